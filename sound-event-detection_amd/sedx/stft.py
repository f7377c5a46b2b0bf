"""Frontend construction (host side, construction time only).

The reference builds these with librosa at model construction and stores them
in the state_dict (pytorch/stft.py:157-221 STFT conv weights; :674-692
melW).  The FFT kernel in libsedx only needs the window (row 0 of
conv_real) and the mel band weights, but the state_dict layout is kept so a
reference .pth loads unchanged.  librosa is not a dependency: the periodic
Hann window and the librosa-0.8 Slaney mel filterbank are computed here.
"""
import numpy as np
import torch
import torch.nn as nn


def hann_periodic(n):
    """scipy.signal.get_window('hann', n, fftbins=True) (pytorch/stft.py:192)."""
    return 0.5 - 0.5 * np.cos(2.0 * np.pi * np.arange(n) / n)


def stft_conv_weights(n_fft):
    """Re/Im(DFT[:, :n_fft//2+1] * window).T -> 2 x [n_fft//2+1, 1, n_fft]
    (pytorch/stft.py:20-24, :209-217)."""
    n = np.arange(n_fft)
    k = np.arange(n_fft // 2 + 1)
    ang = -2.0 * np.pi * np.outer(n, k) / n_fft
    w = hann_periodic(n_fft)[:, None]
    return ((np.cos(ang) * w).T.astype(np.float32)[:, None, :],
            (np.sin(ang) * w).T.astype(np.float32)[:, None, :])


def _hz_to_mel(f):
    f = np.asarray(f, dtype=np.float64)
    lin = f * 3.0 / 200.0
    return np.where(f >= 1000.0, 15.0 + np.log(np.maximum(f, 1e-300) / 1000.0) * 27.0 / np.log(6.4), lin)


def _mel_to_hz(m):
    m = np.asarray(m, dtype=np.float64)
    return np.where(m >= 15.0, 1000.0 * np.exp((m - 15.0) * np.log(6.4) / 27.0), m * 200.0 / 3.0)


def mel_weights(sr, n_fft, n_mels, fmin, fmax):
    """librosa.filters.mel(sr, n_fft, n_mels, fmin, fmax).T (librosa 0.8:
    Slaney scale, Slaney area norm, float32) -> [n_fft//2+1, n_mels]
    (pytorch/stft.py:688-689)."""
    if fmax is None:
        fmax = sr // 2
    n_bins = n_fft // 2 + 1
    freqs = np.linspace(0.0, sr / 2.0, n_bins)
    mel_f = _mel_to_hz(np.linspace(_hz_to_mel(fmin), _hz_to_mel(fmax), n_mels + 2))
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, freqs)
    w = np.zeros((n_mels, n_bins), dtype=np.float32)
    for i in range(n_mels):
        w[i] = np.maximum(0.0, np.minimum(-ramps[i] / fdiff[i], ramps[i + 2] / fdiff[i + 1]))
    w *= (2.0 / (mel_f[2:n_mels + 2] - mel_f[:n_mels]))[:, None]
    return np.ascontiguousarray(w.T)


class STFT(nn.Module):
    """Parameter container with the reference's keys (conv_real / conv_imag).
    The transform itself runs in libsedx (FFT kernel)."""

    def __init__(self, n_fft=2048, hop_length=None, win_length=None, window='hann', center=True,
                 pad_mode='reflect', freeze_parameters=True):
        super().__init__()
        if window != 'hann' or not center or pad_mode != 'reflect' or (win_length not in (None, n_fft)):
            raise ValueError('sedx implements the reference configuration only '
                             "(hann, center=True, reflect, win_length=n_fft)")
        self.n_fft = n_fft
        self.hop_length = hop_length if hop_length is not None else n_fft // 4
        out = n_fft // 2 + 1
        self.conv_real = nn.Conv1d(1, out, n_fft, stride=self.hop_length, bias=False)
        self.conv_imag = nn.Conv1d(1, out, n_fft, stride=self.hop_length, bias=False)
        wr, wi = stft_conv_weights(n_fft)
        self.conv_real.weight.data = torch.from_numpy(wr)
        self.conv_imag.weight.data = torch.from_numpy(wi)
        if freeze_parameters:
            for p in self.parameters():
                p.requires_grad = False

    def forward(self, input):
        raise RuntimeError('STFT is fused into the native model forward (libsedx)')


class Spectrogram(nn.Module):
    """pytorch/stft.py:636-670 (container; computed natively)."""

    def __init__(self, n_fft=2048, hop_length=None, win_length=None, window='hann', center=True,
                 pad_mode='reflect', power=2.0, freeze_parameters=True):
        super().__init__()
        if power != 2.0:
            raise ValueError('only power=2.0 is on the reference path')
        self.stft = STFT(n_fft, hop_length, win_length, window, center, pad_mode, True)

    def forward(self, input):
        raise RuntimeError('Spectrogram is fused into the native model forward (libsedx)')


class LogmelFilterBank(nn.Module):
    """pytorch/stft.py:673-734 (container; computed natively, top_db=None)."""

    def __init__(self, sr=22050, n_fft=2048, n_mels=64, fmin=0.0, fmax=None, is_log=True,
                 ref=1.0, amin=1e-10, top_db=80.0, freeze_parameters=True):
        super().__init__()
        if not is_log or ref != 1.0 or amin != 1e-10 or top_db is not None:
            raise ValueError('sedx implements the models\' configuration (is_log, ref=1, '
                             'amin=1e-10, top_db=None)')
        self.melW = nn.Parameter(torch.from_numpy(mel_weights(sr, n_fft, n_mels, fmin, fmax)))
        if freeze_parameters:
            self.melW.requires_grad = False

    def forward(self, input):
        raise RuntimeError('LogmelFilterBank is fused into the native model forward (libsedx)')
