"""librosa 0.8 ``filters.get_window`` / ``filters.mel`` (Slaney scale + Slaney
area norm), restated.  Test-only (see package docstring)."""
import numpy as np
import scipy.signal


def get_window(window, Nx, fftbins=True):
    return scipy.signal.get_window(window, Nx, fftbins=fftbins)


def hz_to_mel(frequencies, htk=False):
    f = np.asanyarray(frequencies, dtype=np.float64)
    if htk:
        return 2595.0 * np.log10(1.0 + f / 700.0)
    f_sp = 200.0 / 3
    mels = f / f_sp
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if f.ndim:
        sel = f >= min_log_hz
        mels = np.array(mels, dtype=np.float64)
        mels[sel] = min_log_mel + np.log(f[sel] / min_log_hz) / logstep
    elif f >= min_log_hz:
        mels = min_log_mel + np.log(f / min_log_hz) / logstep
    return mels


def mel_to_hz(mels, htk=False):
    m = np.asanyarray(mels, dtype=np.float64)
    if htk:
        return 700.0 * (10.0 ** (m / 2595.0) - 1.0)
    f_sp = 200.0 / 3
    freqs = f_sp * m
    min_log_hz = 1000.0
    min_log_mel = min_log_hz / f_sp
    logstep = np.log(6.4) / 27.0
    if m.ndim:
        sel = m >= min_log_mel
        freqs = np.array(freqs, dtype=np.float64)
        freqs[sel] = min_log_hz * np.exp(logstep * (m[sel] - min_log_mel))
    elif m >= min_log_mel:
        freqs = min_log_hz * np.exp(logstep * (m - min_log_mel))
    return freqs


def mel(sr, n_fft, n_mels=128, fmin=0.0, fmax=None, htk=False, norm='slaney',
        dtype=np.float32):
    if fmax is None:
        fmax = float(sr) / 2
    n_bins = int(1 + n_fft // 2)
    weights = np.zeros((int(n_mels), n_bins), dtype=dtype)
    fftfreqs = np.linspace(0, float(sr) / 2, n_bins, endpoint=True)
    mel_pts = np.linspace(hz_to_mel(fmin, htk), hz_to_mel(fmax, htk), int(n_mels) + 2)
    mel_f = mel_to_hz(mel_pts, htk)
    fdiff = np.diff(mel_f)
    ramps = np.subtract.outer(mel_f, fftfreqs)
    for i in range(int(n_mels)):
        lower = -ramps[i] / fdiff[i]
        upper = ramps[i + 2] / fdiff[i + 1]
        weights[i] = np.maximum(0, np.minimum(lower, upper))
    if norm in ('slaney', 1):
        enorm = 2.0 / (mel_f[2:int(n_mels) + 2] - mel_f[:int(n_mels)])
        weights *= enorm[:, np.newaxis]
    return weights
