"""Audio input: librosa.core.load(path, sr, mono=True) as the
reference's drivers call it (pytorch/predict.py:295, pytorch/main_strong.py:787).

Parity status: soundfile, librosa and resampy are neither installed nor part
of /root/reference, so nothing here is pinned by a reference output.  The CPU
restatement (oracle/audio_oracle.py) is checked against exact known answers
(libsndfile's integer scaling) and band-limited reconstruction of sinusoids;
the HIP path (sedx.audio) is checked bit-exactly against the restatement for
decoding and within 1e-6 for resampling (float64 filter-table evaluation
order differs between numpy and C++ in the last bits).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import audio_oracle as A

FORMATS = [('pcm', 8), ('pcm', 16), ('pcm', 24), ('pcm', 32), ('float', 32), ('float', 64)]


def _signal(ch, n, sr, seed=0):
    rng = np.random.default_rng(seed)
    t = np.arange(n) / sr
    s = [0.5 * np.sin(2 * np.pi * (300 + 200 * c) * t) + 0.05 * rng.standard_normal(n) for c in range(ch)]
    return np.clip(np.stack(s), -0.99, 0.99)


# ---------------------------------------------------------------- CPU tests
def test_oracle_decode_known_answers():
    for fmt, bits in FORMATS:
        raw = A.write_wav(np.array([[0.0, 0.5, -0.25, 0.75]]), 16000, bits, fmt)
        y, sr = A.decode(raw)
        assert sr == 16000 and y.shape == (1, 4) and y.dtype == np.float32
        tol = {8: 2 ** -7, 16: 2 ** -15, 24: 2 ** -23}.get(bits, 0) if fmt == 'pcm' else 0
        np.testing.assert_allclose(y[0], [0.0, 0.5, -0.25, 0.75], atol=tol)
    # int16 -32768 .. 32767 -> x / 32768 exactly (libsndfile normalisation)
    raw = A.write_wav(np.array([[-1.0, 32767 / 32768, 1 / 32768]]), 8000, 16)
    np.testing.assert_array_equal(A.decode(raw)[0][0], np.float32([-1.0, 32767 / 32768, 1 / 32768]))


def test_oracle_to_mono_is_float32_mean():
    y = np.float32([[0.1, 0.2], [0.3, 0.7], [0.5, 0.9]])
    np.testing.assert_array_equal(A.to_mono(y), np.mean(y, axis=0))
    assert A.to_mono(y).dtype == np.float32


@pytest.mark.parametrize('sr_in,sr_out', [(44100, 16000), (32000, 16000), (48000, 16000), (8000, 16000)])
def test_oracle_resample_bandlimited(sr_in, sr_out):
    """A sinusoid well inside both bands is reproduced at the new rate (away
    from the edges, where the filter runs off the signal), up to resampy's
    passband gain: resample_f steps the filter table by int(scale * 512)
    (185 for 44.1 -> 16 kHz instead of 185.76), which leaves a passband gain
    of 1.0027 at 440 Hz; reproduced as the library has it."""
    n = sr_in // 2
    t = np.arange(n) / sr_in
    f0 = 440.0
    y = A.resample(np.sin(2 * np.pi * f0 * t).astype(np.float32), sr_in, sr_out, 'kaiser_best')
    assert y.shape == (int(np.ceil(n * sr_out / sr_in)),)
    tt = np.arange(y.size) / sr_out
    ref = np.sin(2 * np.pi * f0 * tt)
    mid = slice(200, y.size - 200)
    gain = float(np.dot(y[mid], ref[mid]) / np.dot(ref[mid], ref[mid]))
    exact_step = min(1.0, sr_out / sr_in) * 512 == int(min(1.0, sr_out / sr_in) * 512)
    assert abs(gain - 1.0) < (2e-4 if exact_step else 5e-3), gain
    assert np.max(np.abs(y[mid] - gain * ref[mid])) < 2e-4


def test_oracle_resample_fast_filter_bandlimited():
    sr_in, sr_out = 44100, 16000
    t = np.arange(sr_in // 2) / sr_in
    y = A.resample(np.sin(2 * np.pi * 1000 * t).astype(np.float32), sr_in, sr_out, 'kaiser_fast')
    tt = np.arange(y.size) / sr_out
    ref = np.sin(2 * np.pi * 1000 * tt)[100:-100]
    gain = float(np.dot(y[100:-100], ref) / np.dot(ref, ref))
    assert abs(gain - 1.0) < 1e-2
    assert np.max(np.abs(y[100:-100] - gain * ref)) < 5e-3


def test_wav_parse_abi_matches_oracle():
    """sedx_wav_parse (host code of libsedx, no GPU) on every format,
    WAVE_FORMAT_EXTENSIBLE and an odd-sized extra chunk."""
    from sedx import audio
    for fmt, bits in FORMATS:
        for ext in (False, True):
            for ch in (1, 2, 3):
                raw = A.write_wav(_signal(ch, 101, 22050), 22050, bits, fmt, extensible=ext)
                info = audio.wav_info(raw)
                tag, ch_o, sr, bits_o, data = A.parse_wav(raw)
                assert (info.channels, info.sample_rate, info.bits_per_sample) == (ch_o, sr, bits_o)
                assert info.format == tag and info.frames == 101
                assert bytes(raw[info.data_offset:info.data_offset + info.data_bytes]) == data
    with pytest.raises(RuntimeError):
        audio.wav_info(b'RIFF\x00\x00\x00\x00WAVEjunk')


# ---------------------------------------------------------------- GPU tests
@pytest.mark.gpu
@pytest.mark.parametrize('fmt,bits', FORMATS)
@pytest.mark.parametrize('ch', [1, 2, 3])
def test_gpu_decode_mono_bit_exact(tmp_path, fmt, bits, ch):
    from sedx import audio
    raw = A.write_wav(_signal(ch, 5000, 16000, seed=ch), 16000, bits, fmt)
    p = os.path.join(tmp_path, 'a.wav')
    open(p, 'wb').write(raw)
    y, sr = audio.load(p, sr=None)
    ref, sr_ref = A.load(raw, sr=None)
    assert sr == sr_ref == 16000
    np.testing.assert_array_equal(y.cpu().numpy(), ref)


@pytest.mark.gpu
@pytest.mark.parametrize('sr_in,ch,res_type', [(44100, 2, 'kaiser_best'), (32000, 1, 'kaiser_best'),
                                                (48000, 2, 'kaiser_fast'), (22050, 1, 'kaiser_best'),
                                                (8000, 1, 'kaiser_best')])
def test_gpu_load_resample_vs_oracle(tmp_path, sr_in, ch, res_type):
    from sedx import audio
    raw = A.write_wav(_signal(ch, int(sr_in * 1.3), sr_in, seed=sr_in), sr_in, 16)
    p = os.path.join(tmp_path, 'b.wav')
    open(p, 'wb').write(raw)
    y, sr = audio.load(p, sr=16000, res_type=res_type)
    ref, _ = A.load(raw, sr=16000, res_type=res_type)
    assert sr == 16000 and y.shape[0] == ref.shape[0]
    d = float(np.max(np.abs(y.cpu().numpy().astype(np.float64) - ref)))
    print('resample %d -> 16000 (%s, %d ch): max|d| = %.3g' % (sr_in, res_type, ch, d))
    assert d <= 1e-6


@pytest.mark.gpu
def test_gpu_load_feeds_the_windowed_driver(tmp_path):
    """A 10 s 44.1 kHz stereo WAV -> load(sr=16000) -> predict_windows: the
    merged framewise output equals the one from the oracle-loaded waveform
    run through the same GPU model (the input side adds no error beyond
    the resampler's 1e-6)."""
    from sedx import audio, inference, models, synth
    mt = 'Cnn_9layers_Gru_FrameAtt'
    m = models.Cnn_9layers_Gru_FrameAtt(16000, 512, 160, 64, 25, 7000, 25, 'logmel')
    sd = m.state_dict()
    for k, v in synth.make_state_dict(mt, seed=0).items():
        sd[k] = torch.from_numpy(v)
    m.load_state_dict(sd)
    m = m.cuda().eval()
    raw = A.write_wav(_signal(2, 441000, 44100, seed=9) * 0.5, 44100, 16)
    p = os.path.join(tmp_path, 'c.wav')
    open(p, 'wb').write(raw)
    y, _ = audio.load(p, sr=16000)
    ref, _ = A.load(raw, sr=16000)
    with torch.no_grad():
        a = inference.predict_windows(m, y[None], 5, 1)
        b = inference.predict_windows(m, torch.from_numpy(ref)[None].cuda(), 5, 1)
    assert a.shape == b.shape == (1, 1000, 25)
    assert float((a - b).abs().max()) <= 1e-3
