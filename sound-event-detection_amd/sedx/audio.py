"""Audio input on the GPU: ``librosa.core.load(path, sr=..., mono=True)`` as
the reference's drivers call it (pytorch/predict.py:295, pytorch/main_strong.py:787,
utils/features.py:356) before slicing windows, plus the HDF5 int16 packing's
dequantisation (utils/utilities.py:73-79, which ``sedx_forward_i16`` fuses
into the frontend).

librosa 0.8 ``load`` = soundfile read (float32, libsndfile scaling) ->
``to_mono`` (mean over channels) -> ``resample(res_type='kaiser_best')`` =
resampy band-limited interpolation + ``fix_length`` to ceil(n * sr / sr_native).
Here: the WAV header is parsed on the host (``sedx_wav_parse``), the sample
bytes are copied to the device once, and decode + downmix
(``sedx_wav_decode_mono``) and resampling (``sedx_resample``) run as HIP
kernels.  WAV only (the reference converts other containers with ffmpeg
first, pytorch/predict.py:287-294).
"""
import ctypes

import numpy as np
import torch

from . import _lib


def wav_info(data):
    """Parse a WAV file image (bytes / uint8 array) -> sedx_wav_info fields."""
    buf = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    info = _lib.SedxWavInfo()
    st = _lib.lib().sedx_wav_parse(buf.ctypes.data_as(ctypes.c_void_p), buf.nbytes, ctypes.byref(info))
    if st != _lib.SEDX_OK:
        raise RuntimeError('sedx_wav_parse: not a PCM (8/16/24/32-bit) or IEEE-float (32/64-bit) WAV file')
    return info


def _stream(dev):
    return ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)


def resample(y, orig_sr, target_sr, res_type='kaiser_best'):
    """librosa.resample (0.8) of a 1-D float32 HIP tensor on the GPU."""
    if y.device.type != 'cuda':
        raise RuntimeError('sedx resample needs a HIP tensor (no CPU fallback)')
    if res_type not in _lib.RESAMPLE:
        raise ValueError('res_type must be one of %s' % sorted(_lib.RESAMPLE))
    y = y.to(torch.float32).contiguous()
    L = _lib.lib()
    n_in = y.numel()
    n_out = ctypes.c_int64()
    _lib.check(L.sedx_resample_size(n_in, int(orig_sr), int(target_sr), ctypes.byref(n_out)), None,
               'resample_size')
    out = torch.empty(n_out.value, dtype=torch.float32, device=y.device)
    q = _lib.RESAMPLE[res_type]
    wsz = ctypes.c_size_t(0)
    if orig_sr != target_sr:
        _lib.check(L.sedx_resample_workspace_size(n_in, int(orig_sr), int(target_sr), q, ctypes.byref(wsz)),
                   None, 'resample_workspace_size')
    ws = torch.empty(max(wsz.value, 1), dtype=torch.uint8, device=y.device)
    with torch.cuda.device(y.device):
        _lib.check(L.sedx_resample(ctypes.c_void_p(y.data_ptr()), n_in, int(orig_sr), int(target_sr), q,
                                   ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ws.data_ptr()), wsz.value,
                                   _stream(y.device)), None, 'resample')
    return out


def load(path, sr=22050, mono=True, res_type='kaiser_best', device=None):
    """``librosa.core.load(path, sr=sr, mono=True, res_type=res_type)`` with
    the decode, downmix and resampling on the GPU.  Returns (float32 HIP
    tensor [n], sample_rate)."""
    if not mono:
        raise NotImplementedError('the reference loads mono audio only (mono=True)')
    dev = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
    if dev.type != 'cuda':
        raise RuntimeError('sedx audio loading runs on HIP devices only (no CPU fallback)')
    raw = np.fromfile(path, dtype=np.uint8)
    info = wav_info(raw)
    data = torch.from_numpy(raw[info.data_offset:info.data_offset + info.frames * info.channels *
                                (info.bits_per_sample // 8)].copy()).to(dev)
    y = torch.empty(info.frames, dtype=torch.float32, device=dev)
    with torch.cuda.device(dev):
        _lib.check(_lib.lib().sedx_wav_decode_mono(ctypes.c_void_p(data.data_ptr()), ctypes.byref(info),
                                                   ctypes.c_void_p(y.data_ptr()), _stream(dev)),
                   None, 'wav_decode_mono')
    if sr is None or sr == info.sample_rate:
        return y, info.sample_rate
    return resample(y, info.sample_rate, sr, res_type), sr
