"""ctypes binding of libsedx.so (C ABI declared in include/sedx.h).

torch is imported first on purpose: the PyTorch-ROCm wheel ships its own
libamdhip64.so with the same SONAME (libamdhip64.so.7) as /opt/rocm's, so
loading libsedx after torch binds it to the HIP runtime torch already runs
(one runtime per process, device pointers shared)."""
import ctypes
import os

import torch  # noqa: F401  (see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, 'libsedx.so')

SEDX_OK = 0
STATUS = {0: 'OK', 1: 'EINVAL', 2: 'ENOMEM', 3: 'EHIP', 4: 'ESTATE', 5: 'EKEY'}

EXPORTS = ['sedx_create', 'sedx_destroy', 'sedx_last_error', 'sedx_version', 'sedx_load_param',
           'sedx_finalize_weights', 'sedx_output_geometry', 'sedx_workspace_size',
           'sedx_forward', 'sedx_forward_features', 'sedx_gamma_features',
           'sedx_window_geometry', 'sedx_forward_windows', 'sedx_window_workspace_size',
           'sedx_events', 'sedx_set_profiling', 'sedx_stage_times', 'sedx_set_precision', 'sedx_set_pipelined',
           'sedx_forward_windows_vote', 'sedx_events_workspace_size', 'sedx_events_device',
           'sedx_forward_i16', 'sedx_wav_parse', 'sedx_wav_decode_mono', 'sedx_resample_size',
           'sedx_resample_workspace_size', 'sedx_resample', 'sedx_gamma_workspace_size',
           'sedx_set_tuning', 'sedx_set_capture', 'sedx_window_starts', 'sedx_merge_host', 'sedx_check_error',
           'sedx_abi_version']
TUNE_GRU_KERNEL, TUNE_GRU_HANDOFF, TUNE_WINO_BLOCK1, TUNE_MEL_MFMA, TUNE_GRU_SPIN, TUNE_WINO_ORDER = 0, 1, 2, 3, 4, 5
TUNE_GAMMA_SPEC = 6
TUNE_WINO_F43 = 7
PRECISION = {'exact': 0, 'x3': 1, 'winograd': 2}
STAGES = ['frontend', 'b1c1', 'b1c2', 'b2c1', 'b2c2', 'b3c1', 'b3c2', 'b4c1', 'b4c2', 'seq', 'head', 'pipeline_wait']


class SedxWavInfo(ctypes.Structure):
    _fields_ = [('format', ctypes.c_int32), ('channels', ctypes.c_int32),
                ('sample_rate', ctypes.c_int32), ('bits_per_sample', ctypes.c_int32),
                ('frames', ctypes.c_int64), ('data_offset', ctypes.c_int64),
                ('data_bytes', ctypes.c_int64)]


RESAMPLE = {'kaiser_best': 0, 'kaiser_fast': 1}

DRIVER = {'predict': 0, 'main_strong': 1}

ABI_VERSION = 5   # include/sedx.h SEDX_ABI_VERSION


class SedxWindowSpec(ctypes.Structure):
    _fields_ = [('driver', ctypes.c_int32), ('overlap', ctypes.c_int32),
                ('sample_duration', ctypes.c_int32), ('vote', ctypes.c_int32),
                ('overlap_value', ctypes.c_double), ('audio_duration', ctypes.c_double)]


def window_spec(sample_duration, overlap_value, driver='predict', overlap=True, audio_duration=None, vote=False):
    """sedx_window_spec of one windowed-driver call (include/sedx.h); vote=True
    for sedx_forward_windows_vote (its geometry / workspace queries then size
    the vote merge, which accepts a zero merge step)."""
    if driver not in DRIVER:
        raise ValueError('driver must be one of %s' % sorted(DRIVER))
    if int(sample_duration) != sample_duration:
        raise ValueError('sample_duration is an int number of seconds in the reference (predict.py:701)')
    return SedxWindowSpec(DRIVER[driver], int(bool(overlap)), int(sample_duration), int(bool(vote)),
                          float(overlap_value),
                          float(audio_duration) if audio_duration is not None else 0.0)


class SedxConfig(ctypes.Structure):
    _fields_ = [('model_type', ctypes.c_int32), ('feature_type', ctypes.c_int32),
                ('sample_rate', ctypes.c_int32), ('window_size', ctypes.c_int32),
                ('hop_size', ctypes.c_int32), ('mel_bins', ctypes.c_int32),
                ('fmin', ctypes.c_float), ('fmax', ctypes.c_float),
                ('classes_num', ctypes.c_int32)]


_lib = None

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int32
F32 = ctypes.c_float
F64 = ctypes.c_double
SZ = ctypes.c_size_t
PI64 = ctypes.POINTER(ctypes.c_int64)
PSZ = ctypes.POINTER(ctypes.c_size_t)
PSPEC = ctypes.POINTER(SedxWindowSpec)


def lib():
    """Load libsedx.so (fails loudly if it was not built: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError('libsedx.so not found at %s: build it with `make -C '
                           'sound-event-detection_amd` or __graft_entry__.build()' % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    sig = {
        'sedx_create': ([ctypes.POINTER(SedxConfig), ctypes.c_int, ctypes.POINTER(P)], I32),
        'sedx_destroy': ([P], None),
        'sedx_last_error': ([P], ctypes.c_char_p),
        'sedx_version': ([], ctypes.c_char_p),
        'sedx_abi_version': ([], I32),
        'sedx_load_param': ([P, ctypes.c_char_p, P, PI64, I32], I32),
        'sedx_finalize_weights': ([P], I32),
        'sedx_output_geometry': ([P, I64, PI64, PI64], I32),
        'sedx_workspace_size': ([P, I64, I64, PSZ], I32),
        'sedx_forward': ([P, P, I64, I64, P, P, P, P, SZ, P], I32),
        'sedx_forward_features': ([P, P, I64, I64, P, P, P, P, SZ, P], I32),
        'sedx_forward_i16': ([P, P, I64, I64, P, P, P, P, SZ, P], I32),
        'sedx_gamma_features': ([P, P, I64, I64, P, PI64, P, SZ, P], I32),
        'sedx_gamma_workspace_size': ([P, I64, I64, PSZ], I32),
        'sedx_set_tuning': ([P, I32, I32], I32),
        'sedx_check_error': ([P], I32),
        'sedx_set_capture': ([P, I32, P, SZ], I32),
        'sedx_window_starts': ([I32, I64, PSPEC, P, P, I64, PI64], I32),
        'sedx_merge_host': ([P, P, I64, I64, I32, F64, I32, P, I64, PI64], I32),
        'sedx_window_geometry': ([P, I64, PSPEC, PI64, PI64, PI64], I32),
        'sedx_forward_windows': ([P, P, I64, I64, PSPEC, P, P, SZ, P], I32),
        'sedx_window_workspace_size': ([P, I64, I64, PSPEC, PSZ], I32),
        'sedx_events': ([P, I64, I64, I64, P, P, I32, P, P, P, I64, PI64], I32),
        'sedx_forward_windows_vote': ([P, P, I64, I64, PSPEC, P, P, P, SZ, P], I32),
        'sedx_events_workspace_size': ([I64, I64, I64, PSZ], I32),
        'sedx_events_device': ([P, I64, I64, I64, P, P, I32, P, P, I32, F64, I32, P, I64, P, P, SZ, P],
                               I32),
        'sedx_set_profiling': ([P, I32], I32),
        'sedx_set_precision': ([P, I32], I32),
        'sedx_set_pipelined': ([P, I32], I32),
        'sedx_stage_times': ([P, ctypes.POINTER(ctypes.c_float), I32, ctypes.POINTER(I32)], I32),
        'sedx_wav_parse': ([P, SZ, ctypes.POINTER(SedxWavInfo)], I32),
        'sedx_wav_decode_mono': ([P, ctypes.POINTER(SedxWavInfo), P, P], I32),
        'sedx_resample_size': ([I64, I32, I32, PI64], I32),
        'sedx_resample_workspace_size': ([I64, I32, I32, I32, PSZ], I32),
        'sedx_resample': ([P, I64, I32, I32, I32, P, P, SZ, P], I32),
    }
    # an ABI <= 4 library has no sedx_abi_version (nor later entry points):
    # say "rebuild" before the argtypes loop trips over a missing symbol
    if not hasattr(L, 'sedx_abi_version'):
        raise RuntimeError('libsedx.so ABI <= 4 (no sedx_abi_version), this binding expects %d '
                           '(include/sedx.h SEDX_ABI_VERSION): rebuild the library' % ABI_VERSION)
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.sedx_abi_version() != ABI_VERSION:
        raise RuntimeError('libsedx.so ABI %d, this binding expects %d (include/sedx.h SEDX_ABI_VERSION): '
                           'rebuild the library' % (L.sedx_abi_version(), ABI_VERSION))
    _lib = L
    return L


def check(status, handle=None, what=''):
    if status != SEDX_OK:
        msg = lib().sedx_last_error(handle).decode() if handle else ''
        raise RuntimeError('libsedx %s failed (%s): %s' % (what, STATUS.get(status, status), msg))
