"""librosa.core subset (test-only): power_to_db as in librosa 0.8."""
import numpy as np


def power_to_db(S, ref=1.0, amin=1e-10, top_db=80.0):
    S = np.asarray(S)
    magnitude = S
    ref_value = ref(magnitude) if callable(ref) else np.abs(ref)
    log_spec = 10.0 * np.log10(np.maximum(amin, magnitude))
    log_spec -= 10.0 * np.log10(np.maximum(amin, ref_value))
    if top_db is not None:
        log_spec = np.maximum(log_spec, log_spec.max() - top_db)
    return log_spec


def load(*args, **kwargs):  # I/O is out of scope; never reached by the harness
    raise NotImplementedError('librosa.load is not available in the oracle shim')


def get_duration(*args, **kwargs):
    raise NotImplementedError
