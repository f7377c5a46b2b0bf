"""librosa.util subset (test-only)."""
import numpy as np
from . import exceptions  # noqa: F401


def pad_center(data, size, axis=-1, **kwargs):
    kwargs.setdefault('mode', 'constant')
    n = data.shape[axis]
    lpad = int((size - n) // 2)
    lengths = [(0, 0)] * data.ndim
    lengths[axis] = (lpad, int(size - n - lpad))
    if lpad < 0:
        raise exceptions.ParameterError('Target size must be at least input size')
    return np.pad(data, lengths, **kwargs)
