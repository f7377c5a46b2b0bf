"""Test-only stand-in for the subset of librosa the reference touches on the
inference path (construction-time filter design + power_to_db).

NOT product code.  Used only by ``oracle/make_golden.py`` to import the
reference (``/root/reference``) in this container, where librosa is absent.
The reference's requirements.txt leaves librosa unpinned; its positional
``pad_center(w, n_fft)`` call (pytorch/stft.py:195) implies librosa < 0.10, so
the algorithms below restate the published librosa 0.8 behaviour.
"""
from . import filters, util, core, display  # noqa: F401
from .core import power_to_db  # noqa: F401
