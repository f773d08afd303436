"""CPython ``random`` state <-> the 625-word layout the C-ABI takes
(include/rg_hip.h: 624 MT19937 words + position), so the device sampler
continues exactly the stream ``random.getstate()`` describes (implicit.py:352
draws with the module-level ``random``)."""
import random

import numpy as np


def from_python(py_state):
    """random.getstate() -> np.uint32[625]."""
    version, internal, _gauss = py_state
    if version != 3 or len(internal) != 625:
        raise ValueError("unexpected random.getstate() layout")
    return np.asarray(internal, dtype=np.uint32).copy()


def to_python(state, gauss_next=None):
    """np.uint32[625] -> a tuple for random.setstate()."""
    return (3, tuple(int(x) for x in np.asarray(state, dtype=np.uint32)), gauss_next)


def current():
    """State of the module-level ``random`` generator."""
    return from_python(random.getstate())


def restore(state):
    """Write a device-advanced state back into the module-level generator."""
    random.setstate(to_python(state, random.getstate()[2]))
