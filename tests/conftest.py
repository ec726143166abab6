import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: CPU test taking more than a few seconds")


@pytest.fixture(scope="session")
def golden():
    cache = {}

    def load(name):
        if name not in cache:
            cache[name] = np.load(os.path.join(GOLDEN, name))
        return cache[name]
    return load


def rel_err(a, ref):
    """max |a - ref| / max |ref|  (the parity metric; frames are in (0,1), states contain
    exact zeros from softshrink, so elementwise relative error is normalised per tensor)."""
    a = np.asarray(a, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.abs(a - ref).max() / max(np.abs(ref).max(), 1e-30))


def elem_rel_err(a, ref):
    """max over elements of |a - ref| / |ref|: the frame metric of SURVEY section 7 (frames lie in
    (0, 1), so each pixel is held to its own magnitude -- a dark pixel of 1e-3 may not be off by
    1e-7 absolute more than 1e-4 of itself).  Not for states, which contain exact zeros."""
    a = np.asarray(a, np.float64)
    ref = np.asarray(ref, np.float64)
    return float((np.abs(a - ref) / np.maximum(np.abs(ref), 1e-30)).max())
