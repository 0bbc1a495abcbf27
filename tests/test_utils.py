"""Driver helpers (reference python/utils/kernel_utils.py)."""
import numpy as np

from utils_amd.kernel_utils import ns_logscale


def test_ns_logscale_grid():
    n = ns_logscale(6)
    assert len(n) == 460
    assert list(n[:10]) == list(range(1, 11))
    assert list(n[10:100]) == list(range(11, 101))
    assert list(n[100:103]) == [110, 120, 130]
    assert n[-1] == 10 ** 6 and np.all(np.diff(n) > 0)
    assert list(ns_logscale(0)) == [1]
