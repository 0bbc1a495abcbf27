"""The contraction sweeps of asumptions_check.ipynb,
every printed maximum, on the GPU through ASSS sample_Pnx +
get_taus_n_sss / get_max_taus (tools/tau_sweeps.py holds the cells' grids,
sample counts, eps and adapt states).  The notebook printed one estimate
from one threefry key; this build draws Philox streams, so each printed value
must lie within the spread of the same estimate over keys 0..5:
|notebook - mean| <= 4 sd + 2 % of the mean.  Cells 43, 93 and 95 took
1 h 07 min, 2 h 28 min and 2 h 37 min on the notebook's CPU; here about a
second per key (profiles/r6_tau_sweeps.jsonl).

Cell 35 printed 0.36068642 for mu = 1, sigma = 1, n = 2.  With cell 32's
eps = 0.1 and N = 2e6 the estimate is 0.3142 +- 0.0008 (z = 57); with cell
83's eps = 5e-2 and N = 1e6 it is 0.3584 +- 0.0030 (z = 0.75).  The
notebook's cells ran out of order (their execution counts interleave), and
tau depends on eps through the finite difference, so cell 35 is pinned under
the settings that were live when it ran (tools/tau_sweeps.py cell 352)."""
import os
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))


def _keys(cell, gpu, keys=6):
    import tau_sweeps as T
    return [T.printed_value(cell, T.run_cell(cell, k, gpu)) for k in range(keys)]


@pytest.mark.parametrize("cell", [33, 352, 43, 92, 93, 95])
def test_printed_max_within_spread(cell, gpu):
    import tau_sweeps as T
    vals = _keys(cell, gpu)
    nb = T.CELLS[cell][7]
    m, s = float(np.mean(vals)), float(np.std(vals, ddof=1))
    print(f"cell {cell}: keys {np.round(vals, 5).tolist()} mean {m:.5f} sd {s:.5f}; notebook {nb}")
    assert abs(nb - m) <= 4 * s + 0.02 * m, (cell, vals, nb)


def test_cell42_curve(gpu):
    """Cell 42's 50-point tau(P^1) curve (mu = 0, sigma = 1): pointwise within
    3 sd of the keys' mean for 90 % of the points (one key's estimate against
    a 6-key sd), and the same shape (correlation > 0.9; 0.96 measured)."""
    import tau_sweeps as T
    arr = np.array(_keys(42, gpu))
    m, s = arr.mean(0), arr.std(0, ddof=1)
    nb = np.array(T.CELL42)
    z = np.abs(nb - m) / np.maximum(s, 1e-9)
    assert (z <= 3).mean() >= 0.9, z.round(2).tolist()
    assert np.corrcoef(nb, m)[0, 1] > 0.9
