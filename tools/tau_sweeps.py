"""Reproduce the contraction sweeps of asumptions_check.ipynb on the GPU
(the many-chain workloads f3 exists for).

Each cell runs ASSS sample_Pnx through get_taus_n_sss / get_max_taus
(utils_amd.kernel_utils, the notebook's cells 31/41/82/91) with the
notebook's grid, sample count, eps and adapt states, for several rng keys:
the notebook printed one value from one threefry key, this build draws
Philox streams, so a printed value is compared with the spread of the same
estimate over keys 0..K-1.  One JSON line per cell: the notebook's value and
wall time, every key's value, mean / sd, and this run's wall time per key.

  normal target (cell 4: -Normal(0, 1).log_prob), states cell 7:
    s1 (0, 1)  s2 (0, 0.1)  s3 (0, 10)  s4 (1, 1)  s5 (1, 0.1)  s6 (1, 10)
  cell 33  s1, 100 points in +-arctan(5), N = 2e6, eps 0.1: max tau(P^2) = 0.022612354
  cell 35  s4, same grid:                                   max tau(P^2) = 0.36068642
  cell 42  s1, 50 points in +-arctan(2.5), N = 5e5, eps 0.1: tau(P^1) per point (50 values)
  cell 43  n = 1..5, s1..s6 (50 points, N = 5e5):           s6 at n = 5 = 0.008646628 (1 h 07 min)
  mixture target (cells 61-62), states of cell 7:
  cell 92  s1, n = 1 (50 points, N = 5e5, eps 0.1):          max = 1.3503939
  cell 93  n = 1, 5, 10, 20, s1..s3:                         s3 at n = 20 = 0.005598169 (2 h 28 min)
  cell 95  n = 1, 5, 10, 20, s4..s6:                         s6 at n = 20 = 0.005381542 (2 h 37 min)

Usage: python3 tools/tau_sweeps.py [--keys K] [--cells 33,35,42,43,92,93,95] [--out FILE]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))

STATES = {"s1": (0.0, 1.0), "s2": (0.0, 0.1), "s3": (0.0, 10.0), "s4": (1.0, 1.0), "s5": (1.0, 0.1), "s6": (1.0, 10.0)}

# cell 42's printed array (tau_x(P^1), s1, normal target)
CELL42 = [0.13749427, 0.13784078, 0.13309874, 0.12080273, 0.12760013, 0.17321618, 0.16587035, 0.11561218,
          0.04040072, 0.04384528, 0.09744439, 0.12681857, 0.14603475, 0.15111035, 0.14886083, 0.14444587,
          0.12653562, 0.10962022, 0.10412868, 0.07945453, 0.05619029, 0.04250671, 0.0353291, 0.0255759,
          0.02115004, 0.02858813, 0.02533795, 0.02444958, 0.02693902, 0.03665483, 0.04882394, 0.06087109,
          0.07091778, 0.08357223, 0.1012999, 0.11778017, 0.12223762, 0.14037713, 0.13296156, 0.10337605,
          0.05073283, 0.03696393, 0.11621223, 0.16249697, 0.16987962, 0.1222439, 0.1161537, 0.13087057,
          0.13662301, 0.13695103]

# cell: (target, grid half-width as arctan(w), points, N, n_list, states, the printed quantity, value, wall s, eps)
CELLS = {
    33: ("normal", 5.0, 100, 2000000, [2], ["s1"], "max", 0.022612354, None, 0.1),
    35: ("normal", 5.0, 100, 2000000, [2], ["s4"], "max", 0.36068642, None, 0.1),
    42: ("normal", 2.5, 50, 500000, [1], ["s1"], "curve", CELL42, 43.2, 0.1),
    43: ("normal", 2.5, 50, 500000, [1, 2, 3, 4, 5], ["s1", "s2", "s3", "s4", "s5", "s6"], "max_last", 0.008646628,
         4018.0, 0.1),
    92: ("mixture", 2.5, 50, 500000, [1], ["s1"], "max", 1.3503939, 104.0, 0.1),
    93: ("mixture", 2.5, 50, 500000, [1, 5, 10, 20], ["s1", "s2", "s3"], "max_last", 0.005598169, 8908.0, 0.1),
    95: ("mixture", 2.5, 50, 500000, [1, 5, 10, 20], ["s4", "s5", "s6"], "max_last", 0.005381542, 9448.0, 0.1),
    # cell 35 under the settings other cells of the notebook leave behind
    # (its cells ran out of order): eps = 5e-2 and N = 1e6 are cell 83's
    351: ("normal", 5.0, 100, 2000000, [2], ["s4"], "max", 0.36068642, None, 0.05),
    352: ("normal", 5.0, 100, 1000000, [2], ["s4"], "max", 0.36068642, None, 0.05),
    353: ("normal", 2.5, 100, 1000000, [2], ["s4"], "max", 0.36068642, None, 0.05),
}


def kernel_for(target, device):
    import posteriors as P
    from kernels_amd import ASSS
    if target == "normal":
        return ASSS(potential_fn=P.gaussian(np.zeros(1), cov=np.eye(1)), device=device)
    return ASSS(potential_fn=P.notebook_mixture(), device=device)


def run_cell(cell, key, device):
    """Everything the cell computes, for one key: {state: [max tau per n]}
    (or the tau curve for cell 42)."""
    import torch
    from kernels_amd import PRNGKey
    from utils_amd.kernel_utils import get_max_taus, get_taus_n_sss
    target, w, npts, N, n_list, states, kind, _, _, eps = CELLS[cell]
    phis = np.linspace(-np.arctan(w), np.arctan(w), npts).astype(np.float32)
    X = np.tan(phis).reshape(-1, 1)
    k = kernel_for(target, device)
    out = {}
    for s in states:
        loc, sc = STATES[s]
        st = (np.array([loc], np.float32), np.array([[sc]], np.float32))
        if kind == "curve":
            out[s] = get_taus_n_sss(PRNGKey(key), k, X, st, n=n_list[0], n_samples=N, eps=eps).tolist()
        else:
            out[s] = get_max_taus(PRNGKey(key), k, X, st, n_list, n_samples=N, eps=eps)
    torch.cuda.synchronize()
    return out


def printed_value(cell, res):
    """The quantity the notebook printed, from one key's results."""
    _, _, _, _, _, states, kind, _, _, _ = CELLS[cell]
    if kind == "curve":
        return res[states[0]]
    if kind == "max":
        return res[states[0]][-1]
    return res[states[-1]][-1]  # max_taus_s<last>[-1]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--keys", type=int, default=6)
    ap.add_argument("--cells", default="33,35,42,43,92,93,95")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    fo = open(a.out, "a") if a.out else None
    for cell in [int(c) for c in a.cells.split(",")]:
        vals, full, secs = [], [], []
        for key in range(a.keys):
            t0 = time.perf_counter()
            res = run_cell(cell, key, dev)
            secs.append(time.perf_counter() - t0)
            vals.append(printed_value(cell, res))
            full.append(res)
            print(f"cell {cell} key {key}: {secs[-1]:.1f} s", flush=True)
        nb, nb_s = CELLS[cell][7], CELLS[cell][8]
        line = {"cell": cell, "notebook": nb, "notebook_wall_s": nb_s, "wall_s_per_key": [round(s, 2) for s in secs],
                "keys": a.keys, "n_samples": CELLS[cell][3], "points": CELLS[cell][2], "n_list": CELLS[cell][4],
                "eps": CELLS[cell][9], "grid_atan": CELLS[cell][1],
                "states": {s: STATES[s] for s in CELLS[cell][5]}}
        if CELLS[cell][6] == "curve":
            arr = np.array(vals)
            m, sd = arr.mean(0), arr.std(0, ddof=1)
            z = (np.array(nb) - m) / np.maximum(sd, 1e-12)
            line.update(mean=m.round(6).tolist(), sd=sd.round(6).tolist(), max_abs_z=float(np.abs(z).max()),
                        frac_within_3sd=float((np.abs(z) <= 3).mean()))
        else:
            m, sd = float(np.mean(vals)), float(np.std(vals, ddof=1))
            line.update(values=[round(v, 8) for v in vals], mean=m, sd=sd, z=(nb - m) / sd if sd > 0 else None,
                        all_max_taus=full)
        print(json.dumps(line), flush=True)
        if fo:
            fo.write(json.dumps(line) + "\n")
            fo.flush()


if __name__ == "__main__":
    main()
