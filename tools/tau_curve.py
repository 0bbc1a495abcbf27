"""tau_x(P^n) curves of the ASSS kernel on the normal target for one adapt
state over several grids / eps / sample counts (asumptions_check.ipynb cells
31-36; a diagnostic for cell 35).  Usage: python3 tools/tau_curve.py LOC SCALE N_STEPS"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from kernels_amd import PRNGKey  # noqa: E402
from tau_sweeps import kernel_for  # noqa: E402
from utils_amd.kernel_utils import get_taus_n_sss  # noqa: E402

loc, sc, n = float(sys.argv[1]), float(sys.argv[2]), int(sys.argv[3])
k = kernel_for("normal", torch.device("cuda", 0))
st = (np.array([loc], np.float32), np.array([[sc]], np.float32))
grids = {
    "atan5_100": np.tan(np.linspace(-np.arctan(5), np.arctan(5), 100).astype(np.float32)),
    "lin5_50": np.linspace(-5, 5, 50).astype(np.float32),
    "lin5_400": np.linspace(-5, 5, 400).astype(np.float32),
}
for gname, x in grids.items():
    for eps in (0.1, 0.05):
        for N in (2000000, 500000):
            if gname == "lin5_400" and (eps != 0.1 or N != 2000000):
                continue
            t = get_taus_n_sss(PRNGKey(0), k, x.reshape(-1, 1), st, n=n, n_samples=N, eps=eps)
            i = int(np.argmax(t))
            print(json.dumps({"loc": loc, "scale": sc, "n": n, "grid": gname, "eps": eps, "N": N, "max": float(t.max()),
                              "argmax_x": float(x[i]), "curve": np.round(t, 4).tolist() if gname == "lin5_400" else None}),
                  flush=True)
