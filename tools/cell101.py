"""asumptions_check.ipynb cell 101 (rho(P, Q), frozen 1-D N(0, 1) kernels with
scale 1 and 0.1) over several keys, with what the trained network is: the
final gradient norm (the notebook: 1000 steps, 0.436), rho, and the trained
f's actual Lipschitz constant on a fine grid (the spectral normalisation's ten
power iterations from a fixed start vector can leave f above 1-Lipschitz,
which raises rho).  Usage (GPU box): python3 tools/cell101.py [n_keys]"""
import contextlib
import io
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))

import torch  # noqa: E402

import posteriors as P  # noqa: E402
from kernels_amd import ARWMH, PRNGKey  # noqa: E402
from utils_amd import lipschitz as Lz  # noqa: E402


def main():
    n_keys = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    g = P.gaussian(np.zeros(1), cov=np.eye(1))
    k = ARWMH(potential_fn=g, num_chains=1)
    s_p = (torch.zeros(1), torch.ones(1, 1), torch.zeros(()))
    s_q = (torch.zeros(1), 0.1 * torch.ones(1, 1), torch.zeros(()))
    fp = lambda key, x, n: k.sample_Pnx(key, x, s_p, 1, n)
    fq = lambda key, x, n: k.sample_Pnx(key, x, s_q, 1, n)
    x = torch.linspace(-5, 5, 100)
    grid = torch.linspace(-8, 8, 20001, device="cuda").reshape(-1, 1)
    rhos = []
    for seed in range(n_keys):
        buf = io.StringIO()
        Lz.TRAIN_LOG = []
        with contextlib.redirect_stdout(buf):
            rho, model, _ = Lz.compute_kernel_distance_1d(fp, fq, PRNGKey(seed), x, sample_batch_size=1000,
                                                          n_train_batches=1, n_eval_batches=1000, max_steps=1000,
                                                          lr=0.1, ratio_rad=5)
        with torch.no_grad():
            f = model(grid)
            lip = float((f[1:] - f[:-1]).abs().max() / (grid[1, 0] - grid[0, 0]))
        rhos.append(rho)
        traj = {s_: (l_, g_) for s_, l_, g_ in Lz.TRAIN_LOG}
        tr = " ".join(f"{s_}:{-traj[s_][0]:.3f}/{traj[s_][1]:.3g}" for s_ in (1, 10, 100, 300, 600, 1000) if s_ in traj)
        print(f"key {seed}: rho {rho:.4f}; {buf.getvalue().strip()}; Lipschitz constant of the trained f "
              f"on [-8, 8]: {lip:.4f}; training ratio/grad-norm at steps {tr}", flush=True)
        Lz.TRAIN_LOG = None
    print(f"rho mean {np.mean(rhos):.4f} sd {np.std(rhos, ddof=1):.4f} (notebook 0.544187)")


if __name__ == "__main__":
    main()
