"""asumptions_check.ipynb cell 101 by exact quadrature (CPU, float64).

The notebook prints rho(P, Q) = 0.544187 for the frozen 1-D N(0, 1) kernels
with scale 1 (P) and 0.1 (Q), x = linspace(-5, 5, 100) and rho_conf (1000 Adam
steps at lr 0.1, ratio_rad 5, 1000 x 1000-sample evaluation).  This tool
separates the three things that number mixes (oracle/metropolis_1d.py):

  1. the Kantorovich-Rubinstein supremum over ALL 1-Lipschitz f, per adjacent
     pair, by quadrature of |F_mu|: the largest value the estimator can
     approach without noise;
  2. what the reference's training procedure (lipschitz.py:396-491 restated on
     the CPU in float64: the same LipschitzNN, spectral normalisation, Adam,
     element-wise clipping, ratio_rad 5, stopping rule) attains, with the
     trained f evaluated EXACTLY -- trained once on the exact objective
     (noise-free (P - Q) f) and once on Monte Carlo draws of the kernel
     (1000 per point for P and for Q, as sample_batch_size = 1000);
  3. the evaluation's Monte Carlo bias for each trained f: the expected max
     over the 99 noisy adjacent ratios (10^6 draws per point) minus the
     noise-free max, and the probability of reaching 0.544187.

Usage: python tools/cell101_exact.py [n_keys] [--seed0 S] [--modes exact,mc] [--build-keys]
       [--out profiles/r5_cell101_exact.txt]
(--build-keys: the initial networks of the build's keys PRNGKey(S..), for a
per-key comparison with tests/test_lipschitz.py's GPU run)
"""
import argparse
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "adaptive-mcmc_amd"))
sys.path.insert(0, ROOT)

from oracle import metropolis_1d as M  # noqa: E402
from kernels_amd.random import PRNGKey, split  # noqa: E402
from utils_amd.lipschitz import LipschitzNN, _init_seed  # noqa: E402

NOTEBOOK = 0.544187
SP, SQ = 1.0 + 1e-6, 0.1 + 1e-6  # arwmh.py:166: L e^lam + eps


def train(seed, x, mode, steps=1000, lr=0.1, rad=5, n_samp=1000, init_seed=None):
    torch.manual_seed(seed)
    model = LipschitzNN(1, seed=seed if init_seed is None else init_seed).double()
    h = float(x[1] - x[0])
    kern = []
    for s in (SP, SQ):
        y, K, r = M.quadrature(x, s)
        kern.append((torch.tensor(K), torch.tensor(r)))
    Y = torch.tensor(y).reshape(-1, 1)
    Xt = torch.tensor(x).reshape(-1, 1)
    rng = np.random.default_rng(1000 + seed)
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    gn = 1.0
    it = 0
    while it < steps and gn > 1e-10:
        it += 1
        opt.zero_grad()
        if mode == "exact":
            fy, fx = model(Y), model(Xt)
            d = (kern[0][0] @ fy + kern[0][1] * fx) - (kern[1][0] @ fy + kern[1][1] * fx)
        else:  # Monte Carlo: the kernel drawn as arwmh.py:165-178 draws it
            means = []
            for s in (SP, SQ):
                X = x[:, None]
                yp = X + s * rng.standard_normal((len(x), n_samp))
                a = np.minimum(1.0, np.exp(np.minimum((X * X - yp * yp) / 2, 0.0)))
                z = np.where(rng.random((len(x), n_samp)) < a, yp, X)
                means.append(model(torch.tensor(z).reshape(len(x), n_samp, 1)).mean(-1))
            d = means[0] - means[1]
        loss = -((d[:-rad] - d[rad:]).abs() / (rad * h)).max()
        loss.backward()
        gn = 0.0
        for p in model.parameters():
            p.grad.clamp_(-1.0, 1.0)
            gn += float((p.grad ** 2).sum())
        opt.step()
    return model, it, gn


def analyse(model, x, rng, n_eval=10 ** 6, n_mc=20000):
    f = lambda t: model(torch.tensor(t).reshape(-1, 1)).detach().numpy()  # noqa: E731
    r, vP, vQ = M.exact_ratios(f, x, SP, SQ)
    v = np.maximum(vP + vQ, 0.0) / n_eval
    h = np.abs(np.diff(x))
    # the estimator: d_j + e_j per point, e_j ~ N(0, v_j) independent
    y, K, rr = M.quadrature(x, SP)
    dP = M.expectations(f(y), f(x), K, rr)[0]
    y, K, rr = M.quadrature(x, SQ)
    dQ = M.expectations(f(y), f(x), K, rr)[0]
    d = dP - dQ
    e = rng.standard_normal((n_mc, len(x))) * np.sqrt(v)[None]
    est = (np.abs(np.diff(d[None] + e, axis=1)) / h[None]).max(axis=1)
    t = np.linspace(-8, 8, 160001)
    ft = f(t)
    lip = float(np.max(np.abs(np.diff(ft)) / (t[1] - t[0])))
    return dict(rho_exact=float(r.max()), arg=float(x[int(r.argmax())]), est_mean=float(est.mean()),
                est_sd=float(est.std()), bias=float(est.mean() - r.max()), p_notebook=float((est >= NOTEBOOK).mean()),
                lip=lip, sd_ratio_max=float(M.mc_sd(vP, vQ, x, n_eval).max()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("n_keys", type=int, nargs="?", default=4)
    ap.add_argument("--modes", default="exact,mc")
    ap.add_argument("--seed0", type=int, default=0)
    ap.add_argument("--build-keys", action="store_true",
                    help="initialise from the networks the build's compute_kernel_distance_1d(PRNGKey(seed)) starts from")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    torch.set_num_threads(int(os.environ.get("CELL101_THREADS", max(1, min(8, os.cpu_count() or 1)))))
    lines = []

    def say(s):
        print(s, flush=True)
        lines.append(s)

    x = np.linspace(-5, 5, 100, dtype=np.float32).astype(np.float64)
    t0 = time.time()
    kr = M.kr_bound(x, SP, SQ)
    say(f"cell 101: P = N(0,1) RWM scale {SP}, Q scale {SQ}, x = linspace(-5, 5, 100)")
    say(f"1. KR supremum over all 1-Lipschitz f, adjacent pairs: max {kr.max():.6f} at x = {x[kr.argmax()]:.4f} "
        f"(min {kr.min():.4f}); ratio_rad 5 pairs: max {M.kr_bound(x, SP, SQ, rad=5).max():.6f}  [{time.time() - t0:.1f} s]")
    rng = np.random.default_rng(7)
    for mode in a.modes.split(","):
        res = []
        for seed in range(a.seed0, a.seed0 + a.n_keys):
            t1 = time.time()
            init = None
            if a.build_keys:
                init = _init_seed(split(PRNGKey(seed))[0])
            model, it, gn = train(seed, x, mode, init_seed=init)
            r = analyse(model, x, rng)
            res.append(r)
            say(f"2. [{mode:5s}] key {seed}: {it} steps, last clipped-grad norm {gn:.3g}; trained f: Lipschitz "
                f"{r['lip']:.4f}, rho exact {r['rho_exact']:.4f} at x = {r['arg']:.3f}; 3. notebook estimator "
                f"{r['est_mean']:.4f} +- {r['est_sd']:.4f} (bias {r['bias']:+.4f}, max ratio sd {r['sd_ratio_max']:.4f}), "
                f"P(>= {NOTEBOOK}) = {r['p_notebook']:.2g}  [{time.time() - t1:.0f} s]")
        ex = np.array([r["rho_exact"] for r in res])
        es = np.array([r["est_mean"] for r in res])
        say(f"   [{mode}] over {len(res)} keys: rho exact {ex.mean():.4f} (sd {ex.std(ddof=1) if len(ex) > 1 else 0:.4f}, "
            f"range {ex.min():.4f}..{ex.max():.4f}); notebook-style estimate {es.mean():.4f}; "
            f"notebook {NOTEBOOK} - mean estimate = {NOTEBOOK - es.mean():+.4f}")
    if a.out:
        with open(a.out, "w") as fh:
            fh.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
