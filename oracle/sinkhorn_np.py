"""TEST INFRASTRUCTURE ONLY (never imported by the product path).

Float64 restatement of the log-domain Sinkhorn iteration behind the
reference's wasserstein_sinkhorn (python/utils/evaluation.py:69-101), which
calls ott-jax (PointCloud(x, y, cost_fn=costs.Euclidean(), epsilon),
linear.solve, .ent_reg_cost).  ott-jax is not vendored under /root/reference,
is unpinned in python/environment.yml, and is not importable here: this is
the published algorithm with ott's defaults (epsilon = 0.05 x std of the cost
matrix when None, threshold 1e-3 on the marginal error checked every 10
iterations, at most 2,000 iterations, ent_reg_cost = <a, f> + <b, g> +
eps (1 - mass)).  Parity against ott itself is unpinned.

It mirrors the iteration order of utils_amd.evaluation.sinkhorn exactly, so
the GPU result can be compared at a fixed iteration count.
"""
import numpy as np
from scipy.special import logsumexp


def cost_matrix(x, y, cost_fn="euclidean"):
    x = np.asarray(x, np.float64)
    y = np.asarray(y, np.float64)
    d2 = ((x[:, None, :] - y[None, :, :]) ** 2).sum(-1)
    return np.sqrt(d2) if cost_fn == "euclidean" else d2


def sinkhorn(x, y, cost_fn="euclidean", epsilon=None, threshold=1e-3, max_iterations=2000, inner_iterations=10,
             relative_epsilon="std"):
    C = cost_matrix(x, y, cost_fn)
    if epsilon is None:
        epsilon = 0.05 * (C.std() if relative_epsilon == "std" else C.mean())
    eps = float(epsilon)
    n, m = C.shape
    la, lb = -np.log(n), -np.log(m)
    f, g = np.zeros(n), np.zeros(m)
    err, it, converged = np.inf, 0, False
    while it < max_iterations:
        f = -eps * logsumexp((g[None, :] - C) / eps + lb, axis=1)
        h = -eps * logsumexp((f[:, None] - C) / eps + la, axis=0)
        it += 1
        if it % inner_iterations == 0 or it == max_iterations:
            err = float(np.abs(np.exp((g - h) / eps) - 1.0).sum() / m)
            if err < threshold:
                converged = True
                g = h
                break
        g = h
    return dict(cost=float(f.mean() + g.mean()), f=f, g=g, epsilon=eps, iterations=it, error=err,
                converged=converged)


def transport_plan(C, f, g, eps):
    n, m = C.shape
    return np.exp((f[:, None] + g[None, :] - C) / eps) / (n * m)
