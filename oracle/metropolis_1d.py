"""Exact transition kernel of the 1-D random-walk Metropolis step on N(0, 1),
and the Kantorovich-Rubinstein value of asumptions_check.ipynb cell 101.

TEST INFRASTRUCTURE ONLY: imported by tests/ and tools/, never by the product
package.

The kernel.  ARWMH.sample with a frozen adapt state (arwmh.py:162-178, the
sample_Pnx path arwmh.py:230-249) on the notebook's target
potential_fn = -Normal(0, 1).log_prob (asumptions_check.ipynb cell 4) with
scale L, log step size 0 and eps = 1e-6 moves x to y = x + s xi, s = L + eps
(arwmh.py:166-167), accepted with alpha = min(1, exp(x^2/2 - y^2/2))
(arwmh.py:173-174).  So

    P_s(x, dy) = q_s(x, y) alpha(x, y) dy + r_s(x) delta_x(dy),
    q_s(x, y) = N(y; x, s^2),  r_s(x) = 1 - int q_s alpha.

On |y| <= |x| alpha = 1; outside it q_s alpha is a Gaussian in y again:
q_s(x, y) e^{(x^2 - y^2)/2} = e^c / sqrt(1 + s^2) N(y; m, s'^2) with
m = x / (1 + s^2), s' = s / sqrt(1 + s^2), c = x^2 s^2 / (2 (1 + s^2)).
Everything below is closed form in the normal CDF (float64).

Cell 101.  compute_kernel_distance_1d (lipschitz.py:347-494) trains one
1-Lipschitz network f and reports max_i |(P - Q) f(x_{i+1}) - (P - Q) f(x_i)|
/ (x_{i+1} - x_i) over adjacent grid points (lipschitz.py:488-491).  For one
pair the supremum over all 1-Lipschitz f is, by Kantorovich-Rubinstein in 1-D,
int |F_mu(t)| dt with mu = P(x_{i+1}) - Q(x_{i+1}) - P(x_i) + Q(x_i) (a signed
measure of mass 0, F_mu its distribution function); sup over f of the max over
pairs is the max over pairs of those integrals (kr_bound).  `expectations`
gives (P f)(x) and (P f^2)(x) of any f by Gauss-Legendre quadrature on the
kernel's continuous part plus the atom, so a trained network's value can be
computed without Monte Carlo noise (exact_ratios) and the Monte Carlo spread
of the notebook's estimator with it (mc_sd).
"""
from __future__ import annotations

import numpy as np
from numpy.polynomial.legendre import leggauss
from scipy.special import ndtr

__all__ = ["cont_cdf", "cdf", "kr_pair", "kr_bound", "quadrature", "expectations", "exact_ratios", "mc_sd"]


def _tilt(x, s):
    k = 1.0 + s * s
    return x / k, s / np.sqrt(k), np.exp(x * x * s * s / (2.0 * k)) / np.sqrt(k)


def cont_cdf(x: float, s: float, t):
    """int_{-inf}^t q_s(x, y) alpha(x, y) dy (the accepted moves' mass below t)."""
    t = np.asarray(t, dtype=np.float64)
    a = abs(x)
    m, sp, w = _tilt(x, s)
    lo = w * ndtr((np.minimum(t, -a) - m) / sp)
    mid = ndtr((np.clip(t, -a, a) - x) / s) - ndtr((-a - x) / s)
    hi = np.where(t > a, w * (ndtr((t - m) / sp) - ndtr((a - m) / sp)), 0.0)
    return lo + mid + hi


def accept_mass(x: float, s: float) -> float:
    return float(cont_cdf(x, s, np.array([np.inf]))[0])


def cdf(x: float, s: float, t):
    """F of P_s(x, .): the continuous part plus the rejection atom at x."""
    t = np.asarray(t, dtype=np.float64)
    return cont_cdf(x, s, t) + (1.0 - accept_mass(x, s)) * (t >= x)


def _segments(bps, L, nseg, ng):
    gx, gw = leggauss(ng)
    ts, ws = [], []
    for a, b in zip(bps[:-1], bps[1:]):
        if b <= a:
            continue
        e = np.linspace(a, b, max(2, int(nseg * (b - a) / (2 * L)) + 1))
        lo, hi = e[:-1], e[1:]
        ts.append((0.5 * (hi - lo)[:, None] * gx + 0.5 * (hi + lo)[:, None]).ravel())
        ws.append((0.5 * (hi - lo)[:, None] * gw).ravel())
    return np.concatenate(ts), np.concatenate(ws)


def kr_pair(x0: float, x1: float, sP: float, sQ: float, L: float = 14.0, nseg: int = 4000, ng: int = 8) -> float:
    """int |F_mu| for mu = P(x1) - Q(x1) - P(x0) + Q(x0): the sup over 1-Lipschitz
    f of (P - Q) f(x1) - (P - Q) f(x0).  The integrand is smooth between the
    atoms x0, x1 and the acceptance kinks +-|x0|, +-|x1|, so those are segment
    ends of the Gauss-Legendre rule."""
    bps = sorted({-L, L, x0, x1, -abs(x0), abs(x0), -abs(x1), abs(x1)})
    t, w = _segments(bps, L, nseg, ng)
    F = cdf(x1, sP, t) - cdf(x1, sQ, t) - cdf(x0, sP, t) + cdf(x0, sQ, t)
    return float(np.sum(w * np.abs(F)))


def kr_bound(x, sP: float, sQ: float, rad: int = 1) -> np.ndarray:
    """Per-pair sup ratios int |F_mu| / |x_{i+rad} - x_i|; its max is the
    largest value compute_kernel_distance_1d can report without noise."""
    x = np.asarray(x, dtype=np.float64)
    return np.array([kr_pair(x[i], x[i + rad], sP, sQ) / abs(x[i + rad] - x[i]) for i in range(len(x) - rad)])


def quadrature(x, s: float, L: float = 12.0, nseg: int = 12000, ng: int = 4):
    """Nodes y [M] and weights K [n, M] with int g dP_s(x_i) ~= K[i] @ g(y) +
    r[i] g(x_i) (the atom r returned separately); node spacing 5e-4, well
    below the narrowest proposal scale of the notebook (0.1)."""
    x = np.asarray(x, dtype=np.float64)
    y, w = _segments([-L, L], L, nseg, ng)
    X = x[:, None]
    q = np.exp(-0.5 * ((y[None] - X) / s) ** 2) / (s * np.sqrt(2 * np.pi))
    a = np.minimum(1.0, np.exp(np.minimum((X * X - y[None] ** 2) / 2.0, 0.0)))
    K = q * a * w[None]
    r = np.array([1.0 - accept_mass(float(xi), s) for xi in x])
    return y, K, r


def expectations(fy: np.ndarray, fx: np.ndarray, K: np.ndarray, r: np.ndarray):
    """(P f)(x_i) and (P f^2)(x_i) from f at the nodes and at the grid points."""
    return K @ fy + r * fx, K @ (fy * fy) + r * fx * fx


def exact_ratios(f, x, sP: float, sQ: float):
    """Noise-free adjacent ratios |(P-Q)f(x_{i+1}) - (P-Q)f(x_i)| / h_i of a
    callable f (numpy in, numpy out) and the per-point variances of f under
    P and Q (for mc_sd)."""
    x = np.asarray(x, dtype=np.float64)
    out = []
    for s in (sP, sQ):
        y, K, r = quadrature(x, s)
        fy, fx = f(y), f(x)
        m1, m2 = expectations(fy, fx, K, r)
        out.append((m1, np.maximum(m2 - m1 * m1, 0.0)))  # (rounding can leave -1e-17)
    d = out[0][0] - out[1][0]
    h = np.abs(np.diff(x))
    return np.abs(np.diff(d)) / h, out[0][1], out[1][1]


def mc_sd(varP: np.ndarray, varQ: np.ndarray, x, n_per_point: int) -> np.ndarray:
    """Standard deviation of each adjacent ratio of the notebook's estimator
    (independent draws per point for P and Q, n_per_point each;
    lipschitz.py:407-420, 484-491)."""
    v = (varP + varQ) / n_per_point
    return np.sqrt(v[1:] + v[:-1]) / np.abs(np.diff(np.asarray(x, dtype=np.float64)))
