"""oracle/metropolis_1d.py: the exact 1-D Metropolis kernel on N(0, 1) that
pins asumptions_check.ipynb cell 101 (tests/test_lipschitz.py) -- checked
here against independent computations: the kernel's closed-form stationary
acceptance rate, brute-force integration of the accepted-move density, Monte
Carlo draws of the kernel as arwmh.py:162-178 draws it, and a dense-grid
integral of |F_mu| for the Kantorovich-Rubinstein value."""
import math

import numpy as np
import pytest
from scipy.special import ndtr

from oracle import metropolis_1d as M

SP, SQ = 1.0 + 1e-6, 0.1 + 1e-6  # cell 101: L e^lam + eps (arwmh.py:166)


def _draw(x, s, n, rng):
    """The kernel drawn literally: y = x + s xi, accepted with
    min(1, exp(x^2/2 - y^2/2)) (arwmh.py:165-178 on -log N(0, 1))."""
    y = x + s * rng.standard_normal(n)
    a = np.minimum(1.0, np.exp(np.minimum((x * x - y * y) / 2.0, 0.0)))
    return np.where(rng.random(n) < a, y, x)


@pytest.mark.parametrize("s", [0.1, 0.5, 1.0, 2.4])
def test_stationary_acceptance_closed_form(s):
    """Under pi = N(0, 1) the RWM acceptance rate is (2 / pi) atan(2 / s)."""
    t = np.linspace(-12, 12, 48001)
    acc = np.array([M.accept_mass(float(x), s) for x in t])
    rate = np.trapezoid(acc * np.exp(-t * t / 2) / math.sqrt(2 * math.pi), t)
    assert rate == pytest.approx(2 / math.pi * math.atan(2 / s), abs=1e-7)


@pytest.mark.parametrize("x", [-3.1, -0.4, 0.0, 0.7, 2.5])
@pytest.mark.parametrize("s", [0.1, 1.0])
def test_cont_cdf_matches_brute_force_integral(x, s):
    """The piecewise tilted-Gaussian CDF equals a dense trapezoid integral of
    q_s(x, y) alpha(x, y), kinks at +-|x| included."""
    y = np.linspace(x - 12 * s, x + 12 * s, 400001)
    dens = np.exp(-0.5 * ((y - x) / s) ** 2) / (s * math.sqrt(2 * math.pi))
    dens *= np.minimum(1.0, np.exp((x * x - y * y) / 2.0))
    cum = np.concatenate([[0.0], np.cumsum(0.5 * (dens[1:] + dens[:-1]) * np.diff(y))])
    for t in (x - s, -abs(x), x, abs(x), x + 0.5 * s, x + 3 * s):
        want = np.interp(t, y, cum)
        assert float(M.cont_cdf(x, s, np.array([t]))[0]) == pytest.approx(want, abs=2e-8)
    # no acceptance test ever fails for |y| <= |x|: the mass of that interval is q's
    if x != 0.0:
        a = abs(x)
        inner = float(M.cont_cdf(x, s, np.array([a]))[0] - M.cont_cdf(x, s, np.array([-a]))[0])
        assert inner == pytest.approx(ndtr((a - x) / s) - ndtr((-a - x) / s), abs=1e-14)


def test_cdf_is_a_distribution_with_the_rejection_atom():
    for x, s in ((0.3, 1.0), (-2.0, 0.1), (4.0, 1.0)):
        t = np.linspace(-15, 15, 20001)
        F = M.cdf(x, s, t)
        assert F[0] == pytest.approx(0.0, abs=1e-12) and F[-1] == pytest.approx(1.0, abs=1e-12)
        assert np.all(np.diff(F) >= -1e-15)
        jump = float(M.cdf(x, s, np.array([x]))[0] - M.cdf(x, s, np.array([np.nextafter(x, -np.inf)]))[0])
        assert jump == pytest.approx(1.0 - M.accept_mass(x, s), abs=1e-12)


def test_expectations_match_the_kernel_drawn_literally():
    """(P f)(x) by quadrature + atom vs 4e6 literal draws, for a 1-Lipschitz
    f with a kink; the Monte Carlo error bound is 5 standard errors."""
    rng = np.random.default_rng(11)
    x = np.array([-4.0, -1.3, 0.0, 0.9, 3.2])
    f = lambda t: np.abs(t - 0.25) - 0.5 * np.tanh(t)  # noqa: E731
    for s in (SP, SQ):
        y, K, r = M.quadrature(x, s)
        assert np.allclose(K.sum(axis=1) + r, 1.0, atol=1e-10)  # f = 1: total mass
        m1, m2 = M.expectations(f(y), f(x), K, r)
        for i, xi in enumerate(x):
            z = f(_draw(xi, s, 4_000_000, rng))
            se = z.std() / math.sqrt(z.size)
            assert abs(z.mean() - m1[i]) < 5 * se + 1e-9, (s, xi, z.mean(), m1[i], se)
            assert m2[i] - m1[i] ** 2 == pytest.approx(z.var(), rel=2e-2, abs=1e-6)


def test_kr_pair_matches_dense_grid_integral():
    """int |F_mu| for one adjacent pair of the cell-101 grid (its maximiser)
    against a plain trapezoid on a 2e6-point grid."""
    x = np.linspace(-5, 5, 100, dtype=np.float32).astype(np.float64)
    i = int(np.argmin(np.abs(x - 1.2626)))
    x0, x1 = x[i], x[i + 1]
    t = np.linspace(-14, 14, 2_000_001)
    F = M.cdf(x1, SP, t) - M.cdf(x1, SQ, t) - M.cdf(x0, SP, t) + M.cdf(x0, SQ, t)
    dense = np.trapezoid(np.abs(F), t)
    assert M.kr_pair(x0, x1, SP, SQ) == pytest.approx(dense, rel=2e-5)


def test_cell101_supremum():
    """The largest value cell 101's estimator can approach without noise --
    the supremum over ALL 1-Lipschitz f, adjacent pairs of linspace(-5, 5,
    100) -- is 0.9591 at x = 1.263 (profiles/r5_cell101_exact.txt): the
    notebook's 0.544187 is reachable, and it is a property of the trained
    network, not of rho(P, Q) alone."""
    x = np.linspace(-5, 5, 100, dtype=np.float32).astype(np.float64)
    kr = M.kr_bound(x, SP, SQ)
    assert kr.max() == pytest.approx(0.959093, abs=2e-6)
    assert x[int(kr.argmax())] == pytest.approx(1.2626, abs=1e-3)
    assert kr.min() > 0.82
    assert 0.544187 < kr.max()


def test_exact_ratios_of_a_linear_f():
    """For f(t) = t the ratios are exact first moments: (P - Q) f(x) is
    E_P[y] - E_Q[y] from the closed-form tilted Gaussians."""
    x = np.linspace(-2, 2, 9)
    r, vP, vQ = M.exact_ratios(lambda t: t, x, SP, SQ)

    def mean(xv, s):
        k = 1 + s * s
        m, sp = xv / k, s / math.sqrt(k)
        w = math.exp(xv * xv * s * s / (2 * k)) / math.sqrt(k)
        a = abs(xv)
        # accepted part: int y q alpha over (-inf, -a), [-a, a], (a, inf)
        phi = lambda u: math.exp(-u * u / 2) / math.sqrt(2 * math.pi)  # noqa: E731
        lo = w * (m * ndtr((-a - m) / sp) - sp * phi((-a - m) / sp))
        mid = xv * (ndtr((a - xv) / s) - ndtr((-a - xv) / s)) - s * (phi((a - xv) / s) - phi((-a - xv) / s))
        hi = w * (m * (1 - ndtr((a - m) / sp)) + sp * phi((a - m) / sp))
        return lo + mid + hi + (1 - M.accept_mass(xv, s)) * xv

    d = np.array([mean(v, SP) - mean(v, SQ) for v in x])
    want = np.abs(np.diff(d)) / np.diff(x)
    assert np.allclose(r, want, atol=2e-9)
    assert np.all(vP >= 0) and np.all(vQ >= 0)


def test_mc_sd_formula():
    """The estimator's per-ratio spread: independent P and Q means at each
    point, n draws each."""
    x = np.array([0.0, 0.5, 1.5])
    vP, vQ = np.array([1.0, 2.0, 3.0]), np.array([0.5, 0.5, 0.5])
    sd = M.mc_sd(vP, vQ, x, 100)
    want = np.sqrt(((vP + vQ) / 100)[1:] + ((vP + vQ) / 100)[:-1]) / np.diff(x)
    assert np.allclose(sd, want)


def test_cell101_training_restatement_runs():
    """tools/cell101_exact.py: a few steps of the float64 restatement of the
    reference's training (lipschitz.py:396-491) on the exact objective and on
    Monte Carlo draws; the trained f stays 1-Lipschitz and its exact ratios
    stay below the pairs' Kantorovich-Rubinstein suprema."""
    import os
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import cell101_exact as T
    x = np.linspace(-5, 5, 100, dtype=np.float32).astype(np.float64)
    kr = M.kr_bound(x, SP, SQ)
    for mode in ("exact", "mc"):
        model, it, gn = T.train(0, x, mode, steps=3, n_samp=200)
        assert it == 3 and np.isfinite(gn)
        r = T.analyse(model, x, np.random.default_rng(0), n_mc=200)
        assert r["lip"] <= 1.0 + 1e-6
        assert 0.0 < r["rho_exact"] <= kr.max()
