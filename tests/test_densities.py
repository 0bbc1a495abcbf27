"""The literal restatement's log-densities (oracle/arwmh_np.py:150-201) against
scipy.stats, which stands in for the NumPyro distributions the reference's
models use (run_eight_schools_lr_decay.py:26-35, run_kidiq_kidscore_lr_decay.py:29-41,
run_diamonds_lr_decay.py:24-40, the Gaussian raw potential of
asumptions_check.ipynb:81-83).  NumPyro itself is not importable here
(SURVEY.md §8c); scipy's densities are an independent implementation of the
same published formulas.

Also pinned: the log-transform Jacobian of the positive sites (+u in the
potential, numpyro's biject_to(positive) = exp): the unconstrained density
of a HalfCauchy / folded StudentT scale integrates to one over u."""
import math

import numpy as np
import pytest
from scipy import integrate, stats

import arwmh_np as lit


def test_normal_lp():
    x = np.linspace(-30, 30, 241)
    for loc, scale in [(0.0, 1.0), (0.0, 5.0), (3.5, 0.123), (-2.0, 18.0)]:
        np.testing.assert_allclose(lit.normal_lp(x, loc, scale), stats.norm.logpdf(x, loc, scale), rtol=1e-12,
                                   atol=1e-12)


def test_halfcauchy_lp():
    x = np.geomspace(1e-6, 1e6, 200)
    for scale in (2.5, 5.0):
        np.testing.assert_allclose(lit.halfcauchy_lp(x, scale), stats.halfcauchy.logpdf(x, scale=scale),
                                   rtol=1e-12, atol=1e-12)


def test_studentt_lp():
    x = np.linspace(-200, 200, 401)
    for df, loc, scale in [(3.0, 8.0, 10.0), (3.0, 0.0, 10.0), (1.5, -1.0, 0.5)]:
        np.testing.assert_allclose(lit.studentt_lp(x, df, loc, scale), stats.t.logpdf(x, df, loc, scale),
                                   rtol=1e-12, atol=1e-12)


def test_folded_studentt_is_log2_plus_base():
    """numpyro FoldedDistribution(StudentT(3, 0, 10)) (run_diamonds_lr_decay.py:33):
    log(p(x) + p(-x)) for x >= 0, = log 2 + log p(x) for a symmetric base."""
    x = np.geomspace(1e-4, 1e4, 200)
    folded = np.log(stats.t.pdf(x, 3, 0, 10) + stats.t.pdf(-x, 3, 0, 10))
    np.testing.assert_allclose(math.log(2.0) + lit.studentt_lp(x, 3.0, 0.0, 10.0), folded, rtol=1e-12, atol=1e-12)


@pytest.mark.parametrize("lp", [lambda s: lit.halfcauchy_lp(s, 5.0), lambda s: lit.halfcauchy_lp(s, 2.5),
                                lambda s: math.log(2.0) + lit.studentt_lp(s, 3.0, 0.0, 10.0)])
def test_log_jacobian_normalises(lp):
    """p_u(u) = p(e^u) e^u: the '+ log sigma' / '+ log tau' term of the potentials."""
    val, err = integrate.quad(lambda u: math.exp(lp(math.exp(u)) + u), -60, 60, limit=400)
    assert abs(val - 1.0) < 1e-6


def _eight_schools_scipy(z, y, sigma):
    mu, lt, tb = z[0], z[1], z[2:]
    tau = math.exp(lt)
    lp = (stats.norm.logpdf(mu, 0, 5) + stats.halfcauchy.logpdf(tau, scale=5) + lt
          + stats.norm.logpdf(tb, 0, 1).sum() + stats.norm.logpdf(y, mu + tau * tb, sigma).sum())
    return -lp


def _kidiq_scipy(z, ks, hs, iq):
    b, ls = z[:3], z[3]
    s = math.exp(ls)
    mu = b[0] + b[1] * hs + b[2] * iq
    return -(stats.halfcauchy.logpdf(s, scale=2.5) + ls + stats.norm.logpdf(ks, mu, s).sum())


def _diamonds_scipy(z, Xc, Y):
    K = Xc.shape[1]
    a, b, ls = z[0], z[1:1 + K], z[1 + K]
    s = math.exp(ls)
    folded = math.log(stats.t.pdf(s, 3, 0, 10) + stats.t.pdf(-s, 3, 0, 10))
    return -(stats.norm.logpdf(b, 0, 1).sum() + stats.t.logpdf(a, 3, 8, 10) + folded + ls
             + stats.norm.logpdf(Y, a + Xc @ b, s).sum())


def test_model_potentials_against_scipy():
    import posteriors as P
    rng = np.random.default_rng(5)
    es = P.EIGHT_SCHOOLS_DATA
    y, sg = es["y"].astype(np.float64), es["sigma"].astype(np.float64)
    kd = P.synthetic_kidiq()
    ks, hs, iq = (np.asarray(kd[k], np.float64) for k in ("kid_score", "mom_hs", "mom_iq"))
    dm = P.synthetic_diamonds(N=300)
    arr, (N, K) = P.diamonds.pack_fn(dm)
    arr = arr.astype(np.float64)
    Xc, Y = arr[:N * (K - 1)].reshape(N, K - 1), arr[N * (K - 1):N * (K - 1) + N]
    for _ in range(20):
        z = rng.uniform(-2, 2, size=10)
        assert lit.eight_schools_potential(z, y, sg) == pytest.approx(_eight_schools_scipy(z, y, sg), rel=1e-12)
        z = np.concatenate([rng.normal(size=3) * [20, 5, 0.5], rng.uniform(-1, 3, size=1)])
        assert lit.kidiq_potential(z, ks, hs, iq) == pytest.approx(_kidiq_scipy(z, ks, hs, iq), rel=1e-12)
        z = np.concatenate([[7.8 + rng.normal()], rng.normal(size=K - 1), [rng.uniform(-3, 1)]])
        assert lit.diamonds_potential(z, Xc, Y) == pytest.approx(_diamonds_scipy(z, Xc, Y), rel=1e-11)


def test_gaussian_potential_against_scipy():
    """U(x) = 1/2 (x-m)^T P (x-m) + c0 with c0 = 1/2 log|2 pi Sigma| is -log N(x; m, Sigma)."""
    import posteriors as P
    for d in (8, 64):
        g = P.correlated_gaussian(d)
        data, _ = g.pack("cpu")
        data = data.numpy().astype(np.float64)
        m, Pm, c0 = data[:d], data[d:d + d * d].reshape(d, d), data[d + d * d]
        cov = np.linalg.inv(Pm)
        cov = 0.5 * (cov + cov.T)
        x = np.random.default_rng(d).normal(size=(10, d))
        want = -stats.multivariate_normal(m, cov).logpdf(x)
        got = np.array([lit.gaussian_potential(xx, m, Pm, c0) for xx in x])
        # data are the float32-rounded precision and constant: compare at float32 resolution
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-4)


def test_mixture_potential_against_scipy():
    """asumptions_check.ipynb cell 61: -log(1/2 N(x; -1, .1) + 1/2 N(x; 1, .1)),
    summed over coordinates; the literal restatement, the host evaluation of
    posteriors.Mixture and the C oracle against scipy's densities."""
    import orc
    import posteriors as P
    mx = P.notebook_mixture()
    x = np.linspace(-3.0, 3.0, 601)
    ref = -np.log(0.5 * stats.norm.pdf(x, -1.0, 0.1) + 0.5 * stats.norm.pdf(x, 1.0, 0.1))
    lit_u = np.array([lit.mixture_potential(v, [0.5, 0.5], [-1.0, 1.0], [0.1, 0.1]) for v in x])
    np.testing.assert_allclose(lit_u, ref, rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(mx(x[:, None]), ref, rtol=1e-12, atol=1e-12)
    data, ip = mx.pack("cpu")
    om = orc.Model(orc.MIXTURE, 1, data.numpy(), n_data=ip[0])
    u32 = orc.potential(om, x.astype(np.float32)[:, None])
    np.testing.assert_allclose(u32, ref, rtol=2e-6, atol=2e-5)
    # far tails: log-sum-exp keeps the potential finite (no underflow to +inf)
    far = orc.potential(om, np.array([[-30.0], [30.0]], np.float32))
    np.testing.assert_allclose(far, [-(np.log(0.5) + stats.norm.logpdf(-30.0, -1, .1)),
                                     -(np.log(0.5) + stats.norm.logpdf(30.0, 1, .1))], rtol=1e-6)
    # several coordinates and three components
    m3 = P.mixture([0.2, 0.3, 0.5], [-2.0, 0.0, 1.5], [0.5, 1.0, 0.25], dim=5)
    d3, ip3 = m3.pack("cpu")
    om3 = orc.Model(orc.MIXTURE, 5, d3.numpy(), n_data=ip3[0])
    z = np.random.default_rng(0).normal(size=(200, 5))
    ref3 = -np.log(sum(w * stats.norm.pdf(z, m, s) for w, m, s in [(0.2, -2, .5), (0.3, 0, 1), (0.5, 1.5, .25)])).sum(1)
    np.testing.assert_allclose(orc.potential(om3, z.astype(np.float32)), ref3, rtol=3e-6, atol=3e-5)
    with pytest.raises(ValueError):
        P.mixture([0.5, 0.6], [0, 1], [1, 1])
