"""Pin the C oracle (bit spec, oracle/amh_oracle.c) against the literal
float64 restatement of the reference (oracle/arwmh_np.py) and against known
answers.  The reference itself (JAX/NumPyro) is not importable here, so these
are the anchors: the Krause-Igel rank-one update vs np.linalg.cholesky, the
gamma_1 = 1 keep-L quirk, NaN -> reject, the analytic stationary acceptance
of the frozen 1-D kernel, adaptation to the target acceptance, and the
eight-schools posterior summary printed in the reference notebook."""
import math

import numpy as np
import pytest

import arwmh_np as lit
from helpers import make_case

# fp32 potentials of magnitude |U| carry ~|U| * 2^-23 absolute error into alpha,
# hence into lambda and mean_accept_prob.
TOL = dict(z=(1e-5, 1e-5), mu=(1e-5, 1e-5), pe=(2e-5, 1e-3), lam=(0, 3e-5), macc=(0, 3e-5))


def lit_potential(kind, om):
    d = om.d
    if kind == "diamonds_ss":  # same posterior: the literal model reads the direct data
        import posteriors as P
        arr, (N, K) = P.diamonds.pack_fn(P.synthetic_diamonds(N=500))
        arr = arr.astype(np.float64)
        return lambda z: lit.diamonds_potential(z, arr[:N * (K - 1)].reshape(N, K - 1), arr[N * (K - 1):])
    # (the diamonds_ss buffer holds float64 statistics as float32 word pairs,
    # so it is never cast; the other models' data are plain float32)
    data = np.asarray(om.data, np.float64)
    if kind == "gaussian":
        m, P, c0 = data[:d], data[d:d + d * d].reshape(d, d), data[d + d * d]
        return lambda z: lit.gaussian_potential(z, m, P, c0)
    if kind == "eight_schools":
        J = d - 2
        return lambda z: lit.eight_schools_potential(z, data[:J], data[J:2 * J])
    if kind == "kidiq":
        N = om.n_data
        return lambda z: lit.kidiq_potential(z, data[:N], data[N:2 * N], data[2 * N:3 * N])
    if kind == "diamonds":
        N, Kc = om.n_data, om.k_data - 1
        return lambda z: lit.diamonds_potential(z, data[:N * Kc].reshape(N, Kc), data[N * Kc:])
    if kind == "mixture":  # the notebook's weights / locs / scales (helpers.make_case)
        return lambda z: lit.mixture_potential(z, [0.5, 0.5], [-1.0, 1.0], [0.1, 0.1])
    raise ValueError(kind)


def unpack(Lp, d):
    L = np.zeros((d, d), np.float64)
    k = 0
    for j in range(d):
        for r in range(j, d):
            L[r, j] = Lp[k]
            k += 1
    return L


# ---------------------------------------------------------------- cholupdate --
@pytest.mark.parametrize("d", [1, 2, 5, 26, 64])
def test_cholupdate_matches_cholesky(d):
    rng = np.random.default_rng(d)
    A = rng.normal(size=(d, d))
    S = A @ A.T + d * np.eye(d)
    L = np.linalg.cholesky(S)
    for gamma in (0.5, 0.01, 1e-4):
        x = rng.normal(size=d)
        out = lit.cholesky_update(np.sqrt(1 - gamma) * L, x, gamma)
        ref = np.linalg.cholesky((1 - gamma) * S + gamma * np.outer(x, x))
        assert np.max(np.abs(out - ref)) < 1e-10 * np.max(np.abs(ref))


def test_gamma_one_keeps_factor():
    """arwmh.py:183-191: gamma_1 = 1 -> sqrt(1-gamma) L = 0 -> NaN -> keep L;
    mu jumps to z_new."""
    d = 4
    L = np.eye(d) * 0.7
    state = lit.ARWMHState(0, np.ones(d), 1.0, 0.0, lit.ARWMHAdaptState(np.zeros(d), L, 0.0), 0.0, None)
    new, acc, a = lit.sample(state, lambda z: 0.5 * z @ z, np.full(d, 0.1), 0.5)
    assert np.array_equal(new.adapt_state.scale, L)
    np.testing.assert_allclose(new.adapt_state.loc, new.z)


def test_nan_potential_rejects():
    d = 3
    state = lit.ARWMHState(5, np.zeros(d), 1.0, 0.2, lit.ARWMHAdaptState(np.zeros(d), np.eye(d), 0.0), 0.0, None)
    new, acc, a = lit.sample(state, lambda z: np.nan, np.ones(d), 0.0)
    assert not acc and a == 0.0 and np.array_equal(new.z, state.z)


# ------------------------------------------------- C oracle vs literal numpy --
@pytest.mark.parametrize("kind,dim", [("gaussian", 12), ("eight_schools", None), ("kidiq", None),
                                      ("diamonds", None), ("diamonds_ss", None), ("gaussian", 128),
                                      ("gaussian", 256), ("mixture", 1), ("mixture", 3),
                                      # large d off the 32-multiples: a ragged MFMA tile,
                                      # dword-DMA column blocks, an odd d
                                      ("gaussian", 72), ("gaussian", 100), ("gaussian", 97)])
@pytest.mark.parametrize("pre_steps", [0, 1, 37])
def test_oracle_step_matches_literal(kind, dim, pre_steps, orc):
    """One teacher-forced transition (identical noise) of the C oracle against
    the literal float64 restatement; d = 128 / 256 exercise the large-d bit
    spec (wave-per-chain passes, MFMA-order potential)."""
    from kernels_amd import PRNGKey
    _, _, om = make_case(kind, dim)
    d, C, W = om.d, (48 if om.d <= 64 else 12), 20
    st = orc.init(om, PRNGKey(3), C)
    if pre_steps:
        orc.step(om, st, pre_steps, num_warmup=W)
    before = st.copy()
    orc.step(om, st, 1, num_warmup=W)
    U = lit_potential(kind, om)
    bits, ubits = lit.step_noise(before.rng_key, before.i, d)
    checked = 0
    for c in range(C):
        xi = lit.normal_from_bits(bits[c])
        u = float(lit.unif01_from_bits(ubits[c]))
        L0 = unpack(before.scale[c], d)
        s0 = lit.ARWMHState(int(before.i[c]), before.z[c].astype(np.float64), float(before.potential_energy[c]),
                            float(before.mean_accept_prob[c]),
                            lit.ARWMHAdaptState(before.loc[c].astype(np.float64), L0, float(before.log_step_size[c])),
                            0.0, None)
        new, acc, alpha = lit.sample(s0, U, xi, u, num_warmup=W)
        if abs(u - alpha) < 1e-4:
            continue  # decision within rounding of the threshold
        checked += 1
        ctx = f"{kind} chain {c}"
        np.testing.assert_allclose(st.z[c], new.z, rtol=TOL["z"][0], atol=TOL["z"][1], err_msg=ctx)
        np.testing.assert_allclose(st.potential_energy[c], new.potential_energy, rtol=TOL["pe"][0],
                                   atol=TOL["pe"][1], err_msg=ctx)
        np.testing.assert_allclose(st.loc[c], new.adapt_state.loc, rtol=TOL["mu"][0], atol=TOL["mu"][1], err_msg=ctx)
        np.testing.assert_allclose(st.log_step_size[c], new.adapt_state.log_step_size, atol=TOL["lam"][1], err_msg=ctx)
        np.testing.assert_allclose(st.mean_accept_prob[c], new.mean_accept_prob, atol=TOL["macc"][1], err_msg=ctx)
        L1 = unpack(st.scale[c], d)
        S1, Sr = L1 @ L1.T, new.adapt_state.scale @ new.adapt_state.scale.T
        assert np.max(np.abs(S1 - Sr)) <= 1e-4 * np.max(np.abs(Sr)) + 1e-6, ctx
        assert abs(st.as_change[c] - new.as_change) <= 1e-3 * abs(new.as_change) + 1e-5, ctx
        assert st.i[c] == new.i
    assert checked >= C - 2


# ------------------------------------------------------------ known answers --
def test_frozen_kernel_stationary_acceptance(orc):
    """1-D N(0,1) target, frozen L = 1, lambda = 0 (asumptions_check.ipynb):
    stationary acceptance of RWM with proposal sd s is (2/pi) atan(2/s)."""
    import posteriors as P
    from kernels_amd import PRNGKey
    g = P.gaussian(np.zeros(1), cov=np.eye(1))
    data, _ = g.pack("cpu")
    om = orc.Model(orc.GAUSSIAN, 1, data.numpy())
    x = np.random.default_rng(0).normal(size=(2000, 1)).astype(np.float32)
    out = orc.sample_pnx(om, PRNGKey(1), x, np.zeros(1), np.ones(1), 0.0, 1, 500)
    acc = np.mean(out[:, :, 0] != x[:, None, 0])
    s = 1.0 + 1e-6
    assert abs(acc - (2 / math.pi) * math.atan(2 / s)) < 0.005


def test_adaptation_reaches_target(orc):
    from kernels_amd import PRNGKey
    _, _, om = make_case("gaussian", 8)
    st = orc.init(om, PRNGKey(0), 64)
    acc = np.zeros(64, np.int32)
    orc.step(om, st, 3000, accept_count=acc)
    assert abs(st.mean_accept_prob.mean() - 0.234) < 0.02
    L = np.stack([unpack(s, 8) for s in st.scale])
    import posteriors as P
    cov = np.linalg.inv(P.correlated_gaussian(8).precision)
    est = np.mean(L @ np.transpose(L, (0, 2, 1)), axis=0)
    # the adapted factor tracks the target covariance (Haario et al. AM):
    # ~0.2 relative error after 3,000 steps, ~0.04 after 30,000
    assert np.linalg.norm(est - cov) / np.linalg.norm(cov) < 0.35


def test_eight_schools_posterior(orc):
    """posteriordb_eight-schools.ipynb:858-867 (NumPyro summary of the
    reference ARWMH run): mu 4.40 (sd 3.29), tau 3.63 (sd 3.21),
    theta_base[0] 0.32 (sd 0.99)."""
    from kernels_amd import PRNGKey
    _, _, om = make_case("eight_schools")
    C = 128
    st = orc.init(om, PRNGKey(11), C)
    orc.step(om, st, 5000)
    cz = orc.step(om, st, 4000, collect_z=True)[::10]  # thin 10
    mu, tau, tb0 = cz[:, :, 0].ravel(), np.exp(cz[:, :, 1]).ravel(), cz[:, :, 2].ravel()
    assert abs(mu.mean() - 4.40) < 0.35 and abs(mu.std() - 3.29) < 0.35
    assert abs(tau.mean() - 3.63) < 0.4 and abs(tau.std() - 3.21) < 0.6
    assert abs(tb0.mean() - 0.32) < 0.1 and abs(tb0.std() - 0.99) < 0.1


@pytest.mark.parametrize("N,K,seed", [(500, 25, 26), (5000, 25, 26), (77, 10, 5)])
def test_diamonds_suffstat_potential(N, K, seed, orc):
    """The sufficient-statistics potential against the literal float64 model
    and against the direct float32 contraction, near the posterior mode and
    far from it.  Tolerance: |dU| <= 2e-6 |U| + 1e-3 (the direct float32 sum of
    N squared residuals carries ~N * 2^-24 relative error; the float64 form is
    the more accurate of the two)."""
    import posteriors as P
    mk = P.synthetic_diamonds(N=N, K=K, seed=seed)
    arr, _ = P.diamonds.pack_fn(mk)
    ss, _ = P.diamonds_suffstat.pack_fn(mk)
    om_d = orc.Model(orc.DIAMONDS, K + 1, arr, n_data=N, k_data=K)
    om_s = orc.Model(orc.DIAMONDS_SS, K + 1, ss, n_data=N, k_data=K)
    rng = np.random.default_rng(0)
    Kc = K - 1
    X = np.asarray(mk["X"], np.float64)
    Y = np.asarray(mk["Y"], np.float64)
    b_ls = np.linalg.lstsq(X, Y, rcond=None)[0]
    mode = np.concatenate([[b_ls[0] + (X[:, 1:].mean(0) @ b_ls[1:])], b_ls[1:], [np.log(0.123)]])
    z = np.concatenate([mode + 1e-3 * rng.normal(size=(200, K + 1)),
                        rng.normal(size=(200, K + 1))]).astype(np.float32)
    u_s = orc.potential(om_s, z).astype(np.float64)
    u_d = orc.potential(om_d, z).astype(np.float64)
    Xc = arr[:N * Kc].reshape(N, Kc).astype(np.float64)
    u_l = np.array([lit.diamonds_potential(zz.astype(np.float64), Xc, arr[N * Kc:].astype(np.float64)) for zz in z])
    tol = 2e-6 * np.abs(u_l) + 1e-3
    assert np.all(np.abs(u_s - u_l) <= tol), np.max(np.abs(u_s - u_l) / tol)
    assert np.all(np.abs(u_d - u_l) <= 10 * tol), np.max(np.abs(u_d - u_l) / tol)


def test_diamonds_suffstat_same_chain_statistics(orc):
    """Both diamonds forms driven by the same keys for 500 transitions (C oracle,
    256 chains, N = 5000).  The rounding differences make the trajectories part
    bitwise within tens of steps (MCMC is chaotic in the last bits), but the
    chains sample the same posterior: mean acceptance agrees to 2e-3 (measured
    4e-5)."""
    import posteriors as P
    from kernels_amd import PRNGKey
    mk = P.synthetic_diamonds()
    a, (N, K) = P.diamonds.pack_fn(mk)
    s, _ = P.diamonds_suffstat.pack_fn(mk)
    md = orc.Model(orc.DIAMONDS, K + 1, a, n_data=N, k_data=K)
    ms = orc.Model(orc.DIAMONDS_SS, K + 1, s, n_data=N, k_data=K)
    sd, ss = orc.init(md, PRNGKey(7), 256), orc.init(ms, PRNGKey(7), 256)
    np.testing.assert_allclose(ss.potential_energy, sd.potential_energy, rtol=2e-6)
    orc.step(md, sd, 500)
    orc.step(ms, ss, 500)
    assert abs(float(sd.mean_accept_prob.mean()) - float(ss.mean_accept_prob.mean())) < 2e-3
