"""ARWMH.sample_Pnx (arwmh.py:230-270) for 64 < d <= 256, dense Gaussian:
the C oracle's large-d mirror (orc_sample_pnx -> orc_sample_pnx_big, the bit
spec of big_pnx_kernel) pinned to the float64 literal restatement with the
same draws (oracle/arwmh_np.py: split keys, step words W_j), plus a known
answer (a frozen kernel with the target's own factor keeps the target).

Tolerance of the one-step comparison (float32 oracle vs float64 literal):
z' rtol 1e-5 / atol 1e-5; a chain whose accept test is within 1e-4 of the
uniform (a decision float32 rounding can flip) is skipped, at most 2 %."""
import math

import numpy as np
import pytest

import arwmh_np as lit


def _case(d, seed=0):
    import orc
    import posteriors as P
    g = P.correlated_gaussian(d)
    data, _ = g.pack("cpu")
    om = orc.Model(orc.GAUSSIAN, d, data.numpy())
    Sigma = np.linalg.inv(np.asarray(g.precision, np.float64))
    return g, om, Sigma


def _packed(L):
    d = L.shape[0]
    return np.concatenate([L[j:, j] for j in range(d)]).astype(np.float32)


def _split_keys(key, n):
    g = np.arange(n, dtype=np.uint64)
    o = lit.philox4x32_10((g & np.uint64(0xFFFFFFFF)).astype(np.uint32), (g >> np.uint64(32)).astype(np.uint32), 0,
                          lit.TAG_SPLIT, np.uint32(key[0]), np.uint32(key[1]))
    return np.stack([o[0], o[1]], axis=-1)


@pytest.mark.parametrize("d", [96, 128, 256, 72, 100, 97])
def test_one_step_matches_literal(d, orc):
    from kernels_amd import PRNGKey
    g, om, Sigma = _case(d)
    rng = np.random.default_rng(d)
    L = np.linalg.cholesky(Sigma) * (1.0 + 0.1 * rng.random((d, 1)))  # a factor that is not the target's
    L = np.tril(L)
    sp = _packed(L)
    lam = math.log(2.38 / math.sqrt(d))
    npts, ns = 6, 8
    x = rng.multivariate_normal(np.asarray(g.mean), Sigma, size=npts).astype(np.float32)
    key = np.asarray(PRNGKey(11), np.uint32)
    out = orc.sample_pnx(om, key, x, np.zeros(d, np.float32), sp, lam, 1, ns)
    keys = _split_keys(key, npts * ns)
    wbits, ubits = lit.step_noise(keys, 0, d)
    xi = lit.normal_from_bits(wbits)
    u = lit.unif01_from_bits(ubits)
    Lf = np.tril(np.zeros((d, d)))
    for j in range(d):
        Lf[j:, j] = sp[sum(d - k for k in range(j)):sum(d - k for k in range(j + 1))]
    m, P = np.asarray(g.mean, np.float64), 0.5 * (g.precision + g.precision.T)
    c0 = 0.5 * g.logdet_2pi_cov
    skipped = 0
    for c in range(npts * ns):
        z = x[c // ns].astype(np.float64)
        zp = z + math.exp(lam) * (Lf @ xi[c]) + 1e-6 * xi[c]
        a = min(1.0, math.exp(lit.gaussian_potential(z, m, P, c0) - lit.gaussian_potential(zp, m, P, c0)))
        if abs(a - u[c]) < 1e-4:
            skipped += 1
            continue
        want = zp if u[c] < a else z
        np.testing.assert_allclose(out[c // ns, c % ns], want, rtol=1e-5, atol=1e-5, err_msg=f"chain {c}")
    assert skipped <= max(1, npts * ns // 50)


def test_frozen_target_factor_keeps_target(orc):
    """With the target's own Cholesky factor the frozen kernel leaves the
    target invariant: start points drawn from N(m, Sigma), 10 steps each,
    the output's mean and per-coordinate variance stay the target's."""
    from kernels_amd import PRNGKey
    d = 96
    g, om, Sigma = _case(d)
    L = np.linalg.cholesky(Sigma)
    rng = np.random.default_rng(5)
    npts, ns = 400, 4
    x = rng.multivariate_normal(np.asarray(g.mean), Sigma, size=npts).astype(np.float32)
    out = orc.sample_pnx(om, np.asarray(PRNGKey(3), np.uint32), x, np.zeros(d, np.float32), _packed(L),
                         math.log(2.38 / math.sqrt(d)), 10, ns).reshape(-1, d).astype(np.float64)
    moved = np.mean(np.any(out.reshape(npts, ns, d) != x[:, None, :], axis=-1))
    assert 0.5 < moved < 1.0  # 10 steps at the optimal scale: most chains moved
    sd = np.sqrt(np.diag(Sigma))
    zmean = (out.mean(0) - np.asarray(g.mean)) / (sd / math.sqrt(npts))  # points independent, samples not
    assert np.max(np.abs(zmean)) < 5.0
    ratio = out.var(0) / np.diag(Sigma)
    assert 0.75 < np.median(ratio) < 1.25


def test_oracle_pooled_refuses_ragged_large_d(orc):
    """The pooled mode has no d > 64 off the 32-multiples (the library's
    amh_pooled_stats returns AMH_EINVAL); the oracle answers NaN sums and
    leaves the shared state alone instead of running its d <= 64 arrays."""
    from kernels_amd import PRNGKey
    d, C = 100, 8
    _, om, _ = _case(d)
    st = orc.init(om, PRNGKey(0), C)
    sh = orc.pooled_init_shared(d)
    L0 = sh["L"].copy()
    _, _, sums = orc.pooled_stats(om, 0, st.z, st.potential_energy, st.rng_key, sh["mu"], sh["L"],
                                  float(sh["lam"][0]))
    assert np.isnan(sums).all()
    orc.pooled_update(om, sums, sh)
    assert np.array_equal(sh["L"], L0)


def test_callable_potential_becomes_external():
    """arwmh.py:69-70 takes any callable as potential_fn: a callable without
    a registry model id is wrapped as posteriors.TorchPotential (the
    AMH_MODEL_EXTERNAL path, dim from init_params), still XOR with model."""
    import posteriors as P
    from kernels_amd import ARWMH
    from kernels_amd import _lib
    k = ARWMH(potential_fn=lambda z: (z * z).sum(-1))
    assert isinstance(k._potential_fn, P.TorchPotential) and k._potential_fn.dim is None
    assert k._potential_fn.model_id == _lib.AMH_MODEL_EXTERNAL == 7
    with pytest.raises(ValueError):
        ARWMH(model=P.eight_schools, potential_fn=lambda z: z)
    with pytest.raises(TypeError):
        ARWMH(potential_fn=3.0)
    with pytest.raises(ValueError):
        P.torch_potential(lambda z: z, dim=257)
