"""ASSS (asss.py:99-269): pin the C oracle's bit spec (orc_asss_step, the
mirror of amh_asss.hip) against the literal float64 restatement
oracle/asss_np.py with the same injected draws, plus known answers.

Tolerances (one teacher-forced step, float32 oracle vs float64 literal):
x', mu' rtol 1e-4 / atol 1e-5 (x' goes through S^-1 and S at condition
number up to ~1e2); U(x') rtol 1e-4; L'L'^T rel 1e-4; as_change rel 1e-3.
A chain whose shrinkage took a different number of steps (a slice test
within float32 rounding of the level) is skipped, and at most 2 % may be."""
import numpy as np
import pytest

import asss_np as lit
from helpers import make_case
from test_oracle import lit_potential, unpack


def _step_compare(kind, pre, orc, C=48, d=None):
    _, _, om = make_case(kind, d)
    from kernels_amd import PRNGKey
    st = orc.init(om, PRNGKey(7), C)
    if pre:
        orc.asss_step(om, st, pre)
    before = st.copy()
    orc.asss_step(om, st, 1)
    U = lit_potential(kind, om)
    dd = om.d
    skipped = 0
    for c in range(C):
        v, ut, th0, uks = lit.draws(before.rng_key[c], int(before.i[c]), dd)
        s0 = lit.ASSSState(int(before.i[c]), before.z[c].astype(np.float64), float(before.potential_energy[c]),
                           lit.ASSSAdaptState(before.loc[c].astype(np.float64), unpack(before.scale[c], dd)),
                           0.0, None)
        new, n_iter = lit.sample(s0, U, v, ut, th0, uks)
        # the oracle's iteration count is not exported: compare the endpoint
        # directly and skip chains whose slice decision flipped (endpoint far)
        if not np.allclose(st.z[c], new.z, rtol=1e-3, atol=1e-3):
            skipped += 1
            continue
        np.testing.assert_allclose(st.z[c], new.z, rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(st.loc[c], new.adapt_state.loc, rtol=1e-4, atol=1e-5)
        np.testing.assert_allclose(st.potential_energy[c], new.potential_energy, rtol=1e-4, atol=1e-4)
        Lg = unpack(st.scale[c], dd)
        Ll = new.adapt_state.scale
        S_g, S_l = Lg @ Lg.T, Ll @ Ll.T
        assert np.linalg.norm(S_g - S_l) <= 1e-4 * np.linalg.norm(S_l) + 1e-7
        assert abs(st.as_change[c] - new.as_change) <= 1e-3 * abs(new.as_change) + 1e-6
        assert int(st.i[c]) == new.i
    assert skipped <= max(1, C // 50), f"{skipped} of {C} chains took a different slice path"


@pytest.mark.parametrize("kind,d", [("gaussian", 12), ("gaussian", 64), ("eight_schools", None), ("kidiq", None),
                                    ("diamonds", None), ("mixture", 1), ("mixture", 3),
                                    # large d (asss_step_big1: streamed factor, potential along the circle)
                                    ("gaussian", 96), ("gaussian", 128), ("gaussian", 100), ("gaussian", 97)])
@pytest.mark.parametrize("pre", [0, 1, 23])
def test_oracle_step_matches_literal(kind, d, pre, orc):
    _step_compare(kind, pre, orc, C=24 if kind in ("diamonds", "gaussian") else 48, d=d)


def test_first_step_keeps_factor(orc):
    """gamma_1 = 1: sqrt(1-gamma) L = 0 -> NaN -> keep L; mu jumps to x'."""
    _, _, om = make_case("eight_schools")
    from kernels_amd import PRNGKey
    st = orc.init(om, PRNGKey(1), 16)
    L0 = st.scale.copy()
    orc.asss_step(om, st, 1)
    assert np.array_equal(st.scale, L0)
    assert np.array_equal(st.loc, st.z)


def test_draws_layout():
    """v_d, u_t and theta_0 come from lane 0's Philox words 1-3."""
    key = np.array([5, 9], np.uint32)
    v, ut, th0, uks = lit.draws(key, 3, 4)
    assert v.shape == (5,) and uks.shape == (50,)
    assert 0.0 <= ut < 1.0 and 0.0 <= th0 < 2 * np.pi + 1e-6


def test_gaussian_moments(orc):
    """Slice sampling leaves the target invariant: a correlated 4-d Gaussian's
    mean and covariance are recovered."""
    import posteriors as P
    import orc as O
    g = P.gaussian(np.zeros(4), cov=np.array([[1.0, 0.5, 0, 0], [0.5, 2.0, 0, 0], [0, 0, 0.5, 0.1],
                                              [0, 0, 0.1, 1.0]]))
    data, _ = g.pack("cpu")
    om = O.Model(O.GAUSSIAN, 4, data.numpy())
    from kernels_amd import PRNGKey
    st = orc.init(om, PRNGKey(2), 256)
    orc.asss_step(om, st, 300)
    cz, _ = orc.asss_step(om, st, 400, collect_z=True)
    x = cz[::4].reshape(-1, 4).astype(np.float64)
    assert np.abs(x.mean(0)).max() < 0.05
    np.testing.assert_allclose(np.cov(x.T), np.linalg.inv(g.precision), atol=0.08)


def test_zero_norm_tangent_keeps_state(orc):
    """A tangent that rounds to zero in every component (|v| = 0: the
    reference's v / norm(v) is NaN, asss.py:222, and would poison the chain)
    takes the shrinkage's own fallback, theta = 0 (asss.py:94): x' is x
    re-projected through the sphere, U(x') its potential, and the adaptation
    runs with delta = x' - mu.  Forced here with the oracle's test hook (the
    event is measure-zero after the fmaf projection); the kernel
    (amh_asss.h) makes the same decisions."""
    from kernels_amd import PRNGKey
    _, _, om = make_case("gaussian", 12)
    st = orc.init(om, PRNGKey(3), 16)
    orc.asss_step(om, st, 5)
    before = st.copy()
    L = orc.lib()
    L.orc_set_test_zero_tangent(1)
    try:
        orc.asss_step(om, st, 1)
    finally:
        L.orc_set_test_zero_tangent(0)
    assert np.all(np.isfinite(st.z)) and np.all(np.isfinite(st.potential_energy))
    assert np.all(np.isfinite(st.scale)) and np.all(np.isfinite(st.loc))
    np.testing.assert_allclose(st.z, before.z, rtol=1e-5, atol=1e-5)  # kept, up to the re-projection
    np.testing.assert_allclose(st.potential_energy, orc.potential(om, st.z), rtol=1e-6)
    assert np.all(st.i == before.i + 1)
    assert not np.array_equal(st.loc, before.loc)  # adaptation ran
