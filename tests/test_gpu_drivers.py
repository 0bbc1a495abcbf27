"""The reference's collect_states_logscale driver (python/utils/kernel_utils.py:20-38)
on the device, against the committed golden trajectory (tests/golden/eight_schools.npz,
made by the literal float64 restatement, tests/golden/make_golden.py).

4 chains of eight schools, n_pow = 3: 1,000 steps with W = 0 and the state
recorded at the 190 grid points of ns_logscale(3), exactly the golden file's
record.  Every thinning interval is one fused launch, so this also covers the
fused path against the float64 literal restatement over 1,000 steps."""
import os

import numpy as np
import pytest
import torch

from test_golden import tol

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_collect_states_logscale_eight_schools_golden(gpu):
    import posteriors as P
    from kernels_amd import ARWMH
    from utils_amd.kernel_utils import collect_states_logscale, ns_logscale
    f = np.load(os.path.join(G, "eight_schools.npz"))
    d = 10
    assert np.array_equal(ns_logscale(3), f["steps_recorded"])
    k = ARWMH(model=P.eight_schools, num_chains=4, device=gpu)
    st = collect_states_logscale(f["run_key"], k, dict(P.EIGHT_SCHOOLS_DATA), n_pow=3,
                                 init_params=torch.as_tensor(f["init_z"]))
    torch.cuda.synchronize()
    n = len(f["steps_recorded"])
    assert st.z.shape == (n, 4, d) and st.adapt_state.scale.shape == (n, 4, d * (d + 1) // 2)
    assert np.array_equal(st.rng_key[0].cpu().numpy().view(np.uint32), f["chain_keys"])
    i = st.i.cpu().numpy()
    assert np.array_equal(i, f["i"])
    z, loc = st.z.cpu().numpy(), st.adapt_state.loc.cpu().numpy()
    pe = st.potential_energy.cpu().numpy()
    lam = st.adapt_state.log_step_size.cpu().numpy()
    macc = st.mean_accept_prob.cpu().numpy()
    sc = st.adapt_state.scale.cpu().numpy()

    def unpack(p):
        L = np.zeros((d, d))
        o = 0
        for j in range(d):
            L[j:, j] = p[o:o + d - j]
            o += d - j
        return L

    for kk, t in enumerate(f["steps_recorded"]):
        tl = tol(int(t))
        np.testing.assert_allclose(z[kk], f["z"][kk], rtol=tl["z"][0], atol=tl["z"][1], err_msg=f"z t={t}")
        np.testing.assert_allclose(loc[kk], f["loc"][kk], rtol=tl["loc"][0], atol=tl["loc"][1], err_msg=f"loc t={t}")
        np.testing.assert_allclose(pe[kk], f["pe"][kk], rtol=tl["pe"][0], atol=tl["pe"][1], err_msg=f"pe t={t}")
        assert np.max(np.abs(lam[kk] - f["lam"][kk])) <= tl["lam"], t
        assert np.max(np.abs(macc[kk] - f["macc"][kk])) <= tl["macc"], t
        for c in range(4):
            L1, Lg = unpack(sc[kk, c]), unpack(f["scale"][kk, c])
            S1, Sg = L1 @ L1.T, Lg @ Lg.T
            assert np.max(np.abs(S1 - Sg)) <= 1e-3 * np.max(np.abs(Sg)) + 1e-5, (int(t), c)


@pytest.mark.parametrize("kind,d", [("arwmh", 64), ("arwmh", 256), ("asss", 12), ("pooled", 128),
                                    ("pooled_overlap", 64), ("pooled_overlap", 128)])
def test_checkpoint_resume_is_exact(kind, d, gpu, tmp_path):
    """SURVEY.md §5 checkpoint / resume: save the state after 7 transitions,
    load it into a fresh kernel of the same configuration and continue for 5;
    the result equals 12 uninterrupted transitions bit for bit (the step is a
    pure function of the state; d = 256 also crosses the chained proposal).
    With overlap=True the sums pending in the sampler travel in the
    checkpoint and are handed to the fresh kernel."""
    import posteriors as P
    from kernels_amd import ARWMH, ASSS, PRNGKey, PooledARWMH, load_state, save_state
    cls = {"arwmh": ARWMH, "asss": ASSS, "pooled": PooledARWMH, "pooled_overlap": PooledARWMH}[kind]
    kw = dict(overlap=True) if kind == "pooled_overlap" else {}
    pooled = kind.startswith("pooled")
    C = 300
    z0 = torch.empty(C, d, device=gpu).uniform_(-2, 2)

    def fresh():
        k = cls(potential_fn=P.correlated_gaussian(d), num_chains=C, device=gpu, **kw)
        return k, k.init(PRNGKey(11), 4, z0, (), {})

    k, s = fresh()
    for _ in range(12):
        s = k.sample(s, (), {}) if not pooled else k.sample(s)
    k2, s2 = fresh()
    for _ in range(7):
        s2 = k2.sample(s2, (), {}) if not pooled else k2.sample(s2)
    path = str(tmp_path / "ckpt")  # ".npz" is appended
    marker = torch.arange(C, dtype=torch.int32, device=gpu)  # an extra array rides along
    assert save_state(path, s2, kernel=k2, marker=marker).endswith(".npz")
    k3, _ = fresh()
    if kind == "pooled_overlap":
        with pytest.raises(ValueError):
            load_state(path, gpu)  # pending sums need the kernel that continues the run
    s3, extra = load_state(path, gpu, kernel=k3, with_extras=True)
    assert list(extra) == ["marker"] and np.array_equal(extra["marker"], marker.cpu().numpy())
    for _ in range(5):
        s3 = k3.sample(s3, (), {}) if not pooled else k3.sample(s3)
    torch.cuda.synchronize()
    for a, b in zip(torch.utils._pytree.tree_leaves(s), torch.utils._pytree.tree_leaves(s3)):
        assert a.dtype == b.dtype and torch.equal(a, b)
