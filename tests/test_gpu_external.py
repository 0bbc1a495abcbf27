"""The external-potential path (AMH_MODEL_EXTERNAL: amh_propose, the
caller's U, amh_step_external; arwmh.py:69-70's arbitrary potential_fn) on
the GPU.  With U = the library's own Gaussian potential (amh_potential,
bit-identical to the oracle's) the transitions must equal orc_step bit for
bit -- single launches, in-place multi-step runs and thinned collection --
at d where the fused Gaussian kernel's lane group is the external path's
(32 for 17 <= d <= 32, 64 above; d = 64's fused kernel is the step64
specialisation, bit-identical to the generic one); above d = 64 the large-d
propose / step passes take the caller's U as they take the MFMA potential's.  A potential written in torch samples its target."""
import math

import numpy as np
import pytest
import torch

from helpers import assert_state_bitequal, make_case

pytestmark = pytest.mark.gpu


def _pair(d, C, gpu, orc, W=4, seed=0):
    from kernels_amd import ARWMH, PRNGKey
    kw, mk, om = make_case("gaussian", d)
    z0 = np.random.default_rng(seed).uniform(-2, 2, size=(C, d)).astype(np.float32)
    kg = ARWMH(num_chains=8, **kw)  # the registry kernel, for its potential only
    kg.init(PRNGKey(1), 0, torch.as_tensor(z0[:8]), (), mk)
    ke = ARWMH(potential_fn=lambda z: kg.potential(z), num_chains=C)
    st = ke.init(PRNGKey(seed), W, torch.as_tensor(z0), (), {})
    ost = orc.init(om, PRNGKey(seed), C, init_z=z0)
    torch.cuda.synchronize()
    return ke, st, om, ost


@pytest.mark.parametrize("d,C", [(24, 333), (32, 200), (17, 65), (48, 130), (64, 77), (100, 40), (128, 33)])
def test_external_matches_oracle_bitexact(d, C, gpu, orc):
    ke, st, om, ost = _pair(d, C, gpu, orc)
    assert_state_bitequal(st, ost, f"d={d} init")
    acc = np.zeros(C, np.int32)
    for t in range(8):  # crosses gamma_1 = 1 (keep L) and the warmup reset at W + 1
        st = ke.sample(st, (), {})
        orc.step(om, ost, 1, num_warmup=4, accept_count=acc)
        torch.cuda.synchronize()
        assert_state_bitequal(st, ost, f"d={d} step {t}")
    np.testing.assert_array_equal(ke.accept_count.cpu().numpy(), acc)
    # every external transition is its own launch (the state goes through
    # HBM, L = U diag(dl) stored and re-read), so the oracle runs one step per
    # call -- its fused n-step call keeps U across steps, as the fused kernels
    ke.sample_(st, 5)  # in place: the chained proposals of amh_step_external
    for _ in range(5):
        orc.step(om, ost, 1, num_warmup=4)
    torch.cuda.synchronize()
    assert_state_bitequal(st, ost, f"d={d} in-place")
    st2, cz, cp = ke.run(st, 6, thinning=3, collect_z=True, collect_pe=True)
    ozs, ops = [], []
    for _ in range(6):
        orc.step(om, ost, 1, num_warmup=4)
        ozs.append(ost.z.copy())
        ops.append(ost.potential_energy.copy())
    torch.cuda.synchronize()
    assert_state_bitequal(st2, ost, f"d={d} run")
    np.testing.assert_array_equal(cz.cpu().numpy().view(np.uint32), np.stack(ozs)[2::3].view(np.uint32))
    np.testing.assert_array_equal(cp.cpu().numpy().view(np.uint32), np.stack(ops)[2::3].view(np.uint32))


def test_torch_potential_samples_target(gpu):
    """U written in torch (a correlated 3-D Gaussian): after adaptation the
    chains' moments are the target's and acceptance is near 0.234."""
    from kernels_amd import ARWMH, PRNGKey
    S = torch.tensor([[1.0, 0.5, 0.0], [0.5, 2.0, -0.3], [0.0, -0.3, 0.5]], dtype=torch.float64)
    Pm = torch.linalg.inv(S).to(torch.float32).cuda()
    m = torch.tensor([1.0, -2.0, 0.5], device="cuda")

    def U(z):
        x = z - m
        return 0.5 * ((x @ Pm) * x).sum(-1)

    C = 4096
    k = ARWMH(potential_fn=U, num_chains=C)
    st = k.init(PRNGKey(3), 0, torch.rand(C, 3) * 4 - 2, (), {})
    k.sample_(st, 1500)
    st, cz, _ = k.run(st, 400, thinning=20, collect_z=True)
    z = cz.reshape(-1, 3).double().cpu()
    np.testing.assert_allclose(z.mean(0).numpy(), m.cpu().numpy(), atol=0.05)
    np.testing.assert_allclose(torch.cov(z.T).numpy(), S.numpy(), atol=0.08)
    assert abs(float(st.mean_accept_prob.mean()) - 0.234) < 0.03
    np.testing.assert_allclose(st.potential_energy.cpu().numpy(), U(st.z).cpu().numpy(), rtol=1e-6, atol=1e-6)


def test_external_limits(gpu):
    """What the external path does not take: ASSS (the slice kernel
    evaluates U inside), d > 256, a potential that
    returns the wrong number of values; NaN rejects (arwmh.py:171)."""
    from kernels_amd import ARWMH, ASSS, PRNGKey
    from kernels_amd._lib import AmhError
    U = lambda z: 0.5 * (z * z).sum(-1)  # noqa: E731
    k = ARWMH(potential_fn=U, num_chains=64)
    st = k.init(PRNGKey(0), 0, torch.zeros(64, 4), (), {})
    with pytest.raises(AmhError, match="device potential"):
        a = ASSS(potential_fn=U, num_chains=64)
        a.sample(a.init(PRNGKey(0), 0, torch.zeros(64, 4), (), {}))
    with pytest.raises(AmhError, match=r"dim must be in \[1, 256\]"):
        ARWMH(potential_fn=U, num_chains=8).init(PRNGKey(0), 0, torch.zeros(8, 300), (), {})
    bad = ARWMH(potential_fn=lambda z: z.sum(), num_chains=8)
    with pytest.raises(ValueError, match="one each"):
        bad.init(PRNGKey(0), 0, torch.zeros(8, 4), (), {})
    nan = ARWMH(potential_fn=lambda z: torch.where(z[:, 0] > 0, torch.nan, 0.5 * (z * z).sum(-1)), num_chains=256)
    s = nan.init(PRNGKey(2), 0, -torch.ones(256, 2), (), {})
    nan.sample_(s, 200)
    assert bool((s.z[:, 0] <= 0).all())  # every proposal into the NaN half was rejected
    assert math.isfinite(float(s.potential_energy.max()))


def test_external_large_d_state_check(gpu):
    """d > 64: amh_step_external takes only the state whose proposals the
    handle holds the solves of (a stale state is refused, not stepped)."""
    import ctypes
    from kernels_amd import ARWMH, PRNGKey, _lib
    from kernels_amd._lib import AmhError
    from kernels_amd.arwmh import ctypes_state
    U = lambda z: 0.5 * (z * z).sum(-1)  # noqa: E731
    k = ARWMH(potential_fn=U, num_chains=16)
    st = k.init(PRNGKey(0), 0, torch.zeros(16, 96), (), {})
    other = k.init(PRNGKey(1), 0, torch.zeros(16, 96), (), {})
    zp = torch.empty(16, 96, device=st.z.device)
    L = _lib.lib()
    s = _lib.stream_ptr(st.z.device.index)
    _lib.check(L.amh_propose(k._handle.h, 16, ctypes_state(k, st), _lib.ptr(zp), s), k._handle.h)
    pe = U(zp).contiguous()
    rc = L.amh_step_external(k._handle.h, 16, ctypes_state(k, other), ctypes_state(k, other), _lib.ptr(zp),
                             _lib.ptr(pe), None, None, s)
    with pytest.raises(AmhError, match="proposals of this state"):
        _lib.check(rc, k._handle.h)
    _lib.check(L.amh_step_external(k._handle.h, 16, ctypes_state(k, st), ctypes_state(k, st), _lib.ptr(zp),
                                   _lib.ptr(pe), None, None, s), k._handle.h)
    assert int(st.i[0]) == 1


@pytest.mark.parametrize("d", [5, 24, 48])
def test_external_sample_pnx_bitexact(d, gpu, orc):
    """sample_Pnx with the caller's U (amh_pnx_propose / amh_pnx_accept):
    with U = the library's own Gaussian potential, bit for bit the oracle's
    orc_sample_pnx (the fused frozen kernel's spec), start points included."""
    from kernels_amd import ARWMH, PRNGKey
    kw, mk, om = make_case("gaussian", d)
    kg = ARWMH(num_chains=8, **kw)
    z0 = np.random.default_rng(0).uniform(-2, 2, size=(8, d)).astype(np.float32)
    st = kg.init(PRNGKey(1), 0, torch.as_tensor(z0), (), mk)
    st = kg.sample_(st, 30)
    ad = st.adapt_state
    ke = ARWMH(potential_fn=lambda z: kg.potential(z), num_chains=8)
    ke.init(PRNGKey(1), 0, torch.as_tensor(z0), (), {})
    x = np.random.default_rng(3).normal(size=(4, d)).astype(np.float32)
    out = ke.sample_Pnx(PRNGKey(7), x, (ad.loc[2], ad.scale[2], ad.log_step_size[2]), n=6, n_samples=33)
    ref = orc.sample_pnx(om, PRNGKey(7), x, ad.loc[2].cpu().numpy(), ad.scale[2].cpu().numpy(),
                         float(ad.log_step_size[2].cpu()), 6, 33)
    assert out.shape == (4, 33, d)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    assert np.mean(np.any(ref != x[:, None, :], axis=-1)) > 0.2


def test_mcmc_driver_with_torch_eight_schools(gpu):
    """The reference's usage with a hand-written potential: the non-centred
    eight-schools density (run_eight_schools_lr_decay.py:26-35) written in
    torch by the caller, driven by infer_amd.MCMC through the external path;
    the posterior means match the notebook's (cell 28: mu 4.40, theta_base[0]
    0.32) within this shorter run's spread."""
    import posteriors as P
    from infer_amd import MCMC
    from kernels_amd import ARWMH, PRNGKey
    y = torch.tensor(P.EIGHT_SCHOOLS_DATA["y"], dtype=torch.float32, device="cuda")
    sg = torch.tensor(P.EIGHT_SCHOOLS_DATA["sigma"], dtype=torch.float32, device="cuda")
    half_log_2pi = 0.5 * math.log(2 * math.pi)

    def U(z):  # z = [mu, log tau, theta_base (8)]: sorted site order, tau unconstrained
        mu, ltau, tb = z[:, 0], z[:, 1], z[:, 2:]
        tau = torch.exp(ltau)
        lp = -0.5 * (mu / 5.0) ** 2 - math.log(5.0) - half_log_2pi
        lp = lp + math.log(2 / math.pi) - math.log(5.0) - torch.log1p((tau / 5.0) ** 2) + ltau
        lp = lp + (-0.5 * tb ** 2 - half_log_2pi).sum(-1)
        r = (y - (mu[:, None] + tau[:, None] * tb)) / sg
        lp = lp + (-0.5 * r ** 2 - torch.log(sg) - half_log_2pi).sum(-1)
        return -lp

    C = 256
    k = ARWMH(potential_fn=U, num_chains=C)
    m = MCMC(k, num_warmup=5000, num_samples=40000, thinning=40)
    m.run(PRNGKey(0), init_params=torch.rand(C, 10) * 4 - 2)
    z = m.get_samples()
    z = z if torch.is_tensor(z) else torch.as_tensor(np.asarray(z))
    z = z.reshape(-1, 10).double()
    assert z.shape[0] == C * 1000
    assert float(z[:, 0].mean()) == pytest.approx(4.40, abs=0.4)
    assert float(z[:, 2].mean()) == pytest.approx(0.32, abs=0.08)
