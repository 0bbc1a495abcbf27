"""Steady-state parity at the BASELINE sizes.

The persistent step kernels hand chains over inside a wave: launch_step64
gives a wave more than one chain only when C > 4,096 (256 blocks x 16 waves),
the generic step kernel when C exceeds CPW x (its co-resident waves), ASSS
when the chain groups exceed 8,192 blocks x 4 waves.  Every test here runs at
a size where each wave owns several chains (the hand-over: store of chain
k-1, the swap through LDS, the flush, the ticket draws) and compares the
WHOLE chain range with the C oracle, bit for bit, through:

  * single sample() launches across the W + 1 warmup reset,
  * a fused run() with thinned collection of z,
  * an in-place sample_() of several steps,
  * the accept counters.

Ragged sizes (4,097 and 65,537 at d = 64) leave one block with one more chain
than the rest.  Reference semantics: python/kernels/arwmh.py:140-207 (ARWMH),
python/kernels/asss.py:197-251 (ASSS)."""
import numpy as np
import pytest
import torch

from helpers import assert_state_bitequal, make_case

pytestmark = pytest.mark.gpu


def _init(kind, C, orc, d=None, num_warmup=0, seed=0, cls="ARWMH"):
    import kernels_amd
    kw, mk, om = make_case(kind, d)
    k = getattr(kernels_amd, cls)(num_chains=C, **kw)
    key = kernels_amd.PRNGKey(seed)
    if "potential_fn" in kw:
        z0 = np.random.default_rng(seed + C).uniform(-2, 2, size=(C, om.d)).astype(np.float32)
        st = k.init(key, num_warmup, torch.as_tensor(z0), (), mk)
        ost = orc.init(om, key, C, init_z=z0)
    else:
        st = k.init(key, num_warmup, None, (), mk)
        ost = orc.init(om, key, C)
    torch.cuda.synchronize()
    return k, st, mk, om, ost


def _arwmh_sequence(kind, d, C, W, gpu, orc, n_single=5):
    k, st, mk, om, ost = _init(kind, C, orc, d=d, num_warmup=W)
    assert_state_bitequal(st, ost, f"{kind} C={C} init")
    acc = np.zeros(C, np.int32)
    for t in range(n_single):  # i = 1..n_single: gamma_1 = 1 keep-L, the reset at W + 1
        st = k.sample(st, (), mk)
        orc.step(om, ost, 1, num_warmup=W, accept_count=acc)
        if t in (0, W, n_single - 1):
            torch.cuda.synchronize()
            assert_state_bitequal(st, ost, f"{kind} C={C} sample {t + 1}")
    st, cz, _ = k.run(st, 7, thinning=3, collect_z=True)
    ocz = orc.step(om, ost, 7, num_warmup=W, accept_count=acc, collect_z=True)
    torch.cuda.synchronize()
    assert_state_bitequal(st, ost, f"{kind} C={C} run(7, thinning=3)")
    assert cz.shape == (2, C, om.d)
    np.testing.assert_array_equal(cz.cpu().numpy().view(np.uint32), ocz[2::3].view(np.uint32))
    del cz, ocz
    k.sample_(st, 6)
    orc.step(om, ost, 6, num_warmup=W, accept_count=acc)
    torch.cuda.synchronize()
    assert_state_bitequal(st, ost, f"{kind} C={C} sample_(6)")
    np.testing.assert_array_equal(k.accept_count.cpu().numpy(), acc)
    assert int(st.i.min()) == int(st.i.max()) == n_single + 13


@pytest.mark.parametrize("C", [65536, 4097, 65537])
def test_step64_steady_state_bitexact(C, gpu, orc):
    """arwmh_step64_kernel<16> (the headline kernel) at configs[1]'s size and
    at ragged sizes either side of one chain per wave: every chain, every field."""
    _arwmh_sequence("gaussian", 64, C, 3, gpu, orc)


@pytest.mark.parametrize("kind,C", [("eight_schools", 262144), ("diamonds_ss", 262144), ("kidiq", 131072),
                                    ("gaussian32", 100003)])
def test_generic_step_steady_state_bitexact(kind, C, gpu, orc):
    """arwmh_step_kernel<DMAX, M> with several chain groups per wave:
    eight schools (G = 16, 4 chains per wave), the diamonds sufficient-
    statistics model at configs[2]'s 262,144 chains (compile-time d = 26),
    kidiq (G = 4) and a ragged d = 32 Gaussian."""
    d = None
    if kind == "gaussian32":
        kind, d = "gaussian", 32
    _arwmh_sequence(kind, d, C, 2, gpu, orc, n_single=4)


@pytest.mark.parametrize("kind,d,C", [("gaussian", 64, 65536), ("eight_schools", None, 262144)])
def test_asss_steady_state_bitexact(kind, d, C, gpu, orc):
    """ASSS (amh_asss.hip) with two or more chain groups per wave (grid-stride
    past 8,192 blocks): single launches, a fused run with collection, in place."""
    from test_gpu_asss import assert_bitequal
    k, st, mk, om, ost = _init(kind, C, orc, d=d, num_warmup=2, cls="ASSS")
    for t in range(3):
        st = k.sample(st, (), mk)
        orc.asss_step(om, ost, 1, num_warmup=2)
    torch.cuda.synchronize()
    assert_bitequal(st, ost, f"asss {kind} C={C} sample x3")
    st, cz, cp = k.run(st, 4, thinning=2, collect_z=True, collect_pe=True)
    ocz, ocp = orc.asss_step(om, ost, 4, num_warmup=2, collect_z=True, collect_pe=True)
    torch.cuda.synchronize()
    assert_bitequal(st, ost, f"asss {kind} C={C} run(4)")
    np.testing.assert_array_equal(cz.cpu().numpy().view(np.uint32), ocz[1::2].view(np.uint32))
    np.testing.assert_array_equal(cp.cpu().numpy().view(np.uint32), ocp[1::2].view(np.uint32))
    k.sample_(st, 3)
    orc.asss_step(om, ost, 3, num_warmup=2)
    torch.cuda.synchronize()
    assert_bitequal(st, ost, f"asss {kind} C={C} in place")
