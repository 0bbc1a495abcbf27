"""GPU parity: the HIP kernels (through the C ABI, via kernels.ARWMH) against
the C oracle on identical inputs.  The bit spec makes the
expected agreement exact: every float of every state field, every step."""
import numpy as np
import pytest
import torch

from helpers import assert_state_bitequal, make_case, state_to_orc

pytestmark = pytest.mark.gpu


def _init(kind, C, gpu, orc, seed=0, d=None, num_warmup=0):
    from kernels_amd import ARWMH, PRNGKey
    kw, mk, om = make_case(kind, d)
    k = ARWMH(num_chains=C, **kw)
    key = PRNGKey(seed)
    if "potential_fn" in kw:
        z0 = np.random.default_rng(seed).uniform(-2, 2, size=(C, om.d)).astype(np.float32)
        st = k.init(key, num_warmup, torch.as_tensor(z0), (), mk)
        ost = orc.init(om, key, C, init_z=z0)
    else:
        st = k.init(key, num_warmup, None, (), mk)
        ost = orc.init(om, key, C)
    torch.cuda.synchronize()
    return k, st, om, ost


@pytest.mark.parametrize("kind", ["gaussian", "eight_schools", "kidiq", "diamonds", "diamonds_ss", "mixture"])
def test_init_bitexact(kind, gpu, orc):
    k, st, om, ost = _init(kind, 333, gpu, orc)
    assert_state_bitequal(st, ost, f"{kind} init")


@pytest.mark.parametrize("kind,d", [("gaussian", 64), ("gaussian", 5), ("gaussian", 16), ("gaussian", 33),
                                    ("eight_schools", None), ("kidiq", None), ("diamonds", None), ("diamonds_ss", None),
                                    ("gaussian", 96), ("gaussian", 256), ("gaussian", 72), ("gaussian", 100),
                                    ("gaussian", 97), ("mixture", 1), ("mixture", 3),
                                    ("mixture", 16)])
def test_potential_bitexact(kind, d, gpu, orc):
    k, st, om, ost = _init(kind, 8, gpu, orc, d=d)
    z = np.random.default_rng(1).normal(size=(1000, om.d)).astype(np.float32)
    pe = k.potential(torch.as_tensor(z, device=gpu)).cpu().numpy()
    ref = orc.potential(om, z)
    np.testing.assert_array_equal(pe.view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("kind,d,C", [("gaussian", 64, 1000), ("gaussian", 7, 517), ("gaussian", 32, 300),
                                      ("eight_schools", None, 400), ("kidiq", None, 257),
                                      ("diamonds", None, 66), ("diamonds_ss", None, 333), ("mixture", 1, 1000),
                                      ("mixture", 5, 300), ("gaussian", 1, 1000), ("gaussian", 2, 333)])
def test_single_steps_bitexact(kind, d, C, gpu, orc):
    """ARWMH.sample (one launch per step) vs oracle step(n_steps=1), 40 steps."""
    k, st, om, ost = _init(kind, C, gpu, orc, d=d, num_warmup=10)
    acc = np.zeros(C, np.int32)
    for t in range(40):
        st = k.sample(st, (), {})
        orc.step(om, ost, 1, num_warmup=10, accept_count=acc)
        torch.cuda.synchronize()
        assert_state_bitequal(st, ost, f"{kind} step {t}")
    np.testing.assert_array_equal(k.accept_count.cpu().numpy(), acc)


@pytest.mark.parametrize("kind,d,C", [("gaussian", 64, 2000), ("eight_schools", None, 1000), ("gaussian", 1, 777),
                                      ("diamonds", None, 130), ("diamonds_ss", None, 1000)])
def test_fused_steps_bitexact(kind, d, C, gpu, orc):
    """ARWMH.run (n steps in one launch, z collected) vs oracle step(n_steps)."""
    k, st, om, ost = _init(kind, C, gpu, orc, d=d)
    acc = np.zeros(C, np.int32)
    for n in (1, 7, 100):
        st, cz, _ = k.run(st, n, thinning=1, collect_z=True)
        ocz = orc.step(om, ost, n, accept_count=acc, collect_z=True)
        torch.cuda.synchronize()
        assert_state_bitequal(st, ost, f"{kind} fused {n}")
        np.testing.assert_array_equal(cz.cpu().numpy().view(np.uint32), ocz.view(np.uint32))
    np.testing.assert_array_equal(k.accept_count.cpu().numpy(), acc)


def test_inplace_and_thinning(gpu, orc):
    k, st, om, ost = _init("gaussian", 257, gpu, orc, d=12)
    st2, cz, cp = k.run(st, 30, thinning=10, collect_z=True, collect_pe=True)
    ocz = orc.step(om, ost, 30, collect_z=True)
    assert cz.shape == (3, 257, 12)
    np.testing.assert_array_equal(cz.cpu().numpy().view(np.uint32), ocz[9::10].view(np.uint32))
    k.sample_(st2, 5)
    orc.step(om, ost, 5)
    assert_state_bitequal(st2, ost, "in-place")


def test_split_path_generic_k(gpu, orc):
    """Diamonds through the split transition (propose / lane-per-chain
    potential / step) with a data shape off the compile-time fast path
    (K = 10, ragged N = 77): collection with thinning and in-place steps
    stay bit-identical to the oracle."""
    import posteriors as P
    from kernels_amd import ARWMH, PRNGKey
    mk = P.synthetic_diamonds(N=77, K=10, seed=5)
    arr, (N, K) = P.diamonds.pack_fn(mk)
    om = orc.Model(orc.DIAMONDS, K + 1, arr, n_data=N, k_data=K)
    C = 199
    k = ARWMH(model=P.diamonds, num_chains=C)
    st = k.init(PRNGKey(4), 5, None, (), mk)
    ost = orc.init(om, PRNGKey(4), C)
    assert_state_bitequal(st, ost, "split init")
    st2, cz, cp = k.run(st, 12, thinning=4, collect_z=True, collect_pe=True)
    ocz = orc.step(om, ost, 12, num_warmup=5, collect_z=True)
    np.testing.assert_array_equal(cz.cpu().numpy().view(np.uint32), ocz[3::4].view(np.uint32))
    k.sample_(st2, 3)
    orc.step(om, ost, 3, num_warmup=5)
    assert_state_bitequal(st2, ost, "split in-place")
    z = np.random.default_rng(2).normal(size=(300, K + 1)).astype(np.float32)
    pe = k.potential(torch.as_tensor(z, device=gpu)).cpu().numpy()
    np.testing.assert_array_equal(pe.view(np.uint32), orc.potential(om, z).view(np.uint32))


@pytest.mark.parametrize("d,C,steps", [(128, 77, 12), (256, 33, 6), (72, 70, 8), (100, 65, 8), (97, 41, 8),
                                        (160, 40, 6), (150, 33, 5), (192, 30, 5)])
def test_big_dim_bitexact(d, C, steps, gpu, orc):
    """64 < d <= 256 (amh_big.hip: propose pass, MFMA potential, step pass):
    init, single launches (gamma_1 = 1 keep-L at step 1, the warmup reset at
    step W + 1) and a multi-step launch with thinned collection, bit for bit."""
    k, st, om, ost = _init("gaussian", C, gpu, orc, d=d, num_warmup=3)
    assert_state_bitequal(st, ost, f"d={d} init")
    acc = np.zeros(C, np.int32)
    for t in range(steps):
        st = k.sample(st, (), {})
        orc.step(om, ost, 1, num_warmup=3, accept_count=acc)
        torch.cuda.synchronize()
        assert_state_bitequal(st, ost, f"d={d} step {t}")
    np.testing.assert_array_equal(k.accept_count.cpu().numpy(), acc)
    st2, cz, cp = k.run(st, 4, thinning=2, collect_z=True, collect_pe=True)
    ocz = orc.step(om, ost, 4, num_warmup=3, collect_z=True)
    torch.cuda.synchronize()
    assert_state_bitequal(st2, ost, f"d={d} run")
    np.testing.assert_array_equal(cz.cpu().numpy().view(np.uint32), ocz[1::2].view(np.uint32))


def test_sample_pnx_bitexact(gpu, orc):
    from kernels_amd import PRNGKey
    k, st, om, ost = _init("gaussian", 4, gpu, orc, d=16)
    st = k.sample_(st, 50)
    ad = st.adapt_state
    loc = ad.loc[0].cpu().numpy()
    scale = ad.scale[0].cpu().numpy()
    lam = float(ad.log_step_size[0].cpu())
    x = np.random.default_rng(3).normal(size=(5, 16)).astype(np.float32)
    out = k.sample_Pnx(PRNGKey(7), x, (ad.loc[0], ad.scale[0], ad.log_step_size[0]), n=6, n_samples=99)
    ref = orc.sample_pnx(om, PRNGKey(7), x, loc, scale, lam, 6, 99)
    assert out.shape == (5, 99, 16)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))


@pytest.mark.parametrize("d", [96, 128, 256, 100, 97, 160, 150])
def test_sample_pnx_large_d_bitexact(d, gpu, orc):
    """ARWMH.sample_Pnx at 64 < d <= 256 (big_pnx_kernel: the shared factor
    streamed per step, U by P's rows in the MFMA potential's order) against
    orc_sample_pnx's large-d mirror, bit for bit; the adapted state of a
    short run as the frozen theta, and the start point's potential included."""
    from kernels_amd import PRNGKey
    k, st, om, ost = _init("gaussian", 16, gpu, orc, d=d)
    st = k.sample_(st, 12)
    ad = st.adapt_state
    loc = ad.loc[5].cpu().numpy()
    scale = ad.scale[5].cpu().numpy()
    lam = float(ad.log_step_size[5].cpu())
    x = st.z[:3].cpu().numpy()
    out = k.sample_Pnx(PRNGKey(7), x, (ad.loc[5], ad.scale[5], ad.log_step_size[5]), n=5, n_samples=13)
    ref = orc.sample_pnx(om, PRNGKey(7), x, loc, scale, lam, 5, 13)
    assert out.shape == (3, 13, d)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), ref.view(np.uint32))
    moved = np.mean(np.any(ref != x[:, None, :], axis=-1))
    assert moved > 0.2  # the comparison covers accepted moves, not only rejections


def test_headline_size_properties(gpu):
    """65,536 chains x d = 64 (BASELINE config 2): after 200 steps every factor
    has a positive finite diagonal, acceptance moves toward 0.234, and the
    launch is deterministic (two runs from one state agree bit for bit)."""
    from kernels_amd import ARWMH, PRNGKey, unpack_scale
    import posteriors as P
    g = P.correlated_gaussian(64)
    C = 65536
    k = ARWMH(potential_fn=g, num_chains=C)
    z0 = torch.empty(C, 64, device=gpu).uniform_(-2, 2)
    st = k.init(PRNGKey(0), 0, z0, (), {})
    a, _, _ = k.run(st, 200, collect_z=False)
    b, _, _ = k.run(st, 200, collect_z=False)
    torch.cuda.synchronize()
    for x, y in zip(a[:4] + (a.as_change,), b[:4] + (b.as_change,)):
        assert torch.equal(x, y)
    assert torch.equal(a.adapt_state.scale, b.adapt_state.scale)
    L = unpack_scale(a.adapt_state.scale[:256], 64)
    dg = torch.diagonal(L, dim1=-2, dim2=-1)
    assert torch.isfinite(dg).all() and (dg > 0).all()
    macc = a.mean_accept_prob.mean().item()
    assert 0.05 < macc < 0.6, macc


def test_sharded_equals_unsharded(gpu):
    """Regime A sharding: two shards run with chain_offset
    reproduce the unsharded run bit for bit, including a ragged split."""
    from kernels_amd import ARWMH, PRNGKey
    from kernels_amd.distributed import shard_range
    import posteriors as P
    g = P.correlated_gaussian(64)
    C = 3001
    z0 = torch.empty(C, 64, device=gpu).uniform_(-2, 2)
    full = ARWMH(potential_fn=g, num_chains=C)
    sf = full.init(PRNGKey(3), 10, z0, (), {})
    full.sample_(sf, 30)
    parts = []
    for r in range(3):
        off, cnt = shard_range(C, r, 3)
        k = ARWMH(potential_fn=g, num_chains=cnt, chain_offset=off)
        s = k.init(PRNGKey(3), 10, z0[off:off + cnt].contiguous(), (), {})
        k.sample_(s, 30)
        parts.append(s)
    torch.cuda.synchronize()
    assert torch.equal(torch.cat([p.z for p in parts]), sf.z)
    assert torch.equal(torch.cat([p.adapt_state.scale for p in parts]), sf.adapt_state.scale)
    assert torch.equal(torch.cat([p.rng_key for p in parts]), sf.rng_key)


def test_edge_sizes(gpu, orc):
    """One chain, a chain count that leaves most of the last work item empty,
    and d = 1 (the frozen-acceptance model of asumptions_check.ipynb)."""
    from kernels_amd import ARWMH, PRNGKey
    import posteriors as P
    for d, C in ((64, 1), (3, 17), (1, 5), (2, 1)):
        g = P.correlated_gaussian(d)
        kw, om = dict(potential_fn=g), orc.Model(orc.GAUSSIAN, d, g.pack("cpu")[0].numpy())
        k = ARWMH(num_chains=C, **kw)
        z0 = np.random.default_rng(d).uniform(-2, 2, size=(C, d)).astype(np.float32)
        st = k.init(PRNGKey(1), 3, torch.as_tensor(z0), (), {})
        ost = orc.init(om, PRNGKey(1), C, init_z=z0)
        k.sample_(st, 9)
        orc.step(om, ost, 9, num_warmup=3)
        torch.cuda.synchronize()
        assert_state_bitequal(st, ost, f"d={d} C={C}")


@pytest.mark.parametrize("name", ["eight_schools", "gaussian64"])
def test_gpu_follows_golden(name, gpu):
    """The device path against the golden vectors of tests/golden (literal
    float64 restatement): identical accept decisions at every step, states
    within the tolerances of tests/test_golden.py."""
    import os
    import posteriors as P
    from kernels_amd import ARWMH
    from test_golden import tol
    f = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", name + ".npz"))
    C = f["init_z"].shape[0]
    if name == "eight_schools":
        k = ARWMH(model=P.eight_schools, num_chains=C)
        st = k.init(f["run_key"], 0, torch.as_tensor(f["init_z"]), (), dict(P.EIGHT_SCHOOLS_DATA))
    else:
        g = P.correlated_gaussian(64)
        assert np.array_equal(g.pack("cpu")[0].numpy(), f["model_data"])
        k = ARWMH(potential_fn=g, num_chains=C)
        st = k.init(f["run_key"], 0, torch.as_tensor(f["init_z"]), (), {})
    rec = {int(t): j for j, t in enumerate(f["steps_recorded"])}
    prev = k.accept_count.clone()
    for t in range(f["accept"].shape[1]):
        k.sample_(st, 1)
        now = k.accept_count.clone()
        assert np.array_equal((now - prev).bool().cpu().numpy(), f["accept"][:, t]), f"step {t + 1}"
        prev = now
        if t + 1 in rec:
            j, tl = rec[t + 1], tol(t + 1)
            np.testing.assert_allclose(st.z.cpu().numpy(), f["z"][j], rtol=tl["z"][0], atol=tl["z"][1])
            np.testing.assert_allclose(st.adapt_state.loc.cpu().numpy(), f["loc"][j], rtol=tl["loc"][0],
                                       atol=tl["loc"][1])


def test_diamonds_suffstat_generic_k(gpu, orc):
    """Sufficient-statistics diamonds off the reference shape (K = 10, N = 77,
    d = 11 in the G = 32 group): init, thinned collection and the potential
    bit-identical to the oracle."""
    import posteriors as P
    from kernels_amd import ARWMH, PRNGKey
    mk = P.synthetic_diamonds(N=77, K=10, seed=5)
    arr, (N, K) = P.diamonds_suffstat.pack_fn(mk)
    om = orc.Model(orc.DIAMONDS_SS, K + 1, arr, n_data=N, k_data=K)
    C = 199
    k = ARWMH(model=P.diamonds_suffstat, num_chains=C)
    st = k.init(PRNGKey(4), 5, None, (), mk)
    ost = orc.init(om, PRNGKey(4), C)
    assert_state_bitequal(st, ost, "suffstat init")
    st2, cz, cp = k.run(st, 12, thinning=4, collect_z=True, collect_pe=True)
    ocz = orc.step(om, ost, 12, num_warmup=5, collect_z=True)
    np.testing.assert_array_equal(cz.cpu().numpy().view(np.uint32), ocz[3::4].view(np.uint32))
    assert_state_bitequal(st2, ost, "suffstat run")
    z = np.random.default_rng(2).normal(size=(300, K + 1)).astype(np.float32)
    pe = k.potential(torch.as_tensor(z, device=gpu)).cpu().numpy()
    np.testing.assert_array_equal(pe.view(np.uint32), orc.potential(om, z).view(np.uint32))


@pytest.mark.parametrize("kind,d,C", [("gaussian", 128, 65), ("diamonds", None, 66)])
def test_big_dim_chained_proposal_invalidation(kind, d, C, gpu, orc):
    """d > 64 and the literal diamonds split path: sample() reuses the proposal
    the previous step pass formed only for the unchanged state it returned: an
    in-place edit of z between calls (torch version counter) or a different
    state object forces the propose pass, and every path stays bit-identical
    to the oracle."""
    k, st, om, ost = _init(kind, C, gpu, orc, d=d, num_warmup=2)
    for t in range(3):
        st = k.sample(st, (), {})
        orc.step(om, ost, 1, num_warmup=2)
    st.z[:, 0] += 0.25  # in place: the kept proposal is stale
    ost.z[:, 0] += np.float32(0.25)
    for t in range(3):
        st = k.sample(st, (), {})
        orc.step(om, ost, 1, num_warmup=2)
        torch.cuda.synchronize()
        assert_state_bitequal(st, ost, f"after edit, step {t}")
    other = st._replace(z=st.z.clone())  # same values, another tensor
    st = k.sample(other, (), {})
    orc.step(om, ost, 1, num_warmup=2)
    k.sample_(st, 2)
    orc.step(om, ost, 2, num_warmup=2)
    torch.cuda.synchronize()
    assert_state_bitequal(st, ost, "clone + in-place")
    # a zero-step call in between must not hand s1's kept proposal to s0
    s0 = st
    ost0 = ost.copy()
    s1 = k.sample(s0, (), {})
    k.sample_(s0, 0)
    s0b = k.sample(s0, (), {})
    orc.step(om, ost0, 1, num_warmup=2)
    torch.cuda.synchronize()
    assert_state_bitequal(s0b, ost0, "zero-step call between")
    assert_state_bitequal(s1, ost0, "s1 = step(s0)")
    z0 = k.run(s0b, 0)
    assert z0[1] is None and torch.equal(z0[0].z, s0b.z) and z0[0].z.data_ptr() != s0b.z.data_ptr()
    # inference-mode tensors carry no version counter: never chained, still exact
    with torch.inference_mode():
        si = k.sample(s0b, (), {})
        si = k.sample(si, (), {})
    orc.step(om, ost0, 2, num_warmup=2)
    torch.cuda.synchronize()
    assert_state_bitequal(si, ost0, "inference mode")
