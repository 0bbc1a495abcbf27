"""Pooled-covariance mode on the GPU (amh_pooled_*) against the oracle
(orc_pooled_*): per-chain state, the sums vector and the shared state bit
for bit over several steps (the summation order is part of the spec)."""
import numpy as np
import pytest
import torch

from helpers import make_case

pytestmark = pytest.mark.gpu


def _run(kind, d, C, steps, gpu, orc, seed=0, K=1):
    from kernels_amd import PooledARWMH, PRNGKey
    kw, mk, om = make_case(kind, d)
    k = PooledARWMH(num_chains=C, sync_every=K, **kw)
    z0 = np.random.default_rng(seed).uniform(-2, 2, size=(C, om.d)).astype(np.float32)
    st = k.init(PRNGKey(seed), 0, torch.as_tensor(z0), (), mk)
    ost = orc.init(om, PRNGKey(seed), C, init_z=z0)
    z, pe, keys = ost.z, ost.potential_energy, ost.rng_key
    assert np.array_equal(st.rng_key.cpu().numpy().view(np.uint32), keys)
    assert np.array_equal(st.potential_energy.cpu().numpy().view(np.uint32), pe.view(np.uint32))
    sh = orc.pooled_init_shared(om.d)
    for t in range(steps):
        st = k.sample(st)
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]),
                                       k_steps=K)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(k._sums.cpu().numpy().view(np.uint64), sums.view(np.uint64),
                                      err_msg=f"{kind} sums step {t + 1}")
        orc.pooled_update(om, sums, sh, k_steps=K)
        got = dict(z=st.z, pe=st.potential_energy, mu=st.adapt_state.loc, L=st.adapt_state.scale,
                   lam=st.adapt_state.log_step_size, macc=st.mean_accept_prob, asc=st.as_change, cov=st.cov,
                   i=st.i)
        want = dict(z=z, pe=pe, mu=sh["mu"], L=sh["L"], lam=sh["lam"], macc=sh["macc"], asc=sh["asc"],
                    cov=sh["cov"], i=sh["i"])
        for f in got:
            a = got[f].cpu().numpy()
            b = np.asarray(want[f])
            assert a.shape == b.shape, (f, a.shape, b.shape)
            assert a.tobytes() == b.astype(a.dtype).tobytes(), f"{kind} {f} differs at step {t + 1}"
    return k, st


@pytest.mark.parametrize("kind,d,C,steps", [("gaussian", 64, 3000, 6), ("gaussian", 64, 70000, 3),
                                            ("gaussian", 7, 517, 8), ("eight_schools", None, 64, 8),
                                            ("kidiq", None, 100, 5), ("diamonds", None, 40, 3),
                                            ("diamonds_ss", None, 1000, 4),
                                            ("gaussian", 128, 700, 4), ("gaussian", 256, 600, 3),
                                            # 3, 5 and 7 column tiles of the d > 64 update
                                            ("gaussian", 96, 500, 3), ("gaussian", 160, 400, 3),
                                            ("gaussian", 224, 300, 3)])
def test_pooled_bitexact(kind, d, C, steps, gpu, orc):
    _run(kind, d, C, steps, gpu, orc)


@pytest.mark.parametrize("d,C", [(16, 999), (128, 300), (256, 257), (64, 70000), (64, 4097)])
def test_pooled_inplace_multistep(d, C, gpu, orc):
    """sample_ (amh_pooled_step, in place: in and out states alias) equals
    repeated out-of-place sample(); covers the large-d update's staging."""
    from kernels_amd import PooledARWMH, PRNGKey
    kw, mk, om = make_case("gaussian", d)
    z0 = torch.empty(C, d, device=gpu).uniform_(-2, 2)
    a = PooledARWMH(num_chains=C, **kw)
    sa = a.init(PRNGKey(4), 5, z0, (), mk)
    b = PooledARWMH(num_chains=C, **kw)
    sb = b.init(PRNGKey(4), 5, z0, (), mk)
    assert d <= 64 or torch.equal(sa.cov, sb.cov)
    a.sample_(sa, 12)
    for _ in range(12):
        sb = b.sample(sb)
    torch.cuda.synchronize()
    assert torch.equal(sa.z, sb.z) and torch.equal(sa.adapt_state.scale, sb.adapt_state.scale)
    assert torch.equal(sa.cov, sb.cov) and int(sa.i[0]) == 12
    assert torch.equal(sa.adapt_state.loc, sb.adapt_state.loc) and torch.equal(sa.as_change, sb.as_change)


@pytest.mark.parametrize("C,K,n", [(70000, 1, 3), (70000, 4, 8), (3000, 1, 5), (4097, 2, 6)])
def test_pooled64_inplace_vs_oracle(C, K, n, gpu, orc):
    """d = 64 in place (amh_pooled_step_k with the fused stats kernel and the
    update launch that folds in the last step's chunk reduction: reduce blocks
    write their sums write-through, take an agent-scope ticket, the last
    arriver runs the update, accumulating over the K steps of a block).  C =
    70,000 gives 547 chunks = 35 reduce groups (> 16).  Per-chain state, the
    last block's sums (k._sums) and the shared state bit for bit against the
    oracle's n / K blocks, and against n / K out-of-place sample() calls."""
    from kernels_amd import PooledARWMH, PRNGKey
    kw, mk, om = make_case("gaussian", 64)
    z0 = np.random.default_rng(11).uniform(-2, 2, size=(C, 64)).astype(np.float32)
    a = PooledARWMH(num_chains=C, sync_every=K, **kw)
    sa = a.init(PRNGKey(11), 0, torch.as_tensor(z0), (), mk)
    b = PooledARWMH(num_chains=C, sync_every=K, **kw)
    sb = b.init(PRNGKey(11), 0, torch.as_tensor(z0), (), mk)
    a.sample_(sa, n)
    for _ in range(n // K):
        sb = b.sample(sb)
    ost = orc.init(om, PRNGKey(11), C, init_z=z0)
    z, pe, keys = ost.z, ost.potential_energy, ost.rng_key
    sh = orc.pooled_init_shared(64)
    for _ in range(n // K):
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]),
                                       k_steps=K)
        orc.pooled_update(om, sums, sh, k_steps=K)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(a._sums.cpu().numpy().view(np.uint64), sums.view(np.uint64))
    np.testing.assert_array_equal(b._sums.cpu().numpy().view(np.uint64), sums.view(np.uint64))
    for st in (sa, sb):
        got = dict(z=st.z, pe=st.potential_energy, mu=st.adapt_state.loc, L=st.adapt_state.scale,
                   lam=st.adapt_state.log_step_size, macc=st.mean_accept_prob, asc=st.as_change, cov=st.cov, i=st.i)
        want = dict(z=z, pe=pe, mu=sh["mu"], L=sh["L"], lam=sh["lam"], macc=sh["macc"], asc=sh["asc"],
                    cov=sh["cov"], i=sh["i"])
        for f in got:
            g = got[f].cpu().numpy()
            assert g.tobytes() == np.asarray(want[f]).astype(g.dtype).tobytes(), f"{f} differs (C={C} K={K})"
    assert int(sa.i[0]) == n


@pytest.mark.parametrize("kind,d,C,blocks,K", [("gaussian", 64, 3000, 3, 4), ("gaussian", 64, 70000, 2, 16),
                                               ("gaussian", 7, 517, 3, 5), ("eight_schools", None, 64, 3, 16),
                                               ("diamonds", None, 40, 2, 3), ("diamonds_ss", None, 1000, 2, 4),
                                               ("gaussian", 128, 700, 2, 3),
                                               ("gaussian", 256, 600, 2, 2)])
def test_pooled_blocks_bitexact(kind, d, C, blocks, K, gpu, orc):
    """sync_every = K (one update per K transitions): per-chain state, the
    block's sums and the shared state bit for bit against orc_pooled_*_k."""
    _run(kind, d, C, blocks, gpu, orc, K=K)


@pytest.mark.parametrize("d,C,K", [(16, 999, 4), (128, 300, 3), (64, 70000, 4), (64, 70000, 1),
                                   (96, 300, 4), (160, 260, 3), (224, 200, 2)])
def test_pooled_blocks_inplace(d, C, K, gpu, orc):
    """sample_(12) with sync_every = K in place (amh_pooled_step_k) equals
    12 / K out-of-place block samples."""
    from kernels_amd import PooledARWMH, PRNGKey
    kw, mk, om = make_case("gaussian", d)
    z0 = torch.empty(C, d, device=gpu).uniform_(-2, 2)
    a = PooledARWMH(num_chains=C, sync_every=K, **kw)
    sa = a.init(PRNGKey(4), 0, z0, (), mk)
    b = PooledARWMH(num_chains=C, sync_every=K, **kw)
    sb = b.init(PRNGKey(4), 0, z0, (), mk)
    a.sample_(sa, 12)
    for _ in range(12 // K):
        sb = b.sample(sb)
    torch.cuda.synchronize()
    assert int(sa.i[0]) == 12 and int(sb.i[0]) == 12
    assert torch.equal(sa.z, sb.z) and torch.equal(sa.adapt_state.scale, sb.adapt_state.scale)
    assert torch.equal(sa.cov, sb.cov) and torch.equal(sa.adapt_state.loc, sb.adapt_state.loc)
    if K > 1:
        with pytest.raises(ValueError):
            a.sample_(sa, 5 if K != 5 else 7)


@pytest.mark.parametrize("kind,d,C,blocks,K", [("gaussian", 64, 3000, 5, 1), ("gaussian", 64, 2000, 4, 4),
                                               ("eight_schools", None, 64, 5, 2), ("gaussian", 128, 300, 3, 1)])
def test_pooled_overlap_bitexact(kind, d, C, blocks, K, gpu, orc):
    """overlap = True (lag-one pooling, the all-reduce in flight while the next
    block computes): theta_{b+1} = update(theta_b, sums_{b-1}), theta_1 =
    theta_0, bit for bit against the oracle's stats / update in that order;
    the last block's sums stay pending and are applied by the next call."""
    from kernels_amd import PooledARWMH, PRNGKey
    kw, mk, om = make_case(kind, d)
    k = PooledARWMH(num_chains=C, sync_every=K, overlap=True, **kw)
    z0 = np.random.default_rng(3).uniform(-2, 2, size=(C, om.d)).astype(np.float32)
    st = k.init(PRNGKey(3), 0, torch.as_tensor(z0), (), mk)
    ost = orc.init(om, PRNGKey(3), C, init_z=z0)
    z, pe, keys = ost.z, ost.potential_energy, ost.rng_key
    sh = orc.pooled_init_shared(om.d)
    pending = None
    for b in range(blocks):
        st = k.sample(st) if b % 2 == 0 else k.sample_(st, K)
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]),
                                       k_steps=K)
        if pending is None:
            sh["i"] += K
        else:
            orc.pooled_update(om, pending, sh, k_steps=K)
        pending = sums
        torch.cuda.synchronize()
        got = dict(z=st.z, pe=st.potential_energy, mu=st.adapt_state.loc, L=st.adapt_state.scale,
                   lam=st.adapt_state.log_step_size, macc=st.mean_accept_prob, cov=st.cov, i=st.i)
        want = dict(z=z, pe=pe, mu=sh["mu"], L=sh["L"], lam=sh["lam"], macc=sh["macc"], cov=sh["cov"], i=sh["i"])
        for f in got:
            a_, b_ = got[f].cpu().numpy(), np.asarray(want[f])
            assert a_.tobytes() == b_.astype(a_.dtype).tobytes(), f"{kind} {f} differs at block {b + 1}"
    # run() (draws at block ends) continues the same recurrence
    st2, cz, cp = k.run(st, 2 * K, thinning=K, collect_z=True, collect_pe=True)
    for t in range(2):
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]),
                                       k_steps=K)
        orc.pooled_update(om, pending, sh, k_steps=K)
        pending = sums
        torch.cuda.synchronize()
        assert cz[t].cpu().numpy().tobytes() == z.tobytes() and cp[t].cpu().numpy().tobytes() == pe.tobytes()
    assert st2.adapt_state.scale.cpu().numpy().tobytes() == sh["L"].tobytes()


def test_pooled_run_matches_sample(gpu):
    """PooledARWMH.run (collect at block ends) equals sample_ block by block."""
    import posteriors as P
    from kernels_amd import PooledARWMH, PRNGKey
    g = P.correlated_gaussian(16)
    z0 = torch.empty(500, 16, device=gpu).uniform_(-2, 2)
    a = PooledARWMH(potential_fn=g, num_chains=500, sync_every=2)
    sa = a.init(PRNGKey(1), 0, z0, (), {})
    b = PooledARWMH(potential_fn=g, num_chains=500, sync_every=2)
    sb = b.init(PRNGKey(1), 0, z0, (), {})
    out, cz, cp = a.run(sa, 13 * 2, thinning=4, collect_z=True, collect_pe=True)
    assert cz.shape == (6, 500, 16) and cp.shape == (6, 500)
    for t in range(6):
        b.sample_(sb, 4)
        assert torch.equal(cz[t], sb.z) and torch.equal(cp[t], sb.potential_energy)
    b.sample_(sb, 2)
    torch.cuda.synchronize()
    assert torch.equal(out.z, sb.z) and torch.equal(out.adapt_state.scale, sb.adapt_state.scale)
    assert int(out.i[0]) == 26 and int(sa.i[0]) == 0  # run() leaves its input alone
    with pytest.raises(ValueError):
        a.run(sa, 4, thinning=3)


def _gpu_worker(rank, world, port, C, steps, out_path, d=32, K=1, overlap=False):
    import os
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)  # the ranks share the box's one GPU
    import posteriors as P
    from kernels_amd import PooledARWMH, PRNGKey
    from kernels_amd.distributed import gather_chains, shard_range
    g = P.correlated_gaussian(d)
    off, cnt = shard_range(C, rank, world)
    z0 = torch.as_tensor(np.random.default_rng(0).uniform(-2, 2, size=(C, d)).astype(np.float32))
    k = PooledARWMH(potential_fn=g, num_chains=cnt, chain_offset=off, device=torch.device("cuda", 0),
                    sync_every=K, overlap=overlap)
    st = k.init(PRNGKey(2), 0, z0[off:off + cnt].cuda(), (), {})
    k.sample_(st, steps)
    z = gather_chains(st.z.cpu(), C)
    if rank == 0:
        np.savez(out_path, z=z.numpy(), L=st.adapt_state.scale.cpu().numpy(), i=st.i.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("d,C,steps,K,overlap,world", [(32, 2001, 25, 1, False, 2), (64, 3001, 12, 1, False, 2),
                                                       (64, 3001, 16, 4, False, 3), (64, 2001, 12, 1, True, 2),
                                                       (64, 2001, 16, 4, True, 2)])
def test_pooled_two_ranks(d, C, steps, K, overlap, world, gpu, tmp_path):
    """The distributed path of PooledARWMH (all-reduce of the sums every
    block; with overlap, lag-one pooling) over several ranks equals the
    1-rank run up to the association order of the sums (BASELINE config 5's
    d = 64 workload, at test size)."""
    import socket
    import torch.multiprocessing as mp
    import posteriors as P
    from kernels_amd import PooledARWMH, PRNGKey
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "g.npz")
    mp.start_processes(_gpu_worker, args=(world, port, C, steps, out, d, K, overlap), nprocs=world, join=True,
                       start_method="spawn")
    r = np.load(out)
    g = P.correlated_gaussian(d)
    z0 = torch.as_tensor(np.random.default_rng(0).uniform(-2, 2, size=(C, d)).astype(np.float32))
    k = PooledARWMH(potential_fn=g, num_chains=C, sync_every=K, overlap=overlap)
    st = k.init(PRNGKey(2), 0, z0.to(gpu), (), {})
    k.sample_(st, steps)
    assert int(r["i"][0]) == steps
    np.testing.assert_allclose(r["L"], st.adapt_state.scale.cpu().numpy(), rtol=1e-4, atol=1e-5)
    # a chain whose u sits within rounding of alpha may decide differently
    # under the other association order; allow a handful of such chains
    zd = np.abs(r["z"] - st.z.cpu().numpy()).max(axis=1) > 1e-4 * (1 + np.abs(r["z"]).max(axis=1))
    assert zd.sum() <= max(2, C // 1000), zd.sum()


@pytest.mark.parametrize("steps,K", [(6, 1), (48, 16)])
def test_config5_eight_ranks_full_shape(steps, K, gpu, tmp_path):
    """BASELINE configs[4] at its own shape: 8 ranks x 65,536 chains = 524,288,
    d = 64, pooled every step and every 16 steps.  The ranks share the box's
    one GPU and exchange over gloo (the RCCL path needs one GPU per rank);
    the result equals one process holding all 524,288 chains up to the
    association order of the all-reduced sums: L within rtol 1e-4, and at
    most C / 1000 chains whose accept decision flips."""
    test_pooled_two_ranks(64, 524288, steps, K, False, 8, gpu, tmp_path)


@pytest.mark.parametrize("d,C", [(64, 3000), (128, 700), (256, 300)])
def test_pooled_noise_ahead_invalidation(d, C, gpu, orc):
    """From d = 64 up the update launch draws the next step's noise ahead of
    time; each chain's record (i, key) decides whether the stats kernel may
    use it.  Editing the keys or the counter between steps must fall back to
    drawing, bit for bit against the oracle."""
    from kernels_amd import PooledARWMH, PRNGKey
    kw, mk, om = make_case("gaussian", d)
    k = PooledARWMH(num_chains=C, **kw)
    z0 = np.random.default_rng(9).uniform(-2, 2, size=(C, d)).astype(np.float32)
    st = k.init(PRNGKey(9), 0, torch.as_tensor(z0), (), mk)
    ost = orc.init(om, PRNGKey(9), C, init_z=z0)
    z, pe, keys = ost.z, ost.potential_energy, ost.rng_key.copy()
    sh = orc.pooled_init_shared(d)
    for t in range(6):
        if t == 2:  # rotate the keys of the first 37 chains in place
            kk = st.rng_key[:37].clone()
            st.rng_key[:37] = torch.roll(kk, 1, dims=0)
            keys[:37] = np.roll(keys[:37].copy(), 1, axis=0)
        if t == 4:  # rewind the shared counter: records of i + 1 no longer match
            st.i.sub_(1)
            sh["i"] = sh["i"] - 1
        st = k.sample(st)
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]))
        orc.pooled_update(om, sums, sh)
        torch.cuda.synchronize()
        assert st.z.cpu().numpy().tobytes() == z.tobytes(), f"z differs at step {t + 1}"
        assert st.adapt_state.scale.cpu().numpy().tobytes() == np.asarray(sh["L"]).tobytes(), f"L at step {t + 1}"
        assert st.as_change.cpu().numpy().tobytes() == np.asarray(sh["asc"]).astype(np.float32).tobytes()


@pytest.mark.parametrize("d,C", [(64, 500), (128, 300)])
def test_pooled_keep_factor_when_not_pd(d, C, gpu, orc):
    """The update's keep-L branch (arwmh.py:191) through the large-d path:
    after two steps the shared covariance is replaced by a negative one, so
    Sigma' is not positive definite and the factor and covariance are kept;
    as_change, mu, lambda still move.  d = 64 runs the update's in-block
    prep / post, d = 128 the all-CU prep / post kernels with the
    last-arriver as_change sum.  Bit for bit against the oracle."""
    from kernels_amd import PooledARWMH, PRNGKey
    kw, mk, om = make_case("gaussian", d)
    k = PooledARWMH(num_chains=C, **kw)
    z0 = np.random.default_rng(5).uniform(-2, 2, size=(C, d)).astype(np.float32)
    st = k.init(PRNGKey(5), 0, torch.as_tensor(z0), (), mk)
    ost = orc.init(om, PRNGKey(5), C, init_z=z0)
    z, pe, keys = ost.z, ost.potential_energy, ost.rng_key
    sh = orc.pooled_init_shared(d)
    for t in range(4):
        if t == 2:
            neg = -1000.0 * np.asarray(sh["cov"])
            st.cov.copy_(torch.as_tensor(neg))
            sh["cov"] = neg.copy()
        L_before = np.asarray(sh["L"]).copy()
        st = k.sample(st)
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]))
        orc.pooled_update(om, sums, sh)
        torch.cuda.synchronize()
        if t == 2:
            assert np.array_equal(np.asarray(sh["L"]), L_before), "oracle did not keep the factor"
        for name, a, b in (("z", st.z, z), ("L", st.adapt_state.scale, sh["L"]), ("cov", st.cov, sh["cov"]),
                           ("mu", st.adapt_state.loc, sh["mu"]), ("asc", st.as_change, sh["asc"]),
                           ("lam", st.adapt_state.log_step_size, sh["lam"])):
            a = a.cpu().numpy()
            assert a.tobytes() == np.asarray(b).astype(a.dtype).tobytes(), f"{name} differs at step {t + 1}"


@pytest.mark.parametrize("K", [1, 16])
def test_rccl_branch_one_rank_bitexact(K):
    """The RCCL exchange in a 1-rank `nccl` group, forced on one GPU: RCCL on
    the compute stream (pooled.py _allreduce, distributed.rccl_allreduce_sum)
    and through torch.distributed's side stream are both bit-equal to the
    fused one-rank path, per step and with sync_every = 16
    (tools/rccl_one_rank.py, its own process so this process keeps no process
    group)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run([sys.executable, os.path.join(root, "tools", "rccl_one_rank.py"), "65536", "64",
                        "20" if K == 1 else "32", str(K)], capture_output=True, text=True, timeout=240, env=env)
    print(r.stdout[-2000:], r.stderr[-2000:])
    assert r.returncode == 0
    assert "bit-equal to the fused path" in r.stdout


def test_pooled_rejects_unsupported_large_d(gpu):
    """d > 64 off the 32-multiples binds (regime A, sample_Pnx and ASSS take
    any d up to 256), but the pooled mode's MFMA tiles need d % 32 == 0:
    PooledARWMH.init raises ValueError, and the C entry itself returns
    AMH_EINVAL instead of running the d <= 64 kernels."""
    import ctypes
    from kernels_amd import ARWMH, PooledARWMH, PRNGKey, _lib
    from kernels_amd._lib import AmhError
    kw, mk, om = make_case("gaussian", 100)
    z0 = torch.as_tensor(np.random.default_rng(0).uniform(-2, 2, size=(64, 100)).astype(np.float32))
    with pytest.raises(ValueError, match="pooled mode"):
        PooledARWMH(num_chains=64, **kw).init(PRNGKey(0), 0, z0, (), mk)
    k = ARWMH(num_chains=64, **kw)  # a handle bound to d = 100, driven through the pooled C entry
    st = k.init(PRNGKey(0), 0, z0, (), mk)
    dev = st.z.device
    cov = torch.zeros(100 * 101 // 2, dtype=torch.float64, device=dev)
    one = torch.zeros(1, dtype=torch.float32, device=dev)
    ps = _lib.AmhPooledState(torch.zeros(1, dtype=torch.int32, device=dev).data_ptr(), st.z.data_ptr(),
                             st.potential_energy.data_ptr(), st.rng_key.data_ptr(), one.data_ptr(),
                             st.adapt_state.loc.data_ptr(), st.adapt_state.scale.data_ptr(), one.data_ptr(),
                             one.data_ptr(), cov.data_ptr())
    zo, po = torch.empty_like(st.z), torch.empty_like(st.potential_energy)
    sums = torch.zeros(100 + 5050 + 2, dtype=torch.float64, device=dev)
    rc = _lib.lib().amh_pooled_stats(k._handle.h, 64, ctypes.byref(ps), _lib.ptr(zo), _lib.ptr(po), _lib.ptr(sums),
                                     _lib.stream_ptr(dev.index))
    with pytest.raises(AmhError, match="d % 32 == 0"):
        _lib.check(rc, k._handle.h)
