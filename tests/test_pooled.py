"""Pooled-covariance mode (regime B, kernels_amd/pooled.py + orc_pooled_*) on
the CPU: the oracle's pooled step with ONE chain reproduces the reference
recurrence (golden vectors of the literal restatement), the pooled
adaptation converges to the target covariance with many chains, and a
2-rank gloo run with an all-reduce of the sums matches the single-process
run."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _unpack(p, d):
    L = np.zeros((d, d))
    k = 0
    for j in range(d):
        L[j:, j] = p[k:k + d - j]
        k += d - j
    return L


def test_layout(orc):
    assert orc.pooled_cpw(1) == 1 and orc.pooled_cpw(4096) == 1 and orc.pooled_cpw(4097) == 2
    assert orc.pooled_cpw(65536) == 16 and orc.pooled_cpw(10 ** 7) == 16


@pytest.mark.parametrize("name,model_id,d", [("eight_schools", 2, 10), ("gaussian64", 1, 64)])
def test_one_chain_is_the_reference_recurrence(name, model_id, d, orc):
    """N = 1: mu' = mu + gamma delta, Sigma' = (1-gamma) Sigma + gamma delta delta^T
    refactorised -- the reference's rank-one update (arwmh.py:188-191), so the
    pooled chain follows the golden trajectory of chain 0."""
    from test_golden import tol
    f = np.load(os.path.join(G, name + ".npz"))
    om = orc.Model(model_id, d, f["model_data"])
    z = f["init_z"][:1].copy()
    pe = orc.potential(om, z)
    keys = f["chain_keys"][:1].copy()
    sh = orc.pooled_init_shared(d)
    sh["mu"][:] = z[0]  # the reference starts mu at z0 (irrelevant after step 1: gamma_1 = 1)
    rec = {int(t): k for k, t in enumerate(f["steps_recorded"])}
    for t in range(f["accept"].shape[1]):
        zo, po, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]))
        accepted = not np.array_equal(zo, z)
        assert accepted == bool(f["accept"][0, t]), f"step {t + 1}"
        assert sums[-1] == 1.0
        z, pe = zo, po
        orc.pooled_update(om, sums, sh)
        if t + 1 in rec:
            k, tl = rec[t + 1], tol(t + 1)
            np.testing.assert_allclose(z[0], f["z"][k, 0], rtol=tl["z"][0], atol=tl["z"][1])
            np.testing.assert_allclose(sh["mu"], f["loc"][k, 0], rtol=tl["loc"][0], atol=tl["loc"][1])
            assert abs(sh["lam"][0] - f["lam"][k, 0]) <= tl["lam"]
            assert abs(sh["macc"][0] - f["macc"][k, 0]) <= tl["macc"]
            Lg = _unpack(f["scale"][k, 0], d)
            L1 = _unpack(sh["L"], d)
            assert np.max(np.abs(L1 @ L1.T - Lg @ Lg.T)) <= 1e-3 * np.max(np.abs(Lg @ Lg.T)) + 1e-5
            Sg = _unpack(sh["cov"], d)
            Sg = Sg + np.tril(Sg, -1).T
            assert np.max(np.abs(Sg - L1 @ L1.T)) <= 1e-5 * np.max(np.abs(Sg))


def test_pooled_adaptation_converges(orc):
    """512 chains on the 8-d correlated Gaussian: the shared factor tracks
    the target covariance after 300 pooled steps, acceptance near 0.234."""
    import posteriors as P
    d, C = 8, 512
    g = P.correlated_gaussian(d)
    om = orc.Model(orc.GAUSSIAN, d, g.pack("cpu")[0].numpy())
    st = orc.init(om, np.array([0, 5], np.uint32), C)
    z, pe, keys = st.z, st.potential_energy, st.rng_key
    sh = orc.pooled_init_shared(d)
    for _ in range(300):
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]))
        orc.pooled_update(om, sums, sh)
    L = _unpack(sh["L"], d)
    cov = np.linalg.inv(g.precision)
    assert np.linalg.norm(L @ L.T - cov) / np.linalg.norm(cov) < 0.15
    assert abs(float(sh["macc"][0]) - 0.234) < 0.05


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _pooled_worker(rank, world, port, C, steps, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import orc
    from helpers import make_case
    from kernels_amd import PRNGKey
    from kernels_amd.distributed import gather_chains, shard_range
    _, _, om = make_case("gaussian", 12)
    off, cnt = shard_range(C, rank, world)
    st = orc.init(om, PRNGKey(9), cnt, chain_offset=off)
    z, pe, keys = st.z, st.potential_energy, st.rng_key
    sh = orc.pooled_init_shared(om.d)
    for _ in range(steps):
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]))
        t = torch.from_numpy(sums.copy())
        dist.all_reduce(t)  # the step's only exchange
        orc.pooled_update(om, t.numpy(), sh)
    zall = gather_chains(torch.from_numpy(z), C).numpy()
    if rank == 0:
        np.savez(out_path, z=zall, L=sh["L"], mu=sh["mu"], lam=sh["lam"], i=sh["i"])
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_match_one(tmp_path, orc):
    from helpers import make_case
    from kernels_amd import PRNGKey
    C, steps = 301, 40
    out = str(tmp_path / "p.npz")
    mp.start_processes(_pooled_worker, args=(2, _free_port(), C, steps, out), nprocs=2, join=True,
                       start_method="spawn")
    g = np.load(out)
    _, _, om = make_case("gaussian", 12)
    st = orc.init(om, PRNGKey(9), C)
    z, pe, keys = st.z, st.potential_energy, st.rng_key
    sh = orc.pooled_init_shared(om.d)
    for _ in range(steps):
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]))
        orc.pooled_update(om, sums, sh)
    assert int(g["i"][0]) == steps
    # the sums differ only in association order (two partial sums vs one)
    np.testing.assert_allclose(g["mu"], sh["mu"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(g["L"], sh["L"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(g["z"], z, rtol=1e-4, atol=1e-4)


@pytest.mark.parametrize("d", [128, 256])
def test_one_chain_big_is_the_reference_recurrence(d, orc):
    """Large-d pooled spec (float32 refactorisation, MFMA-order proposal and
    potential) with ONE chain against the literal float64 restatement of
    ARWMH.sample driven by the same noise, 40 steps (W = 10 covers the
    gamma_1 = 1 keep-L quirk twice)."""
    import arwmh_np as lit
    import posteriors as P
    from kernels_amd import PRNGKey
    g = P.correlated_gaussian(d)
    data, _ = g.pack("cpu")
    om = orc.Model(orc.GAUSSIAN, d, data.numpy())
    m, Pm, c0 = (data.numpy().astype(np.float64)[:d], data.numpy().astype(np.float64)[d:d + d * d].reshape(d, d),
                 float(data[d + d * d]))
    U = lambda z: lit.gaussian_potential(z, m, Pm, c0)  # noqa: E731
    keys = orc.chain_keys(PRNGKey(5), 0, 1)
    z = np.random.default_rng(d).uniform(-2, 2, size=(1, d)).astype(np.float32)
    pe = orc.potential(om, z)
    sh = orc.pooled_init_shared(d)
    sh["mu"][:] = z[0]
    W = 10
    ref = lit.ARWMHState(0, z[0].astype(np.float64), float(pe[0]), 0.0,
                         lit.ARWMHAdaptState(z[0].astype(np.float64), np.eye(d), 0.0), 0.0, None)
    for t in range(40):
        bits, ubits = lit.step_noise(keys, int(sh["i"][0]), d)
        xi, u = lit.normal_from_bits(bits[0]), float(lit.unif01_from_bits(ubits[0]))
        zo, po, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]))
        ref, acc, alpha = lit.sample(ref, U, xi, u, num_warmup=W)
        assert (not np.array_equal(zo, z)) == bool(acc), f"step {t + 1}"
        z, pe = zo, po
        orc.pooled_update(om, sums, sh, num_warmup=W)
        np.testing.assert_allclose(z[0], ref.z, rtol=1e-4, atol=1e-4)
        np.testing.assert_allclose(sh["mu"], ref.adapt_state.loc, rtol=1e-4, atol=1e-4)
        assert abs(sh["lam"][0] - ref.adapt_state.log_step_size) < 1e-4
        L1 = _unpack(sh["L"], d)
        Lr = ref.adapt_state.scale
        assert np.max(np.abs(L1 @ L1.T - Lr @ Lr.T)) <= 1e-3 * np.max(np.abs(Lr @ Lr.T)) + 1e-5, f"step {t + 1}"


# ------------------------------------------------ pool every K (sync_every) --
def _shared_copy(sh):
    return {k: v.copy() for k, v in sh.items()}


@pytest.mark.parametrize("kind,d,C,K", [("gaussian", 12, 37, 4), ("eight_schools", None, 70, 3),
                                        ("gaussian", 128, 40, 3), ("gaussian", 64, 300, 5)])
def test_block_is_k_frozen_steps(kind, d, C, K, orc):
    """A block of K transitions (orc_pooled_stats_k) is K single pooled steps
    with the shared state frozen: per-chain z / pe bit for bit, the sums equal
    up to association order (d < 64: one float32 accumulator per wave over
    all K steps; d = 64: one per 128-chain chunk over (sub-chunk, step, chain),
    orc_pooled_stats64_k; d > 64: the per-step sums added in step order,
    exactly)."""
    from helpers import make_case
    from kernels_amd import PRNGKey
    _, _, om = make_case(kind, d)
    st = orc.init(om, PRNGKey(3), C)
    z, pe, keys = st.z, st.potential_energy, st.rng_key
    sh = orc.pooled_init_shared(om.d)
    for _ in range(3):  # move off the identity first
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]))
        orc.pooled_update(om, sums, sh)
    i0 = int(sh["i"][0])
    zb, peb, sb = orc.pooled_stats(om, i0, z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]), k_steps=K)
    tot = None
    for t in range(K):
        z, pe, s = orc.pooled_stats(om, i0 + t, z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]))
        tot = s.copy() if tot is None else tot + s
    assert zb.tobytes() == z.tobytes() and peb.tobytes() == pe.tobytes()
    assert sb[-1] == K * C
    if om.d > 64:
        assert sb.tobytes() == tot.tobytes()
    else:
        np.testing.assert_allclose(sb, tot, rtol=2e-5, atol=1e-6 * np.abs(tot).max())


def test_block_update_counts_blocks(orc):
    """update_k: i advances by K; gamma = 1/n^a with n the block count
    (i / K + 1), reset at num_warmup; K = 1 is the per-step rule."""
    from helpers import make_case
    from kernels_amd import PRNGKey
    K, W, C, a = 4, 8, 50, 2 / 3
    _, _, om = make_case("gaussian", 6)
    st = orc.init(om, PRNGKey(1), C)
    z, pe, keys = st.z, st.potential_energy, st.rng_key
    sh = orc.pooled_init_shared(om.d)
    for blk in range(4):
        i = int(sh["i"][0])
        n = (i // K + 1) if i < W else ((i - W) // K + 1)
        z, pe, sums = orc.pooled_stats(om, i, z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]), k_steps=K)
        before = _shared_copy(sh)
        orc.pooled_update(om, sums, sh, num_warmup=W, k_steps=K)
        assert int(sh["i"][0]) == i + K
        gamma = float(orc.lr_gamma([n], a)[0])
        mu = before["mu"] + np.float32(gamma) * (sums[:6] / sums[-1]).astype(np.float32)
        np.testing.assert_array_equal(sh["mu"], mu)
        P = 21
        S = (1 - gamma) * before["cov"] + gamma * (sums[6:6 + P] / sums[-1])
        np.testing.assert_allclose(sh["cov"], S, rtol=1e-12)
    assert int(sh["i"][0]) == 4 * K


def _pooled_block_worker(rank, world, port, C, steps, K, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import orc
    from helpers import make_case
    from kernels_amd import PRNGKey
    from kernels_amd.distributed import gather_chains, shard_range
    _, _, om = make_case("gaussian", 12)
    off, cnt = shard_range(C, rank, world)
    st = orc.init(om, PRNGKey(9), cnt, chain_offset=off)
    z, pe, keys = st.z, st.potential_energy, st.rng_key
    sh = orc.pooled_init_shared(om.d)
    for _ in range(steps // K):
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]),
                                       k_steps=K)
        t = torch.from_numpy(sums.copy())
        dist.all_reduce(t)  # one exchange per K transitions
        orc.pooled_update(om, t.numpy(), sh, k_steps=K)
    zall = gather_chains(torch.from_numpy(z), C).numpy()
    if rank == 0:
        np.savez(out_path, z=zall, L=sh["L"], mu=sh["mu"], i=sh["i"])
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_match_one_blocks(tmp_path, orc):
    """sync_every = 4 over 2 gloo ranks (one all-reduce per block) equals the
    single-process block run up to the association order of the sums."""
    from helpers import make_case
    from kernels_amd import PRNGKey
    C, steps, K = 301, 40, 4
    out = str(tmp_path / "pb.npz")
    mp.start_processes(_pooled_block_worker, args=(2, _free_port(), C, steps, K, out), nprocs=2, join=True,
                       start_method="spawn")
    g = np.load(out)
    _, _, om = make_case("gaussian", 12)
    st = orc.init(om, PRNGKey(9), C)
    z, pe, keys = st.z, st.potential_energy, st.rng_key
    sh = orc.pooled_init_shared(om.d)
    for _ in range(steps // K):
        z, pe, sums = orc.pooled_stats(om, int(sh["i"][0]), z, pe, keys, sh["mu"], sh["L"], float(sh["lam"][0]),
                                       k_steps=K)
        orc.pooled_update(om, sums, sh, k_steps=K)
    assert int(g["i"][0]) == steps
    np.testing.assert_allclose(g["mu"], sh["mu"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(g["L"], sh["L"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(g["z"], z, rtol=1e-4, atol=1e-4)


def test_sync_every_argument_checks():
    from kernels_amd import PooledARWMH
    import posteriors as P
    with pytest.raises(ValueError):
        PooledARWMH(potential_fn=P.correlated_gaussian(4), num_chains=8, sync_every=0)
    k = PooledARWMH(potential_fn=P.correlated_gaussian(4), num_chains=8, sync_every=4)
    with pytest.raises(ValueError):
        k.init(np.array([0, 1], np.uint32), 6, None, (), {})
