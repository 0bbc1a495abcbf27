"""Pooled-covariance mode (regime B, kernels/pooled.py + orc_pooled_*) on
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
    from kernels import PRNGKey
    from kernels.distributed import gather_chains, shard_range
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
    from kernels import PRNGKey
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
    from kernels import PRNGKey
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
