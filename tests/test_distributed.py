"""Chain sharding (kernels_amd/distributed.py) with world_size 2 over gloo on the
CPU: shard ranges tile the global chain ids, and two ranks running their
shards with chain_offset reproduce the unsharded run bit for bit (the C
oracle stands in for the device step here; tests/test_gpu_parity.py checks
the device against the oracle, and test_sharded_equals_unsharded there)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from kernels_amd.distributed import shard_range


def test_shard_range_tiles():
    for C in (0, 1, 7, 101, 65536):
        for W in (1, 2, 3, 8):
            seen = []
            for r in range(W):
                off, cnt = shard_range(C, r, W)
                seen.extend(range(off, off + cnt))
            assert seen == list(range(C))
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, C, steps, out_path):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import orc
    from helpers import make_case
    from kernels_amd import PRNGKey
    from kernels_amd.distributed import gather_chains, max_over_ranks, shard_range
    _, _, om = make_case("gaussian", 8)
    off, cnt = shard_range(C, rank, world)
    st = orc.init(om, PRNGKey(7), cnt, chain_offset=off)
    orc.step(om, st, steps)
    z = gather_chains(torch.from_numpy(st.z), C)
    L = gather_chains(torch.from_numpy(st.scale), C)
    keys = gather_chains(torch.from_numpy(st.rng_key.view(np.int32)), C)
    m = max_over_ranks(float(rank))
    if rank == 0:
        np.savez(out_path, z=z.numpy(), L=L.numpy(), keys=keys.numpy(), m=m)
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_run_equals_unsharded(tmp_path, orc):
    from helpers import make_case
    from kernels_amd import PRNGKey
    C, steps = 101, 25
    out = str(tmp_path / "g.npz")
    mp.start_processes(_worker, args=(2, _free_port(), C, steps, out), nprocs=2, join=True, start_method="spawn")
    g = np.load(out)
    _, _, om = make_case("gaussian", 8)
    st = orc.init(om, PRNGKey(7), C)
    orc.step(om, st, steps)
    assert g["z"].tobytes() == st.z.tobytes()
    assert g["L"].tobytes() == st.scale.tobytes()
    assert g["keys"].view(np.uint32).tobytes() == st.rng_key.tobytes()
    assert float(g["m"]) == 1.0
