"""The pooled exchange's own RCCL communicator (kernels_amd/distributed.py
RcclComm) on the CPU: the unique id is made on the group's first rank and
reaches every rank intact over gloo (world 2 and 3); RCCL error results
raise RcclError instead of being retried elsewhere; a process without RCCL
mapped fails setup with OSError, which is the only case PooledARWMH turns
into torch's stream.  Communicator creation and the collective itself need a
GPU (tests/test_gpu_pooled.py::test_rccl_branch_one_rank_bitexact)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _uid_worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from kernels_amd.distributed import rccl_unique_id
    a = rccl_unique_id()
    b = rccl_unique_id()  # a second id: a fresh one, not a cached copy
    np.save(os.path.join(out_dir, f"uid{rank}.npy"), np.frombuffer(a + b, dtype=np.uint8))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_unique_id_broadcast(tmp_path, world):
    mp.start_processes(_uid_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    ids = [np.load(tmp_path / f"uid{r}.npy") for r in range(world)]
    assert all(i.size == 256 for i in ids)
    for i in ids[1:]:
        assert i.tobytes() == ids[0].tobytes()
    a, b = ids[0][:128], ids[0][128:]
    assert a.any() and b.any() and a.tobytes() != b.tobytes()


class _FakeLib:
    """Stands in for librccl: every entry point returns `rc`."""

    def __init__(self, rc):
        self.rc = rc
        self.calls = []

    def ncclAllReduce(self, *a):
        self.calls.append("ncclAllReduce")
        return self.rc

    def ncclGetErrorString(self, rc):
        return b"unhandled system error"


def test_allreduce_error_raises(monkeypatch):
    import kernels_amd.distributed as D
    fake = _FakeLib(2)
    monkeypatch.setattr(D, "_rccl_lib", lambda: fake)

    class _T:  # a device tensor's surface, no GPU needed
        dtype = torch.float64
        is_cuda = True

        def is_contiguous(self):
            return True

        def data_ptr(self):
            return 4096

        def numel(self):
            return 17

    class _S:
        cuda_stream = 0

    with pytest.raises(D.RcclError, match="ncclAllReduce: unhandled system error"):
        D.rccl_allreduce_sum(_T(), comm=1234, stream=_S())
    assert fake.calls == ["ncclAllReduce"]  # issued once, never retried
    fake.rc = 0
    D.rccl_allreduce_sum(_T(), comm=1234, stream=_S())
    with pytest.raises(ValueError):
        D.rccl_allreduce_sum(torch.zeros(3), comm=1234, stream=_S())  # host tensor


def test_no_rccl_mapped_is_oserror(monkeypatch):
    import builtins
    import kernels_amd.distributed as D
    monkeypatch.setattr(D, "_rccl", None)
    real_open = builtins.open

    def fake_open(p, *a, **k):
        if p == "/proc/self/maps":
            import io
            return io.StringIO("00400000-00452000 r-xp 00000000 08:02 173521 /usr/bin/python3\n")
        return real_open(p, *a, **k)

    monkeypatch.setattr(builtins, "open", fake_open)
    with pytest.raises(OSError):
        D._rccl_lib()


def test_pooled_allreduce_error_propagates(monkeypatch):
    """PooledARWMH._allreduce does not swallow an RCCL error: it
    reaches the caller, and the sampler is not switched to another path."""
    import kernels_amd.distributed as D
    import kernels_amd.pooled as PM
    import posteriors as P

    class _Comm:
        def __init__(self, group, device):
            pass

        def all_reduce_sum(self, buf, stream, handle=None):
            raise D.RcclError("ncclAllReduce: remote process exited (ncclResult 6)")

    monkeypatch.setattr(D, "RcclComm", _Comm)
    k = PM.PooledARWMH(potential_fn=P.correlated_gaussian(4), num_chains=8, device=torch.device("cpu"))
    monkeypatch.setattr(k, "_world", lambda: 2)
    monkeypatch.setattr(PM.dist, "get_backend", lambda group=None: "nccl")
    monkeypatch.setattr(PM.torch.cuda, "current_stream", lambda dev=None: None)
    with pytest.raises(D.RcclError):
        k._allreduce(torch.zeros(4, dtype=torch.float64), 0)
    assert k.torch_stream_collective is False
