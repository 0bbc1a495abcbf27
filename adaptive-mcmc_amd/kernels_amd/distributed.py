"""Chain sharding across the GPUs of a node (one process per GPU).

Regime A (the reference's per-chain adaptation, arwmh.py:140-207) has no
data-path exchange: every chain is independent and its noise stream depends
only on (run key, global chain id), so rank r running chains
[offset_r, offset_r + count_r) with ARWMH(..., chain_offset=offset_r)
reproduces exactly those chains of a single-process run.  The only
collectives are the optional gathers of results/diagnostics below
(torch.distributed: RCCL over xGMI on GPUs, gloo on CPU).
"""
from __future__ import annotations

import os
from typing import Tuple

import torch
import torch.distributed as dist


def shard_range(num_chains: int, rank: int, world: int) -> Tuple[int, int]:
    """(offset, count) of rank's contiguous block of global chain ids; the
    first num_chains % world ranks get one extra chain."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of world {world}")
    if num_chains < 0:
        raise ValueError("num_chains must be >= 0")
    base, extra = divmod(num_chains, world)
    count = base + (1 if rank < extra else 0)
    offset = rank * base + min(rank, extra)
    return offset, count


def env_rank() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run env."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def init_process_group(backend: str = None):
    """Initialise the default group from the launcher's env (127.0.0.1
    rendezvous by default); 'nccl' (= RCCL) when a GPU is visible."""
    rank, world, local = env_rank()
    if world <= 1 or dist.is_initialized():
        return rank, world, local
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group(backend, device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(backend)
    return rank, world, local


def gather_chains(t: torch.Tensor, num_chains: int, group=None) -> torch.Tensor:
    """All-gather a per-chain tensor [count_r, ...] from every rank into the
    global [num_chains, ...] in global chain order (ragged shards padded)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return t
    world = dist.get_world_size(group)
    counts = [shard_range(num_chains, r, world)[1] for r in range(world)]
    m = max(counts)
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    outs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return torch.cat([o[:c] for o, c in zip(outs, counts)], dim=0)


def max_over_ranks(x: float, device=None, group=None) -> float:
    """max of a host scalar over ranks (bench timing)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


# ------------------------------------------------- RCCL on the compute stream --
# torch.distributed's nccl backend runs every collective on an internal stream
# of its own, fenced to the caller's stream by events in both directions.  On
# the pooled step's critical path (stats -> all_reduce -> update)
# those two cross-queue hops cost ~29 us on MI355X (profiles/r5a_rccl_trace.txt)
# against a 17 KB message.  rccl_allreduce_sum enqueues ncclAllReduce on the
# caller's stream instead, with the communicator torch created for the group
# (ProcessGroupNCCL._comm_ptr) and the RCCL library torch itself loaded, so
# the update kernel follows the collective in stream order with no event.
_NCCL_DTYPE = {torch.float64: 8, torch.float32: 7, torch.int32: 2, torch.int64: 4}
_NCCL_SUM = 0
_NCCL_IN_PROGRESS = 7  # ncclInProgress (non-blocking communicators)
_rccl = None


def _rccl_lib():
    global _rccl
    if _rccl is None:
        import ctypes
        path = None
        try:  # the librccl torch mapped (same library instance as the communicator)
            with open("/proc/self/maps") as f:
                for line in f:
                    p = line.split()[-1] if line.split() else ""
                    if "librccl.so" in p:
                        path = p
                        break
        except OSError:
            pass
        if path is None:
            raise RuntimeError("librccl is not loaded by torch (no nccl process group?)")
        L = ctypes.CDLL(path)
        L.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p]
        L.ncclAllReduce.restype = ctypes.c_int
        L.ncclGetErrorString.argtypes = [ctypes.c_int]
        L.ncclGetErrorString.restype = ctypes.c_char_p
        L.ncclCommGetAsyncError.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
        L.ncclCommGetAsyncError.restype = ctypes.c_int
        _rccl = L
    return _rccl


def rccl_comm_ptr(group, device: torch.device) -> int:
    """The ncclComm_t torch holds for `group` on `device` (initialised on
    first use by one collective through torch)."""
    pg = group if group is not None else dist.group.WORLD
    be = pg._get_backend(device)
    ptr = be._comm_ptr()
    if not ptr:
        t = torch.zeros(1, device=device)
        dist.all_reduce(t, group=group)  # creates the communicator
        torch.cuda.synchronize(device)
        ptr = be._comm_ptr()
    if not ptr:
        raise RuntimeError("no RCCL communicator for this group")
    return int(ptr)


def rccl_allreduce_sum(buf: torch.Tensor, comm: int, stream=None):
    """In-place all_reduce(sum) of a contiguous device tensor, enqueued on
    `stream` (default: the current stream of buf's device) with RCCL."""
    dt = _NCCL_DTYPE.get(buf.dtype)
    if dt is None or not buf.is_cuda or not buf.is_contiguous():
        raise ValueError("rccl_allreduce_sum: contiguous float64/float32/int device tensor expected")
    s = stream if stream is not None else torch.cuda.current_stream(buf.device)
    L = _rccl_lib()
    rc = L.ncclAllReduce(buf.data_ptr(), buf.data_ptr(), buf.numel(), dt, _NCCL_SUM, comm, s.cuda_stream)
    if rc == _NCCL_IN_PROGRESS:  # a non-blocking communicator: wait until the call is enqueued
        import ctypes
        st = ctypes.c_int(_NCCL_IN_PROGRESS)
        while st.value == _NCCL_IN_PROGRESS:
            rc = L.ncclCommGetAsyncError(comm, ctypes.byref(st))
            if rc != 0:
                break
        rc = rc or st.value
    if rc != 0:
        raise RuntimeError(f"ncclAllReduce: {L.ncclGetErrorString(rc).decode()}")
