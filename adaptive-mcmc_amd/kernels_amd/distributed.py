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
# against a 17 KB message.  RcclComm is a communicator of this package's own
# -- ncclGetUniqueId on the group's first rank, the 128-byte id broadcast over
# torch.distributed, ncclCommInitRank on every rank -- in the RCCL library
# torch already mapped (one RCCL instance per process), and its all_reduce is
# enqueued on the caller's stream, so the update kernel follows the collective
# in stream order with no event.  It never shares a communicator with torch's
# own collectives (barrier, max_over_ranks, gather_chains), which keep torch's.
_NCCL_DTYPE = {torch.float64: 8, torch.float32: 7, torch.int32: 2, torch.int64: 4}
_NCCL_SUM = 0
_NCCL_ID_BYTES = 128
_rccl = None


class RcclError(RuntimeError):
    """An RCCL call returned an error (after a collective may have been issued:
    never retried or routed elsewhere, since the ranks would disagree)."""


def _rccl_lib():
    global _rccl
    if _rccl is None:
        import ctypes
        path = None
        try:  # the librccl torch mapped (the same library instance torch uses)
            with open("/proc/self/maps") as f:
                for line in f:
                    p = line.split()[-1] if line.split() else ""
                    if "librccl.so" in p:
                        path = p
                        break
        except OSError:
            pass
        if path is None:
            raise OSError("librccl is not mapped into this process (torch without RCCL?)")
        L = ctypes.CDLL(path)
        L.ncclGetUniqueId.argtypes = [ctypes.c_void_p]
        L.ncclGetUniqueId.restype = ctypes.c_int
        L.ncclCommInitRank.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int, _UniqueId, ctypes.c_int]
        L.ncclCommInitRank.restype = ctypes.c_int
        L.ncclCommDestroy.argtypes = [ctypes.c_void_p]
        L.ncclCommDestroy.restype = ctypes.c_int
        L.ncclAllReduce.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                    ctypes.c_void_p, ctypes.c_void_p]
        L.ncclAllReduce.restype = ctypes.c_int
        L.ncclGetErrorString.argtypes = [ctypes.c_int]
        L.ncclGetErrorString.restype = ctypes.c_char_p
        _rccl = L
    return _rccl


def _uid_type():
    import ctypes

    class UniqueId(ctypes.Structure):  # ncclUniqueId: 128 opaque bytes, passed by value
        _fields_ = [("internal", ctypes.c_char * _NCCL_ID_BYTES)]
    return UniqueId


_UniqueId = _uid_type()


def _check(L, rc: int, what: str):
    if rc != 0:
        raise RcclError(f"{what}: {L.ncclGetErrorString(rc).decode()} (ncclResult {rc})")


def rccl_unique_id(group=None, device=None) -> bytes:
    """ncclGetUniqueId on the group's first rank, broadcast to every rank of
    the group over torch.distributed (gloo or nccl); returns the 128 bytes."""
    import ctypes
    rank = dist.get_rank(group)
    raw = bytes(_NCCL_ID_BYTES)
    if rank == 0:
        L = _rccl_lib()
        uid = _UniqueId()
        _check(L, L.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
        raw = ctypes.string_at(ctypes.addressof(uid), _NCCL_ID_BYTES)
    on_dev = dist.get_backend(group) == "nccl"
    t = torch.tensor(list(raw), dtype=torch.uint8, device=device if on_dev else "cpu")
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast(t, src=src, group=group)
    return bytes(t.cpu().tolist())


class RcclComm:
    """A blocking RCCL communicator over the ranks of `group` (one GPU each),
    owned by this package (created here, destroyed by close()).

    all_reduce_sum enqueues ncclAllReduce on a given stream and raises
    RcclError on any non-success result -- there is no fallback once a
    collective may have been issued, because a rank that retried elsewhere
    would leave the others with a different collective count."""

    def __init__(self, group=None, device=None):
        import ctypes
        if not dist.is_initialized():
            raise RuntimeError("RcclComm needs an initialised torch.distributed group")
        dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        L = _rccl_lib()
        uid = _UniqueId()
        ctypes.memmove(ctypes.addressof(uid), rccl_unique_id(group, dev), _NCCL_ID_BYTES)
        comm = ctypes.c_void_p()
        with torch.cuda.device(dev.index):
            _check(L, L.ncclCommInitRank(ctypes.byref(comm), self.world, uid, self.rank), "ncclCommInitRank")
        self._ptr = comm.value

    @property
    def ptr(self) -> int:
        if self._ptr is None:
            raise RuntimeError("RcclComm is closed")
        return self._ptr

    def all_reduce_sum(self, buf: torch.Tensor, stream=None, handle=None):
        """In-place all_reduce(sum) of a contiguous device tensor on `stream`
        (default: the current stream of buf's device).  With a library
        `handle` (kernels_amd._lib.Handle) and float64 sums the call goes
        through the C ABI's amh_pooled_allreduce (include/amh.h), the entry a
        non-Python binding uses; otherwise through ctypes into librccl."""
        if handle is not None and buf.dtype == torch.float64 and buf.is_cuda and buf.is_contiguous():
            from . import _lib
            s = stream if stream is not None else torch.cuda.current_stream(buf.device)
            L = _lib.lib()
            rc = L.amh_pooled_allreduce(handle.h, buf.data_ptr(), buf.numel(), self.ptr, s.cuda_stream)
            if rc != 0:
                msg = L.amh_last_error(handle.h)
                raise RcclError(msg.decode() if msg else f"amh_pooled_allreduce: {rc}")
            return
        rccl_allreduce_sum(buf, self.ptr, stream)

    def close(self):
        """ncclCommDestroy (waits for this communicator's outstanding work)."""
        if self._ptr is not None:
            L = _rccl_lib()
            p, self._ptr = self._ptr, None
            with torch.cuda.device(self.device.index):
                _check(L, L.ncclCommDestroy(p), "ncclCommDestroy")


def rccl_allreduce_sum(buf: torch.Tensor, comm: int, stream=None):
    """In-place all_reduce(sum) of a contiguous device tensor, enqueued on
    `stream` (default: the current stream of buf's device) with RCCL on the
    blocking communicator `comm` (RcclComm.ptr).  Raises RcclError."""
    dt = _NCCL_DTYPE.get(buf.dtype)
    if dt is None or not buf.is_cuda or not buf.is_contiguous():
        raise ValueError("rccl_allreduce_sum: contiguous float64/float32/int device tensor expected")
    s = stream if stream is not None else torch.cuda.current_stream(buf.device)
    L = _rccl_lib()
    _check(L, L.ncclAllReduce(buf.data_ptr(), buf.data_ptr(), buf.numel(), dt, _NCCL_SUM, comm, s.cuda_stream),
           "ncclAllReduce")
