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
