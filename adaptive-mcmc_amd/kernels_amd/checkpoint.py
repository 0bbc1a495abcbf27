"""Checkpoint / resume of chain-major device states.

The reference pickles whole runs per seed and resumes by skipping finished
ones (`run_eight_schools_lr_decay.py:63-67`, `run_diamonds_lr_decay.py:55-56`).
Here a state is a namedtuple of torch tensors with a leading chain axis, and a
transition is a pure function of (kernel configuration, state): the noise of
step i is Philox(i, chain key), so saving the state and stepping a fresh
kernel of the same configuration from the loaded copy continues the run bit
for bit (tests/test_gpu_drivers.py).

    sd = state_dict(state)            # {"z": ndarray, "adapt_state.loc": ..., "__kind__": ...}
    state = load_state_dict(sd, dev)  # the same namedtuple on `dev`
    save_state("run.npz", state)      # numpy .npz, no pickles
    state = load_state("run.npz", dev)

A PooledARWMH with overlap=True keeps the all-reduced sums of its last block
pending in the sampler (they update the shared state at the start of the next
block).  Pass the kernel (`state_dict(state, kernel)`, `save_state(path,
state, kernel=k)`) to store them, and the kernel that continues the run to
`load_state_dict` / `load_state`, which hands them back to it; a checkpoint
with pending sums refuses to load without one.

`load_state` reads with numpy's default `allow_pickle=False`, so a file only
ever yields arrays.  ARWMHState, ASSSState and PooledState are supported.
"""
from __future__ import annotations

import numpy as np
import torch

from .arwmh import ARWMHAdaptState, ARWMHState
from .asss import ASSSAdaptState, ASSSState
from .pooled import PooledAdaptState, PooledState

_KINDS = {
    "ARWMHState": (ARWMHState, ARWMHAdaptState),
    "ASSSState": (ASSSState, ASSSAdaptState),
    "PooledState": (PooledState, PooledAdaptState),
}
PENDING = "__pooled_pending_sums__"


def state_dict(state, kernel=None) -> dict:
    """Flatten a state into {field path: host ndarray} plus its kind (and,
    for an overlap PooledARWMH `kernel`, the sums still pending for it)."""
    kind = type(state).__name__
    if kind not in _KINDS:
        raise TypeError(f"unsupported state type {kind}")
    out = {"__kind__": np.array(kind)}
    for name, v in zip(state._fields, state):
        if name == "adapt_state":
            for an, av in zip(v._fields, v):
                out[f"adapt_state.{an}"] = av.detach().cpu().numpy()
        else:
            out[name] = v.detach().cpu().numpy()
    if kernel is not None and getattr(kernel, "overlap", False):
        last = kernel._last_out() if kernel._last_out is not None else None
        pend = kernel.pending_sums() if last is state.z else None
        if pend is not None:
            out[PENDING] = pend
    return out


def load_state_dict(sd: dict, device=None, kernel=None):
    """Inverse of state_dict: the namedtuple with its leaves on `device`;
    pending pooled sums go to `kernel` (required when the checkpoint has them)."""
    kind = str(np.asarray(sd["__kind__"]))
    if kind not in _KINDS:
        raise ValueError(f"unknown state kind {kind!r}")
    cls, acls = _KINDS[kind]
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())

    def leaf(key):
        if key not in sd:
            raise KeyError(f"checkpoint lacks {key!r} for {kind}")
        return torch.from_numpy(np.ascontiguousarray(sd[key])).to(dev)

    fields = []
    for name in cls._fields:
        if name == "adapt_state":
            fields.append(acls(*[leaf(f"adapt_state.{an}") for an in acls._fields]))
        else:
            fields.append(leaf(name))
    state = cls(*fields)
    if PENDING in sd:
        if kernel is None or not getattr(kernel, "overlap", False):
            raise ValueError("checkpoint holds pending pooled sums (overlap=True): pass the PooledARWMH(overlap=True) "
                             "kernel that continues the run as `kernel=`")
        kernel.set_pending_sums(state, sd[PENDING])
    return state


def _npz(path: str) -> str:
    p = str(path)
    return p if p.endswith(".npz") else p + ".npz"  # np.savez appends it otherwise


def save_state(path: str, state, kernel=None, **extra) -> str:
    """state_dict(state, kernel) plus any extra arrays (e.g. accept_count) to
    .npz; returns the path written (".npz" appended when missing)."""
    sd = state_dict(state, kernel)
    for k, v in extra.items():
        if k in sd or k.startswith("__") or k.startswith("adapt_state."):
            raise ValueError(f"extra key {k!r} collides with a state field")
        sd[k] = v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
    path = _npz(path)
    np.savez(path, **sd)
    return path


def load_state(path: str, device=None, kernel=None, with_extras: bool = False):
    """load_state_dict of a save_state file (no pickles: allow_pickle=False).
    with_extras=True returns (state, {name: ndarray} of the extra arrays)."""
    with np.load(_npz(path), allow_pickle=False) as f:
        sd = {k: f[k] for k in f.files}
    state = load_state_dict(sd, device, kernel)
    if not with_extras:
        return state
    kind = str(np.asarray(sd["__kind__"]))
    cls, acls = _KINDS[kind]
    known = {"__kind__", PENDING} | {f for f in cls._fields if f != "adapt_state"} | \
        {f"adapt_state.{an}" for an in acls._fields}
    return state, {k: v for k, v in sd.items() if k not in known}
