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


def state_dict(state) -> dict:
    """Flatten a state into {field path: host ndarray} plus its kind."""
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
    return out


def load_state_dict(sd: dict, device=None):
    """Inverse of state_dict: the namedtuple with its leaves on `device`."""
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
    return cls(*fields)


def save_state(path: str, state, **extra) -> None:
    """state_dict(state) (plus any extra arrays, e.g. accept_count) to .npz."""
    sd = state_dict(state)
    for k, v in extra.items():
        if k in sd:
            raise ValueError(f"extra key {k!r} collides with a state field")
        sd[k] = v.detach().cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)
    np.savez(path, **sd)


def load_state(path: str, device=None):
    """load_state_dict of a save_state file (no pickles: allow_pickle=False)."""
    with np.load(path, allow_pickle=False) as f:
        sd = {k: f[k] for k in f.files}
    return load_state_dict(sd, device)
