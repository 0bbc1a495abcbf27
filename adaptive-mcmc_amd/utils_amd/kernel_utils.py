"""Drivers around ARWMH.sample: the log-spaced state collection of the
reference (python/utils/kernel_utils.py:8-38) on device state.

The reference runs `fori_collect(0, 10^p - 10^(p-1), sample, state,
thinning=10^max(0, p-2))` per decade p and concatenates the collected state
pytrees.  Here every thinning interval is one fused step launch
(ARWMH.sample_, state in registers between steps) followed by a snapshot of
the state tensors; the snapshots are stacked along a new leading axis.
"""
from __future__ import annotations

from typing import List

import numpy as np
import torch

from kernels_amd.arwmh import ARWMHAdaptState, ARWMHState


def ns_logscale(n_pow: int = 6) -> np.ndarray:
    """Step counts at which collect_states_logscale records a state
    (kernel_utils.py:8-12): 1..10, 11..100, then 10^(p-2)-spaced up to 10^n_pow."""
    parts = []
    for p in range(n_pow + 1):
        lo = 0 if p < 1 else 10 ** (p - 1)
        step = 10 ** max(0, p - 2)
        parts.append(np.arange(lo, 10 ** p, step) + step)
    return np.concatenate(parts)


def _snapshot(s: ARWMHState) -> ARWMHState:
    a = s.adapt_state
    return ARWMHState(s.i.clone(), s.z.clone(), s.potential_energy.clone(), s.mean_accept_prob.clone(),
                      ARWMHAdaptState(a.loc.clone(), a.scale.clone(), a.log_step_size.clone()),
                      s.as_change.clone(), s.rng_key.clone())


def concat_trees(trees: List[ARWMHState]) -> ARWMHState:
    """Stack a list of states along a new leading axis (kernel_utils.py:14-18
    concatenates fori_collect outputs that already carry that axis)."""
    def st(xs):
        return torch.stack(list(xs), dim=0)
    a = [t.adapt_state for t in trees]
    return ARWMHState(st(t.i for t in trees), st(t.z for t in trees), st(t.potential_energy for t in trees),
                      st(t.mean_accept_prob for t in trees),
                      ARWMHAdaptState(st(x.loc for x in a), st(x.scale for x in a), st(x.log_step_size for x in a)),
                      st(t.as_change for t in trees), st(t.rng_key for t in trees))


def collect_states_logscale(rng_key, sampler, model_data: dict, n_pow: int = 6, init_params=None) -> ARWMHState:
    """kernel_utils.py:20-38: init with num_warmup = 0, then record the state
    after every step count in ns_logscale(n_pow).  Returns the stacked states,
    leaves shaped [len(ns_logscale(n_pow)), C, ...].

    `init_params`: the reference passes {} (init_to_uniform) for models; a
    potential_fn sampler needs explicit starting points, as in the reference."""
    state = sampler.init(rng_key, 0, {} if init_params is None else init_params, (), model_data)
    snaps = []
    for p in range(n_pow + 1):
        lo = 0 if p < 1 else 10 ** (p - 1)
        thin = 10 ** max(0, p - 2)
        for _ in range((10 ** p - lo) // thin):
            sampler.sample_(state, thin)
            snaps.append(_snapshot(state))
    return concat_trees(snaps)
