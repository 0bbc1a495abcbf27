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


# ------------------------------------------------ local contraction estimates --
# asumptions_check.ipynb cells 81-82 (notebook-local helpers the analysis runs
# through sample_Pnx + wasserstein_1d): tau_x(P^n) = W1(P^n(x_l, .),
# P^n(x_r, .)) / (x_r - x_l) for a pair of points around every x of a 1-D grid.
# As in the notebook, every x's pair is drawn with the same rng_key (so the
# pairs at different x share their per-sample keys).
def _taus_from_pairs(kernel, rng_key, pairs: np.ndarray, adapt_state, n: int, n_samples: int,
                     divisor: float = None) -> np.ndarray:
    from utils_amd.evaluation import wasserstein_1d
    out = np.empty(pairs.shape[0], np.float64)
    for i, (xl, xr) in enumerate(pairs):
        X = np.array([[xl], [xr]], np.float32)
        P = kernel.sample_Pnx(rng_key, X, adapt_state, n, n_samples)  # [2, n_samples, 1]
        w = wasserstein_1d(P[0, :, 0], P[1, :, 0])
        out[i] = float(w) / (divisor if divisor is not None else float(np.float32(xr) - np.float32(xl)))
    return out


def get_taus_n(rng_key, kernel, X, adapt_state, n: int = 1, n_samples: int = 10000, eps: float = 5e-2) -> np.ndarray:
    """Cell 81 (ARWMH): the pair (x - eps, x + eps), W1 / (2 eps)."""
    x = np.asarray(X.cpu() if hasattr(X, "cpu") else X, np.float32).reshape(-1)
    e = np.float32(eps)
    pairs = np.stack([x - e, x + e], axis=1)
    return _taus_from_pairs(kernel, rng_key, pairs, adapt_state, n, n_samples, divisor=2 * eps)


def get_taus_n_sss(rng_key, kernel, X, adapt_state, n: int = 1, n_samples: int = 10000,
                   eps: float = 1e-1) -> np.ndarray:
    """Cell 82 (ASSS): the pair is +-eps in the stereographic angle,
    phi = 2 arctan((x - loc) / scale), x_lr = tan((phi -+ eps) / 2) scale + loc,
    divided by x_r - x_l (float32, as the notebook's jnp arithmetic)."""
    loc = np.float32(np.asarray(adapt_state[0].cpu() if hasattr(adapt_state[0], "cpu") else adapt_state[0]).reshape(-1)[0])
    sc = np.float32(np.asarray(adapt_state[1].cpu() if hasattr(adapt_state[1], "cpu") else adapt_state[1]).reshape(-1)[0])
    x = np.asarray(X.cpu() if hasattr(X, "cpu") else X, np.float32).reshape(-1)
    phi = np.float32(2) * np.arctan((x - loc) / sc)
    e = np.float32(eps)
    xl = np.tan((phi - e) / np.float32(2)) * sc + loc
    xr = np.tan((phi + e) / np.float32(2)) * sc + loc
    return _taus_from_pairs(kernel, rng_key, np.stack([xl, xr], axis=1).astype(np.float32), adapt_state, n, n_samples)


def get_max_taus(rng_key, kernel, X, adapt_state, n_list, n_samples: int = 500000, eps: float = 1e-1) -> list:
    """Cells 41 / 91 (`get_max_taus`): max over the grid X of
    get_taus_n_sss(..., n) for every n in n_list (the same rng_key each time)."""
    return [float(get_taus_n_sss(rng_key, kernel, X, adapt_state, n=n, n_samples=n_samples, eps=eps).max())
            for n in n_list]
