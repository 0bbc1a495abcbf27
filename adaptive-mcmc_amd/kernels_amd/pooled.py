"""Pooled-covariance ARWMH (regime B): one shared adapt state for all chains
of all ranks (include/amh.h, amh_pooled_*).

Every chain proposes with the shared (loc, scale, log_step_size) exactly as
ARWMH.sample does with its own (arwmh.py:162-178).  The adaptation
(arwmh.py:180-197) then consumes the pooled statistics

    S_d = sum_c delta_c,  S_dd = sum_c delta_c delta_c^T,  S_a = sum_c alpha_c

so mu moves by gamma * mean delta, Sigma = L L^T is blended with the mean
outer product and refactorised (kept if not positive definite), and lambda
follows the mean acceptance.  With one chain in total this is the
reference's recurrence.  Across ranks the sums vector (d + d(d+1)/2 + 2
doubles) is the only exchange: one all-reduce(sum) per step over
torch.distributed (RCCL over xGMI on MI355X).
"""
from __future__ import annotations

import ctypes
from collections import namedtuple

import torch
import torch.distributed as dist

from . import _lib
from .arwmh import ARWMH, packed_size
from .random import as_key

PooledState = namedtuple("PooledState", ["i", "z", "potential_energy", "mean_accept_prob", "adapt_state",
                                         "as_change", "rng_key", "cov"])
PooledAdaptState = namedtuple("PooledAdaptState", ["loc", "scale", "log_step_size"])


class AmhPooledState(ctypes.Structure):
    _fields_ = [(n, ctypes.c_void_p) for n in ("i", "z", "potential_energy", "rng_key", "mean_accept_prob", "loc",
                                               "scale", "log_step_size", "as_change", "cov")]


def _bind_pooled(L):
    if getattr(L, "_pooled_bound", False):
        return L
    P, I32, I64 = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64
    PS = ctypes.POINTER(AmhPooledState)
    L.amh_pooled_sums_size.argtypes = [I32, ctypes.POINTER(I64)]
    L.amh_pooled_stats.argtypes = [P, I64, PS, P, P, P, P]
    L.amh_pooled_update.argtypes = [P, P, PS, PS, P]
    L.amh_pooled_step.argtypes = [P, I64, PS, PS, I32, P, P]
    L.amh_pooled_stats_k.argtypes = [P, I64, PS, I32, P, P, P]
    L.amh_pooled_update_k.argtypes = [P, P, PS, PS, I32, P]
    L.amh_pooled_step_k.argtypes = [P, I64, PS, PS, I32, I32, P, P]
    for n in ("amh_pooled_sums_size", "amh_pooled_stats", "amh_pooled_update", "amh_pooled_step",
              "amh_pooled_stats_k", "amh_pooled_update_k", "amh_pooled_step_k"):
        getattr(L, n).restype = ctypes.c_int
    L._pooled_bound = True
    return L


def sums_size(d: int) -> int:
    return d + packed_size(d) + 2


class PooledARWMH(ARWMH):
    """ARWMH with one adapt state shared by every chain (and every rank).

    Same constructor and init arguments as ARWMH; `group` is the
    torch.distributed process group whose chains are pooled (default: the
    default group when initialised, else this process alone).

    sync_every = K pools every K transitions: the shared
    state is frozen for a block of K transitions of every chain, the sums
    (and, across ranks, the one all-reduce) cover the block's K * C
    chain-steps, and one update ends it, with gamma counting blocks.  Then
    `sample` advances one block and `sample_(n)` needs n % K == 0;
    num_warmup must be a multiple of K."""

    pooled = True  # adapt-state leaves carry no chain axis

    def __init__(self, model=None, potential_fn=None, lr_decay=2 / 3, target_accept_prob=0.234, eps=1e-6,
                 num_chains=None, device=None, chain_offset=0, group=None, sync_every: int = 1, **kw):
        super().__init__(model=model, potential_fn=potential_fn, lr_decay=lr_decay,
                         target_accept_prob=target_accept_prob, eps=eps, num_chains=num_chains, device=device,
                         chain_offset=chain_offset, **kw)
        if int(sync_every) < 1:
            raise ValueError("sync_every must be >= 1")
        self._group = group
        self._sums = None
        self.sync_every = int(sync_every)

    def _world(self) -> int:
        if not dist.is_available() or not dist.is_initialized():
            return 1
        return dist.get_world_size(self._group)

    def init(self, rng_key, num_warmup, init_params, model_args, model_kwargs):
        """Per-chain z0 / pe0 / keys as ARWMH.init (arwmh.py:84-138); shared
        state mu = 0, L = Sigma = I, lambda = 0, i = 0 (mu_0 is irrelevant
        after step 1, where gamma_1 = 1)."""
        if int(num_warmup) % self.sync_every != 0:
            raise ValueError(f"num_warmup ({num_warmup}) must be a multiple of sync_every ({self.sync_every})")
        st = super().init(rng_key, num_warmup, init_params, model_args, model_kwargs)
        d, dev = self._dim, st.z.device
        f = dict(dtype=torch.float32, device=dev)
        eye = torch.eye(d, dtype=torch.float64, device=dev)
        from .arwmh import pack_scale
        cov = pack_scale(eye)
        adapt = PooledAdaptState(torch.zeros(d, **f), cov.to(torch.float32), torch.zeros(1, **f))
        self._sums = torch.zeros(sums_size(d), dtype=torch.float64, device=dev)
        return PooledState(torch.zeros(1, dtype=torch.int32, device=dev), st.z, st.potential_energy,
                           torch.zeros(1, **f), adapt, torch.zeros(1, **f), st.rng_key, cov)

    @staticmethod
    def _c(s: PooledState) -> AmhPooledState:
        a = s.adapt_state
        return AmhPooledState(s.i.data_ptr(), s.z.data_ptr(), s.potential_energy.data_ptr(), s.rng_key.data_ptr(),
                              s.mean_accept_prob.data_ptr(), a.loc.data_ptr(), a.scale.data_ptr(),
                              a.log_step_size.data_ptr(), s.as_change.data_ptr(), s.cov.data_ptr())

    def _check(self, s: PooledState):
        if self._handle is None:
            raise RuntimeError("call init() first")
        d = self._dim
        C = s.z.shape[0]
        want = [(s.i, (1,), torch.int32), (s.z, (C, d), torch.float32), (s.potential_energy, (C,), torch.float32),
                (s.mean_accept_prob, (1,), torch.float32), (s.adapt_state.loc, (d,), torch.float32),
                (s.adapt_state.scale, (packed_size(d),), torch.float32),
                (s.adapt_state.log_step_size, (1,), torch.float32), (s.as_change, (1,), torch.float32),
                (s.rng_key, (C, 2), torch.int32), (s.cov, (packed_size(d),), torch.float64)]
        for t, shape, dt in want:
            _lib.require_gpu(t)
            if tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous():
                raise ValueError(f"pooled state leaf has shape {tuple(t.shape)} {t.dtype}, expected {shape} {dt}")
        return C

    def _new_like(self, s: PooledState) -> PooledState:
        a = s.adapt_state
        return PooledState(torch.empty_like(s.i), torch.empty_like(s.z), torch.empty_like(s.potential_energy),
                           torch.empty_like(s.mean_accept_prob),
                           PooledAdaptState(torch.empty_like(a.loc), torch.empty_like(a.scale),
                                            torch.empty_like(a.log_step_size)),
                           torch.empty_like(s.as_change), s.rng_key, torch.empty_like(s.cov))

    def _one(self, sin: PooledState, sout: PooledState):
        L = _bind_pooled(_lib.lib())
        dev = sin.z.device.index
        C = sin.z.shape[0]
        cin, cout = self._c(sin), self._c(sout)
        K = self.sync_every
        with torch.cuda.device(dev):
            stream = _lib.stream_ptr(dev)
            _lib.check(L.amh_pooled_stats_k(self._handle.h, C, ctypes.byref(cin), K, _lib.ptr(sout.z),
                                            _lib.ptr(sout.potential_energy), _lib.ptr(self._sums), stream),
                       self._handle.h)
            if self._world() > 1:
                dist.all_reduce(self._sums, op=dist.ReduceOp.SUM, group=self._group)
            _lib.check(L.amh_pooled_update_k(self._handle.h, _lib.ptr(self._sums), ctypes.byref(cin),
                                             ctypes.byref(cout), K, stream), self._handle.h)

    def sample(self, state, model_args=(), model_kwargs=None):
        """One pooled transition of every chain (sync_every > 1: one block of
        them); returns a new state."""
        self._check(state)
        out = self._new_like(state)
        self._one(state, out)
        return out

    def sample_(self, state, n_steps: int = 1):
        """n_steps pooled transitions in place (a multiple of sync_every)."""
        C = self._check(state)
        K = self.sync_every
        if int(n_steps) % K != 0:
            raise ValueError(f"n_steps ({n_steps}) must be a multiple of sync_every ({K})")
        if self._world() == 1:
            L = _bind_pooled(_lib.lib())
            dev = state.z.device.index
            c = self._c(state)
            with torch.cuda.device(dev):
                _lib.check(L.amh_pooled_step_k(self._handle.h, C, ctypes.byref(c), ctypes.byref(c), int(n_steps), K,
                                               _lib.ptr(self._sums), _lib.stream_ptr(dev)), self._handle.h)
            return state
        for _ in range(int(n_steps) // K):
            self._one(state, state)
        return state

    def run(self, *a, **k):
        raise NotImplementedError("pooled mode: use sample / sample_")

    def get_diagnostics_str(self, state):
        acc = float(state.mean_accept_prob[0])
        step = float(torch.exp(state.adapt_state.log_step_size[0]))
        return f"Acceptance rate: {acc:.2f}, Step size: {step:.3f}"
