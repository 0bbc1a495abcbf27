"""ASSS: adaptive stereographic slice sampler on MI355X.

Drop-in for the reference kernel python/kernels/asss.py (savelovme/
adaptive-mcmc): same constructor arguments (model XOR potential_fn, lr_decay,
eps, init_strategy), method names (init, sample, postprocess_fn,
get_diagnostics_str, sample_Pnx, get_init_adapt_state) and state namedtuples
ASSSState / ASSSAdaptState, with a leading chain axis on every leaf.  Every
transition of every chain runs in the HIP kernel amh_asss.hip (C-ABI
amh_asss_step / amh_asss_sample_pnx, include/amh.h); there is no CPU path.

Differences a caller can see are those of ARWMH (kernels_amd/arwmh.py): torch
leaves on the GPU, packed column-major `scale`, counter-based Philox noise
(`rng_key` fixed per chain, stream position `i`), registry models.
"""
from __future__ import annotations

from collections import namedtuple

import numpy as np
import torch

from . import _lib
from .arwmh import ARWMH, ARWMHAdaptState, ARWMHState, _device_index, init_to_uniform, pack_scale, packed_size
from .random import as_key

ASSSState = namedtuple(
    "ASSSState",
    [
        "i",  # Iteration                                   [C] int32
        "z",  # Current point (unconstrained, flat)         [C, d]
        "potential_energy",  # Current potential energy     [C]
        "adapt_state",  # Mean & Cholesky factor estimates
        "as_change",  # ||mu' - mu|| + ||L' - L||_F           [C]
        "rng_key",  # Per-chain Philox key                  [C, 2] int32 (uint32 bits)
    ],
)

ASSSAdaptState = namedtuple("ASSSAdaptState", ["loc", "scale"])


class ASSS(ARWMH):
    """
    Adaptive Stereographic Slice Sampler kernel (reference: python/kernels/
    asss.py:99-303), batched over chains.

    Parameters (asss.py:106-136): model XOR potential_fn, lr_decay (gamma_n =
    1 / n^lr_decay, default 2/3), eps (default 1e-6), init_strategy
    (init_to_uniform only); plus num_chains, device, chain_offset as ARWMH.
    """

    sample_field = "z"

    def __init__(self, model=None, potential_fn=None, lr_decay=2 / 3, eps=1e-6, init_strategy=init_to_uniform,
                 num_chains=None, device=None, chain_offset=0):
        super().__init__(model=model, potential_fn=potential_fn, lr_decay=lr_decay, eps=eps,
                         init_strategy=init_strategy, num_chains=num_chains, device=device,
                         chain_offset=chain_offset)

    # ------------------------------------------------------------------ state --
    @staticmethod
    def _to_asss(s: ARWMHState) -> ASSSState:
        a = s.adapt_state
        return ASSSState(s.i, s.z, s.potential_energy, ASSSAdaptState(a.loc, a.scale), s.as_change, s.rng_key)

    @staticmethod
    def _c_state(s) -> _lib.AmhState:
        if isinstance(s, ARWMHState):  # ARWMH.init's output, before conversion
            return ARWMH._c_state(s)
        a = s.adapt_state
        return _lib.AmhState(s.i.data_ptr(), s.z.data_ptr(), s.potential_energy.data_ptr(), None,
                             a.loc.data_ptr(), a.scale.data_ptr(), None, s.as_change.data_ptr(),
                             s.rng_key.data_ptr())

    def _alloc(self, C: int, d: int, device) -> ASSSState:
        f = dict(dtype=torch.float32, device=device)
        return ASSSState(torch.empty(C, dtype=torch.int32, device=device), torch.empty(C, d, **f),
                         torch.empty(C, **f), ASSSAdaptState(torch.empty(C, d, **f), torch.empty(C, packed_size(d), **f)),
                         torch.empty(C, **f), torch.empty(C, 2, dtype=torch.int32, device=device))

    def _check(self, s: ASSSState) -> int:
        if self._handle is None:
            raise RuntimeError("call init() first")
        d, C = self._dim, s.z.shape[0]
        leaves = [(s.i, (C,), torch.int32), (s.z, (C, d), torch.float32), (s.potential_energy, (C,), torch.float32),
                  (s.adapt_state.loc, (C, d), torch.float32),
                  (s.adapt_state.scale, (C, packed_size(d)), torch.float32), (s.as_change, (C,), torch.float32),
                  (s.rng_key, (C, 2), torch.int32)]
        for t, shape, dt in leaves:
            _lib.require_gpu(t)
            if tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous():
                raise ValueError(f"state leaf has shape {tuple(t.shape)} {t.dtype}, expected {shape} {dt}")
        return C

    # -------------------------------------------------------------------- API --
    def init(self, rng_key, num_warmup, init_params, model_args, model_kwargs):
        """asss.py:138-189: z0 (init_to_uniform unless init_params), pe0 = U(z0),
        loc = z0, scale = I, i = 0, as_change = 0."""
        if self._model is None and init_params is None:
            raise ValueError("Valid value of `init_params` must be provided with `potential_fn`.")
        st = super().init(rng_key, num_warmup, init_params, model_args, model_kwargs)
        if self._dim > 64 and not self._big_ok():
            raise ValueError("ASSS supports d <= 64, or the dense Gaussian up to d = 256")
        return self._to_asss(st)

    def _big_ok(self) -> bool:
        """64 < d <= 256: the large-d kernel (amh_big.hip asss_big_step_kernel)
        takes the dense Gaussian at any such d (the reference has no dimension
        limit, asss.py:192-269; other models stop at d = 64)."""
        mid = self._model.model_id if self._model is not None else getattr(self._potential_fn, "model_id", None)
        return mid == _lib.AMH_MODEL_GAUSSIAN and self._dim <= 256

    def sample(self, state, model_args=(), model_kwargs=None):
        """asss.py:191-258: one transition of every chain; returns a new state."""
        C = self._check(state)
        out = self._alloc(C, self._dim, state.z.device)
        self._launch(state, out, 1, None)
        return out

    def sample_(self, state, n_steps: int = 1):
        """In-place variant: advance `state` by n_steps (one fused launch)."""
        self._check(state)
        self._launch(state, state, n_steps, None)
        return state

    def run(self, state, n_steps: int, thinning: int = 1, collect_z: bool = True, collect_pe: bool = False):
        """Fused n_steps transitions; returns (new_state, z [n_steps // thinning, C, d]
        or None, pe or None)."""
        C = self._check(state)
        out = self._alloc(C, self._dim, state.z.device)
        keep = n_steps // thinning
        dev = state.z.device
        cz = torch.empty(keep, C, self._dim, dtype=torch.float32, device=dev) if collect_z and keep else None
        cp = torch.empty(keep, C, dtype=torch.float32, device=dev) if collect_pe and keep else None
        self._launch(state, out, n_steps, (cz, cp, thinning))
        return out, cz, cp

    def _launch(self, sin, sout, n_steps, collect):
        cz, cp, thin = collect if collect is not None else (None, None, 1)
        col = _lib.AmhCollect(cz.data_ptr() if cz is not None else None,
                              cp.data_ptr() if cp is not None else None, None, thin)
        dev = sin.z.device.index
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().amh_asss_step(self._handle.h, sin.z.shape[0], self._c_state(sin),
                                                self._c_state(sout), n_steps, col, _lib.stream_ptr(dev)),
                       self._handle.h)

    def get_diagnostics_str(self, state):
        """asss.py:264-265 (chain-averaged potential energy for a batch)."""
        return f"Iteration: {int(state.i.max())}, Potential Energy: {float(state.potential_energy.mean()):.2f}"

    def sample_Pnx(self, rng_key, x, adapt_state, n=1, n_samples=1000, jit_inner=True):
        """asss.py:267-296: n frozen-kernel transitions from every x[i] for
        n_samples chains each, sharing adapt_state = (loc, scale); returns
        [n_points, n_samples, d]."""
        self._ensure_bound()
        dev = torch.device("cuda", _device_index(self._device))
        d = self._dim

        def host(a):
            return torch.as_tensor(a.cpu() if hasattr(a, "cpu") else np.asarray(a), dtype=torch.float32)

        x = host(x).reshape(-1, d).to(dev).contiguous()
        loc, scale = adapt_state[0], adapt_state[1]
        scale = host(scale)
        if scale.dim() >= 2 and scale.shape[-1] == d and scale.shape[-2] == d:
            scale = pack_scale(scale.reshape(-1, d, d)[0])
        scale = scale.reshape(-1)[:packed_size(d)].to(dev).contiguous()
        loc = host(loc).reshape(-1)[:d].to(dev).contiguous()
        out = torch.empty(x.shape[0], n_samples, d, dtype=torch.float32, device=dev)
        with torch.cuda.device(dev.index):
            _lib.check(_lib.lib().amh_asss_sample_pnx(self._handle.h, _lib.key_arr(as_key(rng_key)), _lib.ptr(x),
                                                      x.shape[0], n_samples, _lib.ptr(loc), _lib.ptr(scale), n,
                                                      _lib.ptr(out), _lib.stream_ptr(dev.index)), self._handle.h)
        return out

    def get_init_adapt_state(self, rng_key, init_params, model_args=(), model_kwargs={}):
        """asss.py:298-303."""
        return self.init(rng_key, 0, init_params, model_args, model_kwargs).adapt_state
