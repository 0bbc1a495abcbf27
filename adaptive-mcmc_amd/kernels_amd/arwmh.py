"""ARWMH: adaptive random-walk Metropolis-Hastings on MI355X.

Drop-in for the reference kernel python/kernels/arwmh.py (savelovme/
adaptive-mcmc): same constructor arguments, method names, state namedtuples
and ValueErrors, with a leading chain axis on every state leaf.  One call of
`sample` advances every chain by one transition in one HIP launch
(libamh.so, include/amh.h); there is no CPU path.

Differences a caller can see (DESIGN.md lists them with their reasons):
  * state leaves are torch tensors on the GPU with a leading chain axis C;
    `z` / `loc` are flat [C, d] (sorted-site ravel order, as ravel_pytree),
    `scale` is the packed lower triangle [C, d(d+1)/2] (column-major;
    `unpack_scale` gives [C, d, d]);
  * noise comes from counter-based Philox streams: `rng_key` [C, 2] is the
    chain's key and the stream position is `i`, so the key does not change
    between steps (the reference splits its threefry key every step);
  * models are registry entries (adaptive-mcmc_amd/posteriors), since device
    code cannot call a Python potential.
"""
from __future__ import annotations

import weakref
from collections import namedtuple

import numpy as np
import torch

from . import _lib
from .random import as_key

ARWMHState = namedtuple(
    "ARWMHState",
    [
        "i",  # Iteration                                   [C] int32
        "z",  # Current point (unconstrained, flat)         [C, d]
        "potential_energy",  # Current potential energy     [C]
        "mean_accept_prob",  # Running mean of acceptance   [C]
        "adapt_state",  # Mean & Cholesky factor + log step size
        "as_change",  # || L' e^lam' - L e^lam ||_F         [C]
        "rng_key",  # Per-chain Philox key                  [C, 2] int32 (uint32 bits)
    ],
)

ARWMHAdaptState = namedtuple("ARWMHAdaptState", ["loc", "scale", "log_step_size"])


def init_to_uniform(*args, **kwargs):
    """Marker for numpyro's init_to_uniform (U(-2, 2) per unconstrained site)."""
    return None


def packed_size(d: int) -> int:
    return d * (d + 1) // 2


def _tril_index(d: int, device=None):
    rows, cols = [], []
    for j in range(d):
        for r in range(j, d):
            rows.append(r)
            cols.append(j)
    return torch.tensor(rows, device=device), torch.tensor(cols, device=device)


def pack_scale(L: torch.Tensor) -> torch.Tensor:
    """[..., d, d] lower-triangular -> [..., d(d+1)/2] column-major packing."""
    d = L.shape[-1]
    r, c = _tril_index(d, L.device)
    return L[..., r, c].contiguous()


def unpack_scale(Lp: torch.Tensor, d: int) -> torch.Tensor:
    """[..., d(d+1)/2] -> [..., d, d] (zeros above the diagonal)."""
    r, c = _tril_index(d, Lp.device)
    out = torch.zeros(Lp.shape[:-1] + (d, d), dtype=Lp.dtype, device=Lp.device)
    out[..., r, c] = Lp
    return out


def _device_index(device) -> int:
    if device is None:
        return torch.cuda.current_device()
    d = torch.device(device)
    return d.index if d.index is not None else torch.cuda.current_device()


class ARWMH:
    """
    ARWMH kernel for adaptive random walk-based Markov Chain Monte Carlo
    (reference: python/kernels/arwmh.py:31-276), batched over chains.

    Parameters (arwmh.py:43-78)
    ----------
    model : posteriors.Model, optional
        Registry model; its data are passed as `model_kwargs` to `init`.
    potential_fn : posteriors.Gaussian / Mixture, or any callable, optional
        Device potential (raw potential_fn plug-in), fused into the kernel;
        any other callable (a batched torch function z [n, d] -> U [n], or a
        posteriors.TorchPotential) runs between the kernel's proposal and
        step launches (AMH_MODEL_EXTERNAL, d <= 256).  Exactly one of `model`
        and `potential_fn` must be given.
    lr_decay : float, gamma_n = 1 / n^lr_decay (default 2/3).
    target_accept_prob : float (default 0.234).
    eps : float, added to the diagonal of the scaled factor (default 1e-6).
    init_strategy : only init_to_uniform (U(-2, 2)) is supported.
    num_chains : int, optional; otherwise taken from init_params' leading axis.
    device : torch device of the chains (default: current CUDA device).
    chain_offset : global id of this shard's first chain; chain keys depend
        only on (rng_key, global id), so a sharded run equals an unsharded one.
    """

    sample_field = "z"

    def __init__(self, model=None, potential_fn=None, lr_decay=2 / 3, target_accept_prob=0.234, eps=1e-6,
                 init_strategy=init_to_uniform, num_chains=None, device=None, chain_offset=0):
        if not (model is None) ^ (potential_fn is None):
            raise ValueError("Only one of `model` or `potential_fn` must be specified.")
        if potential_fn is not None and not hasattr(potential_fn, "model_id"):
            if not callable(potential_fn):
                raise TypeError("potential_fn must be callable")
            import posteriors as _P
            potential_fn = _P.TorchPotential(potential_fn)  # dim from init_params
        self._model = model
        self._potential_fn = potential_fn
        self._lr_decay = lr_decay
        self._target_accept_prob = target_accept_prob
        self._eps = eps
        self._postprocess_fn = None
        self._init_strategy = init_strategy
        self._num_warmup = 0
        self._num_chains = num_chains
        self._device = device
        self._chain_offset = int(chain_offset)  # global id of chain 0 (sharding)
        self._handle = None
        self._model_kwargs = None
        self._dim = None
        self.accept_count = None  # [C] int32 accepted proposals since init (diagnostic)
        self.chain_proposals = True  # d > 64 / diamonds: reuse the step pass's next proposal across sample() calls

    @property
    def model(self):
        return self._model

    # ------------------------------------------------------------------ setup --
    def _bind(self, num_warmup: int, model_kwargs: dict, device_index: int):
        if self._model is not None:
            dim = self._model.dim(model_kwargs)
            data, ip = self._model.pack(model_kwargs, torch.device("cuda", device_index))
            model_id = self._model.model_id
        else:
            dim = self._potential_fn.dim
            data, ip = self._potential_fn.pack(torch.device("cuda", device_index))
            model_id = self._potential_fn.model_id
        if self._handle is not None:
            self._handle.close()
        self._handle = _lib.Handle(dim, num_warmup, self._lr_decay, self._target_accept_prob, self._eps,
                                   device_index)
        self._handle.bind_model(model_id, data, ip)
        self._dim = dim
        self._num_warmup = num_warmup
        self._model_kwargs = model_kwargs

    def _alloc_state(self, C: int, d: int, device) -> ARWMHState:
        f = dict(dtype=torch.float32, device=device)
        adapt = ARWMHAdaptState(torch.empty(C, d, **f), torch.empty(C, packed_size(d), **f),
                                torch.empty(C, **f))
        return ARWMHState(torch.empty(C, dtype=torch.int32, device=device), torch.empty(C, d, **f),
                          torch.empty(C, **f), torch.empty(C, **f), adapt, torch.empty(C, **f),
                          torch.empty(C, 2, dtype=torch.int32, device=device))

    @staticmethod
    def _c_state(s: ARWMHState) -> _lib.AmhState:
        return _lib.AmhState(s.i.data_ptr(), s.z.data_ptr(), s.potential_energy.data_ptr(),
                             s.mean_accept_prob.data_ptr(), s.adapt_state.loc.data_ptr(),
                             s.adapt_state.scale.data_ptr(), s.adapt_state.log_step_size.data_ptr(),
                             s.as_change.data_ptr(), s.rng_key.data_ptr())

    def _check_state(self, s: ARWMHState):
        if self._handle is None:
            raise RuntimeError("call init() first")
        d, C = self._dim, s.z.shape[0]
        leaves = [(s.i, (C,), torch.int32), (s.z, (C, d), torch.float32), (s.potential_energy, (C,), torch.float32),
                  (s.mean_accept_prob, (C,), torch.float32), (s.adapt_state.loc, (C, d), torch.float32),
                  (s.adapt_state.scale, (C, packed_size(d)), torch.float32),
                  (s.adapt_state.log_step_size, (C,), torch.float32), (s.as_change, (C,), torch.float32),
                  (s.rng_key, (C, 2), torch.int32)]
        for t, shape, dt in leaves:
            _lib.require_gpu(t)
            if tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous():
                raise ValueError(f"state leaf has shape {tuple(t.shape)} {t.dtype}, expected {shape} {dt}")
        return C

    # -------------------------------------------------------------------- API --
    def init(self, rng_key, num_warmup, init_params, model_args, model_kwargs):
        """arwmh.py:84-138: z0 (init_to_uniform unless init_params), pe0 = U(z0),
        loc = z0, scale = I, log_step_size = 0, i = 0."""
        if self._model is None and init_params is None:
            raise ValueError("Valid value of `init_params` must be provided with `potential_fn`.")
        device_index = _device_index(self._device)
        device = torch.device("cuda", device_index)
        if self._external() and self._potential_fn.dim is None:
            x = init_params.cpu() if hasattr(init_params, "cpu") else np.asarray(init_params)
            self._potential_fn.dim = int(np.asarray(x).shape[-1]) if np.ndim(x) else 1
        self._bind(int(num_warmup), dict(model_kwargs or {}), device_index)
        d = self._dim
        iz = None
        if init_params is not None and not (isinstance(init_params, dict) and len(init_params) == 0):
            iz = self._flat_params(init_params, device)
        C = self._num_chains or (iz.shape[0] if iz is not None else 1)
        if iz is not None and iz.shape[0] == 1 and C > 1:
            iz = iz.expand(C, d).contiguous()
        if iz is not None and iz.shape != (C, d):
            raise ValueError(f"init_params has shape {tuple(iz.shape)}, expected ({C}, {d})")
        self._num_chains = C
        state = self._alloc_state(C, d, device)
        key = _lib.key_arr(as_key(rng_key))
        with torch.cuda.device(device_index):
            _lib.check(_lib.lib().amh_init(self._handle.h, key, self._chain_offset, C, _lib.ptr(iz),
                                           ctypes_state(self, state), _lib.stream_ptr(device_index)),
                       self._handle.h)
        self.accept_count = torch.zeros(C, dtype=torch.int32, device=device)
        if self._external():  # pe0 = U(z0) by the caller's potential (amh_init left 0)
            with torch.cuda.device(device_index):
                state.potential_energy.copy_(self._potential_fn.evaluate(state.z))
            self._zprop = None
        if self._model is not None:
            mk = self._model_kwargs
            self._postprocess_fn = lambda *a, **k: (lambda z: self._model.postprocess(z, mk))
        return state

    def _flat_params(self, init_params, device) -> torch.Tensor:
        if isinstance(init_params, dict):
            if self._model is None:
                raise ValueError("dict init_params need a model")
            parts = []
            for s in self._model.sites(self._model_kwargs):
                v = torch.as_tensor(np.asarray(init_params[s.name]), dtype=torch.float32)
                v = v.reshape(-1, s.size) if v.dim() > (0 if s.size == 1 else 1) else v.reshape(1, s.size)
                parts.append(v)
            x = torch.cat(parts, dim=-1)
        else:
            x = torch.as_tensor(init_params.cpu() if hasattr(init_params, "cpu") else np.asarray(init_params),
                                dtype=torch.float32)
            x = x.reshape(-1, self._dim)
        return x.to(device).contiguous()

    def sample(self, state, model_args, model_kwargs):
        """arwmh.py:140-207: one transition of every chain; returns a new state."""
        C = self._check_state(state)
        out = self._alloc_state(C, self._dim, state.z.device)
        self._launch(state, out, 1, None)
        return out

    def sample_(self, state, n_steps: int = 1):
        """In-place variant: advance `state` by n_steps (one fused launch)."""
        C = self._check_state(state)
        self._launch(state, state, n_steps, None)
        return state

    def run(self, state, n_steps: int, thinning: int = 1, collect_z: bool = True, collect_pe: bool = False):
        """Fused n_steps transitions (numpyro fori_collect over sample); returns
        (new_state, z [n_steps // thinning, C, d] or None, pe or None)."""
        C = self._check_state(state)
        if int(n_steps) == 0:  # nothing to run: a copy of the input, no collections
            return _clone_state(state), None, None
        out = self._alloc_state(C, self._dim, state.z.device)
        keep = n_steps // thinning
        dev = state.z.device
        cz = torch.empty(keep, C, self._dim, dtype=torch.float32, device=dev) if collect_z and keep else None
        cp = torch.empty(keep, C, dtype=torch.float32, device=dev) if collect_pe and keep else None
        self._launch(state, out, n_steps, (cz, cp, thinning))
        return out, cz, cp

    @staticmethod
    def _leaves(state):
        a = state.adapt_state
        return (state.i, state.z, state.potential_energy, state.mean_accept_prob, a.loc, a.scale,
                a.log_step_size, state.as_change, state.rng_key)

    def _external(self) -> bool:
        return self._potential_fn is not None and self._potential_fn.model_id == _lib.AMH_MODEL_EXTERNAL

    def _launch_external(self, sin, sout, n_steps, collect):
        """AMH_MODEL_EXTERNAL: per transition amh_step_external with the
        caller's U of the proposals, which the previous launch formed (the
        first by amh_propose).  Collection as the fused launch (thinning)."""
        cz, cp, thin = collect if collect is not None else (None, None, 1)
        C, d, dev = sin.z.shape[0], self._dim, sin.z.device
        zp = torch.empty(C, d, dtype=torch.float32, device=dev)
        lib = _lib.lib()
        acc = self.accept_count.data_ptr() if self.accept_count is not None else None
        with torch.cuda.device(dev.index):
            st = _lib.stream_ptr(dev.index)
            _lib.check(lib.amh_propose(self._handle.h, C, ctypes_state(self, sin), _lib.ptr(zp), st), self._handle.h)
            for t in range(int(n_steps)):
                src = sin if t == 0 else sout
                pe = self._potential_fn.evaluate(zp)
                keep = (t + 1) % thin == 0
                k = t // thin
                col = _lib.AmhCollect(cz[k].data_ptr() if (keep and cz is not None) else None,
                                      cp[k].data_ptr() if (keep and cp is not None) else None, acc, 1)
                nxt = _lib.ptr(zp) if t + 1 < n_steps else None
                _lib.check(lib.amh_step_external(self._handle.h, C, ctypes_state(self, src), ctypes_state(self, sout),
                                                 _lib.ptr(zp), _lib.ptr(pe), nxt, col, st), self._handle.h)

    def _launch(self, sin, sout, n_steps, collect):
        if int(n_steps) == 0:
            return  # no launch: the chained proposal (if any) stays with the tensors it was made for
        if self._external():
            return self._launch_external(sin, sout, n_steps, collect)
        cz, cp, thin = collect if collect is not None else (None, None, 1)
        col = _lib.AmhCollect(cz.data_ptr() if cz is not None else None,
                              cp.data_ptr() if cp is not None else None,
                              self.accept_count.data_ptr() if self.accept_count is not None else None, thin)
        dev = sin.z.device.index
        flags = 0
        if self._chained_path() and self.chain_proposals and not any(t.is_inference() for t in self._leaves(sin)):
            # d > 64 and the literal diamonds model: the step pass forms the
            # next proposal (amh_step_chained).
            # It is reused only for the very tensors the last call returned
            # (weak references: a dead one never matches, so recycled storage
            # cannot pass), unmodified since (torch's in-place version counters;
            # inference-mode tensors have none, so they are never chained).
            # Edits that bypass the version counter (`.data`, DLPack) are not
            # seen: set `chain_proposals = False` when state is edited that way.
            # The library checks too: READY holds only for the buffers it wrote.
            leaves = self._leaves(sin)
            last = getattr(self, "_chained", None)
            if last is not None and all(w() is t for w, t in zip(last[0], leaves)) and \
                    all(t._version == v for t, v in zip(leaves, last[1])):
                flags |= _lib.AMH_STEP_PROPOSAL_READY
            flags |= _lib.AMH_STEP_KEEP_PROPOSAL
            self._chained = None
        with torch.cuda.device(dev):
            _lib.check(_lib.lib().amh_step_chained(self._handle.h, sin.z.shape[0], ctypes_state(self, sin),
                                                   ctypes_state(self, sout), n_steps, col, flags,
                                                   _lib.stream_ptr(dev)), self._handle.h)
        if flags:
            out = self._leaves(sout)
            if any(t.is_inference() for t in out):
                self._chained = None
            else:
                self._chained = (tuple(weakref.ref(t) for t in out), tuple(t._version for t in out))

    def _ensure_bound(self):
        """sample_Pnx needs no init() with a raw potential_fn (arwmh.py:230-270
        calls only self._potential_fn and self.sample): bind the device
        potential on first use.  A model needs its data (init's model_kwargs)."""
        if self._handle is None:
            if self._potential_fn is None:
                raise RuntimeError("call init() (or get_init_adapt_state()) first")
            self._bind(0, {}, _device_index(self._device))

    def _chained_path(self) -> bool:
        """Paths whose step pass forms the next transition's proposal: d > 64
        (amh_big.hip) and the literal diamonds model's split transition
        (amh_split.hip; include/amh.h AMH_STEP_KEEP_PROPOSAL)."""
        if self._dim > 64:
            return True
        mid = self._model.model_id if self._model is not None else self._potential_fn.model_id
        return mid == _lib.AMH_MODEL_DIAMONDS and 3 <= self._dim <= 32

    def potential(self, z: torch.Tensor) -> torch.Tensor:
        """potential_fn(z) for a batch of flat points [n, d] (device)."""
        _lib.require_gpu(z)
        if self._external():
            return self._potential_fn.evaluate(z.to(torch.float32).contiguous().reshape(-1, self._dim))
        z = z.to(torch.float32).contiguous().reshape(-1, self._dim)
        pe = torch.empty(z.shape[0], dtype=torch.float32, device=z.device)
        with torch.cuda.device(z.device.index):
            _lib.check(_lib.lib().amh_potential(self._handle.h, _lib.ptr(z), _lib.ptr(pe), z.shape[0],
                                                _lib.stream_ptr(z.device.index)), self._handle.h)
        return pe

    def postprocess_fn(self, args, kwargs):
        if self._postprocess_fn is None:
            return lambda z: z
        return self._postprocess_fn(*args, **kwargs)

    def get_diagnostics_str(self, state):
        """arwmh.py:214-228 (chain-averaged for a batch)."""
        acc = float(state.mean_accept_prob.float().mean())
        step = float(torch.exp(state.adapt_state.log_step_size.float()).mean())
        return f"Acceptance rate: {acc:.2f}, Step size: {step:.3f}"

    def sample_Pnx(self, rng_key, x, adapt_state, n=1, n_samples=1000, jit_inner=True):
        """arwmh.py:230-270: n frozen-kernel steps from every x[i] for n_samples
        chains each, all sharing one adapt_state; returns [n_points, n_samples, d]."""
        self._ensure_bound()
        dev = torch.device("cuda", _device_index(self._device))
        x = torch.as_tensor(x.cpu() if hasattr(x, "cpu") else np.asarray(x), dtype=torch.float32)
        x = x.reshape(-1, self._dim).to(dev).contiguous()
        loc, scale, lam = adapt_state
        scale = torch.as_tensor(scale.cpu() if hasattr(scale, "cpu") else np.asarray(scale), dtype=torch.float32)
        if scale.dim() >= 2 and scale.shape[-1] == self._dim and scale.shape[-2] == self._dim:
            scale = pack_scale(scale.reshape(-1, self._dim, self._dim)[0])
        scale = scale.reshape(-1)[:packed_size(self._dim)].to(dev).contiguous()
        loc_t = torch.as_tensor(loc.cpu() if hasattr(loc, "cpu") else np.asarray(loc), dtype=torch.float32)
        loc_t = loc_t.reshape(-1)[:self._dim].to(dev).contiguous()
        lam = float(np.asarray(lam.cpu() if hasattr(lam, "cpu") else lam).reshape(-1)[0])
        if self._external():
            return self._sample_pnx_external(rng_key, x, scale, lam, int(n), int(n_samples), dev)
        out = torch.empty(x.shape[0], n_samples, self._dim, dtype=torch.float32, device=dev)
        with torch.cuda.device(dev.index):
            _lib.check(_lib.lib().amh_sample_pnx(self._handle.h, _lib.key_arr(as_key(rng_key)), _lib.ptr(x),
                                                 x.shape[0], n_samples, _lib.ptr(loc_t), _lib.ptr(scale), lam, n,
                                                 _lib.ptr(out), _lib.stream_ptr(dev.index)), self._handle.h)
        return out

    def _sample_pnx_external(self, rng_key, x, scale, lam, n, n_samples, dev):
        """sample_Pnx with the caller's potential: every step t is
        amh_pnx_propose, U of the proposals, amh_pnx_accept (include/amh.h)."""
        d, npts = self._dim, x.shape[0]
        C = npts * n_samples
        z = x.repeat_interleave(n_samples, dim=0).contiguous()  # chain p * n_samples + s starts at x[p]
        zp = torch.empty_like(z)
        key = _lib.key_arr(as_key(rng_key))
        L = _lib.lib()
        with torch.cuda.device(dev.index):
            st = _lib.stream_ptr(dev.index)
            pe = self._potential_fn.evaluate(z)
            for t in range(n):
                _lib.check(L.amh_pnx_propose(self._handle.h, key, _lib.ptr(z), C, _lib.ptr(scale), lam, t,
                                             _lib.ptr(zp), st), self._handle.h)
                pp = self._potential_fn.evaluate(zp)
                _lib.check(L.amh_pnx_accept(self._handle.h, key, _lib.ptr(z), _lib.ptr(pe), C, _lib.ptr(zp),
                                            _lib.ptr(pp), t, st), self._handle.h)
        return z.reshape(npts, n_samples, d)

    def get_init_adapt_state(self, rng_key, init_params, model_args=(), model_kwargs={}):
        """arwmh.py:272-276."""
        num_warmup = 0
        init_state = self.init(rng_key, num_warmup, init_params, model_args, model_kwargs)
        return init_state.adapt_state

    def unravel(self, z: torch.Tensor):
        """flat unconstrained z -> dict of sites (ravel_pytree inverse)."""
        if self._model is None:
            return z
        return self._model.unravel(z, self._model_kwargs)


def _clone_state(s: ARWMHState) -> ARWMHState:
    a = s.adapt_state
    return ARWMHState(s.i.clone(), s.z.clone(), s.potential_energy.clone(), s.mean_accept_prob.clone(),
                      ARWMHAdaptState(a.loc.clone(), a.scale.clone(), a.log_step_size.clone()),
                      s.as_change.clone(), s.rng_key.clone())


def ctypes_state(kernel: ARWMH, s: ARWMHState):
    return kernel._c_state(s)
