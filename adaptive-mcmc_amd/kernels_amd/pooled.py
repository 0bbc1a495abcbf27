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
doubles) is the only exchange: one all-reduce(sum) per step (per K steps
with sync_every = K) over RCCL on xGMI, on this package's own communicator
(distributed.RcclComm) through the C ABI's amh_pooled_allreduce.
"""
from __future__ import annotations

import ctypes
import weakref
from collections import namedtuple

import torch
import torch.distributed as dist

from . import _lib
from .arwmh import ARWMH, packed_size
from .random import as_key

PooledState = namedtuple("PooledState", ["i", "z", "potential_energy", "mean_accept_prob", "adapt_state",
                                         "as_change", "rng_key", "cov"])
PooledAdaptState = namedtuple("PooledAdaptState", ["loc", "scale", "log_step_size"])


AmhPooledState = _lib.AmhPooledState


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
    num_warmup must be a multiple of K.

    The all-reduce (RCCL, the package's own communicator) is enqueued on the
    compute stream between the stats and update launches; with overlap it
    runs on a side stream and the compute stream waits on its event only
    where the sums are consumed.

    overlap = True (the all-reduce overlapped with the next
    proposal) pools with a lag of one block: block b+1 runs with the shared
    state that block b-1's sums produced while block b's sums are still being
    all-reduced, i.e.

        theta_{b+1} = update(theta_b, sums_{b-1}),   theta_1 = theta_0,

    with the noise position advancing every block as usual.  The update rule
    is unchanged (delta measured from the mean of the block the sums come
    from); only which sums it consumes differs, so this is a delayed
    stochastic-approximation step.  The sums of the last block stay pending
    in the sampler and are applied by the next call.  Results do not depend on
    the rank count (up to the association order of the sums across ranks)."""

    pooled = True  # adapt-state leaves carry no chain axis

    def __init__(self, model=None, potential_fn=None, lr_decay=2 / 3, target_accept_prob=0.234, eps=1e-6,
                 num_chains=None, device=None, chain_offset=0, group=None, sync_every: int = 1,
                 overlap: bool = False, **kw):
        super().__init__(model=model, potential_fn=potential_fn, lr_decay=lr_decay,
                         target_accept_prob=target_accept_prob, eps=eps, num_chains=num_chains, device=device,
                         chain_offset=chain_offset, **kw)
        if int(sync_every) < 1:
            raise ValueError("sync_every must be >= 1")
        self._group = group
        self._sums = None
        self._bufs = None
        self._pending = None  # overlap: (buffer index, all-reduce event or None) not yet applied
        self._last_out = None  # overlap: weak reference to the z leaf of the state the pending sums belong to
        self._comm = None
        self.sync_every = int(sync_every)
        self.overlap = bool(overlap)
        # testing / profiling: run the multi-rank step (stats launch, the
        # all-reduce on the side stream, update launch) even in a world of one
        # rank, so the RCCL branch can be exercised and timed on one GPU
        self.force_collective = False
        # A/B: the non-overlapped all-reduce through torch.distributed on its
        # side stream (the round-4 path) instead of RCCL on the compute stream
        self.torch_stream_collective = False
        self._rccl_comm = None

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
        if d > 64 and d % 32 != 0:  # the pooled MFMA tiles (amh_pooled_stats returns AMH_EINVAL)
            raise ValueError(f"the pooled mode takes d <= 64 or a multiple of 32 up to 256, not d = {d}")
        f = dict(dtype=torch.float32, device=dev)
        eye = torch.eye(d, dtype=torch.float64, device=dev)
        from .arwmh import pack_scale
        cov = pack_scale(eye)
        adapt = PooledAdaptState(torch.zeros(d, **f), cov.to(torch.float32), torch.zeros(1, **f))
        self._bufs = torch.zeros(2, sums_size(d), dtype=torch.float64, device=dev)
        self._sums = self._bufs[0]
        self._pending = None
        self._last_out = None
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

    # ------------------------------------------------------- the exchange --
    def _allreduce(self, buf: torch.Tensor, dev: int):
        """all_reduce(sum) of one sums buffer.  RCCL without overlap: on the
        compute stream itself (kernels_amd.distributed.rccl_allreduce_sum:
        the update follows in stream order, no cross-stream event); returns
        None.  RCCL with overlap: enqueued on the side stream after the
        compute stream's work so far; returns the event the consumer waits
        on.  gloo (ranks sharing a device, CPU tests): done in place,
        host-synchronous; returns None."""
        if self._world() == 1 and not (self.force_collective and dist.is_available() and dist.is_initialized()):
            return None
        if dist.get_backend(self._group) != "nccl":
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self._group)
            return None
        if not self.overlap and not self.torch_stream_collective:
            # this package's own communicator (distributed.RcclComm), the
            # collective on the compute stream.  Setup (the id broadcast and
            # ncclCommInitRank) runs on every rank in the same host order;
            # any RCCL error raises -- no fallback once a collective may have
            # been issued.  Only a process without RCCL mapped (OSError, the
            # same on every rank) takes torch's stream instead.
            from .distributed import RcclComm
            if self._rccl_comm is None:
                try:
                    self._rccl_comm = RcclComm(self._group, buf.device)
                except OSError as e:
                    import warnings
                    warnings.warn(f"RCCL not mapped ({e}); using torch.distributed's stream", RuntimeWarning)
                    self.torch_stream_collective = True
            if self._rccl_comm is not None:
                self._rccl_comm.all_reduce_sum(buf, torch.cuda.current_stream(dev), handle=self._handle)
                return None
        if self._comm is None:
            self._comm = torch.cuda.Stream(device=dev)
        self._comm.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(self._comm):
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self._group)
            ev = torch.cuda.Event()
            ev.record(self._comm)
        return ev

    def close_comm(self):
        """Destroy this sampler's own RCCL communicator (collective over the
        group's ranks in the same host order; a later multi-rank step creates
        a new one)."""
        if self._rccl_comm is not None:
            c, self._rccl_comm = self._rccl_comm, None
            c.close()

    def _stats(self, L, cin, sout, buf, C):
        dev = sout.z.device.index
        _lib.check(L.amh_pooled_stats_k(self._handle.h, C, ctypes.byref(cin), self.sync_every, _lib.ptr(sout.z),
                                        _lib.ptr(sout.potential_energy), _lib.ptr(buf), _lib.stream_ptr(dev)),
                   self._handle.h)

    def _update(self, L, buf, cin, cout):
        dev = buf.device.index
        _lib.check(L.amh_pooled_update_k(self._handle.h, _lib.ptr(buf), ctypes.byref(cin), ctypes.byref(cout),
                                         self.sync_every, _lib.stream_ptr(dev)), self._handle.h)

    def _one(self, sin: PooledState, sout: PooledState):
        L = _lib.lib()
        dev = sin.z.device.index
        C = sin.z.shape[0]
        cin, cout = self._c(sin), self._c(sout)
        with torch.cuda.device(dev):
            if not self.overlap:
                buf = self._bufs[0]
                self._stats(L, cin, sout, buf, C)
                ev = self._allreduce(buf, dev)
                if ev is not None:
                    torch.cuda.current_stream(dev).wait_event(ev)
                self._update(L, buf, cin, cout)
                self._sums = buf
                return
            last = self._last_out() if self._last_out is not None else None
            if self._pending is not None and last is not sin.z:
                # a state this sampler did not just produce: the pending sums
                # belong to another trajectory, so this block starts afresh
                # (theta_1 = theta_0).  A checkpoint carries them instead
                # (checkpoint.state_dict(state, kernel)).
                self._pending = None
            b = 0 if self._pending is None else 1 - self._pending[0]
            buf = self._bufs[b]
            self._stats(L, cin, sout, buf, C)
            ev = self._allreduce(buf, dev)  # in flight while the next block computes
            if self._pending is not None:
                pb, pev = self._pending
                if pev is not None:
                    torch.cuda.current_stream(dev).wait_event(pev)
                self._update(L, self._bufs[pb], cin, cout)
            else:  # first block: theta_1 = theta_0, the noise position advances
                if sout is not sin:
                    for a, c in ((sin.adapt_state.loc, sout.adapt_state.loc),
                                 (sin.adapt_state.scale, sout.adapt_state.scale),
                                 (sin.adapt_state.log_step_size, sout.adapt_state.log_step_size),
                                 (sin.mean_accept_prob, sout.mean_accept_prob), (sin.as_change, sout.as_change),
                                 (sin.cov, sout.cov)):
                        c.copy_(a)
                torch.add(sin.i, self.sync_every, out=sout.i)
            self._pending = (b, ev)
            self._last_out = weakref.ref(sout.z)
            self._sums = buf

    # ------------------------------------------------ checkpoint (overlap) --
    def pending_sums(self):
        """overlap = True: the all-reduced sums of the last block, not yet
        applied (they update the shared state at the start of the next block),
        as a host float64 array; None when nothing is pending."""
        if self._pending is None:
            return None
        b, ev = self._pending
        if ev is not None:
            ev.synchronize()
        torch.cuda.synchronize(self._bufs.device)
        return self._bufs[b].detach().cpu().numpy().copy()

    def set_pending_sums(self, state, sums):
        """Make `sums` the pending sums of `state` (resume of an overlap run:
        the next block applies them exactly as the uninterrupted run would)."""
        if not self.overlap:
            raise ValueError("pending sums exist only with overlap=True")
        if self._bufs is None:
            raise RuntimeError("call init() first")
        self._bufs[0].copy_(torch.as_tensor(sums, dtype=torch.float64))
        self._pending = (0, None)
        self._last_out = weakref.ref(state.z)

    def check_device(self, synchronize: bool = True):
        """Raise if a launch of this sampler flagged a device-side failure (the
        d = 64 update's bounded wait ran out, so that update kept the shared
        factor: amh_check_device).  synchronize=False reads the flag without
        waiting, which covers every launch that has already finished; sample,
        sample_ and run call it that way after each call (and run, which
        synchronises anyway, with True); the handle's destruction reports what
        is left as a RuntimeWarning."""
        if self._handle is None:
            return
        if synchronize:
            torch.cuda.synchronize(self._handle.device)
        _lib.check(_lib.lib().amh_check_device(self._handle.h), self._handle.h)

    def sample(self, state, model_args=(), model_kwargs=None):
        """One pooled transition of every chain (sync_every > 1: one block of
        them); returns a new state."""
        self._check(state)
        out = self._new_like(state)
        self._one(state, out)
        self.check_device(synchronize=False)
        return out

    def sample_(self, state, n_steps: int = 1):
        """n_steps pooled transitions in place (a multiple of sync_every)."""
        C = self._check(state)
        K = self.sync_every
        if int(n_steps) % K != 0:
            raise ValueError(f"n_steps ({n_steps}) must be a multiple of sync_every ({K})")
        if self._world() == 1 and not self.overlap and not self.force_collective:
            L = _lib.lib()
            dev = state.z.device.index
            c = self._c(state)
            with torch.cuda.device(dev):
                _lib.check(L.amh_pooled_step_k(self._handle.h, C, ctypes.byref(c), ctypes.byref(c), int(n_steps), K,
                                               _lib.ptr(self._bufs[0]), _lib.stream_ptr(dev)), self._handle.h)
            self._sums = self._bufs[0]
            self.check_device(synchronize=False)
            return state
        for _ in range(int(n_steps) // K):
            self._one(state, state)
        self.check_device(synchronize=False)
        return state

    def run(self, state, n_steps: int, thinning: int = 1, collect_z: bool = True, collect_pe: bool = False):
        """n_steps pooled transitions (numpyro fori_collect over sample):
        returns (new_state, z [n_steps // thinning, C, d] or None, pe or None).
        Draws are taken at block ends, so thinning must be a multiple of
        sync_every (and n_steps of both)."""
        C = self._check(state)
        K = self.sync_every
        if int(thinning) < 1 or int(thinning) % K != 0 or int(n_steps) % K != 0:
            raise ValueError(f"thinning ({thinning}) and n_steps ({n_steps}) must be multiples of sync_every ({K})")
        out = self._new_like(state)  # (shares the constant rng_key leaf)
        for t, src in ((out.i, state.i), (out.z, state.z), (out.potential_energy, state.potential_energy),
                       (out.mean_accept_prob, state.mean_accept_prob), (out.as_change, state.as_change),
                       (out.cov, state.cov)) + tuple(zip(out.adapt_state, state.adapt_state)):
            t.copy_(src)
        if self._last_out is not None and self._last_out() is state.z:
            self._last_out = weakref.ref(out.z)  # the pending sums continue with the copy
        keep = int(n_steps) // int(thinning)
        dev = state.z.device
        cz = torch.empty(keep, C, self._dim, dtype=torch.float32, device=dev) if collect_z and keep else None
        cp = torch.empty(keep, C, dtype=torch.float32, device=dev) if collect_pe and keep else None
        done = 0
        for k in range(keep):
            self.sample_(out, int(thinning))
            done += int(thinning)
            if cz is not None:
                cz[k].copy_(out.z)
            if cp is not None:
                cp[k].copy_(out.potential_energy)
        if int(n_steps) > done:
            self.sample_(out, int(n_steps) - done)
        self.check_device(synchronize=True)
        return out, cz, cp

    def get_diagnostics_str(self, state):
        acc = float(state.mean_accept_prob[0])
        step = float(torch.exp(state.adapt_state.log_step_size[0]))
        return f"Acceptance rate: {acc:.2f}, Step size: {step:.3f}"
