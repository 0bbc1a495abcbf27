"""MCMC driver: warmup, sampling with thinning, extra fields, constrained
samples and the summary table -- the caller side of `sample()` in the
reference (numpyro `infer.MCMC(ARWMH(model), num_warmup, num_samples,
thinning).run(key, **data, extra_fields=...)`, python/scripts/
run_*_wasserstein.py:48-52, posteriordb_eight-schools.ipynb cells 27-29).

numpyro runs `num_chains` copies of a single-chain kernel; here the kernel is
already batched over chains (ARWMH(num_chains=C)), so `num_chains` is the
kernel's chain count and every step advances all chains in one launch.

Collection follows numpyro's fori_collect: after `num_warmup` steps, the
state is recorded after step num_warmup + r + k * thinning for k = 1 ..
num_samples // thinning, r = num_samples % thinning.  z and
potential_energy are written by the step kernel itself during one fused
launch (ARWMH.run); any other extra field (e.g. "adapt_state",
"mean_accept_prob", "as_change") is snapshot on device after each
thinning-long fused launch.  Both launch partitions are bit-reproducible
(each equals the oracle run with the same partition); they differ from each
other at ULP level, because a fused launch carries the factor in unit-lower
form between its steps.
"""
from __future__ import annotations

from operator import attrgetter
from typing import Dict, Sequence

import torch

from . import diagnostics

__all__ = ["MCMC"]


def _tmap(f, x):
    """Apply f to every tensor leaf of a (nested) namedtuple / tuple / dict."""
    if isinstance(x, torch.Tensor):
        return f(x)
    if isinstance(x, dict):
        return {k: _tmap(f, v) for k, v in x.items()}
    if isinstance(x, tuple) and hasattr(x, "_fields"):
        return type(x)(*[_tmap(f, v) for v in x])
    if isinstance(x, (tuple, list)):
        return type(x)(_tmap(f, v) for v in x)
    return x


def _stack(xs):
    first = xs[0]
    if isinstance(first, torch.Tensor):
        return torch.stack(xs, dim=0)
    if isinstance(first, tuple) and hasattr(first, "_fields"):
        return type(first)(*[_stack([x[i] for x in xs]) for i in range(len(first))])
    if isinstance(first, dict):
        return {k: _stack([x[k] for x in xs]) for k in first}
    raise TypeError(f"cannot collect a field of type {type(first).__name__}")


class MCMC:
    """numpyro.infer.MCMC for the device kernels (ARWMH, PooledARWMH).

    Parameters follow numpyro: num_warmup, num_samples, num_chains (must
    match the kernel's chain count if given), thinning, postprocess_fn
    (default: the kernel's postprocess_fn, i.e. the model's constraining
    transforms), progress_bar / chain_method / jit_model_args (accepted and
    ignored: there is one launch per step for all chains)."""

    def __init__(self, sampler, *, num_warmup, num_samples, num_chains=None, thinning=1, postprocess_fn=None,
                 chain_method="vectorized", progress_bar=False, jit_model_args=False):
        if int(thinning) < 1:
            raise ValueError("thinning must be a positive integer")
        if int(num_warmup) < 0 or int(num_samples) < 0:
            raise ValueError("num_warmup and num_samples must be >= 0")
        self.sampler = sampler
        self.num_warmup = int(num_warmup)
        self.num_samples = int(num_samples)
        self.num_chains = num_chains
        self.thinning = int(thinning)
        self.postprocess_fn = postprocess_fn
        self.chain_method = chain_method
        self.progress_bar = progress_bar
        self._states = None  # {"z": [C, K, d], field: [C, K, ...]}
        self._last_state = None
        self._warmup_state = None
        self._args = ((), {})

    # ------------------------------------------------------------ properties --
    @property
    def last_state(self):
        return self._last_state

    @property
    def post_warmup_state(self):
        return self._warmup_state

    @post_warmup_state.setter
    def post_warmup_state(self, state):
        self._warmup_state = state

    # ----------------------------------------------------------------- setup --
    def _init(self, rng_key, args, kwargs, init_params):
        if self.num_chains is not None:
            nc = getattr(self.sampler, "_num_chains", None)
            if nc is None:
                self.sampler._num_chains = int(self.num_chains)
            elif int(nc) != int(self.num_chains):
                raise ValueError(f"num_chains={self.num_chains} but the kernel holds {nc} chains")
        state = self.sampler.init(rng_key, self.num_warmup, init_params, args, kwargs)
        self.num_chains = int(state.z.shape[0])
        self._args = (args, kwargs)
        return state

    def warmup(self, rng_key, *args, extra_fields=(), collect_warmup=False, init_params=None, **kwargs):
        """Run num_warmup steps only; the result becomes post_warmup_state and a
        following run() continues from it."""
        state = self._init(rng_key, args, kwargs, init_params)
        if collect_warmup:
            state, self._states = self._collect(state, self.num_warmup, 1, extra_fields)
        else:
            self.sampler.sample_(state, self.num_warmup)
        self._warmup_state = state
        self._last_state = state
        return state

    def run(self, rng_key, *args, extra_fields: Sequence[str] = (), init_params=None, **kwargs):
        """Warmup (unless post_warmup_state is set) then num_samples steps,
        recording every thinning-th state."""
        if self._warmup_state is not None:
            state = _tmap(torch.clone, self._warmup_state)
        else:
            state = self._init(rng_key, args, kwargs, init_params)
            self.sampler.sample_(state, self.num_warmup)
            self._warmup_state = _tmap(torch.clone, state)
        state, self._states = self._collect(state, self.num_samples, self.thinning, extra_fields)
        self._last_state = state
        return None

    def _collect(self, state, n: int, thinning: int, fields: Sequence[str]):
        s = self.sampler
        fields = tuple(fields)
        for f in fields:
            attrgetter(f)(state)  # AttributeError for an unknown field, as numpyro
        rem, keep = n % thinning, n // thinning
        if rem:
            s.sample_(state, rem)
        C = state.z.shape[0]
        out: Dict[str, object] = {}
        pooled = getattr(s, "pooled", False)
        fused = not pooled and set(fields) <= {"potential_energy"}
        if keep == 0:
            out["z"] = state.z.new_empty((C, 0) + tuple(state.z.shape[1:]))
            for f in fields:
                out[f] = _tmap(lambda t: t.new_empty((C, 0) + tuple(t.shape[1:])), attrgetter(f)(state))
            return state, out
        if fused:
            state, cz, cp = s.run(state, keep * thinning, thinning, collect_z=True,
                                  collect_pe="potential_energy" in fields)
            out["z"] = cz.transpose(0, 1).contiguous()
            if cp is not None:
                out["potential_energy"] = cp.transpose(0, 1).contiguous()
            return state, out
        zs, ex = [], {f: [] for f in fields}
        for _ in range(keep):
            s.sample_(state, thinning)
            zs.append(state.z.clone())
            for f in fields:
                ex[f].append(_tmap(torch.clone, attrgetter(f)(state)))

        def chain_major(t):
            # [K, C, ...] -> [C, K, ...]
            return t.transpose(0, 1).contiguous()

        def shared(t):
            # a pooled kernel's shared leaf [K, ...] -> [1, K, ...]
            return t.unsqueeze(0)

        out["z"] = chain_major(torch.stack(zs, 0))
        for f in fields:
            per_chain = not pooled or f in ("potential_energy", "rng_key")
            out[f] = _tmap(chain_major if per_chain else shared, _stack(ex[f]))
        return state, out

    # --------------------------------------------------------------- results --
    def _require(self):
        if self._states is None:
            raise RuntimeError("call run() first")

    @staticmethod
    def _flatten(x, group_by_chain):
        if group_by_chain:
            return x
        return _tmap(lambda t: t.reshape((-1,) + tuple(t.shape[2:])), x)

    def _constrained(self):
        z = self._states["z"]
        fn = self.postprocess_fn
        if fn is None:
            args, kwargs = self._args
            fn = self.sampler.postprocess_fn(args, kwargs)
        return fn(z)

    def get_samples(self, group_by_chain: bool = False):
        """Constrained samples: dict site -> [C * K, ...] ([C, K, ...] with
        group_by_chain), or the flat z array for a potential_fn kernel."""
        self._require()
        return self._flatten(self._constrained(), group_by_chain)

    def get_extra_fields(self, group_by_chain: bool = False):
        self._require()
        return {k: self._flatten(v, group_by_chain) for k, v in self._states.items() if k != "z"}

    def _summary_sites(self, exclude_deterministic: bool):
        sites = self._constrained()
        model = getattr(self.sampler, "model", None)
        if isinstance(sites, dict) and exclude_deterministic and model is not None:
            names = {s.name for s in model.sites(self._args[1] or self.sampler._model_kwargs)}
            sites = {k: v for k, v in sites.items() if k in names}
        return sites

    def summary_str(self, prob: float = 0.9, exclude_deterministic: bool = True) -> str:
        self._require()
        return diagnostics.format_summary(self._summary_sites(exclude_deterministic), prob=prob)

    def print_summary(self, prob: float = 0.9, exclude_deterministic: bool = True) -> None:
        """numpyro MCMC.print_summary: mean, std, median, HPDI, n_eff, r_hat
        per site over all chains (grouped by chain)."""
        print(self.summary_str(prob, exclude_deterministic))
