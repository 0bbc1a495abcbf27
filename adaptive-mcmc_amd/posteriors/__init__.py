"""PosteriorDB model plug-in surface.

The reference plugs models in as NumPyro model functions (data passed as
model_kwargs, python/scripts/run_*_lr_decay.py) or as a raw potential_fn
callable (python/jupyter/asumptions_check.ipynb).  Device code cannot run a
Python callable, so each model here is a registry entry that knows

  * the flat unconstrained layout (ravel_pytree order = sorted site names),
  * how to pack the model's data for the device potential (include/amh.h),
  * how to map unconstrained draws back to constrained sites (postprocess).

Entries: eight_schools (non-centred), kidiq_kidscore_momhsiq, diamonds, a
dense Gaussian potential (the build's benchmark targets) and the notebook's
normal mixture potential (asumptions_check.ipynb cells 61-62).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Tuple

import numpy as np
import torch

from kernels_amd import _lib


@dataclass
class Site:
    name: str
    size: int
    transform: str = "identity"  # "identity" | "exp" (positive support, log-transformed)


@dataclass
class Model:
    """A registry entry: ARWMH(model=<Model>) with data in model_kwargs."""
    name: str
    model_id: int
    sites_fn: Callable[[dict], List[Site]]
    pack_fn: Callable[[dict], Tuple[np.ndarray, Tuple[int, ...]]]
    deterministic_fn: Callable[[Dict[str, torch.Tensor], dict], Dict[str, torch.Tensor]] = None
    doc: str = ""

    def sites(self, data: dict) -> List[Site]:
        return self.sites_fn(data)

    def dim(self, data: dict) -> int:
        return sum(s.size for s in self.sites(data))

    def pack(self, data: dict, device) -> Tuple[torch.Tensor, Tuple[int, ...]]:
        arr, ip = self.pack_fn(data)
        return torch.as_tensor(np.ascontiguousarray(arr, dtype=np.float32), device=device), ip

    def unravel(self, z: torch.Tensor, data: dict) -> Dict[str, torch.Tensor]:
        out, k = {}, 0
        for s in self.sites(data):
            v = z[..., k:k + s.size]
            out[s.name] = v[..., 0] if s.size == 1 else v
            k += s.size
        return out

    def postprocess(self, z: torch.Tensor, data: dict) -> Dict[str, torch.Tensor]:
        """unconstrained flat draws -> constrained sites (+ deterministic sites)."""
        raw = self.unravel(z, data)
        tr = {s.name: s.transform for s in self.sites(data)}
        out = {k: (torch.exp(v) if tr[k] == "exp" else v) for k, v in raw.items()}
        if self.deterministic_fn is not None:
            out.update(self.deterministic_fn(out, data))
        return out


def _np(x) -> np.ndarray:
    return np.asarray(x.cpu() if hasattr(x, "cpu") else x)


# ---------------------------------------------------------------- eight schools --
# run_eight_schools_lr_decay.py:26-35; data = PosteriorDB eight_schools (J = 8)
EIGHT_SCHOOLS_DATA = {
    "y": np.array([28.0, 8.0, -3.0, 7.0, -1.0, 1.0, 18.0, 12.0], np.float32),
    "sigma": np.array([15.0, 10.0, 16.0, 11.0, 9.0, 11.0, 10.0, 18.0], np.float32),
}  # posteriordb_eight-schools.ipynb:502-503


def _es_sites(data):
    J = len(_np(data["sigma"]))
    return [Site("mu", 1), Site("tau", 1, "exp"), Site("theta_base", J)]


def _es_pack(data):
    y = _np(data["y"]).astype(np.float32)
    s = _np(data["sigma"]).astype(np.float32)
    return np.concatenate([y, s, np.log(s.astype(np.float64)).astype(np.float32)]), (len(s),)


def _es_det(out, data):
    return {"theta": out["mu"][..., None] + out["tau"][..., None] * out["theta_base"]}


eight_schools = Model("eight_schools_noncentered", _lib.AMH_MODEL_EIGHT_SCHOOLS, _es_sites, _es_pack, _es_det,
                      "mu ~ N(0,5), tau ~ HalfCauchy(5), theta = mu + tau * theta_base, y ~ N(theta, sigma)")


# --------------------------------------------------------------------- kidiq --
# run_kidiq_kidscore_lr_decay.py:29-41
def _kid_sites(data):
    return [Site("beta", 3), Site("sigma", 1, "exp")]


def _kid_pack(data):
    kid = _np(data["kid_score"]).astype(np.float32)
    hs = _np(data["mom_hs"]).astype(np.float32)
    iq = _np(data["mom_iq"]).astype(np.float32)
    return np.concatenate([kid, hs, iq]), (len(kid),)


kidiq = Model("kidiq_kidscore_momhsiq", _lib.AMH_MODEL_KIDIQ, _kid_sites, _kid_pack, None,
              "beta ~ ImproperUniform, sigma ~ HalfCauchy(2.5), kid ~ N(b0 + b1 hs + b2 iq, sigma)")


def synthetic_kidiq(N: int = 434, seed: int = 434) -> dict:
    """kidiq-shaped synthetic data (the PosteriorDB file is not available offline)."""
    rng = np.random.default_rng(seed)
    hs = (rng.random(N) < 0.79).astype(np.float32)
    iq = rng.normal(100.0, 15.0, N).astype(np.float32)
    kid = (26.0 + 6.0 * hs + 0.56 * iq + rng.normal(0.0, 18.1, N)).astype(np.float32)
    return {"kid_score": kid, "mom_hs": hs, "mom_iq": iq}


# ------------------------------------------------------------------ diamonds --
# run_diamonds_lr_decay.py:24-40
def _dia_sites(data):
    K = _np(data["X"]).shape[1]
    return [Site("Intercept", 1), Site("b", K - 1), Site("sigma", 1, "exp")]


def _dia_pack(data):
    X = _np(data["X"]).astype(np.float32)
    Y = _np(data["Y"]).astype(np.float32)
    N, K = X.shape
    Xc = X[:, 1:] - X[:, 1:].mean(axis=0, dtype=np.float32)  # the model centres in fp32
    return np.concatenate([Xc.reshape(-1), Y]), (N, K)


diamonds = Model("diamonds", _lib.AMH_MODEL_DIAMONDS, _dia_sites, _dia_pack, None,
                 "Intercept ~ t3(8,10), b ~ N(0,1), sigma ~ |t3(0,10)|, Y ~ N(Intercept + Xc b, sigma)")


def diamonds_suffstats(data) -> np.ndarray:
    """float64 statistics of the float32 centred design the direct model reads
    (_dia_pack): [N, ybar, A = T'T, sT = sum T, t = Xc'T (Kc), sx = sum_n Xc_n
    (Kc), Gm = Xc'Xc (Kc x Kc, row-major)], T = Y - ybar."""
    flat, (N, K) = _dia_pack(data)
    Kc = K - 1
    Xc = flat[:N * Kc].reshape(N, Kc).astype(np.float64)
    Y = flat[N * Kc:].astype(np.float64)
    ybar = Y.mean()
    T = Y - ybar
    head = np.array([N, ybar, T @ T, T.sum()])
    return np.concatenate([head, Xc.T @ T, Xc.sum(axis=0), (Xc.T @ Xc).reshape(-1)])


def _dia_ss_pack(data):
    st = np.ascontiguousarray(diamonds_suffstats(data), dtype=np.float64)
    N, K = _np(data["X"]).shape
    return st.view(np.float32), (N, K)


# The same posterior with the likelihood's residual sum taken from float64
# sufficient statistics (O(K^2) per evaluation instead of O(N K)); it runs in
# the one-launch step kernel.  U differs from `diamonds` by the rounding of
# the float32 residual sum only.
diamonds_suffstat = Model("diamonds_suffstat", _lib.AMH_MODEL_DIAMONDS_SS, _dia_sites, _dia_ss_pack, None,
                          "diamonds, residual sum from float64 sufficient statistics")

# mean of the stored PosteriorDB reference draws for b[:4], Intercept, sigma
# (python/mcmc_runs/diamonds-example-references.pkl, read byte-wise)
_DIAMONDS_B_HEAD = np.array([6.660, 6.363, -4.684, 1.447])


def synthetic_diamonds(N: int = 5000, K: int = 25, seed: int = 26) -> dict:
    """Diamonds-shaped synthetic data: one-factor
    predictors with pairwise correlation 0.95-0.999, Y = 7.79 + Xc b* + 0.123 e."""
    rng = np.random.default_rng(seed)
    f = rng.normal(size=(N, 1))
    load = np.sqrt(rng.uniform(0.95, 0.999, size=(1, K - 1)))
    Xp = f * load + rng.normal(size=(N, K - 1)) * np.sqrt(1.0 - load ** 2)
    X = np.concatenate([np.ones((N, 1)), Xp], axis=1).astype(np.float32)
    b = np.zeros(K - 1)
    b[:4] = _DIAMONDS_B_HEAD
    b[4:] = rng.normal(0.0, 0.3, size=K - 5)
    Xc = X[:, 1:] - X[:, 1:].mean(axis=0)
    Y = (7.79 + Xc @ b + 0.123 * rng.normal(size=N)).astype(np.float32)
    return {"Y": Y, "X": X}


# ------------------------------------------------------------------ gaussian --
@dataclass
class Gaussian:
    """Dense Gaussian potential U(x) = 1/2 (x-m)' P (x-m) + 1/2 log|2 pi Sigma|
    (a raw potential_fn plug-in; arwmh.py:69-70 allows model XOR potential_fn)."""
    mean: np.ndarray
    precision: np.ndarray
    logdet_2pi_cov: float
    model_id: int = field(default=_lib.AMH_MODEL_GAUSSIAN, init=False)
    name: str = field(default="gaussian", init=False)

    @property
    def dim(self) -> int:
        return int(self.mean.shape[0])

    def pack(self, device) -> Tuple[torch.Tensor, Tuple[int, ...]]:
        d = self.dim
        P = np.asarray(self.precision, np.float64)
        P = 0.5 * (P + P.T)  # exactly symmetric after rounding
        arr = np.concatenate([np.asarray(self.mean, np.float64), P.reshape(-1),
                              [0.5 * self.logdet_2pi_cov]]).astype(np.float32)
        assert arr.size == d + d * d + 1
        return torch.as_tensor(arr, device=device), ()

    def __call__(self, z):
        """Host evaluation (float64), for diagnostics only."""
        x = np.asarray(_np(z), np.float64) - self.mean
        return 0.5 * np.einsum("...i,ij,...j->...", x, self.precision, x) + 0.5 * self.logdet_2pi_cov


def gaussian(mean, cov=None, precision=None) -> Gaussian:
    mean = np.asarray(mean, np.float64)
    d = mean.shape[0]
    if (cov is None) == (precision is None):
        raise ValueError("give exactly one of cov / precision")
    if cov is not None:
        cov = np.asarray(cov, np.float64)
        precision = np.linalg.inv(cov)
        sign, ld = np.linalg.slogdet(cov)
    else:
        precision = np.asarray(precision, np.float64)
        sign, ld = np.linalg.slogdet(precision)
        ld = -ld
    return Gaussian(mean, precision, float(d * math.log(2 * math.pi) + ld))


def correlated_gaussian(d: int = 64, log10_kappa: float = 2.0, seed: int = None) -> Gaussian:
    """Sigma = Q diag(s) Q', s_i = 10^(-k/2 + k i/(d-1)), Q from
    QR of an N(0,1) matrix drawn with default_rng(d) (config 2: d=64, kappa=1e2;
    config 4: d=256, kappa=1e4)."""
    rng = np.random.default_rng(d if seed is None else seed)
    Q, _ = np.linalg.qr(rng.normal(size=(d, d)))
    k = log10_kappa
    s = 10.0 ** (-k / 2 + k * np.arange(d) / max(d - 1, 1))
    cov = (Q * s) @ Q.T
    return gaussian(np.zeros(d), cov=cov)


# ------------------------------------------------------------------- mixture --
@dataclass
class Mixture:
    """Univariate normal mixture on every coordinate, a raw potential_fn
    plug-in: U(x) = -sum_r log sum_k w_k N(x_r; m_k, s_k) (asumptions_check.ipynb
    cells 61-62, `-mixture.log_prob(x)` of numpyro's MixtureSameFamily; the
    notebook's x is 1-D, so its vector-valued potential has one entry)."""
    weights: np.ndarray
    locs: np.ndarray
    scales: np.ndarray
    dim: int = 1
    model_id: int = field(default=_lib.AMH_MODEL_MIXTURE, init=False)
    name: str = field(default="mixture", init=False)

    def pack(self, device) -> Tuple[torch.Tensor, Tuple[int, ...]]:
        w = np.asarray(self.weights, np.float64)
        s = np.asarray(self.scales, np.float64)
        c = np.log(w) - np.log(np.sqrt(2 * np.pi) * s)
        arr = np.concatenate([c, np.asarray(self.locs, np.float64), s]).astype(np.float32)
        return torch.as_tensor(arr, device=device), (len(w),)

    def __call__(self, z):
        """Host evaluation (float64), for diagnostics only."""
        x = np.asarray(_np(z), np.float64)[..., None]
        lp = np.log(np.asarray(self.weights, np.float64)) - 0.5 * ((x - self.locs) / self.scales) ** 2 \
            - np.log(np.sqrt(2 * np.pi) * np.asarray(self.scales, np.float64))
        mx = lp.max(axis=-1, keepdims=True)
        return -(np.log(np.exp(lp - mx).sum(axis=-1)) + mx[..., 0]).sum(axis=-1)


def mixture(weights, locs, scales, dim: int = 1) -> Mixture:
    w = np.asarray(weights, np.float64).reshape(-1)
    m = np.asarray(locs, np.float64).reshape(-1)
    s = np.asarray(scales, np.float64).reshape(-1)
    if not (w.shape == m.shape == s.shape) or not 1 <= w.size <= 8:
        raise ValueError("mixture needs 1..8 components with matching weights / locs / scales")
    if np.any(w <= 0) or abs(w.sum() - 1.0) > 1e-6 or np.any(s <= 0):
        raise ValueError("mixture weights must be positive and sum to 1, scales positive")
    if not 1 <= int(dim) <= 16:
        raise ValueError("mixture supports 1 <= dim <= 16")
    return Mixture(w, m, s, int(dim))


# asumptions_check.ipynb cell 61: 1/2 N(-1, 0.1) + 1/2 N(1, 0.1)
def notebook_mixture() -> Mixture:
    return mixture([0.5, 0.5], [-1.0, 1.0], [0.1, 0.1])


# ------------------------------------------------------------------ external --
@dataclass
class TorchPotential:
    """Any potential the caller writes (arwmh.py:69-70: `potential_fn` is an
    arbitrary callable there): `fn` maps a device batch z [n, d] float32 to
    U(z) [n] (-log density, NaN allowed: it rejects).  ARWMH runs the rest
    of the transition in its kernels around it (include/amh.h
    AMH_MODEL_EXTERNAL: amh_propose, fn, amh_step_external), 1 <= d <= 256.
    `dim` may be left None: init() takes it from init_params."""
    fn: Callable
    dim: int = None
    model_id: int = field(default=_lib.AMH_MODEL_EXTERNAL, init=False)
    name: str = field(default="external", init=False)

    def pack(self, device) -> Tuple[torch.Tensor, Tuple[int, ...]]:
        return torch.zeros(1, dtype=torch.float32, device=device), ()  # no data (the library reads none)

    def evaluate(self, z: torch.Tensor) -> torch.Tensor:
        u = self.fn(z)
        u = torch.as_tensor(u, device=z.device).to(torch.float32).reshape(-1)
        if u.shape[0] != z.shape[0]:
            raise ValueError(f"potential_fn returned {tuple(u.shape)} values for {z.shape[0]} points (one each)")
        return u.contiguous()

    def __call__(self, z):
        return self.fn(z)


def torch_potential(fn: Callable, dim: int = None) -> TorchPotential:
    if dim is not None and not 1 <= int(dim) <= 256:
        raise ValueError("an external potential supports 1 <= dim <= 256")
    return TorchPotential(fn, None if dim is None else int(dim))


REGISTRY = {
    "eight_schools": eight_schools,
    "eight_schools_noncentered": eight_schools,
    "kidiq": kidiq,
    "kidiq_kidscore_momhsiq": kidiq,
    "diamonds": diamonds,
    "diamonds_suffstat": diamonds_suffstat,
}
