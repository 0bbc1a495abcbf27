"""MCMC diagnostics behind `MCMC.print_summary` (the reference prints these
tables in posteriordb_eight-schools.ipynb cells 27-29 and uses n_eff / ESS in
its evaluation).

The reference gets them from numpyro.diagnostics (third party, version
unpinned in python/environment.yml:10, not importable here).  This module
restates numpyro's published estimators on host arrays:

  autocorrelation / autocovariance  FFT of the centred signal, zero-padded to
                                    twice the next fast length; biased
                                    estimator by default
  effective_sample_size             Stan's multi-chain estimator (BDA3 11.5):
                                    rho_k = 1 - (W - mean_c acov_c(k)) / var+,
                                    Geyer's initial positive sequence over lag
                                    pairs made monotone, tau = -1 + 2 sum
  gelman_rubin / split_gelman_rubin sqrt(var+ / W), split = halves as chains
  hpdi                              narrowest interval holding int(prob * n)
  summary / print_summary           mean, std (ddof 0), median, HPDI bounds,
                                    n_eff, r_hat; numpyro's table layout

Inputs are [num_chains, num_draws, ...] (group_by_chain) numpy arrays or
torch tensors (moved to host: these are post-processing, not the hot path).
Parity: against the numbers printed by the reference notebook only in
distribution (different draws); the estimator definitions are pinned by the
known-answer tests in tests/test_infer.py (AR(1) chains with closed-form
tau, iid chains, split-R-hat of shifted chains).
"""
from __future__ import annotations

from collections import OrderedDict
from itertools import product

import numpy as np

__all__ = ["autocorrelation", "autocovariance", "effective_sample_size", "gelman_rubin", "split_gelman_rubin",
           "hpdi", "summary", "print_summary"]


def _host(x) -> np.ndarray:
    if hasattr(x, "detach"):
        x = x.detach().cpu().numpy()
    return np.asarray(x)


def _fft_next_fast_len(target: int) -> int:
    # numpyro: the next integer >= target of the form 2^a 3^b 5^c
    if target <= 2:
        return target
    while True:
        m = target
        while m % 2 == 0:
            m //= 2
        while m % 3 == 0:
            m //= 3
        while m % 5 == 0:
            m //= 5
        if m == 1:
            return target
        target += 1


def autocorrelation(x, axis: int = 0, bias: bool = True) -> np.ndarray:
    """Autocorrelation of x along `axis` (lag 0 normalised to 1)."""
    x = _host(x).astype(np.float64, copy=False)
    N = x.shape[axis]
    M2 = 2 * _fft_next_fast_len(N)
    x = np.swapaxes(x, axis, -1)
    centred = x - x.mean(axis=-1, keepdims=True)
    f = np.fft.rfft(centred, n=M2, axis=-1)
    ac = np.fft.irfft(f * np.conjugate(f), n=M2, axis=-1)[..., :N]
    if not bias:
        ac = ac / np.arange(N, 0.0, -1)
    with np.errstate(invalid="ignore", divide="ignore"):
        ac = ac / ac[..., :1]
    return np.swapaxes(ac, axis, -1)


def autocovariance(x, axis: int = 0, bias: bool = True) -> np.ndarray:
    x = _host(x).astype(np.float64, copy=False)
    return autocorrelation(x, axis, bias) * x.var(axis=axis, keepdims=True)


def _chain_variance_stats(x: np.ndarray):
    C, N = x.shape[:2]
    var_within = x.var(axis=1, ddof=1).mean(axis=0)
    var_estimator = var_within * (N - 1) / N
    if C > 1:
        var_estimator = var_estimator + x.mean(axis=1).var(axis=0, ddof=1)
    else:
        var_within = var_estimator
    return var_within, var_estimator


def _effective_sample_size_torch(x):
    """The same estimator on a torch tensor's own device (float64): many-chain
    draws (65,536 chains x 1,000 draws in bench.py) stay in HBM.  Line for
    line the numpy path below; tests/test_infer.py checks the two agree."""
    import torch
    x = x.detach().to(torch.float64)
    C, N = x.shape[:2]
    M2 = 2 * _fft_next_fast_len(N)
    xs = x.movedim(1, -1)
    centred = xs - xs.mean(dim=-1, keepdim=True)
    f = torch.fft.rfft(centred, n=M2, dim=-1)
    ac = torch.fft.irfft(f * f.conj(), n=M2, dim=-1)[..., :N]
    ac = ac / ac[..., :1]
    gamma = (ac * xs.var(dim=-1, unbiased=False, keepdim=True)).movedim(-1, 1)
    var_within = x.var(dim=1, unbiased=True).mean(dim=0)
    var_estimator = var_within * (N - 1) / N
    if C > 1:
        var_estimator = var_estimator + x.mean(dim=1).var(dim=0, unbiased=True)
    else:
        var_within = var_estimator
    rho = 1.0 - (var_within - gamma.mean(dim=0)) / var_estimator
    rho[0] = 1.0
    Rho = rho[:-1:2] + rho[1::2]
    tail = torch.cummin(Rho[1:].clamp(min=0.0), dim=0).values
    Rho = torch.cat([Rho[:1], tail], dim=0)
    tau = -1.0 + 2.0 * Rho.sum(dim=0)
    return (C * N / tau).cpu().numpy()


def effective_sample_size(x) -> np.ndarray:
    """Multi-chain ESS of x [num_chains, num_draws, ...] (a torch tensor is
    reduced on its own device)."""
    if hasattr(x, "detach"):
        if x.ndim < 2 or x.shape[1] < 2:
            raise ValueError("effective_sample_size needs x of shape [chains, draws >= 2, ...]")
        return _effective_sample_size_torch(x)
    x = _host(x).astype(np.float64, copy=False)
    if x.ndim < 2 or x.shape[1] < 2:
        raise ValueError("effective_sample_size needs x of shape [chains, draws >= 2, ...]")
    gamma = autocovariance(x, axis=1)
    var_within, var_estimator = _chain_variance_stats(x)
    rho = 1.0 - (var_within - gamma.mean(axis=0)) / var_estimator
    rho[0] = 1.0
    Rho = rho[:-1:2, ...] + rho[1::2, ...]
    Rho = np.concatenate([Rho[:1], np.minimum.accumulate(np.clip(Rho[1:, ...], 0.0, None), axis=0)], axis=0)
    tau = -1.0 + 2.0 * np.sum(Rho, axis=0)
    return np.prod(x.shape[:2]) / tau


def gelman_rubin(x) -> np.ndarray:
    x = _host(x).astype(np.float64, copy=False)
    if x.ndim < 2 or x.shape[1] < 2:
        raise ValueError("gelman_rubin needs x of shape [chains, draws >= 2, ...]")
    var_within, var_estimator = _chain_variance_stats(x)
    return np.sqrt(var_estimator / var_within)


def split_gelman_rubin(x) -> np.ndarray:
    x = _host(x).astype(np.float64, copy=False)
    if x.ndim < 2 or x.shape[1] < 4:
        raise ValueError("split_gelman_rubin needs x of shape [chains, draws >= 4, ...]")
    h = x.shape[1] // 2
    return gelman_rubin(np.concatenate([x[:, :h], x[:, -h:]], axis=0))


def hpdi(x, prob: float = 0.90, axis: int = 0) -> np.ndarray:
    """Highest posterior density interval: [lower, upper] stacked on `axis`."""
    x = np.swapaxes(_host(x), axis, 0)
    s = np.sort(x, axis=0)
    mass = x.shape[0]
    k = int(prob * mass)
    start = (s[k:] - s[: mass - k]).argmin(axis=0)
    lo = np.take_along_axis(s, start[None, ...], axis=0)
    hi = np.take_along_axis(s, (start + k)[None, ...], axis=0)
    return np.swapaxes(np.concatenate([lo, hi], axis=0), axis, 0)


def summary(samples, prob: float = 0.90, group_by_chain: bool = True) -> "OrderedDict[str, dict]":
    """Per-site statistics.  samples: dict name -> [chains, draws, ...] (or
    [draws, ...] with group_by_chain=False), or one array."""
    if not isinstance(samples, dict):
        samples = {"Param:0": samples}
    out = OrderedDict()
    lo_name, hi_name = "{:.1f}%".format(50 * (1 - prob)), "{:.1f}%".format(50 * (1 + prob))
    for name, v in samples.items():
        v = _host(v).astype(np.float64, copy=False)
        if not group_by_chain:
            v = v[None, ...]
        flat = v.reshape((-1,) + v.shape[2:])
        iv = hpdi(flat, prob)
        out[name] = OrderedDict([
            ("mean", v.mean(axis=(0, 1))),
            ("std", v.std(axis=(0, 1))),
            ("median", np.median(v, axis=(0, 1))),
            (lo_name, iv[0]),
            (hi_name, iv[1]),
            ("n_eff", effective_sample_size(v)),
            ("r_hat", split_gelman_rubin(v)),
        ])
    return out


def format_summary(samples, prob: float = 0.90, group_by_chain: bool = True) -> str:
    """numpyro's print_summary table as a string."""
    if not isinstance(samples, dict):
        samples = {"Param:0": samples}
    if not group_by_chain:
        samples = {k: _host(v)[None, ...] for k, v in samples.items()}
    stats = summary(samples, prob, group_by_chain=True)
    shapes = {k: _host(v).shape[2:] for k, v in samples.items()}
    labels = []
    for k, shp in shapes.items():
        if len(shp) == 0:
            labels.append(k)
        else:
            labels += [k + "[" + ",".join(map(str, idx)) + "]" for idx in product(*map(range, shp))]
    w = max(max(len(s) for s in labels), 10)
    name_f = "{:>" + str(w) + "}"
    cols = [""] + list(next(iter(stats.values())).keys())
    lines = ["", (name_f + " {:>9}" * 7).format(*cols)]
    row_f = name_f + " {:>9.2f}" * 7
    for name, st in stats.items():
        shp = st["mean"].shape
        if len(shp) == 0:
            lines.append(row_f.format(name, *st.values()))
        else:
            for idx in product(*map(range, shp)):
                lines.append(row_f.format(name + "[{}]".format(",".join(map(str, idx))), *[v[idx] for v in st.values()]))
    lines.append("")
    return "\n".join(lines)


def print_summary(samples, prob: float = 0.90, group_by_chain: bool = True) -> None:
    print(format_summary(samples, prob, group_by_chain))
