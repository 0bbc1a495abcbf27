"""Literal numpy restatement of the reference ARWMH hot path.

TEST INFRASTRUCTURE ONLY (never imported by the product package).

This is the *semantic* oracle: it follows the reference statement by
statement, in the reference's own arithmetic order, at a selectable precision
(float64 "shadow" by default, float32 to mimic the reference's dtype).  It
pins the bit-level C oracle (oracle/amh_oracle.c, whose operation order
matches the HIP kernels) within floating-point tolerance.

Reference anchors (/root/reference):
  ARWMH.init             python/kernels/arwmh.py:84-138
  ARWMH.sample           python/kernels/arwmh.py:140-207
  ARWMH.sample_Pnx       python/kernels/arwmh.py:230-270
  cholesky_update        numpyro.distributions.util.cholesky_update (called at
                         arwmh.py:190; unpinned numpyro, Krause & Igel 2015)
  ns_logscale            python/utils/kernel_utils.py:8-12
  eight_schools model    python/scripts/run_eight_schools_lr_decay.py:26-35
  kidiq model            python/scripts/run_kidiq_kidscore_lr_decay.py:29-41
  diamonds model         python/scripts/run_diamonds_lr_decay.py:24-40
"""
from __future__ import annotations

import math
from collections import namedtuple

import numpy as np
from scipy.special import gammaln

ARWMHState = namedtuple("ARWMHState", ["i", "z", "potential_energy", "mean_accept_prob",
                                       "adapt_state", "as_change", "rng_key"])
ARWMHAdaptState = namedtuple("ARWMHAdaptState", ["loc", "scale", "log_step_size"])

# ----------------------------------------------------------------- philox --
M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
TAG_CHAINKEY, TAG_INIT, TAG_STEP, TAG_SPLIT = 0x4B48434D, 0x54494E49, 0x50455453, 0x54494C50
_MASK = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 (Salmon et al. SC'11). uint32 arrays in/out."""
    c0, c1, c2, c3 = (np.asarray(c, np.uint32) for c in (c0, c1, c2, c3))
    c0, c1, c2, c3 = np.broadcast_arrays(c0, c1, c2, c3)
    k0 = np.asarray(k0, np.uint32)
    k1 = np.asarray(k1, np.uint32)
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & _MASK).astype(np.uint32)
            hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & _MASK).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = (k0 + W0).astype(np.uint32)
            k1 = (k1 + W1).astype(np.uint32)
    return c0, c1, c2, c3


def unif01_from_bits(b):
    """jax.random.uniform's bits -> [0,1) construction, exact in float32."""
    b = np.asarray(b, np.uint32)
    return ((b >> np.uint32(9)) | np.uint32(0x3F800000)).view(np.float32) - np.float32(1.0)


def normal_from_bits(b, dtype=np.float64):
    """sqrt(2) * erfinv(u), u uniform on [nextafter(-1, 0), 1) (jax.random.normal)."""
    from scipy.special import erfinv
    f = unif01_from_bits(b)
    lo = np.float32(np.nextafter(np.float32(-1), np.float32(0)))
    u = np.maximum(lo, f * np.float32(2.0) + lo)
    return (np.sqrt(2.0) * erfinv(u.astype(np.float64))).astype(dtype)


def chain_keys(key, chain_offset, n):
    g = np.arange(chain_offset, chain_offset + n, dtype=np.uint64)
    o = philox4x32_10((g & _MASK).astype(np.uint32), (g >> np.uint64(32)).astype(np.uint32), 0,
                      TAG_CHAINKEY, np.uint32(key[0]), np.uint32(key[1]))
    return np.stack([o[0], o[1]], axis=-1)


def step_noise(keys, ctr, d):
    """Per-chain proposal noise bits [C, d] and accept-uniform bits [C] for a step at
    stream position ctr (= state.i for ARWMH.sample): the words
    W_j = Philox(j >> 2, ctr, 0, TAG_STEP; key)[j & 3], xi_r from W_r (r < d),
    u from W_d (include/amh_math.h amh_step_word)."""
    keys = np.asarray(keys, np.uint32).reshape(-1, 2)
    nc = d // 4 + 1
    c = np.arange(nc, dtype=np.uint32)[None, :]
    ctr = np.broadcast_to(np.asarray(ctr, np.uint32).reshape(-1, 1), (keys.shape[0], 1))
    o = philox4x32_10(c, ctr, 0, TAG_STEP, keys[:, 0:1], keys[:, 1:2])
    words = np.stack(o, axis=-1).reshape(keys.shape[0], 4 * nc)  # W_j at [:, j]
    return words[:, :d], words[:, d]


# ------------------------------------------------------------ cholupdate --
def cholesky_update(L, x, coef, dtype=np.float64):
    """numpyro.distributions.util.cholesky_update, literal (Krause & Igel 2015):
    returns the Cholesky factor of L L^T + coef x x^T."""
    L = np.asarray(L, dtype)
    x = np.asarray(x, dtype)
    coef = dtype(coef)
    with np.errstate(all="ignore"):
        diag = np.diagonal(L).copy()
        U = L / diag[None, :]
        D = np.square(diag)
        b = dtype(1.0)
        w = x.copy()
        Dn = np.empty_like(D)
        for j in range(L.shape[0]):
            Dj, Lj = D[j], U[:, j].copy()
            wj = w[j]
            gamma = b * Dj + coef * np.square(wj)
            Dn[j] = gamma / b
            b = gamma / Dj
            w = w - wj * Lj
            U[:, j] = Lj + (coef * wj / gamma) * w
        return U * np.sqrt(Dn)[None, :]


# ------------------------------------------------------------------ step --
def lr_gamma(n, a, dtype=np.float64):
    return dtype(1) / dtype(n) ** dtype(a)


def sample(state: ARWMHState, potential_fn, xi, u, num_warmup=0, lr_decay=2 / 3,
           target_accept_prob=0.234, eps=1e-6, dtype=np.float64):
    """ARWMH.sample (arwmh.py:140-207) for ONE chain with injected noise xi [d], u."""
    i, z, pe, macc, adapt, _, key = state
    mu, L, lam = adapt
    z = np.asarray(z, dtype)
    dim = z.shape[0]
    with np.errstate(all="ignore"):
        prop_scale = np.asarray(L, dtype) * np.exp(dtype(lam)) + np.eye(dim, dtype=dtype) * dtype(eps)
        zp = z + prop_scale @ np.asarray(xi, dtype)
        pep = dtype(potential_fn(zp))
        pep = dtype(np.inf) if np.isnan(pep) else pep
        accept_prob = np.minimum(np.exp(dtype(pe) - pep), dtype(1))
        accepted = bool(dtype(u) < accept_prob)
        zn = zp if accepted else z
        pen = pep if accepted else dtype(pe)
        itr = int(i) + 1
        n = itr if int(i) < num_warmup else itr - num_warmup
        gamma = lr_gamma(n, lr_decay, dtype)
        maccn = dtype(macc) + (accept_prob - dtype(macc)) / dtype(n)
        delta = zn - np.asarray(mu, dtype)
        mun = np.asarray(mu, dtype) + gamma * delta
        chol = cholesky_update(np.sqrt(dtype(1) - gamma) * np.asarray(L, dtype), delta, gamma, dtype)
        Ln = np.asarray(L, dtype) if np.any(np.isnan(chol)) else chol
        lamn = dtype(lam) + gamma * (accept_prob - dtype(target_accept_prob))
        asc = np.linalg.norm(Ln * np.exp(lamn) - np.asarray(L, dtype) * np.exp(dtype(lam)), "fro")
    return ARWMHState(itr, zn, pen, maccn, ARWMHAdaptState(mun, Ln, lamn), asc, key), accepted, accept_prob


# ---------------------------------------------------------------- models --
HALF_LOG_2PI = 0.5 * math.log(2 * math.pi)


def normal_lp(x, loc, scale):
    return -0.5 * ((x - loc) / scale) ** 2 - np.log(scale) - HALF_LOG_2PI


def halfcauchy_lp(x, scale):
    return math.log(2.0) - math.log(math.pi) - np.log(scale) - np.log1p((x / scale) ** 2)


def studentt_lp(x, df, loc, scale):
    t = (x - loc) / scale
    return (gammaln((df + 1) / 2) - gammaln(df / 2) - 0.5 * np.log(df * np.pi) - np.log(scale)
            - (df + 1) / 2 * np.log1p(t * t / df))


def eight_schools_potential(z, y, sigma):
    """Non-centred eight schools, z = [mu, log tau, theta_base (J)] (sorted sites)."""
    mu, lt, tb = z[0], z[1], np.asarray(z[2:])
    tau = np.exp(lt)
    lp = normal_lp(mu, 0.0, 5.0) + halfcauchy_lp(tau, 5.0) + lt
    lp = lp + np.sum(normal_lp(tb, 0.0, 1.0)) + np.sum(normal_lp(np.asarray(y), mu + tau * tb, np.asarray(sigma)))
    return -lp


def kidiq_potential(z, kid_score, mom_hs, mom_iq):
    """z = [beta (3), log sigma]; beta ImproperUniform, sigma HalfCauchy(2.5)."""
    beta, ls = np.asarray(z[:3]), z[3]
    sigma = np.exp(ls)
    X = np.stack([np.ones_like(mom_hs), mom_hs, mom_iq], axis=1)
    mu = X @ beta
    lp = halfcauchy_lp(sigma, 2.5) + ls + np.sum(normal_lp(np.asarray(kid_score), mu, sigma))
    return -lp


def diamonds_potential(z, Xc, Y):
    """z = [Intercept, b (Kc), log sigma]; Xc = centred X[:, 1:] (N, Kc)."""
    Kc = Xc.shape[1]
    icpt, b, ls = z[0], np.asarray(z[1:1 + Kc]), z[1 + Kc]
    sigma = np.exp(ls)
    mu = icpt + Xc @ b
    lp = (np.sum(normal_lp(b, 0.0, 1.0)) + studentt_lp(icpt, 3.0, 8.0, 10.0)
          + math.log(2.0) + studentt_lp(sigma, 3.0, 0.0, 10.0) + ls
          + np.sum(normal_lp(np.asarray(Y), mu, sigma)))
    return -lp


def mixture_potential(z, weights, locs, scales):
    """asumptions_check.ipynb cells 61-62: -MixtureSameFamily(Categorical(w),
    Normal(m, s)).log_prob(x), summed over the coordinates of z (a scalar at
    d = 1, the notebook's case)."""
    x = np.atleast_1d(np.asarray(z, np.float64))[:, None]
    lp = np.log(np.asarray(weights, np.float64)) + normal_lp(x, np.asarray(locs, np.float64),
                                                            np.asarray(scales, np.float64))
    mx = lp.max(axis=1, keepdims=True)
    return -float(np.sum(np.log(np.exp(lp - mx).sum(axis=1)) + mx[:, 0]))


def gaussian_potential(z, m, P, c0):
    diff = np.asarray(z) - m
    return 0.5 * diff @ (P @ diff) + c0


# ---------------------------------------------------------------- driver --
def ns_logscale(n_pow=6):
    """kernel_utils.py:8-12: the 1-based step indices collect_states_logscale keeps."""
    return np.concatenate([
        np.arange(0 if p < 1 else 10 ** (p - 1), 10 ** p, 10 ** max(0, p - 2)) + 10 ** max(0, p - 2)
        for p in range(n_pow + 1)
    ])
