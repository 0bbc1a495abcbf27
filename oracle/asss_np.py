"""Literal numpy restatement of the reference ASSS kernel.

TEST INFRASTRUCTURE ONLY (never imported by the product package).

Follows python/kernels/asss.py statement by statement at float64 (or a
selected dtype), with the random draws injected so the bit-level C oracle
(oracle/amh_oracle.c, orc_asss_step) and the HIP kernel (amh_asss.hip) can
be fed the same noise:

  _stereographic_project   asss.py:33-45
  _stereographic_inverse   asss.py:48-56
  _shrinkage               asss.py:59-96
  ASSS.sample              asss.py:197-251  (one chain)
  cholesky_update          numpyro (asss.py:242; arwmh_np.cholesky_update)
"""
from __future__ import annotations

from collections import namedtuple

import numpy as np

from arwmh_np import TAG_STEP, cholesky_update, lr_gamma, normal_from_bits, philox4x32_10, unif01_from_bits

ASSSState = namedtuple("ASSSState", ["i", "z", "potential_energy", "adapt_state", "as_change", "rng_key"])
ASSSAdaptState = namedtuple("ASSSAdaptState", ["loc", "scale"])

TAG_ASSS = 0x53535341
MAX_ITERATIONS = 50


def stereographic_project(x, loc, scale):
    """asss.py:33-45 (scale lower triangular)."""
    from scipy.linalg import solve_triangular
    xr = solve_triangular(scale, x - loc, lower=True)
    ns = np.sum(xr ** 2)
    return np.concatenate([2 * xr / (ns + 1), [(ns - 1) / (ns + 1)]])


def stereographic_inverse(z, loc, scale):
    """asss.py:48-56."""
    x_base = z[:-1] / (1 - z[-1])
    return scale @ x_base + loc


def draws(key, it, d):
    """The build's noise for one step at stream position it (amh_asss.hip):
    v [d+1], u_t, theta_0 and the 50 shrink uniforms."""
    k0, k1 = np.uint32(key[0]), np.uint32(key[1])
    o = philox4x32_10(np.arange(d, dtype=np.uint32), np.uint32(it), 0, TAG_ASSS, k0, k1)
    v = np.concatenate([normal_from_bits(o[0]), normal_from_bits(o[1][:1])])
    u_t = float(unif01_from_bits(o[2][0]))
    th0 = float(np.float32(6.28318548) * unif01_from_bits(o[3][0]))
    s = philox4x32_10(np.arange(MAX_ITERATIONS, dtype=np.uint32), np.uint32(it), 1, TAG_ASSS, k0, k1)
    return v, u_t, th0, unif01_from_bits(s[0]).astype(np.float64)


def shrinkage(z, v, t_pe, transformed_pe_fn, th0, uks, eps=1e-6):
    """asss.py:59-96 with the initial angle th0 and the loop's uniforms uks."""
    theta = th0
    theta_min, theta_max = theta - 2 * np.pi, theta
    it = 0

    def cond(theta, it):
        zt = z * np.cos(theta) + v * np.sin(theta)
        pe = transformed_pe_fn(zt)
        pe = np.inf if np.isnan(pe) else pe
        return it < MAX_ITERATIONS and (pe > t_pe or (1.0 - zt[-1]) < eps)

    while cond(theta, it):
        theta_min = theta if theta < 0.0 else theta_min
        theta_max = theta if theta >= 0.0 else theta_max
        theta = theta_min + (theta_max - theta_min) * uks[it]
        it += 1
    theta = 0.0 if it >= MAX_ITERATIONS else theta
    return z * np.cos(theta) + v * np.sin(theta), it


def sample(state: ASSSState, potential_fn, v, u_t, th0, uks, num_warmup=0, lr_decay=2 / 3, eps=1e-6,
           dtype=np.float64):
    """ASSS.sample (asss.py:197-251) for ONE chain with injected draws."""
    i, x, _, adapt, _, key = state
    loc, scale = (np.asarray(a, dtype) for a in adapt)
    x = np.asarray(x, dtype)
    dim = loc.shape[-1]
    with np.errstate(all="ignore"):
        sigma_sqrt = (scale + eps * np.eye(dim)) * dim ** 0.5

        def transformed_pe(z):
            xf = stereographic_inverse(z, loc, sigma_sqrt)
            return potential_fn(xf) + dim * np.log(1.0 - z[-1])

        z = stereographic_project(x, loc, sigma_sqrt)
        pe_t = transformed_pe(z)
        v = np.asarray(v, dtype)
        v = v - np.dot(v, z) * z
        v = v / np.linalg.norm(v)
        t_pe = pe_t - np.log(u_t)
        z_new, n_iter = shrinkage(z, v, t_pe, transformed_pe, th0, uks, eps)
        x_new = stereographic_inverse(z_new, loc, sigma_sqrt)
        pe_new = potential_fn(x_new)
        pe_new = np.inf if np.isnan(pe_new) else pe_new
        itr = int(i) + 1
        n = itr if int(i) < num_warmup else itr - num_warmup
        gamma = lr_gamma(n, lr_decay, dtype)
        delta = x_new - loc
        loc_new = loc + gamma * delta
        chol = cholesky_update(np.sqrt(1 - gamma) * scale, delta, gamma, dtype)
        scale_new = scale if np.any(np.isnan(chol)) else chol
        asc = np.linalg.norm(loc_new - loc) + np.linalg.norm(scale_new - scale, "fro")
    return ASSSState(itr, x_new, pe_new, ASSSAdaptState(loc_new, scale_new), asc, key), n_iter
