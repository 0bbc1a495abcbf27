/*
 * amh_math.h -- the bit-level specification of the sampler's noise stream and
 * of every elementary function the ARWMH step evaluates.
 *
 * Shared by the HIP kernels (adaptive-mcmc_amd/csrc) and by the C oracle
 * (oracle/amh_oracle.c) so that a GPU step and a CPU step fed the same state
 * produce the same bits.  Everything here is built from IEEE-754 basic
 * operations (+ - * / sqrt, fmaf, rint) in a fixed order; no libm/ocml
 * transcendental is called, because those differ between host and device.
 * Both sides are compiled with -ffp-contract=off so nothing else fuses.
 *
 * The functions are pinned independently of this file by tests/test_math.py
 * (numpy/scipy float64 references) and tests/test_rng.py (Random123 KAT
 * vectors for Philox4x32-10).
 *
 * Reference anchors (what the noise stands in for):
 *   arwmh.py:162  rng_key, key_proposal, key_accept = random.split(rng_key, 3)
 *   arwmh.py:165  dist.Normal().sample(key_proposal, (dim,))   -> amh_normal_from_bits
 *   arwmh.py:174  dist.Uniform().sample(key_accept)            -> amh_unif01_from_bits
 *   jax.random.normal = sqrt(2) * erf_inv(uniform(nextafter(-1,0), 1)); XLA's
 *   f32 erf_inv uses Giles' single-precision polynomials, restated below.
 */
#ifndef AMH_MATH_H
#define AMH_MATH_H

#include <stdint.h>
#include <string.h>
#include <math.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define AMH_HD __host__ __device__ __forceinline__
#else
#define AMH_HD static inline
#endif

/* ---------------------------------------------------------------- bits ---- */
AMH_HD uint32_t amh_f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
AMH_HD float amh_u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
AMH_HD uint64_t amh_d2u(double f) { uint64_t u; memcpy(&u, &f, 8); return u; }
AMH_HD double amh_u2d(uint64_t u) { double f; memcpy(&f, &u, 8); return f; }

AMH_HD int amh_isnan(float x) { return x != x; }
AMH_HD int amh_isfinite(float x) { return (amh_f2u(x) & 0x7f800000u) != 0x7f800000u; }

/* ------------------------------------------------------- Philox4x32-10 ---- */
/* Salmon et al., "Parallel random numbers: as easy as 1, 2, 3" (SC'11);
 * constants and round function as in Random123 philox4x32. */
#define AMH_PHILOX_M0 0xD2511F53u
#define AMH_PHILOX_M1 0xCD9E8D57u
#define AMH_PHILOX_W0 0x9E3779B9u
#define AMH_PHILOX_W1 0xBB67AE85u

typedef struct { uint32_t v[4]; } amh_u32x4;

AMH_HD amh_u32x4 amh_philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                   uint32_t k0, uint32_t k1) {
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)AMH_PHILOX_M0 * (uint64_t)c0;
    const uint64_t p1 = (uint64_t)AMH_PHILOX_M1 * (uint64_t)c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += AMH_PHILOX_W0;
    k1 += AMH_PHILOX_W1;
  }
  amh_u32x4 o;
  o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}

/* The same function with the rounds unrolled (device code only): for
 * batched draws where several independent streams should interleave (the
 * pooled noise-ahead blocks).  Not used by default: unrolled rounds raise the
 * register count of the step kernels. */
#if defined(__HIPCC__)
__device__ __forceinline__ amh_u32x4 amh_philox4x32_10_unrolled(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                                uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)AMH_PHILOX_M0 * (uint64_t)c0;
    const uint64_t p1 = (uint64_t)AMH_PHILOX_M1 * (uint64_t)c2;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c0 = hi1 ^ c1 ^ k0;
    c1 = lo1;
    c2 = hi0 ^ c3 ^ k1;
    c3 = lo0;
    k0 += AMH_PHILOX_W0;
    k1 += AMH_PHILOX_W1;
  }
  amh_u32x4 o;
  o.v[0] = c0; o.v[1] = c1; o.v[2] = c2; o.v[3] = c3;
  return o;
}
#endif

/* Stream tags (counter word 3).  A chain key plus (tag, counter words) never
 * collides between uses. */
#define AMH_TAG_CHAINKEY 0x4B48434Du /* derive per-chain key from the run key */
#define AMH_TAG_INIT     0x54494E49u /* init_to_uniform draws                 */
#define AMH_TAG_STEP     0x50455453u /* per-step proposal / accept draws      */
#define AMH_TAG_SPLIT    0x54494C50u /* key splitting (sample_Pnx keys)       */
#define AMH_TAG_EVAL     0x4C415645u /* evaluation draws (sliced directions) */
#define AMH_TAG_ASSS     0x53535341u /* ASSS per-step draws (c2 = 0: v, u_t,
                                        theta_0; c2 = 1: shrink uniforms)   */

/* The step's noise stream (ARWMH.sample, arwmh.py:162-165, 174; round 5):
 * words W_j = Philox4x32-10(c0 = j >> 2, c1 = ctr, c2 = 0, c3 = TAG_STEP;
 * chain key).v[j & 3] for j = 0, 1, ..; the proposal noise is
 * xi_r = N(W_r) for r < d and the accept uniform u = U(W_d) -- four words
 * of every Philox call used, floor(d / 4) + 1 calls per chain-step (was one
 * call per coordinate, three words discarded).  ctr is the stream position
 * (state.i; the step index in sample_Pnx). */
AMH_HD uint32_t amh_step_word(uint32_t j, uint32_t ctr, uint32_t k0, uint32_t k1) {
  const amh_u32x4 o = amh_philox4x32_10(j >> 2, ctr, 0u, AMH_TAG_STEP, k0, k1);
  const uint32_t q = j & 3u; /* selects, not an indexed load: no stack array on the device */
  return (q == 0u) ? o.v[0] : ((q == 1u) ? o.v[1] : ((q == 2u) ? o.v[2] : o.v[3]));
}

/* 32 random bits -> float in [0,1): jax.random.uniform's construction
 * (mantissa fill of [1,2) then subtract 1). */
AMH_HD float amh_unif01_from_bits(uint32_t b) {
  return amh_u2f((b >> 9) | 0x3F800000u) - 1.0f;
}

/* ------------------------------------------------------------ logf/expf ---- */
/* Cephes-style single precision log: x = 2^e * m, m in [sqrt(.5), sqrt(2)).
 * Branch-free core (lanes of a wavefront never diverge on it); special
 * arguments are patched by selects at the end. */
AMH_HD float amh_logf(float x) {
  const int sub = x < 1.17549435e-38f;           /* subnormal (or <= 0) */
  const float xs = sub ? x * 33554432.0f : x;
  const uint32_t bits = amh_f2u(xs);
  int e = (int)((bits >> 23) & 0xFFu) - 126 - (sub ? 25 : 0);
  float m = amh_u2f((bits & 0x007FFFFFu) | 0x3F000000u); /* [0.5, 1) */
  const int lo = m < 0.707106781186547524f;
  e -= lo;
  m = lo ? ((m + m) - 1.0f) : (m - 1.0f);
  const float z = m * m;
  float y = 7.0376836292e-2f;
  y = fmaf(y, m, -1.1514610310e-1f);
  y = fmaf(y, m, 1.1676998740e-1f);
  y = fmaf(y, m, -1.2420140846e-1f);
  y = fmaf(y, m, 1.4249322787e-1f);
  y = fmaf(y, m, -1.6668057665e-1f);
  y = fmaf(y, m, 2.0000714765e-1f);
  y = fmaf(y, m, -2.4999993993e-1f);
  y = fmaf(y, m, 3.3333331174e-1f);
  y = (y * m) * z;
  const float fe = (float)e;
  y = fmaf(fe, -2.12194440e-4f, y);
  y = fmaf(-0.5f, z, y);
  float r = m + y;
  r = fmaf(fe, 0.693359375f, r);
  r = (x == INFINITY) ? x : r;
  r = (x == 0.0f) ? -INFINITY : r;
  r = ((x < 0.0f) | amh_isnan(x)) ? amh_u2f(0x7FC00000u) : r;
  return r;
}

/* 2^n for n in [-126, 127] as an exact float. */
AMH_HD float amh_exp2i(int n) { return amh_u2f((uint32_t)(n + 127) << 23); }

/* Cephes-style single precision exp with a two-step 2^n scaling so gradual
 * underflow is rounded once.  Branch-free; out-of-range arguments are
 * clamped before the reduction and patched after it. */
AMH_HD float amh_expf(float x) {
  const float xc = (x > 88.7228317f) ? 88.7228317f : ((x < -103.972084f) ? -103.972084f : x);
  const float xr = amh_isnan(x) ? 0.0f : xc;
  const float fn = rintf(xr * 1.44269504088896341f);
  const int n = (int)fn;
  float r = fmaf(fn, -0.693359375f, xr);
  r = fmaf(fn, 2.12194440e-4f, r);
  const float z = r * r;
  float y = 1.9875691500e-4f;
  y = fmaf(y, r, 1.3981999507e-3f);
  y = fmaf(y, r, 8.3334519073e-3f);
  y = fmaf(y, r, 4.1665795894e-2f);
  y = fmaf(y, r, 1.6666665459e-1f);
  y = fmaf(y, r, 5.0000001201e-1f);
  y = fmaf(y, z, r);
  y = y + 1.0f;
  const int n1 = n >> 1;           /* floor(n/2) */
  const int n2 = n - n1;
  float res = (y * amh_exp2i(n1)) * amh_exp2i(n2);
  res = (x > 88.7228317f) ? INFINITY : res;
  res = (x < -103.972084f) ? 0.0f : res;
  res = amh_isnan(x) ? x : res;
  return res;
}

/* log1p(x) = log(u) * x / (u - 1) with u = 1 + x (Goldberg's trick). */
AMH_HD float amh_log1pf(float x) {
  const float u = 1.0f + x;
  if (u == 1.0f) return x;
  if (u == INFINITY) return u;
  return amh_logf(u) * (x / (u - 1.0f));
}

/* ------------------------------------------------------------- erfinv ---- */
/* Giles (2010) single precision erfinv, as XLA's ErfInv32 evaluates it. */
AMH_HD float amh_erfinvf(float x) {
  const float w0 = -amh_logf((1.0f - x) * (1.0f + x));
  const float ws = w0 - 2.5f;
  float ps = 2.81022636e-08f;
  ps = fmaf(ps, ws, 3.43273939e-07f);
  ps = fmaf(ps, ws, -3.5233877e-06f);
  ps = fmaf(ps, ws, -4.39150654e-06f);
  ps = fmaf(ps, ws, 0.00021858087f);
  ps = fmaf(ps, ws, -0.00125372503f);
  ps = fmaf(ps, ws, -0.00417768164f);
  ps = fmaf(ps, ws, 0.246640727f);
  ps = fmaf(ps, ws, 1.50140941f);
  const float wl = sqrtf(w0) - 3.0f;
  float pl = -0.000200214257f;
  pl = fmaf(pl, wl, 0.000100950558f);
  pl = fmaf(pl, wl, 0.00134934322f);
  pl = fmaf(pl, wl, -0.00367342844f);
  pl = fmaf(pl, wl, 0.00573950773f);
  pl = fmaf(pl, wl, -0.0076224613f);
  pl = fmaf(pl, wl, 0.00943887047f);
  pl = fmaf(pl, wl, 1.00167406f);
  pl = fmaf(pl, wl, 2.83297682f);
  const float p = (w0 < 5.0f) ? ps : pl;
  return p * x;
}

/* 32 random bits -> standard normal, jax.random.normal's construction:
 * u in [nextafter(-1,0), 1), xi = sqrt(2) * erfinv(u). */
AMH_HD float amh_normal_from_bits(uint32_t b) {
  const float lo = -0.99999994f; /* nextafter(-1, 0) */
  const float f = amh_unif01_from_bits(b);
  float u = (f * 2.0f) + lo;     /* (hi - lo) rounds to 2 in fp32 */
  u = (u < lo) ? lo : u;
  return 1.41421356f * amh_erfinvf(u);
}

/* The whole step stream of one chain-step on the host (oracle): xi[0..d)
 * and u, one Philox call per four words. */
AMH_HD void amh_step_noise(int d, uint32_t ctr, uint32_t k0, uint32_t k1, float* xi, float* u) {
  amh_u32x4 o = amh_philox4x32_10(0u, ctr, 0u, AMH_TAG_STEP, k0, k1);
  for (int j = 0; j <= d; ++j) {
    if (j > 0 && (j & 3) == 0) o = amh_philox4x32_10((uint32_t)(j >> 2), ctr, 0u, AMH_TAG_STEP, k0, k1);
    if (j < d) xi[j] = amh_normal_from_bits(o.v[j & 3]);
    else *u = amh_unif01_from_bits(o.v[j & 3]);
  }
}

#if defined(__HIPCC__)
/* amh_normal_from_bits split for batched draws on the device (the same
 * value): the head gives u, w and the central polynomial; the tail
 * polynomial of erfinv (w >= 5, |u| > 0.9966: ~0.3% of draws, so about one
 * wave in five has a lane there) and its sqrtf are needed only when some
 * lane of the wave has w >= 5, which the caller tests wave-uniformly; the
 * normal is then 1.41421356 * ((w < 5 ? ps : pl) * u). */
__device__ __forceinline__ float amh_normal_head(uint32_t b, float* u_out, float* w_out) {
  const float lo = -0.99999994f;
  const float f = amh_unif01_from_bits(b);
  float u = (f * 2.0f) + lo;
  u = (u < lo) ? lo : u;
  const float w0 = -amh_logf((1.0f - u) * (1.0f + u));
  const float ws = w0 - 2.5f;
  float ps = 2.81022636e-08f;
  ps = fmaf(ps, ws, 3.43273939e-07f);
  ps = fmaf(ps, ws, -3.5233877e-06f);
  ps = fmaf(ps, ws, -4.39150654e-06f);
  ps = fmaf(ps, ws, 0.00021858087f);
  ps = fmaf(ps, ws, -0.00125372503f);
  ps = fmaf(ps, ws, -0.00417768164f);
  ps = fmaf(ps, ws, 0.246640727f);
  ps = fmaf(ps, ws, 1.50140941f);
  *u_out = u;
  *w_out = w0;
  return ps;
}
__device__ __forceinline__ float amh_erfinv_tail(float w0) {
  const float wl = sqrtf(w0) - 3.0f;
  float pl = -0.000200214257f;
  pl = fmaf(pl, wl, 0.000100950558f);
  pl = fmaf(pl, wl, 0.00134934322f);
  pl = fmaf(pl, wl, -0.00367342844f);
  pl = fmaf(pl, wl, 0.00573950773f);
  pl = fmaf(pl, wl, -0.0076224613f);
  pl = fmaf(pl, wl, 0.00943887047f);
  pl = fmaf(pl, wl, 1.00167406f);
  pl = fmaf(pl, wl, 2.83297682f);
  return pl;
}
#endif

/* ----------------------------------------------------------- sin/cos ---- */
/* Cephes-style single precision sin and cos of one argument (the slice
 * angle of ASSS, asss.py:69, :95: |theta| < 2 pi).  theta = k pi/2 + r with
 * k = rint(theta 2/pi) and a three-part Cody-Waite reduction (fmaf), then the
 * sinf / cosf minimax polynomials on |r| <= pi/4 and the quadrant swap. */
AMH_HD void amh_sincosf(float x, float* s_out, float* c_out) {
  const float kf = rintf(x * 0.636619772367581343f);
  const int k = (int)kf;
  float r = fmaf(kf, -1.57079637050628662109375f, x);
  r = fmaf(kf, 4.37113882867379e-08f, r);
  r = fmaf(kf, 1.7151245100059596e-15f, r);
  const float z = r * r;
  float ps = -1.9515295891e-4f;
  ps = fmaf(ps, z, 8.3321608736e-3f);
  ps = fmaf(ps, z, -1.6666654611e-1f);
  const float sr = fmaf(ps * z, r, r);
  float pc = 2.443315711809948e-5f;
  pc = fmaf(pc, z, -1.388731625493765e-3f);
  pc = fmaf(pc, z, 4.166664568298827e-2f);
  const float cr = fmaf(pc * z, z, fmaf(-0.5f, z, 1.0f));
  const int q = k & 3;
  const float s = (q == 0) ? sr : ((q == 1) ? cr : ((q == 2) ? -sr : -cr));
  const float c = (q == 0) ? cr : ((q == 1) ? -sr : ((q == 2) ? -cr : sr));
  *s_out = s;
  *c_out = c;
}

/* ------------------------------------------------- double log/exp/pow ---- */
/* Used only for the learning-rate schedule gamma = 1 / n^a (arwmh.py:183);
 * computed in double and rounded once to float. */
AMH_HD double amh_log_d(double x) { /* x > 0, finite, normal */
  const uint64_t bits = amh_d2u(x);
  int e = (int)((bits >> 52) & 0x7FFu) - 1022;
  double m = amh_u2d((bits & 0x000FFFFFFFFFFFFFull) | 0x3FE0000000000000ull); /* [0.5,1) */
  if (m < 0.70710678118654752440) { e -= 1; m = m + m; }
  const double f = m - 1.0;
  const double s = f / (2.0 + f);
  const double s2 = s * s;
  double t = 1.0 / 23.0;
  t = fma(t, s2, 1.0 / 21.0);
  t = fma(t, s2, 1.0 / 19.0);
  t = fma(t, s2, 1.0 / 17.0);
  t = fma(t, s2, 1.0 / 15.0);
  t = fma(t, s2, 1.0 / 13.0);
  t = fma(t, s2, 1.0 / 11.0);
  t = fma(t, s2, 1.0 / 9.0);
  t = fma(t, s2, 1.0 / 7.0);
  t = fma(t, s2, 1.0 / 5.0);
  t = fma(t, s2, 1.0 / 3.0);
  t = t * s2;
  const double lm = fma(2.0 * s, t, 2.0 * s);
  const double fe = (double)e;
  return fma(fe, 6.93147180369123816490e-01, fma(fe, 1.90821492927058770002e-10, lm));
}

AMH_HD double amh_exp_d(double x) { /* |x| < 700 */
  const double kf = rint(x * 1.44269504088896338700e+00);
  const int k = (int)kf;
  double r = fma(kf, -6.93147180369123816490e-01, x);
  r = fma(kf, -1.90821492927058770002e-10, r);
  double p = 1.0 / 6227020800.0; /* 1/13! */
  p = fma(p, r, 1.0 / 479001600.0);
  p = fma(p, r, 1.0 / 39916800.0);
  p = fma(p, r, 1.0 / 3628800.0);
  p = fma(p, r, 1.0 / 362880.0);
  p = fma(p, r, 1.0 / 40320.0);
  p = fma(p, r, 1.0 / 5040.0);
  p = fma(p, r, 1.0 / 720.0);
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return p * amh_u2d((uint64_t)(k + 1023) << 52);
}

/* gamma_n = 1 / n^a  (arwmh.py:183: `1 / n ** self._lr_decay`): n^a is
 * evaluated in double, rounded to float, then the float reciprocal is taken
 * as the reference does in fp32. */
AMH_HD float amh_lr_gamma(int32_t n, float a) {
  const double na = amh_exp_d((double)a * amh_log_d((double)n));
  return 1.0f / (float)na;
}

/* ---------------------------------------------- shared-factor pivot ---- */
/* The pooled (shared) factorisation's column scaling (regime B, d >= 64):
 * 1/sqrt(x) by three Newton steps from the bit-pattern seed (3.4 % ->
 * 1.7e-3 -> 4.6e-6 -> rounding), in fmaf / mul only, so the device and the
 * host give the same bits; L_kk = x * y and the column below is multiplied
 * by y.  Eleven dependent operations in place of IEEE sqrtf followed by an
 * IEEE division (about 30): the pivot chain is the factorisation's critical
 * path.
 * Callers accept only normal, finite pivots (amh_pivot_ok). */
AMH_HD int amh_pivot_ok(float x) { return x >= 1.17549435e-38f && amh_isfinite(x); }
AMH_HD float amh_rsqrt_nr(float x) {
  const float h = 0.5f * x;
  float y = amh_u2f(0x5F375A86u - (amh_f2u(x) >> 1));
  float t = y * y;
  t = fmaf(-h, t, 1.5f);
  y = y * t;
  t = y * y;
  t = fmaf(-h, t, 1.5f);
  y = y * t;
  t = y * y;
  t = fmaf(-h, t, 1.5f);
  return y * t;
}

#endif /* AMH_MATH_H */
