/*
 * amh_oracle.c -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
 * ARWMH hot path, used as the parity checker for the HIP kernels and as the
 * `cpu_baseline` leg of bench.py.  Nothing in the product (the package under
 * adaptive-mcmc_amd/) links, imports or calls this file.
 *
 * What it restates (reference = /root/reference, savelovme/adaptive-mcmc):
 *   orc_init        arwmh.py:84-138   ARWMH.init (mu = z0, L = I, lambda = 0)
 *                   + numpyro init_to_uniform: U(-2, 2) per unconstrained site
 *   orc_step        arwmh.py:140-207  ARWMH.sample, one or more steps
 *     cholupdate    numpyro.distributions.util.cholesky_update (called at
 *                   arwmh.py:190; Krause & Igel 2015 rank-one update)
 *   orc_sample_pnx  arwmh.py:230-270  ARWMH.sample_Pnx (frozen shared theta)
 *   potentials      run_eight_schools_lr_decay.py:26-35,
 *                   run_kidiq_kidscore_lr_decay.py:29-41,
 *                   run_diamonds_lr_decay.py:24-40, and the build-defined
 *                   dense Gaussian
 *
 * Arithmetic order follows the HIP kernel's (documented in DESIGN.md, "bit
 * spec"), so GPU and oracle agree bit for bit; the order's faithfulness to
 * the reference is pinned separately by tests/test_oracle.py against the
 * literal numpy restatement oracle/arwmh_np.py (float64) within tolerance.
 *
 * Build: make -C oracle   (gcc -O2 -ffp-contract=off -fopenmp)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <math.h>
#include "../include/amh_math.h"

#define ORC_DMAX 64

enum { ORC_GAUSSIAN = 1, ORC_EIGHT_SCHOOLS = 2, ORC_KIDIQ = 3, ORC_DIAMONDS = 4, ORC_DIAMONDS_SS = 5, ORC_MIXTURE = 6 };

typedef struct {
  int32_t model_id;
  int32_t d;
  int32_t num_warmup;
  float lr_decay;
  float target_accept_prob;
  float eps;
  const float* data;   /* model data, layout per model (see potential) */
  int64_t n_data;      /* N rows for regression models                 */
  int64_t k_data;      /* K columns for diamonds                       */
} orc_cfg;

/* Group (lane) width the GPU uses for dimension d: next power of two. */
int orc_group_width(int d) {
  int g = 1;
  while (g < d) g <<= 1;
  return g;
}

/* Group width of the per-chain kernels for a model (amh_device.h dispatch):
 * eight schools runs at G = 16 and diamonds at G = 32 for every d they take. */
static int orc_gw(const orc_cfg* cfg) {
  if (cfg->model_id == ORC_DIAMONDS || cfg->model_id == ORC_DIAMONDS_SS) return 32;
  if (cfg->model_id == ORC_EIGHT_SCHOOLS) return 16;
  return orc_group_width(cfg->d);
}

/* ----------------------------------------------------- lane-group ops ---- */
/* butterfly sum: for off = 1,2,4,..: x[r] = x[r] + x[r ^ off] */
static float group_sum(const float* in, int G) {
  float x[ORC_DMAX], y[ORC_DMAX];
  memcpy(x, in, sizeof(float) * G);
  for (int off = 1; off < G; off <<= 1) {
    for (int r = 0; r < G; ++r) y[r] = x[r] + x[r ^ off];
    memcpy(x, y, sizeof(float) * G);
  }
  return x[0];
}

/* exclusive scan with the kernel's association (Grp::excl_scan): shift by one
 * lane; inclusive Hillis-Steele inside 16-lane rows (DPP row_shr 1,2,4,8);
 * then odd rows add lane 15 of the row before (row_bcast15) and, for G = 64,
 * rows 2-3 add lane 31 (row_bcast31).  Each round reads the previous round's
 * values (simultaneous update). */
static void group_excl_scan(const float* t, float* out, int G) {
  float x[ORC_DMAX], y[ORC_DMAX];
  for (int r = 0; r < G; ++r) x[r] = (r >= 1) ? t[r - 1] : 0.0f;
  for (int off = 1; off < 16 && off < G; off <<= 1) {
    for (int r = 0; r < G; ++r) {
      const int ok = (G >= 16) ? ((r % 16) >= off) : (r >= off);
      y[r] = ok ? x[r] + x[r - off] : x[r];
    }
    memcpy(x, y, sizeof(float) * G);
  }
  if (G >= 32) {
    for (int r = 0; r < G; ++r) y[r] = ((r / 16) % 2 == 1) ? x[r] + x[(r / 16) * 16 - 1] : x[r];
    memcpy(x, y, sizeof(float) * G);
  }
  if (G == 64) {
    for (int r = 0; r < G; ++r) y[r] = (r >= 32) ? x[r] + x[31] : x[r];
    memcpy(x, y, sizeof(float) * G);
  }
  memcpy(out, x, sizeof(float) * G);
}

/* ------------------------------------------------------------- models ---- */
#define HALF_LOG_2PI 0.918938533204672742f

/* Dense Gaussian: data = [m (d) | P (d*d, symmetric precision) | c0].
 * U(x) = 0.5 (x-m)' P (x-m) + c0. */
static float pot_gaussian(const orc_cfg* cfg, const float* x, int G) {
  const int d = cfg->d;
  const float* m = cfg->data;
  const float* P = cfg->data + d;
  const float c0 = cfg->data[d + d * d];
  float diff[ORC_DMAX], q[ORC_DMAX];
  for (int r = 0; r < G; ++r) diff[r] = (r < d) ? x[r] - m[r] : 0.0f;
  for (int r = 0; r < G; ++r) {
    if (r >= d) { q[r] = 0.0f; continue; }
    float y4[4] = {0.0f, 0.0f, 0.0f, 0.0f}; /* partial sums over j mod 4 (kernel order) */
    for (int j = 0; j < d; ++j) y4[j & 3] = fmaf(P[r * d + j], diff[j], y4[j & 3]); /* row r */
    const float y = (y4[0] + y4[1]) + (y4[2] + y4[3]);
    q[r] = diff[r] * y;
  }
  const float S = group_sum(q, G);
  return (0.5f * S) + c0;
}

/* Eight schools, non-centred (run_eight_schools_lr_decay.py:26-35).
 * z = [mu, log tau, theta_base_0..J-1] (ravel_pytree sorted-key order).
 * data = [y (J) | sigma (J) | log sigma (J)]. */
static float pot_eight_schools(const orc_cfg* cfg, const float* x, int G) {
  const int d = cfg->d, J = d - 2;
  const float* y = cfg->data;
  const float* sg = cfg->data + J;
  const float* lsg = cfg->data + 2 * J;
  const float mu = x[0], lt = x[1];
  const float tau = amh_expf(lt);
  float lp[ORC_DMAX];
  for (int r = 0; r < G; ++r) {
    float v = 0.0f;
    if (r == 0) {
      const float t = mu / 5.0f;
      v = ((-0.5f * (t * t)) - 1.60943791243410037f) - HALF_LOG_2PI;
    } else if (r == 1) {
      const float t = tau / 5.0f;
      /* log HalfCauchy(tau; 5) + log|d tau / d lt| */
      v = ((-0.451582705289454865f - 1.60943791243410037f) - amh_log1pf(t * t)) + lt;
    } else if (r < d) {
      const int j = r - 2;
      const float th = x[r];
      const float lpt = (-0.5f * (th * th)) - HALF_LOG_2PI;
      const float e = (y[j] - (mu + tau * th)) / sg[j];
      const float lpy = ((-0.5f * (e * e)) - lsg[j]) - HALF_LOG_2PI;
      v = lpt + lpy;
    }
    lp[r] = v;
  }
  return -group_sum(lp, G);
}

/* kidiq-kidscore_momhsiq (run_kidiq_kidscore_lr_decay.py:29-41).
 * z = [beta0, beta1, beta2, log sigma]; data = [kid (N) | hs (N) | iq (N)].
 * Lane r sums rows n = r, r+G, r+2G, ... */
static float pot_kidiq(const orc_cfg* cfg, const float* x, int G) {
  const int64_t N = cfg->n_data;
  const float* kid = cfg->data;
  const float* hs = cfg->data + N;
  const float* iq = cfg->data + 2 * N;
  const float b0 = x[0], b1 = x[1], b2 = x[2], ls = x[3];
  const float sg = amh_expf(ls);
  const float isg = 1.0f / sg;
  float part[ORC_DMAX];
  for (int r = 0; r < G; ++r) {
    float acc = 0.0f;
    for (int64_t n = r; n < N; n += G) {
      const float mu = fmaf(b2, iq[n], fmaf(b1, hs[n], b0));
      const float e = (kid[n] - mu) * isg;
      acc = fmaf(e, e, acc);
    }
    part[r] = acc;
  }
  const float S = group_sum(part, G);
  const float t = sg / 2.5f;
  /* -[ N*(-log sigma - HALF_LOG_2PI) - S/2 + logHalfCauchy(sigma;2.5) + ls ] */
  const float ll = fmaf(-0.5f, S, (float)N * ((-ls) - HALF_LOG_2PI));
  const float lpr = ((-0.451582705289454865f - 0.916290731874155065f) - amh_log1pf(t * t)) + ls;
  return -(ll + lpr);
}

/* log StudentT(x; nu=3, loc, scale) up to the data-independent constant
 * folded into c (= lgamma(2) - lgamma(1.5) - 0.5 log(3 pi) - log scale). */
static float lp_student3(float x, float loc, float scale, float c) {
  const float t = (x - loc) / scale;
  return c - 2.0f * amh_log1pf((t * t) / 3.0f);
}

/* diamonds (run_diamonds_lr_decay.py:24-40).
 * z = [Intercept, b_0..b_{K-2}, log sigma]; data = [Xc (N x Kc, row-major,
 * centred) | Y (N)].  Lane r sums rows n = r, r+G, ... */
static float pot_diamonds(const orc_cfg* cfg, const float* x, int G) {
  const int64_t N = cfg->n_data;
  const int Kc = (int)cfg->k_data - 1;
  const float* X = cfg->data;
  const float* Y = cfg->data + N * Kc;
  const float icpt = x[0], ls = x[Kc + 1];
  const float sg = amh_expf(ls);
  const float isg = 1.0f / sg;
  float part[ORC_DMAX];
  for (int r = 0; r < G; ++r) {
    float acc = 0.0f;
    for (int64_t n = r; n < N; n += G) {
      float mu = 0.0f;
      for (int k = 0; k < Kc; ++k) mu = fmaf(X[n * Kc + k], x[1 + k], mu);
      const float e = (Y[n] - (icpt + mu)) * isg;
      acc = fmaf(e, e, acc);
    }
    part[r] = acc;
  }
  const float S = group_sum(part, G);
  float bb[ORC_DMAX];
  for (int r = 0; r < G; ++r) bb[r] = (r >= 1 && r <= Kc) ? x[r] * x[r] : 0.0f;
  const float B = group_sum(bb, G);
  const float cst = -3.30347394261755545f; /* lgamma(2)-lgamma(1.5)-.5log(3pi) - log 10 */
  const float ll = fmaf(-0.5f, S, (float)N * ((-ls) - HALF_LOG_2PI));
  const float lpb = fmaf(-0.5f, B, -(float)Kc * HALF_LOG_2PI);
  const float lpi = lp_student3(icpt, 8.0f, 10.0f, cst);
  const float lps = (0.693147181f + lp_student3(sg, 0.0f, 10.0f, cst)) + ls;
  return -(((ll + lpb) + lpi) + lps);
}

/* diamonds through float64 sufficient statistics (amh_device.h DiamondsSSM;
 * model run_diamonds_lr_decay.py:24-40 as pot_diamonds).  data = float64
 * [N, ybar, A, sT, t (Kc), sx (Kc), Gm (Kc x Kc)]; the residual sum is
 * A + a (N a - 2 sT) + sum_i [b_i (2 rr_i + Gm_ii b_i) - 2 b_i (t_i - a sx_i)]
 * with rr_i = sum_{j<i} Gm_ij b_j, the per-coordinate terms summed by the
 * group butterfly in float64. */
static double dgroup_sum(const double* in, int G) {
  double x[ORC_DMAX], y[ORC_DMAX];
  memcpy(x, in, sizeof(double) * G);
  for (int off = 1; off < G; off <<= 1) {
    for (int r = 0; r < G; ++r) y[r] = x[r] + x[r ^ off];
    memcpy(x, y, sizeof(double) * G);
  }
  return x[0];
}

static float pot_diamonds_ss(const orc_cfg* cfg, const float* x, int G) {
  const int Kc = cfg->d - 2;
  const double* D = (const double*)cfg->data;
  const double N = D[0], ybar = D[1], A = D[2], sT = D[3];
  const double* t = D + 4;
  const double* sx = D + 4 + Kc;
  const double* Gm = D + 4 + 2 * Kc;
  const float icpt = x[0], ls = x[Kc + 1];
  const float sg = amh_expf(ls);
  const float isg = 1.0f / sg;
  const double a = (double)icpt - ybar;
  double v[ORC_DMAX];
  float bb[ORC_DMAX];
  for (int r = 0; r < G; ++r) {
    v[r] = 0.0;
    bb[r] = 0.0f;
    if (r < 1 || r > Kc) continue;
    const int i = r - 1;
    const double bi = (double)x[r];
    double rr = 0.0;
    for (int j = 0; j < Kc; ++j) rr = fma(j < i ? Gm[i * Kc + j] : 0.0, (double)x[1 + j], rr);
    const double quad = bi * fma(2.0, rr, Gm[i * Kc + i] * bi);
    const double lin = bi * fma(-a, sx[i], t[i]);
    v[r] = fma(-2.0, lin, quad);
    bb[r] = x[r] * x[r];
  }
  const double Q = dgroup_sum(v, G);
  const double qa = fma(a, fma(N, a, -2.0 * sT), A);
  const double q = qa + Q;
  const double isgd = (double)isg;
  const float S = (float)(q * (isgd * isgd));
  const float B = group_sum(bb, G);
  const float cst = -3.30347394261755545f;
  const float ll = fmaf(-0.5f, S, (float)N * ((-ls) - HALF_LOG_2PI));
  const float lpb = fmaf(-0.5f, B, -(float)Kc * HALF_LOG_2PI);
  const float lpi = lp_student3(icpt, 8.0f, 10.0f, cst);
  const float lps = (0.693147181f + lp_student3(sg, 0.0f, 10.0f, cst)) + ls;
  return -(((ll + lpb) + lpi) + lps);
}

/* K-component univariate normal mixture on every coordinate
 * (asumptions_check.ipynb cells 61-62; amh_device.h MixtureM).  data =
 * [c (K) | m (K) | s (K)], c_k = log w_k - log(sqrt(2 pi) s_k); n_data = K.
 * Per coordinate: lp_k = c_k - 0.5 t^2, t = (x - m_k) / s_k; the
 * jax.nn.logsumexp over k (max, non-finite max -> 0, sum in k order). */
static float pot_mixture(const orc_cfg* cfg, const float* x, int G) {
  const int K = (int)cfg->n_data;
  const float* c = cfg->data;
  const float* m = cfg->data + K;
  const float* s = cfg->data + 2 * K;
  float v[ORC_DMAX];
  for (int r = 0; r < G; ++r) {
    if (r >= cfg->d) { v[r] = 0.0f; continue; }
    float lp[8];
    float mx = -INFINITY;
    for (int k = 0; k < K; ++k) {
      const float t = (x[r] - m[k]) / s[k];
      lp[k] = c[k] - 0.5f * (t * t);
      mx = (lp[k] > mx) ? lp[k] : mx;
    }
    mx = (mx == INFINITY || mx == -INFINITY || mx != mx) ? 0.0f : mx;
    float S = 0.0f;
    for (int k = 0; k < K; ++k) S = S + amh_expf(lp[k] - mx);
    v[r] = amh_logf(S) + mx;
  }
  return -group_sum(v, G);
}

static float pot_gaussian_big(const orc_cfg* cfg, const float* x);

float orc_potential1(const orc_cfg* cfg, const float* x) {
  const int G = orc_gw(cfg);
  if (cfg->d > ORC_DMAX) return (cfg->model_id == ORC_GAUSSIAN) ? pot_gaussian_big(cfg, x) : NAN;
  switch (cfg->model_id) {
    case ORC_GAUSSIAN: return pot_gaussian(cfg, x, G);
    case ORC_EIGHT_SCHOOLS: return pot_eight_schools(cfg, x, G);
    case ORC_KIDIQ: return pot_kidiq(cfg, x, G);
    case ORC_DIAMONDS: return pot_diamonds(cfg, x, G);
    case ORC_DIAMONDS_SS: return pot_diamonds_ss(cfg, x, G);
    case ORC_MIXTURE: return pot_mixture(cfg, x, G);
    default: return NAN;
  }
}

void orc_potential(const orc_cfg* cfg, const float* z, float* pe, int64_t n) {
#pragma omp parallel for schedule(static)
  for (int64_t c = 0; c < n; ++c) pe[c] = orc_potential1(cfg, z + c * cfg->d);
}

/* ---------------------------------------------------------------- keys ---- */
void orc_chain_keys(const uint32_t* key, int64_t chain_offset, int64_t n, uint32_t* out) {
  for (int64_t c = 0; c < n; ++c) {
    const uint64_t g = (uint64_t)(chain_offset + c);
    const amh_u32x4 o = amh_philox4x32_10((uint32_t)g, (uint32_t)(g >> 32), 0u, AMH_TAG_CHAINKEY,
                                          key[0], key[1]);
    out[2 * c] = o.v[0];
    out[2 * c + 1] = o.v[1];
  }
}

/* ----------------------------------------------------------------- init ---- */
static inline int64_t packed_size(int d) { return (int64_t)d * (d + 1) / 2; }
static inline int64_t col_off(int d, int j) { return (int64_t)j * d - (int64_t)j * (j - 1) / 2; }

void orc_init(const orc_cfg* cfg, const uint32_t* key, int64_t chain_offset, int64_t C,
              const float* init_z, int32_t* i_, float* z, float* pe, float* macc, float* mu,
              float* L, float* lam, float* asc, uint32_t* keys) {
  const int d = cfg->d;
  orc_chain_keys(key, chain_offset, C, keys);
#pragma omp parallel for schedule(static)
  for (int64_t c = 0; c < C; ++c) {
    float* zc = z + c * d;
    for (int r = 0; r < d; ++r) {
      if (init_z) {
        zc[r] = init_z[c * d + r];
      } else {
        const amh_u32x4 o = amh_philox4x32_10((uint32_t)r, 0u, 0u, AMH_TAG_INIT, keys[2 * c], keys[2 * c + 1]);
        float v = (amh_unif01_from_bits(o.v[0]) * 4.0f) + (-2.0f);
        zc[r] = (v < -2.0f) ? -2.0f : v;
      }
      mu[c * d + r] = zc[r];
    }
    pe[c] = orc_potential1(cfg, zc);
    float* Lc = L + c * packed_size(d);
    for (int64_t k = 0; k < packed_size(d); ++k) Lc[k] = 0.0f;
    for (int j = 0; j < d; ++j) Lc[col_off(d, j)] = 1.0f;
    i_[c] = 0;
    macc[c] = 0.0f;
    lam[c] = 0.0f;
    asc[c] = 0.0f;
  }
}

/* ----------------------------------------------------------------- step ---- */
/* A chain between steps, as the kernel keeps it in registers: the factor in
 * unit-lower form U (U_rr = 1, U_rj = L_rj / L_jj) plus its diagonal dl. */
typedef struct {
  int32_t i;
  float pe, macc, lam, asc;
  float z[ORC_DMAX], mu[ORC_DMAX], dl[ORC_DMAX];
  float U[ORC_DMAX][ORC_DMAX];
  int updated;
} chain_t;

/* One ARWMH transition of one chain (arwmh.py:140-207). Returns accept. */
static int chain_step(const orc_cfg* cfg, chain_t* s, uint32_t k0, uint32_t k1, uint32_t ctr) {
  const int d = cfg->d;
  const int G = orc_gw(cfg);
  /* arwmh.py:162-165: proposal noise and accept uniform */
  float xi[ORC_DMAX], u;
  amh_step_noise(d, ctr, k0, k1, xi, &u); /* W_j = Philox(j >> 2, ctr)[j & 3]: xi_r = N(W_r), u = U(W_d) */
  /* arwmh.py:166-167: z' = z + (L e^lam + eps I) xi,  L xi = U (dl * xi) */
  const float el = amh_expf(s->lam);
  float eta[ORC_DMAX], zp[ORC_DMAX];
  for (int r = 0; r < d; ++r) eta[r] = s->dl[r] * xi[r];
  for (int r = 0; r < d; ++r) {
    float a4[4] = {0.0f, 0.0f, 0.0f, 0.0f}; /* partial sums over j mod 4 (kernel order) */
    for (int j = 0; j < d; ++j) a4[j & 3] = fmaf(s->U[r][j], eta[j], a4[j & 3]);
    const float acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    zp[r] = s->z[r] + fmaf(el, acc, cfg->eps * xi[r]);
  }
  /* arwmh.py:169-171 */
  float pep = orc_potential1(cfg, zp);
  if (amh_isnan(pep)) pep = INFINITY;
  /* arwmh.py:173-178 */
  const float ex = amh_expf(s->pe - pep);
  const float alpha = (ex > 1.0f) ? 1.0f : ex;
  const int acc = u < alpha;
  float zn[ORC_DMAX];
  for (int r = 0; r < d; ++r) zn[r] = acc ? zp[r] : s->z[r];
  const float pen = acc ? pep : s->pe;
  /* arwmh.py:180-185 */
  const int32_t itr = s->i + 1;
  const int32_t n = (s->i < cfg->num_warmup) ? itr : itr - cfg->num_warmup;
  const float gamma = amh_lr_gamma(n, cfg->lr_decay);
  const float maccn = s->macc + (alpha - s->macc) / (float)n;
  /* arwmh.py:188-189 */
  float delta[ORC_DMAX], mun[ORC_DMAX];
  for (int r = 0; r < d; ++r) {
    delta[r] = zn[r] - s->mu[r];
    mun[r] = s->mu[r] + gamma * delta[r];
  }
  /* arwmh.py:193 */
  const float lamn = s->lam + gamma * (alpha - cfg->target_accept_prob);
  const float e1 = amh_expf(lamn);
  /* arwmh.py:190-191: cholesky_update(sqrt(1-gamma) L, delta, gamma), NaN -> keep L */
  const float sq = sqrtf(1.0f - gamma);
  float Dg[ORC_DMAX], one[ORC_DMAX];
  for (int j = 0; j < d; ++j) {
    const float ajj = sq * s->dl[j];
    Dg[j] = ajj * ajj;
    one[j] = (amh_isfinite(ajj) && ajj != 0.0f) ? 1.0f : NAN;
  }
  /* sweep 1: forward solve U w* = delta; w*_j captured when column j is applied */
  float w[ORC_DMAX], ws[ORC_DMAX];
  for (int r = 0; r < d; ++r) w[r] = delta[r];
  for (int j = 0; j < d; ++j) {
    const float wj = w[j];
    ws[j] = wj;
    for (int r = 0; r < d; ++r) w[r] = fmaf(-wj, s->U[r][j], w[r]);
  }
  /* per-column scalars, all columns at once; b_j by exclusive scan */
  float t[ORC_DMAX], bsc[ORC_DMAX], cc[ORC_DMAX], qq[ORC_DMAX], gw2[ORC_DMAX], dnew[ORC_DMAX];
  for (int r = 0; r < G; ++r) {
    gw2[r] = (r < d) ? gamma * (ws[r] * ws[r]) : 0.0f;
    t[r] = (r < d) ? gw2[r] / Dg[r] : 0.0f;
  }
  group_excl_scan(t, bsc, G);
  int revert = 0;
  for (int r = 0; r < d; ++r) {
    const float b = 1.0f + bsc[r];
    const float g = (b * Dg[r]) + gw2[r];
    const float dn = g / b;
    cc[r] = (gamma * ws[r]) / g;
    qq[r] = sqrtf(dn);
    dnew[r] = fmaf(cc[r], 0.0f, one[r]) * qq[r];
    revert |= amh_isnan(dnew[r]);
  }
  float sacc[ORC_DMAX], s4[ORC_DMAX][4]; /* as_change partial sums over j mod 4 */
  for (int r = 0; r < G; ++r) { sacc[r] = 0.0f; s4[r][0] = s4[r][1] = s4[r][2] = s4[r][3] = 0.0f; }
  if (!revert) {
    /* sweep 2: U'_rj = U_rj + c_j w_r^(j+1); as_change terms */
    /* L'_rj e1 - L_rj e0 = U_rj (q_j e1 - dl_j e0) + (c_j q_j e1) w_r^(j+1) */
    float ac[ORC_DMAX], bc[ORC_DMAX];
    for (int r = 0; r < d; ++r) { ac[r] = (qq[r] * e1) - (s->dl[r] * el); bc[r] = (cc[r] * qq[r]) * e1; }
    for (int r = 0; r < d; ++r) w[r] = delta[r];
    for (int j = 0; j < d; ++j) {
      for (int r = 0; r < d; ++r) {
        const float uo = s->U[r][j];
        w[r] = fmaf(-ws[j], uo, w[r]);
        const float un = fmaf(cc[j], w[r], uo);
        const float tt = fmaf(uo, ac[j], bc[j] * w[r]);
        s4[r][j & 3] = fmaf(tt, tt, s4[r][j & 3]);
        s->U[r][j] = un;
      }
    }
    for (int r = 0; r < d; ++r) sacc[r] = (s4[r][0] + s4[r][1]) + (s4[r][2] + s4[r][3]);
    s->asc = sqrtf(group_sum(sacc, G));
    for (int r = 0; r < d; ++r) s->dl[r] = qq[r];
    s->updated = 1;
  } else {
    /* factor unchanged: L_rj (e1 - e0) = U_rj (dl_j e1 - dl_j e0) */
    float ac[ORC_DMAX];
    for (int r = 0; r < d; ++r) ac[r] = (s->dl[r] * e1) - (s->dl[r] * el);
    for (int j = 0; j < d; ++j)
      for (int r = 0; r < d; ++r) {
        const float tt = s->U[r][j] * ac[j];
        s4[r][j & 3] = fmaf(tt, tt, s4[r][j & 3]);
      }
    for (int r = 0; r < d; ++r) sacc[r] = (s4[r][0] + s4[r][1]) + (s4[r][2] + s4[r][3]);
    s->asc = sqrtf(group_sum(sacc, G));
  }
  s->i = itr;
  for (int r = 0; r < d; ++r) { s->z[r] = zn[r]; s->mu[r] = mun[r]; }
  s->pe = pen;
  s->macc = maccn;
  s->lam = lamn;
  return acc;
}

/* launch-input conversion L -> (U, dl), kernel mirror */
static void chain_load(const orc_cfg* cfg, chain_t* s, int64_t c, const int32_t* i_, const float* z,
                       const float* pe, const float* macc, const float* mu, const float* L,
                       const float* lam, const float* asc) {
  const int d = cfg->d;
  const float* Lc = L + c * packed_size(d);
  float inv[ORC_DMAX];
  for (int r = 0; r < d; ++r) {
    s->dl[r] = Lc[col_off(d, r)];
    inv[r] = (amh_isfinite(s->dl[r]) && s->dl[r] != 0.0f) ? 1.0f / s->dl[r] : 0.0f;
  }
  for (int r = 0; r < d; ++r)
    for (int j = 0; j < d; ++j) {
      const float x = (r > j) ? Lc[col_off(d, j) + (r - j)] : 0.0f;
      s->U[r][j] = (r == j) ? 1.0f : x * inv[j];
    }
  for (int r = 0; r < d; ++r) { s->z[r] = z[c * d + r]; s->mu[r] = mu[c * d + r]; }
  s->i = i_[c];
  s->pe = pe[c];
  s->macc = macc[c];
  s->lam = lam[c];
  s->asc = asc[c];
  s->updated = 0;
}

/* L = U diag(dl) if any step of this launch updated the factor, else the
 * launch-input factor verbatim (kernel mirror) */
static void chain_store(const orc_cfg* cfg, const chain_t* s, int64_t c, const float* Lin, int32_t* i_,
                        float* z, float* pe, float* macc, float* mu, float* L, float* lam, float* asc) {
  const int d = cfg->d;
  float* Lc = L + c * packed_size(d);
  const float* L0 = Lin + c * packed_size(d);
  for (int j = 0; j < d; ++j)
    for (int r = j; r < d; ++r)
      Lc[col_off(d, j) + (r - j)] = s->updated ? s->U[r][j] * s->dl[j] : L0[col_off(d, j) + (r - j)];
  for (int r = 0; r < d; ++r) { z[c * d + r] = s->z[r]; mu[c * d + r] = s->mu[r]; }
  i_[c] = s->i;
  pe[c] = s->pe;
  macc[c] = s->macc;
  lam[c] = s->lam;
  asc[c] = s->asc;
}

/* n_steps transitions of chains [0, C), in place (one kernel launch).  If
 * collect_z is given it receives z after every step: collect_z[t][c][r].
 * accept_count (nullable) is incremented per accepted proposal. */
static void orc_step_big(const orc_cfg* cfg, int64_t C, int32_t n_steps, int32_t* i_, float* z, float* pe,
                         float* macc, float* mu, float* L, float* lam, float* asc, const uint32_t* keys,
                         int32_t* accept_count, float* collect_z);

void orc_step(const orc_cfg* cfg, int64_t C, int32_t n_steps, int32_t* i_, float* z, float* pe,
              float* macc, float* mu, float* L, float* lam, float* asc, const uint32_t* keys,
              int32_t* accept_count, float* collect_z) {
  const int d = cfg->d;
  if (d > ORC_DMAX) {
    orc_step_big(cfg, C, n_steps, i_, z, pe, macc, mu, L, lam, asc, keys, accept_count, collect_z);
    return;
  }
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t c = 0; c < C; ++c) {
    chain_t* s = (chain_t*)malloc(sizeof(chain_t));
    /* the split transition (data-heavy models, amh_split.hip) is one launch
     * per step: the state goes through HBM (L = U diag(dl)) between steps */
    const int split = cfg->model_id == ORC_DIAMONDS && d >= 3 && d <= 32;
    chain_load(cfg, s, c, i_, z, pe, macc, mu, L, lam, asc);
    int nacc = 0;
    for (int32_t t = 0; t < n_steps; ++t) {
      if (split && t > 0) chain_load(cfg, s, c, i_, z, pe, macc, mu, L, lam, asc);
      nacc += chain_step(cfg, s, keys[2 * c], keys[2 * c + 1], (uint32_t)s->i);
      if (collect_z)
        for (int r = 0; r < d; ++r) collect_z[((int64_t)t * C + c) * d + r] = s->z[r];
      if (split && t + 1 < n_steps) chain_store(cfg, s, c, L, i_, z, pe, macc, mu, L, lam, asc);
    }
    chain_store(cfg, s, c, L, i_, z, pe, macc, mu, L, lam, asc);
    if (accept_count) accept_count[c] += nacc;
    free(s);
  }
}

/* ----------------------------------------------------------- sample_Pnx ---- */
/* arwmh.py:230-270: every chain (p, s) starts at x[p] with key
 * split(rng_key, (n_points, n_samples))[p, s] and runs n frozen-theta steps;
 * only z (and pe) are carried.  Step t draws its noise at stream position t. */
void orc_split_keys(const uint32_t* key, int64_t n, uint32_t* out) {
  for (int64_t c = 0; c < n; ++c) {
    const uint64_t g = (uint64_t)c;
    const amh_u32x4 o = amh_philox4x32_10((uint32_t)g, (uint32_t)(g >> 32), 0u, AMH_TAG_SPLIT, key[0], key[1]);
    out[2 * c] = o.v[0];
    out[2 * c + 1] = o.v[1];
  }
}

static void orc_sample_pnx_big(const orc_cfg* cfg, const uint32_t* keys, const float* x, int64_t n_points,
                               int64_t n_samples, const float* Lpacked, float log_step_size, int32_t n, float* out);

void orc_sample_pnx(const orc_cfg* cfg, const uint32_t* key, const float* x, int64_t n_points,
                    int64_t n_samples, const float* loc, const float* Lpacked, float log_step_size,
                    int32_t n, float* out) {
  const int d = cfg->d;
  const int64_t C = n_points * n_samples;
  if (d > ORC_DMAX) {
    uint32_t* bkeys = (uint32_t*)malloc(sizeof(uint32_t) * 2 * (size_t)C);
    orc_split_keys(key, C, bkeys);
    orc_sample_pnx_big(cfg, bkeys, x, n_points, n_samples, Lpacked, log_step_size, n, out);
    free(bkeys);
    return;
  }
  uint32_t* keys = (uint32_t*)malloc(sizeof(uint32_t) * 2 * (size_t)C);
  orc_split_keys(key, C, keys);
  (void)loc;
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t c = 0; c < C; ++c) {
    const int64_t p = c / n_samples;
    float A[ORC_DMAX][ORC_DMAX];
    memset(A, 0, sizeof(A));
    for (int j = 0; j < d; ++j)
      for (int r = j; r < d; ++r) A[r][j] = Lpacked[col_off(d, j) + (r - j)];
    float z[ORC_DMAX], zp[ORC_DMAX], xi[ORC_DMAX];
    for (int r = 0; r < d; ++r) z[r] = x[p * d + r];
    float pe = orc_potential1(cfg, z);
    const float el = amh_expf(log_step_size);
    for (int32_t t = 0; t < n; ++t) {
      float u;
      amh_step_noise(d, (uint32_t)t, keys[2 * c], keys[2 * c + 1], xi, &u);
      for (int r = 0; r < d; ++r) {
        float acc = 0.0f;
        for (int j = 0; j < d; ++j) acc = fmaf(A[r][j], xi[j], acc);
        zp[r] = z[r] + fmaf(el, acc, cfg->eps * xi[r]);
      }
      float pep = orc_potential1(cfg, zp);
      if (amh_isnan(pep)) pep = INFINITY;
      const float ex = amh_expf(pe - pep);
      const float alpha = (ex > 1.0f) ? 1.0f : ex;
      if (u < alpha) {
        for (int r = 0; r < d; ++r) z[r] = zp[r];
        pe = pep;
      }
    }
    for (int r = 0; r < d; ++r) out[c * d + r] = z[r];
  }
  free(keys);
}

/* ------------------------------------------- elementwise math (for tests) ---- */
void orc_philox(const uint32_t* ctr, const uint32_t* key, uint32_t* out, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    const amh_u32x4 o = amh_philox4x32_10(ctr[4 * i], ctr[4 * i + 1], ctr[4 * i + 2], ctr[4 * i + 3],
                                          key[2 * i], key[2 * i + 1]);
    memcpy(out + 4 * i, o.v, 16);
  }
}
void orc_logf(const float* x, float* y, int64_t n) { for (int64_t i = 0; i < n; ++i) y[i] = amh_logf(x[i]); }
void orc_expf(const float* x, float* y, int64_t n) { for (int64_t i = 0; i < n; ++i) y[i] = amh_expf(x[i]); }
void orc_log1pf(const float* x, float* y, int64_t n) { for (int64_t i = 0; i < n; ++i) y[i] = amh_log1pf(x[i]); }
void orc_erfinvf(const float* x, float* y, int64_t n) { for (int64_t i = 0; i < n; ++i) y[i] = amh_erfinvf(x[i]); }
void orc_normal_bits(const uint32_t* b, float* y, int64_t n) { for (int64_t i = 0; i < n; ++i) y[i] = amh_normal_from_bits(b[i]); }
void orc_lr_gamma(const int32_t* nn, float a, float* y, int64_t n) { for (int64_t i = 0; i < n; ++i) y[i] = amh_lr_gamma(nn[i], a); }
int orc_num_threads(void) {
#ifdef _OPENMP
  extern int omp_get_max_threads(void);
  return omp_get_max_threads();
#else
  return 1;
#endif
}

/* ================================================= pooled covariance ==== */
/* Regime B (build-defined): every chain proposes with ONE
 * shared adapt state (mu, L, lambda); the adaptation consumes the pooled
 * statistics of all chains (all ranks):
 *   S_d = sum_c delta_c,  S_dd = sum_c delta_c delta_c^T,  S_a = sum_c alpha_c
 *   mu'  = mu + gamma S_d / N
 *   Sig' = (1 - gamma) Sig + gamma S_dd / N,   L' = chol(Sig')  (else keep)
 *   lam' = lam + gamma (S_a / N - target),     macc' = macc + (S_a/N - macc)/n
 * With N = 1 this is the reference recurrence (arwmh.py:180-197) with the
 * rank-one update replaced by a refactorisation.
 *
 * Kernel mirror: one chain per 64-lane wave (G = 64 for every d <= 64);
 * chunks of 16 waves x cpw consecutive chains; per wave float32 accumulators
 * over its chains in order, the 16 wave partials of a chunk combined by a
 * float32 pairwise tree (w += w + h for h = 8, 4, 2, 1) and converted to
 * double, chunk partials summed in double in groups of 16
 * chunks (chunk order), the group sums in group order.
 * sums layout (V = d + P + 2 doubles): [S_d (d) | S_dd packed col-major (P) |
 * S_a | N]. */
#define ORC_POOLED_WAVES 16
#define ORC_BIG_D 256

int orc_pooled_cpw(int64_t C) {
  const int64_t c = (C + 4095) / 4096;
  return c < 1 ? 1 : (c > 16 ? 16 : (int)c);
}

static float orc_potential_g(const orc_cfg* cfg, const float* x, int G) {
  switch (cfg->model_id) {
    case ORC_GAUSSIAN: return pot_gaussian(cfg, x, G);
    case ORC_EIGHT_SCHOOLS: return pot_eight_schools(cfg, x, G);
    case ORC_KIDIQ: return pot_kidiq(cfg, x, G);
    case ORC_DIAMONDS: return pot_diamonds(cfg, x, G);
    case ORC_DIAMONDS_SS: return pot_diamonds_ss(cfg, x, G);
    case ORC_MIXTURE: return pot_mixture(cfg, x, G);
    default: return NAN;
  }
}

/* Per-chain transition with the shared state; writes z/pe out and the
 * pooled sums.  i: shared iteration (noise stream position). */
static void orc_pooled_stats_big(const orc_cfg* cfg, int64_t C, int32_t i, const float* z, const float* pe,
                                 const uint32_t* keys, const float* mu, const float* Lpacked, float lam,
                                 float* z_out, float* pe_out, double* sums);
static int orc_pooled_update_big(const orc_cfg* cfg, const double* sums, int32_t K, int32_t* i_, float* macc,
                                 float* mu, float* Lpacked, float* lam, float* asc, double* cov);

/* The MFMA path of the pooled mode (amh_big_pooled.hip): the dense Gaussian
 * with d % 32 == 0, 64 <= d <= 256 (amh_internal.h pooled_big_model). */
static int orc_pooled_big(const orc_cfg* cfg) {
  return cfg->model_id == ORC_GAUSSIAN && cfg->d >= 64 && cfg->d <= ORC_BIG_D && cfg->d % 32 == 0;
}

/* Pool every K (amh_pooled_stats_k): K transitions per chain with the frozen
 * shared state at noise positions i .. i+K-1, the sums over all K*C
 * chain-steps.  Lane-per-row path: one kernel, each wave's chains in order
 * with each chain's K steps in order.  MFMA path, d = 64: one launch, the
 * chunk sums over (sub-chunk, step, chain) (orc_pooled_stats64_k); d > 64: K
 * launch sequences, sums accumulated in step order (sums = s_0, then
 * sums + s_t). */
static void orc_pooled_stats64_k(const orc_cfg* cfg, int64_t C, int32_t i, int32_t K, const float* z,
                                 const float* pe, const uint32_t* keys, const float* mu, const float* Lpacked,
                                 float lam, float* z_out, float* pe_out, double* sums);

void orc_pooled_stats_k(const orc_cfg* cfg, int64_t C, int32_t i, int32_t K, const float* z, const float* pe,
                        const uint32_t* keys, const float* mu, const float* Lpacked, float lam,
                        float* z_out, float* pe_out, double* sums) {
  const int d = cfg->d;
  if (d > ORC_DMAX && !orc_pooled_big(cfg)) { /* no pooled mode there (the library returns AMH_EINVAL) */
    for (int64_t v = 0; v < d + packed_size(d) + 2; ++v) sums[v] = NAN;
    return;
  }
  if (orc_pooled_big(cfg) && d == 64) {
    orc_pooled_stats64_k(cfg, C, i, K, z, pe, keys, mu, Lpacked, lam, z_out, pe_out, sums);
    return;
  }
  if (orc_pooled_big(cfg)) {
    const int64_t V = d + packed_size(d) + 2;
    double* tmp = (double*)malloc((size_t)V * sizeof(double));
    for (int32_t t = 0; t < K; ++t) {
      orc_pooled_stats_big(cfg, C, i + t, t ? z_out : z, t ? pe_out : pe, keys, mu, Lpacked, lam, z_out, pe_out,
                           t ? tmp : sums);
      if (t)
        for (int64_t v = 0; v < V; ++v) sums[v] = sums[v] + tmp[v];
    }
    free(tmp);
    return;
  }
  const int64_t P = packed_size(d);
  const int64_t V = d + P + 2;
  const int cpw = orc_pooled_cpw(C);
  const int64_t chunk = (int64_t)ORC_POOLED_WAVES * cpw;
  const int64_t n_chunks = (C + chunk - 1) / chunk;
  float L[ORC_DMAX][ORC_DMAX];
  memset(L, 0, sizeof(L));
  for (int j = 0; j < d; ++j)
    for (int r = j; r < d; ++r) L[r][j] = Lpacked[col_off(d, j) + (r - j)];
  const float el = amh_expf(lam);
  double* part = (double*)calloc((size_t)(n_chunks * V), sizeof(double));
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t ch = 0; ch < n_chunks; ++ch) {
    double* acc = part + ch * V;
    double cnt = 0.0;
    /* per-wave float32 partials: S[w][r][k] (k <= r), sd[w][r], sa[w] */
    float (*S)[ORC_DMAX][ORC_DMAX] = calloc(ORC_POOLED_WAVES, sizeof(*S));
    float sd[ORC_POOLED_WAVES][ORC_DMAX], sa[ORC_POOLED_WAVES];
    memset(sd, 0, sizeof(sd));
    memset(sa, 0, sizeof(sa));
    for (int w = 0; w < ORC_POOLED_WAVES; ++w) {
      for (int t = 0; t < cpw; ++t) {
        const int64_t c = ch * chunk + (int64_t)w * cpw + t;
        if (c >= C) continue;
        const uint32_t k0 = keys[2 * c], k1 = keys[2 * c + 1];
        float zc[ORC_DMAX], pec = pe[c];
        for (int r = 0; r < d; ++r) zc[r] = z[c * d + r];
        for (int32_t s = 0; s < K; ++s) {
          cnt += 1.0;
          float xi[ORC_DMAX], zp[ORC_DMAX], delta[ORC_DMAX];
          float u;
          amh_step_noise(d, (uint32_t)(i + s), k0, k1, xi, &u);
          for (int r = 0; r < d; ++r) {
            float a4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            for (int j = 0; j < d; ++j) a4[j & 3] = fmaf(L[r][j], xi[j], a4[j & 3]);
            const float a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
            zp[r] = zc[r] + fmaf(el, a, cfg->eps * xi[r]);
          }
          float pep = orc_potential_g(cfg, zp, 64);
          if (amh_isnan(pep)) pep = INFINITY;
          const float ex = amh_expf(pec - pep);
          const float alpha = (ex > 1.0f) ? 1.0f : ex;
          const int accept = u < alpha;
          for (int r = 0; r < d; ++r) {
            zc[r] = accept ? zp[r] : zc[r];
            delta[r] = zc[r] - mu[r];
          }
          pec = accept ? pep : pec;
          for (int r = 0; r < d; ++r) {
            sd[w][r] = sd[w][r] + delta[r];
            for (int k = 0; k <= r; ++k) S[w][r][k] = fmaf(delta[r], delta[k], S[w][r][k]);
          }
          sa[w] = sa[w] + alpha;
        }
        for (int r = 0; r < d; ++r) z_out[c * d + r] = zc[r];
        pe_out[c] = pec;
      }
    }
    /* pairwise tree over the 16 waves (h = 8, 4, 2, 1), float32 */
    for (int h = ORC_POOLED_WAVES / 2; h >= 1; h /= 2)
      for (int w = 0; w < h; ++w) {
        for (int r = 0; r < d; ++r) {
          for (int k = 0; k <= r; ++k) S[w][r][k] = S[w][r][k] + S[w + h][r][k];
          sd[w][r] = sd[w][r] + sd[w + h][r];
        }
        sa[w] = sa[w] + sa[w + h];
      }
    for (int r = 0; r < d; ++r) acc[r] = (double)sd[0][r];
    for (int k = 0; k < d; ++k)
      for (int r = k; r < d; ++r) acc[d + col_off(d, k) + (r - k)] = (double)S[0][r][k];
    acc[d + P] = (double)sa[0];
    free(S);
    acc[d + P + 1] = cnt;
  }
  /* chunk partials: groups of 16 chunks in chunk order, then the groups in
   * group order (pooled_reduce_kernel) */
  const int64_t n_groups = (n_chunks + 15) / 16;
  for (int64_t v = 0; v < V; ++v) {
    double tot = 0.0;
    for (int64_t g = 0; g < n_groups; ++g) {
      double s = 0.0;
      for (int64_t ch = g * 16; ch < n_chunks && ch < (g + 1) * 16; ++ch) s += part[ch * V + v];
      tot += s;
    }
    sums[v] = tot;
  }
  free(part);
}

void orc_pooled_stats(const orc_cfg* cfg, int64_t C, int32_t i, const float* z, const float* pe,
                      const uint32_t* keys, const float* mu, const float* Lpacked, float lam,
                      float* z_out, float* pe_out, double* sums) {
  orc_pooled_stats_k(cfg, C, i, 1, z, pe, keys, mu, Lpacked, lam, z_out, pe_out, sums);
}

/* Shared-state update from the (all-reduced) sums.  Returns 1 if the factor
 * was refactorised, 0 if kept. */
/* the block counter of amh_internal.h pooled_block_n: n = it / K + 1 (reset at W) */
static int32_t orc_block_n(int32_t it, int32_t W, int32_t K) { return (it < W) ? it / K + 1 : (it - W) / K + 1; }

int orc_pooled_update_k(const orc_cfg* cfg, const double* sums, int32_t K, int32_t* i_, float* macc, float* mu,
                        float* Lpacked, float* lam, float* asc, double* cov) {
  const int d = cfg->d;
  if (orc_pooled_big(cfg)) return orc_pooled_update_big(cfg, sums, K, i_, macc, mu, Lpacked, lam, asc, cov);
  if (d > ORC_DMAX) return 0; /* no pooled mode at this d (see orc_pooled_stats_k) */
  const int64_t P = packed_size(d);
  const double N = sums[d + P + 1];
  const int32_t it = *i_;
  const int32_t itr = it + K;
  const int32_t n = orc_block_n(it, cfg->num_warmup, K);
  const float gamma = amh_lr_gamma(n, cfg->lr_decay);
  const float abar = (float)(sums[d + P] / N);
  const float maccn = *macc + (abar - *macc) / (float)n;
  const float lamn = *lam + gamma * (abar - cfg->target_accept_prob);
  for (int r = 0; r < d; ++r) mu[r] = mu[r] + gamma * (float)(sums[r] / N);
  const double g = (double)gamma;
  /* Sig' and its Cholesky factor, lower triangle A[r][k], k <= r */
  double A[ORC_DMAX][ORC_DMAX];
  memset(A, 0, sizeof(A));
  for (int k = 0; k < d; ++k)
    for (int r = k; r < d; ++r) {
      const int64_t o = col_off(d, k) + (r - k);
      const double a = (1.0 - g) * cov[o];
      const double b = g * (sums[d + o] / N);
      A[r][k] = a + b;
    }
  double Sn[ORC_DMAX][ORC_DMAX];
  memcpy(Sn, A, sizeof(A));
  int ok = 1;
  for (int j = 0; j < d; ++j) {
    const double piv = A[j][j];
    if (!(piv > 0.0) || !isfinite(piv)) { ok = 0; break; }
    const double ljj = sqrt(piv);
    for (int r = j + 1; r < d; ++r) A[r][j] = A[r][j] / ljj;
    A[j][j] = ljj;
    for (int k = j + 1; k < d; ++k)
      for (int r = k; r < d; ++r) A[r][k] = fma(-A[r][j], A[k][j], A[r][k]);
  }
  const float e0 = amh_expf(*lam), e1 = amh_expf(lamn);
  float part[ORC_DMAX];
  for (int r = 0; r < 64; ++r) part[r] = 0.0f;
  for (int r = 0; r < d; ++r) {
    float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int j = 0; j <= r; ++j) {
      const float lo = Lpacked[col_off(d, j) + (r - j)];
      const float ln = ok ? (float)A[r][j] : lo;
      const float tt = (ln * e1) - (lo * e0);
      s4[j & 3] = fmaf(tt, tt, s4[j & 3]);
    }
    part[r] = (s4[0] + s4[1]) + (s4[2] + s4[3]);
  }
  *asc = sqrtf(group_sum(part, 64));
  if (ok) {
    for (int k = 0; k < d; ++k)
      for (int r = k; r < d; ++r) {
        const int64_t o = col_off(d, k) + (r - k);
        Lpacked[o] = (float)A[r][k];
        cov[o] = Sn[r][k];
      }
  }
  *i_ = itr;
  *macc = maccn;
  *lam = lamn;
  return ok;
}

int orc_pooled_update(const orc_cfg* cfg, const double* sums, int32_t* i_, float* macc, float* mu,
                      float* Lpacked, float* lam, float* asc, double* cov) {
  return orc_pooled_update_k(cfg, sums, 1, i_, macc, mu, Lpacked, lam, asc, cov);
}

/* ====================================== large dimensions (64 < d <= 256) ==== */
/* Dense Gaussian only, any 64 < d <= 256 (amh_big.hip).  Kernel mirror:
 *
 * potential  batched over chains on MFMA (v_mfma_f32_32x32x2_f32, a k-ordered
 *            fmaf chain): y_r = fmaf chain over k = 0..d-1 of P_rk D_k with
 *            D = x - m; q_r = D_r y_r (q_r = 0 for the rows d .. 32 ceil(d /
 *            32) - 1 of a ragged last tile); each 32-row tile I is summed as two
 *            sequential halves over the accumulator layout (rows (reg & 3) +
 *            8 (reg >> 2) + 4 h, reg = 0..15, h = 0, 1), t_I = p_I0 + p_I1,
 *            S = sequential sum of t_I over I; U = 0.5 S + c0.
 * transition one wave per chain, lane l holds rows r = 64 s + l (slots s).
 *            propose pass (column order j = 0..d-1): acc_r = fmaf chain of
 *            U_rj eta_j over j <= r (U_rr = 1); at column r the row's
 *            proposal is complete and both forward solves of the rank-one
 *            update finalise  wa_r = (z'_r - mu_r) - sa_r,
 *            wr_r = (z_r - mu_r) - sr_r,  with sa_r, sr_r the fmaf chains of
 *            U_rj wa_j, U_rj wr_j over j < r (w = U^-1 delta for the accepted
 *            and the rejected delta).  Step pass: b by a 64-lane scan per slot
 *            plus carries, then column order again: s_r = fmaf(U_rj, ws_j,
 *            s_r), w = delta_r - s_r, U'_rj = fmaf(c_j, w, U_rj) for r > j
 *            (U'_jj stays 1), as_change terms sequential per row; row sums
 *            by the 64-lane butterfly per slot, then (s0 + s1) + (s2 + s3).
 *            Each step is one launch sequence (state through HBM). */
#define ORC_BIG 256

static float pot_gaussian_big(const orc_cfg* cfg, const float* x) {
  const int d = cfg->d;
  const float* m = cfg->data;
  const float* P = cfg->data + d;
  const float c0 = cfg->data[d + d * d];
  float D[ORC_BIG], q[ORC_BIG];
  for (int k = 0; k < d; ++k) D[k] = x[k] - m[k];
  for (int r = 0; r < d; ++r) {
    float y = 0.0f;
    for (int k = 0; k < d; ++k) y = fmaf(P[r * d + k], D[k], y);
    q[r] = D[r] * y;
  }
  for (int r = d; r < ((d + 31) & ~31); ++r) q[r] = 0.0f; /* a ragged last tile: zero rows */
  float S = 0.0f;
  for (int I = 0; I < (d + 31) / 32; ++I) {
    float ph[2];
    for (int h = 0; h < 2; ++h) {
      float p = 0.0f;
      for (int reg = 0; reg < 16; ++reg) p = p + q[32 * I + (reg & 3) + 8 * (reg >> 2) + 4 * h];
      ph[h] = p;
    }
    S = S + (ph[0] + ph[1]);
  }
  return (0.5f * S) + c0;
}

/* sum over rows: 64-lane butterfly per slot, then (s0 + s1) + (s2 + s3) */
static float big_sum(const float* v, int d) {
  float sl[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  for (int k = 0; k < 4; ++k) {
    float x[64];
    for (int l = 0; l < 64; ++l) x[l] = (64 * k + l < d) ? v[64 * k + l] : 0.0f;
    sl[k] = group_sum(x, 64);
  }
  return (sl[0] + sl[1]) + (sl[2] + sl[3]);
}

/* exclusive scan over rows: 64-lane scan per slot plus the carry of the
 * slots before (carry_s = carry_{s-1} + total_{s-1}) */
static void big_excl_scan(const float* t, float* out, int d) {
  float carry = 0.0f;
  for (int k = 0; k < 4; ++k) {
    float x[64], e[64];
    for (int l = 0; l < 64; ++l) x[l] = (64 * k + l < d) ? t[64 * k + l] : 0.0f;
    group_excl_scan(x, e, 64);
    for (int l = 0; l < 64; ++l)
      if (64 * k + l < d) out[64 * k + l] = (k == 0) ? e[l] : e[l] + carry;
    const float tot = e[63] + x[63];
    carry = (k == 0) ? tot : carry + tot;
  }
}

typedef struct {
  float z[ORC_BIG], mu[ORC_BIG], dl[ORC_BIG], inv[ORC_BIG];
  float U[ORC_BIG][ORC_BIG]; /* U_rj = L_rj / L_jj for r > j (others unused) */
} bigchain_t;

/* one transition of chain c in place (propose pass, potential, step pass) */
static int big_step1(const orc_cfg* cfg, bigchain_t* s, int64_t c, int32_t* i_, float* z, float* pe, float* macc,
                     float* mu, float* L, float* lam, float* asc, const uint32_t* keys) {
  const int d = cfg->d;
  const int64_t P = packed_size(d);
  float* Lc = L + c * P;
  for (int r = 0; r < d; ++r) {
    s->dl[r] = Lc[col_off(d, r)];
    s->inv[r] = (amh_isfinite(s->dl[r]) && s->dl[r] != 0.0f) ? 1.0f / s->dl[r] : 0.0f;
    s->z[r] = z[c * d + r];
    s->mu[r] = mu[c * d + r];
  }
  for (int j = 0; j < d; ++j)
    for (int r = j + 1; r < d; ++r) s->U[r][j] = Lc[col_off(d, j) + (r - j)] * s->inv[j];
  const int32_t it = i_[c];
  const uint32_t k0 = keys[2 * c], k1 = keys[2 * c + 1];
  float xi[ORC_BIG], eta[ORC_BIG], acc[ORC_BIG], sa[ORC_BIG], sr[ORC_BIG], zp[ORC_BIG], wa[ORC_BIG], wr[ORC_BIG];
  float u;
  amh_step_noise(d, (uint32_t)it, k0, k1, xi, &u);
  for (int r = 0; r < d; ++r) {
    eta[r] = s->dl[r] * xi[r];
    acc[r] = sa[r] = sr[r] = 0.0f;
  }
  const float el = amh_expf(lam[c]);
  /* propose pass */
  for (int j = 0; j < d; ++j) {
    acc[j] = fmaf(1.0f, eta[j], acc[j]);
    zp[j] = s->z[j] + fmaf(el, acc[j], cfg->eps * xi[j]);
    wa[j] = (zp[j] - s->mu[j]) - sa[j];
    wr[j] = (s->z[j] - s->mu[j]) - sr[j];
    for (int r = j + 1; r < d; ++r) {
      const float uo = s->U[r][j];
      acc[r] = fmaf(uo, eta[j], acc[r]);
      sa[r] = fmaf(uo, wa[j], sa[r]);
      sr[r] = fmaf(uo, wr[j], sr[r]);
    }
  }
  float pep = pot_gaussian_big(cfg, zp);
  if (amh_isnan(pep)) pep = INFINITY;
  /* step pass */
  const float ex = amh_expf(pe[c] - pep);
  const float alpha = (ex > 1.0f) ? 1.0f : ex;
  const int accept = u < alpha;
  const int32_t itr = it + 1;
  const int32_t n = (it < cfg->num_warmup) ? itr : itr - cfg->num_warmup;
  const float gamma = amh_lr_gamma(n, cfg->lr_decay);
  const float maccn = macc[c] + (alpha - macc[c]) / (float)n;
  float delta[ORC_BIG], ws[ORC_BIG], t[ORC_BIG], gw2[ORC_BIG], Dg[ORC_BIG], one[ORC_BIG], bsc[ORC_BIG];
  float cc[ORC_BIG], qq[ORC_BIG], sacc[ORC_BIG];
  for (int r = 0; r < d; ++r) {
    const float zn = accept ? zp[r] : s->z[r];
    delta[r] = zn - s->mu[r];
    ws[r] = accept ? wa[r] : wr[r];
  }
  const float lamn = lam[c] + gamma * (alpha - cfg->target_accept_prob);
  const float e1 = amh_expf(lamn);
  const float sq = sqrtf(1.0f - gamma);
  for (int r = 0; r < d; ++r) {
    const float ajj = sq * s->dl[r];
    Dg[r] = ajj * ajj;
    one[r] = (amh_isfinite(ajj) && ajj != 0.0f) ? 1.0f : NAN;
    gw2[r] = gamma * (ws[r] * ws[r]);
    t[r] = gw2[r] / Dg[r];
  }
  big_excl_scan(t, bsc, d);
  int revert = 0;
  for (int r = 0; r < d; ++r) {
    const float b = 1.0f + bsc[r];
    const float g = (b * Dg[r]) + gw2[r];
    const float dn = g / b;
    cc[r] = (gamma * ws[r]) / g;
    qq[r] = sqrtf(dn);
    revert |= amh_isnan(fmaf(cc[r], 0.0f, one[r]) * qq[r]);
  }
  for (int r = 0; r < d; ++r) sacc[r] = 0.0f;
  if (!revert) {
    float ac[ORC_BIG], bc[ORC_BIG], sv[ORC_BIG];
    for (int r = 0; r < d; ++r) {
      ac[r] = (qq[r] * e1) - (s->dl[r] * el);
      bc[r] = (cc[r] * qq[r]) * e1;
      sv[r] = 0.0f;
    }
    for (int j = 0; j < d; ++j) {
      {
        const float tt = fmaf(1.0f, ac[j], bc[j] * 0.0f);
        sacc[j] = fmaf(tt, tt, sacc[j]);
        Lc[col_off(d, j)] = 1.0f * qq[j];
      }
      for (int r = j + 1; r < d; ++r) {
        const float uo = s->U[r][j];
        sv[r] = fmaf(uo, ws[j], sv[r]);
        const float w = delta[r] - sv[r];
        const float un = fmaf(cc[j], w, uo);
        const float tt = fmaf(uo, ac[j], bc[j] * w);
        sacc[r] = fmaf(tt, tt, sacc[r]);
        Lc[col_off(d, j) + (r - j)] = un * qq[j];
      }
    }
  } else {
    float ac[ORC_BIG];
    for (int r = 0; r < d; ++r) ac[r] = (s->dl[r] * e1) - (s->dl[r] * el);
    for (int j = 0; j < d; ++j) {
      const float t0 = 1.0f * ac[j];
      sacc[j] = fmaf(t0, t0, sacc[j]);
      for (int r = j + 1; r < d; ++r) {
        const float tt = s->U[r][j] * ac[j];
        sacc[r] = fmaf(tt, tt, sacc[r]);
      }
    }
  }
  asc[c] = sqrtf(big_sum(sacc, d));
  for (int r = 0; r < d; ++r) {
    z[c * d + r] = accept ? zp[r] : s->z[r];
    mu[c * d + r] = s->mu[r] + gamma * delta[r];
  }
  i_[c] = itr;
  pe[c] = accept ? pep : pe[c];
  macc[c] = maccn;
  lam[c] = lamn;
  return accept;
}

static void orc_step_big(const orc_cfg* cfg, int64_t C, int32_t n_steps, int32_t* i_, float* z, float* pe,
                         float* macc, float* mu, float* L, float* lam, float* asc, const uint32_t* keys,
                         int32_t* accept_count, float* collect_z) {
  const int d = cfg->d;
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t c = 0; c < C; ++c) {
    bigchain_t* s = (bigchain_t*)malloc(sizeof(bigchain_t));
    int nacc = 0;
    for (int32_t t = 0; t < n_steps; ++t) {
      nacc += big_step1(cfg, s, c, i_, z, pe, macc, mu, L, lam, asc, keys);
      if (collect_z)
        for (int r = 0; r < d; ++r) collect_z[((int64_t)t * C + c) * d + r] = z[c * d + r];
    }
    if (accept_count) accept_count[c] += nacc;
    free(s);
  }
}

/* arwmh.py:230-270 (ARWMH.sample_Pnx) for 64 < d <= 256, dense Gaussian,
 * mirror of big_pnx_kernel (amh_big.hip): the d <= 64 rule (above) with
 * acc_r the fmaf chain of L_rj xi_j over j <= r (the zero terms j > r of the
 * small-d loop leave acc unchanged: acc starts at +0 and an fmaf with a zero
 * product never makes it -0) and U by pot_gaussian_big, the start point's
 * included. */
static void orc_sample_pnx_big(const orc_cfg* cfg, const uint32_t* keys, const float* x, int64_t n_points,
                               int64_t n_samples, const float* Lpacked, float log_step_size, int32_t n, float* out) {
  const int d = cfg->d;
  const int64_t C = n_points * n_samples;
  const float el = amh_expf(log_step_size);
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t c = 0; c < C; ++c) {
    const int64_t p = c / n_samples;
    float z[ORC_BIG], zp[ORC_BIG], xi[ORC_BIG];
    for (int r = 0; r < d; ++r) z[r] = x[p * d + r];
    float pe = pot_gaussian_big(cfg, z);
    for (int32_t t = 0; t < n; ++t) {
      float u = 0.0f;
      amh_step_noise(d, (uint32_t)t, keys[2 * c], keys[2 * c + 1], xi, &u);
      for (int r = 0; r < d; ++r) {
        float acc = 0.0f;
        for (int j = 0; j <= r; ++j) acc = fmaf(Lpacked[col_off(d, j) + (r - j)], xi[j], acc);
        zp[r] = z[r] + fmaf(el, acc, cfg->eps * xi[r]);
      }
      float pep = pot_gaussian_big(cfg, zp);
      if (amh_isnan(pep)) pep = INFINITY;
      const float ex = amh_expf(pe - pep);
      const float alpha = (ex > 1.0f) ? 1.0f : ex;
      if (u < alpha) {
        for (int r = 0; r < d; ++r) z[r] = zp[r];
        pe = pep;
      }
    }
    for (int r = 0; r < d; ++r) out[c * d + r] = z[r];
  }
}

/* ------------------------------------- pooled mode, large dimensions ---- */
/* Kernel mirror (amh_big_pooled.hip):
 *  proposal  z' = z + fmaf(e^lam, acc, eps xi), acc_r = fmaf chain over
 *            k < 32 (floor(r / 32) + 1) of L_rk xi_k (L_rk = 0 above the
 *            diagonal; MFMA on 32-row tiles), U(z') in the MFMA order.
 *  sums      chunks of 128 consecutive chains: float32 S_dd (fmaf chain over
 *            the chunk's chains in order, MFMA), S_d and S_a (sequential
 *            adds), written in double; chunks reduced as in the d <= 64 mode.
 *  update    Sigma' in double as the d <= 64 mode; its Cholesky factor in
 *            float32 (element (r, k) updated in column order j < k, then
 *            divided by L_kk = sqrtf(A_kk)); as_change: squared terms of
 *            column j (rows j + t) by big_sum, then the columns by big_sum. */
/* chains per chunk: 128 (pooled_fused64_kernel and pooled_fused_big_kernel:
 * two 64-chain sub-chunks per chunk) */
static int64_t orc_big_chunk(int d) { (void)d; return 128; }

static void orc_pooled_stats_big(const orc_cfg* cfg, int64_t C, int32_t i, const float* z, const float* pe,
                                 const uint32_t* keys, const float* mu, const float* Lpacked, float lam,
                                 float* z_out, float* pe_out, double* sums) {
  const int d = cfg->d;
  const int64_t P = packed_size(d);
  const int64_t V = d + P + 2;
  const int64_t chunk = orc_big_chunk(d);
  const int64_t n_chunks = (C + chunk - 1) / chunk;
  const float el = amh_expf(lam);
  double* part = (double*)calloc((size_t)(n_chunks * V), sizeof(double));
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t ch = 0; ch < n_chunks; ++ch) {
    float* S = (float*)calloc((size_t)d * d, sizeof(float));
    float sd[ORC_BIG], xi[ORC_BIG], zp[ORC_BIG], dl[ORC_BIG];
    float sa = 0.0f;
    double cnt = 0.0;
    for (int r = 0; r < d; ++r) sd[r] = 0.0f;
    for (int64_t c = ch * chunk; c < C && c < (ch + 1) * chunk; ++c) {
      cnt += 1.0;
      const uint32_t k0 = keys[2 * c], k1 = keys[2 * c + 1];
      float u;
      amh_step_noise(d, (uint32_t)i, k0, k1, xi, &u);
      for (int r = 0; r < d; ++r) {
        float acc = 0.0f;
        const int kend = 32 * (r / 32 + 1);
        for (int k = 0; k < kend; ++k) {
          const float lrk = (k <= r) ? Lpacked[col_off(d, k) + (r - k)] : 0.0f;
          acc = fmaf(lrk, xi[k], acc);
        }
        zp[r] = z[c * d + r] + fmaf(el, acc, cfg->eps * xi[r]);
      }
      float pep = pot_gaussian_big(cfg, zp);
      if (amh_isnan(pep)) pep = INFINITY;
      const float ex = amh_expf(pe[c] - pep);
      const float alpha = (ex > 1.0f) ? 1.0f : ex;
      const int accept = u < alpha;
      for (int r = 0; r < d; ++r) {
        const float zn = accept ? zp[r] : z[c * d + r];
        z_out[c * d + r] = zn;
        dl[r] = zn - mu[r];
      }
      pe_out[c] = accept ? pep : pe[c];
      for (int r = 0; r < d; ++r) {
        sd[r] = sd[r] + dl[r];
        for (int k = 0; k <= r; ++k) S[r * d + k] = fmaf(dl[r], dl[k], S[r * d + k]);
      }
      sa = sa + alpha;
    }
    double* acc = part + ch * V;
    for (int r = 0; r < d; ++r) acc[r] = (double)sd[r];
    for (int k = 0; k < d; ++k)
      for (int r = k; r < d; ++r) acc[d + col_off(d, k) + (r - k)] = (double)S[r * d + k];
    acc[d + P] = (double)sa;
    acc[d + P + 1] = cnt;
    free(S);
  }
  const int64_t n_groups = (n_chunks + 15) / 16;
  for (int64_t v = 0; v < V; ++v) {
    double tot = 0.0;
    for (int64_t g = 0; g < n_groups; ++g) {
      double s = 0.0;
      for (int64_t c2 = g * 16; c2 < n_chunks && c2 < (g + 1) * 16; ++c2) s += part[c2 * V + v];
      tot += s;
    }
    sums[v] = tot;
  }
  free(part);
}

/* d = 64 (pooled_fused64_kernel, round 5): the K steps of a block run in one
 * launch.  Each 128-chain chunk is two 64-chain sub-chunks; the chunk's
 * float32 sums run over its chain-steps in the order (sub-chunk, step, chain)
 * -- sub-chunk 0's K steps chain by chain, then sub-chunk 1's -- and the
 * chunks are reduced in double as for one step.  K = 1 is the per-step order
 * of orc_pooled_stats_big. */
static void orc_pooled_stats64_k(const orc_cfg* cfg, int64_t C, int32_t i, int32_t K, const float* z,
                                 const float* pe, const uint32_t* keys, const float* mu, const float* Lpacked,
                                 float lam, float* z_out, float* pe_out, double* sums) {
  const int d = cfg->d;
  const int64_t P = packed_size(d);
  const int64_t V = d + P + 2;
  const int64_t chunk = orc_big_chunk(d), sub = 64;
  const int64_t n_chunks = (C + chunk - 1) / chunk;
  const float el = amh_expf(lam);
  double* part = (double*)calloc((size_t)(n_chunks * V), sizeof(double));
  for (int64_t c = 0; c < C; ++c) {
    for (int r = 0; r < d; ++r) z_out[c * d + r] = z[c * d + r];
    pe_out[c] = pe[c];
  }
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t ch = 0; ch < n_chunks; ++ch) {
    float* S = (float*)calloc((size_t)d * d, sizeof(float));
    float sd[ORC_BIG], xi[ORC_BIG], zp[ORC_BIG], dl[ORC_BIG];
    float sa = 0.0f;
    double cnt = 0.0;
    for (int r = 0; r < d; ++r) sd[r] = 0.0f;
    for (int64_t s0 = ch * chunk; s0 < C && s0 < (ch + 1) * chunk; s0 += sub) {
      for (int32_t t = 0; t < K; ++t) {
        for (int64_t c = s0; c < C && c < s0 + sub; ++c) {
          cnt += 1.0;
          float* zc = z_out + c * d;
          float u;
          amh_step_noise(d, (uint32_t)(i + t), keys[2 * c], keys[2 * c + 1], xi, &u);
          for (int r = 0; r < d; ++r) {
            float acc = 0.0f;
            const int kend = 32 * (r / 32 + 1);
            for (int k = 0; k < kend; ++k) {
              const float lrk = (k <= r) ? Lpacked[col_off(d, k) + (r - k)] : 0.0f;
              acc = fmaf(lrk, xi[k], acc);
            }
            zp[r] = zc[r] + fmaf(el, acc, cfg->eps * xi[r]);
          }
          float pep = pot_gaussian_big(cfg, zp);
          if (amh_isnan(pep)) pep = INFINITY;
          const float ex = amh_expf(pe_out[c] - pep);
          const float alpha = (ex > 1.0f) ? 1.0f : ex;
          const int accept = u < alpha;
          for (int r = 0; r < d; ++r) {
            if (accept) zc[r] = zp[r];
            dl[r] = zc[r] - mu[r];
          }
          if (accept) pe_out[c] = pep;
          for (int r = 0; r < d; ++r) {
            sd[r] = sd[r] + dl[r];
            for (int k = 0; k <= r; ++k) S[r * d + k] = fmaf(dl[r], dl[k], S[r * d + k]);
          }
          sa = sa + alpha;
        }
      }
    }
    double* acc = part + ch * V;
    for (int r = 0; r < d; ++r) acc[r] = (double)sd[r];
    for (int k = 0; k < d; ++k)
      for (int r = k; r < d; ++r) acc[d + col_off(d, k) + (r - k)] = (double)S[r * d + k];
    acc[d + P] = (double)sa;
    acc[d + P + 1] = cnt;
    free(S);
  }
  const int64_t n_groups = (n_chunks + 15) / 16;
  for (int64_t v = 0; v < V; ++v) {
    double tot = 0.0;
    for (int64_t g = 0; g < n_groups; ++g) {
      double s = 0.0;
      for (int64_t c2 = g * 16; c2 < n_chunks && c2 < (g + 1) * 16; ++c2) s += part[c2 * V + v];
      tot += s;
    }
    sums[v] = tot;
  }
  free(part);
}

static int orc_pooled_update_big(const orc_cfg* cfg, const double* sums, int32_t K, int32_t* i_, float* macc,
                                 float* mu, float* Lpacked, float* lam, float* asc, double* cov) {
  const int d = cfg->d;
  const int64_t P = packed_size(d);
  const double N = sums[d + P + 1];
  const int32_t it = *i_;
  const int32_t itr = it + K;
  const int32_t n = orc_block_n(it, cfg->num_warmup, K);
  const float gamma = amh_lr_gamma(n, cfg->lr_decay);
  const float abar = (float)(sums[d + P] / N);
  const float maccn = *macc + (abar - *macc) / (float)n;
  const float lamn = *lam + gamma * (abar - cfg->target_accept_prob);
  for (int r = 0; r < d; ++r) mu[r] = mu[r] + gamma * (float)(sums[r] / N);
  const double g = (double)gamma;
  double* Sn = (double*)malloc(sizeof(double) * (size_t)P);
  float* A = (float*)malloc(sizeof(float) * (size_t)d * d);
  for (int k = 0; k < d; ++k)
    for (int r = k; r < d; ++r) {
      const int64_t o = col_off(d, k) + (r - k);
      const double a = (1.0 - g) * cov[o];
      const double b = g * (sums[d + o] / N);
      Sn[o] = a + b;
      A[r * d + k] = (float)Sn[o];
    }
  int ok = 1;
  for (int j = 0; j < d && ok; ++j) {
    const float piv = A[j * d + j];
    if (!amh_pivot_ok(piv)) { ok = 0; break; }
    const float y = amh_rsqrt_nr(piv); /* L_kk = piv y, column scaled by y (amh_math.h) */
    const float ljj = piv * y;
    for (int r = j + 1; r < d; ++r) A[r * d + j] = A[r * d + j] * y;
    A[j * d + j] = ljj;
    for (int k = j + 1; k < d; ++k)
      for (int r = k; r < d; ++r) A[r * d + k] = fmaf(-A[r * d + j], A[k * d + j], A[r * d + k]);
  }
  const float e0 = amh_expf(*lam), e1 = amh_expf(lamn);
  float part[ORC_BIG];
  for (int j = 0; j < d; ++j) {  /* column j's squared terms, rows j + t, big_sum order */
    float col[ORC_BIG];
    for (int t = 0; t < d; ++t) {
      col[t] = 0.0f;
      if (t < d - j) {
        const int r = j + t;
        const float lo = Lpacked[col_off(d, j) + (r - j)];
        const float ln = ok ? A[r * d + j] : lo;
        const float tt = (ln * e1) - (lo * e0);
        col[t] = tt * tt;
      }
    }
    part[j] = big_sum(col, d);
  }
  *asc = sqrtf(big_sum(part, d));
  if (ok) {
    for (int k = 0; k < d; ++k)
      for (int r = k; r < d; ++r) {
        const int64_t o = col_off(d, k) + (r - k);
        Lpacked[o] = A[r * d + k];
        cov[o] = Sn[o];
      }
  }
  free(Sn);
  free(A);
  *i_ = itr;
  *macc = maccn;
  *lam = lamn;
  return ok;
}

/* ================================================================= ASSS ==== */
/* Test hook (tests/test_asss.py): treat every tangent as zero-norm. */
int orc_test_zero_tangent = 0;
void orc_set_test_zero_tangent(int on) { orc_test_zero_tangent = on; }

/* asss.py:197-251 (ASSS.sample), kernel mirror of amh_asss.hip: the chain is
 * held as (U, dl) between the steps of one launch like chain_t; the factor
 * is written back as U diag(dl) if any step updated it, else verbatim.
 * Noise at stream position i: v_r = N(Philox(r, i, 0)[0]); v_d, u_t, th_0
 * from words 1-3 of Philox(0, i, 0); shrink step k: U(Philox(k, i, 1)[0]). */
static void asss_chain_step(const orc_cfg* cfg, chain_t* s, uint32_t k0, uint32_t k1, int adapt) {
  const int d = cfg->d;
  const int G = orc_gw(cfg);
  const uint32_t it = (uint32_t)s->i;
  const float sd = sqrtf((float)d);
  const float epsd = cfg->eps * sd;
  const float fd = (float)d;
  /* draws (asss.py:207, 219, 225, 60) */
  float v[ORC_DMAX];
  uint32_t w1 = 0, w2 = 0, w3 = 0;
  for (int r = 0; r < d; ++r) {
    const amh_u32x4 o = amh_philox4x32_10((uint32_t)r, it, 0u, AMH_TAG_ASSS, k0, k1);
    v[r] = amh_normal_from_bits(o.v[0]);
    if (r == 0) { w1 = o.v[1]; w2 = o.v[2]; w3 = o.v[3]; }
  }
  float vd = amh_normal_from_bits(w1);
  const float ut = amh_unif01_from_bits(w2);
  const float th0 = 6.28318548f * amh_unif01_from_bits(w3);
  /* y = S^-1 (x - mu), S = (L + eps I) sqrt(d): S_rj = U_rj e_j, S_rr = D_r */
  float e[ORC_DMAX], invD[ORC_DMAX], b[ORC_DMAX], y[ORC_DMAX];
  for (int r = 0; r < d; ++r) {
    e[r] = s->dl[r] * sd;
    invD[r] = 1.0f / ((s->dl[r] + cfg->eps) * sd);
    b[r] = s->z[r] - s->mu[r];
  }
  for (int j = 0; j < d; ++j) {
    const float yj = b[j] * invD[j];
    y[j] = yj;
    const float gj = yj * e[j];
    for (int r = 0; r < d; ++r) b[r] = fmaf(-s->U[r][j], gj, b[r]);
  }
  /* stereographic projection (asss.py:40-45) */
  float t[ORC_DMAX];
  for (int r = 0; r < G; ++r) t[r] = (r < d) ? y[r] * y[r] : 0.0f;
  const float ns = group_sum(t, G);
  const float den = ns + 1.0f;
  float zr[ORC_DMAX];
  for (int r = 0; r < d; ++r) zr[r] = (2.0f * y[r]) / den;
  const float zd = (ns - 1.0f) / den;
  /* v on the tangent space of z, normalised (asss.py:219-222) */
  for (int r = 0; r < G; ++r) t[r] = (r < d) ? v[r] * zr[r] : 0.0f;
  const float dot = group_sum(t, G) + (vd * zd);
  for (int r = 0; r < d; ++r) v[r] = fmaf(-dot, zr[r], v[r]); /* one rounding: no exact cancellation */
  vd = fmaf(-dot, zd, vd);
  for (int r = 0; r < G; ++r) t[r] = (r < d) ? v[r] * v[r] : 0.0f;
  float nv = sqrtf(group_sum(t, G) + (vd * vd));
  if (orc_test_zero_tangent) nv = 0.0f; /* test hook: the measure-zero case, on demand */
  /* |v| = 0 (every component rounded to 0; the reference's v / norm(v) is
   * NaN): theta = 0, the shrinkage's own fallback (asss.py:94) -- the state
   * is kept (re-projected) and the adaptation runs as usual */
  const int degen = !(nv > 0.0f);
  for (int r = 0; r < d; ++r) v[r] = degen ? 0.0f : v[r] / nv;
  vd = degen ? 0.0f : vd / nv;
  /* S z_1d and S v_1d */
  float Sz[ORC_DMAX], Sv[ORC_DMAX], hz[ORC_DMAX], hv[ORC_DMAX];
  for (int j = 0; j < d; ++j) { hz[j] = e[j] * zr[j]; hv[j] = e[j] * v[j]; }
  for (int r = 0; r < d; ++r) {
    float a4[4] = {0.0f, 0.0f, 0.0f, 0.0f}, c4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int j = 0; j < d; ++j) {
      a4[j & 3] = fmaf(s->U[r][j], hz[j], a4[j & 3]);
      c4[j & 3] = fmaf(s->U[r][j], hv[j], c4[j & 3]);
    }
    Sz[r] = ((a4[0] + a4[1]) + (a4[2] + a4[3])) + epsd * zr[r];
    Sv[r] = ((c4[0] + c4[1]) + (c4[2] + c4[3])) + epsd * v[r];
  }
  /* slice level at z (asss.py:216-217, 224-226) */
  float x0[ORC_DMAX], xt[ORC_DMAX];
  float om0;
  {
    const float zdt = (zd * 1.0f) + (vd * 0.0f);
    om0 = 1.0f - zdt;
    for (int r = 0; r < d; ++r) x0[r] = (((Sz[r] * 1.0f) + (Sv[r] * 0.0f)) / om0) + s->mu[r];
  }
  const float U0 = orc_potential1(cfg, x0);
  const float tpe = (U0 + fd * amh_logf(om0)) - amh_logf(ut);
  /* shrinkage (asss.py:59-96) */
  float th = th0, thmin = th0 - 6.28318548f, thmax = th0;
  int iter = 0;
  float ux;
  int cont;
  {
    float sn, cs;
    amh_sincosf(th, &sn, &cs);
    const float om = 1.0f - ((zd * cs) + (vd * sn));
    for (int r = 0; r < d; ++r) xt[r] = (((Sz[r] * cs) + (Sv[r] * sn)) / om) + s->mu[r];
    ux = orc_potential1(cfg, xt);
    float pt = ux + fd * amh_logf(om);
    if (amh_isnan(pt)) pt = INFINITY;
    cont = !degen && ((pt > tpe) || (om < cfg->eps));
  }
  while (cont) {
    if (th < 0.0f) thmin = th;
    if (th >= 0.0f) thmax = th;
    const amh_u32x4 o = amh_philox4x32_10((uint32_t)iter, it, 1u, AMH_TAG_ASSS, k0, k1);
    th = thmin + (thmax - thmin) * amh_unif01_from_bits(o.v[0]);
    float sn, cs;
    amh_sincosf(th, &sn, &cs);
    const float om = 1.0f - ((zd * cs) + (vd * sn));
    for (int r = 0; r < d; ++r) xt[r] = (((Sz[r] * cs) + (Sv[r] * sn)) / om) + s->mu[r];
    ux = orc_potential1(cfg, xt);
    float pt = ux + fd * amh_logf(om);
    if (amh_isnan(pt)) pt = INFINITY;
    iter += 1;
    cont = (iter < 50) && ((pt > tpe) || (om < cfg->eps));
  }
  const int capped = degen || iter >= 50;
  float xn[ORC_DMAX];
  for (int r = 0; r < d; ++r) xn[r] = capped ? x0[r] : xt[r];
  float pen = capped ? U0 : ux;
  if (amh_isnan(pen)) pen = INFINITY;
  if (!adapt) { /* frozen kernel (sample_Pnx) */
    for (int r = 0; r < d; ++r) s->z[r] = xn[r];
    s->pe = pen;
    return;
  }
  /* adaptation (asss.py:237-251) */
  const int32_t itr = s->i + 1;
  const int32_t n = (s->i < cfg->num_warmup) ? itr : itr - cfg->num_warmup;
  const float gamma = amh_lr_gamma(n, cfg->lr_decay);
  float delta[ORC_DMAX], mun[ORC_DMAX];
  for (int r = 0; r < G; ++r) t[r] = 0.0f;
  for (int r = 0; r < d; ++r) {
    delta[r] = xn[r] - s->mu[r];
    mun[r] = s->mu[r] + gamma * delta[r];
    const float dm = mun[r] - s->mu[r];
    t[r] = dm * dm;
  }
  const float locd = sqrtf(group_sum(t, G));
  const float sq = sqrtf(1.0f - gamma);
  float Dg[ORC_DMAX], one[ORC_DMAX];
  for (int j = 0; j < d; ++j) {
    const float ajj = sq * s->dl[j];
    Dg[j] = ajj * ajj;
    one[j] = (amh_isfinite(ajj) && ajj != 0.0f) ? 1.0f : NAN;
  }
  float w[ORC_DMAX], ws[ORC_DMAX];
  for (int r = 0; r < d; ++r) w[r] = delta[r];
  for (int j = 0; j < d; ++j) {
    const float wj = w[j];
    ws[j] = wj;
    for (int r = 0; r < d; ++r) w[r] = fmaf(-wj, s->U[r][j], w[r]);
  }
  float tsc[ORC_DMAX], bsc[ORC_DMAX], cc[ORC_DMAX], qq[ORC_DMAX], gw2[ORC_DMAX];
  for (int r = 0; r < G; ++r) {
    gw2[r] = (r < d) ? gamma * (ws[r] * ws[r]) : 0.0f;
    tsc[r] = (r < d) ? gw2[r] / Dg[r] : 0.0f;
  }
  group_excl_scan(tsc, bsc, G);
  int revert = 0;
  for (int r = 0; r < d; ++r) {
    const float bb = 1.0f + bsc[r];
    const float g2 = (bb * Dg[r]) + gw2[r];
    const float dn = g2 / bb;
    cc[r] = (gamma * ws[r]) / g2;
    qq[r] = sqrtf(dn);
    revert |= amh_isnan(fmaf(cc[r], 0.0f, one[r]) * qq[r]);
  }
  float sdiff = 0.0f;
  if (!revert) {
    float ac[ORC_DMAX], bc[ORC_DMAX], s4[ORC_DMAX][4];
    for (int r = 0; r < d; ++r) {
      ac[r] = qq[r] - s->dl[r];
      bc[r] = cc[r] * qq[r];
      s4[r][0] = s4[r][1] = s4[r][2] = s4[r][3] = 0.0f;
      w[r] = delta[r];
    }
    for (int j = 0; j < d; ++j)
      for (int r = 0; r < d; ++r) {
        const float uo = s->U[r][j];
        w[r] = fmaf(-ws[j], uo, w[r]);
        const float un = fmaf(cc[j], w[r], uo);
        const float tt = fmaf(uo, ac[j], bc[j] * w[r]);
        s4[r][j & 3] = fmaf(tt, tt, s4[r][j & 3]);
        s->U[r][j] = un;
      }
    for (int r = 0; r < G; ++r) t[r] = (r < d) ? (s4[r][0] + s4[r][1]) + (s4[r][2] + s4[r][3]) : 0.0f;
    sdiff = sqrtf(group_sum(t, G));
    for (int r = 0; r < d; ++r) s->dl[r] = qq[r];
    s->updated = 1;
  }
  s->asc = locd + sdiff;
  s->i = itr;
  for (int r = 0; r < d; ++r) { s->z[r] = xn[r]; s->mu[r] = mun[r]; }
  s->pe = pen;
}

/* n_steps ASSS transitions of chains [0, C) in place (one kernel launch);
 * collect_z [n_steps][C][d] / collect_pe [n_steps][C] nullable. */
/* ASSS for large dimensions (asss.py:192-269; 64 < d <= 256,
 * the dense Gaussian; round 5, passes folded in round 6).  Kernel mirror of
 * amh_big.hip asss_big_chain: one wave per chain, lane l owns rows 64 s + l,
 * the factor streamed column by column (the large-d ARWMH path's layout),
 * two passes over it per transition:
 *   A  one column sweep, four accumulators per row (U = L / diag(L), unit
 *      diagonal; S = (L + eps I) sqrt(d) = U diag(e) + eps sqrt(d) I, e =
 *      dl sqrt(d)):
 *        y = S^-1 (x - mu) (asss.py:214, :33-45): y_j = b_j / D_j,
 *          b_r = fmaf(-U_rj, y_j e_j, b_r)
 *        av = U (e * v)  (S v_raw = av + eps sqrt(d) v_raw)
 *        wy = U^-1 y     (wy_j = y_j - ty_j, ty_r = fmaf(U_rj, wy_j, ty_r))
 *        wv = U^-1 v_raw (wv_j = v_j - tv_j, tv_r = fmaf(U_rj, wv_j, tv_r))
 *      Since S y = x - mu, S z = 2 (x - mu) / den and S v = (S v_raw - dot
 *      S z) / |v|; U^-1 z and U^-1 v follow the same way from wy, wv.  The
 *      round-5 passes B (S z, S v) and C (w = U^-1 delta) are gone: with q =
 *      (z c + v s) / om at the accepted angle, delta = S q, so U^-1 delta =
 *      sqrt(d) (dl q + eps U^-1 q) -- the same quantities up to rounding.
 *   the potential along the slice circle: with a = S z, b = S v, g = mu - m,
 *      D(th) = (a c + b s) / om + g and Y(th) = (Pa c + Pb s) / om + Pg, where
 *      Pa, Pb, Pg are fmaf chains over k of P[k][r] (once per transition);
 *      U(th) = 0.5 big_sum(D Y) + c0 -- each shrink step is O(d).  The stored
 *      potential is this U at the accepted angle (the model potential of the
 *      stored x' up to rounding, not re-evaluated at it)
 *   D  the rank-one update as the large-d ARWMH step pass with a_j = q_j -
 *      dl_j, b_j = c_j q_j (no step size), sdiff = sqrt(big_sum(row sums)).
 * Draws as the d <= 64 kernel (Philox(r, i, 0, TAG_ASSS)).  as_change =
 * ||mu' - mu|| + ||L' - L||_F (asss.py:259-267). */
static void asss_step_big1(const orc_cfg* cfg, bigchain_t* s, int64_t c, int32_t* i_, float* z, float* pe,
                           float* mu, float* L, float* asc, const uint32_t* keys, int adapt,
                           const float* Lshared, const float* mushared) {
  const int d = cfg->d;
  const int64_t P = packed_size(d);
  const float* Lc = adapt ? L + c * P : Lshared;
  const float* mc = adapt ? mu + c * d : mushared;
  const float* m = cfg->data;
  const float* Pm = cfg->data + d;
  const float c0 = cfg->data[d + d * d];
  for (int r = 0; r < d; ++r) {
    s->dl[r] = Lc[col_off(d, r)];
    s->inv[r] = (amh_isfinite(s->dl[r]) && s->dl[r] != 0.0f) ? 1.0f / s->dl[r] : 0.0f;
    s->z[r] = z[c * d + r];
    s->mu[r] = mc[r];
  }
  for (int j = 0; j < d; ++j)
    for (int r = j + 1; r < d; ++r) s->U[r][j] = Lc[col_off(d, j) + (r - j)] * s->inv[j];
  const uint32_t it = (uint32_t)i_[c];
  const uint32_t k0 = keys[2 * c], k1 = keys[2 * c + 1];
  const float sd = sqrtf((float)d);
  const float epsd = cfg->eps * sd;
  const float fd = (float)d;
  /* draws (asss.py:207, 219, 225, 60) */
  float v[ORC_BIG];
  for (int r = 0; r < d; ++r) v[r] = amh_normal_from_bits(amh_philox4x32_10((uint32_t)r, it, 0u, AMH_TAG_ASSS, k0, k1).v[0]);
  const amh_u32x4 o0 = amh_philox4x32_10(0u, it, 0u, AMH_TAG_ASSS, k0, k1);
  float vd = amh_normal_from_bits(o0.v[1]);
  const float ut = amh_unif01_from_bits(o0.v[2]);
  const float th0 = 6.28318548f * amh_unif01_from_bits(o0.v[3]);
  /* pass A */
  float e[ORC_BIG], invD[ORC_BIG], b[ORC_BIG], y[ORC_BIG], t[ORC_BIG];
  float hv[ORC_BIG], av[ORC_BIG], ty[ORC_BIG], tv[ORC_BIG], wy[ORC_BIG], wv[ORC_BIG];
  for (int r = 0; r < d; ++r) {
    e[r] = s->dl[r] * sd;
    invD[r] = 1.0f / ((s->dl[r] + cfg->eps) * sd);
    b[r] = s->z[r] - s->mu[r];
    hv[r] = e[r] * v[r];
    av[r] = ty[r] = tv[r] = 0.0f;
  }
  for (int j = 0; j < d; ++j) {
    const float yl = b[j] * invD[j];
    y[j] = yl;
    const float g = yl * e[j];
    av[j] = fmaf(1.0f, hv[j], av[j]);
    wy[j] = yl - ty[j];
    wv[j] = v[j] - tv[j];
    for (int r = j + 1; r < d; ++r) {
      const float uo = s->U[r][j];
      b[r] = fmaf(-uo, g, b[r]);
      av[r] = fmaf(uo, hv[j], av[r]);
      ty[r] = fmaf(uo, wy[j], ty[r]);
      tv[r] = fmaf(uo, wv[j], tv[r]);
    }
  }
  float svr[ORC_BIG];
  for (int r = 0; r < d; ++r) svr[r] = av[r] + epsd * v[r]; /* S v_raw */
  for (int r = 0; r < d; ++r) t[r] = y[r] * y[r];
  const float ns = big_sum(t, d);
  const float den = ns + 1.0f;
  float zr[ORC_BIG];
  for (int r = 0; r < d; ++r) zr[r] = (2.0f * y[r]) / den;
  const float zd = (ns - 1.0f) / den;
  /* tangent v (the d <= 64 kernel's rule for |v| = 0) */
  for (int r = 0; r < d; ++r) t[r] = v[r] * zr[r];
  const float dot = big_sum(t, d) + (vd * zd);
  for (int r = 0; r < d; ++r) v[r] = fmaf(-dot, zr[r], v[r]);
  vd = fmaf(-dot, zd, vd);
  for (int r = 0; r < d; ++r) t[r] = v[r] * v[r];
  float nv = sqrtf(big_sum(t, d) + (vd * vd));
  if (orc_test_zero_tangent) nv = 0.0f;
  const int degen = !(nv > 0.0f);
  for (int r = 0; r < d; ++r) v[r] = degen ? 0.0f : v[r] / nv;
  vd = degen ? 0.0f : vd / nv;
  float Sz[ORC_BIG], Sv[ORC_BIG], gm[ORC_BIG], Pa[ORC_BIG], Pb[ORC_BIG], Pg[ORC_BIG];
  float Wz[ORC_BIG], Wv[ORC_BIG];
  for (int r = 0; r < d; ++r) {
    Sz[r] = (2.0f * (s->z[r] - s->mu[r])) / den; /* S z = 2 S y / den, S y = x - mu */
    Sv[r] = degen ? 0.0f : fmaf(-dot, Sz[r], svr[r]) / nv;
    Wz[r] = (2.0f * wy[r]) / den; /* U^-1 z */
    Wv[r] = degen ? 0.0f : fmaf(-dot, Wz[r], wv[r]) / nv;
    gm[r] = s->mu[r] - m[r];
    Pa[r] = Pb[r] = Pg[r] = 0.0f;
  }
  for (int k = 0; k < d; ++k)
    for (int r = 0; r < d; ++r) {
      const float pk = Pm[k * d + r];
      Pa[r] = fmaf(pk, Sz[k], Pa[r]);
      Pb[r] = fmaf(pk, Sv[k], Pb[r]);
      Pg[r] = fmaf(pk, gm[k], Pg[r]);
    }
  /* the point at angle (cs, sn): potential and x */
  float xt[ORC_BIG], x0[ORC_BIG];
#define ASSS_BIG_EVAL(CS, SN, XOUT, OM, UOUT)                                   \
  do {                                                                         \
    OM = 1.0f - ((zd * (CS)) + (vd * (SN)));                                   \
    for (int r = 0; r < d; ++r) {                                              \
      const float num = (Sz[r] * (CS)) + (Sv[r] * (SN));                       \
      const float Dr = (num / OM) + gm[r];                                     \
      const float Yr = (((Pa[r] * (CS)) + (Pb[r] * (SN))) / OM) + Pg[r];      \
      t[r] = Dr * Yr;                                                          \
      XOUT[r] = (num / OM) + s->mu[r];                                         \
    }                                                                          \
    UOUT = (0.5f * big_sum(t, d)) + c0;                                        \
  } while (0)
  float om0, U0;
  ASSS_BIG_EVAL(1.0f, 0.0f, x0, om0, U0);
  const float tpe = (U0 + fd * amh_logf(om0)) - amh_logf(ut);
  float th = th0, thmin = th0 - 6.28318548f, thmax = th0;
  int iter = 0;
  float ux;
  int cont;
  float cst, snt, omt; /* the angle of xt */
  {
    float sn, cs, om;
    amh_sincosf(th, &sn, &cs);
    ASSS_BIG_EVAL(cs, sn, xt, om, ux);
    cst = cs;
    snt = sn;
    omt = om;
    float pt = ux + fd * amh_logf(om);
    if (amh_isnan(pt)) pt = INFINITY;
    cont = !degen && ((pt > tpe) || (om < cfg->eps));
  }
  while (cont) {
    if (th < 0.0f) thmin = th;
    if (th >= 0.0f) thmax = th;
    const amh_u32x4 o = amh_philox4x32_10((uint32_t)iter, it, 1u, AMH_TAG_ASSS, k0, k1);
    th = thmin + (thmax - thmin) * amh_unif01_from_bits(o.v[0]);
    float sn, cs, om;
    amh_sincosf(th, &sn, &cs);
    ASSS_BIG_EVAL(cs, sn, xt, om, ux);
    cst = cs;
    snt = sn;
    omt = om;
    float pt = ux + fd * amh_logf(om);
    if (amh_isnan(pt)) pt = INFINITY;
    iter += 1;
    cont = (iter < 50) && ((pt > tpe) || (om < cfg->eps));
  }
#undef ASSS_BIG_EVAL
  const int capped = degen || iter >= 50;
  if (capped) { /* theta = 0 (asss.py:94) */
    cst = 1.0f;
    snt = 0.0f;
    omt = om0;
  }
  float xn[ORC_BIG];
  for (int r = 0; r < d; ++r) xn[r] = capped ? x0[r] : xt[r];
  float pen = capped ? U0 : ux;
  if (amh_isnan(pen)) pen = INFINITY;
  if (!adapt) {
    for (int r = 0; r < d; ++r) z[c * d + r] = xn[r];
    pe[c] = pen;
    return;
  }
  /* adaptation (asss.py:246-267) */
  const int32_t itr = (int32_t)it + 1;
  const int32_t n = ((int32_t)it < cfg->num_warmup) ? itr : itr - cfg->num_warmup;
  const float gamma = amh_lr_gamma(n, cfg->lr_decay);
  float delta[ORC_BIG], mun[ORC_BIG], Dg[ORC_BIG], one[ORC_BIG], ws[ORC_BIG], gw2[ORC_BIG];
  float bsc[ORC_BIG], cc[ORC_BIG], qq[ORC_BIG], sacc[ORC_BIG];
  const float sq = sqrtf(1.0f - gamma);
  for (int r = 0; r < d; ++r) {
    delta[r] = xn[r] - s->mu[r];
    mun[r] = s->mu[r] + gamma * delta[r];
    const float dm = mun[r] - s->mu[r];
    t[r] = dm * dm;
    const float ajj = sq * s->dl[r];
    Dg[r] = ajj * ajj;
    one[r] = (amh_isfinite(ajj) && ajj != 0.0f) ? 1.0f : NAN;
  }
  const float locd = sqrtf(big_sum(t, d));
  /* w = U^-1 delta = sqrt(d) (dl q + eps U^-1 q), q = (z c + v s) / om */
  for (int r = 0; r < d; ++r) {
    const float q = ((zr[r] * cst) + (v[r] * snt)) / omt;
    const float wq = ((Wz[r] * cst) + (Wv[r] * snt)) / omt;
    ws[r] = ((s->dl[r] * q) + (cfg->eps * wq)) * sd;
  }
  for (int r = 0; r < d; ++r) {
    gw2[r] = gamma * (ws[r] * ws[r]);
    t[r] = gw2[r] / Dg[r];
  }
  big_excl_scan(t, bsc, d);
  int revert = 0;
  for (int r = 0; r < d; ++r) {
    const float bq = 1.0f + bsc[r];
    const float g2 = (bq * Dg[r]) + gw2[r];
    const float dn = g2 / bq;
    cc[r] = (gamma * ws[r]) / g2;
    qq[r] = sqrtf(dn);
    revert |= amh_isnan(fmaf(cc[r], 0.0f, one[r]) * qq[r]);
  }
  float sdiff = 0.0f;
  if (!revert) {
    /* pass D */
    float* Lw = L + c * P;
    float ac[ORC_BIG], bc[ORC_BIG], sv[ORC_BIG];
    for (int r = 0; r < d; ++r) {
      ac[r] = qq[r] - s->dl[r];
      bc[r] = cc[r] * qq[r];
      sv[r] = 0.0f;
      sacc[r] = 0.0f;
    }
    for (int j = 0; j < d; ++j) {
      {
        const float tt = fmaf(1.0f, ac[j], bc[j] * 0.0f);
        sacc[j] = fmaf(tt, tt, sacc[j]);
        Lw[col_off(d, j)] = 1.0f * qq[j];
      }
      for (int r = j + 1; r < d; ++r) {
        const float uo = s->U[r][j];
        sv[r] = fmaf(uo, ws[j], sv[r]);
        const float w = delta[r] - sv[r];
        const float un = fmaf(cc[j], w, uo);
        const float tt = fmaf(uo, ac[j], bc[j] * w);
        sacc[r] = fmaf(tt, tt, sacc[r]);
        Lw[col_off(d, j) + (r - j)] = un * qq[j];
      }
    }
    sdiff = sqrtf(big_sum(sacc, d));
  }
  asc[c] = locd + sdiff;
  for (int r = 0; r < d; ++r) {
    z[c * d + r] = xn[r];
    mu[c * d + r] = mun[r];
  }
  i_[c] = itr;
  pe[c] = pen;
}

static int orc_asss_big(const orc_cfg* cfg) {
  return cfg->model_id == ORC_GAUSSIAN && cfg->d > ORC_DMAX && cfg->d <= ORC_BIG;
}

void orc_asss_step(const orc_cfg* cfg, int64_t C, int32_t n_steps, int32_t* i_, float* z, float* pe, float* mu,
                   float* L, float* asc, const uint32_t* keys, float* collect_z, float* collect_pe) {
  const int d = cfg->d;
  if (orc_asss_big(cfg)) {
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t c = 0; c < C; ++c) {
      bigchain_t* s = (bigchain_t*)malloc(sizeof(bigchain_t));
      for (int32_t t = 0; t < n_steps; ++t) {
        asss_step_big1(cfg, s, c, i_, z, pe, mu, L, asc, keys, 1, NULL, NULL);
        if (collect_z)
          for (int r = 0; r < d; ++r) collect_z[((int64_t)t * C + c) * d + r] = z[c * d + r];
        if (collect_pe) collect_pe[(int64_t)t * C + c] = pe[c];
      }
      free(s);
    }
    return;
  }
  if (d > ORC_DMAX) return;
#pragma omp parallel for schedule(dynamic, 16)
  for (int64_t c = 0; c < C; ++c) {
    chain_t* s = (chain_t*)malloc(sizeof(chain_t));
    const float* Lc = L + c * packed_size(d);
    float inv[ORC_DMAX];
    for (int r = 0; r < d; ++r) {
      s->dl[r] = Lc[col_off(d, r)];
      inv[r] = (amh_isfinite(s->dl[r]) && s->dl[r] != 0.0f) ? 1.0f / s->dl[r] : 0.0f;
    }
    for (int r = 0; r < d; ++r)
      for (int j = 0; j < d; ++j) {
        const float x = (r > j) ? Lc[col_off(d, j) + (r - j)] : 0.0f;
        s->U[r][j] = (r == j) ? 1.0f : x * inv[j];
      }
    for (int r = 0; r < d; ++r) { s->z[r] = z[c * d + r]; s->mu[r] = mu[c * d + r]; }
    s->i = i_[c];
    s->pe = pe[c];
    s->asc = asc[c];
    s->updated = 0;
    for (int32_t t = 0; t < n_steps; ++t) {
      asss_chain_step(cfg, s, keys[2 * c], keys[2 * c + 1], 1);
      if (collect_z)
        for (int r = 0; r < d; ++r) collect_z[((int64_t)t * C + c) * d + r] = s->z[r];
      if (collect_pe) collect_pe[(int64_t)t * C + c] = s->pe;
    }
    if (s->updated) {
      float* Lw = L + c * packed_size(d);
      for (int j = 0; j < d; ++j)
        for (int r = j; r < d; ++r) Lw[col_off(d, j) + (r - j)] = s->U[r][j] * s->dl[j];
    }
    for (int r = 0; r < d; ++r) { z[c * d + r] = s->z[r]; mu[c * d + r] = s->mu[r]; }
    i_[c] = s->i;
    pe[c] = s->pe;
    asc[c] = s->asc;
    free(s);
  }
}

/* asss.py:271-303 (ASSS.sample_Pnx), mirror of asss_pnx_kernel: chain
 * c = (p, s) starts at x[p] with key split(key, C)[c], frozen shared
 * (loc, L); transition t at stream position t. */
void orc_asss_sample_pnx(const orc_cfg* cfg, const uint32_t* key, const float* x, int64_t n_points,
                         int64_t n_samples, const float* loc, const float* Lpacked, int32_t n, float* out) {
  const int d = cfg->d;
  const int64_t C = n_points * n_samples;
  if (orc_asss_big(cfg)) { /* the frozen large-d transition (asss_step_big1, adapt = 0) */
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t c = 0; c < C; ++c) {
      bigchain_t* s = (bigchain_t*)malloc(sizeof(bigchain_t));
      const int64_t p = c / n_samples;
      const amh_u32x4 kk = amh_philox4x32_10((uint32_t)c, (uint32_t)((uint64_t)c >> 32), 0u, AMH_TAG_SPLIT, key[0],
                                             key[1]);
      const uint32_t k2[2] = {kk.v[0], kk.v[1]};
      float zc[ORC_BIG], pe1 = 0.0f;
      for (int r = 0; r < d; ++r) zc[r] = x[p * d + r];
      for (int32_t t = 0; t < n; ++t) {
        int32_t i1 = t;
        asss_step_big1(cfg, s, 0, &i1, zc, &pe1, NULL, NULL, NULL, k2, 0, Lpacked, loc);
      }
      for (int r = 0; r < d; ++r) out[c * d + r] = zc[r];
      free(s);
    }
    return;
  }
#pragma omp parallel for schedule(dynamic, 64)
  for (int64_t c = 0; c < C; ++c) {
    chain_t* s = (chain_t*)malloc(sizeof(chain_t));
    float inv[ORC_DMAX];
    for (int r = 0; r < d; ++r) {
      s->dl[r] = Lpacked[col_off(d, r)];
      inv[r] = (amh_isfinite(s->dl[r]) && s->dl[r] != 0.0f) ? 1.0f / s->dl[r] : 0.0f;
    }
    for (int r = 0; r < d; ++r)
      for (int j = 0; j < d; ++j) {
        const float xx = (r > j) ? Lpacked[col_off(d, j) + (r - j)] : 0.0f;
        s->U[r][j] = (r == j) ? 1.0f : xx * inv[j];
      }
    const int64_t p = c / n_samples;
    const amh_u32x4 kk = amh_philox4x32_10((uint32_t)c, (uint32_t)((uint64_t)c >> 32), 0u, AMH_TAG_SPLIT, key[0],
                                           key[1]);
    for (int r = 0; r < d; ++r) { s->z[r] = x[p * d + r]; s->mu[r] = loc[r]; }
    s->pe = orc_potential1(cfg, s->z);
    for (int32_t t = 0; t < n; ++t) {
      s->i = t;
      asss_chain_step(cfg, s, kk.v[0], kk.v[1], 0);
    }
    for (int r = 0; r < d; ++r) out[c * d + r] = s->z[r];
    free(s);
  }
}
