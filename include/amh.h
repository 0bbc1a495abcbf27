/*
 * amh.h -- C ABI of libamh.so, the MI355X (gfx950) adaptive random-walk
 * Metropolis-Hastings engine.
 *
 * The reference (savelovme/adaptive-mcmc) has no FFI: its boundary is the
 * NumPyro MCMCKernel object python/kernels/arwmh.py:31.  Each entry point
 * below replaces one method of that object for a whole batch of chains; the
 * Python mirror (adaptive-mcmc_amd/kernels_amd/arwmh.py, _lib.py) binds them with ctypes.
 *
 *   amh_create / amh_bind_model   ARWMH.__init__        arwmh.py:43-78
 *                                 + model plug-in        arwmh.py:109-116
 *   amh_init                      ARWMH.init            arwmh.py:84-138
 *   amh_step                      ARWMH.sample          arwmh.py:140-207
 *                                 (n_steps > 1: numpyro fori_collect over
 *                                 sample, kernel_utils.py:29-33)
 *   amh_potential                 potential_fn          arwmh.py:121,170
 *   amh_sample_pnx                ARWMH.sample_Pnx      arwmh.py:230-270
 *   amh_pooled_*                  build-defined pooled-covariance mode
 *                                 (SURVEY.md §8(e)); ARWMH.sample's
 *                                 adaptation (arwmh.py:180-197) driven by
 *                                 the statistics of all chains
 *
 * Conventions
 *   - Every pointer in amh_state / model data / outputs is a DEVICE pointer
 *     owned by the caller (PyTorch allocates them).  The library never frees
 *     caller memory.
 *   - Layout is chain-major: z/loc [C][d], scale [C][d(d+1)/2] (lower
 *     triangle packed column by column: column j holds rows j..d-1),
 *     scalars [C], rng_key [C][2] uint32.
 *   - All work is enqueued on `stream` (a hipStream_t; NULL = default
 *     stream).  No call synchronises the device (amh_destroy's hipFree
 *     calls wait for outstanding device work as HIP defines).
 *   - Return value: 0 on success, a negative AMH_E* code on failure;
 *     amh_last_error(h) describes the failure (thread-local when h is NULL).
 *   - One handle per device; handles are not shared between host threads.
 */
#ifndef AMH_H
#define AMH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AMH_ABI_VERSION 1

enum {
  AMH_OK = 0,
  AMH_EINVAL = -1,   /* bad argument (shape, pointer, unsupported d)     */
  AMH_ENOMODEL = -2, /* amh_step/amh_init before amh_bind_model          */
  AMH_EHIP = -3,     /* HIP runtime error (message in amh_last_error)    */
  AMH_ENOMEM = -4
};

/* Model plug-in registry (PosteriorDB models of the reference + Gaussian). */
enum {
  AMH_MODEL_GAUSSIAN = 1,      /* data: [m (d) | P (d*d) | c0]; U = .5 (x-m)'P(x-m) + c0   */
  AMH_MODEL_EIGHT_SCHOOLS = 2, /* data: [y (J) | sigma (J) | log sigma (J)], d = J + 2     */
  AMH_MODEL_KIDIQ = 3,         /* data: [kid (N) | mom_hs (N) | mom_iq (N)], d = 4          */
  AMH_MODEL_DIAMONDS = 4,      /* data: [Xc (N*Kc) | Y (N)], d = Kc + 2, Kc = K - 1        */
  AMH_MODEL_DIAMONDS_SS = 5,   /* diamonds through float64 sufficient statistics, passed as
                                  2 floats each: [N, ybar, A, sT, t (Kc), sx (Kc), Gm (Kc*Kc)],
                                  n_data = 2 (4 + 2 Kc + Kc^2), iparams {N, K}, 3 <= d <= 32 */
  AMH_MODEL_MIXTURE = 6,       /* K-component univariate normal mixture on every coordinate
                                  (asumptions_check.ipynb cells 61-62): data [c (K) | m (K) |
                                  s (K)], c_k = log w_k - log(sqrt(2 pi) s_k); iparams {K},
                                  1 <= K <= 8, n_data = 3 K, 1 <= d <= 16 */
  AMH_MODEL_EXTERNAL = 7       /* the caller's potential (arwmh.py:69-70 potential_fn, any
                                  callable): the library never evaluates U; amh_init leaves
                                  pe0 = 0 for the caller to fill, transitions run through
                                  amh_propose / amh_step_external; data ignored (non-null,
                                  n_data >= 0, no iparams), 1 <= d <= 256 */
};

typedef struct amh_config {
  int32_t dim;                /* d, flat unconstrained dimension: 1..64 for
                                 every model; 64 < d <= 256 for the dense
                                 Gaussian (regime A, sample_Pnx and ASSS; the
                                 pooled mode needs d % 32 == 0) */
  int32_t num_warmup;         /* W (ARWMH.init's num_warmup)                 */
  float lr_decay;             /* a: gamma_n = 1 / n^a          (default 2/3) */
  float target_accept_prob;   /*                               (default .234)*/
  float eps;                  /* eps added to the scaled factor (default 1e-6)*/
  int32_t reserved[3];
} amh_config;

typedef struct amh_state {
  int32_t* i;                 /* [C]      iteration                          */
  float* z;                   /* [C][d]   current point (unconstrained)      */
  float* potential_energy;    /* [C]                                          */
  float* mean_accept_prob;    /* [C]                                          */
  float* loc;                 /* [C][d]   adapt_state.loc                    */
  float* scale;               /* [C][P]   adapt_state.scale, packed lower    */
  float* log_step_size;       /* [C]      adapt_state.log_step_size          */
  float* as_change;           /* [C]                                          */
  uint32_t* rng_key;          /* [C][2]   per-chain Philox key               */
} amh_state;

/* Optional per-launch collection (numpyro fori_collect / extra_fields). */
typedef struct amh_collect {
  float* z;                   /* [n_keep][C][d] or NULL                      */
  float* potential_energy;    /* [n_keep][C] or NULL                         */
  int32_t* accept_count;      /* [C] incremented per accepted step, or NULL  */
  int32_t thinning;           /* keep every `thinning`-th step (>= 1)        */
} amh_collect;

typedef struct amh_handle amh_handle;

int amh_version(void);
const char* amh_last_error(const amh_handle* h);

/* arwmh.py:43-78 (constructor config). */
int amh_create(const amh_config* cfg, int device, amh_handle** out);
int amh_destroy(amh_handle* h);

/* A device-side failure flagged by a completed launch of this handle (the
 * d = 64 pooled update's bounded wait running out: that update kept the shared
 * factor, so the run no longer follows the bit spec).  Returns AMH_EHIP with
 * the message in amh_last_error and clears the flag, else AMH_OK.  Reads a
 * host-mapped word, no synchronisation: a launch still in flight is covered
 * by a call after the caller has synchronised its stream (amh_destroy reads
 * the flag as it stands, without synchronising, and returns the same code
 * when it is set).  No counterpart in the reference,
 * whose guards (arwmh.py:171, :191) cannot fail this way. */
int amh_check_device(amh_handle* h);

/* Model plug-in (arwmh.py:109-116 / the scripts' numpyro models).
 * data: device pointer, n_data floats; iparams model-specific:
 *   GAUSSIAN: none.  EIGHT_SCHOOLS: {J}.  KIDIQ: {N}.  DIAMONDS: {N, K}. */
int amh_bind_model(amh_handle* h, int32_t model_id, const float* data, int64_t n_data,
                   const int64_t* iparams, int32_t n_iparams);

/* arwmh.py:84-138 for chains [chain_offset, chain_offset + C) of the run
 * keyed by key[2] (host memory).  init_z: device [C][d] starting points, or
 * NULL for init_to_uniform (U(-2, 2) per coordinate).  Writes *out. */
int amh_init(amh_handle* h, const uint32_t key[2], int64_t chain_offset, int64_t num_chains,
             const float* init_z, const amh_state* out, void* stream);

/* arwmh.py:140-207 applied n_steps times to every chain.  `in` and `out` may
 * alias (in-place update).  collect may be NULL. */
int amh_step(amh_handle* h, int64_t num_chains, const amh_state* in, const amh_state* out,
             int32_t n_steps, const amh_collect* collect, void* stream);

/* amh_step with flags (64 < d <= 256 and the literal diamonds model's split
 * transition; other shapes ignore them).  The step pass of those paths forms
 * the next transition's proposal while it streams L' out (so the factor is
 * read once per transition); AMH_STEP_KEEP_PROPOSAL keeps the one after the last step in
 * the handle, and AMH_STEP_PROPOSAL_READY tells the next call that its `in` is
 * that unchanged output (same chains), so its propose pass is skipped.  The
 * handle drops a kept proposal whenever its scratch is used otherwise, and
 * READY without one falls back to the propose pass.  Same bits either way. */
enum { AMH_STEP_PROPOSAL_READY = 1, AMH_STEP_KEEP_PROPOSAL = 2 };
int amh_step_chained(amh_handle* h, int64_t num_chains, const amh_state* in, const amh_state* out,
                     int32_t n_steps, const amh_collect* collect, int32_t flags, void* stream);

/* AMH_MODEL_EXTERNAL: ARWMH.sample (arwmh.py:140-207) with U evaluated by the
 * caller between two launches.  amh_propose writes every chain's proposal
 * z' = z + (L e^lam + eps I) xi (arwmh.py:162-167, the step stream at in.i)
 * to zprop[C][d].  amh_step_external then runs the rest of the transition
 * (accept with pe_prop[C] = U(zprop), NaN -> +inf as arwmh.py:171; the
 * schedule, mean, rank-one update and step size) from `in` to `out`; with
 * zprop_next non-null it also writes the NEXT transition's proposals (from
 * `out`, in the same pass over the factor; zprop_next may equal zprop), so a
 * chain of transitions is propose once, then {U; step_external}.  collect:
 * z / potential_energy after the transition (thinning 1) and accept_count.
 * `in` and `out` may alias.  Same bits as the fused kernels with the same U.
 * d > 64: the solves of the proposals stay in the handle, so amh_step_external
 * takes only the state the last amh_propose / amh_step_external formed them
 * from, and zprop_next must be null or zprop (AMH_EINVAL otherwise). */
int amh_propose(amh_handle* h, int64_t num_chains, const amh_state* in, float* zprop, void* stream);
int amh_step_external(amh_handle* h, int64_t num_chains, const amh_state* in, const amh_state* out,
                      const float* zprop, const float* pe_prop, float* zprop_next, const amh_collect* collect,
                      void* stream);

/* ARWMH.sample_Pnx (arwmh.py:230-270) with AMH_MODEL_EXTERNAL, d <= 64: step
 * t of every chain c (key split(key)[c], as amh_sample_pnx) in two calls
 * around the caller's U.  The caller starts z[C][d] at the points (chain
 * p * n_samples + s at x[p]) and pe[C] = U(z); per step t = 0..n-1:
 * amh_pnx_propose writes zprop from z and the shared (scale_packed,
 * log_step_size), the caller evaluates pe_prop = U(zprop), amh_pnx_accept
 * moves accepted chains (u < min(1, exp(pe - pe_prop)), NaN -> +inf) into z,
 * pe.  Same bits as amh_sample_pnx given the same U. */
int amh_pnx_propose(amh_handle* h, const uint32_t key[2], const float* z, int64_t num_chains,
                    const float* scale_packed, float log_step_size, int32_t t, float* zprop, void* stream);
int amh_pnx_accept(amh_handle* h, const uint32_t key[2], float* z, float* pe, int64_t num_chains,
                   const float* zprop, const float* pe_prop, int32_t t, void* stream);

/* potential_fn(z) for n points: pe[n] from z[n][d] (arwmh.py:121). */
int amh_potential(amh_handle* h, const float* z, float* pe, int64_t n, void* stream);

/* arwmh.py:230-270.  x: device [n_points][d]; adapt state (loc[d],
 * scale_packed[P], log_step_size) shared by every chain; out: device
 * [n_points][n_samples][d].  key[2] in host memory. */
int amh_sample_pnx(amh_handle* h, const uint32_t key[2], const float* x, int64_t n_points,
                   int64_t n_samples, const float* loc, const float* scale_packed,
                   float log_step_size, int32_t n, float* out, void* stream);

/* Per-chain key derivation used by amh_init (device out[n][2]); exposed so
 * callers can reproduce chain streams. */
int amh_chain_keys(const uint32_t key[2], int64_t chain_offset, int64_t n, uint32_t* out,
                   void* stream);

/* ------------------------------------------------------------------ ASSS ----
 * asss.py:197-251 (ASSS.sample) applied n_steps times to every chain: the
 * adaptive stereographic slice sampler with the same adaptation as ARWMH
 * (mean, rank-one Cholesky update, NaN -> keep L) and as_change =
 * ||mu' - mu|| + ||L' - L||_F.  Uses i, z, potential_energy, loc, scale,
 * as_change and rng_key of the states (mean_accept_prob / log_step_size are
 * not read or written and may be NULL).  Initial states come from amh_init
 * (asss.py:134-189 equals arwmh.py:84-138 on these leaves).  d <= 64.
 * `in` and `out` may alias.  collect: as amh_step (z / potential_energy). */
int amh_asss_step(amh_handle* h, int64_t num_chains, const amh_state* in, const amh_state* out,
                  int32_t n_steps, const amh_collect* collect, void* stream);

/* asss.py:271-303 (ASSS.sample_Pnx): n transitions with the frozen shared
 * adapt state (loc[d], scale_packed[P]) from every x[pt] for n_samples chains
 * each; out: device [n_points][n_samples][d].  Chain keys as amh_sample_pnx;
 * transition t draws at stream position t.  key[2] in host memory. */
int amh_asss_sample_pnx(amh_handle* h, const uint32_t key[2], const float* x, int64_t n_points,
                        int64_t n_samples, const float* loc, const float* scale_packed, int32_t n,
                        float* out, void* stream);

/* ----------------------------------------------------------- evaluation ----
 * python/utils/evaluation.py:223-294 (gaussian_kernel / mmd2_unbiased /
 * mmd_heuristic).  No handle: work goes to `stream` on the current device.
 * amh_kernel_sum: *out (device double) = sum over i < n, j < m of
 * exp(-gamma ||a_i - b_j||^2), pairs i == j skipped if skip_diag; a [n][d],
 * b [m][d] device float; scratch: amh_kernel_sum_scratch(n, m) device
 * doubles.  Deterministic (fixed-order reduction). */
int64_t amh_kernel_sum_scratch(int64_t n, int64_t m);
int amh_kernel_sum(const float* a, int64_t n, const float* b, int64_t m, int32_t d, float gamma,
                   int32_t skip_diag, double* scratch, double* out, void* stream);
/* out[i] = standard normal i of the stream keyed by key[2] (host memory),
 * for the random directions of max_sliced_wasserstein (evaluation.py:189). */
/* One half-iteration of log-domain Sinkhorn (the OT solver behind
 * wasserstein_sinkhorn, python/utils/evaluation.py:69-101, ott-jax linear.solve):
 * out[i] = -eps * log sum_j exp((pot[j] - cost[i][j]) / eps + log_w), cost
 * row-major [rows][cols] on the device.  The other half runs on the
 * transposed cost matrix. */
int amh_sinkhorn_lse(const float* cost, int64_t rows, int64_t cols, const float* pot, float log_w, float eps,
                     float* out, void* stream);
int amh_normals(const uint32_t key[2], int64_t n, float* out, void* stream);
/* out [n][m] = ||a_i - b_j||^2 (the median bandwidth heuristic, evaluation.py:286). */
int amh_pairwise_dist2(const float* a, int64_t n, const float* b, int64_t m, int32_t d, float* out,
                       void* stream);

/* ---------------------------------------------------- pooled covariance ----
 * Regime B (build-defined, no reference analogue): every chain
 * proposes with ONE shared adapt state, and the adaptation of arwmh.py:180-197
 * consumes the statistics of all chains (of all ranks):
 *   mu'  = mu + gamma S_d / N,   Sig' = (1 - gamma) Sig + gamma S_dd / N,
 *   L'   = chol(Sig') (kept, with Sig, if Sig' is not positive definite),
 *   lam' = lam + gamma (S_a / N - target), macc' = macc + (S_a / N - macc) / n
 * where S_d = sum delta_c, S_dd = sum delta_c delta_c^T, S_a = sum alpha_c,
 * delta_c = z_c' - mu.  With N = 1 this is the reference recurrence.
 * A step is amh_pooled_stats (per-chain transition + local sums), an
 * all-reduce(sum) of the sums across ranks by the caller (RCCL through
 * torch.distributed), then amh_pooled_update on every rank. */
typedef struct amh_pooled_state {
  int32_t* i;                 /* [1]      shared iteration                   */
  float* z;                   /* [C][d]   per chain                          */
  float* potential_energy;    /* [C]                                         */
  uint32_t* rng_key;          /* [C][2]   per-chain Philox key               */
  float* mean_accept_prob;    /* [1]                                         */
  float* loc;                 /* [d]      shared mu                          */
  float* scale;               /* [P]      shared L, packed lower             */
  float* log_step_size;       /* [1]                                         */
  float* as_change;           /* [1]                                         */
  double* cov;                /* [P]      shared Sigma (= L L^T), packed     */
} amh_pooled_state;

/* Number of doubles in the sums vector: d + d(d+1)/2 + 2, laid out as
 * [S_d (d) | S_dd packed lower (P) | S_a | N]. */
int amh_pooled_sums_size(int32_t dim, int64_t* v);

/* Per-chain transition with the shared state `in`, z / pe written to
 * z_out / pe_out (may alias in), and this rank's sums (device, V doubles). */
int amh_pooled_stats(amh_handle* h, int64_t num_chains, const amh_pooled_state* in, float* z_out,
                     float* pe_out, double* sums, void* stream);

/* Shared-state update from the (all-reduced) sums; writes i, mean accept,
 * loc, scale, log_step_size, as_change, cov of `out` (may alias `in`). */
int amh_pooled_update(amh_handle* h, const double* sums, const amh_pooled_state* in,
                      const amh_pooled_state* out, void* stream);

/* Single-process convenience: n_steps of stats + update (no all-reduce).
 * sums: device scratch of amh_pooled_sums_size doubles. */
int amh_pooled_step(amh_handle* h, int64_t num_chains, const amh_pooled_state* in,
                    const amh_pooled_state* out, int32_t n_steps, double* sums, void* stream);

/* Pool every K steps (one exchange per K transitions).  The
 * shared state stays frozen for a block of K transitions of every chain
 * (noise positions i .. i+K-1), the sums cover all K * C chain-steps (delta
 * against the frozen mu, N = K * C), and one update ends the block: i += K,
 * gamma = 1 / n^a with n = the block count (i / K + 1, reset at num_warmup,
 * which must be a multiple of K).  K = 1 is amh_pooled_stats / _update. */
int amh_pooled_stats_k(amh_handle* h, int64_t num_chains, const amh_pooled_state* in, int32_t k_steps,
                       float* z_out, float* pe_out, double* sums, void* stream);
int amh_pooled_update_k(amh_handle* h, const double* sums, const amh_pooled_state* in,
                        const amh_pooled_state* out, int32_t k_steps, void* stream);
/* n_steps (a multiple of sync_every) transitions, one update per sync_every. */
int amh_pooled_step_k(amh_handle* h, int64_t num_chains, const amh_pooled_state* in,
                      const amh_pooled_state* out, int32_t n_steps, int32_t sync_every, double* sums,
                      void* stream);

/* The exchange between amh_pooled_stats_k and amh_pooled_update_k on N > 1
 * ranks (SURVEY.md §8(b) amh_pooled_allreduce; no counterpart in the
 * reference, whose adaptation is per chain): in-place ncclAllReduce(sum) of
 * the n = amh_pooled_sums_size doubles at `sums` on `stream`, over the
 * caller's RCCL communicator `rccl_comm` (an ncclComm_t made by
 * ncclCommInitRank in the same RCCL instance; kernels_amd.distributed.RcclComm
 * does that).  The RCCL already loaded in the process is used (looked up by
 * soname), else the system librccl.so.1.  An RCCL error returns AMH_EHIP with
 * its text in amh_last_error; nothing is retried. */
int amh_pooled_allreduce(amh_handle* h, double* sums, int64_t n, void* rccl_comm, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* AMH_H */
