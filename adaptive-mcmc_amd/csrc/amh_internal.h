// amh_internal.h -- kernel parameter blocks shared by amh_kernels.hip and the
// C-ABI layer amh_capi.hip.  Not part of the public ABI (include/amh.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/amh.h"

// the phase-stamp build is a diagnostic build: it also honours the A/B
// environment switches (amh_kernels.hip, amh_capi.hip)
#if defined(AMH_STAMPS) && !defined(AMH_DIAG)
#define AMH_DIAG 1
#endif

namespace amh {

// Learning-rate table size: gamma_n for n < 2^20 is precomputed on the host
// with the same amh_lr_gamma the device would run (bit-identical); larger n
// fall back to the device routine.
constexpr int32_t kGammaTab = 1 << 20;

struct ModelArgs {
  const float* data;  // device, model-specific layout (include/amh.h)
  int64_t n;          // N rows (regression models)
  int64_t k;          // K columns (diamonds)
};

struct StepParams {
  amh_state in, out;
  int64_t C;
  int32_t d, W;
  float a, target, eps;
  int32_t n_steps;
  float* col_z;            // [n_keep][C][d] or null
  float* col_pe;           // [n_keep][C] or null
  int32_t* accept_count;   // [C] or null
  int32_t thinning;
  const float* gamma_tab;  // gamma_n = amh_lr_gamma(n, a) for n < gamma_tab_n
  int32_t gamma_tab_n;
  ModelArgs model;
  const float* ext_pe;     // split path: U(z') per chain from the batched potential (n_steps == 1)
  const float* ext_z;      // split path: the proposals z' [C][d] that U(z') was evaluated at
  float* xprop_next;       // split path: the NEXT transition's proposal [C][d] (or null), formed as
                           // the propose pass would form it from the stored state
};

struct InitParams {
  amh_state out;
  int64_t C, chain_offset;
  int32_t d;
  uint32_t key0, key1;
  const float* init_z;
  ModelArgs model;
};

struct PotParams {
  const float* z;
  float* pe;
  int64_t n;
  int32_t d;
  ModelArgs model;
  const float* xpack = nullptr;  // diamonds: the design matrix in MFMA tile order (diamonds_pack_kernel)
};

struct PnxParams {
  const float* x;
  int64_t n_points, n_samples;
  const float* scale;  // packed shared factor
  float log_step_size, eps;
  int32_t n, d;
  uint32_t key0, key1;
  float* out;
  ModelArgs model;
};

// ASSS.sample_Pnx (amh_asss.hip): frozen shared (loc, scale) for every chain
struct AsssPnxParams {
  const float* x;
  int64_t n_points, n_samples;
  const float* loc;    // shared mu [d]
  const float* scale;  // shared packed factor
  float eps;
  int32_t n, d;
  uint32_t key0, key1;
  float* out;
  ModelArgs model;
};

// pooled covariance (amh_pooled.hip)
constexpr int kPoolWaves = 16;  // waves (of one chain each) per chunk block

// chains each wave of a chunk takes (bit spec: fixes the summation order)
__host__ __device__ inline int pooled_cpw(int64_t C) {
  const int64_t c = (C + 4095) / 4096;
  return c < 1 ? 1 : (c > 16 ? 16 : (int)c);
}

// pooled_final_kernel may also form the large-d update's Sigma' (what
// pooled_big_prep_kernel does) when the update follows in the same library
// call with no exchange in between (amh_pooled_step_k, one rank): scratch
// non-null, N = the chain-steps the sums cover
struct FinalPrep {
  const double* cov;
  const int32_t* i;
  float* scratch;
  double N;
  int32_t W, K;
  float a;
};

struct PooledStatsParams {
  int64_t C;
  int32_t d;
  const int32_t* i;
  const float *z, *pe;
  const uint32_t* keys;
  const float *mu, *L, *lam;
  float eps;
  float *z_out, *pe_out;
  double* partials;  // [n_chunks][V]
  ModelArgs model;
  int32_t k_steps;     // d <= 64: transitions per chain with the frozen shared state
  int32_t i_add;       // d > 64: this launch is step i + i_add of the block
  int32_t accumulate;  // d > 64: sums += this launch's sums (steps after the first)
  // d > 64: noise made ahead of time (pooled_big_update_kernel's extra
  // blocks): xi [cap][d] and per-chain records (i, key0, key1, u bits); a
  // chain uses them only if its record matches (i, its key), else it draws
  const float* xi;
  const uint4* xrec;
  int64_t xi_cap;
  FinalPrep prep;  // scratch == nullptr: none
  // d = 64: the chunk partials are left for the update launch to reduce
  // (amh_pooled_step_k on one rank: the update follows with no exchange)
  int32_t defer_reduce;
  // d > 64: the A-operand copies are current (the previous update's post
  // kernel wrote the factor's tiles; the precision's are from the first pack)
  int32_t pack_ready;
};

// Pool-every-K: the update after a block of K transitions that started at
// shared iteration it counts blocks, n = it / K + 1 (reset at W, W % K == 0);
// K = 1 is arwmh.py:181.
__host__ __device__ inline int32_t pooled_block_n(int32_t it, int32_t W, int32_t K) {
  return (it < W) ? it / K + 1 : (it - W) / K + 1;
}

struct PooledUpdateParams {
  int32_t d, W;
  float a, target;
  const double* sums;
  amh_pooled_state in, out;
  float* scratch;  // d >= 64: d(d+4)/2 floats (4-row-aligned factor), ok, gamma, e^lam, e^lam', 4 spare, d column sums
  int32_t K;       // transitions per pooled update (the sums cover K * C chain-steps)
  // d > 64: the next step's noise for chains [0, noise_C) is drawn by the
  // update launch's extra blocks into xi / xrec (PooledStatsParams)
  int64_t noise_C;
  const uint32_t* keys;
  float* xi;
  uint4* xrec;
  // d = 64, red_blocks > 0: the launch first reduces the stats launch's chunk
  // partials into sums_out (== sums; the last reduce block to finish runs
  // the update)
  const float* red_partials;
  int64_t red_chunks;
  int32_t red_accumulate, red_blocks;
  double* sums_out;
  // host-mapped flag (the handle's): set when the d = 64 update's bounded
  // wait on an earlier wave's columns runs out (the factor is then kept);
  // the next library call on the handle reports it (amh_capi.hip)
  int* err_flag;
  // d > 64, one rank (amh_pooled_step_k): pooled_big_post_kernel also writes
  // the new factor's lower tiles in A-operand order here, for the next
  // step's stats launch (its pooled_pack_kernel launch is then skipped)
  float* pack_out;
};
int pooled_reduce64_blocks(int64_t V);  // reduce blocks of the d = 64 partial rows

hipError_t run_pooled_stats(int model_id, const PooledStatsParams& p, double* sums, hipStream_t s);
// large dimensions (amh_big_pooled.hip): chunks of 256 chains
int64_t pooled_big_chunks(int64_t C, int d);
int64_t pooled_big_pack_floats(int d);
int64_t pooled_big_tile_V(int d);  // partial row length of the fused large-d stats (d > 64)  // scratch floats of the fused large-d stats (A-operand tiles)
int64_t pooled_scratch_rows(int64_t n_chunks);  // partials + group sums of pooled_reduce
hipError_t run_pooled_big_stats(const PooledStatsParams& p, float* xprop, float* pep, double* sums, hipStream_t s);
hipError_t run_pooled_big_update(const PooledUpdateParams& p, hipStream_t s, bool sigma_ready = false);
hipError_t run_asss_step(int model_id, const StepParams& p, hipStream_t s);  // amh_asss.hip
hipError_t run_asss_step64(const StepParams& p, hipStream_t s);  // amh_kernels.hip (d = 64 Gaussian)
hipError_t run_asss_pnx(int model_id, const AsssPnxParams& p, hipStream_t s);
// evaluation metrics (amh_eval.hip)
int64_t kernel_sum_blocks(int64_t n, int64_t m);
hipError_t run_kernel_sum(const float* A, int64_t n, const float* B, int64_t m, int d, float gamma, int skip_diag,
                          double* partials, double* out, hipStream_t s);
hipError_t run_dist2(const float* A, int64_t n, const float* B, int64_t m, int d, float* out, hipStream_t s);
hipError_t run_normals(uint32_t k0, uint32_t k1, int64_t n, float* out, hipStream_t s);
hipError_t run_pooled_update(const PooledUpdateParams& p, hipStream_t s);

hipError_t run_step(int model_id, const StepParams& p, hipStream_t s);
hipError_t run_lse_rows(const float* Cm, int64_t rows, int64_t cols, const float* pot, float logw, float eps,
                        float* out, hipStream_t s);
hipError_t run_init(int model_id, const InitParams& p, hipStream_t s);
hipError_t run_potential(int model_id, const PotParams& p, hipStream_t s);
hipError_t run_pnx(int model_id, const PnxParams& p, hipStream_t s);
// sample_Pnx with the caller's potential (AMH_MODEL_EXTERNAL, d <= 64): one
// step t of every chain in two launches around the caller's U
struct PnxExtParams {
  float* z;              // [C][d] current points (accept: updated)
  float* pe;             // [C] their U (accept: updated)
  float* zprop;          // [C][d] proposals (propose: written)
  const float* pe_prop;  // [C] U(zprop) (accept)
  int64_t C;
  const float* scale;    // shared packed factor
  float log_step_size, eps;
  int32_t t, d;
  uint32_t key0, key1;
};
hipError_t run_pnx_ext(const PnxExtParams& p, bool accept, hipStream_t s);
// large dimensions (64 < d <= 256, Gaussian; amh_big.hip)
struct BigParams {
  amh_state in, out;
  int64_t C;
  int32_t d, W;
  float a, target, eps;
  const float* gamma_tab;
  int32_t gamma_tab_n;
  float *xprop, *wa, *wr;  // propose -> step scratch [C][d]
  float* dg;               // the factor's diagonal [C][d] (propose / step<NEXT> -> step)
  const float* pep;        // U(z') [C]
  int32_t* accept_count;   // [C] or null
  float* col_z;            // this step's collection slot [C][d] or null
  float* col_pe;           // [C] or null
};
bool big_model(int model_id, int d);
bool pooled_big_model(int model_id, int d);
hipError_t run_big_init(const InitParams& p, hipStream_t s);
hipError_t run_big_propose(const BigParams& p, hipStream_t s);
// next: also form the next transition's proposal and solves (multi-step launches)
hipError_t run_big_step(const BigParams& p, hipStream_t s, bool next = false);
hipError_t run_big_potential(const PotParams& p, hipStream_t s);
// ASSS for the large-d Gaussian (big_model): one transition per launch; the
// frozen kernel of sample_Pnx
hipError_t run_asss_big_step(const StepParams& p, hipStream_t s);
// ARWMH.sample_Pnx for the large-d Gaussian (big_model)
hipError_t run_big_pnx(const PnxParams& p, hipStream_t s);
hipError_t run_asss_big_pnx(const AsssPnxParams& p, hipStream_t s);

// split path for data-heavy models (diamonds): proposal kernel, lane-per-chain
// batched potential, then the step kernel reading U(z') (amh_split.hip)
bool split_model(int model_id, int d);
constexpr int kDiaMfmaKc = 24;  // diamonds on MFMA: the reference data set's Kc (amh_split.hip)
int64_t diamonds_pack_floats(int64_t N, int64_t K);  // 0: no MFMA path for this shape
hipError_t run_diamonds_pack(const ModelArgs& m, float* xp, hipStream_t s);
// the reference diamonds data (K = 25 columns): d = 26, compiled as a fixed
// dimension on the split path
constexpr int kDiamondsD = 26;
hipError_t run_propose(const StepParams& p, float* xprop, hipStream_t s);
hipError_t run_step_ext(const StepParams& p, hipStream_t s);
hipError_t run_init_nopot(const InitParams& p, hipStream_t s);
hipError_t run_potential_lane(int model_id, const PotParams& p, hipStream_t s);
hipError_t run_chain_keys(uint32_t k0, uint32_t k1, int64_t offset, int64_t n, uint32_t* out,
                          hipStream_t s);
#ifdef AMH_STAMPS
hipError_t diag_stamps_copy(void* host, size_t bytes);
hipError_t diag_upd_stamps_copy(void* host);
hipError_t diag_f64_stamps_copy(void* host);
hipError_t diag_u64_timeline_copy(void* host);
#endif

}  // namespace amh
