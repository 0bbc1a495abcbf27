// amh_asss.hip -- ASSS, the adaptive stereographic slice sampler
// (python/kernels/asss.py:99-269), for d <= 64 on gfx950.
//
// Same lane mapping as the ARWMH step kernel: a group of G lanes owns one
// chain, lane r holds row r of the factor in unit-lower form (U[j] = L_rj /
// L_jj, U_rr = 1) plus dl = L_rr, x_r and mu_r.  One transition:
//
//   S = (L + eps I) sqrt(d)                        asss.py:214
//   y = S^-1 (x - mu)     column sweep, one broadcast pair per column
//   z = stereographic projection of y on S^d       asss.py:33-45
//   v ~ N(0, I_{d+1}), projected to the tangent space of z and normalised
//   t = U~(z) - log u,  U~(z) = U(x(z)) + d log(1 - z_d)
//   shrinkage on the great circle z cos th + v sin th (asss.py:59-96)
//   x' = x(z'),  then the reference's mean / rank-one Cholesky adaptation
//
// The slice circle is mapped back through S once per transition: x(th) =
// (cos th S z + sin th S v) / (1 - z_d(th)) + mu, so each shrinkage step
// costs O(d) plus one potential evaluation.  Groups of one wave that finish
// their shrinkage early keep their values (selects) while the wave loops on
// (wave ballot), so potentials run converged as the model code requires.
//
// Noise at stream position i (counter-based, AMH_TAG_ASSS): lane r of
// Philox(r, i, 0) gives v_r; lane 0's other words give v_d, u_t and th_0;
// shrink step k draws Philox(k, i, 1).  The bit spec is mirrored by
// oracle/amh_oracle.c (orc_asss_step); tests/test_asss.py pins it against a
// literal float64 restatement of asss.py.
#include "amh_asss.h"

namespace amh {

template <int DMAX, template <int> class M, bool EXACT>
__global__ __launch_bounds__(kBlock, (EXACT && DMAX == 64) ? 4 : 1) void asss_step_kernel(StepParams p) {
  constexpr int G = DMAX;
  using Gp = Grp<G>;
  extern __shared__ float lds[];
  const int d = EXACT ? DMAX : p.d;
  M<G>::stage(lds, p.model, d);
  __syncthreads();
  const auto mctx = M<G>::prepare(p.model, d, lane_id() & (G - 1));
  const int64_t C = p.C;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const int64_t n_items = (C + Geo<G>::CPW - 1) / Geo<G>::CPW;
  const int64_t wave0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t wstride = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t item = wave0; item < n_items; item += wstride) {
    int lane = lane_id();
    asm volatile("" : "+v"(lane));  // keep per-column lane masks inside the item loop
    const int r = lane & (G - 1);
    const int rr = r;
    const bool act = r < d;
    const int64_t chain = item_chain<G>(item);
    const bool chain_ok = chain < C;
    const int64_t cl = chain_ok ? chain : C - 1;

    // ---- state (L -> U, dl as the ARWMH kernel)
    const float* Lin = p.in.scale + cl * P;
    float dl = act ? Lin[col_off(d, r)] : 0.0f;
    const float inv = (amh_isfinite(dl) && dl != 0.0f) ? 1.0f / dl : 0.0f;
    float U[DMAX];
    static_for<DMAX>([&](auto J) {
      constexpr int j = J;
      U[j] = 0.0f;
      if (j < d) {
        const float lv = (act && r > j) ? Lin[col_off(d, j) + (r - j)] : 0.0f;
        U[j] = set_one_at<G, j>(keep_above<G, j>(lv * Gp::template bcast<j>(inv), rr), rr);
      }
    });
    float x = act ? p.in.z[cl * d + r] : 0.0f;
    float mu = act ? p.in.loc[cl * d + r] : 0.0f;
    int32_t it = p.in.i[cl];
    float pe = p.in.potential_energy[cl];
    float asc = p.in.as_change[cl];
    const uint32_t k0 = (uint32_t)p.in.rng_key[2 * cl], k1 = (uint32_t)p.in.rng_key[2 * cl + 1];
    bool updated = false;

    for (int32_t t = 0; t < p.n_steps; ++t) {
      asss_transition<DMAX, M, true>(p, U, dl, x, mu, pe, asc, updated, it, k0, k1, d, r, rr, act, mctx, lds);
      it += 1;
      if (p.col_z != nullptr || p.col_pe != nullptr) {
        if ((t + 1) % p.thinning == 0 && chain_ok) {
          const int64_t k = t / p.thinning;
          if (p.col_z != nullptr && act) p.col_z[(k * C + chain) * d + r] = x;
          if (p.col_pe != nullptr && r == 0) p.col_pe[k * C + chain] = pe;
        }
      }
    }

    // ---- store: L = U diag(dl) if any step updated it, else verbatim
    if (chain_ok) {
      float* Lout = p.out.scale + chain * P;
      static_for<DMAX>([&](auto J) {
        constexpr int j = J;
        if (j < d) {
          const float dj = Gp::template bcast<j>(dl);
          if (act && r >= j) {
            const int64_t o = col_off(d, j) + (r - j);
            if (updated) {
              Lout[o] = U[j] * dj;
            } else if (Lout != Lin) {
              Lout[o] = Lin[o];
            }
          }
        }
      });
      if (act) {
        p.out.z[chain * d + r] = x;
        p.out.loc[chain * d + r] = mu;
      }
      if (r == 0) {
        p.out.i[chain] = it;
        p.out.potential_energy[chain] = pe;
        p.out.as_change[chain] = asc;
        p.out.rng_key[2 * chain] = k0;
        p.out.rng_key[2 * chain + 1] = k1;
      }
    }
  }
}

// ----------------------------------------------------------- sample_Pnx ----
// asss.py:271-303: chain c = (pt, s) starts at x[pt] with key split(rng_key,
// C)[c] (as the ARWMH sample_Pnx kernel) and runs n transitions with the
// frozen shared (loc, scale); transition t draws at stream position t.
template <int DMAX, template <int> class M, bool EXACT>
__global__ __launch_bounds__(kBlock) void asss_pnx_kernel(AsssPnxParams q) {
  constexpr int G = DMAX;
  using Gp = Grp<G>;
  extern __shared__ float lds[];
  const int d = EXACT ? DMAX : q.d;
  M<G>::stage(lds, q.model, d);
  __syncthreads();
  const auto mctx = M<G>::prepare(q.model, d, lane_id() & (G - 1));
  StepParams p{};
  p.eps = q.eps;
  const int r0 = Gp::r();
  const bool act0 = r0 < d;
  float dl = act0 ? q.scale[col_off(d, r0)] : 0.0f;
  const float inv = (amh_isfinite(dl) && dl != 0.0f) ? 1.0f / dl : 0.0f;
  float U[DMAX];
  static_for<DMAX>([&](auto J) {
    constexpr int j = J;
    U[j] = 0.0f;
    if (j < d) {
      const float lv = (act0 && r0 > j) ? q.scale[col_off(d, j) + (r0 - j)] : 0.0f;
      U[j] = set_one_at<G, j>(keep_above<G, j>(lv * Gp::template bcast<j>(inv), r0), r0);
    }
  });
  float mu = act0 ? q.loc[r0] : 0.0f;
  const int64_t C = q.n_points * q.n_samples;
  const int64_t n_items = (C + Geo<G>::CPW - 1) / Geo<G>::CPW;
  const int64_t wave0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t wstride = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t item = wave0; item < n_items; item += wstride) {
    int lane = lane_id();
    asm volatile("" : "+v"(lane));
    const int r = lane & (G - 1);
    const bool act = r < d;
    const int64_t chain = item_chain<G>(item);
    const bool chain_ok = chain < C;
    const int64_t cl = chain_ok ? chain : C - 1;
    const int64_t pt = cl / q.n_samples;
    const amh_u32x4 kk = amh_philox4x32_10((uint32_t)cl, (uint32_t)((uint64_t)cl >> 32), 0u, AMH_TAG_SPLIT,
                                           q.key0, q.key1);
    float x = act ? q.x[pt * d + r] : 0.0f;
    float pe = M<G>::potential(x, r, d, mctx, lds);
    float asc = 0.0f;
    bool updated = false;
    for (int32_t t = 0; t < q.n; ++t) {
      asss_transition<DMAX, M, false>(p, U, dl, x, mu, pe, asc, updated, t, kk.v[0], kk.v[1], d, r, r, act, mctx,
                                      lds);
    }
    if (chain_ok && act) q.out[cl * d + r] = x;
  }
}

// ------------------------------------------------------------- launchers ----
template <int DMAX, template <int> class M, bool EXACT>
hipError_t launch_asss(const StepParams& p, hipStream_t s) {
  const int64_t n_items = (p.C + Geo<DMAX>::CPW - 1) / Geo<DMAX>::CPW;
  const size_t shm = M<DMAX>::lds_bytes(p.model, EXACT ? DMAX : p.d);
  if (shm > 163840) return hipErrorInvalidConfiguration;
  int64_t blocks = (n_items + kBlock / 64 - 1) / (kBlock / 64);
  if (blocks > 256 * 32) blocks = 256 * 32;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((asss_step_kernel<DMAX, M, EXACT>), dim3((unsigned)blocks), dim3(kBlock), shm, s, p);
  return hipGetLastError();
}

struct AsssF {
  const StepParams& p;
  hipStream_t s;
  template <int D, template <int> class M, bool E>
  hipError_t operator()() const {
    return launch_asss<D, M, E>(p, s);
  }
};

hipError_t run_asss_step(int model_id, const StepParams& p, hipStream_t s) {
  // the d = 64 Gaussian (BASELINE configs[1] shape): the persistent step
  // kernel's data movement (LDS-DMA prefetch, dwordx4 write-back, 16 waves
  // per CU) around the same transition -- the same bits
  if (model_id == AMH_MODEL_GAUSSIAN && p.d == 64) return run_asss_step64(p, s);
  return dispatch(model_id, p.d, AsssF{p, s});
}

template <int DMAX, template <int> class M, bool EXACT>
hipError_t launch_asss_pnx(const AsssPnxParams& p, hipStream_t s) {
  const int64_t C = p.n_points * p.n_samples;
  const int64_t n_items = (C + Geo<DMAX>::CPW - 1) / Geo<DMAX>::CPW;
  const size_t shm = M<DMAX>::lds_bytes(p.model, EXACT ? DMAX : p.d);
  if (shm > 163840) return hipErrorInvalidConfiguration;
  int64_t blocks = (n_items + kBlock / 64 - 1) / (kBlock / 64);
  if (blocks > 256 * 32) blocks = 256 * 32;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL((asss_pnx_kernel<DMAX, M, EXACT>), dim3((unsigned)blocks), dim3(kBlock), shm, s, p);
  return hipGetLastError();
}

struct AsssPnxF {
  const AsssPnxParams& p;
  hipStream_t s;
  template <int D, template <int> class M, bool E>
  hipError_t operator()() const {
    return launch_asss_pnx<D, M, E>(p, s);
  }
};

hipError_t run_asss_pnx(int model_id, const AsssPnxParams& p, hipStream_t s) {
  return dispatch(model_id, p.d, AsssPnxF{p, s});
}

}  // namespace amh
