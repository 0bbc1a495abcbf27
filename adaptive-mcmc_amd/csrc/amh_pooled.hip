// amh_pooled.hip -- pooled-covariance adaptation (regime B, include/amh.h):
// every chain proposes with one shared (mu, L, lambda); the adaptation of
// arwmh.py:180-197 consumes the statistics of all chains.
//
//   pooled_stats_kernel   per-chain transition (arwmh.py:162-178 with the
//                         shared factor staged in LDS) + the chunk's sums
//                         S_d, S_dd, S_a (float32 per wave over its chains,
//                         double across the chunk's waves)
//   pooled_reduce_kernel  chunk partials -> this rank's sums (double, chunk
//                         order); ranks then all-reduce them (RCCL)
//   pooled_update_kernel  mu, Sigma, lambda, mean-accept update and the
//                         Cholesky refactorisation of Sigma' (one wave, rows
//                         in registers, double precision)
//
// The order of every sum is fixed (oracle: orc_pooled_stats/_update), so the
// result does not depend on which CU runs which chunk.
#include "amh_device.h"

namespace amh {

namespace {

// Shared-factor row r as stored in LDS (dense, zero above the diagonal, rows
// padded like the Gaussian precision) dotted with v broadcast from lane j:
// partial sums over j mod 4, read 16 columns at a time.
__device__ __forceinline__ float lds_row_dot64(uint32_t prow, int d, float v, bool act) {
  using Gp = Grp<64>;
  float y4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  static_for<4>([&](auto B) {
    constexpr int b = B;
    if (16 * b < d) {
      f32x4 pv[4];
      static_for<4>([&](auto Q) {
        pv[Q] = (4 * (4 * b + Q) < d) ? lds_ld4<16 * (4 * b + Q)>(prow) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      });
      lds_wait(pv[0], pv[1], pv[2], pv[3]);
      static_for<16>([&](auto K) {
        constexpr int j = 16 * b + K;
        if (j < d) y4[K & 3] = fmaf(act ? pv[K / 4][K % 4] : 0.0f, Gp::template bcast<j>(v), y4[K & 3]);
      });
      __builtin_amdgcn_sched_barrier(0);
    }
  });
  return (y4[0] + y4[1]) + (y4[2] + y4[3]);
}

__host__ __device__ inline int pooled_ld(int d) { return ((d + 3) & ~3) + 4; }

template <template <int> class M>
__host__ __device__ inline size_t pooled_lds_model_floats(const ModelArgs& m, int d) {
  return (M<64>::lds_bytes(m, d) / sizeof(float) + 3) & ~(size_t)3;
}
template <template <int> class M>
__host__ __device__ inline size_t pooled_lds_bytes(const ModelArgs& m, int d) {
  const size_t f = pooled_lds_model_floats<M>(m, d) + (size_t)d * pooled_ld(d);
  const size_t f8 = (f + 1) & ~(size_t)1;  // 8-B align the double area
  return f8 * sizeof(float) + (64 * 64 + 64 + 2) * sizeof(double);
}

__device__ __forceinline__ int64_t packed_col(int d, int64_t o) {  // column of packed index o
  int k = 0;
  while (k + 1 < d && col_off(d, k + 1) <= o) ++k;
  return k;
}

}  // namespace

template <template <int> class M, bool EXACT>
__global__ __launch_bounds__(kPoolWaves * 64) void pooled_stats_kernel(PooledStatsParams p) {
  constexpr int G = 64;
  using Gp = Grp<G>;
  extern __shared__ float lds[];
  const int d = EXACT ? 64 : p.d;
  const int ld = pooled_ld(d);
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const int64_t V = d + P + 2;
  float* lrow = lds + pooled_lds_model_floats<M>(p.model, d);
  double* cmb = (double*)(lds + (((size_t)(lrow - lds) + (size_t)d * ld + 1) & ~(size_t)1));
  double* cmb_sd = cmb + 64 * 64;
  double* cmb_sa = cmb_sd + 64;

  M<G>::stage(lds, p.model, d);
  for (int k = threadIdx.x; k < d * ld; k += blockDim.x) {
    const int row = k / ld, col = k - row * ld;
    lrow[k] = (col <= row && col < d) ? p.L[col_off(d, col) + (row - col)] : 0.0f;
  }
  for (int k = threadIdx.x; k < 64 * 64 + 64 + 2; k += blockDim.x) cmb[k] = 0.0;
  __syncthreads();

  const int lane = lane_id();
  const int r = lane;
  const bool act = r < d;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  const auto mctx = M<G>::prepare(p.model, d, r);
  const int32_t it = __builtin_amdgcn_readfirstlane(p.i[0]);
  const float el = amh_expf(p.lam[0]);
  const float mu = act ? p.mu[r] : 0.0f;
  const uint32_t prow = lds_addr(lrow + (act ? r : 0) * ld);

  const int cpw = pooled_cpw(p.C);
  const int64_t chunk0 = (int64_t)blockIdx.x * kPoolWaves * cpw;
  const int64_t base = chunk0 + (int64_t)w * cpw;
  float S[64];
  static_for<64>([&](auto K) { S[K] = 0.0f; });
  float sd = 0.0f, sa = 0.0f;
  for (int t = 0; t < cpw; ++t) {
    const int64_t c = base + t;
    if (c >= p.C) break;
    const float z = act ? p.z[c * d + r] : 0.0f;
    const float pe = p.pe[c];
    const uint32_t k0 = p.keys[2 * c], k1 = p.keys[2 * c + 1];
    // noise at the shared stream position (arwmh.py:162-165, 174)
    const amh_u32x4 o = amh_philox4x32_10((uint32_t)r, (uint32_t)it, 0u, AMH_TAG_STEP, k0, k1);
    const float xi = act ? amh_normal_from_bits(o.v[0]) : 0.0f;
    const float u = amh_unif01_from_bits(Gp::template bcast_u<0>(o.v[1]));
    // proposal with the shared factor (arwmh.py:166-167)
    const float acc = lds_row_dot64(prow, d, xi, act);
    const float zp = act ? z + fmaf(el, acc, p.eps * xi) : 0.0f;
    float pep = M<G>::potential(zp, r, d, mctx, lds);
    if (amh_isnan(pep)) pep = INFINITY;
    const float ex = amh_expf(pe - pep);
    const float alpha = (ex > 1.0f) ? 1.0f : ex;
    const bool accept = u < alpha;
    const float zn = accept ? zp : z;
    if (act) p.z_out[c * d + r] = zn;
    if (r == 0) p.pe_out[c] = accept ? pep : pe;
    // pooled statistics (float32 over this wave's chains, in chain order)
    const float delta = act ? zn - mu : 0.0f;
    sd = sd + delta;
    static_for<64>([&](auto K) {
      constexpr int k = K;
      if (k < d) S[k] = fmaf(delta, Gp::template bcast<k>(delta), S[k]);
      column_fence<k>();
    });
    sa = sa + alpha;
  }
  // the chunk's waves add their partials in wave order (double)
  for (int ww = 0; ww < kPoolWaves; ++ww) {
    if (w == ww) {
      if (act) {
        static_for<64>([&](auto K) {
          constexpr int k = K;
          if (k <= r && k < d) cmb[r * 64 + k] += (double)S[k];
        });
        cmb_sd[r] += (double)sd;
      }
      if (lane == 0) *cmb_sa += (double)sa;
    }
    __syncthreads();
  }
  double* out = p.partials + (int64_t)blockIdx.x * V;
  const int64_t left = p.C - chunk0;
  const double cnt = (double)(left < (int64_t)kPoolWaves * cpw ? left : (int64_t)kPoolWaves * cpw);
  for (int64_t v = threadIdx.x; v < V; v += blockDim.x) {
    double val;
    if (v < d) {
      val = cmb_sd[v];
    } else if (v < d + P) {
      const int64_t o = v - d;
      const int64_t k = packed_col(d, o);
      const int64_t rr = k + (o - col_off(d, (int)k));
      val = cmb[rr * 64 + k];
    } else if (v == d + P) {
      val = *cmb_sa;
    } else {
      val = cnt;
    }
    out[v] = val;
  }
}

__global__ __launch_bounds__(256) void pooled_reduce_kernel(const double* partials, int64_t n_chunks, int64_t V,
                                                            double* sums) {
  const int64_t v = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (v >= V) return;
  double s = 0.0;
  for (int64_t ch = 0; ch < n_chunks; ++ch) s += partials[ch * V + v];
  sums[v] = s;
}

namespace {
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffLL), lane);
  const int hi = __builtin_amdgcn_readlane((int)(unsigned)((unsigned long long)b >> 32), lane);
  return __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
}
}  // namespace

// One wave: lane r holds row r of Sigma' (double) and factors it in place
// (right-looking; element (r, k) is updated in column order, oracle mirror).
__global__ __launch_bounds__(64) void pooled_update_kernel(PooledUpdateParams p) {
  const int d = p.d;
  const int r = lane_id();
  const bool act = r < d;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const double* sums = p.sums;
  const double N = sums[d + P + 1];
  const int32_t it = p.in.i[0];
  const int32_t itr = it + 1;
  const int32_t n = (it < p.W) ? itr : itr - p.W;
  const float gamma = amh_lr_gamma(n, p.a);
  const float macc = p.in.mean_accept_prob[0];
  const float lam = p.in.log_step_size[0];
  const float abar = (float)(sums[d + P] / N);
  const float maccn = macc + (abar - macc) / (float)n;
  const float lamn = lam + gamma * (abar - p.target);
  const float mun = act ? p.in.loc[r] + gamma * (float)(sums[r] / N) : 0.0f;
  const double g = (double)gamma;

  double A[64];
  float Lo[64];
  static_for<64>([&](auto K) {
    constexpr int k = K;
    A[k] = 0.0;
    Lo[k] = 0.0f;
    if (k < d && act && k <= r) {
      const int64_t o = col_off(d, k) + (r - k);
      const double a = (1.0 - g) * p.in.cov[o];
      const double b = g * (sums[d + o] / N);
      A[k] = a + b;
      Lo[k] = p.in.scale[o];
    }
  });
  bool ok = true;
  static_for<64>([&](auto J) {
    constexpr int j = J;
    if (j < d) {
      const double piv = readlane_f64(A[j], j);
      ok = ok && (piv > 0.0) && __builtin_isfinite(piv);
      const double ljj = sqrt(piv);
      A[j] = (r > j) ? A[j] / ljj : ((r == j) ? ljj : A[j]);
      static_for<64>([&](auto K) {
        constexpr int k = K;
        if constexpr (k > j) {
          if (k < d) {
            const double lkj = readlane_f64(A[j], k);
            A[k] = (r >= k) ? fma(-A[j], lkj, A[k]) : A[k];
          }
        }
      });
    }
  });
  const float e0 = amh_expf(lam), e1 = amh_expf(lamn);
  float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  static_for<64>([&](auto J) {
    constexpr int j = J;
    if (j < d) {
      const float lo = Lo[j];
      const float ln = ok ? (float)A[j] : lo;
      const float tt = (j <= r && act) ? (ln * e1) - (lo * e0) : 0.0f;
      s4[j & 3] = fmaf(tt, tt, s4[j & 3]);
    }
  });
  const float part = act ? (s4[0] + s4[1]) + (s4[2] + s4[3]) : 0.0f;
  const float asc = sqrtf(Grp<64>::sum(part));
  // writes (each lane reads then writes only its own row: in-place safe)
  if (act) {
    static_for<64>([&](auto K) {
      constexpr int k = K;
      if (k < d && k <= r) {
        const int64_t o = col_off(d, k) + (r - k);
        if (ok) {
          const double a = (1.0 - g) * p.in.cov[o];
          const double b = g * (sums[d + o] / N);
          p.out.cov[o] = a + b;
          p.out.scale[o] = (float)A[k];
        } else {
          p.out.cov[o] = p.in.cov[o];
          p.out.scale[o] = Lo[k];
        }
      }
    });
    p.out.loc[r] = mun;
  }
  if (r == 0) {
    p.out.i[0] = itr;
    p.out.mean_accept_prob[0] = maccn;
    p.out.log_step_size[0] = lamn;
    p.out.as_change[0] = asc;
  }
}

template <int DMAX, template <int> class M, bool EXACT>
hipError_t launch_pooled_stats(const PooledStatsParams& p, double* sums, hipStream_t s) {
  static_assert(DMAX == 64, "pooled kernels run one chain per wave");
  const int d = EXACT ? 64 : p.d;
  const size_t shm = pooled_lds_bytes<M>(p.model, d);
  if (shm > 163840) return hipErrorInvalidConfiguration;
  const int cpw = pooled_cpw(p.C);
  const int64_t chunk = (int64_t)kPoolWaves * cpw;
  const int64_t n_chunks = (p.C + chunk - 1) / chunk;
  const int64_t V = d + (int64_t)d * (d + 1) / 2 + 2;
  hipLaunchKernelGGL((pooled_stats_kernel<M, EXACT>), dim3((unsigned)n_chunks), dim3(kPoolWaves * 64), shm, s, p);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(pooled_reduce_kernel, dim3((unsigned)((V + 255) / 256)), dim3(256), 0, s, p.partials,
                     n_chunks, V, sums);
  return hipGetLastError();
}

namespace {
struct PooledF {
  const PooledStatsParams& p;
  double* sums;
  hipStream_t s;
  template <int D, template <int> class M, bool E>
  hipError_t operator()() {
    return launch_pooled_stats<64, M, E>(p, sums, s);
  }
};
}  // namespace

hipError_t run_pooled_stats(int model_id, const PooledStatsParams& p, double* sums, hipStream_t s) {
  const int d = p.d;
  if (d < 1 || d > 64) return hipErrorInvalidValue;
  PooledF f{p, sums, s};
  switch (model_id) {
    case AMH_MODEL_GAUSSIAN:
      return d == 64 ? f.template operator()<64, GaussianM, true>() : f.template operator()<64, GaussianM, false>();
    case AMH_MODEL_EIGHT_SCHOOLS:
      return f.template operator()<64, EightSchoolsM, false>();
    case AMH_MODEL_KIDIQ:
      return f.template operator()<64, KidiqM, false>();
    case AMH_MODEL_DIAMONDS:
      return f.template operator()<64, DiamondsM, false>();
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t run_pooled_update(const PooledUpdateParams& p, hipStream_t s) {
  if (p.d < 1 || p.d > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pooled_update_kernel, dim3(1), dim3(64), 0, s, p);
  return hipGetLastError();
}

}  // namespace amh
