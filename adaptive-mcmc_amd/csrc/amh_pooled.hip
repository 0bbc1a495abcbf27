// amh_pooled.hip -- pooled-covariance adaptation (regime B, include/amh.h):
// every chain proposes with one shared (mu, L, lambda); the adaptation of
// arwmh.py:180-197 consumes the statistics of all chains.
//
//   pooled_stats_kernel   per-chain transition (arwmh.py:162-178 with the
//                         shared factor staged in LDS) + the chunk's sums
//                         S_d, S_dd, S_a (float32 per wave over its chains,
//                         double across the chunk's waves)
//   pooled_reduce_kernel  chunk partials -> this rank's sums (double, fixed
//                         two-level order); ranks then all-reduce them (RCCL)
//   pooled_update_kernel  mu, Sigma, lambda, mean-accept update and the
//                         Cholesky refactorisation of Sigma' (one wave, rows
//                         in registers, columns broadcast through LDS, double)
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
  f32x2v y01 = {0.0f, 0.0f}, y23 = {0.0f, 0.0f};
  static_for<4>([&](auto B) {
    constexpr int b = B;
    if (16 * b < d) {
      f32x4 pv[4];
      static_for<4>([&](auto Q) {
        pv[Q] = (4 * (4 * b + Q) < d) ? lds_ld4<16 * (4 * b + Q)>(prow) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
      });
      lds_wait(pv[0], pv[1], pv[2], pv[3]);
      // columns (j, j+1) through one v_pk_fma_f32 into accumulators (j mod 4,
      // j+1 mod 4); a column past d adds 0 * 0 (padded row, inactive lane)
      static_for<8>([&](auto K2) {
        constexpr int j = 16 * b + 2 * K2;
        if (j < d) {
          const f32x4 q = pv[K2 / 2];
          const f32x2v pp = (K2 % 2 == 0) ? f32x2v{q[0], q[1]} : f32x2v{q[2], q[3]};
          const f32x2v pa = act ? pp : f32x2v{0.0f, 0.0f};
          const f32x2v bp = {Gp::template bcast<j>(v), Gp::template bcast<j + 1>(v)};
          if constexpr (K2 % 2 == 0) {
            y01 = __builtin_elementwise_fma(pa, bp, y01);
          } else {
            y23 = __builtin_elementwise_fma(pa, bp, y23);
          }
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    }
  });
  return (y01[0] + y01[1]) + (y23[0] + y23[1]);
}

__host__ __device__ inline int pooled_ld(int d) { return ((d + 3) & ~3) + 4; }

template <template <int> class M>
__host__ __device__ inline size_t pooled_lds_model_floats(const ModelArgs& m, int d) {
  return (M<64>::lds_bytes(m, d) / sizeof(float) + 3) & ~(size_t)3;
}
// combine-tree slot: rows r = 0..63 as [S_r0 .. S_rr, sd_r], then sa
constexpr int kTreeSlot = 64 * 65 / 2 + 64 + 1;

template <template <int> class M>
__host__ __device__ inline size_t pooled_lds_bytes(const ModelArgs& m, int d) {
  const size_t f = pooled_lds_model_floats<M>(m, d) + (size_t)d * pooled_ld(d);
  return (f + (size_t)(kPoolWaves / 2) * kTreeSlot) * sizeof(float);
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
  float* tree = lrow + (size_t)d * ld;

  M<G>::stage(lds, p.model, d);
  for (int k = threadIdx.x; k < d * ld; k += blockDim.x) {
    const int row = k / ld, col = k - row * ld;
    lrow[k] = (col <= row && col < d) ? p.L[col_off(d, col) + (row - col)] : 0.0f;
  }
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
  // this wave's chains [base, end); the next chain's z / pe / key are loaded
  // while the current one is computed
  // (buffer descriptors with a wave-uniform base: no 64-bit per-lane
  // addresses to keep live, lanes r >= d read 0 / store nothing)
  const int64_t end = (base + cpw < p.C) ? base + cpw : p.C;
  const uint32_t vr = 4u * (uint32_t)r;
  auto load_chain = [&](int64_t c, float& zz, float& pp, uint32_t& q0, uint32_t& q1) {
    const Buf bz(uniform_ptr(p.z + c * d), 4u * (uint32_t)d);
    zz = bz.ld(vr, 0);
    pp = p.pe[c];
    q0 = p.keys[2 * c];
    q1 = p.keys[2 * c + 1];
  };
  float zq = 0.0f, peq = 0.0f;
  uint32_t k0q = 0, k1q = 0;
  if (base < end) load_chain(base, zq, peq, k0q, k1q);
  const int K = p.k_steps;
  for (int64_t c = base; c < end; ++c) {
    float z = zq, pe = peq;
    const uint32_t k0 = k0q, k1 = k1q;
    if (c + 1 < end) load_chain(c + 1, zq, peq, k0q, k1q);
    // K transitions with the frozen shared state (K = 1: one pooled step)
    for (int t = 0; t < K; ++t) {
      // noise at the shared stream position i + t (arwmh.py:162-165, 174)
      float xi, u;
      step_noise<G>(r, d, (uint32_t)(it + t), k0, k1, xi, u);
      xi = act ? xi : 0.0f;
      // proposal with the shared factor (arwmh.py:166-167)
      const float acc = lds_row_dot64(prow, d, xi, act);
      const float zp = act ? z + fmaf(el, acc, p.eps * xi) : 0.0f;
      float pep = M<G>::potential(zp, r, d, mctx, lds);
      if (amh_isnan(pep)) pep = INFINITY;
      const float ex = amh_expf(pe - pep);
      const float alpha = (ex > 1.0f) ? 1.0f : ex;
      const bool accept = u < alpha;
      z = accept ? zp : z;
      pe = accept ? pep : pe;
      // pooled statistics (float32 over this wave's chain-steps: chains in
      // order, each chain's K steps in order)
      const float delta = act ? z - mu : 0.0f;
      sd = sd + delta;
      // (S_k, S_k+1) += delta_r (delta_k, delta_k+1): one v_pk_fma_f32 per pair
      // (each half is the same fmaf; past d the broadcast delta is 0)
      static_for<32>([&](auto K2) {
        constexpr int k = 2 * K2;
        if (k < d) {
          const f32x2v bp = {Gp::template bcast<k>(delta), Gp::template bcast<k + 1>(delta)};
          const f32x2v sp = __builtin_elementwise_fma(f32x2v{delta, delta}, bp, f32x2v{S[k], S[k + 1]});
          S[k] = sp[0];
          S[k + 1] = sp[1];
        }
        column_fence<k + 1>();
      });
      sa = sa + alpha;
    }
    const Buf bo(uniform_ptr(p.z_out + c * d), 4u * (uint32_t)d);
    bo.st(z, vr, 0);
    if (r == 0) p.pe_out[c] = pe;
  }
  // The chunk's 16 wave partials are combined by a fixed pairwise tree in
  // float32 (h = 8, 4, 2, 1: wave w < h adds wave w + h), through LDS slots
  // holding each row r as [S_r0 .. S_rr, sd_r] (row offset r(r+3)/2) and sa
  // last; the chunk total is then written in double (oracle mirror).
  const uint32_t rowoff = (uint32_t)(r * (r + 3) / 2);
  static_for<4>([&](auto H) {
    constexpr int h = 8 >> H;
    if (w >= h && w < 2 * h) {
      float* slot = tree + (size_t)(w - h) * kTreeSlot;
      if (act) {
        static_for<64>([&](auto K) {
          constexpr int k = K;
          if (k <= r) slot[rowoff + k] = S[k];
        });
        slot[rowoff + r + 1] = sd;
      }
      if (lane == 0) slot[kTreeSlot - 1] = sa;
    }
    __syncthreads();
    if (w < h) {
      const float* slot = tree + (size_t)w * kTreeSlot;
      if (act) {
        static_for<64>([&](auto K) {
          constexpr int k = K;
          if (k <= r) S[k] = S[k] + slot[rowoff + k];
        });
        sd = sd + slot[rowoff + r + 1];
      }
      sa = sa + slot[kTreeSlot - 1];
    }
    __syncthreads();
  });
  if (w == 0) {
    double* out = p.partials + (int64_t)blockIdx.x * V;
    if (act) {
      static_for<64>([&](auto K) {
        constexpr int k = K;
        if (k <= r) out[d + col_off(d, k) + (r - k)] = (double)S[k];
      });
      out[r] = (double)sd;
    }
    if (lane == 0) {
      const int64_t left = p.C - chunk0;
      out[d + P] = (double)sa;
      out[d + P + 1] = (double)K * (double)(left < (int64_t)kPoolWaves * cpw ? left : (int64_t)kPoolWaves * cpw);
    }
  }
}

// Chunk partials -> sums, in a fixed two-level order (oracle mirror):
// groups of kRedGroup consecutive chunks are summed in chunk order, then the
// group sums in group order.  Two launches, each with a thread per (group, v)
// or per v: pooled_group_kernel writes the group sums after the partials
// (the scratch holds n_chunks + n_groups rows of V doubles), and
// pooled_final_kernel adds them in group order.
constexpr int kRedGroup = 16;

// T = float: the large-d stats kernel's partials, which are float32 sums
// (their conversion to double is exact, so storing them as float halves the
// traffic and changes no bit)
template <typename T>
__global__ __launch_bounds__(256) void pooled_group_kernel(const T* __restrict__ partials, int64_t n_chunks,
                                                           int64_t V, double* __restrict__ gsum) {
  const int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t g = blockIdx.y;
  if (v >= V) return;
  const int64_t c1 = (g + 1) * kRedGroup < n_chunks ? (g + 1) * kRedGroup : n_chunks;
  double x[kRedGroup];
#pragma unroll
  for (int q = 0; q < kRedGroup; ++q) x[q] = (g * kRedGroup + q < c1) ? (double)partials[(g * kRedGroup + q) * V + v] : 0.0;
  double s = 0.0;  // chunk order; a missing tail chunk adds nothing (it is not added at all)
#pragma unroll
  for (int q = 0; q < kRedGroup; ++q)
    if (g * kRedGroup + q < c1) s += x[q];
  gsum[g * V + v] = s;
}

__global__ __launch_bounds__(256) void pooled_final_kernel(const double* __restrict__ gsum, int64_t n_groups, int64_t V,
                                                           double* sums, int accumulate, int tile_d, FinalPrep fp) {
  const int64_t u = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (u >= V) return;
  if (tile_d && tile_to_packed(u, V, tile_d) < 0) return;
  double tot = 0.0;
  int64_t g = 0;
  for (; g + 32 <= n_groups; g += 32) {  // 32 loads in flight, adds in group order
    double x[32];
#pragma unroll
    for (int q = 0; q < 32; ++q) x[q] = gsum[(g + q) * V + u];
#pragma unroll
    for (int q = 0; q < 32; ++q) tot += x[q];
  }
  for (; g + 8 <= n_groups; g += 8) {
    double x[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) x[q] = gsum[(g + q) * V + u];
#pragma unroll
    for (int q = 0; q < 8; ++q) tot += x[q];
  }
  for (; g < n_groups; ++g) tot += gsum[g * V + u];
  final_entry(u, tot, V, sums, accumulate, tile_d, fp);
}

int64_t pooled_scratch_rows(int64_t n_chunks) { return n_chunks + (n_chunks + kRedGroup - 1) / kRedGroup; }

// d < 64: double partial rows, two launches (group sums, then the groups);
// d >= 64 reduces its float32 tile rows in one launch
// (amh_big_pooled.hip, pooled_reduce_tiles_kernel)
hipError_t pooled_reduce(const double* partials, int64_t n_chunks, int64_t V, double* sums, int accumulate,
                         hipStream_t s, int tile_d = 0, FinalPrep fp = FinalPrep{}) {
  const int64_t n_groups = (n_chunks + kRedGroup - 1) / kRedGroup;
  double* gsum = const_cast<double*>(partials) + n_chunks * V;
  const unsigned vb = (unsigned)((V + 255) / 256);
  hipLaunchKernelGGL(pooled_group_kernel<double>, dim3(vb, (unsigned)n_groups), dim3(256), 0, s, partials,
                     n_chunks, V, gsum);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(pooled_final_kernel, dim3(vb), dim3(256), 0, s, (const double*)gsum, n_groups, V, sums,
                     accumulate, tile_d, fp);
  return hipGetLastError();
}

namespace {
__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(unsigned)(b & 0xffffffffLL), lane);
  const int hi = __builtin_amdgcn_readlane((int)(unsigned)((unsigned long long)b >> 32), lane);
  return __longlong_as_double(((long long)(unsigned)hi << 32) | (unsigned)lo);
}
}  // namespace

// 8 waves move the packed matrices between HBM and LDS with coalesced
// column accesses; wave 0 holds row r of Sigma' (double) in lane r and
// factors it in registers (right-looking; element (r, k) is updated in column
// order, oracle mirror).
constexpr int kUpdLd = 65;  // LDS row stride of the [r][k] staging arrays

__global__ __launch_bounds__(512) void pooled_update_kernel(PooledUpdateParams p) {
  const int d = p.d;
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane(tid / 64);
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const double* sums = p.sums;
  const double N = sums[d + P + 1];
  const int32_t it = p.in.i[0];
  const int32_t itr = it + p.K;
  const int32_t n = pooled_block_n(it, p.W, p.K);
  const float gamma = amh_lr_gamma(n, p.a);
  const double g = (double)gamma;
  __shared__ double As[64 * kUpdLd];  // Sigma' [r][k], then the new factor (float view)
  __shared__ float Los[64 * kUpdLd];  // old factor [r][k]
  __shared__ int okv;

  // (1) Sigma' = (1-g) Sigma + g S_dd / N and the old factor into LDS;
  // wave w takes columns w, w + 8, ..; lane = row offset
  for (int k = w; k < d; k += 8) {
    const int r = k + lane;
    if (r < d) {
      const int64_t o = col_off(d, k) + (r - k);
      const double a = (1.0 - g) * p.in.cov[o];
      const double b = g * (sums[d + o] / N);
      As[r * kUpdLd + k] = a + b;
      Los[r * kUpdLd + k] = p.in.scale[o];
    }
  }
  __syncthreads();

  if (w == 0) {
    const int r = lane;
    const bool act = r < d;
    const float macc = p.in.mean_accept_prob[0];
    const float lam = p.in.log_step_size[0];
    const float abar = (float)(sums[d + P] / N);
    const float maccn = macc + (abar - macc) / (float)n;
    const float lamn = lam + gamma * (abar - p.target);
    const float mun = act ? p.in.loc[r] + gamma * (float)(sums[r] / N) : 0.0f;
    double A[64];
    static_for<64>([&](auto K) {
      constexpr int k = K;
      A[k] = (k < d && act && k <= r) ? As[r * kUpdLd + k] : 0.0;
    });
    // Right-looking Cholesky, lane r = row r, in registers.  Column j goes
    // through LDS once and is read back as 16-B broadcasts; the entries above
    // the diagonal are updated too (never used), so no lane masks.
    __shared__ __attribute__((aligned(16))) double colb[64];
    bool ok = true;
    static_for<64>([&](auto J) {
      constexpr int j = J;
      if (j < d) {
        const double piv = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(A[j]), j),
                                            __builtin_amdgcn_readlane(__double2loint(A[j]), j));
        ok = ok && (piv > 0.0) && __builtin_isfinite(piv);
        const double ljj = sqrt(piv);
        const double lrj = A[j] / ljj;
        A[j] = (r == j) ? ljj : lrj;
        colb[r] = lrj;
        // columns k >= d are updated with garbage and never read: no branches
        static_for<(64 - ((j + 1) & ~1)) / 2>([&](auto Q) {
          constexpr int k0 = ((j + 1) & ~1) + 2 * Q;
          typedef double f64x2 __attribute__((ext_vector_type(2)));
          const f64x2 v = *(const f64x2*)&colb[k0];
          if constexpr (k0 > j) A[k0] = fma(-lrj, v[0], A[k0]);
          A[k0 + 1] = fma(-lrj, v[1], A[k0 + 1]);
        });
        asm volatile("" ::: "memory");
      }
    });
    const float e0 = amh_expf(lam), e1 = amh_expf(lamn);
    float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    float* Lns = (float*)As;  // the new factor, float [r][k] (row r's doubles are already in registers)
    static_for<64>([&](auto J) {
      constexpr int j = J;
      if (j < d) {
        const float lo = (j <= r && act) ? Los[r * kUpdLd + j] : 0.0f;
        const float ln = ok ? (float)A[j] : lo;
        const float tt = (j <= r && act) ? (ln * e1) - (lo * e0) : 0.0f;
        s4[j & 3] = fmaf(tt, tt, s4[j & 3]);
      }
    });
    const float part = act ? (s4[0] + s4[1]) + (s4[2] + s4[3]) : 0.0f;
    const float asc = sqrtf(Grp<64>::sum(part));
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_wave_barrier();
    static_for<64>([&](auto K) {
      constexpr int k = K;
      if (k < d && act && k <= r) Lns[r * kUpdLd + k] = (float)A[k];
    });
    if (act) p.out.loc[r] = mun;
    if (r == 0) {
      okv = ok ? 1 : 0;
      p.out.i[0] = itr;
      p.out.mean_accept_prob[0] = maccn;
      p.out.log_step_size[0] = lamn;
      p.out.as_change[0] = asc;
    }
  }
  __syncthreads();

  // (3) write-out by column (in-place safe: every element is read and written
  // by the same thread)
  const bool ok = okv != 0;
  const float* Lns = (const float*)As;
  for (int k = w; k < d; k += 8) {
    const int r = k + lane;
    if (r < d) {
      const int64_t o = col_off(d, k) + (r - k);
      if (ok) {
        const double a = (1.0 - g) * p.in.cov[o];
        const double b = g * (sums[d + o] / N);
        p.out.cov[o] = a + b;
        p.out.scale[o] = Lns[r * kUpdLd + k];
      } else {  // kept (rare: gamma = 1 at n = 1, or Sigma' not positive definite)
        p.out.cov[o] = p.in.cov[o];
        p.out.scale[o] = Los[r * kUpdLd + k];
      }
    }
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
  return pooled_reduce(p.partials, n_chunks, V, sums, 0, s);
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
    case AMH_MODEL_DIAMONDS_SS:
      if (d < 3 || d > 32) return hipErrorInvalidValue;
      return f.template operator()<64, DiamondsSSM, false>();
    default:
      return hipErrorInvalidValue;
  }
}

hipError_t run_pooled_update(const PooledUpdateParams& p, hipStream_t s) {
  if (p.d < 1 || p.d > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pooled_update_kernel, dim3(1), dim3(512), 0, s, p);
  return hipGetLastError();
}

}  // namespace amh
