// amh_big_pooled.hip -- pooled-covariance mode (regime B) for 64 < d <= 256
// (Gaussian, d % 32 == 0): BASELINE config 4's headline, d = 256 with one
// shared factor for 32,768 chains.
//
// With one shared L every per-chain product is a GEMM over chains, so the
// three O(d^2) pieces run on MFMA (v_mfma_f32_32x32x2_f32, a k-ordered fmaf
// chain -- bit-reproducible by the oracle):
//
//   pooled_big_propose_kernel  Z' = Z + e^lam (L Xi) + eps Xi for 64 chains
//                              per block; Xi drawn straight into LDS
//                              (arwmh.py:162-167), L read from L2
//   gauss_pot_mfma_kernel      U(Z') (amh_big.hip)
//   pooled_big_stats_kernel    accept (arwmh.py:173-178) and the chunk sums
//                              S_d, S_a and S_dd = sum delta delta^T, the
//                              latter as a K = chains MFMA over 32x32 tile
//                              pairs of the lower triangle
//   pooled_reduce_kernel       chunk partials -> sums (amh_pooled.hip)
//   pooled_big_update_kernel   Sigma' = (1-g) Sigma + g S_dd / N (double) and
//                              its blocked Cholesky factor (float32, 32-column
//                              panels, the matrix resident in LDS)
// Bit spec: oracle/amh_oracle.c, "pooled mode, large dimensions".
#include "amh_device.h"

namespace amh {

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kLd = 65;          // LDS row stride of [k][chain] tiles
constexpr int kBigChunk = 256;   // chains per stats block (bit spec)

__device__ __forceinline__ float rdlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int64_t pk(int d, int r, int k) { return col_off(d, k) + (r - k); }
}  // namespace

// ----------------------------------------------------------------- propose --
__global__ __launch_bounds__(256) void pooled_big_propose_kernel(PooledStatsParams p, float* xprop) {
  extern __shared__ float lds[];
  const int d = p.d;
  const int nt = d / 32;
  float* Xi = lds;
  float* Zt = lds + (size_t)d * kLd;
  const int32_t it = p.i[0];
  const float el = amh_expf(p.lam[0]);
  const int64_t c0 = (int64_t)blockIdx.x * 64;
  for (int idx = threadIdx.x; idx < 64 * d; idx += 256) {
    const int cc = idx / d, k = idx - cc * d;
    int64_t ch = c0 + cc;
    if (ch >= p.C) ch = p.C - 1;
    const amh_u32x4 o = amh_philox4x32_10((uint32_t)k, (uint32_t)it, 0u, AMH_TAG_STEP, p.keys[2 * ch],
                                          p.keys[2 * ch + 1]);
    Xi[k * kLd + cc] = amh_normal_from_bits(o.v[0]);
    Zt[k * kLd + cc] = p.z[ch * d + k];
  }
  __syncthreads();
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  const int h = lane >> 5, i = lane & 31;
  static_for<2>([&](auto I2) {
    const int tile = 2 * w + I2;
    if (tile < nt) {
      const int row = 32 * tile + i;
      f32x16 acc0 = f32x16{}, acc1 = f32x16{};
      for (int kk = 0; kk < 32 * (tile + 1); kk += 2) {
        const int col = kk + h;
        const float a = (row >= col) ? p.L[pk(d, row, col)] : 0.0f;
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Xi[col * kLd + i], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a, Xi[col * kLd + 32 + i], acc1, 0, 0, 0);
      }
      // z' in place of z: each (row, chain) is owned by exactly one lane
      static_for<16>([&](auto R) {
        const int rr = 32 * tile + (R & 3) + 8 * (R >> 2) + 4 * h;
        float* z0 = &Zt[rr * kLd + i];
        float* z1 = &Zt[rr * kLd + 32 + i];
        *z0 = *z0 + fmaf(el, acc0[(int)R], p.eps * Xi[rr * kLd + i]);
        *z1 = *z1 + fmaf(el, acc1[(int)R], p.eps * Xi[rr * kLd + 32 + i]);
      });
    }
  });
  __syncthreads();
  for (int idx = threadIdx.x; idx < 64 * d; idx += 256) {
    const int cc = idx / d, k = idx - cc * d;
    const int64_t ch = c0 + cc;
    if (ch < p.C) xprop[ch * d + k] = Zt[k * kLd + cc];
  }
}

// ------------------------------------------------------------------- stats --
// 8 waves; 36 (at d = 256) lower tile pairs (I >= J) of S_dd, wave w owns
// pairs w, w + 8, ...; the chunk's chains feed the MFMA K dimension in order.
__global__ __launch_bounds__(512) void pooled_big_stats_kernel(PooledStatsParams p, const float* xprop,
                                                               const float* pep) {
  extern __shared__ float lds[];
  const int d = p.d;
  const int nt = d / 32;
  const int npairs = nt * (nt + 1) / 2;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const int64_t V = d + P + 2;
  float* Dl = lds;                         // [d][kLd]
  int* flag = (int*)(lds + (size_t)d * kLd);  // [64]
  float* alph = lds + (size_t)d * kLd + 64;   // [64]
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane((int)(tid / 64));
  const int h = lane >> 5, i = lane & 31;
  const int32_t it = p.i[0];
  const int64_t base = (int64_t)blockIdx.x * kBigChunk;
  float sd = 0.0f, sa = 0.0f;
  int64_t cnt = 0;
  f32x16 acc[5];
  int pI[5], pJ[5];
  static_for<5>([&](auto S) {
    acc[S] = f32x16{};
    const int pp = w + 8 * S;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= pp) ++I;
    pI[S] = I;
    pJ[S] = pp - I * (I + 1) / 2;
  });
  for (int t = 0; t < kBigChunk / 64; ++t) {
    const int64_t c0 = base + 64 * t;
    const int64_t left = p.C - c0;
    if (left <= 0) break;
    const int nv = left < 64 ? (int)left : 64;
    if (tid < 64) {
      int acc_f = 0;
      float a = 0.0f;
      if (tid < nv) {
        const int64_t c = c0 + tid;
        const amh_u32x4 o = amh_philox4x32_10(0u, (uint32_t)it, 0u, AMH_TAG_STEP, p.keys[2 * c], p.keys[2 * c + 1]);
        const float u = amh_unif01_from_bits(o.v[1]);
        float pp = pep[c];
        if (amh_isnan(pp)) pp = INFINITY;
        const float pe = p.pe[c];
        const float ex = amh_expf(pe - pp);
        a = (ex > 1.0f) ? 1.0f : ex;
        acc_f = u < a;
        p.pe_out[c] = acc_f ? pp : pe;
      }
      flag[tid] = acc_f;
      alph[tid] = a;
    }
    __syncthreads();
    for (int idx = tid; idx < 64 * d; idx += 512) {
      const int cc = idx / d, k = idx - cc * d;
      float dv = 0.0f;
      if (cc < nv) {
        const int64_t c = c0 + cc;
        const float zn = flag[cc] ? xprop[c * d + k] : p.z[c * d + k];
        p.z_out[c * d + k] = zn;
        dv = zn - p.mu[k];
      }
      Dl[k * kLd + cc] = dv;
    }
    __syncthreads();
    if (tid < d) {
      for (int c = 0; c < nv; ++c) sd = sd + Dl[tid * kLd + c];
    }
    if (tid == 511) {
      for (int c = 0; c < nv; ++c) sa = sa + alph[c];
    }
    cnt += nv;
    static_for<5>([&](auto S) {
      if (w + 8 * S < npairs) {
        const int ra = (32 * pI[S] + i) * kLd, rb = (32 * pJ[S] + i) * kLd;
        for (int kk = 0; kk < nv; kk += 2) {
          acc[S] = __builtin_amdgcn_mfma_f32_32x32x2f32(Dl[ra + kk + h], Dl[rb + kk + h], acc[S], 0, 0, 0);
        }
      }
    });
    __syncthreads();
  }
  double* out = p.partials + (int64_t)blockIdx.x * V;
  if (tid < d) out[tid] = (double)sd;
  if (tid == 511) {
    out[d + P] = (double)sa;
    out[d + P + 1] = (double)cnt;
  }
  static_for<5>([&](auto S) {
    if (w + 8 * S < npairs) {
      static_for<16>([&](auto R) {
        const int row = 32 * pI[S] + (R & 3) + 8 * (R >> 2) + 4 * h;
        const int col = 32 * pJ[S] + i;
        if (row >= col) out[d + pk(d, row, col)] = (double)acc[S][(int)R];
      });
    }
  });
}

// ------------------------------------------------------------------ update --
__global__ __launch_bounds__(1024) void pooled_big_update_kernel(PooledUpdateParams p) {
  extern __shared__ float A[];  // packed lower, column-major, float32
  const int d = p.d;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  __shared__ int okv;
  __shared__ float rowpart[256];
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane((int)(tid / 64));
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
  const double g = (double)gamma;
  for (int64_t o = tid; o < P; o += 1024) {
    const double a = (1.0 - g) * p.in.cov[o];
    const double b = g * (sums[d + o] / N);
    A[o] = (float)(a + b);
  }
  if (tid == 0) okv = 1;
  __syncthreads();
  for (int p0 = 0; p0 < d; p0 += 32) {
    // (1) diagonal block: wave 0, lane i < 32 holds row p0 + i
    if (w == 0) {
      const int ii = lane & 31;
      float a[32];
      static_for<32>([&](auto K) { a[K] = (K <= ii) ? A[pk(d, p0 + ii, p0 + K)] : 0.0f; });
      bool ok = true;
      static_for<32>([&](auto K) {
        constexpr int k = K;
        const float piv = rdlane(a[k], k);
        ok = ok && (piv > 0.0f) && amh_isfinite(piv);
        const float ljj = sqrtf(piv);
        if (ii > k) a[k] = a[k] / ljj;
        if (ii == k) a[k] = ljj;
        static_for<32>([&](auto M) {
          constexpr int m = M;
          if constexpr (m > k) {
            const float lmk = rdlane(a[k], m);
            if (ii >= m) a[m] = fmaf(-a[k], lmk, a[m]);
          }
        });
      });
      if (lane < 32) static_for<32>([&](auto K) { if (K <= ii) A[pk(d, p0 + ii, p0 + K)] = a[K]; });
      if (lane == 0 && !ok) okv = 0;
    }
    __syncthreads();
    // (2) panel below the block: one thread per row
    const int q0 = p0 + 32;
    if (tid < d - q0) {
      const int r = q0 + tid;
      float a[32];
      static_for<32>([&](auto K) { a[K] = A[pk(d, r, p0 + K)]; });
      static_for<32>([&](auto K) {
        constexpr int k = K;
        const float lrk = a[k] / A[pk(d, p0 + k, p0 + k)];
        a[k] = lrk;
        static_for<32>([&](auto M) {
          constexpr int m = M;
          if constexpr (m > k) a[m] = fmaf(-lrk, A[pk(d, p0 + m, p0 + k)], a[m]);
        });
      });
      static_for<32>([&](auto K) { A[pk(d, r, p0 + K)] = a[K]; });
    }
    __syncthreads();
    // (3) trailing update with the panel's 32 columns, 4x4 element tiles
    const int nb = (d - q0) / 4;
    for (int tix = tid; tix < nb * (nb + 1) / 2; tix += 1024) {
      int R = 0;
      while ((R + 1) * (R + 2) / 2 <= tix) ++R;
      const int Cb = tix - R * (R + 1) / 2;
      const int r0 = q0 + 4 * R, c0 = q0 + 4 * Cb;
      float t[4][4];
      static_for<4>([&](auto X) {
        static_for<4>([&](auto Y) {
          const int r = r0 + X, c = c0 + Y;
          t[X][Y] = (c <= r) ? A[pk(d, r, c)] : 0.0f;
        });
      });
      for (int j = 0; j < 32; ++j) {
        const int64_t cj = col_off(d, p0 + j) - (p0 + j);
        float lr[4], lc[4];
        static_for<4>([&](auto X) {
          lr[X] = A[cj + r0 + X];
          lc[X] = A[cj + c0 + X];
        });
        static_for<4>([&](auto X) {
          static_for<4>([&](auto Y) { t[X][Y] = fmaf(-lr[X], lc[Y], t[X][Y]); });
        });
      }
      static_for<4>([&](auto X) {
        static_for<4>([&](auto Y) {
          const int r = r0 + X, c = c0 + Y;
          if (c <= r) A[pk(d, r, c)] = t[X][Y];
        });
      });
    }
    __syncthreads();
  }
  const bool ok = okv != 0;
  const float e0 = amh_expf(lam), e1 = amh_expf(lamn);
  if (tid < d) {
    const int r = tid;
    float s = 0.0f;
    for (int j = 0; j <= r; ++j) {
      const int64_t o = pk(d, r, j);
      const float lo = p.in.scale[o];
      const float ln = ok ? A[o] : lo;
      const float tt = (ln * e1) - (lo * e0);
      s = fmaf(tt, tt, s);
    }
    rowpart[r] = s;
  }
  __syncthreads();
  if (w == 0) {
    float sl[4];
    static_for<4>([&](auto K) { sl[K] = Grp<64>::sum((64 * K + lane < d) ? rowpart[64 * K + lane] : 0.0f); });
    const float asc = sqrtf((sl[0] + sl[1]) + (sl[2] + sl[3]));
    if (lane == 0) {
      p.out.i[0] = itr;
      p.out.mean_accept_prob[0] = maccn;
      p.out.log_step_size[0] = lamn;
      p.out.as_change[0] = asc;
    }
  }
  if (tid < d) p.out.loc[tid] = p.in.loc[tid] + gamma * (float)(sums[tid] / N);
  for (int64_t o = tid; o < P; o += 1024) {
    if (ok) {
      const double a = (1.0 - g) * p.in.cov[o];
      const double b = g * (sums[d + o] / N);
      p.out.cov[o] = a + b;
      p.out.scale[o] = A[o];
    } else {
      p.out.cov[o] = p.in.cov[o];
      p.out.scale[o] = p.in.scale[o];
    }
  }
}

// --------------------------------------------------------------- launchers --
hipError_t pooled_reduce(const double* partials, int64_t n_chunks, int64_t V, double* sums, hipStream_t s);

int64_t pooled_big_chunks(int64_t C) { return (C + kBigChunk - 1) / kBigChunk; }

hipError_t run_pooled_big_stats(const PooledStatsParams& p, float* xprop, float* pep, double* sums, hipStream_t s) {
  const int d = p.d;
  const int64_t V = d + (int64_t)d * (d + 1) / 2 + 2;
  hipLaunchKernelGGL(pooled_big_propose_kernel, dim3((unsigned)((p.C + 63) / 64)), dim3(256),
                     (size_t)2 * d * kLd * sizeof(float), s, p, xprop);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  PotParams q{xprop, pep, p.C, d, p.model};
  e = run_big_potential(q, s);
  if (e != hipSuccess) return e;
  const int64_t nch = pooled_big_chunks(p.C);
  hipLaunchKernelGGL(pooled_big_stats_kernel, dim3((unsigned)nch), dim3(512),
                     ((size_t)d * kLd + 128) * sizeof(float), s, p, (const float*)xprop, (const float*)pep);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  return pooled_reduce(p.partials, nch, V, sums, s);
}

hipError_t run_pooled_big_update(const PooledUpdateParams& p, hipStream_t s) {
  const size_t shm = (size_t)p.d * (p.d + 1) / 2 * sizeof(float);
  hipLaunchKernelGGL(pooled_big_update_kernel, dim3(1), dim3(1024), shm, s, p);
  return hipGetLastError();
}

}  // namespace amh
