// amh_eval.hip -- sample-quality metrics of the reference's evaluation
// (python/utils/evaluation.py:223-294) on gfx950: the Gaussian-kernel sums
// behind mmd2_unbiased / mmd_heuristic and the pairwise squared distances
// behind the median bandwidth heuristic.
//
//   kernel_sum_kernel  sum_{i,j} exp(-gamma ||a_i - b_j||^2) over a 128 x 128
//                      pair tile per block: both point tiles staged in LDS
//                      column-major ([k][i], 32 coordinates per stage), each
//                      thread accumulates an 8 x 8 block of squared
//                      distances with direct differences (the reference's
//                      ((x - y)^2).sum(-1), no |x|^2 + |y|^2 - 2 x.y
//                      cancellation), then exp and a fixed-order reduction to
//                      one double per block; a second kernel adds the block
//                      partials in block order.  The sum is deterministic.
//   dist2_kernel       the same tiles, writing ||a_i - b_j||^2 to [n][m].
//
// Bound: VALU.  3 FLOP per pair-coordinate plus one exp per pair; at
// n = m = 10^4, d = 26 that is 7.8 GFLOP per kernel sum.
#include "amh_device.h"

namespace amh {

namespace {
constexpr int kTile = 128;  // points per tile side
constexpr int kKc = 32;     // coordinates staged per pass
constexpr int kTLd = kTile + 4;

// squared distances of this thread's 8 x 8 pairs, tile rows a0.., b0..
__device__ __forceinline__ void tile_dist2(const float* A, int64_t n, const float* B, int64_t m, int d, int64_t a0,
                                           int64_t b0, float (&acc)[8][8], float* As, float* Bs) {
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  static_for<8>([&](auto X) { static_for<8>([&](auto Y) { acc[X][Y] = 0.0f; }); });
  for (int k0 = 0; k0 < d; k0 += kKc) {
    __syncthreads();
    for (int idx = threadIdx.x; idx < kTile * kKc; idx += 256) {
      const int i = idx / kKc, k = idx - i * kKc;
      const bool kin = k0 + k < d;
      As[k * kTLd + i] = (kin && a0 + i < n) ? A[(a0 + i) * d + k0 + k] : 0.0f;
      Bs[k * kTLd + i] = (kin && b0 + i < m) ? B[(b0 + i) * d + k0 + k] : 0.0f;
    }
    __syncthreads();
    const int kn = (d - k0 < kKc) ? d - k0 : kKc;
    for (int k = 0; k < kn; ++k) {
      const f32x4 a_lo = *(const f32x4*)&As[k * kTLd + ty * 8];
      const f32x4 a_hi = *(const f32x4*)&As[k * kTLd + ty * 8 + 4];
      const f32x4 b_lo = *(const f32x4*)&Bs[k * kTLd + tx * 8];
      const f32x4 b_hi = *(const f32x4*)&Bs[k * kTLd + tx * 8 + 4];
      const float a[8] = {a_lo[0], a_lo[1], a_lo[2], a_lo[3], a_hi[0], a_hi[1], a_hi[2], a_hi[3]};
      const float b[8] = {b_lo[0], b_lo[1], b_lo[2], b_lo[3], b_hi[0], b_hi[1], b_hi[2], b_hi[3]};
      static_for<8>([&](auto X) {
        static_for<8>([&](auto Y) {
          const float df = a[X] - b[Y];
          acc[X][Y] = fmaf(df, df, acc[X][Y]);
        });
      });
    }
  }
}
}  // namespace

__global__ __launch_bounds__(256) void kernel_sum_kernel(const float* __restrict__ A, int64_t n,
                                                         const float* __restrict__ B, int64_t m, int d, float gamma,
                                                         int skip_diag, double* __restrict__ partials) {
  __shared__ __attribute__((aligned(16))) float As[kKc * kTLd];
  __shared__ __attribute__((aligned(16))) float Bs[kKc * kTLd];
  __shared__ double red[256];
  const int64_t a0 = (int64_t)blockIdx.y * kTile, b0 = (int64_t)blockIdx.x * kTile;
  float acc[8][8];
  tile_dist2(A, n, B, m, d, a0, b0, acc, As, Bs);
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  float s = 0.0f;
  static_for<8>([&](auto X) {
    static_for<8>([&](auto Y) {
      const int64_t i = a0 + ty * 8 + X, j = b0 + tx * 8 + Y;
      const bool valid = i < n && j < m && !(skip_diag && i == j);
      const float e = amh_expf(-gamma * acc[X][Y]);
      s += valid ? e : 0.0f;
    });
  });
  red[threadIdx.x] = (double)s;
  __syncthreads();
  for (int h = 128; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) partials[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = red[0];
}

__global__ __launch_bounds__(1024) void ordered_sum_kernel(const double* __restrict__ partials, int64_t nb,
                                                           double* __restrict__ out) {
  __shared__ double red[1024];
  double s = 0.0;
  for (int64_t b = threadIdx.x; b < nb; b += 1024) s += partials[b];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int h = 512; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = red[0];
}

__global__ __launch_bounds__(256) void dist2_kernel(const float* __restrict__ A, int64_t n,
                                                    const float* __restrict__ B, int64_t m, int d,
                                                    float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float As[kKc * kTLd];
  __shared__ __attribute__((aligned(16))) float Bs[kKc * kTLd];
  const int64_t a0 = (int64_t)blockIdx.y * kTile, b0 = (int64_t)blockIdx.x * kTile;
  float acc[8][8];
  tile_dist2(A, n, B, m, d, a0, b0, acc, As, Bs);
  const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
  static_for<8>([&](auto X) {
    const int64_t i = a0 + ty * 8 + X;
    if (i < n) {
      static_for<8>([&](auto Y) {
        const int64_t j = b0 + tx * 8 + Y;
        if (j < m) out[i * m + j] = acc[X][Y];
      });
    }
  });
}

// out[i] = N(0, 1) from Philox(i, i >> 32, 0, AMH_TAG_EVAL) word 0 (the
// random directions of max_sliced_wasserstein, evaluation.py:189-190)
__global__ void normals_kernel(uint32_t k0, uint32_t k1, int64_t n, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const amh_u32x4 o = amh_philox4x32_10((uint32_t)i, (uint32_t)((uint64_t)i >> 32), 0u, AMH_TAG_EVAL, k0, k1);
  out[i] = amh_normal_from_bits(o.v[0]);
}

hipError_t run_normals(uint32_t k0, uint32_t k1, int64_t n, float* out, hipStream_t s) {
  hipLaunchKernelGGL(normals_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, k0, k1, n, out);
  return hipGetLastError();
}

int64_t kernel_sum_blocks(int64_t n, int64_t m) { return ((n + kTile - 1) / kTile) * ((m + kTile - 1) / kTile); }

hipError_t run_kernel_sum(const float* A, int64_t n, const float* B, int64_t m, int d, float gamma, int skip_diag,
                          double* partials, double* out, hipStream_t s) {
  const dim3 grid((unsigned)((m + kTile - 1) / kTile), (unsigned)((n + kTile - 1) / kTile));
  hipLaunchKernelGGL(kernel_sum_kernel, grid, dim3(256), 0, s, A, n, B, m, d, gamma, skip_diag, partials);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(ordered_sum_kernel, dim3(1), dim3(1024), 0, s, (const double*)partials,
                     kernel_sum_blocks(n, m), out);
  return hipGetLastError();
}

hipError_t run_dist2(const float* A, int64_t n, const float* B, int64_t m, int d, float* out, hipStream_t s) {
  const dim3 grid((unsigned)((m + kTile - 1) / kTile), (unsigned)((n + kTile - 1) / kTile));
  hipLaunchKernelGGL(dist2_kernel, grid, dim3(256), 0, s, A, n, B, m, d, out);
  return hipGetLastError();
}

// ------------------------------------------------------------- Sinkhorn --
// One half-iteration of log-domain Sinkhorn (the solver behind the
// reference's wasserstein_sinkhorn, evaluation.py:69-101, ott-jax
// linear.solve): for every row i of the cost matrix C [rows][cols]
//   out_i = -eps * log sum_j exp((pot_j - C_ij) / eps + log_w)
// (uniform weights w = 1 / cols).  One 256-thread block per row streams the
// row once (coalesced) with a running (max, sum) per thread, then combines the
// pairs across the block.  The column half runs on the transposed matrix.
// Bound: HBM (4 bytes of C per element, one exp each).
__global__ __launch_bounds__(256) void lse_rows_kernel(const float* __restrict__ Cm, int64_t rows, int64_t cols,
                                                       const float* __restrict__ pot, float logw, float eps,
                                                       float* __restrict__ out) {
  const int64_t i = blockIdx.x;
  if (i >= rows) return;
  const float* row = Cm + i * cols;
  float mx = -INFINITY, sm = 0.0f;
  for (int64_t j = threadIdx.x; j < cols; j += 256) {
    const float a = (pot[j] - row[j]) / eps + logw;
    if (a > mx) {
      sm = sm * expf(mx - a) + 1.0f;
      mx = a;
    } else {
      sm += expf(a - mx);
    }
  }
  // combine (max, sum) pairs: lanes of the wave, then the four waves
  for (int off = 32; off >= 1; off >>= 1) {
    const float om = __shfl_xor(mx, off, 64);
    const float os = __shfl_xor(sm, off, 64);
    const float nm = fmaxf(mx, om);
    sm = (nm == -INFINITY) ? 0.0f : sm * expf(mx - nm) + os * expf(om - nm);
    mx = nm;
  }
  __shared__ float wm[4], wsum[4];
  if ((threadIdx.x & 63) == 0) {
    wm[threadIdx.x >> 6] = mx;
    wsum[threadIdx.x >> 6] = sm;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = wm[0], S = wsum[0];
    for (int k = 1; k < 4; ++k) {
      const float nm = fmaxf(M, wm[k]);
      S = (nm == -INFINITY) ? 0.0f : S * expf(M - nm) + wsum[k] * expf(wm[k] - nm);
      M = nm;
    }
    out[i] = -eps * (M + logf(S));
  }
}

hipError_t run_lse_rows(const float* Cm, int64_t rows, int64_t cols, const float* pot, float logw, float eps,
                        float* out, hipStream_t s) {
  hipLaunchKernelGGL(lse_rows_kernel, dim3((unsigned)rows), dim3(256), 0, s, Cm, rows, cols, pot, logw, eps, out);
  return hipGetLastError();
}

}  // namespace amh
