// membw.hip -- achievable HBM bandwidth on this MI355X for the access shapes
// of the d = 64 step kernel (tools/membw; diagnostic, not part of libamh):
//   read-only, write-only and copy streams of 580 MB (the headline's state in
//   each direction), 16 B per lane, plain and nt cache policy, 1..4 loads in
//   flight per lane.  Prints GB/s per variant (best of 20 launches).
//   hipcc --offload-arch=gfx950 -O3 -o tools/membw tools/membw.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

template <int U, int AUX>
__global__ __launch_bounds__(256) void copy_k(const f4* __restrict__ src, f4* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + (U - 1) * stride < n; i += U * stride) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = __builtin_nontemporal_load(&src[i + u * stride]);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (AUX) __builtin_nontemporal_store(v[u], &dst[i + u * stride]);
      else dst[i + u * stride] = v[u];
    }
  }
  for (; i < n; i += stride) dst[i] = src[i];
}

template <int U>
__global__ __launch_bounds__(256) void read_k(const f4* __restrict__ src, float* __restrict__ sink, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  f4 acc = {0, 0, 0, 0};
  for (; i + (U - 1) * stride < n; i += U * stride) {
#pragma unroll
    for (int u = 0; u < U; ++u) acc += __builtin_nontemporal_load(&src[i + u * stride]);
  }
  if (acc[0] == 1234.5f) sink[0] = acc[1];
}

__global__ __launch_bounds__(256) void write_k(f4* __restrict__ dst, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    __builtin_nontemporal_store(f4{1, 2, 3, 4}, &dst[i]);
}

template <class F>
float best_ms(F f) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int r = 0; r < 30; ++r) f();  // clocks up
  float best = 1e9f;
  for (int r = 0; r < 20; ++r) {
    hipEventRecord(a);
    f();
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    if (ms < best) best = ms;
  }
  return best;
}

int main() {
  const size_t bytes = (size_t)65536 * 17712 / 2;  // one direction of the headline state
  const size_t n = bytes / 16;
  f4 *src, *dst;
  float* sink;
  hipMalloc(&src, bytes);
  hipMalloc(&dst, bytes);
  hipMalloc(&sink, 4);
  hipMemset(src, 0, bytes);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  for (int bpc : {4, 8, 16, 32}) {
    const int grid = cus * bpc;
    float ms;
    ms = best_ms([&] { hipLaunchKernelGGL((copy_k<1, 0>), dim3(grid), dim3(256), 0, 0, src, dst, n); });
    printf("blocks/CU %2d copy U=1          %7.0f GB/s\n", bpc, 2 * bytes / ms / 1e6);
    ms = best_ms([&] { hipLaunchKernelGGL((copy_k<4, 0>), dim3(grid), dim3(256), 0, 0, src, dst, n); });
    printf("blocks/CU %2d copy U=4          %7.0f GB/s\n", bpc, 2 * bytes / ms / 1e6);
    ms = best_ms([&] { hipLaunchKernelGGL((copy_k<4, 1>), dim3(grid), dim3(256), 0, 0, src, dst, n); });
    printf("blocks/CU %2d copy U=4 nt-store %7.0f GB/s\n", bpc, 2 * bytes / ms / 1e6);
    ms = best_ms([&] { hipLaunchKernelGGL((read_k<4>), dim3(grid), dim3(256), 0, 0, src, sink, n); });
    printf("blocks/CU %2d read U=4          %7.0f GB/s\n", bpc, bytes / ms / 1e6);
    ms = best_ms([&] { hipLaunchKernelGGL(write_k, dim3(grid), dim3(256), 0, 0, dst, n); });
    printf("blocks/CU %2d write nt          %7.0f GB/s\n", bpc, bytes / ms / 1e6);
  }
  return 0;
}
