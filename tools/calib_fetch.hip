// calib_fetch.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for
// the access patterns of the step kernel (MI355X_MICROARCH.md: "other access
// widths are uncalibrated: calibrate on a known byte count").
//
// Each kernel moves exactly BYTES (1 GiB, four times the 256 MiB Infinity
// Cache) once:
//   rd_lds16_aux<A>   buffer_load ... lds, 16 B/lane (the factor's DMA loads),
//                     cache policy A (0 = default, 2 = nt as AMH_LOAD_AUX)
//   rd_lds4           buffer_load ... lds, 4 B/lane, default policy (z, loc)
//   rd_global16       plain global_load_dwordx4 (the guide's reference case)
//   wr_b32_aux<A>     buffer_store_dword, 4 B/lane, policy A (state stores)
// Build: hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o tools/calib_fetch
// Run:   rocprofv3 --pmc FETCH_SIZE -- tools/calib_fetch   (then WRITE_SIZE)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(3))) void lds_void;

constexpr uint32_t BYTES = 1u << 30;
constexpr int WAVES_PER_BLOCK = 4;
constexpr int BLOCKS = 2048;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)BYTES, 0x00020000);
}

template <int W, int AUX>
__device__ __forceinline__ void rd_lds(const float* src, float* sink) {
  __shared__ __attribute__((aligned(16))) float buf[WAVES_PER_BLOCK][64 * 4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  auto rs = rsrc(src);
  const uint32_t chunk = 64u * W;  // bytes per wave per load
  const uint32_t nwaves = gridDim.x * WAVES_PER_BLOCK;
  for (uint32_t o = (blockIdx.x * WAVES_PER_BLOCK + w) * chunk; o < BYTES; o += nwaves * chunk) {
    if constexpr (W == 16)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)&buf[w][0], 16, (int)(o + 16u * lane), 0, 0, AUX);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)&buf[w][0], 4, (int)(o + 4u * lane), 0, 0, AUX);
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (buf[w][lane] == 12345.f) sink[0] = 1.f;  // keep the loads alive
}

template <int AUX>
__global__ __launch_bounds__(256) void rd_lds16_aux(const float* src, float* sink) { rd_lds<16, AUX>(src, sink); }
__global__ __launch_bounds__(256) void rd_lds4(const float* src, float* sink) { rd_lds<4, 0>(src, sink); }

__global__ __launch_bounds__(256) void rd_global16(const float4* src, float* sink) {
  float acc = 0.f;
  const uint32_t n = BYTES / 16, stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    float4 v = src[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.f) sink[0] = acc;
}

template <int AUX>
__global__ __launch_bounds__(256) void wr_b32_aux(float* dst) {
  auto rs = rsrc(dst);
  const uint32_t n = BYTES / 4, stride = gridDim.x * blockDim.x;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)i, rs, (int)(4u * i), 0, AUX);
}

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                       \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

int main() {
  float *a, *b, *sink;
  CK(hipMalloc(&a, BYTES));
  CK(hipMalloc(&b, BYTES));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 0, BYTES));
  CK(hipMemset(b, 0, BYTES));
  CK(hipDeviceSynchronize());
  // alternate the two buffers so nothing is resident in the Infinity Cache
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(rd_lds16_aux<0>, dim3(BLOCKS), dim3(256), 0, 0, a, sink);
    hipLaunchKernelGGL(wr_b32_aux<0>, dim3(BLOCKS), dim3(256), 0, 0, b);
    hipLaunchKernelGGL(rd_lds16_aux<2>, dim3(BLOCKS), dim3(256), 0, 0, a, sink);
    hipLaunchKernelGGL(wr_b32_aux<2>, dim3(BLOCKS), dim3(256), 0, 0, b);
    hipLaunchKernelGGL(rd_lds4, dim3(BLOCKS), dim3(256), 0, 0, a, sink);
    hipLaunchKernelGGL(wr_b32_aux<0>, dim3(BLOCKS), dim3(256), 0, 0, b);
    hipLaunchKernelGGL(rd_global16, dim3(BLOCKS), dim3(256), 0, 0, (const float4*)a, sink);
    hipLaunchKernelGGL(wr_b32_aux<0>, dim3(BLOCKS), dim3(256), 0, 0, b);
  }
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  printf("calib_fetch: each kernel moved %u bytes (%.1f KiB)\n", BYTES, BYTES / 1024.0);
  return 0;
}
