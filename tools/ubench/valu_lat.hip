// Lone-wave VALU issue / latency microbenchmark (tools only, not shipped):
// one wave per launch runs a fixed instruction pattern N times between two
// s_memtime reads; prints cycles per pattern instance.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP 256

template <int MODE>
__global__ void kern(float* out, unsigned long long* t, float s) {
  float a = threadIdx.x * 1e-3f, b = 1.0001f, c = 0.9999f, e = 0.5f, f = 0.25f, g = 0.125f, h = 0.3f, k = 0.7f;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p = {a, b}, q = {c, e}, r = {f, g};
  asm volatile("" : "+s"(s));
  int li = threadIdx.x;
  asm volatile("" : "+v"(li));
  __syncthreads();
  unsigned long long t0, t1;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0));
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(e), "+v"(f), "+v"(g), "+v"(h), "+v"(k), "+v"(p), "+v"(q), "+v"(r));
#pragma unroll
  for (int i = 0; i < REP; ++i) {
    if constexpr (MODE == 0) {  // 8 dependent fma
      a = fmaf(a, b, c); a = fmaf(a, b, c); a = fmaf(a, b, c); a = fmaf(a, b, c);
      a = fmaf(a, b, c); a = fmaf(a, b, c); a = fmaf(a, b, c); a = fmaf(a, b, c);
    } else if constexpr (MODE == 1) {  // 8 independent fma (4 chains x 2)
      a = fmaf(a, s, c); e = fmaf(e, s, c); f = fmaf(f, s, c); g = fmaf(g, s, c);
      h = fmaf(h, s, c); k = fmaf(k, s, c); b = fmaf(b, s, c); q[0] = fmaf(q[0], s, c);
    } else if constexpr (MODE == 2) {  // 8 independent v_pk_fma_f32
      p = __builtin_elementwise_fma(p, q, r); q = __builtin_elementwise_fma(q, r, p);
      r = __builtin_elementwise_fma(r, p, q); p = __builtin_elementwise_fma(p, q, r);
      q = __builtin_elementwise_fma(q, r, p); r = __builtin_elementwise_fma(r, p, q);
      p = __builtin_elementwise_fma(p, q, r); q = __builtin_elementwise_fma(q, r, p);
    } else if constexpr (MODE == 3) {  // readlane -> fma chain (8 pairs)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float x = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a), (i + j) & 63));
        a = fmaf(a, x, c);
      }
    } else if constexpr (MODE == 4) {  // dependent chain interleaved with 1 independent fma each
      a = fmaf(a, b, c); e = fmaf(e, s, c); a = fmaf(a, b, c); f = fmaf(f, s, c);
      a = fmaf(a, b, c); g = fmaf(g, s, c); a = fmaf(a, b, c); h = fmaf(h, s, c);
    } else if constexpr (MODE == 5) {  // 8 independent fma, 8 chains (no reuse within 8)
      a = fmaf(a, s, c); e = fmaf(e, s, c); f = fmaf(f, s, c); g = fmaf(g, s, c);
      h = fmaf(h, s, c); k = fmaf(k, s, c); b = fmaf(b, s, c); q[0] = fmaf(q[0], s, c);
      __builtin_amdgcn_sched_barrier(0);
    } else if constexpr (MODE == 7) {  // 8 independent v_mad_u64_u32 (4 chains x 2)
      uint64_t* u = (uint64_t*)nullptr;
      (void)u;
      unsigned x0 = __float_as_uint(a), x1 = __float_as_uint(e), x2 = __float_as_uint(f), x3 = __float_as_uint(g);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const unsigned long long m0 = (unsigned long long)x0 * 0xD2511F53u, m1 = (unsigned long long)x1 * 0xCD9E8D57u;
        const unsigned long long m2 = (unsigned long long)x2 * 0xD2511F53u, m3 = (unsigned long long)x3 * 0xCD9E8D57u;
        x0 = (unsigned)(m0 >> 32) ^ (unsigned)m1; x1 = (unsigned)(m1 >> 32) ^ (unsigned)m2;
        x2 = (unsigned)(m2 >> 32) ^ (unsigned)m3; x3 = (unsigned)(m3 >> 32) ^ (unsigned)m0;
      }
      a = __uint_as_float(x0); e = __uint_as_float(x1); f = __uint_as_float(x2); g = __uint_as_float(x3);
    } else if constexpr (MODE == 6) {  // cmp + cndmask dependent pairs
#pragma unroll
      for (int j = 0; j < 4; ++j) { a = (li == ((i + j) & 63)) ? b : a * c; }
    }
  }
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(e), "+v"(f), "+v"(g), "+v"(h), "+v"(k), "+v"(p), "+v"(q), "+v"(r));
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1));
  out[threadIdx.x] = a + b + c + e + f + g + h + k + p[0] + p[1] + q[0] + q[1] + r[0] + r[1];
  if (threadIdx.x == 0) t[0] = t1 - t0;
}

template <int MODE>
void run(const char* name, int instr_per, int nthreads) {
  float* o; unsigned long long* t;
  hipMalloc(&o, 4096 * 4); hipMalloc(&t, 8);
  unsigned long long best = ~0ull;
  for (int r = 0; r < 5; ++r) {
    hipLaunchKernelGGL(kern<MODE>, dim3(1), dim3(nthreads), 0, 0, o, t, 1.0f);
    unsigned long long h; hipMemcpy(&h, t, 8, hipMemcpyDeviceToHost);
    if (h < best) best = h;
  }
  printf("%-40s threads %4d: %.2f ticks per instruction\n", name, nthreads, (double)best / (REP * instr_per));
  hipFree(o); hipFree(t);
}

int main() {
  for (int nt : {64, 256, 512}) {
    run<0>("dependent v_fma_f32", 8, nt);
    run<1>("independent v_fma_f32", 8, nt);
    run<2>("v_pk_fma_f32 (3 rotating)", 8, nt);
    run<3>("readlane+fma (per pair)", 8, nt);
    run<4>("dep chain + 1 indep interleaved", 8, nt);
    run<6>("cmp+cndmask+mul (per triple)", 4, nt);
    run<7>("mad_u64_u32 x8 + xor x8 (per mad)", 8, nt);
  }
  // s_memtime vs realtime calibration
  return 0;
}
