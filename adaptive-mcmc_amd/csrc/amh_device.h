// amh_device.h -- device building blocks shared by the step kernels
// (amh_kernels.hip: per-chain adaptation; amh_pooled.hip: pooled adaptation):
// lane-group primitives, model potentials (the PosteriorDB plug-in surface),
// buffer descriptors and the (model, d) dispatch table.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "../../include/amh.h"
#include "../../include/amh_math.h"
#include "amh_internal.h"

namespace amh {

__device__ __forceinline__ int lane_id() { return (int)__lane_id(); }

// ------------------------------------------------------------ lane groups --
// Cross-lane primitives inside a group of G lanes (G | 64), built on DPP,
// ds_swizzle, permlane and readlane so that no lane-address VGPRs are needed.
// Their association orders are part of the bit spec (oracle: group_sum,
// group_excl_scan).
namespace dpp {
constexpr int quad(int a, int b, int c, int d) { return a | (b << 2) | (c << 4) | (d << 6); }
constexpr int kRowShr0 = 0x110;
constexpr int kRowRor0 = 0x120;
constexpr int kWaveShr1 = 0x138;
constexpr int kRowBcast15 = 0x142;
constexpr int kRowBcast31 = 0x143;
constexpr int kRowNewBcast0 = 0x150;
}  // namespace dpp

// compile-time unrolled loop: f(std::integral_constant<int, j>) for j < N
template <int N, int I = 0, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

// Scheduling fence every K unrolled columns: the serial column sweeps have
// little ILP to gain, and without fences the scheduler hoists independent
// per-column products (64 of them) and runs out of VGPRs.
template <int J, int K = 8>
__device__ __forceinline__ void column_fence() {
  if constexpr ((J % K) == K - 1) __builtin_amdgcn_sched_barrier(0);
}

template <int CTRL, int ROWMASK = 0xF, bool BC = true>
__device__ __forceinline__ float dppf(float old, float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(old), __float_as_int(v), CTRL, ROWMASK, 0xF, BC));
}
template <int PATTERN>
__device__ __forceinline__ float swz(float v) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), PATTERN));
}

template <int G>
struct Grp {
  static_assert(G >= 1 && G <= 64 && (G & (G - 1)) == 0, "group width must be a power of two");
  static __device__ __forceinline__ int r() { return lane_id() & (G - 1); }

  // value of lane J of this lane's group
  template <int J>
  static __device__ __forceinline__ float bcast(float v) {
    static_assert(J >= 0 && J < G, "lane index out of group");
    if constexpr (G == 64) {
      return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), J));
    } else if constexpr (G == 32) {
      const int t = __builtin_amdgcn_update_dpp(0, __float_as_int(v), dpp::kRowNewBcast0 + (J & 15), 0xF, 0xF, false);
      const auto sw = __builtin_amdgcn_permlane16_swap(t, t, false, false);
      return __int_as_float(J < 16 ? sw[0] : sw[1]);
    } else if constexpr (G == 16) {
      return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), dpp::kRowNewBcast0 + J, 0xF, 0xF, false));
    } else if constexpr (G == 8) {
      return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x18 | (J << 5)));
    } else if constexpr (G == 4) {
      return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), dpp::quad(J, J, J, J), 0xF, 0xF, false));
    } else if constexpr (G == 2) {
      return __int_as_float(
          __builtin_amdgcn_update_dpp(0, __float_as_int(v), dpp::quad(J, J, 2 + J, 2 + J), 0xF, 0xF, false));
    } else {
      return v;
    }
  }
  // A value broadcast to many columns: at G = 32 one permlane16_swap per value
  // (lo: rows 0 / 2 copied over rows 1 / 3; hi: rows 1 / 3 over rows 0 / 2),
  // then each column is a single row_newbcast DPP of lo (J < 16) or hi --
  // instead of a copy, a swap and a DPP per column as bcast<J> needs
  struct Src {
    int lo, hi;
  };
  static __device__ __forceinline__ Src src(float v) {
    if constexpr (G == 32) {
      const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_int(v), __float_as_int(v), false, false);
      return Src{(int)sw[0], (int)sw[1]};
    } else {
      return Src{__float_as_int(v), 0};
    }
  }
  template <int J>
  static __device__ __forceinline__ float bcast(const Src& s) {
    if constexpr (G == 32) {
      return __int_as_float(
          __builtin_amdgcn_update_dpp(0, J < 16 ? s.lo : s.hi, dpp::kRowNewBcast0 + (J & 15), 0xF, 0xF, false));
    } else {
      return bcast<J>(__int_as_float(s.lo));
    }
  }
  template <int J>
  static __device__ __forceinline__ uint32_t bcast_u(uint32_t v) {
    return (uint32_t)__float_as_int(bcast<J>(__int_as_float((int)v)));
  }
  // runtime lane index (model code with data-dependent layout)
  static __device__ __forceinline__ float bcast_rt(float v, int j) {
    if constexpr (G == 64) {
      return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), j));
    } else if constexpr (G == 1) {
      return v;
    } else {
      return __shfl(v, (lane_id() & ~(G - 1)) | j, 64);
    }
  }

  // butterfly: for off = 1, 2, 4, ..: x_r = x_r + x_{r ^ off}  (oracle: group_sum)
  static __device__ __forceinline__ float sum(float v) {
    if constexpr (G >= 2) v = v + dppf<dpp::quad(1, 0, 3, 2)>(0.0f, v);
    if constexpr (G >= 4) v = v + dppf<dpp::quad(2, 3, 0, 1)>(0.0f, v);
    if constexpr (G >= 8) v = v + swz<0x1F | (4 << 10)>(v);
    if constexpr (G >= 16) v = v + dppf<dpp::kRowRor0 + 8>(0.0f, v);
    if constexpr (G >= 32) v = v + swz<0x1F | (16 << 10)>(v);
    if constexpr (G == 64) {
      // every lane of each 32-lane half holds that half's total here
      v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0)) +
          __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    }
    return v;
  }

  // exclusive scan (oracle: group_excl_scan): shift by one lane, inclusive
  // Hillis-Steele inside 16-lane rows, then row totals via row_bcast15/31.
  static __device__ __forceinline__ float excl_scan(float t, int rr) {
    if constexpr (G == 1) {
      return 0.0f;
    } else {
      float x = dppf<dpp::kWaveShr1>(0.0f, t);
      if constexpr (G < 64) x = (rr == 0) ? 0.0f : x;
      if constexpr (G >= 2) { const float y = dppf<dpp::kRowShr0 + 1>(0.0f, x); x = (G >= 16 || rr >= 1) ? x + y : x; }
      if constexpr (G >= 4) { const float y = dppf<dpp::kRowShr0 + 2>(0.0f, x); x = (G >= 16 || rr >= 2) ? x + y : x; }
      if constexpr (G >= 8) { const float y = dppf<dpp::kRowShr0 + 4>(0.0f, x); x = (G >= 16 || rr >= 4) ? x + y : x; }
      if constexpr (G >= 16) { const float y = dppf<dpp::kRowShr0 + 8>(0.0f, x); x = x + y; }
      if constexpr (G >= 32) { x = x + dppf<dpp::kRowBcast15, 0xA>(0.0f, x); }
      if constexpr (G == 64) { x = x + dppf<dpp::kRowBcast31, 0xC>(0.0f, x); }
      return x;
    }
  }

  static __device__ __forceinline__ bool any(bool p) {
    const unsigned long long m = __ballot(p);
    if constexpr (G == 64) {
      return m != 0ull;
    } else {
      const int g0 = lane_id() & ~(G - 1);
      constexpr unsigned long long gm = (1ull << G) - 1ull;
      return ((m >> g0) & gm) != 0ull;
    }
  }
};

// ------------------------------------------------------ the step's noise --
// Bit spec (include/amh_math.h amh_step_word): words W_j = Philox(j >> 2, it,
// 0, TAG_STEP; key)[j & 3]; xi_r = N(W_r) for r < d, u = U(W_d).  In a
// chain's G-lane group (G >= d) lane r computes call r >> 2 itself (four
// lanes the same call: no cross-lane traffic, one call per lane as before)
// and keeps word r & 3.  u is word d & 3 of call d >> 2, which lane
// 4 (d >> 2) computed when that lane is in the group (d < G, or d % 4 != 0);
// else (d = G, a multiple of 4) lane G - 1 computes call d >> 2 instead of a
// fourth copy of call G/4 - 1 and takes its own word from lane G - 4 (two
// broadcasts instead of a second Philox call per lane).
template <int G>
__device__ __forceinline__ void step_noise(int r, int d, uint32_t it, uint32_t k0, uint32_t k1, float& xi, float& u) {
  const int src = 4 * (d >> 2);
  const bool full = src >= G;  // d == G: word d is in call G / 4, which no lane computes
  const bool last = full && r == G - 1;
  const amh_u32x4 o = amh_philox4x32_10(last ? (uint32_t)(d >> 2) : (uint32_t)(r >> 2), it, 0u, AMH_TAG_STEP, k0, k1);
  const int q = r & 3;
  uint32_t w = (q == 0) ? o.v[0] : ((q == 1) ? o.v[1] : ((q == 2) ? o.v[2] : o.v[3]));
  uint32_t ub;
  if (!full) {
    const int qd = d & 3;
    const uint32_t us = (qd == 0) ? o.v[0] : ((qd == 1) ? o.v[1] : ((qd == 2) ? o.v[2] : o.v[3]));
    ub = (uint32_t)__float_as_int(Grp<G>::bcast_rt(__int_as_float((int)us), src));
  } else if constexpr (G >= 4) {  // (d <= G < 4 never fills a call)
    const uint32_t wl = (uint32_t)__float_as_int(Grp<G>::bcast_rt(__int_as_float((int)o.v[3]), G - 4));
    ub = (uint32_t)__float_as_int(Grp<G>::bcast_rt(__int_as_float((int)o.v[0]), G - 1));
    w = last ? wl : w;
  } else {
    ub = 0u;
  }
  xi = amh_normal_from_bits(w);
  u = amh_unif01_from_bits(ub);
}

// One chain per wave at d = 64 (arwmh_step64_kernel): lane r computes call
// r >> 2 itself (four lanes the same call -- no cross-lane traffic, and the
// registers of the bpermute form, which made the kernel spill) and keeps word
// r & 3.  u is word 64 (call 16): lane 63 computes call 16 instead of a
// fourth copy of call 15 and takes its own word (word 3 of call 15) from lane
// 60 -- two v_readlane and two selects instead of a second Philox call (the
// round-5 form ran call 16 on the scalar unit: ~60 more instructions per
// chain-step, AMH_S64_NOISE_SCALAR=1 keeps it for A/B).  The same bits as
// step_noise<64>.
__device__ __forceinline__ void step_noise_w64(int r, uint32_t it, uint32_t k0, uint32_t k1, float& xi, float& u) {
#if AMH_S64_NOISE_SCALAR
  const amh_u32x4 o = amh_philox4x32_10((uint32_t)(r >> 2), it, 0u, AMH_TAG_STEP, k0, k1);
  const int q = r & 3;
  const uint32_t w = (q == 0) ? o.v[0] : ((q == 1) ? o.v[1] : ((q == 2) ? o.v[2] : o.v[3]));
  xi = amh_normal_from_bits(w);
  const uint32_t ks0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k0);
  const uint32_t ks1 = (uint32_t)__builtin_amdgcn_readfirstlane((int)k1);
  const uint32_t its = (uint32_t)__builtin_amdgcn_readfirstlane((int)it);
  u = amh_unif01_from_bits(amh_philox4x32_10(16u, its, 0u, AMH_TAG_STEP, ks0, ks1).v[0]);
#else
  const bool l63 = (r == 63);
  const amh_u32x4 o = amh_philox4x32_10(l63 ? 16u : (uint32_t)(r >> 2), it, 0u, AMH_TAG_STEP, k0, k1);
  const int q = r & 3;
  const uint32_t w = (q == 0) ? o.v[0] : ((q == 1) ? o.v[1] : ((q == 2) ? o.v[2] : o.v[3]));
  const uint32_t w63 = (uint32_t)__builtin_amdgcn_readlane((int)o.v[3], 60);  // word 63
  const uint32_t ub = (uint32_t)__builtin_amdgcn_readlane((int)o.v[0], 63);   // word 64
  xi = amh_normal_from_bits(l63 ? w63 : w);
  u = amh_unif01_from_bits(ub);
#endif
}

// The same stream for one chain per wave with lane l owning rows 64 K + l
// (the large-d kernels, NS row slices): row 64 K + l is word l & 3 of call
// 16 K + (l >> 2), computed by the lane itself (NS calls per lane, as one per
// row was; no cross-lane traffic).  Rows >= d get 0.  *ubits (if given)
// receives word d, the accept uniform's bits (one more call).
template <int NS>
__device__ __forceinline__ void step_noise_rows(int lane, int d, uint32_t it, uint32_t k0, uint32_t k1,
                                                float (&xi)[NS], uint32_t* ubits = nullptr) {
  static_assert(NS <= 4, "64 calls cover 256 rows");
  const int q = lane & 3;
  static_for<NS>([&](auto K) {
    const amh_u32x4 o = amh_philox4x32_10((uint32_t)(16 * (int)K + (lane >> 2)), it, 0u, AMH_TAG_STEP, k0, k1);
    const uint32_t w = (q == 0) ? o.v[0] : ((q == 1) ? o.v[1] : ((q == 2) ? o.v[2] : o.v[3]));
    xi[K] = (64 * (int)K + lane < d) ? amh_normal_from_bits(w) : 0.0f;
  });
  if (ubits != nullptr) *ubits = amh_step_word((uint32_t)d, it, k0, k1);
}

// ----------------------------------------------------------- lane masks --
// Per-column lane predicates of the load/store phases.  For a full-wave
// group they are compile-time lane masks built by one SALU shift inside the
// asm (so the compiler can neither hoist 64 mask constants into SGPRs nor
// keep them live across the chain loop); smaller groups compare an opaque
// per-item copy of the lane index.
template <int G, int J>
__device__ __forceinline__ float keep_above(float x, int rr) {  // lanes r > J keep x, else 0
  if constexpr (G == 64) {
    if constexpr (J >= 63) {
      return 0.0f;
    } else {
      float out;
      unsigned long long m;
      asm("s_lshl_b64 %1, -1, %3\n\tv_cndmask_b32_e64 %0, 0, %2, %1" : "=v"(out), "=&s"(m) : "v"(x), "n"(J + 1));
      return out;
    }
  } else {
    return (rr > J) ? x : 0.0f;
  }
}
template <int G, int J>
__device__ __forceinline__ float set_one_at(float x, int rr) {  // lane r == J gets 1.0
  if constexpr (G == 64) {
    float out;
    unsigned long long m;
    asm("s_lshl_b64 %1, 1, %3\n\tv_cndmask_b32_e64 %0, %2, 1.0, %1" : "=v"(out), "=&s"(m) : "v"(x), "n"(J));
    return out;
  } else {
    return (rr == J) ? 1.0f : x;
  }
}
template <int G, int J>
__device__ __forceinline__ uint32_t off_from(uint32_t v, uint32_t oob, int rr) {  // lanes r >= J keep v, else oob
  if constexpr (G == 64) {
    uint32_t out;
    unsigned long long m;
    asm("s_lshl_b64 %1, -1, %4\n\tv_cndmask_b32_e64 %0, %3, %2, %1" : "=v"(out), "=&s"(m) : "v"(v), "v"(oob), "n"(J));
    return out;
  } else {
    return (rr >= J) ? v : oob;
  }
}

// packed column-major lower triangle: column j starts at j*d - j(j-1)/2
__device__ __forceinline__ int64_t col_off(int d, int j) {
  return (int64_t)j * d - (int64_t)j * (j - 1) / 2;
}

#define HALF_LOG_2PI 0.918938533204672742f

// ------------------------------------------------------ model-data LDS reads --
// Model data staged in LDS is never a DMA destination, but the compiler cannot
// tell it from the step kernel's prefetch buffers (one LDS allocation): a plain
// LDS load makes it wait vmcnt(0) for the in-flight buffer_load..lds prefetch.
// These reads are issued as asm (invisible to the wait-count pass) and
// completed by lds_wait(), which ties the loaded values so no use can be
// scheduled before the wait.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) const float lds_cfloat;
__device__ __forceinline__ uint32_t lds_addr(const float* p) {
  return (uint32_t)(uintptr_t)(lds_cfloat*)p;
}
template <int OFF>
__device__ __forceinline__ f32x4 lds_ld4(uint32_t a) {
  f32x4 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
  return v;
}
template <int OFF>
__device__ __forceinline__ float lds_ld1(uint32_t a) {
  float v;
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(a), "n"(OFF));
  return v;
}
template <class T>
__device__ __forceinline__ void lds_wait(T& a, T& b, T& c) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c));
}
template <class T>
__device__ __forceinline__ void lds_wait(T& a, T& b, T& c, T& d) {
  asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
}
template <int N, class T>
__device__ __forceinline__ void lds_wait_n(T (&v)[N]) {
  static_assert(N == 1 || N == 2 || N == 4, "lds_wait_n: 1, 2 or 4 values");
  if constexpr (N == 1) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]));
  if constexpr (N == 2) asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]));
  if constexpr (N == 4) lds_wait(v[0], v[1], v[2], v[3]);
}

// ------------------------------------------------------------------ models --
// Every model: static potential(x_r, r, d, args, lds) -> U (same value in all
// lanes of the group), evaluated with all lanes converged.

// Model interface (every potential runs with all lanes of the group
// converged and returns the same U in every lane of the group):
//   lds_bytes(args, d)             model data staged in LDS per block
//   stage(lds, args, d)            block-cooperative staging
//   Ctx prepare(args, d, r)        per-lane constants, loaded once per kernel
//   potential(x_r, r, d, ctx, lds) U(x)
// Nothing is read from global memory inside potential() for the Gaussian,
// eight-schools and kidiq models: inside the step kernel a global load would
// make the compiler drain the in-flight LDS-DMA prefetch (vmcnt(0)).

template <int G>
struct GaussianM {
  // data = [m (d) | P (d*d) | c0].  P is symmetric; LDS holds row r of P at
  // lds[r * ld + j] with ld = d rounded up to 4 plus 4 floats of padding, so
  // lane r reads its own row with ds_read_b128 (4 columns per read) and the
  // 16-B slots of the 16 lanes of a read group fall on distinct banks.
  struct Ctx {
    float mr, c0;
  };
  static __host__ __device__ int ld(int d) { return ((d + 3) & ~3) + 4; }
  static __host__ __device__ size_t lds_bytes(const ModelArgs&, int d) { return (size_t)d * ld(d) * sizeof(float); }
  static __device__ void stage(float* lds, const ModelArgs& m, int d) {
    const float* P = m.data + d;
    const int L = ld(d);
    for (int k = threadIdx.x; k < d * L; k += blockDim.x) {
      const int row = k / L, col = k - row * L;
      lds[k] = (col < d) ? P[row * d + col] : 0.0f;
    }
  }
  static __device__ __forceinline__ Ctx prepare(const ModelArgs& m, int d, int r) {
    return Ctx{(r < d) ? m.data[r] : 0.0f, m.data[d + d * d]};
  }
  static __device__ __forceinline__ float potential(float x, int r, int d, const Ctx& c, const float* lds) {
    const bool act = r < d;
    const float diff = act ? x - c.mr : 0.0f;
    const uint32_t prow = lds_addr(lds + (act ? r : 0) * ld(d));
    // partial sums over columns j mod 4 (four independent FMA chains); the
    // row is read 16 columns at a time (four ds_read_b128 then one wait).
    // Columns (j, j+1) go through one v_pk_fma_f32 into the accumulator pair
    // (j mod 4, j+1 mod 4): each half is the same fmaf.  A column past d
    // pairs a zero (padded row) with a zero (inactive lane's diff) and
    // leaves its accumulator unchanged.
    float y4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    f32x2v y01 = {0.0f, 0.0f}, y23 = {0.0f, 0.0f};
    static_for<(G + 15) / 16>([&](auto B) {
      constexpr int b = B;
      if (16 * b < d) {
        f32x4 pv[4];
        static_for<4>([&](auto Q) {
          // a block that starts below d lies inside the padded row
          pv[Q] = (4 * (4 * b + Q) < d) ? lds_ld4<16 * (4 * b + Q)>(prow) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        });
        lds_wait(pv[0], pv[1], pv[2], pv[3]);
        if constexpr (G == 1) {
          y4[0] = fmaf(act ? pv[0][0] : 0.0f, diff, y4[0]);
        } else {
          static_for<8>([&](auto K2) {
            constexpr int j = 16 * b + 2 * K2;
            if constexpr (j < G) {
              if (j < d) {
                const f32x4 q = pv[K2 / 2];
                const f32x2v pp = (K2 % 2 == 0) ? f32x2v{q[0], q[1]} : f32x2v{q[2], q[3]};
                const f32x2v pa = act ? pp : f32x2v{0.0f, 0.0f};
                const f32x2v bp = {Grp<G>::template bcast<j>(diff), Grp<G>::template bcast<j + 1>(diff)};
                if constexpr (K2 % 2 == 0) {
                  y01 = __builtin_elementwise_fma(pa, bp, y01);
                } else {
                  y23 = __builtin_elementwise_fma(pa, bp, y23);
                }
              }
            }
          });
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    });
    if constexpr (G > 1) {
      y4[0] = y01[0];
      y4[1] = y01[1];
      y4[2] = y23[0];
      y4[3] = y23[1];
    }
    const float y = (y4[0] + y4[1]) + (y4[2] + y4[3]);
    const float q = act ? diff * y : 0.0f;
    const float S = Grp<G>::sum(q);
    return (0.5f * S) + c.c0;
  }
};

template <int G>
struct EightSchoolsM {
  // z = [mu, log tau, theta_base (J)]; data = [y (J) | sigma (J) | log sigma (J)]
  struct Ctx {
    float y, sg, lsg;  // school r - 2 (lanes 2 .. d-1)
  };
  static __host__ __device__ size_t lds_bytes(const ModelArgs&, int) { return 0; }
  static __device__ void stage(float*, const ModelArgs&, int) {}
  static __device__ __forceinline__ Ctx prepare(const ModelArgs& m, int d, int r) {
    const int J = d - 2;
    const bool sch = r >= 2 && r < d;
    const int j = sch ? r - 2 : 0;
    return Ctx{sch ? m.data[j] : 0.0f, sch ? m.data[J + j] : 1.0f, sch ? m.data[2 * J + j] : 0.0f};
  }
  static __device__ __forceinline__ float potential(float x, int r, int d, const Ctx& c, const float*) {
    const float mu = Grp<G>::template bcast<0>(x);
    const float lt = Grp<G>::template bcast<1>(x);
    const float tau = amh_expf(lt);
    float v = 0.0f;
    if (r == 0) {
      const float t = mu / 5.0f;
      v = ((-0.5f * (t * t)) - 1.60943791243410037f) - HALF_LOG_2PI;
    } else if (r == 1) {
      const float t = tau / 5.0f;
      v = ((-0.451582705289454865f - 1.60943791243410037f) - amh_log1pf(t * t)) + lt;
    } else if (r < d) {
      const float th = x;
      const float lpt = (-0.5f * (th * th)) - HALF_LOG_2PI;
      const float e = (c.y - (mu + tau * th)) / c.sg;
      const float lpy = ((-0.5f * (e * e)) - c.lsg) - HALF_LOG_2PI;
      v = lpt + lpy;
    }
    return -Grp<G>::sum(v);
  }
};

template <int G>
struct KidiqM {
  // z = [beta0, beta1, beta2, log sigma]; data = [kid | hs | iq] (N each),
  // staged in LDS
  struct Ctx {
    int64_t N;
  };
  static __host__ __device__ size_t lds_bytes(const ModelArgs& m, int) { return (size_t)(3 * m.n) * sizeof(float); }
  static __device__ void stage(float* lds, const ModelArgs& m, int) {
    for (int64_t k = threadIdx.x; k < 3 * m.n; k += blockDim.x) lds[k] = m.data[k];
  }
  static __device__ __forceinline__ Ctx prepare(const ModelArgs& m, int, int) { return Ctx{m.n}; }
  static __device__ __forceinline__ float potential(float x, int r, int, const Ctx& c, const float* lds) {
    const int64_t N = c.N;
    const float b0 = Grp<G>::template bcast<0>(x), b1 = Grp<G>::template bcast<1>(x);
    const float b2 = Grp<G>::template bcast<2>(x), ls = Grp<G>::template bcast<3>(x);
    const float sg = amh_expf(ls);
    const float isg = 1.0f / sg;
    const uint32_t a0 = lds_addr(lds);
    const uint32_t nb = (uint32_t)N * 4u;
    float acc = 0.0f;
    for (int64_t n = r; n < N; n += G) {
      const uint32_t an = a0 + (uint32_t)n * 4u;
      float kid = lds_ld1<0>(an), hs = lds_ld1<0>(an + nb), iq = lds_ld1<0>(an + 2u * nb);
      lds_wait(kid, hs, iq);
      const float mu = fmaf(b2, iq, fmaf(b1, hs, b0));
      const float e = (kid - mu) * isg;
      acc = fmaf(e, e, acc);
    }
    const float S = Grp<G>::sum(acc);
    const float t = sg / 2.5f;
    const float ll = fmaf(-0.5f, S, (float)N * ((-ls) - HALF_LOG_2PI));
    const float lpr = ((-0.451582705289454865f - 0.916290731874155065f) - amh_log1pf(t * t)) + ls;
    return -(ll + lpr);
  }
};

__device__ __forceinline__ float lp_student3(float x, float loc, float scale, float c) {
  const float t = (x - loc) / scale;
  return c - 2.0f * amh_log1pf((t * t) / 3.0f);
}

template <int G>
struct DiamondsM {
  // z = [Intercept, b (Kc), log sigma]; data = [Xc (N x Kc) | Y (N)]
  // Straight VALU restatement (parity path; the data stream from L2).
  struct Ctx {
    int64_t N;
    const float* data;
  };
  static __host__ __device__ size_t lds_bytes(const ModelArgs&, int) { return 0; }
  static __device__ void stage(float*, const ModelArgs&, int) {}
  static __device__ __forceinline__ Ctx prepare(const ModelArgs& m, int, int) { return Ctx{m.n, m.data}; }
  static __device__ __forceinline__ float potential(float x, int r, int d, const Ctx& c, const float*) {
    const int64_t N = c.N;
    const float* data = c.data;
    const int Kc = d - 2;
    const float* X = data;
    const float* Y = data + N * Kc;
    float xb[G];
    static_for<G>([&](auto J) { xb[J] = Grp<G>::template bcast<J>(x); });
    const float icpt = xb[0];
    const float ls = Grp<G>::bcast_rt(x, Kc + 1);
    const float sg = amh_expf(ls);
    const float isg = 1.0f / sg;
    float acc = 0.0f;
    for (int64_t n = r; n < N; n += G) {
      float mu = 0.0f;
#pragma unroll
      for (int k = 0; k < G - 1; ++k) {
        if (k >= Kc) continue;
        mu = fmaf(X[n * Kc + k], xb[1 + k], mu);
      }
      const float e = (Y[n] - (icpt + mu)) * isg;
      acc = fmaf(e, e, acc);
    }
    const float S = Grp<G>::sum(acc);
    const float bb = (r >= 1 && r <= Kc) ? x * x : 0.0f;
    const float B = Grp<G>::sum(bb);
    const float cst = -3.30347394261755545f;
    const float ll = fmaf(-0.5f, S, (float)N * ((-ls) - HALF_LOG_2PI));
    const float lpb = fmaf(-0.5f, B, -(float)Kc * HALF_LOG_2PI);
    const float lpi = lp_student3(icpt, 8.0f, 10.0f, cst);
    const float lps = (0.693147181f + lp_student3(sg, 0.0f, 10.0f, cst)) + ls;
    return -(((ll + lpb) + lpi) + lps);
  }
};

// Diamonds through sufficient statistics (AMH_MODEL_DIAMONDS_SS).  The
// likelihood's residual sum is an exact quadratic in (Intercept, b):
//   sum_n (Y_n - I - Xc_n b)^2 = A + a (N a - 2 sT) - 2 b'(t - a sx) + b'Gm b,
// a = I - ybar, T = Y - ybar, A = T'T, sT = sum T, t = Xc'T, sx = sum Xc_n,
// Gm = Xc'Xc, all float64 statistics of the same float32 Xc and Y the direct
// model reads (posteriors.diamonds_suffstat).  Per chain-step this is
// O(Kc^2) float64 work instead of the N*Kc float32 contraction, so the model
// runs inside the one-launch step kernel with the factor read once.  Only the
// residual sum differs from DiamondsM (float64, then rounded); priors and
// the rest of U are the same float ops.
// data = float64 [N, ybar, A, sT, t (Kc), sx (Kc), Gm (Kc x Kc, row-major)]
// passed as pairs of floats.  Everything lives in LDS (float64), so a lane
// keeps no model registers between chain groups:
//   row i (i < Kc) at i * ldr: [Gm_i0 .. Gm_i,i-1, 0 .. 0 (to Kc), Gm_ii, t_i, sx_i, pad]
//   header at Kc * ldr:        [N, ybar, A, sT]
template <int G>
struct DiamondsSSM {
  struct Ctx {};
  static __host__ __device__ int ldr(int Kc) { return (Kc + 4) & ~1; }  // doubles per row (16-B rows)
  static __host__ __device__ size_t lds_bytes(const ModelArgs&, int d) {
    return (size_t)((d - 2) * ldr(d - 2) + 4) * sizeof(double);
  }
  static __device__ void stage(float* lds, const ModelArgs& m, int d) {
    const int Kc = d - 2, L = ldr(Kc);
    const double* D = (const double*)m.data;
    const double* Gm = D + 4 + 2 * Kc;
    double* out = (double*)lds;
    for (int k = threadIdx.x; k < Kc * L + 4; k += blockDim.x) {
      const int i = k / L, j = k - i * L;
      double v = 0.0;
      if (i >= Kc) v = D[j];                         // header
      else if (j < i) v = Gm[i * Kc + j];
      else if (j == Kc) v = Gm[i * Kc + i];
      else if (j == Kc + 1) v = D[4 + i];            // t_i
      else if (j == Kc + 2) v = D[4 + Kc + i];       // sx_i
      out[k] = v;
    }
  }
  static __device__ __forceinline__ Ctx prepare(const ModelArgs&, int, int) { return Ctx{}; }
  // float64 Grp::sum: the same DPP / swizzle partners on both halves
  template <int CTRL>
  static __device__ __forceinline__ double dpp_d(double v) {
    const f32x2v h = __builtin_bit_cast(f32x2v, v);
    return __builtin_bit_cast(double, f32x2v{dppf<CTRL>(0.0f, h[0]), dppf<CTRL>(0.0f, h[1])});
  }
  template <int PATTERN>
  static __device__ __forceinline__ double swz_d(double v) {
    const f32x2v h = __builtin_bit_cast(f32x2v, v);
    return __builtin_bit_cast(double, f32x2v{swz<PATTERN>(h[0]), swz<PATTERN>(h[1])});
  }
  static __device__ __forceinline__ double dsum(double v) {
    if constexpr (G >= 2) v = v + dpp_d<dpp::quad(1, 0, 3, 2)>(v);
    if constexpr (G >= 4) v = v + dpp_d<dpp::quad(2, 3, 0, 1)>(v);
    if constexpr (G >= 8) v = v + swz_d<0x1F | (4 << 10)>(v);
    if constexpr (G >= 16) v = v + dpp_d<dpp::kRowRor0 + 8>(v);
    if constexpr (G >= 32) v = v + swz_d<0x1F | (16 << 10)>(v);
    if constexpr (G == 64) v = v + __shfl_xor(v, 32, 64);
    return v;
  }
  static __device__ __forceinline__ double lo(const f32x4& q) { return __builtin_bit_cast(double, f32x2v{q[0], q[1]}); }
  static __device__ __forceinline__ double hi(const f32x4& q) { return __builtin_bit_cast(double, f32x2v{q[2], q[3]}); }
  static __device__ __forceinline__ float potential(float x, int r, int d, const Ctx&, const float* lds) {
    const int Kc = d - 2;
    const int L = ldr(Kc);
    const float icpt = Grp<G>::template bcast<0>(x);
    // lane Kc + 1 (log sigma): a compile-time DPP broadcast once d is fixed
    float ls = 0.0f;
    static_for<G>([&](auto J) {
      if (J == Kc + 1) ls = Grp<G>::template bcast<J>(x);
    });
    const float sg = amh_expf(ls);
    const float isg = 1.0f / sg;
    const bool act = r >= 1 && r <= Kc;
    const uint32_t prow = lds_addr(lds + 2 * (act ? r - 1 : 0) * L);
    const uint32_t phdr = lds_addr(lds + 2 * Kc * L);
    // rr = sum_{j < i} Gm_ij b_j in j order (the row's zeros at j >= i add +0)
    double rr = 0.0;
    static_for<(G + 3) / 4>([&](auto B) {  // 4 columns (two ds_read_b128) per wait
      constexpr int b = B;
      if (4 * b < Kc) {
        f32x4 p0 = lds_ld4<32 * b>(prow);
        f32x4 p1 = (4 * b + 2 < Kc) ? lds_ld4<32 * b + 16>(prow) : f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(p0), "+v"(p1));
        static_for<4>([&](auto K) {
          constexpr int j = 4 * b + K;
          if constexpr (j + 1 < G) {
            if (j < Kc) {
              const f32x4& q = (K < 2) ? p0 : p1;
              const double g = (K % 2 == 0) ? lo(q) : hi(q);
              rr = __builtin_fma(act ? g : 0.0, (double)Grp<G>::template bcast<1 + j>(x), rr);
            }
          }
        });
      }
    });
    // Gm_ii, t_i, sx_i at columns Kc .. Kc+2 of the row; header N, ybar, A, sT
    const uint32_t pdiag = prow + 8u * (uint32_t)Kc;  // Kc even or odd: 8-B aligned reads
    f32x2v g2, t2, s2;
    asm volatile("ds_read_b64 %0, %1 offset:0" : "=v"(g2) : "v"(pdiag));
    asm volatile("ds_read_b64 %0, %1 offset:8" : "=v"(t2) : "v"(pdiag));
    asm volatile("ds_read_b64 %0, %1 offset:16" : "=v"(s2) : "v"(pdiag));
    f32x4 h0 = lds_ld4<0>(phdr), h1 = lds_ld4<16>(phdr);
    asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(g2), "+v"(t2), "+v"(s2), "+v"(h0), "+v"(h1));
    const double gii = __builtin_bit_cast(double, g2), ti = __builtin_bit_cast(double, t2);
    const double sxi = __builtin_bit_cast(double, s2);
    const double N = lo(h0), ybar = hi(h0), A = lo(h1), sT = hi(h1);
    const double a = (double)icpt - ybar;
    const double bi = act ? (double)x : 0.0;
    const double quad = bi * __builtin_fma(2.0, rr, gii * bi);
    const double lin = bi * __builtin_fma(-a, sxi, ti);
    double v = act ? __builtin_fma(-2.0, lin, quad) : 0.0;
    v = dsum(v);  // xor butterfly over the group (oracle dgroup_sum)
    const double qa = __builtin_fma(a, __builtin_fma(N, a, -2.0 * sT), A);
    const double q = qa + v;
    const double isgd = (double)isg;
    const float S = (float)(q * (isgd * isgd));
    const float bb = act ? x * x : 0.0f;
    const float B = Grp<G>::sum(bb);
    const float cst = -3.30347394261755545f;
    const float ll = fmaf(-0.5f, S, (float)N * ((-ls) - HALF_LOG_2PI));
    const float lpb = fmaf(-0.5f, B, -(float)Kc * HALF_LOG_2PI);
    const float lpi = lp_student3(icpt, 8.0f, 10.0f, cst);
    const float lps = (0.693147181f + lp_student3(sg, 0.0f, 10.0f, cst)) + ls;
    return -(((ll + lpb) + lpi) + lps);
  }
};

// Mixture of K <= 8 univariate normals, applied to every coordinate
// (asumptions_check.ipynb cells 61-62: potential_fn = -MixtureSameFamily(
// Categorical(w), Normal(m, s)).log_prob(x), summed over coordinates, which
// at d = 1 -- the notebook's case -- is the scalar it returns).
// data = [c (K) | m (K) | s (K)] with c_k = log w_k - log(sqrt(2 pi) s_k)
// (host, float64, then rounded), staged in LDS.  Per coordinate:
//   lp_k = c_k - 0.5 t_k^2, t_k = (x - m_k) / s_k  (numpyro Normal.log_prob)
//   v = log(sum_k exp(lp_k - M)) + M, M = max_k lp_k or 0 if not finite
//   (jax.nn.logsumexp; the sum in k order from 0).
constexpr int kMixtureKMax = 8;
template <int G>
struct MixtureM {
  struct Ctx {
    int K;
  };
  static __host__ __device__ size_t lds_bytes(const ModelArgs& m, int) { return (size_t)(3 * m.n) * sizeof(float); }
  static __device__ void stage(float* lds, const ModelArgs& m, int) {
    for (int64_t k = threadIdx.x; k < 3 * m.n; k += blockDim.x) lds[k] = m.data[k];
  }
  static __device__ __forceinline__ Ctx prepare(const ModelArgs& m, int, int) { return Ctx{(int)m.n}; }
  static __device__ __forceinline__ float potential(float x, int r, int d, const Ctx& c, const float* lds) {
    const int K = c.K;
    const uint32_t a0 = lds_addr(lds);
    const uint32_t nb = (uint32_t)K * 4u;
    float lp[kMixtureKMax];
    float mx = -INFINITY;
    static_for<kMixtureKMax>([&](auto Kc) {
      constexpr int k = Kc;
      lp[k] = 0.0f;
      if (k < K) {
        float ck = lds_ld1<4 * k>(a0), mk = lds_ld1<4 * k>(a0 + nb), sk = lds_ld1<4 * k>(a0 + 2u * nb);
        lds_wait(ck, mk, sk);
        const float t = (x - mk) / sk;
        lp[k] = ck - 0.5f * (t * t);
        mx = (lp[k] > mx) ? lp[k] : mx;
      }
    });
    mx = (mx == INFINITY || mx == -INFINITY || mx != mx) ? 0.0f : mx;
    float S = 0.0f;
    static_for<kMixtureKMax>([&](auto Kc) {
      constexpr int k = Kc;
      if (k < K) S = S + amh_expf(lp[k] - mx);
    });
    const float v = (r < d) ? (amh_logf(S) + mx) : 0.0f;
    return -Grp<G>::sum(v);
  }
};

// Potential evaluated outside the step kernel (split path, amh_split.hip):
// the step kernel reads U(z') from StepParams::ext_pe instead of calling
// potential(); init leaves pe for the batched potential kernel to fill.
template <int G>
struct ExtPotM {
  struct Ctx {};
  static constexpr bool kExternal = true;
  static __host__ __device__ size_t lds_bytes(const ModelArgs&, int) { return 0; }
  static __device__ void stage(float*, const ModelArgs&, int) {}
  static __device__ __forceinline__ Ctx prepare(const ModelArgs&, int, int) { return Ctx{}; }
  static __device__ __forceinline__ float potential(float, int, int, const Ctx&, const float*) { return 0.0f; }
};
template <class T, class = void>
struct is_external : std::false_type {};
template <class T>
struct is_external<T, std::void_t<decltype(T::kExternal)>> : std::bool_constant<T::kExternal> {};

// --------------------------------------------------------------- geometry --
constexpr int kBlock = 256;       // 4 waves (init / potential / sample_Pnx kernels)
constexpr int kBlockStep = 1024;  // 16 waves per CU share one staged copy of the model data
#ifndef AMH_STEP_MIN_WAVES
#define AMH_STEP_MIN_WAVES 1  // waves per SIMD the step kernel must fit (VGPR budget)
#endif

template <int G>
struct Geo {
  static constexpr int CPW = 64 / G;  // chains per wave
};

// Chain owned by this lane's group for work item `item`; clamped to C-1 so
// that tail groups run converged on valid memory and simply do not store.
template <int G>
__device__ __forceinline__ int64_t item_chain(int64_t item) {
  int64_t c = item * Geo<G>::CPW + (lane_id() / G);
  if constexpr (G == 64) c = (int64_t)__builtin_amdgcn_readfirstlane((int)c);  // wave-uniform
  return c;
}

// gamma_n beyond the host-built table (n >= 2^20): same bits, kept out of line
// so its double-precision constants do not occupy registers in the step loop.
static __device__ __noinline__ float lr_gamma_slow(int32_t n, float a) { return amh_lr_gamma(n, a); }

// gamma_n from the host-built table through the scalar cache (constant
// address space): a vector load here would drain the LDS-DMA prefetch.
typedef __attribute__((address_space(4))) const float const_float;

template <int G>
__device__ __forceinline__ float lookup_gamma(const StepParams& p, int32_t n) {
  const const_float* tab = (const const_float*)p.gamma_tab;
  if constexpr (G == 64) {
    const int32_t nu = __builtin_amdgcn_readfirstlane(n);
    return (nu < p.gamma_tab_n) ? tab[nu] : lr_gamma_slow(nu, p.a);
  } else {
    float g = 0.0f;
    const int gi_lane = lane_id() / G;
    static_for<64 / G>([&](auto GI) {
      const int32_t ng = __builtin_amdgcn_readlane(n, GI * G);
      const float gv = (ng < p.gamma_tab_n) ? tab[ng] : lr_gamma_slow(ng, p.a);
      g = (gi_lane == GI) ? gv : g;
    });
    return g;
  }
}

// ------------------------------------------------------------ buffer I/O --
// Raw buffer descriptor over one wave's chain block: the base is wave-uniform
// (SGPRs), per-lane offsets are 32-bit VGPRs and the per-column part of an
// offset is an SGPR, so the 64 column loads of a chain share one VGPR.  Lanes
// that must not touch memory get an out-of-range voffset (loads return 0,
// stores are dropped by the hardware range check).
constexpr uint32_t kOOB = 0x80000000u;
#ifndef AMH_STORE_AUX
#define AMH_STORE_AUX 2  // cache policy of state stores: nt (streaming, written once per launch)
#endif
#ifndef AMH_LOAD_AUX
#define AMH_LOAD_AUX 2  // cache policy of the factor's DMA loads: nt (read once per launch)
#endif

struct Buf {
  __amdgpu_buffer_rsrc_t rs;
  __device__ __forceinline__ Buf(const void* base, uint32_t bytes) {
    rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  }
  __device__ __forceinline__ float ld(uint32_t voff, uint32_t soff) const {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, (int)voff, (int)soff, 0));
  }
  __device__ __forceinline__ void st(float v, uint32_t voff, uint32_t soff) const {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), rs, (int)voff, (int)soff, AMH_STORE_AUX);
  }
};

__device__ __forceinline__ const void* uniform_ptr(const void* p) {
  const uint64_t u = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)u);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(u >> 32));
  return (const void*)(((uint64_t)hi << 32) | lo);
}

// The launch parameters re-read from the kernarg segment (scalar loads through
// an opaque pointer) where a persistent loop would otherwise keep every field
// live in SGPRs -- past the SGPR budget they spill to VGPR lanes, and each use
// costs a v_readlane + hazard nop.  `p` must be the kernel's first argument.
template <class T>
__device__ __forceinline__ const T& reload_kernarg(const T& p) {
  typedef __attribute__((address_space(4))) const T kconst_t;
  kconst_t* pk = (kconst_t*)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(pk));
  (void)p;
  return *(const T*)pk;
}

// v_writelane through the LLVM intrinsic (no clang builtin in ROCm 7.2)
__device__ int amh_writelane_i32(int val, int lane, int old) __asm("llvm.amdgcn.writelane.i32");

// lane J of the group takes `v` (uniform in the group), other lanes keep `old`
template <int G, int J>
__device__ __forceinline__ float capture(float old, float v, int rr) {
  if constexpr (G == 64) {
    return __int_as_float(amh_writelane_i32(__float_as_int(v), J, __float_as_int(old)));
  } else {
    return (rr == J) ? v : old;
  }
}


// Dispatch table over (model, d).  Instantiated shapes:
//   Gaussian: exact d = 64 (headline), dynamic d <= 1,2,4,8,16,32,64
//   eight schools: d <= 16;  kidiq: d = 4;  diamonds: d <= 32
template <template <int> class M, class F>
static hipError_t dispatch_dim(int d, bool allow_exact64, F&& f) {
  if (d < 1 || d > 64) return hipErrorInvalidValue;
  if (d == 64 && allow_exact64) return f.template operator()<64, M, true>();
  if (d <= 1) return f.template operator()<1, M, false>();
  if (d <= 2) return f.template operator()<2, M, false>();
  if (d <= 4) return f.template operator()<4, M, false>();
  if (d <= 8) return f.template operator()<8, M, false>();
  if (d <= 16) return f.template operator()<16, M, false>();
  if (d <= 32) return f.template operator()<32, M, false>();
  return f.template operator()<64, M, false>();
}

template <class F>
static hipError_t dispatch(int model_id, int d, F&& f) {
  switch (model_id) {
    case AMH_MODEL_GAUSSIAN:
      return dispatch_dim<GaussianM>(d, true, f);
    case AMH_MODEL_EIGHT_SCHOOLS:
      if (d > 16) return hipErrorInvalidValue;
      return f.template operator()<16, EightSchoolsM, false>();
    case AMH_MODEL_KIDIQ:
      if (d != 4) return hipErrorInvalidValue;
      return f.template operator()<4, KidiqM, true>();
    case AMH_MODEL_DIAMONDS:
      if (d > 32) return hipErrorInvalidValue;
      return f.template operator()<32, DiamondsM, false>();
    case AMH_MODEL_DIAMONDS_SS:
      if (d < 3 || d > 32) return hipErrorInvalidValue;
      return f.template operator()<32, DiamondsSSM, false>();
    case AMH_MODEL_MIXTURE:
      if (d <= 1) return f.template operator()<1, MixtureM, false>();
      if (d <= 2) return f.template operator()<2, MixtureM, false>();
      if (d <= 4) return f.template operator()<4, MixtureM, false>();
      if (d <= 8) return f.template operator()<8, MixtureM, false>();
      if (d <= 16) return f.template operator()<16, MixtureM, false>();
      return hipErrorInvalidValue;
    default:
      return hipErrorInvalidValue;
  }
}


// Row u of a "tile" partial (pooled_fused_big_kernel, d > 64): [d S_d | NPAIR
// 32x32 tiles of S_dd in MFMA register order (pair, reg R, lane) | S_a | N]
// -> its index in the packed sums vector (-1: above the diagonal of a
// diagonal tile, not part of the sums).
__device__ inline int64_t tile_to_packed(int64_t u, int64_t Vt, int d, int* prow = nullptr, int* pcol = nullptr) {
  const int64_t P = (int64_t)d * (d + 1) / 2;
  if (u < d) return u;
  if (u >= Vt - 2) return u - Vt + d + P + 2;
  if (u >= Vt - 4) return -1;  // padding (V % 4 == 0)
  const int64_t q = u - d;
  const int pair = (int)(q >> 10), R = (int)((q >> 6) & 15), lane = (int)(q & 63);
  int I = 0;
  while ((I + 1) * (I + 2) / 2 <= pair) ++I;
  const int J = pair - I * (I + 1) / 2;
  const int row = 32 * I + (R & 3) + 8 * (R >> 2) + 4 * (lane >> 5), col = 32 * J + (lane & 31);
  if (row < col) return -1;
  if (prow) *prow = row;
  if (pcol) *pcol = col;
  return d + (int64_t)col * d - (int64_t)col * (col - 1) / 2 + (row - col);
}


// the update's 4-row-aligned layout (amh_big_pooled.hip a4_base)
__device__ __forceinline__ int fp_a4_base(int d, int j) {
  const int q = j >> 2;
  return 4 * (q * d - 2 * q * (q - 1)) + (j & 3) * (d - 4 * q) - (j & ~3);
}

// entry u of the sums once its total over the groups is known: the packed
// index (tile layout above d = 64), accumulation over the steps of a pooled
// block, and (one rank, amh_pooled_step_k) the update's Sigma' entry
__device__ __forceinline__ void final_entry(int64_t u, double tot, int64_t V, double* sums, int accumulate,
                                            int tile_d, const FinalPrep& fp, bool coherent = false) {
  int row = -1, col = -1;
  const int64_t v = tile_d ? tile_to_packed(u, V, tile_d, &row, &col) : u;
  if (v < 0) return;
  const double sv = accumulate ? sums[v] + tot : tot;
  if (coherent) {  // read by another block, maybe in another XCD: write-through
    __hip_atomic_store(&sums[v], sv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    sums[v] = sv;
  }
  if (fp.scratch != nullptr && col >= 0) {
    // Sigma' = (1-g) Sigma + g S_dd / N in float, as pooled_big_prep_kernel
    const int d = tile_d;
    const int32_t it = fp.i[0];
    const double gm = (double)amh_lr_gamma(pooled_block_n(it, fp.W, fp.K), fp.a);
    const int64_t o = v - d;
    const double a = (1.0 - gm) * fp.cov[o];
    const double b = gm * (sv / fp.N);
    fp.scratch[fp_a4_base(d, col) + row] = (float)(a + b);
    if (u == d) ((int*)fp.scratch)[d * (d + 4) / 2 + 4] = it + fp.K;  // the next step's i (noise blocks)
  }
}


}  // namespace amh
