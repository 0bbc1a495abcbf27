// amh_kernels.hip -- gfx950 (CDNA4) kernels for the ARWMH hot path.
//
// Reference: savelovme/adaptive-mcmc python/kernels/arwmh.py (ARWMH.sample
// :140-207, ARWMH.init :84-138, ARWMH.sample_Pnx :230-270) and the NumPyro
// rank-one cholesky_update it calls at :190.  This is not a translation: the
// reference runs one chain per XLA:CPU program; here one wavefront lane-group
// owns one chain and the whole transition (RNG, proposal, potential, accept,
// mean / Cholesky / step-size adaptation) runs in registers.
//
// Lane mapping ("lane = row"): a chain of dimension d <= DMAX is owned by a
// group of G = DMAX lanes (G in {1,..,64}); lane r holds row r of the packed
// lower-triangular factor L in DMAX registers A[0..DMAX-1] (A[j] = L_rj, zero
// above the diagonal), plus z_r, mu_r and the per-column scalars of the
// rank-one update.  Column j of L is stored contiguously in HBM (packed,
// column-major), so the load of register j is one coalesced dword access over
// lanes j..d-1 -- no LDS staging and no transposition.
//
// Bit spec: the arithmetic order here is mirrored exactly by the C oracle
// oracle/amh_oracle.c; both compile with -ffp-contract=off and take every
// transcendental from include/amh_math.h.  See DESIGN.md "bit spec".
#include "amh_asss.h"
#include "amh_device.h"

#include <cstdlib>

namespace amh {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) float lds_float;
__device__ __forceinline__ lds_void* to_lds(const float* p) { return (lds_void*)(p); }

// Per-wave LDS staging buffer of the step kernel, in floats:
//   [ L: CPW*P (rounded to 4) | z: CPW*d | loc: CPW*d | scalars: 8 x CPW ]
__host__ __device__ __forceinline__ int wbuf_L(int cpw, int d) { return ((cpw * d * (d + 1) / 2) + 3) & ~3; }
__host__ __device__ __forceinline__ int wbuf_zd(int cpw, int d) { return ((cpw * d) + 3) & ~3; }
__host__ __device__ __forceinline__ int wbuf_floats(int cpw, int d) {
  return wbuf_L(cpw, d) + 2 * wbuf_zd(cpw, d) + 8 * cpw;
}

// Issue the DMA of one work item's chain state (global -> this wave's LDS
// buffer).  Out-of-range bytes (past C) read as zero.
template <int G, bool EXT>
__device__ __forceinline__ void prefetch_item(const StepParams& p, int64_t first, int d, float* wb, int lane) {
  constexpr int CPW = Geo<G>::CPW;
  const uint32_t P = (uint32_t)(d * (d + 1) / 2);
  const int64_t nvalid = (p.C - first) < CPW ? (p.C - first) : CPW;  // chains of this item in range
  float* wL = wb;
  float* wz = wb + wbuf_L(CPW, d);
  float* wm = wz + wbuf_zd(CPW, d);
  float* ws = wm + wbuf_zd(CPW, d);
  {
    const uint32_t bytes = (uint32_t)nvalid * P * 4u;
    const Buf b(uniform_ptr(p.in.scale + first * P), bytes);
    const bool vec = ((P * 4u) % 16u) == 0u;  // 16-B aligned chain blocks
    const uint32_t total = (uint32_t)CPW * P * 4u;
    // whole 1 KB pieces as dwordx4, the tail as dwords; exec masks keep every
    // DMA inside this wave's buffer (an LDS-DMA writes base + 4*size*lane)
    const uint32_t n16 = vec ? (total / 1024u) * 1024u : 0u;
    for (uint32_t o = 0; o < n16; o += 1024u)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b.rs, to_lds(wL + o / 4u), 16, (int)(o + 16u * lane), 0, 0, AMH_LOAD_AUX);
    for (uint32_t o = n16; o < total; o += 256u) {
      if (o + 4u * lane < total)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(b.rs, to_lds(wL + o / 4u), 4, (int)(o + 4u * lane), 0, 0, AMH_LOAD_AUX);
    }
  }
  {
    const uint32_t bytes = (uint32_t)(nvalid * d) * 4u;
    const uint32_t total = (uint32_t)(CPW * d) * 4u;
    const Buf bz(uniform_ptr(p.in.z + first * d), bytes);
    const Buf bm(uniform_ptr(p.in.loc + first * d), bytes);
    for (uint32_t o = 0; o < total; o += 256u) {
      if (o + 4u * lane < total) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(bz.rs, to_lds(wz + o / 4u), 4, (int)(o + 4u * lane), 0, 0, 0);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(bm.rs, to_lds(wm + o / 4u), 4, (int)(o + 4u * lane), 0, 0, 0);
      }
    }
  }
  if (lane < CPW) {
    const uint32_t bytes = (uint32_t)nvalid * 4u;
    const uint32_t vo = 4u * lane;
    const Buf b0(uniform_ptr(p.in.i + first), bytes);
    const Buf b1(uniform_ptr(p.in.potential_energy + first), bytes);
    // (ASSS states have no mean_accept_prob / log_step_size: an empty range, so
    // those DMAs read zeros and touch no memory)
    const Buf b2(p.in.mean_accept_prob ? uniform_ptr(p.in.mean_accept_prob + first) : p.in.i,
                 p.in.mean_accept_prob ? bytes : 0u);
    const Buf b3(p.in.log_step_size ? uniform_ptr(p.in.log_step_size + first) : p.in.i,
                 p.in.log_step_size ? bytes : 0u);
    const Buf b4(uniform_ptr(p.in.as_change + first), bytes);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(b0.rs, to_lds(ws + 0 * CPW), 4, (int)vo, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(b1.rs, to_lds(ws + 1 * CPW), 4, (int)vo, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(b2.rs, to_lds(ws + 2 * CPW), 4, (int)vo, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(b3.rs, to_lds(ws + 3 * CPW), 4, (int)vo, 0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(b4.rs, to_lds(ws + 4 * CPW), 4, (int)vo, 0, 0, 0);
  }
  {
    // 2 CPW key words: two DMAs of 64 lanes when a wave holds 64 chains (G = 1)
    const Buf bk(uniform_ptr(p.in.rng_key + 2 * first), (uint32_t)nvalid * 8u);
    static_for<(2 * CPW + 63) / 64>([&](auto H) {
      constexpr int o = 64 * H;
      if (lane + o < 2 * CPW)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(bk.rs, to_lds(ws + 5 * CPW + o), 4, (int)(4u * (lane + o)), 0, 0, 0);
    });
  }
  if (EXT && lane < CPW) {  // split path: U(z') of the batched potential kernel
    const Buf be(uniform_ptr(p.ext_pe + first), (uint32_t)nvalid * 4u);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(be.rs, to_lds(ws + 7 * CPW), 4, (int)(4u * lane), 0, 0, 0);
  }
}

// ------------------------------------------------------- phase stamps --
// Diagnostic build only (-DAMH_STAMPS, tools/stamps.py): per-wave cycle
// totals of the step kernel's phases, read back with amh_diag_stamps().
#ifdef AMH_STAMPS
constexpr int kStampWaves = 1 << 16;
constexpr int kStampSlots = 8;  // wait, store, lds->reg, prefetch, compute, tail, items, wall
__device__ unsigned long long g_stamps[kStampWaves * kStampSlots];
hipError_t diag_stamps_copy(void* host, size_t bytes) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
#define AMH_STAMP_INIT                             \
  unsigned long long st_acc[kStampSlots] = {0};    \
  unsigned long long st_t0 = __builtin_amdgcn_s_memtime(); \
  unsigned long long st_prev = st_t0;
#define AMH_STAMP(k)                                          \
  {                                                           \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t_ - st_prev;                                \
    st_prev = t_;                                             \
  }
#define AMH_STAMP_COUNT(k) st_acc[k] += 1;
#define AMH_STAMP_FLUSH(w)                                                                         \
  {                                                                                                \
    st_acc[7] = __builtin_amdgcn_s_memtime() - st_t0;                                              \
    if ((w) < kStampWaves && lane_id() < kStampSlots) g_stamps[(w) * kStampSlots + lane_id()] = 0; \
    if ((w) < kStampWaves && lane_id() == 0)                                                       \
      for (int k_ = 0; k_ < kStampSlots; ++k_) g_stamps[(w) * kStampSlots + k_] = st_acc[k_];      \
  }
#else
#define AMH_STAMP_INIT
#define AMH_STAMP(k)
#define AMH_STAMP_COUNT(k)
#define AMH_STAMP_FLUSH(w)
#endif

// -------------------------------------------------------------- step kernel --
// One or more ARWMH transitions (arwmh.py:140-207) per chain with the state
// held in registers between steps.
//
// Persistent waves walk the chain groups; while a wave computes one group
// (state in registers) the DMA engine streams the next group's state from HBM
// into the wave's LDS buffer (buffer_load ... lds), so the HBM traffic of
// the state round trip overlaps the arithmetic.
//
// Between steps the factor lives in registers in unit-lower form: U[j] holds
// U_rj = L_rj / L_jj (U_rr = 1 exactly, zero above the diagonal) and `dl`
// holds L_rr.  numpyro's cholesky_update works on exactly this pair (it
// divides the scaled factor by its diagonal, arwmh.py:190), so the update
// needs no per-column masks: the w_r of a row is zeroed exactly when its own
// column passes (w - w*1), which keeps the upper triangle at exact zeros.
// L = U diag(dl) is formed only when the state is written back.
// Step-kernel LDS, in floats: [ model data | WPB wave buffers | ticket ]
template <int G, template <int> class M>
__host__ __device__ __forceinline__ size_t step_wbuf_off(const ModelArgs& m, int d) {
  return (M<G>::lds_bytes(m, d) / sizeof(float) + 3) & ~(size_t)3;
}
template <int G, template <int> class M>
__host__ __device__ __forceinline__ size_t tickets_off(const ModelArgs& m, int d) {
  return step_wbuf_off<G, M>(m, d) + (size_t)(kBlockStep / 64) * wbuf_floats(Geo<G>::CPW, d);
}
// G = 32: per-wave broadcast scratch (64 lanes x 4 floats) after the ticket --
// the column sweeps read a column's four per-column scalars with one
// ds_read_b128 instead of four DPP + permlane16 broadcasts (three
// instructions each at this width)
template <int G, template <int> class M>
__host__ __device__ __forceinline__ size_t bcast_off(const ModelArgs& m, int d) {
  return (tickets_off<G, M>(m, d) + 4 + 3) & ~(size_t)3;
}
constexpr int kBcastFloats = 64 * 4;
template <int G, template <int> class M>
__host__ __device__ __forceinline__ size_t step_lds_bytes(const ModelArgs& m, int d) {
  if (G == 32) return (bcast_off<G, M>(m, d) + (size_t)(kBlockStep / 64) * kBcastFloats) * sizeof(float);
  return (tickets_off<G, M>(m, d) + 4) * sizeof(float);
}
__device__ __forceinline__ void lds_st4(uint32_t a, f32x4 v) {
  asm volatile("ds_write_b128 %0, %1" : : "v"(a), "v"(v) : "memory");
}

// DFIX > 0: d fixed at compile time below the group width (the diamonds
// split path, d = 26 in groups of 32): column offsets become immediates.
template <int DMAX, template <int> class M, bool EXACT, int DFIX = 0>
__global__ __launch_bounds__(kBlockStep) void arwmh_step_kernel(StepParams p) {
  const StepParams& p_outer = p;
  constexpr int G = DMAX;
  constexpr int CPW = Geo<G>::CPW;
  constexpr bool kExt = is_external<M<G>>::value;
  using Gp = Grp<G>;
  extern __shared__ float lds[];
  const int d = EXACT ? DMAX : (DFIX > 0 ? DFIX : p.d);
  M<G>::stage(lds, p.model, d);
  if (threadIdx.x == 0) lds[tickets_off<G, M>(p.model, d)] = 0.0f;  // ticket counter (bits 0)
  __syncthreads();
  const auto mctx = M<G>::prepare(p.model, d, lane_id() & (G - 1));

  const int64_t C = p.C;
  const uint32_t P = (uint32_t)(d * (d + 1) / 2);
  const int64_t n_items = (C + CPW - 1) / CPW;
  [[maybe_unused]] const int64_t wave = (int64_t)blockIdx.x * (kBlockStep / 64) + threadIdx.x / 64;
  const int wave_in_block = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));  // wave-uniform
  float* wb = lds + step_wbuf_off<G, M>(p.model, d) + (size_t)wave_in_block * wbuf_floats(CPW, d);
  const float* wL = wb;
  const float* wz = wb + wbuf_L(CPW, d);
  const float* wm = wz + wbuf_zd(CPW, d);
  const float* wsc = wm + wbuf_zd(CPW, d);
  const uint32_t oob = kOOB;
  // G = 32 at a fixed d: sweep 2 and the next proposal's broadcasts through
  // the wave's LDS scratch (the next-proposal form spilled in the ExtPotM
  // instance, 128 VGPRs, so it keeps the one-swap DPP broadcasts there)
  constexpr bool kLdsS2 = G == 32 && DFIX > 0;
  constexpr bool kLdsSP = G == 32 && DFIX > 0 && !kExt;
  constexpr int NB = 4;  // columns per LDS wait
  [[maybe_unused]] const uint32_t bs_a =
      lds_addr(lds + bcast_off<G, M>(p.model, d) + (size_t)wave_in_block * kBcastFloats);

  // Registers carry one chain group at a time.  Iteration k: wait for the
  // DMA of item k, write item k-1 back (its registers are still live), read
  // item k from LDS, start the DMA of item k+1, compute item k.  Stores are
  // issued after the wait, so the next wait never has to drain them.
  float U[DMAX];
  float dl = 0.0f, z = 0.0f, mu = 0.0f, pe = 0.0f, macc = 0.0f, lam = 0.0f, asc = 0.0f;
  [[maybe_unused]] float pe_ext = 0.0f;  // split path: U(z') computed outside
  // split path: the proposal U(z') was evaluated at, read from the split
  // buffer (loaded for the next item while this one computes) instead of
  // formed again -- the same bits (the propose pass / the previous step
  // pass made it from this state), one column sweep and the normals fewer
  [[maybe_unused]] float zp_nx = 0.0f, zp_cur = 0.0f;
  auto load_zp = [&](const StepParams& p, int64_t it_item, int ln) {
    const int rq = ln & (G - 1);
    const int64_t ch = it_item * CPW + ln / G;
    zp_nx = (rq < d && ch < C) ? p.ext_z[ch * d + rq] : 0.0f;
  };
  int32_t it = 0, nacc = 0, acc0 = 0;
  uint32_t k0 = 0, k1 = 0;
  bool updated = false;
  int64_t prev = -1;  // item whose state the registers hold
  static_for<DMAX>([&](auto J) { U[J] = 0.0f; });

  // write the registers' chain group (item `it_item`) back to HBM
  auto store_item = [&](const StepParams& p, int64_t it_item, int lane) {
    const int r = lane & (G - 1);
    const int rr = r;
    const bool act = r < d;
    const int g = lane / G;
    const int64_t first = it_item * CPW;
    const int64_t chain = first + g;
    const bool chain_ok = chain < C;
    // L = U diag(dl); factors no step of this launch updated are copied from
    // the launch input verbatim
    const bool any_upd = Gp::any(updated);
    const uint32_t vrow = (act && chain_ok) ? ((uint32_t)g * P + (uint32_t)r) * 4u : kOOB;
    const uint32_t wave_bytes = (uint32_t)CPW * P * 4u;
    const Buf Lout(uniform_ptr(p.out.scale + first * P), wave_bytes);
    const Buf Lin(uniform_ptr(p.in.scale + first * P), wave_bytes);
    // (the branch is outside the column loop: a per-column select between a
    // load and a product made the compiler wait vmcnt(0) before every store)
    if (any_upd) {
      const auto dls = Gp::src(dl);
      static_for<DMAX>([&](auto J) {
        constexpr int j = J;
        if (j < d) {
          const uint32_t so = (uint32_t)(col_off(d, j) - j) * 4u;
          const float v = U[j] * Gp::template bcast<j>(dls);
          if constexpr (EXACT || DFIX > 0) {
            // d fixed: the column offset as the instruction's immediate (an
            // SGPR offset costs an s_movk + hazard nop per column; kOOB + so
            // stays out of range)
            Lout.st(v, off_from<G, j>(vrow, oob, rr) + so, 0u);
          } else {
            Lout.st(v, off_from<G, j>(vrow, oob, rr), so);
          }
        }
        column_fence<j>();
      });
    } else {
      // verbatim copy: all loads first (into the now dead U registers), then
      // all stores, so the copy waits for memory once
      static_for<(DMAX + 15) / 16>([&](auto B) {  // batches of 16 columns
        static_for<16>([&](auto K) {
          constexpr int j = 16 * B + K;
          if constexpr (j < DMAX) {
            if (j < d) U[j] = Lin.ld(off_from<G, j>(vrow, oob, rr), (uint32_t)(col_off(d, j) - j) * 4u);
          }
        });
        static_for<16>([&](auto K) {
          constexpr int j = 16 * B + K;
          if constexpr (j < DMAX) {
            if (j < d) Lout.st(U[j], off_from<G, j>(vrow, oob, rr), (uint32_t)(col_off(d, j) - j) * 4u);
          }
        });
        __builtin_amdgcn_sched_barrier(0);
      });
    }
    if (chain_ok) {
      if (act) {
        p.out.z[chain * d + r] = z;
        p.out.loc[chain * d + r] = mu;
      }
      if (r == 0) {
        p.out.i[chain] = it;
        p.out.potential_energy[chain] = pe;
        p.out.mean_accept_prob[chain] = macc;
        p.out.log_step_size[chain] = lam;
        p.out.as_change[chain] = asc;
        p.out.rng_key[2 * chain] = k0;
        p.out.rng_key[2 * chain + 1] = k1;
        if (p.accept_count != nullptr) p.accept_count[chain] = acc0 + nacc;  // loaded with the item
      }
    }
  };

  // Chain groups are split into one contiguous range per block; inside a
  // block the waves take groups from an LDS ticket counter, so waves that
  // lose the SIMD's issue arbitration simply process fewer groups (static
  // striding left the slowest wave ~1.4x behind the mean).  The ticket for
  // the group after next is drawn right after a prefetch is issued.  (A
  // single device-wide counter was tried: its global atomics serialise and
  // stall the memory pipeline behind them.)
  const int64_t blk_lo = n_items * (int64_t)blockIdx.x / gridDim.x;
  const int64_t blk_hi = n_items * ((int64_t)blockIdx.x + 1) / gridDim.x;
  const uint32_t tk_addr = lds_addr(lds) + (uint32_t)(tickets_off<G, M>(p.model, d) * sizeof(float));
  auto ticket = [&]() -> int64_t {
    uint32_t v = 0;
    if (lane_id() == 0) {
      asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(tk_addr), "v"(1u) : "memory");
    }
    return blk_lo + (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)v);
  };
  AMH_STAMP_INIT
  int64_t item = ticket();
  int64_t nxt = item < blk_hi ? ticket() : blk_hi;

  if (item < blk_hi) {
    prefetch_item<G, kExt>(p, item * CPW, d, wb, lane_id());
    if constexpr (kExt) load_zp(p, item, lane_id());
  }
  for (; item < blk_hi;) {
    // Every lane-dependent quantity is derived from an opaque copy of the lane
    // id inside the loop: otherwise the compiler hoists dozens of per-column
    // addresses and masks out of this persistent loop and runs out of VGPRs.
    int lane = lane_id();
    asm volatile("" : "+v"(lane));
    // the launch parameters re-read from the kernarg segment each item
    // (scalar loads through an opaque pointer): kept live across the loop,
    // their ~60 SGPRs spilled to VGPR lanes and every item paid hundreds of
    // v_readlane / v_writelane + hazard nops
    const StepParams& p = reload_kernarg(p_outer);
    const int r = lane & (G - 1);
    const int rr = r;
    const bool act = r < d;
    const int64_t first = item * CPW;
    const int g = lane / G;
    const int64_t chain = first + g;
    const bool chain_ok = chain < C;

    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this item's DMA has landed
    __builtin_amdgcn_s_setprio(3);  // hand-over phase first (as arwmh_step64_kernel): diamonds_ss +1.8 %
    AMH_STAMP(0)
    if (prev >= 0) store_item(p, prev, lane);
    AMH_STAMP(1)

    // ---- state: LDS -> registers
    {
      // LDS addresses made opaque per item so the 64 column addresses are
      // not hoisted out of the chain loop (one base VGPR + immediate offsets)
      lds_float* Lrow = (lds_float*)(wL + g * P + r);
      asm volatile("" : "+v"(Lrow));
      const lds_float* Lg = (const lds_float*)(wL + g * P);
      dl = act ? Lg[col_off(d, r)] : 0.0f;
      const float inv = (amh_isfinite(dl) && dl != 0.0f) ? 1.0f / dl : 0.0f;
      const auto invs = Gp::src(inv);
      static_for<DMAX>([&](auto J) {
        constexpr int j = J;
        U[j] = 0.0f;
        if (j < d) {
          const float x = Lrow[col_off(d, j) - j];  // garbage for r < j: masked below
          U[j] = set_one_at<G, j>(keep_above<G, j>(x * Gp::template bcast<j>(invs), rr), rr);
        }
        column_fence<j>();
      });
      z = act ? wz[g * d + r] : 0.0f;
      mu = act ? wm[g * d + r] : 0.0f;
      it = __float_as_int(wsc[0 * CPW + g]);
      if constexpr (G == 64) it = __builtin_amdgcn_readfirstlane(it);  // wave-uniform: scalar table lookups
      acc0 = (p.accept_count != nullptr && chain_ok && r == 0) ? p.accept_count[chain] : 0;
      pe = wsc[1 * CPW + g];
      macc = wsc[2 * CPW + g];
      lam = wsc[3 * CPW + g];
      asc = wsc[4 * CPW + g];
      k0 = (uint32_t)__float_as_int(wsc[5 * CPW + 2 * g]);
      k1 = (uint32_t)__float_as_int(wsc[5 * CPW + 2 * g + 1]);
      if constexpr (kExt) {
        pe_ext = wsc[7 * CPW + g];
        zp_cur = zp_nx;
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): buffer consumed before it is refilled
    AMH_STAMP(2)
    int64_t nxt2 = blk_hi;
    if (nxt < blk_hi) {
      prefetch_item<G, kExt>(p, nxt * CPW, d, wb, lane);
      if constexpr (kExt) load_zp(p, nxt, lane);
      nxt2 = ticket();
    }
    __builtin_amdgcn_s_setprio(0);
    AMH_STAMP(3)

    nacc = 0;
    updated = false;
    for (int32_t t = 0; t < p.n_steps; ++t) {
      // ---- noise (arwmh.py:162-165, 174): stream position = state.i
      float u, zp;
      const float el = amh_expf(lam);
      if constexpr (kExt) {
        // split path (n_steps == 1): z' from the split buffer, u = U(W_d)
        u = amh_unif01_from_bits(amh_step_word((uint32_t)d, (uint32_t)it, k0, k1));
        zp = act ? zp_cur : 0.0f;
      } else {
        float xi;
        step_noise<G>(r, d, (uint32_t)it, k0, k1, xi, u);
        xi = act ? xi : 0.0f;

        // ---- proposal z' = z + (L e^lam + eps I) xi  (arwmh.py:166-167),
        //      L xi = U (dl * xi)
        const float eta = dl * xi;
        // four interleaved partial sums (columns j mod 4): four independent
        // FMA chains instead of one 64-long dependency chain
        float a4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        static_for<DMAX>([&](auto J) {
          if (J < d) a4[J & 3] = fmaf(U[J], Gp::template bcast<J>(eta), a4[J & 3]);
          column_fence<J, 16>();
        });
        const float acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        zp = act ? z + fmaf(el, acc, p.eps * xi) : 0.0f;
      }

      // ---- potential, NaN -> +inf (arwmh.py:169-171)
      float pep;
      if constexpr (kExt) {
        pep = pe_ext;  // n_steps == 1 (host-enforced)
      } else {
        pep = M<G>::potential(zp, r, d, mctx, lds);
      }
      if (amh_isnan(pep)) pep = INFINITY;

      // ---- accept / reject (arwmh.py:173-178)
      const float ex = amh_expf(pe - pep);
      const float alpha = (ex > 1.0f) ? 1.0f : ex;
      const bool accept = u < alpha;
      const float zn = accept ? zp : z;
      const float pen = accept ? pep : pe;
      nacc += accept ? 1 : 0;

      // ---- schedule (arwmh.py:180-185)
      const int32_t itr = it + 1;
      const int32_t n = (it < p.W) ? itr : itr - p.W;
      const float gamma = lookup_gamma<G>(p, n);
      const float maccn = macc + (alpha - macc) / (float)n;

      // ---- mean and step size (arwmh.py:188-189, 193)
      const float delta = act ? zn - mu : 0.0f;
      const float mun = act ? mu + gamma * delta : 0.0f;
      const float lamn = lam + gamma * (alpha - p.target);
      const float e1 = amh_expf(lamn);

      // ---- rank-one update of sqrt(1-gamma) L by (delta, gamma)
      //      (arwmh.py:190-191 -> numpyro cholesky_update), NaN -> keep L.
      const float sq = sqrtf(1.0f - gamma);
      const float ajj = sq * dl;
      const float Dg = ajj * ajj;
      const float one = (amh_isfinite(ajj) && ajj != 0.0f) ? 1.0f : __int_as_float(0x7FC00000);

      // sweep 1: w*_j = w_j when column j is applied (forward solve U w* = delta)
      float w = delta;
      float ws = 0.0f;
      static_for<DMAX>([&](auto J) {
        if (J < d) {
          const float wj = Gp::template bcast<J>(w);
          ws = capture<G, J>(ws, wj, rr);
          w = fmaf(-wj, U[J], w);
        }
        column_fence<J>();
      });

      // per-column scalars, one column per lane; b_j by exclusive scan
      const float gw2 = act ? gamma * (ws * ws) : 0.0f;
      const float tsc = act ? gw2 / Dg : 0.0f;
      const float b = 1.0f + Gp::excl_scan(tsc, rr);
      const float g2 = (b * Dg) + gw2;
      const float dn = g2 / b;
      const float c = (gamma * ws) / g2;
      const float q = sqrtf(dn);
      const float dnew = fmaf(c, 0.0f, one) * q;  // new diagonal of column r

      // A NaN anywhere in numpyro's updated factor shows up in its new diagonal
      // (fmaf(c, 0, U_jj) q_j): c_j, q_j and U_jj = A_jj / A_jj are the only
      // per-column quantities, and every off-diagonal entry is finite whenever
      // they are ("keep-L rule").  So the keep-L test of
      // arwmh.py:191 is decided before the factor is touched.
      const bool revert = Gp::any(act && amh_isnan(dnew));
      float sacc = 0.0f;
      float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // as_change partial sums (columns j mod 4)
      if (!revert) {
        // sweep 2: U'_rj = U_rj + c_j w_r^{(j+1)};  as_change terms
        //   L'_rj e1 - L_rj e0 = U'_rj (q_j e1) - U_rj (dl_j e0)
        //   = U_rj (q_j e1 - dl_j e0) + (c_j q_j e1) w_r^{(j+1)}
        const float ac = (q * e1) - (dl * el);
        const float bc = (c * q) * e1;
        w = delta;
        auto col2 = [&](auto J, float wj, float cj, float aj, float bj) {
          const float uo = U[J];
          w = fmaf(-wj, uo, w);
          const float un = fmaf(cj, w, uo);
          const float tt = fmaf(uo, aj, bj * w);
          s4[J & 3] = fmaf(tt, tt, s4[J & 3]);
          U[J] = un;
        };
        if constexpr (kLdsS2) {
          // the group's (ws, c, ac, bc) through the wave's LDS scratch, four
          // columns per wait (asm reads: no vmcnt wait on the DMA prefetch)
          lds_st4(bs_a + 16u * (uint32_t)lane, f32x4{ws, c, ac, bc});
          const uint32_t ga = bs_a + 16u * (uint32_t)(g * G);
          static_for<(DMAX + NB - 1) / NB>([&](auto B) {
            f32x4 qv[NB];
            static_for<NB>([&](auto Q) {
              constexpr int j = NB * B + Q;
              qv[Q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
              if (j < d) qv[Q] = lds_ld4<16 * j>(ga);
            });
            lds_wait_n<NB>(qv);
            static_for<NB>([&](auto Q) {
              constexpr int j = NB * B + Q;
              if (j < d) col2(std::integral_constant<int, j>{}, qv[Q][0], qv[Q][1], qv[Q][2], qv[Q][3]);
            });
            column_fence<NB * B + NB - 1>();
          });
        } else {
          static_for<DMAX>([&](auto J) {
            if (J < d) {
              col2(J, Gp::template bcast<J>(ws), Gp::template bcast<J>(c), Gp::template bcast<J>(ac),
                   Gp::template bcast<J>(bc));
            }
            column_fence<J>();
          });
        }
        sacc = (s4[0] + s4[1]) + (s4[2] + s4[3]);
        asc = sqrtf(Gp::sum(act ? sacc : 0.0f));
        dl = act ? q : 0.0f;
        updated = true;
      } else {
        // factor unchanged: as_change = || L (e1 - e0) ||_F, L_rj = U_rj dl_j
        const float ac = (dl * e1) - (dl * el);
        static_for<DMAX>([&](auto J) {
          if (J < d) {
            const float tt = U[J] * Gp::template bcast<J>(ac);
            s4[J & 3] = fmaf(tt, tt, s4[J & 3]);
          }
          column_fence<J>();
        });
        sacc = (s4[0] + s4[1]) + (s4[2] + s4[3]);
        asc = sqrtf(Gp::sum(act ? sacc : 0.0f));
      }

      // ---- commit (arwmh.py:199-207)
      it = itr;
      z = zn;
      pe = pen;
      macc = maccn;
      mu = mun;
      lam = lamn;

      if (p.col_z != nullptr || p.col_pe != nullptr) {
        if ((t + 1) % p.thinning == 0 && chain_ok) {
          const int64_t k = t / p.thinning;
          if (p.col_z != nullptr && act) p.col_z[(k * C + chain) * d + r] = z;
          if (p.col_pe != nullptr && r == 0) p.col_pe[k * C + chain] = pe;
        }
      }
    }
    if constexpr (kExt) {
      // split path: the next transition's proposal, exactly as propose_kernel
      // forms it from the state this launch stores -- L = U diag(dl) if a step
      // updated the factor (else the input factor, whose U these registers
      // already are), reloaded as U = L / L_jj -- so the batched potential of
      // the next launch can run without a propose pass over the factor
      if (p.xprop_next != nullptr) {
        const bool any_upd = Gp::any(updated);
        const float inv = (amh_isfinite(dl) && dl != 0.0f) ? 1.0f / dl : 0.0f;
        float xi, u_unused;
        step_noise<G>(r, d, (uint32_t)it, k0, k1, xi, u_unused);
        xi = act ? xi : 0.0f;
        const float el = amh_expf(lam);
        const float eta = dl * xi;
        float a4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        auto colp = [&](auto J, float dj, float ij, float ej) {
          constexpr int j = J;
          const float un = set_one_at<G, j>(keep_above<G, j>((U[j] * dj) * ij, rr), rr);
          a4[j & 3] = fmaf(any_upd ? un : U[j], ej, a4[j & 3]);
        };
        if constexpr (kLdsSP) {
          // (dl, 1 / dl, eta) through the LDS scratch, as sweep 2
          lds_st4(bs_a + 16u * (uint32_t)lane, f32x4{dl, inv, eta, 0.0f});
          const uint32_t ga = bs_a + 16u * (uint32_t)(g * G);
          static_for<(DMAX + NB - 1) / NB>([&](auto B) {
            f32x4 qv[NB];
            static_for<NB>([&](auto Q) {
              constexpr int j = NB * B + Q;
              qv[Q] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
              if (j < d) qv[Q] = lds_ld4<16 * j>(ga);
            });
            lds_wait_n<NB>(qv);
            static_for<NB>([&](auto Q) {
              constexpr int j = NB * B + Q;
              if (j < d) colp(std::integral_constant<int, j>{}, qv[Q][0], qv[Q][1], qv[Q][2]);
            });
            column_fence<NB * B + NB - 1, 16>();
          });
        } else {
          const auto dls = Gp::src(dl), invs = Gp::src(inv), etas = Gp::src(eta);
          static_for<DMAX>([&](auto J) {
            constexpr int j = J;
            if (j < d) {
              // the broadcasts run with every lane of the group active (a
              // broadcast under a lane-dependent branch would read an inactive
              // source lane); then the load path's own masking
              colp(J, Gp::template bcast<j>(dls), Gp::template bcast<j>(invs), Gp::template bcast<j>(etas));
            }
            column_fence<j, 16>();
          });
        }
        const float acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
        const float zp = act ? z + fmaf(el, acc, p.eps * xi) : 0.0f;
        if (chain_ok && act) p.xprop_next[chain * d + r] = zp;
      }
    }

    prev = item;
    item = nxt;
    nxt = nxt2;
    AMH_STAMP(4)
    AMH_STAMP_COUNT(6)
  }
  if (prev >= 0) {
    int lane = lane_id();
    asm volatile("" : "+v"(lane));
    store_item(p, prev, lane);
  }
  __builtin_amdgcn_s_waitcnt(0);
  AMH_STAMP(5)
  AMH_STAMP_FLUSH(wave)
}

// -------------------------------------------------------------- init kernel --
// arwmh.py:84-138 with numpyro init_to_uniform (U(-2,2) per coordinate).
template <int DMAX, template <int> class M, bool EXACT>
__global__ __launch_bounds__(kBlock) void arwmh_init_kernel(InitParams p) {
  constexpr int G = DMAX;
  using Gp = Grp<G>;
  extern __shared__ float lds[];
  const int d = EXACT ? DMAX : p.d;
  M<G>::stage(lds, p.model, d);
  __syncthreads();
  const auto mctx = M<G>::prepare(p.model, d, lane_id() & (G - 1));
  const int r = Gp::r();
  const bool act = r < d;
  const int64_t C = p.C;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const int64_t n_items = (C + Geo<G>::CPW - 1) / Geo<G>::CPW;
  const int64_t wave0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t wstride = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t item = wave0; item < n_items; item += wstride) {
    const int64_t chain = item_chain<G>(item);
    const bool chain_ok = chain < C;
    const int64_t cl = chain_ok ? chain : C - 1;
    const uint64_t gc = (uint64_t)(p.chain_offset + cl);
    const amh_u32x4 kk = amh_philox4x32_10((uint32_t)gc, (uint32_t)(gc >> 32), 0u, AMH_TAG_CHAINKEY,
                                           p.key0, p.key1);
    float z0 = 0.0f;
    if (act) {
      if (p.init_z != nullptr) {
        z0 = p.init_z[cl * d + r];
      } else {
        const amh_u32x4 o = amh_philox4x32_10((uint32_t)r, 0u, 0u, AMH_TAG_INIT, kk.v[0], kk.v[1]);
        const float v = (amh_unif01_from_bits(o.v[0]) * 4.0f) + (-2.0f);
        z0 = (v < -2.0f) ? -2.0f : v;
      }
    }
    const float pe0 = M<G>::potential(z0, r, d, mctx, lds);
    if (chain_ok) {
      float* Lout = p.out.scale + chain * P;
      if (act) {
        p.out.z[chain * d + r] = z0;
        p.out.loc[chain * d + r] = z0;
        // row r of the identity: entries (r, j), j <= r
        for (int j = 0; j <= r; ++j) Lout[col_off(d, j) + (r - j)] = (j == r) ? 1.0f : 0.0f;
      }
      if (r == 0) {
        p.out.i[chain] = 0;
        p.out.potential_energy[chain] = pe0;
        p.out.mean_accept_prob[chain] = 0.0f;
        p.out.log_step_size[chain] = 0.0f;
        p.out.as_change[chain] = 0.0f;
        p.out.rng_key[2 * chain] = kk.v[0];
        p.out.rng_key[2 * chain + 1] = kk.v[1];
      }
    }
  }
}

// --------------------------------------------------------- potential kernel --
template <int DMAX, template <int> class M, bool EXACT>
__global__ __launch_bounds__(kBlock) void potential_kernel(PotParams p) {
  constexpr int G = DMAX;
  using Gp = Grp<G>;
  extern __shared__ float lds[];
  const int d = EXACT ? DMAX : p.d;
  M<G>::stage(lds, p.model, d);
  __syncthreads();
  const auto mctx = M<G>::prepare(p.model, d, lane_id() & (G - 1));
  const int r = Gp::r();
  const bool act = r < d;
  const int64_t C = p.n;
  const int64_t n_items = (C + Geo<G>::CPW - 1) / Geo<G>::CPW;
  const int64_t wave0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t wstride = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t item = wave0; item < n_items; item += wstride) {
    const int64_t chain = item_chain<G>(item);
    const bool chain_ok = chain < C;
    const int64_t cl = chain_ok ? chain : C - 1;
    const float x = act ? p.z[cl * d + r] : 0.0f;
    const float pe = M<G>::potential(x, r, d, mctx, lds);
    if (chain_ok && r == 0) p.pe[chain] = pe;
  }
}

// -------------------------------------------------------- sample_Pnx kernel --
// arwmh.py:230-270: all chains share one frozen adapt state; chain c = (pt, s)
// starts at x[pt] with key split(rng_key, C)[c] and runs n steps, noise at
// stream position t.  L stays in registers for every chain the wave visits.
template <int DMAX, template <int> class M, bool EXACT>
__global__ __launch_bounds__(kBlock) void sample_pnx_kernel(PnxParams p) {
  constexpr int G = DMAX;
  using Gp = Grp<G>;
  extern __shared__ float lds[];
  const int d = EXACT ? DMAX : p.d;
  M<G>::stage(lds, p.model, d);
  __syncthreads();
  const auto mctx = M<G>::prepare(p.model, d, lane_id() & (G - 1));
  const int r = Gp::r();
  const bool act = r < d;
  const int64_t C = p.n_points * p.n_samples;
  const int64_t n_items = (C + Geo<G>::CPW - 1) / Geo<G>::CPW;
  const int64_t wave0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t wstride = (int64_t)gridDim.x * (kBlock / 64);
  float A[DMAX];
#pragma unroll
  for (int j = 0; j < DMAX; ++j) {
    A[j] = 0.0f;
    if (j < d) {
      if (r >= j && act) A[j] = p.scale[col_off(d, j) + (r - j)];
    }
  }
  const float el = amh_expf(p.log_step_size);
  for (int64_t item = wave0; item < n_items; item += wstride) {
    const int64_t chain = item_chain<G>(item);
    const bool chain_ok = chain < C;
    const int64_t cl = chain_ok ? chain : C - 1;
    const int64_t pt = cl / p.n_samples;
    const amh_u32x4 kk = amh_philox4x32_10((uint32_t)cl, (uint32_t)((uint64_t)cl >> 32), 0u, AMH_TAG_SPLIT,
                                           p.key0, p.key1);
    float z = act ? p.x[pt * d + r] : 0.0f;
    float pe = M<G>::potential(z, r, d, mctx, lds);
    for (int32_t t = 0; t < p.n; ++t) {
      float xi, u;
      step_noise<G>(r, d, (uint32_t)t, kk.v[0], kk.v[1], xi, u);
      xi = act ? xi : 0.0f;
      float acc = 0.0f;
      static_for<DMAX>([&](auto J) {
        if (J < d) acc = fmaf(A[J], Gp::template bcast<J>(xi), acc);
      });
      const float zp = act ? z + fmaf(el, acc, p.eps * xi) : 0.0f;
      float pep = M<G>::potential(zp, r, d, mctx, lds);
      if (amh_isnan(pep)) pep = INFINITY;
      const float ex = amh_expf(pe - pep);
      const float alpha = (ex > 1.0f) ? 1.0f : ex;
      const bool accept = u < alpha;
      z = accept ? zp : z;
      pe = accept ? pep : pe;
    }
    if (chain_ok && act) p.out[cl * d + r] = z;
  }
}

// ------------------------------------------------------------ chain keys ----
__global__ void chain_keys_kernel(uint32_t key0, uint32_t key1, int64_t offset, int64_t n, uint32_t* out) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  const uint64_t g = (uint64_t)(offset + c);
  const amh_u32x4 o = amh_philox4x32_10((uint32_t)g, (uint32_t)(g >> 32), 0u, AMH_TAG_CHAINKEY, key0, key1);
  out[2 * c] = o.v[0];
  out[2 * c + 1] = o.v[1];
}

// ------------------------------------------------------ d = 64 step kernel --
// The headline shape (BASELINE configs[1]: the d = 64 Gaussian, one chain per
// wave).  The same transition and the same float operations as
// arwmh_step_kernel<64, GaussianM, true> (bit-identical, oracle: orc_step);
// what differs is how data moves between HBM, LDS and registers:
//
// * Write-back through LDS.  After the DMA of item k has landed, one pass over
//   the columns reads item k's column j from the wave's LDS buffer and, at the
//   same addresses, writes item k-1's column j of L' = U diag(dl) (LDS is in
//   order within a wave, so the read sees the input).  The buffer then holds
//   item k-1's factor in the packed layout and goes to HBM as 9 full-lane
//   buffer_store_dwordx4 instead of 64 partially masked buffer_store_dword.
// * Exec-masked column ops.  Column j's LDS read and its normalisation touch
//   lanes r > j only (exec set by one SALU shift inside the asm), so the unit
//   diagonal and the zeros above it stay in the registers from the previous
//   chain; sweep 1 runs on lanes r > j, so lane r keeps its w_r when its own
//   column passes -- that is the forward-solve value the general kernel
//   captures with a v_writelane per column.
// * Broadcasts from LDS.  The per-column values every lane needs (dl_j and
//   1/l_j in the swap, eta_j of the proposal, diff_j of the potential, and the
//   four coefficients of sweep 2) are written once per lane into a 1 KiB
//   per-wave scratch and read back four columns at a time with broadcast
//   ds_read_b128, in place of v_readlane + s_nop per column.  Only sweep 1,
//   whose w_j is serial, still uses v_readlane.
#ifndef AMH_S64_WAVES
#define AMH_S64_WAVES 16
#endif
constexpr int kS64Waves = AMH_S64_WAVES;
#ifndef AMH_S64_EB
#define AMH_S64_EB 8
#endif
#ifndef AMH_S64_PB
#define AMH_S64_PB 8
#endif
constexpr int kS64EB = AMH_S64_EB;  // proposal: broadcast columns per LDS wait (16 or 8)
constexpr int kS64PB = AMH_S64_PB;  // potential: columns per LDS wait (16 or 8)
static_assert((kS64EB == 16 || kS64EB == 8) && (kS64PB == 16 || kS64PB == 8), "batch sizes");
typedef uint32_t uint32x4_t_ __attribute__((ext_vector_type(4)));
constexpr int kS64P = 2080;                   // d(d+1)/2
constexpr int kS64Z = 2080, kS64M = 2144, kS64S = 2208, kS64X = 2216;  // wave-buffer offsets (floats)
constexpr int kS64WB = kS64X + 64;            // floats per wave buffer (9,120 B): 64-float scratch
constexpr int kS64Model = 64 * 68;            // GaussianM<64> rows (lds_bytes / 4)
static_assert(kS64Z == 2080 && kS64S == kS64M + 64, "layout of prefetch_item<64>");
// + 32 floats: the ticket, and slack for flush_factor's 9 KiB read of the last wave buffer
template <int WPB = kS64Waves>
constexpr size_t s64_lds_bytes() { return ((size_t)kS64Model + (size_t)WPB * kS64WB + 32) * sizeof(float); }

constexpr int s64_col(int j) { return j * 64 - j * (j - 1) / 2; }  // packed column offset

// lanes r > J read the dword at a + OFF into x (others keep x); pending until lds_wait
template <int J, int OFF>
__device__ __forceinline__ void s64_rd_above(float& x, uint32_t a) {
  uint64_t sv;
  asm volatile("s_mov_b64 %1, exec\n\ts_lshl_b64 exec, -1, %3\n\tds_read_b32 %0, %2 offset:%4\n\ts_mov_b64 exec, %1"
               : "+v"(x), "=&s"(sv) : "v"(a), "n"(J + 1), "n"(OFF));
}
// lanes r >= J write v to a + OFF
template <int J, int OFF>
__device__ __forceinline__ void s64_wr_from(uint32_t a, float v) {
  uint64_t sv;
  asm volatile("s_mov_b64 %0, exec\n\ts_lshl_b64 exec, -1, %3\n\tds_write_b32 %1, %2 offset:%4\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(a), "v"(v), "n"(J), "n"(OFF) : "memory");
}
// lanes r > J: u = t * s
template <int J>
__device__ __forceinline__ void s64_mul_above(float& u, float t, float s) {
  uint64_t sv;
  asm volatile("s_mov_b64 %1, exec\n\ts_lshl_b64 exec, -1, %4\n\tv_mul_f32 %0, %2, %3\n\ts_mov_b64 exec, %1"
               : "+v"(u), "=&s"(sv) : "v"(t), "v"(s), "n"(J + 1));
}
// sweep 1, column J: w_J broadcast, then w -= w_J U_rJ on lanes r > J.  A VALU
// read of an SGPR written by v_readlane needs two wait states, and SALU
// instructions in between do not provide them (measured: with only the exec
// setup in between, a few chains per thousand read the previous column's
// w_j), so the s_nop 1 stays.
template <int J>
__device__ __forceinline__ void s64_sweep1(float& w, float u) {
  uint64_t sv;
  uint32_t t;
  asm volatile("s_mov_b64 %2, exec\n\ts_lshl_b64 exec, -1, %5\n\tv_readlane_b32 %1, %0, %4\n\ts_nop 1\n\t"
               "v_fma_f32 %0, -%1, %3, %0\n\ts_mov_b64 exec, %2"
               : "+v"(w), "=&s"(t), "=&s"(sv) : "v"(u), "n"(J), "n"(J + 1));
}
// LDS batches read and waited for in ONE statement (outputs "=&v"): per
// batch one boundary pad instead of two (the separate read and wait
// statements each had hipcc's pad around them).  AMH_S64_LDSW=0 keeps the
// separate statements (A/B).
#ifndef AMH_S64_LDSW
#define AMH_S64_LDSW 1
#endif
template <int O0, int O1>
__device__ __forceinline__ void lds_ld4x2w(f32x4& a, f32x4& b, uint32_t addr) {
  asm volatile("ds_read_b128 %0, %2 offset:%3\n\tds_read_b128 %1, %2 offset:%4\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(a), "=&v"(b)
               : "v"(addr), "n"(O0), "n"(O1));
}
// a, b from addr0 (offsets O0, O1); c, d from addr1 (O2, O3)
template <int O0, int O1, int O2, int O3>
__device__ __forceinline__ void lds_ld4x4w(f32x4& a, f32x4& b, f32x4& c, f32x4& d, uint32_t addr0, uint32_t addr1) {
  asm volatile("ds_read_b128 %0, %4 offset:%6\n\tds_read_b128 %1, %4 offset:%7\n\t"
               "ds_read_b128 %2, %5 offset:%8\n\tds_read_b128 %3, %5 offset:%9\n\ts_waitcnt lgkmcnt(0)"
               : "=&v"(a), "=&v"(b), "=&v"(c), "=&v"(d)
               : "v"(addr0), "v"(addr1), "n"(O0), "n"(O1), "n"(O2), "n"(O3));
}

// sweep 1 over eight columns J0 .. J0 + 7 (seven when J0 = 56: columns up to
// 62) in one statement: exec saved once and restored once, each column
// s_lshl exec (lanes r > J) / v_readlane / s_nop 1 / v_fma / s_nop 0 -- the
// s_nop 0 is the VALU-write -> v_readlane wait state of the next column (the
// per-column statements had hipcc's boundary pad there, plus an exec save
// and restore per column: 8 slots per column, now 5).  The same fma, in the
// same order, as s64_sweep1.
#define AMH_SW1_COL(k)                                                          \
  "s_lshl_b64 exec, -1, %[s" #k "]\n\tv_readlane_b32 %[t], %[w], %[l" #k "]\n\t" \
  "s_nop 1\n\tv_fma_f32 %[w], -%[t], %[u" #k "], %[w]\n\ts_nop 0\n\t"
template <int J0>
__device__ __forceinline__ void s64_sweep1x8(float& w, const float (&U)[64]) {
  uint64_t sv;
  uint32_t t;
  if constexpr (J0 + 7 <= 62) {
    asm volatile("s_mov_b64 %[sv], exec\n\t" AMH_SW1_COL(0) AMH_SW1_COL(1) AMH_SW1_COL(2) AMH_SW1_COL(3)
                 AMH_SW1_COL(4) AMH_SW1_COL(5) AMH_SW1_COL(6) AMH_SW1_COL(7) "s_mov_b64 exec, %[sv]"
                 : [w] "+v"(w), [t] "=&s"(t), [sv] "=&s"(sv)
                 : [u0] "v"(U[J0]), [u1] "v"(U[J0 + 1]), [u2] "v"(U[J0 + 2]), [u3] "v"(U[J0 + 3]),
                   [u4] "v"(U[J0 + 4]), [u5] "v"(U[J0 + 5]), [u6] "v"(U[J0 + 6]), [u7] "v"(U[J0 + 7]),
                   [s0] "n"(J0 + 1), [s1] "n"(J0 + 2), [s2] "n"(J0 + 3), [s3] "n"(J0 + 4), [s4] "n"(J0 + 5),
                   [s5] "n"(J0 + 6), [s6] "n"(J0 + 7), [s7] "n"(J0 + 8), [l0] "n"(J0), [l1] "n"(J0 + 1),
                   [l2] "n"(J0 + 2), [l3] "n"(J0 + 3), [l4] "n"(J0 + 4), [l5] "n"(J0 + 5), [l6] "n"(J0 + 6),
                   [l7] "n"(J0 + 7));
  } else {
    static_assert(J0 == 56, "sweep 1 covers columns 0 .. 62");
    asm volatile("s_mov_b64 %[sv], exec\n\t" AMH_SW1_COL(0) AMH_SW1_COL(1) AMH_SW1_COL(2) AMH_SW1_COL(3)
                 AMH_SW1_COL(4) AMH_SW1_COL(5) AMH_SW1_COL(6) "s_mov_b64 exec, %[sv]"
                 : [w] "+v"(w), [t] "=&s"(t), [sv] "=&s"(sv)
                 : [u0] "v"(U[J0]), [u1] "v"(U[J0 + 1]), [u2] "v"(U[J0 + 2]), [u3] "v"(U[J0 + 3]),
                   [u4] "v"(U[J0 + 4]), [u5] "v"(U[J0 + 5]), [u6] "v"(U[J0 + 6]), [s0] "n"(J0 + 1),
                   [s1] "n"(J0 + 2), [s2] "n"(J0 + 3), [s3] "n"(J0 + 4), [s4] "n"(J0 + 5), [s5] "n"(J0 + 6),
                   [s6] "n"(J0 + 7), [l0] "n"(J0), [l1] "n"(J0 + 1), [l2] "n"(J0 + 2), [l3] "n"(J0 + 3),
                   [l4] "n"(J0 + 4), [l5] "n"(J0 + 5), [l6] "n"(J0 + 6));
  }
}
#undef AMH_SW1_COL
#ifndef AMH_S64_SW1_PERCOL
#define AMH_S64_SW1_PERCOL 0  // 1: the per-column statements (A/B)
#endif
// the whole sweep 1 (columns 0 .. 62)
__device__ __forceinline__ void s64_sweep1_all(float& w, const float (&U)[64]) {
#if AMH_S64_SW1_PERCOL
  static_for<63>([&](auto J) {
    s64_sweep1<J>(w, U[J]);
    column_fence<J>();
  });
#else
  static_for<8>([&](auto B) {
    s64_sweep1x8<8 * B>(w, U);
    __builtin_amdgcn_sched_barrier(0);
  });
#endif
}

// lanes 16Q .. 16Q+15 write v0..v3 at a, a+64, a+128, a+192 (a = scratch + 4 (r mod 16))
template <int Q>
__device__ __forceinline__ void s64_wr4_quarter(uint32_t a, float v0, float v1, float v2, float v3) {
  uint64_t sv;
  asm volatile("s_mov_b64 %0, exec\n\ts_bfm_b64 exec, 16, %6\n\tds_write_b32 %1, %2\n\t"
               "ds_write_b32 %1, %3 offset:64\n\tds_write_b32 %1, %4 offset:128\n\t"
               "ds_write_b32 %1, %5 offset:192\n\ts_mov_b64 exec, %0"
               : "=&s"(sv) : "v"(a), "v"(v0), "v"(v1), "v"(v2), "v"(v3), "n"(16 * Q) : "memory");
}
__device__ __forceinline__ void s64_wr(uint32_t a, float v) {  // this lane's dword at a
  asm volatile("ds_write_b32 %0, %1" : : "v"(a), "v"(v) : "memory");
}
template <int OFF>
__device__ __forceinline__ void s64_wr_off(uint32_t a, float v) {
  asm volatile("ds_write_b32 %0, %1 offset:%2" : : "v"(a), "v"(v), "n"(OFF) : "memory");
}
__device__ __forceinline__ void s64_wait() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
template <class T>
__device__ __forceinline__ void s64_tie(T& a) { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a)); }
template <class T>
__device__ __forceinline__ void s64_tie(T& a, T& b) { asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(a), "+v"(b)); }

// lane J takes v (its own value), the others keep old -- capture<64, J> of a
// broadcast of lane J's own value, without the v_readlane / v_writelane pair
template <int J>
__device__ __forceinline__ float s64_keep_at(float old, float v) {
  float out;
  unsigned long long m;
  asm("s_lshl_b64 %1, 1, %4\n\tv_cndmask_b32_e64 %0, %2, %3, %1" : "=v"(out), "=&s"(m) : "v"(old), "v"(v), "n"(J));
  return out;
}

// The d = 64 Gaussian potential (GaussianM<64>::potential, the same float
// operations and order) with diff_j read back from the wave's scratch x_a
// (one ds_write, then 16-B broadcast reads) instead of 64 v_readlane.
__device__ __forceinline__ float s64_gauss_pot(float diff, uint32_t x_a, uint32_t prow, uint32_t r, float c0) {
  s64_wr(x_a + r * 4u, diff);
  f32x2v y01 = {0.0f, 0.0f}, y23 = {0.0f, 0.0f};
  static_for<64 / kS64PB>([&](auto B) {
    constexpr int b = B;
    constexpr int NQ = kS64PB / 4;
    f32x4 pv[NQ], dv[NQ];
    if constexpr (NQ == 2 && AMH_S64_LDSW) {
      lds_ld4x4w<16 * (2 * b), 16 * (2 * b + 1), 16 * (2 * b), 16 * (2 * b + 1)>(pv[0], pv[1], dv[0], dv[1], prow, x_a);
    } else {
      static_for<NQ>([&](auto Q) {
        pv[(int)Q] = lds_ld4<16 * (NQ * b + Q)>(prow);
        dv[(int)Q] = lds_ld4<16 * (NQ * b + Q)>(x_a);
      });
      if constexpr (NQ == 4) {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pv[0]), "+v"(pv[1]), "+v"(pv[2]), "+v"(pv[3]), "+v"(dv[0]),
                     "+v"(dv[1]), "+v"(dv[2]), "+v"(dv[3]));
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pv[0]), "+v"(pv[1]), "+v"(dv[0]), "+v"(dv[1]));
      }
    }
    static_for<2 * NQ>([&](auto K2) {
      const f32x4 q = pv[(int)K2 / 2];
      const f32x4 dq = dv[(int)K2 / 2];
      const f32x2v pp = (K2 % 2 == 0) ? f32x2v{q[0], q[1]} : f32x2v{q[2], q[3]};
      const f32x2v bp = (K2 % 2 == 0) ? f32x2v{dq[0], dq[1]} : f32x2v{dq[2], dq[3]};
      if constexpr (K2 % 2 == 0) {
        y01 = __builtin_elementwise_fma(pp, bp, y01);
      } else {
        y23 = __builtin_elementwise_fma(pp, bp, y23);
      }
    });
    __builtin_amdgcn_sched_barrier(0);
  });
  const float y = (y01[0] + y01[1]) + (y23[0] + y23[1]);
  const float S = Grp<64>::sum(diff * y);
  return (0.5f * S) + c0;
}

// asss_transition<64, GaussianM, true> (amh_asss.h; asss.py:197-251) for the
// d = 64 persistent kernel: the same float operations in the same order (so
// the same bits as the generic transition and orc_asss_step), with the
// column broadcasts of the step64 ARWMH path -- the matrix-vector products
// S z, S v and every potential read their broadcast vector from the wave's
// LDS scratch, sweep 1 is s64_sweep1, sweep 2 the quarter-vector LDS scheme,
// and the forward solve keeps one v_readlane per column (its own y_j by a
// select).  The generic form spent ~576 + 64 (shrink steps + 2) v_readlane per
// transition.
__device__ __forceinline__ void asss_transition64(const StepParams& p, float (&U)[64], float& dl, float& x, float& mu,
                                                  float& pe, float& asc, bool& updated, int32_t it, uint32_t k0,
                                                  uint32_t k1, int r, const GaussianM<64>::Ctx& mctx, uint32_t x_a,
                                                  uint32_t xq_a, uint32_t prow) {
  using Gp = Grp<64>;
  constexpr int d = 64;
  const float sd = sqrtf((float)d);
  const float epsd = p.eps * sd;
  const float fd = (float)d;
  const uint32_t ur = (uint32_t)r;
  // ---- draws (asss.py:207, 219, 225, 60)
  const amh_u32x4 o = amh_philox4x32_10((uint32_t)r, (uint32_t)it, 0u, AMH_TAG_ASSS, k0, k1);
  float v = amh_normal_from_bits(o.v[0]);
  float vd = amh_normal_from_bits(Gp::template bcast_u<0>(o.v[1]));
  const float ut = amh_unif01_from_bits(Gp::template bcast_u<0>(o.v[2]));
  const float th0 = 6.28318548f * amh_unif01_from_bits(Gp::template bcast_u<0>(o.v[3]));

  // ---- y = S^-1 (x - mu)
  const float e = dl * sd;
  const float Dr = (dl + p.eps) * sd;
  const float invD = 1.0f / Dr;
  float b = x - mu;
  float y = 0.0f;
  static_for<d>([&](auto J) {
    constexpr int j = J;
    const float yl = b * invD;
    y = s64_keep_at<j>(y, yl);
    const float gj = Gp::template bcast<j>(yl * e);
    b = fmaf(-U[j], gj, b);
    column_fence<j>();
  });

  // ---- stereographic projection (asss.py:40-45)
  const float ns = Gp::sum(y * y);
  const float den = ns + 1.0f;
  const float zr = (2.0f * y) / den;
  const float zd = (ns - 1.0f) / den;

  // ---- v orthogonal to z on S^d (asss.py:219-222), as amh_asss.h
  const float dot = Gp::sum(v * zr) + (vd * zd);
  v = fmaf(-dot, zr, v);
  vd = fmaf(-dot, zd, vd);
  const float nv = sqrtf(Gp::sum(v * v) + (vd * vd));
  const bool degen = !(nv > 0.0f);
  v = degen ? 0.0f : v / nv;
  vd = degen ? 0.0f : vd / nv;

  // ---- S z_1d and S v_1d: U times the broadcast vectors hz, hv from the scratch
  auto svec = [&](float h) -> float {
    s64_wr(x_a + ur * 4u, h);
    float a4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    static_for<d / kS64EB>([&](auto B) {
      constexpr int bb = B;
      f32x4 ev[kS64EB / 4];
      if constexpr (kS64EB == 8 && AMH_S64_LDSW) {
        lds_ld4x2w<16 * (2 * bb), 16 * (2 * bb + 1)>(ev[0], ev[1], x_a);
      } else {
        static_for<kS64EB / 4>([&](auto Q) { ev[(int)Q] = lds_ld4<16 * (kS64EB / 4 * bb + Q)>(x_a); });
        if constexpr (kS64EB == 16) {
          lds_wait(ev[0], ev[1], ev[2], ev[3]);
        } else {
          s64_tie(ev[0], ev[1]);
        }
      }
      static_for<kS64EB>([&](auto K) {
        constexpr int j = kS64EB * bb + K;
        a4[j & 3] = fmaf(U[j], ev[(int)K / 4][(int)K % 4], a4[j & 3]);
      });
      __builtin_amdgcn_sched_barrier(0);
    });
    s64_wait();  // every lane's reads are done before the scratch is written again
    return (a4[0] + a4[1]) + (a4[2] + a4[3]);
  };
  const float Sz = svec(e * zr) + epsd * zr;
  const float Sv = svec(e * v) + epsd * v;

  auto x_at = [&](float c, float s, float& om) -> float {
    const float zdt = (zd * c) + (vd * s);
    om = 1.0f - zdt;
    return (((Sz * c) + (Sv * s)) / om) + mu;
  };
  auto pot = [&](float xv) -> float {
    const float u = s64_gauss_pot(xv - mctx.mr, x_a, prow, ur, mctx.c0);
    s64_wait();
    return u;
  };

  // ---- slice level at z (asss.py:216-217, 224-226)
  float om0;
  const float x0 = x_at(1.0f, 0.0f, om0);
  const float U0 = pot(x0);
  const float tpe = (U0 + fd * amh_logf(om0)) - amh_logf(ut);

  // ---- shrinkage (asss.py:59-96)
  float th = th0, thmin = th0 - 6.28318548f, thmax = th0;
  int32_t iter = 0;
  float xt, ux;
  bool cont;
  {
    float s, c, om;
    amh_sincosf(th, &s, &c);
    xt = x_at(c, s, om);
    ux = pot(xt);
    float pt = ux + fd * amh_logf(om);
    if (amh_isnan(pt)) pt = INFINITY;
    cont = !degen && ((pt > tpe) || (om < p.eps));
  }
  while (cont) {  // wave-uniform: one chain per wave
    const float thmin_n = (th < 0.0f) ? th : thmin;
    const float thmax_n = (th >= 0.0f) ? th : thmax;
    const amh_u32x4 ok = amh_philox4x32_10((uint32_t)iter, (uint32_t)it, 1u, AMH_TAG_ASSS, k0, k1);
    const float th_n = thmin_n + (thmax_n - thmin_n) * amh_unif01_from_bits(ok.v[0]);
    float s, c, om;
    amh_sincosf(th_n, &s, &c);
    const float xn = x_at(c, s, om);
    const float un = pot(xn);
    float pt = un + fd * amh_logf(om);
    if (amh_isnan(pt)) pt = INFINITY;
    thmin = thmin_n;
    thmax = thmax_n;
    th = th_n;
    xt = xn;
    ux = un;
    iter += 1;
    cont = (iter < kAsssMaxIter) && ((pt > tpe) || (om < p.eps));
  }
  const bool capped = degen || iter >= kAsssMaxIter;  // asss.py:94: theta = 0
  const float xnew = capped ? x0 : xt;
  float pen = capped ? U0 : ux;
  if (amh_isnan(pen)) pen = INFINITY;  // asss.py:234

  // ---- adaptation (asss.py:237-251)
  const int32_t itr = it + 1;
  const int32_t n = (it < p.W) ? itr : itr - p.W;
  const float gamma = lookup_gamma<64>(p, n);
  const float delta = xnew - mu;
  const float mun = mu + gamma * delta;
  const float dmu = mun - mu;
  const float locd = sqrtf(Gp::sum(dmu * dmu));

  const float sq = sqrtf(1.0f - gamma);
  const float ajj = sq * dl;
  const float Dg = ajj * ajj;
  const float one = (amh_isfinite(ajj) && ajj != 0.0f) ? 1.0f : __int_as_float(0x7FC00000);
  float ws = delta;  // sweep 1: lane r ends with w*_r (s64_sweep1_all)
  s64_sweep1_all(ws, U);
  const float gw2 = gamma * (ws * ws);
  const float tsc = gw2 / Dg;
  const float bb = 1.0f + Gp::excl_scan(tsc, r);
  const float g2 = (bb * Dg) + gw2;
  const float dn = g2 / bb;
  const float cc = (gamma * ws) / g2;
  const float q = sqrtf(dn);
  const float dnew = fmaf(cc, 0.0f, one) * q;
  const bool revert = Gp::any(amh_isnan(dnew));
  float sdiff = 0.0f;
  if (!revert) {
    const float ac = q - dl;
    const float bc = cc * q;
    float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    float w = delta;
    static_for<16>([&](auto G4) {
      constexpr int g = G4;
      if constexpr (g % 4 == 0) s64_wr4_quarter<g / 4>(xq_a, ws, cc, ac, bc);
      constexpr int gq = g % 4;
      f32x4 cw, cv, ca, cb;
#if AMH_S64_LDSW
      lds_ld4x4w<16 * gq, 64 + 16 * gq, 128 + 16 * gq, 192 + 16 * gq>(cw, cv, ca, cb, x_a, x_a);
#else
      cw = lds_ld4<16 * gq>(x_a), cv = lds_ld4<64 + 16 * gq>(x_a);
      ca = lds_ld4<128 + 16 * gq>(x_a), cb = lds_ld4<192 + 16 * gq>(x_a);
      lds_wait(cw, cv, ca, cb);
#endif
      static_for<4>([&](auto Q) {
        constexpr int j = 4 * g + Q;
        const float uo = U[j];
        w = fmaf(-cw[(int)Q], uo, w);
        const float un = fmaf(cv[(int)Q], w, uo);
        const float tt = fmaf(uo, ca[(int)Q], cb[(int)Q] * w);
        s4[j & 3] = fmaf(tt, tt, s4[j & 3]);
        U[j] = un;
      });
      column_fence<g, 2>();
    });
    const float sacc = (s4[0] + s4[1]) + (s4[2] + s4[3]);
    sdiff = sqrtf(Gp::sum(sacc));
    dl = q;
    updated = true;
  }
  asc = locd + sdiff;  // asss.py:248-250
  x = xnew;
  pe = pen;
  mu = mun;
}

// kASSS: the same persistent data movement around one ASSS transition
// (asss_transition, amh_asss.h; asss.py:197-251) instead of the ARWMH one --
// the state is the same but for mean_accept_prob / log_step_size (absent).
template <int WPB, bool kASSS = false>
__global__ __launch_bounds__(WPB * 64) void arwmh_step64_kernel(StepParams p) {
  constexpr int D = 64;
  constexpr uint32_t P = kS64P;
  using Gp = Grp<64>;
  using M = GaussianM<64>;
  extern __shared__ float lds[];
  M::stage(lds, p.model, D);
  float* tick = lds + kS64Model + WPB * kS64WB;
  if (threadIdx.x == 0) tick[0] = 0.0f;
  __syncthreads();
  const auto mctx = M::prepare(p.model, D, lane_id());
#ifdef AMH_STAMPS
  // diagnostic build: per-wave start / end on the constant 100 MHz clock and
  // the items taken (tools/s64_tail.py: how long the launch drains)
  const unsigned long long st_start = __builtin_amdgcn_s_memrealtime();
  int st_items = 0;
#endif

  const int64_t C = p.C;
  const int64_t n_items = C;  // one chain per wave
  const int wave_in_block = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  float* wb = lds + kS64Model + wave_in_block * kS64WB;
  const uint32_t wb_a = lds_addr(wb);
  const uint32_t x_a = wb_a + kS64X * 4;            // scratch (64 floats: broadcast vectors)
  const uint32_t zm_a = wb_a + kS64Z * 4;           // z / loc region (swap vectors once read)
  const uint32_t xq_a = x_a + (uint32_t)(lane_id() & 15) * 4u;  // sweep-2 quarter slot
  const uint32_t prow = lds_addr(lds) + (uint32_t)lane_id() * (uint32_t)(M::ld(D) * 4);  // row r of P

  float U[D];  // row r of U = L / diag(L): unit diagonal, zeros above (kept between chains)
  static_for<D>([&](auto J) { U[J] = set_one_at<64, J>(0.0f, lane_id()); });
  float dl = 0.0f, z = 0.0f, mu = 0.0f, pe = 0.0f, macc = 0.0f, lam = 0.0f, asc = 0.0f;
  int32_t it = 0, nacc = 0, acc0 = 0;
  uint32_t k0 = 0, k1 = 0;
  int64_t prev = -1;
  bool prev_upd = false;

  const int64_t blk_lo = n_items * (int64_t)blockIdx.x / gridDim.x;
  const int64_t blk_hi = n_items * ((int64_t)blockIdx.x + 1) / gridDim.x;
  const int64_t kEnd = blk_hi;  // "no item" sentinel
  const uint32_t tk_addr = lds_addr(tick);
  auto ticket = [&]() -> int64_t {
    uint32_t v = 0;
    if (lane_id() == 0) {
      asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(tk_addr), "v"(1u) : "memory");
    }
    return blk_lo + (int64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)v);
  };

  // z, loc and the scalars of chain `c` from registers
  auto store_small = [&](int64_t c, int r) {
    p.out.z[c * D + r] = z;
    p.out.loc[c * D + r] = mu;
    if (r == 0) {
      p.out.i[c] = it;
      p.out.potential_energy[c] = pe;
      if constexpr (!kASSS) {
        p.out.mean_accept_prob[c] = macc;
        p.out.log_step_size[c] = lam;
      }
      p.out.as_change[c] = asc;
      p.out.rng_key[2 * c] = k0;
      p.out.rng_key[2 * c + 1] = k1;
      if (!kASSS && p.accept_count != nullptr) p.accept_count[c] = acc0 + nacc;
    }
  };
  // factor of chain `c` copied verbatim from the launch input (no step of this
  // launch updated it); U is used as scratch and reset to the unit pattern
  auto copy_verbatim = [&](int64_t c, int r) {
    const uint32_t vrow = (uint32_t)r * 4u;
    const Buf Lout(uniform_ptr(p.out.scale + c * P), P * 4u);
    const Buf Lin(uniform_ptr(p.in.scale + c * P), P * 4u);
    static_for<4>([&](auto B) {
      static_for<16>([&](auto K) {
        constexpr int j = 16 * B + K;
        U[j] = Lin.ld(off_from<64, j>(vrow, kOOB, r), (uint32_t)(s64_col(j) - j) * 4u);
      });
      static_for<16>([&](auto K) {
        constexpr int j = 16 * B + K;
        Lout.st(U[j], off_from<64, j>(vrow, kOOB, r), (uint32_t)(s64_col(j) - j) * 4u);
      });
      __builtin_amdgcn_sched_barrier(0);
    });
    __builtin_amdgcn_s_waitcnt(0);  // loads landed and store data read before U is reused
    static_for<D>([&](auto J) { U[J] = set_one_at<64, J>(0.0f, r); });
  };
  // the wave buffer's factor region (packed, column-major) -> chain `c` in HBM
  auto flush_factor = [&](int64_t c) {
    const Buf Lout(uniform_ptr(p.out.scale + c * P), P * 4u);
    const uint32_t la = wb_a + (uint32_t)lane_id() * 16u;
    static_for<3>([&](auto G) {  // three dwordx4 per lane in flight per wait
      f32x4 v[3];
      static_for<3>([&](auto Q) { v[(int)Q] = lds_ld4<1024 * (3 * G + Q)>(la); });
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]));
      static_for<3>([&](auto Q) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(uint32x4_t_, v[(int)Q]), Lout.rs,
                                               (int)(1024u * (3 * G + Q) + 16u * (uint32_t)lane_id()), 0,
                                               AMH_STORE_AUX);
      });
    });
  };

  int64_t item = ticket();
  int64_t nxt = item < kEnd ? ticket() : kEnd;
  if (item < kEnd) prefetch_item<64, false>(p, item, D, wb, lane_id());
  for (; item < kEnd;) {
    int lane = lane_id();
    asm volatile("" : "+v"(lane));
    const int r = lane;
    const uint32_t la = wb_a + (uint32_t)r * 4u;  // this lane's dword in the factor region

    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): item k has landed
    // the hand-over phase (stores, LDS -> registers, the next DMA) at high
    // wave priority so the memory queue is re-armed before other waves'
    // compute: 239 -> 236 us per launch (tools/gpu_prio.sh A/B)
    __builtin_amdgcn_s_setprio(3);
    // ---- item k-1's z / loc / scalars leave from registers
    if (prev >= 0) store_small(prev, r);
    const bool wr = prev >= 0 && prev_upd;
    if (prev >= 0 && !prev_upd) copy_verbatim(prev, r);

    // ---- diagonal of item k
    float lnew = lds_ld1<0>(wb_a + (uint32_t)s64_col(r) * 4u);
    s64_tie(lnew);
    const float inv = (amh_isfinite(lnew) && lnew != 0.0f) ? 1.0f / lnew : 0.0f;
    // ---- item k's z / loc / scalars: LDS -> registers
    {
      float zz = lds_ld1<kS64Z * 4>(la), mm = lds_ld1<kS64M * 4>(la);
      const uint32_t sa = wb_a + kS64S * 4;
      float s0 = lds_ld1<0>(sa), s1 = lds_ld1<4>(sa), s2 = lds_ld1<8>(sa), s3 = lds_ld1<12>(sa);
      float s4v = lds_ld1<16>(sa), s5 = lds_ld1<20>(sa), s6 = lds_ld1<24>(sa);
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(zz), "+v"(mm), "+v"(s0), "+v"(s1), "+v"(s2), "+v"(s3), "+v"(s4v),
                   "+v"(s5), "+v"(s6));
      z = zz;
      mu = mm;
      it = __builtin_amdgcn_readfirstlane(__float_as_int(s0));
      pe = s1;
      macc = s2;
      lam = s3;
      asc = s4v;
      k0 = (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(s5));
      k1 = (uint32_t)__builtin_amdgcn_readfirstlane(__float_as_int(s6));
      // broadcast vectors [dl of k-1 | 1 / l of k] over item k's z / loc, now in registers
      s64_wr(zm_a + (uint32_t)r * 4u, dl);
      s64_wr_off<256>(zm_a + (uint32_t)r * 4u, inv);
      dl = lnew;
      acc0 = (!kASSS && p.accept_count != nullptr && r == 0) ? p.accept_count[item] : 0;
    }

    // ---- swap: read item k's column j (lanes > j), write item k-1's column j
    //      of L' = U diag(dl) (lanes >= j) at the same addresses, normalise
    static_for<16>([&](auto G4) {
      constexpr int g = G4;
      f32x4 dl4 = lds_ld4<16 * g>(zm_a);
      f32x4 in4 = lds_ld4<256 + 16 * g>(zm_a);
      s64_tie(dl4, in4);
      float t[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      static_for<4>([&](auto Q) {
        constexpr int j = 4 * g + Q;
        constexpr int off = (s64_col(j) - j) * 4;
        if constexpr (j < D - 1) s64_rd_above<j, off>(t[(int)Q], la);
        if (wr) s64_wr_from<j, off>(la, U[j] * dl4[(int)Q]);
      });
      asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(t[0]), "+v"(t[1]), "+v"(t[2]), "+v"(t[3]));
      static_for<4>([&](auto Q) {
        constexpr int j = 4 * g + Q;
        if constexpr (j < D - 1) s64_mul_above<j>(U[j], t[(int)Q], in4[(int)Q]);
      });
    });
    if (wr) flush_factor(prev);

    s64_wait();  // every LDS read of the buffer is done before the DMA refills it
    int64_t nxt2 = kEnd;
    if (nxt < kEnd) {
      prefetch_item<64, false>(p, nxt, D, wb, lane);
      nxt2 = ticket();
    }
    __builtin_amdgcn_s_setprio(0);

    nacc = 0;
    bool updated = false;
    for (int32_t t = 0; t < p.n_steps; ++t) {
     if constexpr (kASSS) {
#if AMH_S64_ASSS_GENERIC
      asss_transition<64, GaussianM, true>(p, U, dl, z, mu, pe, asc, updated, it, k0, k1, D, r, r, true, mctx, lds);
#else
      asss_transition64(p, U, dl, z, mu, pe, asc, updated, it, k0, k1, r, mctx, x_a, xq_a, prow);
#endif
      it += 1;
     } else {
      // ---- noise (arwmh.py:162-165, 174): stream position = state.i
      float xi, u;
      step_noise_w64(r, (uint32_t)it, k0, k1, xi, u);  // bit spec: amh_step_word

      // ---- proposal z' = z + (L e^lam + eps I) xi  (arwmh.py:166-167), L xi = U (dl * xi)
      const float el = amh_expf(lam);
      const float eta = dl * xi;
      s64_wr(x_a + (uint32_t)r * 4u, eta);
      float a4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      static_for<D / kS64EB>([&](auto B) {  // kS64EB columns per batch
        constexpr int b = B;
        f32x4 e[kS64EB / 4];
        if constexpr (kS64EB == 8 && AMH_S64_LDSW) {
          lds_ld4x2w<16 * (2 * b), 16 * (2 * b + 1)>(e[0], e[1], x_a);
        } else {
          static_for<kS64EB / 4>([&](auto Q) { e[(int)Q] = lds_ld4<16 * (kS64EB / 4 * b + Q)>(x_a); });
          if constexpr (kS64EB == 16) {
            lds_wait(e[0], e[1], e[2], e[3]);
          } else {
            s64_tie(e[0], e[1]);
          }
        }
        static_for<kS64EB>([&](auto K) {
          constexpr int j = kS64EB * b + K;
          a4[j & 3] = fmaf(U[j], e[(int)K / 4][(int)K % 4], a4[j & 3]);
        });
        __builtin_amdgcn_sched_barrier(0);
      });
      const float acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
      const float zp = z + fmaf(el, acc, p.eps * xi);

      // ---- potential (GaussianM<64>::potential with diff_j from the scratch), NaN -> +inf
      float pep;
      {
        const float diff = zp - mctx.mr;
        s64_wr(x_a + (uint32_t)r * 4u, diff);
        f32x2v y01 = {0.0f, 0.0f}, y23 = {0.0f, 0.0f};
        static_for<D / kS64PB>([&](auto B) {
          constexpr int b = B;
          constexpr int NQ = kS64PB / 4;
          f32x4 pv[NQ], dv[NQ];
          if constexpr (NQ == 2 && AMH_S64_LDSW) {
            lds_ld4x4w<16 * (2 * b), 16 * (2 * b + 1), 16 * (2 * b), 16 * (2 * b + 1)>(pv[0], pv[1], dv[0], dv[1], prow, x_a);
          } else {
            static_for<NQ>([&](auto Q) {
              pv[(int)Q] = lds_ld4<16 * (NQ * b + Q)>(prow);
              dv[(int)Q] = lds_ld4<16 * (NQ * b + Q)>(x_a);
            });
            if constexpr (NQ == 4) {
              asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pv[0]), "+v"(pv[1]), "+v"(pv[2]), "+v"(pv[3]), "+v"(dv[0]),
                           "+v"(dv[1]), "+v"(dv[2]), "+v"(dv[3]));
            } else {
              asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(pv[0]), "+v"(pv[1]), "+v"(dv[0]), "+v"(dv[1]));
            }
          }
          static_for<2 * NQ>([&](auto K2) {
            const f32x4 q = pv[(int)K2 / 2];
            const f32x4 dq = dv[(int)K2 / 2];
            const f32x2v pp = (K2 % 2 == 0) ? f32x2v{q[0], q[1]} : f32x2v{q[2], q[3]};
            const f32x2v bp = (K2 % 2 == 0) ? f32x2v{dq[0], dq[1]} : f32x2v{dq[2], dq[3]};
            if constexpr (K2 % 2 == 0) {
              y01 = __builtin_elementwise_fma(pp, bp, y01);
            } else {
              y23 = __builtin_elementwise_fma(pp, bp, y23);
            }
          });
          __builtin_amdgcn_sched_barrier(0);
        });
        const float y = (y01[0] + y01[1]) + (y23[0] + y23[1]);
        const float S = Gp::sum(diff * y);
        pep = (0.5f * S) + mctx.c0;
      }
      if (amh_isnan(pep)) pep = INFINITY;

      // ---- accept / reject (arwmh.py:173-178)
      const float ex = amh_expf(pe - pep);
      const float alpha = (ex > 1.0f) ? 1.0f : ex;
      const bool accept = u < alpha;
      const float zn = accept ? zp : z;
      const float pen = accept ? pep : pe;
      nacc += accept ? 1 : 0;

      // ---- schedule (arwmh.py:180-185)
      const int32_t itr = it + 1;
      const int32_t n = (it < p.W) ? itr : itr - p.W;
      const float gamma = lookup_gamma<64>(p, n);
      const float maccn = macc + (alpha - macc) / (float)n;

      // ---- mean and step size (arwmh.py:188-189, 193)
      const float delta = zn - mu;
      const float mun = mu + gamma * delta;
      const float lamn = lam + gamma * (alpha - p.target);
      const float e1 = amh_expf(lamn);

      // ---- rank-one update of sqrt(1-gamma) L by (delta, gamma), NaN -> keep L
      const float sq = sqrtf(1.0f - gamma);
      const float ajj = sq * dl;
      const float Dg = ajj * ajj;
      const float one = (amh_isfinite(ajj) && ajj != 0.0f) ? 1.0f : __int_as_float(0x7FC00000);

      // sweep 1 (lanes r > j): afterwards lane r holds w*_r (forward solve U w* = delta)
      float ws = delta;
      s64_sweep1_all(ws, U);

      const float gw2 = gamma * (ws * ws);
      const float tsc = gw2 / Dg;
      const float b = 1.0f + Gp::excl_scan(tsc, r);
      const float g2 = (b * Dg) + gw2;
      const float dn = g2 / b;
      const float c = (gamma * ws) / g2;
      const float q = sqrtf(dn);
      const float dnew = fmaf(c, 0.0f, one) * q;
      const bool revert = Gp::any(amh_isnan(dnew));
      float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      if (!revert) {
        // sweep 2: U'_rj = U_rj + c_j w_r^{(j+1)}; as_change terms
        //   U_rj (q_j e1 - dl_j e0) + (c_j q_j e1) w_r^{(j+1)}
        const float ac = (q * e1) - (dl * el);
        const float bc = (c * q) * e1;
        float w = delta;
        static_for<16>([&](auto G4) {
          constexpr int g = G4;
          // the four coefficient vectors of columns 16(g/4) .. +15 (lanes of that quarter write)
          if constexpr (g % 4 == 0) s64_wr4_quarter<g / 4>(xq_a, ws, c, ac, bc);
          constexpr int gq = g % 4;
          f32x4 cw, cc, ca, cb;
#if AMH_S64_LDSW
          lds_ld4x4w<16 * gq, 64 + 16 * gq, 128 + 16 * gq, 192 + 16 * gq>(cw, cc, ca, cb, x_a, x_a);
#else
          cw = lds_ld4<16 * gq>(x_a), cc = lds_ld4<64 + 16 * gq>(x_a);
          ca = lds_ld4<128 + 16 * gq>(x_a), cb = lds_ld4<192 + 16 * gq>(x_a);
          lds_wait(cw, cc, ca, cb);
#endif
          static_for<4>([&](auto Q) {
            constexpr int j = 4 * g + Q;
            const float uo = U[j];
            w = fmaf(-cw[(int)Q], uo, w);
            const float un = fmaf(cc[(int)Q], w, uo);
            const float tt = fmaf(uo, ca[(int)Q], cb[(int)Q] * w);
            s4[j & 3] = fmaf(tt, tt, s4[j & 3]);
            U[j] = un;
          });
          column_fence<g, 2>();
        });
        const float sacc = (s4[0] + s4[1]) + (s4[2] + s4[3]);
        asc = sqrtf(Gp::sum(sacc));
        dl = q;
        updated = true;
      } else {
        // factor unchanged: as_change = || L (e1 - e0) ||_F, L_rj = U_rj dl_j
        const float ac = (dl * e1) - (dl * el);
        static_for<D>([&](auto J) {
          const float tt = U[J] * Gp::template bcast<J>(ac);
          s4[J & 3] = fmaf(tt, tt, s4[J & 3]);
          column_fence<J>();
        });
        const float sacc = (s4[0] + s4[1]) + (s4[2] + s4[3]);
        asc = sqrtf(Gp::sum(sacc));
      }

      // ---- commit (arwmh.py:199-207)
      it = itr;
      z = zn;
      pe = pen;
      macc = maccn;
      mu = mun;
      lam = lamn;
     }
      if (p.col_z != nullptr || p.col_pe != nullptr) {
        if ((t + 1) % p.thinning == 0) {
          const int64_t kk = t / p.thinning;
          if (p.col_z != nullptr) p.col_z[(kk * C + item) * D + r] = z;
          if (p.col_pe != nullptr && r == 0) p.col_pe[kk * C + item] = pe;
        }
      }
    }
    prev = item;
    prev_upd = Gp::any(updated);
    item = nxt;
    nxt = nxt2;
#ifdef AMH_STAMPS
    ++st_items;
#endif
  }
  if (prev >= 0) {
    int lane = lane_id();
    asm volatile("" : "+v"(lane));
    const uint32_t la = wb_a + (uint32_t)lane * 4u;
    store_small(prev, lane);
    if (prev_upd) {
      s64_wr(x_a + (uint32_t)lane * 4u, dl);
      static_for<16>([&](auto G4) {
        constexpr int g = G4;
        f32x4 dl4 = lds_ld4<16 * g>(x_a);
        s64_tie(dl4);
        static_for<4>([&](auto Q) {
          constexpr int j = 4 * g + Q;
          s64_wr_from<j, (s64_col(j) - j) * 4>(la, U[j] * dl4[(int)Q]);
        });
      });
      flush_factor(prev);
    } else {
      copy_verbatim(prev, lane);
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
#ifdef AMH_STAMPS
  {
    const unsigned long long st_end = __builtin_amdgcn_s_memrealtime();
    const int64_t w = (int64_t)blockIdx.x * WPB + wave_in_block;
    if (w < kStampWaves && lane_id() == 0) {
      g_stamps[w * kStampSlots + 0] = st_start;
      g_stamps[w * kStampSlots + 1] = st_end;
      g_stamps[w * kStampSlots + 2] = (unsigned long long)st_items;
      g_stamps[w * kStampSlots + 3] = (unsigned long long)blockIdx.x;
      g_stamps[w * kStampSlots + 7] = 1;
    }
  }
#endif
}

template <int WPB, bool kASSS = false>
hipError_t launch_step64(const StepParams& p, hipStream_t s) {
  constexpr size_t shm = s64_lds_bytes<WPB>();
  static_assert(shm <= 163840, "d = 64 step kernel: LDS budget");
  auto kern = arwmh_step64_kernel<WPB, kASSS>;
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, WPB * 64, shm);
  if (e != hipSuccess) return e;
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (per_cu < 1) per_cu = 1;
  const int64_t need = (p.C + WPB - 1) / WPB;
  int64_t blocks = (int64_t)cus * per_cu;
  if (blocks > need) blocks = need;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(WPB * 64), shm, s, p);
  return hipGetLastError();
}

// ------------------------------------------------------------- launchers ----
static int grid_for(int64_t n_items, int waves_per_block) {
  // enough waves to cover 256 CUs x 8 waves/CU several times; grid-stride past it
  const int64_t blocks = (n_items + waves_per_block - 1) / waves_per_block;
  const int64_t cap = 256 * 32;
  return (int)(blocks < cap ? (blocks > 0 ? blocks : 1) : cap);
}

template <int DMAX, template <int> class M, bool EXACT, int DFIX = 0>
hipError_t launch_step(const StepParams& p, hipStream_t s) {
  constexpr int CPW = Geo<DMAX>::CPW;
  constexpr int WPB = kBlockStep / 64;
  const int d = EXACT ? DMAX : p.d;
  const int64_t n_items = (p.C + CPW - 1) / CPW;
  const size_t shm = step_lds_bytes<DMAX, M>(p.model, d);
  if (shm > 163840) return hipErrorInvalidConfiguration;
  auto kern = arwmh_step_kernel<DMAX, M, EXACT, DFIX>;
  // persistent grid: as many blocks as are co-resident (each wave then walks
  // chain groups wave, wave + total_waves, ...)
  int per_cu = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kBlockStep, shm);
  if (e != hipSuccess) return e;
  int dev = 0, cus = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (per_cu < 1) per_cu = 1;
  const int64_t need = (n_items + WPB - 1) / WPB;
  int64_t blocks = (int64_t)cus * per_cu;
  if (blocks > need) blocks = need;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kBlockStep), shm, s, p);
  return hipGetLastError();
}

template <int DMAX, template <int> class M, bool EXACT>
hipError_t launch_init(const InitParams& p, hipStream_t s) {
  const int64_t n_items = (p.C + Geo<DMAX>::CPW - 1) / Geo<DMAX>::CPW;
  const size_t shm = M<DMAX>::lds_bytes(p.model, EXACT ? DMAX : p.d);
  hipLaunchKernelGGL((arwmh_init_kernel<DMAX, M, EXACT>), dim3(grid_for(n_items, kBlock / 64)), dim3(kBlock),
                     shm, s, p);
  return hipGetLastError();
}

template <int DMAX, template <int> class M, bool EXACT>
hipError_t launch_pot(const PotParams& p, hipStream_t s) {
  const int64_t n_items = (p.n + Geo<DMAX>::CPW - 1) / Geo<DMAX>::CPW;
  const size_t shm = M<DMAX>::lds_bytes(p.model, EXACT ? DMAX : p.d);
  hipLaunchKernelGGL((potential_kernel<DMAX, M, EXACT>), dim3(grid_for(n_items, kBlock / 64)), dim3(kBlock),
                     shm, s, p);
  return hipGetLastError();
}

// sample_pnx_kernel's step t split around the caller's potential
// (AMH_MODEL_EXTERNAL): ACCEPT = false forms every chain's proposal from the
// shared factor (the same fmaf chain over j as sample_pnx_kernel), ACCEPT =
// true takes U(z') from memory and applies the test with the step's u
template <int G, bool ACCEPT>
__global__ __launch_bounds__(kBlock) void pnx_ext_kernel(PnxExtParams p) {
  using Gp = Grp<G>;
  const int d = p.d;
  const int r = Gp::r();
  const bool act = r < d;
  const int64_t C = p.C;
  const int64_t n_items = (C + Geo<G>::CPW - 1) / Geo<G>::CPW;
  const int64_t wave0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t wstride = (int64_t)gridDim.x * (kBlock / 64);
  float A[G];
  if constexpr (!ACCEPT) {
    static_for<G>([&](auto J) {
      constexpr int j = J;
      A[j] = (j < d && r >= j && act) ? p.scale[col_off(d, j) + (r - j)] : 0.0f;
    });
  }
  const float el = amh_expf(p.log_step_size);
  for (int64_t item = wave0; item < n_items; item += wstride) {
    const int64_t chain = item_chain<G>(item);
    const bool chain_ok = chain < C;
    const int64_t cl = chain_ok ? chain : C - 1;
    const amh_u32x4 kk = amh_philox4x32_10((uint32_t)cl, (uint32_t)((uint64_t)cl >> 32), 0u, AMH_TAG_SPLIT,
                                           p.key0, p.key1);
    const float z = act ? p.z[cl * d + r] : 0.0f;
    if constexpr (!ACCEPT) {
      float xi, u;
      step_noise<G>(r, d, (uint32_t)p.t, kk.v[0], kk.v[1], xi, u);
      xi = act ? xi : 0.0f;
      float acc = 0.0f;
      static_for<G>([&](auto J) {
        if (J < d) acc = fmaf(A[J], Gp::template bcast<J>(xi), acc);
      });
      const float zp = act ? z + fmaf(el, acc, p.eps * xi) : 0.0f;
      if (chain_ok && act) p.zprop[cl * d + r] = zp;
    } else {
      const float u = amh_unif01_from_bits(amh_step_word((uint32_t)d, (uint32_t)p.t, kk.v[0], kk.v[1]));  // W_d
      const float pe = p.pe[cl];
      float pep = p.pe_prop[cl];
      if (amh_isnan(pep)) pep = INFINITY;
      const float ex = amh_expf(pe - pep);
      const float alpha = (ex > 1.0f) ? 1.0f : ex;
      if (u < alpha && chain_ok) {  // group-uniform: one chain per group
        if (act) p.z[cl * d + r] = p.zprop[cl * d + r];
        if (r == 0) p.pe[cl] = pep;
      }
    }
  }
}

hipError_t run_pnx_ext(const PnxExtParams& p, bool accept, hipStream_t s) {
  if (p.d < 1 || p.d > 64 || p.C < 1) return hipErrorInvalidValue;
  auto go = [&](auto kern, int64_t cpw) {
    const int64_t n_items = (p.C + cpw - 1) / cpw;
    hipLaunchKernelGGL(kern, dim3(grid_for(n_items, kBlock / 64)), dim3(kBlock), 0, s, p);
    return hipGetLastError();
  };
  if (p.d <= 32) return accept ? go(pnx_ext_kernel<32, true>, Geo<32>::CPW) : go(pnx_ext_kernel<32, false>, Geo<32>::CPW);
  return accept ? go(pnx_ext_kernel<64, true>, Geo<64>::CPW) : go(pnx_ext_kernel<64, false>, Geo<64>::CPW);
}

template <int DMAX, template <int> class M, bool EXACT>
hipError_t launch_pnx(const PnxParams& p, hipStream_t s) {
  const int64_t n_items = (p.n_points * p.n_samples + Geo<DMAX>::CPW - 1) / Geo<DMAX>::CPW;
  const size_t shm = M<DMAX>::lds_bytes(p.model, EXACT ? DMAX : p.d);
  hipLaunchKernelGGL((sample_pnx_kernel<DMAX, M, EXACT>), dim3(grid_for(n_items, kBlock / 64)), dim3(kBlock),
                     shm, s, p);
  return hipGetLastError();
}

struct StepF {
  const StepParams& p;
  hipStream_t s;
  template <int D, template <int> class M, bool E>
  hipError_t operator()() { return launch_step<D, M, E>(p, s); }
};
struct InitF {
  const InitParams& p;
  hipStream_t s;
  template <int D, template <int> class M, bool E>
  hipError_t operator()() { return launch_init<D, M, E>(p, s); }
};
struct PotF {
  const PotParams& p;
  hipStream_t s;
  template <int D, template <int> class M, bool E>
  hipError_t operator()() { return launch_pot<D, M, E>(p, s); }
};
struct PnxF {
  const PnxParams& p;
  hipStream_t s;
  template <int D, template <int> class M, bool E>
  hipError_t operator()() { return launch_pnx<D, M, E>(p, s); }
};

// A/B switches (the general kernel for d = 64; the data movement alone) exist
// only in the diagnostic build (-DAMH_DIAG, `make stamps`): the release
// library never reads the environment, so no setting can change its work.
static bool step64_enabled() {
#ifdef AMH_DIAG
  static const bool on = [] {
    const char* e = getenv("AMH_STEP64");
    return !(e != nullptr && e[0] == '0');
  }();
  return on;
#else
  return true;
#endif
}

hipError_t run_step(int model_id, const StepParams& p, hipStream_t s) {
  // the headline shape: d = 64 Gaussian, LDS-staged write-back
  if (model_id == AMH_MODEL_GAUSSIAN && p.d == 64 && p.ext_pe == nullptr && step64_enabled()) {
#ifdef AMH_DIAG
    static const bool move_only = [] {  // diagnostic: the data movement alone (tools/membound.py)
      const char* e = getenv("AMH_S64_MOVE_ONLY");
      return e != nullptr && e[0] == '1';
    }();
    if (move_only) {
      StepParams q = p;
      q.n_steps = 0;
      return launch_step64<kS64Waves>(q, s);
    }
#endif
    return launch_step64<kS64Waves>(p, s);
  }
  // diamonds at the reference shape: compile-time d (immediate offsets)
  if (model_id == AMH_MODEL_DIAMONDS_SS && p.d == kDiamondsD) return launch_step<32, DiamondsSSM, false, kDiamondsD>(p, s);
  return dispatch(model_id, p.d, StepF{p, s});
}
// ASSS at the d = 64 Gaussian (amh_asss.hip run_asss_step): the persistent
// LDS-staged kernel around the ASSS transition
#ifndef AMH_ASSS64_WAVES
// 16 waves (128 VGPRs, 64 B of spill) measured 0.343 ms per sample() against
// 0.363 ms at 12 waves (170 VGPRs, no spill): the occupancy pays for the spill
#define AMH_ASSS64_WAVES 16
#endif
hipError_t run_asss_step64(const StepParams& p, hipStream_t s) {
  return launch_step64<AMH_ASSS64_WAVES, true>(p, s);
}

hipError_t run_init(int model_id, const InitParams& p, hipStream_t s) {
  return dispatch(model_id, p.d, InitF{p, s});
}
hipError_t run_potential(int model_id, const PotParams& p, hipStream_t s) {
  return dispatch(model_id, p.d, PotF{p, s});
}
hipError_t run_pnx(int model_id, const PnxParams& p, hipStream_t s) {
  return dispatch(model_id, p.d, PnxF{p, s});
}
// split path (amh_split.hip): the step kernel with U(z') read from p.ext_pe,
// and init without the potential (filled by the batched potential kernel)
hipError_t run_step_ext(const StepParams& p, hipStream_t s) {
  if (p.d < 1 || p.d > 64 || p.n_steps != 1 || p.ext_pe == nullptr) return hipErrorInvalidValue;
  if (p.d == kDiamondsD) return launch_step<32, ExtPotM, false, kDiamondsD>(p, s);
  if (p.d > 32) return launch_step<64, ExtPotM, false>(p, s);  // the external potential's 33..64
  return launch_step<32, ExtPotM, false>(p, s);
}
hipError_t run_init_nopot(const InitParams& p, hipStream_t s) {
  if (p.d < 1 || p.d > 64) return hipErrorInvalidValue;
  if (p.d > 32) return launch_init<64, ExtPotM, false>(p, s);
  return launch_init<32, ExtPotM, false>(p, s);
}

hipError_t run_chain_keys(uint32_t k0, uint32_t k1, int64_t offset, int64_t n, uint32_t* out, hipStream_t s) {
  const int blocks = (int)((n + 255) / 256);
  hipLaunchKernelGGL(chain_keys_kernel, dim3(blocks > 0 ? blocks : 1), dim3(256), 0, s, k0, k1, offset, n, out);
  return hipGetLastError();
}

}  // namespace amh
