// amh_big_pooled.hip -- pooled-covariance mode (regime B) for the Gaussian
// with d % 32 == 0, 64 <= d <= 256: BASELINE config 4's headline (d = 256,
// one shared factor for 32,768 chains) and config 5's per-GPU work (d = 64,
// 65,536 chains).
//
// With one shared L every per-chain product is a GEMM over chains, so the
// three O(d^2) pieces run on MFMA (v_mfma_f32_32x32x2_f32, a k-ordered fmaf
// chain -- bit-reproducible by the oracle), fused into one persistent kernel
// per step:
//
//   pooled_fused64_kernel      d = 64: proposal Z' = Z + e^lam (L Xi) + eps Xi
//                              (arwmh.py:162-167), U(Z'), accept
//                              (arwmh.py:173-178) and the chunk sums S_d, S_a,
//                              S_dd = sum delta delta^T of a 64-chain chunk;
//                              L and P staged in LDS
//   pooled_pack_kernel +       d > 64: the same for 128-chain chunks, L and
//   pooled_fused_big_kernel    P read from L2 in MFMA A-operand order
//   pooled_reduce              chunk partials -> sums (amh_pooled.hip)
//   pooled_big_update_kernel   Sigma' = (1-g) Sigma + g S_dd / N (double) and
//                              its blocked Cholesky factor (float32, 32-column
//                              panels, the matrix resident in LDS)
// Bit spec: oracle/amh_oracle.c, "pooled mode, large dimensions".
#include "amh_device.h"

namespace amh {

// The d = 64 update's cross-block hand-off.  The reduce blocks' sums go out
// as agent-scope (write-through, sc1) stores and each block waits for them
// to complete (vmcnt(0)) before its arrival ticket, so the ticket itself is a
// relaxed RMW: an agent-scope release would add an L2 write-back
// (buffer_wbl2) of the whole XCD, whose L2 then holds the noise blocks'
// dirty rows -- measured 3.1 us from the last slice to the ticket, 0.7 us
// without (tools/u64_timeline.py, r4p).  The last arriver reads the sums with
// agent-scope (sc1) loads only; with sc1 stores drained before every add that
// is the guide's write-through hand-off, which needs no acquire fence (round
// 6: the buffer_inv removed, AMH_HANDOFF_FENCE=1 restores it).  Diagnostic
// variant -DAMH_TICKET_ACQREL: the acquire-release RMW instead.
#ifdef AMH_TICKET_ACQREL
#define AMH_TICKET_ORDER __ATOMIC_ACQ_REL
#else
#define AMH_TICKET_ORDER __ATOMIC_RELAXED
#endif
#ifndef AMH_HANDOFF_FENCE
#define AMH_HANDOFF_FENCE 0
#endif

// fused stats kernel, drawn-ahead noise rows loaded early (diagnostic
// variants; measured at C = 65,536, r4h): AMH_F64_PRE=1 loads sub-chunk 0's
// with its z in the prologue, =2 also the next sub-chunk's during the current
// one (phase (5), written in (6)): 31.5 us without, 33.9 us with both
#ifndef AMH_F64_PRE
#define AMH_F64_PRE 0
#endif
constexpr bool kF64Pre0 = AMH_F64_PRE >= 1;
constexpr bool kF64Pre = AMH_F64_PRE >= 2;

namespace {
typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int kLd = 65;          // LDS row stride of [k][chain] tiles

__device__ __forceinline__ float rdlane(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ int64_t pk(int d, int r, int k) { return col_off(d, k) + (r - k); }
}  // namespace

// -------------------------------------------------- fused stats, d = 64 --
// BASELINE configs[4]'s per-GPU work (d = 64, 65,536 chains): proposal,
// potential, accept and the pooled sums of 64-chain sub-chunks, two
// persistent 256-thread blocks per CU.  A block walks the chunks of the sums
// (128 chains, the bit spec of every d >= 64) blockIdx.x, + gridDim.x, ..,
// each as two sub-chunks whose fp32 sums accumulate in chain order.
//
// Phases per sub-chunk (wave w; lane = (i, h), i = lane & 31, h = lane >> 5):
//   (1) noise: chains w, w + 4, ..; lane = coordinate k (arwmh.py:162-165, 174)
//   (2) proposal on MFMA (row tile T = w >> 1, chain half w & 1):
//       xprop = z + fmaf(e^lam, L xi, eps xi) (arwmh.py:166-167)
//   (3) U(xprop) on MFMA, D = xprop - m formed as the B operand is read
//   (4) accept (wave 0, lane = chain; arwmh.py:173-178)
//   (5) z' out, delta = z' - mu
//   (6) S_dd on MFMA (waves 0..2: tile pairs (0,0), (1,0), (1,1)), S_d and S_a
//       sequential in chain order (wave 3); after a chunk's last sub-chunk its
//       float32 partial row in the tile layout ([S_d | S_dd tiles in register
//       order | 2 pad | S_a | N], 256-B stores; pooled_group4_kernel widens it
//       exactly).
// Operands: the A tile of L (proposal) lives in registers for the whole
// launch (one VGPR per MFMA); P (the potential's A operand) and the B operands
// are read from LDS arrays whose k index is stored in the MFMA's pair order, fperm(k) =
// 32 (k & 1) + (k >> 1), so lane half h finds the k = h, h + 2, h + 4, h + 6
// of four consecutive MFMAs in one ds_read_b128.  The next sub-chunk's z and
// keys are loaded into registers during the current one; the barriers are
// LDS-only (a __syncthreads() would drain those loads).
// Oracle: orc_pooled_stats_big (float operations and their order).
constexpr int kF = 64;       // d
constexpr int kFS = 68;      // LDS row stride (floats): rows 16-B aligned
constexpr int kFSub = 64;    // chains per sub-chunk
constexpr int kFChunk = 128; // chains per chunk of the sums (bit spec, all d >= 64)
__host__ __device__ constexpr int fperm(int k) { return (k & 1) * 32 + (k >> 1); }
namespace f64 {  // LDS layout (floats)
constexpr int kT = kF * kFS;
constexpr int Z_ = 0 /* [chain][k] z */, XI = kT /* [chain][fperm k] xi, then [k][fperm chain] delta */,
              XP = 2 * kT /* [chain][fperm k] xprop */, U_ = 3 * kT, TS = U_ + 64 /* [2][64] */, FL = TS + 128,
              AL = FL + 64, MP = AL + 64 /* m[fperm k] */, MN = MP + 64 /* m[k] */,
              PP = MN + 64 /* [r][fperm k] precision rows */, END = PP + kT;
}  // namespace f64
constexpr size_t fused64_lds_bytes() { return (size_t)f64::END * sizeof(float); }

__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// Diagnostic build only (make stamps, tools/f64_stamps.py): thread 0 of block
// 0 accumulates s_memtime ticks per phase of the d = 64 fused kernel (even
// slots: the phase's own work, odd slots: the barrier after it).
#ifdef AMH_STAMPS
__device__ unsigned long long g_f64_stamps[16];
#define FS_INIT                                   \
  unsigned long long fs_acc[16] = {0};            \
  unsigned long long fs_prev = __builtin_amdgcn_s_memtime();
#define FS(k)                                                 \
  {                                                           \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    fs_acc[k] += t_ - fs_prev;                                \
    fs_prev = t_;                                             \
  }
#define FS_FLUSH \
  if (threadIdx.x == 0 && blockIdx.x == 0) for (int k_ = 0; k_ < 16; ++k_) g_f64_stamps[k_] = fs_acc[k_];
hipError_t diag_f64_stamps_copy(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_f64_stamps), sizeof(unsigned long long) * 16, 0, hipMemcpyDeviceToHost);
}
#else
#define FS_INIT
#define FS(k)
#define FS_FLUSH
#endif
__device__ __forceinline__ f32x4 ld4(const float* a) { return *(const f32x4*)a; }

// MULTI = false: one step (sync_every = 1), the step loop compiled away.
template <bool MULTI>
__global__ __launch_bounds__(256, 2) void pooled_fused64_kernel(PooledStatsParams p, int64_t n_chunks) {
  const PooledStatsParams& p_outer = p;
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int d = kF;
  constexpr int kSub = kFChunk / kFSub;  // sub-chunks per chunk
  const int64_t Vt = d + 3 * 1024 + 4;   // pooled_big_tile_V(64)
  float* Zs = lds + f64::Z_;
  // the noise / delta tile and the proposal tile swap roles every sub-chunk:
  // sub-chunk t + 1's noise is written into this sub-chunk's proposal tile
  // during phase (6), once phase (5) has read it
  float* const XA = lds + f64::XI;
  float* const XB = lds + f64::XP;
  float* Xi = XA;
  float* Xp = XB;
  float* uu = lds + f64::U_;
  float* tsum = lds + f64::TS;
  int* flag = (int*)(lds + f64::FL);
  float* alph = lds + f64::AL;
  const float* mp = lds + f64::MP;
  const float* mn = lds + f64::MN;
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane((int)(tid / 64));
  const int h = lane >> 5, i = lane & 31;
  const int T = w >> 1, hf = w & 1;
  FS_INIT
  const float c0p = p.model.data[d + d * d];
  const int32_t it = p.i[0] + p.i_add;  // step i_add of a pooled block
  const float el = amh_expf(p.lam[0]);
  const float mu_l = p.mu[lane];  // lane = coordinate k in the chain-major phases
  float aL[32];
  // the block's sub-chunks, flat: t -> chunk blockIdx.x + gridDim.x (t / kSub),
  // sub-chunk t % kSub; only the grid's last chunk can be ragged, so the valid
  // ones are a prefix
  const int64_t G = gridDim.x;
  int64_t nmine = 0;
  if ((int64_t)blockIdx.x < n_chunks) {
    const int64_t nchk = (n_chunks - 1 - (int64_t)blockIdx.x) / G + 1;
    const int64_t last_c0 = ((int64_t)blockIdx.x + G * (nchk - 1)) * kFChunk;
    const int64_t last_subs = (p.C - last_c0 + kFSub - 1) / kFSub;
    nmine = kSub * (nchk - 1) + (last_subs < kSub ? last_subs : kSub);
  }
  auto sub_c0 = [&](int64_t t) { return ((int64_t)blockIdx.x + G * (t / kSub)) * kFChunk + kFSub * (t % kSub); };
  // z and keys of a sub-chunk's chains w + 4 N (lane = coordinate; the key's
  // two words alternate over the lanes and come back with v_readlane), pe of
  // its chains (wave 0, lane = chain)
  // (keys: lane l < 32 holds word l >> 4 of chain w + 4 (l & 15); one VGPR;
  // lanes 0..15 hold the noise record of chain w + 4 lane when noise drawn
  // ahead exists: (i, key0, key1, u bits))
  float zr[16];
  uint32_t kr = 0u;
  uint4 rec = make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
  float pev = 0.0f;
  const bool ahead = p.xi != nullptr;
  auto load_sub = [&](const PooledStatsParams& p, int64_t t) {
    const int64_t c0 = sub_c0(t);
    static_for<16>([&](auto N) {
      int64_t ch = c0 + w + 4 * N;
      if (ch >= p.C) ch = p.C - 1;
      zr[N] = p.z[ch * d + lane];
    });
    int64_t kc = c0 + w + 4 * (lane & 15);
    if (kc >= p.C) kc = p.C - 1;
    kr = p.keys[2 * kc + ((lane >> 4) & 1)];
    if (ahead) rec = (kc < p.xi_cap) ? p.xrec[kc] : make_uint4(0xFFFFFFFFu, 0u, 0u, 0u);
  };
  auto load_pe = [&](const PooledStatsParams& p, int64_t t) {
    const int64_t c0 = sub_c0(t);
    pev = (w == 0 && c0 + lane < p.C) ? p.pe[c0 + lane] : 0.0f;
  };
  auto store_z = [&]() { static_for<16>([&](auto N) { Zs[(w + 4 * N) * kFS + lane] = zr[N]; }); };
  f32x16 sacc = f32x16{};  // S_dd of the chunk so far (waves 0..2)
  float sd = 0.0f, sa = 0.0f;  // S_d (wave 3, lane = coordinate), S_a (wave 3 lane 0)
  int cnt = 0;
  // ---- (1) noise of chains w + 4 N of sub-chunk t: drawn ahead by the
  // previous update launch when the chain's record is this draw's (i, key),
  // else here.  PRE: the rows are already in xr0 (sub-chunk 0: the prologue)
  float xr0[16];
  auto noise_phase = [&](const PooledStatsParams& p, int64_t c0, auto PRE, int32_t its, uint32_t krv, bool records) {
    uint64_t usem = 0;
    if (ahead && records) {
      // lane N < 16: key word 0 of chain N is its own krv, word 1 lane N + 16's
      const uint32_t kw1 = (uint32_t)__shfl_down((int)krv, 16, 64);
      const bool ok = (lane < 16) && rec.x == (uint32_t)its && rec.y == krv && rec.z == kw1;
      usem = __ballot(ok);
    }
    if (usem == 0xFFFFull) {  // every chain of the wave: rows of the buffer (one latency)
      float xr[16];
      // the rows through one buffer descriptor with a wave-uniform base (rows
      // past C read 0 -- unused): 64-bit per-lane addresses here were hoisted
      // out of the step loop and spilled, 16 of them
      const int64_t cw = c0 + w;
      // range: the rows this wave reads (cw + 4 N, N < 16: at most 64) -- the
      // byte count stays below 2^32 for any C
      const int64_t nrow = p.C - cw;
      const int64_t nr = nrow < 64 ? (nrow > 0 ? nrow : 0) : 64;
      const Buf xb(uniform_ptr(p.xi + cw * d), (uint32_t)(nr * d) * 4u);
      static_for<16>([&](auto N) {
        if constexpr (decltype(PRE)::value) {
          xr[N] = xr0[N];
        } else {
          xr[N] = xb.ld(4u * (uint32_t)lane, 4u * (uint32_t)(4 * (int)N * d));
        }
      });
      static_for<16>([&](auto N) {
        const int cc = w + 4 * N;
        Xi[cc * kFS + fperm(lane)] = xr[N];
        const uint32_t ub = (uint32_t)__builtin_amdgcn_readlane((int)rec.w, N);
        if (lane == 0) uu[cc] = amh_unif01_from_bits(ub);
      });
    } else {
      // not every chain's row was drawn ahead: the wave draws all 16 here (the
      // buffer holds the same values).  Bit spec (amh_step_word): pass g
      // draws chains w + 4 (4 g + (lane >> 4)), call c = lane & 15 = the
      // coordinates 4c .. 4c + 3; one more pass the uniforms (call 16, word
      // 0).  Five Philox calls per lane for 16 chains (one per normal: 16).
      // (an opaque copy of the lane id: the shuffle addresses are formed here,
      // not hoisted out of the step loop -- they spilled)
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const int cq = ln & 15;
      static_for<4>([&](auto G4) {
        const int N = 4 * G4 + (ln >> 4);
        const uint32_t k0 = (uint32_t)__shfl((int)krv, N, 64), k1 = (uint32_t)__shfl((int)krv, 16 + N, 64);
        const amh_u32x4 o = amh_philox4x32_10((uint32_t)cq, (uint32_t)its, 0u, AMH_TAG_STEP, k0, k1);
        float* row = Xi + (w + 4 * N) * kFS;
        static_for<4>([&](auto E) {
          row[fperm(4 * cq + E)] = amh_normal_from_bits(o.v[E]);
          __builtin_amdgcn_sched_barrier(0);  // one normal at a time (registers for the rest of the kernel)
        });
      });
      {
        const int N = ln & 15;
        const uint32_t k0 = (uint32_t)__shfl((int)krv, N, 64), k1 = (uint32_t)__shfl((int)krv, 16 + N, 64);
        const amh_u32x4 o = amh_philox4x32_10(16u, (uint32_t)its, 0u, AMH_TAG_STEP, k0, k1);
        if (ln < 16) uu[w + 4 * ln] = amh_unif01_from_bits(o.v[0]);
      }
    }
  };
  // the first sub-chunk's loads -- z, keys, records, pe and (speculatively)
  // its noise rows -- go out before the shared operands' (one memory latency
  // in the prologue instead of three)
  if (nmine > 0) {
    load_sub(p, 0);
    load_pe(p, 0);
    const int64_t c00 = sub_c0(0);
    if constexpr (kF64Pre0) static_for<16>([&](auto N) {
      int64_t ch = c00 + w + 4 * N;
      if (ch >= p.C) ch = p.C - 1;
      xr0[N] = (ahead && ch < p.xi_cap) ? p.xi[ch * d + lane] : 0.0f;
    });
  }
  // A operands in registers: lane (i, h) of MFMA m holds row 32 T + i, column 2 m + h
  {
    // unconditional loads in one batch (above the diagonal: the row's
    // diagonal entry, replaced by 0 once loaded); P rows to LDS in fperm order
    const int r = 32 * T + i;
    float pv[16];
    static_for<32>([&](auto M) {
      const int k = 2 * M + h;
      aL[M] = p.L[pk(d, r, k <= r ? k : r)];
    });
    static_for<16>([&](auto N) { pv[N] = p.model.data[d + ((tid >> 6) + 4 * (int)N) * d + (tid & 63)]; });
    static_for<32>([&](auto M) {
      if (2 * M + h > r) aL[M] = 0.0f;
    });
    static_for<16>([&](auto N) {
      const int row = (tid >> 6) + 4 * N, k = tid & 63;
      lds[f64::PP + row * kFS + fperm(k)] = pv[N];
    });
    if (tid < d) {
      lds[f64::MP + fperm(tid)] = p.model.data[tid];
      lds[f64::MN + tid] = p.model.data[tid];
    }
  }
  if (nmine > 0) {
    store_z();
    if constexpr (kF64Pre0) noise_phase(p, sub_c0(0), std::true_type{}, it, kr, true);  // sub-chunk 0's phase (1), its rows already loaded
    else noise_phase(p, sub_c0(0), std::false_type{}, it, kr, true);
  }
  lds_barrier();
  FS(14)
  bool pre_ok = false;  // this sub-chunk's noise rows were written during the previous one
  // A pooled block of K steps (sync_every = K) runs in this one launch: a
  // sub-chunk's chains take their K transitions back to back (z in LDS, pe
  // in wave 0's registers between them) before the next sub-chunk, and the
  // chunk's sums run over (sub-chunk, step, chain) -- orc_pooled_stats64_k.
  // Step 0's noise may come from the buffer the update launch drew ahead;
  // the others are drawn here (noise_phase).
  const int32_t K = MULTI ? p.k_steps : 1;
  int64_t q = 0;  // steps of this block so far (tile parity)
  for (int64_t t = 0; t < nmine; ++t) {
    const int64_t c0 = sub_c0(t);
    const int64_t left = p.C - c0;
    const int nv = left < kFSub ? (int)left : kFSub;
    const bool more = t + 1 < nmine;
#pragma unroll 1
   for (int32_t s = 0; s < K; ++s, ++q) {
    const bool fin = s == K - 1;  // the sub-chunk's last step: z, pe go out, the next sub-chunk comes in
    // per-lane LDS / memory offsets from an opaque copy of the lane id, formed
    // in each step: hoisted out of the step loop they exceeded the registers
    // (two waves per SIMD) and spilled
    int lane_o = lane_id();
    asm volatile("" : "+v"(lane_o));
    const int lane = lane_o;
    const int h = lane >> 5, i = lane & 31;
    const PooledStatsParams& p = reload_kernarg(p_outer);  // (SGPR pressure: reload_kernarg)
    Xi = (q & 1) ? XB : XA;
    Xp = (q & 1) ? XA : XB;
    // (records are for step 0: the update launch draws the next block's first step)
    if ((t > 0 || s > 0) && !pre_ok) noise_phase(p, c0, std::false_type{}, it + s, kr, s == 0);
    if (fin && more) load_sub(p, t + 1);  // in flight through phases (2) .. (6) of the last step
    FS(0)
    lds_barrier();
    FS(1)
    // ---- (2) proposal: acc = L xi over k < 32 (T + 1)
    {
      f32x16 acc = f32x16{};
      const float* bp = Xi + (32 * hf + i) * kFS + 32 * h;
      static_for<8>([&](auto G4) {
        if (G4 < 4 * (T + 1)) {
          const f32x4 bv = ld4(bp + 4 * G4);
          static_for<4>([&](auto Q) { acc = __builtin_amdgcn_mfma_f32_32x32x2f32(aL[4 * G4 + Q], bv[(int)Q], acc, 0, 0, 0); });
        }
      });
      const int ch = 32 * hf + i;
      static_for<16>([&](auto R) {
        const int rr = 32 * T + (R & 3) + 8 * (R >> 2) + 4 * h;
        const float v = fmaf(el, acc[(int)R], p.eps * Xi[ch * kFS + fperm(rr)]);
        Xp[ch * kFS + fperm(rr)] = Zs[ch * kFS + rr] + v;  // xprop = z + (e^lam L xi + eps xi)
      });
    }
    FS(2)
    lds_barrier();
    FS(3)
    // ---- (3) U(xprop) on MFMA: Y = P D with D = xprop - m, q_r = D_r y_r
    {
      f32x16 acc = f32x16{};
      const int ch = 32 * hf + i;
      const float* bp = Xp + ch * kFS + 32 * h;
      const float* ap = lds + f64::PP + (32 * T + i) * kFS + 32 * h;
      static_for<8>([&](auto G4) {
        const f32x4 av = ld4(ap + 4 * G4);
        const f32x4 xv = ld4(bp + 4 * G4);
        const f32x4 mv = ld4(mp + 32 * h + 4 * G4);
        static_for<4>([&](auto Q) {
          acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[(int)Q], xv[(int)Q] - mv[(int)Q], acc, 0, 0, 0);
        });
      });
      float ps = 0.0f;
      static_for<16>([&](auto R) {
        const int row = 32 * T + (R & 3) + 8 * (R >> 2) + 4 * h;
        ps = ps + (Xp[ch * kFS + fperm(row)] - mn[row]) * acc[(int)R];
      });
      const float other = __shfl_xor(ps, 32, 64);
      const float tI = (h == 0) ? ps + other : other + ps;
      if (h == 0) tsum[T * 64 + ch] = tI;
    }
    FS(4)
    lds_barrier();
    FS(5)
    // ---- (4) accept / reject
    if (w == 0) {
      int acc_f = 0;
      float a = 0.0f;
      if (lane < nv) {
        float S = 0.0f;
        S = S + tsum[lane];
        S = S + tsum[64 + lane];
        float pp = (0.5f * S) + c0p;
        if (amh_isnan(pp)) pp = INFINITY;
        const float ex = amh_expf(pev - pp);
        a = (ex > 1.0f) ? 1.0f : ex;
        acc_f = uu[lane] < a;
        pev = acc_f ? pp : pev;
        if (fin) p.pe_out[c0 + lane] = pev;
      }
      flag[lane] = acc_f;
      alph[lane] = a;
      if (fin && more) load_pe(p, t + 1);
    }
    FS(6)
    lds_barrier();
    FS(7)
    // ---- the next sub-chunk's noise rows, loaded now (its records came with
    // load_sub(t + 1) in phase (1)) and written to its tile in phase (6)
    float xn[16];
    bool pre_next = false;
    if (kF64Pre && K == 1 && more && ahead) {
      const int64_t c1 = sub_c0(t + 1);
      static_for<16>([&](auto N) {
        int64_t ch = c1 + w + 4 * N;
        if (ch >= p.C) ch = p.C - 1;
        xn[N] = (ch < p.xi_cap) ? p.xi[ch * d + lane] : 0.0f;
      });
      const uint32_t kw1 = (uint32_t)__shfl_down((int)kr, 16, 64);
      const bool ok = (lane < 16) && rec.x == (uint32_t)it && rec.y == kr && rec.z == kw1;
      pre_next = __ballot(ok) == 0xFFFFull;
    }
    // ---- (5) z' out, delta = z' - mu as [k][fperm chain] over the xi array
    //      (every LDS read first, then the stores)
    {
      // LDS addresses from opaque per-lane bases + immediate offsets, and z'
      // out through a buffer descriptor whose range ends at the sub-chunk's
      // last valid chain: formed from the step's tile pointers directly, the
      // 16 per-chain addresses went to SGPRs, spilled to VGPR lanes, and the
      // phase ran ~200 v_readlane (r5l stamps: 6.9k of a sub-chunk's ~30k ticks)
      uint32_t xp_a = lds_addr(Xp) + 4u * (uint32_t)(w * kFS + fperm(lane));
      uint32_t zs_a = lds_addr(Zs) + 4u * (uint32_t)(w * kFS + lane);
      uint32_t xi_a = lds_addr(Xi) + 4u * (uint32_t)(lane * kFS + 32 * (w & 1) + (w >> 1));
      asm volatile("" : "+v"(xp_a), "+v"(zs_a), "+v"(xi_a));
      typedef __attribute__((address_space(3))) float lds_f;
      const lds_f* xpp = (const lds_f*)(uintptr_t)xp_a;
      lds_f* zsp = (lds_f*)(uintptr_t)zs_a;
      lds_f* xip = (lds_f*)(uintptr_t)xi_a;
      float zn[16];
      static_for<16>([&](auto N) {
        const int cc = w + 4 * N;
        const float xp = xpp[4 * kFS * N], zo = zsp[4 * kFS * N];
        zn[N] = flag[cc] ? xp : zo;
      });
      const int64_t rows = (int64_t)nv - w;  // chains w + 4 N < nv of this wave
      const Buf zb(uniform_ptr(p.z_out + (c0 + w) * d), rows > 0 ? (uint32_t)rows * (uint32_t)d * 4u : 0u);
      static_for<16>([&](auto N) {
        const int cc = w + 4 * N;
        if (fin) zb.st(zn[N], 4u * (uint32_t)lane, 4u * (uint32_t)(4 * d * N));  // (past nv: dropped)
        const float dv = (cc < nv) ? zn[N] - mu_l : 0.0f;
        if (!fin) zsp[4 * kFS * N] = zn[N];  // the next step's z (this lane read the slot above)
        xip[2 * N] = dv;  // Xi[lane][fperm(w + 4 N)]: fperm(w + 4 N) = fperm(w) + 2 N
      });
    }
    FS(8)
    lds_barrier();
    FS(9)
    if (pre_next) {  // the proposal tile is free now: sub-chunk t + 1's noise and u
      static_for<16>([&](auto N) {
        const int cc = w + 4 * N;
        Xp[cc * kFS + fperm(lane)] = xn[N];
        const uint32_t ub = (uint32_t)__builtin_amdgcn_readlane((int)rec.w, N);
        if (lane == 0) uu[cc] = amh_unif01_from_bits(ub);
      });
    }
    pre_ok = pre_next;
    // ---- (6) the chunk's sums, accumulated over its sub-chunks in chain order
    {
      const bool last = fin && ((t % kSub == kSub - 1) || !more);  // the chunk's last sub-chunk, last step
      float* out = (float*)p.partials + (c0 / kFChunk) * Vt;
      if (w < 3) {
        const int pI = (w == 0) ? 0 : 1, pJ = (w == 2) ? 1 : 0;
        const float* ap = Xi + (32 * pI + i) * kFS + 32 * h;
        const float* bp = Xi + (32 * pJ + i) * kFS + 32 * h;
        if (nv == kFSub) {
          static_for<8>([&](auto G4) {
            const f32x4 av = ld4(ap + 4 * G4), bv = ld4(bp + 4 * G4);
            static_for<4>([&](auto Q) { sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[(int)Q], bv[(int)Q], sacc, 0, 0, 0); });
          });
        } else {
          // ragged tail: chain pairs (2m, 2m + 1) for 2m < nv (a chain past nv
          // in the last pair holds delta = +0)
          for (int m = 0; 2 * m < nv; ++m) sacc = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[m], bp[m], sacc, 0, 0, 0);
        }
        if (last) {
          float* o = out + d + (int64_t)w * 1024 + lane;  // pair index I (I + 1) / 2 + J = w
          static_for<16>([&](auto R) { o[64 * R] = sacc[(int)R]; });
          sacc = f32x16{};
        }
      } else {
        // sequential adds in chain order (slots past nv hold +0: adding +0 to a
        // sum that started at +0 changes no bit); even chains at fperm 0..31,
        // odd ones at 32..63
        const float* rp = Xi + lane * kFS;
        static_for<8>([&](auto G4) {
          const f32x4 ev = ld4(rp + 4 * G4), ov = ld4(rp + 32 + 4 * G4);
          static_for<4>([&](auto Q) {
            sd = sd + ev[(int)Q];
            sd = sd + ov[(int)Q];
          });
        });
        if (lane == 0) {
          static_for<16>([&](auto G4) {
            const f32x4 av = ld4(alph + 4 * G4);
            static_for<4>([&](auto Q) { sa = sa + av[(int)Q]; });
          });
        }
        cnt += nv;
        if (last) {
          out[lane] = sd;
          if (lane == 0) {
            out[Vt - 2] = sa;
            out[Vt - 1] = (float)cnt;
          }
          sd = 0.0f;
          sa = 0.0f;
          cnt = 0;
        }
      }
    }
    if (fin && more) store_z();  // every wave is past its phase-(5) reads of z
    FS(10)
    lds_barrier();
    FS(11)
   }
  }
  FS_FLUSH
}

// --------------------------------------------------- fused stats, d > 64 --
// BASELINE configs[3] regime B (d = 256, 32,768 chains) and every pooled
// d = 32 NT > 64: proposal, potential, accept and the chunk sums in one
// persistent 512-thread block per CU (8 waves, 2 per SIMD: 256 registers for
// the S_dd accumulators that live across the chunk), a 128-chain chunk (the
// bit spec's chunk above d = 64) in two 64-chain halves.  The MFMA A operands (the
// shared factor's lower tiles and the precision's tiles) come from a
// per-launch copy in "A-operand order" (pooled_pack_kernel): lane (i, h)
// reads one 16-B vector = rows 32T + i, columns 32J + 8kb + 2e + h, e = 0..3,
// i.e. four consecutive v_mfma_f32_32x32x2_f32 -- the tile's 16 MFMAs are 4
// coalesced dwordx4 loads per lane, double-buffered one tile ahead.  The B
// operands (noise, D = xprop - m, delta) are [k][chain] tiles in LDS.
// Work split, per 64 chains (MFMA counts): proposal 16 NT(NT+1), wave w one
// row tile for both chain halves (at NT = 8 the waves w, w+4 that share a
// SIMD take tiles 7-w and w: equal sums per SIMD); potential 32 NT^2, wave w
// row tile w; S_dd 16 NT(NT+1) in NT(NT+1)/2 tile pairs (wave w: pairs w,
// w+8, .., accumulated over the chunk's 128 chains).  Partials are written
// in "tile" order (coalesced; pooled_final_kernel maps them to the packed
// sums).  Float operations and their
// order: those of orc_pooled_stats_big (the MFMA k order of
// gauss_pot_mfma_kernel for the potential).
constexpr int kFB = 128;  // chains per chunk above d = 64 (bit spec)
constexpr int kFBWaves = 8;
template <int NT>
constexpr size_t fused_big_lds_bytes() {
  return ((size_t)2 * 32 * NT * kLd + (size_t)NT * 64 + 3 * 64 + 32 * NT) * sizeof(float);
}
__host__ __device__ constexpr int64_t pooled_big_tile_V_dev(int d) {
  return d + (int64_t)((d / 32) * (d / 32 + 1) / 2) * 1024 + 4;
}
int64_t pooled_big_tile_V(int d) {  // [S_d | S_dd tiles | 2 pad | S_a | N]: a multiple of 4
  const int nt = d / 32;
  return d + (int64_t)(nt * (nt + 1) / 2) * 1024 + 4;
}
int64_t pooled_big_pack_floats(int d) {
  const int nt = d / 32;
  return (int64_t)(nt * (nt + 1) / 2 + nt * nt) * 1024;
}

// one block per tile: lower tiles of L (zeros above the diagonal), then the
// NT x NT tiles of the precision P (row-major in the model data)
__global__ __launch_bounds__(256) void pooled_pack_kernel(const float* __restrict__ L, const float* __restrict__ Pm,
                                                          int d, float* __restrict__ pack) {
  const int nt = d / 32;
  const int npair = nt * (nt + 1) / 2;
  const int b = blockIdx.x;
  const int t = threadIdx.x;            // = kb * 64 + lane
  const int lane = t & 63, kb = t >> 6;
  const int i = lane & 31, h = lane >> 5;
  f32x4 v;
  if (b < npair) {
    int T = 0;
    while ((T + 1) * (T + 2) / 2 <= b) ++T;
    const int J = b - T * (T + 1) / 2;
    const int row = 32 * T + i;
    static_for<4>([&](auto E) {
      const int col = 32 * J + 8 * kb + 2 * E + h;
      v[(int)E] = (col <= row) ? L[pk(d, row, col)] : 0.0f;
    });
  } else {
    const int b2 = b - npair;
    const int T = b2 / nt, J = b2 - T * nt;
    const int row = 32 * T + i;
    static_for<4>([&](auto E) { v[(int)E] = Pm[(int64_t)row * d + 32 * J + 8 * kb + 2 * E + h]; });
  }
  ((f32x4*)pack)[(int64_t)b * 256 + t] = v;
}

template <int NT>
__global__ __launch_bounds__(512) void pooled_fused_big_kernel(PooledStatsParams p, const float* __restrict__ pack,
                                                               int64_t n_chunks) {
  constexpr int D = 32 * NT;
  constexpr int NPAIR = NT * (NT + 1) / 2;
  constexpr int64_t V = D + (int64_t)NPAIR * 1024 + 4;  // "tile" partial row (pooled_final_kernel maps it)
  constexpr int NS = (NPAIR + kFBWaves - 1) / kFBWaves;  // S_dd tile pairs per wave (<= 5)
  constexpr int NQ = (D + 63) / 64;  // coordinates per lane in the chain-major phases
  constexpr int CPW = 64 / kFBWaves;  // chains per wave in the chain-major phases
  static_assert(CPW % 4 == 0, "chain-major phases take four chains at a time");
  extern __shared__ float lds[];
  float* Xb = lds;                      // [k][chain] xi, then xprop
  float* Zb = Xb + D * kLd;             // [k][chain] z, then D = xprop - m, then delta
  float* tsum = Zb + D * kLd;           // [NT][64] potential partials per row tile
  float* uu = tsum + NT * 64;           // [64]
  int* flag = (int*)(uu + 64);          // [64]
  float* alph = (float*)(flag + 64);    // [64]
  float* msh = alph + 64;               // [D] target mean m
  const f32x4* LP = (const f32x4*)pack;
  const f32x4* PP = LP + NPAIR * 256;
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane((int)(tid / 64));
  const float c0p = p.model.data[D + D * D];
  const int32_t it = p.i[0] + p.i_add;  // step i_add of a pooled block
  const float el = amh_expf(p.lam[0]);
  for (int k = tid; k < D; k += 64 * kFBWaves) msh[k] = p.model.data[k];
  float mu_l[NQ];
  static_for<NQ>([&](auto Q) { mu_l[Q] = (64 * Q + lane < D) ? p.mu[64 * Q + lane] : 0.0f; });
  // row tile of this wave in the proposal (both chain halves): at NT = 8 the
  // waves w and w + 4 that share a SIMD take T and 7 - T (equal MFMA sums)
  const int pT = (NT == 8) ? ((w < 4) ? 7 - w : w - 4) : ((w < NT) ? w : -1);
  const int qT = (w < NT) ? w : -1;  // potential row tile (both chain halves)
  int sI[NS], sJ[NS];
  static_for<NS>([&](auto S) {
    const int u = w + kFBWaves * S;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= u) ++I;
    sI[S] = (u < NPAIR) ? I : -1;
    sJ[S] = u - I * (I + 1) / 2;
  });

  for (int64_t chunk = blockIdx.x; chunk < n_chunks; chunk += gridDim.x) {
    // float32 partials (pooled_group4_kernel widens them exactly); the S_dd
    // accumulators live in registers only during (6): after each half they
    // are parked in the chunk's own partial row (tile / register order) and
    // the next half continues from them, so (1)-(5) keep their registers
    float* out = (float*)p.partials + chunk * V;
    float sd = 0.0f, sa = 0.0f;
    int cnt = 0;
#pragma unroll 1
    for (int half = 0; half < kFB / 64; ++half) {
      const int64_t c0 = chunk * kFB + 64 * half;
      const int64_t left = p.C - c0;
      if (left <= 0) break;
      const int nv = left < 64 ? (int)left : 64;
      // lane indices as opaque values: keeps the per-register addresses of
      // every phase from being hoisted out of the loops (register budget)
      int lo_ = lane;
      asm volatile("" : "+v"(lo_));
      const int h = lo_ >> 5, i = lo_ & 31;
      // (1) z and the noise xi (arwmh.py:162-165), k-major; wave w takes the
      // chains w, w + 8, ..; lane = coordinate k mod 64
      float pe_c = 0.0f;
      {
        __syncthreads();  // the previous half's readers of Zb / Xb / uu are done
#pragma unroll 1
        for (int n0 = 0; n0 < CPW; n0 += 4) {  // four chains' z (and noise) loads in flight at a time
        float zv[4][NQ], xv[4][NQ];
        bool use[4];
        uint32_t ub[4];
        static_for<4>([&](auto N) {
          int64_t ch = c0 + w + kFBWaves * (n0 + N);
          if (ch >= p.C) ch = p.C - 1;
          use[N] = false;
          ub[N] = 0u;
          if (p.xi != nullptr && ch < p.xi_cap) {  // noise drawn ahead: only if its record is this draw's
            const uint4 rec = p.xrec[ch];
            use[N] = rec.x == (uint32_t)it && rec.y == p.keys[2 * ch] && rec.z == p.keys[2 * ch + 1];
            ub[N] = rec.w;
          }
          static_for<NQ>([&](auto Q) { zv[N][Q] = (64 * Q + lane < D) ? p.z[ch * D + 64 * Q + lane] : 0.0f; });
          if (use[N]) static_for<NQ>([&](auto Q) { xv[N][Q] = (64 * Q + lane < D) ? p.xi[ch * D + 64 * Q + lane] : 0.0f; });
        });
        static_for<4>([&](auto N) {
          const int cc = w + kFBWaves * (n0 + N);
          int64_t ch = c0 + cc;
          if (ch >= p.C) ch = p.C - 1;
          if (use[N]) {
            static_for<NQ>([&](auto Q) {
              const int k = 64 * Q + lane;
              if (k < D) {
                Xb[k * kLd + cc] = xv[N][Q];
                if (k == 0) uu[cc] = amh_unif01_from_bits(ub[N]);
                Zb[k * kLd + cc] = zv[N][Q];
              }
            });
          } else {
          const uint32_t kk0 = p.keys[2 * ch], kk1 = p.keys[2 * ch + 1];
#ifndef AMH_FB_NORNG
          float xr[NQ];
          uint32_t ubw;
          step_noise_rows<NQ>(lane, D, (uint32_t)it, kk0, kk1, xr, &ubw);  // bit spec: amh_step_word
#endif
          static_for<NQ>([&](auto Q) {
            const int k = 64 * Q + lane;
            if (k < D) {
#ifndef AMH_FB_NORNG
              Xb[k * kLd + cc] = xr[Q];
              if (k == 0) uu[cc] = amh_unif01_from_bits(ubw);
#else
              Xb[k * kLd + cc] = (float)((kk0 + k) & 15) * 0.1f - 0.75f;
              if (k == 0) uu[cc] = 0.5f;
#endif
              Zb[k * kLd + cc] = zv[N][Q];
            }
          });
          }
        });
        }
        pe_c = (tid < nv) ? p.pe[c0 + tid] : 0.0f;
      }
      __syncthreads();
      // (2) proposal: acc = L xi over k < 32 (T + 1) (arwmh.py:166-167), both
      // chain halves from one A tile
      {
        float v0[16], v1[16];
        if (pT >= 0) {
          const int T = pT;
          f32x16 acc0 = f32x16{}, acc1 = f32x16{};
          const f32x4* a = LP + (T * (T + 1) / 2) * 256 + lane;
#ifndef AMH_FB_NOPROP
          // the next A tile is prefetched unconditionally (a conditional load
          // is sunk next to its use); the B operands of a tile are read in
          // one batch ahead of its MFMAs
          auto tile = [&](const f32x4 (&at)[4], int J) {
            const float* xb = Xb + (32 * J + h) * kLd + i;
            float b0[16], b1[16];
            static_for<16>([&](auto Q) {
              b0[Q] = xb[2 * Q * kLd];
              b1[Q] = xb[2 * Q * kLd + 32];
            });
            __builtin_amdgcn_sched_barrier(0);
            static_for<4>([&](auto KB) {
              static_for<4>([&](auto E) {
                acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(at[KB][(int)E], b0[4 * KB + E], acc0, 0, 0, 0);
                acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(at[KB][(int)E], b1[4 * KB + E], acc1, 0, 0, 0);
              });
            });
          };
          f32x4 cur[4], nxt[4];
          static_for<4>([&](auto KB) { cur[KB] = a[64 * KB]; });
#pragma unroll 1
          for (int J = 0; J <= T; ++J) {
            const f32x4* an = a + 256 * (J < T ? J + 1 : T);  // unconditional prefetch (the last re-reads T)
            static_for<4>([&](auto KB) { nxt[KB] = an[64 * KB]; });
            tile(cur, J);
            __builtin_amdgcn_sched_barrier(0);  // the hand-over stays behind the MFMAs
            static_for<4>([&](auto KB) { cur[KB] = nxt[KB]; });
          }
#endif
          static_for<16>([&](auto R) {
            const int rr = 32 * T + (R & 3) + 8 * (R >> 2) + 4 * h;
            v0[R] = fmaf(el, acc0[(int)R], p.eps * Xb[rr * kLd + i]);
            v1[R] = fmaf(el, acc1[(int)R], p.eps * Xb[rr * kLd + 32 + i]);
          });
        }
        __syncthreads();
        // xprop = z + (e^lam L xi + eps xi) -> Xb; D = xprop - m -> Zb
        if (pT >= 0) {
          static_for<16>([&](auto R) {
            const int rr = 32 * pT + (R & 3) + 8 * (R >> 2) + 4 * h;
            const int o = rr * kLd + i;
            const float xp0 = Zb[o] + v0[R];
            const float xp1 = Zb[o + 32] + v1[R];
            Xb[o] = xp0;
            Xb[o + 32] = xp1;
            Zb[o] = xp0 - msh[rr];
            Zb[o + 32] = xp1 - msh[rr];
          });
        }
      }
      __syncthreads();
      // (3) U(xprop) on MFMA: Y = P D, q_r = D_r y_r, tile partials in row order
      if (qT >= 0) {
        const int T = qT;
        f32x16 acc0 = f32x16{}, acc1 = f32x16{};
        const f32x4* a = PP + (T * NT) * 256 + lane;
#ifndef AMH_FB_NOPOT
        auto tile = [&](const f32x4 (&at)[4], int J) {
          const float* zb = Zb + (32 * J + h) * kLd + i;
          float b0[16], b1[16];
          static_for<16>([&](auto Q) {
            b0[Q] = zb[2 * Q * kLd];
            b1[Q] = zb[2 * Q * kLd + 32];
          });
          __builtin_amdgcn_sched_barrier(0);
          static_for<4>([&](auto KB) {
            static_for<4>([&](auto E) {
              acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(at[KB][(int)E], b0[4 * KB + E], acc0, 0, 0, 0);
              acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(at[KB][(int)E], b1[4 * KB + E], acc1, 0, 0, 0);
            });
          });
        };
        f32x4 cur[4], nxt[4];
        static_for<4>([&](auto KB) { cur[KB] = a[64 * KB]; });
#pragma unroll 1
        for (int J = 0; J < NT; ++J) {
          const f32x4* an = a + 256 * (J + 1 < NT ? J + 1 : NT - 1);  // unconditional prefetch
          static_for<4>([&](auto KB) { nxt[KB] = an[64 * KB]; });
          tile(cur, J);
          __builtin_amdgcn_sched_barrier(0);  // the hand-over stays behind the MFMAs
          static_for<4>([&](auto KB) { cur[KB] = nxt[KB]; });
        }
#endif
        float ps0 = 0.0f, ps1 = 0.0f;
        static_for<16>([&](auto R) {
          const int row = 32 * T + (R & 3) + 8 * (R >> 2) + 4 * h;
          ps0 = ps0 + Zb[row * kLd + i] * acc0[(int)R];
          ps1 = ps1 + Zb[row * kLd + 32 + i] * acc1[(int)R];
        });
        const float o0 = __shfl_xor(ps0, 32, 64), o1 = __shfl_xor(ps1, 32, 64);
        const float t0 = (h == 0) ? ps0 + o0 : o0 + ps0;
        const float t1 = (h == 0) ? ps1 + o1 : o1 + ps1;
        if (h == 0) {
          tsum[T * 64 + i] = t0;
          tsum[T * 64 + 32 + i] = t1;
        }
      }
      __syncthreads();
      // (4) accept / reject (arwmh.py:173-178)
      if (tid < 64) {
        int acc_f = 0;
        float a = 0.0f;
        if (tid < nv) {
          float S = 0.0f;
          static_for<NT>([&](auto I) { S = S + tsum[I * 64 + tid]; });
          float pp = (0.5f * S) + c0p;
          if (amh_isnan(pp)) pp = INFINITY;
          const float ex = amh_expf(pe_c - pp);
          a = (ex > 1.0f) ? 1.0f : ex;
          acc_f = uu[tid] < a;
          p.pe_out[c0 + tid] = acc_f ? pp : pe_c;
        }
        flag[tid] = acc_f;
        alph[tid] = a;
      }
      __syncthreads();
      // (5) z' out, delta = z' - mu in place of D (k-major; z re-read, L2-hot)
#pragma unroll 1
      for (int n0 = 0; n0 < CPW; n0 += 4) {
        float zr[4][NQ];  // z of the rejected chains, four chains' loads in flight
        static_for<4>([&](auto N) {
          const int cc = w + kFBWaves * (n0 + N);
          const int64_t ch = c0 + cc;
          const bool ld = cc < nv && flag[cc] == 0;
          static_for<NQ>([&](auto Q) {
            const int k = 64 * Q + lane;
            zr[N][Q] = (ld && k < D) ? p.z[ch * D + k] : 0.0f;
          });
        });
        static_for<4>([&](auto N) {
          const int cc = w + kFBWaves * (n0 + N);
          const int64_t ch = c0 + cc;
          const bool fl = flag[cc] != 0;
          static_for<NQ>([&](auto Q) {
            const int k = 64 * Q + lane;
            if (k < D) {
              float dv = 0.0f;
              if (cc < nv) {
                const float zn = fl ? Xb[k * kLd + cc] : zr[N][Q];
                p.z_out[ch * D + k] = zn;
                dv = zn - mu_l[Q];
              }
              Zb[k * kLd + cc] = dv;
            }
          });
        });
      }
      __syncthreads();
      // (6) the chunk's sums: S_d, S_a sequential over chains, S_dd on MFMA
      // sequential adds in chain order, the LDS reads batched 16 at a time
      // (the slots past nv hold +0, and adding +0 to a sum that started at
      // +0 changes no bit, so all 64 are added)
      if (tid < D) {
        static_for<4>([&](auto B) {
          float x[16];
          static_for<16>([&](auto Q) { x[Q] = Zb[tid * kLd + 16 * B + Q]; });
          static_for<16>([&](auto Q) { sd = sd + x[Q]; });
        });
      }
      if (tid == 64 * kFBWaves - 1) {
        static_for<4>([&](auto B) {
          float x[16];
          static_for<16>([&](auto Q) { x[Q] = alph[16 * B + Q]; });
          static_for<16>([&](auto Q) { sa = sa + x[Q]; });
        });
      }
      cnt += nv;
      {
      int lq_ = lane;
      asm volatile("" : "+v"(lq_));
      f32x16 sacc[NS];
      static_for<NS>([&](auto S) {
        if (half == 0 || sI[S] < 0) {
          sacc[S] = f32x16{};
        } else {
          const float* o = out + D + (int64_t)(w + kFBWaves * S) * 1024 + lq_;
          static_for<16>([&](auto R) { sacc[S][(int)R] = o[64 * R]; });
        }
      });
#ifndef AMH_FB_NOSDD
      {
        // all of the wave's tile pairs per 8-chain block: the block's
        // operands read in one LDS batch, then the pairs' MFMAs interleaved
        // (independent accumulators); each accumulator still takes the
        // chains in order
        int ra[NS], rb[NS];
        static_for<NS>([&](auto S) {
          ra[S] = (32 * (sI[S] >= 0 ? sI[S] : 0) + i) * kLd;
          rb[S] = (32 * (sI[S] >= 0 ? sJ[S] : 0) + i) * kLd;
        });
        const bool lastS = sI[NS - 1] >= 0;  // wave-uniform: the last pair may be absent
        int kk = 0;
#pragma unroll 1
        for (; kk + 8 <= nv; kk += 8) {
          float a[NS][4], b[NS][4];
          static_for<NS>([&](auto S) {
            static_for<4>([&](auto Q) {
              a[S][Q] = Zb[ra[S] + kk + 2 * Q + h];
              b[S][Q] = Zb[rb[S] + kk + 2 * Q + h];
            });
          });
          __builtin_amdgcn_sched_barrier(0);
          static_for<4>([&](auto Q) {
            static_for<NS>([&](auto S) {
              if (S + 1 < NS || lastS) sacc[S] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[S][Q], b[S][Q], sacc[S], 0, 0, 0);
            });
          });
        }
        for (; kk < nv; kk += 2)
          static_for<NS>([&](auto S) {
            if (S + 1 < NS || lastS)
              sacc[S] = __builtin_amdgcn_mfma_f32_32x32x2f32(Zb[ra[S] + kk + h], Zb[rb[S] + kk + h], sacc[S], 0, 0, 0);
          });
      }
#endif
      // S_dd tiles in register order: one coalesced 256-B row per register
      // (the final values after the chunk's last half)
      static_for<NS>([&](auto S) {
        if (sI[S] >= 0) {
          float* o = out + D + (int64_t)(w + kFBWaves * S) * 1024 + lq_;
          static_for<16>([&](auto R) { o[64 * R] = sacc[S][(int)R]; });
        }
      });
      }
    }
    if (tid < D) out[tid] = sd;
    if (tid == 64 * kFBWaves - 1) {
      out[V - 2] = sa;
      out[V - 1] = (float)cnt;
    }
  }
}

// ------------------------------------------------------------------ update --
// Diagnostic build (make stamps, tools/upd_stamps.py): thread 0's s_memtime
// totals per phase: init, diagonal blocks, panel solves, trailing updates,
// write-out, as_change rows, final reduction.
#ifdef AMH_STAMPS
__device__ unsigned long long g_upd_stamps[8];
#define US_INIT                                   \
  unsigned long long us_acc[8] = {0};             \
  unsigned long long us_prev = __builtin_amdgcn_s_memtime();
#define US(k)                                                 \
  {                                                           \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    us_acc[k] += t_ - us_prev;                                \
    us_prev = t_;                                             \
  }
#define US_FLUSH \
  if (threadIdx.x == 0) for (int k_ = 0; k_ < 8; ++k_) g_upd_stamps[k_] = us_acc[k_];
hipError_t diag_upd_stamps_copy(void* host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_upd_stamps), sizeof(unsigned long long) * 8, 0, hipMemcpyDeviceToHost);
}
// d = 64 update launch timeline on the 100 MHz constant clock (thread 0 of
// each block; atomicMax of the value, or of ~value for a minimum): [0] ~first
// block entry, [1] last reduce slice done, [2] ticket won, [3] Sigma' formed,
// [4] factorisation done, [5] update end, [6] last noise worker end,
// [7] ~first noise worker start, [8] last reduce block's group sums in LDS,
// [9] last reduce block's sums stored (before the vmcnt wait).  Copied and cleared by amh_diag_u64_timeline.
__device__ unsigned long long g_u64_rt[16];
// (kept in LDS while the block runs and flushed with atomicMax when it
// ends, so no stamp puts a memory round trip on the path it measures)
__shared__ unsigned long long g_urt_s[16];
#define URT_INIT \
  if (threadIdx.x < 16) g_urt_s[threadIdx.x] = 0ull;
#define URT_MAX(k, v) \
  if (threadIdx.x == 0) g_urt_s[k] = (unsigned long long)(v);
#define URT_FLUSH \
  if (threadIdx.x == 0)           \
    for (int k_ = 0; k_ < 16; ++k_) \
      if (g_urt_s[k_] != 0ull) atomicMax(&g_u64_rt[k_], g_urt_s[k_]);
#define URT_NOW() __builtin_amdgcn_s_memrealtime()
hipError_t diag_u64_timeline_copy(void* host) {
  hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_u64_rt), sizeof(unsigned long long) * 16, 0, hipMemcpyDeviceToHost);
  if (e != hipSuccess) return e;
  static const unsigned long long z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_u64_rt), z, sizeof(z), 0, hipMemcpyHostToDevice);
}
#else
#define US_INIT
#define US(k)
#define US_FLUSH
#define URT_MAX(k, v) ;
#define URT_INIT
#define URT_FLUSH
#define URT_NOW() 0ull
#endif

// LDS layout of the update ("A4"): column-major lower triangle where column j
// holds rows (j & ~3) .. d-1 (its first j & 3 slots are padding).  Column
// starts are multiples of 4 floats, so rows 4q .. 4q+3 of any column are one
// aligned 16-B vector: d(d+4)/2 floats, 133,120 B at d = 256.
__device__ __forceinline__ int a4_col(int d, int j) {
  const int q = j >> 2;
  return 4 * (q * d - 2 * q * (q - 1)) + (j & 3) * (d - 4 * q);
}
// index of row 0 of column j (rows r >= (j & ~3) are valid)
__device__ __forceinline__ int a4_base(int d, int j) { return a4_col(d, j) - (j & ~3); }

typedef float f32x2 __attribute__((ext_vector_type(2)));

// 16 waves (115 VGPRs with d a compile-time constant; 8 waves measured
// 2 % slower at d = 256)
#ifndef AMH_UPD_WAVES
#define AMH_UPD_WAVES 16
#endif
constexpr int kUpdWaves = AMH_UPD_WAVES;

// Trailing update of one 32x32 tile (I >= J, in 32-row blocks of the
// trailing matrix that starts at row / column q0) by the panel of columns
// p0 .. p0 + 31 on MFMA: acc = A_IJ and 16 v_mfma_f32_32x32x2_f32 with
// A = -L_I (rows x panel columns) and B = L_J^T -- per element the fmaf chain
// fmaf(-L_rj, L_cj, .) over j = p0 .. p0 + 31 in order, the oracle's bits.
__device__ __forceinline__ void trailing_tile(float* A, int d, int p0, int q0, int I, int J, int lane) {
  // The tile is formed transposed, D' = L_J (-L_I)^T: lane ii then holds row
  // rI + ii of A_IJ and its registers the columns cJ + (R & 3) + 8 (R >> 2)
  // + 4 hh, so each accumulator load / store is 32 consecutive rows of one
  // column of the column-major A4 layout (conflict-free).  Formed as
  // L_I (-L_J)^T instead, a register held one row of 32 different columns,
  // 256 - 4q floats apart: a 32-way LDS bank conflict at d = 256.  The
  // products are the same (a b = b a) in the same k order, so the bits are.
  const int hh = lane >> 5, ii = lane & 31;
  const int rI = q0 + 32 * I, cJ = q0 + 32 * J;
  f32x16 acc;
  const int row = rI + ii;
  // a4_base(d, j) = gb(q) + (j & 3) s(q) with q = j >> 2, s(q) = d - 4q and
  // gb(q) = 4 (q d - 2 q (q - 1)) - 4q: the four column groups of this lane's
  // registers (q = cJ / 4 + 2 G + hh) once, then adds
  int gb[4], gs[4];
  static_for<4>([&](auto G) {
    const int q = (cJ >> 2) + 2 * G + hh;
    gs[G] = d - 4 * q;
    gb[G] = 4 * (q * d - 2 * q * (q - 1)) - 4 * q + row;
  });
  static_for<16>([&](auto R) {
    constexpr int G = R >> 2, c3 = R & 3;
    const int col = cJ + c3 + 8 * G + 4 * hh;
    acc[(int)R] = (row >= (col & ~3)) ? A[gb[G] + c3 * gs[G]] : 0.0f;
  });
  {
    // k = p0 + 2 K2 + hh = p0 + 4 g + c, g = K2 / 2, c = 2 (K2 & 1) + hh:
    // a4_base(d, k) = a4_base(d, p0) + g (4d + 4 - 4 p0) - 8 g^2 + c (d - p0 - 4 g)
    const int kb0 = a4_base(d, p0), pt16 = 4 * d + 4 - 4 * p0, ps0 = d - p0;
    static_for<16>([&](auto K2) {
      constexpr int g = K2 >> 1, c2 = 2 * (K2 & 1);
      const int kb = kb0 + g * pt16 - 8 * g * g + (c2 + hh) * (ps0 - 4 * g);
      const float av = A[kb + cJ + ii];
      const float bv = -A[kb + rI + ii];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc, 0, 0, 0);
    });
  }
  static_for<16>([&](auto R) {
    constexpr int G = R >> 2, c3 = R & 3;
    const int col = cJ + c3 + 8 * G + 4 * hh;
    if (row >= col) A[gb[G] + c3 * gs[G]] = acc[(int)R];
  });
}

// The shared factor's column k: y = amh_rsqrt_nr(x) (three Newton steps from
// the bit-pattern seed, include/amh_math.h), L_kk = x y and q = n y -- the
// oracle's operations in the same order, so the same bits.  Eleven dependent
// VALU operations (the IEEE sqrtf + division expansions were about 30 and set
// the factorisation's pivot-chain latency).  fill(S), S = 0..15, runs between
// the chain's steps with a scheduling barrier on both sides: independent work
// (the previous column's updates) placed in the chain's dependency stalls,
// which an in-order wave cannot fill by itself.
template <class F>
__device__ __forceinline__ void nr_sqrt_div(float x, float n, float& sq, float& qt, float& yo, F&& fill) {
  auto step = [&](auto S) {
    __builtin_amdgcn_sched_barrier(0);
    fill(S);
    __builtin_amdgcn_sched_barrier(0);
  };
  using namespace std;
  const float h = 0.5f * x;
  float y = __uint_as_float(0x5F375A86u - (__float_as_uint(x) >> 1));
  step(integral_constant<int, 0>{});
  float t = y * y;
  step(integral_constant<int, 1>{});
  t = fmaf(-h, t, 1.5f);
  step(integral_constant<int, 2>{});
  y = y * t;
  step(integral_constant<int, 3>{});
  t = y * y;
  step(integral_constant<int, 4>{});
  t = fmaf(-h, t, 1.5f);
  step(integral_constant<int, 5>{});
  y = y * t;
  step(integral_constant<int, 6>{});
  t = y * y;
  step(integral_constant<int, 7>{});
  t = fmaf(-h, t, 1.5f);
  step(integral_constant<int, 8>{});
  y = y * t;
  step(integral_constant<int, 9>{});
  sq = x * y;
  qt = n * y;
  yo = y;
  step(integral_constant<int, 10>{});
  step(integral_constant<int, 11>{});
  step(integral_constant<int, 12>{});
  step(integral_constant<int, 13>{});
  step(integral_constant<int, 14>{});
  step(integral_constant<int, 15>{});
}
template <class F>
__device__ __forceinline__ void nr_sqrt_div(float x, float n, float& sq, float& qt, F&& fill) {
  float y;
  nr_sqrt_div(x, n, sq, qt, y, static_cast<F&&>(fill));
}

template <int NT>
__global__ __launch_bounds__(64 * kUpdWaves) void pooled_big_update_kernel(PooledUpdateParams p) {
  extern __shared__ __attribute__((aligned(16))) float A[];  // A4 layout, float32
  constexpr int d = 32 * NT;  // compile-time: the A4 offsets of every phase fold to constants
  if (blockIdx.x > 0) {
    // extra blocks (one per CU, beside the single-workgroup factorisation):
    // the next step's noise xi and u bits of every chain at i' = i + K
    // (the step stream, amh_step_word; pooled_big_prep_kernel left i' in the
    // staging buffer), each chain's row with its record
    const int32_t inext = ((const int*)p.scratch)[d * (d + 4) / 2 + 4];
    const int lane = lane_id();
    const int64_t wv = (int64_t)(blockIdx.x - 1) * kUpdWaves + threadIdx.x / 64;
    const int64_t nw = (int64_t)(gridDim.x - 1) * kUpdWaves;
    for (int64_t ch = wv; ch < p.noise_C; ch += nw) {
      const uint32_t kk0 = p.keys[2 * ch], kk1 = p.keys[2 * ch + 1];
      uint32_t ubits = 0u;
      float xr[(d + 63) / 64];
      step_noise_rows<(d + 63) / 64>(lane, d, (uint32_t)inext, kk0, kk1, xr, &ubits);  // bit spec: amh_step_word
      static_for<(d + 63) / 64>([&](auto Q) {
        const int k = 64 * Q + lane;
        if (k < d) p.xi[ch * d + k] = xr[Q];
      });
      if (lane == 0) p.xrec[ch] = make_uint4((uint32_t)inext, kk0, kk1, ubits);
    }
    return;
  }
  __shared__ int okv;
  __shared__ __attribute__((aligned(16))) float colbuf[kUpdWaves * 128];  // per-wave column broadcasts
  const int tid = threadIdx.x;
  US_INIT
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane((int)(tid / 64));
  const double* sums = p.sums;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const double N = sums[d + P + 1];
  const int32_t it = p.in.i[0];
  const int32_t itr = it + p.K;
  const int32_t n = pooled_block_n(it, p.W, p.K);
  const float gamma = amh_lr_gamma(n, p.a);
  const float macc = p.in.mean_accept_prob[0];
  const float lam = p.in.log_step_size[0];
  const float abar = (float)(sums[d + P] / N);
  const float maccn = macc + (abar - macc) / (float)n;
  const float lamn = lam + gamma * (abar - p.target);
  // (0) A = float((1-g) Sigma + g S_dd / N), formed in the 4-row-aligned
  // layout by pooled_big_prep_kernel (all CUs): one coalesced 16-B copy.
  // d = 64 (2,080 entries) forms it here, wave w for columns w + 16 q, lane
  // = row offset, with the same double arithmetic (one launch instead of
  // three, see (4)).  Every global operand of the d = 64 update -- the old
  // covariance and factor for the write-out, S_d and mu for the mean -- is
  // loaded here in one batch and kept in registers (one memory latency
  // instead of one per phase and column).
  constexpr int kQ = NT == 2 ? d / kUpdWaves : 1;
  double sig[kQ], cvo[kQ];
  float lvo[kQ];
  float loc_in = 0.0f;
  double sd_in = 0.0;
  if constexpr (NT == 2) {
    static_assert(d % kUpdWaves == 0, "d = 64: whole columns per wave");
    const double g = (double)gamma;
    double sv[kQ];
    static_for<kQ>([&](auto Q) {
      const int k = w + kUpdWaves * Q;
      const int64_t o = col_off(d, k) + (lane < d - k ? lane : 0);
      cvo[Q] = p.in.cov[o];
      sv[Q] = sums[d + o];
      lvo[Q] = p.in.scale[o];
    });
    if (tid < d) {
      loc_in = p.in.loc[tid];
      sd_in = sums[tid];
    }
    static_for<kQ>([&](auto Q) {
      const int k = w + kUpdWaves * Q;
      const double a = (1.0 - g) * cvo[Q];
      const double b = g * (sv[Q] / N);
      sig[Q] = a + b;
      if (lane < d - k) A[a4_base(d, k) + k + lane] = (float)sig[Q];
    });
  } else {
    const int nA = d * (d + 4) / 2;
    const f32x4* src = (const f32x4*)p.scratch;
    f32x4* dst = (f32x4*)A;
    for (int q = tid; q < nA / 4; q += 64 * kUpdWaves) dst[q] = src[q];
  }
  if (tid == 0) okv = 1;
  __syncthreads();
  US(0)
#pragma unroll 1
  for (int p0 = 0; p0 < d; p0 += 32) {
    // (1) the panel's 32 columns, rows p0 .. d-1, in registers: wave v holds
    // the diagonal block's rows p0 + ii in lanes ii < 32 (every wave a copy,
    // so no wave waits for another) and the rows p0 + 32 (v + 1) + ii below
    // it in lanes 32 + ii.  Column k: pivot from lane k, y = rsqrt_nr, the
    // whole column scaled by y, then column k's update of the panel's later
    // columns with L_mk broadcast from lane m (v_readlane) -- per element the
    // oracle's fmaf chain in column order.  Lanes above the diagonal compute
    // values that are never used.
    {
      const int nbelow = (d - p0 - 32) / 32;  // 32-row blocks below the diagonal block
      const int nwv = nbelow > 0 ? nbelow : 1;
      if (w < nwv) {
        int ln = lane;  // opaque: keeps the per-column lane tests from being hoisted into SGPR spills
        asm volatile("" : "+v"(ln));
        const int ii = ln & 31;
        const bool below = ln >= 32;
        const bool live = !below || w < nbelow;
        const int r = below ? (live ? p0 + 32 * (w + 1) + ii : d - 1) : p0 + ii;
        // unconditional loads: entries above the diagonal read in-range
        // neighbours (never used), rows past d read row d - 1
        float a[32];
        const int ab0 = a4_base(d, p0) + r;
        // a4_base(d, p0 + K) - a4_base(d, p0) for K = 4 g + c (p0 = 4 q0):
        // g (4d + 4 - 16 q0) - 8 g^2 + c (d - 4 q0 - 4 g) -- two runtime
        // values, the rest folds (the quadratic evaluated per K was the
        // panel's load and write-back time)
        const int pt16 = 4 * d + 4 - 4 * p0, ps0 = d - p0;
        auto poff = [&](auto K) {
          constexpr int g = K >> 2, c = K & 3;
          return g * pt16 - 8 * g * g + c * (ps0 - 4 * g);
        };
        static_for<32>([&](auto K) { a[K] = A[ab0 + poff(K)]; });
        US(2)
        bool ok = true;
        float* cb = colbuf + 128 * w;  // this wave's two column broadcast rows
        // Software pipeline over the columns: column k's pivot, square root
        // and division come first; then column k-1's LDS-broadcast updates
        // (m >= k+1, read while column k was being formed) are applied; then
        // column k goes to LDS and its next-column update a[k+1] is done with
        // v_readlane.  Every element still sees its updates in column order.
        f32x4 pv[8];  // column k-1's broadcast values (rows 4q .. 4q+3)
        float am1 = 0.0f;
        // the pivot chain on wave-uniform values and the lean column of
        // pooled_update64_kernel: next pivot = fmaf(-l1, l1, sa), l1 = n1 y;
        // column k (unscaled) and column k + 1 to the wave's two broadcast
        // rows at the column's start (n1, the panel rows and sa come back
        // while the chain runs), the rows scaled by y on the way back (the
        // vector path's q, bit for bit), column k's updates of columns k + 1
        // and k + 2 right after it, no select for the diagonal
        float pivu = rdlane(a[0], 0);
        asm volatile("" : "+v"(pivu));  // a VGPR value: the seed's integer ops stay on the VALU
        static_for<32>([&](auto K) {
          constexpr int k = K;
          f32x4 pn[8];
          float sa = 0.0f;
          if constexpr (k + 1 < 32) {
            cb[ln] = a[k];
            cb[64 + ln] = a[k + 1];
            static_for<8>([&](auto Q) {
              if constexpr (4 * Q + 3 >= k + 1) pn[(int)Q] = *(const f32x4*)&cb[4 * Q];
            });
            sa = cb[64 + k + 1];
          }
          ok = ok && amh_pivot_ok(pivu);
          // y = amh_rsqrt_nr(piv), q = a[k] y, with column k-1's updates of
          // the panel's columns m >= k+2 (packed pairs (m, m + 1), m even;
          // column k + 2 alone when odd) in the chain's stalls (nr_sqrt_div;
          // the oracle's bits)
          float ljj, q, y;
          nr_sqrt_div(pivu, a[k], ljj, q, y, [&](auto Sl) {
            if constexpr (k >= 1) {
              constexpr int m0 = ((k + 2) % 2 == 0) ? k + 2 : k + 3;
              if constexpr (Sl == 0 && m0 != k + 2 && k + 2 < 32) a[k + 2] = fmaf(-am1, pv[(k + 2) / 4][(k + 2) % 4], a[k + 2]);
              constexpr int m = m0 + 2 * Sl;
              if constexpr (m + 1 < 32) {
                const f32x2v rr = __builtin_elementwise_fma(f32x2v{-am1, -am1},
                                                            f32x2v{pv[m / 4][m % 4], pv[m / 4][m % 4 + 1]},
                                                            f32x2v{a[m], a[m + 1]});
                a[m] = rr[0];
                a[m + 1] = rr[1];
              }
            }
          });
          a[k] = q;
          if constexpr (k + 1 < 32) {
            static_for<8>([&](auto Q) {
              if constexpr (4 * Q + 3 >= k + 1) {
                f32x4& pq = pn[(int)Q];  // whole vector live to here (pooled_update64_kernel)
                asm volatile("" : "+v"(pq));
              }
            });
            const float n1 = pn[(k + 1) / 4][(k + 1) % 4];
            const float l1 = n1 * y;
            pivu = fmaf(-l1, l1, sa);
            static_for<8>([&](auto Q) {
              if constexpr (4 * Q + 3 >= k + 2) {  // v_pk_mul_f32 pairs
                const f32x2v lo = f32x2v{pn[(int)Q][0], pn[(int)Q][1]} * f32x2v{y, y};
                const f32x2v hi = f32x2v{pn[(int)Q][2], pn[(int)Q][3]} * f32x2v{y, y};
                pv[(int)Q] = f32x4{lo[0], lo[1], hi[0], hi[1]};
              }
            });
            am1 = q;
            a[k + 1] = fmaf(-q, l1, a[k + 1]);
            if constexpr (k + 2 < 32) a[k + 2] = fmaf(-q, pv[(k + 2) / 4][(k + 2) % 4], a[k + 2]);
          }
          __builtin_amdgcn_sched_barrier(0);
        });
        US(1)
        if (w == 0 && lane == 0 && !ok) okv = 0;
        // branch-free write-back: lanes with nothing to write (above the
        // diagonal, past d, or a diagonal copy of a wave other than 0) store
        // to this wave's scratch slot instead
        {
          const int dummy = (int)(colbuf + 128 * w + 64 + ln - A);
          // last column this lane writes: all 32 below the block, K <= ii in
          // wave 0's copy of the block, none otherwise
          const int kmax = below ? (live ? 31 : -1) : (w == 0 ? ii : -1);
          static_for<32>([&](auto K) {
            const int o = ((int)K <= kmax) ? ab0 + poff(K) : dummy;
            A[o] = a[K];
          });
        }
      }
    }
    US(7)
    // (2) look-ahead: while the panel's columns are factored, the other waves
    // apply the previous panel's trailing update to the column blocks right
    // of this panel (that panel's tiles with J >= 1; its J = 0 column block
    // -- this panel -- was updated before this panel was loaded)
    if (p0 >= 32) {
      const int nbelow = (d - p0 - 32) / 32;
      const int nwv = nbelow > 0 ? nbelow : 1;
      const int q0 = p0;  // first row / column of the previous panel's trailing matrix
      const int mt = (d - q0) / 32;
      const int npair1 = mt * (mt - 1) / 2;  // tile pairs with J >= 1
      for (int u = w - nwv; u >= 0 && u < npair1; u += kUpdWaves - nwv) {
        int I = 0;
        while ((I + 1) * (I + 2) / 2 <= u) ++I;
        trailing_tile(A, d, p0 - 32, q0, I + 1, u - I * (I + 1) / 2 + 1, lane);
      }
    }
    __syncthreads();
    US(3)
    // (3) this panel's trailing update of the next column block (tiles J = 0)
    if (p0 + 32 < d) {
      const int mt = (d - p0 - 32) / 32;
      if (w < mt) trailing_tile(A, d, p0, p0 + 32, w, 0, lane);
    }
    __syncthreads();
    US(5)
  }
  const bool ok = okv != 0;
  if constexpr (NT == 2) {
    // d = 64: pooled_big_post_kernel's work in this block, the same float
    // ops and sum order (a column's rows fit one wave, so of its 256-lane
    // big_sum only the first 64-lane butterfly is non-zero)
    __shared__ float colsum[64];
    const float e0 = amh_expf(lam), e1 = amh_expf(lamn);
    static_for<kQ>([&](auto Q) {
      const int k = w + kUpdWaves * Q;
      const int64_t co = col_off(d, k);
      const int ab = a4_base(d, k);
      float sq = 0.0f;
      if (lane < d - k) {
        const int64_t o = co + lane;
        const float lo = lvo[Q];
        const float ln = ok ? A[ab + k + lane] : lo;
        const float tt = (ln * e1) - (lo * e0);
        sq = tt * tt;
        p.out.cov[o] = ok ? sig[Q] : cvo[Q];
        p.out.scale[o] = ln;
      }
      const float s0 = Grp<64>::sum(sq);
      if (lane == 0) colsum[k] = (s0 + 0.0f) + (0.0f + 0.0f);
    });
    __syncthreads();
    if (w == 0) {
      const float S = Grp<64>::sum(colsum[lane]);
      if (lane == 0) {
        p.out.as_change[0] = sqrtf((S + 0.0f) + (0.0f + 0.0f));
        p.out.i[0] = itr;
        p.out.mean_accept_prob[0] = maccn;
        p.out.log_step_size[0] = lamn;
      }
    }
  } else {
  // (4) the new factor back to the staging buffer (coalesced) with the ok
  // flag, gamma and e^lam, e^lam' for pooled_big_post_kernel (all CUs), which
  // copies it to out.scale / out.cov and forms the as_change terms
  {
    const int nA = d * (d + 4) / 2;
    f32x4* dst = (f32x4*)p.scratch;
    const f32x4* src = (const f32x4*)A;
    for (int q = tid; q < nA / 4; q += 64 * kUpdWaves) dst[q] = src[q];
    if (tid == 0) {
      ((int*)p.scratch)[nA] = ok ? 1 : 0;
      p.scratch[nA + 1] = gamma;
      p.scratch[nA + 2] = amh_expf(lam);
      p.scratch[nA + 3] = amh_expf(lamn);
      p.out.i[0] = itr;
      p.out.mean_accept_prob[0] = maccn;
      p.out.log_step_size[0] = lamn;
    }
  }
  }
  if constexpr (NT == 2) {
    if (tid < d) p.out.loc[tid] = loc_in + gamma * (float)(sd_in / N);
  } else {
    if (tid < d) p.out.loc[tid] = p.in.loc[tid] + gamma * (float)(sums[tid] / N);
  }
  US(4)
  US_FLUSH
}

// d = 64 (BASELINE configs[4]): the whole shared-state update in one
// 256-thread workgroup.  Every global operand (Sigma, S_dd, the old factor,
// S_d, mu) is loaded in one batch by the four waves (wave w: columns w + 4 q,
// lane = row offset), Sigma' = (1-g) Sigma + g S_dd / N is formed in double
// and rounded into LDS row by row, then wave 0 factors it with lane r holding
// row r in 64 registers: column k's pivot comes from lane k (v_readlane),
// L_kk = piv y (y = amh_rsqrt_nr), the column scaled by y, column k's update of column k + 1
// follows through v_readlane (the next pivot is then ready), and its update
// of the columns beyond arrives through a 64-float LDS broadcast applied
// after the next column's pivot and division (software-pipelined; per
// element the oracle's fmaf chain in column order, so the bits are those of
// the panel kernel it replaces and of orc_pooled_update_big).  The write-out
// and as_change (column sums by the 64-lane butterfly, then the columns)
// follow on all four waves.
// ------------------------------------------------ chunk reduction, d >= 64 --
// The fused stats kernels' float32 partial rows (tile layout, V floats per
// 128-chain chunk) -> the packed double sums, in the bit spec's order
// (pooled_group4_kernel + pooled_final_kernel): per entry, the chunks of each
// group of 16 summed in chunk order from 0.0, then the group sums in group
// order from 0.0 (then += the sums so far when accumulating over a pooled
// block; with `fp`, the update's Sigma' entry as pooled_final_kernel forms
// it).  One 512-thread block owns 16 float4 columns of the row for every
// group: thread (tg, c) sums group 32 gt + tg of column c into LDS, then 64
// threads (column, component) add the group sums in order, tile by tile.
// One launch instead of two; with `coherent` the sums go out write-through
// (agent-scope stores) for a reader in another XCD.
constexpr int kRedCols = 16;  // float4 columns per reduce block (32 groups per pass)
constexpr int kRedGrp = 16;   // chunks per group (pooled_reduce's kRedGroup)
int pooled_reduce64_blocks(int64_t V) { return (int)((V / 4 + kRedCols - 1) / kRedCols); }

// NCOL float4 columns x (512 / NCOL) groups per pass: 16 x 32, or 32 x 16
// when there are at most 16 groups (d = 256 at C = 32,768), so no thread idles
template <int NCOL = kRedCols>
__device__ __forceinline__ void reduce_tiles_slice(const float* __restrict__ partials, int64_t n_chunks, int64_t V,
                                                   double* sums, int accumulate, int blk, int tile_d,
                                                   const FinalPrep& fp, bool coherent) {
  constexpr int GT = 512 / NCOL;  // groups per pass
  __shared__ double gs[GT][NCOL][4];
  const int tid = threadIdx.x;
  const int c = tid % NCOL, tg = tid / NCOL;
  const int64_t v4 = (int64_t)blk * NCOL + c;
  const bool col_ok = 4 * v4 < V;
  const int64_t n_groups = (n_chunks + kRedGrp - 1) / kRedGrp;
  const int fc = tid >> 2, comp = tid & 3;  // finishing threads (tid < 4 NCOL)
  double tot = 0.0;
  for (int64_t g0 = 0; g0 < n_groups; g0 += GT) {
    const int64_t g = g0 + tg;
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    if (g < n_groups && col_ok) {
      const int64_t q0 = g * kRedGrp;
      const int64_t q1 = q0 + kRedGrp < n_chunks ? q0 + kRedGrp : n_chunks;
      float4 x[kRedGrp];
#pragma unroll
      for (int q = 0; q < kRedGrp; ++q) x[q] = (q0 + q < q1) ? ((const float4*)(partials + (q0 + q) * V))[v4] : float4{};
#pragma unroll
      for (int q = 0; q < kRedGrp; ++q)
        if (q0 + q < q1) {  // chunk order; a missing tail chunk is not added at all
          s0 += (double)x[q].x;
          s1 += (double)x[q].y;
          s2 += (double)x[q].z;
          s3 += (double)x[q].w;
        }
    }
    gs[tg][c][0] = s0;
    gs[tg][c][1] = s1;
    gs[tg][c][2] = s2;
    gs[tg][c][3] = s3;
    __syncthreads();
    if (coherent) URT_MAX(8, URT_NOW())
    if (tid < 4 * NCOL) {
      const int ng = (int)(n_groups - g0 < GT ? n_groups - g0 : GT);
      // group order; eight LDS reads in flight ahead of their adds (one read
      // and one add at a time was a dependent LDS round trip per group)
      for (int q0 = 0; q0 < ng; q0 += 8) {
        double v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = gs[q0 + e < ng ? q0 + e : ng - 1][fc][comp];
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (q0 + e < ng) tot += v[e];
      }
    }
    __syncthreads();
  }
  if (tid < 4 * NCOL) {
    const int64_t u = 4 * ((int64_t)blk * NCOL + fc) + comp;
    if (u < V) final_entry(u, tot, V, sums, accumulate, tile_d, fp, coherent);
  }
  if (coherent) URT_MAX(9, URT_NOW())
}

template <int NCOL>
__global__ __launch_bounds__(512) void pooled_reduce_tiles_kernel(const float* __restrict__ partials, int64_t n_chunks,
                                                                  int64_t V, double* sums, int accumulate, int tile_d,
                                                                  FinalPrep fp) {
  reduce_tiles_slice<NCOL>(partials, n_chunks, V, sums, accumulate, (int)blockIdx.x, tile_d, fp, false);
}

hipError_t launch_reduce_tiles(const float* partials, int64_t n_chunks, int64_t V, double* sums, int accumulate,
                               int tile_d, const FinalPrep& fp, hipStream_t s) {
  const int64_t n_groups = (n_chunks + kRedGrp - 1) / kRedGrp;
  if (n_groups <= 16) {
    hipLaunchKernelGGL(pooled_reduce_tiles_kernel<32>, dim3((unsigned)((V / 4 + 31) / 32)), dim3(512), 0, s, partials,
                       n_chunks, V, sums, accumulate, tile_d, fp);
  } else {
    hipLaunchKernelGGL(pooled_reduce_tiles_kernel<16>, dim3((unsigned)((V / 4 + 15) / 16)), dim3(512), 0, s, partials,
                       n_chunks, V, sums, accumulate, tile_d, fp);
  }
  return hipGetLastError();
}

__global__ __launch_bounds__(512) void pooled_update64_kernel(PooledUpdateParams p) {
  constexpr int d = 64, P = d * (d + 1) / 2;
  constexpr int S = d + 1;  // LDS row stride of the factor
  constexpr int kQ8 = d / 8;  // columns per wave in the load / write-out phases
  __shared__ float A[d * S];
  __shared__ __attribute__((aligned(16))) float cols[64][64];  // finished factor columns (broadcast)
  __shared__ float colsum[64];
  __shared__ int okv, done[64];
  __shared__ __attribute__((aligned(16))) float bc[4][2][64];  // a factoring wave's column broadcast rows
  // the factoring waves' write-out operands, parked here while they factor
  // (they would otherwise stay live across the factorisation)
  __shared__ double park_s[kQ8][256], park_c[kQ8][256];
  __shared__ float park_l[kQ8][256];
  const int nred = p.red_blocks;        // > 0: reduce the chunk partials first
  const int base = nred > 0 ? nred : 1;  // blocks [0, base): reduce / update; the rest draw noise
  // the next step's noise xi and u bits of every chain at i' = i + K (the
  // step stream, amh_step_word), each chain's row with its
  // record (the stats kernel uses a row only if the record is its draw), by
  // `nworkers` 8-wave workers: the noise blocks, and the reduce blocks that
  // do not run the update (after their slice) -- every CU but the update's
  // The reduce blocks join ~5 us late (their slice, the write-through and
  // the ticket first), so they take the chains [split, C) at 70 % of a noise
  // block's share per wave; the noise blocks take [0, split).
  const int nnoise = (int)gridDim.x - base;  // noise blocks ([base, gridDim.x))
  const int nlate = (nnoise > 0 && nred > 0) ? nred - 1 : 0;
  const int64_t split =
      nlate > 0 ? (int64_t)((double)p.noise_C * (double)nnoise / ((double)nnoise + 0.7 * (double)nlate)) : p.noise_C;
  // the noise position, read before any block can reach the update's write of
  // out.i (in place, in == out): a late reduce worker reads it in a register
  const int32_t inext = p.in.i[0] + p.K;
  URT_INIT
  URT_MAX(0, ~URT_NOW())
  auto draw_noise = [&](int64_t worker, int64_t nworkers, int64_t cbeg, int64_t cend) {
    const int lane = lane_id();
    // wave wv takes the chains cbeg + wv, + nw, .. in batches of 64 (lane l
    // loads the key of the batch's l-th).  Bit spec (amh_step_word): per
    // chain the 16 calls 0..15 give the 64 normals (word k of call c is
    // coordinate 4c + k) and call 16's word 0 the accept uniform.  One pass
    // draws four chains (lane >> 4) x 16 calls (lane & 15) -- four normals
    // per lane, stored as one 16-B vector (each chain's 256-B row
    // contiguous) -- and one more pass per batch the 64 uniforms with the
    // records: 17 Philox calls per 64 chains per lane where one call per
    // normal took 64.
    const int64_t wv = cbeg + worker * 8 + threadIdx.x / 64;
    const int64_t nw = nworkers * 8;
    for (int64_t c64 = wv; c64 < cend; c64 += 64 * nw) {
      const int64_t mc = c64 + nw * lane;
      const int64_t mcl = mc < cend ? mc : cend - 1;
      const uint32_t mk0 = p.keys[2 * mcl], mk1 = p.keys[2 * mcl + 1];
      {
        const amh_u32x4 o = amh_philox4x32_10(16u, (uint32_t)inext, 0u, AMH_TAG_STEP, mk0, mk1);
        if (mc < cend) p.xrec[mc] = make_uint4((uint32_t)inext, mk0, mk1, o.v[0]);
      }
      const int cq = lane & 15;
      for (int g = 0; g < 16; ++g) {
        if (c64 + nw * (4 * g) >= cend) break;  // (wave-uniform) no chain of this pass left
        const int j = 4 * g + (lane >> 4);
        const uint32_t k0 = (uint32_t)__shfl((int)mk0, j, 64), k1 = (uint32_t)__shfl((int)mk1, j, 64);
        const amh_u32x4 o = amh_philox4x32_10_unrolled((uint32_t)cq, (uint32_t)inext, 0u, AMH_TAG_STEP, k0, k1);
        float xv[4], uv[4], wv0[4];
        static_for<4>([&](auto E) { xv[E] = amh_normal_head(o.v[E], &uv[E], &wv0[E]); });
        static_for<4>([&](auto E) {  // the erfinv tail only where some lane needs it
          if (__builtin_amdgcn_ballot_w64(!(wv0[E] < 5.0f)) != 0) {
            const float pl = amh_erfinv_tail(wv0[E]);
            xv[E] = (wv0[E] < 5.0f) ? xv[E] : pl;
          }
          xv[E] = 1.41421356f * (xv[E] * uv[E]);
        });
        const int64_t ch = c64 + nw * j;
        if (ch < cend) *(f32x4*)(p.xi + ch * d + 4 * cq) = f32x4{xv[0], xv[1], xv[2], xv[3]};
      }
    }
  };
  // one call site of draw_noise (two inlined copies cost the update path
  // its registers): noise blocks go straight there, the reduce blocks that
  // lose the ticket after their slice
  int64_t nz_worker = (int64_t)blockIdx.x - base, nz_count = nnoise, nz_beg = 0, nz_end = split;
  bool noise_role = (int)blockIdx.x >= base;
  const bool coh = nred > 0;  // the sums were just written by other blocks (maybe other XCDs)
  if (!noise_role && nred > 0) {
    reduce_tiles_slice(p.red_partials, p.red_chunks, pooled_big_tile_V_dev(d), p.sums_out, p.red_accumulate,
                       (int)blockIdx.x, d, FinalPrep{}, true);
    // the last block to finish its slice runs the update: write-through
    // stores done (vmcnt(0)), then an agent-scope ticket; the last arriver
    // reads the sums with agent-scope loads (the cross-XCD hand-off of
    // pooled_big_post_kernel)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    URT_MAX(1, URT_NOW())
    __shared__ int tk;
    int* ticket = (int*)p.scratch + d * (d + 4) / 2 + 5;
    // a relaxed ticket after the write-through stores completed; the last
    // arriver acquires (AMH_TICKET_ORDER above)
    if (threadIdx.x == 0) tk = __hip_atomic_fetch_add(ticket, 1, AMH_TICKET_ORDER, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    // The last arriver reads every block's sums with sc1 (agent-scope relaxed)
    // loads only, the producers stored them sc1 and drained before their add:
    // the write-through form that replaces the acquire (MI355X_MICROARCH.md,
    // inter-workgroup visibility, "Valid forms", first table row), so no
    // buffer_inv (~1.7 us) sits on the update's critical path.
    // AMH_HANDOFF_FENCE=1 keeps the acquire (A/B).
    if (AMH_HANDOFF_FENCE && tk == nred - 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    if (tk != nred - 1) {  // not the last: a noise worker
      if (nlate == 0) {
        URT_FLUSH
        return;
      }
      noise_role = true;
      nz_worker = tk;
      nz_count = nlate;
      nz_beg = split;
      nz_end = p.noise_C;
    } else if (threadIdx.x == 0) {
      __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // next launch
    }
  }
  if (noise_role) {
    URT_MAX(7, ~URT_NOW())
    draw_noise(nz_worker, nz_count, nz_beg, nz_end);
#ifdef AMH_STAMPS
    __syncthreads();
#endif
    URT_MAX(6, URT_NOW())
    URT_FLUSH
    return;
  }
  URT_MAX(2, URT_NOW())
  // eight waves: wave w loads / forms / writes out the columns w + 8 Q;
  // waves 0..3 factor (wave f owns the columns 16 f .. 16 f + 15)
  const int tid = threadIdx.x;
  US_INIT
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane((int)(tid / 64));
  const double* sums = p.sums;
  auto ldsum = [&](int64_t i) -> double {
    return coh ? __hip_atomic_load(&sums[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : sums[i];
  };
  if (tid == 0) {
    done[0] = 0;
    okv = 1;
  }
  // (0) one batch of loads (issued before anything waits on the scalars)
  double sig[kQ8], cvo[kQ8], sv[kQ8];
  float lvo[kQ8];
  static_for<kQ8>([&](auto Q) {
    const int k = w + 8 * Q;
    const int64_t o = col_off(d, k) + (lane < d - k ? lane : 0);
    cvo[Q] = p.in.cov[o];
    sv[Q] = ldsum(d + o);
    lvo[Q] = p.in.scale[o];
  });
  const float loc_in = p.in.loc[lane];
  const double sd_in = ldsum(lane);
  const double N = ldsum(d + P + 1);
  const int32_t it = p.in.i[0];
  const int32_t itr = it + p.K;
  const int32_t n = pooled_block_n(it, p.W, p.K);
  const float gamma = amh_lr_gamma(n, p.a);
  const float macc = p.in.mean_accept_prob[0];
  const float lam = p.in.log_step_size[0];
  const float abar = (float)(ldsum(d + P) / N);
  const float maccn = macc + (abar - macc) / (float)n;
  const float lamn = lam + gamma * (abar - p.target);
  // Sigma' in double, rounded into LDS rows
  {
    const double g = (double)gamma;
    static_for<kQ8>([&](auto Q) {
      const int k = w + 8 * Q;
      const double a = (1.0 - g) * cvo[Q];
      const double b = g * (sv[Q] / N);
      sig[Q] = a + b;
      if (lane < d - k) A[(k + lane) * S + k] = (float)sig[Q];
    });
  }
  if (w < 4) {  // the factoring waves park their write-out operands
    static_for<kQ8>([&](auto Q) {
      park_s[Q][tid] = sig[Q];
      park_c[Q][tid] = cvo[Q];
      park_l[Q][tid] = lvo[Q];
    });
  }
  US(0)
  __syncthreads();
  US(1)
  URT_MAX(3, URT_NOW())
  // (1) the factorisation, column block f = w on waves 0..3, lane = row.
  // Every element receives column k's update for k = 0, 1, .. in order (the
  // oracle's fmaf chain), whichever wave applies it: wave f first applies
  // the finished columns 0 .. 16 f - 1 of the earlier waves as they appear
  // in `cols` (LDS, all 64 kept; `done` counts the finished ones), then
  // factors its own 16 columns.  Column k: pivot (v_readlane), the
  // rsqrt_nr chain (nr_sqrt_div) with column k-1's updates of the block's later
  // columns in its stalls, column k's update of column k + 1 through
  // v_readlane (the next pivot ready), column k to `cols`.  Entries above
  // the diagonal are never operands of valid ones.
  if (w < 4) {
    const int f = w;
    const int c0 = 16 * f;
    int ln = lane;  // opaque: keeps the per-column lane tests from being hoisted
    asm volatile("" : "+v"(ln));
    float a[16];
    static_for<16>([&](auto J) { a[J] = A[ln * S + c0 + J]; });
    // the earlier waves' columns, in order (the wait is bounded: a wave
    // that never sees its column marks the update failed -- the factor is
    // then kept -- rather than hang the GPU; producers never wait, so this
    // does not happen)
    bool stuck = false;
    int spins = 0;
    for (int k = 0; k < c0;) {
      int avail = __hip_atomic_load(&done[0], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
      if (avail <= k) {
        if (++spins > (1 << 22)) {
          stuck = true;
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        continue;
      }
      if (avail > c0) avail = c0;
      for (; k < avail; ++k) {
        const float lr = cols[k][ln];
        f32x4 pv[4];
        static_for<4>([&](auto Q) { pv[Q] = *(const f32x4*)&cols[k][c0 + 4 * Q]; });
        static_for<8>([&](auto J2) {
          constexpr int j = 2 * J2;
          const f32x2v r = __builtin_elementwise_fma(f32x2v{-lr, -lr}, f32x2v{pv[j / 4][j % 4], pv[j / 4][j % 4 + 1]},
                                                     f32x2v{a[j], a[j + 1]});
          a[j] = r[0];
          a[j + 1] = r[1];
        });
      }
    }
    bool ok = true;
    f32x4 pv[4];  // column k-1's entries of this block's rows c0 .. c0 + 15
    float am1 = 0.0f;
    // The pivot chain runs on wave-uniform values: with l1 = L_{k+1,k} =
    // n1 y (n1 = column k's unscaled row k + 1) the next pivot is
    // fmaf(-l1, l1, sa) (sa = row k + 1 of column k + 1 before column k's
    // update) -- the very operations the vector update makes in lane k + 1 --
    // so no v_readlane or LDS round trip sits between two pivots.  A lone wave
    // is issue-bound here (tools/ubench: ~5 ticks per VALU op, dependent or
    // not; ~15 per v_readlane feeding a VALU op; ~9 per v_cmp/v_cndmask), so
    // the column's other work is kept small: at its start column k (unscaled)
    // and column k + 1 go to the wave's two broadcast rows -- n1 and the
    // rows c0 .. c0 + 15 come back from the first, sa from the second, all
    // while the chain runs -- and the rows return scaled as pv = row y (the
    // vector path's q, bit for bit) for the next column's fills.  Column k's
    // updates of columns k + 1 and k + 2 are made right after it (so column
    // k + 1 is final when its turn comes); no select for the diagonal (lane
    // k holds the pivot itself, so its q = piv y is L_kk).
    float pivu = rdlane(a[0], c0);
    asm volatile("" : "+v"(pivu));  // a VGPR value: the seed's integer ops stay on the VALU
    static_for<16>([&](auto J) {
      constexpr int j = J;
      const int k = c0 + j;
      f32x4 pn[4];
      float sa = 0.0f;
      if constexpr (j + 1 < 16) {
        bc[w][0][ln] = a[j];
        bc[w][1][ln] = a[j + 1];
        static_for<4>([&](auto Q) {
          if constexpr (4 * Q + 3 >= j + 1) pn[(int)Q] = *(const f32x4*)&bc[w][0][c0 + 4 * Q];
        });
        sa = bc[w][1][k + 1];
      }
      ok = ok && amh_pivot_ok(pivu);
      float ljj, q, y;
      nr_sqrt_div(pivu, a[j], ljj, q, y, [&](auto Sl) {
        // column k-1's updates of this block's columns m >= k + 2 (packed
        // pairs (m, m + 1), m - c0 even; column k + 2 alone when odd)
        if constexpr (j >= 1) {
          constexpr int m0 = ((j + 2) % 2 == 0) ? j + 2 : j + 3;
          if constexpr (Sl == 0 && m0 != j + 2 && j + 2 < 16) a[j + 2] = fmaf(-am1, pv[(j + 2) / 4][(j + 2) % 4], a[j + 2]);
          constexpr int m = m0 + 2 * Sl;
          if constexpr (m + 1 < 16) {
            const f32x2v r = __builtin_elementwise_fma(f32x2v{-am1, -am1}, f32x2v{pv[m / 4][m % 4], pv[m / 4][m % 4 + 1]},
                                                       f32x2v{a[m], a[m + 1]});
            a[m] = r[0];
            a[m + 1] = r[1];
          }
        }
      });
      a[j] = q;
      cols[k][ln] = q;
      if constexpr (j + 1 < 16) {
        // the whole vectors live to here: an element never used would
        // otherwise have its register reused while the load is in flight,
        // and the wait for it would land inside the chain
        static_for<4>([&](auto Q) {
          if constexpr (4 * Q + 3 >= j + 1) {
            f32x4& pq = pn[(int)Q];  // (a named reference: an asm operand alone is not a capture)
            asm volatile("" : "+v"(pq));
          }
        });
        const float n1 = pn[(j + 1) / 4][(j + 1) % 4];
        const float l1 = n1 * y;
        pivu = fmaf(-l1, l1, sa);
        static_for<4>([&](auto Q) {
          if constexpr (4 * Q + 3 >= j + 2) {  // v_pk_mul_f32 pairs
            const f32x2v lo = f32x2v{pn[(int)Q][0], pn[(int)Q][1]} * f32x2v{y, y};
            const f32x2v hi = f32x2v{pn[(int)Q][2], pn[(int)Q][3]} * f32x2v{y, y};
            pv[(int)Q] = f32x4{lo[0], lo[1], hi[0], hi[1]};
          }
        });
        am1 = q;
        a[j + 1] = fmaf(-q, l1, a[j + 1]);
        if constexpr (j + 2 < 16) a[j + 2] = fmaf(-q, pv[(j + 2) / 4][(j + 2) % 4], a[j + 2]);
      }
      // columns out.  A wave's LDS operations are performed in issue order,
      // so the column's writes above land before this flag; the empty asm
      // keeps the compiler from moving them past it.  Every lane stores (lane
      // 0 to done[0], the word the readers poll): no branch.  Every second
      // column and the block's last.
      if constexpr (j % 2 == 1) {
        asm volatile("" ::: "memory");
        __hip_atomic_store(&done[ln], k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    static_for<16>([&](auto J) {
      if (c0 + (int)J <= ln) A[ln * S + c0 + J] = a[J];
    });
    if ((!ok || stuck) && ln == 0) okv = 0;
    if (stuck && ln == 0 && p.err_flag != nullptr) *p.err_flag = 1;  // reported by the next call
  }
  US(2)
  __syncthreads();
  URT_MAX(4, URT_NOW())
  asm volatile("" ::: "memory");  // the parked values are reloaded, not kept in registers
  if (w < 4) {
    static_for<kQ8>([&](auto Q) {
      sig[Q] = park_s[Q][tid];
      cvo[Q] = park_c[Q][tid];
      lvo[Q] = park_l[Q][tid];
    });
  }
  US(3)
  // (2) write-out and as_change: column k's squared terms (rows k + t) by the
  // 64-lane butterfly, then the columns (pooled_big_post_kernel's order)
  const bool ok = okv != 0;
  const float e0 = amh_expf(lam), e1 = amh_expf(lamn);
  float sq[kQ8];
  static_for<kQ8>([&](auto Q) {
    const int k = w + 8 * Q;
    const int64_t co = col_off(d, k);
    sq[Q] = 0.0f;
    const float lf = A[((k + lane) < d ? k + lane : d - 1) * S + k];
    if (lane < d - k) {
      const int64_t o = co + lane;
      const float lo = lvo[Q];
      const float lnw = ok ? lf : lo;
      const float tt = (lnw * e1) - (lo * e0);
      sq[Q] = tt * tt;
      p.out.cov[o] = ok ? sig[Q] : cvo[Q];
      p.out.scale[o] = lnw;
    }
  });
  static_for<kQ8>([&](auto Q) {  // independent butterflies, interleaved
    const float s0 = Grp<64>::sum(sq[Q]);
    if (lane == 0) colsum[w + 8 * Q] = (s0 + 0.0f) + (0.0f + 0.0f);
  });
  __syncthreads();
  if (w == 0) {
    const float Ssum = Grp<64>::sum(colsum[lane]);
    if (lane == 0) {
      p.out.as_change[0] = sqrtf((Ssum + 0.0f) + (0.0f + 0.0f));
      p.out.i[0] = itr;
      p.out.mean_accept_prob[0] = maccn;
      p.out.log_step_size[0] = lamn;
    }
  }
  if (w == 0) p.out.loc[lane] = loc_in + gamma * (float)(sd_in / N);
  US(4)
  US_FLUSH
#ifdef AMH_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
#endif
  URT_MAX(5, URT_NOW())
  URT_FLUSH
}

// Sigma' = (1-g) Sigma + g S_dd / N rounded to float, in the update's
// 4-row-aligned layout (block k = column k; all CUs)
__global__ __launch_bounds__(256) void pooled_big_prep_kernel(PooledUpdateParams p) {
  const int d = p.d;
  const int k = blockIdx.x;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const double N = p.sums[d + P + 1];
  const int32_t it = p.in.i[0];
  const int32_t n = pooled_block_n(it, p.W, p.K);
  const double g = (double)amh_lr_gamma(n, p.a);
  const int64_t co = col_off(d, k);
  const int ab = a4_base(d, k);
  if (k == 0 && threadIdx.x == 0) ((int*)p.scratch)[d * (d + 4) / 2 + 4] = it + p.K;  // the next step's i (noise blocks)
  for (int rr = threadIdx.x; rr < d - k; rr += 256) {
    const double a = (1.0 - g) * p.in.cov[co + rr];
    const double b = g * (p.sums[d + co + rr] / N);
    p.scratch[ab + k + rr] = (float)(a + b);
  }
}

// out.scale = the new factor (or the kept one), out.cov = Sigma' (or the kept
// one); element-wise, in-place safe (block k = column k; all CUs).  Column
// k's as_change terms t_rk = L'_rk e^lam' - L_rk e^lam (arwmh.py:197) are
// squared and summed over the column's rows r = k + t by the 256-thread
// big_sum order (four 64-lane butterflies, (s0 + s1) + (s2 + s3)); the column
// sums are handed to the block that finishes last, which forms as_change.
// With pack_out (amh_pooled_step_k) the new factor also goes to the next
// step's A-operand copy (pooled_pack_kernel's slots), so that step skips
// its pack launch.
__global__ __launch_bounds__(256) void pooled_big_post_kernel(PooledUpdateParams p) {
  const int d = p.d;
  const int k = blockIdx.x;
  const int t = threadIdx.x;
  const int nA = d * (d + 4) / 2;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  __shared__ float wsum[4];
  // ok flag, gamma, e^lam, e^lam' from the update kernel (p.in may alias
  // p.out, which the update kernel has already advanced)
  const bool ok = ((const int*)p.scratch)[nA] != 0;
  const double g = (double)p.scratch[nA + 1];
  const float e0 = p.scratch[nA + 2], e1 = p.scratch[nA + 3];
  const double N = p.sums[d + P + 1];
  const int64_t co = col_off(d, k);
  const int ab = a4_base(d, k);
  float sq = 0.0f;
  if (t < d - k) {  // d <= 256: one element per thread
    const int64_t o = co + t;
    const float lo = p.in.scale[o];
    const float ln = ok ? p.scratch[ab + k + t] : lo;
    const float tt = (ln * e1) - (lo * e0);
    sq = tt * tt;
    if (ok) {
      const double a = (1.0 - g) * p.in.cov[o];
      const double b = g * (p.sums[d + o] / N);
      p.out.cov[o] = a + b;
      p.out.scale[o] = ln;
    } else {
      p.out.cov[o] = p.in.cov[o];
      p.out.scale[o] = lo;
    }
    if (p.pack_out != nullptr) {  // pooled_pack_kernel's slot of L[r][k], r = k + t
      const int r = k + t, c = k & 31;
      const int T = r >> 5, J = k >> 5;
      const int b = T * (T + 1) / 2 + J;
      const int lane = (r & 31) + 32 * (c & 1);
      p.pack_out[((int64_t)b * 256 + (c >> 3) * 64 + lane) * 4 + ((c & 7) >> 1)] = ln;
    }
  }
  const float ws = Grp<64>::sum(sq);
  if ((t & 63) == 0) wsum[t >> 6] = ws;
  __syncthreads();
  // the column sum goes out write-through (sc1) and the block takes a ticket;
  // the block that takes the last one sums the columns (cross-XCD hand-off:
  // sc1 stores, vmcnt(0), relaxed agent-scope add, acquire + sc1 loads by the
  // last arriver -- cdna_hip_programming.md's write-through counter recipe)
  uint32_t* colsum = (uint32_t*)(p.scratch + nA + 8);
  int* ticket = (int*)p.scratch + nA + 5;
  __shared__ int last;
  if (t == 0) {
    const float cs = (wsum[0] + wsum[1]) + (wsum[2] + wsum[3]);
    __hip_atomic_store(&colsum[k], __float_as_uint(cs), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    last = __hip_atomic_fetch_add(ticket, 1, AMH_TICKET_ORDER, __HIP_MEMORY_SCOPE_AGENT) == d - 1;
  }
  __syncthreads();
  if (!last) return;
  if (AMH_HANDOFF_FENCE) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // sc1 loads below (see update64)
  // as_change = sqrtf(big_sum of the column sums)
  const float v = t < d ? __uint_as_float(__hip_atomic_load(&colsum[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                        : 0.0f;
  const float vs = Grp<64>::sum(v);
  __syncthreads();  // every wave has read wsum above
  if ((t & 63) == 0) wsum[t >> 6] = vs;
  __syncthreads();
  if (t == 0) {
    p.out.as_change[0] = sqrtf((wsum[0] + wsum[1]) + (wsum[2] + wsum[3]));
    __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // for the next launch
  }
}

// --------------------------------------------------------------- launchers --
// chains per chunk of the sums (bit spec): 128 at every d >= 64
int64_t pooled_big_chunks(int64_t C, int d) {
  const int64_t ch = (d == kF) ? kFChunk : kFB;
  return (C + ch - 1) / ch;
}

hipError_t run_pooled_big_stats(const PooledStatsParams& p, float* xprop, float* pep, double* sums, hipStream_t s) {
  const int d = p.d;
  const int64_t V = d + (int64_t)d * (d + 1) / 2 + 2;
  if (d == kF) {  // one launch (+ the reduction) per step
    const int64_t nch = pooled_big_chunks(p.C, d);
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t grid = nch < 2 * (int64_t)cus ? nch : 2 * (int64_t)cus;  // persistent, two per CU
    if (p.k_steps > 1)
      hipLaunchKernelGGL(pooled_fused64_kernel<true>, dim3((unsigned)grid), dim3(256), fused64_lds_bytes(), s, p, nch);
    else
      hipLaunchKernelGGL(pooled_fused64_kernel<false>, dim3((unsigned)grid), dim3(256), fused64_lds_bytes(), s, p, nch);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    (void)V;
    if (p.defer_reduce) return hipSuccess;  // the update launch reduces (run_pooled_big_update)
    return launch_reduce_tiles((const float*)p.partials, nch, pooled_big_tile_V(d), sums, p.accumulate, d, FinalPrep{},
                               s);
  }
  {
    const int nt = d / 32;
    const int64_t nch = pooled_big_chunks(p.C, d);
    float* pack = xprop;  // the caller's scratch: pooled_big_pack_floats(d) floats
    hipError_t e = hipSuccess;
    if (!p.pack_ready) {
      hipLaunchKernelGGL(pooled_pack_kernel, dim3((unsigned)(nt * (nt + 1) / 2 + nt * nt)), dim3(256), 0, s, p.L,
                         p.model.data + d, d, pack);
      e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    const int64_t grid = nch < (int64_t)cus ? nch : (int64_t)cus;
    switch (nt) {
#define AMH_FB(NT_)                                                                                          \
  case NT_:                                                                                                  \
    hipLaunchKernelGGL(pooled_fused_big_kernel<NT_>, dim3((unsigned)grid), dim3(64 * kFBWaves), fused_big_lds_bytes<NT_>(), s, \
                       p, (const float*)pack, nch);                                                          \
    break;
      AMH_FB(3) AMH_FB(4) AMH_FB(5) AMH_FB(6) AMH_FB(7) AMH_FB(8)
#undef AMH_FB
      default:
        return hipErrorInvalidValue;
    }
    e = hipGetLastError();
    if (e != hipSuccess) return e;
    (void)pep;
    // one launch (was pooled_group4_kernel + pooled_final_kernel)
    return launch_reduce_tiles((const float*)p.partials, nch, pooled_big_tile_V(d), sums, p.accumulate, d, p.prep, s);
  }
}

hipError_t run_pooled_big_update(const PooledUpdateParams& p, hipStream_t s, bool sigma_ready) {
  const size_t shm = (size_t)p.d * (p.d + 4) / 2 * sizeof(float);
  hipError_t e = hipSuccess;
  const bool in_block = p.d == 64;  // d = 64: prep and post run inside the update block
  if (!sigma_ready && !in_block) {  // else pooled_final_kernel formed Sigma' already
    hipLaunchKernelGGL(pooled_big_prep_kernel, dim3((unsigned)p.d), dim3(256), 0, s, p);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (p.d == 64) {
    // blocks: the reduce blocks (red_blocks > 0; the last to finish runs the
    // update) or the one update block, then noise blocks up to one per CU
    // when the next step's noise is drawn ahead
    const unsigned head = p.red_blocks > 0 ? (unsigned)p.red_blocks : 1u;
    unsigned nb = head;
    if (p.noise_C > 0 && p.xi != nullptr) {
      int dev = 0, cus = 0;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      nb = (unsigned)cus > head + 1 ? (unsigned)cus : head + 1;
    }
    hipLaunchKernelGGL(pooled_update64_kernel, dim3(nb), dim3(512), 0, s, p);
    return hipGetLastError();
  }
  unsigned nblk = 1;  // + one noise block per other CU when the next step's noise is drawn ahead
  if (p.noise_C > 0 && p.xi != nullptr) {
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    nblk = (unsigned)(cus > 1 ? cus : 2);
  }
  switch (p.d / 32) {
#define AMH_UPD(NT_)                                                                                    \
  case NT_:                                                                                            \
    hipLaunchKernelGGL(pooled_big_update_kernel<NT_>, dim3(nblk), dim3(64 * kUpdWaves), shm, s, p);    \
    break;
    AMH_UPD(2) AMH_UPD(3) AMH_UPD(4) AMH_UPD(5) AMH_UPD(6) AMH_UPD(7) AMH_UPD(8)
#undef AMH_UPD
    default:
      return hipErrorInvalidValue;
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (in_block) return hipSuccess;
  hipLaunchKernelGGL(pooled_big_post_kernel, dim3((unsigned)p.d), dim3(256), 0, s, p);
  return hipGetLastError();
}

}  // namespace amh
