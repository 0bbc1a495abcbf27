// amh_split.hip -- the split transition for data-heavy models (diamonds).
//
// The fused step kernel evaluates the potential with the chain's lane group
// (lane r sums rows n = r, r+G, ...), so every chain streams the whole data
// set (diamonds: N x Kc = 5000 x 24 floats, 480 KB) through the cache per
// step: 262,144 chains move 126 GB of L2 traffic per transition.  Here one
// transition is three launches:
//
//   propose_kernel      z' = z + (L e^lam + eps I) xi   (arwmh.py:162-167)
//   *_pot_lane_kernel   U(z'), ONE LANE PER CHAIN: the data rows arrive as
//                       wave-uniform scalar loads shared by 64 chains, the
//                       chain's coefficients sit in the lane's registers
//                       (run_diamonds_lr_decay.py:24-40)
//   step kernel (ExtPotM) accept / adaptation with U(z') read from memory
//                       (arwmh.py:168-207), recomputing z' in registers
//
// Bit spec: the proposal is the step kernel's expression, evaluated in the
// same order (so the step kernel's recomputed z' is the one evaluated here),
// and the lane kernel keeps the group kernel's summation order -- 32 partial
// sums over rows n = r (mod 32), each in row order, then the group's xor
// butterfly (oracle: pot_diamonds, group_sum).  The split path is therefore
// bit-identical to the fused one (tests/test_gpu_parity.py).
#include "amh_device.h"

namespace amh {

bool split_model(int model_id, int d) { return model_id == AMH_MODEL_DIAMONDS && d >= 3 && d <= 32; }

// ---------------------------------------------------------------- propose --
// Lane group of G = 32 per chain, lane r = row r; the factor is read straight
// from HBM (each column of a chain is one coalesced access).  U_rj and the
// four partial sums follow arwmh_step_kernel exactly.
template <int G, int DFIX = 0>
__global__ __launch_bounds__(kBlock) void propose_kernel(StepParams p, float* __restrict__ xprop) {
  using Gp = Grp<G>;
  const int d = DFIX > 0 ? DFIX : p.d;
  const int64_t C = p.C;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const int64_t n_items = (C + Geo<G>::CPW - 1) / Geo<G>::CPW;
  const int64_t wave0 = (int64_t)blockIdx.x * (kBlock / 64) + threadIdx.x / 64;
  const int64_t wstride = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t item = wave0; item < n_items; item += wstride) {
    // lane-dependent values from an opaque lane id inside the loop, so the
    // per-column load offsets are not hoisted out of it (VGPR pressure)
    int lane = lane_id();
    asm volatile("" : "+v"(lane));
    const int r = lane & (G - 1);
    const bool act = r < d;
    const int64_t chain = item * Geo<G>::CPW + lane / G;
    const bool chain_ok = chain < C;
    const int64_t cl = chain_ok ? chain : C - 1;
    // The item's factors through one buffer descriptor (wave-uniform base,
    // range = the item's chains): every column load is unconditional, lanes
    // above the diagonal and chains past C read 0 out of range, so all the
    // loads are in flight together (per-lane conditional loads were issued
    // one round trip at a time).
    const int64_t first = item * Geo<G>::CPW;
    const int64_t nvalid = (C - first) < Geo<G>::CPW ? (C - first) : Geo<G>::CPW;
    const Buf Lb(uniform_ptr(p.in.scale + first * P), (uint32_t)(nvalid * P) * 4u);
    const int g = lane / G;
    const uint32_t vrow = act ? ((uint32_t)g * (uint32_t)P + (uint32_t)r) * 4u : kOOB;
    const float dl = Lb.ld(act ? ((uint32_t)g * (uint32_t)P + (uint32_t)col_off(d, r)) * 4u : kOOB, 0);
    float U[G];
    static_for<G>([&](auto J) {
      constexpr int j = J;
      U[j] = (j < d) ? Lb.ld(off_from<G, j>(vrow, kOOB, r), (uint32_t)(col_off(d, j) - j) * 4u) : 0.0f;
    });
    const int32_t it = p.in.i[cl];
    const uint32_t k0 = p.in.rng_key[2 * cl], k1 = p.in.rng_key[2 * cl + 1];
    const float zr = p.in.z[cl * d + (act ? r : 0)];
    const float z = act ? zr : 0.0f;
    const float lam = p.in.log_step_size[cl];
    const float inv = (amh_isfinite(dl) && dl != 0.0f) ? 1.0f / dl : 0.0f;
    static_for<G>([&](auto J) {
      constexpr int j = J;
      if (j < d) {
        const float ij = Gp::template bcast<j>(inv);
        U[j] = (r == j) ? 1.0f : ((r > j) ? U[j] * ij : 0.0f);
      }
    });
    float xi, u_unused;
    step_noise<G>(r, d, (uint32_t)it, k0, k1, xi, u_unused);  // (bit spec: amh_step_word)
    xi = act ? xi : 0.0f;
    const float el = amh_expf(lam);
    const float eta = dl * xi;
    float a4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    static_for<G>([&](auto J) {
      if (J < d) a4[J & 3] = fmaf(U[J], Gp::template bcast<J>(eta), a4[J & 3]);
    });
    const float acc = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    const float zp = act ? z + fmaf(el, acc, p.eps * xi) : 0.0f;
    if (chain_ok && act) xprop[chain * d + r] = zp;
  }
}

// ------------------------------------------------ diamonds, lane per chain --
// xor butterfly of the G = 32 group (Grp<32>::sum / oracle group_sum) on 32
// values held by one lane
__device__ __forceinline__ float butterfly32(float (&x)[32]) {
  static_for<5>([&](auto S) {
    constexpr int off = 1 << S;
    float y[32];
    static_for<32>([&](auto R) { y[R] = x[R] + x[R ^ off]; });
    static_for<32>([&](auto R) { x[R] = y[R]; });
  });
  return x[0];
}

typedef __attribute__((address_space(4))) const float cfloat;

// z = [Intercept, b (Kc), log sigma]; data = [Xc (N x Kc) | Y (N)].  KC > 0:
// compile-time Kc (the reference data set: K = 25); KC == 0: any Kc <= 30.
//
// A block of 4 waves serves 128 chains: lane l holds chains 128 * block + l
// and + 64 side by side, so one v_pk_fma_f32 with the row's Xc entry as a
// broadcast scalar operand (op_sel) advances both chains' fmaf chains, and
// every scalar load of the data feeds 128 chains.  The 32 partial sums of
// the bit spec are independent FMA chains (rows n = r mod 32, each in row
// order), so wave w owns residues r in [8w, 8w + 8) and reads only those
// rows (the scalar-load latency of one row is hidden by the other waves of
// the SIMD) at unchanged bits.  The partials then meet in LDS, and waves 0
// and 1 finish the block's first and second 64 chains.
constexpr int kDiaWaves = 4;
constexpr int kDiaRes = 32 / kDiaWaves;  // residues per wave

template <int KC>
__global__ __launch_bounds__(64 * kDiaWaves) void diamonds_pot_lane_kernel(PotParams p) {
  constexpr int KMAX = KC > 0 ? KC : 30;
  __shared__ float pl[32][128];
  const int Kc = KC > 0 ? KC : (int)p.model.k - 1;
  const int d = p.d;
  const int64_t N = p.model.n;
  const int64_t n_ch = p.n;
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  const int64_t c0 = (int64_t)blockIdx.x * 128 + lane;
  const float* z0 = p.z + (c0 < n_ch ? c0 : n_ch - 1) * d;
  const float* z1 = p.z + (c0 + 64 < n_ch ? c0 + 64 : n_ch - 1) * d;
  f32x2v b2[KMAX];
  static_for<KMAX>([&](auto K) { b2[K] = (K < Kc) ? f32x2v{z0[1 + K], z1[1 + K]} : f32x2v{0.0f, 0.0f}; });
  const f32x2v icpt2 = {z0[0], z1[0]};
  const f32x2v ls2 = {z0[Kc + 1], z1[Kc + 1]};
  const f32x2v sg2 = {amh_expf(ls2[0]), amh_expf(ls2[1])};
  const f32x2v isg2 = {1.0f / sg2[0], 1.0f / sg2[1]};
  const cfloat* X = (const cfloat*)p.model.data;
  const cfloat* Y = X + N * Kc;
  f32x2v part2[kDiaRes];
  static_for<kDiaRes>([&](auto Q) { part2[Q] = f32x2v{0.0f, 0.0f}; });
  auto row = [&](const float (&xr)[KMAX], float yn, f32x2v& acc) {
    f32x2v mu = {0.0f, 0.0f};
    static_for<KMAX>([&](auto K) {
      if (K < Kc) mu = __builtin_elementwise_fma(f32x2v{xr[K], xr[K]}, b2[K], mu);
    });
    const f32x2v e = (f32x2v{yn, yn} - (icpt2 + mu)) * isg2;
    acc = __builtin_elementwise_fma(e, e, acc);
  };
  auto load = [&](int64_t n, float (&xr)[KMAX], float& yn) {
    static_for<KMAX>([&](auto K) { xr[K] = (K < Kc) ? X[n * Kc + K] : 0.0f; });
    yn = Y[n];
  };
  // whole blocks of 32 rows: the next row's scalar loads are issued before
  // this row's FMAs
  const int64_t Mfull = N / 32;
  const int64_t r0 = kDiaRes * w;
  if (Mfull > 0) {
    float cur[KMAX], ycur;
    load(r0, cur, ycur);
    for (int64_t m = 0; m < Mfull; ++m) {
      static_for<kDiaRes>([&](auto Q) {
        float nxt[KMAX], ynxt;
        int64_t nn;
        if constexpr (Q + 1 < kDiaRes) {
          nn = 32 * m + r0 + Q + 1;
        } else {
          nn = (m + 1 < Mfull) ? 32 * (m + 1) + r0 : 32 * m + r0 + Q;
        }
        load(nn, nxt, ynxt);
        row(cur, ycur, part2[Q]);
        static_for<KMAX>([&](auto K) { cur[K] = nxt[K]; });
        ycur = ynxt;
      });
    }
  }
  static_for<kDiaRes>([&](auto Q) {  // ragged tail: rows 32 Mfull .. N-1
    const int64_t n = 32 * Mfull + r0 + Q;
    if (n < N) {
      float xr[KMAX], yn;
      load(n, xr, yn);
      row(xr, yn, part2[Q]);
    }
  });
  static_for<kDiaRes>([&](auto Q) {
    pl[r0 + Q][lane] = part2[Q][0];
    pl[r0 + Q][64 + lane] = part2[Q][1];
  });
  __syncthreads();
  if (w >= 2) return;
  const int h = w;  // this wave finishes chain c0 + 64 h
  const int64_t c = c0 + 64 * h;
  float all[32];
  static_for<32>([&](auto R) { all[R] = pl[R][64 * h + lane]; });
  const float S = butterfly32(all);
  float bb[32];  // group lane r holds coordinate r: b_{r-1}^2 for 1 <= r <= Kc
  static_for<32>([&](auto R) {
    constexpr int r = R;
    if constexpr (r >= 1 && r - 1 < KMAX) {
      const float br = h ? b2[r - 1][1] : b2[r - 1][0];
      bb[r] = (r <= Kc) ? br * br : 0.0f;
    } else {
      bb[r] = 0.0f;
    }
  });
  const float B = butterfly32(bb);
  const float icpt = h ? icpt2[1] : icpt2[0];
  const float ls = h ? ls2[1] : ls2[0];
  const float sg = h ? sg2[1] : sg2[0];
  const float cst = -3.30347394261755545f;
  const float ll = fmaf(-0.5f, S, (float)N * ((-ls) - HALF_LOG_2PI));
  const float lpb = fmaf(-0.5f, B, -(float)Kc * HALF_LOG_2PI);
  const float lpi = lp_student3(icpt, 8.0f, 10.0f, cst);
  const float lps = (0.693147181f + lp_student3(sg, 0.0f, 10.0f, cst)) + ls;
  if (c < n_ch) p.pe[c] = -(((ll + lpb) + lpi) + lps);
}

// --------------------------------------------------- diamonds on MFMA --
// mu = Xc b for 32 rows x 32 chains per v_mfma_f32_32x32x2_f32 accumulation
// (A = a 32-row tile of Xc, B = the chains' coefficients; KC/2 MFMAs over k
// in order from 0 -- per element the fmaf chain of the bit spec, so the bits
// equal the lane kernel's).  Accumulator register R of lane (i, h) holds row
// 32 m + (R&3) + 8 (R>>2) + 4 h of chain i: the residue of the bit spec's 32
// partial sums is fixed per register, and the tiles arrive in row order, so
// part[R] = fmaf(e, e, part[R]) keeps every residue's row order.  Xc and Y
// are read from a per-model tile copy in A-operand / register order
// (diamonds_pack_kernel, made when the model is bound).  A wave serves 64
// chains (two B tiles sharing each A tile); rows past N add nothing.
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int KC>
struct DiaMfma {
  static constexpr int S = (KC + 1) / 2;   // MFMA k steps per tile
  static constexpr int G = (S + 3) / 4;    // 16-B A vectors per lane per tile
  static constexpr int64_t tiles(int64_t N) { return (N + 31) / 32; }
  static constexpr int64_t floats(int64_t N) { return tiles(N) * (G * 256 + 32); }
};

template <int KC>
__global__ __launch_bounds__(256) void diamonds_pack_kernel(const float* __restrict__ data, int64_t N,
                                                            float* __restrict__ xp) {
  using T = DiaMfma<KC>;
  const int64_t m = blockIdx.x;
  const int t = threadIdx.x;
  const float* X = data;
  const float* Y = data + N * KC;
  if (t < T::G * 64) {
    const int g = t >> 6, lane = t & 63, i = lane & 31, h = lane >> 5;
    const int64_t row = 32 * m + i;
    f32x4 v;
    static_for<4>([&](auto E) {
      const int k = 2 * (4 * g + E) + h;
      v[(int)E] = (row < N && k < KC) ? X[row * KC + k] : 0.0f;
    });
    ((f32x4*)xp)[(m * T::G + g) * 64 + lane] = v;
  } else if (t < T::G * 64 + 32) {
    const int q = t - T::G * 64, h = q >> 4, R = q & 15;
    const int64_t row = 32 * m + (R & 3) + 8 * (R >> 2) + 4 * h;
    xp[T::tiles(N) * T::G * 256 + 32 * m + q] = row < N ? Y[row] : 0.0f;
  }
}

// NB B tiles (32 chains each) per wave share every A tile.  NB = 4 halves
// the A / Y operand loads per chain and doubles the wave's independent MFMA
// chains, but at two waves per SIMD instead of three it was slower: 0.995
// against 0.956 ms per transition (tools/gpu_ab_dia.sh, r5x).  (This form of
// the NB = 2 kernel keeps its per-chain operands in registers where the
// previous one moved 30 dwords through scratch in every tile: 0.976 -> 0.956.)
constexpr int kDiaNB = 2;
template <int KC, int NB>
__global__ __launch_bounds__(256, (NB == 2 ? 2 : 1)) void diamonds_pot_mfma_kernel(PotParams p) {
  using T = DiaMfma<KC>;
  constexpr int S = T::S, G = T::G;
  const int d = p.d;
  const int64_t N = p.model.n;
  const int64_t NT = T::tiles(N);
  const int64_t n_ch = p.n;
  const int lane = lane_id();
  const int i = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  const int64_t cb = ((int64_t)blockIdx.x * 4 + w) * (32 * NB);
  int64_t cq[NB];
  const float* zq[NB];
  float B[NB][S];
  float icq[NB], isq[NB];
  static_for<NB>([&](auto J) {
    cq[J] = cb + 32 * J + i;
    zq[J] = p.z + (cq[J] < n_ch ? cq[J] : n_ch - 1) * d;
    static_for<S>([&](auto Q) {
      const int k = 2 * Q + h;
      B[J][Q] = k < KC ? zq[J][1 + k] : 0.0f;
    });
    icq[J] = zq[J][0];
    isq[J] = 1.0f / amh_expf(zq[J][KC + 1]);
  });
  const f32x4* xa = (const f32x4*)p.xpack + lane;
  const f32x4* ya = (const f32x4*)(p.xpack + NT * G * 256) + 4 * h;
  float part[NB][16];
  static_for<NB>([&](auto J) { static_for<16>([&](auto R) { part[J][R] = 0.0f; }); });
  f32x4 a[G], y[4];
  static_for<G>([&](auto Q) { a[Q] = xa[64 * Q]; });
  static_for<4>([&](auto Q) { y[Q] = ya[Q]; });
  // one tile: KC/2 MFMA steps for each B tile, then the residues; FULL: every
  // row exists (all tiles but the last: no per-register row test)
  auto tile = [&](int64_t m, auto FULL) {
    f32x4 an[G], yn[4];
    const int64_t mn = (m + 1 < NT) ? m + 1 : m;  // next tile's loads in flight during this one
    static_for<G>([&](auto Q) { an[Q] = xa[(mn * G + Q) * 64]; });
    static_for<4>([&](auto Q) { yn[Q] = ya[8 * mn + Q]; });
    f32x16 acc[NB];
    static_for<NB>([&](auto J) { acc[J] = f32x16{}; });
    static_for<S>([&](auto Q) {
      const float av = a[Q / 4][Q % 4];
      static_for<NB>([&](auto J) { acc[J] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, B[J][Q], acc[J], 0, 0, 0); });
    });
    const int64_t nrem = N - 32 * m;  // rows of this tile that exist
    static_for<16>([&](auto R) {
      const int rr = (R & 3) + 8 * (R >> 2) + 4 * h;
      const float yv = y[R / 4][R % 4];
      static_for<NB>([&](auto J) {
        const float e = (yv - (icq[J] + acc[J][(int)R])) * isq[J];
        if constexpr (decltype(FULL)::value) {
          part[J][R] = fmaf(e, e, part[J][R]);
        } else {
          const bool ok = rr < nrem;
          part[J][R] = ok ? fmaf(e, e, part[J][R]) : part[J][R];
        }
      });
    });
    static_for<G>([&](auto Q) { a[Q] = an[Q]; });
    static_for<4>([&](auto Q) { y[Q] = yn[Q]; });
  };
#ifdef AMH_DIA_SELECT_ALL
#pragma unroll 1
  for (int64_t m = 0; m < NT; ++m) tile(m, std::false_type{});
#else
#pragma unroll 1
  for (int64_t m = 0; m + 1 < NT; ++m) tile(m, std::true_type{});
  if (NT > 0) tile(NT - 1, std::false_type{});
#endif
  // chain pair (2P, 2P + 1): lane (i, 0) finishes chain 2P, lane (i, 1) chain
  // 2P + 1; the other half's residues arrive by a 32-lane swap
  static_for<NB / 2>([&](auto PP) {
    constexpr int P0 = 2 * PP, P1 = 2 * PP + 1;
    float all[32];
    static_for<16>([&](auto R) {
      const float mine = h ? part[P1][R] : part[P0][R];
      const float other = __shfl_xor(h ? part[P0][R] : part[P1][R], 32, 64);
      const int rm = (R & 3) + 8 * (R >> 2);
      if (h == 0) {
        all[rm] = mine;
        all[rm + 4] = other;
      } else {
        all[rm + 4] = mine;
        all[rm] = other;
      }
    });
    const float Ssum = butterfly32(all);
    const int64_t c = h ? cq[P1] : cq[P0];
    const float* zc = h ? zq[P1] : zq[P0];
    float bb[32];
    static_for<32>([&](auto R) {
      constexpr int r = R;
      if constexpr (r >= 1 && r <= KC) {
        const float br = zc[r];
        bb[r] = br * br;
      } else {
        bb[r] = 0.0f;
      }
    });
    const float Bsum = butterfly32(bb);
    const float icpt = zc[0];
    const float ls = zc[KC + 1];
    const float sg = amh_expf(ls);
    const float cst = -3.30347394261755545f;
    const float ll = fmaf(-0.5f, Ssum, (float)N * ((-ls) - HALF_LOG_2PI));
    const float lpb = fmaf(-0.5f, Bsum, -(float)KC * HALF_LOG_2PI);
    const float lpi = lp_student3(icpt, 8.0f, 10.0f, cst);
    const float lps = (0.693147181f + lp_student3(sg, 0.0f, 10.0f, cst)) + ls;
    if (c < n_ch) p.pe[c] = -(((ll + lpb) + lpi) + lps);
  });
}

int64_t diamonds_pack_floats(int64_t N, int64_t K) {
  return (K - 1 == kDiaMfmaKc) ? DiaMfma<kDiaMfmaKc>::floats(N) : 0;
}

hipError_t run_diamonds_pack(const ModelArgs& m, float* xp, hipStream_t s) {
  if (m.k - 1 != kDiaMfmaKc || m.n < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(diamonds_pack_kernel<kDiaMfmaKc>, dim3((unsigned)DiaMfma<kDiaMfmaKc>::tiles(m.n)), dim3(256), 0,
                     s, m.data, m.n, xp);
  return hipGetLastError();
}

// ---------------------------------------------------------------- launchers --
hipError_t run_propose(const StepParams& p, float* xprop, hipStream_t s) {
  if (p.d < 1 || p.d > 64) return hipErrorInvalidValue;
  if (p.d > 32) {  // the external potential's 33 <= d <= 64: one chain per wave
    int64_t blocks = (p.C + kBlock / 64 - 1) / (kBlock / 64);
    if (blocks > 256 * 32) blocks = 256 * 32;
    hipLaunchKernelGGL(propose_kernel<64>, dim3((unsigned)(blocks > 0 ? blocks : 1)), dim3(kBlock), 0, s, p, xprop);
    return hipGetLastError();
  }
  const int64_t n_items = (p.C + Geo<32>::CPW - 1) / Geo<32>::CPW;
  int64_t blocks = (n_items + kBlock / 64 - 1) / (kBlock / 64);
  if (blocks > 256 * 32) blocks = 256 * 32;
  if (p.d == kDiamondsD) {
    hipLaunchKernelGGL((propose_kernel<32, kDiamondsD>), dim3((unsigned)(blocks > 0 ? blocks : 1)), dim3(kBlock), 0, s,
                       p, xprop);
  } else {
    hipLaunchKernelGGL(propose_kernel<32>, dim3((unsigned)(blocks > 0 ? blocks : 1)), dim3(kBlock), 0, s, p, xprop);
  }
  return hipGetLastError();
}

hipError_t run_potential_lane(int model_id, const PotParams& p, hipStream_t s) {
  if (!split_model(model_id, p.d)) return hipErrorInvalidValue;
  if (p.xpack != nullptr && p.model.k - 1 == kDiaMfmaKc && p.d == kDiaMfmaKc + 2) {
    constexpr int per_block = 4 * 32 * kDiaNB;
    hipLaunchKernelGGL((diamonds_pot_mfma_kernel<kDiaMfmaKc, kDiaNB>), dim3((unsigned)((p.n + per_block - 1) / per_block)),
                       dim3(256), 0, s, p);
    return hipGetLastError();
  }
  const int64_t blocks = (p.n + 127) / 128;
  if (p.model.k - 1 == 24) {
    hipLaunchKernelGGL(diamonds_pot_lane_kernel<24>, dim3((unsigned)blocks), dim3(64 * kDiaWaves), 0, s, p);
  } else {
    hipLaunchKernelGGL(diamonds_pot_lane_kernel<0>, dim3((unsigned)blocks), dim3(64 * kDiaWaves), 0, s, p);
  }
  return hipGetLastError();
}

}  // namespace amh
