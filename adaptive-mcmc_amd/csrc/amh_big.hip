// amh_big.hip -- ARWMH for large dimensions (64 < d <= 256, dense Gaussian
// potential; BASELINE config 4: d = 256, kappa = 1e4).
//
// At d = 256 a chain's packed factor is 131.6 KB: it cannot live in one
// wave's registers, and the dense precision (256 KB) cannot sit in LDS next
// to anything else.  One transition is therefore three launches:
//
//   big_propose_kernel   one wave per chain, lane l owns rows 64 s + l.  One
//                        pass over the factor in column order computes the
//                        proposal z' = z + (L e^lam + eps I) xi (arwmh.py:
//                        166-167) and, because row r's proposal is complete
//                        once column r has passed, BOTH forward solves of the
//                        rank-one update (w = U^-1 delta for the accepted and
//                        for the rejected delta) in the same pass.
//   gauss_pot_mfma_kernel U(z') for 64 chains per block on MFMA
//                        (v_mfma_f32_32x32x2_f32: Y = P D, D = z' - m; the
//                        f32 MFMA is a k-ordered fmaf chain, so the oracle
//                        can mirror it bit for bit).  Shared by init and
//                        amh_potential.
//   big_step_kernel      one wave per chain: accept (arwmh.py:173-178), the
//                        schedule and mean / step-size updates (:180-193) and
//                        the second pass over the factor, which applies the
//                        rank-one update column by column and streams L' out
//                        (cholesky_update at :190, keep-L rule at :191).
//
// The factor is read twice and written once per transition (the algorithmic
// count is one read and one write); the passes stream it with coalesced
// column accesses and keep nothing but O(d) per chain on chip.
// Bit spec: oracle/amh_oracle.c, "large dimensions".
#include "amh_device.h"

namespace amh {

namespace {

constexpr int kNSMAX = 4;  // row slots per lane: d <= 64 * NS, NS = 2 (d <= 128) or 4
constexpr int kAsssBigMaxIter = 50;  // asss.py:59 max_iterations
#ifndef AMH_ABL_NOPASSD
#define AMH_ABL_NOPASSD 0
#endif

__device__ __forceinline__ float rdl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// gamma_n (scalar cache table, as the step kernel)
__device__ __forceinline__ float big_gamma(const BigParams& p, int32_t n) {
  typedef __attribute__((address_space(4))) const float cf;
  const cf* tab = (const cf*)p.gamma_tab;
  return (n < p.gamma_tab_n) ? tab[n] : amh_lr_gamma(n, p.a);
}

// sum over rows: 64-lane butterfly per slot, then (s0 + s1) + (s2 + s3)
// (NS = 2: s2 = s3 = +0, added as such -- the bits of the four-slot form)
template <int NS>
__device__ __forceinline__ float big_sum(const float (&v)[NS]) {
  float s[kNSMAX];
  static_for<kNSMAX>([&](auto K) {
    if constexpr (K < NS) {
      s[K] = Grp<64>::sum(v[K]);
    } else {
      s[K] = 0.0f;
    }
  });
  return (s[0] + s[1]) + (s[2] + s[3]);
}

typedef __attribute__((address_space(3))) void lds_void_t;

// Column stream of one chain's packed factor (column-major, column j at
// col_off(d, j)): blocks of 8 columns are contiguous in HBM (and 16-B aligned
// for d % 8 == 0: col_off(d, 8b) and d (d + 1) / 2 are multiples of 4), so
// each block is one bulk LDS-DMA of dwordx4 pieces -- dword pieces for other
// d -- into the wave's double buffer while the previous block is consumed; a
// ragged last block holds d % 8 columns.  LDS reads
// go through asm (lds_ld1) so the compiler's wait-count pass does not drain
// the in-flight DMA before them (see amh_device.h).
constexpr int kColBlk = 8;

template <bool RAG>
__device__ __forceinline__ void issue_block(const float* Lc, int d, int64_t P, int b, float* wbuf, int lane) {
  const int j0 = kColBlk * b;
  const int j1 = j0 + kColBlk;
  const int64_t o0 = col_off(d, j0);
  const int64_t o1 = (j1 < d) ? col_off(d, j1) : P;
  const uint32_t bytes = (uint32_t)(o1 - o0) * 4u;
  const Buf rb(uniform_ptr(Lc + o0), bytes);
  if constexpr (!RAG) {
    for (uint32_t o = 0; o < bytes; o += 1024u) {
      if (o + 16u * (uint32_t)lane < bytes)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb.rs, (lds_void_t*)(wbuf + o / 4u), 16, (int)(o + 16u * lane), 0, 0, 0);
    }
  } else {
    for (uint32_t o = 0; o < bytes; o += 256u) {
      if (o + 4u * (uint32_t)lane < bytes)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb.rs, (lds_void_t*)(wbuf + o / 4u), 4, (int)(o + 4u * lane), 0, 0, 0);
    }
  }
}

// f(KB, j, v) for every column j in order, v[K] = L_rj for rows r = 64 K + l
// (only rows j < r < d are meaningful; the diagonal L_jj is v[j / 64] of
// lane j % 64).  KB = j / 64 is a compile-time slot index.
template <bool RAG, int NS, class F>
__device__ __forceinline__ void for_columns(const float* Lc, int d, int64_t P, float* wb0, float* wb1, int lane,
                                            F&& f) {
  const int nb = (d + kColBlk - 1) / kColBlk;
  issue_block<RAG>(Lc, d, P, 0, wb0, lane);
  static_for<NS>([&](auto KB) {
    constexpr int kb = KB;
    if (64 * kb < d) {
      for (int bb = 0; bb < 64 / kColBlk; ++bb) {
        const int b = (64 / kColBlk) * kb + bb;
        if (b >= nb) break;
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): block b has landed
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): reads of the other buffer done
        float* cur = (b & 1) ? wb1 : wb0;
        if (b + 1 < nb) issue_block<RAG>(Lc, d, P, b + 1, (b & 1) ? wb0 : wb1, lane);
        const int64_t ob = col_off(d, kColBlk * b);
        // element (r, j) sits at cur[col_off(d, j) - ob + r - j]; column q + 1's
        // reads are issued before f runs on column q (one LDS round trip off
        // each column but the block's first)
        auto rd = [&](int q, float (&v)[NS]) {
          const int j = kColBlk * b + q;
          const uint32_t a0 = lds_addr(cur) + 4u * (uint32_t)(col_off(d, j) - ob - j + lane);
          static_for<NS>([&](auto K) {
            if constexpr (K >= kb) {
              v[K] = lds_ld1<0>(a0 + 256u * K);
            } else {
              v[K] = 0.0f;
            }
          });
        };
        // (the wait sits at the end of the iteration, so no loop-carried
        // register is copied while its read is in flight)
        float vn[NS];
        rd(0, vn);
        if constexpr (NS == 3) { lds_wait(vn[0], vn[1], vn[2]); } else { lds_wait_n(vn); }
        // RAG (d % 8 != 0): a run-time column count for the ragged last
        // block; the aligned instantiation keeps the compile-time trip count
        // (a run-time bound in it cost 12-17 % at d = 256)
        const int qn = RAG ? ((d - kColBlk * b) < kColBlk ? (d - kColBlk * b) : kColBlk) : kColBlk;
        for (int q = 0; q < qn; ++q) {
          float v[NS];
          static_for<NS>([&](auto K) { v[K] = vn[K]; });
#if AMH_BIG_NOPIPE
          f(KB, kColBlk * b + q, v);
          if (q + 1 < qn) rd(q + 1, vn);
#else
          if (q + 1 < qn) rd(q + 1, vn);
          f(KB, kColBlk * b + q, v);
#endif
          if constexpr (NS == 3) { lds_wait(vn[0], vn[1], vn[2]); } else { lds_wait_n(vn); }
        }
      }
    }
  });
}

}  // namespace

// --------------------------------------------------------------- init ----
// arwmh.py:84-138 (init_to_uniform), one wave per chain; pe0 is filled by
// the MFMA potential afterwards.
template <int NS>
__global__ __launch_bounds__(256) void big_init_kernel(InitParams p) {
  const int d = p.d;
  const int lane = lane_id();
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t c = (int64_t)blockIdx.x * 4 + threadIdx.x / 64; c < p.C; c += nw) {
    const uint64_t gc = (uint64_t)(p.chain_offset + c);
    const amh_u32x4 kk = amh_philox4x32_10((uint32_t)gc, (uint32_t)(gc >> 32), 0u, AMH_TAG_CHAINKEY, p.key0, p.key1);
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      if (r < d) {
        float z0;
        if (p.init_z != nullptr) {
          z0 = p.init_z[c * d + r];
        } else {
          const amh_u32x4 o = amh_philox4x32_10((uint32_t)r, 0u, 0u, AMH_TAG_INIT, kk.v[0], kk.v[1]);
          const float v = (amh_unif01_from_bits(o.v[0]) * 4.0f) + (-2.0f);
          z0 = (v < -2.0f) ? -2.0f : v;
        }
        p.out.z[c * d + r] = z0;
        p.out.loc[c * d + r] = z0;
      }
    });
    float* Lc = p.out.scale + c * P;
    for (int j = 0; j < d; ++j) {
      static_for<NS>([&](auto K) {
        const int r = 64 * K + lane;
        if (r >= j && r < d) Lc[col_off(d, j) + (r - j)] = (r == j) ? 1.0f : 0.0f;
      });
    }
    if (lane == 0) {
      p.out.i[c] = 0;
      p.out.potential_energy[c] = 0.0f;
      p.out.mean_accept_prob[c] = 0.0f;
      p.out.log_step_size[c] = 0.0f;
      p.out.as_change[c] = 0.0f;
      p.out.rng_key[2 * c] = kk.v[0];
      p.out.rng_key[2 * c + 1] = kk.v[1];
    }
  }
}

// ------------------------------------------------------------- propose ----
template <bool RAG, int NS>
__global__ __launch_bounds__(256) void big_propose_kernel(BigParams p) {
  extern __shared__ float lds_big[];
  const int d = p.d;
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  float* wb0 = lds_big + (size_t)wv * 2 * kColBlk * d;
  float* wb1 = wb0 + kColBlk * d;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t c = (int64_t)blockIdx.x * 4 + threadIdx.x / 64; c < p.C; c += nw) {
    const float* Lc = p.in.scale + c * P;
    const int32_t it = p.in.i[c];
    const uint32_t k0 = p.in.rng_key[2 * c], k1 = p.in.rng_key[2 * c + 1];
    const float el = amh_expf(p.in.log_step_size[c]);
    float inv[NS], xi[NS], eta[NS], zz[NS], mu[NS], acc[NS], sa[NS], sr[NS], zp[NS], wa[NS], wr[NS];
    float pdl[NS];
    step_noise_rows<NS>(lane, d, (uint32_t)it, k0, k1, xi);  // bit spec: amh_step_word
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      const bool act = r < d;
      const float dl = act ? Lc[col_off(d, act ? r : 0)] : 0.0f;
      pdl[K] = dl;
      inv[K] = (amh_isfinite(dl) && dl != 0.0f) ? 1.0f / dl : 0.0f;
      eta[K] = dl * xi[K];
      zz[K] = act ? p.in.z[c * d + r] : 0.0f;
      mu[K] = act ? p.in.loc[c * d + r] : 0.0f;
      acc[K] = sa[K] = sr[K] = zp[K] = wa[K] = wr[K] = 0.0f;
    });
    for_columns<RAG, NS>(Lc, d, P, wb0, wb1, lane, [&](auto KB, int j, const float (&v)[NS]) {
      constexpr int kb = KB;
      const int jl = j - 64 * kb;
      const float etaj = rdl(eta[kb], jl);
      const float invj = rdl(inv[kb], jl);
      // row j completes its proposal and both solves at its own column
      if (lane == jl) {
        acc[kb] = fmaf(1.0f, etaj, acc[kb]);
        zp[kb] = zz[kb] + fmaf(el, acc[kb], p.eps * xi[kb]);
        wa[kb] = (zp[kb] - mu[kb]) - sa[kb];
        wr[kb] = (zz[kb] - mu[kb]) - sr[kb];
      }
      const float waj = rdl(wa[kb], jl);
      const float wrj = rdl(wr[kb], jl);
      static_for<NS>([&](auto K) {
        if constexpr (K >= kb) {
          const int r = 64 * K + lane;
          if (r > j && r < d) {
            const float uo = v[K] * invj;
            acc[K] = fmaf(uo, etaj, acc[K]);
            sa[K] = fmaf(uo, waj, sa[K]);
            sr[K] = fmaf(uo, wrj, sr[K]);
          }
        }
      });
    });
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      if (r < d) {
        p.xprop[c * d + r] = zp[K];
        p.wa[c * d + r] = wa[K];
        p.wr[c * d + r] = wr[K];
        p.dg[c * d + r] = pdl[K];
      }
    });
  }
}

// ---------------------------------------------------------------- step ----
// NEXT: the pass that streams L' out also runs the next transition's propose
// pass on the columns of L' as they are formed (the same float ops as
// big_propose_kernel on the stored values), so a multi-step launch reads the
// factor once per transition.  The wave's own xprop / wa / wr rows were read
// at the top of its chain, so the next ones overwrite them in place.
template <bool NEXT, bool RAG, int NS>
__global__ __launch_bounds__(256) void big_step_kernel(BigParams p) {
  extern __shared__ float lds_big[];
  const int d = p.d;
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  float* wb0 = lds_big + (size_t)wv * 2 * kColBlk * d;
  float* wb1 = wb0 + kColBlk * d;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t c = (int64_t)blockIdx.x * 4 + threadIdx.x / 64; c < p.C; c += nw) {
    const float* Lin = p.in.scale + c * P;
    float* Lout = p.out.scale + c * P;
    const int32_t it = p.in.i[c];
    const uint32_t k0 = p.in.rng_key[2 * c], k1 = p.in.rng_key[2 * c + 1];
    const float pe = p.in.potential_energy[c];
    const float macc = p.in.mean_accept_prob[c];
    const float lam = p.in.log_step_size[c];
    float pep = p.pep[c];
    const float u = amh_unif01_from_bits(amh_step_word((uint32_t)d, (uint32_t)it, k0, k1));  // W_d
    if (amh_isnan(pep)) pep = INFINITY;
    const float ex = amh_expf(pe - pep);
    const float alpha = (ex > 1.0f) ? 1.0f : ex;
    const bool accept = u < alpha;
    const int32_t itr = it + 1;
    const int32_t n = (it < p.W) ? itr : itr - p.W;
    const float gamma = big_gamma(p, n);
    const float maccn = macc + (alpha - macc) / (float)n;
    const float lamn = lam + gamma * (alpha - p.target);
    const float e1 = amh_expf(lamn);
    const float el = amh_expf(lam);
    const float sq = sqrtf(1.0f - gamma);
    float dl[NS], inv[NS], zn[NS], delta[NS], mun[NS], ws[NS], Dg[NS], one[NS], gw2[NS], t[NS];
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      const bool act = r < d;
      dl[K] = act ? p.dg[c * d + r] : 0.0f;  // the diagonal, coalesced (propose / previous step pass)
      inv[K] = (amh_isfinite(dl[K]) && dl[K] != 0.0f) ? 1.0f / dl[K] : 0.0f;
      const float z = act ? p.in.z[c * d + r] : 0.0f;
      const float mu = act ? p.in.loc[c * d + r] : 0.0f;
      const float zpv = act ? p.xprop[c * d + r] : 0.0f;
      const float w = act ? (accept ? p.wa[c * d + r] : p.wr[c * d + r]) : 0.0f;
      zn[K] = accept ? zpv : z;
      delta[K] = act ? zn[K] - mu : 0.0f;
      mun[K] = act ? mu + gamma * delta[K] : 0.0f;
      ws[K] = w;
      const float ajj = sq * dl[K];
      Dg[K] = ajj * ajj;
      one[K] = (amh_isfinite(ajj) && ajj != 0.0f) ? 1.0f : __int_as_float(0x7FC00000);
      gw2[K] = act ? gamma * (w * w) : 0.0f;
      t[K] = act ? gw2[K] / Dg[K] : 0.0f;
    });
    // b_j: 64-lane exclusive scan per slot plus the carry of the slots before
    float cc[NS], qq[NS];
    bool bad = false;
    float carry = 0.0f;
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      const bool act = r < d;
      const float e = Grp<64>::excl_scan(t[K], lane);
      const float bs = (K == 0) ? e : e + carry;
      const float tot = rdl(e + t[K], 63);
      carry = (K == 0) ? tot : carry + tot;
      const float b = 1.0f + bs;
      const float g2 = (b * Dg[K]) + gw2[K];
      const float dn = g2 / b;
      cc[K] = (gamma * ws[K]) / g2;
      qq[K] = sqrtf(dn);
      const float dnew = fmaf(cc[K], 0.0f, one[K]) * qq[K];
      bad = bad || (act && amh_isnan(dnew));
    });
    const bool revert = __ballot(bad) != 0ull;
    float sacc[NS];
    static_for<NS>([&](auto K) { sacc[K] = 0.0f; });
    // next transition's propose state (big_propose_kernel on the output state)
    float ninv[NS], nxi[NS], neta[NS], nacc[NS], nsa[NS], nsr[NS], nzp[NS], nwa[NS], nwr[NS], ndg[NS];
    if constexpr (NEXT) {
      step_noise_rows<NS>(lane, d, (uint32_t)itr, k0, k1, nxi);
      static_for<NS>([&](auto K) {
        const int r = 64 * K + lane;
        const bool act = r < d;
        const float ndl = act ? (revert ? dl[K] : 1.0f * qq[K]) : 0.0f;
        ndg[K] = ndl;
        ninv[K] = (amh_isfinite(ndl) && ndl != 0.0f) ? 1.0f / ndl : 0.0f;
        neta[K] = ndl * nxi[K];
        nacc[K] = nsa[K] = nsr[K] = nzp[K] = nwa[K] = nwr[K] = 0.0f;
      });
    }
    // column j of L' (rows > j in nv) into the next proposal and both solves
    auto next_col = [&](auto KB, int j, const float (&nv)[NS]) {
      if constexpr (NEXT) {
        constexpr int kb = KB;
        const int jl = j - 64 * kb;
        const float etaj = rdl(neta[kb], jl);
        const float invj = rdl(ninv[kb], jl);
        if (lane == jl) {
          nacc[kb] = fmaf(1.0f, etaj, nacc[kb]);
          nzp[kb] = zn[kb] + fmaf(e1, nacc[kb], p.eps * nxi[kb]);
          nwa[kb] = (nzp[kb] - mun[kb]) - nsa[kb];
          nwr[kb] = (zn[kb] - mun[kb]) - nsr[kb];
        }
        const float waj = rdl(nwa[kb], jl);
        const float wrj = rdl(nwr[kb], jl);
        static_for<NS>([&](auto K) {
          if constexpr (K >= kb) {
            const int r = 64 * K + lane;
            if (r > j && r < d) {
              const float uo = nv[K] * invj;
              nacc[K] = fmaf(uo, etaj, nacc[K]);
              nsa[K] = fmaf(uo, waj, nsa[K]);
              nsr[K] = fmaf(uo, wrj, nsr[K]);
            }
          }
        });
      }
    };
    if (!revert) {
      float ac[NS], bc[NS], sv[NS];
      static_for<NS>([&](auto K) {
        ac[K] = (qq[K] * e1) - (dl[K] * el);
        bc[K] = (cc[K] * qq[K]) * e1;
        sv[K] = 0.0f;
      });
      for_columns<RAG, NS>(Lin, d, P, wb0, wb1, lane, [&](auto KB, int j, const float (&v)[NS]) {
        constexpr int kb = KB;
        const int jl = j - 64 * kb;
        const float wsj = rdl(ws[kb], jl), cj = rdl(cc[kb], jl), acj = rdl(ac[kb], jl);
        const float bcj = rdl(bc[kb], jl), invj = rdl(inv[kb], jl), qj = rdl(qq[kb], jl);
        float* ocol = Lout + col_off(d, j) - j;
        if (lane == jl) {
          const float tt = fmaf(1.0f, acj, bcj * 0.0f);
          sacc[kb] = fmaf(tt, tt, sacc[kb]);
          ocol[j] = 1.0f * qj;
        }
        float nv[NS];
        static_for<NS>([&](auto K) {
          nv[K] = 0.0f;
          if constexpr (K >= kb) {
            const int r = 64 * K + lane;
            if (r > j && r < d) {
              const float uo = v[K] * invj;
              sv[K] = fmaf(uo, wsj, sv[K]);
              const float w = delta[K] - sv[K];
              const float un = fmaf(cj, w, uo);
              const float tt = fmaf(uo, acj, bcj * w);
              sacc[K] = fmaf(tt, tt, sacc[K]);
              nv[K] = un * qj;
              ocol[r] = nv[K];
            }
          }
        });
        next_col(KB, j, nv);
      });
    } else {
      // factor kept (arwmh.py:191): copied verbatim; as_change = ||L (e1 - e0)||_F
      float ac[NS];
      static_for<NS>([&](auto K) { ac[K] = (dl[K] * e1) - (dl[K] * el); });
      for_columns<RAG, NS>(Lin, d, P, wb0, wb1, lane, [&](auto KB, int j, const float (&v)[NS]) {
        constexpr int kb = KB;
        const int jl = j - 64 * kb;
        const float acj = rdl(ac[kb], jl), invj = rdl(inv[kb], jl);
        float* ocol = Lout + col_off(d, j) - j;
        if (lane == jl) {
          const float t0 = 1.0f * acj;
          sacc[kb] = fmaf(t0, t0, sacc[kb]);
          ocol[j] = dl[kb];
        }
        static_for<NS>([&](auto K) {
          if constexpr (K >= kb) {
            const int r = 64 * K + lane;
            if (r > j && r < d) {
              const float x = v[K];
              const float tt = (x * invj) * acj;
              sacc[K] = fmaf(tt, tt, sacc[K]);
              ocol[r] = x;
            }
          }
        });
        next_col(KB, j, v);
      });
    }
    const float asc = sqrtf(big_sum(sacc));
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      if (r < d) {
        p.out.z[c * d + r] = zn[K];
        p.out.loc[c * d + r] = mun[K];
        if (p.col_z != nullptr) p.col_z[c * d + r] = zn[K];
        if constexpr (NEXT) {
          p.xprop[c * d + r] = nzp[K];
          p.wa[c * d + r] = nwa[K];
          p.wr[c * d + r] = nwr[K];
          p.dg[c * d + r] = ndg[K];
        }
      }
    });
    if (lane == 0) {
      p.out.i[c] = itr;
      p.out.potential_energy[c] = accept ? pep : pe;
      p.out.mean_accept_prob[c] = maccn;
      p.out.log_step_size[c] = lamn;
      p.out.as_change[c] = asc;
      p.out.rng_key[2 * c] = k0;
      p.out.rng_key[2 * c + 1] = k1;
      if (p.accept_count != nullptr) p.accept_count[c] += accept ? 1 : 0;
      if (p.col_pe != nullptr) p.col_pe[c] = accept ? pep : pe;
    }
  }
}

// ------------------------------------------------- potential on MFMA ----
// 64 chains per block (two 32-chain tiles), 4 waves; wave w owns the 32-row
// tiles 2w and 2w + 1.  D = z' - m is staged k-major in LDS ([k][chain],
// rows padded to 65 floats); A = P rows straight from L2.  For d % 32 != 0
// the last tile and the k steps past d see zeros (A and the LDS rows d ..
// 32 nt - 1): an fmaf with a zero product leaves a sum that started at +0
// unchanged, so the bits are the k < d chain's.
constexpr int kPotChains = 64;
constexpr int kPotLd = 65;

typedef float f32x16 __attribute__((ext_vector_type(16)));

__host__ __device__ inline int pot_rows(int d) { return (d + 31) & ~31; }
__host__ __device__ inline size_t pot_mfma_lds(int d) { return ((size_t)pot_rows(d) * kPotLd + 8 * kPotChains) * sizeof(float); }

template <bool PAD>  // d % 32 != 0: the zero rows / k steps past d
__global__ __launch_bounds__(256) void gauss_pot_mfma_kernel(PotParams p) {
  extern __shared__ float lds_pot[];
  const int d = p.d;
  float* Dt = lds_pot;
  const int dp = pot_rows(d);
  float(*tsum)[kPotChains] = (float(*)[kPotChains])(lds_pot + (size_t)dp * kPotLd);
  const int nt = dp / 32;
  const float* m = p.model.data;
  const float* Pm = p.model.data + d;
  const float c0 = p.model.data[d + d * d];
  const int64_t cbase = (int64_t)blockIdx.x * kPotChains;
  for (int idx = threadIdx.x; idx < kPotChains * d; idx += 256) {
    const int cc = idx / d, k = idx - cc * d;
    int64_t ch = cbase + cc;
    if (ch >= p.n) ch = p.n - 1;
    Dt[k * kPotLd + cc] = p.z[ch * d + k] - m[k];
  }
  if constexpr (PAD) {
    for (int idx = threadIdx.x; idx < kPotChains * (dp - d); idx += 256) {
      const int cc = idx % kPotChains, k = d + idx / kPotChains;
      Dt[k * kPotLd + cc] = 0.0f;
    }
  }
  __syncthreads();
  const int lane = lane_id();
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  const int h = lane >> 5, i = lane & 31;
  f32x16 acc[2][2];
  static_for<2>([&](auto I) { static_for<2>([&](auto T) { acc[I][T] = f32x16{}; }); });
  const bool has1 = 2 * w + 1 < nt;
  const bool has0 = 2 * w < nt;
  const bool in0 = !PAD || 32 * (2 * w) + i < d, in1 = !PAD || 32 * (2 * w + 1) + i < d;  // rows of P (else zero)
  const float* prow0 = Pm + (int64_t)(in0 ? 32 * (2 * w) + i : 0) * d;
  const float* prow1 = Pm + (int64_t)(in1 ? 32 * (2 * w + 1) + i : 0) * d;
  // A operands (P rows, L2) in batches of 8 k-steps, the next batch loaded
  // while the current one feeds the MFMAs
  if (has0) {
    constexpr int NB = 8;
    float an0[NB], an1[NB];
    auto load = [&](int kk0) {
      static_for<NB>([&](auto S) {
        const int k = kk0 + 2 * S + h;
        if constexpr (PAD) {
          an0[S] = (in0 && k < d) ? prow0[k] : 0.0f;
          an1[S] = (has1 && in1 && k < d) ? prow1[k] : 0.0f;
        } else {
          an0[S] = prow0[k];
          an1[S] = has1 ? prow1[k] : 0.0f;
        }
      });
    };
    load(0);
    for (int kk0 = 0; kk0 < d; kk0 += 2 * NB) {
      float a0[NB], a1[NB];
      static_for<NB>([&](auto S) {
        a0[S] = an0[S];
        a1[S] = an1[S];
      });
      if (kk0 + 2 * NB < d) load(kk0 + 2 * NB);
      static_for<NB>([&](auto S) {
        const int kk = kk0 + 2 * S;
        const float b0 = Dt[(kk + h) * kPotLd + i];
        const float b1 = Dt[(kk + h) * kPotLd + 32 + i];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[S], b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[S], b1, acc[0][1], 0, 0, 0);
        if (has1) {
          acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[S], b0, acc[1][0], 0, 0, 0);
          acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[S], b1, acc[1][1], 0, 0, 0);
        }
      });
    }
  }
  // q = D_r y_r summed over the accumulator layout, then the two lane halves
  static_for<2>([&](auto I) {
    const int tile = 2 * w + I;
    if (tile < nt) {
      static_for<2>([&](auto T) {
        float ps = 0.0f;
        static_for<16>([&](auto R) {
          const int row = 32 * tile + (R & 3) + 8 * (R >> 2) + 4 * h;
          ps = ps + Dt[row * kPotLd + 32 * T + i] * acc[I][T][(int)R];
        });
        const float other = __shfl_xor(ps, 32, 64);
        const float tI = (h == 0) ? ps + other : other + ps;
        if (h == 0) tsum[tile][32 * T + i] = tI;
      });
    }
  });
  __syncthreads();
  if (w == 0) {
    float S = 0.0f;
    for (int t = 0; t < nt; ++t) S = S + tsum[t][lane];
    const int64_t ch = cbase + lane;
    if (ch < p.n) p.pe[ch] = (0.5f * S) + c0;
  }
}

// ------------------------------------------------------------------ ASSS ----
// ASSS (asss.py:192-269) for 64 < d <= 256, dense Gaussian:
// one wave per chain, lane l owns rows 64 s + l, the factor streamed column
// by column through the wave's LDS double buffer (for_columns).  Two passes
// over the factor per transition (bit spec: oracle asss_step_big1; round 5
// had four):
//   A  one column sweep, at column j lane j's y_j = b_j / D_j (y = S^-1 (x -
//      mu), S = (L + eps I) sqrt(d); asss.py:33-45) and three more running
//      sums: av = U (e v) (S v = av + eps sqrt(d) v for the raw draw v),
//      wy = U^-1 y and wv = U^-1 v (ADAPT only).  S y = x - mu, so S z =
//      2 (x - mu) / den and S v_tangent = (S v - dot S z) / |v| need no pass
//   -- the potential along the slice circle: Pa, Pb, Pg = P a, P b, P g
//      (g = mu - m; P's rows read coalesced, an fmaf chain over k), then
//      every shrink step is O(d): D = (a c + b s) / om + g, Y = (Pa c + Pb s)
//      / om + Pg, U = 0.5 sum D Y + c0                      (asss.py:59-96)
//   -- w = U^-1 delta without a pass: delta = S q, q = (z c + v s) / om at
//      the accepted angle, so w = sqrt(d) (dl q + eps U^-1 q)
//   D  the rank-one update streaming L' out, as the large-d ARWMH step pass
//      (no step size)                                     (asss.py:246-267)
// ADAPT = false is the frozen kernel of sample_Pnx (shared loc / factor).
namespace {

template <bool ADAPT, bool RAG, int NS>
__device__ __forceinline__ void asss_big_chain(const float* Lc, float* Lout, const float (&dl)[NS],
                                               const float (&inv)[NS], float (&x)[NS], float (&mu)[NS],
                                               float& pe, float& asc, int32_t it, uint32_t k0, uint32_t k1, int d,
                                               int64_t P, float eps, int32_t W, float gamma_in, const ModelArgs& model,
                                               float* wb0, float* wb1, int lane) {
  const float* m = model.data;
  const float* Pm = model.data + d;
  const float c0 = model.data[d + d * d];
  const float sd = sqrtf((float)d);
  const float epsd = eps * sd;
  const float fd = (float)d;
  // ---- draws (asss.py:207, 219, 225, 60): the d <= 64 kernel's stream
  float v[NS];
  static_for<NS>([&](auto K) {
    const int r = 64 * K + lane;
    v[K] = (r < d) ? amh_normal_from_bits(amh_philox4x32_10((uint32_t)r, (uint32_t)it, 0u, AMH_TAG_ASSS, k0, k1).v[0])
                   : 0.0f;
  });
  const amh_u32x4 o0 = amh_philox4x32_10(0u, (uint32_t)it, 0u, AMH_TAG_ASSS, k0, k1);
  float vd = amh_normal_from_bits(o0.v[1]);
  const float ut = amh_unif01_from_bits(o0.v[2]);
  const float th0 = 6.28318548f * amh_unif01_from_bits(o0.v[3]);
  // ---- pass A: y = S^-1 (x - mu), av = U (e v), wy = U^-1 y, wv = U^-1 v
  float e[NS], invD[NS], b[NS], y[NS], tt[NS], hv[NS], av[NS], ty[NS], tv[NS], wy[NS], wv[NS];
  static_for<NS>([&](auto K) {
    const bool act = 64 * K + lane < d;
    e[K] = dl[K] * sd;
    invD[K] = 1.0f / ((dl[K] + eps) * sd);
    b[K] = act ? x[K] - mu[K] : 0.0f;
    hv[K] = e[K] * v[K];
    y[K] = av[K] = ty[K] = tv[K] = wy[K] = wv[K] = 0.0f;
  });
#if !AMH_ABL_NOPASSA
  for_columns<RAG, NS>(Lc, d, P, wb0, wb1, lane, [&](auto KB, int j, const float (&vv)[NS]) {
    constexpr int kb = KB;
    const int jl = j - 64 * kb;
    const float yl = rdl(b[kb] * invD[kb], jl);
    const float g = yl * rdl(e[kb], jl);
    const float hvj = rdl(hv[kb], jl);
    const float invj = rdl(inv[kb], jl);
    float wyj = 0.0f, wvj = 0.0f;
    if constexpr (ADAPT) {
      wyj = yl - rdl(ty[kb], jl);
      wvj = rdl(v[kb] - tv[kb], jl);
    }
    if (lane == jl) {
      y[kb] = yl;
      av[kb] = fmaf(1.0f, hvj, av[kb]);
      wy[kb] = wyj;
      wv[kb] = wvj;
    }
    static_for<NS>([&](auto K) {
      if constexpr (K >= kb) {
        const int r = 64 * K + lane;
        if (r > j && r < d) {
          const float uo = vv[K] * invj;
          b[K] = fmaf(-uo, g, b[K]);
          av[K] = fmaf(uo, hvj, av[K]);
          if constexpr (ADAPT) {
            ty[K] = fmaf(uo, wyj, ty[K]);
            tv[K] = fmaf(uo, wvj, tv[K]);
          }
        }
      }
    });
  });
#endif
  float svr[NS];  // S v for the raw draw
  static_for<NS>([&](auto K) { svr[K] = av[K] + epsd * v[K]; });
  // ---- stereographic projection, tangent v (asss.py:40-45, 219-222)
  static_for<NS>([&](auto K) { tt[K] = y[K] * y[K]; });
  const float ns = big_sum(tt);
  const float den = ns + 1.0f;
  float zr[NS];
  static_for<NS>([&](auto K) { zr[K] = (2.0f * y[K]) / den; });
  const float zd = (ns - 1.0f) / den;
  static_for<NS>([&](auto K) { tt[K] = v[K] * zr[K]; });
  const float dot = big_sum(tt) + (vd * zd);
  static_for<NS>([&](auto K) { v[K] = (64 * K + lane < d) ? fmaf(-dot, zr[K], v[K]) : 0.0f; });
  vd = fmaf(-dot, zd, vd);
  static_for<NS>([&](auto K) { tt[K] = v[K] * v[K]; });
  const float nv = sqrtf(big_sum(tt) + (vd * vd));
  const bool degen = !(nv > 0.0f);  // the d <= 64 kernel's rule (amh_asss.h)
  static_for<NS>([&](auto K) { v[K] = degen ? 0.0f : v[K] / nv; });
  vd = degen ? 0.0f : vd / nv;
  // ---- S z = 2 (x - mu) / den, S v = (S v_raw - dot S z) / |v|; U^-1 z, U^-1 v
  float Sz[NS], Sv[NS], Wz[NS], Wv[NS], gm[NS], Pa[NS], Pb[NS], Pg[NS];
  static_for<NS>([&](auto K) {
    const int r = 64 * K + lane;
    const bool act = r < d;
    Sz[K] = act ? (2.0f * (x[K] - mu[K])) / den : 0.0f;
    Sv[K] = (degen || !act) ? 0.0f : fmaf(-dot, Sz[K], svr[K]) / nv;
    if constexpr (ADAPT) {
      Wz[K] = (2.0f * wy[K]) / den;
      Wv[K] = (degen || !act) ? 0.0f : fmaf(-dot, Wz[K], wv[K]) / nv;
    }
    gm[K] = act ? mu[K] - m[act ? r : 0] : 0.0f;
    Pa[K] = Pb[K] = Pg[K] = 0.0f;
  });
  // ---- P a, P b, P g: row k of P (= column k) coalesced, k in order
#if !AMH_ABL_NOPMV  // (timing ablations only: AMH_ABL_*)
  static_for<NS>([&](auto KB) {
    constexpr int kb = KB;
    if (64 * kb < d) {
      const int kmax = (d - 64 * kb) < 64 ? (d - 64 * kb) : 64;
      for (int k2 = 0; k2 < kmax; k2 += 8) {
        float pr[8][NS];  // rows k >= d read as zeros (their terms leave the chains unchanged)
        static_for<8>([&](auto T) {
          const bool kin = !RAG || k2 + T < kmax;  // d % 8 == 0: kmax is a multiple of 8
          const float* row = Pm + (int64_t)(kin ? 64 * kb + k2 + T : 0) * d;
          static_for<NS>([&](auto K) { pr[T][K] = (kin && 64 * K + lane < d) ? row[64 * K + lane] : 0.0f; });
        });
        static_for<8>([&](auto T) {
          const int kl = k2 + T;
          const float sa = rdl(Sz[kb], kl), sb = rdl(Sv[kb], kl), sg = rdl(gm[kb], kl);
          static_for<NS>([&](auto K) {
            Pa[K] = fmaf(pr[T][K], sa, Pa[K]);
            Pb[K] = fmaf(pr[T][K], sb, Pb[K]);
            Pg[K] = fmaf(pr[T][K], sg, Pg[K]);
          });
        });
      }
    }
  });
#endif
  // the point at angle (cs, sn) of the slice circle: x and U
  auto eval = [&](float cs, float sn, float (&xo)[NS], float& om) -> float {
    om = 1.0f - ((zd * cs) + (vd * sn));
    float t4[NS];
    static_for<NS>([&](auto K) {
      const bool act = 64 * K + lane < d;
      const float num = (Sz[K] * cs) + (Sv[K] * sn);
      const float Dr = (num / om) + gm[K];
      const float Yr = (((Pa[K] * cs) + (Pb[K] * sn)) / om) + Pg[K];
      t4[K] = act ? Dr * Yr : 0.0f;
      xo[K] = act ? (num / om) + mu[K] : 0.0f;
    });
    return (0.5f * big_sum(t4)) + c0;
  };
  // ---- slice level and shrinkage (asss.py:216-239, 59-96)
  float x0[NS], xt[NS], om0;
  const float U0 = eval(1.0f, 0.0f, x0, om0);
  const float tpe = (U0 + fd * amh_logf(om0)) - amh_logf(ut);
  float th = th0, thmin = th0 - 6.28318548f, thmax = th0;
  int32_t iter = 0;
  float ux, cst, snt, omt;  // the angle of xt
  bool cont;
  {
    float sn, cs, om;
    amh_sincosf(th, &sn, &cs);
    ux = eval(cs, sn, xt, om);
    cst = cs;
    snt = sn;
    omt = om;
    float pt = ux + fd * amh_logf(om);
    if (amh_isnan(pt)) pt = INFINITY;
    cont = !degen && ((pt > tpe) || (om < eps));
  }
  while (cont) {  // wave-uniform: one chain per wave
    if (th < 0.0f) thmin = th;
    if (th >= 0.0f) thmax = th;
    const amh_u32x4 o = amh_philox4x32_10((uint32_t)iter, (uint32_t)it, 1u, AMH_TAG_ASSS, k0, k1);
    th = thmin + (thmax - thmin) * amh_unif01_from_bits(o.v[0]);
    float sn, cs, om;
    amh_sincosf(th, &sn, &cs);
    ux = eval(cs, sn, xt, om);
    cst = cs;
    snt = sn;
    omt = om;
    float pt = ux + fd * amh_logf(om);
    if (amh_isnan(pt)) pt = INFINITY;
    iter += 1;
    cont = (iter < kAsssBigMaxIter) && ((pt > tpe) || (om < eps));
  }
  const bool capped = degen || iter >= kAsssBigMaxIter;  // asss.py:94: theta = 0
  if (capped) {
    cst = 1.0f;
    snt = 0.0f;
    omt = om0;
  }
  float xn[NS];
  static_for<NS>([&](auto K) { xn[K] = capped ? x0[K] : xt[K]; });
  float pen = capped ? U0 : ux;
  if (amh_isnan(pen)) pen = INFINITY;
  if constexpr (!ADAPT) {
    static_for<NS>([&](auto K) { x[K] = xn[K]; });
    pe = pen;
    (void)Lout;
    (void)W;
    (void)gamma_in;
    (void)asc;
    return;
  } else {
    // ---- adaptation (asss.py:246-267): mean, rank-one update, as_change
    const float gamma = gamma_in;
    float delta[NS], mun[NS], Dg[NS], one[NS], ws[NS], gw2[NS];
    const float sq = sqrtf(1.0f - gamma);
    static_for<NS>([&](auto K) {
      const bool act = 64 * K + lane < d;
      delta[K] = act ? xn[K] - mu[K] : 0.0f;
      mun[K] = act ? mu[K] + gamma * delta[K] : 0.0f;
      const float dm = mun[K] - mu[K];
      tt[K] = act ? dm * dm : 0.0f;
      const float ajj = sq * dl[K];
      Dg[K] = ajj * ajj;
      one[K] = (amh_isfinite(ajj) && ajj != 0.0f) ? 1.0f : __int_as_float(0x7FC00000);
      // w = U^-1 delta = sqrt(d) (dl q + eps U^-1 q), q = (z c + v s) / om
      const float q = ((zr[K] * cst) + (v[K] * snt)) / omt;
      const float wq = ((Wz[K] * cst) + (Wv[K] * snt)) / omt;
      ws[K] = act ? ((dl[K] * q) + (eps * wq)) * sd : 0.0f;
    });
    const float locd = sqrtf(big_sum(tt));
    float cc[NS], qq[NS];
    bool bad = false;
    {
      float carry = 0.0f;
      static_for<NS>([&](auto K) {
        const bool act = 64 * K + lane < d;
        gw2[K] = act ? gamma * (ws[K] * ws[K]) : 0.0f;
        const float t = act ? gw2[K] / Dg[K] : 0.0f;
        const float ex = Grp<64>::excl_scan(t, lane);
        const float bs = (K == 0) ? ex : ex + carry;
        const float tot = rdl(ex + t, 63);
        carry = (K == 0) ? tot : carry + tot;
        const float bq = 1.0f + bs;
        const float g2 = (bq * Dg[K]) + gw2[K];
        const float dn = g2 / bq;
        cc[K] = (gamma * ws[K]) / g2;
        qq[K] = sqrtf(dn);
        const float dnew = fmaf(cc[K], 0.0f, one[K]) * qq[K];
        bad = bad || (act && amh_isnan(dnew));
      });
    }
    const bool revert = __ballot(bad) != 0ull || AMH_ABL_NOPASSD;
    float sdiff = 0.0f;
    if (!revert) {
      // pass D: the update, L' streamed out (in place allowed: block b + 1 is
      // in flight before block b's columns are written)
      float ac[NS], bc[NS], sv[NS], sacc[NS];
      static_for<NS>([&](auto K) {
        ac[K] = qq[K] - dl[K];
        bc[K] = cc[K] * qq[K];
        sv[K] = sacc[K] = 0.0f;
      });
      for_columns<RAG, NS>(Lc, d, P, wb0, wb1, lane, [&](auto KB, int j, const float (&vv)[NS]) {
        constexpr int kb = KB;
        const int jl = j - 64 * kb;
        const float wsj = rdl(ws[kb], jl), cj = rdl(cc[kb], jl), acj = rdl(ac[kb], jl);
        const float bcj = rdl(bc[kb], jl), invj = rdl(inv[kb], jl), qj = rdl(qq[kb], jl);
        float* ocol = Lout + col_off(d, j) - j;
        if (lane == jl) {
          const float t0 = fmaf(1.0f, acj, bcj * 0.0f);
          sacc[kb] = fmaf(t0, t0, sacc[kb]);
          ocol[j] = 1.0f * qj;
        }
        static_for<NS>([&](auto K) {
          if constexpr (K >= kb) {
            const int r = 64 * K + lane;
            if (r > j && r < d) {
              const float uo = vv[K] * invj;
              sv[K] = fmaf(uo, wsj, sv[K]);
              const float w = delta[K] - sv[K];
              const float un = fmaf(cj, w, uo);
              const float t1 = fmaf(uo, acj, bcj * w);
              sacc[K] = fmaf(t1, t1, sacc[K]);
              ocol[r] = un * qj;
            }
          }
        });
      });
      sdiff = sqrtf(big_sum(sacc));
    } else if (Lout != Lc && !AMH_ABL_NOPASSD) {  // factor kept (asss.py:255): copied verbatim
      for_columns<RAG, NS>(Lc, d, P, wb0, wb1, lane, [&](auto KB, int j, const float (&vv)[NS]) {
        constexpr int kb = KB;
        float* ocol = Lout + col_off(d, j) - j;
        static_for<NS>([&](auto K) {
          if constexpr (K >= kb) {
            const int r = 64 * K + lane;
            if (r >= j && r < d) ocol[r] = vv[K];
          }
        });
      });
    }
    asc = locd + sdiff;
    static_for<NS>([&](auto K) {
      x[K] = xn[K];
      mu[K] = mun[K];
    });
    pe = pen;
  }
}

}  // namespace

// ASSS.sample: one transition of every chain per launch (host loops n_steps)
template <bool RAG, int NS>
__global__ __launch_bounds__(256) void asss_big_step_kernel(StepParams p) {
  extern __shared__ float lds_big[];
  const int d = p.d;
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  float* wb0 = lds_big + (size_t)wv * 2 * kColBlk * d;
  float* wb1 = wb0 + kColBlk * d;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const int64_t nw = (int64_t)gridDim.x * 4;
  typedef __attribute__((address_space(4))) const float cf;
  for (int64_t c = (int64_t)blockIdx.x * 4 + threadIdx.x / 64; c < p.C; c += nw) {
    const float* Lc = p.in.scale + c * P;
    float* Lo = p.out.scale + c * P;
    const int32_t it = p.in.i[c];
    const uint32_t k0 = p.in.rng_key[2 * c], k1 = p.in.rng_key[2 * c + 1];
    float dl[NS], inv[NS], x[NS], mu[NS];
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      const bool act = r < d;
      dl[K] = act ? Lc[col_off(d, act ? r : 0)] : 0.0f;
      inv[K] = (amh_isfinite(dl[K]) && dl[K] != 0.0f) ? 1.0f / dl[K] : 0.0f;
      x[K] = act ? p.in.z[c * d + r] : 0.0f;
      mu[K] = act ? p.in.loc[c * d + r] : 0.0f;
    });
    const int32_t itr = it + 1;
    const int32_t n = (it < p.W) ? itr : itr - p.W;
    const float gamma = (n < p.gamma_tab_n) ? ((const cf*)p.gamma_tab)[n] : amh_lr_gamma(n, p.a);
    float pe = p.in.potential_energy[c];
    float asc = 0.0f;
    asss_big_chain<true, RAG, NS>(Lc, Lo, dl, inv, x, mu, pe, asc, it, k0, k1, d, P, p.eps, p.W, gamma, p.model, wb0, wb1,
                         lane);
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      if (r < d) {
        p.out.z[c * d + r] = x[K];
        p.out.loc[c * d + r] = mu[K];
        if (p.col_z != nullptr) p.col_z[c * d + r] = x[K];
      }
    });
    if (lane == 0) {
      p.out.i[c] = itr;
      p.out.potential_energy[c] = pe;
      p.out.as_change[c] = asc;
      p.out.rng_key[2 * c] = k0;
      p.out.rng_key[2 * c + 1] = k1;
      if (p.col_pe != nullptr) p.col_pe[c] = pe;
    }
  }
}

// ASSS.sample_Pnx: chain c = (point, sample) from x[point] with key split(c),
// n frozen transitions with the shared (loc, factor), the transition's
// stream position the step index
template <bool RAG, int NS>
__global__ __launch_bounds__(256) void asss_big_pnx_kernel(AsssPnxParams p) {
  extern __shared__ float lds_big[];
  const int d = p.d;
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  float* wb0 = lds_big + (size_t)wv * 2 * kColBlk * d;
  float* wb1 = wb0 + kColBlk * d;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t C = p.n_points * p.n_samples;
  float dl[NS], inv[NS];
  static_for<NS>([&](auto K) {
    const int r = 64 * K + lane;
    const bool act = r < d;
    dl[K] = act ? p.scale[col_off(d, act ? r : 0)] : 0.0f;
    inv[K] = (amh_isfinite(dl[K]) && dl[K] != 0.0f) ? 1.0f / dl[K] : 0.0f;
  });
  for (int64_t c = (int64_t)blockIdx.x * 4 + threadIdx.x / 64; c < C; c += nw) {
    const int64_t pt = c / p.n_samples;
    const amh_u32x4 kk = amh_philox4x32_10((uint32_t)c, (uint32_t)((uint64_t)c >> 32), 0u, AMH_TAG_SPLIT, p.key0, p.key1);
    float x[NS], mu[NS];
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      const bool act = r < d;
      x[K] = act ? p.x[pt * d + r] : 0.0f;
      mu[K] = act ? p.loc[r] : 0.0f;
    });
    float pe = 0.0f, asc = 0.0f;
    for (int32_t t = 0; t < p.n; ++t)
      asss_big_chain<false, RAG, NS>(p.scale, nullptr, dl, inv, x, mu, pe, asc, t, kk.v[0], kk.v[1], d, P, p.eps, 0, 0.0f,
                            p.model, wb0, wb1, lane);
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      if (r < d) p.out[c * d + r] = x[K];
    });
  }
}

// ARWMH.sample_Pnx (arwmh.py:230-270) for the large-d Gaussian: chain c =
// (point, sample) from x[point] with key split(c), n frozen-theta steps at
// stream positions 0..n-1 (bit spec: orc_sample_pnx, large d).  The proposal's
// L xi streams the shared factor column by column (lane l: the fmaf chain of
// L_rj xi_j over j <= r, rows r = 64 s + l); U(z') takes P's rows in k order
// (an fmaf chain per row, the MFMA potential's bits) and sums D_r Y_r in the
// MFMA kernel's tile order (pot_gaussian_big).
template <bool RAG, int NS>
__global__ __launch_bounds__(256) void big_pnx_kernel(PnxParams p) {
  extern __shared__ float lds_big[];
  const int d = p.d;
  const int lane = lane_id();
  const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x / 64));
  float* wb0 = lds_big + (size_t)wv * 2 * kColBlk * d;
  float* wb1 = wb0 + kColBlk * d;
  const int64_t P = (int64_t)d * (d + 1) / 2;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t C = p.n_points * p.n_samples;
  const float* m = p.model.data;
  const float* Pm = p.model.data + d;
  const float c0 = p.model.data[d + d * d];
  const float el = amh_expf(p.log_step_size);
  // U(zz) = 0.5 sum_r D_r Y_r + c0, Y = P D, D = zz - m
  auto potential = [&](const float (&zz)[NS]) -> float {
    float D[NS], Y[NS];
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      const bool act = r < d;
      D[K] = act ? zz[K] - m[act ? r : 0] : 0.0f;
      Y[K] = 0.0f;
    });
    static_for<NS>([&](auto KB) {
      constexpr int kb = KB;
      if (64 * kb < d) {
        const int kmax = (d - 64 * kb) < 64 ? (d - 64 * kb) : 64;
        for (int k2 = 0; k2 < kmax; k2 += 8) {
          float pr[8][NS];  // rows k >= d read as zeros
          static_for<8>([&](auto T) {
            const bool kin = !RAG || k2 + T < kmax;  // d % 8 == 0: kmax is a multiple of 8
            const float* row = Pm + (int64_t)(kin ? 64 * kb + k2 + T : 0) * d;  // row k = column k (P symmetric)
            static_for<NS>([&](auto K) { pr[T][K] = (kin && 64 * K + lane < d) ? row[64 * K + lane] : 0.0f; });
          });
          static_for<8>([&](auto T) {
            const float dk = rdl(D[kb], k2 + T);
            static_for<NS>([&](auto K) { Y[K] = fmaf(pr[T][K], dk, Y[K]); });
          });
        }
      }
    });
    float q[NS];
    static_for<NS>([&](auto K) { q[K] = (64 * K + lane < d) ? D[K] * Y[K] : 0.0f; });
    // tile order: 32-row tiles in order, each (ph_0 + ph_1), ph_h the
    // sequential sum of rows 32 I + (g & 3) + 8 (g >> 2) + 4 h, g = 0..15
    float S = 0.0f;
    static_for<NS>([&](auto K) {
      static_for<2>([&](auto I2) {
        if (64 * K + 32 * I2 < d) {
          float ph[2];
          static_for<2>([&](auto H) {
            float a = 0.0f;
            static_for<16>([&](auto G) {
              constexpr int l = 32 * I2 + (G & 3) + 8 * (G >> 2) + 4 * H;
              a = a + rdl(q[K], l);
            });
            ph[(int)H] = a;
          });
          S = S + (ph[0] + ph[1]);
        }
      });
    });
    return (0.5f * S) + c0;
  };
  for (int64_t c = (int64_t)blockIdx.x * 4 + threadIdx.x / 64; c < C; c += nw) {
    const int64_t pt = c / p.n_samples;
    const amh_u32x4 kk = amh_philox4x32_10((uint32_t)c, (uint32_t)((uint64_t)c >> 32), 0u, AMH_TAG_SPLIT, p.key0, p.key1);
    const uint32_t k0 = kk.v[0], k1 = kk.v[1];
    float z[NS];
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      z[K] = (r < d) ? p.x[pt * d + r] : 0.0f;
    });
    float pe = potential(z);
    for (int32_t t = 0; t < p.n; ++t) {
      float xi[NS], acc[NS], zp[NS];
      step_noise_rows<NS>(lane, d, (uint32_t)t, k0, k1, xi);  // bit spec: amh_step_word
      const float u = amh_unif01_from_bits(amh_step_word((uint32_t)d, (uint32_t)t, k0, k1));  // W_d
      static_for<NS>([&](auto K) { acc[K] = 0.0f; });
      for_columns<RAG, NS>(p.scale, d, P, wb0, wb1, lane, [&](auto KB, int j, const float (&vv)[NS]) {
        constexpr int kb = KB;
        const float xj = rdl(xi[kb], j - 64 * kb);
        static_for<NS>([&](auto K) {
          if constexpr (K >= kb) {
            const int r = 64 * K + lane;
            if (r >= j && r < d) acc[K] = fmaf(vv[K], xj, acc[K]);
          }
        });
      });
      static_for<NS>([&](auto K) {
        const bool act = 64 * K + lane < d;
        zp[K] = act ? z[K] + fmaf(el, acc[K], p.eps * xi[K]) : 0.0f;
      });
      float pep = potential(zp);
      if (amh_isnan(pep)) pep = INFINITY;
      const float ex = amh_expf(pe - pep);
      const float alpha = (ex > 1.0f) ? 1.0f : ex;
      if (u < alpha) {  // wave-uniform: one chain per wave
        static_for<NS>([&](auto K) { z[K] = zp[K]; });
        pe = pep;
      }
    }
    static_for<NS>([&](auto K) {
      const int r = 64 * K + lane;
      if (r < d) p.out[c * d + r] = z[K];
    });
  }
}

// ------------------------------------------------------------- launchers ----
bool big_model(int model_id, int d) { return model_id == AMH_MODEL_GAUSSIAN && d > 64 && d <= 256; }
// pooled mode: the MFMA path also takes d = 64 (every per-chain product is a
// GEMM over chains once the factor is shared)
bool pooled_big_model(int model_id, int d) {
  return model_id == AMH_MODEL_GAUSSIAN && d >= 64 && d <= 256 && d % 32 == 0;
}

// row slots per lane by d: two up to 128, three up to 192, four up to 256
// (each a separate instantiation; big_sum adds the absent slots as +0)
#ifndef AMH_BIG_NS3
#define AMH_BIG_NS3 1
#endif
static int row_slots(int d) { return d <= 128 ? 2 : ((AMH_BIG_NS3 && d <= 192) ? 3 : 4); }
static int wave_grid(int64_t n) {
  int64_t b = (n + 3) / 4;
  if (b > 256 * 16) b = 256 * 16;
  return (int)(b > 0 ? b : 1);
}

hipError_t run_big_init(const InitParams& p, hipStream_t s) {
  const int ns = row_slots(p.d);
  auto k = ns == 2 ? big_init_kernel<2> : (ns == 3 ? big_init_kernel<3> : big_init_kernel<4>);
  hipLaunchKernelGGL(k, dim3(wave_grid(p.C)), dim3(256), 0, s, p);
  return hipGetLastError();
}
static size_t stream_lds(int d) { return (size_t)4 * 2 * kColBlk * d * sizeof(float); }
#define AMH_BY_NS(NAME, ...) \
  (ns == 2 ? NAME<__VA_ARGS__, 2> : (ns == 3 ? NAME<__VA_ARGS__, 3> : NAME<__VA_ARGS__, 4>))
hipError_t run_big_propose(const BigParams& p, hipStream_t s) {
  const bool rag = p.d % kColBlk != 0;
  const int ns = row_slots(p.d);
  auto k = rag ? AMH_BY_NS(big_propose_kernel, true) : AMH_BY_NS(big_propose_kernel, false);
  hipLaunchKernelGGL(k, dim3(wave_grid(p.C)), dim3(256), stream_lds(p.d), s, p);
  return hipGetLastError();
}
hipError_t run_big_step(const BigParams& p, hipStream_t s, bool next) {
  const bool rag = p.d % kColBlk != 0;
  const int ns = row_slots(p.d);
  auto k = next ? (rag ? AMH_BY_NS(big_step_kernel, true, true) : AMH_BY_NS(big_step_kernel, true, false))
                : (rag ? AMH_BY_NS(big_step_kernel, false, true) : AMH_BY_NS(big_step_kernel, false, false));
  hipLaunchKernelGGL(k, dim3(wave_grid(p.C)), dim3(256), stream_lds(p.d), s, p);
  return hipGetLastError();
}
hipError_t run_asss_big_step(const StepParams& p, hipStream_t s) {
  const bool rag = p.d % kColBlk != 0;
  const int ns = row_slots(p.d);
  auto k = rag ? AMH_BY_NS(asss_big_step_kernel, true) : AMH_BY_NS(asss_big_step_kernel, false);
  hipLaunchKernelGGL(k, dim3(wave_grid(p.C)), dim3(256), stream_lds(p.d), s, p);
  return hipGetLastError();
}
hipError_t run_big_pnx(const PnxParams& p, hipStream_t s) {
  const bool rag = p.d % kColBlk != 0;
  const int ns = row_slots(p.d);
  auto k = rag ? AMH_BY_NS(big_pnx_kernel, true) : AMH_BY_NS(big_pnx_kernel, false);
  hipLaunchKernelGGL(k, dim3(wave_grid(p.n_points * p.n_samples)), dim3(256), stream_lds(p.d), s, p);
  return hipGetLastError();
}
hipError_t run_asss_big_pnx(const AsssPnxParams& p, hipStream_t s) {
  const bool rag = p.d % kColBlk != 0;
  const int ns = row_slots(p.d);
  auto k = rag ? AMH_BY_NS(asss_big_pnx_kernel, true) : AMH_BY_NS(asss_big_pnx_kernel, false);
  hipLaunchKernelGGL(k, dim3(wave_grid(p.n_points * p.n_samples)), dim3(256), stream_lds(p.d), s, p);
  return hipGetLastError();
}
hipError_t run_big_potential(const PotParams& p, hipStream_t s) {
  const int64_t blocks = (p.n + kPotChains - 1) / kPotChains;
  auto k = (p.d % 32) ? gauss_pot_mfma_kernel<true> : gauss_pot_mfma_kernel<false>;
  hipLaunchKernelGGL(k, dim3((unsigned)blocks), dim3(256), pot_mfma_lds(p.d), s, p);
  return hipGetLastError();
}

}  // namespace amh
