// amh_asss.h -- one ASSS transition (python/kernels/asss.py:197-251) of a
// lane group's chain, shared by the ASSS kernels (amh_asss.hip) and the d = 64
// persistent step kernel's ASSS instantiation (amh_kernels.hip).  Bit spec:
// oracle/amh_oracle.c orc_asss_step.
#pragma once
#include "amh_device.h"

namespace amh {

constexpr int kAsssMaxIter = 50;  // asss.py:59 max_iterations

// One ASSS transition of the group's chain (asss.py:197-251) at stream
// position `it`.  ADAPT = false is the frozen kernel of sample_Pnx
// (asss.py:281-296): the shared (U, dl, mu) are used and left unchanged.
template <int DMAX, template <int> class M, bool ADAPT>
__device__ __forceinline__ void asss_transition(const StepParams& p, float (&U)[DMAX], float& dl, float& x,
                                                float& mu, float& pe, float& asc, bool& updated, int32_t it,
                                                uint32_t k0, uint32_t k1, int d, int r, int rr, bool act,
                                                const typename M<DMAX>::Ctx& mctx, const float* lds) {
  constexpr int G = DMAX;
  using Gp = Grp<G>;
  const float sd = sqrtf((float)d);
  const float epsd = p.eps * sd;
  const float fd = (float)d;
  // ---- draws (asss.py:207, 219, 225, 60)
  const amh_u32x4 o = amh_philox4x32_10((uint32_t)r, (uint32_t)it, 0u, AMH_TAG_ASSS, k0, k1);
  float v = act ? amh_normal_from_bits(o.v[0]) : 0.0f;
  float vd = amh_normal_from_bits(Gp::template bcast_u<0>(o.v[1]));
  const float ut = amh_unif01_from_bits(Gp::template bcast_u<0>(o.v[2]));
  const float th0 = 6.28318548f * amh_unif01_from_bits(Gp::template bcast_u<0>(o.v[3]));

  // ---- y = S^-1 (x - mu): S_rj = U_rj e_j below the diagonal, S_rr = D_r
  const float e = dl * sd;
  const float Dr = (dl + p.eps) * sd;
  const float invD = 1.0f / Dr;
  float b = act ? x - mu : 0.0f;
  float y = 0.0f;
  static_for<DMAX>([&](auto J) {
    constexpr int j = J;
    if (j < d) {
      const float yl = b * invD;
      y = capture<G, j>(y, Gp::template bcast<j>(yl), rr);
      const float gj = Gp::template bcast<j>(yl * e);
      b = fmaf(-U[j], gj, b);
    }
    column_fence<j>();
  });

  // ---- stereographic projection (asss.py:40-45)
  const float ns = Gp::sum(act ? y * y : 0.0f);
  const float den = ns + 1.0f;
  const float zr = act ? (2.0f * y) / den : 0.0f;
  const float zd = (ns - 1.0f) / den;

  // ---- v orthogonal to z on S^d (asss.py:219-222)
  // v - (v.z) z with one rounding per component (fmaf): with the product
  // rounded first, a draw numerically parallel to z (about 1e-9 per
  // transition at d = 1) cancelled to exactly 0 -- a mitigation, not a cure:
  // if every component still rounds to 0 (|v| = 0, where the reference's
  // v / norm(v) is NaN and would poison the chain), the transition is the
  // shrinkage's own fallback, theta = 0 (asss.py:94): the state is kept
  // (re-projected), the adaptation runs as usual.  Oracle: asss_chain_step.
  const float dot = Gp::sum(act ? v * zr : 0.0f) + (vd * zd);
  v = act ? fmaf(-dot, zr, v) : 0.0f;
  vd = fmaf(-dot, zd, vd);
  const float nv = sqrtf(Gp::sum(v * v) + (vd * vd));
  const bool degen = !(nv > 0.0f);  // group-uniform
  v = degen ? 0.0f : v / nv;
  vd = degen ? 0.0f : vd / nv;

  // ---- S z_1d and S v_1d (asss.py:48-56 for both circle directions)
  float sz4[4] = {0.0f, 0.0f, 0.0f, 0.0f}, sv4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
  const float hz = e * zr, hv = e * v;
  static_for<DMAX>([&](auto J) {
    if (J < d) {
      sz4[J & 3] = fmaf(U[J], Gp::template bcast<J>(hz), sz4[J & 3]);
      sv4[J & 3] = fmaf(U[J], Gp::template bcast<J>(hv), sv4[J & 3]);
    }
    column_fence<J, 16>();
  });
  const float Sz = ((sz4[0] + sz4[1]) + (sz4[2] + sz4[3])) + epsd * zr;
  const float Sv = ((sv4[0] + sv4[1]) + (sv4[2] + sv4[3])) + epsd * v;

  // x on the circle at angle (c, s); om = 1 - z_d(th)
  auto x_at = [&](float c, float s, float& om) -> float {
    const float zdt = (zd * c) + (vd * s);
    om = 1.0f - zdt;
    return act ? (((Sz * c) + (Sv * s)) / om) + mu : 0.0f;
  };

  // ---- slice level at z (asss.py:216-217, 224-226)
  float om0;
  const float x0 = x_at(1.0f, 0.0f, om0);
  const float U0 = M<G>::potential(x0, r, d, mctx, lds);
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
    ux = M<G>::potential(xt, r, d, mctx, lds);
    float pt = ux + fd * amh_logf(om);
    if (amh_isnan(pt)) pt = INFINITY;
    cont = !degen && ((pt > tpe) || (om < p.eps));
  }
  while (__ballot(cont) != 0ull) {
    const float thmin_n = (th < 0.0f) ? th : thmin;
    const float thmax_n = (th >= 0.0f) ? th : thmax;
    const amh_u32x4 ok = amh_philox4x32_10((uint32_t)iter, (uint32_t)it, 1u, AMH_TAG_ASSS, k0, k1);
    const float th_n = thmin_n + (thmax_n - thmin_n) * amh_unif01_from_bits(ok.v[0]);
    float s, c, om;
    amh_sincosf(th_n, &s, &c);
    const float xn = x_at(c, s, om);
    const float un = M<G>::potential(xn, r, d, mctx, lds);
    float pt = un + fd * amh_logf(om);
    if (amh_isnan(pt)) pt = INFINITY;
    if (cont) {
      thmin = thmin_n;
      thmax = thmax_n;
      th = th_n;
      xt = xn;
      ux = un;
      iter += 1;
      cont = (iter < kAsssMaxIter) && ((pt > tpe) || (om < p.eps));
    }
  }
  const bool capped = degen || iter >= kAsssMaxIter;  // asss.py:94: theta = 0
  const float xnew = capped ? x0 : xt;
  float pen = capped ? U0 : ux;
  if (amh_isnan(pen)) pen = INFINITY;  // asss.py:234

  if constexpr (!ADAPT) {
    x = xnew;
    pe = pen;
    return;
  } else {
    // ---- adaptation (asss.py:237-251): as ARWMH without the step size
    const int32_t itr = it + 1;
    const int32_t n = (it < p.W) ? itr : itr - p.W;
    const float gamma = lookup_gamma<G>(p, n);
    const float delta = act ? xnew - mu : 0.0f;
    const float mun = act ? mu + gamma * delta : 0.0f;
    const float dmu = mun - mu;
    const float locd = sqrtf(Gp::sum(dmu * dmu));

    const float sq = sqrtf(1.0f - gamma);
    const float ajj = sq * dl;
    const float Dg = ajj * ajj;
    const float one = (amh_isfinite(ajj) && ajj != 0.0f) ? 1.0f : __int_as_float(0x7FC00000);
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
    const float gw2 = act ? gamma * (ws * ws) : 0.0f;
    const float tsc = act ? gw2 / Dg : 0.0f;
    const float bb = 1.0f + Gp::excl_scan(tsc, rr);
    const float g2 = (bb * Dg) + gw2;
    const float dn = g2 / bb;
    const float cc = (gamma * ws) / g2;
    const float q = sqrtf(dn);
    const float dnew = fmaf(cc, 0.0f, one) * q;
    const bool revert = Gp::any(act && amh_isnan(dnew));
    float sdiff = 0.0f;
    if (!revert) {
      // U'_rj = U_rj + c_j w_r^(j+1);  L'_rj - L_rj = U_rj (q_j - dl_j) + (c_j q_j) w_r^(j+1)
      const float ac = q - dl;
      const float bc = cc * q;
      float s4[4] = {0.0f, 0.0f, 0.0f, 0.0f};
      w = delta;
      static_for<DMAX>([&](auto J) {
        if (J < d) {
          const float wj = Gp::template bcast<J>(ws);
          const float cj = Gp::template bcast<J>(cc);
          const float aj = Gp::template bcast<J>(ac);
          const float bj = Gp::template bcast<J>(bc);
          const float uo = U[J];
          w = fmaf(-wj, uo, w);
          const float un = fmaf(cj, w, uo);
          const float tt = fmaf(uo, aj, bj * w);
          s4[J & 3] = fmaf(tt, tt, s4[J & 3]);
          U[J] = un;
        }
        column_fence<J>();
      });
      const float sacc = (s4[0] + s4[1]) + (s4[2] + s4[3]);
      sdiff = sqrtf(Gp::sum(act ? sacc : 0.0f));
      dl = act ? q : 0.0f;
      updated = true;
    }
    asc = locd + sdiff;  // asss.py:248-250
    x = xnew;
    pe = pen;
    mu = mun;
  }
}

}  // namespace amh
