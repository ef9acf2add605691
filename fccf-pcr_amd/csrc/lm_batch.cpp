// lm_batch.cpp — quick_verify's Ceres-1.14-style LM (host_stages.cpp lm_solve; FCCF.cpp
// :210-249, App. A10) for up to L problems at once, SIMD across the problems: lane l
// runs problem l's own iteration with exactly the scalar form's operations in the same
// order (IEEE add, multiply, divide and square root give the same bits in a vector lane;
// no contraction: -ffp-contract=off), so every lane's result equals lm_solve's bit for
// bit.  Where the problems' paths differ (row counts, accepted steps, termination) a
// lane's state changes only under its mask: a masked sum skips a row instead of adding
// zero (which could turn a -0 into +0).  sin, cos and pow (the quaternion plus and the
// trust-region radius) run per lane through the same libm calls as lm_solve.  Written
// with clang vector types; built for AVX-512 (8 lanes) or AVX2 (4 lanes), chosen at run
// time; other CPUs run lm_solve.
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "host_stages.h"

// Host code only: the Makefile compiles every .cpp as HIP, and the device pass has no
// CPU feature detection or x86 target attributes.
#ifndef __HIP_DEVICE_COMPILE__
namespace fccf {
constexpr int LB_MAXP_PUBLIC = 17;  // lm_solve's limit (host_stages.cpp LM_MAXM / 2)
namespace {

constexpr int LB_MAXP = 17, LB_MAXM = 2 * LB_MAXP, LB_LD = LB_MAXM + 6;
static_assert(LB_MAXP == LB_MAXP_PUBLIC, "one pair limit");
#define LB_AI __attribute__((always_inline)) inline

template <int L>
struct VT {
  typedef double V __attribute__((ext_vector_type(L)));
  typedef long M __attribute__((ext_vector_type(L)));  // lane masks: -1 true, 0 false
};

template <int L>
LB_AI typename VT<L>::V vsqrt(typename VT<L>::V a) {
  return __builtin_elementwise_sqrt(a);
}
template <int L>
LB_AI typename VT<L>::M vfinite(typename VT<L>::V a) {  // std::isfinite per lane (NaN compares false)
  return __builtin_elementwise_abs(a) < (typename VT<L>::V)(INFINITY);
}
template <int L>
LB_AI bool vany(typename VT<L>::M m) {
  for (int l = 0; l < L; ++l)
    if (m[l]) return true;
  return false;
}

template <int L>
struct LbData {
  using V = typename VT<L>::V;
  using M = typename VT<L>::M;
  int Pmax, Mmax;
  M P, m, Mr;  // per lane: pairs, rows, rows + 6
  V p1[LB_MAXP][3], n1[LB_MAXP][3], p2[LB_MAXP][3], n2[LB_MAXP][3], w[LB_MAXP];
};

template <int L>
LB_AI void cross_v(const typename VT<L>::V* a, const typename VT<L>::V* b, typename VT<L>::V* r) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}

// host_stages.cpp rotq: v' = v + w*uv + u x uv, uv = 2(u x v); Jacobian wrt (x,y,z,w)
template <int L, bool WJ>
LB_AI void rotq_v(const typename VT<L>::V* q, const typename VT<L>::V* v, typename VT<L>::V* f,
                  typename VT<L>::V (*J)[4]) {
  using V = typename VT<L>::V;
  const V u[3] = {q[0], q[1], q[2]};
  V a[3], uv[3], c[3];
  cross_v<L>(u, v, a);
  for (int i = 0; i < 3; ++i) uv[i] = a[i] + a[i];
  cross_v<L>(u, uv, c);
  for (int i = 0; i < 3; ++i) f[i] = (v[i] + q[3] * uv[i]) + c[i];
  if (!WJ) return;
  for (int k = 0; k < 3; ++k) {
    V e[3], ekv[3], eka[3], uekv[3];
    for (int i = 0; i < 3; ++i) e[i] = (V)(i == k ? 1.0 : 0.0);
    cross_v<L>(e, v, ekv);
    cross_v<L>(e, a, eka);
    cross_v<L>(u, ekv, uekv);
    for (int i = 0; i < 3; ++i) J[i][k] = (V)(2.0) * q[3] * ekv[i] + (V)(2.0) * (eka[i] + uekv[i]);
  }
  for (int i = 0; i < 3; ++i) J[i][3] = uv[i];
}

// host_stages.cpp lm_eval for the lanes in `act`: their cost (when ok), residual rows and
// (WJ) Jacobian rows are written; other lanes' outputs are left as they were.  Returns
// the lanes of `act` whose residuals and Jacobian entries are all finite.
template <int L, bool WJ>
LB_AI typename VT<L>::M lm_eval_v(const LbData<L>& D, const typename VT<L>::V* x, typename VT<L>::M act,
                                  typename VT<L>::V& cost, typename VT<L>::V* r, typename VT<L>::V (*J)[6]) {
  using V = typename VT<L>::V;
  using M = typename VT<L>::M;
  const V Pj[4][3] = {{x[3], x[2], -x[1]}, {-x[2], x[3], x[0]}, {x[1], -x[0], x[3]}, {-x[0], -x[1], -x[2]}};
  V c = (V)(0.0);
  M bad = (M)(0);
  for (int b = 0; b < D.Pmax; ++b) {
    M in = act & ~bad & (D.P > b);
    V n2r[3], p2r[3], Jn[3][4], Jp[3][4], cr[3];
    rotq_v<L, WJ>(x, D.n2[b], n2r, Jn);
    rotq_v<L, WJ>(x, D.p2[b], p2r, Jp);
    for (int i = 0; i < 3; ++i) p2r[i] = p2r[i] + x[4 + i];
    cross_v<L>(D.n1[b], n2r, cr);
    const V nrm = vsqrt<L>((cr[0] * cr[0] + cr[1] * cr[1]) + cr[2] * cr[2]);
    const V d = ((D.n1[b][0] * D.p1[b][0] + D.n1[b][1] * D.p1[b][1]) + D.n1[b][2] * D.p1[b][2]) -
                ((n2r[0] * p2r[0] + n2r[1] * p2r[1]) + n2r[2] * p2r[2]);
    const V sdd = vsqrt<L>(d * d);
    const V r0 = D.w[b] * nrm, r1 = D.w[b] * sdd;
    r[2 * b] = in ? r0 : r[2 * b];
    r[2 * b + 1] = in ? r1 : r[2 * b + 1];
    c = in ? c + (V)(0.5) * (r0 * r0 + r1 * r1) : c;
    const M rf = vfinite<L>(r0) & vfinite<L>(r1);
    bad = bad | (in & ~rf);
    in = in & rf;
    if (WJ) {
      V g0[4], g1[7];
      for (int k = 0; k < 4; ++k) {
        const V col[3] = {Jn[0][k], Jn[1][k], Jn[2][k]};
        V dc[3];
        cross_v<L>(D.n1[b], col, dc);
        g0[k] = D.w[b] * (((cr[0] * dc[0] + cr[1] * dc[1]) + cr[2] * dc[2]) / nrm);
        const V dd = -(((Jn[0][k] * p2r[0] + Jn[1][k] * p2r[1]) + Jn[2][k] * p2r[2]) +
                       ((n2r[0] * Jp[0][k] + n2r[1] * Jp[1][k]) + n2r[2] * Jp[2][k]));
        g1[k] = D.w[b] * ((d * dd) / sdd);
      }
      for (int k = 0; k < 3; ++k) g1[4 + k] = D.w[b] * ((d * -n2r[k]) / sdd);
      M jf = (M)(-1);
      for (int j = 0; j < 3; ++j) {
        const V j0 = ((g0[0] * Pj[0][j] + g0[1] * Pj[1][j]) + g0[2] * Pj[2][j]) + g0[3] * Pj[3][j];
        const V j1 = ((g1[0] * Pj[0][j] + g1[1] * Pj[1][j]) + g1[2] * Pj[2][j]) + g1[3] * Pj[3][j];
        J[2 * b][j] = in ? j0 : J[2 * b][j];
        J[2 * b + 1][j] = in ? j1 : J[2 * b + 1][j];
        J[2 * b][3 + j] = in ? (V)(0.0) : J[2 * b][3 + j];
        J[2 * b + 1][3 + j] = in ? g1[4 + j] : J[2 * b + 1][3 + j];
        jf = jf & vfinite<L>(j0) & vfinite<L>(j1) & vfinite<L>(g1[4 + j]);
      }
      bad = bad | (in & ~jf);
    }
  }
  const M ok = act & ~bad;
  cost = ok ? c : cost;
  return ok;
}

// host_stages.cpp qr_solve: min || [A; diag(Dg)] y - [b; 0] || by Householder QR, per lane
// over its own M = m + 6 rows (rows past a lane's M take no part in any sum).  Returns
// the lanes whose y is finite.
template <int L>
LB_AI typename VT<L>::M qr_solve_v(const LbData<L>& D, const typename VT<L>::V (*A)[6], const typename VT<L>::V* Dg,
                                   const typename VT<L>::V* b, typename VT<L>::V* y) {
  using V = typename VT<L>::V;
  using M = typename VT<L>::M;
  constexpr int n = 6;
  V C[n + 1][LB_LD];
  const int Mmax = D.Mmax;
  for (int i = 0; i < Mmax; ++i) {
    const M rowA = D.m > i;
    for (int j = 0; j < n; ++j) C[j][i] = rowA ? A[i][j] : ((D.m + j == i) ? Dg[j] : (V)(0.0));
    C[n][i] = rowA ? b[i] : (V)(0.0);
  }
  for (int k = 0; k < n; ++k) {
    const V c0 = C[k][k];
    V tail = (V)(0.0);
    for (int i = k + 1; i < Mmax; ++i) tail = (D.Mr > i) ? tail + C[k][i] * C[k][i] : tail;
    const M small = tail <= (V)(DBL_MIN);
    V bt = vsqrt<L>(c0 * c0 + tail);
    bt = (c0 >= (V)(0.0)) ? -bt : bt;
    const V beta = small ? c0 : bt;
    const V tau = small ? (V)(0.0) : (bt - c0) / bt;
    const V den = c0 - beta;
    for (int i = k + 1; i < Mmax; ++i) {
      const M row = D.Mr > i;
      C[k][i] = row ? (small ? (V)(0.0) : C[k][i] / den) : C[k][i];
    }
    C[k][k] = beta;
    V tmp[n + 1];
    for (int j = k + 1; j <= n; ++j) tmp[j] = (V)(0.0);
    for (int i = k + 1; i < Mmax; ++i) {
      const M row = D.Mr > i;
      const V v = C[k][i];
      for (int j = k + 1; j <= n; ++j) tmp[j] = row ? tmp[j] + v * C[j][i] : tmp[j];
    }
    for (int j = k + 1; j <= n; ++j) {
      const V t = tmp[j] + C[j][k];
      C[j][k] = C[j][k] - tau * t;
      for (int i = k + 1; i < Mmax; ++i) {
        const M row = D.Mr > i;
        C[j][i] = row ? C[j][i] - tau * C[k][i] * t : C[j][i];
      }
    }
  }
  for (int i = 0; i < n; ++i) y[i] = C[n][i];
  for (int k = n - 1; k >= 0; --k) {
    y[k] = y[k] / C[k][k];
    for (int i = 0; i < k; ++i) y[i] = y[i] - y[k] * C[k][i];
  }
  M fin = (M)(-1);
  for (int i = 0; i < n; ++i) fin = fin & vfinite<L>(y[i]);
  return fin;
}

// host_stages.cpp plus7 (EigenQuaternionParameterization::Plus, Euclidean t) for the
// lanes in `act`; sin and cos per lane
template <int L>
LB_AI void plus7_v(const typename VT<L>::V* x, const typename VT<L>::V* d, typename VT<L>::V* o,
                   typename VT<L>::M act) {
  using V = typename VT<L>::V;
  using M = typename VT<L>::M;
  const V nd = vsqrt<L>(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  const M pos = nd > (V)(0.0);
  V s = (V)(0.0), cs = (V)(1.0);
  for (int l = 0; l < L; ++l)
    if (act[l] && pos[l]) {
      s[l] = std::sin(nd[l]) / nd[l];
      cs[l] = std::cos(nd[l]);
    }
  const V ax = s * d[0], ay = s * d[1], az = s * d[2], aw = cs;
  const V bx = x[0], by = x[1], bz = x[2], bw = x[3];
  o[0] = pos ? (aw * bx + ay * bz) - (az * by - ax * bw) : x[0];
  o[1] = pos ? (aw * by + ay * bw) + (az * bx - ax * bz) : x[1];
  o[2] = pos ? (aw * bz - ay * bx) + (az * bw + ax * by) : x[2];
  o[3] = pos ? (aw * bw - ay * by) - (az * bz + ax * bx) : x[3];
  for (int i = 0; i < 3; ++i) o[4 + i] = x[4 + i] + d[3 + i];
}

// lm_solve's finish(): the gradient, the largest change of its plus step (gmax) and the
// column scaling of J -- for the lanes in `sel`.  (Helpers that take vectors are
// always_inline functions, not lambdas: a lambda is compiled for the default target, and
// passing an AVX-512 vector into it breaks the calling convention.)
template <int L>
LB_AI void lb_finish(const LbData<L>& D, const typename VT<L>::V* x, const typename VT<L>::V* r,
                     typename VT<L>::V (*J)[6], const typename VT<L>::V* scale, typename VT<L>::V& gmax,
                     typename VT<L>::M sel) {
  using V = typename VT<L>::V;
  using M = typename VT<L>::M;
  V ng[6], xp[7];
  for (int j = 0; j < 6; ++j) {
    V s = (V)(0.0);
    for (int i = 0; i < LB_MAXM; ++i) s = (D.m > i) ? s + J[i][j] * r[i] : s;
    ng[j] = -s;
  }
  plus7_v<L>(x, ng, xp, sel);
  V mx = (V)(0.0);
  for (int j = 0; j < 7; ++j) {
    const V dlt = __builtin_elementwise_abs(x[j] - xp[j]);
    mx = (mx < dlt) ? dlt : mx;  // std::max(mx, |.|)
  }
  gmax = sel ? mx : gmax;
  for (int i = 0; i < LB_MAXM; ++i) {
    const M row = sel & (D.m > i);
    for (int j = 0; j < 6; ++j) J[i][j] = row ? J[i][j] * scale[j] : J[i][j];
  }
}
template <int L>
LB_AI typename VT<L>::V lb_norm7(const typename VT<L>::V* x) {
  typename VT<L>::V s = (typename VT<L>::V)(0.0);
  for (int i = 0; i < 7; ++i) s += x[i] * x[i];
  return vsqrt<L>(s);
}

// host_stages.cpp lm_solve, lane-parallel: problems pf[0..n) (n <= L) with P[l] pairs
template <int L>
LB_AI void lm_solve_v(const float* const* pf, const int* Pin, int n, double (*best)[7]) {
  using V = typename VT<L>::V;
  using M = typename VT<L>::M;
  LbData<L> D;
  D.Pmax = 0;
  D.Mmax = 0;
  M act;
  for (int l = 0; l < L; ++l) {
    const int P = l < n ? Pin[l] : 0;
    D.P[l] = P;
    D.m[l] = 2 * P;
    D.Mr[l] = 2 * P + 6;
    act[l] = l < n ? -1 : 0;
    D.Pmax = std::max(D.Pmax, P);
    D.Mmax = std::max(D.Mmax, 2 * P + 6);
  }
  for (int b = 0; b < LB_MAXP; ++b) {
    for (int i = 0; i < 3; ++i) D.p1[b][i] = D.n1[b][i] = D.p2[b][i] = D.n2[b][i] = (V)(0.0);
    D.w[b] = (V)(0.0);
    for (int l = 0; l < L; ++l) {
      if (b >= D.P[l]) continue;
      const float* s = pf[l] + 13 * b;
      for (int i = 0; i < 3; ++i) {
        D.p1[b][i][l] = (double)s[i];
        D.n1[b][i][l] = (double)s[3 + i];
        D.p2[b][i][l] = (double)s[6 + i];
        D.n2[b][i][l] = (double)s[9 + i];
      }
      D.w[b][l] = (double)s[12];
    }
  }
  V x[7], r[LB_MAXM], J[LB_MAXM][6], rc[LB_MAXM], cost = (V)(0.0);
  for (int i = 0; i < 7; ++i) x[i] = (V)(i == 3 ? 1.0 : 0.0);
  for (int l = 0; l < n; ++l)
    for (int i = 0; i < 7; ++i) best[l][i] = x[i][l];
  for (int i = 0; i < LB_MAXM; ++i) {
    r[i] = rc[i] = (V)(0.0);
    for (int j = 0; j < 6; ++j) J[i][j] = (V)(0.0);
  }
  act = lm_eval_v<L, true>(D, x, act, cost, r, J);
  V scale[6], gmax = (V)(0.0);
  for (int j = 0; j < 6; ++j) {
    V s = (V)(0.0);
    for (int i = 0; i < LB_MAXM; ++i) s = (D.m > i) ? s + J[i][j] * J[i][j] : s;
    scale[j] = (V)(1.0) / ((V)(1.0) + vsqrt<L>(s));
  }
  lb_finish<L>(D, x, r, J, scale, gmax, act);
  V min_cost = cost, x_norm = lb_norm7<L>(x), radius = (V)(1e4), decrease = (V)(2.0), diag[6];
  for (int j = 0; j < 6; ++j) diag[j] = (V)(0.0);
  M reuse = (M)(0);
  int iteration[L], invalid[L];
  for (int l = 0; l < L; ++l) iteration[l] = invalid[l] = 0;
  act = act & ~(gmax <= (V)(1e-10));
  while (vany<L>(act)) {
    for (int l = 0; l < L; ++l)
      if (act[l]) ++iteration[l];
    const M newdiag = act & ~reuse;
    if (vany<L>(newdiag))
      for (int j = 0; j < 6; ++j) {
        V s = (V)(0.0);
        for (int i = 0; i < LB_MAXM; ++i) s = (D.m > i) ? s + J[i][j] * J[i][j] : s;
        s = (s < (V)(1e-6)) ? (V)(1e-6) : s;  // std::max(s, 1e-6)
        s = ((V)(1e32) < s) ? (V)(1e32) : s;  // std::min(., 1e32)
        diag[j] = newdiag ? s : diag[j];
      }
    V Dg[6], y[6], step[6];
    for (int j = 0; j < 6; ++j) Dg[j] = vsqrt<L>(diag[j] / radius);
    const M solved = qr_solve_v<L>(D, J, Dg, r, y);
    reuse = reuse | act;
    for (int j = 0; j < 6; ++j) step[j] = -y[j];
    V dot = (V)(0.0);
    for (int i = 0; i < LB_MAXM; ++i) {
      V mr = (V)(0.0);
      for (int j = 0; j < 6; ++j) mr += J[i][j] * step[j];
      dot = (D.m > i) ? dot + mr * (r[i] + mr / (V)(2.0)) : dot;
    }
    const V mcc = solved ? -dot : (V)(0.0);
    const M valid = solved & (mcc > (V)(0.0));
    const M tv = act & valid;  // the lanes that evaluate a candidate step
    const M inv = act & ~valid;
    for (int l = 0; l < L; ++l) {
      if (inv[l] && ++invalid[l] >= 5) act[l] = 0;
      if (tv[l]) invalid[l] = 0;
    }
    const M shrink_inv = inv & act;
    radius = shrink_inv ? radius / decrease : radius;
    decrease = shrink_inv ? decrease * (V)(2.0) : decrease;
    M acc = (M)(0);  // rho > 1e-3: the step is taken
    V rho = (V)(0.0);
    if (vany<L>(tv)) {
      V delta[6], cand[7], ccost = (V)(0.0);
      for (int j = 0; j < 6; ++j) delta[j] = step[j] * scale[j];
      plus7_v<L>(x, delta, cand, tv);
      const M cok = lm_eval_v<L, false>(D, cand, tv, ccost, rc, nullptr);
      ccost = (tv & ~cok) ? (V)(DBL_MAX) : ccost;
      V sn = (V)(0.0);
      for (int i = 0; i < 7; ++i) sn += (x[i] - cand[i]) * (x[i] - cand[i]);
      sn = vsqrt<L>(sn);
      const M stop1 = tv & (sn <= (V)(1e-8) * (x_norm + (V)(1e-8)));
      const M stop2 = tv & ~stop1 & (__builtin_elementwise_abs(cost - ccost) <= (V)(1e-6) * cost);
      act = act & ~stop1 & ~stop2;
      const M go = tv & ~stop1 & ~stop2;
      rho = (cost - ccost) / mcc;
      acc = go & (rho > (V)(1e-3));
      const M rej = go & ~acc;
      radius = rej ? radius / decrease : radius;
      decrease = rej ? decrease * (V)(2.0) : decrease;
      for (int i = 0; i < 7; ++i) x[i] = acc ? cand[i] : x[i];
      x_norm = acc ? lb_norm7<L>(x) : x_norm;
      if (vany<L>(acc)) {
        const M aok = lm_eval_v<L, true>(D, x, acc, cost, r, J);
        act = act & ~(acc & ~aok);
        acc = acc & aok;
        lb_finish<L>(D, x, r, J, scale, gmax, acc);
      }
    }
    for (int l = 0; l < L; ++l) {
      if (!acc[l]) continue;
      const double rad = radius[l] / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rho[l] - 1.0, 3));
      radius[l] = std::min(1e16, rad);
      decrease[l] = 2.0;
    }
    const M successful = acc;
    reuse = reuse & ~acc;
    const M better = act & successful & (cost < min_cost);
    min_cost = better ? cost : min_cost;
    for (int l = 0; l < L; ++l) {
      if (better[l] && l < n)
        for (int i = 0; i < 7; ++i) best[l][i] = x[i][l];
      if (act[l] && (iteration[l] >= 50 || (successful[l] && gmax[l] <= 1e-10) || radius[l] <= 1e-32)) act[l] = 0;
    }
  }
}

__attribute__((target("avx512f,avx512dq,avx512vl,avx2,bmi2"))) void lm_solve_x8(const float* const* pf, const int* P,
                                                                               int n, double (*best)[7]) {
  lm_solve_v<8>(pf, P, n, best);
}
__attribute__((target("avx2,bmi2"))) void lm_solve_x4(const float* const* pf, const int* P, int n,
                                                    double (*best)[7]) {
  lm_solve_v<4>(pf, P, n, best);
}

int lm_lanes_detect() {
  __builtin_cpu_init();
  if (__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") && __builtin_cpu_supports("avx512vl"))
    return 8;
  if (__builtin_cpu_supports("avx2")) return 4;
  return 1;
}

}  // namespace

int lm_batch_lanes() {
  static const int lanes = lm_lanes_detect();
  return lanes;
}

void lm_solve_batch(const float* const* pf, const int* P, int n, double (*best)[7], int lanes) {
  if (lanes <= 0) lanes = lm_batch_lanes();
  for (int i = 0; i < n; ++i)
    if (P[i] > LB_MAXP) throw std::length_error("lm_solve: too many plane pairs");
  for (int i0 = 0; i0 < n;) {
    const int k = lanes >= 4 ? std::min(n - i0, lanes) : 1;
    if (lanes >= 8) lm_solve_x8(pf + i0, P + i0, k, best + i0);
    else if (lanes >= 4) lm_solve_x4(pf + i0, P + i0, k, best + i0);
    else lm_solve(pf[i0], P[i0], best[i0]);
    i0 += k;
  }
}

}  // namespace fccf

extern "C" int fccf_debug_lm_batch(const float* pairs, const int32_t* P, int32_t n, int32_t lanes, double* best) {
  if (n < 0 || (n && (!pairs || !P || !best)) || lanes < 0) return FCCF_E_ARG;
  if (lanes == 0) lanes = fccf::lm_batch_lanes();
  __builtin_cpu_init();
  if ((lanes >= 8 && !(__builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512dq") &&
                       __builtin_cpu_supports("avx512vl"))) ||
      (lanes >= 4 && !__builtin_cpu_supports("avx2")))
    return FCCF_E_ARG;
  std::vector<const float*> pf((size_t)n);
  size_t off = 0;
  for (int i = 0; i < n; ++i) {
    if (P[i] < 0 || P[i] > fccf::LB_MAXP_PUBLIC) return FCCF_E_ARG;
    pf[(size_t)i] = pairs + 13 * off;
    off += (size_t)P[i];
  }
  fccf::lm_solve_batch(pf.data(), P, n, reinterpret_cast<double (*)[7]>(best), lanes >= 8 ? 8 : (lanes >= 4 ? 4 : 1));
  return FCCF_OK;
}
#endif  // __HIP_DEVICE_COMPILE__
