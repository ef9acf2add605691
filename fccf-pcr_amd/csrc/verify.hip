// verify.hip — f1: quick_verify with its Ceres-1.14 LM refinement
// on the GPU, one wave per candidate transform, every candidate of all three types
// in one launch.  Reference: quick_verify FCCF.cpp:680-783, ceres_refine :210-249,
// LidarPlaneFactor :178-208; the host form is host_stages.cpp (quick_verify,
// lm_solve), whose operations and orders this file follows one for one.
//
// Mapping: lane i < |F1| finds source plane i's best partner (the pair records are
// compacted in i order by ballot); the LM keeps J, r and the QR workspace in LDS;
// lane b evaluates residual block b; lane j owns column j in the column sums
// (J^T J, J^T r, the QR's column dots), each summed over ascending rows as the host
// does; every reduction the host performs left to right is performed left to right
// by one lane here.  Control flow is uniform across the wave.
//
// Transcendentals: the quaternion plus (EigenQuaternionParameterization) calls double
// sin/cos, and the trust-region update calls pow(2 rho - 1, 3).  The device has no
// libm with glibc's bits, so these are evaluated in double-double and rounded once
// (correctly rounded).  glibc 2.35's sin/cos/pow agree with the correctly rounded
// value on 99.95% / 99.99% / 99.91% of random arguments (DESIGN.md §5b measures the
// disagreement rate); where they disagree, a double differs in its last bit and the
// float outputs almost always still agree.  Arguments the reduction does not cover
// (|x| >= 2^20) set the item's status and the host redoes that candidate.
#define KT_TU 11  // ktrace.h source tag
#include <float.h>

#include "ktrace.h"
#include "kernels.h"
#include "match.h"

namespace fccf {
namespace {

// ---------------------------------------------------------------- double-double
struct dd {
  double hi, lo;
};
__device__ __forceinline__ dd two_sum(double a, double b) {
  const double s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
__device__ __forceinline__ dd quick_two_sum(double a, double b) {
  const double s = a + b;
  return {s, b - (s - a)};
}
__device__ __forceinline__ dd two_prod(double a, double b) {
  const double p = a * b;
  return {p, fma(a, b, -p)};
}
__device__ __forceinline__ dd dd_add(dd a, dd b) {
  dd s = two_sum(a.hi, b.hi);
  const dd t = two_sum(a.lo, b.lo);
  s.lo = s.lo + t.hi;
  s = quick_two_sum(s.hi, s.lo);
  s.lo = s.lo + t.lo;
  return quick_two_sum(s.hi, s.lo);
}
__device__ __forceinline__ dd dd_mul(dd a, dd b) {
  dd p = two_prod(a.hi, b.hi);
  p.lo = p.lo + (a.hi * b.lo + a.lo * b.hi);
  return quick_two_sum(p.hi, p.lo);
}

// 1/n! for n = 0..30 as double-double (generated with 80-digit decimal arithmetic)
__constant__ double kInvFact[31][2] = {
    {1.0, 0.0}, {1.0, 0.0}, {0x1.0000000000000p-1, 0.0},
    {0x1.5555555555555p-3, 0x1.5555555555555p-57}, {0x1.5555555555555p-5, 0x1.5555555555555p-59},
    {0x1.1111111111111p-7, 0x1.1111111111111p-63}, {0x1.6c16c16c16c17p-10, -0x1.f49f49f49f49fp-65},
    {0x1.a01a01a01a01ap-13, 0x1.a01a01a01a01ap-73}, {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76},
    {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73}, {0x1.27e4fb7789f5cp-22, 0x1.cbbc05b4fa99ap-76},
    {0x1.ae64567f544e4p-26, -0x1.c062e06d1f209p-80}, {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83},
    {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87}, {0x1.93974a8c07c9dp-37, 0x1.05d6f8a2efd1fp-92},
    {0x1.ae7f3e733b81fp-41, 0x1.1d8656b0ee8cbp-97}, {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101},
    {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103}, {0x1.6827863b97d97p-53, 0x1.eec01221a8b0bp-107},
    {0x1.2f49b46814157p-57, 0x1.2650f61dbdcb4p-112}, {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120},
    {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120}, {0x1.0ce396db7f853p-70, -0x1.aebcdbd20331cp-124},
    {0x1.761b41316381ap-75, -0x1.3423c7d91404fp-130}, {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135},
    {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139}, {0x1.88e85fc6a4e5ap-89, -0x1.71c37ebd16540p-143},
    {0x1.d1ab1c2dccea3p-94, 0x1.054d0c78aea14p-149}, {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153},
    {0x1.259f98b4358adp-103, 0x1.eaf8c39dd9bc5p-157}, {0x1.3932c5047d60ep-108, 0x1.832b7b530a627p-162}};

// sin and cos of x, correctly rounded (double-double evaluation, one final rounding).
// Cody-Waite reduction by pi/2 split in three doubles; false when |x| >= 2^20.
__device__ bool cr_sincos(double x, double* sn, double* cs) {
  if (!(fabs(x) < 1048576.0)) return false;
  const double P1 = 0x1.921fb54442d18p+0, P2 = 0x1.1a62633145c07p-54, P3 = -0x1.f1976b7ed8fbcp-110;
  const double k = rint(x * 0x1.45f306dc9c883p-1);
  const dd p1 = two_prod(k, P1), p2 = two_prod(k, P2), p3 = two_prod(k, P3);
  dd r = dd_add(dd{x, 0.0}, dd{-p1.hi, -p1.lo});
  r = dd_add(r, dd{-p2.hi, -p2.lo});
  r = dd_add(r, dd{-p3.hi, -p3.lo});
  const dd r2 = dd_mul(r, r);
  // sin(r) = r * sum (-1)^k r^2k / (2k+1)!, cos(r) = sum (-1)^k r^2k / (2k)!  (Horner in r^2)
  dd ps = {kInvFact[29][0], kInvFact[29][1]};
  for (int n = 27; n >= 1; n -= 2) {
    const double sg = ((n >> 1) & 1) ? -1.0 : 1.0;
    ps = dd_add(dd{sg * kInvFact[n][0], sg * kInvFact[n][1]}, dd_mul(r2, ps));
  }
  const dd sr = dd_mul(r, ps);
  dd pc = {kInvFact[30][0], kInvFact[30][1]};  // (-1)^15 / 30! -> negated below
  pc.hi = -pc.hi;
  pc.lo = -pc.lo;
  for (int n = 28; n >= 0; n -= 2) {
    const double sg = ((n >> 1) & 1) ? -1.0 : 1.0;
    pc = dd_add(dd{sg * kInvFact[n][0], sg * kInvFact[n][1]}, dd_mul(r2, pc));
  }
  const int q = (int)(((long long)k % 4 + 4) % 4);
  const double s = sr.hi + sr.lo, c = pc.hi + pc.lo;
  *sn = q == 0 ? s : q == 1 ? c : q == 2 ? -s : -c;
  *cs = q == 0 ? c : q == 1 ? -s : q == 2 ? -c : s;
  return true;
}
// the ps polynomial's first sign: n = 29 -> k = 14, (+); the loop applies (-1)^((n-1)/2)
// through ((n >> 1) & 1), which is the same parity for odd n.

// y^3 correctly rounded
__device__ __forceinline__ double cr_cube(double y) {
  const dd y2 = two_prod(y, y);
  const dd y3 = dd_mul(y2, dd{y, 0.0});
  return y3.hi + y3.lo;
}

// ---------------------------------------------------------------- the host LM's helpers
__device__ __forceinline__ void crossd(const double a[3], const double b[3], double r[3]) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}
__device__ __forceinline__ void qmul(const double a[4], const double b[4], double r[4]) {
  const double ax = a[0], ay = a[1], az = a[2], aw = a[3], bx = b[0], by = b[1], bz = b[2], bw = b[3];
  r[0] = (aw * bx + ay * bz) - (az * by - ax * bw);
  r[1] = (aw * by + ay * bw) + (az * bx - ax * bz);
  r[2] = (aw * bz - ay * bx) + (az * bw + ax * by);
  r[3] = (aw * bw - ay * by) - (az * bz + ax * bx);
}
// false: the argument left the reduction's range (status set by the caller)
__device__ __forceinline__ bool plus7(const double x[7], const double d[6], double o[7]) {
  const double nd = sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  bool ok = true;
  if (nd > 0.0) {
    double sn = 0.0, cs = 1.0;
    ok = cr_sincos(nd, &sn, &cs);
    const double s = sn / nd;
    const double dq[4] = {s * d[0], s * d[1], s * d[2], cs};
    qmul(dq, x, o);
  } else {
    o[0] = x[0]; o[1] = x[1]; o[2] = x[2]; o[3] = x[3];
  }
  for (int i = 0; i < 3; ++i) o[4 + i] = x[4 + i] + d[3 + i];
  return ok;
}
__device__ __forceinline__ void rotq(const double q[4], const double v[3], double f[3], double (*J)[4]) {
  const double u[3] = {q[0], q[1], q[2]}, w = q[3];
  double a[3], uv[3], c[3];
  crossd(u, v, a);
  uv[0] = a[0] + a[0]; uv[1] = a[1] + a[1]; uv[2] = a[2] + a[2];
  crossd(u, uv, c);
  for (int i = 0; i < 3; ++i) f[i] = (v[i] + w * uv[i]) + c[i];
  if (!J) return;
  for (int k = 0; k < 3; ++k) {
    double e[3] = {0, 0, 0};
    e[k] = 1.0;
    double ekv[3], eka[3], uekv[3];
    crossd(e, v, ekv);
    crossd(e, a, eka);
    crossd(u, ekv, uekv);
    for (int i = 0; i < 3; ++i) J[i][k] = 2.0 * w * ekv[i] + 2.0 * (eka[i] + uekv[i]);
  }
  for (int i = 0; i < 3; ++i) J[i][3] = uv[i];
}

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

constexpr int LM_MAXP = MAX_PLANES;        // plane pairs (one per source plane)
constexpr int LM_MAXM = 2 * LM_MAXP;       // residual rows
constexpr int LM_LD = LM_MAXM + 6;

struct VerLds {
  double J[LM_MAXM * 6];
  double r[LM_MAXM], rc[LM_MAXM], mr[LM_MAXM];
  double C[7][LM_LD];
  double col[8];                 // per-column results broadcast through LDS
  float pf[LM_MAXP * 13];        // plane pair records (FCCF.cpp:735-741 order)
  float c2[MAX_PLANES * 3], n2[MAX_PLANES * 3];
  uint32_t bad;
};

// LidarPlaneFactor residuals (and the local 6-column Jacobian when withJ), lane b for
// block b; cost summed over blocks in order by lane 0.  False (uniform) on a
// non-finite residual or Jacobian entry, as the host's early return.
__device__ bool lm_eval(VerLds& S, const float* pf, int P, const double x[7], double* cost, double* r, bool withJ) {
  const uint32_t lane = threadIdx.x;
  const double* q = x;
  const double* t = x + 4;
  bool okl = true;
  if ((int)lane < P) {
    const int b = (int)lane;
    const double Pj[4][3] = {{q[3], q[2], -q[1]}, {-q[2], q[3], q[0]}, {q[1], -q[0], q[3]}, {-q[0], -q[1], -q[2]}};
    const float* s = pf + 13 * b;
    const double p1[3] = {s[0], s[1], s[2]}, n1[3] = {s[3], s[4], s[5]};
    const double p2[3] = {s[6], s[7], s[8]}, n2[3] = {s[9], s[10], s[11]};
    const double w = s[12];
    double n2r[3], p2r[3], Jn[3][4], Jp[3][4];
    rotq(q, n2, n2r, withJ ? Jn : nullptr);
    rotq(q, p2, p2r, withJ ? Jp : nullptr);
    for (int i = 0; i < 3; ++i) p2r[i] = p2r[i] + t[i];
    double cr[3];
    crossd(n1, n2r, cr);
    const double nrm = sqrt((cr[0] * cr[0] + cr[1] * cr[1]) + cr[2] * cr[2]);
    const double d = ((n1[0] * p1[0] + n1[1] * p1[1]) + n1[2] * p1[2]) -
                     ((n2r[0] * p2r[0] + n2r[1] * p2r[1]) + n2r[2] * p2r[2]);
    const double r0 = w * nrm, r1 = w * sqrt(d * d);
    r[2 * b] = r0;
    r[2 * b + 1] = r1;
    okl = isfinite(r0) && isfinite(r1);
    if (withJ) {
      double g0[7] = {0, 0, 0, 0, 0, 0, 0}, g1[7] = {0, 0, 0, 0, 0, 0, 0};
      for (int k = 0; k < 4; ++k) {
        const double cl[3] = {Jn[0][k], Jn[1][k], Jn[2][k]};
        double dc[3];
        crossd(n1, cl, dc);
        g0[k] = w * (((cr[0] * dc[0] + cr[1] * dc[1]) + cr[2] * dc[2]) / nrm);
        const double dd_ = -(((Jn[0][k] * p2r[0] + Jn[1][k] * p2r[1]) + Jn[2][k] * p2r[2]) +
                             ((n2r[0] * Jp[0][k] + n2r[1] * Jp[1][k]) + n2r[2] * Jp[2][k]));
        g1[k] = w * ((d * dd_) / sqrt(d * d));
      }
      for (int k = 0; k < 3; ++k) g1[4 + k] = w * ((d * -n2r[k]) / sqrt(d * d));
      double* J0 = S.J + (2 * b) * 6;
      double* J1 = S.J + (2 * b + 1) * 6;
      for (int j = 0; j < 3; ++j) {
        J0[j] = ((g0[0] * Pj[0][j] + g0[1] * Pj[1][j]) + g0[2] * Pj[2][j]) + g0[3] * Pj[3][j];
        J1[j] = ((g1[0] * Pj[0][j] + g1[1] * Pj[1][j]) + g1[2] * Pj[2][j]) + g1[3] * Pj[3][j];
        J0[3 + j] = 0.0;
        J1[3 + j] = g1[4 + j];
      }
      for (int j = 0; j < 6; ++j) okl = okl && isfinite(J0[j]) && isfinite(J1[j]);
    }
  }
  const bool ok = __ballot(!okl) == 0;
  wsync();
  double c = 0.0;
  for (int b = 0; b < P; ++b) c += 0.5 * (r[2 * b] * r[2 * b] + r[2 * b + 1] * r[2 * b + 1]);
  if (ok) *cost = c;
  return ok;
}

// per-column sums over ascending rows, lane j < 6 for column j: sum_i J[i][j] * v[i]
// (v = null: J[i][j]^2); the results land in S.col
__device__ __forceinline__ void col_sums(VerLds& S, int m, const double* v) {
  const uint32_t lane = threadIdx.x;
  if (lane < 6) {
    double s = 0.0;
    for (int i = 0; i < m; ++i) s += S.J[(size_t)i * 6 + lane] * (v ? v[i] : S.J[(size_t)i * 6 + lane]);
    S.col[lane] = s;
  }
  wsync();
}

// DENSE_QR solve of min || [A; diag(D)] y - [b; 0] || (host qr_solve's operations)
__device__ bool qr_solve(VerLds& S, int m, const double D[6], const double* b, double y[6]) {
  constexpr int n = 6;
  const uint32_t lane = threadIdx.x;
  const int M = m + n;
  for (int e = (int)lane; e < (n + 1) * LM_LD; e += 64) S.C[e / LM_LD][e % LM_LD] = 0.0;
  wsync();
  for (int e = (int)lane; e < m * n; e += 64) S.C[e % n][e / n] = S.J[e];
  if ((int)lane < n) S.C[lane][m + lane] = D[lane];
  for (int i = (int)lane; i < m; i += 64) S.C[n][i] = b[i];
  wsync();
  for (int k = 0; k < n; ++k) {
    double* ck = S.C[k];
    const double c0 = ck[k];
    double tail = 0.0;
    for (int i = k + 1; i < M; ++i) tail += ck[i] * ck[i];
    double tau, beta;
    wsync();
    if (tail <= DBL_MIN) {
      tau = 0.0;
      beta = c0;
      for (int i = k + 1 + (int)lane; i < M; i += 64) ck[i] = 0.0;
    } else {
      beta = sqrt(c0 * c0 + tail);
      if (c0 >= 0.0) beta = -beta;
      const double den = c0 - beta;
      for (int i = k + 1 + (int)lane; i < M; i += 64) ck[i] = ck[i] / den;
      tau = (beta - c0) / beta;
    }
    wsync();
    if (lane == 0) ck[k] = beta;
    // tmp[j] = sum_{i > k} v_i C[j][i] over ascending i, lane j
    double tj = 0.0;
    if ((int)lane > k && (int)lane <= n) {
      const double* cj = S.C[lane];
      for (int i = k + 1; i < M; ++i) tj += ck[i] * cj[i];
    }
    wsync();
    if ((int)lane > k && (int)lane <= n) {
      double* cj = S.C[lane];
      const double t = tj + cj[k];
      cj[k] = cj[k] - tau * t;
      for (int i = k + 1; i < M; ++i) cj[i] = cj[i] - tau * ck[i] * t;
    }
    wsync();
  }
  for (int i = 0; i < n; ++i) y[i] = S.C[n][i];
  for (int k = n - 1; k >= 0; --k) {
    y[k] = y[k] / S.C[k][k];
    for (int i = 0; i < k; ++i) y[i] = y[i] - y[k] * S.C[k][i];
  }
  bool ok = true;
  for (int i = 0; i < n; ++i) ok = ok && isfinite(y[i]);
  return ok;
}

__device__ __forceinline__ double dmax(double a, double b) { return (a < b) ? b : a; }  // std::max
__device__ __forceinline__ double dmin(double a, double b) { return (b < a) ? b : a; }  // std::min

// Host lm_solve (TrustRegionMinimizer + LevenbergMarquardtStrategy, Ceres 1.14 defaults).
// Returns false when a sin/cos argument left the reduction's range.
__device__ bool lm_solve(VerLds& S, const float* pf, int P, double best[7]) {
  const uint32_t lane = threadIdx.x;
  const int m = 2 * P;
  double x[7] = {0, 0, 0, 1, 0, 0, 0};
  for (int i = 0; i < 7; ++i) best[i] = x[i];
  bool range_ok = true;
  double cost;
  if (!lm_eval(S, pf, P, x, &cost, S.r, true)) return true;
  double scale[6], gmax = 0.0;
  col_sums(S, m, nullptr);
  for (int j = 0; j < 6; ++j) scale[j] = 1.0 / (1.0 + sqrt(S.col[j]));
  wsync();
  auto finish = [&]() {
    col_sums(S, m, S.r);
    double ng[6], xp[7];
    for (int j = 0; j < 6; ++j) ng[j] = -S.col[j];
    range_ok = plus7(x, ng, xp) && range_ok;
    double mx = 0.0;
    for (int j = 0; j < 7; ++j) mx = dmax(mx, fabs(x[j] - xp[j]));
    gmax = mx;
    wsync();
    for (int e = (int)lane; e < m * 6; e += 64) S.J[e] *= scale[e % 6];
    wsync();
  };
  finish();
  double min_cost = cost;
  auto norm7 = [](const double* v) {
    double s = 0.0;
    for (int i = 0; i < 7; ++i) s += v[i] * v[i];
    return sqrt(s);
  };
  double x_norm = norm7(x);
  double radius = 1e4, decrease = 2.0, diag[6];
  bool reuse = false;
  int iteration = 0, invalid = 0;
  if (gmax <= 1e-10) return range_ok;
  while (true) {
    ++iteration;
    bool successful = false;
    if (!reuse) {
      col_sums(S, m, nullptr);
      for (int j = 0; j < 6; ++j) diag[j] = dmin(dmax(S.col[j], 1e-6), 1e32);
      wsync();
    }
    double D[6], y[6], step[6];
    for (int j = 0; j < 6; ++j) D[j] = sqrt(diag[j] / radius);
    const bool solved = qr_solve(S, m, D, S.r, y);
    reuse = true;
    bool valid = false;
    double mcc = 0.0;
    if (solved) {
      for (int j = 0; j < 6; ++j) step[j] = -y[j];
      if ((int)lane < m) {
        double v = 0.0;
        for (int j = 0; j < 6; ++j) v += S.J[(size_t)lane * 6 + j] * step[j];
        S.mr[lane] = v;
      }
      wsync();
      double dot = 0.0;
      for (int i = 0; i < m; ++i) dot += S.mr[i] * (S.r[i] + S.mr[i] / 2.0);
      mcc = -dot;
      valid = mcc > 0.0;
      wsync();
    }
    if (!valid) {
      if (++invalid >= 5) return range_ok;
      radius = radius / decrease;
      decrease *= 2.0;
    } else {
      invalid = 0;
      double delta[6], cand[7];
      for (int j = 0; j < 6; ++j) delta[j] = step[j] * scale[j];
      range_ok = plus7(x, delta, cand) && range_ok;
      double ccost;
      if (!lm_eval(S, pf, P, cand, &ccost, S.rc, false)) ccost = DBL_MAX;
      double sn = 0.0;
      for (int i = 0; i < 7; ++i) sn += (x[i] - cand[i]) * (x[i] - cand[i]);
      sn = sqrt(sn);
      if (sn <= 1e-8 * (x_norm + 1e-8)) return range_ok;
      if (fabs(cost - ccost) <= 1e-6 * cost) return range_ok;
      const double rho = (cost - ccost) / mcc;
      if (rho > 1e-3) {
        for (int i = 0; i < 7; ++i) x[i] = cand[i];
        x_norm = norm7(x);
        wsync();
        if (!lm_eval(S, pf, P, x, &cost, S.r, true)) return range_ok;
        finish();
        successful = true;
        radius = radius / dmax(1.0 / 3.0, 1.0 - cr_cube(2.0 * rho - 1.0));
        radius = dmin(1e16, radius);
        decrease = 2.0;
        reuse = false;
      } else {
        radius = radius / decrease;
        decrease *= 2.0;
      }
    }
    if (successful && cost < min_cost) {
      min_cost = cost;
      for (int i = 0; i < 7; ++i) best[i] = x[i];
    }
    if (iteration >= 50) return range_ok;
    if (successful && gmax <= 1e-10) return range_ok;
    if (radius <= 1e-32) return range_ok;
  }
}

// One wave per candidate: T from its quaternion record, quick_verify's pairing, the
// LM refinement (T <- dT * T), and the score (FCCF.cpp:680-783).
__global__ void __launch_bounds__(64) k_verify(VerifyIn in, VerifyOut out) {
  KT();
  __shared__ VerLds S;
  const uint32_t lane = threadIdx.x;
  const int item = (int)blockIdx.x;
  const QTd qt = in.q[item];
  m44 T = eye44();
  {
    const m33 R = rot_from_quat(quatf{qt.qw, qt.qx, qt.qy, qt.qz});
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) T.m[i][j] = R.m[i][j];
    T.m[0][3] = qt.tx; T.m[1][3] = qt.ty; T.m[2][3] = qt.tz;
  }
  const MatchIn* M = in.planes;
  const int nF1 = M->nF1, nF2 = M->nF2;
  if ((int)lane < nF2) {
    const MPlane& f = M->F2[lane];
    const f3 c = tf_se3(T, f.c[0], f.c[1], f.c[2]);
    const f3 nn = tf_so3(T, f.n[0], f.n[1], f.n[2]);
    S.c2[3 * lane] = c.x; S.c2[3 * lane + 1] = c.y; S.c2[3 * lane + 2] = c.z;
    S.n2[3 * lane] = nn.x; S.n2[3 * lane + 1] = nn.y; S.n2[3 * lane + 2] = nn.z;
  }
  wsync();
  bool find = false;
  float rec[13];
  if ((int)lane < nF1) {
    const MPlane& a = M->F1[lane];
    int best = 0;
    float best_imp = 0, best_score = 0;
    for (int j = 0; j < nF2; ++j) {
      const float nx = S.n2[3 * j], ny = S.n2[3 * j + 1], nz = S.n2[3 * j + 2];
      const bool ang_ok = angle_lt(normal_cos(a.n[0], a.n[1], a.n[2], nx, ny, nz), in.qcut);
      const float d1 = (float)dot3d(a.n[0], a.n[1], a.n[2], a.c[0], a.c[1], a.c[2]);
      const float d2 = (float)dot3d(nx, ny, nz, S.c2[3 * j], S.c2[3 * j + 1], S.c2[3 * j + 2]);
      const float dist = fabsf(d1 - d2);
      if (ang_ok && dist < in.dist_thr) {
        find = true;
        const float s1 = a.fps, s2 = M->F2[j].fps;
        const float mn = s1 < s2 ? s1 : s2, mx = s1 > s2 ? s1 : s2;
        const float sc = mn / mx;
        const float imp = (2 * mn) / (float)in.fs12;
        if (sc > best_score) { best_imp = imp; best_score = sc; best = j; }
      }
    }
    const float r13[13] = {a.c[0], a.c[1], a.c[2], a.n[0], a.n[1], a.n[2], S.c2[3 * best], S.c2[3 * best + 1],
                           S.c2[3 * best + 2], S.n2[3 * best], S.n2[3 * best + 1], S.n2[3 * best + 2], best_imp};
    for (int k = 0; k < 13; ++k) rec[k] = r13[k];
  }
  const uint64_t fm = __ballot(find);
  const int np = (int)__popcll(fm);
  if (find) {
    const uint32_t slot = mbcnt(fm);
    for (int k = 0; k < 13; ++k) S.pf[13 * slot + k] = rec[k];
  }
  wsync();
  uint32_t status = 0;
  if ((float)np >= in.required) {
    double b[7];
    if (!lm_solve(S, S.pf, np, b)) status = 1;
    const m33 R = rot_from_quat(quatf{(float)b[3], (float)b[0], (float)b[1], (float)b[2]});
    m44 dT = eye44();
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) dT.m[i][j] = R.m[i][j];
    dT.m[0][3] = (float)b[4]; dT.m[1][3] = (float)b[5]; dT.m[2][3] = (float)b[6];
    T = mul44(dT, T);
  }
  float score = 0;
  for (int k = 0; k < np; ++k) score = score + S.pf[13 * k + 12];
  if (lane < 16) out.T[16 * (size_t)item + lane] = T.m[lane >> 2][lane & 3];
  if (lane == 0) {
    out.score[item] = score;
    out.npairs[item] = np;
    out.status[item] = status;
  }
}

// debug probe: the device's correctly rounded sin/cos (status 0 where out of range)
__global__ void k_sincos_probe(const double* x, int n, double* s, double* c, uint32_t* ok) {
  const int i = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  if (i >= n) return;
  double a = 0.0, b = 0.0;
  ok[i] = cr_sincos(x[i], &a, &b) ? 1u : 0u;
  s[i] = a;
  c[i] = b;
}

}  // namespace

void sincos_probe(const double* x, int n, double* s, double* c, uint32_t* ok, hipStream_t st) {
  if (n > 0) k_sincos_probe<<<(n + 255) / 256, 256, 0, st>>>(x, n, s, c, ok);
}

void verify_device(const VerifyIn& in, int n, const VerifyOut& out, hipStream_t st) {
  if (n <= 0) return;
  k_verify<<<n, 64, 0, st>>>(in, out);
}

}  // namespace fccf
