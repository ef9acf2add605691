// exactsum.h — exact emulation of a left-to-right float32 sum, in parallel.
//
// The reference computes several sums as s = ((0 + x0) + x1) + ... in float
// (pcl::compute3DCentroid, FCCF.cpp:473; fine_verify's similar_num, :830-835).  The
// bits of s depend on every intermediate rounding, so the GPU must reproduce the
// sequence exactly.  Within one binade the sequence is translation-equivariant:
// if s is a multiple of the quantum u = 2^(E-23) and the exact partial r = s + x
// lies in binade E (2^E <= |r| < 2^(E+1)), then
//      fl(s + x) = s + q*u,  q = RNE(x/u) with ties broken towards even s/u + q.
// A run of inputs is therefore summarised, for a hypothesis (E, parity p of s/u),
// by Q = sum of q and the integer envelope [lo, hi] of Q_k + floor(x_k/u) (units
// of u); "every partial of this run stays in binade E" is then a pure integer
// test on the actual start M = s/u.  Summaries of consecutive runs compose
// (xs_compose is associative), so a wave reduces a 256-input chunk in O(log)
// depth, and one ordered wave scan composes 64 chunk summaries.  Hypotheses cover
// the 3 binades around a double-precision prefix prediction.  A short serial
// chain then applies up to 64 chunks (16384 inputs) per scan and replays with
// plain float adds a chunk that does not validate (binade crossings,
// zero/subnormal starts, non-finite inputs).  XS_G (64-chunk groups) survives
// only in the host fuzz model (tests/xs_fuzz.cpp): any grouping composes.
// Result bits are identical to the naive loop (tests/test_exactsum.py fuzzes it).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "fccf_math.h"

namespace fccf {

constexpr int XS_L = 256;   // inputs per chunk (one wave x 4)
constexpr int XS_G = 64;    // chunks per group
constexpr int XS_NE = 3;    // binade hypotheses per table: Ebase, Ebase+1, Ebase+2
constexpr int32_t XS_INF = 1 << 30;             // empty-envelope sentinel
constexpr int32_t XS_LIM = 1 << 26;             // |Q|, |lo|, |hi| of any applicable summary stay below
constexpr double XS_YMAX = 33554432.0;          // 2^25: a step this large always leaves binade E
constexpr int XS_NOE = -100000;                 // "no prediction" Ebase

// Summary of a run under one binade E, for start parity 0 / 1.  A summary can only
// validate at a start |M| < 2^24 if every envelope bound and Q is below 2^26 in
// magnitude, so anything larger is recorded as "bad" and int32 suffices.
struct XsSum {
  int32_t Q[2], lo[2], hi[2];
  int32_t ok, pad;
};

FH XsSum xs_identity() {
  XsSum s;
  for (int p = 0; p < 2; ++p) { s.Q[p] = 0; s.lo[p] = XS_INF; s.hi[p] = -XS_INF; }
  s.ok = 1;
  s.pad = 0;
  return s;
}

FH XsSum xs_bad() {
  XsSum s = xs_identity();
  s.ok = 0;
  return s;
}

// one input x under binade E (inv_u = 2^(23-E)); x/u is exact in double
FH XsSum xs_elem(float x, double inv_u) {
  if (!isfinite(x)) return xs_bad();
  const double y = (double)x * inv_u;
  if (!(fabs(y) < XS_YMAX)) return xs_bad();
  const double fl = floor(y);
  const int32_t f = (int32_t)fl;
  const double fr = y - fl;  // exact
  XsSum s;
  for (int p = 0; p < 2; ++p) {
    int32_t q;
    if (fr < 0.5) q = f;
    else if (fr > 0.5) q = f + 1;
    else q = ((p + f) & 1) ? f + 1 : f;  // tie: the new s/u is even
    s.Q[p] = q;
    s.lo[p] = f;
    s.hi[p] = f;
  }
  s.ok = 1;
  s.pad = 0;
  return s;
}

// a[p & 1] as a mask blend (a `p ? a[1] : a[0]` select is folded back into an
// indexed load, which sends the whole struct to scratch memory)
FH int32_t xs_sel(const int32_t a[2], int64_t p) {
  const int32_t a0 = a[0], a1 = a[1], m = -(int32_t)(p & 1);
  return a0 ^ ((a0 ^ a1) & m);
}

// run a then run b
FH XsSum xs_compose(const XsSum& a, const XsSum& b) {
  XsSum r;
  r.pad = 0;
  int ok = a.ok & b.ok;
  for (int p = 0; p < 2; ++p) {
    const int32_t qa = a.Q[p];
    const int32_t pb = p + qa;
    const int32_t q = qa + xs_sel(b.Q, pb);
    const int32_t blo = xs_sel(b.lo, pb), bhi = xs_sel(b.hi, pb);
    const int32_t bl = blo == XS_INF ? XS_INF : qa + blo;
    const int32_t bh = bhi == -XS_INF ? -XS_INF : qa + bhi;
    const int32_t lo = a.lo[p] < bl ? a.lo[p] : bl;
    const int32_t hi = a.hi[p] > bh ? a.hi[p] : bh;
    // inputs are within +-2^26 (or sentinels), so nothing above overflows int32
    ok &= (q > -XS_LIM && q < XS_LIM) & (lo == XS_INF || lo > -XS_LIM) & (hi == -XS_INF || hi < XS_LIM);
    r.Q[p] = q;
    r.lo[p] = lo;
    r.hi[p] = hi;
  }
  if (!ok) return xs_bad();
  r.ok = 1;
  return r;
}

// c ? b : a field by field, as mask blends (keeps tables in registers)
FH XsSum xs_blend(const XsSum& a, const XsSum& b, bool c) {
  const int32_t m = -(int32_t)c;
  XsSum r;
  for (int p = 0; p < 2; ++p) {
    r.Q[p] = a.Q[p] ^ ((a.Q[p] ^ b.Q[p]) & m);
    r.lo[p] = a.lo[p] ^ ((a.lo[p] ^ b.lo[p]) & m);
    r.hi[p] = a.hi[p] ^ ((a.hi[p] ^ b.hi[p]) & m);
  }
  r.ok = a.ok ^ ((a.ok ^ b.ok) & m);
  r.pad = 0;
  return r;
}

// Tables of one unit (chunk or group): summaries under Eb, Eb+1, Eb+2.
struct XsTab3 {
  XsSum t0, t1, t2;
  int32_t Eb;
};

// the summary of unit T under binade E (bad if E is not covered)
FH XsSum xs_pick(const XsTab3& T, int E) {
  const int h = E - T.Eb;
  if (T.Eb == XS_NOE || h < 0 || h > 2) return xs_bad();
  return xs_blend(xs_blend(T.t0, T.t1, h == 1), T.t2, h == 2);
}

// binade exponent and signed integer mantissa M (s = M * 2^(E-23)) of a normal float
FH bool xs_decompose(float s, int* E, int64_t* M) {
  uint32_t b;
  __builtin_memcpy(&b, &s, 4);
  const int ex = (int)((b >> 23) & 0xFF);
  if (ex == 0 || ex == 0xFF) return false;  // zero/subnormal/inf/nan: no binade hypothesis
  *E = ex - 127;
  const int64_t m = (int64_t)((b & 0x7FFFFFu) | 0x800000u);
  *M = (b >> 31) ? -m : m;
  return true;
}

// Does summary h (parity p = M & 1) apply at start M: every partial r_k/u in
// [M + lo, M + hi + 1) stays inside binade E on M's side of zero?
FH bool xs_valid(const XsSum& h, int64_t M) {
  if (!h.ok) return false;
  const int32_t hl = xs_sel(h.lo, M), hh = xs_sel(h.hi, M);
  if (hl == XS_INF) return true;  // empty run
  const int64_t lo = M + hl, hi = M + hh;
  if (M > 0) return lo >= ((int64_t)1 << 23) && hi + 1 <= ((int64_t)1 << 24);
  return hi + 1 <= -((int64_t)1 << 23) && lo >= -((int64_t)1 << 24) + 1;
}

// The same test for one unit at its own start Me (int64, any sign; the side of
// zero is M's, the start of the whole scan): the composed run is valid iff every
// unit is valid at its own start, because a valid unit ends inside the binade
// (Q lies in [lo, hi + 1]).  The device chain uses this form (k_xs_chain).
FH bool xs_valid_unit(const XsSum& h, int64_t Me, bool pos) {
  if (!h.ok) return false;
  const int32_t hl = xs_sel(h.lo, Me), hh = xs_sel(h.hi, Me);
  if (hl == XS_INF) return true;
  const int64_t lo = Me + hl, hi = Me + hh;
  if (pos) return lo >= ((int64_t)1 << 23) && hi + 1 <= ((int64_t)1 << 24);
  return hi + 1 <= -((int64_t)1 << 23) && lo >= -((int64_t)1 << 24) + 1;
}

// end of the run: (M + Q) u, exact (it is the float the last rounding produced)
FH float xs_apply(const XsSum& h, int64_t M, int E) {
  return (float)ldexp((double)(M + xs_sel(h.Q, M)), E - 23);
}

// Ebase (= predicted binade - 1) of a run starting at prefix value pre;
// XS_NOE when the prefix is too close to zero to be useful.
FH int xs_predict(double pre) {
  const double a = fabs(pre);
  if (!(a >= 1.1754943508222875e-38) || !(a < 3.0e38)) return XS_NOE;
  int e;
  frexp(a, &e);  // a = f * 2^e, f in [0.5, 1)
  return e - 2;
}

// Device scratch of exact_sum (devprim.h): per row (problem x component) NC chunk
// tables.
struct XsBufs {
  double* pre;     // rows x (NC + 1): chunk sums, then exclusive prefix
  XsSum* ctab;     // rows x NC x XS_NE
  int32_t* cE;     // rows x NC: Ebase per chunk
  uint32_t NC;
  int rows;
};

// Summary of the run x[0..n) under binade E (host / reference walk).
FH XsSum xs_run(const float* x, int64_t stride, int n, int E) {
  const double inv_u = ldexp(1.0, 23 - E);
  XsSum s = xs_identity();
  for (int k = 0; k < n; ++k) s = xs_compose(s, xs_elem(x[k * stride], inv_u));
  return s;
}

}  // namespace fccf
