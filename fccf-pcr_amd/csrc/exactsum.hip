// exactsum.hip — exact parallel left-to-right float32 sums (algorithm: exactsum.h).
//
// Four launches per call, all sized from device counts:
//   k_xs_csum    one wave per (problem, 256-input chunk): double chunk sums (K comps)
//   k_xs_prefix  one block per row (problem x component): exclusive double prefix
//   k_xs_chunk   one wave per chunk: 3 binade hypotheses x 2 parities, wave-composed
//   k_xs_chain   one wave per row: one ordered scan per 64-chunk window, a plain
//                replay of each chunk that crosses a binade
// The first three are bandwidth-bound streaming passes over the inputs; the chain
// costs one wave scan per window plus one scan and a 256-add replay per crossing,
// with its loads issued one or two windows ahead.
#define KT_TU 4  // ktrace.h source tag
#include "probe.h"
#include "devprim.h"
#include "exactsum.h"
#include "ctx.h"

namespace fccf {
namespace {

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  return v;
}

// Inclusive ordered scan of parity maps.  Unit l maps a start parity p to its
// quantum count Q_l[p] (and so to the end parity p + Q_l[p]); lane l ends with
// the count of units 0..l for each parity at unit 0.  Two int32 per lane per
// step instead of a whole summary: this is the chain's critical path.
// Every DPP step reads 0 where its source lane is out of range or its row is masked
// off (update_dpp's old value): 0 is the identity map (no quanta, parity kept), so no
// step needs a lane condition.
// Wrap-around in lanes past the first invalid unit is harmless (never read).
__device__ __forceinline__ void pmap_scan(uint32_t& q0, uint32_t& q1) {
  auto step = [&](uint32_t o0, uint32_t o1) {
    // earlier run o, then this run: Q[p] = o[p] + this[(p + o[p]) & 1]
    const uint32_t m0 = 0u - (o0 & 1u), m1 = 0u - ((o1 + 1u) & 1u);
    const uint32_t n0 = o0 + (q0 ^ ((q0 ^ q1) & m0));
    const uint32_t n1 = o1 + (q0 ^ ((q0 ^ q1) & m1));
    q0 = n0;
    q1 = n1;
  };
#define XS_PSTEP(CTRL, ROWS)                                                     \
  step((uint32_t)__builtin_amdgcn_update_dpp(0, (int)q0, CTRL, ROWS, 0xf, false), \
       (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q1, CTRL, ROWS, 0xf, false));
  XS_PSTEP(0x111, 0xf)  // row_shr:1
  XS_PSTEP(0x112, 0xf)  // row_shr:2
  XS_PSTEP(0x114, 0xf)  // row_shr:4
  XS_PSTEP(0x118, 0xf)  // row_shr:8
  XS_PSTEP(0x142, 0xa)  // row_bcast:15 into rows 1, 3
  XS_PSTEP(0x143, 0xc)  // row_bcast:31 into rows 2, 3
#undef XS_PSTEP
}

// parity-free form (no unit of the scan depends on the start parity; 0 is the identity)
__device__ __forceinline__ uint32_t add_scan(uint32_t q) {
  q += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x111, 0xf, 0xf, false);
  q += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x112, 0xf, 0xf, false);
  q += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x114, 0xf, 0xf, false);
  q += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x118, 0xf, 0xf, false);
  q += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x142, 0xa, 0xf, false);
  q += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)q, 0x143, 0xc, 0xf, false);
  return q;
}

// value of lane l-1 (0 in lane 0): DPP wave_shr:1
__device__ __forceinline__ uint32_t wave_shr1(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xf, 0xf, false);
}

// Inclusive ordered min / max over the wave (lane 63 ends with the total).  Lanes
// without a source read the operation's identity (INT32_MAX / INT32_MIN), so no step
// needs a lane condition.
template <bool MAX>
__device__ __forceinline__ int32_t mm_scan(int32_t q) {
  constexpr int32_t I = MAX ? INT32_MIN : INT32_MAX;
#define XS_MM(CTRL, ROWS)                                                  \
  {                                                                        \
    const int32_t o = __builtin_amdgcn_update_dpp(I, q, CTRL, ROWS, 0xf, false); \
    q = MAX ? max(q, o) : min(q, o);                                       \
  }
  XS_MM(0x111, 0xf)
  XS_MM(0x112, 0xf)
  XS_MM(0x114, 0xf)
  XS_MM(0x118, 0xf)
  XS_MM(0x142, 0xa)
  XS_MM(0x143, 0xc)
#undef XS_MM
  return q;
}

// The composition of the 64 lanes' summaries (lane 0 first), valid in lane 63.
// Instead of composing whole summaries along the scan, the quantum counts are
// scanned as parity maps, every lane shifts its envelope by its exclusive count
// (under its own start parity), and the envelopes reduce by min / max.  Same
// summary as folding xs_compose over the lanes (the bounds check differs only in
// where it rejects: any summary it accepts is exact, XS_LIM keeps int32 safe,
// since consecutive counts differ by less than 2^26).
__device__ __forceinline__ XsSum wave_total(const XsSum& a) {
  uint32_t q0 = (uint32_t)a.Q[0], q1 = (uint32_t)a.Q[1];
  pmap_scan(q0, q1);
  const uint32_t e[2] = {wave_shr1(q0), wave_shr1(q1)};
  XsSum t;
  int ok = a.ok;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int32_t ep = (int32_t)e[p];
    const int32_t alo = xs_sel(a.lo, p + ep), ahi = xs_sel(a.hi, p + ep);
    const int32_t lo = alo == XS_INF ? XS_INF : ep + alo;
    const int32_t hi = ahi == -XS_INF ? -XS_INF : ep + ahi;
    const int32_t qi = (int32_t)(p ? q1 : q0);
    ok &= (ep > -XS_LIM && ep < XS_LIM) & (qi > -XS_LIM && qi < XS_LIM) & (lo == XS_INF || lo > -XS_LIM) &
          (hi == -XS_INF || hi < XS_LIM);
    t.Q[p] = qi;
    t.lo[p] = mm_scan<false>(lo);
    t.hi[p] = mm_scan<true>(hi);
  }
  t.ok = __ballot(!ok) == 0;
  t.pad = 0;
  if (!t.ok) t = xs_bad();
  return t;
}

struct Prob {
  const float* base;  // first element of the problem
  uint32_t n, nch;
};

// Where the problems live: either one array with per-problem offsets/counts
// (off may be null), or (multi != 0) up to four separate arrays, problem b = dp[b]
// with count *cp[b] (the clouds' centroids of a cloud stage).
struct XsIn {
  const float* data;
  const uint32_t* off;
  const uint32_t* cnt;
  int multi;
  const float* dp[BMAX];
  const uint32_t* cp[BMAX];
};

template <class T>
__device__ __forceinline__ T sel4(const T (&a)[BMAX], int b) {  // a select chain, not a dynamic index
  T r = a[0];
#pragma unroll
  for (int q = 1; q < BMAX; ++q) r = b == q ? a[q] : r;
  return r;
}

__device__ __forceinline__ uint32_t prob_n(const XsIn& in, int b) {
  return in.multi ? *sel4(in.cp, b) : in.cnt[b];
}

__device__ __forceinline__ Prob prob_of(const XsIn& in, int S, int b) {
  Prob p;
  p.n = prob_n(in, b);
  p.base = in.multi ? sel4(in.dp, b) : in.data + (size_t)(in.off ? in.off[b] : 0u) * S;
  p.nch = (p.n + XS_L - 1) / XS_L;
  return p;
}

// lane's 4 consecutive inputs of chunk c, components k < K (non-finite allowed)
template <int S>
__device__ __forceinline__ void load4(const Prob& P, uint32_t c, int lane, int K, float v[4][S], bool ok[4]) {
  // all loads issued before use: clamped indices (P.n >= 1 whenever a chunk exists)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t i = c * XS_L + lane * 4 + j;
    ok[j] = i < P.n;
    const size_t ic = min(i, P.n - 1u);
#pragma unroll
    for (int k = 0; k < S; ++k) v[j][k] = P.base[ic * S + k];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < S; ++k)
      if (!ok[j] || k >= K) v[j][k] = 0.f;
}

template <int S>
__global__ void __launch_bounds__(256) k_xs_csum(XsIn in, int K, double* __restrict__ pre, uint32_t NC) {
  KT();
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const Prob P = prob_of(in, S, b);
  for (uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6); c < P.nch; c += gridDim.x * 4) {
    float v[4][S];
    bool ok[4];
    load4<S>(P, c, lane, K, v, ok);
#pragma unroll
    for (int k = 0; k < S; ++k) {
      if (k >= K) break;
      double a = 0.0;
#pragma unroll
      for (int j = 0; j < 4; ++j) a += ok[j] ? (double)v[j][k] : 0.0;
      a = wave_sum_d(a);
      if (lane == 0) pre[(size_t)(b * K + k) * (NC + 1) + c + 1] = a;
    }
  }
}

// in-place: pre[row][1..nch] chunk sums -> pre[row][0..nch] exclusive prefix
__global__ void __launch_bounds__(256) k_xs_prefix(XsIn in, int K, double* __restrict__ pre, uint32_t NC) {
  KT();
  __shared__ double sh[256];
  const int row = blockIdx.x, t = threadIdx.x;
  const uint32_t nch = (prob_n(in, row / K) + XS_L - 1) / XS_L;
  double* p = pre + (size_t)row * (NC + 1);
  double carry = 0.0;
  if (t == 0) p[0] = 0.0;
  for (uint32_t b0 = 1; b0 <= nch; b0 += 256) {
    const uint32_t i = b0 + t;
    double v = i <= nch ? p[i] : 0.0;
    sh[t] = v;
    __syncthreads();
    for (int d = 1; d < 256; d <<= 1) {
      const double o = t >= d ? sh[t - d] : 0.0;
      __syncthreads();
      v += o;
      sh[t] = v;
      __syncthreads();
    }
    if (i <= nch) p[i] = carry + v;
    carry += sh[255];
    __syncthreads();
  }
}

// The lane's run of (up to) four inputs under inv_u = 2^(23-E): the left fold
// xs_compose(...xs_compose(xs_identity(), xs_elem(x0)), ...) over the present inputs,
// computed directly.  Both start parities share each input's y, floor f and fraction;
// with e = Q + f (the input's envelope point), the input adds f + 1 when its fraction
// is above 1/2, or exactly 1/2 with p + e odd (the tie goes to the even quantum), and
// f otherwise.  The bounds are checked after every input, as each xs_compose checks
// its result, so the accepted summaries and the bad ones are those of the fold.
template <int S>
__device__ __forceinline__ XsSum xs_lane4(const float (&v)[4][S], int k, const bool (&ok)[4], double inv_u) {
  int32_t Q0 = 0, Q1 = 0, lo0 = XS_INF, lo1 = XS_INF, hi0 = -XS_INF, hi1 = -XS_INF;
  bool good = true;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float x = v[j][k];
    const double y = (double)x * inv_u;
    const bool fin = isfinite(x) && fabs(y) < XS_YMAX;
    const double fl = floor(y);
    const int32_t f = fin ? (int32_t)fl : 0;
    const double fr = y - fl;
    const uint32_t up = fr > 0.5 ? 1u : 0u, tie = fr == 0.5 ? 1u : 0u;
    // (unsigned arithmetic: a run already out of bounds keeps going without overflow)
    const int32_t e0 = (int32_t)((uint32_t)Q0 + (uint32_t)f), e1 = (int32_t)((uint32_t)Q1 + (uint32_t)f);
    const int32_t n0 = (int32_t)((uint32_t)e0 + (up | (tie & (uint32_t)e0 & 1u)));
    const int32_t n1 = (int32_t)((uint32_t)e1 + (up | (tie & ~(uint32_t)e1 & 1u)));
    const bool in = ok[j];
    Q0 = in ? n0 : Q0;
    Q1 = in ? n1 : Q1;
    lo0 = in ? min(lo0, e0) : lo0;
    lo1 = in ? min(lo1, e1) : lo1;
    hi0 = in ? max(hi0, e0) : hi0;
    hi1 = in ? max(hi1, e1) : hi1;
    good = good && (!in || (fin && Q0 > -XS_LIM && Q0 < XS_LIM && Q1 > -XS_LIM && Q1 < XS_LIM &&
                            lo0 > -XS_LIM && lo1 > -XS_LIM && hi0 < XS_LIM && hi1 < XS_LIM));
  }
  if (!good) return xs_bad();
  XsSum a;
  a.Q[0] = Q0;
  a.Q[1] = Q1;
  a.lo[0] = lo0;
  a.lo[1] = lo1;
  a.hi[0] = hi0;
  a.hi[1] = hi1;
  a.ok = 1;
  a.pad = 0;
  return a;
}

template <int S>
__global__ void __launch_bounds__(256) k_xs_chunk(XsIn in, int K, const double* __restrict__ pre,
                                                  XsSum* __restrict__ ctab, int32_t* __restrict__ cE, uint32_t NC) {
  KT();
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const Prob P = prob_of(in, S, b);
  for (uint32_t c = blockIdx.x * 4 + (threadIdx.x >> 6); c < P.nch; c += gridDim.x * 4) {
    float v[4][S];
    bool ok[4];
    load4<S>(P, c, lane, K, v, ok);
#pragma unroll
    for (int k = 0; k < S; ++k) {
      if (k >= K) break;
      const size_t row = (size_t)b * K + k;
      const int Eb = xs_predict(pre[row * (NC + 1) + c]);
      if (lane == 0) cE[row * NC + c] = Eb;
      if (Eb == XS_NOE) continue;
      for (int h = 0; h < XS_NE; ++h) {
        const double inv_u = ldexp(1.0, 23 - (Eb + h));
        const XsSum a = wave_total(xs_lane4<S>(v, k, ok, inv_u));
        if (lane == 63) ctab[(row * NC + c) * XS_NE + h] = a;
      }
    }
  }
}

__device__ __forceinline__ XsTab3 load_tab3(const XsSum* tab, const int32_t* eb, size_t u, bool have) {
  XsTab3 T;
  if (have) {
    T.t0 = tab[u * XS_NE];
    T.t1 = tab[u * XS_NE + 1];
    T.t2 = tab[u * XS_NE + 2];
    T.Eb = eb[u];
  } else {
    T.t0 = T.t1 = T.t2 = xs_identity();
    T.Eb = XS_NOE;
  }
  return T;
}

#ifdef XS_PROBE
__device__ unsigned long long xs_probe[8];  // scans, replays, decompose misses, replay cycles, scan cycles, prefetch misses
#define XS_COUNT(i, v) (threadIdx.x == 0 ? (void)atomicAdd(&xs_probe[i], (unsigned long long)(v)) : (void)0)
#else
#define XS_COUNT(i, v) ((void)0)
#endif

// Apply units cur..cnt-1 (lane l holds unit l's tables) to s.  Each unit is
// picked under s's binade E; an ordered scan of the units' quantum counts gives
// every unit its own start M_l, each unit checks its envelope there
// (xs_valid_unit), the first invalid lane f is found by a ballot, units cur..f-1
// are applied in one step and unit f goes to `descend`.
template <class Descend>
__device__ __forceinline__ void scan_jump(float& s, const XsTab3& T, int cnt, Descend descend) {
  const int lane = threadIdx.x & 63;
  int cur = 0;
  while (cur < cnt) {
    int E;
    int64_t M;
    if (!xs_decompose(s, &E, &M)) {  // zero / subnormal / non-finite start
      XS_COUNT(2, 1);
      descend(cur);
      ++cur;
      continue;
    }
#ifdef XS_PROBE
    const long long t0 = wall_clock64();
#endif
    const bool mine = lane >= cur && lane < cnt;
    const XsSum h = mine ? xs_pick(T, E) : xs_identity();
    uint32_t q0 = (uint32_t)h.Q[0], q1 = (uint32_t)h.Q[1];
    const int P = (int)(M & 1);
    uint32_t qi;  // inclusive count for the scan's start parity P
    if (__ballot(q0 != q1) == 0) {
      qi = add_scan(q0);
    } else {
      pmap_scan(q0, q1);
      qi = P ? q1 : q0;
    }
    const uint32_t qe = wave_shr1(qi);
    const int64_t Me = M + (int64_t)(int32_t)qe;
    const uint64_t bad = __ballot(mine && !xs_valid_unit(h, Me, M > 0));
    const int f = bad ? (int)__builtin_ctzll(bad) : cnt;
    if (f > cur) {
      const int64_t Q = (int32_t)__builtin_amdgcn_readlane(qi, f - 1);
      s = (float)ldexp((double)(M + Q), E - 23);
    }
    XS_COUNT(0, 1);
#ifdef XS_PROBE
    XS_COUNT(4, wall_clock64() - t0);
#endif
    if (f >= cnt) break;
    descend(f);
    cur = f + 1;
  }
}

// A window of 64 consecutive chunks: lane l holds chunk w*64+l's tables and the
// double prefix at its start and end (used only to predict binade crossings).
struct XsWin {
  XsTab3 T;
  double p0, p1;
};

// Chunk data prefetched for one window: up to XS_PF predicted crossing chunks,
// lane l holding inputs 4l..4l+3 of each.
constexpr int XS_PF = 4;
struct XsPf {
  uint32_t c[XS_PF];  // chunk ids (uniform); UINT32_MAX = empty slot
  float v[XS_PF][4];
};

// One wave per row: stream the row's chunk tables window by window (64 chunks per
// ordered scan), with tables loaded two windows ahead and the data of the chunks
// whose double prefix predicts a binade or sign change loaded one window ahead, so
// the serial chain rarely waits on memory.  A chunk that does not validate under
// the running sum's binade is replayed with plain float adds.  s is identical in
// every lane, so all control flow is uniform.
template <int S>
__global__ void __launch_bounds__(64) k_xs_chain(XsIn in, int K, const double* __restrict__ pre,
                                                 const XsSum* __restrict__ ctab, const int32_t* __restrict__ cE,
                                                 uint32_t NC, float* __restrict__ out, int divide) {
  KT();
  const int row = blockIdx.x, lane = threadIdx.x;
  const int b = row / K, k = row % K;
  const Prob P = prob_of(in, S, b);
  const float* x = P.base + k;
  const uint32_t nch = P.nch, nw = (nch + 63) / 64;
  const size_t t0 = (size_t)row * NC;
  const double* pr = pre + (size_t)row * (NC + 1);
  float s = 0.f;
  __shared__ __attribute__((aligned(16))) float rb[XS_L + 16];

  auto load_win = [&](uint32_t w, XsWin& W) {
    const uint32_t c = w * 64 + lane;
    const bool have = w < nw && c < nch;
    W.T = load_tab3(ctab, cE, t0 + c, have);
    W.p0 = have ? pr[c] : 0.0;
    W.p1 = have ? pr[c + 1] : 0.0;
  };
  auto load_chunk = [&](uint32_t c, float v[4]) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = c * XS_L + lane * 4 + j;
      v[j] = x[(size_t)min(i, P.n - 1u) * S];
    }
  };
  // issue the data loads of window w's predicted crossing chunks
  auto prefetch = [&](uint32_t w, const XsWin& W, XsPf& D) {
    const uint32_t c = w * 64 + lane;
    bool p = false;
    if (w < nw && c < nch)
      p = W.T.Eb == XS_NOE || xs_predict(W.p1) != W.T.Eb || ((W.p0 < 0.0) != (W.p1 < 0.0));
    uint64_t m = __ballot(p);
#pragma unroll
    for (int q = 0; q < XS_PF; ++q) {
      D.c[q] = m ? w * 64 + (uint32_t)__builtin_ctzll(m) : 0xffffffffu;
      m &= m - 1;
      if (D.c[q] != 0xffffffffu) load_chunk(D.c[q], D.v[q]);
    }
  };
  // Replay: the chunk is staged in LDS and summed with broadcast reads into a
  // VGPR accumulator (a uniform SGPR chain would cost a readlane/readfirstlane
  // round trip per add); reads of add group g+1 overlap the adds of group g.
  auto replay = [&](uint32_t c, const XsPf& D) {
    XS_COUNT(1, 1);
#ifdef XS_PROBE
    const long long tr = wall_clock64();
#endif
    float v[4];
    bool hit = false;
#pragma unroll
    for (int q = 0; q < XS_PF; ++q)
      if (D.c[q] == c) {
        hit = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) v[j] = D.v[q][j];
      }
    if (!hit) {
      XS_COUNT(5, 1);
      load_chunk(c, v);
    }
    const uint32_t m = min((uint32_t)XS_L, P.n - c * XS_L);
#pragma unroll
    for (int j = 0; j < 4; ++j) rb[lane * 4 + j] = v[j];
    __syncthreads();
    float acc = s;
    constexpr int GR = 16;
    const uint32_t ng16 = m / GR;
    float cur[GR];
#pragma unroll
    for (int q = 0; q < GR; ++q) cur[q] = rb[q];
    for (uint32_t g = 0; g < ng16; ++g) {
      float nxt[GR];
      const float* src = rb + GR * ((g + 1) & 15);  // wraps harmlessly on the last group
#pragma unroll
      for (int q = 0; q < GR; ++q) nxt[q] = src[q];
#pragma unroll
      for (int q = 0; q < GR; ++q) acc += cur[q];
#pragma unroll
      for (int q = 0; q < GR; ++q) cur[q] = nxt[q];
    }
    for (uint32_t j = GR * ng16; j < m; ++j) acc += rb[j];
    s = acc;
    __syncthreads();
#ifdef XS_PROBE
    XS_COUNT(3, wall_clock64() - tr);
#endif
  };
  // window w: tables in Wc (loaded two windows ago), data in Dc (one window ago);
  // issues the tables of w+2 into Wl and the data of w+1 into Dn.  Three-way
  // rotation by unrolling, so no register holding an in-flight load is copied.
  auto step = [&](uint32_t w, const XsWin& Wc, const XsWin& Wn, XsWin& Wl, const XsPf& Dc, XsPf& Dn) {
    load_win(w + 2, Wl);
    prefetch(w + 1, Wn, Dn);
    const int nc = (int)min(64u, nch - w * 64);
    scan_jump(s, Wc.T, nc, [&](int f) { replay(w * 64 + (uint32_t)f, Dc); });
  };
  XsWin W0, W1, W2;
  XsPf D0, D1, D2;
  load_win(0, W0);
  load_win(1, W1);
  prefetch(0, W0, D0);
  for (uint32_t w = 0; w < nw; w += 3) {
    step(w, W0, W1, W2, D0, D1);
    if (w + 1 >= nw) break;
    step(w + 1, W1, W2, W0, D1, D2);
    if (w + 2 >= nw) break;
    step(w + 2, W2, W0, W1, D2, D0);
  }
  if (lane == 0) out[row] = divide ? (P.n ? s / (float)P.n : 0.f) : s;
}

inline uint32_t clampg(uint32_t v, uint32_t mx) { return v < 1 ? 1 : (v > mx ? mx : v); }

}  // namespace

static size_t up256(size_t b) { return (b + 255) & ~size_t(255); }

size_t exact_sum_bytes(int rows, uint32_t cap) {
  const size_t NC = cap / XS_L + 1;
  return up256(rows * (NC + 1) * sizeof(double)) + up256(rows * NC * XS_NE * sizeof(XsSum)) +
         up256(rows * NC * sizeof(int32_t)) + 256;
}

XsBufs exact_sum_carve(void* base, int rows, uint32_t cap) {
  XsBufs x;
  x.NC = cap / XS_L + 1;
  x.rows = rows;
  char* p = (char*)(((uintptr_t)base + 255) & ~(uintptr_t)255);
  const size_t NC = x.NC;
  x.pre = (double*)p;
  p += up256(rows * (NC + 1) * sizeof(double));
  x.ctab = (XsSum*)p;
  p += up256(rows * NC * XS_NE * sizeof(XsSum));
  x.cE = (int32_t*)p;
  return x;
}

namespace {
void exact_sum_in(const XsIn& in, int S, int K, int nprob, float* out, bool divide, XsBufs x, hipStream_t st) {
  if (nprob <= 0) return;
  const int rows = nprob * K;
  if (rows > x.rows) throw Error(FCCF_E_INTERNAL, "exact_sum: scratch carved for fewer rows");
  const dim3 gc(clampg((x.NC + 3) / 4, 1024), nprob);
  if (S == 3) {
    k_xs_csum<3><<<gc, 256, 0, st>>>(in, K, x.pre, x.NC);
    k_xs_prefix<<<rows, 256, 0, st>>>(in, K, x.pre, x.NC);
    // probe bytes: 12 B per element of every problem (separate arrays: one count each)
    ProbeBytes pb;
    if (in.multi)
      for (int e = 0; e < nprob && e < BMAX; ++e) pb.add(in.cp[e], 12.0);
    else
      pb.add(in.cnt, 12.0);
    FCCF_LAUNCH("k_xs_chunk", (pb), k_xs_chunk<3>, gc, 256, 0, st, in, K, x.pre, x.ctab, x.cE, x.NC);
    FCCF_LAUNCH("k_xs_chain", (pb), k_xs_chain<3>, rows, 64, 0, st, in, K, x.pre, x.ctab, x.cE, x.NC, out, divide);
  } else {
    k_xs_csum<1><<<gc, 256, 0, st>>>(in, K, x.pre, x.NC);
    k_xs_prefix<<<rows, 256, 0, st>>>(in, K, x.pre, x.NC);
    FCCF_LAUNCH("k_xs_chunk", (in.cnt, 4.0 * 1), k_xs_chunk<1>, gc, 256, 0, st, in, K, x.pre, x.ctab, x.cE, x.NC);
    FCCF_LAUNCH("k_xs_chain", (in.cnt, 4.0 * 1), k_xs_chain<1>, rows, 64, 0, st, in, K, x.pre, x.ctab, x.cE, x.NC, out, divide);
  }
}
}  // namespace

void exact_sum(const float* data, int S, int K, const uint32_t* off, const uint32_t* cnt, int nprob, float* out,
               bool divide, XsBufs x, hipStream_t st) {
  XsIn in{};
  in.data = data;
  in.off = off;
  in.cnt = cnt;
  exact_sum_in(in, S, K, nprob, out, divide, x, st);
}

void exact_sum_n(const float* const* data, const uint32_t* const* cnt, int nprob, int S, int K, float* out, bool divide,
                 XsBufs x, hipStream_t st) {
  if (nprob < 1 || nprob > BMAX) throw Error(FCCF_E_INTERNAL, "exact_sum_n: 1 to BMAX arrays");
  XsIn in{};
  in.multi = 1;
  for (int b = 0; b < BMAX; ++b) {
    in.dp[b] = data[b < nprob ? b : nprob - 1];
    in.cp[b] = cnt[b < nprob ? b : nprob - 1];
  }
  exact_sum_in(in, S, K, nprob, out, divide, x, st);
}

void exact_sum2(const float* a, const uint32_t* na, const float* b, const uint32_t* nb, int S, int K, float* out,
                bool divide, XsBufs x, hipStream_t st) {
  const float* d[2] = {a, b};
  const uint32_t* c[2] = {na, nb};
  exact_sum_n(d, c, 2, S, K, out, divide, x, st);
}

}  // namespace fccf
