// exactsum.hip — exact parallel left-to-right float32 sums (algorithm: exactsum.h).
//
// Five launches per call, all sized from device counts:
//   k_xs_csum    one wave per (problem, 256-input chunk): double chunk sums (K comps)
//   k_xs_prefix  one block per row (problem x component): exclusive double prefix
//   k_xs_chunk   one wave per chunk: 3 binade hypotheses x 2 parities, wave-composed
//   k_xs_group   one wave per (row, 64-chunk group): compose chunk tables per binade
//   k_xs_chain   one wave per row: scan-jump over groups, then over the chunks of
//                a group that crosses a binade, then a plain replay of the chunk
// The first four are bandwidth-bound streaming passes over the inputs; the chain
// costs one wave scan per binade crossing (plus one 256-add replay).
#define KT_TU 4  // ktrace.h source tag
#include "probe.h"
#include "devprim.h"
#include "exactsum.h"
#include "ctx.h"

namespace fccf {
namespace {

// XsSum moved across lanes by one DPP control (row_shr:n / row_bcast:15 / :31);
// lanes the control does not address keep their own value.
template <int CTRL, int ROWS>
__device__ __forceinline__ XsSum dpp_sum(const XsSum& a) {
  XsSum o;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    o.Q[p] = __builtin_amdgcn_update_dpp(a.Q[p], a.Q[p], CTRL, ROWS, 0xf, false);
    o.lo[p] = __builtin_amdgcn_update_dpp(a.lo[p], a.lo[p], CTRL, ROWS, 0xf, false);
    o.hi[p] = __builtin_amdgcn_update_dpp(a.hi[p], a.hi[p], CTRL, ROWS, 0xf, false);
  }
  o.ok = __builtin_amdgcn_update_dpp(a.ok, a.ok, CTRL, ROWS, 0xf, false);
  o.pad = 0;
  return o;
}

// Inclusive ordered scan over the wave: lane l ends with units 0..l composed
// (earlier lanes first).  Four row_shr steps scan each 16-lane row, then
// row_bcast:15 / row_bcast:31 carry row totals forward.  No LDS traffic.
__device__ __forceinline__ XsSum wave_scan(XsSum a) {
  const int lane = threadIdx.x & 63, r = lane & 15;
  XsSum o;
  o = dpp_sum<0x111, 0xf>(a);
  if (r >= 1) a = xs_compose(o, a);
  o = dpp_sum<0x112, 0xf>(a);
  if (r >= 2) a = xs_compose(o, a);
  o = dpp_sum<0x114, 0xf>(a);
  if (r >= 4) a = xs_compose(o, a);
  o = dpp_sum<0x118, 0xf>(a);
  if (r >= 8) a = xs_compose(o, a);
  o = dpp_sum<0x142, 0xa>(a);
  if (lane & 16) a = xs_compose(o, a);
  o = dpp_sum<0x143, 0xc>(a);
  if (lane >= 32) a = xs_compose(o, a);
  return a;
}

__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d);
  return v;
}

struct Prob {
  const float* base;  // first element of the problem
  uint32_t n, nch;
};

// Where the problems live: either one array with per-problem offsets/counts
// (off may be null), or (data2 != null) two separate arrays, problem 0 = data with
// count *cnt and problem 1 = data2 with count *cnt2 (both clouds' centroids).
struct XsIn {
  const float* data;
  const uint32_t* off;
  const uint32_t* cnt;
  const float* data2;
  const uint32_t* cnt2;
};

__device__ __forceinline__ uint32_t prob_n(const XsIn& in, int b) {
  return (in.data2 && b == 1) ? *in.cnt2 : in.cnt[b];
}

__device__ __forceinline__ Prob prob_of(const XsIn& in, int S, int b) {
  Prob p;
  p.n = prob_n(in, b);
  p.base = (in.data2 && b == 1) ? in.data2 : in.data + (size_t)(in.off ? in.off[b] : 0u) * S;
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
        XsSum a = xs_identity();
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (ok[j]) a = xs_compose(a, xs_elem(v[j][k], inv_u));
        a = wave_scan(a);
        if (lane == 63) ctab[(row * NC + c) * XS_NE + h] = a;
      }
    }
  }
}

__global__ void __launch_bounds__(256) k_xs_group(XsIn in, int K, const double* __restrict__ pre,
                                                  const XsSum* __restrict__ ctab, const int32_t* __restrict__ cE,
                                                  XsSum* __restrict__ gtab, int32_t* __restrict__ gE, uint32_t NC,
                                                  uint32_t NG) {
  KT();
  const size_t row = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const uint32_t nch = (prob_n(in, (int)(row / K)) + XS_L - 1) / XS_L;
  const uint32_t ng = (nch + XS_G - 1) / XS_G;
  for (uint32_t g = blockIdx.x * 4 + (threadIdx.x >> 6); g < ng; g += gridDim.x * 4) {
    const int Eg = xs_predict(pre[row * (NC + 1) + (size_t)g * XS_G]);
    if (lane == 0) gE[row * NG + g] = Eg;
    if (Eg == XS_NOE) continue;
    const uint32_t c = g * XS_G + lane;
    const int Ec = c < nch ? cE[row * NC + c] : XS_NOE;
    for (int h = 0; h < XS_NE; ++h) {
      XsSum a = xs_identity();
      if (c < nch) {
        const int hc = Eg + h - Ec;
        a = (Ec != XS_NOE && hc >= 0 && hc < XS_NE) ? ctab[(row * NC + c) * XS_NE + hc] : xs_bad();
      }
      a = wave_scan(a);
      if (lane == 63) gtab[(row * NG + g) * XS_NE + h] = a;
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

// Apply units cur..cnt-1 (lane l holds unit l's tables) to s.  One ordered scan
// composes every prefix under s's binade; validity is monotone in the prefix
// length (envelopes only widen), so the first invalid lane f is found by a
// ballot, prefix f-1 is applied in one step and unit f goes to `descend`.
#ifdef XS_PROBE
__device__ unsigned long long xs_probe[8];  // scans, replays, decompose misses, replay cycles, scan cycles
#define XS_COUNT(i, v) (threadIdx.x == 0 ? (void)atomicAdd(&xs_probe[i], (unsigned long long)(v)) : (void)0)
#else
#define XS_COUNT(i, v) ((void)0)
#endif

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
    XsSum a = mine ? xs_pick(T, E) : xs_identity();
    a = wave_scan(a);
    const uint64_t bad = __ballot(mine && !xs_valid(a, M));
    const int f = bad ? (int)__builtin_ctzll(bad) : cnt;
    if (f > cur) {
      const int64_t Q = __builtin_amdgcn_readlane(xs_sel(a.Q, M), f - 1);
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

// One wave per row: groups (scan-jump) -> chunks (scan-jump) -> plain replay.
// s is identical in every lane, so all control flow is uniform.
template <int S>
__global__ void __launch_bounds__(64) k_xs_chain(XsIn in, int K, const XsSum* __restrict__ ctab,
                                                 const int32_t* __restrict__ cE, const XsSum* __restrict__ gtab,
                                                 const int32_t* __restrict__ gE, uint32_t NC, uint32_t NG,
                                                 float* __restrict__ out, int divide) {
  KT();
  const int row = blockIdx.x, lane = threadIdx.x;
  const int b = row / K, k = row % K;
  const Prob P = prob_of(in, S, b);
  const float* x = P.base + k;
  const uint32_t ng = (P.nch + XS_G - 1) / XS_G;
  float s = 0.f;
  // Replay: the chunk is staged in LDS and summed with broadcast reads into a
  // VGPR accumulator (a uniform SGPR chain would cost a readlane/readfirstlane
  // round trip per add); reads of group g+1 overlap the adds of group g.
  __shared__ __attribute__((aligned(16))) float rb[XS_L + 16];
  auto replay = [&](uint32_t c) {
    XS_COUNT(1, 1);
#ifdef XS_PROBE
    const long long t0 = wall_clock64();
#endif
    const uint32_t m = min((uint32_t)XS_L, P.n - c * XS_L);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t i = c * XS_L + lane * 4 + j;
      rb[lane * 4 + j] = i < P.n ? x[(size_t)i * S] : 0.f;
    }
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
    XS_COUNT(3, wall_clock64() - t0);
#endif
  };
  auto group = [&](uint32_t g) {
    const uint32_t c0 = g * XS_G;
    const int nc = (int)min((uint32_t)XS_G, P.nch - c0);
    const XsTab3 C = load_tab3(ctab, cE, (size_t)row * NC + c0 + lane, lane < nc);
    scan_jump(s, C, nc, [&](int f) { replay(c0 + (uint32_t)f); });
  };
  for (uint32_t gb = 0; gb < ng; gb += 64) {
    const int na = (int)min(64u, ng - gb);
    const XsTab3 G = load_tab3(gtab, gE, (size_t)row * NG + gb + lane, lane < na);
    scan_jump(s, G, na, [&](int f) { group(gb + (uint32_t)f); });
  }
  if (lane == 0) out[row] = divide ? (P.n ? s / (float)P.n : 0.f) : s;
}

inline uint32_t clampg(uint32_t v, uint32_t mx) { return v < 1 ? 1 : (v > mx ? mx : v); }

}  // namespace

static size_t up256(size_t b) { return (b + 255) & ~size_t(255); }

size_t exact_sum_bytes(int rows, uint32_t cap) {
  const size_t NC = cap / XS_L + 1, NG = NC / XS_G + 1;
  return up256(rows * (NC + 1) * sizeof(double)) + up256(rows * NC * XS_NE * sizeof(XsSum)) +
         up256(rows * NC * sizeof(int32_t)) + up256(rows * NG * XS_NE * sizeof(XsSum)) +
         up256(rows * NG * sizeof(int32_t)) + 256;
}

XsBufs exact_sum_carve(void* base, int rows, uint32_t cap) {
  XsBufs x;
  x.NC = cap / XS_L + 1;
  x.NG = x.NC / XS_G + 1;
  x.rows = rows;
  char* p = (char*)(((uintptr_t)base + 255) & ~(uintptr_t)255);
  const size_t NC = x.NC, NG = x.NG;
  x.pre = (double*)p;
  p += up256(rows * (NC + 1) * sizeof(double));
  x.ctab = (XsSum*)p;
  p += up256(rows * NC * XS_NE * sizeof(XsSum));
  x.cE = (int32_t*)p;
  p += up256(rows * NC * sizeof(int32_t));
  x.gtab = (XsSum*)p;
  p += up256(rows * NG * XS_NE * sizeof(XsSum));
  x.gE = (int32_t*)p;
  return x;
}

namespace {
void exact_sum_in(const XsIn& in, int S, int K, int nprob, float* out, bool divide, XsBufs x, hipStream_t st) {
  if (nprob <= 0) return;
  const int rows = nprob * K;
  if (rows > x.rows) throw Error(FCCF_E_INTERNAL, "exact_sum: scratch carved for fewer rows");
  const dim3 gc(clampg((x.NC + 3) / 4, 1024), nprob), gg(clampg((x.NG + 3) / 4, 256), rows);
  if (S == 3) {
    k_xs_csum<3><<<gc, 256, 0, st>>>(in, K, x.pre, x.NC);
    k_xs_prefix<<<rows, 256, 0, st>>>(in, K, x.pre, x.NC);
    // probe bytes: 12 B per element of every problem (two-array form: both counts)
    const uint32_t* c2 = in.data2 ? in.cnt2 : nullptr;
    FCCF_LAUNCH("k_xs_chunk", (in.cnt, 12.0, c2, 12.0, 0.0), k_xs_chunk<3>, gc, 256, 0, st, in, K, x.pre, x.ctab, x.cE, x.NC);
    k_xs_group<<<gg, 256, 0, st>>>(in, K, x.pre, x.ctab, x.cE, x.gtab, x.gE, x.NC, x.NG);
    FCCF_LAUNCH("k_xs_chain", (in.cnt, 12.0, c2, 12.0, 0.0), k_xs_chain<3>, rows, 64, 0, st, in, K, x.ctab, x.cE, x.gtab, x.gE, x.NC, x.NG, out, divide);
  } else {
    k_xs_csum<1><<<gc, 256, 0, st>>>(in, K, x.pre, x.NC);
    k_xs_prefix<<<rows, 256, 0, st>>>(in, K, x.pre, x.NC);
    FCCF_LAUNCH("k_xs_chunk", (in.cnt, 4.0 * 1), k_xs_chunk<1>, gc, 256, 0, st, in, K, x.pre, x.ctab, x.cE, x.NC);
    k_xs_group<<<gg, 256, 0, st>>>(in, K, x.pre, x.ctab, x.cE, x.gtab, x.gE, x.NC, x.NG);
    FCCF_LAUNCH("k_xs_chain", (in.cnt, 4.0 * 1), k_xs_chain<1>, rows, 64, 0, st, in, K, x.ctab, x.cE, x.gtab, x.gE, x.NC, x.NG, out, divide);
  }
}
}  // namespace

void exact_sum(const float* data, int S, int K, const uint32_t* off, const uint32_t* cnt, int nprob, float* out,
               bool divide, XsBufs x, hipStream_t st) {
  exact_sum_in(XsIn{data, off, cnt, nullptr, nullptr}, S, K, nprob, out, divide, x, st);
}

void exact_sum2(const float* a, const uint32_t* na, const float* b, const uint32_t* nb, int S, int K, float* out,
                bool divide, XsBufs x, hipStream_t st) {
  exact_sum_in(XsIn{a, nullptr, na, b, nb}, S, K, 2, out, divide, x, st);
}

}  // namespace fccf
