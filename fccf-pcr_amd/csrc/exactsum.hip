// exactsum.hip — exact parallel left-to-right float32 sums (algorithm: exactsum.h).
//
// Five launches per call, all sized from device counts:
//   k_xs_csum    one wave per (problem, 256-input chunk): double chunk sums (K comps)
//   k_xs_prefix  one block per row (problem x component): exclusive double prefix
//   k_xs_chunk   one wave per chunk: 3 binade hypotheses x 2 parities, wave-composed
//   k_xs_group   one wave per (row, 64-chunk group): compose chunk tables per binade
//   k_xs_chain   one wave per row: serial apply, group -> chunk -> replay
// The first four are bandwidth-bound streaming passes over the inputs; the chain
// touches one table per 16384 inputs except around binade crossings.
#include "devprim.h"
#include "exactsum.h"
#include "ctx.h"

namespace fccf {
namespace {

__device__ __forceinline__ XsSum shfl_down_sum(const XsSum& a, int d) {
  XsSum o;
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    o.Q[p] = __shfl_down(a.Q[p], d);
    o.lo[p] = __shfl_down(a.lo[p], d);
    o.hi[p] = __shfl_down(a.hi[p], d);
  }
  o.ok = __shfl_down(a.ok, d);
  o.pad = 0;
  return o;
}

// ordered reduction over the 64 lanes (lane 0 = first run); result in lane 0
__device__ __forceinline__ XsSum wave_compose(XsSum a) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const XsSum o = shfl_down_sum(a, d);
    if ((lane & (2 * d - 1)) == 0) a = xs_compose(a, o);
  }
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

__device__ __forceinline__ Prob prob_of(const float* data, int S, const uint32_t* off, const uint32_t* cnt, int b) {
  Prob p;
  p.n = cnt[b];
  p.base = data + (size_t)(off ? off[b] : 0u) * S;
  p.nch = (p.n + XS_L - 1) / XS_L;
  return p;
}

// lane's 4 consecutive inputs of chunk c, components k < K (non-finite allowed)
template <int S>
__device__ __forceinline__ void load4(const Prob& P, uint32_t c, int lane, int K, float v[4][S], bool ok[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const uint32_t i = c * XS_L + lane * 4 + j;
    ok[j] = i < P.n;
#pragma unroll
    for (int k = 0; k < S; ++k) v[j][k] = (ok[j] && k < K) ? P.base[(size_t)i * S + k] : 0.f;
  }
}

template <int S>
__global__ void __launch_bounds__(256) k_xs_csum(const float* __restrict__ data, int K, const uint32_t* __restrict__ off,
                                                 const uint32_t* __restrict__ cnt, double* __restrict__ pre,
                                                 uint32_t NC) {
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const Prob P = prob_of(data, S, off, cnt, b);
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
__global__ void __launch_bounds__(256) k_xs_prefix(const uint32_t* __restrict__ cnt, int K, double* __restrict__ pre,
                                                   uint32_t NC) {
  __shared__ double sh[256];
  const int row = blockIdx.x, t = threadIdx.x;
  const uint32_t nch = (cnt[row / K] + XS_L - 1) / XS_L;
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
__global__ void __launch_bounds__(256) k_xs_chunk(const float* __restrict__ data, int K, const uint32_t* __restrict__ off,
                                                  const uint32_t* __restrict__ cnt, const double* __restrict__ pre,
                                                  XsSum* __restrict__ ctab, int32_t* __restrict__ cE, uint32_t NC) {
  const int b = blockIdx.y, lane = threadIdx.x & 63;
  const Prob P = prob_of(data, S, off, cnt, b);
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
        a = wave_compose(a);
        if (lane == 0) ctab[(row * NC + c) * XS_NE + h] = a;
      }
    }
  }
}

__global__ void __launch_bounds__(256) k_xs_group(const uint32_t* __restrict__ cnt, int K, const double* __restrict__ pre,
                                                  const XsSum* __restrict__ ctab, const int32_t* __restrict__ cE,
                                                  XsSum* __restrict__ gtab, int32_t* __restrict__ gE, uint32_t NC,
                                                  uint32_t NG) {
  const size_t row = blockIdx.y;
  const int lane = threadIdx.x & 63;
  const uint32_t nch = (cnt[row / K] + XS_L - 1) / XS_L;
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
      a = wave_compose(a);
      if (lane == 0) gtab[(row * NG + g) * XS_NE + h] = a;
    }
  }
}

__device__ __forceinline__ bool xs_try(float& s, const XsSum* tab, int Eb) {
  int E;
  int64_t M;
  if (Eb == XS_NOE || !xs_decompose(s, &E, &M)) return false;
  const int h = E - Eb;
  if (h < 0 || h >= XS_NE) return false;
  const XsSum t = tab[h];
  if (!xs_valid(t, M)) return false;
  s = xs_apply(t, M, E);
  return true;
}

// One wave per row.  s is identical in every lane, so control flow is uniform.
template <int S>
__global__ void __launch_bounds__(64) k_xs_chain(const float* __restrict__ data, int K, const uint32_t* __restrict__ off,
                                                 const uint32_t* __restrict__ cnt, const XsSum* __restrict__ ctab,
                                                 const int32_t* __restrict__ cE, const XsSum* __restrict__ gtab,
                                                 const int32_t* __restrict__ gE, uint32_t NC, uint32_t NG,
                                                 float* __restrict__ out, int divide) {
  __shared__ XsSum tg[XS_G * XS_NE], tc[XS_G * XS_NE];
  __shared__ int32_t eg[XS_G], ec[XS_G];
  const int row = blockIdx.x, lane = threadIdx.x;
  const int b = row / K, k = row % K;
  const Prob P = prob_of(data, S, off, cnt, b);
  const float* x = P.base + k;
  const uint32_t ng = (P.nch + XS_G - 1) / XS_G;
  float s = 0.f;
  for (uint32_t gb = 0; gb < ng; gb += 64) {
    __syncthreads();
    if (gb + lane < ng) {
      const size_t gi = (size_t)row * NG + gb + lane;
      for (int h = 0; h < XS_NE; ++h) tg[lane * XS_NE + h] = gtab[gi * XS_NE + h];
      eg[lane] = gE[gi];
    }
    __syncthreads();
    for (uint32_t gi = 0; gi < 64 && gb + gi < ng; ++gi) {
      if (xs_try(s, &tg[gi * XS_NE], eg[gi])) continue;
      const uint32_t g = gb + gi;
      __syncthreads();
      {
        const uint32_t c = g * XS_G + lane;
        if (c < P.nch) {
          const size_t ci = (size_t)row * NC + c;
          for (int h = 0; h < XS_NE; ++h) tc[lane * XS_NE + h] = ctab[ci * XS_NE + h];
          ec[lane] = cE[ci];
        }
      }
      __syncthreads();
      for (uint32_t cj = 0; cj < XS_G; ++cj) {
        const uint32_t c = g * XS_G + cj;
        if (c >= P.nch) break;
        if (xs_try(s, &tc[cj * XS_NE], ec[cj])) continue;
        // replay the chunk with plain float adds in input order
        const uint32_t m = min((uint32_t)XS_L, P.n - c * XS_L);
        float v[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t i = c * XS_L + lane * 4 + j;
          v[j] = i < P.n ? x[(size_t)i * S] : 0.f;
        }
        for (uint32_t l = 0; l * 4 < m; ++l) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (l * 4 + j < m) s += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v[j]), (int)l));
        }
      }
    }
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

void exact_sum(const float* data, int S, int K, const uint32_t* off, const uint32_t* cnt, int nprob, float* out,
               bool divide, XsBufs x, hipStream_t st) {
  if (nprob <= 0) return;
  const int rows = nprob * K;
  if (rows > x.rows) throw Error(FCCF_E_INTERNAL, "exact_sum: scratch carved for fewer rows");
  const dim3 gc(clampg((x.NC + 3) / 4, 1024), nprob), gg(clampg((x.NG + 3) / 4, 256), rows);
  if (S == 3) {
    k_xs_csum<3><<<gc, 256, 0, st>>>(data, K, off, cnt, x.pre, x.NC);
    k_xs_prefix<<<rows, 256, 0, st>>>(cnt, K, x.pre, x.NC);
    k_xs_chunk<3><<<gc, 256, 0, st>>>(data, K, off, cnt, x.pre, x.ctab, x.cE, x.NC);
    k_xs_group<<<gg, 256, 0, st>>>(cnt, K, x.pre, x.ctab, x.cE, x.gtab, x.gE, x.NC, x.NG);
    k_xs_chain<3><<<rows, 64, 0, st>>>(data, K, off, cnt, x.ctab, x.cE, x.gtab, x.gE, x.NC, x.NG, out, divide);
  } else {
    k_xs_csum<1><<<gc, 256, 0, st>>>(data, K, off, cnt, x.pre, x.NC);
    k_xs_prefix<<<rows, 256, 0, st>>>(cnt, K, x.pre, x.NC);
    k_xs_chunk<1><<<gc, 256, 0, st>>>(data, K, off, cnt, x.pre, x.ctab, x.cE, x.NC);
    k_xs_group<<<gg, 256, 0, st>>>(cnt, K, x.pre, x.ctab, x.cE, x.gtab, x.gE, x.NC, x.NG);
    k_xs_chain<1><<<rows, 64, 0, st>>>(data, K, off, cnt, x.ctab, x.cE, x.gtab, x.gE, x.NC, x.NG, out, divide);
  }
}

}  // namespace fccf
