// fine.hip — K7: fine_verify (FCCF.cpp:785-839) for all <= 12 candidate transforms
// of one registration in one batch.
//
// Per evaluation e: S2' = T_e * S2 (PCL SSE transformer), fused cloud S1 ++ S2',
// OctreePointCloudSearch(0.5) anchored at the fused cloud's first point, then for
// each occupied leaf in DFS (Morton) order: s/t counts and the sequential float sums
//   allinvec += s + t ;  similar += (s+t) * (min/max)   (if s >= 1 and t >= 1)
// score = similar / allinvec.  The S1 half of the octree bound replay is shared by
// all evaluations.  Each workgroup counts its tile's points per leaf in an LDS hash
// (the residual clouds come in 1 m leaf order, so a tile of 2048 points holds a few
// hundred 0.5 m leaves) and emits one entry per leaf: key (e | morton), value
// (source | target << 16).  The entries are sorted by key, every leaf's entries summed
// -- counts are exact integers, so neither the tiles nor the entry order change them --
// and the float sum runs in the reference's leaf order (one lane per evaluation).
#define KT_TU 5  // ktrace.h source tag
#include <algorithm>
#include <cstdlib>

#include "probe.h"
#include "kernels.h"
#include "match.h"
#include "mail.h"

namespace fccf {
namespace {

// scal: [0] leaf entries (counted by k_fv_entries), [1] nbits = 3*Dmax + eb, [3] shift
// = 3*Dmax + 1 (the is_target bit of the per-point layout kept: the key of a leaf is
// (e << (shift-1)) | morton), [4] n1, [5] n2, [6] E; pts[e] = 0
__global__ void k_fv_bits(const OctState* __restrict__ st, uint32_t* __restrict__ scal, uint32_t* __restrict__ range,
                          uint32_t* __restrict__ pts, uint32_t n1, uint32_t n2, int E) {
  KT();
  if (threadIdx.x != 0) return;
  uint32_t D = 0;
  for (int e = 0; e < E; ++e)
    if (st[e].defined && st[e].depth > D) D = st[e].depth;
  uint32_t eb = 1;
  while ((1u << eb) <= (uint32_t)E) ++eb;
  scal[0] = 0u;
  scal[2] = 0u;  // segment count (stays 0 when there are no keys)
  for (int i = 0; i < 2 * MAX_EVAL; ++i) range[i] = 0u;
  for (int i = 0; i < MAX_EVAL; ++i) pts[i] = 0u;
  scal[3] = 3u * D + 1u;
  scal[1] = 3u * D + eb;
  scal[4] = n1;
  scal[5] = n2;
  scal[6] = (uint32_t)E;
}

// Exclusive scan over the 256 threads of a block; sh needs 4 u32.
__device__ __forceinline__ uint32_t fv_scan_256(uint32_t v, uint32_t* sh, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  uint32_t wp = 0;
  for (uint32_t w = 0; w < wave; ++w) wp += sh[w];
  const uint32_t tot = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  *total = tot;
  return wp + x - v;
}

// One workgroup per (tile of FV_TILE points of the fused cloud S1 ++ T_e S2, evaluation
// e): every finite point's leaf counted in an LDS hash (open addressing, FV_SLOTS = 2 x
// FV_TILE slots: it never fills), then the tile's leaves appended to the entry list at
// an offset taken with one atomic, and the tile's finite points added to pts[e].
constexpr uint32_t FV_TILE = 2048, FV_SLOTS = 4096;
constexpr unsigned long long FV_EMPTY = ~0ull;
// ecnt (the LDS form): evaluation e's entries go to its own region keys[e * (n1 + n2) ..]
// with their count in ecnt[e], and the key is the morton code alone.
__global__ void __launch_bounds__(256) k_fv_entries(const float* __restrict__ s1, const float* __restrict__ s2t,
                                                    const OctState* __restrict__ st, uint32_t* __restrict__ scal,
                                                    double res, uint64_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                                    uint32_t* __restrict__ pts, uint32_t* __restrict__ ecnt) {
  KT();
  __shared__ unsigned long long hk[FV_SLOTS];
  __shared__ uint32_t hc[FV_SLOTS];
  __shared__ uint32_t sh[4], sbase;
  const int e = blockIdx.y;
  const uint32_t n1 = scal[4], n2 = scal[5], shift = ecnt ? 63u : scal[3] - 1u;
  const uint32_t n = n1 + n2, i0 = blockIdx.x * FV_TILE;
  if (i0 >= n) return;
  const OctState S = st[e];
  const double inv = 1.0 / res;
  const float* b = s2t + (size_t)e * 3 * n2;
  for (uint32_t j = threadIdx.x; j < FV_SLOTS; j += 256) {
    hk[j] = FV_EMPTY;
    hc[j] = 0u;
  }
  __syncthreads();
  uint32_t fin = 0;
  const uint32_t lane = threadIdx.x & 63u;
  for (uint32_t j = 0; j < FV_TILE / 256; ++j) {
    if (i0 + j * 256 >= n) break;  // (uniform)
    const uint32_t i = i0 + j * 256 + threadIdx.x;
    const bool tgt = i >= n1;
    bool act = i < n;
    unsigned long long key = 0ull;
    if (act) {
      const float* p = tgt ? b + 3 * (i - n1) : s1 + 3 * i;
      const float x = p[0], y = p[1], z = p[2];
      act = finite3(x, y, z);
      if (act) key = (ecnt ? 0ull : (unsigned long long)e << shift) | oct_code(S, res, inv, x, y, z);
    }
    fin += act ? 1u : 0u;
    // A wave's points lie in a few leaves (the clouds come in 1 m leaf order): one lane
    // per distinct key inserts it and adds the wave's source and target counts, instead
    // of every lane hitting the same few LDS slots with atomics.
    const uint64_t tmask = __ballot(act && tgt);
    uint64_t pending = __ballot(act);
    while (pending) {
      const uint32_t leader = (uint32_t)__ffsll((unsigned long long)pending) - 1u;
      const uint32_t klo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)key, (int)leader);
      const uint32_t khi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(key >> 32), (int)leader);
      const unsigned long long lk = ((unsigned long long)khi << 32) | klo;
      const uint64_t same = __ballot(act && key == lk) & pending;
      if (lane == leader) {
        uint32_t h = (uint32_t)((lk * 0x9E3779B97F4A7C15ull) >> 52);  // 12 bits: FV_SLOTS
        for (;;) {
          const unsigned long long old = atomicCAS(&hk[h], FV_EMPTY, lk);
          if (old == FV_EMPTY || old == lk) break;
          h = (h + 1u) & (FV_SLOTS - 1u);
        }
        const uint32_t nt = (uint32_t)__popcll(same & tmask), ns = (uint32_t)__popcll(same) - nt;
        atomicAdd(&hc[h], ns | (nt << 16));
      }
      pending &= ~same;
    }
  }
  __syncthreads();
  // the occupied slots, compacted: FV_SLOTS / 256 consecutive slots per thread
  constexpr uint32_t PER = FV_SLOTS / 256;
  uint32_t occ = 0;
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) occ += hk[threadIdx.x * PER + q] != FV_EMPTY ? 1u : 0u;
  uint32_t tot, ftot;
  uint32_t pos = fv_scan_256(occ, sh, &tot);
  fv_scan_256(fin, sh, &ftot);
  if (threadIdx.x == 0) {
    sbase = ecnt ? (uint32_t)e * n + atomicAdd(&ecnt[e], tot) : atomicAdd(&scal[0], tot);
    if (ftot) atomicAdd(&pts[e], ftot);
  }
  __syncthreads();
  pos += sbase;
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q) {
    const uint32_t j = threadIdx.x * PER + q;
    if (hk[j] == FV_EMPTY) continue;
    keys[pos] = hk[j];
    vals[pos] = hc[j];
    ++pos;
  }
}

// similar_num (:830-835): the sequential float sum of the U terms in ht (float bits), by
// one lane -- groups of 16 without per-term conditions, the next group's 16-byte LDS
// loads issued before the current group's adds, then the tail
__device__ __forceinline__ float seq_sum(const uint32_t* ht, uint32_t U) {
  float s = 0.f;
  const uint4* __restrict__ t4 = reinterpret_cast<const uint4*>(ht);
  const uint32_t full = U & ~15u;
  uint4 cur[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) cur[u] = t4[u];
  for (uint32_t g = 0; g < full; g += 16) {
    uint4 nxt[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) nxt[u] = t4[((g + 16) >> 2) + u];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      s += __uint_as_float(cur[u].x);
      s += __uint_as_float(cur[u].y);
      s += __uint_as_float(cur[u].z);
      s += __uint_as_float(cur[u].w);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) cur[u] = nxt[u];
  }
  for (uint32_t g = full; g < U; ++g) s += __uint_as_float(ht[g]);
  return s;
}

// The LDS form, one 1024-thread workgroup per evaluation e: its entries merged into an
// LDS table (leaf code -> source, target counts; FV_LDS_SLOTS = 2 x FV_LDS_MAX slots),
// each leaf's term (:830-835) formed, the nonzero terms placed in code order by rank
// (c3: ~1700 leaves, ~900 nonzero terms per evaluation), and summed in that order by
// one lane -- the reference's sequential similar_num -- then score = similar_num /
// allinvec.  More than lds_cap leaves: FV_ERR_LDS, no score (the caller reruns in the
// sorted form).
constexpr uint32_t FV_LDS_SLOTS = 2 * FV_LDS_MAX;
__global__ void __launch_bounds__(1024) k_fv_eval(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                  const uint32_t* __restrict__ ecnt, const uint32_t* __restrict__ pts,
                                                  uint32_t* __restrict__ scal, float* __restrict__ scores,
                                                  FineMail* __restrict__ mail, uint32_t lds_cap) {
  KT();
  __shared__ __attribute__((aligned(16))) unsigned long long hk[FV_LDS_SLOTS];
  __shared__ __attribute__((aligned(16))) uint32_t hs[FV_LDS_SLOTS];
  __shared__ uint32_t ht[FV_LDS_SLOTS];
  __shared__ uint32_t snu, snz, sover;
  const int e = blockIdx.x;
#ifdef FV_PHASES
  unsigned long long fvt[8];  // dev (make VAR=fvph EXTRA=-DFV_PHASES): thread 0's phase stamps, printed for e = 0
#define FV_PH(k) do { if (threadIdx.x == 0) fvt[k] = __builtin_amdgcn_s_memtime(); } while (0)
  FV_PH(0);
#else
#define FV_PH(k) do {} while (0)
#endif
  const uint32_t n = scal[4] + scal[5], m = ecnt[e];
  const uint64_t* __restrict__ ke = keys + (size_t)e * n;
  const uint32_t* __restrict__ ve = vals + (size_t)e * n;
  for (uint32_t j = threadIdx.x; j < FV_LDS_SLOTS; j += 1024) {
    hk[j] = FV_EMPTY;
    hs[j] = 0u;
    ht[j] = 0u;
  }
  if (threadIdx.x == 0) {
    snu = 0u;
    snz = 0u;
    sover = 0u;
  }
  __syncthreads();
  FV_PH(1);
  for (uint32_t j = threadIdx.x; j < m; j += 1024) {
    const unsigned long long key = ke[j];
    const uint32_t c = ve[j];
    uint32_t h = (uint32_t)((key * 0x9E3779B97F4A7C15ull) >> 51);  // 13 bits: FV_LDS_SLOTS
    bool ok = false;
    for (uint32_t probe = 0; probe < FV_LDS_SLOTS; ++probe) {
      const unsigned long long old = atomicCAS(&hk[h], FV_EMPTY, key);
      if (old == FV_EMPTY) {
        if (atomicAdd(&snu, 1u) >= lds_cap) sover = 1u;
        ok = true;
        break;
      }
      if (old == key) {
        ok = true;
        break;
      }
      h = (h + 1u) & (FV_LDS_SLOTS - 1u);
    }
    if (!ok) {
      sover = 1u;
      continue;
    }
    atomicAdd(&hs[h], c & 0xFFFFu);
    atomicAdd(&ht[h], c >> 16);
  }
  __syncthreads();
  FV_PH(2);
  if (sover) {  // (uniform) more leaves than the LDS form takes
    if (threadIdx.x == 0) atomicOr(&scal[7], FV_ERR_LDS);  // (k_fv_mail_err copies the word to the mailbox)
    return;
  }
  // Each occupied leaf's term (:830-835).  Only the leaves with both counts >= 1 have a
  // nonzero term; the others add +0.0f to a sum that is never -0, which leaves it
  // unchanged, so only the Z nonzero terms are ordered and summed.  They are appended
  // in any order as (code, term) to the front of hk / ht (every thread reads its slots
  // before the barrier, then writes), and each one's place in code order is its rank:
  // the number of smaller codes among the Z (codes are distinct, one slot per leaf),
  // found by sorted 64-pair chunks and binary searches.
  {
    constexpr uint32_t PER = FV_LDS_SLOTS / 1024;
    unsigned long long k8[PER];
    uint32_t s8[PER], t8[PER];
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {  // (all loads first: an empty slot has counts 0)
      const uint32_t j = q * 1024 + threadIdx.x;  // (consecutive lanes, consecutive slots)
      k8[q] = hk[j];
      s8[q] = hs[j];
      t8[q] = ht[j];
    }
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q) {
      const float sn = (float)s8[q], tn = (float)t8[q];
      t8[q] = 0u;
      if (sn >= 1.f && tn >= 1.f) {
        const float mn = sn < tn ? sn : tn, mx = sn > tn ? sn : tn;
        t8[q] = __float_as_uint((sn + tn) * (mn / mx));  // > 0
      }
    }
    __syncthreads();
#pragma unroll
    for (uint32_t q = 0; q < PER; ++q)
      if (t8[q]) {
        const uint32_t o = atomicAdd(&snz, 1u);
        hk[o] = k8[q];
        ht[o] = t8[q];
      }
  }
  __syncthreads();
  FV_PH(3);
  const uint32_t Z = snz, nch = (Z + 63) / 64;
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  // chunks of 64 pairs sorted by code in registers (a wave's bitonic network over
  // shuffles), written back in place; pads (past Z) carry the empty code, above every
  // real one, so each chunk's valid pairs come first
  for (uint32_t c = wv; c < nch; c += 16) {
    const uint32_t i = c * 64 + lane;
    unsigned long long v = i < Z ? hk[i] : FV_EMPTY;
    uint32_t t = i < Z ? ht[i] : 0u;
#pragma unroll
    for (uint32_t k = 2; k <= 64; k <<= 1)
#pragma unroll
      for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
        const uint32_t olo = (uint32_t)__shfl_xor((int)(uint32_t)v, (int)jj, 64);
        const uint32_t ohi = (uint32_t)__shfl_xor((int)(uint32_t)(v >> 32), (int)jj, 64);
        const uint32_t ot = (uint32_t)__shfl_xor((int)t, (int)jj, 64);
        const unsigned long long o = ((unsigned long long)ohi << 32) | olo;
        const bool keep_min = ((lane & k) == 0) == ((lane & jj) == 0);
        const bool take = keep_min ? o < v : o > v;
        v = take ? o : v;
        t = take ? ot : t;
      }
    hk[i] = v;
    ht[i] = t;
  }
  __syncthreads();
  FV_PH(4);
  // each pair's place in code order: its lane in its sorted chunk plus, per other chunk,
  // the count of smaller codes there (a branchless binary search over the 64 entries)
  for (uint32_t c = wv; c < nch; c += 16) {
    const uint32_t i = c * 64 + lane;
    if (i >= Z) continue;
    const unsigned long long key = hk[i];
    uint32_t r = lane;
    for (uint32_t d = 0; d < nch; ++d) {
      if (d == c) continue;
      const unsigned long long* __restrict__ A = hk + d * 64;
      uint32_t pos = 0;
#pragma unroll
      for (uint32_t st = 32; st > 0; st >>= 1) pos += A[pos + st - 1] < key ? st : 0u;
      pos += A[pos] < key ? 1u : 0u;
      r += pos;
    }
    hs[r] = ht[i];  // the terms in code order in hs[0, Z)
  }
  __syncthreads();
  FV_PH(5);
  if (threadIdx.x == 0) {
    const float similar = seq_sum(hs, Z);  // similar_num += term, leaf by leaf
    const uint32_t p = pts[e];
    if (p >= (1u << 24)) atomicOr(&scal[7], FV_ERR_POINTS);  // float allinvec would round: unsupported size
    const float sc = similar / (float)p;
    scores[e] = sc;
    if (mail) mail->scores[e] = sc;
#ifdef FV_PHASES
    FV_PH(6);
    if (e == 0) printf("fv_eval e0 m %u U %u Z %u | init %llu merge %llu terms %llu chunks %llu search %llu sum %llu (s_memtime ticks)\n", m, snu, Z,
                       fvt[1] - fvt[0], fvt[2] - fvt[1], fvt[3] - fvt[2], fvt[4] - fvt[3], fvt[5] - fvt[4], fvt[6] - fvt[5]);
#endif
  }
}

// Per leaf (a run of equal keys among the sorted entries): source/target counts, the
// sums of its entries' counts (exact), and the similar_num term (:830-835):
// (s+t)*(min/max) when both are >= 1, else +0.0f (adding +0 leaves the float sum
// unchanged).  Also the per-evaluation segment ranges.
__global__ void __launch_bounds__(256) k_fv_counts(const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
                                                   const uint32_t* __restrict__ starts,
                                                   const uint32_t* __restrict__ scal, float* __restrict__ term,
                                                   uint32_t* __restrict__ range) {
  KT();
  const uint32_t ns = scal[2], sh = scal[3] - 1u;
  for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < ns; s += gridDim.x * 256) {
    const uint32_t b = starts[s], e = starts[s + 1];
    uint32_t src = 0, tg = 0;
    for (uint32_t j = b; j < e; ++j) {
      const uint32_t c = vals[j];
      src += c & 0xFFFFu;
      tg += c >> 16;
    }
    const float sn = (float)src, tn = (float)tg;
    float t = 0.f;
    if (sn >= 1.f && tn >= 1.f) {
      const float mn = sn < tn ? sn : tn, mx = sn > tn ? sn : tn;
      t = (sn + tn) * (mn / mx);
    }
    term[s] = t;
    const uint32_t ev = (uint32_t)(keys[b] >> sh);
    if (s == 0 || (uint32_t)(keys[starts[s - 1]] >> sh) != ev) range[2 * ev] = s;
    if (s + 1 == ns || (uint32_t)(keys[starts[s + 1]] >> sh) != ev) range[2 * ev + 1] = s + 1;
  }
}

// count of leaves per evaluation (exact_sum input) and allinvec: the float sum of
// integer counts is exact below 2^24, so it equals the integer point count.
__global__ void k_fv_ranges(const uint32_t* __restrict__ pts_e, uint32_t* __restrict__ range,
                            uint32_t* __restrict__ nseg_e, float* __restrict__ all, uint32_t* __restrict__ scal, int E) {
  KT();
  const int e = threadIdx.x;
  if (e >= E) return;
  const uint32_t f = range[2 * e], l = range[2 * e + 1];
  nseg_e[e] = l - f;
  nseg_e[MAX_EVAL + e] = f;  // first leaf of evaluation e (exact_sum offsets)
  const uint32_t pts = pts_e[e];
  if (pts >= (1u << 24)) atomicOr(&scal[7], 1u);  // float allinvec would round: unsupported size
  all[e] = (float)pts;
}

__global__ void k_fv_score(const float* __restrict__ similar, const float* __restrict__ all, float* __restrict__ scores,
                           int E, const uint32_t* __restrict__ scal, FineMail* __restrict__ mail) {
  KT();
  const int e = threadIdx.x;
  if (e < E) {
    const float sc = similar[e] / all[e];
    scores[e] = sc;
    if (mail) mail->scores[e] = sc;
  }
  if (mail && e == 0) {
    mail->err = scal[7];
    mail->stamp[1] = __builtin_amdgcn_s_memrealtime();
  }
  if (mail) {  // the mailbox is complete: its flag after a system-scope fence (phase B2 polls it)
    __syncthreads();
    if (e == 0) {
      __threadfence_system();
      __hip_atomic_store(&mail->done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

// the LDS form's scores (again: this kernel's own writes then precede the flag) and
// error word into the mailbox, then its flag (k_fv_score does this in the sorted form)
__global__ void k_fv_mail_err(const uint32_t* __restrict__ scal, const float* __restrict__ scores, int E,
                              FineMail* __restrict__ mail) {
  KT();
  if (threadIdx.x == 0) mail->stamp[1] = __builtin_amdgcn_s_memrealtime();
  if ((int)threadIdx.x < E) mail->scores[threadIdx.x] = scores[threadIdx.x];
  if (threadIdx.x == 0) mail->err = scal[7];
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    __hip_atomic_store(&mail->done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

inline uint32_t grid_for(uint32_t cap, uint32_t per = 256, uint32_t mx = 4096) {
  uint32_t g = (cap + per - 1) / per;
  return g < 1 ? 1 : (g > mx ? mx : g);
}

}  // namespace

void fine_verify_batch(const float* s1, uint32_t n1, const OctState* s1_state, const float* s2, uint32_t n2, int E,
                       double res, FineBufs b, hipStream_t st, FineMail* mail, int mode, uint32_t lds_cap) {
  if (E <= 0) return;
  const size_t astride = aggr_floats(n2);
  // scal[5] holds n2 for the device-count interfaces
  uint32_t* d_n2 = b.scal + 5;
  SeqStrides sd;  // evaluation e: its own transformed S2 copy, aggregates and state; shared count
  sd.xyz = 12 * (size_t)n2;
  sd.aggr = 4 * astride;
  sd.state = sizeof(OctState);
  // T_e * S2, its block aggregates and each evaluation's octree start (from S1's bounds)
  // in one launch
  {
    FvTransform tf{s2, b.T, b.s2t, s1_state, b.state, b.scal, b.nseg_e, b.pts, n1, n2};
    block_aggr_transform(tf, d_n2, n2, b.aggr2, st, E, sd, mail ? &mail->stamp[0] : nullptr);
  }
  octree_sim(b.s2t, d_n2, n2, res, b.aggr2, b.state, st, E, sd);
  const dim3 ge(std::max<uint32_t>(1u, (n1 + n2 + FV_TILE - 1) / FV_TILE), E);
  if (mode == FV_LEAVES_LDS) {
    // the leaves of each evaluation merged, sorted and summed in LDS: two launches
    // after the octrees instead of ~20 (scal[7] was zeroed by the transform launch)
    k_fv_entries<<<ge, 256, 0, st>>>(s1, b.s2t, b.state, b.scal, res, b.k0, b.v0, b.pts, b.nseg_e);
    k_fv_eval<<<E, 1024, 0, st>>>(b.k0, b.v0, b.nseg_e, b.pts, b.scal, b.scores, mail, std::min<uint32_t>(lds_cap, FV_LDS_MAX));
    if (mail) k_fv_mail_err<<<1, 64, 0, st>>>(b.scal, b.scores, E, mail);
    return;
  }
  k_fv_bits<<<1, 64, 0, st>>>(b.state, b.scal, b.range, b.pts, n1, n2, E);
  const uint32_t n = (uint32_t)E * (n1 + n2);  // the entry count's bound (one per point)
  k_fv_entries<<<ge, 256, 0, st>>>(s1, b.s2t, b.state, b.scal, res, b.k0, b.v0, b.pts, nullptr);
  // (e | morton) entries with their counts: 4 fast passes cover depth <= 9 with <= 15
  // evaluations; a third buffer, so no copy-back launch
  radix_sort_u64(b.k0, b.v0, b.k1, b.v1, b.scal, n, b.scal + 1, 32, false, b.ss, st, 1, B4<const uint32_t*>(nullptr),
                 B4<uint64_t*>(b.k2), B4<uint32_t*>(b.v2));
  segment_heads_u64(b.k0, b.scal, n, b.starts, b.scal + 2, b.ss, st);
  FCCF_LAUNCH("k_fv_counts", (b.scal, 12.0, b.scal + 2, 12.0), k_fv_counts, grid_for(n), 256, 0, st, b.k0, b.v0, b.starts, b.scal, b.term, b.range);
  k_fv_ranges<<<1, 64, 0, st>>>(b.pts, b.range, b.nseg_e, b.all, b.scal, E);
  exact_sum(b.term, 1, 1, b.nseg_e + MAX_EVAL, b.nseg_e, E, b.similar, false, b.xs, st);  // similar_num, leaf order
  k_fv_score<<<1, 64, 0, st>>>(b.similar, b.all, b.scores, E, b.scal, mail);
}

int fine_mode_env(int sticky_sorted) {
  const char* e = std::getenv("FCCF_FINE_SORTED");
  return (sticky_sorted || (e && e[0] == '1')) ? FV_LEAVES_SORTED : FV_LEAVES_LDS;
}
uint32_t fine_lds_cap_env() {
  const char* e = std::getenv("FCCF_FINE_LDS_CAP");
  const long v = e ? std::atol(e) : (long)FV_LDS_MAX;
  return v < 1 ? 1u : (v > (long)FV_LDS_MAX ? FV_LDS_MAX : (uint32_t)v);
}

}  // namespace fccf
