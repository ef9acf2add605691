// devprim.hip — stable LSD radix sort, run-length segmentation and exclusive scan
// for gfx950.  Wave64-native: per-digit ranks come from 8 ballots per 64-key
// chunk (no 32-lane warp idioms), block = 4 waves, tile = 2048 keys.
#define KT_TU 1  // ktrace.h source tag
#include "probe.h"
#include "devprim.h"
#include "ctx.h"

namespace fccf {

namespace {

constexpr int T = RS_THREADS;

__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }
// popcount(mask & lanes_below_me)
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Exclusive scan over the 256 threads of a block; sh needs 4 u32.
__device__ __forceinline__ uint32_t block_scan_256(uint32_t v, uint32_t* sh, uint32_t* total) {
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
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

__device__ __forceinline__ uint32_t passes_of(uint32_t nbits) { return (nbits + 7u) / 8u; }

// Digit plan of the device-wide passes for an nbits-wide key: up to RS_MAXW * 3 bits,
// the fewest passes of <= RS_MAXW-bit digits (19..27 bits: three 9-bit passes instead
// of four 8-bit ones), wider keys 8-bit digits (the fast launches then cover 32 bits
// and the single-workgroup tail the rest).  Every kernel of a sort derives the same
// plan from the device-side nbits.  RS_MAXW 10 (two passes for the c3 face codes,
// three for fine verification's keys) measured no faster: 1024-bucket tiles write
// ~4-key digit runs.
#ifndef RS_MAXW
#define RS_MAXW 9
#endif
constexpr int RS_MAXD = 1 << RS_MAXW;  // buckets of the widest digit (<= SORT_THREADS)
static_assert(RS_MAXD <= SORT_THREADS, "one digit bucket per sort thread");
struct RsPlan {
  uint32_t passes, width;
};
__device__ __forceinline__ RsPlan rs_plan(uint32_t nbits) {
  if (nbits == 0) return {0u, 8u};
  const uint32_t p = nbits <= 3u * RS_MAXW ? (nbits + RS_MAXW - 1u) / RS_MAXW : (nbits + 7u) / 8u;
  return {p, (nbits + p - 1u) / p};
}

// Exclusive scan of v over the first RS_MAXD threads of an ST-thread block (threads
// >= RS_MAXD pass 0 and get garbage); sh needs SW u32.  Every thread must call it.
__device__ __forceinline__ uint32_t scan_digits_of(uint32_t v, uint32_t* sh, uint32_t* total) {
  constexpr uint32_t NW = RS_MAXD / 64;  // waves holding digits
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  if (threadIdx.x >= (uint32_t)RS_MAXD) v = 0;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63 && wave < NW) sh[wave] = x;
  __syncthreads();
  uint32_t wp = 0, tot = 0;
  for (uint32_t w = 0; w < NW; ++w) {
    wp += w < wave ? sh[w] : 0u;
    tot += sh[w];
  }
  __syncthreads();
  *total = tot;
  return wp + x - v;
}

// Radix-sort tiles: 4096 keys per block of ST = 1024 threads (16 waves x 4 chunks of
// 64 keys).  A fat block keeps the per-tile ranking short (each wave ranks 256
// keys) while the tile count, and with it the digit x tile histogram, stays small.
constexpr int ST = SORT_THREADS;
constexpr int SW = ST / 64;  // waves per sort block

// Exclusive scan of v over the first 256 threads of an ST-thread block (threads
// >= 256 pass 0 and get garbage); sh needs SW u32.  Every thread must call it.
__device__ __forceinline__ uint32_t scan_256_of(uint32_t v, uint32_t* sh, uint32_t* total) {
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6;
  if (threadIdx.x >= 256) v = 0;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63 && wave < 4) sh[wave] = x;
  __syncthreads();
  uint32_t wp = 0;
  for (uint32_t w = 0; w < wave && w < 4; ++w) wp += sh[w];
  const uint32_t tot = sh[0] + sh[1] + sh[2] + sh[3];
  __syncthreads();
  *total = tot;
  return wp + x - v;
}

// The buffers of one sort: k[0]/v[0] in and out, k[1]/v[1] ping-pong, k[2]/v[2] an
// optional third buffer.  With it, a sort of exactly three active passes rotates
// 0 -> 2 -> 1 -> 0 and ends in buffer 0 without the copy-back an odd pass count
// otherwise needs; every kernel derives the same route from the device-side plan.
template <class K>
struct RsRing {
  K* k[3];
  uint32_t* v[3];
};
// buffer i of problem e, by selects only (no struct or array copy of the argument:
// no reference to a part of it either, which would make the compiler store it to scratch)
template <class K>
__device__ __forceinline__ K* ring_key(const B4<RsRing<K>>& R2, int e, int i) {
  return R2.v[e].k[i];
}
template <class K>
__device__ __forceinline__ uint32_t* ring_val(const B4<RsRing<K>>& R2, int e, int i) {
  return R2.v[e].v[i];
}
__device__ __forceinline__ uint32_t rs_active(uint32_t nbits, int fast_passes) {
  return min(rs_plan(nbits).passes, (uint32_t)fast_passes);
}
__device__ __forceinline__ int rs_src(int p, uint32_t P, bool three) {
  return (three && P == 3u) ? (p == 0 ? 0 : (p == 1 ? 2 : 1)) : (p & 1);
}
__device__ __forceinline__ int rs_dst(int p, uint32_t P, bool three) {
  return (three && P == 3u) ? (p == 0 ? 2 : (p == 1 ? 1 : 0)) : ((p & 1) ^ 1);
}

template <class K>
__global__ void __launch_bounds__(ST) k_rs_hist(B4<RsRing<K>> R2, B4<const uint32_t*> d_n2,
                                                B4<const uint32_t*> d_nbits2, int pass, B4<SortScratch> ss,
                                                uint32_t nblocks, int fast_passes) {
  KT();
  const int e = blockIdx.y;
  const bool three = ring_key(R2, e, 2) != nullptr;
  const K* __restrict__ keys = ring_key(R2, e, rs_src(pass, rs_active(*d_nbits2[e], fast_passes), three));
  uint32_t* __restrict__ hist = ss[e].hist;
  const RsPlan pl = rs_plan(*d_nbits2[e]);
  if ((uint32_t)pass >= pl.passes) return;
  const uint32_t shift = (uint32_t)pass * pl.width, W = pl.width, nd = 1u << W, mask = nd - 1u;
  const uint32_t n = *d_n2[e];
  __shared__ uint32_t cnt[RS_MAXD];
  // the grid is capped (rs_grid), not sized for the capacity: each workgroup takes the
  // problem's tiles blockIdx.x, + gridDim.x, ... (the face stage sorts the downsampled
  // cloud, a fifth of the capacity at c3; tiles past n are neither counted nor scanned)
  for (uint32_t t = blockIdx.x; t * (uint32_t)SORT_TILE < n; t += gridDim.x) {
    const uint32_t base = t * SORT_TILE;
    if (threadIdx.x < RS_MAXD) cnt[threadIdx.x] = 0;
    __syncthreads();
    const uint32_t end = min(base + (uint32_t)SORT_TILE, n);
    // all loads of the tile are issued before any is consumed (clamped indices, no
    // branches), then one LDS atomic per distinct digit per 64 keys (ballot match):
    // neighbouring keys share their high digits
    K kk[SORT_CHUNKS];
    const uint32_t last = n ? n - 1u : 0u;
#pragma unroll
    for (int c = 0; c < SORT_CHUNKS; ++c) kk[c] = keys[min(base + c * ST + threadIdx.x, last)];
#pragma unroll
    for (int c = 0; c < SORT_CHUNKS; ++c) {
      const bool ok = base + c * ST + threadIdx.x < end;
      const uint32_t d = (uint32_t)(kk[c] >> shift) & mask;
      uint64_t m = __ballot(ok);
      for (uint32_t b = 0; b < W; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
      }
      if (ok && mbcnt(m) == 0) atomicAdd(&cnt[d], (uint32_t)__popcll(m));
    }
    __syncthreads();
    if (threadIdx.x < nd) hist[threadIdx.x * nblocks + t] = cnt[threadIdx.x];
    __syncthreads();
  }
}

// One block per digit: exclusive scan of that digit's per-block counts in place.
__global__ void __launch_bounds__(T) k_rs_rowscan(B4<SortScratch> ss, uint32_t nblocks, B4<const uint32_t*> d_n2,
                                                  B4<const uint32_t*> d_nbits2, int pass) {
  KT();
  const int e = blockIdx.y;
  uint32_t* __restrict__ hist = ss[e].hist;
  uint32_t* __restrict__ tot = ss[e].tot;
  const RsPlan pl = rs_plan(*d_nbits2[e]);
  if ((uint32_t)pass >= pl.passes || blockIdx.x >= (1u << pl.width)) return;
  __shared__ uint32_t sh[4];
  const uint32_t d = blockIdx.x;
  const uint32_t ntl = min(nblocks, (*d_n2[e] + SORT_TILE - 1u) / SORT_TILE);  // the problem's tiles
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < ntl; b0 += T) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t v = i < ntl ? hist[d * nblocks + i] : 0u;
    uint32_t t;
    const uint32_t ex = block_scan_256(v, sh, &t);
    if (i < ntl) hist[d * nblocks + i] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) tot[d] = carry;
}

// Ranks a 4096-key tile (wave ballots), stages it in LDS in digit order, then
// writes each digit run to its global slot with consecutive lanes on consecutive
// addresses.  *active (probe, may be null) is cleared when the pass is skipped.
template <class K>
__global__ void __launch_bounds__(ST) k_rs_scatter(B4<RsRing<K>> R2, B4<const uint32_t*> d_n2,
                                                   B4<const uint32_t*> d_nbits2, int pass, B4<SortScratch> ss,
                                                   uint32_t nblocks, int iota, uint32_t* __restrict__ active,
                                                   int fast_passes) {
  KT();
  const int e = blockIdx.y;
  const uint32_t P = rs_active(*d_nbits2[e], fast_passes);
  const bool three = ring_key(R2, e, 2) != nullptr;
  const int si = rs_src(pass, P, three), di = rs_dst(pass, P, three);
  const K* __restrict__ kin = ring_key(R2, e, si);
  const uint32_t* __restrict__ vin = ring_val(R2, e, si);
  K* __restrict__ kout = ring_key(R2, e, di);
  uint32_t* __restrict__ vout = ring_val(R2, e, di);
  const uint32_t* __restrict__ hist = ss[e].hist;
  const uint32_t* __restrict__ tot = ss[e].tot;
  const RsPlan pl = rs_plan(*d_nbits2[e]);
  const bool run = (uint32_t)pass < pl.passes;
  if (active && e == 0 && blockIdx.x == 0 && threadIdx.x == 0) {  // probe: any problem of the batch active
    bool any = run;
#pragma unroll
    for (int q = 1; q < BMAX; ++q)  // (constant indices: a dynamic one would copy the argument to scratch)
      if (q < (int)gridDim.y) any = any || (uint32_t)pass < rs_plan(*d_nbits2.v[q]).passes;
    *active = any ? 1u : 0u;
  }
  const uint32_t n = *d_n2[e];
  if (!run) return;
  const uint32_t shift = (uint32_t)pass * pl.width, W = pl.width, nd = 1u << W, mask = nd - 1u;
  __shared__ uint32_t gofs[RS_MAXD];     // global slot of the tile's first key of each digit
  __shared__ uint32_t tex[RS_MAXD];      // exclusive digit offsets inside the tile
  __shared__ uint16_t wcnt[SW][RS_MAXD]; // per-wave digit counts, then per-wave offsets (<= 4096)
  __shared__ uint32_t sh[SW];
  __shared__ K sk[SORT_TILE];
  __shared__ uint32_t sv[SORT_TILE];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  const bool hv = vout != nullptr;  // keys-only sorts pass no value buffers
  // (capped grid: the problem's tiles blockIdx.x, + gridDim.x, ..., as in k_rs_hist)
  for (uint32_t tl = blockIdx.x; tl * (uint32_t)SORT_TILE < n; tl += gridDim.x) {
    const uint32_t tile0 = tl * SORT_TILE;
    const uint32_t base = tile0 + wave * (SORT_CHUNKS * 64);
    K kk[SORT_CHUNKS];
    uint32_t vv[SORT_CHUNKS], rk[SORT_CHUNKS], dg[SORT_CHUNKS];
    const uint32_t last = n - 1u;  // n > tile0 >= 0
#pragma unroll
    for (int c = 0; c < SORT_CHUNKS; ++c) {  // all loads in flight before the ranking
      const uint32_t i = min(base + c * 64 + lane, last);
      kk[c] = kin[i];
      vv[c] = (iota || !hv) ? i : vin[i];
    }
    {
      uint32_t t;
      const uint32_t g = tid < nd ? tot[tid] : 0u;
      const uint32_t h = tid < nd ? hist[tid * nblocks + tl] : 0u;
      const uint32_t ex = scan_digits_of(g, sh, &t);
      if (tid < nd) gofs[tid] = ex + h;
    }
    for (uint32_t j = tid; j < SW * RS_MAXD; j += ST) (&wcnt[0][0])[j] = 0;
    __syncthreads();
#pragma unroll
    for (int c = 0; c < SORT_CHUNKS; ++c) {
      const uint32_t i = base + c * 64 + lane;
      const bool ok = i < n;
      const uint32_t d = (uint32_t)(kk[c] >> shift) & mask;
      dg[c] = ok ? d : RS_MAXD;
      uint64_t m = __ballot(ok);
      for (uint32_t b = 0; b < W; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
      }
      const uint32_t r = mbcnt(m);
      const uint32_t pre = ok ? wcnt[wave][d] : 0u;
      rk[c] = pre + r;
      if (ok && r == 0) wcnt[wave][d] = (uint16_t)(pre + (uint32_t)__popcll(m));
    }
    __syncthreads();
    {  // per-wave offsets within a digit, tile digit totals, their exclusive scan
      uint32_t acc = 0;
      if (tid < nd)
        for (int w = 0; w < SW; ++w) {
          const uint32_t t = wcnt[w][tid];
          wcnt[w][tid] = (uint16_t)acc;
          acc += t;
        }
      uint32_t t;
      const uint32_t ex = scan_digits_of(acc, sh, &t);
      if (tid < nd) tex[tid] = ex;
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < SORT_CHUNKS; ++c) {
      const uint32_t d = dg[c];
      if (d >= (uint32_t)RS_MAXD) continue;
      const uint32_t lp = tex[d] + wcnt[wave][d] + rk[c];
      sk[lp] = kk[c];
      if (hv) sv[lp] = vv[c];
    }
    __syncthreads();
    const uint32_t m = min((uint32_t)SORT_TILE, n - tile0);
    for (uint32_t j = tid; j < m; j += ST) {
      const K k = sk[j];
      const uint32_t d = (uint32_t)(k >> shift) & mask;
      const uint32_t pos = gofs[d] + (j - tex[d]);
      kout[pos] = k;
      if (hv) vout[pos] = sv[j];
    }
    __syncthreads();  // (the tile's LDS reads before the next tile's writes)
  }
}

// The high passes of a sort, for keys wider than the fast passes cover (octree
// codes of very large extents), or the whole sort of keys that are normally already
// in order (VoxelGrid's second pass; `need` = its "unsorted" flag): one workgroup per
// problem runs the stable 8-bit LSD passes [lo, nbits) over all tiles in order, lo =
// the bits the fast_passes launched passes of the device plan covered.
// Slow (one CU) but a single launch that exits at once in the common case, where
// the launches of never-needed fast passes would each cost a kernel boundary.
// copy_home (a sort with a third buffer, which launches no copy-back kernel): the one
// plan that still ends outside buffer 0 -- a single active pass, 0 -> 1 -- is copied
// home here, by this one workgroup (tiny key widths only: nbits <= RS_MAXW).
template <class K>
__global__ void __launch_bounds__(ST) k_rs_tail(B4<K*> k02, B4<uint32_t*> v02, B4<K*> k12, B4<uint32_t*> v12,
                                                B4<const uint32_t*> d_n2, B4<const uint32_t*> d_nbits2,
                                                int fast_passes, B4<const uint32_t*> need2, int copy_home) {
  KT();
  const int e = blockIdx.y;
  const uint32_t nbits = *d_nbits2[e], n = *d_n2[e];
  K* kb[2] = {k02[e], k12[e]};
  uint32_t* vb[2] = {v02[e], v12[e]};
  if (copy_home && rs_active(nbits, fast_passes) == 1u) {
    for (uint32_t i = threadIdx.x; i < n; i += ST) {
      kb[0][i] = kb[1][i];
      if (vb[0]) vb[0][i] = vb[1][i];
    }
    __syncthreads();
  }
  const RsPlan pl = rs_plan(nbits);
  const uint32_t lo_bit = pl.passes <= (uint32_t)fast_passes ? nbits : (uint32_t)fast_passes * pl.width;
  if (lo_bit >= nbits || n < 2) return;
  if (need2[e] && *need2[e] == 0u) return;
  __shared__ uint32_t run_ofs[256], cnt[256], tex[256], tcnt[256];
  __shared__ uint32_t wcnt[SW][256];
  __shared__ uint32_t sh[SW];
  __shared__ K sk[SORT_TILE];
  __shared__ uint32_t sv[SORT_TILE];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  int src = 0;
  for (uint32_t shift = lo_bit; shift < nbits; shift += 8) {
    const K* __restrict__ kin = kb[src];
    const uint32_t* __restrict__ vin = vb[src];
    K* __restrict__ kout = kb[src ^ 1];
    uint32_t* __restrict__ vout = vb[src ^ 1];
    if (tid < 256) cnt[tid] = 0;
    __syncthreads();
    for (uint32_t b0 = 0; b0 < n; b0 += ST) {  // digit histogram of the whole array
      const uint32_t i = b0 + tid;
      const bool ok = i < n;
      const uint32_t d = ok ? (uint32_t)(kin[i] >> shift) & 255u : 0u;
      uint64_t m = __ballot(ok);
#pragma unroll
      for (int b = 0; b < 8; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
      }
      if (ok && mbcnt(m) == 0) atomicAdd(&cnt[d], (uint32_t)__popcll(m));
    }
    __syncthreads();
    {
      uint32_t t;
      const uint32_t ex = scan_256_of(tid < 256 ? cnt[tid] : 0u, sh, &t);
      if (tid < 256) run_ofs[tid] = ex;
    }
    __syncthreads();
    for (uint32_t tile0 = 0; tile0 < n; tile0 += SORT_TILE) {  // stable scatter, tile by tile
      const uint32_t base = tile0 + wave * (SORT_CHUNKS * 64);
      K kk[SORT_CHUNKS];
      uint32_t vv[SORT_CHUNKS], rk[SORT_CHUNKS], dg[SORT_CHUNKS];
#pragma unroll
      for (int c = 0; c < SORT_CHUNKS; ++c) {
        const uint32_t i = min(base + c * 64 + lane, n - 1u);
        kk[c] = kin[i];
        vv[c] = vin ? vin[i] : 0u;
      }
      for (uint32_t j = tid; j < SW * 256; j += ST) (&wcnt[0][0])[j] = 0;
      __syncthreads();
#pragma unroll
      for (int c = 0; c < SORT_CHUNKS; ++c) {
        const uint32_t i = base + c * 64 + lane;
        const bool ok = i < n;
        const uint32_t d = (uint32_t)(kk[c] >> shift) & 255u;
        dg[c] = ok ? d : 256u;
        uint64_t m = __ballot(ok);
#pragma unroll
        for (int b = 0; b < 8; ++b) {
          const bool bit = (d >> b) & 1u;
          const uint64_t bb = __ballot(bit);
          m &= bit ? bb : ~bb;
        }
        const uint32_t r = mbcnt(m);
        const uint32_t pre = ok ? wcnt[wave][d] : 0u;
        rk[c] = pre + r;
        if (ok && r == 0) wcnt[wave][d] = pre + (uint32_t)__popcll(m);
      }
      __syncthreads();
      {
        uint32_t acc = 0;
        if (tid < 256)
          for (int w = 0; w < SW; ++w) {
            const uint32_t t = wcnt[w][tid];
            wcnt[w][tid] = acc;
            acc += t;
          }
        if (tid < 256) tcnt[tid] = acc;
        uint32_t t;
        const uint32_t ex = scan_256_of(acc, sh, &t);
        if (tid < 256) tex[tid] = ex;
      }
      __syncthreads();
#pragma unroll
      for (int c = 0; c < SORT_CHUNKS; ++c) {
        const uint32_t d = dg[c];
        if (d > 255u) continue;
        const uint32_t lp = tex[d] + wcnt[wave][d] + rk[c];
        sk[lp] = kk[c];
        sv[lp] = vv[c];
      }
      __syncthreads();
      const uint32_t m = min((uint32_t)SORT_TILE, n - tile0);
      for (uint32_t j = tid; j < m; j += ST) {
        const K k = sk[j];
        const uint32_t d = (uint32_t)(k >> shift) & 255u;
        const uint32_t pos = run_ofs[d] + (j - tex[d]);
        kout[pos] = k;
        if (vout) vout[pos] = sv[j];
      }
      __syncthreads();
      if (tid < 256) run_ofs[tid] += tcnt[tid];
      __syncthreads();
    }
    src ^= 1;
  }
  if (src)
    for (uint32_t i = tid; i < n; i += ST) {
      kb[0][i] = kb[1][i];
      if (vb[0]) vb[0][i] = vb[1][i];
    }
}

template <class K>
__global__ void k_rs_copyback(B4<RsRing<K>> R2, B4<const uint32_t*> d_n2, B4<const uint32_t*> d_nbits2,
                              int max_passes) {
  KT();
  const int e = blockIdx.y;
  const uint32_t p = rs_active(*d_nbits2[e], max_passes);
  if ((p & 1u) == 0u || (p == 3u && ring_key(R2, e, 2) != nullptr)) return;  // even, or rotated home
  const K* __restrict__ k1 = ring_key(R2, e, 1);
  const uint32_t* __restrict__ v1 = ring_val(R2, e, 1);
  K* __restrict__ k0 = ring_key(R2, e, 0);
  uint32_t* __restrict__ v0 = ring_val(R2, e, 0);
  const uint32_t n = *d_n2[e];
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    k0[i] = k1[i];
    if (v0) v0[i] = v1[i];
  }
}

// Workgroups per problem of the radix passes: the capacity's tiles, at most ~1024
// workgroups per launch over the batch (two 1024-thread tiles fit a CU, so that is two
// rounds of the chip).  Grids sized for the capacity launched ~2,000 workgroups per
// ten-cloud face sort of which a fifth had a tile.
#ifndef RS_GRID_MAX
#define RS_GRID_MAX 1024
#endif
static uint32_t rs_grid(uint32_t nb, int nbatch) {
  return std::max(1u, std::min(nb, (uint32_t)RS_GRID_MAX / (uint32_t)std::max(1, nbatch)));
}

template <class K>
void radix_sort(B4<K*> k0, B4<uint32_t*> v0, B4<K*> k1, B4<uint32_t*> v1, B4<const uint32_t*> d_n, uint32_t cap,
                B4<const uint32_t*> d_nbits, int fast_bits, bool iota, B4<SortScratch> s, hipStream_t st,
                int nbatch, B4<const uint32_t*> tail_need, B4<K*> k2, B4<uint32_t*> v2) {
  const uint32_t nb = sort_blocks(cap);
  if (nb == 0) return;
  if (fast_bits == 0 && iota) throw Error(FCCF_E_INTERNAL, "radix_sort: a tail-only sort takes its values as input");
  if ((v0[0] == nullptr) != (v1[0] == nullptr)) throw Error(FCCF_E_INTERNAL, "radix_sort: both or no value buffers");
  if ((k2[0] == nullptr) != (k2[nbatch - 1] == nullptr) || (k2[0] && (v2[0] == nullptr) != (v0[0] == nullptr)))
    throw Error(FCCF_E_INTERNAL, "radix_sort: third buffer on every problem, values with values");
  const int fast_passes = fast_bits / 8;
  B4<RsRing<K>> R;
  for (int e = 0; e < BMAX; ++e) R.v[e] = RsRing<K>{{k0[e], k1[e], k2[e]}, {v0[e], v1[e], v2[e]}};  // host side
  const uint32_t g = rs_grid(nb, nbatch);
  for (int p = 0; p < fast_passes; ++p) {  // pass p: digit p of the device-side plan (rs_plan)
    k_rs_hist<K><<<dim3(g, nbatch), ST, 0, st>>>(R, d_n, d_nbits, p, s, nb, fast_passes);
    k_rs_rowscan<<<dim3(RS_MAXD, nbatch), T, 0, st>>>(s, nb, d_n, d_nbits, p);
    const double eb = 2.0 * (sizeof(K) + (v0[0] ? 4 : 0));  // algorithmic bytes per element
    ProbeBytes pb;
    for (int e = 0; e < nbatch; ++e) pb.add(d_n[e], eb);
    FCCF_LAUNCH("k_rs_scatter", (pb), k_rs_scatter<K>, dim3(g, nbatch), ST, 0, st, R, d_n, d_nbits, p, s, nb, (iota && p == 0) ? 1 : 0, _probe.active(), fast_passes);
  }
  // With a third buffer every plan but a single pass ends in buffer 0 (an even pass
  // count by ping-pong, three passes by rotation), so no copy-back kernel is launched
  // (a dependent launch, ~5 us, that exited at once); the tail copies that one case home.
  const bool three = k2[0] != nullptr;
  if (fast_passes && !three) {
    const uint32_t g = min(nb * 8u, 2048u);
    k_rs_copyback<K><<<dim3(g, nbatch), 256, 0, st>>>(R, d_n, d_nbits, fast_passes);
  }
  if (fast_bits < (int)(8 * sizeof(K)) || (three && fast_passes))
    k_rs_tail<K><<<dim3(1, nbatch), ST, 0, st>>>(k0, v0, k1, v1, d_n, d_nbits, fast_passes, tail_need, three ? 1 : 0);
}

// ---------------------------------------------------------------- segments / scan
// Two launches each: per-tile counts, then the writes.  Each write block forms its
// tile's exclusive prefix itself from the counts of the tiles before it (a block
// reduction over <= a few thousand words, all L2 hits), which saves the separate
// scan-of-tile-counts launch; the block owning the last element writes the total.
// keys[i0-1 .. i0+RS_CHUNKS] into registers, all loads issued before use
// (clamped indices; positions outside [0, n) are masked by the callers)
template <class K>
__device__ __forceinline__ void load_run(const K* keys, uint32_t i0, uint32_t n, K kk[RS_CHUNKS + 2]) {
  const uint32_t last = n ? n - 1u : 0u;
#pragma unroll
  for (int j = 0; j < RS_CHUNKS + 2; ++j) {
    // kk[j] = keys[i0 - 1 + j]; for i0 == 0 the wrapped index clamps to `last`, and
    // kk[0] is then never read (position 0 is always a head)
    kk[j] = keys[min(i0 + (uint32_t)j - 1u, last)];
  }
}

template <class K, bool HasInvalid>
__device__ __forceinline__ bool head_at(const K kk[RS_CHUNKS + 2], int j, uint32_t i, uint32_t n, K invalid) {
  if (i >= n) return false;
  const K k = kk[j + 1];
  if (HasInvalid && k == invalid) return false;
  return i == 0 || kk[j] != k;
}

// sum of blk[0 .. blockIdx.x) over the block (every thread gets it)
__device__ __forceinline__ uint32_t tiles_before(const uint32_t* __restrict__ blk, uint32_t* sh) {
  uint32_t v = 0;
  for (uint32_t i = threadIdx.x; i < blockIdx.x; i += T) v += blk[i];
  uint32_t t;
  block_scan_256(v, sh, &t);
  return t;
}

// the block that owns the last element (block 0 when n == 0) reports the total
__device__ __forceinline__ bool owns_last(uint32_t n) { return blockIdx.x == (n ? (n - 1u) / RS_TILE : 0u); }

template <class K, bool HasInvalid>
__global__ void __launch_bounds__(T) k_seg_count(B4<const K*> keys2, B4<const uint32_t*> d_n2, K invalid,
                                                 B4<SortScratch> ss, B4<const uint32_t*> run2) {
  KT();
  __shared__ uint32_t sh[4];
  const int e = blockIdx.y;
  if (run2[e] && *run2[e] == 0u) return;
  const uint32_t n = *d_n2[e];
  const uint32_t i0 = blockIdx.x * RS_TILE + threadIdx.x * RS_CHUNKS;
  if (blockIdx.x * RS_TILE >= n && blockIdx.x) return;
  K kk[RS_CHUNKS + 2];
  load_run<K>(keys2[e], i0, n, kk);
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < RS_CHUNKS; ++j) c += head_at<K, HasInvalid>(kk, j, i0 + j, n, invalid) ? 1u : 0u;
  uint32_t t;
  block_scan_256(c, sh, &t);
  if (threadIdx.x == 0) ss[e].blk[blockIdx.x] = t;
}

template <class K, bool HasInvalid>
__global__ void __launch_bounds__(T) k_seg_write(B4<const K*> keys2, B4<const uint32_t*> d_n2, K invalid,
                                                 B4<SortScratch> ss, B4<uint32_t*> starts2, B4<uint32_t*> d_nseg2,
                                                 B4<uint32_t*> seg_of2, B4<const uint32_t*> run2) {
  KT();
  __shared__ uint32_t sh[4];
  const int e = blockIdx.y;
  if (run2[e] && *run2[e] == 0u) return;
  const uint32_t n = *d_n2[e];
  if (blockIdx.x * RS_TILE >= n && blockIdx.x) return;
  uint32_t* __restrict__ starts = starts2[e];
  uint32_t* __restrict__ seg_of = seg_of2[e];
  const uint32_t i0 = blockIdx.x * RS_TILE + threadIdx.x * RS_CHUNKS;
  K kk[RS_CHUNKS + 2];
  load_run<K>(keys2[e], i0, n, kk);
  const uint32_t before = tiles_before(ss[e].blk, sh);
  bool h[RS_CHUNKS];
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < RS_CHUNKS; ++j) {
    h[j] = head_at<K, HasInvalid>(kk, j, i0 + j, n, invalid);
    c += h[j] ? 1u : 0u;
  }
  uint32_t t;
  uint32_t pos = before + block_scan_256(c, sh, &t);
  if (threadIdx.x == 0 && owns_last(n)) *d_nseg2[e] = before + t;
#pragma unroll
  for (int j = 0; j < RS_CHUNKS; ++j) {
    const uint32_t i = i0 + j;
    if (h[j]) starts[pos++] = i;
    // end of the valid prefix: close the last segment
    if (i < n) {
      const bool valid = !HasInvalid || kk[j + 1] != invalid;
      if (seg_of && valid) seg_of[i] = pos - 1;
      const bool next_valid = (i + 1 < n) && (!HasInvalid || kk[j + 2] != invalid);
      if (valid && !next_valid) starts[pos] = i + 1;  // pos == segment count here
    }
  }
}

template <class K, bool HasInvalid>
void segment_heads(B4<const K*> keys, B4<const uint32_t*> d_n, uint32_t cap, K invalid, B4<uint32_t*> starts,
                   B4<uint32_t*> d_nseg, B4<SortScratch> s, hipStream_t st, B4<uint32_t*> seg_of, int nbatch,
                   B4<const uint32_t*> run) {
  const uint32_t nb = rs_blocks(cap) ? rs_blocks(cap) : 1u;
  k_seg_count<K, HasInvalid><<<dim3(nb, nbatch), T, 0, st>>>(keys, d_n, invalid, s, run);
  k_seg_write<K, HasInvalid><<<dim3(nb, nbatch), T, 0, st>>>(keys, d_n, invalid, s, starts, d_nseg, seg_of, run);
}

// Two independent scans may share the launches (gridDim.z = 2): z = 1 scans in2b into
// out2b with its tile totals in the scratch's hist words (free outside a radix sort).
__device__ __forceinline__ uint32_t* scan_blk(const SortScratch& s) { return blockIdx.z ? s.hist : s.blk; }

__global__ void __launch_bounds__(T) k_sum_tiles(B4<const uint32_t*> in2, B4<const uint32_t*> in2b,
                                                 B4<const uint32_t*> d_n2, B4<SortScratch> ss) {
  KT();
  __shared__ uint32_t sh[4];
  const int e = blockIdx.y;
  const uint32_t n = *d_n2[e];
  if (blockIdx.x * RS_TILE >= n && blockIdx.x) return;
  const uint32_t* __restrict__ in = blockIdx.z ? in2b[e] : in2[e];
  const uint32_t i0 = blockIdx.x * RS_TILE + threadIdx.x * RS_CHUNKS;
  uint32_t v[RS_CHUNKS], c = 0;
#pragma unroll
  for (int j = 0; j < RS_CHUNKS; ++j) v[j] = in[min(i0 + j, n ? n - 1u : 0u)];
#pragma unroll
  for (int j = 0; j < RS_CHUNKS; ++j) c += (i0 + j < n) ? v[j] : 0u;
  uint32_t t;
  block_scan_256(c, sh, &t);
  if (threadIdx.x == 0) scan_blk(ss[e])[blockIdx.x] = t;
}

__global__ void __launch_bounds__(T) k_scan_tiles(B4<const uint32_t*> in2, B4<uint32_t*> out2, B4<uint32_t*> d_total2,
                                                  B4<const uint32_t*> in2b, B4<uint32_t*> out2b,
                                                  B4<uint32_t*> d_total2b, B4<const uint32_t*> d_n2,
                                                  B4<SortScratch> ss) {
  KT();
  __shared__ uint32_t sh[4];
  const int e = blockIdx.y;
  const uint32_t n = *d_n2[e];
  if (blockIdx.x * RS_TILE >= n && blockIdx.x) return;
  const uint32_t* __restrict__ in = blockIdx.z ? in2b[e] : in2[e];
  uint32_t* __restrict__ out = blockIdx.z ? out2b[e] : out2[e];
  uint32_t* d_total = blockIdx.z ? d_total2b[e] : d_total2[e];
  const uint32_t i0 = blockIdx.x * RS_TILE + threadIdx.x * RS_CHUNKS;
  uint32_t v[RS_CHUNKS], c = 0;
#pragma unroll
  for (int j = 0; j < RS_CHUNKS; ++j) v[j] = in[min(i0 + j, n ? n - 1u : 0u)];
#pragma unroll
  for (int j = 0; j < RS_CHUNKS; ++j) {
    v[j] = (i0 + j < n) ? v[j] : 0u;
    c += v[j];
  }
  const uint32_t before = tiles_before(scan_blk(ss[e]), sh);
  uint32_t t;
  uint32_t run = before + block_scan_256(c, sh, &t);
  if (threadIdx.x == 0 && owns_last(n) && d_total) *d_total = before + t;
#pragma unroll
  for (int j = 0; j < RS_CHUNKS; ++j) {
    if (i0 + j < n) out[i0 + j] = run;
    run += v[j];
  }
}

}  // namespace

// hist: max(256 words per segment-kernel tile, RS_MAXD per radix tile)
static size_t hist_words(uint32_t cap) {
  return std::max<size_t>(256 * ((size_t)rs_blocks(cap) + 1), (size_t)RS_MAXD * ((size_t)sort_blocks(cap) + 1));
}
size_t sort_scratch_bytes(uint32_t cap) {
  const size_t nb = rs_blocks(cap) + 1;
  return sizeof(uint32_t) * (hist_words(cap) + RS_MAXD + nb + 1) + 256;
}

SortScratch sort_scratch_carve(void* base, uint32_t cap) {
  uint32_t* p = (uint32_t*)base;
  SortScratch s;
  s.hist = p;
  s.tot = p + hist_words(cap);
  s.blk = s.tot + RS_MAXD;
  return s;
}

void radix_sort_u32(B4<uint32_t*> k0, B4<uint32_t*> v0, B4<uint32_t*> k1, B4<uint32_t*> v1, B4<const uint32_t*> d_n,
                    uint32_t cap, B4<const uint32_t*> d_nbits, int fast_bits, bool iota, B4<SortScratch> s,
                    hipStream_t st, int nbatch, B4<const uint32_t*> tail_need) {
  radix_sort<uint32_t>(k0, v0, k1, v1, d_n, cap, d_nbits, fast_bits, iota, s, st, nbatch, tail_need,
                       B4<uint32_t*>(nullptr), B4<uint32_t*>(nullptr));
}
void radix_sort_u64(B4<uint64_t*> k0, B4<uint32_t*> v0, B4<uint64_t*> k1, B4<uint32_t*> v1, B4<const uint32_t*> d_n,
                    uint32_t cap, B4<const uint32_t*> d_nbits, int fast_bits, bool iota, B4<SortScratch> s,
                    hipStream_t st, int nbatch, B4<const uint32_t*> tail_need, B4<uint64_t*> k2, B4<uint32_t*> v2) {
  radix_sort<uint64_t>(k0, v0, k1, v1, d_n, cap, d_nbits, fast_bits, iota, s, st, nbatch, tail_need, k2, v2);
}
void segment_heads_u32(B4<const uint32_t*> keys, B4<const uint32_t*> d_n, uint32_t cap, uint32_t invalid,
                       B4<uint32_t*> starts, B4<uint32_t*> d_nseg, B4<SortScratch> s, hipStream_t st,
                       B4<uint32_t*> seg_of, int nbatch, B4<const uint32_t*> run) {
  segment_heads<uint32_t, true>(keys, d_n, cap, invalid, starts, d_nseg, s, st, seg_of, nbatch, run);
}
void segment_heads_u64(B4<const uint64_t*> keys, B4<const uint32_t*> d_n, uint32_t cap, B4<uint32_t*> starts,
                       B4<uint32_t*> d_nseg, B4<SortScratch> s, hipStream_t st, B4<uint32_t*> seg_of, int nbatch) {
  segment_heads<uint64_t, true>(keys, d_n, cap, ~(uint64_t)0, starts, d_nseg, s, st, seg_of, nbatch,
                                B4<const uint32_t*>(nullptr));
}
void exclusive_scan_u32(B4<const uint32_t*> in, B4<uint32_t*> out, B4<const uint32_t*> d_n, uint32_t cap,
                        B4<uint32_t*> d_total, B4<SortScratch> s, hipStream_t st, int nbatch) {
  const uint32_t nb = rs_blocks(cap) ? rs_blocks(cap) : 1u;
  k_sum_tiles<<<dim3(nb, nbatch), T, 0, st>>>(in, in, d_n, s);
  k_scan_tiles<<<dim3(nb, nbatch), T, 0, st>>>(in, out, d_total, in, out, d_total, d_n, s);
}

void exclusive_scan2_u32(B4<const uint32_t*> in_a, B4<uint32_t*> out_a, B4<uint32_t*> total_a,
                         B4<const uint32_t*> in_b, B4<uint32_t*> out_b, B4<uint32_t*> total_b,
                         B4<const uint32_t*> d_n, uint32_t cap, B4<SortScratch> s, hipStream_t st, int nbatch) {
  const uint32_t nb = rs_blocks(cap) ? rs_blocks(cap) : 1u;
  if ((size_t)nb > hist_words(cap)) throw Error(FCCF_E_INTERNAL, "exclusive_scan2_u32: scratch");
  k_sum_tiles<<<dim3(nb, nbatch, 2), T, 0, st>>>(in_a, in_b, d_n, s);
  k_scan_tiles<<<dim3(nb, nbatch, 2), T, 0, st>>>(in_a, out_a, total_a, in_b, out_b, total_b, d_n, s);
}

}  // namespace fccf
