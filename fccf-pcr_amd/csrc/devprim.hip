// devprim.hip — stable LSD radix sort, run-length segmentation and exclusive scan
// for gfx950.  Wave64-native: per-digit ranks come from 8 ballots per 64-key
// chunk (no 32-lane warp idioms), block = 4 waves, tile = 2048 keys.
#include "probe.h"
#include "devprim.h"

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

template <class K>
__global__ void __launch_bounds__(T) k_rs_hist(const K* __restrict__ keys, const uint32_t* __restrict__ d_n,
                                               const uint32_t* __restrict__ d_nbits, int shift,
                                               uint32_t* __restrict__ hist, uint32_t nblocks) {
  if ((uint32_t)shift >= *d_nbits) return;
  __shared__ uint32_t cnt[256];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t n = *d_n;
  const uint32_t base = blockIdx.x * SORT_TILE;
  const uint32_t end = min(base + (uint32_t)SORT_TILE, n);
  // all 16 loads of the tile are issued before any is consumed (clamped indices,
  // no branches), then one LDS atomic per distinct digit per 64 keys (ballot
  // match): neighbouring keys share their high digits
  K kk[SORT_CHUNKS];
  const uint32_t last = n ? n - 1u : 0u;
#pragma unroll
  for (int c = 0; c < SORT_CHUNKS; ++c) kk[c] = keys[min(base + c * T + threadIdx.x, last)];
#pragma unroll
  for (int c = 0; c < SORT_CHUNKS; ++c) {
    const bool ok = base + c * T + threadIdx.x < end;
    const uint32_t d = (uint32_t)(kk[c] >> shift) & 255u;
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
  hist[threadIdx.x * nblocks + blockIdx.x] = cnt[threadIdx.x];
}

// One block per digit: exclusive scan of that digit's per-block counts in place.
__global__ void __launch_bounds__(T) k_rs_rowscan(uint32_t* __restrict__ hist, uint32_t nblocks,
                                                  uint32_t* __restrict__ tot, const uint32_t* __restrict__ d_nbits,
                                                  int shift) {
  if ((uint32_t)shift >= *d_nbits) return;
  __shared__ uint32_t sh[4];
  const uint32_t d = blockIdx.x;
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nblocks; b0 += T) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t v = i < nblocks ? hist[d * nblocks + i] : 0u;
    uint32_t t;
    const uint32_t ex = block_scan_256(v, sh, &t);
    if (i < nblocks) hist[d * nblocks + i] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) tot[d] = carry;
}

// Ranks a 4096-key tile (wave ballots), stages it in LDS in digit order, then
// writes each digit run to its global slot with consecutive lanes on consecutive
// addresses.  *active (probe, may be null) is cleared when the pass is skipped.
template <class K>
__global__ void __launch_bounds__(T) k_rs_scatter(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                  K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                  const uint32_t* __restrict__ d_n,
                                                  const uint32_t* __restrict__ d_nbits, int shift,
                                                  const uint32_t* __restrict__ hist,
                                                  const uint32_t* __restrict__ tot, uint32_t nblocks, int iota,
                                                  uint32_t* __restrict__ active) {
  const bool run = (uint32_t)shift < *d_nbits;
  if (active && blockIdx.x == 0 && threadIdx.x == 0) *active = run ? 1u : 0u;
  const uint32_t n = *d_n;
  const uint32_t tile0 = blockIdx.x * SORT_TILE;
  if (!run || tile0 >= n) return;  // grids are sized for the capacity; tiles past n are empty
  __shared__ uint32_t gofs[256];     // global slot of the tile's first key of each digit
  __shared__ uint32_t tex[256];      // exclusive digit offsets inside the tile
  __shared__ uint32_t wcnt[4][256];
  __shared__ uint32_t sh[4];
  __shared__ K sk[SORT_TILE];
  __shared__ uint32_t sv[SORT_TILE];
  const uint32_t tid = threadIdx.x, lane = lane_id(), wave = tid >> 6;
  {
    uint32_t t;
    gofs[tid] = block_scan_256(tot[tid], sh, &t) + hist[tid * nblocks + blockIdx.x];
  }
  for (int w = 0; w < 4; ++w) wcnt[w][tid] = 0;
  __syncthreads();
  const uint32_t base = tile0 + wave * (SORT_CHUNKS * 64);
  K kk[SORT_CHUNKS];
  uint32_t vv[SORT_CHUNKS], rk[SORT_CHUNKS], dg[SORT_CHUNKS];
  const uint32_t last = n - 1u;  // n > tile0 >= 0
#pragma unroll
  for (int c = 0; c < SORT_CHUNKS; ++c) {  // all loads in flight before the ranking
    const uint32_t i = min(base + c * 64 + lane, last);
    kk[c] = kin[i];
    vv[c] = iota ? i : vin[i];
  }
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
  {  // per-wave offsets within a digit, tile digit totals, their exclusive scan
    uint32_t acc = 0;
    for (int w = 0; w < 4; ++w) {
      const uint32_t t = wcnt[w][tid];
      wcnt[w][tid] = acc;
      acc += t;
    }
    uint32_t t;
    tex[tid] = block_scan_256(acc, sh, &t);
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
  for (uint32_t j = tid; j < m; j += T) {
    const K k = sk[j];
    const uint32_t d = (uint32_t)(k >> shift) & 255u;
    const uint32_t pos = gofs[d] + (j - tex[d]);
    kout[pos] = k;
    vout[pos] = sv[j];
  }
}

template <class K>
__global__ void k_rs_copyback(const K* __restrict__ k1, const uint32_t* __restrict__ v1, K* __restrict__ k0,
                              uint32_t* __restrict__ v0, const uint32_t* __restrict__ d_n,
                              const uint32_t* __restrict__ d_nbits, int max_passes) {
  const uint32_t p = min(passes_of(*d_nbits), (uint32_t)max_passes);
  if ((p & 1u) == 0u) return;
  const uint32_t n = *d_n;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    k0[i] = k1[i];
    v0[i] = v1[i];
  }
}

template <class K>
void radix_sort(K* k0, uint32_t* v0, K* k1, uint32_t* v1, const uint32_t* d_n, uint32_t cap,
                const uint32_t* d_nbits, int max_bits, bool iota, SortScratch s, hipStream_t st) {
  const uint32_t nb = sort_blocks(cap);
  if (nb == 0) return;
  const int max_passes = (max_bits + 7) / 8;
  K* kb[2] = {k0, k1};
  uint32_t* vb[2] = {v0, v1};
  for (int p = 0; p < max_passes; ++p) {
    const int shift = 8 * p;
    const int src = p & 1, dst = src ^ 1;
    k_rs_hist<K><<<nb, T, 0, st>>>(kb[src], d_n, d_nbits, shift, s.hist, nb);
    k_rs_rowscan<<<256, T, 0, st>>>(s.hist, nb, s.tot, d_nbits, shift);
    FCCF_LAUNCH("k_rs_scatter", (d_n, 2.0 * (sizeof(K) + 4)), k_rs_scatter<K>, nb, T, 0, st, kb[src], vb[src], kb[dst], vb[dst], d_n, d_nbits, shift, s.hist, s.tot, nb, (iota && p == 0) ? 1 : 0, _probe.active());
  }
  const uint32_t g = min(nb * 8u, 2048u);
  k_rs_copyback<K><<<g, 256, 0, st>>>(k1, v1, k0, v0, d_n, d_nbits, max_passes);
}

// ---------------------------------------------------------------- segments / scan
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

template <class K, bool HasInvalid>
__global__ void __launch_bounds__(T) k_seg_count(const K* __restrict__ keys, const uint32_t* __restrict__ d_n,
                                                 K invalid, uint32_t* __restrict__ blk) {
  __shared__ uint32_t sh[4];
  const uint32_t n = *d_n;
  const uint32_t i0 = blockIdx.x * RS_TILE + threadIdx.x * RS_CHUNKS;
  K kk[RS_CHUNKS + 2];
  load_run<K>(keys, i0, n, kk);
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < RS_CHUNKS; ++j) c += head_at<K, HasInvalid>(kk, j, i0 + j, n, invalid) ? 1u : 0u;
  uint32_t t;
  block_scan_256(c, sh, &t);
  if (threadIdx.x == 0) blk[blockIdx.x] = t;
}

// single block: exclusive scan of blk[0..nb) in place, blk[nb] = total, *d_out = total
__global__ void __launch_bounds__(T) k_scan_blocks(uint32_t* __restrict__ blk, uint32_t nb, uint32_t* __restrict__ d_out) {
  __shared__ uint32_t sh[4];
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += T) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t v = i < nb ? blk[i] : 0u;
    uint32_t t;
    const uint32_t ex = block_scan_256(v, sh, &t);
    if (i < nb) blk[i] = carry + ex;
    carry += t;
  }
  if (threadIdx.x == 0) {
    blk[nb] = carry;
    if (d_out) *d_out = carry;
  }
}

template <class K, bool HasInvalid>
__global__ void __launch_bounds__(T) k_seg_write(const K* __restrict__ keys, const uint32_t* __restrict__ d_n,
                                                 K invalid, const uint32_t* __restrict__ blk,
                                                 uint32_t* __restrict__ starts, uint32_t* __restrict__ seg_of) {
  __shared__ uint32_t sh[4];
  const uint32_t n = *d_n;
  const uint32_t i0 = blockIdx.x * RS_TILE + threadIdx.x * RS_CHUNKS;
  K kk[RS_CHUNKS + 2];
  load_run<K>(keys, i0, n, kk);
  bool h[RS_CHUNKS];
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < RS_CHUNKS; ++j) {
    h[j] = head_at<K, HasInvalid>(kk, j, i0 + j, n, invalid);
    c += h[j] ? 1u : 0u;
  }
  uint32_t t;
  uint32_t pos = blk[blockIdx.x] + block_scan_256(c, sh, &t);
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
void segment_heads(const K* keys, const uint32_t* d_n, uint32_t cap, K invalid, uint32_t* starts, uint32_t* d_nseg,
                   SortScratch s, hipStream_t st, uint32_t* seg_of) {
  const uint32_t nb = rs_blocks(cap);
  if (nb == 0) return;
  k_seg_count<K, HasInvalid><<<nb, T, 0, st>>>(keys, d_n, invalid, s.blk);
  k_scan_blocks<<<1, T, 0, st>>>(s.blk, nb, d_nseg);
  k_seg_write<K, HasInvalid><<<nb, T, 0, st>>>(keys, d_n, invalid, s.blk, starts, seg_of);
}

__global__ void __launch_bounds__(T) k_sum_tiles(const uint32_t* __restrict__ in, const uint32_t* __restrict__ d_n,
                                                 uint32_t* __restrict__ blk) {
  __shared__ uint32_t sh[4];
  const uint32_t n = *d_n;
  const uint32_t i0 = blockIdx.x * RS_TILE + threadIdx.x * RS_CHUNKS;
  uint32_t c = 0;
  for (int j = 0; j < RS_CHUNKS; ++j) c += (i0 + j < n) ? in[i0 + j] : 0u;
  uint32_t t;
  block_scan_256(c, sh, &t);
  if (threadIdx.x == 0) blk[blockIdx.x] = t;
}

__global__ void __launch_bounds__(T) k_scan_tiles(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                  const uint32_t* __restrict__ d_n, const uint32_t* __restrict__ blk) {
  __shared__ uint32_t sh[4];
  const uint32_t n = *d_n;
  const uint32_t i0 = blockIdx.x * RS_TILE + threadIdx.x * RS_CHUNKS;
  uint32_t v[RS_CHUNKS], c = 0;
  for (int j = 0; j < RS_CHUNKS; ++j) {
    v[j] = (i0 + j < n) ? in[i0 + j] : 0u;
    c += v[j];
  }
  uint32_t t;
  uint32_t run = blk[blockIdx.x] + block_scan_256(c, sh, &t);
  for (int j = 0; j < RS_CHUNKS; ++j) {
    if (i0 + j < n) out[i0 + j] = run;
    run += v[j];
  }
}

}  // namespace

size_t sort_scratch_bytes(uint32_t cap) {
  const size_t nb = rs_blocks(cap) + 1;
  return sizeof(uint32_t) * (256 * nb + 256 + nb + 1) + 256;
}

SortScratch sort_scratch_carve(void* base, uint32_t cap) {
  const size_t nb = rs_blocks(cap) + 1;
  uint32_t* p = (uint32_t*)base;
  SortScratch s;
  s.hist = p;
  s.tot = p + 256 * nb;
  s.blk = s.tot + 256;
  return s;
}

void radix_sort_u32(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, const uint32_t* d_n, uint32_t cap,
                    const uint32_t* d_nbits, int max_bits, bool iota, SortScratch s, hipStream_t st) {
  radix_sort<uint32_t>(k0, v0, k1, v1, d_n, cap, d_nbits, max_bits, iota, s, st);
}
void radix_sort_u64(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, const uint32_t* d_n, uint32_t cap,
                    const uint32_t* d_nbits, int max_bits, bool iota, SortScratch s, hipStream_t st) {
  radix_sort<uint64_t>(k0, v0, k1, v1, d_n, cap, d_nbits, max_bits, iota, s, st);
}
void segment_heads_u32(const uint32_t* keys, const uint32_t* d_n, uint32_t cap, uint32_t invalid, uint32_t* starts,
                       uint32_t* d_nseg, SortScratch s, hipStream_t st, uint32_t* seg_of) {
  segment_heads<uint32_t, true>(keys, d_n, cap, invalid, starts, d_nseg, s, st, seg_of);
}
void segment_heads_u64(const uint64_t* keys, const uint32_t* d_n, uint32_t cap, uint32_t* starts, uint32_t* d_nseg,
                       SortScratch s, hipStream_t st, uint32_t* seg_of) {
  segment_heads<uint64_t, true>(keys, d_n, cap, ~(uint64_t)0, starts, d_nseg, s, st, seg_of);
}
void exclusive_scan_u32(const uint32_t* in, uint32_t* out, const uint32_t* d_n, uint32_t cap, uint32_t* d_total,
                        SortScratch s, hipStream_t st) {
  const uint32_t nb = rs_blocks(cap);
  if (nb == 0) return;
  k_sum_tiles<<<nb, T, 0, st>>>(in, d_n, s.blk);
  k_scan_blocks<<<1, T, 0, st>>>(s.blk, nb, d_total);
  k_scan_tiles<<<nb, T, 0, st>>>(in, out, d_n, s.blk);
}

}  // namespace fccf
