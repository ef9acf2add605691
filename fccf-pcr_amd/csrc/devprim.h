// devprim.h — device-wide primitives used by the FCCF kernels (gfx950, wave64).
// Every size is read from device memory (d_n) so the whole pipeline can be
// enqueued without host round-trips; grids are sized for the capacity.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exactsum.h"

namespace fccf {

constexpr int RS_THREADS = 256;               // 4 waves
constexpr int RS_CHUNKS = 8;                  // 64-key chunks per wave
constexpr int RS_TILE = RS_THREADS * RS_CHUNKS;  // 2048 keys per block

inline uint32_t rs_blocks(uint32_t cap) { return (cap + RS_TILE - 1) / RS_TILE; }

// Radix sort tiles: 4096 keys per block (hist and scatter).
constexpr int SORT_CHUNKS = 16;
constexpr int SORT_TILE = RS_THREADS * SORT_CHUNKS;
inline uint32_t sort_blocks(uint32_t cap) { return (cap + SORT_TILE - 1) / SORT_TILE; }

// Scratch for radix_sort_pairs / segment_heads: hist needs 256*blocks u32,
// tot 256 u32, blk blocks+1 u32.
struct SortScratch {
  uint32_t* hist;
  uint32_t* tot;
  uint32_t* blk;
};
size_t sort_scratch_bytes(uint32_t cap);
SortScratch sort_scratch_carve(void* base, uint32_t cap);

// Stable LSD radix sort of (key, val) by the low *d_nbits bits of key (8-bit
// digits).  The sorted result is always left in (k0, v0); (k1, v1) are temporaries.
// If vals_iota, v0 is ignored on input and the values are the input positions.
void radix_sort_u32(uint32_t* k0, uint32_t* v0, uint32_t* k1, uint32_t* v1, const uint32_t* d_n,
                    uint32_t cap, const uint32_t* d_nbits, int max_bits, bool vals_iota,
                    SortScratch s, hipStream_t st);
void radix_sort_u64(uint64_t* k0, uint32_t* v0, uint64_t* k1, uint32_t* v1, const uint32_t* d_n,
                    uint32_t cap, const uint32_t* d_nbits, int max_bits, bool vals_iota,
                    SortScratch s, hipStream_t st);

// Run-length segmentation of sorted keys[0..*d_n): starts[s] = first index of
// segment s, starts[S] = *d_n, *d_nseg = S.  Keys equal to `invalid` (which sort
// last) are excluded: the valid prefix ends at the first invalid key.
// seg_of (optional): segment index of every valid element.
void segment_heads_u32(const uint32_t* keys, const uint32_t* d_n, uint32_t cap, uint32_t invalid,
                       uint32_t* starts, uint32_t* d_nseg, SortScratch s, hipStream_t st,
                       uint32_t* seg_of = nullptr);
void segment_heads_u64(const uint64_t* keys, const uint32_t* d_n, uint32_t cap, uint32_t* starts,
                       uint32_t* d_nseg, SortScratch s, hipStream_t st, uint32_t* seg_of = nullptr);

// Sequential float sums in the reference's left-to-right order, s = ((0 + v0) + v1) + ...
// bit-exact, computed in parallel (exactsum.h).  Problem b sums elements
// [off[b], off[b] + cnt[b]) of `data` (off may be null = 0); an element is S
// consecutive floats (S = 1 or 3) and its first K components are summed
// independently into out[b*K + k] (divided by the count if `divide`).
// Scratch: exact_sum_carve(rows = nprob*K, cap = max elements per problem).
size_t exact_sum_bytes(int rows, uint32_t cap);
XsBufs exact_sum_carve(void* base, int rows, uint32_t cap);
void exact_sum(const float* data, int S, int K, const uint32_t* off, const uint32_t* cnt, int nprob, float* out,
               bool divide, XsBufs x, hipStream_t st);

// The same for two separate arrays: problem 0 = a[0..*na), problem 1 = b[0..*nb);
// out[0..K) and out[K..2K).  Scratch: rows = 2*K, cap = max of both counts.
void exact_sum2(const float* a, const uint32_t* na, const float* b, const uint32_t* nb, int S, int K, float* out,
                bool divide, XsBufs x, hipStream_t st);

// Exclusive scan of u32 values in[0..*d_n) -> out, *d_total = sum.
void exclusive_scan_u32(const uint32_t* in, uint32_t* out, const uint32_t* d_n, uint32_t cap,
                        uint32_t* d_total, SortScratch s, hipStream_t st);

}  // namespace fccf
