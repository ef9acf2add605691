// devprim.h — device-wide primitives used by the FCCF kernels (gfx950, wave64).
// Every size is read from device memory (d_n) so the whole pipeline can be
// enqueued without host round-trips; grids are sized for the capacity.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "exactsum.h"
#include "ktrace.h"

namespace fccf {

constexpr int RS_THREADS = 256;               // 4 waves
constexpr int RS_CHUNKS = 8;                  // 64-key chunks per wave
constexpr int RS_TILE = RS_THREADS * RS_CHUNKS;  // 2048 keys per block

inline uint32_t rs_blocks(uint32_t cap) { return (cap + RS_TILE - 1) / RS_TILE; }

// Radix sort tiles: 4096 keys per block of 1024 threads (hist and scatter).
constexpr int SORT_THREADS = 1024;
#ifndef SORT_CHUNKS_VAL
#define SORT_CHUNKS_VAL 4
#endif
constexpr int SORT_CHUNKS = SORT_CHUNKS_VAL;
constexpr int SORT_TILE = SORT_THREADS * SORT_CHUNKS;
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

// Per-problem arguments of a batched launch: problem e = blockIdx.y uses v[e].
// The primitives below run `nbatch` (1 to BMAX) independent problems -- the clouds of
// one registration, or of the registrations that a pipelined batch runs together --
// in the same launches (a kernel boundary costs ~1.7 us on gfx950 and two streams of
// dependent kernels interfere, so one stream of batched launches is the fast shape).
// A single value converts to a batch of one; entries past the ones given repeat the
// last (never read: problems past nbatch do not run).
constexpr int BMAX = 10;
template <class T>
struct B4 {
  T v[BMAX];
  B4() = default;
  __host__ __device__ B4(T a) {
    for (int i = 0; i < BMAX; ++i) v[i] = a;
  }
  __host__ __device__ B4(T a, T b) {
    v[0] = a;
    for (int i = 1; i < BMAX; ++i) v[i] = b;
  }
  __host__ __device__ B4(T a, T b, T c, T d) {
    v[0] = a;
    v[1] = b;
    v[2] = c;
    for (int i = 3; i < BMAX; ++i) v[i] = d;
  }
  // the first n of a[] (n >= 1)
  __host__ __device__ B4(const T* a, int n) {
    for (int i = 0; i < BMAX; ++i) v[i] = a[i < n ? i : n - 1];
  }
  template <class U>
  __host__ __device__ B4(const B4<U>& o) {
    for (int i = 0; i < BMAX; ++i) v[i] = o.v[i];
  }
  // (an index into the kernel argument: ROCm 7.2 reads the selected entry from the
  // kernarg segment with scalar loads -- no scratch copy, fewer SGPRs than a select
  // chain, which on structs of four entries made the compiler spill to scratch; an
  // older toolchain copied such arguments to a private array, round 1)
  __host__ __device__ __forceinline__ T operator[](int i) const { return v[i]; }
};

// Stable LSD radix sort of (key, val) by the low *d_nbits bits of key (8-bit
// digits).  The sorted result is always left in (k0, v0); (k1, v1) are temporaries.
// If vals_iota, v0 is ignored on input and the values are the input positions.
// Keys-only: v0 = v1 = null (no value traffic).
// cap bounds every problem's count.  fast_bits / 8 passes of the device-side digit
// plan run as device-wide passes (3 launches each, a pass past the plan exits at
// once); the bits they leave run in one single-workgroup tail launch (k_rs_tail),
// which also exits at once unless needed.  tail_need (optional): the tail runs only
// where *tail_need != 0 (fast_bits == 0: a sort of keys usually already in order).
void radix_sort_u32(B4<uint32_t*> k0, B4<uint32_t*> v0, B4<uint32_t*> k1, B4<uint32_t*> v1, B4<const uint32_t*> d_n,
                    uint32_t cap, B4<const uint32_t*> d_nbits, int fast_bits, bool vals_iota, B4<SortScratch> s,
                    hipStream_t st, int nbatch = 1, B4<const uint32_t*> tail_need = B4<const uint32_t*>(nullptr));
// (k2, v2) optional: a third buffer, so a sort of three active passes ends in (k0, v0)
// without a copy-back.
void radix_sort_u64(B4<uint64_t*> k0, B4<uint32_t*> v0, B4<uint64_t*> k1, B4<uint32_t*> v1, B4<const uint32_t*> d_n,
                    uint32_t cap, B4<const uint32_t*> d_nbits, int fast_bits, bool vals_iota, B4<SortScratch> s,
                    hipStream_t st, int nbatch = 1, B4<const uint32_t*> tail_need = B4<const uint32_t*>(nullptr),
                    B4<uint64_t*> k2 = B4<uint64_t*>(nullptr), B4<uint32_t*> v2 = B4<uint32_t*>(nullptr));

// Run-length segmentation of sorted keys[0..*d_n): starts[s] = first index of
// segment s, starts[S] = *d_n, *d_nseg = S.  Keys equal to `invalid` (which sort
// last) are excluded: the valid prefix ends at the first invalid key.
// seg_of (optional): segment index of every valid element.
// run (optional): skip problems whose *run == 0 (their outputs are left untouched).
void segment_heads_u32(B4<const uint32_t*> keys, B4<const uint32_t*> d_n, uint32_t cap, uint32_t invalid,
                       B4<uint32_t*> starts, B4<uint32_t*> d_nseg, B4<SortScratch> s, hipStream_t st,
                       B4<uint32_t*> seg_of = B4<uint32_t*>(nullptr), int nbatch = 1,
                       B4<const uint32_t*> run = B4<const uint32_t*>(nullptr));
void segment_heads_u64(B4<const uint64_t*> keys, B4<const uint32_t*> d_n, uint32_t cap, B4<uint32_t*> starts,
                       B4<uint32_t*> d_nseg, B4<SortScratch> s, hipStream_t st,
                       B4<uint32_t*> seg_of = B4<uint32_t*>(nullptr), int nbatch = 1);

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
// The same for nprob (1 to 4) separate arrays data[b] with counts *cnt[b]; out = nprob * K values.
void exact_sum_n(const float* const* data, const uint32_t* const* cnt, int nprob, int S, int K, float* out, bool divide,
                 XsBufs x, hipStream_t st);

// Exclusive scan of u32 values in[0..*d_n) -> out, *d_total = sum.
void exclusive_scan_u32(B4<const uint32_t*> in, B4<uint32_t*> out, B4<const uint32_t*> d_n, uint32_t cap,
                        B4<uint32_t*> d_total, B4<SortScratch> s, hipStream_t st, int nbatch = 1);
// Two such scans of the same length in the same two launches (the second's tile
// totals use the scratch's radix histogram words, unused outside a sort).
void exclusive_scan2_u32(B4<const uint32_t*> in_a, B4<uint32_t*> out_a, B4<uint32_t*> total_a,
                         B4<const uint32_t*> in_b, B4<uint32_t*> out_b, B4<uint32_t*> total_b,
                         B4<const uint32_t*> d_n, uint32_t cap, B4<SortScratch> s, hipStream_t st, int nbatch = 1);

}  // namespace fccf
