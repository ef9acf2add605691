// introsort.hip — K1's sort in the reference's order: libstdc++ std::sort
// (introsort) of PCL VoxelGrid's (idx, cloud_point_index) pairs, compared by idx
// only.  Reference: FCCF.cpp:1668-1678 (main) and :1377-1387 (driver), both through
// pcl::VoxelGrid<PointXYZ>::applyFilter, whose std::sort leaves the points of one
// leaf in introsort's (unstable) order; the centroid sums them in that order
// (SURVEY.md App. A2 steps 6-7).  The result equals std::sort bit for bit
// (tests/test_gpu_introsort.py, tools/introsort_model.cpp).
//
// libstdc++ std::sort = __introsort_loop(depth 2*lg(n)) + a final insertion sort:
//  * a segment of more than 16 elements is partitioned after
//    __move_median_to_first(first, first+1, mid, last-1); at depth 0 it is heap sorted;
//  * __unguarded_partition(first+1, last, pivot=*first) swaps the k-th element >= P
//    from the left (L[k]) with the k-th element <= P from the right (R[k]) for
//    k = 1..K, the prefix where L[k] < R[k], and returns cut = min(L[K+1], R[K]).
//    So an element >= P with ge-rank k is swapped iff (#<=P after it) >= k, an
//    element <= P with right-rank k iff (#>=P before it) >= k: prefix counts decide
//    every move, no sequential scan is needed;
//  * the final insertion sort is stable and every leaf segment is bounded by its
//    neighbours, so the output is each leaf segment stably sorted in place.
//
// GPU structure (per cloud; both clouds of a registration in the same launches):
//  k_is_prep   stable compaction of non-finite points (PCL skips them), sort length;
//  rounds      the first R levels over segments > IS_LCAP, many workgroups each:
//              k_is_count (pivot, per-tile ge/le counts and tile-local position
//              lists) and k_is_scatter (ranks from the tile prefix, every element
//              written to its destination in the other buffer, cut by atomicMin);
//  k_is_block  one workgroup per remaining segment (dequeued; single registrations take
//              them longest first, k_is_order): partitions in global memory while a
//              segment exceeds IS_LCAP, then in LDS down to subtrees of <= IS_WCAP,
//              which become wave tasks; leaves are finished here;
//  k_is_wave   every wave of a resident grid finishes tasks in its own LDS slice, the
//              longest first (k_is_torder) from a per-cloud counter (wave partitions,
//              register-resident subtrees of <= 64, stable leaf sort).
// HBM per round: 4 B/elem (count) + 4 B lists + 16 B (scatter); the block and wave
// kernels read and write each element once more each (8 + 8 B).
#ifndef KT_TU
#define KT_TU 9  // ktrace.h source tag (introsort_b2.hip: 13)
#endif
#include <cstdio>
#include <cstdlib>

#include "probe.h"
#include "kernels.h"

namespace fccf {
namespace {

#ifndef IS_TILE_VAL
#define IS_TILE_VAL 2048
#endif
// elements per round tile (small clouds).  4096 (-DIS_TILE_VAL=4096) measured at four
// pairs per stage: pipelined the same (0.865-0.871 vs 0.847-0.870 ms), single
// registration slower (main VoxelGrid 0.83 vs 0.73 ms)
constexpr uint32_t IS_TILE = IS_TILE_VAL;
constexpr uint32_t IS_TILE_L = 4096;  // elements per round tile (large clouds: fewer workgroup latency chains)
// clouds from this size plan each round once (k_is_count_plan; sharded sorts always):
// c5 (10M) 7.93 ms per registration with it vs 10.6 without, c4 (5M) 3.98 vs 3.85
// (profiles/r03l), so the crossover lies between
constexpr uint32_t IS_LARGE_MIN = 1u << 23;
constexpr int IS_NSH = 64;                       // round kernels: completion counter shards (last_block)
constexpr int IS_DONE_WORDS = (IS_NSH + 1) * 32;  // u32 per launch: shards + top, 128 B apart
constexpr int IS_TT = 256;           // round kernels: threads per block
constexpr int IS_TC = IS_TILE / IS_TT;  // 8 elements per thread
#ifndef IS_LCAP_VAL
#define IS_LCAP_VAL 8192
#endif
constexpr uint32_t IS_LCAP = IS_LCAP_VAL;  // largest segment a block kernel workgroup holds in LDS
#ifndef IS_OT_VAL
#define IS_OT_VAL 1024
#endif
constexpr int IS_OT = IS_OT_VAL;     // block kernel: threads per block (16 waves, one block per CU)
constexpr int IS_OW = IS_OT / 64;    // block kernel: waves
constexpr int IS_OC = IS_LCAP / IS_OT;  // 8 elements per thread in a workgroup partition
constexpr uint32_t IS_OE = IS_OC * IS_OW;  // (chunk, wave) count entries of a workgroup partition
#ifndef IS_WCAP_VAL
#define IS_WCAP_VAL 512
#endif
constexpr uint32_t IS_WCAP = IS_WCAP_VAL;  // largest subtree finished by one wave (wave kernel)
constexpr int IS_WC = IS_WCAP / 64;  // 8 elements per lane
constexpr int IS_WT = 256;           // wave kernel: threads per block
constexpr uint32_t IS_TASK_BIG = 128;  // wave tasks above this are dequeued first
constexpr uint32_t IS_THRESHOLD = 16;  // libstdc++ _S_threshold
constexpr int IS_STACK = 96;  // a wave's stack also holds its register-mode subtree (depth <= 48 each)
#ifndef IS_SEGT_MINC
#define IS_SEGT_MINC 2  // wave_task_level: per-segment table from this many chunks per lane up
#endif
// packed u32 subtree of at most IS_WCAP elements: off (13 bits) | len (11) | depth (6)
__device__ __forceinline__ uint32_t wpack(uint32_t off, uint32_t len, int d) { return off | (len << 13) | ((uint32_t)d << 24); }
constexpr uint32_t IS_NONE = 0xFFFFFFFFu;
#ifndef IS_STATS
#define IS_STATS 1  // path counters in IsBufs::ctl[3..], when IsBufs::stats (debug sorts only)
#endif

#ifdef IS_PHASES
// Development (variant builds, make VAR=ph EXTRA=-DIS_PHASES): per-phase shader cycles
// of an instrumented kernel (thread 0 after each barrier), summed over workgroups, read
// with fccf_debug_is_phases (tools/is_phases.py).
__device__ unsigned long long g_is_ph[32];
__device__ unsigned long long g_is_ph_last[4096];
#define IS_PH(k)                                                                   \
  do {                                                                             \
    if (threadIdx.x == 0) {                                                        \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();                  \
      const unsigned slot_ = (blockIdx.x + blockIdx.y * gridDim.x) & 4095u;        \
      atomicAdd(&g_is_ph[(k)], t_ - g_is_ph_last[slot_]);                         \
      atomicAdd(&g_is_ph[16 + (k)], 1ull);                                         \
      g_is_ph_last[slot_] = t_;                                                    \
    }                                                                              \
  } while (0)
#define IS_PH_START()                                                              \
  do {                                                                             \
    if (threadIdx.x == 0)                                                          \
      g_is_ph_last[(blockIdx.x + blockIdx.y * gridDim.x) & 4095u] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define IS_PH(k) do {} while (0)
#define IS_PH_START() do {} while (0)
#endif
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63u; }
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
__device__ __forceinline__ int depth0(uint32_t n) { return n ? 2 * (31 - __clz((int)n)) : 0; }  // 2*std::__lg(n)
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// An invariant violation (IS_FAULT_*, kernels.h): recorded in the sort's ctl[2] and in
// the cloud's VGParams::sort_err, which the host turns into FCCF_E_INTERNAL.
__device__ __forceinline__ void is_fault(uint32_t* ctl, uint32_t* err, uint32_t bits) {
  atomicOr(&ctl[2], bits);
  if (err) atomicOr(err, bits);
}
// Test hook: the injected flags of `bits` (fccf_debug_inject_sort_fault), raised by the
// caller's one designated thread.
__device__ __forceinline__ void is_inject(const IsBufs& W, uint32_t bits) {
  if (!W.inject) return;
  const uint32_t b = *W.inject & bits;
  if (b) is_fault(W.ctl, W.err, b);
}

// A final (key, value) write's point, when the sort writes sorted points (IsBufs::xyzs).
// The points are read and written as one 12-byte global access each (the source pointer
// comes from memory, so without the address-space cast the compiler emits flat loads,
// which also wait on LDS traffic); callers with several points issue every load before
// the first store (load_xyz / store_xyz), so the random gathers overlap instead of each
// waiting out its own memory latency.
struct Pt3 {
  float x, y, z;
};
// (the global address space exists only in the device compilation of this file)
#if defined(__HIP_DEVICE_COMPILE__)
typedef __attribute__((address_space(1))) const Pt3* GPt3c;
typedef __attribute__((address_space(1))) Pt3* GPt3;
#else
typedef const Pt3* GPt3c;
typedef Pt3* GPt3;
#endif
__device__ __forceinline__ Pt3 load_xyz(const float* src, uint32_t v) { return ((GPt3c)(const Pt3*)src)[v]; }
__device__ __forceinline__ void store_xyz(const IsBufs& W, uint32_t pos, const Pt3& q) { ((GPt3)(Pt3*)W.xyzs)[pos] = q; }
__device__ __forceinline__ void put_xyz(const IsBufs& W, const float* __restrict__ src, uint32_t pos, uint32_t v) {
  // (a random 12-B load: one line each, overlapped by the finish kernels' LDS work;
  // a separate gather pass cost 170 us per ten clouds and saved nothing, profiles/r06a)
  store_xyz(W, pos, load_xyz(src, v));
}

// The fence before a workgroup barrier that hands global-memory data between the waves
// of one workgroup (k_is_block's global phase).  Every sort kernel runs with TG_SPLIT = 0
// (COMPUTE_PGM_RSRC3 bit 16; checked in tools/check_tgsplit.py), so all waves of a
// workgroup share one CU and its vector L1, and the segment a workgroup works on is
// touched by no other workgroup during the kernel: a workgroup-scope fence is enough by
// the memory model.  The agent-scope fence is kept as the product default (measured
// cost: DESIGN.md, "Sort edge behaviour"); -DIS_WG_FENCE builds the workgroup form.
__device__ __forceinline__ void hand_off_fence() {
#ifdef IS_WG_FENCE
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
#else
  __threadfence();
#endif
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return v;
}

// __move_median_to_first(first, first+1, mid, last-1): the position whose element
// becomes the pivot (requires l - f > 16, so the three positions are distinct)
template <class KP>
__device__ __forceinline__ uint32_t median_pos(KP K, uint32_t f, uint32_t l) {
  const uint32_t A = f + 1, B = f + (l - f) / 2, C = l - 1;
  const uint32_t a = K[A], b = K[B], c = K[C];
  if (a < b) {
    if (b < c) return B;
    if (a < c) return C;
    return A;
  }
  if (a < c) return A;
  if (b < c) return C;
  return B;
}

// median_pos together with the four values a round's partition needs -- the pivot P =
// K[m] and V[m], the first element K[f], V[f] -- from ONE round of global loads: the
// median is one of the three probed positions, so their values are loaded with the keys
// (the count kernels' thread 0 otherwise chains three dependent round trips: the
// probes, then K[m], then the values; profiles/r03p)
template <class KP, class VP>
__device__ __forceinline__ void median_load(KP K, VP V, uint32_t f, uint32_t l, uint32_t& m, uint32_t& P,
                                            uint32_t& vm, uint32_t& kf, uint32_t& vf) {
  const uint32_t A = f + 1, B = f + (l - f) / 2, C = l - 1;
  const uint32_t a = K[A], b = K[B], c = K[C], va = V[A], vb = V[B], vc = V[C];
  kf = K[f];
  vf = V[f];
  int pick;  // 0: A, 1: B, 2: C (median_pos's comparisons)
  if (a < b) pick = b < c ? 1 : (a < c ? 2 : 0);
  else pick = a < c ? 0 : (b < c ? 2 : 1);
  m = pick == 0 ? A : (pick == 1 ? B : C);
  P = pick == 0 ? a : (pick == 1 ? b : c);
  vm = pick == 0 ? va : (pick == 1 ? vb : vc);
}

// std::__adjust_heap / __make_heap / __sort_heap on (K, V) pairs by key (one thread)
template <class KP, class VP>
__device__ __forceinline__ void adjust_heap(KP K, VP V, int64_t hole, int64_t len, uint32_t vk, uint32_t vv) {
  const int64_t top = hole;
  int64_t sc = hole;
  while (sc < (len - 1) / 2) {
    sc = 2 * (sc + 1);
    if (K[sc] < K[sc - 1]) sc--;
    K[hole] = K[sc];
    V[hole] = V[sc];
    hole = sc;
  }
  if ((len & 1) == 0 && sc == (len - 2) / 2) {
    sc = 2 * (sc + 1);
    K[hole] = K[sc - 1];
    V[hole] = V[sc - 1];
    hole = sc - 1;
  }
  int64_t parent = (hole - 1) / 2;
  while (hole > top && K[parent] < vk) {
    K[hole] = K[parent];
    V[hole] = V[parent];
    hole = parent;
    parent = (hole - 1) / 2;
  }
  K[hole] = vk;
  V[hole] = vv;
}
template <class KP, class VP>
__device__ __forceinline__ void heap_sort(KP K, VP V, int64_t len) {  // std::__partial_sort(first, last, last)
  if (len < 2) return;
  for (int64_t parent = (len - 2) / 2;; parent--) {
    adjust_heap(K, V, parent, len, K[parent], V[parent]);
    if (parent == 0) break;
  }
  for (int64_t last = len - 1; last > 0; --last) {
    const uint32_t vk = K[last], vv = V[last];
    K[last] = K[0];
    V[last] = V[0];
    adjust_heap(K, V, 0, last, vk, vv);
  }
}

// The depth-limit step of std::sort is std::__partial_sort(first, last, last), a heap
// sort, whose only freedom is the order of equal keys.  With pairwise distinct keys the
// sorted order is unique, so the heap sort's result puts every element at its segment
// start + #smaller keys: the parallel forms below rank each element against its
// segment (reporting in dup whether another element has the same key), and only a
// segment with a repeated key keeps the sequential heap sort for its tie order.
__device__ __forceinline__ uint32_t rank_in_segment(const uint32_t* k, uint32_t a, uint32_t b, uint32_t p, uint32_t key,
                                                    bool& dup) {
  uint32_t r = 0;
  for (uint32_t q = a; q < b; ++q) {
    const uint32_t kq = k[q];
    r += kq < key ? 1u : 0u;
    dup |= kq == key && q != p;
  }
  return r;
}

// Exclusive scan over the whole block (blockDim a multiple of 64, <= 1024); sh >= 16 u32.
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* sh, uint32_t* total) {
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  uint32_t wp = 0, tot = 0;
  for (uint32_t w = 0; w < nw; ++w) {
    wp += w < wave ? sh[w] : 0u;
    tot += sh[w];
  }
  __syncthreads();
  *total = tot;
  return wp + x - v;
}

// The same for packed 64-bit counters (several fields summed at once, no carries
// between them by construction); sh >= 16 u64.
__device__ __forceinline__ uint64_t block_excl_scan64(uint64_t v, uint64_t* sh, uint64_t* total) {
  const uint32_t lane = lane_id(), wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint64_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  uint64_t wp = 0, tot = 0;
  for (uint32_t w = 0; w < nw; ++w) {
    wp += w < wave ? sh[w] : 0ull;
    tot += sh[w];
  }
  __syncthreads();
  *total = tot;
  return wp + x - v;
}

struct Child {
  uint32_t f, l;
  int32_t d;
};
// children of round r-1's partitioned segments in position order (r == 0: the root)
__device__ __forceinline__ Child child_of(const IsBufs& W, int r, uint32_t nsort, uint32_t i) {
  if (r == 0) return {0u, nsort, depth0(nsort)};
  const IsSeg s = W.segs[(size_t)(r - 1) * W.segmax + i / 2];
  // a cut lies in (f, l) by construction; clamped so that a defect cannot address
  // outside the segment (it would show as a wrong order, never as a fault)
  const uint32_t c = min(max(W.cuts[(size_t)(r - 1) * W.segmax + i / 2], s.f + 1), s.l - 1);
  return (i & 1) ? Child{c, s.l, s.depth - 1} : Child{s.f, c, s.depth - 1};
}
__device__ __forceinline__ uint32_t nchildren(const IsBufs& W, int r) { return r == 0 ? 1u : 2u * W.rounds[r - 1].nseg; }
__device__ __forceinline__ bool is_large(const Child& c, uint32_t tier) { return c.l - c.f > tier && c.d > 0; }
__device__ __forceinline__ uint32_t tiles_of(uint32_t len) { return (len - 1 + IS_TILE - 1) / IS_TILE; }
constexpr int IS_TC_L = IS_TILE_L / IS_TT;  // 16 elements per thread (large-cloud rounds)
__device__ __forceinline__ uint32_t tiles_of_l(uint32_t len) { return (len - 1 + IS_TILE_L - 1) / IS_TILE_L; }

// largest u < n with pre[u] <= x (pre ascending, pre[0] = 0)
__device__ __forceinline__ uint32_t upper_index(const uint32_t* pre, uint32_t n, uint32_t x) {
  uint32_t lo = 0, hi = n;  // answer in [lo, hi)
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    if (pre[mid] <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}
// the same over a segment's tile prefixes in global memory (component 0: >=, 1: <=)
__device__ __forceinline__ uint32_t upper_index_g(const uint2* pre, uint32_t n, uint32_t x, int comp) {
  uint32_t lo = 0, hi = n;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) >> 1;
    const uint2 v = pre[mid];
    if ((comp ? v.y : v.x) <= x) lo = mid;
    else hi = mid;
  }
  return lo;
}

__device__ void plan_round(const IsBufs& W, int r, uint32_t nsort, uint64_t* sh64);

// ---------------------------------------------------------------- k_is_prep
// PCL pushes only finite points into its index vector, in input order: compact the
// (key, index) pairs of finite points (rare: only when some point is not finite) and
// mark the tail invalid.  ctl[0] = sort length, ctl[1] = k_is_block's dequeue head;
// the rounds' completion counters zeroed and round 0 planned (plan_round).
// exact_gate (the driver's presorted second pass): sort only when the order check failed.
__global__ void __launch_bounds__(1024) k_is_prep(B4<uint32_t*> K2, B4<uint32_t*> V2, B4<const uint32_t*> d_n2,
                                                   B4<const VGParams*> P2, B4<IsBufs> W2, int exact_gate) {
  KT();
  const int e = blockIdx.y;
  const IsBufs W = W2[e];
  const VGParams* P = P2[e];
  const uint32_t n = *d_n2[e];
  uint32_t ns = (P->overflow || P->nfinite == 0) ? 0u : P->nfinite;
  if (exact_gate && P->unsorted == 0u) ns = 0;
  if (threadIdx.x == 0) {
    W.ctl[0] = ns;
    for (int i = 1; i < 32; ++i) W.ctl[i] = 0;
  }
  for (int i = threadIdx.x; i < 2 * IS_RMAX * IS_DONE_WORDS; i += 1024) W.done[i] = 0;
  // Test hook (IS_POISON_XYZS): the sorted points are NaN before the sort, so a final
  // position that no put_xyz writes shows up as a NaN centroid instead of reading the
  // previous registration's point (the arena is reused)
  if (W.xyzs && W.inject && (*W.inject & IS_POISON_XYZS))
    for (uint32_t i = threadIdx.x; i < 3 * n; i += 1024) W.xyzs[i] = __uint_as_float(0x7FC00000u);
  if (ns > 0 && ns < n) {
    uint32_t* K = K2[e];
    uint32_t* V = V2[e];
    __shared__ uint32_t sh[16];
    uint32_t out = 0;
    for (uint32_t b = 0; b < n; b += 1024) {
      const uint32_t i = b + threadIdx.x;
      const uint32_t k = i < n ? K[i] : IS_NONE, v = i < n ? V[i] : 0u;
      const uint32_t keep = k != IS_NONE;
      uint32_t tot;
      const uint32_t o = block_excl_scan(keep, sh, &tot);  // its barriers order these reads before the writes
      if (keep) {
        K[out + o] = k;
        V[out + o] = v;
      }
      out += tot;
      __syncthreads();
    }
    for (uint32_t i = ns + threadIdx.x; i < n; i += 1024) K[i] = IS_NONE;
  }
  __shared__ uint64_t sh64[16];
  plan_round(W, 0, ns, sh64);
}

// ---------------------------------------------------------------- rounds
// Per round r, two launches over maxtiles workgroups (one 2048-element tile each):
//  k_is_count_plan  the tile's ge/le counts against its segment's pivot and the
//                   tile-local position lists; the LAST workgroup to finish turns all
//                   tiles' counts into each segment's exclusive tile prefix (pre) and
//                   its <= total (letot), once for the round;
//  k_is_scatter     ranks from that prefix, every element to its place after the
//                   partition in the other buffer, the cut by atomicMin; the LAST
//                   workgroup plans round r+1 (plan_round).
// Round 0 is planned by k_is_prep.  (Before, every workgroup re-derived the round's
// segment table and re-scanned its whole segment's tile counts: at c5 that was ~10K
// workgroups x up to ~5K entries of block scans per launch, most of the rounds' time.)
//
// Hand-offs inside one launch (to its last workgroup): written with agent-scope
// atomics (performed at the coherence point), read with atomic read-modify-writes
// after an agent-scope acquire, so no stale L1 or L2 copy on another XCD is read
// (MI355X_MICROARCH.md, inter-workgroup visibility); every storing wave drains
// (s_waitcnt vmcnt(0)) before the barrier that precedes its workgroup's counter add.
// Everything else is consumed by a later launch.
__device__ __forceinline__ void drain_vm() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
__device__ __forceinline__ uint32_t coherent_load(uint32_t* p) { return atomicAdd(p, 0u); }

// Whether this workgroup is the last of its grid row to get here.  done: the launch's
// IS_DONE_WORDS counters (zeroed by k_is_prep): IS_NSH shard counters and a top one,
// each on its own 128-byte line -- same-address atomics serialise (~18 ns each), so one
// counter for thousands of workgroups cost ~0.1 ms per launch at c5.  The last of a
// shard adds to the top counter; the last there is the grid's last.  Every thread of
// every workgroup must call it; the last workgroup returns true (in all threads) after
// an agent-scope acquire.
__device__ bool last_block(uint32_t* done, uint32_t* sflag) {
  drain_vm();
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t sh = blockIdx.x % IS_NSH, nsh = min((uint32_t)IS_NSH, gridDim.x);
    const uint32_t members = (gridDim.x - sh + IS_NSH - 1) / IS_NSH;
    bool last = false;
    if (atomicAdd(&done[sh * 32], 1u) == members - 1u) last = atomicAdd(&done[IS_NSH * 32], 1u) == nsh - 1u;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      drain_vm();
    }
    *sflag = last ? 1u : 0u;
  }
  __syncthreads();
  return *sflag != 0u;
}

// child_of, reading round r-1's cut with an atomic (it was set by the atomicMin of
// workgroups of the same launch: the planner in k_is_scatter's last workgroup)
__device__ __forceinline__ Child child_coherent(const IsBufs& W, int r, uint32_t nsort, uint32_t i) {
  if (r == 0) return {0u, nsort, depth0(nsort)};
  const IsSeg s = W.segs[(size_t)(r - 1) * W.segmax + i / 2];
  const uint32_t c = min(max(coherent_load(&W.cuts[(size_t)(r - 1) * W.segmax + i / 2]), s.f + 1), s.l - 1);
  return (i & 1) ? Child{c, s.l, s.depth - 1} : Child{s.f, c, s.depth - 1};
}

// Largest u < n with key(u) <= x, by one wave (key(0) <= x and key ascending): a
// 64-ary search, one load per lane and a ballot per step, ~log64(n) dependent loads.
template <class KeyAt>
__device__ __forceinline__ uint32_t wave_upper_index(KeyAt key, uint32_t n, uint32_t x) {
  const uint32_t lane = lane_id();
  uint32_t lo = 0, hi = n;  // answer in [lo, hi), key(lo) <= x
  while (hi - lo > 1) {
    const uint32_t stride = (hi - lo + 63) / 64;
    const uint32_t idx = lo + lane * stride;
    const uint64_t m = __ballot(idx < hi && key(idx) <= x);  // bit 0 set: key(lo) <= x
    const uint32_t nlo = lo + (63u - (uint32_t)__clzll((long long)m)) * stride;
    hi = min(hi, nlo + stride);
    lo = nlo;
    if (stride == 1) break;
  }
  return lo;
}

// The plan of round r, by one workgroup: the children of round r-1's segments (the
// root for r = 0) longer than the tier become the round's segments (ptab: f, l, depth,
// first tile), the shorter non-empty children go to the owned list, and the IsRound
// record.  PL children per thread per step (their cut loads in flight together).
constexpr int PL = 8;
__device__ void plan_round(const IsBufs& W, int r, uint32_t nsort, uint64_t* sh64) {
  const uint32_t nch = nchildren(W, r);
  const uint32_t own_base = r ? W.rounds[r - 1].nown : 0u;
  uint32_t nseg = 0, ntiles = 0, nown = 0;
  // Row D: from round shard_r0 on only the children starting in this rank's range.  At
  // shard_r0 the bounds are set here: bound j = the first child start >= j * nsort / N
  // (a child's start is always a segment boundary: the owned segments of earlier rounds
  // lie between the children), so every later segment lies within one rank's range.
  const bool shard = W.shard_n > 1 && r >= (int)W.shard_r0;
  __shared__ uint32_t sbound[IS_SHARD_MAX + 1];
  if (shard && r == (int)W.shard_r0) {
    const uint32_t N = W.shard_n;
    for (uint32_t jb = threadIdx.x; jb <= N; jb += blockDim.x) sbound[jb] = jb == 0 ? 0u : nsort;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nch; i += blockDim.x) {
      const uint32_t fi = W.segs[(size_t)(r - 1) * W.segmax + i / 2].f;  // left child: the parent's start
      const uint32_t f = (i & 1) ? min(max(coherent_load(&W.cuts[(size_t)(r - 1) * W.segmax + i / 2]),
                                           fi + 1), W.segs[(size_t)(r - 1) * W.segmax + i / 2].l - 1)
                                 : fi;
      for (uint32_t jb = 1; jb < N; ++jb)
        if ((uint64_t)f * N >= (uint64_t)jb * nsort) atomicMin(&sbound[jb], f);
    }
    __syncthreads();
    for (uint32_t jb = threadIdx.x; jb <= N; jb += blockDim.x) W.bounds[jb] = sbound[jb];
    __syncthreads();
  } else if (shard) {
    for (uint32_t jb = threadIdx.x; jb <= W.shard_n; jb += blockDim.x) sbound[jb] = W.bounds[jb];
    __syncthreads();
  }
  const uint32_t lo = shard ? sbound[W.shard_rank] : 0u, hi = shard ? sbound[W.shard_rank + 1] : 0xFFFFFFFFu;
  for (uint32_t b0 = 0; b0 < nch; b0 += blockDim.x * PL) {
    const uint32_t i0 = b0 + threadIdx.x * PL;  // this thread's PL consecutive children (PL/2 parents)
    uint32_t cut[PL / 2];
    IsSeg sg[PL / 2];
#pragma unroll
    for (int k = 0; k < PL / 2; ++k) {
      const uint32_t i = i0 + 2 * k;
      cut[k] = 0u;
      sg[k] = IsSeg{};
      if (r > 0 && i < nch) {
        sg[k] = W.segs[(size_t)(r - 1) * W.segmax + i / 2];
        cut[k] = coherent_load(&W.cuts[(size_t)(r - 1) * W.segmax + i / 2]);
      }
    }
    Child ch[PL];
    uint64_t tot_t = 0;
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      const uint32_t i = i0 + k;
      Child c = {0u, 0u, 0};
      if (i < nch) {
        if (r == 0) {
          c = Child{0u, nsort, depth0(nsort)};
        } else {
          const IsSeg& q = sg[k / 2];
          const uint32_t cc = min(max(cut[k / 2], q.f + 1), q.l - 1);
          c = (k & 1) ? Child{cc, q.l, q.depth - 1} : Child{q.f, cc, q.depth - 1};
        }
      }
      if (c.f < lo || c.f >= hi) c = Child{0u, 0u, 0};  // another rank's (row D)
      ch[k] = c;
      const bool lg = i < nch && is_large(c, W.tier), ow = i < nch && !lg && c.l > c.f;
      // packed counters: large (21 bits) | owned (21) | tiles (22)
      tot_t += (lg ? 1ull : 0ull) | ((ow ? 1ull : 0ull) << 21) | ((uint64_t)(lg ? tiles_of_l(c.l - c.f) : 0u) << 42);
    }
    uint64_t s_all;
    uint64_t run = block_excl_scan64(tot_t, sh64, &s_all);
#pragma unroll
    for (int k = 0; k < PL; ++k) {
      const uint32_t i = i0 + k;
      const Child c = ch[k];
      const bool lg = i < nch && is_large(c, W.tier), ow = i < nch && !lg && c.l > c.f;
      const uint32_t p_lg = (uint32_t)(run & 0x1FFFFFu), p_ow = (uint32_t)((run >> 21) & 0x1FFFFFu),
                     p_nt = (uint32_t)(run >> 42);
      if (lg) W.ptab[nseg + p_lg] = make_uint4(c.f, c.l, (uint32_t)c.d, ntiles + p_nt);
      if (ow) W.own[own_base + nown + p_ow] = IsOwn{c.f, c.l, c.d, (uint32_t)(r & 1)};
      run += (lg ? 1ull : 0ull) | ((ow ? 1ull : 0ull) << 21) | ((uint64_t)(lg ? tiles_of_l(c.l - c.f) : 0u) << 42);
    }
    nseg += (uint32_t)(s_all & 0x1FFFFFu);
    nown += (uint32_t)((s_all >> 21) & 0x1FFFFFu);
    ntiles += (uint32_t)(s_all >> 42);
  }
  // (pad: elements partitioned this round, the scatter probe's unit count, summed by
  // the scatter's first tiles)
  if (threadIdx.x == 0) W.rounds[r] = IsRound{nseg, ntiles, own_base + nown, 0u};
}

// Tile t of segment j: pivot (its first tile publishes the segment record and the
// initial cut), counts and its segment (atomics: read by this launch's last
// workgroup), lists.
__device__ __forceinline__ void count_tile(const uint32_t* __restrict__ K, const uint32_t* __restrict__ V,
                                           const IsBufs& W, int r, uint32_t t, uint32_t j) {
  __shared__ uint32_t cg[IS_TC_L * 4], cl[IS_TC_L * 4], pg[IS_TC_L * 4], pl[IS_TC_L * 4];
  __shared__ uint32_t bsh[4];
  const uint4 pt = W.ptab[j];
  const uint32_t f = pt.x, l = pt.y, tile0 = pt.w;
  const uint32_t i = t - tile0;
  const uint32_t a = f + 1 + i * IS_TILE_L, b = min(l, a + IS_TILE_L);
  uint32_t kk[IS_TC_L];
  // the tile's keys are loaded before the pivot, so their latency overlaps thread 0's
  // dependent median reads below
#pragma unroll
  for (int c = 0; c < IS_TC_L; ++c) {
    const uint32_t p = a + c * IS_TT + threadIdx.x;
    kk[c] = p < b ? K[p] : 0u;
  }
  if (threadIdx.x == 0) {
    uint32_t m, Pm, vm, kf0, vf0;
    median_load(K, V, f, l, m, Pm, vm, kf0, vf0);
    bsh[0] = m;
    bsh[1] = Pm;
    bsh[2] = kf0;
    const IsSeg rec{f, l, (int32_t)pt.z, tile0, m, Pm, kf0, vf0, vm};
    W.tdesc[t] = IsTile{j, rec};  // the scatter's one-load view of this tile's segment
    atomicExch(&W.tseg[t], j);
    if (t == tile0) {  // the segment's record, once
      W.segs[(size_t)r * W.segmax + j] = rec;
      W.cuts[(size_t)r * W.segmax + j] = l;
    }
  }
  __syncthreads();
  const uint32_t m = bsh[0], P = bsh[1], kf = bsh[2];
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < IS_TC_L; ++c)
    if (a + c * IS_TT + threadIdx.x == m) kk[c] = kf;  // the median-to-first swap
#pragma unroll
  for (int c = 0; c < IS_TC_L; ++c) {
    const bool ok = a + c * IS_TT + threadIdx.x < b;
    const uint64_t bg = __ballot(ok && kk[c] >= P), bl = __ballot(ok && kk[c] <= P);
    if (lane == 0) {
      cg[c * 4 + w] = (uint32_t)__popcll(bg);
      cl[c * 4 + w] = (uint32_t)__popcll(bl);
    }
  }
  __syncthreads();
  if (w == 0) {  // IS_TC_L * 4 (chunk, wave) entries in position order
    const uint32_t xg0 = lane < IS_TC_L * 4 ? cg[lane] : 0u, xl0 = lane < IS_TC_L * 4 ? cl[lane] : 0u;
    uint32_t xg = xg0, xl = xl0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t yg = __shfl_up(xg, o, 64), yl = __shfl_up(xl, o, 64);
      if (lane >= (uint32_t)o) { xg += yg; xl += yl; }
    }
    if (lane < IS_TC_L * 4) {
      pg[lane] = xg - xg0;
      pl[lane] = xl - xl0;
    }
    if (lane == IS_TC_L * 4 - 1) {
      atomicExch(&W.cnt[2 * (size_t)t], xg);
      atomicExch(&W.cnt[2 * (size_t)t + 1], xl);
    }
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < IS_TC_L; ++c) {
    const uint32_t p = a + c * IS_TT + threadIdx.x;
    const bool ok = p < b;
    const bool ge = ok && kk[c] >= P, le = ok && kk[c] <= P;
    const uint64_t bg = __ballot(ge), bl = __ballot(le);
    if (ge) W.gel[a + pg[c * 4 + w] + mbcnt(bg)] = (uint16_t)(p - a);
    if (le) W.lel[a + pl[c * 4 + w] + mbcnt(bl)] = (uint16_t)(p - a);
  }
}

// The round's tile prefixes, by its last count workgroup: per tile the exclusive
// (>=, <=) prefix within its segment (pre), per segment the <= total (letot).  TP
// consecutive tiles per thread per step (their atomic loads in flight together).  A
// tile's two counts (<= IS_TILE_L each) travel packed in one u32 and are re-summed in
// the second pass instead of kept per tile.  The last workgroup's registers set the
// whole kernel's occupancy: 16 tiles per thread took 150 VGPRs (3 waves per SIMD), 4
// take 65 (7 waves per SIMD; c5: 68 -> 38.5 us per count launch, 8.53 -> 7.97 ms per
// registration, profiles/r03i).
// base: LDS scratch of 2 x segmax u32 (the running prefix at each segment's first tile).
#ifndef IS_TP_VAL
#define IS_TP_VAL 4
#endif
constexpr int TP = IS_TP_VAL;
static_assert(IS_TILE_L < 65536, "tile counts packed in 16 bits");
__device__ __forceinline__ uint64_t coherent_load64(uint32_t* p) {
  return atomicAdd(reinterpret_cast<unsigned long long*>(p), 0ull);
}
__device__ __forceinline__ uint64_t unpack_gq(uint32_t gq) { return (uint64_t)(gq & 0xFFFFu) | ((uint64_t)(gq >> 16) << 32); }
__device__ void tile_prefix(const IsBufs& W, int r, uint32_t* base, uint64_t* sh64) {
  const uint32_t ntiles = W.rounds[r].ntiles;
  uint32_t* bg = base;
  uint32_t* bl = base + W.segmax;
  uint64_t run = 0;
  for (uint32_t b0 = 0; b0 < ntiles; b0 += blockDim.x * TP) {
    const uint32_t t0 = b0 + threadIdx.x * TP;
    uint32_t gq[TP], js[TP];
#pragma unroll
    for (int k = 0; k < TP; ++k) {
      const uint32_t t = t0 + k;
      gq[k] = js[k] = 0u;
      if (t < ntiles) {
        const uint64_t c = coherent_load64(&W.cnt[2 * (size_t)t]);  // (>=, <=) of tile t
        gq[k] = (uint32_t)c | ((uint32_t)(c >> 32) << 16);
        js[k] = coherent_load(&W.tseg[t]);
      }
    }
    uint64_t sum = 0;
#pragma unroll
    for (int k = 0; k < TP; ++k) sum += unpack_gq(gq[k]);
    uint64_t tot;  // >= counts (low 32 bits) and <= counts (high): each sums to <= the sort length
    const uint64_t x0 = run + block_excl_scan64(sum, sh64, &tot);
    uint64_t x = x0;
#pragma unroll
    for (int k = 0; k < TP; ++k) {
      const uint32_t t = t0 + k;
      if (t < ntiles && t == W.ptab[js[k]].w) {
        bg[js[k]] = (uint32_t)x;
        bl[js[k]] = (uint32_t)(x >> 32);
      }
      x += unpack_gq(gq[k]);
    }
    __syncthreads();
    x = x0;
#pragma unroll
    for (int k = 0; k < TP; ++k) {
      const uint32_t t = t0 + k;
      if (t >= ntiles) continue;
      const uint32_t j = js[k];
      W.pre[2 * (size_t)t] = (uint32_t)x - bg[j];
      W.pre[2 * (size_t)t + 1] = (uint32_t)(x >> 32) - bl[j];
      x += unpack_gq(gq[k]);
      const uint4 pt = W.ptab[j];
      if (t == pt.w + tiles_of_l(pt.y - pt.x) - 1u) W.letot[j] = (uint32_t)(x >> 32) - bl[j];
    }
    run += tot;
    __syncthreads();
  }
}

// Dynamic LDS: 2 * segmax u32 (tile_prefix).
__global__ void __launch_bounds__(IS_TT) k_is_count_plan(B4<const uint32_t*> K2, B4<const uint32_t*> V2,
                                                         B4<IsBufs> W2, int r) {
  KT();
  extern __shared__ uint32_t dyn[];
  __shared__ uint64_t sh64[16];
  __shared__ uint32_t sflag, sj;
  const int e = blockIdx.y;
  const IsBufs W = W2[e];
  const uint32_t t = blockIdx.x;
  const IsRound rd = W.rounds[r];
  if (t < rd.ntiles) {
    if (threadIdx.x < 64) {  // the tile's segment: the last with first tile <= t
      const uint32_t j = wave_upper_index([&](uint32_t u) { return W.ptab[u].w; }, rd.nseg, t);
      if (threadIdx.x == 0) sj = j;
    }
    __syncthreads();
    count_tile(K2[e], V2[e], W, r, t, sj);
  }
  if (!last_block(W.done + (size_t)(2 * r) * IS_DONE_WORDS, &sflag)) return;
  tile_prefix(W, r, dyn, sh64);
}

// The partitioned tile written out: every element to its destination, so a swapped
// element is a scattered 4-byte store into another tile's lines (two of them: key and
// value), which other workgroups fill too.  (A gather form -- every position reading
// its partner, whole tiles written coalesced -- measured no faster: pipelined
// 0.770/0.768/0.808 against 0.787/0.794/0.770 ms, profiles/r05a/ab_gather.txt.)
template <int TC>
__device__ __forceinline__ void store_partitioned(uint32_t* __restrict__ Ko, uint32_t* __restrict__ Vo,
                                                  const uint32_t (&kk)[TC], const uint32_t (&vv)[TC],
                                                  const uint32_t (&dst)[TC], uint32_t f, uint32_t l, const IsBufs& W) {
#pragma unroll
  for (int c = 0; c < TC; ++c) {
    const uint32_t d = dst[c];
    if (d == IS_NONE) continue;
    if (d <= f || d >= l) {  // cannot happen; never write outside the segment
      is_fault(W.ctl, W.err, IS_FAULT_SCATTER);
      continue;
    }
    Ko[d] = kk[c];
    Vo[d] = vv[c];
  }
}

// Every element of the round's large segments to its place after the partition,
// written to the other buffer; the cut by atomicMin; the last workgroup plans round
// r + 1 (if r + 1 < R).  The partners of a tile's swapped elements have contiguous
// ranks in the other list, so each workgroup locates that window of its segment's
// tile prefix once (wave_upper_index over global memory) and keeps it in LDS.
constexpr uint32_t IS_WIN = 256;  // prefix window in LDS (larger windows: binary search in global memory)

#ifndef IS_SCATTER_MINB
#define IS_SCATTER_MINB 1
#endif
__global__ void __launch_bounds__(IS_TT, IS_SCATTER_MINB) k_is_scatter(B4<const uint32_t*> Ki2, B4<const uint32_t*> Vi2,
                                                      B4<uint32_t*> Ko2, B4<uint32_t*> Vo2, B4<IsBufs> W2, int r,
                                                      int R) {
  KT();
  __shared__ uint64_t sh64[16];
  __shared__ uint32_t cg[IS_TC_L * 4], cl[IS_TC_L * 4], pg[IS_TC_L * 4], pl[IS_TC_L * 4];
  __shared__ uint32_t wing[IS_WIN], winl[IS_WIN];  // windows of the >= / <= prefixes
  __shared__ uint32_t stot[2], swin[4];            // the tile's totals; window bounds
  __shared__ uint32_t scut, sflag;
  const int e = blockIdx.y;
  const IsBufs W = W2[e];
  const uint32_t t = blockIdx.x;
  if (r == 0 && t == 0 && e == 0 && threadIdx.x == 0) is_inject(W, IS_FAULT_SCATTER);
  if (t < W.rounds[r].ntiles) {
    const IsTile td = W.tdesc[t];
    const uint32_t j = td.j;
    const IsSeg s = td.s;
    const uint32_t f = s.f, l = s.l, nt = tiles_of_l(l - f), i = t - s.tile0, m = s.m, P = s.P;
    const uint32_t* __restrict__ K = Ki2[e];
    const uint32_t* __restrict__ V = Vi2[e];
    uint32_t* __restrict__ Ko = Ko2[e];
    uint32_t* __restrict__ Vo = Vo2[e];
    const uint2* pre = reinterpret_cast<const uint2*>(W.pre) + s.tile0;  // the segment's tile prefixes
    const uint32_t a = f + 1 + i * IS_TILE_L, b = min(l, a + IS_TILE_L);
    const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
    if (i == 0 && threadIdx.x == 0) atomicAdd(&W.rounds[r].pad, l - f);
    // the tile's elements are loaded first: their latency overlaps the window searches
    uint32_t kk[IS_TC_L], vv[IS_TC_L];
#pragma unroll
    for (int c = 0; c < IS_TC_L; ++c) {
      const uint32_t p = a + c * IS_TT + threadIdx.x;
      const bool ok = p < b;
      kk[c] = ok ? K[p] : 0u;
      vv[c] = ok ? V[p] : 0u;
      if (p == m) {
        kk[c] = s.kf;
        vv[c] = s.vf;
      }
    }
    if (threadIdx.x == 0) scut = IS_NONE;
    const uint2 own = pre[i];
    const uint32_t le_tot = W.letot[j];
#pragma unroll
    for (int c = 0; c < IS_TC_L; ++c) {
      const bool ok = a + c * IS_TT + threadIdx.x < b;
      const uint64_t bg = __ballot(ok && kk[c] >= P), bl = __ballot(ok && kk[c] <= P);
      if (lane == 0) {
        cg[c * 4 + w] = (uint32_t)__popcll(bg);
        cl[c * 4 + w] = (uint32_t)__popcll(bl);
      }
    }
    __syncthreads();
    if (w == 0) {
      const uint32_t xg0 = lane < IS_TC_L * 4 ? cg[lane] : 0u, xl0 = lane < IS_TC_L * 4 ? cl[lane] : 0u;
      uint32_t xg = xg0, xl = xl0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t yg = __shfl_up(xg, o, 64), yl = __shfl_up(xl, o, 64);
        if (lane >= (uint32_t)o) { xg += yg; xl += yl; }
      }
      if (lane < IS_TC_L * 4) {
        pg[lane] = xg - xg0 + own.x;
        pl[lane] = xl - xl0 + own.y;
      }
      if (lane == IS_TC_L * 4 - 1) {
        stot[0] = xg;
        stot[1] = xl;
      }
    }
    __syncthreads();
    // Partner windows.  A swapped >= element of rank gx in [own.x, own.x + cg) takes
    // R[gx + 1], the <= element of rank le_tot - gx - 1; a swapped <= element of rank
    // lx in [own.y, own.y + cl) takes L[le_tot - lx], the >= element of rank
    // le_tot - lx - 1.  Each rank range spans a window of tiles of the other list.
    const uint32_t cgt = stot[0], clt = stot[1];
    const bool lw_any = cgt > 0 && le_tot > own.x;  // the <= window (partners of swapped >=)
    const uint32_t xl_hi = lw_any ? le_tot - own.x - 1 : 0u;
    const uint32_t xl_lo = lw_any ? (le_tot >= own.x + cgt ? le_tot - own.x - cgt : 0u) : 0u;
    const bool gw_any = clt > 0 && le_tot > own.y;  // the >= window (partners of swapped <=)
    const uint32_t xg_hi = gw_any ? le_tot - own.y - 1 : 0u;
    const uint32_t xg_lo = gw_any ? (le_tot >= own.y + clt ? le_tot - own.y - clt : 0u) : 0u;
    if (w < 4) {
      uint32_t u = 0;
      if (w == 0 && lw_any) u = wave_upper_index([&](uint32_t k) { return pre[k].y; }, nt, xl_lo);
      if (w == 1 && lw_any) u = wave_upper_index([&](uint32_t k) { return pre[k].y; }, nt, xl_hi);
      if (w == 2 && gw_any) u = wave_upper_index([&](uint32_t k) { return pre[k].x; }, nt, xg_lo);
      if (w == 3 && gw_any) u = wave_upper_index([&](uint32_t k) { return pre[k].x; }, nt, xg_hi);
      if (lane == 0) swin[w] = u;
    }
    __syncthreads();
    const uint32_t wl_lo = swin[0], wl_n = lw_any ? swin[1] - swin[0] + 1 : 0u;
    const uint32_t wg_lo = swin[2], wg_n = gw_any ? swin[3] - swin[2] + 1 : 0u;
    for (uint32_t k = threadIdx.x; k < IS_WIN; k += IS_TT) {
      if (k < wl_n) winl[k] = pre[wl_lo + k].y;
      if (k < wg_n) wing[k] = pre[wg_lo + k].x;
    }
    __syncthreads();
    // destinations: the swapped elements' partner positions come from the lists (all
    // list loads issued before any store)
    uint32_t cut = IS_NONE;
    uint32_t dst[IS_TC_L];
#pragma unroll
    for (int c = 0; c < IS_TC_L; ++c) {
      const uint32_t p = a + c * IS_TT + threadIdx.x;
      const bool ok = p < b;
      const bool ge = ok && kk[c] >= P, le = ok && kk[c] <= P;
      const uint64_t bg = __ballot(ge), bl = __ballot(le);
      const uint32_t gx = pg[c * 4 + w] + mbcnt(bg);  // # >= P before p in the segment
      const uint32_t lx = pl[c * 4 + w] + mbcnt(bl);  // # <= P before p
      const bool sg = ge && le_tot - lx - (le ? 1u : 0u) >= gx + 1;
      const bool sl = le && gx >= le_tot - lx;
      if ((ge && !sg) || sl) cut = min(cut, p);  // L[K+1] / R[K]
      dst[c] = ok ? p : IS_NONE;
      if (sg) {  // R[gx+1]: the (le_tot-gx-1)-th <= P from the left
        const uint32_t x = le_tot - gx - 1;
        const uint32_t u = wl_n <= IS_WIN ? wl_lo + upper_index(winl, wl_n, x) : upper_index_g(pre, nt, x, 1);
        const uint32_t au = f + 1 + u * IS_TILE_L;
        dst[c] = au + W.lel[au + (x - (wl_n <= IS_WIN ? winl[u - wl_lo] : pre[u].y))];
      } else if (sl) {  // L[kr]: the (kr-1)-th >= P from the left
        const uint32_t x = le_tot - lx - 1;
        const uint32_t u = wg_n <= IS_WIN ? wg_lo + upper_index(wing, wg_n, x) : upper_index_g(pre, nt, x, 0);
        const uint32_t au = f + 1 + u * IS_TILE_L;
        dst[c] = au + W.gel[au + (x - (wg_n <= IS_WIN ? wing[u - wg_lo] : pre[u].x))];
      }
    }
    store_partitioned<IS_TC_L>(Ko, Vo, kk, vv, dst, f, l, W);
    cut = wave_min_u32(cut);
    if (lane == 0 && cut != IS_NONE) atomicMin(&scut, cut);
    __syncthreads();
    if (threadIdx.x == 0) {
      if (scut != IS_NONE) atomicMin(&W.cuts[(size_t)r * W.segmax + j], scut);
      if (i == 0) {
        Ko[f] = P;
        Vo[f] = s.vm;
      }
    }
  }
  if (r + 1 >= R) return;  // (uniform: no planner after the last round)
  if (!last_block(W.done + (size_t)(2 * r + 1) * IS_DONE_WORDS, &sflag)) return;
  plan_round(W, r + 1, W.ctl[0], sh64);
}

// ---------------------------------------------------------------- rounds, small clouds
// Below IS_LARGE_MIN points the round plan is derived by every workgroup itself (the
// segment table from the previous round's segments and cuts, a few hundred entries)
// and every scatter workgroup scans its segment's tile counts itself: at ~700
// workgroups per launch that costs less than the large form's per-round serial steps
// (last-workgroup hand-offs; c3: 0.76 vs 0.96 ms main VoxelGrid).
//
// k_is_count_plan_s: the round's plan, then per-tile ge/le counts against the segment's
// pivot and the tile-local position lists (offsets from the tile start, in position
// order).  The workgroup of a segment's first tile publishes its IsSeg and initial
// cut, every workgroup its tile's descriptor (IsTile), workgroup 0 the owned list of
// small children and the IsRound; the scatter reads them after the kernel boundary.
__device__ __forceinline__ void is_count_body_s(const uint32_t* __restrict__ K, const uint32_t* __restrict__ V,
                                              const IsBufs& W, int r, uint32_t* dyn) {
  __shared__ uint32_t cg[IS_TC * 4], cl[IS_TC * 4], pg[IS_TC * 4], pl[IS_TC * 4];
  __shared__ uint32_t bsh[4];
  __shared__ uint64_t sh64[16];
  // Tiles blockIdx.x, + gridDim.x, ... of the round (the grid is capped, is_round_grid):
  // the plan is derived once per workgroup, not once per tile.
  if (r > 0) {
    // Round r's large segments are children of round r-1's (which partitioned `pad`
    // elements in nseg segments), so it has at most pad / IS_TILE + 2 nseg tiles: a
    // workgroup whose first tile lies past that bound leaves at once (the late rounds
    // hold a few segments; their launches were all plan derivation).
    const IsRound pr = W.rounds[r - 1];
    if (blockIdx.x >= pr.pad / IS_TILE + 2u * pr.nseg + 1u) return;
  }
  const uint32_t nsort = W.ctl[0];
  uint32_t* tf = dyn;
  uint32_t* tl = tf + W.segmax;
  int32_t* td = (int32_t*)(tl + W.segmax);
  uint32_t* t0 = (uint32_t*)(td + W.segmax);
  const uint32_t nch = nchildren(W, r);
  const uint32_t own_base = r ? W.rounds[r - 1].nown : 0u;
  uint32_t nseg = 0, ntiles = 0, nown = 0;
  for (uint32_t b = 0; b < nch; b += blockDim.x) {
    const uint32_t i = b + threadIdx.x;
    Child c = {0u, 0u, 0};
    if (i < nch) c = child_of(W, r, nsort, i);
    const bool lg = i < nch && is_large(c, W.tier);
    const bool ow = i < nch && !lg && c.l > c.f;
    const uint32_t nt = lg ? tiles_of(c.l - c.f) : 0u;
    // one scan of the three counters packed: large (21 bits) | owned (21) | tiles (22)
    uint64_t s_all;
    const uint64_t p_all =
        block_excl_scan64((lg ? 1ull : 0ull) | ((ow ? 1ull : 0ull) << 21) | ((uint64_t)nt << 42), sh64, &s_all);
    const uint32_t p_lg = (uint32_t)(p_all & 0x1FFFFFu), p_ow = (uint32_t)((p_all >> 21) & 0x1FFFFFu),
                   p_nt = (uint32_t)(p_all >> 42);
    const uint32_t s_lg = (uint32_t)(s_all & 0x1FFFFFu), s_ow = (uint32_t)((s_all >> 21) & 0x1FFFFFu),
                   s_nt = (uint32_t)(s_all >> 42);
    if (lg) {
      tf[nseg + p_lg] = c.f;
      tl[nseg + p_lg] = c.l;
      td[nseg + p_lg] = c.d;
      t0[nseg + p_lg] = ntiles + p_nt;
    }
    if (ow && blockIdx.x == 0) W.own[own_base + nown + p_ow] = IsOwn{c.f, c.l, c.d, (uint32_t)(r & 1)};
    nseg += s_lg;
    ntiles += s_nt;
    nown += s_ow;
  }
  __syncthreads();
  IS_PH(5);  // count: the round's plan
  // (pad: elements partitioned this round, the scatter probe's unit count, summed by
  // the scatter's first tiles)
  if (blockIdx.x == 0 && threadIdx.x == 0) W.rounds[r] = IsRound{nseg, ntiles, own_base + nown, 0u};
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  for (uint32_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const uint32_t j = upper_index(t0, nseg, t);
    const uint32_t f = tf[j], l = tl[j], tile0 = t0[j];
    const uint32_t a = f + 1 + (t - tile0) * IS_TILE, b = min(l, a + IS_TILE);
    // the tile's keys are loaded before the pivot, so their latency overlaps thread 0's
    // dependent median reads below
    uint32_t kk[IS_TC];
#pragma unroll
    for (int c = 0; c < IS_TC; ++c) {
      const uint32_t p = a + c * IS_TT + threadIdx.x;
      kk[c] = p < b ? K[p] : 0u;
    }
    if (threadIdx.x == 0) {
      uint32_t m0, Pm, vm, kf0, vf0;
      median_load(K, V, f, l, m0, Pm, vm, kf0, vf0);
      bsh[0] = m0;
      bsh[1] = Pm;
      bsh[2] = kf0;
      const IsSeg rec{f, l, td[j], tile0, m0, Pm, kf0, vf0, vm};
      W.tseg[t] = j;
      W.tdesc[t] = IsTile{j, rec};  // the scatter's one-load view of this tile's segment
      if (t == tile0) {  // the segment's record, once
        W.segs[(size_t)r * W.segmax + j] = rec;
        W.cuts[(size_t)r * W.segmax + j] = l;
      }
    }
    __syncthreads();
    IS_PH(6);  // count: tile keys, median, descriptor
    const uint32_t m = bsh[0], P = bsh[1], kf = bsh[2];
#pragma unroll
    for (int c = 0; c < IS_TC; ++c)
      if (a + c * IS_TT + threadIdx.x == m) kk[c] = kf;  // the median-to-first swap
#pragma unroll
    for (int c = 0; c < IS_TC; ++c) {
      const bool ok = a + c * IS_TT + threadIdx.x < b;
      const uint64_t bg = __ballot(ok && kk[c] >= P), bl = __ballot(ok && kk[c] <= P);
      if (lane == 0) {
        cg[c * 4 + w] = (uint32_t)__popcll(bg);
        cl[c * 4 + w] = (uint32_t)__popcll(bl);
      }
    }
    __syncthreads();
    IS_PH(7);  // count: ballots
    if (w == 0) {  // IS_TC * 4 (chunk, wave) entries in position order
      const uint32_t xg0 = lane < IS_TC * 4 ? cg[lane] : 0u, xl0 = lane < IS_TC * 4 ? cl[lane] : 0u;
      uint32_t xg = xg0, xl = xl0;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t yg = __shfl_up(xg, o, 64), yl = __shfl_up(xl, o, 64);
        if (lane >= (uint32_t)o) { xg += yg; xl += yl; }
      }
      if (lane < IS_TC * 4) {
        pg[lane] = xg - xg0;
        pl[lane] = xl - xl0;
      }
      if (lane == IS_TC * 4 - 1) {
        W.cnt[2 * (size_t)t] = xg;
        W.cnt[2 * (size_t)t + 1] = xl;
      }
    }
    __syncthreads();
    IS_PH(8);  // count: chunk scan
#pragma unroll
    for (int c = 0; c < IS_TC; ++c) {
      const uint32_t p = a + c * IS_TT + threadIdx.x;
      const bool ok = p < b;
      const bool ge = ok && kk[c] >= P, le = ok && kk[c] <= P;
      const uint64_t bg = __ballot(ge), bl = __ballot(le);
      if (ge) W.gel[a + pg[c * 4 + w] + mbcnt(bg)] = (uint16_t)(p - a);
      if (le) W.lel[a + pl[c * 4 + w] + mbcnt(bl)] = (uint16_t)(p - a);
    }
    IS_PH(9);  // count: lists written
    __syncthreads();  // (this tile's LDS reads before the next tile's writes)
  }
}

// Dynamic LDS: 4 * segmax u32 (the round's segment table).
__global__ void __launch_bounds__(IS_TT) k_is_count_plan_s(B4<const uint32_t*> K2, B4<const uint32_t*> V2,
                                                         B4<IsBufs> W2, int r) {
  KT();
  IS_PH_START();
  extern __shared__ uint32_t dyn[];
  const int e = blockIdx.y;
  is_count_body_s(K2[e], V2[e], W2[e], r, dyn);
}

// Every element of the round's large segments to its place after the partition,
// written to the other buffer; the cut by atomicMin.  Dynamic LDS: 2 * maxtiles u32.
// seven waves per SIMD: 67 VGPRs and no scratch instead of 79 (six waves); 44.7 ->
// 43.0 us per ten-cloud launch (eight: 64 VGPRs with spills, 49.7 us; profiles/r06l)
#ifndef IS_SCATTER_S_WPE
#define IS_SCATTER_S_WPE 7
#endif
__global__ void __launch_bounds__(IS_TT) __attribute__((amdgpu_waves_per_eu(IS_SCATTER_S_WPE)))
k_is_scatter_s(B4<const uint32_t*> Ki2, B4<const uint32_t*> Vi2,
                                                      B4<uint32_t*> Ko2, B4<uint32_t*> Vo2, B4<IsBufs> W2, int r) {
  KT();
  IS_PH_START();
  extern __shared__ uint32_t dyn[];
  __shared__ uint64_t sh64[16];
  __shared__ uint32_t cg[IS_TC * 4], cl[IS_TC * 4], pg[IS_TC * 4], pl[IS_TC * 4];
  __shared__ uint32_t scut, swin[4];
  const int e = blockIdx.y;
  const IsBufs W = W2[e];
  const uint32_t t = blockIdx.x;
  // (the count kernel wrote the round's tile count; descriptors past it are stale, both
  // loads in flight together)
  const uint32_t ntl = W.rounds[r].ntiles;
  const IsTile td = W.tdesc[t];
  if (t >= ntl) return;
  const uint32_t j = td.j;
  const IsSeg s = td.s;
  const uint32_t f = s.f, l = s.l, nt = tiles_of(l - f), i = t - s.tile0, m = s.m, P = s.P;
  uint32_t* preg = dyn;
  uint32_t* prel = preg + W.maxtiles;
  const uint32_t* __restrict__ K = Ki2[e];
  const uint32_t* __restrict__ V = Vi2[e];
  uint32_t* __restrict__ Ko = Ko2[e];
  uint32_t* __restrict__ Vo = Vo2[e];
  const uint32_t a = f + 1 + i * IS_TILE, b = min(l, a + IS_TILE);
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  if (i == 0 && threadIdx.x == 0) atomicAdd(&W.rounds[r].pad, l - f);
  if (r == 0 && t == 0 && e == 0 && threadIdx.x == 0) is_inject(W, IS_FAULT_SCATTER);
  // the tile's elements are loaded first: their latency overlaps the prefix below
  uint32_t kk[IS_TC], vv[IS_TC];
#pragma unroll
  for (int c = 0; c < IS_TC; ++c) {
    const uint32_t p = a + c * IS_TT + threadIdx.x;
    const bool ok = p < b;
    kk[c] = ok ? K[p] : 0u;
    vv[c] = ok ? V[p] : 0u;
    if (p == m) {
      kk[c] = s.kf;
      vv[c] = s.vf;
    }
  }
  if (threadIdx.x == 0) scut = IS_NONE;
  // exclusive prefix of the segment's tile counts
  uint32_t rg = 0, rl = 0;
  for (uint32_t u0 = 0; u0 < nt; u0 += blockDim.x) {
    const uint32_t u = u0 + threadIdx.x;
    const uint32_t g = u < nt ? W.cnt[2 * (size_t)(s.tile0 + u)] : 0u;
    const uint32_t q = u < nt ? W.cnt[2 * (size_t)(s.tile0 + u) + 1] : 0u;
    uint64_t sx;  // >= counts (low 32 bits) and <= counts (high) in one scan: each sums to <= l - f
    const uint64_t xx = block_excl_scan64((uint64_t)g | ((uint64_t)q << 32), sh64, &sx);
    const uint32_t xg = (uint32_t)xx, xl = (uint32_t)(xx >> 32), sg = (uint32_t)sx, sl = (uint32_t)(sx >> 32);
    if (u < nt) {
      preg[u] = rg + xg;
      prel[u] = rl + xl;
    }
    rg += sg;
    rl += sl;
  }
  const uint32_t le_tot = rl;
  IS_PH(0);  // descriptor, tile loads issued, the segment's tile prefix
#pragma unroll
  for (int c = 0; c < IS_TC; ++c) {
    const bool ok = a + c * IS_TT + threadIdx.x < b;
    const uint64_t bg = __ballot(ok && kk[c] >= P), bl = __ballot(ok && kk[c] <= P);
    if (lane == 0) {
      cg[c * 4 + w] = (uint32_t)__popcll(bg);
      cl[c * 4 + w] = (uint32_t)__popcll(bl);
    }
  }
  __syncthreads();
  IS_PH(1);  // ballots, counts
  if (w == 0) {
    const uint32_t xg0 = lane < IS_TC * 4 ? cg[lane] : 0u, xl0 = lane < IS_TC * 4 ? cl[lane] : 0u;
    uint32_t xg = xg0, xl = xl0;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t yg = __shfl_up(xg, o, 64), yl = __shfl_up(xl, o, 64);
      if (lane >= (uint32_t)o) { xg += yg; xl += yl; }
    }
    if (lane < IS_TC * 4) {
      pg[lane] = xg - xg0 + preg[i];
      pl[lane] = xl - xl0 + prel[i];
    }
    // Partner windows (as in k_is_scatter): a swapped >= element of rank gx takes the
    // (le_tot-gx-1)-th <= element, a swapped <= element of rank lx the (le_tot-lx-1)-th
    // >= element; this tile's ranks are contiguous, so their partners lie in a window of
    // tiles found once here (four binary searches, one per lane) instead of per element.
    const uint32_t cgt = (uint32_t)__shfl((int)xg, IS_TC * 4 - 1, 64), clt = (uint32_t)__shfl((int)xl, IS_TC * 4 - 1, 64);
    const uint32_t ox = preg[i], oy = prel[i];
    if (lane < 4) {
      uint32_t x = 0;
      if (lane == 0) x = le_tot > ox + cgt ? le_tot - ox - cgt : 0u;
      if (lane == 1) x = le_tot > ox ? le_tot - ox - 1 : 0u;
      if (lane == 2) x = le_tot > oy + clt ? le_tot - oy - clt : 0u;
      if (lane == 3) x = le_tot > oy ? le_tot - oy - 1 : 0u;
      swin[lane] = upper_index(lane < 2 ? prel : preg, nt, x);
    }
  }
  __syncthreads();
  IS_PH(2);  // chunk prefix, partner windows
  const uint32_t wl_lo = swin[0], wl_hi = swin[1], wg_lo = swin[2], wg_hi = swin[3];
  // largest u in [lo, hi] with pre[u] <= x (pre[lo] <= x and the answer <= hi by the
  // window): a few steps forward when the window is short, else a binary search in it
  auto in_window = [](const uint32_t* pre, uint32_t lo, uint32_t hi, uint32_t x) {
    if (hi - lo <= 4) {
      uint32_t u = lo;
      while (u < hi && pre[u + 1] <= x) ++u;
      return u;
    }
    uint32_t L = lo, H = hi + 1;
    while (H - L > 1) {
      const uint32_t mid = (L + H) >> 1;
      if (pre[mid] <= x) L = mid;
      else H = mid;
    }
    return L;
  };
  // destinations: the swapped elements' partner positions come from the lists (all
  // list loads issued before any store)
  uint32_t cut = IS_NONE;
  uint32_t dst[IS_TC];
#pragma unroll
  for (int c = 0; c < IS_TC; ++c) {
    const uint32_t p = a + c * IS_TT + threadIdx.x;
    const bool ok = p < b;
    const bool ge = ok && kk[c] >= P, le = ok && kk[c] <= P;
    const uint64_t bg = __ballot(ge), bl = __ballot(le);
    const uint32_t gx = pg[c * 4 + w] + mbcnt(bg);  // # >= P before p in the segment
    const uint32_t lx = pl[c * 4 + w] + mbcnt(bl);  // # <= P before p
    const bool sg = ge && le_tot - lx - (le ? 1u : 0u) >= gx + 1;
    const bool sl = le && gx >= le_tot - lx;
    if ((ge && !sg) || sl) cut = min(cut, p);  // L[K+1] / R[K]
    dst[c] = ok ? p : IS_NONE;
    if (sg) {  // R[gx+1]: the (le_tot-gx-1)-th <= P from the left
      const uint32_t x = le_tot - gx - 1;
      const uint32_t u = in_window(prel, wl_lo, wl_hi, x);
      const uint32_t au = f + 1 + u * IS_TILE;
      dst[c] = au + W.lel[au + (x - prel[u])];
    } else if (sl) {  // L[kr]: the (kr-1)-th >= P from the left
      const uint32_t x = le_tot - lx - 1;
      const uint32_t u = in_window(preg, wg_lo, wg_hi, x);
      const uint32_t au = f + 1 + u * IS_TILE;
      dst[c] = au + W.gel[au + (x - preg[u])];
    }
  }
  store_partitioned<IS_TC>(Ko, Vo, kk, vv, dst, f, l, W);
  IS_PH(3);  // destinations (list loads), stores issued
  cut = wave_min_u32(cut);
  if (lane == 0 && cut != IS_NONE) atomicMin(&scut, cut);
  __syncthreads();
  IS_PH(4);  // cut
  if (threadIdx.x == 0) {
    if (scut != IS_NONE) atomicMin(&W.cuts[(size_t)r * W.segmax + j], scut);
    if (i == 0) {
      Ko[f] = P;
      Vo[f] = s.vm;
    }
  }
}


// ---------------------------------------------------------------- finish: block + wave kernels
// After the rounds every segment is at most IS_LCAP long (leftovers beyond it are
// split by one workgroup in global memory first).  k_is_block: one 1024-thread
// workgroup per segment (dequeued), the segment in LDS, workgroup partitions while a
// subtree exceeds IS_WCAP; leaves (<= 16) and heap-sorted ranges are finished there,
// subtrees of <= IS_WCAP become tasks.  k_is_wave: every wave of the GPU takes tasks
// (dequeued), finishes each in its own LDS slice (wave partitions, register-resident
// subtrees of <= 64) and writes it.  Tasks keep the waves of the whole chip busy
// instead of the 16 waves of one workgroup.

// exchange slots of a workgroup partition: it swaps < IS_LCAP / 2 pairs
struct BlockLds {
  uint32_t k[IS_LCAP], v[IS_LCAP];
  uint16_t xch[IS_LCAP / 2];
  uint32_t heads[IS_LCAP / 32];     // leaf starts
  uint32_t intask[IS_LCAP / 32];    // positions handed to the wave kernel
  uint32_t cg[IS_OE], cl[IS_OE], pg[IS_OE], pl[IS_OE];
  uint2 wstk[IS_STACK / 2];         // workgroup-phase stack {off, len | depth << 16}
  uint4 gstk[IS_STACK / 2];         // global-phase stack {f, l, depth, -}
  uint32_t gsp;
  uint32_t bc[8];                   // broadcasts
  uint32_t sh[16];
  uint32_t* stat;                   // IsBufs::ctl
  uint32_t* err;                    // IsBufs::err
  uint32_t son;                     // path counters on (IS_STATS && IsBufs::stats)
  // wave tasks of the current segment, packed off | n << 13 | depth << 24, handed
  // to the global list with one atomic per class when the segment is done
  uint32_t tb[IS_LCAP / (IS_TASK_BIG + 1) + 1];  // > IS_TASK_BIG elements
  uint32_t ts[IS_LCAP / (IS_THRESHOLD + 1) + 1];  // the rest
  uint32_t ntb, nts, units;
};
static_assert(IS_LCAP <= 8192 && IS_WCAP <= 1024, "task packing: 13-bit offsets, 11-bit sizes, 8-bit depths");

// (wave tasks of > 64 elements are partitioned level by level, wave_task_level)

// One wave's slice of the wave kernel
struct WaveLds {
  uint32_t k[IS_WCAP + IS_THRESHOLD], v[IS_WCAP];  // (k: IS_NONE past the task, leaf_rank)
  uint16_t lg[IS_WCAP], ll[IS_WCAP];   // a level's >= / <= positions, in position order
  uint32_t cutv[IS_WCAP];              // per segment (at its first position): its cut, or its end
  uint64_t bw[2][IS_WC + 1];           // the level's >= / <= ballots per chunk
  uint32_t pc[2][IS_WC + 1];           // and their exclusive prefix counts
  union {
    uint16_t xch[IS_WCAP / 2];         // wave_partition's exchange
    uint32_t seg[IS_WCAP / 4];         // wave_task_level: a level's segments to partition, a | b << 16
  };
  uint32_t heads[IS_WCAP / 32];
  uint32_t stk[IS_STACK];
  uint32_t lstat[4];
  uint32_t* stat;
  uint32_t* err;
  uint32_t son;  // path counters on (IS_STATS && IsBufs::stats)
};

template <class SL>
__device__ __forceinline__ void mark_leaf(SL& S, uint32_t off) { atomicOr(&S.heads[off >> 5], 1u << (off & 31)); }

// Exclusive prefix (plus carries) of the IS_OE (chunk, wave) counts in position
// order, by wave 0 (IS_OE / 64 consecutive entries per lane).
__device__ __forceinline__ void block_chunk_scan(BlockLds& S, uint32_t cg0, uint32_t cl0) {
  constexpr uint32_t PER = (IS_OE + 63) / 64;
  const uint32_t lane = lane_id(), i0 = PER * lane;
  uint32_t sg = 0, sl = 0;
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q)
    if (i0 + q < IS_OE) {
      sg += S.cg[i0 + q];
      sl += S.cl[i0 + q];
    }
  uint32_t xg = sg, xl = sl;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t yg = __shfl_up(xg, o, 64), yl = __shfl_up(xl, o, 64);
    if (lane >= (uint32_t)o) { xg += yg; xl += yl; }
  }
  uint32_t rg = cg0 + xg - sg, rl = cl0 + xl - sl;
#pragma unroll
  for (uint32_t q = 0; q < PER; ++q)
    if (i0 + q < IS_OE) {
      S.pg[i0 + q] = rg;
      S.pl[i0 + q] = rl;
      rg += S.cg[i0 + q];
      rl += S.cl[i0 + q];
    }
}

// Position of the r-th (0-based) set bit of m (r < popcount(m)).
__device__ __forceinline__ uint32_t select64(uint64_t m, uint32_t r) {
  uint32_t pos = 0, c = (uint32_t)__popc((uint32_t)m);
  if (r >= c) {
    r -= c;
    m >>= 32;
    pos = 32;
  }
  uint32_t x = (uint32_t)m;
#pragma unroll
  for (int wdt = 16; wdt >= 2; wdt >>= 1) {
    c = (uint32_t)__popc(x & ((1u << wdt) - 1u));
    if (r >= c) {
      r -= c;
      x >>= wdt;
      pos += (uint32_t)wdt;
    }
  }
  return pos + (r >= (x & 1u) ? 1u : 0u);
}

// One partition of [f, l) (17 <= l - f <= 64 * C) in LDS by one wave; returns the cut.
// C (chunks of 64 per lane) is chosen per segment: a wave executes every unrolled
// chunk at full cost whatever its exec mask, and most partitions are small.  The
// median-to-first swap is applied in registers (position m holds the old first
// element, position f receives the pivot).  C == 1: swap partners are selected
// straight from the ballot masks; larger C exchange positions through LDS slots.
// The cut is the first position that is a non-swapped >= element or a swapped <=
// element (min(L[K+1], R[K])), found from ballots.
template <int C, class SL>
__device__ __forceinline__ uint32_t wave_partition(SL& S, uint32_t f, uint32_t l, uint16_t* xch) {
  const uint32_t lane = lane_id();
  const uint32_t m = median_pos(S.k, f, l);
  const uint32_t kf = S.k[f], vf = S.v[f], P = S.k[m], vm = S.v[m];
  const uint32_t n = l - f - 1;
  uint32_t kk[C], vv[C];
  uint32_t le_tot = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint32_t q = c * 64 + lane, p = f + 1 + q;
    const bool ok = q < n;
    kk[c] = ok ? S.k[p] : 0u;
    vv[c] = ok ? S.v[p] : 0u;
    if (p == m) {
      kk[c] = kf;
      vv[c] = vf;
    }
    le_tot += (uint32_t)__popcll(__ballot(ok && kk[c] <= P));
  }
  uint32_t cut = IS_NONE;
  // sw[c]: 1-based swap rank as a >= element (low 16 bits) / as a <= element (high 16)
  uint32_t sw[C];
  uint32_t gx = 0, lx = 0;  // counts before this chunk
  uint64_t bg0 = 0, bl0 = 0;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const bool ok = c * 64 + lane < n;
    const bool ge = ok && kk[c] >= P, le = ok && kk[c] <= P;
    const uint64_t bg = __ballot(ge), bl = __ballot(le);
    if (c == 0) {
      bg0 = bg;
      bl0 = bl;
    }
    const uint32_t g = gx + mbcnt(bg), h = lx + mbcnt(bl);
    const bool sg = ge && le_tot - h - (le ? 1u : 0u) >= g + 1;
    const bool sl = le && g >= le_tot - h;
    sw[c] = (sg ? g + 1 : 0u) | ((sl ? le_tot - h : 0u) << 16);
    const uint64_t cand = __ballot((ge && !sg) || sl);
    if (cut == IS_NONE && cand) cut = f + 1 + (uint32_t)(c * 64) + (uint32_t)(__ffsll((unsigned long long)cand) - 1);
    if (C > 1 && sg) xch[g] = (uint16_t)(f + 1 + c * 64 + lane);
    gx += (uint32_t)__popcll(bg);
    lx += (uint32_t)__popcll(bl);
  }
  if (C == 1) {
    const uint32_t kg = sw[0] & 0xFFFFu, kl = sw[0] >> 16;
    uint32_t d = f + 1 + lane;  // own position: only m must be rewritten when not swapped
    if (kg) d = f + 1 + select64(bl0, le_tot - kg);
    else if (kl) d = f + 1 + select64(bg0, kl - 1);
    if (kg || kl || d == m) {
      S.k[d] = kk[0];
      S.v[d] = vv[0];
    }
  } else {
    wsync();
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const uint32_t kl = sw[c] >> 16;
      if (kl) {  // take L[kr], leave R[kr] (this position) for its partner
        const uint32_t d = xch[kl - 1];
        xch[kl - 1] = (uint16_t)(f + 1 + c * 64 + lane);
        sw[c] = (sw[c] & 0xFFFFu) | (d << 16);
      }
    }
    wsync();
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const uint32_t p = f + 1 + c * 64 + lane, kg = sw[c] & 0xFFFFu, dl = sw[c] >> 16;
      uint32_t d = p;
      if (kg) d = xch[kg - 1];  // R[k]
      if (dl) d = dl;
      if (kg || dl || p == m) {
        S.k[d] = kk[c];
        S.v[d] = vv[c];
      }
    }
  }
  if (lane == 0) {
    S.k[f] = P;
    S.v[f] = vm;
  }
  wsync();
  return min(max(cut, f + 1), l - 1);
}

// The whole introsort subtree of [f, f+n) (n <= 64) in registers, level by level:
// lane i holds position f + i, the segments of a level are bit runs of the head mask
// H (all segments of one level share the depth), and every segment of the level is
// partitioned in the same pass -- per-lane pivots by shuffles, ranks and partners
// from the ballot masks restricted to the lane's segment, one shuffle per word for
// the swaps.  Leaves are then stably sorted by shuffles and written back in final
// order (every position marked as its own leaf).
template <class SL>
__device__ __forceinline__ void wave_sort_regs(SL& S, uint32_t f, uint32_t n, int d, uint32_t* /*stk*/) {
  const uint32_t lane = lane_id();
  const bool live = lane < n;
  uint32_t k = live ? S.k[f + lane] : 0xFFFFFFFFu, v = live ? S.v[f + lane] : 0u;
  const uint64_t below = (1ull << lane) - 1ull;             // lanes < lane
  const uint64_t upto = lane == 63 ? ~0ull : (2ull << lane) - 1ull;  // lanes <= lane
  uint64_t H = 1ull;                                         // segment starts
  uint64_t single = 0ull;                                    // heap-sorted positions (own leaves)
  for (int dd = d, guard = 0; guard < 64; --dd, ++guard) {
    // the lane's segment [a, b)
    const uint32_t a = 63u - (uint32_t)__clzll((long long)(H & upto));
    const uint64_t hi = H & ~upto;
    const uint32_t b = hi ? min(n, (uint32_t)(__ffsll((unsigned long long)hi) - 1)) : n;
    const uint32_t len = live ? b - a : 0u;
    const bool act = len > IS_THRESHOLD && !((single >> lane) & 1ull);
    if (!__ballot(act)) break;
    if (dd == 0) {  // depth limit: heap sort every remaining segment in LDS (rare)
      if (live) {
        S.k[f + lane] = k;
        S.v[f + lane] = v;
      }
      wsync();
      const uint64_t starts = __ballot(act && lane == a);
      if (lane == 0)
        for (uint64_t m = starts; m; m &= m - 1) {
          const uint32_t sa = (uint32_t)(__ffsll((unsigned long long)m) - 1);
          const uint64_t h2 = H & ~((2ull << sa) - 1ull);
          const uint32_t sb = h2 ? min(n, (uint32_t)(__ffsll((unsigned long long)h2) - 1)) : n;
          heap_sort(S.k + f + sa, S.v + f + sa, (int64_t)(sb - sa));
        }
      wsync();
      if (live) {
        k = S.k[f + lane];
        v = S.v[f + lane];
      }
      single |= __ballot(act);
      break;
    }
    // __move_median_to_first(a, a+1, mid, b-1) of the lane's segment
    const uint32_t A = a + 1, B = a + (b - a) / 2, C = b - 1;
    const uint32_t ka = (uint32_t)__shfl((int)k, (int)min(A, 63u), 64), kb = (uint32_t)__shfl((int)k, (int)min(B, 63u), 64),
                   kc = (uint32_t)__shfl((int)k, (int)min(C, 63u), 64);
    uint32_t mm;
    if (ka < kb) mm = kb < kc ? B : (ka < kc ? C : A);
    else mm = ka < kc ? A : (kb < kc ? C : B);
    mm = min(mm, 63u);
    const uint32_t P = (uint32_t)__shfl((int)k, (int)mm, 64), vm = (uint32_t)__shfl((int)v, (int)mm, 64);
    const uint32_t kf = (uint32_t)__shfl((int)k, (int)a, 64), vf = (uint32_t)__shfl((int)v, (int)a, 64);
    if (act) {
      if (lane == a) {
        k = P;
        v = vm;
      } else if (lane == mm) {
        k = kf;
        v = vf;
      }
    }
    const bool in = act && lane > a;
    const uint64_t seg = (b >= 64 ? ~0ull : ((1ull << b) - 1ull)) & ~((2ull << a) - 1ull);  // (a, b)
    const uint64_t bg = __ballot(in && k >= P) & seg, bl = __ballot(in && k <= P) & seg;
    const uint32_t le_tot = (uint32_t)__popcll(bl);
    const bool ge = (bg >> lane) & 1ull, le = (bl >> lane) & 1ull;
    const uint32_t g = (uint32_t)__popcll(bg & below), h = (uint32_t)__popcll(bl & below);
    const bool sg = ge && le_tot - h - (le ? 1u : 0u) >= g + 1;
    const bool sl = le && g >= le_tot - h;
    uint32_t src = lane;  // the lane whose element lands here (swaps are symmetric)
    if (sg) src = select64(bl, le_tot - (g + 1));
    else if (sl) src = select64(bg, le_tot - h - 1);
    const uint64_t cand = __ballot((ge && !sg) || sl) & seg;
    const uint32_t cut = cand ? (uint32_t)(__ffsll((unsigned long long)cand) - 1) : A;
    k = (uint32_t)__shfl((int)k, (int)src, 64);
    v = (uint32_t)__shfl((int)v, (int)src, 64);
    H |= __ballot(act && lane == cut);
  }
  // stable sort of each leaf (<= 16 lanes; heap-sorted positions are their own leaves)
  const uint64_t HL = H | single | (single << 1);
  const uint32_t ls = 63u - (uint32_t)__clzll((long long)(HL & upto));
  const uint64_t above = HL & ~upto;
  const uint32_t le_ = above ? min(n, (uint32_t)(__ffsll((unsigned long long)above) - 1)) : n;
  uint32_t rank = 0;
#pragma unroll
  for (int j = 0; j < (int)IS_THRESHOLD; ++j) {
    const uint32_t q = min(ls + (uint32_t)j, 63u);
    const uint32_t kq = (uint32_t)__shfl((int)k, (int)q, 64);
    if (ls + (uint32_t)j < le_ && (kq < k || (kq == k && ls + (uint32_t)j < lane))) ++rank;
  }
  wsync();
  if (live) {
    S.k[f + ls + rank] = k;
    S.v[f + ls + rank] = v;
  }
  if (lane == 0) {  // every position of the run is final: one leaf each
    for (uint32_t q = 0; q < n; q += 32 - ((f + q) & 31)) {
      const uint32_t bit = (f + q) & 31, cnt = min(32u - bit, n - q);
      atomicOr(&S.heads[(f + q) >> 5], (cnt == 32 ? 0xFFFFFFFFu : ((1u << cnt) - 1u)) << bit);
    }
  }
  wsync();
}

// The introsort subtree of [off, off+len) (len <= IS_WCAP) by one wave, in LDS.
template <class SL>
__device__ __forceinline__ void wave_sort(SL& S, uint32_t packed, uint32_t* stk, uint16_t* xch) {
  const uint32_t lane = lane_id();
  int sp = 0;
  stk[sp++] = packed;
  for (uint32_t guard = 0; sp > 0; ++guard) {
    if (guard > 4 * IS_WCAP || sp >= IS_STACK / 2) {  // cannot happen
      if (lane == 0) is_fault(S.stat, S.err, IS_FAULT_WAVE);
      break;
    }
    const uint32_t it = __builtin_amdgcn_readfirstlane(stk[--sp]);
    const uint32_t f = it & 0x1FFFu, n = (it >> 13) & 0x7FFu;
    const int dd = (int)(it >> 24);
    if (n <= IS_THRESHOLD) {
      if (lane == 0 && n) mark_leaf(S, f);
      continue;
    }
    if (dd == 0) {  // depth limit: rank_in_segment (heap sort on ties)
      uint32_t kd[IS_WC], vd[IS_WC], rd[IS_WC];
      bool dup = false;
#pragma unroll
      for (int c = 0; c < IS_WC; ++c) {
        const uint32_t q = c * 64 + lane;
        kd[c] = vd[c] = rd[c] = 0u;
        if (q < n) {
          kd[c] = S.k[f + q];
          vd[c] = S.v[f + q];
          rd[c] = f + rank_in_segment(S.k, f, f + n, f + q, kd[c], dup);
        }
      }
      const bool ties = __ballot(dup) != 0ull;
      wsync();
      if (!ties) {
#pragma unroll
        for (int c = 0; c < IS_WC; ++c)
          if (c * 64 + lane < n) {
            S.k[rd[c]] = kd[c];
            S.v[rd[c]] = vd[c];
          }
      } else if (lane == 0) {
        heap_sort(S.k + f, S.v + f, (int64_t)n);
      }
      wsync();
      for (uint32_t q = lane; q < n; q += 64) mark_leaf(S, f + q);
      wsync();
      continue;
    }
    if (n <= 64) {  // the rest of this subtree in registers
      if (S.son && lane == 0) atomicAdd(&S.lstat[0], 1u);
      wave_sort_regs(S, f, n, dd, stk + sp);
      continue;
    }
    if (S.son && lane == 0) atomicAdd(&S.lstat[2], 1u);
    uint32_t c;
    if (n <= 128) c = wave_partition<2, SL>(S, f, f + n, xch);
    else if (n <= 256) c = wave_partition<4, SL>(S, f, f + n, xch);
    else if (IS_WC <= 8 || n <= 512) c = wave_partition<(IS_WC < 8 ? IS_WC : 8), SL>(S, f, f + n, xch);
    else c = wave_partition<IS_WC, SL>(S, f, f + n, xch);
    stk[sp++] = wpack(c, f + n - c, dd - 1);
    stk[sp++] = wpack(f, c - f, dd - 1);
  }
}

// The rank of position p (key k[p]) in its leaf [a, b) of a finished wave task, ties
// by position: # of q in [a, b) with (k[q], q) < (key, p).  b - a <= 16, and the scan
// runs over the fixed window [a, a + 16): the positions in [b, a + 16) belong to later
// segments, whose keys are >= every key of the leaf (the partitions' invariant), equal
// ones at q > p, and the 16 positions past the task hold IS_NONE, so none of them
// counts -- sixteen unrolled reads at immediate offsets, no per-lane loop bound.
__device__ __forceinline__ uint32_t leaf_rank(const uint32_t* k, uint32_t a, uint32_t p, uint32_t key) {
  const uint64_t me = (uint64_t)key << 32 | p;
  uint32_t r = 0;
#pragma unroll
  for (uint32_t j = 0; j < IS_THRESHOLD; ++j) r += ((uint64_t)k[a + j] << 32 | (a + j)) < me ? 1u : 0u;
  return r;
}

// # of the level's >= (s = 0) / <= (s = 1) elements before position x (0 <= x <= 64 C)
__device__ __forceinline__ uint32_t level_rank(const WaveLds& S, int s, uint32_t x) {
  const uint32_t c = x >> 6, bit = x & 63u;
  return S.pc[s][c] + (uint32_t)__popcll(S.bw[s][c] & ((1ull << bit) - 1ull));
}

// A whole wave task [f, f+n) (64 < n <= 64 C), in LDS, level by level: every segment
// of a level is partitioned in the same pass, so the task's dependent chain is its
// tree depth instead of its partition count (the <= 64 subtrees of wave_sort_regs
// already work this way).  Position p = 64 c + lane stays with (chunk c, lane), whose
// segment [a, b) is kept in registers.  Per level, for the segments longer than 16:
// each lane takes its segment's median-of-3 pivot itself (three LDS reads), >= / <=
// flags against it, ballots per chunk and their prefix counts (one LDS table), so
// the segment-relative ranks are differences of whole-window ranks and the k-th
// >= / <= element of a segment is read from the window's compacted position lists;
// the swap rule and the cut are wave_partition's.  Depth 0 heap-sorts what is still
// active (rare).  The leaves are then stably sorted by rank and written to K/V.
template <int C>
__device__ __forceinline__ void wave_task_level(WaveLds& S, uint32_t* __restrict__ K, uint32_t* __restrict__ V,
                                                uint32_t f, uint32_t n, int d, const IsBufs& W,
                                                const float* __restrict__ src) {
  const uint32_t lane = lane_id();
  uint32_t ab[C];  // a | b << 16
#pragma unroll
  for (int c = 0; c < C; ++c) ab[c] = n << 16;
  for (int dd = d;; --dd) {
    uint32_t actm = 0;  // bit c: chunk c's position lies in a segment still to partition
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const uint32_t p = c * 64 + lane, a = ab[c] & 0xFFFFu, b = ab[c] >> 16;
      if (p < n && b - a > IS_THRESHOLD) actm |= 1u << c;
    }
    if (!__ballot(actm != 0u)) break;
    if (dd == 0) {  // depth limit: every active segment sorted (rank_in_segment; heap sort on ties)
      {
        uint32_t kd[C], vd[C], rd[C];
        bool dup = false;
#pragma unroll
        for (int c = 0; c < C; ++c) {
          const uint32_t p = c * 64 + lane;
          kd[c] = vd[c] = rd[c] = 0u;
          if ((actm >> c) & 1u) {
            kd[c] = S.k[p];
            vd[c] = S.v[p];
            rd[c] = (ab[c] & 0xFFFFu) + rank_in_segment(S.k, ab[c] & 0xFFFFu, ab[c] >> 16, p, kd[c], dup);
          }
        }
        if (!__ballot(dup)) {
          wsync();
#pragma unroll
          for (int c = 0; c < C; ++c)
            if ((actm >> c) & 1u) {
              S.k[rd[c]] = kd[c];
              S.v[rd[c]] = vd[c];
            }
          wsync();
#pragma unroll
          for (int c = 0; c < C; ++c) {
            const uint32_t p = c * 64 + lane;
            if ((actm >> c) & 1u) ab[c] = p | ((p + 1) << 16);  // sorted: every position its own leaf
          }
          if (S.son && lane == 0) atomicAdd(&S.stat[9], 1u);
          break;
        }
      }
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const uint32_t p = c * 64 + lane;
        if (((actm >> c) & 1u) && p == (ab[c] & 0xFFFFu)) S.cutv[p] = ab[c] >> 16;
      }
      uint64_t hd[C];
#pragma unroll
      for (int c = 0; c < C; ++c) hd[c] = __ballot(((actm >> c) & 1u) && c * 64 + lane == (ab[c] & 0xFFFFu));
      wsync();
      if (lane == 0)
#pragma unroll
        for (int c = 0; c < C; ++c)
          for (uint64_t m = hd[c]; m; m &= m - 1) {
            const uint32_t a = c * 64 + (uint32_t)(__ffsll((unsigned long long)m) - 1);
            heap_sort(S.k + a, S.v + a, (int64_t)(S.cutv[a] - a));
          }
      wsync();
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const uint32_t p = c * 64 + lane;
        if ((actm >> c) & 1u) ab[c] = p | ((p + 1) << 16);  // sorted: every position its own leaf
      }
      break;
    }
    // Per-segment work once per segment instead of once per position: lane s takes
    // the level's s-th segment (its median, pivot and whole-window ranks) and leaves
    // them in the segment's own cutv slots a+1..a+3 (a segment here has > 16
    // positions, so they are its own), which its positions then read.
    constexpr bool SEGT = C >= IS_SEGT_MINC;
    static_assert(IS_WCAP / (IS_THRESHOLD + 1) < 64 && IS_WCAP <= 1023, "one lane per segment; 10-bit ranks");
    uint32_t sa = 0, sb = 0, nsg = 0;
    if constexpr (SEGT) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const bool head = ((actm >> c) & 1u) && c * 64 + lane == (ab[c] & 0xFFFFu);
        const uint64_t hm = __ballot(head);
        if (head) S.seg[nsg + mbcnt(hm)] = ab[c];
        nsg += (uint32_t)__popcll(hm);
      }
      wsync();
      if (lane < nsg) {
        const uint32_t s = S.seg[lane];
        sa = s & 0xFFFFu;
        sb = s >> 16;
        // __move_median_to_first(a, a+1, mid, b-1): a receives the pivot, m the old first
        const uint32_t m = median_pos(S.k, sa, sb);
        S.cutv[sa] = IS_NONE;
        S.cutv[sa + 1] = S.k[m];
        S.cutv[sa + 2] = m;
      }
      wsync();
    }
    uint32_t kk[C], vv[C];
    uint64_t bg[C], bl[C];
    uint32_t moved = 0;  // bit c: chunk c's position is the segment's first or its median (rewritten in place)
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const uint32_t p = c * 64 + lane, a = ab[c] & 0xFFFFu, b = ab[c] >> 16;
      const bool act = (actm >> c) & 1u;
      kk[c] = 0u;
      vv[c] = 0u;
      bool ge = false, le = false;
      if (act) {  // (positions in finished segments are neither read nor written)
        kk[c] = S.k[p];
        vv[c] = S.v[p];
        // __move_median_to_first(a, a+1, mid, b-1): a receives the pivot, m the old first
        uint32_t m, P;
        if constexpr (SEGT) {
          P = S.cutv[a + 1];
          m = S.cutv[a + 2];
        } else {
          m = median_pos(S.k, a, b);
          P = S.k[m];
        }
        if (p == a) {
          kk[c] = P;
          vv[c] = S.v[m];
          if constexpr (!SEGT) S.cutv[a] = IS_NONE;
          moved |= 1u << c;
        } else {
          if (p == m) {
            kk[c] = S.k[a];
            vv[c] = S.v[a];
            moved |= 1u << c;
          }
          ge = kk[c] >= P;
          le = kk[c] <= P;
        }
      }
      bg[c] = __ballot(ge);
      bl[c] = __ballot(le);
    }
    if (lane == 0) {
      uint32_t rg = 0, rl = 0;
#pragma unroll
      for (int c = 0; c <= C; ++c) {
        S.pc[0][c] = rg;
        S.pc[1][c] = rl;
        S.bw[0][c] = c < C ? bg[c] : 0ull;
        S.bw[1][c] = c < C ? bl[c] : 0ull;
        if (c < C) {
          rg += (uint32_t)__popcll(bg[c]);
          rl += (uint32_t)__popcll(bl[c]);
        }
      }
    }
    wsync();  // (every read of S.k above precedes every write below)
    if constexpr (SEGT) {
      if (lane < nsg) {
        const uint32_t g0 = level_rank(S, 0, sa + 1), l0 = level_rank(S, 1, sa + 1);
        S.cutv[sa + 3] = g0 | l0 << 10 | (level_rank(S, 1, sb) - l0) << 20;
      }
      wsync();
    }
    uint32_t li[C];  // 1 + index into S.ll (a swapped >=) or S.lg | 1 << 16 (a swapped <=), 0: stays
#pragma unroll
    for (int c = 0; c < C; ++c) {
      li[c] = 0;
      if (!((actm >> c) & 1u)) continue;
      const uint32_t p = c * 64 + lane, a = ab[c] & 0xFFFFu, b = ab[c] >> 16;
      if (p == a) continue;
      const bool ge = (bg[c] >> lane) & 1ull, le = (bl[c] >> lane) & 1ull;
      uint32_t g0, l0, le_tot;
      if constexpr (SEGT) {
        const uint32_t r = S.cutv[a + 3];
        g0 = r & 0x3FFu;
        l0 = (r >> 10) & 0x3FFu;
        le_tot = r >> 20;
      } else {
        g0 = level_rank(S, 0, a + 1);
        l0 = level_rank(S, 1, a + 1);
        le_tot = level_rank(S, 1, b) - l0;
      }
      const uint32_t ga = S.pc[0][c] + mbcnt(bg[c]), la = S.pc[1][c] + mbcnt(bl[c]);
      const uint32_t g = ga - g0, h = la - l0;  // # >= / # <= of the segment before p
      const bool sg = ge && le_tot - h - (le ? 1u : 0u) >= g + 1;
      const bool sl = le && g >= le_tot - h;
      if (ge) S.lg[ga] = (uint16_t)p;
      if (le) S.ll[la] = (uint16_t)p;
      if ((ge && !sg) || sl) atomicMin(&S.cutv[a], p);  // L[K+1] / R[K]
      if (sg) li[c] = 1u + l0 + (le_tot - g - 1);        // R[g+1]
      else if (sl) li[c] = (1u + g0 + (le_tot - h - 1)) | (1u << 16);  // L[kr]
    }
    wsync();
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (!((actm >> c) & 1u)) continue;
      const uint32_t p = c * 64 + lane;
      uint32_t dst = p;
      if (li[c]) {
        const uint32_t x = (li[c] & 0xFFFFu) - 1u;
        dst = (li[c] >> 16) ? S.lg[x] : S.ll[x];
      } else if (!((moved >> c) & 1u)) {
        continue;  // stays in place
      }
      S.k[dst] = kk[c];
      S.v[dst] = vv[c];
    }
    wsync();
#pragma unroll
    for (int c = 0; c < C; ++c) {
      if (!((actm >> c) & 1u)) continue;
      const uint32_t p = c * 64 + lane, a = ab[c] & 0xFFFFu, b = ab[c] >> 16;
      const uint32_t cut = min(max(S.cutv[a], a + 1), b - 1);
      ab[c] = p >= cut ? (cut | (b << 16)) : (a | (cut << 16));
    }
    wsync();  // (the cut reads precede the next level's resets)
  }
  // stable sort of every leaf (<= 16 positions) by rank, straight to K/V
  uint32_t dpos[C], dval[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint32_t p = c * 64 + lane;
    dpos[c] = IS_NONE;
    dval[c] = 0u;
    if (p >= n) continue;
    const uint32_t a = ab[c] & 0xFFFFu;
    const uint32_t key = S.k[p];
    // (< b - a whenever the partitions' invariant holds; the clamp keeps every store
    // inside the task whatever the data)
    const uint32_t rank = min(leaf_rank(S.k, a, p, key), (ab[c] >> 16) - a - 1u);
    dpos[c] = f + a + rank;
    dval[c] = S.v[p];
    K[dpos[c]] = key;
    V[dpos[c]] = dval[c];
  }
  if (src) {  // every gather issued before the first point store
    Pt3 pt[C];
#pragma unroll
    for (int c = 0; c < C; ++c) pt[c] = load_xyz(src, dval[c]);  // (dval = 0 past n: a valid point, not stored)
#pragma unroll
    for (int c = 0; c < C; ++c)
      if (dpos[c] != IS_NONE) store_xyz(W, dpos[c], pt[c]);
  }
}

// One partition of [f, l) (IS_WCAP < l - f <= IS_OT * C) in LDS by the whole block.
template <int C>
__device__ __forceinline__ uint32_t block_partition(BlockLds& S, uint32_t f, uint32_t l) {
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    const uint32_t m = median_pos(S.k, f, l);
    const uint32_t tk = S.k[f], tv = S.v[f];
    S.k[f] = S.k[m];
    S.v[f] = S.v[m];
    S.k[m] = tk;
    S.v[m] = tv;
    S.bc[4] = IS_NONE;
  }
  for (uint32_t i = C * IS_OW + threadIdx.x; i < IS_OE; i += IS_OT) {  // unused (chunk, wave) entries
    S.cg[i] = 0;
    S.cl[i] = 0;
  }
  __syncthreads();
  const uint32_t P = S.k[f];
  const uint32_t n = l - f - 1;
  uint32_t kk[C], vv[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint32_t q = c * IS_OT + threadIdx.x;
    const bool ok = q < n;
    kk[c] = ok ? S.k[f + 1 + q] : 0u;
    vv[c] = ok ? S.v[f + 1 + q] : 0u;
    const uint64_t bg = __ballot(ok && kk[c] >= P), bl = __ballot(ok && kk[c] <= P);
    if (lane == 0) {
      S.cg[c * IS_OW + w] = (uint32_t)__popcll(bg);
      S.cl[c * IS_OW + w] = (uint32_t)__popcll(bl);
    }
  }
  __syncthreads();
  if (w == 0) block_chunk_scan(S, 0u, 0u);
  __syncthreads();
  const uint32_t le_tot = S.pl[IS_OE - 1] + S.cl[IS_OE - 1];  // read by every thread after the scan's barrier
  uint32_t cut = IS_NONE;
  uint32_t sw[C];  // swap rank as >= (low 16 bits) / as <= (high 16), later the <= destination
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint32_t q = c * IS_OT + threadIdx.x, p = f + 1 + q;
    const bool ok = q < n;
    const bool ge = ok && kk[c] >= P, le = ok && kk[c] <= P;
    const uint64_t bg = __ballot(ge), bl = __ballot(le);
    const uint32_t g = S.pg[c * IS_OW + w] + mbcnt(bg), h = S.pl[c * IS_OW + w] + mbcnt(bl);
    const bool sg = ge && le_tot - h - (le ? 1u : 0u) >= g + 1;
    const bool sl = le && g >= le_tot - h;
    sw[c] = (sg ? g + 1 : 0u) | ((sl ? le_tot - h : 0u) << 16);
    const uint64_t cand = __ballot((ge && !sg) || sl);
    if (cut == IS_NONE && cand) cut = p - lane + (uint32_t)(__ffsll((unsigned long long)cand) - 1);
    if (sg) S.xch[g] = (uint16_t)p;
  }
  if (lane == 0 && cut != IS_NONE) atomicMin(&S.bc[4], cut);
  __syncthreads();
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint32_t kl = sw[c] >> 16;
    if (kl) {
      const uint32_t d = S.xch[kl - 1];
      S.xch[kl - 1] = (uint16_t)(f + 1 + c * IS_OT + threadIdx.x);
      sw[c] = (sw[c] & 0xFFFFu) | (d << 16);
    }
  }
  __syncthreads();
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const uint32_t kg = sw[c] & 0xFFFFu, dl = sw[c] >> 16;
    if (kg || dl) {
      const uint32_t d = kg ? (uint32_t)S.xch[kg - 1] : dl;
      S.k[d] = kk[c];
      S.v[d] = vv[c];
    }
  }
  __syncthreads();
  // (S.bc[4] is reset only by the next partition's thread 0, after the caller's
  // barrier that follows its stack update, so no barrier is needed after this read)
  return min(max(S.bc[4], f + 1), l - 1);
}

// The segment [f, f+len) (len <= IS_LCAP, depth d) from (Ki, Vi): workgroup
// partitions in LDS down to subtrees of <= IS_WCAP, which become wave tasks; the
// leaves and heap-sorted ranges are stably sorted here.  The whole run is written
// to (Ko, Vo) (task ranges in their current order, for the wave kernel).
__device__ __forceinline__ void lds_block(BlockLds& S, const IsBufs& W, const uint32_t* Ki, const uint32_t* Vi,
                                          uint32_t* Ko, uint32_t* Vo, uint32_t f, uint32_t len, int d) {
  IS_PH_START();
  for (uint32_t q = threadIdx.x; q < len; q += IS_OT) {
    S.k[q] = Ki[f + q];
    S.v[q] = Vi[f + q];
  }
  for (uint32_t q = threadIdx.x; q < (len + 31) / 32; q += IS_OT) {
    S.heads[q] = 0;
    S.intask[q] = 0;
  }
  if (threadIdx.x == 0) {
    S.bc[0] = 0;  // stack depth
    S.ntb = S.nts = S.units = 0;
    if (len <= IS_THRESHOLD) {
      S.heads[0] = 1u;
    } else {
      S.wstk[0] = make_uint2(0u, len | ((uint32_t)d << 16));
      S.bc[0] = 1;
    }
  }
  // thread 0 pops the stack until it finds a subtree to partition (leaves, heap
  // ranges and wave tasks are settled on the way); S.bc[3] = found
  auto pop = [&]() {
    if (threadIdx.x == 0) {
      uint32_t go = 0;
      while (S.bc[0] > 0 && !go) {
        const uint2 it = S.wstk[--S.bc[0]];
        const uint32_t off = it.x, n = it.y & 0xFFFFu;
        const int dd = (int)(it.y >> 16);
        if (n <= IS_THRESHOLD) {
          if (n) mark_leaf(S, off);
        } else if (dd == 0) {  // depth limit: the whole workgroup sorts it (below)
          S.bc[6] = off;
          S.bc[7] = it.y;
          go = 2;
        } else if (n <= IS_WCAP) {  // a wave task: large ones from the front, small from the back
          S.units += n;  // the wave probe's unit count
          const uint32_t pk = off | (n << 13) | ((uint32_t)dd << 24);
          if (n > IS_TASK_BIG) S.tb[S.ntb++] = pk;
          else S.ts[S.nts++] = pk;
          for (uint32_t q = off; q < off + n; q += 32 - (q & 31)) {
            const uint32_t bit = q & 31, cnt = min(32u - bit, off + n - q);
            atomicOr(&S.intask[q >> 5], (cnt == 32 ? 0xFFFFFFFFu : ((1u << cnt) - 1u)) << bit);
          }
        } else {
          S.bc[6] = off;
          S.bc[7] = it.y;
          go = 1;
        }
      }
      if (S.bc[0] >= IS_STACK / 2 - 2) {  // cannot happen
        is_fault(S.stat, S.err, IS_FAULT_POP);
        S.bc[0] = 0;
      }
      S.bc[3] = go;
    }
  };
  pop();
  __syncthreads();
  for (;;) {
    if (!S.bc[3]) break;
    const uint32_t off = S.bc[6], n = S.bc[7] & 0xFFFFu;
    const int dd = (int)(S.bc[7] >> 16);
    if (S.bc[3] == 2) {  // depth limit: rank_in_segment by the workgroup (heap sort on ties)
      uint32_t kd[IS_OC], vd[IS_OC], rd[IS_OC];
      bool dup = false;
#pragma unroll
      for (int c = 0; c < IS_OC; ++c) {
        const uint32_t q = c * IS_OT + threadIdx.x;
        kd[c] = vd[c] = rd[c] = 0u;
        if (q < n) {
          kd[c] = S.k[off + q];
          vd[c] = S.v[off + q];
          rd[c] = off + rank_in_segment(S.k, off, off + n, off + q, kd[c], dup);
        }
      }
      if (threadIdx.x == 0) S.bc[5] = 0;
      __syncthreads();
      if (dup) S.bc[5] = 1;
      __syncthreads();
      if (S.bc[5] == 0) {
#pragma unroll
        for (int c = 0; c < IS_OC; ++c)
          if (c * IS_OT + threadIdx.x < n) {
            S.k[rd[c]] = kd[c];
            S.v[rd[c]] = vd[c];
          }
        if (S.son && threadIdx.x == 0) atomicAdd(&S.stat[9], 1u);
      } else if (threadIdx.x == 0) {
        heap_sort(S.k + off, S.v + off, (int64_t)n);
        if (S.son) atomicAdd(&S.stat[7], 1u);
      }
      __syncthreads();
      for (uint32_t q = threadIdx.x; q < n; q += IS_OT) mark_leaf(S, off + q);
      pop();
      __syncthreads();
      continue;
    }
    if (S.son && threadIdx.x == 0) atomicAdd(&S.stat[5], 1u);
    uint32_t c;
    if (n <= 2 * IS_OT) c = block_partition<2>(S, off, off + n);
    else if (n <= 4 * IS_OT) c = block_partition<4>(S, off, off + n);
    else if (n <= 8 * IS_OT) c = block_partition<8>(S, off, off + n);
    else c = block_partition<IS_OC>(S, off, off + n);
    if (threadIdx.x == 0) {  // push both children, then pop the next subtree: one barrier
      const uint32_t nd = (uint32_t)(dd - 1) << 16;
      S.wstk[S.bc[0]++] = make_uint2(c, (off + n - c) | nd);
      S.wstk[S.bc[0]++] = make_uint2(off, (c - off) | nd);
    }
    pop();
    __syncthreads();
  }
  IS_PH(11);  // block item: load and partitions
  // the segment's wave tasks into the global list: one slot reservation per class
  if (threadIdx.x == 0) {
    S.bc[1] = S.ntb ? atomicAdd(&W.ctl[16], S.ntb) : 0u;
    S.bc[2] = S.nts ? atomicAdd(&W.ctl[18], S.nts) : 0u;
    if (S.units) atomicAdd(&W.ctl[19], S.units);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < S.ntb + S.nts; i += IS_OT) {
    const bool big = i < S.ntb;
    const uint32_t pk = big ? S.tb[i] : S.ts[i - S.ntb];
    const uint4 t = make_uint4(f + (pk & 0x1FFFu), (pk >> 13) & 0x7FFu, pk >> 24, 0u);
    if (big) W.tasks[S.bc[1] + i] = t;
    else W.tasks[W.taskmax - 1u - (S.bc[2] + i - S.ntb)] = t;
  }
  IS_PH(12);  // block item: tasks listed
  // leaves: stable sort in place (the final insertion sort); task ranges as they are
  const float* __restrict__ xsrc = W.xyzs ? W.vgp->src : nullptr;
  for (uint32_t p = threadIdx.x; p < len; p += IS_OT) {
    const uint32_t key = S.k[p];
    if ((S.intask[p >> 5] >> (p & 31)) & 1u) {
      Ko[f + p] = key;
      Vo[f + p] = S.v[p];
      continue;
    }
    uint32_t a = 0, b = len;
    {
      uint32_t wi = p >> 5, m = S.heads[wi] & (0xFFFFFFFFu >> (31 - (p & 31)));
      while (!m && wi > 0) m = S.heads[--wi];
      if (m) a = (wi << 5) + 31 - __clz((int)m);
      uint32_t wj = (p + 1) >> 5, nw = (len + 31) >> 5;
      const uint32_t q = (p + 1) & 31;
      uint32_t mm = wj < nw ? (S.heads[wj] & (0xFFFFFFFFu << q)) : 0u;
      while (!mm && ++wj < nw) mm = S.heads[wj];
      if (mm) b = min(len, (wj << 5) + (uint32_t)__ffs((int)mm) - 1);
      // a leaf never reaches into a task range: tasks start at a head-less position
      // bounded by the next head or task start, so clip at the first task position
      for (uint32_t x = p + 1; x < b; ++x)
        if ((S.intask[x >> 5] >> (x & 31)) & 1u) {
          b = x;
          break;
        }
    }
    uint32_t rank = 0;
    for (uint32_t q = a; q < b; ++q) {
      const uint32_t kq = S.k[q];
      rank += (kq < key || (kq == key && q < p)) ? 1u : 0u;
    }
    Ko[f + a + rank] = key;
    Vo[f + a + rank] = S.v[p];
    if (xsrc) put_xyz(W, xsrc, f + a + rank, S.v[p]);  // (the block's leaf elements are few: most go to wave tasks)
  }
  __syncthreads();
  IS_PH(13);  // block item: leaves and write-back
}

// One partition of [f, l) (l - f > IS_LCAP) in global memory by the whole block,
// in place in (K, V); (SK, SV) at the same positions is scratch.  Returns the cut.
// (free != 0: a segment known to hold pairwise distinct keys, whose sorted order is
// unique: the median of three pseudo-random positions instead of std::sort's first+1 /
// mid / last-1, so that an input built against that rule does not stay quadratic.)
__device__ __forceinline__ uint32_t global_partition(BlockLds& S, uint32_t* K, uint32_t* V, uint32_t* SK, uint32_t* SV, uint32_t f,
                                     uint32_t l, uint32_t free = 0) {
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  if (threadIdx.x == 0) {
    uint32_t m;
    if (free) {
      uint32_t x = f * 0x9E3779B9u ^ l * 0x85EBCA6Bu;
      uint32_t r[3];
      for (int i = 0; i < 3; ++i) {
        x ^= x >> 16;
        x *= 0x7FEB352Du;
        x ^= x >> 15;
        x *= 0x846CA68Bu;
        x ^= x >> 16;
        r[i] = f + 1 + x % (l - f - 1);
      }
      const uint32_t a = K[r[0]], b = K[r[1]], c = K[r[2]];
      m = (a < b) ? (b < c ? r[1] : (a < c ? r[2] : r[0])) : (a < c ? r[0] : (b < c ? r[2] : r[1]));
    } else {
      m = median_pos(K, f, l);
    }
    const uint32_t tk = K[f], tv = V[f];
    K[f] = K[m];
    V[f] = V[m];
    K[m] = tk;
    V[m] = tv;
    S.bc[4] = IS_NONE;
    S.bc[0] = 0;  // running >= count
    S.bc[1] = 0;  // running <= count
  }
  hand_off_fence();
  __syncthreads();
  const uint32_t P = K[f];
  const uint32_t n = l - f - 1, H = (l - f) / 2;
  // totals of <= P
  uint32_t lc = 0;
  for (uint32_t q = threadIdx.x; q < n; q += IS_OT) lc += K[f + 1 + q] <= P ? 1u : 0u;
  uint32_t le_tot;
  (void)block_excl_scan(lc, S.sh, &le_tot);
  uint32_t cut = IS_NONE;
  for (int pass = 0; pass < 2; ++pass) {
    if (threadIdx.x == 0) {
      S.bc[0] = 0;
      S.bc[1] = 0;
    }
    __syncthreads();
    for (uint32_t s0 = 0; s0 < n; s0 += IS_LCAP) {
      uint32_t kk[IS_OC], vv[IS_OC];
#pragma unroll
      for (int c = 0; c < IS_OC; ++c) {
        const uint32_t q = s0 + c * IS_OT + threadIdx.x;
        const bool ok = q < n;
        kk[c] = ok ? K[f + 1 + q] : 0u;
        vv[c] = ok ? V[f + 1 + q] : 0u;
        const uint64_t bg = __ballot(ok && kk[c] >= P), bl = __ballot(ok && kk[c] <= P);
        if (lane == 0) {
          S.cg[c * IS_OW + w] = (uint32_t)__popcll(bg);
          S.cl[c * IS_OW + w] = (uint32_t)__popcll(bl);
        }
      }
      __syncthreads();
      if (w == 0) block_chunk_scan(S, S.bc[0], S.bc[1]);
      __syncthreads();
      if (threadIdx.x == 0) {  // running counts for the next superchunk
        S.bc[0] = S.pg[IS_OE - 1] + S.cg[IS_OE - 1];
        S.bc[1] = S.pl[IS_OE - 1] + S.cl[IS_OE - 1];
      }
#pragma unroll
      for (int c = 0; c < IS_OC; ++c) {
        const uint32_t q = s0 + c * IS_OT + threadIdx.x, p = f + 1 + q;
        const bool ok = q < n;
        const bool ge = ok && kk[c] >= P, le = ok && kk[c] <= P;
        const uint64_t bg = __ballot(ge), bl = __ballot(le);
        const uint32_t g = S.pg[c * IS_OW + w] + mbcnt(bg), h = S.pl[c * IS_OW + w] + mbcnt(bl);
        if (ge) {
          const uint32_t k1 = g + 1;
          if (le_tot - h - (le ? 1u : 0u) >= k1) {
            if (pass == 0) {  // publish: the value R[k1] receives
              SK[f + k1 - 1] = kk[c];
              SV[f + k1 - 1] = vv[c];
            } else {  // take L[k1]'s partner's value
              K[p] = SK[f + H + k1 - 1];
              V[p] = SV[f + H + k1 - 1];
            }
          } else {
            cut = min(cut, p);
          }
        }
        if (le) {
          const uint32_t kr = le_tot - h;
          if (g >= kr) {
            if (pass == 0) {
              SK[f + H + kr - 1] = kk[c];
              SV[f + H + kr - 1] = vv[c];
            } else {
              K[p] = SK[f + kr - 1];
              V[p] = SV[f + kr - 1];
            }
            cut = min(cut, p);
          }
        }
      }
      __syncthreads();  // superchunks are independent within a pass
    }
    hand_off_fence();  // pass 0's scratch (or pass 1's in-place writes) visible to every wave
    __syncthreads();
  }
  cut = wave_min_u32(cut);
  if (lane == 0 && cut != IS_NONE) atomicMin(&S.bc[4], cut);
  __syncthreads();
  const uint32_t r = min(max(S.bc[4], f + 1), l - 1);
  __syncthreads();
  return r;
}

// Whether the len keys at K are pairwise distinct (one workgroup): an open-addressing
// table of 2 len slots in the scratch arrays T0[0, len) and T1[0, len) (the other
// buffer at the segment's positions), filled by atomicCAS.  For the depth limit on a
// segment beyond the LDS (see rank_in_segment).
__device__ bool distinct_keys(BlockLds& S, const uint32_t* K, uint32_t* T0, uint32_t* T1, uint32_t len) {
  for (uint32_t q = threadIdx.x; q < len; q += IS_OT) T0[q] = T1[q] = IS_NONE;
  if (threadIdx.x == 0) S.bc[5] = 0;
  hand_off_fence();  // (the table's initial values before any wave's atomics)
  __syncthreads();
  const uint32_t nsl = 2 * len;
  bool dup = false;
  for (uint32_t q = threadIdx.x; q < len && !dup; q += IS_OT) {
    const uint32_t key = K[q];
    uint32_t h = key * 0x9E3779B1u;
    h = (uint32_t)(((uint64_t)(h ^ (h >> 15)) * nsl) >> 32);
    for (uint32_t probe = 0; probe < nsl; ++probe) {
      uint32_t* slot = h < len ? &T0[h] : &T1[h - len];
      const uint32_t old = atomicCAS(slot, IS_NONE, key);
      if (old == IS_NONE) break;
      if (old == key) {
        dup = true;
        break;
      }
      h = h + 1 == nsl ? 0u : h + 1;
    }
  }
  if (dup) S.bc[5] = 1;
  __syncthreads();
  const bool r = S.bc[5] == 0;
  __syncthreads();
  return r;
}

// The block kernel's items -- the last round's final children (index i < nfin), then the
// owned list -- in descending size, as indices into that list (W.ord), so that the
// workgroups dequeue the longest items first and the launch does not end on a long item
// started late (longest-first list scheduling).  One workgroup per cloud: 64 size classes
// of 128 elements, counted and placed with LDS atomics (the order inside a class is free:
// items are disjoint segments, so the result does not depend on it).
constexpr int IS_ORD_CLASSES = 64;
__device__ __forceinline__ uint32_t item_len(const IsBufs& W, int R, uint32_t nsort, uint32_t nfin, uint32_t i) {
  if (i < nfin) {
    const Child c = child_of(W, R, nsort, i);
    return c.l > c.f ? c.l - c.f : 0u;
  }
  const IsOwn o = W.own[i - nfin];
  return o.l > o.f ? o.l - o.f : 0u;
}
__global__ void __launch_bounds__(1024) k_is_order(B4<IsBufs> W2, int R) {
  KT();
  const IsBufs W = W2[blockIdx.y];
  const uint32_t nsort = W.ctl[0];
  if (nsort == 0) return;
  const uint32_t nfin = nchildren(W, R), n = nfin + (R ? W.rounds[R - 1].nown : 0u);
  __shared__ uint32_t cnt[IS_ORD_CLASSES];
  if (threadIdx.x < IS_ORD_CLASSES) cnt[threadIdx.x] = 0u;
  __syncthreads();
  auto slot = [&](uint32_t i) {  // descending: the longest class first
    return (uint32_t)IS_ORD_CLASSES - 1u - min(item_len(W, R, nsort, nfin, i) >> 7, (uint32_t)IS_ORD_CLASSES - 1u);
  };
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&cnt[slot(i)], 1u);
  __syncthreads();
  if (threadIdx.x < 64) {  // exclusive scan of the 64 class counts (one wave)
    const uint32_t v = cnt[threadIdx.x];
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if ((int)threadIdx.x >= o) x += y;
    }
    cnt[threadIdx.x] = x - v;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) W.ord[atomicAdd(&cnt[slot(i)], 1u)] = i;
}

// One workgroup per remaining segment, dequeued from ctl[1]: in W.ord's order (the longest
// first) when `ordered`, else the final children of the last round (which may exceed
// IS_LCAP), then the owned list.
#ifndef IS_BLOCK_WPE
#define IS_BLOCK_WPE 1
#endif
__global__ void __launch_bounds__(IS_OT) __attribute__((amdgpu_waves_per_eu(IS_BLOCK_WPE))) k_is_block(B4<uint32_t*> K02, B4<uint32_t*> V02, B4<uint32_t*> K12,
                                                    B4<uint32_t*> V12, B4<IsBufs> W2, int R, int ordered) {
  KT();
  __shared__ BlockLds S;
  __shared__ uint32_t s_idx;
  const int e = blockIdx.y;
  const IsBufs W = W2[e];
  const uint32_t nsort = W.ctl[0];
  if (blockIdx.x == 0 && e == 0 && threadIdx.x == 0) is_inject(W, IS_FAULT_BLOCK | IS_FAULT_POP);
  if (nsort == 0) return;
  if (threadIdx.x == 0) {
    S.stat = W.ctl;
    S.err = W.err;
    S.son = IS_STATS && W.stats;
  }
  const uint32_t nfin = nchildren(W, R);
  const uint32_t nown = R ? W.rounds[R - 1].nown : 0u;
  const bool shard_on = W.shard_n > 1 && R > (int)W.shard_r0;
  const uint32_t shard_lo = shard_on ? W.bounds[W.shard_rank] : 0u, shard_hi = shard_on ? W.bounds[W.shard_rank + 1] : 0u;
  if (shard_on && blockIdx.x == 0 && threadIdx.x == 0) {  // (debug counters: this rank's range)
    W.ctl[28] = shard_lo;
    W.ctl[29] = shard_hi;
  }
  uint32_t* const K0 = K02[e];
  uint32_t* const V0 = V02[e];
  uint32_t* const K1 = K12[e];
  uint32_t* const V1 = V12[e];
  uint32_t units = 0;  // elements this workgroup sorted in LDS (the block probe's unit count)
  uint32_t xunits = 0;  // ... of which it finished itself (sorted points written: ctl[21])
  for (;;) {
    if (threadIdx.x == 0) {
      // look before taking: once the list is drained, leave without another atomic
      const uint32_t seen = __hip_atomic_load(&W.ctl[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const uint32_t q = seen >= nfin + nown ? seen : atomicAdd(&W.ctl[1], 1u);
      s_idx = q < nfin + nown ? (ordered ? W.ord[q] : q) : IS_NONE;
    }
    __syncthreads();
    const uint32_t idx = s_idx;
    __syncthreads();
    if (idx >= nfin + nown) break;
    uint32_t f, l, buf;
    int d;
    if (idx < nfin) {
      const Child c = child_of(W, R, nsort, idx);
      f = c.f;
      l = c.l;
      d = c.d;
      buf = (uint32_t)(R & 1);
    } else {
      const IsOwn o = W.own[idx - nfin];
      f = o.f;
      l = o.l;
      d = o.depth;
      buf = o.buf;
      // row D: the replicated rounds' owned segments belong to the rank whose range
      // holds their start (the later rounds list only this rank's)
      if (shard_on && (f < shard_lo || f >= shard_hi)) continue;
    }
    if (l <= f) continue;
    const unsigned long long t_item = W.trace ? wall_clock64() : 0ull;
    uint32_t* K = buf ? K1 : K0;  // selects: a dynamically indexed local array lives in scratch
    uint32_t* V = buf ? V1 : V0;
    if (threadIdx.x == 0) {
      S.gstk[0] = make_uint4(f, l, (uint32_t)d, 0u);
      S.gsp = 1;
    }
    __syncthreads();
    for (uint32_t guard = 0;; ++guard) {
      const uint32_t sp = S.gsp;
      __syncthreads();
      if (sp == 0) break;
      if (guard > 4 * (l - f) || sp >= IS_STACK / 2 - 2) {  // cannot happen: every step shrinks a segment
        if (threadIdx.x == 0) is_fault(W.ctl, W.err, IS_FAULT_BLOCK);
        break;
      }
      const uint4 it = S.gstk[sp - 1];
      const uint32_t gf = it.x, gl = it.y, len = gl - gf;
      const int gd = (int)it.z;
      const uint32_t gfree = it.w;  // 1: distinct keys, any exact sort (global_partition's free pivots)
      __syncthreads();
      if (threadIdx.x == 0) S.gsp = sp - 1;
      __syncthreads();
      if (len <= IS_LCAP) {
        if (S.son && threadIdx.x == 0) atomicAdd(&W.ctl[4], 1u);
        units += len;
        // (free: std::sort's depth bounds the LDS stacks; its depth limit there is the
        // parallel rank sort, exact for distinct keys)
        lds_block(S, W, K, V, K0, V0, gf, len, gfree ? depth0(len) : gd);
        if (W.xyzs) xunits += len - S.units;  // (S.units: its elements handed to wave tasks)
      } else if (gd == 0 && distinct_keys(S, K + gf, (buf ? K0 : K1) + gf, (buf ? V0 : V1) + gf, len)) {
        // depth exhausted, distinct keys: the order is unique; go on with free pivots
        if (threadIdx.x == 0) {
          atomicOr(&W.ctl[2], 4u);  // (other workgroups atomicOr fault bits into the same word)
          if (S.son) atomicAdd(&W.ctl[9], 1u);
          S.gstk[S.gsp++] = make_uint4(gf, gl, 60u, 1u);
        }
        __syncthreads();
      } else if (gd == 0) {  // depth exhausted, a repeated key: heap sort in place (slow; adversarial only)
        if (threadIdx.x == 0) {
          heap_sort(K + gf, V + gf, (int64_t)len);
          atomicOr(&W.ctl[2], 2u);
          if (S.son) atomicAdd(&W.ctl[7], 1u);
        }
        hand_off_fence();
        __syncthreads();
        if (buf != 0)
          for (uint32_t q = threadIdx.x; q < len; q += IS_OT) {
            K0[gf + q] = K[gf + q];
            V0[gf + q] = V[gf + q];
          }
        if (W.xyzs) {
          for (uint32_t q = threadIdx.x; q < len; q += IS_OT) put_xyz(W, W.vgp->src, gf + q, V[gf + q]);
          xunits += len;
        }
        __syncthreads();
      } else {
        if (S.son && threadIdx.x == 0) atomicAdd(&W.ctl[3], 1u);
        const uint32_t c = global_partition(S, K, V, buf ? K0 : K1, buf ? V0 : V1, gf, gl, gfree);
        if (threadIdx.x == 0) {
          atomicOr(&W.ctl[2], 1u);
          uint32_t s = S.gsp;
          const uint32_t cd = gfree ? 60u : (uint32_t)(gd - 1);  // (free: depth is irrelevant)
          // the larger child below the smaller (the segments are disjoint, so the order
          // is free): the smaller is done first and the stack stays O(log n) deep
          const uint4 lo = make_uint4(gf, c, cd, gfree), hi = make_uint4(c, gl, cd, gfree);
          const bool lo_small = c - gf <= gl - c;
          S.gstk[s++] = lo_small ? hi : lo;
          S.gstk[s++] = lo_small ? lo : hi;
          S.gsp = s;
        }
        hand_off_fence();
        __syncthreads();
      }
    }
    if (W.trace && threadIdx.x == 0) {  // dev: item timestamps (fccf_debug_sort_keys, FCCF_IS_TRACE_OUT)
      const uint32_t slot = atomicAdd(&W.ctl[24], 1u);
      if (slot < W.taskmax) {
        unsigned long long* r = W.trace + 4 * (size_t)slot;
        r[0] = t_item;
        r[1] = wall_clock64();
        r[2] = l - f;
        r[3] = blockIdx.x;
      }
    }
  }
  if (threadIdx.x == 0 && units) atomicAdd(&W.ctl[20], units);
  if (threadIdx.x == 0 && xunits) atomicAdd(&W.ctl[21], xunits);
}

// The wave tasks' slots (the large list from the front, the small list from the end of
// W.tasks) in descending size (64 classes of 8 elements), for k_is_wave's longest-first
// dequeue.  One workgroup per cloud; the order inside a class is free (disjoint subtrees).
__global__ void __launch_bounds__(1024) k_is_torder(B4<IsBufs> W2) {
  KT();
  const IsBufs W = W2[blockIdx.y];
  const uint32_t nbig = W.ctl[16], n = nbig + W.ctl[18];
  __shared__ uint32_t cnt[64];
  if (threadIdx.x < 64) cnt[threadIdx.x] = 0u;
  __syncthreads();
  auto slot_of = [&](uint32_t i) { return i < nbig ? i : W.taskmax - 1u - (i - nbig); };
  auto cls = [&](uint32_t i) { return 63u - min(W.tasks[slot_of(i)].y >> 3, 63u); };
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&cnt[cls(i)], 1u);
  __syncthreads();
  if (threadIdx.x < 64) {
    const uint32_t v = cnt[threadIdx.x];
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(x, o, 64);
      if ((int)threadIdx.x >= o) x += y;
    }
    cnt[threadIdx.x] = x - v;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) W.tord[atomicAdd(&cnt[cls(i)], 1u)] = slot_of(i);
}

// Every wave takes its share of the wave tasks: the subtree in its LDS slice,
// finished and stably leaf-sorted, written back in place in buffer 0.
#ifndef IS_WAVE_DYN
#define IS_WAVE_DYN 1
#endif
#ifndef IS_WAVE_LB
#define IS_WAVE_LB 4  // 4 waves per SIMD: 128 VGPRs, no spill (1.19 vs 1.21 ms pipelined, profiles/r02j)
#endif
__global__ void __launch_bounds__(IS_WT, IS_WAVE_LB) k_is_wave(B4<uint32_t*> K02, B4<uint32_t*> V02, B4<IsBufs> W2) {
  KT();
  __shared__ WaveLds WL[IS_WT / 64];
  const int e = blockIdx.y;
  const IsBufs W = W2[e];
  const uint32_t lane = lane_id(), w = threadIdx.x >> 6;
  WaveLds& S = WL[w];
  if (lane == 0) {
    S.stat = W.ctl;
    S.err = W.err;
    S.son = IS_STATS && W.stats;
    for (int i = 0; i < 4; ++i) S.lstat[i] = 0;
  }
  if (blockIdx.x == 0 && e == 0 && threadIdx.x == 0) is_inject(W, IS_FAULT_WAVE);
  wsync();
#if IS_WAVE_DYN
  // Longest first (W.tord, k_is_torder): wave g of the grid (which is sized to be
  // resident at once) takes task g, then the next one from a per-cloud counter when it
  // has finished one (greedy list scheduling; the static first task keeps the grid's
  // start free of contention on the counter).
  const uint32_t nbig = W.ctl[16], ntasks = nbig + W.ctl[18];
  const float* __restrict__ xsrc = W.xyzs ? W.vgp->src : nullptr;
  uint32_t* __restrict__ K = K02[e];
  uint32_t* __restrict__ V = V02[e];
  const uint32_t nw = gridDim.x * (IS_WT / 64);
  for (uint32_t idx = blockIdx.x * (IS_WT / 64) + w; idx < ntasks;) {
    const uint4 tk = W.tasks[W.tord[idx]];
#else
  // Static assignment, no queue: wave g of the grid takes tasks g, g + NW, g + 2 NW ...
  // of the list, which holds the large tasks first, so the largest ones are spread
  // one per wave (a dynamic dequeue from one counter serialises on that counter:
  // ~18 ns per atomic, which at thousands of tasks was the kernel's whole time).
  const uint32_t nbig = W.ctl[16], ntasks = nbig + W.ctl[18];
  const float* __restrict__ xsrc = W.xyzs ? W.vgp->src : nullptr;
  uint32_t* __restrict__ K = K02[e];
  uint32_t* __restrict__ V = V02[e];
  const uint32_t nw = gridDim.x * (IS_WT / 64);
  for (uint32_t idx = blockIdx.x * (IS_WT / 64) + w; idx < ntasks; idx += nw) {
    const uint4 tk = W.tasks[idx < nbig ? idx : W.taskmax - 1u - (idx - nbig)];
#endif
    const uint32_t f = __builtin_amdgcn_readfirstlane(tk.x), n = __builtin_amdgcn_readfirstlane(tk.y);
    const int d = (int)__builtin_amdgcn_readfirstlane(tk.z);
#pragma unroll
    for (int c = 0; c < IS_WC; ++c) {
      const uint32_t q = c * 64 + lane;
      if (q < n) {
        S.k[q] = K[f + q];
        S.v[q] = V[f + q];
      }
    }
    if (lane < IS_THRESHOLD) S.k[n + lane] = IS_NONE;  // (leaf_rank's window past the task)
    if (lane < IS_WCAP / 32) S.heads[lane] = 0;
    wsync();
    const unsigned long long t_task = W.trace ? wall_clock64() : 0ull;
    if (n > 64) {
      // (chunk counts 2, 4, 6, 8: 6 for 257-384 elements saved ~2 %; every count from 2 to
      // 8 made the kernel's code 164 KB and it slower, profiles/r06l)
      if (n <= 128) wave_task_level<2>(S, K, V, f, n, d, W, xsrc);
      else if (n <= 256) wave_task_level<4>(S, K, V, f, n, d, W, xsrc);
      else if (n <= 384) wave_task_level<6>(S, K, V, f, n, d, W, xsrc);
      else wave_task_level<IS_WC>(S, K, V, f, n, d, W, xsrc);
      if (S.son && lane == 0) atomicAdd(&S.lstat[2], 1u);
    } else
    {
    wave_sort(S, wpack(0u, n, d), S.stk, S.xch);
    wsync();
    // (n <= 64: a task of more than 16 positions comes back from wave_sort sorted, every
    // position its own leaf (wave_sort_regs or the depth-limit path); one of at most 16
    // is one leaf, ranked here)
    if (lane < n) {
      const uint32_t key = S.k[lane], val = S.v[lane];
      const uint32_t dst = f + (n <= IS_THRESHOLD ? min(leaf_rank(S.k, 0u, lane, key), n - 1u) : lane);
      K[dst] = key;
      V[dst] = val;
      if (xsrc) put_xyz(W, xsrc, dst, val);
    }
    }
    wsync();
    if (W.trace && lane == 0) {
      const uint32_t slot = atomicAdd(&W.ctl[25], 1u);
      if (slot < W.taskmax) {
        unsigned long long* r = W.trace + 4 * ((size_t)W.taskmax + slot);
        r[0] = t_task;
        r[1] = wall_clock64();
        r[2] = n;
        r[3] = blockIdx.x * (IS_WT / 64) + w;
      }
    }
#if IS_WAVE_DYN
    uint32_t nxt = 0;
    if (lane == 0) nxt = nw + atomicAdd(&W.ctl[26], 1u);
    idx = __builtin_amdgcn_readfirstlane(nxt);
#endif
  }
  if (S.son && lane == 0) {
    atomicAdd(&W.ctl[6], S.lstat[2]);
    atomicAdd(&W.ctl[12], S.lstat[0]);
  }
}


}  // namespace

#ifdef IS_KERNEL_VARIANT
// introsort_b2.hip: this file's kernels again with 256-thread block-kernel workgroups over
// 4,096-element segments, three per CU; only the block kernel's launch is taken from this form
void introsort_block_b2(B4<uint32_t*> k0, B4<uint32_t*> v0, B4<uint32_t*> k1, B4<uint32_t*> v1, B4<IsBufs> b, int R,
                        hipStream_t st, int nbatch) {
  ProbeBytes pb;  // algorithmic bytes: see introsort_u32 (block_probe_bytes)
  for (int e = 0; e < nbatch; ++e) pb.add(b[e].ctl + 20, 16.0).add(b[e].ctl + 21, 24.0);
  const int blocks = std::max(1, IS_B2_PER_CU * IS_OWN_BLOCKS / nbatch);
#ifndef IS_B2_ORDERED
#define IS_B2_ORDERED 0  // (ordered, its launch in a pipelined batch read 388-405 against 342-344 us, r06x)
#endif
  if (IS_B2_ORDERED) k_is_order<<<dim3(1, nbatch), 1024, 0, st>>>(b, R);
  FCCF_LAUNCH("k_is_block", (pb), k_is_block, dim3(blocks, nbatch), IS_OT, 0, st, k0, v0, k1, v1, b, R, IS_B2_ORDERED);
}
#else
// the rounds split segments longer than this (8192 / 6144 / 2048 with 13-17 rounds
// measured slower)
uint32_t introsort_tier() { return 4096u; }
// Workgroups per cloud of the small-cloud count kernel, which takes its tiles in a
// grid-stride loop (the plan derived once per workgroup): 1024 over the batch, at most a
// cloud's tile capacity (profiles/r06o).
#ifndef IS_COUNT_GRID
#define IS_COUNT_GRID 1024
#endif
static uint32_t is_round_grid(uint32_t maxtiles, int nbatch, uint32_t total) {
  return std::max(1u, std::min(maxtiles, total / (uint32_t)std::max(1, nbatch)));
}

uint32_t introsort_segmax(uint32_t cap) { return cap / introsort_tier() + 2; }
uint32_t introsort_maxtiles(uint32_t cap) { return cap / IS_TILE + introsort_segmax(cap) + 1; }
uint32_t introsort_maxtiles_l(uint32_t cap) { return cap / IS_TILE_L + introsort_segmax(cap) + 1; }

#ifndef IS_RPLUS
#define IS_RPLUS 7
#endif
int introsort_rounds(uint32_t cap) {
  int r = 0;
  const uint32_t tier = introsort_tier();
  if (cap > tier) {
    // ceil(log2(cap / tier)) balanced levels, plus the deeper tail of unbalanced
    // splits (structured clouds: ~15 rounds at 1M points before all segments are <= 4096)
    while ((uint64_t)tier << r < cap) ++r;
    r += IS_RPLUS;
  }
  return r > IS_RMAX ? IS_RMAX : r;
}

size_t introsort_bytes(uint32_t cap) {
  const size_t sm = introsort_segmax(cap), mt = introsort_maxtiles(cap);
  const size_t own = 2 * sm * (IS_RMAX + 1) + 4;
  return 256 + 256 + 16 * ((size_t)cap / 16 + 64) + 12 * mt + sizeof(IsTile) * mt + 256 + 2 * 2 * ((size_t)cap + 64) + sizeof(IsRound) * IS_RMAX +
         (sizeof(IsSeg) + 4) * sm * IS_RMAX + sizeof(IsOwn) * own + 16 * sm + 8 * mt + 4 * sm + 8 * (size_t)IS_RMAX * IS_DONE_WORDS + 4 * (IS_SHARD_MAX + 1) + 4 * (own + 2 * sm + 4) + 4 * ((size_t)cap / 16 + 64) + 15 * 256;
}

IsBufs introsort_carve(void* base, uint32_t cap) {
  char* p = (char*)base;
  auto take = [&](size_t b) {
    char* r = p;
    p += (b + 255) & ~size_t(255);
    return (void*)r;
  };
  IsBufs b;
  b.segmax = introsort_segmax(cap);
  b.maxtiles = introsort_maxtiles(cap);
  b.ownmax = 2 * b.segmax * (IS_RMAX + 1) + 4;
  b.ctl = (uint32_t*)take(256);
  b.cnt = (uint32_t*)take(8 * (size_t)b.maxtiles);
  b.tseg = (uint32_t*)take(4 * (size_t)b.maxtiles);
  b.tdesc = (IsTile*)take(sizeof(IsTile) * (size_t)b.maxtiles);
  b.gel = (uint16_t*)take(2 * ((size_t)cap + 64));
  b.lel = (uint16_t*)take(2 * ((size_t)cap + 64));
  b.rounds = (IsRound*)take(sizeof(IsRound) * IS_RMAX);
  b.segs = (IsSeg*)take(sizeof(IsSeg) * (size_t)b.segmax * IS_RMAX);
  b.cuts = (uint32_t*)take(4 * (size_t)b.segmax * IS_RMAX);
  b.own = (IsOwn*)take(sizeof(IsOwn) * (size_t)b.ownmax);
  b.taskmax = cap / 16 + 64;
  b.tasks = (uint4*)take(sizeof(uint4) * (size_t)b.taskmax);
  b.tord = (uint32_t*)take(4 * (size_t)b.taskmax);
  b.ptab = (uint4*)take(sizeof(uint4) * (size_t)b.segmax);
  b.pre = (uint32_t*)take(8 * (size_t)b.maxtiles);
  b.letot = (uint32_t*)take(4 * (size_t)b.segmax);
  b.ord = (uint32_t*)take(4 * ((size_t)b.ownmax + 2 * (size_t)b.segmax + 4));
  b.done = (uint32_t*)take(4 * 2 * (size_t)IS_RMAX * IS_DONE_WORDS);
  b.bounds = (uint32_t*)take(4 * (IS_SHARD_MAX + 1));
  b.shard_n = 1;
  b.shard_rank = 0;
  b.shard_r0 = 0;
  b.shard_group = nullptr;
  b.trace = nullptr;
  b.tier = introsort_tier();
  b.stats = 0;
  b.err = nullptr;
  b.inject = nullptr;
  b.vgp = nullptr;
  b.xyzs = nullptr;
  return b;
}

void introsort_u32(B4<uint32_t*> k0, B4<uint32_t*> v0, B4<uint32_t*> k1, B4<uint32_t*> v1, B4<const uint32_t*> d_n,
                   B4<const VGParams*> P, uint32_t cap, B4<IsBufs> b, hipStream_t st, int nbatch, bool exact_gate) {
  const int R = exact_gate ? 0 : introsort_rounds(cap);
  static const bool trace = std::getenv("FCCF_IS_TRACE") != nullptr;  // dev: sync + log after each launch
  auto step = [&](const char* what, int r) {
    if (!trace) return;
    const hipError_t e = hipStreamSynchronize(st);
    std::fprintf(stderr, "introsort %s r=%d: %s\n", what, r, hipGetErrorString(e));
  };
  k_is_prep<<<dim3(1, nbatch), 1024, 0, st>>>(k0, v0, d_n, P, b, exact_gate ? 1 : 0);
  step("prep", 0);
  const uint32_t segmax = introsort_segmax(cap), maxtiles = introsort_maxtiles(cap),
                 maxtiles_l = introsort_maxtiles_l(cap);
  // the round plan's form: once per round (large clouds) or per workgroup (small ones);
  // FCCF_IS_PLAN=large|small overrides (tests run the sort cases in both)
  const char* pm = std::getenv("FCCF_IS_PLAN");
  const bool large = b[0].shard_n > 1 || (pm && pm[0] == 'l' ? true : (pm && pm[0] == 's' ? false : cap >= IS_LARGE_MIN));
  // algorithmic bytes of a launch, summed over its clouds (probe.h)
  auto pb_round = [&](int r, double per) {
    ProbeBytes x;
    for (int e = 0; e < nbatch; ++e) x.add(&b[e].rounds[r].pad, per);
    return x;
  };
  auto pb_block = [&] {
    ProbeBytes x;
    for (int e = 0; e < nbatch; ++e) x.add(b[e].ctl + 20, 16.0).add(b[e].ctl + 21, 24.0);
    return x;
  };
  auto pb_wave = [&] {
    ProbeBytes x;
    for (int e = 0; e < nbatch; ++e) x.add(b[e].ctl + 19, b[e].xyzs ? 40.0 : 16.0);
    return x;
  };
  for (int r = 0; r < R; ++r) {
    const B4<uint32_t*> ki = (r & 1) ? k1 : k0, vi = (r & 1) ? v1 : v0;
    const B4<uint32_t*> ko = (r & 1) ? k0 : k1, vo = (r & 1) ? v0 : v1;
    if (large) {
      // algorithmic bytes: the key read, a 2-byte list entry written (x2: >= and <= lists share a unit)
      FCCF_LAUNCH("k_is_count_plan",
                  (pb_round(r, 8.0)),
                  k_is_count_plan, dim3(maxtiles_l, nbatch), IS_TT, 8 * (size_t)segmax, st, B4<const uint32_t*>(ki),
                  B4<const uint32_t*>(vi), b, r);
      step("count", r);
      // algorithmic bytes: key + value read and written, plus a 2-byte list entry
      FCCF_LAUNCH("k_is_scatter", (pb_round(r, 18.0)), k_is_scatter, dim3(maxtiles_l, nbatch), IS_TT, 0, st,
                  B4<const uint32_t*>(ki), B4<const uint32_t*>(vi), ko, vo, b, r, R);
    } else {
      FCCF_LAUNCH("k_is_count_plan",
                  (pb_round(r, 8.0)),
                  k_is_count_plan_s, dim3(is_round_grid(maxtiles, nbatch, IS_COUNT_GRID), nbatch), IS_TT,
                  16 * (size_t)segmax, st, B4<const uint32_t*>(ki), B4<const uint32_t*>(vi), b, r);
      step("count", r);
      FCCF_LAUNCH("k_is_scatter", (pb_round(r, 18.0)), k_is_scatter_s, dim3(maxtiles, nbatch), IS_TT,
                  8 * (size_t)maxtiles, st, B4<const uint32_t*>(ki), B4<const uint32_t*>(vi), ko, vo, b, r);
    }
    step("scatter", r);
  }
  // Algorithmic bytes of the finish kernels: each element's key and value read once and
  // written once (16 B), and for the elements a kernel finishes while the sort writes
  // sorted points (VoxelGrid's first pass), the point gathered from its original
  // position and written at its final one (12 + 12 B): the wave kernel finishes every
  // element of its tasks (ctl[19]), the block kernel the leaves it settles itself
  // (ctl[21], of its ctl[20] LDS elements).
  // k_is_block: IS_OWN_BLOCKS workgroups (one per CU) split over the clouds, so both
  // clouds' items run at once and 8 CUs stay free for the small kernels of other
  // streams (matching, fine verification); profiles/r03r
  const int own_blocks = std::max(1, IS_OWN_BLOCKS / nbatch);
  // Stage groups of three to five pairs (six to ten clouds per launch): the block
  // kernel's second form, 256-thread workgroups at three per CU (introsort_b2.hip), whose
  // items interleave their partition chains on each CU: pipelined 0.548 against 0.593 ms
  // per registration (profiles/r06u; the earlier 512-thread form read 0.650-0.654 against
  // 0.658-0.665 for the 1024-thread form, r05ap).  Single registrations (two clouds: few
  // items per workgroup) keep the 1024-thread form: main VoxelGrid 0.733 against 0.843 ms
  // with the second form (r06u).
  // FCCF_IS_BLOCK_B2=0 / 1: never / always (dev, tests)
  const char* b2e = std::getenv("FCCF_IS_BLOCK_B2");
  const bool b2 = b2e ? b2e[0] == '1' : nbatch >= 6;
  if (b2) {
    introsort_block_b2(k0, v0, k1, v1, b, R, st, nbatch);
  } else {
    // One 1024-thread workgroup per CU takes 3-4 items per launch: the longest first
    // (k_is_order), so that none starts late: main VoxelGrid 0.727-0.731 -> 0.703-0.707
    // ms.  The second form keeps the list order: its launch in a pipelined batch read
    // 388-405 us ordered against 342-344 us (profiles/r06x).
    k_is_order<<<dim3(1, nbatch), 1024, 0, st>>>(b, R);
    step("order", R);
    FCCF_LAUNCH("k_is_block", (pb_block()), k_is_block,
                dim3(own_blocks, nbatch), IS_OT, 0, st, k0, v0, k1, v1, b, R, 1);
  }
  step("block", R);
  // (other wave grids at ten clouds per launch: no gain, profiles/r05au/ab_wave_grid_width10.txt)
#if IS_WAVE_DYN
  // (the tasks longest first; a grid that is resident at once: four workgroups per CU)
  k_is_torder<<<dim3(1, nbatch), 1024, 0, st>>>(b);
  step("torder", R);
  const int wave_blocks = std::max(1, IS_WAVE_RESIDENT / nbatch);
#else
  const int wave_blocks = IS_WAVE_BLOCKS;
#endif
  FCCF_LAUNCH("k_is_wave", (pb_wave()), k_is_wave,
              dim3(wave_blocks, nbatch), IS_WT, 0, st, k0, v0, b);
  step("wave", R);
}

#endif  // IS_KERNEL_VARIANT

}  // namespace fccf

#ifdef IS_PHASES
// Development export (variant builds only): the instrumented kernel's phase sums since
// the last call (cycles [0..15], counts [16..31]), then reset.
#ifdef IS_KERNEL_VARIANT
extern "C" int fccf_debug_is_phases_b2(unsigned long long out[32]) {  // (the second form's own counters)
#else
extern "C" int fccf_debug_is_phases(unsigned long long out[32]) {
#endif
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(fccf::g_is_ph), 32 * sizeof(unsigned long long)) != hipSuccess) return -2;
  unsigned long long z[32] = {};
  if (hipMemcpyToSymbol(HIP_SYMBOL(fccf::g_is_ph), z, sizeof z) != hipSuccess) return -2;
  return 0;
}
#endif
