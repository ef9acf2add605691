// kernels.h — launchers of the FCCF HIP kernels (one .hip file per stage).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "devprim.h"
#include "fccf_math.h"

namespace fccf {

// ------------------------------------------------ K1: VoxelGrid (FCCF.cpp:1668-1678, :1377-1387)
struct VGParams {
  float mn[3], mx[3];
  float inv;
  uint32_t nfinite;
  int32_t min_b[3];
  int32_t div_b[3];
  int64_t mul1, mul2;
  uint32_t overflow;  // int32 index guard tripped: output = input
  uint32_t nbits;     // radix bits (0 when overflow / empty, or when the keys are already sorted)
  uint32_t unsorted;  // presorted check: some key is not strictly above its predecessor
  uint32_t chk_done;  // presorted check: blocks finished
  uint32_t nonfinite; // some output point is not finite (set by k_vg_centroid when it writes a copy)
  const float* src;   // the pass's input points (set by k_vg_bbox, read by the later kernels)
  uint64_t t_main;    // s_memrealtime at the start of main's pass (k_vg_bbox<0>): stage spans
  uint64_t t_driver;  // ... and of the driver's remove-NaN + second pass (k_finite_fix)
  uint32_t redo;      // VG_OPTIMISTIC pass not in leaf order (output empty): cleared by k_vg_bbox
  uint32_t sort_err;  // K1 sort invariant flags of this cloud's passes (IS_FAULT_*), cleared by main's pass
                      // entry (k_vg_bbox<0>); copied to the cloud mailbox, where the host turns them into
                      // FCCF_E_INTERNAL
};

constexpr int VG_BBOX_BLOCKS = 512;
constexpr int VG_KEY_BLOCKS = 512;

// K1's sort in libstdc++ std::sort order (introsort.hip): workspace of one cloud.
constexpr int IS_RMAX = 24;          // most partition rounds before the owner kernel
constexpr int IS_OWN_BLOCKS = 248;   // block-kernel workgroups of a launch, split over its clouds (one per CU)
constexpr int IS_WAVE_BLOCKS = 512;  // wave-kernel workgroups per cloud (4 waves each; static task assignment)
constexpr int IS_WAVE_RESIDENT = 1024;  // wave-kernel workgroups of a launch (dynamic dequeue): 4 per CU
constexpr int IS_SHARD_MAX = 64;     // most ranks of a sharded sort (row D)
struct IsRound {
  uint32_t nseg, ntiles, nown, pad;  // large segments, their tiles, owned entries so far
};
struct IsSeg {
  uint32_t f, l;
  int32_t depth;
  uint32_t tile0;
  uint32_t m, P, kf, vf, vm;  // median position, pivot key, the first element, the median's value
};
struct IsTile {  // a round tile's segment (j = IS_NONE past the round's tiles): one load for the scatter
  uint32_t j;
  IsSeg s;
};
struct IsOwn {
  uint32_t f, l;
  int32_t depth;
  uint32_t buf;  // which of the two key/value buffers holds the segment
};
struct IsBufs {
  uint32_t* ctl;        // [0] sort length, [1] block dequeue head, [2] slow paths taken (1 global partition,
                        // 2 heap), [3..15] counters, [16] large wave tasks, [18] small wave tasks
                        // (stored from the end), [19]/[20] wave/block probe unit counts
  uint32_t* cnt;        // per round tile: (#>= pivot, #<= pivot), written with atomics
  uint32_t* tseg;       // per round tile: its segment (0xFFFFFFFF past the round's tiles; plan_round)
  IsTile* tdesc;        // per round tile: its segment and the segment's record (the scatter's input)
  uint16_t *gel, *lel;  // tile-local positions of the >= / <= elements, indexed from the tile start
  IsRound* rounds;      // IS_RMAX
  IsSeg* segs;          // IS_RMAX x segmax
  uint32_t* cuts;       // IS_RMAX x segmax
  IsOwn* own;           // ownmax
  uint4* tasks;         // wave tasks {f, n, depth, -} (count in ctl[16])
  uint32_t* tord;       // the wave tasks' slots in descending size (k_is_torder), dequeued by k_is_wave
  uint4* ptab;          // the current round's plan: per segment {f, l, depth, first tile} (plan_round)
  uint32_t* pre;        // per round tile: exclusive (>=, <=) prefix within its segment (k_is_count_plan's last workgroup)
  uint32_t* letot;      // per segment of the round: its <= count
  uint32_t* ord;        // the block kernel's items (final children, then owned) in descending size (k_is_order)
  uint32_t* done;       // per round, count and scatter: sharded completion counters (last-workgroup hand-offs)
  // Row D sharding (group.cpp): from round shard_r0 on, this rank partitions and finishes
  // only the segments starting in its range [bounds[shard_rank], bounds[shard_rank + 1]);
  // plan_round of round shard_r0 writes the shard_n + 1 bounds.  shard_n = 1: off.
  uint32_t shard_n, shard_rank, shard_r0;
  uint32_t* bounds;     // IS_SHARD_MAX + 1
  void* shard_group;    // host only: the Group whose ranks gather the sorted slices
  unsigned long long* trace;  // dev (null = off): per block item / wave task {start, end, size, who},
                              // block records from 0 (count in ctl[24]), wave records from taskmax (ctl[25])
  uint32_t segmax, maxtiles, ownmax, taskmax;
  uint32_t tier;        // rounds split segments longer than this (<= the owner's LDS capacity)
  uint32_t stats;       // path counters in ctl[3..15] (debug sorts; each costs a global atomic)
  uint32_t* err;        // VGParams::sort_err of the pass's cloud (null: ctl[2] only)
  const uint32_t* inject;  // test hook (fccf_debug_inject_sort_fault): IS_FAULT_* bits raised once per
                           // sort by a designated thread at the matching site (null: off)
  // Sorted points (VoxelGrid's first pass, unsharded): every final (key, value) write also
  // writes the point vgp->src[value] to xyzs at the same position, so the centroid kernel
  // reads each leaf's members contiguously instead of gathering them (null: off)
  const struct VGParams* vgp;
  float* xyzs;
};
// Invariant flags of the sort (IsBufs::ctl[2], VGParams::sort_err).  Each marks a
// state the algorithm cannot reach; any of them makes fccf_register* fail with
// FCCF_E_INTERNAL instead of returning a transform from a wrong order.
constexpr uint32_t IS_FAULT_SCATTER = 0x100u;  // a round's scatter destination outside its segment
constexpr uint32_t IS_FAULT_BLOCK = 0x200u;    // a block item's stack or step guard exceeded
constexpr uint32_t IS_FAULT_WAVE = 0x400u;     // a wave task's stack or step guard exceeded
constexpr uint32_t IS_FAULT_POP = 0x1000u;     // a block item's partition stack overran
constexpr uint32_t IS_FAULT_MASK = IS_FAULT_SCATTER | IS_FAULT_BLOCK | IS_FAULT_WAVE | IS_FAULT_POP;
size_t introsort_bytes(uint32_t cap);
IsBufs introsort_carve(void* base, uint32_t cap);
int introsort_rounds(uint32_t cap);
// Sort (k0, v0)[0..n) -- keys with 0xFFFFFFFF for non-finite points, values the input
// positions -- exactly as std::sort orders PCL's index vector of the finite points;
// the result is left in (k0, v0) with the invalid keys after it.  (k1, v1) are the
// other buffer.  exact_gate: sort only if P->unsorted (the presorted second pass).
// k_is_block in its second form (introsort_b2.hip: 512-thread workgroups, two per CU)
void introsort_block_b2(B4<uint32_t*> k0, B4<uint32_t*> v0, B4<uint32_t*> k1, B4<uint32_t*> v1, B4<IsBufs> b, int R,
                        hipStream_t st, int nbatch);
void introsort_u32(B4<uint32_t*> k0, B4<uint32_t*> v0, B4<uint32_t*> k1, B4<uint32_t*> v1, B4<const uint32_t*> d_n,
                   B4<const VGParams*> P, uint32_t cap, B4<IsBufs> b, hipStream_t st, int nbatch, bool exact_gate);

struct VGBufs {
  uint32_t *k0, *v0, *k1, *v1;  // cap each
  uint32_t* starts;             // cap + 1
  float* part;                  // VG_BBOX_BLOCKS * 8
  VGParams* params;
  uint32_t* nseg;
  SortScratch ss;
  IsBufs is;
  float* xyzs;                  // 3 * cap: the first pass's points in sorted order (IsBufs::xyzs)
};

// xyz[0..*d_n) -> out[0..*d_m), PCL VoxelGrid<PointXYZ> semantics: the points of a
// leaf are accumulated in the order libstdc++ std::sort leaves them (introsort.hip).
// presorted: the input is expected to be in (nearly) ascending leaf order -- the
// driver's second pass over main's output (:1377-1387 after :1668-1678).  A check
// kernel then skips the sort when the keys are already strictly increasing (every
// leaf holds one point, so the order cannot matter); otherwise one workgroup per
// cloud runs the whole std::sort.
// nbatch = 2 runs both clouds (argument pairs, blockIdx.y = cloud) in the same launches.
// out_copy (optional): every output point is also written there, and
// VGParams::nonfinite is set when one is not finite (the driver's remove-NaN after
// the first pass, FCCF.cpp:1374-1375, is then an identity unless that flag is set).
// The arguments of a pass's entry kernel (k_vg_bbox), the only launch of the pass
// that takes the input points and their count: a cached graph replays the pass for
// other caller-owned inputs by rewriting this one node (CachedGraph::patch), so the
// inputs are read in place, never staged.  set_n: the count is n (by value) and the
// kernel stores it to d_n for the later kernels; otherwise it is read from d_n.
struct VGEntry {
  B4<const float*> xyz;
  B4<uint32_t*> d_n;
  B4<uint32_t> n;
  int set_n = 0;
  B4<float*> part;
  B4<VGParams*> P;
  void* args[6];
  void bind() {
    args[0] = &xyz; args[1] = &d_n; args[2] = &n; args[3] = &set_n; args[4] = &part; args[5] = &P;
  }
  // the arguments fixed by the workspace layout (all but the inputs xyz and n), as
  // CachedGraph's replay check reads them: {index in args, size}
  static constexpr int LAYOUT_N = 4;
  static constexpr int layout_idx[LAYOUT_N] = {1, 3, 4, 5};
  static constexpr size_t layout_size[LAYOUT_N] = {sizeof(B4<uint32_t*>), sizeof(int), sizeof(B4<float*>),
                                                   sizeof(B4<VGParams*>)};
};
const void* vg_entry_kernel();
// One VoxelGrid pass per batch entry.  n_in (optional): the counts by value (see
// VGEntry.set_n), stored to d_n; entry (optional): receives the entry kernel's arguments.
// presorted: VG_GENERAL; VG_PRESORTED (the driver's second pass over main's output:
// usually every leaf holds one point in order, else the device sorts it exactly);
// VG_OPTIMISTIC (the same without the sort and segmentation launches of the fallback:
// an input that is not in leaf order yields an empty output and sets VGParams::redo,
// and the caller redoes the pass with VG_PRESORTED).
enum { VG_GENERAL = 0, VG_PRESORTED = 1, VG_OPTIMISTIC = 2 };
constexpr uint32_t VG_REDO = 0x80000000u;       // CloudMail::fsc[k][1]: the optimistic pass must be redone
constexpr uint32_t VG_FORCE_REDO = 0x10000u;    // test hook bit (fccf_debug_inject_sort_fault)
constexpr uint32_t VG_FORCE_REDO_LATER = 0x40000u;  // the same for a stage group's later pairs only (clouds >= 2)
// CloudMail::fsc[k][1]: the cloud's face codes are wider than three 9-bit radix digits
// (a 1 m octree deeper than 8 levels): a cloud stage that launched three passes sorted
// the rest in the single-workgroup tail, and the ctx launches four from then on
constexpr uint32_t FACE_DEEP = 0x40000000u;
constexpr uint32_t IS_POISON_XYZS = 0x20000u;   // test hook bit: sorted points filled with NaN before each sort
void voxel_grid(B4<const float*> xyz, B4<uint32_t*> d_n, uint32_t cap, float leaf, B4<float*> out,
                B4<uint32_t*> d_m, B4<VGBufs> b, hipStream_t st, int presorted = VG_GENERAL, int nbatch = 1,
                B4<float*> out_copy = B4<float*>(nullptr), const uint32_t* n_in = nullptr,
                VGEntry* entry = nullptr);

// ------------------------------------------------ K2/K3: 1 m face voxels (FCCF.cpp:470-534)
struct VoxRec {  // one occupied octree leaf, Morton order
  float c[3];
  float n[3];   // oriented normal (planar) / raw eigenvector
  int32_t count;
  float curvature;
};

// ------------------------------------------------ K4: region growing (FCCF.cpp:536-648), grow.hip
constexpr uint32_t GROW_CAP = 3072;  // voxels per cloud held in LDS (larger clouds grow on the host)
struct GrowIn {
  const VoxRec* vox;  // planar voxel records of one cloud, Morton order
  uint32_t nv;        // <= GROW_CAP
};
struct GrowDev {      // per group (<= nv), creation (seed) order; plus the member lists
  float* gac;         // 3 per group: average centre
  float* gan;         // 3 per group: average normal
  float* gfps;        // face_point_size
  float* gsum;        // 7 per group: running sums s, sc[3], sn[3] after stage 1
  double* gna;        // norm3d(an)
  uint32_t *ghead, *gtail, *gnmem, *galloc;
  uint32_t* next;     // nv: next member of the same group (0xFFFFFFFF at a tail)
  uint32_t* ng;       // number of groups
};
struct GrowParams {
  AngleCut cut1, cut2;  // normal_vector_threshold1/2 as cosine cuts
  float l1, k1, l2, k2;
};
void grow_device(const GrowIn in[2], const GrowDev out[2], const GrowParams& P, hipStream_t st);

struct FaceBufs {
  uint64_t *c0, *c1, *c2;  // codes, cap each (c2: the sort's third buffer)
  uint32_t *v0, *v1, *v2;  // cap each
  uint32_t* starts;        // cap + 1
  float* aggr;             // octree-bounds aggregates, aggr_floats(cap) (see block_aggr)
  OctState* oct;
  float* centroid;         // 3 floats (the cloud centroid, exact_sum2 in pipeline.cpp)
  VoxRec* recs;            // cap (all leaves)
  uint32_t* flag_planar;   // cap
  uint32_t* resid_cnt;     // cap
  uint32_t* planar_off;    // cap
  uint32_t* resid_off;     // cap
  float* sp;               // points in leaf order, 3 * cap
  uint32_t* seg_of;        // leaf index of every sorted point, cap
  uint32_t* nleaf;         // scalars
  uint32_t* nbits;
  uint32_t* nplanar;
  uint32_t* nresid;
  uint64_t* t_faces;       // s_memrealtime at the start of the face stage (k_block_aggr)
  const VGParams* vgp;     // the cloud's VoxelGrid parameters (their stage stamps), or null
  SortScratch ss;
};

// Octree leaves (Morton order) of each cloud of the batch.  Batched clouds must be
// carved identically: every pointer of cloud 1 sits `stride` bytes after cloud 0's.
// fast_bits: 8 x the device-wide radix passes launched for the face codes (24: three
// <= 9-bit digits, octrees up to depth 8; 32: four, depth 10; deeper codes finish in the
// single-workgroup tail either way)
void face_voxels_prepare(B4<const float*> xyz, B4<const uint32_t*> d_n, uint32_t cap, double res, B4<FaceBufs> b,
                         hipStream_t st, int nbatch = 1, int fast_bits = 32);
// Row P (the face stage sharded by Morton range of 1 m leaves, group.cpp
// face_voxels_sharded): the codes of every point; this rank's points (in input order)
// and their sort into leaf order; the fit of its leaves into views of the full arrays;
// its residual points; the planar offsets over all leaves after the exchange.
void face_codes(B4<const float*> xyz, B4<const uint32_t*> d_n, uint32_t cap, double res, B4<FaceBufs> b, hipStream_t st,
                int nbatch);
void face_shard_select(B4<const uint32_t*> d_n, uint32_t cap, B4<FaceBufs> b, int rank, int nranks, hipStream_t st,
                       int nbatch);
void face_shard_sort(B4<const float*> xyz, uint32_t cap, B4<FaceBufs> b, hipStream_t st, int nbatch);
void face_shard_fit(uint32_t cap, float vpt, float cthr, B4<FaceBufs> bv, hipStream_t st, int nbatch);
void face_shard_resid(uint32_t cap, B4<FaceBufs> bv, B4<float*> rout, hipStream_t st, int nbatch);
void face_planar_scan(uint32_t cap, B4<FaceBufs> b, hipStream_t st, int nbatch);
// Per-leaf fit, planar/residual flags and the residual cloud.
void face_voxels_fit(B4<const uint32_t*> d_n, uint32_t cap, float voxel_point_threshold, float curvature_threshold, B4<float*> resid_out,
                     B4<FaceBufs> b, hipStream_t st, int nbatch = 1);
// Planar records, oriented towards b.centroid (must be ready: the caller orders streams).
struct CloudMail;
// mail (may be null): pinned mailbox receiving the records and both clouds' counts (sc = scalars of each cloud)
void face_voxels_orient(uint32_t cap, B4<VoxRec*> planar_out, B4<FaceBufs> b, hipStream_t st, int nbatch = 1,
                        CloudMail* mail = nullptr, B4<const uint32_t*> sc = B4<const uint32_t*>(nullptr));

// Byte strides between the sequences of a batched octree launch: sequence e uses
// xyz + e*xyz, aggr + e*aggr, state + e*state, d_n + e*n (bytes; 0 = shared).
struct SeqStrides {
  size_t xyz = 0, aggr = 0, state = 0, n = 0;
  template <class T>
  __host__ __device__ static T* at(T* p, size_t stride, uint32_t e) {
    return (T*)((char*)p + stride * e);
  }
  template <class T>
  __host__ __device__ static const T* at(const T* p, size_t stride, uint32_t e) {
    return (const T*)((const char*)p + stride * e);
  }
};
// Octree bound simulation over xyz[0..*d_n) starting from *state (one workgroup per
// sequence; `batch` sequences laid out by `sd`).
void octree_sim(const float* xyz, const uint32_t* d_n, uint32_t cap, double res, const float* aggr,
                OctState* state, hipStream_t st, int batch = 1, SeqStrides sd = SeqStrides());
// Fresh octree bounds replayed over xyz[0..*d_n) (aggr: aggr_floats(cap) floats).
void octree_replay(const float* xyz, const uint32_t* d_n, uint32_t cap, double res, float* aggr, OctState* state,
                   hipStream_t st);
// reset_state (optional): block 0 of each sequence also writes an empty OctState
// there (sequence e at reset_state + e * sd.state bytes) for the octree_sim that follows.
void block_aggr(const float* xyz, const uint32_t* d_n, uint32_t cap, float* aggr, hipStream_t st, int batch = 1,
                SeqStrides sd = SeqStrides(), OctState* reset_state = nullptr,
                uint64_t* stamp = nullptr);  // stamp: the face stage's start (FaceBufs::t_faces)
// Fine verification's form of block_aggr (fine.hip, FCCF.cpp:785-839): sequence e's
// points are T[e] * s2[i] (tf_se3), written to s2t + e * sd.xyz as they are aggregated,
// and block (0, e) also starts evaluation e's octree from the state after S1 and clears
// its per-evaluation counters (the work of a separate transform launch before).
struct FvTransform {
  const float* s2;  // the untransformed cloud (shared by the evaluations)
  const m44* T;
  float* s2t;       // per evaluation (sd.xyz stride)
  const OctState* s1_state;
  OctState* st;     // per evaluation (sd.state stride)
  uint32_t* scal;   // [4] n1, [5] n2, [7] error word (evaluation 0's block 0)
  uint32_t* ecnt;   // per-evaluation entry counts
  uint32_t* pts;    // per-evaluation finite point counts
  uint32_t n1, n2;  // (n2 also written to scal[5], the later launches' device count)
};
void block_aggr_transform(const FvTransform& tf, const uint32_t* d_n, uint32_t cap, float* aggr, hipStream_t st,
                          int batch, SeqStrides sd, uint64_t* stamp = nullptr);
// Grid of a streaming (grid-stride) launch over up to `cap` items per cloud, `per` items
// per workgroup, `nbatch` clouds: about one chip-full of workgroups in all (2048 per
// launch).  The face stage and the second VoxelGrid pass run on the downsampled clouds,
// a third of `cap` or less, so a grid sized by `cap` is mostly workgroups with no work.
uint32_t grid_stream(uint32_t cap, int nbatch, uint32_t per = 256);
constexpr uint32_t AGGR_BLOCK = 4096;  // points per block aggregate
constexpr uint32_t AGGR_SUB = 64;      // points per sub-aggregate (64 per block)
// aggregates of one sequence: aggr_blocks(cap) block records, then 64 sub-records per
// block; a record is the finite points' min xyz, max xyz (empty: min > max)
inline uint32_t aggr_blocks(uint32_t cap) { return (cap + AGGR_BLOCK - 1) / AGGR_BLOCK + 1; }
inline size_t aggr_floats(uint32_t cap) { return 6 * (size_t)aggr_blocks(cap) * (1 + AGGR_BLOCK / AGGR_SUB); }

}  // namespace fccf
