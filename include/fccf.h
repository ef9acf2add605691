/* fccf.h — C-ABI of libfccf, the MI355X-native FCCF-PCR registration path.
 *
 * Drop-in boundary.  The reference has no library surface of
 * its own: its only entry points are the CLI `./FCCF src.ply tar.ply voxel`
 * (/root/reference/FCCF.cpp:1646-1689) and the in-process driver
 *   void computer_transform_guess(PointCloud<PointXYZ>::Ptr source,
 *                                 PointCloud<PointXYZ>::Ptr target,
 *                                 Eigen::Matrix4f& best)            (FCCF.cpp:1370)
 * which `main` calls as (cloud_tar, cloud_src) after one VoxelGrid pass per cloud
 * (FCCF.cpp:1668-1683).  fccf_register() replaces the whole of main's compute
 * (both VoxelGrid passes + the driver) with plain pointers: inputs in FILE order
 * (src, tar), output T maps src-file points into the tar-file frame, exactly the
 * matrix the reference prints.  Inputs are never mutated (the reference's driver
 * mutates its clouds via removeNaNFromPointCloud, FCCF.cpp:1374-1375).
 *
 * All functions return 0 (FCCF_OK) or a negative FCCF_E_* code; no C++ exception
 * crosses this boundary.  One fccf_ctx per host thread; a ctx is bound to one HIP
 * device and stream.  There is no CPU fallback: fccf_ctx_create fails with
 * FCCF_E_NODEVICE when no gfx950 device is present.
 */
#ifndef FCCF_H_
#define FCCF_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum {
  FCCF_OK = 0,
  FCCF_E_ARG = -1,      /* bad argument (null pointer, leaf <= 0, n < 0 ...)        */
  FCCF_E_HIP = -2,      /* a HIP runtime call failed                                 */
  FCCF_E_RCCL = -3,     /* a collective failed                                       */
  FCCF_E_OOM = -4,      /* device or host allocation failed                          */
  FCCF_E_IO = -5,       /* PLY read/write failed                                     */
  FCCF_E_INTERNAL = -6, /* capacity / invariant violation inside the pipeline        */
  FCCF_E_NODEVICE = -7  /* no usable HIP device                                      */
};

/* The 26 tunables of FCCF.cpp:120-176, same names and reference defaults
 * (fccf_params_default).  Passed explicitly instead of globals. */
typedef struct fccf_params {
  float parameter_l1, parameter_l2, parameter_k1, parameter_k2;          /* :126-129 */
  float normal_vector_threshold1, normal_vector_threshold2;              /* :131-132 */
  float face_voxel_size;                                                 /* :134 (1.0 m; only 1.0 and 0.5 are exact) */
  float voxel_point_threshold;                                           /* :136 */
  float curvature_threshold;                                             /* :138 */
  float select_plane_number;                                             /* :141 */
  float quick_verify_angel_threshold, quick_verify_distance_threshold;   /* :145-146 */
  float required_optimize_plane;                                         /* :147 */
  float fine_verify_voxel_size, fine_verify_number;                      /* :150-151 */
  float included_angle_same_threshold, included_angle_min_threshold,
        included_angle_max_threshold;                                    /* :156-158 */
  float third_plane_threshold, third_plane_normal_threshold;             /* :160,162 */
  float cluster_number_threshold, cluster_angel_threshold,
        cluster_distance_threshold;                                      /* :166-168 */
  float seclct_cluster_number;                                           /* :171 */
  float rough_threshold_gl;                                              /* :175 */
} fccf_params;

/* Per-call counters and per-stage device/host timings (ms). */
enum {
  FCCF_T_DOWNSAMPLE = 0, FCCF_T_VOXELFIT, FCCF_T_GROW, FCCF_T_SELECT, FCCF_T_MATCH,
  FCCF_T_CLUSTER, FCCF_T_VERIFY, FCCF_T_FINE, FCCF_T_FUSE, FCCF_T_H2D, FCCF_T_COUNT
};
typedef struct fccf_stats {
  int64_t n_src, n_tar;          /* input points                                  */
  int64_t m_src, m_tar;          /* after both VoxelGrid passes                   */
  int64_t vox1, vox2;            /* planar 1 m voxels (driver source / target)    */
  int64_t res1, res2;            /* residual (non-planar) points S1, S2           */
  int64_t groups1, groups2;      /* region-growing groups after stage 2           */
  int64_t planes1, planes2;      /* selected planes F1, F2 (<= 16)                */
  int64_t bases1, bases2;        /* coplane pairs B1, B2                          */
  int64_t K;                     /* coplane-pair correspondence tests = B1*B2     */
  int64_t K_pass;                /* tests that passed (computer_transform calls)  */
  int64_t cand[3];               /* candidate transforms per roughness type       */
  int64_t fine[3];               /* cluster-fused candidates per type             */
  int64_t lm_solves;             /* quick_verify refinements run                  */
  int32_t overflow_passthrough;  /* VoxelGrid int32 guard tripped (any pass)      */
  int32_t graph_captures;        /* device-stage graphs (re)captured by this call */
  double ms[FCCF_T_COUNT];       /* stage times: DOWNSAMPLE and VOXELFIT are device
                                    spans (s_memrealtime stamps written by the cloud
                                    stage's own kernels, dev_ms below), H2D a HIP-event
                                    span of the input copy, the others host wall times */
  double ms_total;               /* host arrays (or resident device arrays) -> T  */
  /* appended in round 2 (SURVEY.md §8(d) stage roofline inputs) */
  int64_t m1_src, m1_tar;        /* after main's VoxelGrid pass (FCCF.cpp:1668-1678) */
  int64_t leaves1, leaves2;      /* occupied 1 m octree leaves (driver source / target) */
  int64_t fine_evals;            /* fine_verify evaluations E                      */
  double dev_ms[4];              /* device spans: main's VoxelGrid pass, the driver's
                                    remove-NaN + second pass, face voxels (s_memrealtime
                                    stamps of the cloud stage's kernels), fine verify */
  /* appended in round 3 */
  int64_t stage_redos;           /* cloud stages redone because the driver's VoxelGrid
                                    input was not in leaf order; in a
                                    batch, counted for the pair that found it and the
                                    later pairs of its stage group (an earlier pair of
                                    the group had already finished its phase B1, with
                                    a correct result, and counts 0) */
  /* appended in round 4 */
  int32_t shard_ranks;           /* ranks of the attached group (1: no group)      */
  uint32_t sharded;              /* FCCF_SHARDED_* stages this call split over them */
  int64_t fine_reruns;           /* fine verifications rerun in the sorted leaf form
                                    (an evaluation with more 0.5 m leaves than the
                                    LDS form holds; the scores are the same).  In a
                                    pipelined batch such a pair is registered again
                                    after the batch's last pair (its stage arena may
                                    be recycled by then)                           */
  /* appended in round 6 */
  int64_t xch_bytes[3];          /* bytes this rank received through its group's
                                    exchanges during the call, per channel: matching
                                    (K5 counts and lists), fine (F scores), clouds (D
                                    sorted slices, P face records); a pipelined batch
                                    reports its whole call on every pair.  0 without
                                    a group (fccf_group_bytes: the running totals)  */
} fccf_stats;
/* fccf_stats.sharded bits */
enum {
  FCCF_SHARDED_SEARCH = 1u, /* K5 correspondence search, FCCF.cpp:1410-1428 */
  FCCF_SHARDED_FINE = 2u,   /* F fine_verify evaluations, :785-839          */
  FCCF_SHARDED_SORT = 4u,   /* D VoxelGrid's std::sort ranges, :1668-1678   */
  FCCF_SHARDED_FACES = 8u   /* P 1 m face voxels by Morton range, :470-534  */
};

typedef struct fccf_ctx fccf_ctx;

void fccf_params_default(fccf_params* p);
const char* fccf_strerror(int code);

/* device: HIP ordinal (the ctx creates its own non-blocking stream). */
int fccf_ctx_create(fccf_ctx** ctx, int device);
int fccf_ctx_destroy(fccf_ctx* ctx);
/* Message of the last failing call on ctx ("" if none); valid until the next call. */
const char* fccf_ctx_last_error(fccf_ctx* ctx);
/* Region growing (FCCF.cpp:536-648) on the GPU (K4, one wave
 * per cloud with LDS-resident voxels, bit-identical) instead of the host: applies to
 * fccf_register* and fccf_stage_grow on this ctx; clouds with more planar voxels than
 * the kernel's LDS holds still grow on the host.  Off by default. */
int fccf_ctx_set_grow_device(fccf_ctx* ctx, int on);
/* quick_verify with its Ceres-style LM refinement (FCCF.cpp:680-783, :210-249; SURVEY
 * §8(f) f1) on the GPU, one wave per candidate, all candidates in one launch, instead
 * of the host pool: applies to fccf_register* and fccf_stage_verify on this ctx.  Off
 * by default. */
int fccf_ctx_set_lm_device(fccf_ctx* ctx, int on);
/* transform_cluster's seed pass, range_cluster's exchange sort and the cluster
 * averaging (FCCF.cpp:1040-1231, :1020-1038) on the GPU, after the
 * device radius search, bit-identical: applies to fccf_register* and
 * fccf_stage_cluster on this ctx; a type past the kernels' capacities is clustered on
 * the host.  Off by default. */
int fccf_ctx_set_cluster_device(fccf_ctx* ctx, int on);
/* Keep per-stage intermediates for fccf_debug_get (tests). Off by default. */
int fccf_ctx_set_debug(fccf_ctx* ctx, int on);

/* Whole registration from host arrays (xyz float32, 3*n, FILE order src/tar).
 * leaf = the CLI voxel argument (FCCF.cpp:1650).  params may be NULL (defaults).
 * T_rowmajor receives the 4x4 the reference prints (FCCF.cpp:1687).  stats may be NULL. */
int fccf_register(fccf_ctx* ctx, const float* src_xyz, int64_t n_src, const float* tar_xyz,
                  int64_t n_tar, float leaf, const fccf_params* params, float T_rowmajor[16],
                  fccf_stats* stats);

/* Same, with both clouds already resident in device memory of ctx's device. */
int fccf_register_device(fccf_ctx* ctx, const float* d_src_xyz, int64_t n_src,
                         const float* d_tar_xyz, int64_t n_tar, float leaf,
                         const fccf_params* params, float T_rowmajor[16], fccf_stats* stats);

/* Batch / throughput mode: n independent pairs, pipelined so
 * that pair i+1's cloud stage (VoxelGrid passes, face voxels) runs on the GPU while
 * pair i's later stages run.  Every pair's T and stats equal what fccf_register
 * (fccf_register_device when on_device != 0) returns for it alone.
 * T_rowmajor: 16*n floats; stats: n entries or NULL. */
int fccf_register_batch(fccf_ctx* ctx, int n, const float* const* src_xyz, const int64_t* n_src,
                        const float* const* tar_xyz, const int64_t* n_tar, int on_device, float leaf,
                        const fccf_params* params, float* T_rowmajor, fccf_stats* stats);

/* Device-resident inputs for fccf_register_device (bench / batch users): copy n
 * xyz points to a new HBM buffer on ctx's device; release with fccf_device_free. */
int fccf_device_upload(fccf_ctx* ctx, const float* xyz, int64_t n, float** d_xyz);
int fccf_device_free(fccf_ctx* ctx, float* d_xyz);
/* n xyz points of a device buffer back to host memory (tests). */
int fccf_device_download(fccf_ctx* ctx, const float* d_xyz, int64_t n, float* xyz);

/* Stage export: PCL VoxelGrid<PointXYZ> (FCCF.cpp:1668-1678) on the GPU.
 * out_xyz capacity 3*n floats; *m receives the output count.  Output order is
 * ascending leaf index; the points of one leaf are summed in the order libstdc++
 * std::sort leaves PCL's (leaf, index) pairs (the reference's own order, introsort,
 * unstable), bit-identical to the oracle's INTROSORT mode.  FCCF_E_INTERNAL if the
 * sort's device invariant checks fail. */
int fccf_stage_downsample(fccf_ctx* ctx, const float* xyz, int64_t n, float leaf, float* out_xyz,
                          int64_t* m);
/* The same, as the driver's second pass runs it (FCCF.cpp:1377-1387 over main's
 * output): a check in the key kernel takes the identity shortcut when the keys are
 * already strictly increasing, else a single-workgroup sort.  Same result for any input. */
int fccf_stage_downsample_presorted(fccf_ctx* ctx, const float* xyz, int64_t n, float leaf, float* out_xyz,
                                    int64_t* m);

/* Stage export: pcl::compute3DCentroid of a dense cloud (FCCF.cpp:473 via
 * face_extrate): out = (sum x / n, sum y / n, sum z / n, 1) with each sum a
 * left-to-right float accumulation, bit-identical to the sequential loop (computed
 * in parallel on the GPU, exactsum.h).  n == 0 gives (0, 0, 0, 1). */
int fccf_stage_centroid(fccf_ctx* ctx, const float* xyz, int64_t n, float out[4]);
/* Stage export: s = ((0 + x0) + x1) + ... + x(n-1) in float, the accumulation
 * order of fine_verify's similar_num (FCCF.cpp:830-835); bit-exact. */
int fccf_stage_seqsum(fccf_ctx* ctx, const float* x, int64_t n, float* out);

/* One planar 1 m voxel (FCCF.cpp:500-534): leaf centroid, normal oriented towards the
 * cloud centroid, point count; curvature is the leaf's eigen33 curvature. */
typedef struct fccf_voxel { float c[3], n[3]; int32_t count; float curvature; } fccf_voxel;

/* Stage export: face_extrate's voxel pass (FCCF.cpp:473-534) of one downsampled
 * cloud on the GPU: compute3DCentroid, the face_voxel_size octree anchored at the
 * first point, the per-leaf plane fit and the planar / residual split.  planar
 * receives the planar voxels in octree (Morton) order, resid_xyz the residual points
 * (leaf order); at most cap_* entries are copied, n_* receive the full counts.
 * centroid (may be NULL) receives (cx, cy, cz, 1).  Uses face_voxel_size,
 * voxel_point_threshold and curvature_threshold of params (NULL: defaults). */
int fccf_stage_voxel_planes(fccf_ctx* ctx, const float* xyz, int64_t n, const fccf_params* params,
                            fccf_voxel* planar, int64_t cap_planar, int64_t* n_planar, float* resid_xyz,
                            int64_t cap_resid, int64_t* n_resid, float centroid[4]);

/* A selected plane (facenode summary, FCCF.cpp:47-58) and a coplane pair
 * (face_base + its roughness type, FCCF.cpp:60-65, :454-461), as the matching stage
 * reads them.  type: 0 smooth/smooth, 1 rough/rough, 2 mixed, negative = untyped
 * (NaN roughness: never matches). */
typedef struct fccf_plane { float c[3], n[3]; float fps; int32_t nvox; } fccf_plane;
typedef struct fccf_base { int32_t i1, i2; float angle; int32_t type; } fccf_base;

/* Stage export: region growing (FCCF.cpp:536-648), range_face + plane selection
 * (:409-427, :650-677) and select_base (:429-468) of one cloud's planar voxels
 * (host stage; ctx supplies only the error slot).  side = 1 for the driver source,
 * 2 for the target (the untyped sentinel differs, App. B Q5).  planes (<= 17),
 * theta (roughness per plane, may be NULL) and bases (<= 136): at most cap_* are
 * copied, n_* receive the full counts. */
int fccf_stage_grow(fccf_ctx* ctx, const fccf_voxel* vox, int64_t nv, int side, const fccf_params* params,
                    fccf_plane* planes, int cap_planes, int* n_planes, double* theta, fccf_base* bases,
                    int cap_bases, int* n_bases);

/* Stage export: the coplane-pair correspondence search (FCCF.cpp:1410-1428) and
 * computer_transform (:841-1018) on the GPU, for source pairs b1 in [b1_lo, b1_hi)
 * against all nB2 target pairs (b1_hi < 0 means nB1).  F1/B1 are the driver
 * source's planes and pairs, F2/B2 the target's (<= 17 planes, <= 136 pairs each).
 * Candidates go to cand[t] (type t = 0..2) as row-major 4x4 matrices, 16 floats each,
 * in the reference's (b1, b2, third plane) loop order; at most cap[t] are copied and
 * n_cand[t] receives the full count.  *k_pass = tests with >= 1 candidate.
 * Sharding: splitting [0, nB1) into contiguous ranges and
 * concatenating each type's lists in range order gives the unsharded lists exactly.
 * Uses included_angle_same_threshold, third_plane_threshold and
 * third_plane_normal_threshold of params (NULL: defaults). */
int fccf_stage_match(fccf_ctx* ctx, const fccf_plane* F1, int nF1, const fccf_base* B1, int nB1,
                     const fccf_plane* F2, int nF2, const fccf_base* B2, int nB2, int b1_lo, int b1_hi,
                     const fccf_params* params, float* const cand[3], const int64_t cap[3],
                     int64_t n_cand[3], int64_t* k_pass);

/* Stage export: the quaternion/translation records (FCCF.cpp:1437-1465) and
 * transform_cluster (:1040-1231, with range_cluster :1020-1038 and average_normal
 * :325-367) of one candidate type's list (host stage).  cand: n row-major 4x4
 * matrices in list order, as fccf_stage_match returns them; cluster_num is the
 * caller's int(seclct_cluster_number * n / total over all types) (:1458).  fine
 * receives the fused candidates, 8 floats each (qw, qx, qy, qz, tx, ty, tz,
 * allocated flag); at most cap are copied, *n_fine = the full count.
 * *n_clusters (may be NULL) = clusters formed. */
int fccf_stage_cluster(fccf_ctx* ctx, const float* cand_rowmajor, int64_t n, int cluster_num,
                       const fccf_params* params, float* fine, int64_t cap, int64_t* n_fine, int64_t* n_clusters);
/* Stage export: the fusion of computer_transform_guess (FCCF.cpp:1546-1606, host
 * stage): cand[t] holds n[t] verified candidates of type t in score_range order, 18
 * floats each (row-major 4x4 T, quick_verify score, fine_verify score).  The score
 * sums run over the first analyse_max candidates of every type (:1538-1540), each
 * type's best normalised score picks its T (identity when none), the types above 0.8
 * of the best are fused (fuse_answer :1253-1368).  T receives the result; high (may be
 * NULL) the three per-type bests, 8 floats each (qw qx qy qz tx ty tz score).
 * fccf_stage_grow, fccf_stage_cluster and fccf_stage_fuse are host code: ctx may be
 * NULL for them (no device form is selectable then). */
int fccf_stage_fuse(fccf_ctx* ctx, const float* const cand[3], const int64_t n[3], int analyse_max, float T_rowmajor[16],
                    float high[24]);

/* Stage export: fine_verify (FCCF.cpp:785-839) of E <= 16 transforms on the GPU:
 * scores[e] = score of S2 transformed by T_e against S1 over the fine_verify_voxel
 * octree (the voxel argument).  s1/s2: residual clouds (xyz float32, n1, n2 >= 1);
 * T_rowmajor: 16*E floats.  Bit-identical to the sequential reference arithmetic. */
/* quick_verify + LM of n clustered candidates (8 floats each: qw qx qy qz tx ty tz
 * allocated, as fccf_stage_cluster returns them) against the selected planes F1/F2:
 * refined T (row-major, 16 per candidate), score and plane-pair count per candidate. */
int fccf_stage_verify(fccf_ctx* ctx, const fccf_plane* F1, int nF1, const fccf_plane* F2, int nF2, const float* qt,
                      int64_t n, const fccf_params* params, float* T_out, float* score, int32_t* npairs);
int fccf_stage_fine_verify(fccf_ctx* ctx, const float* s1_xyz, int64_t n1, const float* s2_xyz, int64_t n2,
                           const float* T_rowmajor, int E, float voxel, float* scores);

/* Roofline probe (bench.py): time every launch of one kernel (by name, e.g.
 * "k_vg_centroid") with HIP events on its own stream, also inside the captured
 * graphs, and accumulate its algorithmic bytes ("Measurement").
 * kernel NULL or "" switches the probe off.  Setting it resets the totals. */
int fccf_ctx_set_probe(fccf_ctx* ctx, const char* kernel);
int fccf_probe_read(fccf_ctx* ctx, double* total_ms, int64_t* launches, double* total_bytes);
/* The same totals split by launch width w = 1..max_width (entry w - 1): the clouds one
 * batched launch processes (grid.y of the cloud stage's kernels; a single registration
 * launches two, a pipelined batch of five pairs per stage ten; widths past 16 are not
 * tallied). */
int fccf_probe_read_widths(fccf_ctx* ctx, int max_width, double* ms, int64_t* launches, double* bytes);

/* Named intermediate of the last fccf_register call with debug on (see DESIGN.md
 * "Debug names").  Copies min(cap_bytes, size) bytes; *n_bytes = full size. */
int fccf_debug_get(fccf_ctx* ctx, const char* name, void* buf, int64_t cap_bytes,
                   int64_t* n_bytes);

/* Test hook of K1's sort (the std::sort of pcl::VoxelGrid's index vector,
 * FCCF.cpp:1668-1678): keys[0..n) (0xFFFFFFFF = a non-finite point, skipped as PCL
 * skips it) with values = input positions, sorted on the GPU in libstdc++ std::sort
 * order; perm_out[0..n) receives the values in sorted order (the finite ones first).
 * exact_gate != 0 runs the presorted second pass's single-workgroup form. */
int fccf_debug_sort_keys(fccf_ctx* ctx, const uint32_t* keys, int64_t n, int exact_gate, uint32_t* perm_out);
/* Dev / tests: the same sort of `copies` (1..10) copies of the keys in one batched launch
 * sequence, as a pipelined stage group runs it (grid y = copies), writing the sorted points
 * of xyz (may be NULL) as VoxelGrid's first pass does; perm_out: copy 0's order; dev_ms:
 * the sort's device span. */
int fccf_debug_sort_keys_batch(fccf_ctx* ctx, const uint32_t* keys, int64_t n, int copies, const float* xyz,
                               uint32_t* perm_out, double* dev_ms);
/* Path counters of the last fccf_debug_sort_keys: [0] sort length, [2] slow-path flags
 * (1 global partitions, 2 a sequential heap sort beyond the LDS, 4 a depth-limit segment
 * beyond the LDS with distinct keys), [3] global partitions, [4] LDS segments, [5]
 * workgroup partitions, [6] wave partitions, [7] sequential heap sorts (depth limit,
 * repeated keys), [9] depth-limit segments with pairwise distinct keys (sorted in
 * parallel: their order is unique), [12] register-resident subtrees, [16] wave tasks,
 * [28..29] the rank range of a row-D simulated sort (FCCF_SHARD_D_SIM=r/N, environment),
 * [31] the sort's device time in ns.
 * fccf_debug_sort_keys returns FCCF_E_INTERNAL when an invariant flag is set. */
/* Test hook: the device LM's correctly rounded double sin/cos (verify.hip); ok[i] = 0
 * where |x| is beyond its argument reduction. */
int fccf_debug_sincos(fccf_ctx* ctx, const double* x, int64_t n, double* s, double* c, uint32_t* ok);
int fccf_debug_sort_stats(fccf_ctx* ctx, uint32_t out[32]);
/* Test hook (host only, no ctx): quick_verify's LM (Ceres-style, FCCF.cpp:210-249) for n
 * problems, pairs[13 * (sum of the P before i) ..] holding problem i's P[i] plane pairs
 * (p1 n1 p2 n2 w), solved `lanes` problems at a time with SIMD across the problems
 * (1 = the scalar form, 4 = AVX2, 8 = AVX-512; 0 = the widest the CPU runs); best:
 * n x 7 doubles (q xyzw, t).  FCCF_E_ARG when the CPU lacks the lanes asked for. */
int fccf_debug_lm_batch(const float* pairs, const int32_t* P, int32_t n, int32_t lanes, double* best);
/* Test hook: the round records of the last fccf_debug_sort_keys, 24 x {segments
 * partitioned, their tiles, owned segments so far, elements partitioned}. */
int fccf_debug_sort_rounds(fccf_ctx* ctx, uint32_t out[96]);
/* Test hook: every later sort of K1 on ctx raises the invariant flags in bits (0x100
 * round scatter outside its segment, 0x200 block item guard, 0x400 wave task stack,
 * 0x1000 block partition stack) as if the check had fired, until called with 0.
 * fccf_register* then fails with FCCF_E_INTERNAL, as it does for a real violation.
 * Bit 0x10000 instead makes the pipeline's optimistic driver VoxelGrid pass report its
 * input as out of leaf order, so the registration redoes its cloud stage with the
 * exact second pass (fccf_stats.stage_redos; the result is unchanged); bit 0x40000 does
 * the same for the later pairs of a pipelined batch's stage group only (their clouds
 * share the launches with the group's first pair, which is not flagged).  Bit 0x20000
 * fills the first pass's sorted-point buffer with NaN before every sort, so a sorted
 * position that the sort's finish kernels fail to write turns into a NaN centroid
 * (a wrong result) instead of a stale point of an earlier call. */
int fccf_debug_inject_sort_fault(fccf_ctx* ctx, uint32_t bits);
/* Test hook: the next replay of a cached cloud-stage graph is patched with one
 * workspace-layout argument that differs from the graph's capture (the bug class of a
 * patch state shared by graphs of two layouts).  Every replay compares the patched
 * entry kernel's layout arguments with the captured ones, so that call fails with
 * FCCF_E_INTERNAL before anything is launched; the hook is consumed. */
int fccf_debug_graph_mismatch(fccf_ctx* ctx);
/* Forces a graph capture on one stream concurrent with another thread's wait on
 * an event last recorded on that stream (the pipelined batch's hazard, guarded by
 * the capture lock).  guard 1 = the product's guarded wait, 0 = an unguarded
 * hipStreamWaitEvent.  out: [0] ms in the wait call, [1] ms the capture held after
 * releasing the waiter, [2] the wait's error code, [3] 1 if it returned after the
 * capture ended.  Test hook. */
int fccf_debug_capture_race(fccf_ctx* ctx, int hold_ms, int guard, double out[4]);

/* Multi-GPU over RCCL: one process per GPU, one group per
 * ctx.  Rank 0 makes an id with fccf_group_unique_id and the caller hands it to every
 * rank out of band; each rank calls fccf_group_create with its ctx (collective over
 * the n ranks).  While a group is attached, fccf_register* on that ctx is a
 * collective: every rank passes the same clouds, the coplane-pair correspondence
 * search (FCCF.cpp:1410-1428) is sharded by contiguous source-pair blocks and the
 * candidate lists are gathered in rank order over RCCL; every rank returns the same T,
 * bit-identical to the unsharded registration.  fccf_group_destroy detaches it. */
#define FCCF_GROUP_ID_BYTES 128
typedef struct fccf_group fccf_group;
int fccf_group_unique_id(uint8_t id[FCCF_GROUP_ID_BYTES]);
int fccf_group_create(fccf_ctx* ctx, const uint8_t id[FCCF_GROUP_ID_BYTES], int n_ranks, int rank,
                      fccf_group** group);
int fccf_group_destroy(fccf_group* group);
/* Test hook: n "virtual ranks" of one process on one device, one group per ctx
 * (distinct ctxs of the same device), exchanging through a shared device buffer
 * under host barriers instead of RCCL: the sharded paths' host-side exchange logic
 * with n > 1 ranks on one GPU (RCCL refuses two ranks on one device).  Each rank's
 * calls must come from its own host thread, all ranks calling the same sequence. */
int fccf_group_create_local(fccf_ctx* const* ctxs, int n, fccf_group** groups);
int fccf_group_info(const fccf_group* group, int* n_ranks, int* rank);
/* Bytes this rank has received through the group's collectives since it was created,
 * per channel: [0] the candidate gather (matching stream), [1] the fine scores, [2]
 * the cloud stage's rows D and P (sorted slices, leaf records, residual points).  An
 * all-gather-v is one all-gather of count-padded blocks, so the padding is included.
 * The caller takes differences around the calls it measures (bench.py's group leg). */
int fccf_group_bytes(const fccf_group* group, int64_t rx[3]);
/* Failure handling: every host wait of a registration that may depend on a peer (a
 * stream or event after a collective, the pipelined batch's collective-order gate, a
 * virtual-rank barrier) is bounded by FCCF_GROUP_TIMEOUT_S seconds (environment at
 * group creation, default 30) and polls ncclCommGetAsyncError.  A rank whose
 * registration fails -- an error of its own, an asynchronous RCCL error or a timeout --
 * aborts the group (ncclCommAbort of its communicators, which also ends the kernels
 * waiting in them) and returns the error; its peers end at their bound the same way
 * and return FCCF_E_RCCL.  An aborted group fails every later registration with
 * FCCF_E_RCCL until fccf_group_destroy; then create a new one.
 * fccf_group_aborted: 1 if aborted, 0 if not. */
int fccf_group_aborted(const fccf_group* group);
/* Test hook: this rank fails (FCCF_E_RCCL, "injected failure") when its next
 * registration reaches collective site `site` (1 the candidate gather, 2 the fine-score
 * gather, 3 the sharded sort's gather; 0 = off).  silent != 0: it does not abort its
 * transport either (a peer that died), so the others find out at their time limit. */
int fccf_debug_group_fail(fccf_group* group, int site, int silent);
/* Stage export of the sharded search: fccf_stage_match's arguments without the
 * range; this rank searches its block, and every rank receives the whole lists. */
int fccf_group_stage_match(fccf_group* group, const fccf_plane* F1, int nF1, const fccf_base* B1, int nB1,
                           const fccf_plane* F2, int nF2, const fccf_base* B2, int nB2,
                           const fccf_params* params, float* const cand[3], const int64_t cap[3],
                           int64_t n_cand[3], int64_t* k_pass);

/* PLY I/O (the reference's pcl::io::loadPLYFile<PointXYZ> surface, FCCF.cpp:1655-1665):
 * ascii / binary_little_endian / binary_big_endian, float x,y,z (double converted).
 * *xyz is malloc'd by the library; release with fccf_free. */
int fccf_ply_read(const char* path, float** xyz, int64_t* n);
int fccf_ply_write(const char* path, const float* xyz, int64_t n, int binary);
void fccf_free(void* p);
/* Streaming PLY ingest: the vertex rows of path are decoded in
 * chunks by the ctx's ingest threads into pinned staging slots, each chunk uploaded
 * to a new HBM buffer on the ctx's copy stream while the next is decoded.  Same
 * values as fccf_ply_read.  *d_xyz is released with fccf_device_free; the buffer is
 * complete when the call returns.  FCCF_E_IO for a file loadPLYFile would reject. */
int fccf_ply_load_device(fccf_ctx* ctx, const char* path, float** d_xyz, int64_t* n);

/* Deterministic synthetic scenes; used by tests and bench. */
int fccf_synth_scene(int64_t n, double Lx, double Ly, double Lz, uint64_t seed,
                     double crop_x_frac, float* out_xyz);
int fccf_synth_pair(int64_t n, double Lx, double Ly, double Lz, float* src_xyz,
                    float* tar_xyz, float T_gt_rowmajor[16]);

#ifdef __cplusplus
}
#endif
#endif /* FCCF_H_ */
