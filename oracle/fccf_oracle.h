/* fccf_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of /root/reference/FCCF.cpp (the whole registration path) used
 * as the parity oracle by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg.  The product (libfccf, fccf-pcr_amd/) never links it.
 *
 * Parity status: the reference cannot be compiled here (PCL/Eigen/Ceres/FLANN
 * absent) and ships no tests or fixtures, so this restatement is
 * "parity unpinned" against the original binary; it is pinned by known-answer
 * tests (tests/test_oracle_kat.py) and by recovering the ground-truth transform
 * of the synthetic scenes.  See DESIGN.md §Oracle.
 */
#ifndef FCCF_ORACLE_H_
#define FCCF_ORACLE_H_
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Within-leaf summation order of the VoxelGrid centroid (PCL sorts (leaf, index)
 * pairs with std::sort, which is unstable; FCCF.cpp:1668-1678 / App. A2). */
enum { ORC_ORDER_STABLE = 0, ORC_ORDER_INTROSORT = 1 };

typedef struct orc_ctx orc_ctx;

/* Full registration exactly as `./FCCF src tar leaf` computes it: VoxelGrid on
 * both clouds (main), then computer_transform_guess(tar, src).  Keeps every
 * intermediate for orc_get.  Returns NULL on bad arguments. */
orc_ctx* orc_register(const float* src_xyz, int64_t n_src, const float* tar_xyz, int64_t n_tar,
                      float leaf, int order);
void orc_free(orc_ctx* c);
/* Copy a named intermediate (see oracle/README in DESIGN.md); returns its byte size. */
int64_t orc_get(orc_ctx* c, const char* name, void* buf, int64_t cap_bytes);
/* Per-stage host milliseconds of the last run: [downsample, voxelfit, grow+select,
 * match, cluster, verify, fine, fuse, total]. */
void orc_times(orc_ctx* c, double out_ms[9]);

/* Single stages (known-answer tests). */
int64_t orc_voxel_grid(const float* xyz, int64_t n, float leaf, int order, float* out_xyz,
                       int* overflow);
/* std::sort of PCL VoxelGrid's (idx, cloud_point_index) pairs (compared by idx only)
 * over the keys != 0xFFFFFFFF in input order; perm_out receives cloud_point_index in
 * sorted order.  Returns the number of sorted pairs. */
int64_t orc_sort_pairs(const uint32_t* keys, int64_t n, uint32_t* perm_out);
/* Keys that drive libstdc++ std::sort to its depth limit (McIlroy's adversary run
 * against this std::sort), for the heap-sort fallback tests. */
void orc_sort_adversary(int64_t n, uint32_t* keys_out);
/* pcl::eigen33 + curvature on a symmetric 3x3 (row-major) covariance. */
void orc_eigen33(const float cov[9], float* eigenvalue, float vec[3]);
/* compute_normal_angel (FCCF.cpp:369-377). */
float orc_normal_angle(float x1, float y1, float z1, float x2, float y2, float z2);
/* acos convention of FCCF.cpp:374 used by every angle (0 = float overload,
 * correctly rounded acosf — default; 1 = this host's glibc acosf; 2 = C's
 * double acos).  Returns the previous mode; out-of-range modes are ignored. */
int orc_set_acos_mode(int mode);
/* Octree structure of face_extrate / fine_verify: 1 = PCL's pointer octree (default,
 * the CPU baseline's algorithm), 0 = a Morton stable sort (same leaves).  Returns the
 * previous mode. */
int orc_set_octree_mode(int mode);
/* Per-site decision audit since the last reset, 8 sites (grow, merge, rough,
 * base, third, cluster, verify, pair): out[0..7] evaluations, out[8..15]
 * decision inputs whose bits differ between the conventions, out[16..23]
 * decisions that flip between them.  reset != 0 clears the counters after. */
void orc_acos_audit(uint64_t out[24], int reset);
/* Eigen::Quaternionf(Matrix3f) and toRotationMatrix (row-major). */
void orc_quat_from_rot(const float R[9], float q_wxyz[4]);
void orc_rot_from_quat(const float q_wxyz[4], float R[9]);
/* Ceres-1.14-style LM of ceres_refine (FCCF.cpp:210-249) on P plane pairs laid out
 * as 13 floats each: p1[3] n1[3] p2[3] n2[3] weight.  Outputs q (x,y,z,w), t. */
int orc_lm_refine(const float* pairs, int P, double q_xyzw[4], double t[3]);

/* Single host stages for the known-answer tests (tests/test_host_kat.py), default
 * parameters.  orc_voxel has fccf_voxel's layout. */
typedef struct orc_voxel { float c[3], n[3]; int32_t count; float curvature; } orc_voxel;
/* Region growing, range_face + selection and select_base (FCCF.cpp:536-677, :429-468):
 * planes 8 floats each (c, n, fps, voxel count), theta per plane, bases 4 words each
 * (i1, i2, angle bits, type; past type_index's end the side's sentinel -1 / -2). */
int orc_stage_grow(const orc_voxel* vox, int64_t nv, int side, float* planes, int cap_planes, int* n_planes,
                   double* theta, int32_t* bases, int cap_bases, int* n_bases);
/* transform_cluster (:1040-1231) of n row-major candidates: 8 floats per fused one. */
int orc_stage_cluster(const float* cand, int64_t n, int cluster_num, float* fine, int64_t cap, int64_t* n_fine,
                      int64_t* n_clusters);
/* The fusion (:1546-1606): cand[t] n[t] records of 18 floats (T, score, score2). */
int orc_stage_fuse(const float* const cand[3], const int64_t n[3], int analyse_max, float T[16], float high[24]);

#ifdef __cplusplus
}
#endif
#endif
