// host_stages.h — the serial, tiny-cardinality stages of FCCF-PCR that libfccf
// runs on the host CPU in round 1 (<= a few thousand items each).  Bit-level
// arithmetic follows fccf_math.h, the same conventions as the device kernels.
#pragma once
#include <cstdint>
#include <vector>

#include "../../include/fccf.h"
#include "error.h"
#include "fccf_math.h"
#include "kernels.h"
#include "pool.h"

namespace fccf {

// Exact cut points of theta(c) for a threshold (see pipeline.cpp make_cut).
AngleCut make_cut(float thr);

struct Plane {        // facenode of a selected plane (FCCF.cpp:47-58)
  float c[3], n[3];   // average_centry_*, average_normal_* (never renormalised, App. B Q3)
  float fps;          // face_point_size
  int32_t nvox;       // voxelgrothnode.size()
};

struct Base {         // face_base + type (FCCF.cpp:60-65, :454-461)
  int32_t i1, i2;
  float angle;
  int32_t type;       // 0 smooth/smooth, 1 rough/rough, 2 mixed; -1/-2 = no type (NaN roughness, Q5)
};

struct GrowOut {
  std::vector<Plane> planes;     // <= select_plane_number + 1
  std::vector<double> theta;     // roughness per selected plane
  std::vector<Plane> groups;     // all groups after stage 2 + range_face (debug)
  std::vector<int32_t> galloc;   // their is_allocate flags
  double ms_select = 0.0;        // host time of range_face + selection
};

// A growth group after stage 2 (a facenode of voxel_vector_groth, :595-648).
struct GroupOut {
  float ac[3], an[3], fps;
  bool alloc;
  std::vector<int> mem;  // member voxels in voxelgrothnode order
};
// face_extrate region growing, stages 1 and 2 (:536-648), on the host.
std::vector<GroupOut> grow_groups(const VoxRec* vox, int nv, const fccf_params& P);
// range_face (:409-427) and the plane selection with roughness (:650-677).
GrowOut select_groups(const std::vector<GroupOut>& G, const VoxRec* vox, const fccf_params& P);
// both of the above
GrowOut grow_and_select(const VoxRec* vox, int nv, const fccf_params& P);
// select_base (:429-468); `side` picks the out-of-range type sentinel (-1 / -2).
std::vector<Base> select_base(const std::vector<Plane>& F, const std::vector<double>& theta, const fccf_params& P,
                              int side);

struct QT {  // transform_q_t (FCCF.cpp:74-84)
  float qw, qx, qy, qz, tx, ty, tz;
  uint32_t alloc;
};

// transform_cluster (:1040-1231) incl. range_cluster and average_normal.  pool (may be
// null) builds the neighbour lists of consecutive seeds in parallel.  bits (may be
// null): the device's neighbour rows of these candidates (k_cluster_bits, n rows of
// ceil(n/64) words), which replace the host radius search.
void transform_cluster(std::vector<QT>& in, std::vector<QT>& fine, int cluster_num, const fccf_params& P,
                       int64_t* nclusters, Pool* pool = nullptr, const uint64_t* bits = nullptr);

// quick_verify (:680-783) with ceres_refine (:210-249): refines T in place, returns score.
float quick_verify(m44& T, const std::vector<Plane>& F1, const std::vector<Plane>& F2, const fccf_params& P,
                   int* npairs);

// Ceres-1.14-style LM on plane pairs (13 floats each: p1 n1 p2 n2 w); best x = q(xyzw), t.
void lm_solve(const float* pairs, int P, double best[7]);
// lm_solve of n problems, `lanes` at a time, SIMD across the problems (lm_batch.cpp):
// bit-identical to lm_solve per problem.  lanes 0: the widest the CPU runs (8 with
// AVX-512, 4 with AVX2, else 1 = lm_solve).
void lm_solve_batch(const float* const* pairs, const int* P, int n, double (*best)[7], int lanes = 0);
int lm_batch_lanes();
// quick_verify split for batched LMs: the plane pairs (13 floats each) and their count
// for T, and the score; then quick_verify_refine applies the LM result to T.
float quick_verify_pairs(const m44& T, const std::vector<Plane>& F1, const std::vector<Plane>& F2,
                         const fccf_params& P, std::vector<float>& pairs, int* npairs);
void quick_verify_refine(m44& T, const double best[7]);

struct High {
  QT qt;
  float score;
};
// weight_normal + fuse_answer (:1253-1368)
m44 fuse_answer(const std::vector<High>& hs, float sum);

struct TS { m44 T; float score, score2; };  // a verified candidate: T, quick score, fine score
// The fusion of computer_transform_guess (:1546-1606): score1/score2 sums over the first
// analyse_max candidates of every type (:1538-1540), each type's best normalised score
// (:1548-1596, identity when a type has none), the types above 0.8 of the best
// (:1599-1605) and fuse_answer.  tmp (may be null) receives the three per-type bests.
m44 fuse_types(const std::vector<TS> ctv[3], int analyse_max, std::vector<High>* tmp);

QT qt_from_T(const m44& T);
m44 T_from_qt(const QT& q);

}  // namespace fccf
