// fccf_oracle.cpp — TEST INFRASTRUCTURE ONLY (see fccf_oracle.h).
//
// A single-threaded C++17 restatement of /root/reference/FCCF.cpp with the
// third-party behaviour it depends on (PCL 1.10 VoxelGrid / octree / normal
// estimation, Eigen 3.3 fixed-size arithmetic, FLANN radius search, Ceres 1.14
// LM) re-stated from their published algorithms.
//
// Arithmetic conventions (they decide bit patterns, so they are fixed here and
// restated identically by the HIP product):
//  * build with -O2 -ffp-contract=off: no FMA anywhere (the reference is built
//    for baseline x86-64 = SSE2, which has no FMA; CMakeLists.txt:6-8).
//  * Eigen float Vector3 reductions are a0 + (a1 + a2) (redux_novec_unroller);
//    Eigen double Vector3 reductions are (a0 + a1) + a2 (SSE2 Packet2d redux).
//  * float transcendental f(x) is evaluated as (float)f((double)x)
//    (acos, atan2, cos, sin): correctly rounded except in ~2^-29 of cases.
//  * PCL's SSE Transformer: p' = x*c0 + (y*c1 + (z*c2 + c3)), n' = x*c0 + (y*c1 + z*c2).
#include "fccf_oracle.h"

#include <algorithm>
#include <cfloat>
#include <chrono>
#include <climits>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

// ---------------------------------------------------------------- parameters
// FCCF.cpp:120-176 (global floats; defaults of the shipped source).
struct Params {
  float parameter_l1 = 0.5f, parameter_l2 = 1.0f, parameter_k1 = 5.0f, parameter_k2 = 2.0f;
  float normal_vector_threshold1 = 5.0f, normal_vector_threshold2 = 8.0f;
  float face_voxel_size = 1.0f;
  float voxel_point_threshold = 5;
  float curvature_threshold = 0.05f;
  float select_plane_number = 15;
  float quick_verify_angel_threshold = 10.0f, quick_verify_distance_threshold = 2.0f;
  float required_optimize_plane = 4.0f;
  float fine_verify_voxel_size = 0.5f, fine_verify_number = 4;
  float included_angle_same_threshold = 5.0f, included_angle_min_threshold = 30.0f,
        included_angle_max_threshold = 150.0f;
  float third_plane_threshold = 0.5f, third_plane_normal_threshold = 5.0f;
  float cluster_number_threshold = 10, cluster_angel_threshold = 2.0f,
        cluster_distance_threshold = 0.8f;
  float seclct_cluster_number = 200;
  float rough_threshold_gl = 2;
};

// ------------------------------------------------------ Eigen-order helpers
struct V3f { float x, y, z; };
struct M3f { float m[3][3]; };
struct M4f { float m[4][4]; };

static inline float dotf(const V3f& a, const V3f& b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
static inline float sqnormf(const V3f& a) { return a.x * a.x + (a.y * a.y + a.z * a.z); }
static inline V3f crossf(const V3f& a, const V3f& b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
// Eigen 3.3.7 MatrixBase::normalize(): divide by sqrt(squaredNorm) only if > 0.
static inline V3f normalizedf(V3f a) {
  float z = sqnormf(a);
  if (z > 0.f) {
    float s = std::sqrt(z);
    a.x /= s; a.y /= s; a.z /= s;
  }
  return a;
}
static inline M3f identity3() {
  M3f r{};
  r.m[0][0] = r.m[1][1] = r.m[2][2] = 1.f;
  return r;
}
static inline M4f identity4() {
  M4f r{};
  for (int i = 0; i < 4; ++i) r.m[i][i] = 1.f;
  return r;
}
// 3x3 * 3x3 and 3x3 * 3: coefficient-based product, a0b0 + (a1b1 + a2b2).
static inline M3f mul33(const M3f& a, const M3f& b) {
  M3f r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      r.m[i][j] = a.m[i][0] * b.m[0][j] + (a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j]);
  return r;
}
static inline V3f mul3v(const M3f& a, const V3f& v) {
  return {a.m[0][0] * v.x + (a.m[0][1] * v.y + a.m[0][2] * v.z),
          a.m[1][0] * v.x + (a.m[1][1] * v.y + a.m[1][2] * v.z),
          a.m[2][0] * v.x + (a.m[2][1] * v.y + a.m[2][2] * v.z)};
}
// 4x4 * 4x4: vectorised lazy product, ((a0b0 + a1b1) + a2b2) + a3b3.
static inline M4f mul44(const M4f& a, const M4f& b) {
  M4f r;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      r.m[i][j] = ((a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j]) + a.m[i][2] * b.m[2][j]) +
                  a.m[i][3] * b.m[3][j];
  return r;
}
// Rodrigues-style matrix used by computer_transform / transform_cluster / fuse_answer:
// R = c*I + (1-c)*r r^T + s*[r]x, element-wise left to right.
static inline M3f rodrigues(float c, float s, const V3f& r) {
  const float rv[3] = {r.x, r.y, r.z};
  const float rx[3][3] = {{0, -r.z, r.y}, {r.z, 0, -r.x}, {-r.y, r.x, 0}};
  const M3f I = identity3();
  M3f R;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      R.m[i][j] = (c * I.m[i][j] + (1 - c) * (rv[i] * rv[j])) + s * rx[i][j];
  return R;
}

// double Vector3 (SSE2-vectorised redux): (a0b0 + a1b1) + a2b2.
static inline double dotd(const double a[3], const double b[3]) {
  return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2];
}
static inline double normd(const double a[3]) { return std::sqrt(dotd(a, a)); }

// float transcendental convention.
static inline float acos_f(float x) { return (float)std::acos((double)x); }
static inline float atan2_f(float y, float x) { return (float)std::atan2((double)y, (double)x); }
static inline float cos_f(float x) { return (float)std::cos((double)x); }
static inline float sin_f(float x) { return (float)std::sin((double)x); }

// ------------------------------------------------------ predicates (:369-407)
// The acos convention of FCCF.cpp:374 `float theta=acos(cos_theta)*180/M_PI;`
// (cos_theta is float, no `using namespace std` in FCCF.cpp).  Which overload
// the unqualified call binds to depends on whether some PCL/VTK/FLANN header
// brought libstdc++'s <math.h> wrapper (`using std::acos;`) into the global
// namespace, and acosf's last bit on the glibc the reference was built with.
// The three candidates are switchable (orc_set_acos_mode) so that a test can
// count the threshold decisions that would flip between them:
//   ACOS_CR_FLOAT   float overload, correctly rounded acosf (the default and
//                   the convention the HIP product's cosine cut points follow)
//   ACOS_LIBM_FLOAT float overload, this host's glibc acosf
//   ACOS_DOUBLE     C's double acos: the whole expression in double, then float
enum { ACOS_CR_FLOAT = 0, ACOS_LIBM_FLOAT = 1, ACOS_DOUBLE = 2, ACOS_MODES = 3 };
static int g_acos_mode = ACOS_CR_FLOAT;
static float theta_of_cos(float cos_theta, int mode) {
  switch (mode) {
    case ACOS_LIBM_FLOAT: return (float)((double)(::acosf(cos_theta) * 180.0f) / M_PI);
    case ACOS_DOUBLE: return (float)(std::acos((double)cos_theta) * 180.0 / M_PI);
    default: return (float)((double)(acos_f(cos_theta) * 180.0f) / M_PI);
  }
}
static float normal_cos(float x1, float y1, float z1, float x2, float y2, float z2) {
  const double n1[3] = {x1, y1, z1}, n2[3] = {x2, y2, z2};
  float n1n3 = (float)dotd(n1, n2);
  return (float)((double)n1n3 / (normd(n1) * normd(n2)));
}
static float compute_normal_angel(float x1, float y1, float z1, float x2, float y2, float z2) {
  return theta_of_cos(normal_cos(x1, y1, z1, x2, y2, z2), g_acos_mode);
}

// Decision audit: every thresholded use of the angle (sites below) evaluates
// its predicate under all three conventions; `flips` counts the evaluations
// where the conventions disagree, `differ` those where the angles' bits do.
enum { SITE_GROW = 0, SITE_MERGE, SITE_ROUGH, SITE_BASE, SITE_THIRD, SITE_CLUSTER, SITE_VERIFY, SITE_PAIR, SITE_N, SITE_ANGLE_ONLY = SITE_N };
struct AcosAudit { uint64_t evals[SITE_N + 1], differ[SITE_N + 1], flips[SITE_N + 1]; };
static AcosAudit g_audit;
// Records one evaluation of a decision whose inputs under the three conventions
// are v[] (angles or quantities derived from them) and whose outcomes are d[].
template <class T>
static void audit_site(int site, const T v[ACOS_MODES], const bool d[ACOS_MODES]) {
  g_audit.evals[site]++;
  if (std::memcmp(&v[0], &v[1], sizeof(T)) || std::memcmp(&v[0], &v[2], sizeof(T))) g_audit.differ[site]++;
  if (d[0] != d[1] || d[0] != d[2]) g_audit.flips[site]++;
}
template <class Pred>
static bool angle_decide(int site, float x1, float y1, float z1, float x2, float y2, float z2, Pred pred,
                         float* theta_out = nullptr, float* all_out = nullptr) {
  const float c = normal_cos(x1, y1, z1, x2, y2, z2);
  float th[ACOS_MODES];
  bool d[ACOS_MODES];
  for (int m = 0; m < ACOS_MODES; ++m) { th[m] = theta_of_cos(c, m); d[m] = pred(th[m]); }
  audit_site(site, th, d);
  if (theta_out) *theta_out = th[g_acos_mode];
  if (all_out) std::memcpy(all_out, th, sizeof th);
  return d[g_acos_mode];
}
static bool compare_normal(int site, float x1, float y1, float z1, float x2, float y2, float z2, float thr) {
  return angle_decide(site, x1, y1, z1, x2, y2, z2, [thr](float t) { return !(t > thr); });
}
static bool compare_plane(float nx1, float ny1, float nz1, float cx1, float cy1, float cz1, float nx2,
                          float ny2, float nz2, float cx2, float cy2, float cz2, float l, float k) {
  const double n1[3] = {nx1, ny1, nz1}, n2[3] = {nx2, ny2, nz2};
  float len = std::sqrt((cx1 - cx2) * (cx1 - cx2) + (cy1 - cy2) * (cy1 - cy2) + (cz1 - cz2) * (cz1 - cz2));
  const double n3[3] = {(double)((cx1 - cx2) / len), (double)((cy1 - cy2) / len), (double)((cz1 - cz2) / len)};
  float n1n3 = (float)std::fabs(dotd(n1, n3));
  float n2n3 = (float)std::fabs(dotd(n2, n3));
  float thr = l / (k * len + 1);
  return n1n3 < thr && n2n3 < thr;
}

// ------------------------------------------------------ Eigen quaternion (3.3)
struct Qf { float w, x, y, z; };
static Qf quat_from_rot(const M3f& R) {
  Qf q;
  float t = R.m[0][0] + (R.m[1][1] + R.m[2][2]);  // trace(): diagonal redux
  if (t > 0.f) {
    t = std::sqrt(t + 1.0f);
    q.w = 0.5f * t;
    t = 0.5f / t;
    q.x = (R.m[2][1] - R.m[1][2]) * t;
    q.y = (R.m[0][2] - R.m[2][0]) * t;
    q.z = (R.m[1][0] - R.m[0][1]) * t;
  } else {
    int i = 0;
    if (R.m[1][1] > R.m[0][0]) i = 1;
    if (R.m[2][2] > R.m[i][i]) i = 2;
    int j = (i + 1) % 3, k = (j + 1) % 3;
    t = std::sqrt(R.m[i][i] - R.m[j][j] - R.m[k][k] + 1.0f);
    float c[3];
    c[i] = 0.5f * t;
    t = 0.5f / t;
    q.w = (R.m[k][j] - R.m[j][k]) * t;
    c[j] = (R.m[j][i] + R.m[i][j]) * t;
    c[k] = (R.m[k][i] + R.m[i][k]) * t;
    q.x = c[0]; q.y = c[1]; q.z = c[2];
  }
  return q;
}
static M3f rot_from_quat(const Qf& q) {
  const float tx = 2.f * q.x, ty = 2.f * q.y, tz = 2.f * q.z;
  const float twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const float txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const float tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  M3f r;
  r.m[0][0] = 1.f - (tyy + tzz); r.m[0][1] = txy - twz; r.m[0][2] = txz + twy;
  r.m[1][0] = txy + twz; r.m[1][1] = 1.f - (txx + tzz); r.m[1][2] = tyz - twx;
  r.m[2][0] = txz - twy; r.m[2][1] = tyz + twx; r.m[2][2] = 1.f - (txx + tyy);
  return r;
}
// quat_transform_vector: uv = q.vec x v; uv += uv; v + w*uv + q.vec x uv.
static V3f quat_rotate(const Qf& q, const V3f& v) {
  V3f qv = {q.x, q.y, q.z};
  V3f uv = crossf(qv, v);
  uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
  V3f c = crossf(qv, uv);
  return {(v.x + q.w * uv.x) + c.x, (v.y + q.w * uv.y) + c.y, (v.z + q.w * uv.z) + c.z};
}

// ------------------------------------------------------ PCL Transformer<float>
static inline V3f tf_se3(const M4f& T, float x, float y, float z) {
  return {x * T.m[0][0] + (y * T.m[0][1] + (z * T.m[0][2] + T.m[0][3])),
          x * T.m[1][0] + (y * T.m[1][1] + (z * T.m[1][2] + T.m[1][3])),
          x * T.m[2][0] + (y * T.m[2][1] + (z * T.m[2][2] + T.m[2][3]))};
}
static inline V3f tf_so3(const M4f& T, float x, float y, float z) {
  return {x * T.m[0][0] + (y * T.m[0][1] + z * T.m[0][2]),
          x * T.m[1][0] + (y * T.m[1][1] + z * T.m[1][2]),
          x * T.m[2][0] + (y * T.m[2][1] + z * T.m[2][2])};
}

// ------------------------------------------------------ named intermediates
struct Store {
  std::map<std::string, std::vector<uint8_t>> blobs;
  template <class T>
  void put(const std::string& k, const std::vector<T>& v) {
    auto& b = blobs[k];
    b.resize(v.size() * sizeof(T));
    if (!v.empty()) std::memcpy(b.data(), v.data(), b.size());
  }
  template <class T>
  void put1(const std::string& k, const T& v) { put(k, std::vector<T>{v}); }
};

using Cloud = std::vector<float>;  // xyz interleaved
static inline size_t npts(const Cloud& c) { return c.size() / 3; }

// ------------------------------------------------------ VoxelGrid (App. A2)
struct IdxPair {  // pcl::cloud_point_index_idx
  unsigned int idx, cloud_point_index;
  bool operator<(const IdxPair& p) const { return idx < p.idx; }
};

static Cloud voxel_grid(const Cloud& in, float leaf, int order, int* overflow) {
  const size_t n = npts(in);
  const float inv = 1.0f / leaf;
  float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
  size_t nfinite = 0;
  for (size_t i = 0; i < n; ++i) {
    const float* p = &in[3 * i];
    if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) continue;
    ++nfinite;
    for (int a = 0; a < 3; ++a) {
      mn[a] = std::min(mn[a], p[a]);
      mx[a] = std::max(mx[a], p[a]);
    }
  }
  if (nfinite == 0) return Cloud();
  int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
  int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
  int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
  if (dx * dy * dz > (int64_t)INT32_MAX) {  // "Integer indices would overflow": output = input
    if (overflow) *overflow = 1;
    return in;
  }
  int min_b[3], max_b[3], div_b[3];
  for (int a = 0; a < 3; ++a) {
    min_b[a] = (int)std::floor(mn[a] * inv);
    max_b[a] = (int)std::floor(mx[a] * inv);
    div_b[a] = max_b[a] - min_b[a] + 1;
  }
  const int64_t mul1 = div_b[0], mul2 = (int64_t)div_b[0] * div_b[1];
  std::vector<IdxPair> iv;
  iv.reserve(nfinite);
  for (size_t i = 0; i < n; ++i) {
    const float* p = &in[3 * i];
    if (!std::isfinite(p[0]) || !std::isfinite(p[1]) || !std::isfinite(p[2])) continue;
    int i0 = (int)(std::floor(p[0] * inv) - (float)min_b[0]);
    int i1 = (int)(std::floor(p[1] * inv) - (float)min_b[1]);
    int i2 = (int)(std::floor(p[2] * inv) - (float)min_b[2]);
    int64_t idx = (int64_t)i0 + (int64_t)i1 * mul1 + (int64_t)i2 * mul2;
    iv.push_back({(unsigned int)(uint32_t)idx, (unsigned int)i});
  }
  if (order == ORC_ORDER_INTROSORT)
    std::sort(iv.begin(), iv.end(), std::less<IdxPair>());
  else
    std::stable_sort(iv.begin(), iv.end(), std::less<IdxPair>());
  Cloud out;
  out.reserve(3 * iv.size());
  size_t s = 0;
  while (s < iv.size()) {
    size_t e = s + 1;
    while (e < iv.size() && iv[e].idx == iv[s].idx) ++e;
    float sx = 0.f, sy = 0.f, sz = 0.f;  // CentroidPoint / AccumulatorXYZ: Vector3f +=
    for (size_t k = s; k < e; ++k) {
      const float* p = &in[3 * iv[k].cloud_point_index];
      sx += p[0]; sy += p[1]; sz += p[2];
    }
    const float cnt = (float)(e - s);
    out.push_back(sx / cnt); out.push_back(sy / cnt); out.push_back(sz / cnt);
    s = e;
  }
  return out;
}

static Cloud remove_nan(const Cloud& in) {
  Cloud out;
  out.reserve(in.size());
  for (size_t i = 0; i < npts(in); ++i) {
    const float* p = &in[3 * i];
    if (std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2])) out.insert(out.end(), p, p + 3);
  }
  return out;
}

// ------------------------------------------------------ octree (App. A3)
struct OctBounds {
  double min[3] = {0, 0, 0}, max[3] = {0, 0, 0};
  unsigned depth = 0;
  bool defined = false;
};

static void oct_key_bit_size_first(OctBounds& b, double res) {
  const float minValue = FLT_EPSILON;
  unsigned mk[3];
  for (int a = 0; a < 3; ++a) mk[a] = (unsigned)std::ceil((b.max[a] - b.min[a] - minValue) / res);
  unsigned max_voxels = std::max(std::max(std::max(mk[0], mk[1]), mk[2]), 2u);
  unsigned d = (unsigned)std::ceil(std::log((double)max_voxels) / std::log(2.0) - minValue);
  b.depth = std::max(std::min(32u, d), 0u);
  const double side = (double)(1u << b.depth) * res;
  for (int a = 0; a < 3; ++a) {  // leaf_count_ == 0 branch
    double over = (side - (b.max[a] - b.min[a])) / 2.0;
    if (over > minValue) {
      b.min[a] -= over;
      b.max[a] += over;
    }
  }
}

static void oct_adopt(OctBounds& b, double res, const float* p) {
  const float minValue = FLT_EPSILON;
  while (true) {
    bool lo[3], up[3], any = !b.defined;
    for (int a = 0; a < 3; ++a) {
      lo[a] = (double)p[a] < b.min[a];
      up[a] = (double)p[a] >= b.max[a];
      any = any || lo[a] || up[a];
    }
    if (!any) break;
    if (b.defined) {
      double side = (double)(1 << b.depth) * res;
      for (int a = 0; a < 3; ++a)
        if (!up[a]) b.min[a] -= side;
      b.depth++;
      side = (double)(1 << b.depth) * res - minValue;
      for (int a = 0; a < 3; ++a) b.max[a] = b.min[a] + side;
    } else {
      for (int a = 0; a < 3; ++a) {
        b.min[a] = (double)p[a] - res / 2;
        b.max[a] = (double)p[a] + res / 2;
      }
      oct_key_bit_size_first(b, res);
      b.defined = true;
    }
  }
}

static inline uint64_t morton3(uint32_t kx, uint32_t ky, uint32_t kz, unsigned depth) {
  uint64_t m = 0;
  for (int bit = (int)depth - 1; bit >= 0; --bit)
    m = (m << 3) | ((uint64_t)((kx >> bit) & 1) << 2) | ((uint64_t)((ky >> bit) & 1) << 1) |
        (uint64_t)((kz >> bit) & 1);
  return m;
}

// Occupied leaves in getOccupiedVoxelCenters (DFS = Morton, x most significant)
// order; each leaf lists its point indices in insertion (ascending) order.
struct Leaves {
  std::vector<uint64_t> code;
  std::vector<uint32_t> start;  // CSR into idx
  std::vector<uint32_t> idx;
  OctBounds b;
};

static inline bool finite3(const float* p) {
  return std::isfinite(p[0]) && std::isfinite(p[1]) && std::isfinite(p[2]);
}

// PCL's OctreePointCloudSearch structure (octree_base.hpp / octree_pointcloud.hpp):
// branch nodes with eight child pointers, leaf containers holding the point indices in
// insertion order, a DFS over the children in index order (x bit most significant) for
// the occupied leaves.  The oracle's result does not depend on the structure (the
// Morton stable sort below yields the same leaves, checked in test_oracle_kat.py); it
// is kept so that the CPU baseline times PCL's algorithm (pointer chasing, one heap
// vector per leaf), SURVEY.md §8(d).  orc_set_octree_mode(0) selects the sort.
struct PclOctNode {
  PclOctNode* child[8] = {};
  std::vector<uint32_t>* leaf = nullptr;  // a leaf node's container
  ~PclOctNode() {
    for (PclOctNode* c : child) delete c;
    delete leaf;
  }
};
static int g_octree_mode = 1;  // 1: PCL pointer octree, 0: Morton stable sort

static void pcl_dfs(const PclOctNode* nd, uint64_t code, unsigned level, unsigned depth, Leaves& L) {
  if (level == depth) {
    L.code.push_back(code);
    L.start.push_back((uint32_t)L.idx.size());
    L.idx.insert(L.idx.end(), nd->leaf->begin(), nd->leaf->end());
    return;
  }
  for (unsigned c = 0; c < 8; ++c)
    if (nd->child[c]) pcl_dfs(nd->child[c], (code << 3) | c, level + 1, depth, L);
}

// addPointsFromInputCloud skips non-finite points (isFinite), so they belong to no leaf.
static Leaves octree_leaves(const float* xyz, size_t n, double res) {
  Leaves L;
  for (size_t i = 0; i < n; ++i)
    if (finite3(&xyz[3 * i])) oct_adopt(L.b, res, &xyz[3 * i]);
  if (g_octree_mode == 1) {
    PclOctNode root;
    const unsigned depth = L.b.depth;
    for (size_t i = 0; i < n; ++i) {
      if (!finite3(&xyz[3 * i])) continue;
      uint32_t k[3];
      for (int a = 0; a < 3; ++a) k[a] = (uint32_t)(((double)xyz[3 * i + a] - L.b.min[a]) / res);
      PclOctNode* nd = &root;
      for (int bit = (int)depth - 1; bit >= 0; --bit) {  // createLeafRecursive
        const unsigned c = (((k[0] >> bit) & 1u) << 2) | (((k[1] >> bit) & 1u) << 1) | ((k[2] >> bit) & 1u);
        if (!nd->child[c]) nd->child[c] = new PclOctNode();
        nd = nd->child[c];
      }
      if (!nd->leaf) nd->leaf = new std::vector<uint32_t>();
      nd->leaf->push_back((uint32_t)i);
    }
    if (depth == 0) {
      if (root.leaf) pcl_dfs(&root, 0, 0, 0, L);
    } else {
      pcl_dfs(&root, 0, 0, depth, L);
    }
    L.start.push_back((uint32_t)L.idx.size());
    return L;
  }
  std::vector<std::pair<uint64_t, uint32_t>> kv;
  kv.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    if (!finite3(&xyz[3 * i])) continue;
    uint32_t k[3];
    for (int a = 0; a < 3; ++a) k[a] = (uint32_t)(((double)xyz[3 * i + a] - L.b.min[a]) / res);
    kv.push_back({morton3(k[0], k[1], k[2], L.b.depth), (uint32_t)i});
  }
  n = kv.size();
  std::stable_sort(kv.begin(), kv.end(),
                   [](const std::pair<uint64_t, uint32_t>& a, const std::pair<uint64_t, uint32_t>& b) {
                     return a.first < b.first;
                   });
  L.idx.resize(n);
  for (size_t i = 0; i < n; ++i) {
    if (i == 0 || kv[i].first != kv[i - 1].first) {
      L.code.push_back(kv[i].first);
      L.start.push_back((uint32_t)i);
    }
    L.idx[i] = kv[i].second;
  }
  L.start.push_back((uint32_t)n);
  return L;
}

// ------------------------------------------------------ normals (App. A4-A6)
static void compute_roots2(float b, float c, float roots[3]) {
  roots[0] = 0.f;
  float d = (float)((double)(b * b) - 4.0 * (double)c);
  if (d < 0.0) d = 0.0;
  float sd = std::sqrt(d);
  roots[2] = 0.5f * (b + sd);
  roots[1] = 0.5f * (b - sd);
}

static void compute_roots(const float m[3][3], float roots[3]) {
  float c0 = m[0][0] * m[1][1] * m[2][2] + 2.f * m[0][1] * m[0][2] * m[1][2] - m[0][0] * m[1][2] * m[1][2] -
             m[1][1] * m[0][2] * m[0][2] - m[2][2] * m[0][1] * m[0][1];
  float c1 = m[0][0] * m[1][1] - m[0][1] * m[0][1] + m[0][0] * m[2][2] - m[0][2] * m[0][2] +
             m[1][1] * m[2][2] - m[1][2] * m[1][2];
  float c2 = m[0][0] + m[1][1] + m[2][2];
  if (std::fabs(c0) < FLT_EPSILON) {
    compute_roots2(c2, c1, roots);
    return;
  }
  const float s_inv3 = (float)(1.0 / 3.0);
  const float s_sqrt3 = std::sqrt(3.0f);
  float c2_over_3 = c2 * s_inv3;
  float a_over_3 = (c1 - c2 * c2_over_3) * s_inv3;
  if (a_over_3 > 0.f) a_over_3 = 0.f;
  float half_b = 0.5f * (c0 + c2_over_3 * (2.f * c2_over_3 * c2_over_3 - c1));
  float q = half_b * half_b + a_over_3 * a_over_3 * a_over_3;
  if (q > 0.f) q = 0.f;
  float rho = std::sqrt(-a_over_3);
  float theta = atan2_f(std::sqrt(-q), half_b) * s_inv3;
  float cos_theta = cos_f(theta);
  float sin_theta = sin_f(theta);
  roots[0] = c2_over_3 + 2.f * rho * cos_theta;
  roots[1] = c2_over_3 - rho * (cos_theta + s_sqrt3 * sin_theta);
  roots[2] = c2_over_3 - rho * (cos_theta - s_sqrt3 * sin_theta);
  if (roots[0] >= roots[1]) std::swap(roots[0], roots[1]);
  if (roots[1] >= roots[2]) {
    std::swap(roots[1], roots[2]);
    if (roots[0] >= roots[1]) std::swap(roots[0], roots[1]);
  }
  if (roots[0] <= 0.f) compute_roots2(c2, c1, roots);
}

static void eigen33(const float mat[3][3], float& eigenvalue, V3f& vec) {
  float scale = 0.f;
  for (int i = 0; i < 3; ++i)  // cwiseAbs().maxCoeff(): column-major scan, first max wins
    for (int j = 0; j < 3; ++j) scale = std::max(scale, std::fabs(mat[j][i]));
  if (scale <= FLT_MIN) scale = 1.0f;
  float s[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) s[i][j] = mat[i][j] / scale;
  float roots[3];
  compute_roots(s, roots);
  eigenvalue = roots[0] * scale;
  for (int i = 0; i < 3; ++i) s[i][i] -= roots[0];
  V3f r0 = {s[0][0], s[0][1], s[0][2]}, r1 = {s[1][0], s[1][1], s[1][2]}, r2 = {s[2][0], s[2][1], s[2][2]};
  V3f v1 = crossf(r0, r1), v2 = crossf(r0, r2), v3 = crossf(r1, r2);
  float l1 = sqnormf(v1), l2 = sqnormf(v2), l3 = sqnormf(v3);
  V3f v;
  float d;
  if (l1 >= l2 && l1 >= l3) { v = v1; d = std::sqrt(l1); }
  else if (l2 >= l1 && l2 >= l3) { v = v2; d = std::sqrt(l2); }
  else { v = v3; d = std::sqrt(l3); }
  vec = {v.x / d, v.y / d, v.z / d};
}

// computeMeanAndCovarianceMatrix (PCL 1.10, unshifted single pass) + solvePlaneParameters.
static void point_normal(const float* xyz, const uint32_t* idx, size_t n, float& nx, float& ny, float& nz,
                         float& curvature) {
  if (n < 3) {
    nx = ny = nz = curvature = std::numeric_limits<float>::quiet_NaN();
    return;
  }
  float accu[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
  for (size_t k = 0; k < n; ++k) {
    const float* p = &xyz[3 * idx[k]];
    accu[0] += p[0] * p[0]; accu[1] += p[0] * p[1]; accu[2] += p[0] * p[2];
    accu[3] += p[1] * p[1]; accu[4] += p[1] * p[2]; accu[5] += p[2] * p[2];
    accu[6] += p[0]; accu[7] += p[1]; accu[8] += p[2];
  }
  const float fn = (float)n;
  for (float& a : accu) a /= fn;
  float cov[3][3];
  cov[0][0] = accu[0] - accu[6] * accu[6];
  cov[0][1] = accu[1] - accu[6] * accu[7];
  cov[0][2] = accu[2] - accu[6] * accu[8];
  cov[1][1] = accu[3] - accu[7] * accu[7];
  cov[1][2] = accu[4] - accu[7] * accu[8];
  cov[2][2] = accu[5] - accu[8] * accu[8];
  // covariance_matrix is column-major; coeffRef(1)=(1,0), (2)=(2,0), (5)=(2,1) were
  // written above as (0,1),(0,2),(1,2) of the transpose; it is symmetric.
  cov[1][0] = cov[0][1]; cov[2][0] = cov[0][2]; cov[2][1] = cov[1][2];
  float ev;
  V3f v;
  eigen33(cov, ev, v);
  nx = v.x; ny = v.y; nz = v.z;
  float eig_sum = cov[0][0] + cov[1][1] + cov[2][2];
  curvature = (eig_sum != 0.f) ? std::fabs(ev / eig_sum) : 0.f;
}

// ------------------------------------------------------ face_extrate (:470-678)
struct Voxel { float c[3], n[3]; int size; };
struct Face {
  float ac[3], an[3];   // average_centry_*, average_normal_*
  float fps;            // face_point_size
  bool alloc;
  std::vector<int> members;  // voxelgrothnode (indices into voxel vector)
};

struct FaceOut {
  std::vector<Face> planes;     // face_vecter (<= 16)
  std::vector<double> theta;    // new_theta_vector
  std::vector<Voxel> voxels;    // planar voxels
  Cloud residual;               // cloud_sub
  float centroid[4];
  double oct[4];
  std::vector<int32_t> vstat;   // per occupied voxel: count, flag (0 dropped,1 planar,2 residual)
  std::vector<float> vcurv;
  std::vector<Face> groups_all; // after stage 2 + range_face
};

static void face_recompute(Face& f, const std::vector<Voxel>& vox) {
  float s = 0, cx = 0, cy = 0, cz = 0, nx = 0, ny = 0, nz = 0;
  for (int m : f.members) {
    const Voxel& v = vox[m];
    s = s + v.size;
    cx = cx + v.c[0] * v.size; cy = cy + v.c[1] * v.size; cz = cz + v.c[2] * v.size;
    nx = nx + v.n[0] * v.size; ny = ny + v.n[1] * v.size; nz = nz + v.n[2] * v.size;
  }
  f.fps = s;
  f.ac[0] = cx / s; f.ac[1] = cy / s; f.ac[2] = cz / s;
  f.an[0] = nx / s; f.an[1] = ny / s; f.an[2] = nz / s;
}

static void grow_select(const Params& P, FaceOut& out);
static void face_extrate(const Cloud& cloud, const Params& P, FaceOut& out) {
  const size_t n = npts(cloud);
  // compute3DCentroid (dense): sequential float sums / n
  float c4[4] = {0, 0, 0, 0};
  if (n) {
    for (size_t i = 0; i < n; ++i) {
      c4[0] += cloud[3 * i]; c4[1] += cloud[3 * i + 1]; c4[2] += cloud[3 * i + 2];
    }
    const float fn = (float)n;
    c4[0] /= fn; c4[1] /= fn; c4[2] /= fn; c4[3] = 1;
  }
  std::memcpy(out.centroid, c4, sizeof c4);
  const double res = (double)P.face_voxel_size;
  Leaves L = octree_leaves(cloud.data(), n, res);
  out.oct[0] = L.b.min[0]; out.oct[1] = L.b.min[1]; out.oct[2] = L.b.min[2]; out.oct[3] = L.b.depth;
  std::vector<Voxel>& vox = out.voxels;
  for (size_t v = 0; v + 1 < L.start.size(); ++v) {
    const uint32_t* idx = &L.idx[L.start[v]];
    const size_t cnt = L.start[v + 1] - L.start[v];
    int32_t flag = 0;
    float curv = 0;
    if ((float)cnt > P.voxel_point_threshold) {
      float cx = 0, cy = 0, cz = 0;
      for (size_t k = 0; k < cnt; ++k) {
        cx += cloud[3 * idx[k]]; cy += cloud[3 * idx[k] + 1]; cz += cloud[3 * idx[k] + 2];
      }
      const float fc = (float)cnt;
      cx /= fc; cy /= fc; cz /= fc;
      float nx, ny, nz;
      point_normal(cloud.data(), idx, cnt, nx, ny, nz, curv);
      if (curv < P.curvature_threshold) {
        Voxel vx;
        vx.c[0] = cx; vx.c[1] = cy; vx.c[2] = cz;
        vx.size = (int)cnt;
        V3f to = {cx - c4[0], cy - c4[1], cz - c4[2]}, nv = {nx, ny, nz};
        if (dotf(to, nv) < 0) { vx.n[0] = nx; vx.n[1] = ny; vx.n[2] = nz; }
        else { vx.n[0] = -nx; vx.n[1] = -ny; vx.n[2] = -nz; }
        vox.push_back(vx);
        flag = 1;
      } else {
        for (size_t k = 0; k < cnt; ++k) out.residual.insert(out.residual.end(), &cloud[3 * idx[k]], &cloud[3 * idx[k]] + 3);
        flag = 2;
      }
    }
    out.vstat.push_back((int32_t)cnt);
    out.vstat.push_back(flag);
    out.vcurv.push_back(curv);
  }

  grow_select(P, out);
}

// Region growing stages 1-2, range_face and the selection with roughness
// (:536-677) over out.voxels; fills planes, theta and groups_all.
static void grow_select(const Params& P, FaceOut& out) {
  const std::vector<Voxel>& vox = out.voxels;
  // stage 1: greedy seed growth (:536-593)
  std::vector<char> valloc(vox.size(), 0);
  std::vector<Face> groth;
  for (size_t i = 0; i < vox.size(); ++i) {
    if (valloc[i]) continue;
    Face f;
    valloc[i] = 1;
    f.members.push_back((int)i);
    f.fps = (float)vox[i].size;
    for (int a = 0; a < 3; ++a) { f.an[a] = vox[i].n[a]; f.ac[a] = vox[i].c[a]; }
    for (size_t j = 0; j < vox.size(); ++j) {
      if (valloc[j]) continue;
      bool same = compare_normal(SITE_GROW, f.an[0], f.an[1], f.an[2], vox[j].n[0], vox[j].n[1], vox[j].n[2],
                                 P.normal_vector_threshold1);
      bool cop = compare_plane(f.an[0], f.an[1], f.an[2], f.ac[0], f.ac[1], f.ac[2], vox[j].n[0], vox[j].n[1],
                               vox[j].n[2], vox[j].c[0], vox[j].c[1], vox[j].c[2], P.parameter_l1, P.parameter_k1);
      if (same && cop) {
        f.members.push_back((int)j);
        valloc[j] = 1;
        face_recompute(f, vox);
      }
    }
    f.alloc = false;
    groth.push_back(std::move(f));
  }
  // stage 2: iterative merge (:595-648); seeds never mark themselves allocated.
  for (size_t i = 0; i < groth.size(); ++i) {
    if (groth[i].alloc) continue;
    bool newadd = true;
    while (newadd) {
      newadd = false;
      for (size_t j = 0; j < groth.size(); ++j) {
        if (j == i || groth[j].alloc) continue;
        Face& a = groth[i];
        Face& b = groth[j];
        bool same = compare_normal(SITE_MERGE, a.an[0], a.an[1], a.an[2], b.an[0], b.an[1], b.an[2],
                                   P.normal_vector_threshold2);
        bool cop = compare_plane(a.an[0], a.an[1], a.an[2], a.ac[0], a.ac[1], a.ac[2], b.an[0], b.an[1], b.an[2],
                                 b.ac[0], b.ac[1], b.ac[2], P.parameter_l2, P.parameter_k2);
        if (same && cop) {
          newadd = true;
          b.alloc = true;
          a.members.insert(a.members.end(), b.members.begin(), b.members.end());
          face_recompute(a, vox);
        }
      }
    }
  }
  // range_face (:409-427): exchange sort by member count.
  for (size_t i = 0; i + 1 < groth.size(); ++i)
    for (size_t j = i + 1; j < groth.size(); ++j)
      if (groth[i].members.size() < groth[j].members.size()) std::swap(groth[i], groth[j]);
  out.groups_all = groth;
  // selection + roughness (:652-675)
  int cur = 0;
  for (size_t i = 0; i < groth.size(); ++i) {
    const Face& f = groth[i];
    if (!f.alloc) {
      out.planes.push_back(f);
      double sum = 0, alt[ACOS_MODES] = {0, 0, 0};
      for (int m : f.members) {
        float thf, tha[ACOS_MODES];
        angle_decide(SITE_ANGLE_ONLY, f.an[0], f.an[1], f.an[2], vox[m].n[0], vox[m].n[1], vox[m].n[2],
                     [](float) { return false; }, &thf, tha);
        double th = thf;
        sum += std::fabs(th);
        for (int a = 0; a < ACOS_MODES; ++a) alt[a] += std::fabs((double)tha[a]);
      }
      sum /= (double)f.members.size();
      out.theta.push_back(sum);
      // the roughness class select_base derives from it (:445-452)
      bool rd[ACOS_MODES];
      for (int a = 0; a < ACOS_MODES; ++a) {
        alt[a] /= (double)f.members.size();
        rd[a] = alt[a] <= (double)P.rough_threshold_gl;
      }
      audit_site(SITE_ROUGH, alt, rd);
      cur++;
    }
    if (cur > P.select_plane_number) break;
  }
}

// ------------------------------------------------------ select_base (:429-468)
struct Base { int i1, i2; float angle; float alt[3]; };
static void select_base(const std::vector<Face>& F, const std::vector<double>& th, const Params& P,
                        std::vector<Base>& base, std::vector<int>& type) {
  const double t1 = P.rough_threshold_gl;
  for (size_t i = 0; i < F.size(); ++i)
    for (size_t j = 0; j < F.size(); ++j) {
      if (!(i < j)) continue;
      float ang, alt[ACOS_MODES];
      const float lo = P.included_angle_min_threshold, hi = P.included_angle_max_threshold;
      if (angle_decide(SITE_BASE, F[i].an[0], F[i].an[1], F[i].an[2], F[j].an[0], F[j].an[1], F[j].an[2],
                       [lo, hi](float t) { return lo < t && t < hi; }, &ang, alt)) {
        base.push_back({(int)i, (int)j, ang, {alt[0], alt[1], alt[2]}});
        if (th[i] <= t1 && th[j] <= t1) type.push_back(0);
        else if (th[i] > t1 && th[j] > t1) type.push_back(1);
        else if (th[i] <= t1 && th[j] > t1) type.push_back(2);
        else if (th[i] > t1 && th[j] <= t1) type.push_back(2);
      }
    }
}

// ------------------------------------------------------ computer_transform (:841-1018)
static void computer_transform(std::vector<M4f>* out, int i11, int i12, int i21, int i22, const std::vector<Face>& F1,
                               const std::vector<Face>& F2, int type, const Params& P) {
  M4f T = identity4();
  V3f n1 = {F1[i11].an[0], F1[i11].an[1], F1[i11].an[2]};
  V3f m1 = {F1[i12].an[0], F1[i12].an[1], F1[i12].an[2]};
  V3f n2 = {F2[i21].an[0], F2[i21].an[1], F2[i21].an[2]};
  V3f m2 = {F2[i22].an[0], F2[i22].an[1], F2[i22].an[2]};
  V3f r1 = normalizedf(crossf(n2, n1));
  float n2dn1 = dotf(n2, n1);
  V3f r1cn2 = crossf(r1, n2);
  float r1cn2dn1 = dotf(r1cn2, n1);
  M3f R1 = rodrigues(n2dn1, r1cn2dn1, r1);
  m2 = mul3v(R1, m2);
  V3f r2 = n1;
  float m2dm1 = dotf(m2, m1), m2dr2 = dotf(m2, r2), m1dr2 = dotf(m1, r2);
  V3f r2cm2 = crossf(r2, m2);
  float r2cm2dm1 = dotf(r2cm2, m1);
  float cos2 = (m2dm1 - (m2dr2 * m1dr2)) / (1 - (m2dr2 * m1dr2));
  float sin2 = (r2cm2dm1) / (1 - (m2dr2 * m1dr2));
  M3f R2 = rodrigues(cos2, sin2, r2);
  M3f rot = mul33(R2, R1);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T.m[i][j] = rot.m[i][j];

  std::vector<int> three;
  V3f n1cm1 = normalizedf(crossf(n1, m1));
  for (size_t k = 0; k < F1.size(); ++k) {
    if ((int)k == i11 || (int)k == i12) continue;
    V3f nt = {F1[k].an[0], F1[k].an[1], F1[k].an[2]};
    if (std::fabs(dotf(n1cm1, nt)) > P.third_plane_threshold) three.push_back((int)k);
  }
  V3f n2cm2 = normalizedf(crossf(n2, m2));
  bool getthree = false;
  if (!three.empty()) {
    std::vector<V3f> pc(F2.size()), pn(F2.size());
    for (size_t k = 0; k < F2.size(); ++k) {
      pc[k] = tf_se3(T, F2[k].ac[0], F2[k].ac[1], F2[k].ac[2]);
      pn[k] = tf_so3(T, F2[k].an[0], F2[k].an[1], F2[k].an[2]);
    }
    for (int k3 : three) {
      for (size_t q = 0; q < F2.size(); ++q) {
        if ((int)q == i21 || (int)q == i22) continue;
        const float thr3 = P.third_plane_normal_threshold;
        const bool a3ok = angle_decide(SITE_THIRD, F1[k3].an[0], F1[k3].an[1], F1[k3].an[2], pn[q].x, pn[q].y,
                                       pn[q].z, [thr3](float t) { return t < thr3; });
        if (a3ok && std::fabs(dotf(n2cm2, pn[q])) > P.third_plane_threshold) {
          getthree = true;
          V3f k1 = {F1[k3].an[0], F1[k3].an[1], F1[k3].an[2]};
          V3f k2 = pn[q];
          V3f c11 = {F1[i11].ac[0], F1[i11].ac[1], F1[i11].ac[2]};
          V3f c12 = {F1[i12].ac[0], F1[i12].ac[1], F1[i12].ac[2]};
          V3f c13 = {F1[k3].ac[0], F1[k3].ac[1], F1[k3].ac[2]};
          V3f c21 = {F2[i21].ac[0], F2[i21].ac[1], F2[i21].ac[2]};
          V3f c22 = {F2[i22].ac[0], F2[i22].ac[1], F2[i22].ac[2]};
          V3f c23 = pc[q];
          float d11 = dotf(c11, n1), d12 = dotf(c12, m1), d13 = dotf(c13, k1);
          float d21 = dotf(c21, n2), d22 = dotf(c22, m2), d23 = dotf(c23, k2);
          V3f D = {d11 - d21, d12 - d22, d13 - d23};
          M3f A;
          A.m[0][0] = n1.x; A.m[0][1] = n1.y; A.m[0][2] = n1.z;
          A.m[1][0] = m1.x; A.m[1][1] = m1.y; A.m[1][2] = m1.z;
          A.m[2][0] = k1.x; A.m[2][1] = k1.y; A.m[2][2] = k1.z;
          M3f AT;
          for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) AT.m[i][j] = A.m[j][i];
          M3f M = mul33(AT, A);
          // Eigen 3x3 inverse: cofactors of column 0, det = c00*m00 + (c10*m10 + c20*m20)
          auto cof = [&](int i, int j) {
            int i1 = (i + 1) % 3, i2 = (i + 2) % 3, j1 = (j + 1) % 3, j2 = (j + 2) % 3;
            return M.m[i1][j1] * M.m[i2][j2] - M.m[i1][j2] * M.m[i2][j1];
          };
          float cc0 = cof(0, 0), cc1 = cof(1, 0), cc2 = cof(2, 0);
          float det = cc0 * M.m[0][0] + (cc1 * M.m[1][0] + cc2 * M.m[2][0]);
          float invdet = 1.f / det;
          M3f Mi;
          Mi.m[0][0] = cc0 * invdet; Mi.m[0][1] = cc1 * invdet; Mi.m[0][2] = cc2 * invdet;
          Mi.m[1][0] = cof(0, 1) * invdet; Mi.m[1][1] = cof(1, 1) * invdet; Mi.m[1][2] = cof(2, 1) * invdet;
          Mi.m[2][0] = cof(0, 2) * invdet; Mi.m[2][1] = cof(1, 2) * invdet; Mi.m[2][2] = cof(2, 2) * invdet;
          M3f MiAT = mul33(Mi, AT);
          V3f t = mul3v(MiAT, D);
          T.m[0][3] = t.x; T.m[1][3] = t.y; T.m[2][3] = t.z;
          out[type].push_back(T);
        }
      }
    }
  }
  if (!getthree) {
    const Face &a = F1[i11], &b = F1[i12], &c = F2[i21], &d = F2[i22];
    float sx = (a.ac[0] * a.fps + b.ac[0] * b.fps) / (a.fps + b.fps);
    float sy = (a.ac[1] * a.fps + b.ac[1] * b.fps) / (a.fps + b.fps);
    float sz = (a.ac[2] * a.fps + b.ac[2] * b.fps) / (a.fps + b.fps);
    float tx = (c.ac[0] * c.fps + d.ac[0] * d.fps) / (c.fps + d.fps);
    float ty = (c.ac[1] * c.fps + d.ac[1] * d.fps) / (c.fps + d.fps);
    float tz = (c.ac[2] * c.fps + d.ac[2] * d.fps) / (c.fps + d.fps);
    V3f tc = mul3v(rot, V3f{tx, ty, tz});
    T.m[0][3] = sx - tc.x; T.m[1][3] = sy - tc.y; T.m[2][3] = sz - tc.z;
    out[type].push_back(T);
  }
}

// ------------------------------------------------------ clustering (:1020-1231)
struct QT { float qw, qx, qy, qz, tx, ty, tz; bool alloc; };

// Rotation part built from two averaged axes (shared by transform_cluster :1148-1196
// and fuse_answer :1306-1354).
static M3f axes_to_rot(const V3f& nt1, const V3f& nt2) {
  const V3f ns1 = {1, 0, 0};
  V3f ns2 = {0, 1, 0};
  V3f r1 = normalizedf(crossf(ns1, nt1));
  float c1 = dotf(nt1, ns1);
  float s1 = dotf(nt1, crossf(r1, ns1));
  M3f R1 = rodrigues(c1, s1, r1);
  ns2 = mul3v(R1, ns2);
  V3f r2 = nt1;
  float ns2dnt2 = dotf(ns2, nt2), ns2dr2 = dotf(ns2, r2), nt2dr2 = dotf(nt2, r2);
  V3f r2cns2 = crossf(r2, ns2);
  float r2cns2dnt2 = dotf(r2cns2, nt2);
  float c2 = (ns2dnt2 - (ns2dr2 * nt2dr2)) / (1 - (ns2dr2 * nt2dr2));
  float s2 = (r2cns2dnt2) / (1 - (ns2dr2 * nt2dr2));
  M3f R2 = rodrigues(c2, s2, r2);
  return mul33(R2, R1);
}

static void average_normal(V3f& v1, V3f& v2, const std::vector<QT>& mv) {
  float sx1 = 0, sy1 = 0, sz1 = 0, sx2 = 0, sy2 = 0, sz2 = 0;
  for (const QT& t : mv) {
    Qf q = {t.qw, t.qx, t.qy, t.qz};
    V3f a = quat_rotate(q, V3f{1, 0, 0}), b = quat_rotate(q, V3f{0, 1, 0});
    sx1 = sx1 + a.x; sy1 = sy1 + a.y; sz1 = sz1 + a.z;
    sx2 = sx2 + b.x; sy2 = sy2 + b.y; sz2 = sz2 + b.z;
  }
  const float n = (float)mv.size();
  v1 = normalizedf(V3f{sx1 / n, sy1 / n, sz1 / n});
  v2 = normalizedf(V3f{sx2 / n, sy2 / n, sz2 / n});
}

static void transform_cluster(std::vector<QT>& in, std::vector<QT>& fine, int cluster_num, const Params& P,
                              int64_t* n_clusters) {
  const int n = (int)in.size();
  if ((float)n <= P.cluster_number_threshold) {
    if (n == 0) fine.push_back({1, 0, 0, 0, 0, 0, 0, true});
    else fine.insert(fine.end(), in.begin(), in.end());
    return;
  }
  const float r2 = (float)((double)P.cluster_distance_threshold * (double)P.cluster_distance_threshold);
  // Exact stand-in for KdTreeFLANN radiusSearch: all j with d2 < r2, sorted by (d2, j).
  struct Key { int64_t x, y, z; bool operator==(const Key& o) const { return x == o.x && y == o.y && z == o.z; } };
  struct KH { size_t operator()(const Key& k) const { return (size_t)(k.x * 73856093 ^ k.y * 19349663 ^ k.z * 83492791); } };
  const double cell = std::max(1.0, (double)P.cluster_distance_threshold * 1.25);
  std::unordered_map<Key, std::vector<int>, KH> grid;
  auto key_of = [&](const QT& t) {
    return Key{(int64_t)std::floor(t.tx / cell), (int64_t)std::floor(t.ty / cell), (int64_t)std::floor(t.tz / cell)};
  };
  for (int i = 0; i < n; ++i) grid[key_of(in[i])].push_back(i);
  std::vector<std::vector<QT>> clusters;
  std::vector<std::pair<float, int>> nb;
  for (int i = 0; i < n; ++i) {
    if (i == n - 1) break;  // the last candidate never seeds (:1084)
    if (in[i].alloc) continue;
    nb.clear();
    Key k = key_of(in[i]);
    for (int64_t dx = -1; dx <= 1; ++dx)
      for (int64_t dy = -1; dy <= 1; ++dy)
        for (int64_t dz = -1; dz <= 1; ++dz) {
          auto it = grid.find(Key{k.x + dx, k.y + dy, k.z + dz});
          if (it == grid.end()) continue;
          for (int j : it->second) {
            float ex = in[i].tx - in[j].tx, ey = in[i].ty - in[j].ty, ez = in[i].tz - in[j].tz;
            float d2 = 0.0f;  // flann::L2_Simple: sequential
            d2 += ex * ex; d2 += ey * ey; d2 += ez * ez;
            if (d2 < r2) nb.push_back({d2, j});
          }
        }
    std::sort(nb.begin(), nb.end());
    std::vector<QT> cl;
    Qf q1 = {in[i].qw, in[i].qx, in[i].qy, in[i].qz};
    V3f p1 = quat_rotate(q1, V3f{1, 0, 0});
    for (auto& e : nb) {
      QT& o = in[e.second];
      Qf q2 = {o.qw, o.qx, o.qy, o.qz};
      V3f p2 = quat_rotate(q2, V3f{1, 0, 0});
      const float thrc = P.cluster_angel_threshold;
      if (angle_decide(SITE_CLUSTER, p1.x, p1.y, p1.z, p2.x, p2.y, p2.z, [thrc](float t) { return t < thrc; })) {
        o.alloc = true;
        cl.push_back(o);
      }
    }
    clusters.push_back(std::move(cl));
  }
  if (n_clusters) *n_clusters = (int64_t)clusters.size();
  // range_cluster (:1020-1038)
  for (size_t i = 0; i < clusters.size(); ++i)
    for (size_t j = 0; j < clusters.size(); ++j)
      if (j > i && clusters[i].size() < clusters[j].size()) std::swap(clusters[i], clusters[j]);
  int clusternum = (int)clusters.front().size();
  bool stop = false;
  for (size_t ci = 0; ci < clusters.size(); ++ci) {
    if (stop) continue;
    const std::vector<QT>& c = clusters[ci];
    if ((int)c.size() >= clusternum) {
      float ax = 0, ay = 0, az = 0;
      for (const QT& t : c) { ax = ax + t.tx; ay = ay + t.ty; az = az + t.tz; }
      const float cs = (float)c.size();
      ax = ax / cs; ay = ay / cs; az = az / cs;
      V3f nt1, nt2;
      average_normal(nt1, nt2, c);
      M3f R = axes_to_rot(nt1, nt2);
      Qf q = quat_from_rot(R);
      fine.push_back({q.w, q.x, q.y, q.z, ax, ay, az, true});
      if (fine.size() > (size_t)cluster_num) break;
    } else {
      if ((double)fine.size() < (cluster_num / 2.0)) {
        stop = false;
        clusternum--;
        if (clusternum < 2) break;
      } else {
        stop = true;
      }
    }
  }
}

// ------------------------------------------------------ Ceres 1.14 LM (App. A10)
struct PairFace { float p1[3], n1[3], p2[3], n2[3]; float w; };

// Eigen Quaterniond product with the SSE2 Packet2d grouping (Geometry_SSE.h).
static void quatd_mul(const double a[4], const double b[4], double r[4]) {  // xyzw
  const double ax = a[0], ay = a[1], az = a[2], aw = a[3], bx = b[0], by = b[1], bz = b[2], bw = b[3];
  r[0] = (aw * bx + ay * bz) - (az * by - ax * bw);
  r[1] = (aw * by + ay * bw) + (az * bx - ax * bz);
  r[2] = (aw * bz - ay * bx) + (az * bw + ax * by);
  r[3] = (aw * bw - ay * by) - (az * bz + ax * bx);
}
// EigenQuaternionParameterization::Plus on q, plain + on t.
static void lm_plus(const double x[7], const double d[6], double out[7]) {
  const double nd = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  if (nd > 0.0) {
    const double s = std::sin(nd) / nd;
    const double dq[4] = {s * d[0], s * d[1], s * d[2], std::cos(nd)};
    quatd_mul(dq, x, out);
  } else {
    out[0] = x[0]; out[1] = x[1]; out[2] = x[2]; out[3] = x[3];
  }
  for (int i = 0; i < 3; ++i) out[4 + i] = x[4 + i] + d[3 + i];
}

static inline void crossd(const double a[3], const double b[3], double r[3]) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}
// f(q,v) = v + w*uv + qv x uv with uv = 2 (qv x v); J (3x4, columns x,y,z,w).
static void qrot_d(const double q[4], const double v[3], double f[3], double J[3][4]) {
  const double u[3] = {q[0], q[1], q[2]};
  const double w = q[3];
  double a[3], uv[3], c[3];
  crossd(u, v, a);
  uv[0] = a[0] + a[0]; uv[1] = a[1] + a[1]; uv[2] = a[2] + a[2];
  crossd(u, uv, c);
  for (int i = 0; i < 3; ++i) f[i] = (v[i] + w * uv[i]) + c[i];
  if (!J) return;
  for (int k = 0; k < 3; ++k) {
    double e[3] = {0, 0, 0};
    e[k] = 1.0;
    double ekv[3], eka[3], uekv[3];
    crossd(e, v, ekv);
    crossd(e, a, eka);
    crossd(u, ekv, uekv);
    for (int i = 0; i < 3; ++i) J[i][k] = 2.0 * w * ekv[i] + 2.0 * (eka[i] + uekv[i]);
  }
  for (int i = 0; i < 3; ++i) J[i][3] = uv[i];
}

// Residuals r (2P) and local Jacobian J (2P x 6, row-major). Returns false on non-finite.
static bool lm_eval(const std::vector<PairFace>& pf, const double x[7], double* cost, double* r, double* J) {
  const int m = 2 * (int)pf.size();
  const double* q = x;
  const double* t = x + 4;
  double Pj[4][3] = {{q[3], q[2], -q[1]}, {-q[2], q[3], q[0]}, {q[1], -q[0], q[3]}, {-q[0], -q[1], -q[2]}};
  double c = 0.0;
  for (size_t b = 0; b < pf.size(); ++b) {
    const PairFace& p = pf[b];
    const double n1[3] = {p.n1[0], p.n1[1], p.n1[2]}, p1[3] = {p.p1[0], p.p1[1], p.p1[2]};
    const double n2[3] = {p.n2[0], p.n2[1], p.n2[2]}, p2[3] = {p.p2[0], p.p2[1], p.p2[2]};
    const double w = p.w;
    double n2r[3], p2r[3], Jn[3][4], Jp[3][4];
    qrot_d(q, n2, n2r, J ? Jn : nullptr);
    qrot_d(q, p2, p2r, J ? Jp : nullptr);
    for (int i = 0; i < 3; ++i) p2r[i] = p2r[i] + t[i];
    double cr[3];
    crossd(n1, n2r, cr);
    const double nrm = std::sqrt((cr[0] * cr[0] + cr[1] * cr[1]) + cr[2] * cr[2]);
    const double d = ((n1[0] * p1[0] + n1[1] * p1[1]) + n1[2] * p1[2]) - ((n2r[0] * p2r[0] + n2r[1] * p2r[1]) + n2r[2] * p2r[2]);
    const double r0 = w * nrm, r1 = w * std::sqrt(d * d);
    r[2 * b] = r0;
    r[2 * b + 1] = r1;
    c += 0.5 * (r0 * r0 + r1 * r1);
    if (!std::isfinite(r0) || !std::isfinite(r1)) return false;
    if (J) {
      double g0[7] = {0, 0, 0, 0, 0, 0, 0}, g1[7] = {0, 0, 0, 0, 0, 0, 0};
      // d||n1 x n2r|| / dq = (cr/|cr|)^T [n1]x Jn
      for (int k = 0; k < 4; ++k) {
        double col[3] = {Jn[0][k], Jn[1][k], Jn[2][k]}, dc[3];
        crossd(n1, col, dc);
        g0[k] = w * (((cr[0] * dc[0] + cr[1] * dc[1]) + cr[2] * dc[2]) / nrm);
        double dd = -(((Jn[0][k] * p2r[0] + Jn[1][k] * p2r[1]) + Jn[2][k] * p2r[2]) +
                      ((n2r[0] * Jp[0][k] + n2r[1] * Jp[1][k]) + n2r[2] * Jp[2][k]));
        g1[k] = w * ((d * dd) / std::sqrt(d * d));
      }
      for (int k = 0; k < 3; ++k) g1[4 + k] = w * ((d * -n2r[k]) / std::sqrt(d * d));
      double* J0 = J + (2 * b) * 6;
      double* J1 = J + (2 * b + 1) * 6;
      for (int j = 0; j < 3; ++j) {
        J0[j] = ((g0[0] * Pj[0][j] + g0[1] * Pj[1][j]) + g0[2] * Pj[2][j]) + g0[3] * Pj[3][j];
        J1[j] = ((g1[0] * Pj[0][j] + g1[1] * Pj[1][j]) + g1[2] * Pj[2][j]) + g1[3] * Pj[3][j];
        J0[3 + j] = 0.0;
        J1[3 + j] = g1[4 + j];
      }
      for (int j = 0; j < 6; ++j)
        if (!std::isfinite(J0[j]) || !std::isfinite(J1[j])) return false;
    }
  }
  (void)m;
  *cost = c;
  return true;
}

// min || [A; diag(D)] y - [b; 0] || by Householder QR (Eigen HouseholderQR shape).
static bool qr_solve(const std::vector<double>& A, int m, const double D[6], const double* b, double y[6]) {
  const int n = 6, M = m + n;
  std::vector<double> Q((size_t)M * n), rhs(M, 0.0);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < n; ++j) Q[(size_t)i * n + j] = A[(size_t)i * n + j];
  for (int j = 0; j < n; ++j) {
    for (int k = 0; k < n; ++k) Q[(size_t)(m + j) * n + k] = 0.0;
    Q[(size_t)(m + j) * n + j] = D[j];
  }
  for (int i = 0; i < m; ++i) rhs[i] = b[i];
  for (int k = 0; k < n; ++k) {
    double c0 = Q[(size_t)k * n + k], tail = 0.0;
    for (int i = k + 1; i < M; ++i) tail += Q[(size_t)i * n + k] * Q[(size_t)i * n + k];
    double tau, beta;
    if (tail <= DBL_MIN) {
      tau = 0.0;
      beta = c0;
      for (int i = k + 1; i < M; ++i) Q[(size_t)i * n + k] = 0.0;
    } else {
      beta = std::sqrt(c0 * c0 + tail);
      if (c0 >= 0.0) beta = -beta;
      for (int i = k + 1; i < M; ++i) Q[(size_t)i * n + k] = Q[(size_t)i * n + k] / (c0 - beta);
      tau = (beta - c0) / beta;
    }
    Q[(size_t)k * n + k] = beta;
    auto apply = [&](auto get, auto set) {
      double tmp = 0.0;
      for (int i = k + 1; i < M; ++i) tmp += Q[(size_t)i * n + k] * get(i);
      tmp += get(k);
      set(k, get(k) - tau * tmp);
      for (int i = k + 1; i < M; ++i) set(i, get(i) - tau * Q[(size_t)i * n + k] * tmp);
    };
    for (int j = k + 1; j < n; ++j)
      apply([&](int i) { return Q[(size_t)i * n + j]; }, [&](int i, double v) { Q[(size_t)i * n + j] = v; });
    apply([&](int i) { return rhs[i]; }, [&](int i, double v) { rhs[i] = v; });
  }
  for (int i = 0; i < n; ++i) y[i] = rhs[i];
  for (int k = n - 1; k >= 0; --k) {  // column-oriented back substitution
    y[k] = y[k] / Q[(size_t)k * n + k];
    for (int i = 0; i < k; ++i) y[i] = y[i] - y[k] * Q[(size_t)i * n + k];
  }
  for (int i = 0; i < n; ++i)
    if (!std::isfinite(y[i])) return false;
  return true;
}

// Returns the best parameters seen (Solver writes back parameters_ = argmin cost).
static void lm_solve(const std::vector<PairFace>& pf, double best[7]) {
  const int m = 2 * (int)pf.size();
  double x[7] = {0, 0, 0, 1, 0, 0, 0};
  for (int i = 0; i < 7; ++i) best[i] = x[i];
  std::vector<double> r(m), J((size_t)m * 6), rc(m), Jc((size_t)m * 6);
  double cost;
  if (!lm_eval(pf, x, &cost, r.data(), J.data())) return;
  double scale[6];
  auto finish_jacobian = [&](std::vector<double>& Jm, const std::vector<double>& rr, double* gmax) {
    double g[6];
    for (int j = 0; j < 6; ++j) {
      double s = 0.0;
      for (int i = 0; i < m; ++i) s += Jm[(size_t)i * 6 + j] * rr[i];
      g[j] = s;
    }
    double ng[6], xp[7];
    for (int j = 0; j < 6; ++j) ng[j] = -g[j];
    lm_plus(x, ng, xp);
    double mx = 0.0;
    for (int j = 0; j < 7; ++j) mx = std::max(mx, std::fabs(x[j] - xp[j]));
    *gmax = mx;
    for (int i = 0; i < m; ++i)
      for (int j = 0; j < 6; ++j) Jm[(size_t)i * 6 + j] *= scale[j];
  };
  for (int j = 0; j < 6; ++j) {
    double s = 0.0;
    for (int i = 0; i < m; ++i) s += J[(size_t)i * 6 + j] * J[(size_t)i * 6 + j];
    scale[j] = 1.0 / (1.0 + std::sqrt(s));
  }
  double gmax;
  finish_jacobian(J, r, &gmax);
  double min_cost = cost;
  for (int i = 0; i < 7; ++i) best[i] = x[i];
  auto xnorm_of = [](const double* v) {
    double s = 0.0;
    for (int i = 0; i < 7; ++i) s += v[i] * v[i];
    return std::sqrt(s);
  };
  double x_norm = xnorm_of(x);
  double radius = 1e4, decrease = 2.0;
  bool reuse = false, successful = true;
  double diag[6];
  int iteration = 0, invalid = 0;
  // Finalize(iteration 0)
  if (successful && gmax <= 1e-10) return;
  while (true) {
    ++iteration;
    successful = false;
    if (!reuse) {
      for (int j = 0; j < 6; ++j) {
        double s = 0.0;
        for (int i = 0; i < m; ++i) s += J[(size_t)i * 6 + j] * J[(size_t)i * 6 + j];
        diag[j] = std::min(std::max(s, 1e-6), 1e32);
      }
    }
    double D[6], y[6], step[6];
    for (int j = 0; j < 6; ++j) D[j] = std::sqrt(diag[j] / radius);
    bool solved = qr_solve(J, m, D, r.data(), y);
    reuse = true;
    bool valid = false;
    double mcc = 0.0;
    if (solved) {
      for (int j = 0; j < 6; ++j) step[j] = -y[j];
      double dot = 0.0;
      for (int i = 0; i < m; ++i) {
        double mr = 0.0;
        for (int j = 0; j < 6; ++j) mr += J[(size_t)i * 6 + j] * step[j];
        dot += mr * (r[i] + mr / 2.0);
      }
      mcc = -dot;
      valid = mcc > 0.0;
    }
    if (!valid) {
      if (++invalid >= 5) return;
      radius = radius / decrease;  // StepIsInvalid -> StepRejected(0)
      decrease *= 2.0;
    } else {
      invalid = 0;
      double delta[6], cand[7];
      for (int j = 0; j < 6; ++j) delta[j] = step[j] * scale[j];
      lm_plus(x, delta, cand);
      double ccost;
      if (!lm_eval(pf, cand, &ccost, rc.data(), nullptr)) ccost = DBL_MAX;
      double sn = 0.0;
      for (int i = 0; i < 7; ++i) sn += (x[i] - cand[i]) * (x[i] - cand[i]);
      sn = std::sqrt(sn);
      if (sn <= 1e-8 * (x_norm + 1e-8)) return;           // parameter tolerance
      if (std::fabs(cost - ccost) <= 1e-6 * cost) return;  // function tolerance
      double rho = (cost - ccost) / mcc;
      if (rho > 1e-3) {
        for (int i = 0; i < 7; ++i) x[i] = cand[i];
        x_norm = xnorm_of(x);
        if (!lm_eval(pf, x, &cost, r.data(), J.data())) return;
        finish_jacobian(J, r, &gmax);
        successful = true;
        radius = radius / std::max(1.0 / 3.0, 1.0 - std::pow(2.0 * rho - 1.0, 3));
        radius = std::min(1e16, radius);
        decrease = 2.0;
        reuse = false;
      } else {
        radius = radius / decrease;
        decrease *= 2.0;
      }
    }
    // FinalizeIterationAndCheckIfMinimizerCanContinue
    if (successful && cost < min_cost) {
      min_cost = cost;
      for (int i = 0; i < 7; ++i) best[i] = x[i];
    }
    if (iteration >= 50) return;
    if (successful && gmax <= 1e-10) return;
    if (radius <= 1e-32) return;
  }
}

static M4f ceres_refine_T(const std::vector<PairFace>& pf) {
  double b[7];
  lm_solve(pf, b);
  Qf q = {(float)b[3], (float)b[0], (float)b[1], (float)b[2]};
  M3f R = rot_from_quat(q);
  M4f T = identity4();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T.m[i][j] = R.m[i][j];
  T.m[0][3] = (float)b[4]; T.m[1][3] = (float)b[5]; T.m[2][3] = (float)b[6];
  return T;
}

// ------------------------------------------------------ quick_verify (:680-783)
static float quick_verify(M4f& T, const std::vector<Face>& F1, const std::vector<Face>& F2, const Params& P,
                          int* npairs) {
  int fs1 = 0, fs2 = 0;
  for (const Face& f : F1) fs1 = (int)((float)fs1 + f.fps);
  for (const Face& f : F2) fs2 = (int)((float)fs2 + f.fps);
  std::vector<V3f> c2(F2.size()), n2(F2.size());
  for (size_t k = 0; k < F2.size(); ++k) {
    c2[k] = tf_se3(T, F2[k].ac[0], F2[k].ac[1], F2[k].ac[2]);
    n2[k] = tf_so3(T, F2[k].an[0], F2[k].an[1], F2[k].an[2]);
  }
  std::vector<PairFace> pairs;
  for (size_t i = 0; i < F1.size(); ++i) {
    const Face& a = F1[i];
    std::vector<int> cand;
    bool find = false;
    for (size_t j = 0; j < F2.size(); ++j) {
      const float thrv = P.quick_verify_angel_threshold;
      const bool angok = angle_decide(SITE_VERIFY, a.an[0], a.an[1], a.an[2], n2[j].x, n2[j].y, n2[j].z,
                                      [thrv](float t) { return t < thrv; });
      const double dn1[3] = {a.an[0], a.an[1], a.an[2]}, dn2[3] = {n2[j].x, n2[j].y, n2[j].z};
      const double dc1[3] = {a.ac[0], a.ac[1], a.ac[2]}, dc2[3] = {c2[j].x, c2[j].y, c2[j].z};
      float d1 = (float)dotd(dn1, dc1), d2 = (float)dotd(dn2, dc2);
      float dist = std::fabs(d1 - d2);
      if (angok && dist < P.quick_verify_distance_threshold) {
        find = true;
        cand.push_back((int)j);
      }
    }
    float size1 = a.fps;
    int best = 0;
    float best_imp = 0, best_score = 0;
    for (int j : cand) {
      float size2 = F2[j].fps;
      float mn = size1 < size2 ? size1 : size2;
      float mx = size1 > size2 ? size1 : size2;
      float sc = mn / mx;
      float imp = (2 * mn) / (float)(fs1 + fs2);
      if (sc > best_score) { best_imp = imp; best_score = sc; best = j; }
    }
    if (find) {
      PairFace pf;
      pf.p1[0] = a.ac[0]; pf.p1[1] = a.ac[1]; pf.p1[2] = a.ac[2];
      pf.n1[0] = a.an[0]; pf.n1[1] = a.an[1]; pf.n1[2] = a.an[2];
      pf.p2[0] = c2[best].x; pf.p2[1] = c2[best].y; pf.p2[2] = c2[best].z;
      pf.n2[0] = n2[best].x; pf.n2[1] = n2[best].y; pf.n2[2] = n2[best].z;
      pf.w = best_imp;
      pairs.push_back(pf);
    }
  }
  if (npairs) *npairs = (int)pairs.size();
  if ((float)pairs.size() >= P.required_optimize_plane) {
    M4f dT = ceres_refine_T(pairs);
    T = mul44(dT, T);
  }
  float score = 0;
  for (const PairFace& p : pairs) score = score + p.w;
  return score;
}

// ------------------------------------------------------ fine_verify (:785-839)
static float fine_verify(const M4f& T, const Cloud& s1, const Cloud& s2, const Params& P) {
  const size_t n1 = npts(s1), n2 = npts(s2), n = n1 + n2;
  std::vector<float> fused(3 * n);
  std::memcpy(fused.data(), s1.data(), sizeof(float) * 3 * n1);
  for (size_t i = 0; i < n2; ++i) {
    V3f p = tf_se3(T, s2[3 * i], s2[3 * i + 1], s2[3 * i + 2]);
    fused[3 * (n1 + i)] = p.x; fused[3 * (n1 + i) + 1] = p.y; fused[3 * (n1 + i) + 2] = p.z;
  }
  Leaves L = octree_leaves(fused.data(), n, (double)P.fine_verify_voxel_size);
  float similar = 0, all = 0;
  for (size_t v = 0; v + 1 < L.start.size(); ++v) {
    float sn = 0, tn = 0;
    for (uint32_t k = L.start[v]; k < L.start[v + 1]; ++k) {
      if (L.idx[k] < n1) sn++;
      else tn++;
    }
    all = all + sn + tn;
    if (sn >= 1 && tn >= 1) {
      float mn = sn < tn ? sn : tn, mx = sn > tn ? sn : tn;
      similar = similar + (sn + tn) * (mn / mx);
    }
  }
  return similar / all;
}

// ------------------------------------------------------ fusion (:1253-1368)
struct High { QT qt; float score; };
static M4f fuse_answer(const std::vector<High>& hs, float sum) {
  float tx = 0, ty = 0, tz = 0;
  for (const High& h : hs) {
    tx = tx + h.qt.tx * (h.score / sum);
    ty = ty + h.qt.ty * (h.score / sum);
    tz = tz + h.qt.tz * (h.score / sum);
  }
  float a1 = 0, b1 = 0, c1 = 0, a2 = 0, b2 = 0, c2 = 0;
  for (const High& h : hs) {
    Qf q = {h.qt.qw, h.qt.qx, h.qt.qy, h.qt.qz};
    V3f u = quat_rotate(q, V3f{1, 0, 0}), v = quat_rotate(q, V3f{0, 1, 0});
    a1 = a1 + u.x * (h.score / sum); b1 = b1 + u.y * (h.score / sum); c1 = c1 + u.z * (h.score / sum);
    a2 = a2 + v.x * (h.score / sum); b2 = b2 + v.y * (h.score / sum); c2 = c2 + v.z * (h.score / sum);
  }
  V3f nt1 = normalizedf(V3f{a1, b1, c1}), nt2 = normalizedf(V3f{a2, b2, c2});
  M3f R = axes_to_rot(nt1, nt2);
  M4f T = identity4();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T.m[i][j] = R.m[i][j];
  T.m[0][3] = tx; T.m[1][3] = ty; T.m[2][3] = tz;
  return T;
}

static QT qt_from_T(const M4f& T) {
  M3f R;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R.m[i][j] = T.m[i][j];
  Qf q = quat_from_rot(R);
  return {q.w, q.x, q.y, q.z, T.m[0][3], T.m[1][3], T.m[2][3], false};
}
static M4f T_from_qt(const QT& t) {
  M3f R = rot_from_quat(Qf{t.qw, t.qx, t.qy, t.qz});
  M4f T = identity4();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T.m[i][j] = R.m[i][j];
  T.m[0][3] = t.tx; T.m[1][3] = t.ty; T.m[2][3] = t.tz;
  return T;
}

static void put_faces(Store& st, const std::string& k, const std::vector<Face>& F) {
  std::vector<float> v;
  for (const Face& f : F) {
    v.insert(v.end(), f.ac, f.ac + 3);
    v.insert(v.end(), f.an, f.an + 3);
    v.push_back(f.fps);
    v.push_back((float)f.members.size());
  }
  st.put(k, v);
}
static std::vector<float> flat(const std::vector<M4f>& Ts) {
  std::vector<float> v;
  for (const M4f& T : Ts)
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) v.push_back(T.m[i][j]);
  return v;
}

}  // namespace

// ============================================================== driver (:1370-1608)
struct orc_ctx {
  Store st;
  double ms[9] = {0};
};

using clk = std::chrono::steady_clock;
static double ms_since(clk::time_point t0) {
  return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

// The fusion (:1546-1606): every type's best normalised score over its first
// analyse_max candidates (score1_sum / score2_sum over all types, App. B Q15), the
// types above 0.8 of the best, fuse_answer.
struct TS { M4f T; float score, score2; };
static M4f fuse_stage(const std::vector<TS> ctv[3], int analyse_max, float score1_sum, float score2_sum,
                      std::vector<High>& tmp) {
  float best_best = 0;
  for (int i = 0; i < 3; ++i) {
    int analyse_sum = 0;
    float bs = 0;
    M4f bt = identity4();
    for (auto& ts : ctv[i]) {
      if (analyse_sum < analyse_max) {
        analyse_sum++;
        float s = ts.score / score1_sum + ts.score2 / score2_sum;
        if (s > bs) { bs = s; bt = ts.T; }
      }
    }
    if (best_best < bs) best_best = bs;
    High h;
    h.qt = qt_from_T(bt);
    h.score = bs;
    tmp.push_back(h);
  }
  std::vector<High> hs;
  float score_sum = 0;
  for (const High& h : tmp)
    if (h.score > best_best * 0.8) {
      hs.push_back(h);
      score_sum += h.score;
    }
  return fuse_answer(hs, score_sum);
}

static void computer_transform_guess(Cloud source, Cloud target, float leaf, int order, const Params& P, M4f& best,
                                     orc_ctx* cx) {
  Store& st = cx->st;
  auto t0 = clk::now();
  source = remove_nan(source);
  target = remove_nan(target);
  int ovf = 0;
  Cloud cs = voxel_grid(source, leaf, order, &ovf);
  Cloud ct = voxel_grid(target, leaf, order, &ovf);
  st.put("ds1", cs);
  st.put("ds2", ct);
  cx->ms[0] += ms_since(t0);

  t0 = clk::now();
  FaceOut f1, f2;
  face_extrate(cs, P, f1);
  face_extrate(ct, P, f2);
  cx->ms[1] += ms_since(t0);
  for (int c = 1; c <= 2; ++c) {
    FaceOut& f = c == 1 ? f1 : f2;
    std::string s = std::to_string(c);
    st.put("centroid" + s, std::vector<float>(f.centroid, f.centroid + 4));
    st.put("oct" + s, std::vector<double>(f.oct, f.oct + 4));
    std::vector<float> vv;
    for (const Voxel& v : f.voxels) {
      vv.insert(vv.end(), v.c, v.c + 3);
      vv.insert(vv.end(), v.n, v.n + 3);
      vv.push_back((float)v.size);
      vv.push_back(0.f);
    }
    st.put("vox" + s, vv);
    st.put("vstat" + s, f.vstat);
    st.put("vcurv" + s, f.vcurv);
    st.put("res" + s, f.residual);
    put_faces(st, "groups" + s, f.groups_all);
    put_faces(st, "planes" + s, f.planes);
    st.put("theta" + s, f.theta);
    std::vector<int32_t> gal;
    for (const Face& g : f.groups_all) gal.push_back(g.alloc ? 1 : 0);
    st.put("galloc" + s, gal);
  }

  t0 = clk::now();
  std::vector<int> type1, type2;
  std::vector<Base> b1, b2;
  select_base(f1.planes, f1.theta, P, b1, type1);
  select_base(f2.planes, f2.theta, P, b2, type2);
  for (int c = 1; c <= 2; ++c) {
    auto& b = c == 1 ? b1 : b2;
    auto& ty = c == 1 ? type1 : type2;
    std::vector<int32_t> v;
    for (size_t i = 0; i < b.size(); ++i) {
      int32_t ab;
      std::memcpy(&ab, &b[i].angle, 4);
      v.push_back(b[i].i1); v.push_back(b[i].i2); v.push_back(ab);
      v.push_back(i < ty.size() ? ty[i] : -1);
    }
    st.put("bases" + std::to_string(c), v);
  }
  std::vector<M4f> tv[3];
  int64_t kpass = 0;
  const float angth = P.included_angle_same_threshold;
  for (size_t i1 = 0; i1 < b1.size(); ++i1)
    for (size_t i2 = 0; i2 < b2.size(); ++i2) {
      // type_index may be shorter than base_vecter (NaN roughness, App. B Q5):
      // out-of-range reads are undefined in the reference; here they never match.
      int ta = i1 < type1.size() ? type1[i1] : -1;
      int tb = i2 < type2.size() ? type2[i2] : -2;
      float dv[ACOS_MODES];
      bool dd[ACOS_MODES];
      for (int a = 0; a < ACOS_MODES; ++a) {
        dv[a] = std::fabs(b1[i1].alt[a] - b2[i2].alt[a]);
        dd[a] = dv[a] < angth;
      }
      audit_site(SITE_PAIR, dv, dd);
      if (std::fabs(b1[i1].angle - b2[i2].angle) < angth && ta == tb) {
        ++kpass;
        computer_transform(tv, b1[i1].i1, b1[i1].i2, b2[i2].i1, b2[i2].i2, f1.planes, f2.planes, ta, P);
      }
    }
  cx->ms[3] += ms_since(t0);
  const int transformation_num = (int)(tv[0].size() + tv[1].size() + tv[2].size());
  std::vector<int64_t> counts = {(int64_t)b1.size() * (int64_t)b2.size(), kpass, (int64_t)tv[0].size(),
                                 (int64_t)tv[1].size(), (int64_t)tv[2].size()};
  for (int i = 0; i < 3; ++i) st.put("cand" + std::to_string(i), flat(tv[i]));

  float score1_sum = 0, score2_sum = 0;
  std::vector<TS> ctv[3];
  const int analyse_max = (int)P.fine_verify_number;
  int64_t lm_solves = 0;
  for (int i = 0; i < 3; ++i) {
    t0 = clk::now();
    std::vector<QT> qv;
    for (const M4f& T : tv[i]) qv.push_back(qt_from_T(T));
    std::vector<QT> fine;
    // 0/0 when no type has candidates: unused by transform_cluster in that case (App. B Q17).
    int cluster_num = transformation_num
                          ? (int)(P.seclct_cluster_number * (float)tv[i].size() / (float)transformation_num)
                          : 0;
    int64_t ncl = 0;
    transform_cluster(qv, fine, cluster_num, P, &ncl);
    counts.push_back(ncl);
    cx->ms[4] += ms_since(t0);
    std::vector<float> fv;
    for (const QT& q : fine) {
      float a[8] = {q.qw, q.qx, q.qy, q.qz, q.tx, q.ty, q.tz, q.alloc ? 1.f : 0.f};
      fv.insert(fv.end(), a, a + 8);
    }
    st.put("fine" + std::to_string(i), fv);
    t0 = clk::now();
    std::vector<float> qvd;
    for (const QT& q : fine) {
      TS ts;
      ts.T = T_from_qt(q);
      int np = 0;
      ts.score = quick_verify(ts.T, f1.planes, f2.planes, P, &np);
      ts.score2 = 0;
      if ((float)np >= P.required_optimize_plane) ++lm_solves;
      ctv[i].push_back(ts);
      for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) qvd.push_back(ts.T.m[a][b]);
      qvd.push_back(ts.score);
      qvd.push_back((float)np);
    }
    st.put("qv" + std::to_string(i), qvd);
    // score_range (:1233-1251)
    auto& cv = ctv[i];
    for (size_t a = 0; a + 1 < cv.size(); ++a)
      for (size_t b = a + 1; b < cv.size(); ++b)
        if (cv[a].score < cv[b].score) std::swap(cv[a], cv[b]);
    cx->ms[5] += ms_since(t0);
    t0 = clk::now();
    int analyse_sum = 0;
    std::vector<float> fvd;
    for (auto& ts : cv) {
      if (analyse_sum < analyse_max) {
        analyse_sum++;
        ts.score2 = fine_verify(ts.T, f1.residual, f2.residual, P);
        score2_sum += ts.score2;
        score1_sum += ts.score;
        for (int a = 0; a < 4; ++a)
          for (int b = 0; b < 4; ++b) fvd.push_back(ts.T.m[a][b]);
        fvd.push_back(ts.score);
        fvd.push_back(ts.score2);
      } else {
        break;
      }
    }
    st.put("fv" + std::to_string(i), fvd);
    cx->ms[6] += ms_since(t0);
  }
  t0 = clk::now();
  std::vector<High> tmp;
  M4f T = fuse_stage(ctv, analyse_max, score1_sum, score2_sum, tmp);
  std::vector<float> hv;
  for (const High& h : tmp) {
    float a[8] = {h.qt.qw, h.qt.qx, h.qt.qy, h.qt.qz, h.qt.tx, h.qt.ty, h.qt.tz, h.score};
    hv.insert(hv.end(), a, a + 8);
  }
  st.put("high", hv);
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) best.m[i][j] = T.m[i][j];
  cx->ms[7] += ms_since(t0);
  counts.push_back(lm_solves);
  counts.push_back(ovf);
  st.put("counts", counts);
}

extern "C" orc_ctx* orc_register(const float* src_xyz, int64_t n_src, const float* tar_xyz, int64_t n_tar,
                                 float leaf, int order) {
  if ((!src_xyz && n_src) || (!tar_xyz && n_tar) || n_src < 0 || n_tar < 0 || !(leaf > 0.f)) return nullptr;
  orc_ctx* cx = new orc_ctx();
  Params P;
  auto t_all = clk::now();
  auto t0 = clk::now();
  Cloud src(src_xyz, src_xyz + 3 * n_src), tar(tar_xyz, tar_xyz + 3 * n_tar);
  int ovf = 0;
  Cloud cs = voxel_grid(src, leaf, order, &ovf);  // main :1668-1672
  Cloud ct = voxel_grid(tar, leaf, order, &ovf);  // main :1674-1678
  const double main_vg_ms = ms_since(t0);
  cx->ms[0] += main_vg_ms;
  cx->st.put1("main_vg_ms", main_vg_ms);  // outside the reference's timer window (:1681-1685)
  cx->st.put("ds_src", cs);
  cx->st.put("ds_tar", ct);
  M4f best = identity4();
  computer_transform_guess(ct, cs, leaf, order, P, best, cx);  // (cloud_tar, cloud_src) :1683
  std::vector<float> T;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) T.push_back(best.m[i][j]);
  cx->st.put("T", T);
  cx->st.put1("main_overflow", (int32_t)ovf);
  cx->ms[8] = ms_since(t_all);
  return cx;
}

extern "C" void orc_free(orc_ctx* c) { delete c; }

extern "C" int64_t orc_get(orc_ctx* c, const char* name, void* buf, int64_t cap) {
  if (!c || !name) return -1;
  auto it = c->st.blobs.find(name);
  if (it == c->st.blobs.end()) return -1;
  int64_t n = (int64_t)it->second.size();
  if (buf && cap > 0) std::memcpy(buf, it->second.data(), (size_t)std::min(n, cap));
  return n;
}

extern "C" void orc_times(orc_ctx* c, double out[9]) {
  for (int i = 0; i < 9; ++i) out[i] = c ? c->ms[i] : 0.0;
}

extern "C" int64_t orc_voxel_grid(const float* xyz, int64_t n, float leaf, int order, float* out, int* overflow) {
  if (n < 0 || !(leaf > 0.f)) return -1;
  Cloud in(xyz, xyz + 3 * n);
  int ovf = 0;
  Cloud o = voxel_grid(in, leaf, order, &ovf);
  if (overflow) *overflow = ovf;
  if (out) std::memcpy(out, o.data(), o.size() * sizeof(float));
  return (int64_t)npts(o);
}

extern "C" int64_t orc_sort_pairs(const uint32_t* keys, int64_t n, uint32_t* perm) {
  std::vector<IdxPair> iv;  // pcl::VoxelGrid::applyFilter's index_vector (App. A2 steps 5-6)
  for (int64_t i = 0; i < n; ++i)
    if (keys[i] != 0xFFFFFFFFu) iv.push_back({keys[i], (unsigned int)i});
  std::sort(iv.begin(), iv.end(), std::less<IdxPair>());
  for (size_t i = 0; i < iv.size(); ++i) perm[i] = iv[i].cloud_point_index;
  return (int64_t)iv.size();
}

extern "C" void orc_sort_adversary(int64_t n, uint32_t* keys) {
  // M. D. McIlroy, "A killer adversary for quicksort" (1999): values are frozen lazily
  // so that every partition is as unbalanced as the comparisons allow
  std::vector<int64_t> val((size_t)n, -1);
  std::vector<uint32_t> idx((size_t)n);
  for (int64_t i = 0; i < n; ++i) idx[(size_t)i] = (uint32_t)i;
  int64_t nsolid = 0, candidate = 0;
  const int64_t gas = n;
  std::sort(idx.begin(), idx.end(), [&](uint32_t x, uint32_t y) {
    if (val[x] < 0 && val[y] < 0) val[(int64_t)x == candidate ? x : y] = nsolid++;
    if (val[x] < 0) candidate = x;
    else if (val[y] < 0) candidate = y;
    const int64_t vx = val[x] < 0 ? gas : val[x], vy = val[y] < 0 ? gas : val[y];
    return vx < vy;
  });
  for (int64_t i = 0; i < n; ++i) keys[i] = (uint32_t)(val[(size_t)i] < 0 ? gas : val[(size_t)i]);
}

extern "C" void orc_eigen33(const float cov[9], float* ev, float vec[3]) {
  float m[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) m[i][j] = cov[3 * i + j];
  V3f v;
  eigen33(m, *ev, v);
  vec[0] = v.x; vec[1] = v.y; vec[2] = v.z;
}

extern "C" float orc_normal_angle(float x1, float y1, float z1, float x2, float y2, float z2) {
  return compute_normal_angel(x1, y1, z1, x2, y2, z2);
}
extern "C" int orc_set_octree_mode(int mode) {
  const int prev = g_octree_mode;
  if (mode == 0 || mode == 1) g_octree_mode = mode;
  return prev;
}

extern "C" int orc_set_acos_mode(int mode) {
  const int prev = g_acos_mode;
  if (mode >= 0 && mode < ACOS_MODES) g_acos_mode = mode;
  return prev;
}
extern "C" void orc_acos_audit(uint64_t out[3 * SITE_N], int reset) {
  if (out)
    for (int i = 0; i < SITE_N; ++i) {
      out[i] = g_audit.evals[i];
      out[SITE_N + i] = g_audit.differ[i];
      out[2 * SITE_N + i] = g_audit.flips[i];
    }
  if (reset) g_audit = AcosAudit{};
}

extern "C" void orc_quat_from_rot(const float R[9], float q[4]) {
  M3f m;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) m.m[i][j] = R[3 * i + j];
  Qf r = quat_from_rot(m);
  q[0] = r.w; q[1] = r.x; q[2] = r.y; q[3] = r.z;
}

extern "C" void orc_rot_from_quat(const float q[4], float R[9]) {
  M3f m = rot_from_quat(Qf{q[0], q[1], q[2], q[3]});
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R[3 * i + j] = m.m[i][j];
}

extern "C" int orc_lm_refine(const float* pairs, int P, double q[4], double t[3]) {
  std::vector<PairFace> pf(P);
  for (int i = 0; i < P; ++i) {
    const float* s = pairs + 13 * i;
    std::memcpy(pf[i].p1, s, 12); std::memcpy(pf[i].n1, s + 3, 12);
    std::memcpy(pf[i].p2, s + 6, 12); std::memcpy(pf[i].n2, s + 9, 12);
    pf[i].w = s[12];
  }
  double b[7];
  lm_solve(pf, b);
  for (int i = 0; i < 4; ++i) q[i] = b[i];
  for (int i = 0; i < 3; ++i) t[i] = b[4 + i];
  return 0;
}

// ------------------------------------------------ single host stages (KAT inputs)
extern "C" int orc_stage_grow(const orc_voxel* vox, int64_t nv, int side, float* planes, int cap_planes,
                              int* n_planes, double* theta, int32_t* bases, int cap_bases, int* n_bases) {
  if ((!vox && nv) || nv < 0 || (side != 1 && side != 2) || !n_planes || !n_bases) return -1;
  Params P;
  FaceOut out;
  for (int64_t i = 0; i < nv; ++i) {
    Voxel v;
    for (int a = 0; a < 3; ++a) { v.c[a] = vox[i].c[a]; v.n[a] = vox[i].n[a]; }
    v.size = vox[i].count;
    out.voxels.push_back(v);
  }
  grow_select(P, out);
  std::vector<Base> b;
  std::vector<int> type;
  select_base(out.planes, out.theta, P, b, type);
  *n_planes = (int)out.planes.size();
  *n_bases = (int)b.size();
  for (int i = 0; i < *n_planes && i < cap_planes; ++i) {
    const Face& f = out.planes[(size_t)i];
    const float a[8] = {f.ac[0], f.ac[1], f.ac[2], f.an[0], f.an[1], f.an[2], f.fps, (float)f.members.size()};
    std::memcpy(planes + 8 * i, a, sizeof a);
    if (theta) theta[i] = out.theta[(size_t)i];
  }
  // type_index is shorter than the bases when a roughness is NaN (App. B Q5): positions
  // past its end read as the side's sentinel, as the matching loop does (-1 / -2)
  for (int k = 0; k < *n_bases && k < cap_bases; ++k) {
    int32_t* r = bases + 4 * k;
    r[0] = b[(size_t)k].i1;
    r[1] = b[(size_t)k].i2;
    std::memcpy(&r[2], &b[(size_t)k].angle, 4);
    r[3] = (size_t)k < type.size() ? type[(size_t)k] : (side == 1 ? -1 : -2);
  }
  return 0;
}

extern "C" int orc_stage_cluster(const float* cand, int64_t n, int cluster_num, float* fine, int64_t cap,
                                 int64_t* n_fine, int64_t* n_clusters) {
  if ((!cand && n) || n < 0 || !n_fine) return -1;
  Params P;
  std::vector<QT> qv, out;
  for (int64_t i = 0; i < n; ++i) {
    M4f T;
    std::memcpy(T.m, cand + 16 * i, sizeof T.m);
    qv.push_back(qt_from_T(T));
  }
  int64_t ncl = 0;
  transform_cluster(qv, out, cluster_num, P, &ncl);
  *n_fine = (int64_t)out.size();
  if (n_clusters) *n_clusters = ncl;
  for (int64_t i = 0; i < *n_fine && i < cap; ++i) {
    const QT& q = out[(size_t)i];
    const float a[8] = {q.qw, q.qx, q.qy, q.qz, q.tx, q.ty, q.tz, q.alloc ? 1.f : 0.f};
    std::memcpy(fine + 8 * i, a, sizeof a);
  }
  return 0;
}

extern "C" int orc_stage_fuse(const float* const cand[3], const int64_t n[3], int analyse_max, float T[16],
                              float high[24]) {
  if (!cand || !n || !T) return -1;
  std::vector<TS> ctv[3];
  float s1 = 0, s2 = 0;
  for (int t = 0; t < 3; ++t)
    for (int64_t i = 0; i < n[t]; ++i) {
      TS x;
      const float* r = cand[t] + 18 * i;
      std::memcpy(x.T.m, r, sizeof x.T.m);
      x.score = r[16];
      x.score2 = r[17];
      ctv[t].push_back(x);
      if (i < analyse_max) {  // (:1538-1540: the first analyse_max of every type)
        s2 += x.score2;
        s1 += x.score;
      }
    }
  std::vector<High> tmp;
  const M4f R = fuse_stage(ctv, analyse_max, s1, s2, tmp);
  M4f best = identity4();  // (the caller's matrix: rows 0-2 written, :1606 via fuse_answer)
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 4; ++j) best.m[i][j] = R.m[i][j];
  std::memcpy(T, best.m, sizeof best.m);
  if (high)
    for (int t = 0; t < 3; ++t) {
      const High& h = tmp[(size_t)t];
      const float a[8] = {h.qt.qw, h.qt.qx, h.qt.qy, h.qt.qz, h.qt.tx, h.qt.ty, h.qt.tz, h.score};
      std::memcpy(high + 8 * t, a, sizeof a);
    }
  return 0;
}
