// fccf_math.h — host+device scalar arithmetic of the FCCF-PCR path, in the exact
// evaluation order the reference binary uses (Eigen 3.3 fixed-size expressions,
// PCL 1.10 SSE transformer, SSE2/no-FMA build of FCCF.cpp).  Every kernel and
// every host stage of libfccf goes through these helpers so that discrete
// decisions (thresholds, orderings) come out bit-identical to the CPU oracle.
// Build with -ffp-contract=off (no FMA contraction on host or device).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define FH __host__ __device__ __forceinline__

namespace fccf {

struct f3 { float x, y, z; };
struct m33 { float m[3][3]; };
struct m44 { float m[4][4]; };
struct quatf { float w, x, y, z; };

// Eigen float Vector3 redux (redux_novec_unroller): a0 + (a1 + a2)
FH float dot3(f3 a, f3 b) { return a.x * b.x + (a.y * b.y + a.z * b.z); }
FH float sqn3(f3 a) { return a.x * a.x + (a.y * a.y + a.z * a.z); }
FH f3 cross3(f3 a, f3 b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
// Eigen 3.3.7 normalize(): no-op on a zero vector
FH f3 normalize3(f3 a) {
  float z = sqn3(a);
  if (z > 0.f) {
    float s = sqrtf(z);
    a.x = a.x / s; a.y = a.y / s; a.z = a.z / s;
  }
  return a;
}
FH m33 eye33() {
  m33 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.m[i][j] = (i == j) ? 1.f : 0.f;
  return r;
}
FH m44 eye44() {
  m44 r;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) r.m[i][j] = (i == j) ? 1.f : 0.f;
  return r;
}
FH m33 mul33(const m33& a, const m33& b) {
  m33 r;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) r.m[i][j] = a.m[i][0] * b.m[0][j] + (a.m[i][1] * b.m[1][j] + a.m[i][2] * b.m[2][j]);
  return r;
}
FH f3 mul3v(const m33& a, f3 v) {
  return {a.m[0][0] * v.x + (a.m[0][1] * v.y + a.m[0][2] * v.z), a.m[1][0] * v.x + (a.m[1][1] * v.y + a.m[1][2] * v.z),
          a.m[2][0] * v.x + (a.m[2][1] * v.y + a.m[2][2] * v.z)};
}
// Matrix4f * Matrix4f (vectorised lazy product): ((a0b0 + a1b1) + a2b2) + a3b3
FH m44 mul44(const m44& a, const m44& b) {
  m44 r;
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      r.m[i][j] = ((a.m[i][0] * b.m[0][j] + a.m[i][1] * b.m[1][j]) + a.m[i][2] * b.m[2][j]) + a.m[i][3] * b.m[3][j];
  return r;
}
// c*I + (1-c)*r r^T + s*[r]x   (FCCF.cpp:868, :892, :1170, :1193, :1328, :1351)
FH m33 rodrigues(float c, float s, f3 r) {
  const float rv[3] = {r.x, r.y, r.z};
  const float rx[3][3] = {{0.f, -r.z, r.y}, {r.z, 0.f, -r.x}, {-r.y, r.x, 0.f}};
  m33 R;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R.m[i][j] = (c * (i == j ? 1.f : 0.f) + (1.f - c) * (rv[i] * rv[j])) + s * rx[i][j];
  return R;
}

// double Vector3 (SSE2 Packet2d redux): (a0b0 + a1b1) + a2b2
FH double dot3d(double a0, double a1, double a2, double b0, double b1, double b2) {
  return (a0 * b0 + a1 * b1) + a2 * b2;
}

// compute_normal_angel (FCCF.cpp:369-377) up to the acos: the float cos_theta.
FH float normal_cos(float x1, float y1, float z1, float x2, float y2, float z2) {
  const double a0 = x1, a1 = y1, a2 = z1, b0 = x2, b1 = y2, b2 = z2;
  const float dp = (float)dot3d(a0, a1, a2, b0, b1, b2);
  const double na = sqrt(dot3d(a0, a1, a2, a0, a1, a2));
  const double nb = sqrt(dot3d(b0, b1, b2, b0, b1, b2));
  return (float)((double)dp / (na * nb));
}
FH float normal_cos(f3 a, f3 b) { return normal_cos(a.x, a.y, a.z, b.x, b.y, b.z); }
// normal_cos with both double norms precomputed (same bits: na = sqrt(a.a), nb = sqrt(b.b))
FH double norm3d(float x, float y, float z) {
  const double a0 = x, a1 = y, a2 = z;
  return sqrt(dot3d(a0, a1, a2, a0, a1, a2));
}
FH float normal_cos_pre(float x1, float y1, float z1, double na, float x2, float y2, float z2, double nb) {
  const float dp = (float)dot3d((double)x1, (double)y1, (double)z1, (double)x2, (double)y2, (double)z2);
  return (float)((double)dp / (na * nb));
}

// theta(c) = float(double(acosf(c) * 180.f) / M_PI); acosf(c) := float(acos(double c)).
// Host-only by policy: the device never evaluates acos, it compares c against the
// exact cut points of AngleCuts (theta is monotone non-increasing in c).
inline float theta_of_cos_host(float c) {
  const float a = (float)acos((double)c);
  return (float)((double)(a * 180.0f) / 3.14159265358979323846);
}

// Threshold cut points: theta(c) > thr  <=>  -1 <= c < gt ;  theta(c) < thr  <=>  lt < c <= 1
// (theta(c) is NaN outside [-1,1], which makes both comparisons false, as in the reference).
struct AngleCut { float gt, lt; };
FH bool angle_gt(float c, AngleCut k) { return c >= -1.0f && c < k.gt; }
FH bool angle_lt(float c, AngleCut k) { return c > k.lt && c <= 1.0f; }

// compare_plane (FCCF.cpp:391-407)
FH bool compare_plane(f3 n1, f3 c1, f3 n2, f3 c2, float l, float k) {
  const float dx = c1.x - c2.x, dy = c1.y - c2.y, dz = c1.z - c2.z;
  const float len = sqrtf(dx * dx + dy * dy + dz * dz);
  const double e0 = (double)(dx / len), e1 = (double)(dy / len), e2 = (double)(dz / len);
  const float a = (float)fabs(dot3d(n1.x, n1.y, n1.z, e0, e1, e2));
  const float b = (float)fabs(dot3d(n2.x, n2.y, n2.z, e0, e1, e2));
  const float thr = l / (k * len + 1.f);
  return a < thr && b < thr;
}

// Eigen::Quaternionf(const Matrix3f&) (Shoemake), no normalisation.
FH quatf quat_from_rot(const m33& R) {
  quatf q;
  float t = R.m[0][0] + (R.m[1][1] + R.m[2][2]);
  if (t > 0.f) {
    t = sqrtf(t + 1.0f);
    q.w = 0.5f * t;
    t = 0.5f / t;
    q.x = (R.m[2][1] - R.m[1][2]) * t;
    q.y = (R.m[0][2] - R.m[2][0]) * t;
    q.z = (R.m[1][0] - R.m[0][1]) * t;
  } else {
    int i = 0;
    if (R.m[1][1] > R.m[0][0]) i = 1;
    if (R.m[2][2] > R.m[i][i]) i = 2;
    const int j = (i + 1) % 3, k = (j + 1) % 3;
    t = sqrtf(R.m[i][i] - R.m[j][j] - R.m[k][k] + 1.0f);
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
FH m33 rot_from_quat(quatf q) {
  const float tx = 2.f * q.x, ty = 2.f * q.y, tz = 2.f * q.z;
  const float twx = tx * q.w, twy = ty * q.w, twz = tz * q.w;
  const float txx = tx * q.x, txy = ty * q.x, txz = tz * q.x;
  const float tyy = ty * q.y, tyz = tz * q.y, tzz = tz * q.z;
  m33 r;
  r.m[0][0] = 1.f - (tyy + tzz); r.m[0][1] = txy - twz; r.m[0][2] = txz + twy;
  r.m[1][0] = txy + twz; r.m[1][1] = 1.f - (txx + tzz); r.m[1][2] = tyz - twx;
  r.m[2][0] = txz - twy; r.m[2][1] = tyz + twx; r.m[2][2] = 1.f - (txx + tyy);
  return r;
}
// Quaternionf * Vector3f (quat_transform_vector)
FH f3 quat_rotate(quatf q, f3 v) {
  const f3 qv = {q.x, q.y, q.z};
  f3 uv = cross3(qv, v);
  uv = {uv.x + uv.x, uv.y + uv.y, uv.z + uv.z};
  const f3 c = cross3(qv, uv);
  return {(v.x + q.w * uv.x) + c.x, (v.y + q.w * uv.y) + c.y, (v.z + q.w * uv.z) + c.z};
}

// pcl::detail::Transformer<float> (SSE): se3 = x*c0 + (y*c1 + (z*c2 + c3)), so3 without c3
FH f3 tf_se3(const m44& T, float x, float y, float z) {
  return {x * T.m[0][0] + (y * T.m[0][1] + (z * T.m[0][2] + T.m[0][3])),
          x * T.m[1][0] + (y * T.m[1][1] + (z * T.m[1][2] + T.m[1][3])),
          x * T.m[2][0] + (y * T.m[2][1] + (z * T.m[2][2] + T.m[2][3]))};
}
FH f3 tf_so3(const m44& T, float x, float y, float z) {
  return {x * T.m[0][0] + (y * T.m[0][1] + z * T.m[0][2]), x * T.m[1][0] + (y * T.m[1][1] + z * T.m[1][2]),
          x * T.m[2][0] + (y * T.m[2][1] + z * T.m[2][2])};
}

// Rotation from two averaged axes (transform_cluster :1148-1196, fuse_answer :1306-1354).
FH m33 axes_to_rot(f3 nt1, f3 nt2) {
  const f3 ns1 = {1.f, 0.f, 0.f};
  f3 ns2 = {0.f, 1.f, 0.f};
  const f3 r1 = normalize3(cross3(ns1, nt1));
  const float c1 = dot3(nt1, ns1);
  const float s1 = dot3(nt1, cross3(r1, ns1));
  const m33 R1 = rodrigues(c1, s1, r1);
  ns2 = mul3v(R1, ns2);
  const f3 r2 = nt1;
  const float ns2dnt2 = dot3(ns2, nt2), ns2dr2 = dot3(ns2, r2), nt2dr2 = dot3(nt2, r2);
  const float r2cns2dnt2 = dot3(cross3(r2, ns2), nt2);
  const float c2 = (ns2dnt2 - (ns2dr2 * nt2dr2)) / (1.f - (ns2dr2 * nt2dr2));
  const float s2 = (r2cns2dnt2) / (1.f - (ns2dr2 * nt2dr2));
  const m33 R2 = rodrigues(c2, s2, r2);
  return mul33(R2, R1);
}

// Octree key bounds of PCL OctreePointCloud after adoptBoundingBoxToPoint (App. A3).
struct OctState {
  double min[3];
  double max[3];
  uint32_t depth;
  uint32_t defined;
};

FH void oct_first(OctState& b, double res, const float* p) {
  const float eps = 1.1920928955078125e-07f;  // FLT_EPSILON
  for (int a = 0; a < 3; ++a) {
    b.min[a] = (double)p[a] - res / 2;
    b.max[a] = (double)p[a] + res / 2;
  }
  uint32_t mk[3];
  for (int a = 0; a < 3; ++a) mk[a] = (uint32_t)ceil((b.max[a] - b.min[a] - eps) / res);
  uint32_t mv = mk[0] > mk[1] ? mk[0] : mk[1];
  mv = mv > mk[2] ? mv : mk[2];
  mv = mv > 2u ? mv : 2u;
  uint32_t d = (uint32_t)ceil(log((double)mv) / log(2.0) - eps);
  b.depth = d < 32u ? d : 32u;
  const double side = (double)(1u << b.depth) * res;
  for (int a = 0; a < 3; ++a) {
    const double over = (side - (b.max[a] - b.min[a])) / 2.0;
    if (over > eps) {
      b.min[a] -= over;
      b.max[a] += over;
    }
  }
  b.defined = 1;
}

// One point through adoptBoundingBoxToPoint; returns true if the bounds changed.
FH bool oct_adopt(OctState& b, double res, const float* p) {
  const float eps = 1.1920928955078125e-07f;
  if (!b.defined) {
    oct_first(b, res, p);
    return true;
  }
  bool changed = false;
  while (true) {
    bool up[3], any = false;
    for (int a = 0; a < 3; ++a) {
      const bool lo = (double)p[a] < b.min[a];
      up[a] = (double)p[a] >= b.max[a];
      any = any || lo || up[a];
    }
    if (!any) break;
    changed = true;
    double side = (double)(1 << b.depth) * res;
    for (int a = 0; a < 3; ++a)
      if (!up[a]) b.min[a] -= side;
    b.depth++;
    side = (double)(1 << b.depth) * res - eps;
    for (int a = 0; a < 3; ++a) b.max[a] = b.min[a] + side;
  }
  return changed;
}

FH bool oct_inside(const OctState& b, float x, float y, float z) {
  return !((double)x < b.min[0] || (double)y < b.min[1] || (double)z < b.min[2] || (double)x >= b.max[0] ||
           (double)y >= b.max[1] || (double)z >= b.max[2]);
}

// Morton code of final leaf keys, x most significant within each level (DFS order
// of getOccupiedVoxelCenters, child index (x<<2)|(y<<1)|z).
// bit i of v (i < 21) to bit 3i
FH uint64_t spread3(uint64_t v) {
  v &= 0x1fffffull;
  v = (v | v << 32) & 0x1f00000000ffffull;
  v = (v | v << 16) & 0x1f0000ff0000ffull;
  v = (v | v << 8) & 0x100f00f00f00f00full;
  v = (v | v << 4) & 0x10c30c30c30c30c3ull;
  v = (v | v << 2) & 0x1249249249249249ull;
  return v;
}
FH uint64_t morton_code(uint32_t kx, uint32_t ky, uint32_t kz, uint32_t depth) {
  if (depth <= 21) {  // the loop below, as masked bit spreads (bit b of kx at 3b + 2)
    const uint32_t mk = (uint32_t)((1ull << depth) - 1ull);
    return (spread3(kx & mk) << 2) | (spread3(ky & mk) << 1) | spread3(kz & mk);
  }
  uint64_t m = 0;
  for (int bit = (int)depth - 1; bit >= 0; --bit)
    m = (m << 3) | ((uint64_t)((kx >> bit) & 1u) << 2) | ((uint64_t)((ky >> bit) & 1u) << 1) | (uint64_t)((kz >> bit) & 1u);
  return m;
}
FH uint64_t oct_code(const OctState& b, double res, float x, float y, float z) {
  const uint32_t kx = (uint32_t)(((double)x - b.min[0]) / res);
  const uint32_t ky = (uint32_t)(((double)y - b.min[1]) / res);
  const uint32_t kz = (uint32_t)(((double)z - b.min[2]) / res);
  return morton_code(kx, ky, kz, b.depth);
}
// (uint32_t)(a / res), the key of an offset a from the octree's minimum, with inv = 1.0 /
// res: the quotient through a multiplication (relative error below 2^-52) truncates the
// same way as the IEEE division unless an integer lies within 2^-50 of it; there, and for
// a <= 0, the division itself runs.  Bit-identical to the division form, without a
// double-precision division per coordinate on the device.
FH uint32_t key_div(double a, double res, double inv) {
  const double q = a * inv;
  const double f = floor(q);
  const double m = q * 0x1p-50;
  if (a > 0.0 && q - f > m && (f + 1.0) - q > m) return (uint32_t)f;
  return (uint32_t)(a / res);
}
FH uint64_t oct_code(const OctState& b, double res, double inv, float x, float y, float z) {
  const uint32_t kx = key_div((double)x - b.min[0], res, inv);
  const uint32_t ky = key_div((double)y - b.min[1], res, inv);
  const uint32_t kz = key_div((double)z - b.min[2], res, inv);
  return morton_code(kx, ky, kz, b.depth);
}

FH bool finite3(float x, float y, float z) { return isfinite(x) && isfinite(y) && isfinite(z); }

}  // namespace fccf
