// Deterministic synthetic scene generator.
//
// The reference ships no data and no tests, so every parity case
// and the bench workload come from this generator: an axis-aligned room with
// furniture (≥6 plane orientations, distinct plane sizes) plus ~5 % non-planar
// clutter, sampled uniformly by area with Gaussian noise along the normal.
// RNG is SplitMix64 + Box–Muller in double, so a (seed, N, room) triple always
// yields the same float32 points on the same libm.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <vector>

#include "../../include/fccf.h"

namespace {

struct Rng {
  uint64_t s;
  explicit Rng(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  double uni() { return (double)(next() >> 11) * (1.0 / 9007199254740992.0); }  // [0,1)
  double gauss() {
    double u1 = 1.0 - uni();  // (0,1]
    double u2 = uni();
    return std::sqrt(-2.0 * std::log(u1)) * std::cos(6.283185307179586 * u2);
  }
};

struct V3 { double x, y, z; };
static V3 add(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static V3 mul(V3 a, double s) { return {a.x * s, a.y * s, a.z * s}; }

// A planar parallelogram o + u*a + v*b, u,v in [0,1], unit normal n.
struct Quad { V3 o, a, b, n; double area; };
// Sphere / vertical cylinder clutter.
struct Sphere { V3 c; double r; };
struct Cyl { V3 c; double r, h; };

static Quad quad(V3 o, V3 a, V3 b, V3 n) {
  V3 cr = {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
  return {o, a, b, n, std::sqrt(cr.x * cr.x + cr.y * cr.y + cr.z * cr.z)};
}

// Box resting on the floor: base corner c, extents (w,d,h), yaw (rad). Top + 4 sides.
static void add_box(std::vector<Quad>& q, V3 c, double w, double d, double h, double yaw) {
  double cs = std::cos(yaw), sn = std::sin(yaw);
  V3 ex = {cs * w, sn * w, 0}, ey = {-sn * d, cs * d, 0}, ez = {0, 0, h};
  V3 nx = {cs, sn, 0}, ny = {-sn, cs, 0};
  q.push_back(quad(add(c, ez), ex, ey, {0, 0, 1}));                 // top
  q.push_back(quad(c, ex, ez, mul(ny, -1)));                        // front (-y')
  q.push_back(quad(add(c, ey), ex, ez, ny));                        // back  (+y')
  q.push_back(quad(c, ey, ez, mul(nx, -1)));                        // left  (-x')
  q.push_back(quad(add(c, ex), ey, ez, nx));                        // right (+x')
}

struct Scene {
  std::vector<Quad> quads;
  std::vector<Sphere> spheres;
  std::vector<Cyl> cyls;
  double plane_area = 0, clutter_area = 0;
};

static Scene make_scene(double Lx, double Ly, double Lz) {
  Scene s;
  auto& q = s.quads;
  q.push_back(quad({0, 0, 0}, {Lx, 0, 0}, {0, Ly, 0}, {0, 0, 1}));     // floor
  q.push_back(quad({0, 0, Lz}, {Lx, 0, 0}, {0, Ly, 0}, {0, 0, -1}));   // ceiling
  q.push_back(quad({0, 0, 0}, {0, Ly, 0}, {0, 0, Lz}, {1, 0, 0}));     // wall x=0
  q.push_back(quad({Lx, 0, 0}, {0, Ly, 0}, {0, 0, Lz}, {-1, 0, 0}));   // wall x=Lx
  q.push_back(quad({0, 0, 0}, {Lx, 0, 0}, {0, 0, Lz}, {0, 1, 0}));     // wall y=0
  q.push_back(quad({0, Ly, 0}, {Lx, 0, 0}, {0, 0, Lz}, {0, -1, 0}));   // wall y=Ly
  // 35 degree ramp, 4 m along the slope x 3 m wide, rising along +x.
  const double a35 = 35.0 * 3.14159265358979323846 / 180.0;
  q.push_back(quad({0.15 * Lx, 0.55 * Ly, 0}, {4 * std::cos(a35), 0, 4 * std::sin(a35)}, {0, 3, 0},
                   {-std::sin(a35), 0, std::cos(a35)}));
  add_box(q, {0.55 * Lx, 0.2 * Ly, 0}, 2.0, 1.0, 1.0, 0.0);
  add_box(q, {0.35 * Lx, 0.75 * Ly, 0}, 1.2, 0.8, 0.7, 20.0 * 3.14159265358979323846 / 180.0);
  q.push_back(quad({0.7 * Lx, 0.6 * Ly, 0.75}, {2, 0, 0}, {0, 1, 0}, {0, 0, 1}));  // table top
  for (auto& x : q) s.plane_area += x.area;
  // clutter: 10 spheres resting on the floor, 4 vertical cylinders
  const double fx[10] = {0.08, 0.22, 0.31, 0.47, 0.52, 0.63, 0.74, 0.86, 0.41, 0.27};
  const double fy[10] = {0.12, 0.33, 0.88, 0.45, 0.71, 0.15, 0.38, 0.82, 0.22, 0.57};
  for (int i = 0; i < 10; ++i) {
    double r = 0.3 + 0.3 * (double)i / 9.0;
    s.spheres.push_back({{fx[i] * Lx, fy[i] * Ly, r}, r});
    s.clutter_area += 4 * 3.14159265358979323846 * r * r;
  }
  const double cx[4] = {0.18, 0.44, 0.67, 0.9}, cy[4] = {0.8, 0.1, 0.9, 0.5};
  for (int i = 0; i < 4; ++i) {
    s.cyls.push_back({{cx[i] * Lx, cy[i] * Ly, 0}, 0.2, 1.5});
    s.clutter_area += 2 * 3.14159265358979323846 * 0.2 * 1.5;
  }
  return s;
}

static void sample_point(const Scene& s, Rng& g, double sigma, V3& out) {
  V3 p, n;
  if (g.uni() < 0.05) {  // clutter: ~5 % of points
    double pick = g.uni() * s.clutter_area, acc = 0;
    for (auto& sp : s.spheres) {
      acc += 4 * 3.14159265358979323846 * sp.r * sp.r;
      if (pick < acc) {
        double z = 2 * g.uni() - 1, ph = 6.283185307179586 * g.uni(), rr = std::sqrt(1 - z * z);
        n = {rr * std::cos(ph), rr * std::sin(ph), z};
        p = add(sp.c, mul(n, sp.r));
        double e = sigma * g.gauss();
        out = add(p, mul(n, e));
        return;
      }
    }
    const Cyl& c = s.cyls[(size_t)(g.uni() * s.cyls.size()) % s.cyls.size()];
    double ph = 6.283185307179586 * g.uni(), h = g.uni() * c.h;
    n = {std::cos(ph), std::sin(ph), 0};
    p = {c.c.x + c.r * n.x, c.c.y + c.r * n.y, h};
    out = add(p, mul(n, sigma * g.gauss()));
    return;
  }
  double pick = g.uni() * s.plane_area, acc = 0;
  const Quad* q = &s.quads.back();
  for (auto& x : s.quads) {
    acc += x.area;
    if (pick < acc) { q = &x; break; }
  }
  double u = g.uni(), v = g.uni();
  p = add(q->o, add(mul(q->a, u), mul(q->b, v)));
  out = add(p, mul(q->n, sigma * g.gauss()));
}

}  // namespace

extern "C" int fccf_synth_scene(int64_t n, double Lx, double Ly, double Lz, uint64_t seed,
                                double crop_x_frac, float* out_xyz) {
  if (n < 0 || !out_xyz || Lx <= 0 || Ly <= 0 || Lz <= 0) return FCCF_E_ARG;
  Scene s = make_scene(Lx, Ly, Lz);
  Rng g(seed);
  const double crop = crop_x_frac > 0 ? crop_x_frac * Lx : 1e300;
  for (int64_t i = 0; i < n;) {
    V3 p;
    sample_point(s, g, 0.003, p);
    if (p.x > crop) continue;
    out_xyz[3 * i + 0] = (float)p.x;
    out_xyz[3 * i + 1] = (float)p.y;
    out_xyz[3 * i + 2] = (float)p.z;
    ++i;
  }
  return FCCF_OK;
}

// The registration pair of SURVEY.md §8(d): tar = scene (seed 2) cropped to
// x <= 0.8 Lx; src = scene (seed 1) mapped by T_gt^-1, so the expected output
// of fccf_register(src, tar) is T_gt (yaw 25 deg * roll 2 deg, t = (2,-1,0.5)).
extern "C" int fccf_synth_pair(int64_t n, double Lx, double Ly, double Lz, float* src_xyz,
                               float* tar_xyz, float T_gt_rowmajor[16]) {
  int rc = fccf_synth_scene(n, Lx, Ly, Lz, 2, 0.8, tar_xyz);
  if (rc) return rc;
  rc = fccf_synth_scene(n, Lx, Ly, Lz, 1, 0.0, src_xyz);
  if (rc) return rc;
  const double d2r = 3.14159265358979323846 / 180.0;
  const double cy = std::cos(25 * d2r), sy = std::sin(25 * d2r);
  const double cr = std::cos(2 * d2r), sr = std::sin(2 * d2r);
  // R = Rz(25) * Rx(2)
  const double R[3][3] = {{cy, -sy * cr, sy * sr}, {sy, cy * cr, -cy * sr}, {0, sr, cr}};
  const double t[3] = {2.0, -1.0, 0.5};
  for (int64_t i = 0; i < n; ++i) {
    double p[3] = {src_xyz[3 * i] - t[0], src_xyz[3 * i + 1] - t[1], src_xyz[3 * i + 2] - t[2]};
    for (int r = 0; r < 3; ++r)  // R^T (p - t)
      src_xyz[3 * i + r] = (float)(R[0][r] * p[0] + R[1][r] * p[1] + R[2][r] * p[2]);
  }
  if (T_gt_rowmajor) {
    for (int r = 0; r < 3; ++r) {
      for (int c = 0; c < 3; ++c) T_gt_rowmajor[4 * r + c] = (float)R[r][c];
      T_gt_rowmajor[4 * r + 3] = (float)t[r];
    }
    T_gt_rowmajor[12] = T_gt_rowmajor[13] = T_gt_rowmajor[14] = 0.f;
    T_gt_rowmajor[15] = 1.f;
  }
  return FCCF_OK;
}
