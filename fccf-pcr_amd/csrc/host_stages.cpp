// host_stages.cpp — serial stages of the FCCF-PCR driver kept on the host in
// round 1 (see host_stages.h).  Every expression is written in the evaluation
// order of the reference binary (fccf_math.h conventions).
#include "host_stages.h"

#include <algorithm>
#include <chrono>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <unordered_map>

namespace fccf {

namespace {

// ------------------------------------------------------------ exact angle cuts
// theta(c) is monotone non-increasing on [-1,1]; find c* with theta(c) > thr <=> c < gt
// and theta(c) < thr <=> c > lt, then verify the claim around the cut.
uint32_t okey(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
float okey_inv(uint32_t k) {
  const uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}
AngleCut make_cut_impl(float thr) {
  auto first_true = [](uint32_t lo, uint32_t hi, auto pred) {  // pred monotone false..true on [lo,hi]
    while (lo < hi) {
      const uint32_t mid = lo + (hi - lo) / 2;
      if (pred(mid)) hi = mid;
      else lo = mid + 1;
    }
    return lo;
  };
  const uint32_t lo = okey(-1.0f), hi = okey(1.0f);
  const uint32_t kg = first_true(lo, hi + 1, [&](uint32_t k) { return !(theta_of_cos_host(okey_inv(k)) > thr); });
  const uint32_t kl = first_true(lo, hi + 1, [&](uint32_t k) { return theta_of_cos_host(okey_inv(k)) < thr; });
  AngleCut c;
  c.gt = okey_inv(kg);
  c.lt = okey_inv(kl - 1);
  for (int64_t d = -4096; d <= 4096; ++d) {  // monotonicity check around both cuts
    for (uint32_t base : {kg, kl}) {
      const int64_t k = (int64_t)base + d;
      if (k < (int64_t)lo || k > (int64_t)hi) continue;
      const float v = okey_inv((uint32_t)k);
      const float th = theta_of_cos_host(v);
      if ((th > thr) != (v >= -1.0f && v < c.gt) || (th < thr) != (v > c.lt && v <= 1.0f))
        throw Error(FCCF_E_INTERNAL, "angle cut not monotone");
    }
  }
  return c;
}

}  // namespace

AngleCut make_cut(float thr) {  // memoised per thread: thresholds are few and fixed per call
  static thread_local std::vector<std::pair<float, AngleCut>> memo;
  for (const auto& m : memo)
    if (m.first == thr) return m.second;
  const AngleCut c = make_cut_impl(thr);
  memo.push_back({thr, c});
  return c;
}

static inline float angle_deg(float x1, float y1, float z1, float x2, float y2, float z2) {
  return theta_of_cos_host(normal_cos(x1, y1, z1, x2, y2, z2));
}

// ------------------------------------------------------------------ growing
namespace {
struct Group {
  std::vector<int> mem;             // voxel indices in voxelgrothnode order
  float s = 0, sc[3] = {0, 0, 0}, sn[3] = {0, 0, 0};  // running recompute sums
  float ac[3], an[3], fps;
  double nan_ = 0;                  // norm3d(an), refreshed with the averages
  bool alloc = false;
};

inline void add_member(Group& g, const VoxRec& v) {
  g.s = g.s + (float)v.count;
  for (int a = 0; a < 3; ++a) {
    g.sc[a] = g.sc[a] + v.c[a] * (float)v.count;
    g.sn[a] = g.sn[a] + v.n[a] * (float)v.count;
  }
}
inline void set_avg(Group& g) {  // the recompute's averages (:580-586)
  g.fps = g.s;
  for (int a = 0; a < 3; ++a) {
    g.ac[a] = g.sc[a] / g.s;
    g.an[a] = g.sn[a] / g.s;
  }
  g.nan_ = norm3d(g.an[0], g.an[1], g.an[2]);
}
}  // namespace

// Direction index of unit normals for region growing's scan: cube-map cells (face =
// the dominant axis and its sign, then a DG x DG grid over the other two coordinates
// divided by the dominant one), each with its voxels in ascending index, its mean
// direction and angular radius.  candidates(a, after) lists, ascending, the voxels after
// index `after` and not yet allocated in every cell whose cone could hold a direction
// within `cone` of a -- cos(angle(a, center)) >= cos(cone + radius + slack) -- plus the
// non-finite normals; an undefined a (not finite, or not of unit length) lists them all.
namespace {
struct DirIndex {
  static constexpr int DG = 8, NC = 6 * DG * DG;  // cell NC: non-finite / zero normals
  std::vector<int> idx;                  // voxels by cell, ascending within a cell
  int beg[NC + 2], len[NC + 1];          // cell c: idx[beg[c], beg[c] + len[c]) (allocated ones dropped)
  float cx[NC], cy[NC], cz[NC], ccos[NC];  // unit mean direction, cos(cone + radius + slack)
  int used[NC], nused = 0;               // non-empty cells
  DirIndex(const float* ux, const float* uy, const float* uz, int n, double cone) : idx(n) {
    std::vector<uint16_t> cof(n);
    int cnt[NC + 1] = {};
    for (int j = 0; j < n; ++j) ++cnt[cof[j] = (uint16_t)cell_of(ux[j], uy[j], uz[j])];
    beg[0] = 0;
    for (int c = 0; c <= NC; ++c) {
      beg[c + 1] = beg[c] + cnt[c];
      len[c] = 0;
    }
    for (int j = 0; j < n; ++j) idx[beg[cof[j]] + len[cof[j]]++] = j;
    for (int c = 0; c < NC; ++c) {
      if (!len[c]) continue;
      used[nused++] = c;
      const int* l = idx.data() + beg[c];
      double m[3] = {0, 0, 0};
      for (int q = 0; q < len[c]; ++q) { m[0] += ux[l[q]]; m[1] += uy[l[q]]; m[2] += uz[l[q]]; }
      const double r = std::sqrt(m[0] * m[0] + m[1] * m[1] + m[2] * m[2]);
      for (double& x : m) x /= r;
      double mind = 1.0;  // cos of the cell's angular radius
      for (int q = 0; q < len[c]; ++q) mind = std::min(mind, m[0] * ux[l[q]] + m[1] * uy[l[q]] + m[2] * uz[l[q]]);
      const double lim = cone + std::acos(std::max(-1.0, std::min(1.0, mind))) + 1e-3;
      cx[c] = (float)m[0]; cy[c] = (float)m[1]; cz[c] = (float)m[2];
      ccos[c] = lim >= 3.14159265358979323846 ? -2.f : (float)std::cos(lim) - 1e-5f;
    }
  }
  static int cell_of(float x, float y, float z) {
    if (!(std::isfinite(x) && std::isfinite(y) && std::isfinite(z))) return NC;
    const float ax = std::fabs(x), ay = std::fabs(y), az = std::fabs(z);
    int f;
    float s, t, m;
    if (ax >= ay && ax >= az) { f = x < 0 ? 1 : 0; m = ax; s = y; t = z; }
    else if (ay >= az) { f = y < 0 ? 3 : 2; m = ay; s = x; t = z; }
    else { f = z < 0 ? 5 : 4; m = az; s = x; t = y; }
    if (!(m > 0.f)) return NC;
    auto q = [](float v) { return std::min(DG - 1, std::max(0, (int)((v + 1.f) * (0.5f * DG)))); };
    return f * DG * DG + q(s / m) * DG + q(t / m);
  }
  void candidates(const float a[3], int after, const char* va, std::vector<int>& out) {
    out.clear();
    const bool ok = std::isfinite(a[0]) && std::isfinite(a[1]) && std::isfinite(a[2]) &&
                    std::fabs(a[0] * a[0] + a[1] * a[1] + a[2] * a[2] - 1.f) < 1e-3f;
    auto take = [&](int c) {
      // drop allocated voxels from the cell for good (they never return), keep the rest
      int* l = idx.data() + beg[c];
      int w = 0;
      for (int q = 0; q < len[c]; ++q) {
        const int j = l[q];
        if (va[j]) continue;
        l[w++] = j;
        if (j > after) out.push_back(j);
      }
      len[c] = w;
    };
    for (int u = 0; u < nused; ++u) {
      const int c = used[u];
      if (len[c] && (!ok || a[0] * cx[c] + a[1] * cy[c] + a[2] * cz[c] >= ccos[c])) take(c);
    }
    take(NC);
    std::sort(out.begin(), out.end());
  }
};
}  // namespace

std::vector<GroupOut> grow_groups(const VoxRec* vox, int nv, const fccf_params& P) {
  // compare_normal(...) == !(theta > thr) == !angle_gt(cos, cut): no acos in the O(V^2) loops
  const AngleCut cut1 = make_cut(P.normal_vector_threshold1), cut2 = make_cut(P.normal_vector_threshold2);
  std::vector<char> va(nv, 0);
  std::vector<Group> G;
  // stage 1 (:536-593): recompute-from-scratch == running sums in member order (App. B Q7)
  // The predicate is `same && cop` with no side effects, so `cop` is evaluated only when
  // `same` holds.  A seed's scan visits the still-unallocated voxels in index order and
  // every rejection leaves the state unchanged, so it may skip any voxel the exact angle
  // test would reject: the scan visits only candidates, the voxels whose normals lie in
  // direction buckets (cube-map cells, DirIndex) near the seed's normal, in index order.
  // A voxel that passes the exact test against the group normal g lies within thr1 of g;
  // while g stays within DRIFT of the anchor the candidates were chosen for, it lies
  // within thr1 + DRIFT of the anchor, so its bucket is among those selected (bucket
  // radius and rounding slack included); when g drifts further, the candidates are
  // chosen again for the rest of the scan.  Non-finite or zero normals (NaN cosines,
  // never rejected) are always candidates; an undefined group direction scans all.
  std::vector<double> vnv(nv);
  std::vector<float> ux(nv), uy(nv), uz(nv);
  for (int j = 0; j < nv; ++j) {
    vnv[j] = norm3d(vox[j].n[0], vox[j].n[1], vox[j].n[2]);
    const double r = vnv[j];
    ux[j] = (float)(vox[j].n[0] / r); uy[j] = (float)(vox[j].n[1] / r); uz[j] = (float)(vox[j].n[2] / r);
  }
  constexpr double DRIFT = 0.1, SLACK = 5e-3;  // radians
  const double theta1 = (double)P.normal_vector_threshold1 * (3.14159265358979323846 / 180.0);
  DirIndex dix(ux.data(), uy.data(), uz.data(), nv, theta1 + DRIFT + SLACK);
  const float cos_drift = (float)std::cos(DRIFT);
  std::vector<int> cand;
  for (int i = 0; i < nv; ++i) {
    if (va[i]) continue;
    Group g;
    va[i] = 1;
    g.mem.push_back(i);
    add_member(g, vox[i]);
    g.fps = (float)vox[i].count;
    for (int a = 0; a < 3; ++a) { g.an[a] = vox[i].n[a]; g.ac[a] = vox[i].c[a]; }
    g.nan_ = vnv[i];
    g.mem.reserve(64);
    float anc[3];
    size_t k = 0;
    auto choose = [&](int after) {  // candidates after index `after`, for the current g
      const double r = g.nan_;
      for (int a = 0; a < 3; ++a) anc[a] = (float)(g.an[a] / r);
      dix.candidates(anc, after, va.data(), cand);
      k = 0;
    };
    choose(i);
    while (k < cand.size()) {
      const int jj = cand[k++];
      if (va[jj]) continue;
      const VoxRec& v = vox[jj];
      if (angle_gt(normal_cos_pre(g.an[0], g.an[1], g.an[2], g.nan_, v.n[0], v.n[1], v.n[2], vnv[jj]), cut1)) continue;
      if (compare_plane(f3{g.an[0], g.an[1], g.an[2]}, f3{g.ac[0], g.ac[1], g.ac[2]}, f3{v.n[0], v.n[1], v.n[2]},
                        f3{v.c[0], v.c[1], v.c[2]}, P.parameter_l1, P.parameter_k1)) {
        g.mem.push_back(jj);
        va[jj] = 1;
        add_member(g, v);
        set_avg(g);
        // drift: cos(anchor, g) >= cos(DRIFT), as anc . an >= cos(DRIFT) |an| (an of zero or
        // non-finite length fails it: choose() then scans everything)
        const float cd = anc[0] * g.an[0] + anc[1] * g.an[1] + anc[2] * g.an[2];
        if (!(g.nan_ > 0.0 && cd >= cos_drift * (float)g.nan_)) choose(jj);
      }
    }
    G.push_back(std::move(g));
  }
  // stage 2 (:595-648): seeds never mark themselves allocated (Q6).  The angle test is
  // prefiltered as in stage 1: with unit group normals in float, cf = a.b is within ~1e-6
  // of the exact cosine, so cf < cut2.gt - d and cf > -1 + d reject for sure (every
  // other pair, NaN included, takes the exact test).  Only group i's normal changes
  // during its sweeps.
  const size_t ng = G.size();
  std::vector<float> gx(ng), gy(ng), gz(ng);
  auto unit_of = [&](size_t k) {
    const double r = G[k].nan_;
    gx[k] = (float)(G[k].an[0] / r); gy[k] = (float)(G[k].an[1] / r); gz[k] = (float)(G[k].an[2] / r);
  };
  for (size_t k = 0; k < ng; ++k) unit_of(k);
  constexpr float PF_D = 1e-4f;
  const float pf_hi = cut2.gt - PF_D, pf_lo = -1.0f + PF_D;
  for (size_t i = 0; i < ng; ++i) {
    if (G[i].alloc) continue;
    bool newadd = true;
    while (newadd) {
      newadd = false;
      for (size_t j = 0; j < ng; ++j) {
        if (j == i || G[j].alloc) continue;
        const float cf = gx[i] * gx[j] + gy[i] * gy[j] + gz[i] * gz[j];
        if (cf < pf_hi && cf > pf_lo) continue;
        Group& a = G[i];
        Group& b = G[j];
        if (angle_gt(normal_cos_pre(a.an[0], a.an[1], a.an[2], a.nan_, b.an[0], b.an[1], b.an[2], b.nan_), cut2))
          continue;
        if (compare_plane(f3{a.an[0], a.an[1], a.an[2]}, f3{a.ac[0], a.ac[1], a.ac[2]}, f3{b.an[0], b.an[1], b.an[2]},
                          f3{b.ac[0], b.ac[1], b.ac[2]}, P.parameter_l2, P.parameter_k2)) {
          newadd = true;
          b.alloc = true;
          for (int m : b.mem) {
            a.mem.push_back(m);
            add_member(a, vox[m]);
          }
          set_avg(a);
          unit_of(i);
        }
      }
    }
  }
  std::vector<GroupOut> out(G.size());
  for (size_t i = 0; i < G.size(); ++i) {
    std::memcpy(out[i].ac, G[i].ac, 12);
    std::memcpy(out[i].an, G[i].an, 12);
    out[i].fps = G[i].fps;
    out[i].alloc = G[i].alloc;
    out[i].mem = std::move(G[i].mem);
  }
  return out;
}

GrowOut select_groups(const std::vector<GroupOut>& G, const VoxRec* vox, const fccf_params& P) {
  // range_face (:409-427): exchange sort on voxel counts, emulated on indices
  const auto t_sel = std::chrono::steady_clock::now();  // range_face + selection from here
  std::vector<int> ord(G.size());
  for (size_t i = 0; i < G.size(); ++i) ord[i] = (int)i;
  for (size_t i = 0; i + 1 < ord.size(); ++i)
    for (size_t j = i + 1; j < ord.size(); ++j)
      if (G[ord[i]].mem.size() < G[ord[j]].mem.size()) std::swap(ord[i], ord[j]);
  GrowOut out;
  for (int k : ord) {
    const GroupOut& g = G[k];
    Plane p;
    std::memcpy(p.c, g.ac, 12);
    std::memcpy(p.n, g.an, 12);
    p.fps = g.fps;
    p.nvox = (int32_t)g.mem.size();
    out.groups.push_back(p);
    out.galloc.push_back(g.alloc ? 1 : 0);
  }
  int cur = 0;
  for (size_t r = 0; r < ord.size(); ++r) {
    const GroupOut& g = G[ord[r]];
    if (!g.alloc) {
      out.planes.push_back(out.groups[r]);
      double sum = 0;
      for (int m : g.mem) {
        const double th = angle_deg(g.an[0], g.an[1], g.an[2], vox[m].n[0], vox[m].n[1], vox[m].n[2]);
        sum += std::fabs(th);
      }
      sum /= (double)g.mem.size();
      out.theta.push_back(sum);
      cur++;
    }
    if ((float)cur > P.select_plane_number) break;
  }
  out.ms_select = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t_sel).count();
  return out;
}

GrowOut grow_and_select(const VoxRec* vox, int nv, const fccf_params& P) {
  return select_groups(grow_groups(vox, nv, P), vox, P);
}

std::vector<Base> select_base(const std::vector<Plane>& F, const std::vector<double>& th, const fccf_params& P,
                              int side) {
  std::vector<Base> base;
  std::vector<int32_t> type;
  const double t1 = P.rough_threshold_gl;
  for (size_t i = 0; i < F.size(); ++i)
    for (size_t j = i + 1; j < F.size(); ++j) {
      const float ang = angle_deg(F[i].n[0], F[i].n[1], F[i].n[2], F[j].n[0], F[j].n[1], F[j].n[2]);
      if (P.included_angle_min_threshold < ang && ang < P.included_angle_max_threshold) {
        base.push_back({(int32_t)i, (int32_t)j, ang, 0});
        if (th[i] <= t1 && th[j] <= t1) type.push_back(0);
        else if (th[i] > t1 && th[j] > t1) type.push_back(1);
        else if (th[i] <= t1 && th[j] > t1) type.push_back(2);
        else if (th[i] > t1 && th[j] <= t1) type.push_back(2);
      }
    }
  // type_index is indexed by the pair's position even when NaN roughness made it
  // shorter (Q5); positions past its end get a sentinel that matches nothing.
  for (size_t k = 0; k < base.size(); ++k) base[k].type = k < type.size() ? type[k] : (side == 1 ? -1 : -2);
  return base;
}

// ------------------------------------------------------------------ clustering
QT qt_from_T(const m44& T) {
  m33 R;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) R.m[i][j] = T.m[i][j];
  const quatf q = quat_from_rot(R);
  return {q.w, q.x, q.y, q.z, T.m[0][3], T.m[1][3], T.m[2][3], 0u};
}

m44 T_from_qt(const QT& t) {
  const m33 R = rot_from_quat(quatf{t.qw, t.qx, t.qy, t.qz});
  m44 T = eye44();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T.m[i][j] = R.m[i][j];
  T.m[0][3] = t.tx; T.m[1][3] = t.ty; T.m[2][3] = t.tz;
  return T;
}

// The host radius search of transform_cluster (:1075-1103): clusters in creation
// order (seed, size) with their members in (d2, j) order as ranges of `mem`.
static void cpu_clusters(std::vector<QT>& in, const fccf_params& P, float r2, Pool* pool, std::vector<int>& cseed,
                         std::vector<int>& csize, std::vector<int>& mem, std::vector<int>& cbeg) {
  const int n = (int)in.size();
  std::vector<int> byx;
  byx.reserve(n);
  for (int i = 0; i < n; ++i)
    if (std::isfinite(in[i].tx)) byx.push_back(i);
  std::sort(byx.begin(), byx.end(), [&](int a, int b) { return in[a].tx < in[b].tx || (in[a].tx == in[b].tx && a < b); });
  const size_t nx = byx.size();
  std::vector<float> sx(nx), sy(nx), sz3(nx);
  for (size_t p = 0; p < nx; ++p) {
    sx[p] = in[byx[p]].tx;
    sy[p] = in[byx[p]].ty;
    sz3[p] = in[byx[p]].tz;
  }
  const AngleCut ccut = make_cut(P.cluster_angel_threshold);
  std::vector<f3> xaxis(n);
  for (int i = 0; i < n; ++i) xaxis[i] = quat_rotate(quatf{in[i].qw, in[i].qx, in[i].qy, in[i].qz}, f3{1.f, 0.f, 0.f});
  // A seed's neighbour list does not depend on which candidates are already
  // allocated (:1084-1103 pushes every neighbour that passes the angle test), only
  // whether the seed itself is skipped does.  So the lists of the next NB seeds
  // that are still unallocated are built in parallel (speculatively), then applied
  // in seed order; a seed allocated by an earlier seed of its own batch is dropped.
  auto neighbours = [&](int i, std::vector<std::pair<float, int>>& nb, std::vector<float>& d2w) {
    nb.clear();
    const float xi = in[i].tx, yi = in[i].ty, zi = in[i].tz;
    if (!std::isfinite(xi)) return;
    const size_t lo = std::partition_point(sx.begin(), sx.end(), [&](float x) {
                        const float ex = xi - x;
                        return ex > 0.f && ex * ex >= r2;
                      }) - sx.begin();
    const size_t hi = std::partition_point(sx.begin() + lo, sx.end(), [&](float x) {
                        const float ex = xi - x;
                        return !(ex < 0.f && ex * ex >= r2);
                      }) - sx.begin();
    d2w.resize(hi - lo);
    for (size_t p = lo; p < hi; ++p) {  // contiguous SoA: vectorises
      const float ex = xi - sx[p], ey = yi - sy[p], ez = zi - sz3[p];
      float d2 = 0.0f;
      d2 += ex * ex;
      d2 += ey * ey;
      d2 += ez * ez;
      d2w[p - lo] = d2;
    }
    // neighbours passing the angle test, then ordered by (d2, j): the same
    // sequence as testing the (d2, j)-sorted radius-search result in order
    const f3 a = xaxis[i];
    for (size_t p = lo; p < hi; ++p) {
      if (!(d2w[p - lo] < r2)) continue;
      const int j = byx[p];
      const f3 b = xaxis[j];
      if (angle_lt(normal_cos(a.x, a.y, a.z, b.x, b.y, b.z), ccut)) nb.push_back({d2w[p - lo], j});
    }
    std::sort(nb.begin(), nb.end());
  };
  // Per seed the list costs ~0.2 us at C ~ 1e3 (measured), below a parallel_for's
  // overhead, so the speculative batches only pay for large candidate sets.
  if (n < 16384) pool = nullptr;
  const int NB = pool ? 4 * pool->size() : 1;
  std::vector<std::vector<std::pair<float, int>>> nbs(NB);
  std::vector<std::vector<float>> d2ws(NB);
  std::vector<int> seeds;
  int next = 0;
  while (true) {
    seeds.clear();  // the next NB unallocated seeds; the last candidate never seeds (:1084)
    for (; next + 1 < n && (int)seeds.size() < NB; ++next)
      if (!in[next].alloc) seeds.push_back(next);
    if (seeds.empty()) break;
    if (pool && seeds.size() > 1)
      pool->parallel_for((int)seeds.size(), [&](int b) { neighbours(seeds[b], nbs[b], d2ws[b]); });
    else
      for (size_t b = 0; b < seeds.size(); ++b) neighbours(seeds[b], nbs[b], d2ws[b]);
    for (size_t b = 0; b < seeds.size(); ++b) {
      if (in[seeds[b]].alloc) continue;  // taken by an earlier seed of this batch
      cseed.push_back(seeds[b]);
      csize.push_back((int)nbs[b].size());
      cbeg.push_back((int)mem.size());
      for (auto& e : nbs[b]) {
        in[e.second].alloc = 1u;
        mem.push_back(e.second);
      }
    }
  }
  cbeg.push_back((int)mem.size());
}

void transform_cluster(std::vector<QT>& in, std::vector<QT>& fine, int cluster_num, const fccf_params& P,
                       int64_t* nclp, Pool* pool, const uint64_t* bits) {
  const int n = (int)in.size();
  if (nclp) *nclp = 0;
  if ((float)n <= P.cluster_number_threshold) {
    if (n == 0) fine.push_back({1.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 1u});
    else fine.insert(fine.end(), in.begin(), in.end());
    return;
  }
  // KdTreeFLANN::radiusSearch(q, r): every j with L2_Simple d2 < float(r*r), sorted by (d2, j).
  // d2 = ((0 + ex^2) + ey^2) + ez^2 adds non-negative terms, so d2 < r2 implies
  // fl(ex)^2 < r2; that predicate is monotone along candidates sorted by tx, so two
  // binary searches give a window that contains every neighbour, and the exact d2
  // test inside it decides.  Candidates with non-finite tx have no neighbours
  // (d2 is NaN or inf, even against themselves).
  const float r2 = (float)((double)P.cluster_distance_threshold * (double)P.cluster_distance_threshold);
  // clusters in creation order: seed, size, and (CPU path) the members in
  // (d2, j) order as ranges of one flat list
  std::vector<int> cseed, csize, mem, cbeg;
  if (bits) {
    // Device rows (k_cluster_bits): row i = the neighbour set of seed i.  Seeds are
    // applied in order; a seed already taken is skipped (:1084-1086).
    const int W = (n + 63) / 64;
    std::vector<uint64_t> A(W, 0);
    for (int i = 0; i + 1 < n; ++i) {  // the last candidate never seeds (:1084)
      if ((A[i >> 6] >> (i & 63)) & 1u) continue;
      const uint64_t* row = bits + (size_t)i * W;
      int c = 0;
      for (int w = 0; w < W; ++w) {
        A[w] |= row[w];
        c += __builtin_popcountll(row[w]);
      }
      cseed.push_back(i);
      csize.push_back(c);
    }
  } else {
    cpu_clusters(in, P, r2, pool, cseed, csize, mem, cbeg);
  }
  const int ncl = (int)cseed.size();
  if (nclp) *nclp = (int64_t)ncl;
  if (ncl == 0) return;
  auto sz = [&](int k) { return csize[k]; };
  // members of cluster k in the radius search's (d2, j) order
  std::vector<int> mk;
  std::vector<std::pair<float, int>> mord;
  auto members = [&](int k) -> const std::vector<int>& {
    mk.clear();
    if (!bits) {
      mk.assign(mem.begin() + cbeg[k], mem.begin() + cbeg[k + 1]);
      return mk;
    }
    const int W = (n + 63) / 64;
    const int i = cseed[k];
    const uint64_t* row = bits + (size_t)i * W;
    const float xi = in[i].tx, yi = in[i].ty, zi = in[i].tz;
    mord.clear();
    for (int w = 0; w < W; ++w)
      for (uint64_t m = row[w]; m; m &= m - 1) {
        const int j = w * 64 + __builtin_ctzll(m);
        const float ex = xi - in[j].tx, ey = yi - in[j].ty, ez = zi - in[j].tz;
        float d2 = 0.0f;
        d2 += ex * ex;
        d2 += ey * ey;
        d2 += ez * ez;
        mord.push_back({d2, j});
      }
    std::sort(mord.begin(), mord.end());
    for (auto& e : mord) mk.push_back(e.second);
    return mk;
  };
  // range_cluster (:1020-1038), an exchange sort by size (swap when strictly
  // smaller).  Elements below a threshold never change the relative order of the
  // elements at or above it, and the sorted prefix holds exactly those.  With
  // t = min(max size, 2), only clusters of size >= t can be emitted below
  // (clusternum starts at the max size and the loop breaks before it drops under
  // 2), so the exchange sort is run on those alone; past them only the (smaller)
  // sizes drive the loop.  Equal sizes keep creation order.
  int mx = 0;
  for (int k = 0; k < ncl; ++k) mx = std::max(mx, sz(k));
  const int thr = std::min(mx, 2);
  std::vector<int> big;
  std::vector<int> rest_sizes;
  for (int k = 0; k < ncl; ++k) {
    if (sz(k) >= thr) big.push_back(k);
    else rest_sizes.push_back(sz(k));
  }
  for (size_t a = 0; a < big.size(); ++a)
    for (size_t b = a + 1; b < big.size(); ++b)
      if (sz(big[a]) < sz(big[b])) std::swap(big[a], big[b]);
  std::sort(rest_sizes.begin(), rest_sizes.end(), std::greater<int>());
  int clusternum = mx;
  for (size_t r = 0; r < (size_t)ncl; ++r) {
    const bool is_big = r < big.size();
    const int size_r = is_big ? sz(big[r]) : rest_sizes[r - big.size()];
    if (size_r >= clusternum) {
      const int kk = big[r];  // size_r >= clusternum >= thr: r is in the big prefix
      const std::vector<int>& mm = members(kk);
      float ax = 0, ay = 0, az = 0;
      for (int m : mm) { ax = ax + in[m].tx; ay = ay + in[m].ty; az = az + in[m].tz; }
      const float cs = (float)mm.size();
      ax = ax / cs; ay = ay / cs; az = az / cs;
      float s1[3] = {0, 0, 0}, s2[3] = {0, 0, 0};
      for (int m : mm) {
        const QT& t = in[m];
        const quatf q = {t.qw, t.qx, t.qy, t.qz};
        const f3 u = quat_rotate(q, f3{1.f, 0.f, 0.f}), v = quat_rotate(q, f3{0.f, 1.f, 0.f});
        s1[0] = s1[0] + u.x; s1[1] = s1[1] + u.y; s1[2] = s1[2] + u.z;
        s2[0] = s2[0] + v.x; s2[1] = s2[1] + v.y; s2[2] = s2[2] + v.z;
      }
      const f3 nt1 = normalize3(f3{s1[0] / cs, s1[1] / cs, s1[2] / cs});
      const f3 nt2 = normalize3(f3{s2[0] / cs, s2[1] / cs, s2[2] / cs});
      const quatf q = quat_from_rot(axes_to_rot(nt1, nt2));
      fine.push_back({q.w, q.x, q.y, q.z, ax, ay, az, 1u});
      if (fine.size() > (size_t)cluster_num) break;
    } else {
      if ((double)fine.size() < (cluster_num / 2.0)) {
        clusternum--;
        if (clusternum < 2) break;
      } else {
        break;  // stop: nothing else happens once it is set
      }
    }
  }
}

// ------------------------------------------------------------------ Ceres 1.14 LM
namespace {
inline void crossd(const double a[3], const double b[3], double r[3]) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}
// Eigen Quaterniond product, SSE2 Packet2d grouping; coefficients (x,y,z,w).
inline void qmul(const double a[4], const double b[4], double r[4]) {
  const double ax = a[0], ay = a[1], az = a[2], aw = a[3], bx = b[0], by = b[1], bz = b[2], bw = b[3];
  r[0] = (aw * bx + ay * bz) - (az * by - ax * bw);
  r[1] = (aw * by + ay * bw) + (az * bx - ax * bz);
  r[2] = (aw * bz - ay * bx) + (az * bw + ax * by);
  r[3] = (aw * bw - ay * by) - (az * bz + ax * bx);
}
// EigenQuaternionParameterization::Plus (q) and Euclidean plus (t).
inline void plus7(const double x[7], const double d[6], double o[7]) {
  const double nd = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
  if (nd > 0.0) {
    const double s = std::sin(nd) / nd;
    const double dq[4] = {s * d[0], s * d[1], s * d[2], std::cos(nd)};
    qmul(dq, x, o);
  } else {
    o[0] = x[0]; o[1] = x[1]; o[2] = x[2]; o[3] = x[3];
  }
  for (int i = 0; i < 3; ++i) o[4 + i] = x[4 + i] + d[3 + i];
}
// v' = v + w*uv + u x uv, uv = 2(u x v); Jacobian wrt (x,y,z,w).
inline void rotq(const double q[4], const double v[3], double f[3], double (*J)[4]) {
  const double u[3] = {q[0], q[1], q[2]}, w = q[3];
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

// LidarPlaneFactor (FCCF.cpp:178-208): residuals and local (6-column) Jacobian.
bool lm_eval(const float* pf, int P, const double x[7], double* cost, double* r, double* J) {
  const double* q = x;
  const double* t = x + 4;
  const double Pj[4][3] = {{q[3], q[2], -q[1]}, {-q[2], q[3], q[0]}, {q[1], -q[0], q[3]}, {-q[0], -q[1], -q[2]}};
  double c = 0.0;
  for (int b = 0; b < P; ++b) {
    const float* s = pf + 13 * b;
    const double p1[3] = {s[0], s[1], s[2]}, n1[3] = {s[3], s[4], s[5]};
    const double p2[3] = {s[6], s[7], s[8]}, n2[3] = {s[9], s[10], s[11]};
    const double w = s[12];
    double n2r[3], p2r[3], Jn[3][4], Jp[3][4];
    rotq(q, n2, n2r, J ? Jn : nullptr);
    rotq(q, p2, p2r, J ? Jp : nullptr);
    for (int i = 0; i < 3; ++i) p2r[i] = p2r[i] + t[i];
    double cr[3];
    crossd(n1, n2r, cr);
    const double nrm = std::sqrt((cr[0] * cr[0] + cr[1] * cr[1]) + cr[2] * cr[2]);
    const double d = ((n1[0] * p1[0] + n1[1] * p1[1]) + n1[2] * p1[2]) -
                     ((n2r[0] * p2r[0] + n2r[1] * p2r[1]) + n2r[2] * p2r[2]);
    const double r0 = w * nrm, r1 = w * std::sqrt(d * d);
    r[2 * b] = r0;
    r[2 * b + 1] = r1;
    c += 0.5 * (r0 * r0 + r1 * r1);
    if (!std::isfinite(r0) || !std::isfinite(r1)) return false;
    if (J) {
      double g0[7] = {0, 0, 0, 0, 0, 0, 0}, g1[7] = {0, 0, 0, 0, 0, 0, 0};
      for (int k = 0; k < 4; ++k) {
        const double col[3] = {Jn[0][k], Jn[1][k], Jn[2][k]};
        double dc[3];
        crossd(n1, col, dc);
        g0[k] = w * (((cr[0] * dc[0] + cr[1] * dc[1]) + cr[2] * dc[2]) / nrm);
        const double dd = -(((Jn[0][k] * p2r[0] + Jn[1][k] * p2r[1]) + Jn[2][k] * p2r[2]) +
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
  *cost = c;
  return true;
}

// DENSE_QR: min || [A; diag(D)] y - [b; 0] || by Householder QR (HouseholderQR form).
constexpr int LM_MAXM = 2 * 17;  // <= one pair per source plane
bool qr_solve(const double* A, int m, const double D[6], const double* b, double y[6]) {
  // Column-major [A; diag(D) | b]: column 6 is the right-hand side.  Every output
  // element is computed with the same operations in the same order as the
  // row-major HouseholderQR form (per column j, dot products run over ascending
  // rows i); the seven column dot products of a step are interleaved for ILP.
  constexpr int n = 6;
  constexpr int LD = LM_MAXM + 6;
  const int M = m + n;
  double C[n + 1][LD];
  for (int j = 0; j <= n; ++j)
    for (int i = 0; i < M; ++i) C[j][i] = 0.0;
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < n; ++j) C[j][i] = A[(size_t)i * n + j];
  for (int j = 0; j < n; ++j) C[j][m + j] = D[j];
  for (int i = 0; i < m; ++i) C[n][i] = b[i];
  for (int k = 0; k < n; ++k) {
    double* ck = C[k];
    const double c0 = ck[k];
    double tail = 0.0;
    for (int i = k + 1; i < M; ++i) tail += ck[i] * ck[i];
    double tau, beta;
    if (tail <= DBL_MIN) {
      tau = 0.0;
      beta = c0;
      for (int i = k + 1; i < M; ++i) ck[i] = 0.0;
    } else {
      beta = std::sqrt(c0 * c0 + tail);
      if (c0 >= 0.0) beta = -beta;
      const double den = c0 - beta;
      for (int i = k + 1; i < M; ++i) ck[i] = ck[i] / den;
      tau = (beta - c0) / beta;
    }
    ck[k] = beta;
    double tmp[n + 1];
    for (int j = k + 1; j <= n; ++j) tmp[j] = 0.0;
    for (int i = k + 1; i < M; ++i) {
      const double v = ck[i];
      for (int j = k + 1; j <= n; ++j) tmp[j] += v * C[j][i];
    }
    for (int j = k + 1; j <= n; ++j) {
      double* cj = C[j];
      const double t = tmp[j] + cj[k];
      cj[k] = cj[k] - tau * t;
      for (int i = k + 1; i < M; ++i) cj[i] = cj[i] - tau * ck[i] * t;
    }
  }
  for (int i = 0; i < n; ++i) y[i] = C[n][i];
  for (int k = n - 1; k >= 0; --k) {
    y[k] = y[k] / C[k][k];
    for (int i = 0; i < k; ++i) y[i] = y[i] - y[k] * C[k][i];
  }
  for (int i = 0; i < n; ++i)
    if (!std::isfinite(y[i])) return false;
  return true;
}
}  // namespace

// TrustRegionMinimizer + LevenbergMarquardtStrategy (Ceres 1.14 defaults, App. A10):
// jacobi scaling from iteration 0, LM diagonal clamp [1e-6,1e32], radius 1e4,
// function/gradient/parameter tolerances 1e-6/1e-10/1e-8, 50 iterations, returns
// the parameters of the lowest cost seen at an iteration boundary.
void lm_solve(const float* pf, int P, double best[7]) {
  const int m = 2 * P;
  double x[7] = {0, 0, 0, 1, 0, 0, 0};
  for (int i = 0; i < 7; ++i) best[i] = x[i];
  if (m > LM_MAXM) throw std::length_error("lm_solve: too many plane pairs");
  double r[LM_MAXM], J[LM_MAXM * 6], rc[LM_MAXM];
  double cost;
  if (!lm_eval(pf, P, x, &cost, r, J)) return;
  double scale[6], gmax = 0.0;
  for (int j = 0; j < 6; ++j) {
    double s = 0.0;
    for (int i = 0; i < m; ++i) s += J[(size_t)i * 6 + j] * J[(size_t)i * 6 + j];
    scale[j] = 1.0 / (1.0 + std::sqrt(s));
  }
  auto finish = [&]() {
    double g[6], ng[6], xp[7];
    for (int j = 0; j < 6; ++j) {
      double s = 0.0;
      for (int i = 0; i < m; ++i) s += J[(size_t)i * 6 + j] * r[i];
      g[j] = s;
      ng[j] = -g[j];
    }
    plus7(x, ng, xp);
    double mx = 0.0;
    for (int j = 0; j < 7; ++j) mx = std::max(mx, std::fabs(x[j] - xp[j]));
    gmax = mx;
    for (int i = 0; i < m; ++i)
      for (int j = 0; j < 6; ++j) J[(size_t)i * 6 + j] *= scale[j];
  };
  finish();
  double min_cost = cost;
  auto norm7 = [](const double* v) {
    double s = 0.0;
    for (int i = 0; i < 7; ++i) s += v[i] * v[i];
    return std::sqrt(s);
  };
  double x_norm = norm7(x);
  double radius = 1e4, decrease = 2.0, diag[6];
  bool reuse = false;
  int iteration = 0, invalid = 0;
  if (gmax <= 1e-10) return;
  while (true) {
    ++iteration;
    bool successful = false;
    if (!reuse)
      for (int j = 0; j < 6; ++j) {
        double s = 0.0;
        for (int i = 0; i < m; ++i) s += J[(size_t)i * 6 + j] * J[(size_t)i * 6 + j];
        diag[j] = std::min(std::max(s, 1e-6), 1e32);
      }
    double D[6], y[6], step[6];
    for (int j = 0; j < 6; ++j) D[j] = std::sqrt(diag[j] / radius);
    const bool solved = qr_solve(J, m, D, r, y);
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
      radius = radius / decrease;
      decrease *= 2.0;
    } else {
      invalid = 0;
      double delta[6], cand[7];
      for (int j = 0; j < 6; ++j) delta[j] = step[j] * scale[j];
      plus7(x, delta, cand);
      double ccost;
      if (!lm_eval(pf, P, cand, &ccost, rc, nullptr)) ccost = DBL_MAX;
      double sn = 0.0;
      for (int i = 0; i < 7; ++i) sn += (x[i] - cand[i]) * (x[i] - cand[i]);
      sn = std::sqrt(sn);
      if (sn <= 1e-8 * (x_norm + 1e-8)) return;
      if (std::fabs(cost - ccost) <= 1e-6 * cost) return;
      const double rho = (cost - ccost) / mcc;
      if (rho > 1e-3) {
        for (int i = 0; i < 7; ++i) x[i] = cand[i];
        x_norm = norm7(x);
        if (!lm_eval(pf, P, x, &cost, r, J)) return;
        finish();
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
    if (successful && cost < min_cost) {
      min_cost = cost;
      for (int i = 0; i < 7; ++i) best[i] = x[i];
    }
    if (iteration >= 50) return;
    if (successful && gmax <= 1e-10) return;
    if (radius <= 1e-32) return;
  }
}

float quick_verify(m44& T, const std::vector<Plane>& F1, const std::vector<Plane>& F2, const fccf_params& P,
                   int* npairs) {
  std::vector<float> pairs;
  int np = 0;
  const float score = quick_verify_pairs(T, F1, F2, P, pairs, &np);
  if (npairs) *npairs = np;
  if ((float)np >= P.required_optimize_plane) {
    double b[7];
    lm_solve(pairs.data(), np, b);
    quick_verify_refine(T, b);
  }
  return score;
}

void quick_verify_refine(m44& T, const double b[7]) {
  const m33 R = rot_from_quat(quatf{(float)b[3], (float)b[0], (float)b[1], (float)b[2]});
  m44 dT = eye44();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) dT.m[i][j] = R.m[i][j];
  dT.m[0][3] = (float)b[4]; dT.m[1][3] = (float)b[5]; dT.m[2][3] = (float)b[6];
  T = mul44(dT, T);
}

float quick_verify_pairs(const m44& T, const std::vector<Plane>& F1, const std::vector<Plane>& F2,
                         const fccf_params& P, std::vector<float>& pairs, int* npairs) {
  pairs.clear();
  int fs1 = 0, fs2 = 0;
  for (const Plane& f : F1) fs1 = (int)((float)fs1 + f.fps);
  for (const Plane& f : F2) fs2 = (int)((float)fs2 + f.fps);
  const AngleCut qcut = make_cut(P.quick_verify_angel_threshold);
  std::vector<f3> c2(F2.size()), n2(F2.size());
  for (size_t k = 0; k < F2.size(); ++k) {
    c2[k] = tf_se3(T, F2[k].c[0], F2[k].c[1], F2[k].c[2]);
    n2[k] = tf_so3(T, F2[k].n[0], F2[k].n[1], F2[k].n[2]);
  }
  int np = 0;
  for (size_t i = 0; i < F1.size(); ++i) {
    const Plane& a = F1[i];
    bool find = false;
    int best = 0;
    float best_imp = 0, best_score = 0;
    for (size_t j = 0; j < F2.size(); ++j) {
      const bool ang_ok = angle_lt(normal_cos(a.n[0], a.n[1], a.n[2], n2[j].x, n2[j].y, n2[j].z), qcut);
      const float d1 = (float)dot3d(a.n[0], a.n[1], a.n[2], a.c[0], a.c[1], a.c[2]);
      const float d2 = (float)dot3d(n2[j].x, n2[j].y, n2[j].z, c2[j].x, c2[j].y, c2[j].z);
      const float dist = std::fabs(d1 - d2);
      if (ang_ok && dist < P.quick_verify_distance_threshold) {
        find = true;
        const float s1 = a.fps, s2 = F2[j].fps;
        const float mn = s1 < s2 ? s1 : s2, mx = s1 > s2 ? s1 : s2;
        const float sc = mn / mx;
        const float imp = (2 * mn) / (float)(fs1 + fs2);
        if (sc > best_score) { best_imp = imp; best_score = sc; best = (int)j; }
      }
    }
    if (find) {
      const float rec[13] = {a.c[0], a.c[1], a.c[2], a.n[0], a.n[1], a.n[2], c2[best].x, c2[best].y, c2[best].z,
                             n2[best].x, n2[best].y, n2[best].z, best_imp};
      pairs.insert(pairs.end(), rec, rec + 13);
      ++np;
    }
  }
  if (npairs) *npairs = np;
  float score = 0;
  for (int k = 0; k < np; ++k) score = score + pairs[13 * k + 12];
  return score;
}

m44 fuse_answer(const std::vector<High>& hs, float sum) {
  float tx = 0, ty = 0, tz = 0;
  for (const High& h : hs) {
    tx = tx + h.qt.tx * (h.score / sum);
    ty = ty + h.qt.ty * (h.score / sum);
    tz = tz + h.qt.tz * (h.score / sum);
  }
  float a[3] = {0, 0, 0}, b[3] = {0, 0, 0};
  for (const High& h : hs) {
    const quatf q = {h.qt.qw, h.qt.qx, h.qt.qy, h.qt.qz};
    const f3 u = quat_rotate(q, f3{1.f, 0.f, 0.f}), v = quat_rotate(q, f3{0.f, 1.f, 0.f});
    a[0] = a[0] + u.x * (h.score / sum); a[1] = a[1] + u.y * (h.score / sum); a[2] = a[2] + u.z * (h.score / sum);
    b[0] = b[0] + v.x * (h.score / sum); b[1] = b[1] + v.y * (h.score / sum); b[2] = b[2] + v.z * (h.score / sum);
  }
  const m33 R = axes_to_rot(normalize3(f3{a[0], a[1], a[2]}), normalize3(f3{b[0], b[1], b[2]}));
  m44 T = eye44();
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T.m[i][j] = R.m[i][j];
  T.m[0][3] = tx; T.m[1][3] = ty; T.m[2][3] = tz;
  return T;
}

m44 fuse_types(const std::vector<TS> ctv[3], int analyse_max, std::vector<High>* tmp_out) {
  // sums over every type's first analyse_max candidates (:1499-1541), before any type is
  // normalised (App. B Q15)
  float score1_sum = 0.f, score2_sum = 0.f;
  for (int t = 0; t < 3; ++t)
    for (int i = 0; i < (int)ctv[t].size() && i < analyse_max; ++i) {
      score2_sum += ctv[t][i].score2;
      score1_sum += ctv[t][i].score;
    }
  std::vector<High> tmp;
  float best_best = 0.f;
  for (int t = 0; t < 3; ++t) {
    float bs = 0.f;
    m44 bt = eye44();
    for (int i = 0; i < (int)ctv[t].size() && i < analyse_max; ++i) {
      const float sc = ctv[t][i].score / score1_sum + ctv[t][i].score2 / score2_sum;
      if (sc > bs) { bs = sc; bt = ctv[t][i].T; }  // first best on ties (:1559)
    }
    if (best_best < bs) best_best = bs;
    tmp.push_back({qt_from_T(bt), bs});
  }
  std::vector<High> hs;
  float score_sum = 0.f;
  for (const High& h : tmp)
    if (h.score > best_best * 0.8) {  // (float * double: the cut in double, :1601)
      hs.push_back(h);
      score_sum += h.score;
    }
  if (tmp_out) *tmp_out = tmp;
  return fuse_answer(hs, score_sum);
}

}  // namespace fccf
