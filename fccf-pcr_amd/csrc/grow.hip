// grow.hip — K4: face_extrate's region growing on the GPU (FCCF.cpp:536-648,
// SURVEY.md §8(a) rows a5/a6), bit-identical to the host version
// (host_stages.cpp grow_groups) and the oracle.
//
// Both stages are greedy and sequential: every acceptance changes the group's
// averages, which the next test reads.  The parallel part is the search for the next
// acceptance: one wave per cloud tests 64 candidates at once and takes the first
// passing one by ballot (the reference's scan order), then updates the running sums
// (uniform across lanes) and continues right after it.
//   stage 1 (:536-593): seeds in voxel order; the still-unallocated voxels are a
//     compact ascending list in LDS (compacted after each seed), so the seed is its
//     head and the scan covers only candidates; compare_normal (5 deg, as an exact
//     cosine cut) then compare_plane (l1, k1) against the group's averages.
//   stage 2 (:595-648): for every unallocated group i, repeated passes over all other
//     unallocated groups j (while a pass merged any): compare_normal (8 deg) and
//     compare_plane (l2, k2) of the two groups' averages; a merge appends j's members
//     (linked lists, in order) and re-adds their weighted sums to i's running sums.
//     A group's members are the first nmem nodes from its head (a merged group's
//     tail is extended later by the group that absorbed it).
// Running sums in member order equal the reference's recompute-from-scratch (App. B
// Q7): the recompute sums the same members in the same order from zero.
// Voxel records live in LDS (SoA), so a test step costs LDS reads and ALU only.
#define KT_TU 10  // ktrace.h source tag
#include "ktrace.h"
#include "kernels.h"

namespace fccf {
namespace {

constexpr uint32_t NONE = 0xFFFFFFFFu;

struct GrowLds {
  float nx[GROW_CAP], ny[GROW_CAP], nz[GROW_CAP];
  float cx[GROW_CAP], cy[GROW_CAP], cz[GROW_CAP];
  float w[GROW_CAP];        // (float)count
  double vn[GROW_CAP];      // norm3d of the voxel normal
  uint32_t u[GROW_CAP];     // stage 1: unallocated voxels, ascending (NONE = taken this seed)
  uint32_t nxt[GROW_CAP];   // member lists: next member of the same group, NONE at the tail
};

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// A group's running state, uniform across the wave's lanes.
struct Run {
  float s, sc[3], sn[3];  // running sums (add_member)
  float ac[3], an[3], fps;
  double na;              // norm3d(an)
};
__device__ __forceinline__ void add_member(Run& g, const GrowLds& L, uint32_t v) {
  const float w = L.w[v];
  g.s = g.s + w;
  g.sc[0] = g.sc[0] + L.cx[v] * w;
  g.sc[1] = g.sc[1] + L.cy[v] * w;
  g.sc[2] = g.sc[2] + L.cz[v] * w;
  g.sn[0] = g.sn[0] + L.nx[v] * w;
  g.sn[1] = g.sn[1] + L.ny[v] * w;
  g.sn[2] = g.sn[2] + L.nz[v] * w;
}
__device__ __forceinline__ void set_avg(Run& g) {
  g.fps = g.s;
  for (int a = 0; a < 3; ++a) {
    g.ac[a] = g.sc[a] / g.s;
    g.an[a] = g.sn[a] / g.s;
  }
  g.na = norm3d(g.an[0], g.an[1], g.an[2]);
}

__global__ void __launch_bounds__(64) k_grow(GrowIn in0, GrowIn in1, GrowDev out0, GrowDev out1, GrowParams P) {
  KT();
  __shared__ GrowLds L;
  const GrowIn in = blockIdx.x ? in1 : in0;
  const GrowDev out = blockIdx.x ? out1 : out0;
  const uint32_t lane = threadIdx.x;
  const uint32_t nv = in.nv;
  for (uint32_t v = lane; v < nv; v += 64) {
    const VoxRec r = in.vox[v];
    L.nx[v] = r.n[0]; L.ny[v] = r.n[1]; L.nz[v] = r.n[2];
    L.cx[v] = r.c[0]; L.cy[v] = r.c[1]; L.cz[v] = r.c[2];
    L.w[v] = (float)r.count;
    L.vn[v] = norm3d(r.n[0], r.n[1], r.n[2]);
    L.u[v] = v;
    L.nxt[v] = NONE;
  }
  wsync();
  // ---------------- stage 1
  uint32_t nu = nv, G = 0;
  while (nu > 0) {
    const uint32_t seed = L.u[0];
    Run g;
    g.s = 0.f;
    for (int a = 0; a < 3; ++a) g.sc[a] = g.sn[a] = 0.f;
    add_member(g, L, seed);
    g.fps = L.w[seed];
    g.an[0] = L.nx[seed]; g.an[1] = L.ny[seed]; g.an[2] = L.nz[seed];
    g.ac[0] = L.cx[seed]; g.ac[1] = L.cy[seed]; g.ac[2] = L.cz[seed];
    g.na = L.vn[seed];
    uint32_t tail = seed, nmem = 1;
    if (lane == 0) L.u[0] = NONE;
    uint32_t p = 1;
    while (p < nu) {
      const uint32_t q = p + lane;
      bool ok = false;
      uint32_t j = NONE;
      if (q < nu) {
        j = L.u[q];
        const float c = normal_cos_pre(g.an[0], g.an[1], g.an[2], g.na, L.nx[j], L.ny[j], L.nz[j], L.vn[j]);
        ok = !angle_gt(c, P.cut1) &&
             compare_plane(f3{g.an[0], g.an[1], g.an[2]}, f3{g.ac[0], g.ac[1], g.ac[2]},
                           f3{L.nx[j], L.ny[j], L.nz[j]}, f3{L.cx[j], L.cy[j], L.cz[j]}, P.l1, P.k1);
      }
      const uint64_t b = __ballot(ok);
      if (!b) {
        p += 64;
        continue;
      }
      const uint32_t first = (uint32_t)__builtin_ctzll(b);
      const uint32_t acc = __shfl(j, (int)first, 64);
      if (lane == 0) {
        L.u[p + first] = NONE;
        L.nxt[tail] = acc;
      }
      tail = acc;
      ++nmem;
      add_member(g, L, acc);
      set_avg(g);
      p += first + 1;
    }
    if (lane == 0) {
      out.gac[3 * G] = g.ac[0]; out.gac[3 * G + 1] = g.ac[1]; out.gac[3 * G + 2] = g.ac[2];
      out.gan[3 * G] = g.an[0]; out.gan[3 * G + 1] = g.an[1]; out.gan[3 * G + 2] = g.an[2];
      out.gfps[G] = g.fps;
      out.gsum[7 * G] = g.s;
      for (int a = 0; a < 3; ++a) {
        out.gsum[7 * G + 1 + a] = g.sc[a];
        out.gsum[7 * G + 4 + a] = g.sn[a];
      }
      out.gna[G] = g.na;
      out.ghead[G] = seed;
      out.gtail[G] = tail;
      out.gnmem[G] = nmem;
      out.galloc[G] = 0u;
    }
    ++G;
    wsync();
    // drop this seed's members from the list (in place, in order)
    uint32_t wpos = 0;
    for (uint32_t c0 = 0; c0 < nu; c0 += 64) {
      const uint32_t q = c0 + lane;
      const uint32_t x = q < nu ? L.u[q] : NONE;
      const uint64_t keep = __ballot(x != NONE);
      wsync();
      if (x != NONE) L.u[wpos + mbcnt(keep)] = x;
      wpos += (uint32_t)__popcll(keep);
      wsync();
    }
    nu = wpos;
  }
  // ---------------- stage 2 (group records in global memory, written by lane 0 only;
  // every lane re-reads them after a wave fence)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  __syncthreads();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  for (uint32_t i = 0; i < G; ++i) {
    if (out.galloc[i]) continue;
    Run a;
    a.s = out.gsum[7 * i];
    for (int k = 0; k < 3; ++k) {
      a.sc[k] = out.gsum[7 * i + 1 + k];
      a.sn[k] = out.gsum[7 * i + 4 + k];
      a.ac[k] = out.gac[3 * i + k];
      a.an[k] = out.gan[3 * i + k];
    }
    a.fps = out.gfps[i];
    a.na = out.gna[i];
    uint32_t tail = out.gtail[i], nmem = out.gnmem[i];
    bool changed = false, newadd = true;
    while (newadd) {
      newadd = false;
      uint32_t j0 = 0;
      while (j0 < G) {
        const uint32_t j = j0 + lane;
        bool ok = false;
        if (j < G && j != i && !out.galloc[j]) {
          const float c = normal_cos_pre(a.an[0], a.an[1], a.an[2], a.na, out.gan[3 * j], out.gan[3 * j + 1],
                                         out.gan[3 * j + 2], out.gna[j]);
          ok = !angle_gt(c, P.cut2) &&
               compare_plane(f3{a.an[0], a.an[1], a.an[2]}, f3{a.ac[0], a.ac[1], a.ac[2]},
                             f3{out.gan[3 * j], out.gan[3 * j + 1], out.gan[3 * j + 2]},
                             f3{out.gac[3 * j], out.gac[3 * j + 1], out.gac[3 * j + 2]}, P.l2, P.k2);
        }
        const uint64_t b = __ballot(ok);
        if (!b) {
          j0 += 64;
          continue;
        }
        const uint32_t jj = j0 + (uint32_t)__builtin_ctzll(b);
        newadd = changed = true;
        // append jj's members in order and add them to the running sums
        const uint32_t h = out.ghead[jj], nj = out.gnmem[jj];
        uint32_t m = h;
        for (uint32_t q = 0; q < nj; ++q, m = L.nxt[m]) add_member(a, L, m);
        set_avg(a);
        if (lane == 0) {
          out.galloc[jj] = 1u;
          L.nxt[tail] = h;
        }
        tail = out.gtail[jj];
        nmem += out.gnmem[jj];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
        wsync();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        j0 = jj + 1;
      }
    }
    if (changed && lane == 0) {
      for (int k = 0; k < 3; ++k) {
        out.gac[3 * i + k] = a.ac[k];
        out.gan[3 * i + k] = a.an[k];
      }
      out.gfps[i] = a.fps;
      out.gna[i] = a.na;
      out.gtail[i] = tail;
      out.gnmem[i] = nmem;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    wsync();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
  }
  for (uint32_t v = lane; v < nv; v += 64) out.next[v] = L.nxt[v];
  if (lane == 0) *out.ng = G;
}

}  // namespace

void grow_device(const GrowIn in[2], const GrowDev out[2], const GrowParams& P, hipStream_t st) {
  k_grow<<<2, 64, 0, st>>>(in[0], in[1], out[0], out[1], P);
}

}  // namespace fccf
