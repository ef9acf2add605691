// facefit.hip — K2/K3: the voxel pass of face_extrate (FCCF.cpp:470-534) on gfx950.
//
//  * cloud centroid: pcl::compute3DCentroid, a *sequential* float sum (:473);
//  * OctreePointCloudSearch(1.0): the dynamic bounding box grows as points are
//    inserted in cloud order (App. A3).  Only its final bounds matter for the leaf
//    keys, and bounds change only at "violating" points, so one workgroup finds
//    them with block aggregates + parallel find-first, replaying adoptBoundingBox;
//  * leaves in getOccupiedVoxelCenters DFS order = stable sort by Morton code;
//  * per leaf with > 5 points: centroid, unshifted single-pass covariance
//    (PCL 1.10 computeMeanAndCovarianceMatrix), pcl::eigen33, curvature, planar
//    test and normal orientation towards the cloud centroid (:486-531);
//  * compaction: planar leaves (Morton order) and the residual cloud cloud_sub
//    (points of non-planar leaves, Morton then index order, :527-530).
// Sums run over each leaf's points in ascending index, the reference's order.
#define KT_TU 3  // ktrace.h source tag
#include <algorithm>
#include <cstdlib>

#include "probe.h"
#include "kernels.h"
#include "mail.h"
#include "ctx.h"

namespace fccf {
namespace {


// ---------------------------------------------------------------- octree bounds
// Two-level aggregates of the finite points: per 4096-point block and per 64-point
// sub-block.  One workgroup per block; four threads per sub-block, 16 consecutive
// points each (all loads issued before use), quad shuffles for the sub-record,
// then the wave / block reduction for the block record.
// Batched over blockIdx.y = sequence e.
// TF: fine verification's form (FvTransform): the points are read from tf.s2, moved by
// tf.T[e] and written to tf.s2t's sequence e as they are loaded (xyz0 unused).
template <bool TF>
__global__ void __launch_bounds__(256) k_block_aggr(const float* __restrict__ xyz0, const uint32_t* __restrict__ d_n0,
                                                    float* __restrict__ aggr0, SeqStrides sd,
                                                    uint32_t nbc, OctState* __restrict__ reset0,
                                                    uint64_t* __restrict__ stamp, FvTransform tf) {
  KT();
  if (TF && blockIdx.x == 0 && threadIdx.x == 0) {
    const uint32_t e = blockIdx.y;
    *sd.at(tf.st, sd.state, e) = *tf.s1_state;
    tf.ecnt[e] = 0u;
    tf.pts[e] = 0u;
    if (e == 0) {
      tf.scal[4] = tf.n1;
      tf.scal[5] = tf.n2;
      tf.scal[7] = 0u;
    }
  }
  if (stamp && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)  // the face stage starts
    *stamp = __builtin_amdgcn_s_memrealtime();
  if (reset0 && blockIdx.x == 0 && threadIdx.x == 0) {  // empty octree for k_oct_sim (sequence blockIdx.y)
    OctState z;
    for (int a = 0; a < 3; ++a) z.min[a] = z.max[a] = 0.0;
    z.depth = 0;
    z.defined = 0;
    *sd.at(reset0, sd.state, blockIdx.y) = z;
  }
  __shared__ float sh[4][6];
  const float* xyz = sd.at(xyz0, sd.xyz, blockIdx.y);
  float* aggr = sd.at(aggr0, sd.aggr, blockIdx.y);
  const uint32_t n = TF ? tf.n2 : *sd.at(d_n0, sd.n, blockIdx.y);
  float* sub = aggr + 6 * (size_t)nbc;
  const uint32_t t = threadIdx.x, sb = t >> 2, q = t & 3, lane = t & 63, w = t >> 6;
  const uint32_t p0 = blockIdx.x * AGGR_BLOCK + sb * AGGR_SUB + q * 16;
  const uint32_t last = n ? n - 1u : 0u;
  float v[16][3];
  if constexpr (TF) {
    const m44 M = tf.T[blockIdx.y];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const size_t i = min(p0 + k, last);
      v[k][0] = tf.s2[3 * i];
      v[k][1] = tf.s2[3 * i + 1];
      v[k][2] = tf.s2[3 * i + 2];
    }
    float* o = sd.at(tf.s2t, sd.xyz, blockIdx.y);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const f3 pt = tf_se3(M, v[k][0], v[k][1], v[k][2]);
      v[k][0] = pt.x;
      v[k][1] = pt.y;
      v[k][2] = pt.z;
      if (p0 + k < n) {
        o[3 * (size_t)(p0 + k)] = pt.x;
        o[3 * (size_t)(p0 + k) + 1] = pt.y;
        o[3 * (size_t)(p0 + k) + 2] = pt.z;
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const size_t i = min(p0 + k, last);
      v[k][0] = xyz[3 * i];
      v[k][1] = xyz[3 * i + 1];
      v[k][2] = xyz[3 * i + 2];
    }
  }
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    if (p0 + k >= n || !finite3(v[k][0], v[k][1], v[k][2])) continue;
    for (int a = 0; a < 3; ++a) {
      mn[a] = fminf(mn[a], v[k][a]);
      mx[a] = fmaxf(mx[a], v[k][a]);
    }
  }
  for (int o = 1; o < 4; o <<= 1)  // the four threads of a sub-block
    for (int a = 0; a < 3; ++a) {
      mn[a] = fminf(mn[a], __shfl_xor(mn[a], o, 64));
      mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], o, 64));
    }
  if (q == 0) {
    float* r = sub + 6 * ((size_t)blockIdx.x * (AGGR_BLOCK / AGGR_SUB) + sb);
    for (int a = 0; a < 3; ++a) { r[a] = mn[a]; r[3 + a] = mx[a]; }
  }
  for (int o = 4; o < 64; o <<= 1)
    for (int a = 0; a < 3; ++a) {
      mn[a] = fminf(mn[a], __shfl_xor(mn[a], o, 64));
      mx[a] = fmaxf(mx[a], __shfl_xor(mx[a], o, 64));
    }
  if (lane == 0)
    for (int a = 0; a < 3; ++a) { sh[w][a] = mn[a]; sh[w][3 + a] = mx[a]; }
  __syncthreads();
  if (t < 6) {
    const int a = t;
    float r = sh[0][a];
    for (int ww = 1; ww < 4; ++ww) r = a < 3 ? fminf(r, sh[ww][a]) : fmaxf(r, sh[ww][a]);
    aggr[6 * blockIdx.x + a] = r;
  }
}

struct Box6 {
  float v[6];
};

__device__ __forceinline__ Box6 load_box(const float* a, bool ok) {
  Box6 b;
  for (int k = 0; k < 6; ++k) b.v[k] = ok ? a[k] : (k < 3 ? INFINITY : -INFINITY);
  return b;
}

// a non-empty record some point of which may lie outside the current bounds
__device__ __forceinline__ bool may_violate(const OctState& S, const Box6& b) {
  if (!(b.v[0] <= b.v[3])) return false;  // no finite point
  return !S.defined || !oct_inside(S, b.v[0], b.v[1], b.v[2]) || !oct_inside(S, b.v[3], b.v[4], b.v[5]);
}

// Replays adoptBoundingBoxToPoint over xyz[0..n) in order, starting from *state.
// One wave per sequence (blockIdx.x = e): block records, then the 64 sub-records of
// a candidate block, then the 64 points of a candidate sub-block sit one per lane;
// after each adoption the lanes re-test what they hold with one ballot, so memory is
// touched only when the wave moves to a new block or sub-block, and every lane
// replays the adoption itself (the state stays uniform without broadcasts).
__global__ void __launch_bounds__(64) k_oct_sim(const float* __restrict__ xyz0, const uint32_t* __restrict__ d_n0,
                                                const float* __restrict__ aggr0, double res,
                                                OctState* __restrict__ state0, SeqStrides sd, uint32_t nbc) {
  KT();
  const uint32_t lane = threadIdx.x;
  const float* xyz = sd.at(xyz0, sd.xyz, blockIdx.x);
  const float* aggr = sd.at(aggr0, sd.aggr, blockIdx.x);
  const uint32_t n = *sd.at(d_n0, sd.n, blockIdx.x);
  const float* sub = aggr + 6 * (size_t)nbc;
  OctState* state = sd.at(state0, sd.state, blockIdx.x);
  OctState S = *state;
  const uint32_t nblk = (n + AGGR_BLOCK - 1) / AGGR_BLOCK;
  uint32_t pos = 0;  // points before pos are done
  for (uint32_t bb = 0; bb < nblk; bb += 64) {
    const uint32_t myb = bb + lane;
    const Box6 A = load_box(aggr + 6 * (size_t)myb, myb < nblk);
    while (true) {
      const bool cb = myb < nblk && (myb + 1) * AGGR_BLOCK > pos && may_violate(S, A);
      const uint64_t mb = __ballot(cb);
      if (!mb) break;
      const uint32_t fb = bb + (uint32_t)__builtin_ctzll(mb);
      const uint32_t mys = fb * (AGGR_BLOCK / AGGR_SUB) + lane;
      const Box6 B = load_box(sub + 6 * (size_t)mys, true);
      while (true) {
        const bool cs = (mys + 1) * AGGR_SUB > pos && may_violate(S, B);
        const uint64_t ms = __ballot(cs);
        if (!ms) break;
        const uint32_t s0 = (fb * (AGGR_BLOCK / AGGR_SUB) + (uint32_t)__builtin_ctzll(ms)) * AGGR_SUB;
        const uint32_t i = s0 + lane;
        float p[3] = {0.f, 0.f, 0.f};
        if (i < n) {
          p[0] = xyz[3 * (size_t)i];
          p[1] = xyz[3 * (size_t)i + 1];
          p[2] = xyz[3 * (size_t)i + 2];
        }
        while (true) {
          const bool cp = i >= pos && i < n && finite3(p[0], p[1], p[2]) && (!S.defined || !oct_inside(S, p[0], p[1], p[2]));
          const uint64_t mp = __ballot(cp);
          if (!mp) {
            pos = s0 + AGGR_SUB;
            break;
          }
          const int f = __builtin_ctzll(mp);
          float q[3];
          for (int a = 0; a < 3; ++a) q[a] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p[a]), f));
          oct_adopt(S, res, q);
          pos = s0 + (uint32_t)f + 1;
        }
      }
      pos = max(pos, (fb + 1) * AGGR_BLOCK);
    }
  }
  if (lane == 0) *state = S;
}

__global__ void __launch_bounds__(256) k_oct_codes(B4<const float*> xyz2, B4<const uint32_t*> d_n2,
                                                   B4<const OctState*> state2, double res, B4<uint64_t*> codes2,
                                                   B4<uint32_t*> d_nbits2) {
  KT();
  const int e = blockIdx.y;
  const OctState S = *state2[e];
  const uint32_t n = *d_n2[e];
  const float* __restrict__ xyz = xyz2[e];
  uint64_t* __restrict__ codes = codes2[e];
  uint32_t* __restrict__ d_nbits = d_nbits2[e];
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x, gsz = gridDim.x * 256;
  const double inv = 1.0 / res;
  if (gid == 0) *d_nbits = S.defined ? 3u * S.depth + 1u : 1u;
  // four points per thread: three 16-byte loads, two 16-byte stores (aligned arena
  // buffers; a misaligned base takes the one-point loop for everything)
  const bool al = ((((uintptr_t)xyz) | ((uintptr_t)codes)) & 15u) == 0;
  const uint32_t nq = al ? n / 4 : 0;
  for (uint32_t q = gid; q < nq; q += gsz) {
    const float4* v = reinterpret_cast<const float4*>(xyz) + 3 * (size_t)q;
    const float4 a = v[0], b = v[1], c = v[2];
    const float p[12] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, c.x, c.y, c.z, c.w};
    uint64_t k[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float x = p[3 * j], y = p[3 * j + 1], z = p[3 * j + 2];
      k[j] = finite3(x, y, z) ? oct_code(S, res, inv, x, y, z) : ~(uint64_t)0;
    }
    ulonglong2* o = reinterpret_cast<ulonglong2*>(codes + 4 * (size_t)q);
    o[0] = make_ulonglong2(k[0], k[1]);
    o[1] = make_ulonglong2(k[2], k[3]);
  }
  for (uint32_t i = 4 * nq + gid; i < n; i += gsz) {
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    codes[i] = finite3(x, y, z) ? oct_code(S, res, inv, x, y, z) : ~(uint64_t)0;
  }
}

// ---------------------------------------------------------------- plane fit
__device__ __forceinline__ void roots2(float b, float c, float r[3]) {
  r[0] = 0.f;
  float d = (float)((double)(b * b) - 4.0 * (double)c);
  if (d < 0.0) d = 0.0;
  const float sd = sqrtf(d);
  r[2] = 0.5f * (b + sd);
  r[1] = 0.5f * (b - sd);
}

// pcl::computeRoots (closed-form cubic; float transcendental := f64 evaluation rounded)
__device__ void roots3(const float m[3][3], float r[3]) {
  const float c0 = m[0][0] * m[1][1] * m[2][2] + 2.f * m[0][1] * m[0][2] * m[1][2] - m[0][0] * m[1][2] * m[1][2] -
                   m[1][1] * m[0][2] * m[0][2] - m[2][2] * m[0][1] * m[0][1];
  const float c1 = m[0][0] * m[1][1] - m[0][1] * m[0][1] + m[0][0] * m[2][2] - m[0][2] * m[0][2] +
                   m[1][1] * m[2][2] - m[1][2] * m[1][2];
  const float c2 = m[0][0] + m[1][1] + m[2][2];
  if (fabsf(c0) < 1.1920928955078125e-07f) {
    roots2(c2, c1, r);
    return;
  }
  const float inv3 = (float)(1.0 / 3.0);
  const float sqrt3 = sqrtf(3.0f);
  const float c2o3 = c2 * inv3;
  float a3 = (c1 - c2 * c2o3) * inv3;
  if (a3 > 0.f) a3 = 0.f;
  const float hb = 0.5f * (c0 + c2o3 * (2.f * c2o3 * c2o3 - c1));
  float q = hb * hb + a3 * a3 * a3;
  if (q > 0.f) q = 0.f;
  const float rho = sqrtf(-a3);
  const float th = (float)atan2((double)sqrtf(-q), (double)hb) * inv3;
  const float ct = (float)cos((double)th), sn = (float)sin((double)th);
  r[0] = c2o3 + 2.f * rho * ct;
  r[1] = c2o3 - rho * (ct + sqrt3 * sn);
  r[2] = c2o3 - rho * (ct - sqrt3 * sn);
  float t;
  if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
  if (r[1] >= r[2]) {
    t = r[1]; r[1] = r[2]; r[2] = t;
    if (r[0] >= r[1]) { t = r[0]; r[0] = r[1]; r[1] = t; }
  }
  if (r[0] <= 0.f) roots2(c2, c1, r);
}

// pcl::eigen33(mat, eigenvalue, eigenvector): smallest eigenpair.
__device__ void eig_min(const float A[3][3], float& ev, f3& v) {
  float scale = 0.f;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) scale = fmaxf(scale, fabsf(A[i][j]));
  if (scale <= 1.17549435e-38f) scale = 1.0f;
  float s[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) s[i][j] = A[i][j] / scale;
  float r[3];
  roots3(s, r);
  ev = r[0] * scale;
  for (int i = 0; i < 3; ++i) s[i][i] -= r[0];
  const f3 a = {s[0][0], s[0][1], s[0][2]}, b = {s[1][0], s[1][1], s[1][2]}, c = {s[2][0], s[2][1], s[2][2]};
  const f3 v1 = cross3(a, b), v2 = cross3(a, c), v3 = cross3(b, c);
  const float l1 = sqn3(v1), l2 = sqn3(v2), l3 = sqn3(v3);
  f3 w;
  float d;
  if (l1 >= l2 && l1 >= l3) { w = v1; d = sqrtf(l1); }
  else if (l2 >= l1 && l2 >= l3) { w = v2; d = sqrtf(l2); }
  else { w = v3; d = sqrtf(l3); }
  v = {w.x / d, w.y / d, w.z / d};
}

// Points in leaf order (Morton, then index): the per-leaf loops below then read
// contiguous memory instead of gathering through the sort permutation.
__global__ void __launch_bounds__(256) k_gather(B4<const float*> xyz2, B4<const uint32_t*> vals2,
                                                B4<const uint32_t*> d_n2, B4<float*> sp2) {
  KT();
  const int e = blockIdx.y;
  const uint32_t n = *d_n2[e];
  const float* __restrict__ xyz = xyz2[e];
  const uint32_t* __restrict__ vals = vals2[e];
  float* __restrict__ sp = sp2[e];
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
    const uint32_t j = vals[k];
    sp[3 * k] = xyz[3 * j]; sp[3 * k + 1] = xyz[3 * j + 1]; sp[3 * k + 2] = xyz[3 * j + 2];
  }
}

constexpr uint32_t VFIT_BLOCKS = 512;  // 2048 waves per cloud; leaves are a few thousand at most

// One wave per leaf (Morton order).  Lane k < 9 owns accumulator k of
// computeMeanAndCovarianceMatrix (:495): [xx, xy, xz, yy, yz, zz, x, y, z], each a
// sequential float sum over the leaf's points in index order.  Points are staged in
// LDS as (x, y, z, 1) so every lane computes term = p[i1] * p[i2] (the linear sums
// use i2 = w = 1, and x * 1 == x exactly).  compute3DCentroid (:490) is the same
// sequential x/y/z sum divided by n, i.e. accumulators 6..8 / n bit-for-bit.
#ifndef VFIT_WPE
#define VFIT_WPE 1
#endif
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VFIT_WPE))) k_voxel_fit(B4<FaceBufs> fb, float vpt, float cthr) {
  KT();
  constexpr uint32_t VB = 256;  // points per LDS burst of a wave (four per lane)
  __shared__ __attribute__((aligned(16))) float pts[4][VB * 4];
  const FaceBufs& B = fb.v[blockIdx.y];
  const float* __restrict__ sp = B.sp;
  const uint32_t* __restrict__ starts = B.starts;
  VoxRec* __restrict__ recs = B.recs;
  uint32_t* __restrict__ planar = B.flag_planar;
  uint32_t* __restrict__ resid = B.resid_cnt;
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t nl = *B.nleaf;
  const int i1t[16] = {0, 0, 0, 1, 1, 2, 0, 1, 2, 0, 0, 0, 0, 0, 0, 0};
  const int i2t[16] = {0, 1, 2, 1, 2, 2, 3, 3, 3, 3, 3, 3, 3, 3, 3, 3};
  const int i1 = i1t[lane & 15], i2 = i2t[lane & 15];
  float* P = pts[wave];
  for (uint32_t s = blockIdx.x * 4 + wave; s < nl; s += gridDim.x * 4) {
    const uint32_t b = starts[s], e = starts[s + 1];
    const uint32_t cnt = e - b;
    float acc = 0.f;
    const bool fit = (float)cnt > vpt;
    if (fit) {
      // The leaf streams through LDS in bursts of VB points; the next burst's four
      // points per lane are loaded into registers while this one is summed, so the
      // global-load latency (~1.5 us) hides behind a burst's ~VB dependent adds.
      float nx[4], ny[4], nz[4];
      auto load_burst = [&](uint32_t base) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const uint32_t k = base + u * 64 + lane;
          if (k < cnt) {
            const float* q = sp + 3 * (size_t)(b + k);
            nx[u] = q[0]; ny[u] = q[1]; nz[u] = q[2];
          }
        }
      };
      load_burst(0);
      for (uint32_t base = 0; base < cnt; base += VB) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
          if (base + u * 64 + lane < cnt) *(float4*)(P + 4 * (u * 64 + lane)) = make_float4(nx[u], ny[u], nz[u], 1.0f);
        if (base + VB < cnt) load_burst(base + VB);
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // sequential per accumulator (the reference's summation order); the LDS reads
        // of the next eight points are issued before this eight's adds
        const uint32_t m = __builtin_amdgcn_readfirstlane(min(VB, cnt - base));
        const uint32_t m8 = m & ~7u;
        float a[8], c[8];
        if (m8) {
#pragma unroll
          for (int q = 0; q < 8; ++q) { a[q] = P[4 * q + i1]; c[q] = P[4 * q + i2]; }
        }
        for (uint32_t j = 0; j < m8; j += 8) {
          float an[8], cn[8];
          const bool more = j + 8 < m8;
          if (more) {
#pragma unroll
            for (int q = 0; q < 8; ++q) { an[q] = P[4 * (j + 8 + q) + i1]; cn[q] = P[4 * (j + 8 + q) + i2]; }
          }
#pragma unroll
          for (int q = 0; q < 8; ++q) acc += a[q] * c[q];
          if (more) {
#pragma unroll
            for (int q = 0; q < 8; ++q) { a[q] = an[q]; c[q] = cn[q]; }
          }
        }
        for (uint32_t j = m8; j < m; ++j) acc += P[4 * j + i1] * P[4 * j + i2];
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
    }
    float ac[9];
#pragma unroll
    for (int q = 0; q < 9; ++q) ac[q] = __shfl(acc, q, 64);
    if (lane != 0) continue;
    VoxRec r;
    r.count = (int32_t)cnt;
    r.curvature = 0.f;
    r.c[0] = r.c[1] = r.c[2] = 0.f;
    r.n[0] = r.n[1] = r.n[2] = 0.f;
    uint32_t flag = 0;
    if (fit) {
      const float fc = (float)cnt;
      const float cx = ac[6] / fc, cy = ac[7] / fc, cz = ac[8] / fc;
      for (int i = 0; i < 9; ++i) ac[i] /= fc;
      float cov[3][3];
      cov[0][0] = ac[0] - ac[6] * ac[6];
      cov[0][1] = ac[1] - ac[6] * ac[7];
      cov[0][2] = ac[2] - ac[6] * ac[8];
      cov[1][1] = ac[3] - ac[7] * ac[7];
      cov[1][2] = ac[4] - ac[7] * ac[8];
      cov[2][2] = ac[5] - ac[8] * ac[8];
      cov[1][0] = cov[0][1]; cov[2][0] = cov[0][2]; cov[2][1] = cov[1][2];
      float ev;
      f3 nv;
      eig_min(cov, ev, nv);
      const float es = cov[0][0] + cov[1][1] + cov[2][2];
      const float curv = (es != 0.f) ? fabsf(ev / es) : 0.f;
      r.curvature = curv;
      r.c[0] = cx; r.c[1] = cy; r.c[2] = cz;
      r.n[0] = nv.x; r.n[1] = nv.y; r.n[2] = nv.z;  // oriented later (needs the cloud centroid)
      flag = curv < cthr ? 1u : 2u;
    }
    recs[s] = r;
    planar[s] = flag == 1 ? 1u : 0u;
    resid[s] = flag == 2 ? cnt : 0u;
  }
}

// cloud_sub (:527-530): every point of a non-planar leaf, leaf order then index order.
__global__ void __launch_bounds__(256) k_compact_resid(B4<FaceBufs> fb, B4<const uint32_t*> d_n2, B4<float*> rout2) {
  KT();
  const int e = blockIdx.y;
  const FaceBufs& B = fb.v[e];
  const float* __restrict__ sp = B.sp;
  const uint32_t* __restrict__ seg_of = B.seg_of;
  const uint32_t* __restrict__ starts = B.starts;
  const uint32_t* __restrict__ resid = B.resid_cnt;
  const uint32_t* __restrict__ roff = B.resid_off;
  float* __restrict__ rout = rout2[e];
  const uint32_t n = *d_n2[e];
  for (uint32_t k = blockIdx.x * 256 + threadIdx.x; k < n; k += gridDim.x * 256) {
    const uint32_t s = seg_of[k];
    if (!resid[s]) continue;
    const uint32_t o = roff[s] + (k - starts[s]);
    rout[3 * o] = sp[3 * k]; rout[3 * o + 1] = sp[3 * k + 1]; rout[3 * o + 2] = sp[3 * k + 2];
  }
}

// Planar leaves with the normal oriented towards the cloud centroid (:504-516).
// With a mailbox, the records (up to its capacity) and both clouds' counts are
// also written to pinned host memory: phase B reads them after one event sync.
__global__ void __launch_bounds__(256) k_compact_planar(B4<FaceBufs> fb, B4<VoxRec*> pout2, CloudMail* __restrict__ mail,
                                                        B4<const uint32_t*> sc2) {
  KT();
  const int e = blockIdx.y;
  const FaceBufs& B = fb.v[e];
  const VoxRec* __restrict__ recs = B.recs;
  const uint32_t* __restrict__ planar = B.flag_planar;
  const uint32_t* __restrict__ poff = B.planar_off;
  const float* __restrict__ cc = B.centroid;
  VoxRec* __restrict__ pout = pout2[e];
  const uint32_t nl = *B.nleaf;
  // clouds 2j and 2j + 1 are pair j of the batch: their mailbox is mail[j]
  CloudMail* __restrict__ pm = mail ? mail + (e >> 1) : nullptr;
  const int ce = e & 1;
  if (pm && blockIdx.x == 0 && threadIdx.x < 8) {
    const uint32_t i = threadIdx.x & 3u;
    if (threadIdx.x < 4) pm->sc[ce][i] = sc2[e][i];
    else if (i == 1)  // both passes' sort flags, redo, deep face codes
      pm->fsc[ce][1] = (B.vgp ? B.vgp->sort_err | (B.vgp->redo ? VG_REDO : 0u) : 0u) | (*B.nbits > 27u ? FACE_DEEP : 0u);
    else pm->fsc[ce][i] = B.nleaf[i];
  }
  // the cloud stage's device spans: the stamps of main's pass, the driver's pass and the
  // face stage, and now (this last kernel of the stage, ~5 us, starts) into the mailbox.
  // (A finished-block count to stamp the true end cost 8192 same-address atomics:
  // ~70 us.)
  if (pm && ce == 0 && blockIdx.x == 0 && threadIdx.x == 0 && B.vgp) {
    pm->stamp[3] = __builtin_amdgcn_s_memrealtime();
    pm->stamp[0] = B.vgp->t_main;
    pm->stamp[1] = B.vgp->t_driver;
    pm->stamp[2] = *fb.v[0].t_faces;  // (the batch's face stage starts once, stamped in cloud 0's buffers)
  }
  for (uint32_t s = blockIdx.x * 256 + threadIdx.x; s < nl; s += gridDim.x * 256) {
    if (!planar[s]) continue;
    VoxRec r = recs[s];
    const f3 to = {r.c[0] - cc[0], r.c[1] - cc[1], r.c[2] - cc[2]};
    const f3 nv = {r.n[0], r.n[1], r.n[2]};
    if (!(dot3(to, nv) < 0.f)) { r.n[0] = -nv.x; r.n[1] = -nv.y; r.n[2] = -nv.z; }
    const uint32_t o = poff[s];
    pout[o] = r;
    if (pm && o < CloudMail::REC_CAP) pm->rec[ce][o] = r;
  }
}

// The stage's mailboxes are complete: every record and count was written by the
// kernels before this one on the stream; the flag follows them to host memory after a
// system-scope fence, and phase B1 polls it instead of sleeping in an event wait.
__global__ void k_mail_done(CloudMail* __restrict__ mail, int npairs) {
  KT();
  __threadfence_system();
  if ((int)threadIdx.x < npairs) __hip_atomic_store(&mail[threadIdx.x].done, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}


inline uint32_t grid_for(uint32_t cap, uint32_t per = 256, uint32_t mx = 4096) {
  uint32_t g = (cap + per - 1) / per;
  return g < 1 ? 1 : (g > mx ? mx : g);
}

}  // namespace


void block_aggr(const float* xyz, const uint32_t* d_n, uint32_t cap, float* aggr, hipStream_t st, int batch,
                SeqStrides sd, OctState* reset_state, uint64_t* stamp) {
  const uint32_t nb = (cap + AGGR_BLOCK - 1) / AGGR_BLOCK;
  k_block_aggr<false><<<dim3(nb ? nb : 1, batch), 256, 0, st>>>(xyz, d_n, aggr, sd, aggr_blocks(cap), reset_state, stamp,
                                                                FvTransform{});
}

void block_aggr_transform(const FvTransform& tf, const uint32_t* d_n, uint32_t cap, float* aggr, hipStream_t st,
                          int batch, SeqStrides sd, uint64_t* stamp) {
  const uint32_t nb = (cap + AGGR_BLOCK - 1) / AGGR_BLOCK;
  k_block_aggr<true><<<dim3(nb ? nb : 1, batch), 256, 0, st>>>(tf.s2, d_n, aggr, sd, aggr_blocks(cap), nullptr, stamp,
                                                               tf);
}

void octree_sim(const float* xyz, const uint32_t* d_n, uint32_t cap, double res, const float* aggr, OctState* state,
                hipStream_t st, int batch, SeqStrides sd) {
  FCCF_LAUNCH("k_oct_sim", (d_n, 24.0 * batch / AGGR_BLOCK), k_oct_sim, batch, 64, 0, st, xyz, d_n, aggr, res, state, sd, aggr_blocks(cap));
}

namespace {
// the batched octree launches address sequence e at a fixed byte stride from sequence 0:
// every cloud of a batch is carved alike (pipeline.cpp carve_cloud)
template <class T>
size_t byte_stride(const B4<T*>& p, int nbatch) {
  if (nbatch < 2) return 0;
  const ptrdiff_t d = (const char*)p[1] - (const char*)p[0];
  for (int e = 2; e < nbatch; ++e)
    if ((const char*)p[e] - (const char*)p[0] != e * d) throw Error(FCCF_E_INTERNAL, "face stage: clouds not carved alike");
  return (size_t)d;
}
template <class F>
auto pick(const B4<FaceBufs>& b, F get) -> B4<decltype(get(b[0]))> {
  B4<decltype(get(b[0]))> r;
  for (int e = 0; e < BMAX; ++e) r.v[e] = get(b[e]);
  return r;
}
}  // namespace

namespace {
// ---------------------------------------------------------------- row P (sharded face stage)
// Rank r of N fits only the 1 m leaves of its range of codes: the points are binned by
// the top FACE_BINS_LG bits of their leaf code (a leaf's points share their code, so a bin
// boundary never splits a leaf), the bins are split into N ranges of about equal point
// counts, and the rank's points are compacted in input order (so its sort keeps PCL's
// insertion order within a leaf).  group.cpp face_voxels_sharded runs the exchange.
constexpr int FACE_BINS_LG = 12;
constexpr uint32_t FACE_BINS = 1u << FACE_BINS_LG;
constexpr uint32_t FACE_HIST_BLOCKS = 256;

__device__ __forceinline__ uint32_t face_shift(uint32_t nbits) {
  return nbits > (uint32_t)FACE_BINS_LG ? nbits - (uint32_t)FACE_BINS_LG : 0u;
}

// hist (FACE_BINS u32, zeroed by the caller): points per bin
__global__ void __launch_bounds__(256) k_face_hist(B4<const uint64_t*> codes2, B4<const uint32_t*> d_n2,
                                                   B4<const uint32_t*> nbits2, B4<uint32_t*> hist2) {
  KT();
  __shared__ uint32_t h[FACE_BINS];
  const int e = blockIdx.y;
  for (uint32_t i = threadIdx.x; i < FACE_BINS; i += 256) h[i] = 0u;
  __syncthreads();
  const uint64_t* __restrict__ codes = codes2[e];
  const uint32_t n = *d_n2[e], sh = face_shift(*nbits2[e]);
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
    atomicAdd(&h[(uint32_t)(codes[i] >> sh) & (FACE_BINS - 1u)], 1u);
  __syncthreads();
  uint32_t* __restrict__ hist = hist2[e];
  for (uint32_t i = threadIdx.x; i < FACE_BINS; i += 256)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// One block per cloud: bound j = the first bin b with (points before b) * N >= j * n;
// rank r takes bins [bound_r, bound_{r+1}).  rng = {lo, hi, shift}.
__global__ void __launch_bounds__(1024) k_face_range(B4<const uint32_t*> hist2, B4<const uint32_t*> d_n2,
                                                     B4<const uint32_t*> nbits2, B4<uint32_t*> rng2, int rank,
                                                     int nranks) {
  KT();
  __shared__ uint32_t sb[IS_SHARD_MAX + 1];
  __shared__ uint32_t sh[16];
  const int e = blockIdx.y;
  const uint32_t* __restrict__ hist = hist2[e];
  const uint64_t n = *d_n2[e];
  constexpr int PER = FACE_BINS / 1024;
  for (int j = threadIdx.x; j <= nranks; j += 1024) sb[j] = j == 0 ? 0u : FACE_BINS;
  uint32_t h[PER], tot = 0;
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    h[k] = hist[threadIdx.x * PER + k];
    tot += h[k];
  }
  // exclusive scan of the per-thread totals (points before this thread's first bin)
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t x = tot;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = __shfl_up(x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) sh[wave] = x;
  __syncthreads();
  uint32_t before = x - tot;
  for (uint32_t w = 0; w < wave; ++w) before += sh[w];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint32_t b = threadIdx.x * PER + k;
    for (int j = 1; j < nranks; ++j)
      if ((uint64_t)before * (uint64_t)nranks >= (uint64_t)j * n) atomicMin(&sb[j], b);
    before += h[k];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t* rng = rng2[e];
    rng[0] = sb[rank];
    rng[1] = sb[rank + 1];
    rng[2] = face_shift(*nbits2[e]);
  }
}

__global__ void __launch_bounds__(256) k_face_flag(B4<const uint64_t*> codes2, B4<const uint32_t*> d_n2,
                                                   B4<const uint32_t*> rng2, B4<uint32_t*> flag2) {
  KT();
  const int e = blockIdx.y;
  const uint64_t* __restrict__ codes = codes2[e];
  const uint32_t* rng = rng2[e];
  const uint32_t n = *d_n2[e], lo = rng[0], hi = rng[1], sh = rng[2];
  uint32_t* __restrict__ flag = flag2[e];
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const uint32_t b = (uint32_t)(codes[i] >> sh) & (FACE_BINS - 1u);
    flag[i] = (b >= lo && b < hi) ? 1u : 0u;
  }
}

// this rank's points, in input order: codes to cout, input positions to iout
__global__ void __launch_bounds__(256) k_face_pick(B4<const uint64_t*> codes2, B4<const uint32_t*> d_n2,
                                                   B4<const uint32_t*> flag2, B4<const uint32_t*> off2,
                                                   B4<uint64_t*> cout2, B4<uint32_t*> iout2) {
  KT();
  const int e = blockIdx.y;
  const uint64_t* __restrict__ codes = codes2[e];
  const uint32_t* __restrict__ flag = flag2[e];
  const uint32_t* __restrict__ off = off2[e];
  uint64_t* __restrict__ cout = cout2[e];
  uint32_t* __restrict__ iout = iout2[e];
  const uint32_t n = *d_n2[e];
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
    if (flag[i]) {
      cout[off[i]] = codes[i];
      iout[off[i]] = i;
    }
}

}  // namespace

// block_aggr + octree_sim + codes of every point (replicated in the sharded form)
void face_codes(B4<const float*> xyz, B4<const uint32_t*> d_n, uint32_t cap, double res, B4<FaceBufs> b, hipStream_t st,
                int nbatch) {
  const B4<OctState*> oct = pick(b, [](const FaceBufs& f) { return f.oct; });
  const B4<float*> aggr = pick(b, [](const FaceBufs& f) { return f.aggr; });
  SeqStrides sd;
  sd.xyz = byte_stride(xyz, nbatch);
  sd.aggr = byte_stride(aggr, nbatch);
  sd.state = byte_stride(oct, nbatch);
  sd.n = byte_stride(d_n, nbatch);
  block_aggr(xyz[0], d_n[0], cap, aggr[0], st, nbatch, sd, oct[0], b[0].t_faces);  // also resets the octree states
  octree_sim(xyz[0], d_n[0], cap, res, aggr[0], oct[0], st, nbatch, sd);
  k_oct_codes<<<dim3(grid_stream(cap, nbatch, 1024), nbatch), 256, 0, st>>>(xyz, d_n, B4<const OctState*>(oct), res,
                                                          pick(b, [](const FaceBufs& f) { return f.c0; }),
                                                          pick(b, [](const FaceBufs& f) { return f.nbits; }));
}

void face_shard_select(B4<const uint32_t*> d_n, uint32_t cap, B4<FaceBufs> b, int rank, int nranks, hipStream_t st,
                       int nbatch) {
  if (cap < 2 * FACE_BINS) throw Error(FCCF_E_INTERNAL, "sharded face stage: cloud capacity below the bin table");
  if (nranks < 1 || nranks > IS_SHARD_MAX) throw Error(FCCF_E_INTERNAL, "sharded face stage: rank count");
  // scratch: the histogram in c2 (free until the sort), the flags in v0, their offsets in v2
  const B4<uint32_t*> hist = pick(b, [](const FaceBufs& f) { return (uint32_t*)f.c2; });
  for (int e = 0; e < nbatch; ++e) HIP_CHECK(hipMemsetAsync(hist[e], 0, 4 * FACE_BINS, st));
  const B4<const uint64_t*> c0 = pick(b, [](const FaceBufs& f) { return (const uint64_t*)f.c0; });
  const B4<const uint32_t*> nbits = pick(b, [](const FaceBufs& f) { return (const uint32_t*)f.nbits; });
  const B4<uint32_t*> rng = pick(b, [](const FaceBufs& f) { return f.nleaf + 8; });  // FaceBufs scalars [8..10]
  const B4<uint32_t*> nr = pick(b, [](const FaceBufs& f) { return f.nleaf + 11; });  // [11]: this rank's points
  k_face_hist<<<dim3(FACE_HIST_BLOCKS, nbatch), 256, 0, st>>>(c0, d_n, nbits, hist);
  k_face_range<<<dim3(1, nbatch), 1024, 0, st>>>(B4<const uint32_t*>(hist), d_n, nbits, rng, rank, nranks);
  const B4<uint32_t*> flag = pick(b, [](const FaceBufs& f) { return f.v0; });
  const B4<uint32_t*> off = pick(b, [](const FaceBufs& f) { return f.v2; });
  k_face_flag<<<dim3(grid_for(cap), nbatch), 256, 0, st>>>(c0, d_n, B4<const uint32_t*>(rng), flag);
  exclusive_scan_u32(B4<const uint32_t*>(flag), off, d_n, cap, nr, pick(b, [](const FaceBufs& f) { return f.ss; }), st,
                     nbatch);
  k_face_pick<<<dim3(grid_for(cap), nbatch), 256, 0, st>>>(c0, d_n, B4<const uint32_t*>(flag), B4<const uint32_t*>(off),
                                                          pick(b, [](const FaceBufs& f) { return f.c1; }),
                                                          pick(b, [](const FaceBufs& f) { return f.v1; }));
}

// The rank's points (codes c1, positions v1, count FaceBufs scalar [11]) sorted into leaf
// order, their leaves (local: starts, nleaf, seg_of) and the points in that order (sp).
void face_shard_sort(B4<const float*> xyz, uint32_t cap, B4<FaceBufs> b, hipStream_t st, int nbatch) {
  const B4<const uint32_t*> nr = pick(b, [](const FaceBufs& f) { return (const uint32_t*)(f.nleaf + 11); });
  const B4<uint64_t*> c1 = pick(b, [](const FaceBufs& f) { return f.c1; });
  const B4<uint32_t*> v1 = pick(b, [](const FaceBufs& f) { return f.v1; });
  radix_sort_u64(c1, v1, pick(b, [](const FaceBufs& f) { return f.c0; }), pick(b, [](const FaceBufs& f) { return f.v0; }),
                 nr, cap, pick(b, [](const FaceBufs& f) { return (const uint32_t*)f.nbits; }), 32, false,
                 pick(b, [](const FaceBufs& f) { return f.ss; }), st, nbatch, B4<const uint32_t*>(nullptr),
                 pick(b, [](const FaceBufs& f) { return f.c2; }), pick(b, [](const FaceBufs& f) { return f.v2; }));
  segment_heads_u64(B4<const uint64_t*>(c1), nr, cap, pick(b, [](const FaceBufs& f) { return f.starts; }),
                    pick(b, [](const FaceBufs& f) { return f.nleaf; }), pick(b, [](const FaceBufs& f) { return f.ss; }),
                    st, pick(b, [](const FaceBufs& f) { return f.seg_of; }), nbatch);
  k_gather<<<dim3(grid_stream(cap, nbatch), nbatch), 256, 0, st>>>(xyz, B4<const uint32_t*>(v1), nr,
                                                       pick(b, [](const FaceBufs& f) { return f.sp; }));
}

// The rank's leaves fitted into views of the full arrays (bv: recs, flag_planar,
// resid_cnt, resid_off shifted to the rank's first leaf); its residual offsets (local
// total in scalar [3]).
void face_shard_fit(uint32_t cap, float vpt, float cthr, B4<FaceBufs> bv, hipStream_t st, int nbatch) {
  k_voxel_fit<<<dim3(grid_for(cap, 4, VFIT_BLOCKS), nbatch), 256, 0, st>>>(bv, vpt, cthr);
  exclusive_scan_u32(pick(bv, [](const FaceBufs& f) { return (const uint32_t*)f.resid_cnt; }),
                     pick(bv, [](const FaceBufs& f) { return f.resid_off; }),
                     pick(bv, [](const FaceBufs& f) { return (const uint32_t*)f.nleaf; }), cap,
                     pick(bv, [](const FaceBufs& f) { return f.nresid; }), pick(bv, [](const FaceBufs& f) { return f.ss; }),
                     st, nbatch);
}

// The rank's residual points into rout (already shifted to the rank's first residual point)
void face_shard_resid(uint32_t cap, B4<FaceBufs> bv, B4<float*> rout, hipStream_t st, int nbatch) {
  k_compact_resid<<<dim3(grid_stream(cap, nbatch), nbatch), 256, 0, st>>>(
      bv, pick(bv, [](const FaceBufs& f) { return (const uint32_t*)(f.nleaf + 11); }), rout);
}

// After the exchange: the planar offsets over every leaf (scalar [0] = all leaves)
void face_planar_scan(uint32_t cap, B4<FaceBufs> b, hipStream_t st, int nbatch) {
  exclusive_scan_u32(pick(b, [](const FaceBufs& f) { return (const uint32_t*)f.flag_planar; }),
                     pick(b, [](const FaceBufs& f) { return f.planar_off; }),
                     pick(b, [](const FaceBufs& f) { return (const uint32_t*)f.nleaf; }), cap,
                     pick(b, [](const FaceBufs& f) { return f.nplanar; }), pick(b, [](const FaceBufs& f) { return f.ss; }),
                     st, nbatch);
}

void face_voxels_prepare(B4<const float*> xyz, B4<const uint32_t*> d_n, uint32_t cap, double res, B4<FaceBufs> b,
                         hipStream_t st, int nbatch, int fast_bits) {
  face_codes(xyz, d_n, cap, res, b, st, nbatch);
  const B4<uint32_t*> nbits = pick(b, [](const FaceBufs& f) { return f.nbits; });
  const B4<uint64_t*> c0 = pick(b, [](const FaceBufs& f) { return f.c0; }), c1 = pick(b, [](const FaceBufs& f) { return f.c1; });
  const B4<uint32_t*> v0 = pick(b, [](const FaceBufs& f) { return f.v0; }), v1 = pick(b, [](const FaceBufs& f) { return f.v1; });
  // codes are 3 bits per octree level (+1): the device plan takes 3 passes of <= 9-bit
  // digits up to depth 8 (extents up to ~256 x face_voxel_size; c3-c5: depth 6, 19
  // bits) and 4 passes of 8 bits at depth 9-10 (~1 km at 1 m voxels, outdoor scans).
  // The pipeline launches three (fast_bits 24) until a scene needs the fourth
  // (FACE_DEEP, then 32 for the ctx): a fourth pass that exits at once still costs three
  // dependent launches (~15 us per cloud stage).  Digits past the launched passes are
  // sorted by the single-workgroup tail, exactly.  With the third buffer a three-pass
  // sort ends in (c0, v0) by rotation and a two- or four-pass one by ping-pong.
  radix_sort_u64(c0, v0, c1, v1, d_n, cap, B4<const uint32_t*>(nbits), fast_bits, true,
                 pick(b, [](const FaceBufs& f) { return f.ss; }), st, nbatch, B4<const uint32_t*>(nullptr),
                 pick(b, [](const FaceBufs& f) { return f.c2; }), pick(b, [](const FaceBufs& f) { return f.v2; }));
  segment_heads_u64(B4<const uint64_t*>(c0), d_n, cap, pick(b, [](const FaceBufs& f) { return f.starts; }),
                    pick(b, [](const FaceBufs& f) { return f.nleaf; }), pick(b, [](const FaceBufs& f) { return f.ss; }),
                    st, pick(b, [](const FaceBufs& f) { return f.seg_of; }), nbatch);
  ProbeBytes pb;
  for (int e = 0; e < nbatch; ++e) pb.add(d_n[e], 28.0);
  FCCF_LAUNCH("k_gather", (pb), k_gather, dim3(grid_stream(cap, nbatch), nbatch), 256, 0, st, xyz, B4<const uint32_t*>(v0), d_n, pick(b, [](const FaceBufs& f) { return f.sp; }));
}

void face_voxels_fit(B4<const uint32_t*> d_n, uint32_t cap, float vpt, float cthr, B4<float*> resid_out,
                     B4<FaceBufs> b, hipStream_t st, int nbatch) {
  ProbeBytes pb;
  for (int e = 0; e < nbatch; ++e) pb.add(d_n[e], 12.0).add(b[e].nleaf, (double)sizeof(VoxRec) + 12.0);
  FCCF_LAUNCH("k_voxel_fit", (pb), k_voxel_fit, dim3(grid_for(cap, 4, VFIT_BLOCKS), nbatch), 256, 0, st, b, vpt, cthr);
  const B4<SortScratch> ss = pick(b, [](const FaceBufs& f) { return f.ss; });
  const B4<const uint32_t*> nleaf = pick(b, [](const FaceBufs& f) { return (const uint32_t*)f.nleaf; });
  exclusive_scan2_u32(pick(b, [](const FaceBufs& f) { return (const uint32_t*)f.flag_planar; }),
                      pick(b, [](const FaceBufs& f) { return f.planar_off; }),
                      pick(b, [](const FaceBufs& f) { return f.nplanar; }),
                      pick(b, [](const FaceBufs& f) { return (const uint32_t*)f.resid_cnt; }),
                      pick(b, [](const FaceBufs& f) { return f.resid_off; }),
                      pick(b, [](const FaceBufs& f) { return f.nresid; }), nleaf, cap, ss, st, nbatch);
  k_compact_resid<<<dim3(grid_stream(cap, nbatch), nbatch), 256, 0, st>>>(b, d_n, resid_out);
}

uint32_t grid_stream(uint32_t cap, int nbatch, uint32_t per) {
  constexpr uint32_t total = 2048;  // (1024 / 4096 measured no better)
  uint32_t g = (cap + per - 1) / per;
  const uint32_t mx = std::max(64u, total / (uint32_t)std::max(1, nbatch));
  return g < 1 ? 1 : (g > mx ? mx : g);
}

void octree_replay(const float* xyz, const uint32_t* d_n, uint32_t cap, double res, float* aggr, OctState* state,
                   hipStream_t st) {
  block_aggr(xyz, d_n, cap, aggr, st, 1, SeqStrides(), state);  // also resets the octree state
  octree_sim(xyz, d_n, cap, res, aggr, state, st);
}

void face_voxels_orient(uint32_t cap, B4<VoxRec*> planar_out, B4<FaceBufs> b, hipStream_t st, int nbatch,
                        CloudMail* mail, B4<const uint32_t*> sc) {
  k_compact_planar<<<dim3(grid_stream(cap, nbatch), nbatch), 256, 0, st>>>(b, planar_out, mail, sc);
  if (mail) k_mail_done<<<1, 64, 0, st>>>(mail, (nbatch + 1) / 2);
}

}  // namespace fccf
