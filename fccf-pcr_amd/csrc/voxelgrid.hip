// voxelgrid.hip — K1: pcl::VoxelGrid<PointXYZ>::applyFilter on gfx950.
//
// Reference call sites: FCCF.cpp:1668-1678 (main, one pass per cloud) and
// :1377-1387 (driver, a second pass).  Semantics:
//   bbox over finite points -> int32 overflow guard (output = input) ->
//   idx = ijk0 + ijk1*div0 + ijk2*div0*div1 with ijk = int(floor(p*inv) - float(min_b))
//   -> sort (idx, index) -> one centroid per run, Vector3f sum / n, ascending idx.
// PCL sorts with unstable std::sort; this kernel sums each leaf in ascending input
// index order (a conforming std::sort outcome), exactly as the oracle's stable mode.
//
// HBM traffic per pass (algorithmic): read 12 B/pt, write 12 B/leaf; the radix sort
// adds 2 x (4+4) B/pt per 8-bit digit pass.
#include "probe.h"
#include "kernels.h"

namespace fccf {
namespace {

__device__ __forceinline__ float wave_min(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Per-block partial bbox of finite points: part[b] = {min xyz, max xyz, count(bits), 0}.
__global__ void __launch_bounds__(256) k_vg_bbox(const float* __restrict__ xyz, const uint32_t* __restrict__ d_n,
                                                 float* __restrict__ part) {
  __shared__ float sh[4][7];
  const uint32_t n = *d_n;
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  uint32_t cnt = 0;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    if (!finite3(x, y, z)) continue;
    mn[0] = fminf(mn[0], x); mn[1] = fminf(mn[1], y); mn[2] = fminf(mn[2], z);
    mx[0] = fmaxf(mx[0], x); mx[1] = fmaxf(mx[1], y); mx[2] = fmaxf(mx[2], z);
    ++cnt;
  }
  for (int a = 0; a < 3; ++a) {
    mn[a] = wave_min(mn[a]);
    mx[a] = wave_max(mx[a]);
  }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    for (int a = 0; a < 3; ++a) { sh[w][a] = mn[a]; sh[w][3 + a] = mx[a]; }
    sh[w][6] = __uint_as_float(cnt);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float r[6];
    uint32_t c = 0;
    for (int a = 0; a < 6; ++a) r[a] = sh[0][a];
    for (int ww = 0; ww < 4; ++ww) {
      for (int a = 0; a < 3; ++a) { r[a] = fminf(r[a], sh[ww][a]); r[3 + a] = fmaxf(r[3 + a], sh[ww][3 + a]); }
      c += __float_as_uint(sh[ww][6]);
    }
    float* p = part + 8 * blockIdx.x;
    for (int a = 0; a < 6; ++a) p[a] = r[a];
    p[6] = __uint_as_float(c);
    p[7] = 0.f;
  }
}

__global__ void __launch_bounds__(64) k_vg_params(const float* __restrict__ part, int nparts, float leaf,
                                                 VGParams* __restrict__ P) {
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  uint32_t cnt = 0;
  for (int b = threadIdx.x; b < nparts; b += 64) {
    const float* p = part + 8 * b;
    for (int a = 0; a < 3; ++a) { mn[a] = fminf(mn[a], p[a]); mx[a] = fmaxf(mx[a], p[3 + a]); }
    cnt += __float_as_uint(p[6]);
  }
  for (int a = 0; a < 3; ++a) { mn[a] = wave_min(mn[a]); mx[a] = wave_max(mx[a]); }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  if (threadIdx.x != 0) return;
  VGParams q;
  const float inv = 1.0f / leaf;
  q.inv = inv;
  q.nfinite = cnt;
  for (int a = 0; a < 3; ++a) { q.mn[a] = mn[a]; q.mx[a] = mx[a]; }
  q.overflow = 0;
  q.nbits = 0;
  q.mul1 = q.mul2 = 0;
  for (int a = 0; a < 3; ++a) q.min_b[a] = q.div_b[a] = 0;
  q.unsorted = 0;
  q.chk_done = 0;
  if (cnt > 0) {
    const int64_t dx = (int64_t)((mx[0] - mn[0]) * inv) + 1;
    const int64_t dy = (int64_t)((mx[1] - mn[1]) * inv) + 1;
    const int64_t dz = (int64_t)((mx[2] - mn[2]) * inv) + 1;
    if (dx * dy * dz > (int64_t)2147483647) {
      q.overflow = 1;
    } else {
      for (int a = 0; a < 3; ++a) {
        q.min_b[a] = (int32_t)floorf(mn[a] * inv);
        const int32_t max_b = (int32_t)floorf(mx[a] * inv);
        q.div_b[a] = max_b - q.min_b[a] + 1;
      }
      q.mul1 = q.div_b[0];
      q.mul2 = (int64_t)q.div_b[0] * q.div_b[1];
      const uint64_t total = (uint64_t)q.div_b[0] * (uint64_t)q.div_b[1] * (uint64_t)q.div_b[2];
      uint32_t nb = 1;
      while (nb < 32 && (1ull << nb) <= total) ++nb;  // 2^nbits > total: the invalid key sorts last
      q.nbits = nb;
    }
  }
  *P = q;
}

__global__ void __launch_bounds__(256) k_vg_keys(const float* __restrict__ xyz, const uint32_t* __restrict__ d_n,
                                                 const VGParams* __restrict__ P, uint32_t* __restrict__ keys) {
  const VGParams q = *P;
  if (q.overflow || q.nfinite == 0) return;
  const uint32_t n = *d_n;
  for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
    const float x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
    uint32_t key = 0xFFFFFFFFu;
    if (finite3(x, y, z)) {
      const int i0 = (int)(floorf(x * q.inv) - (float)q.min_b[0]);
      const int i1 = (int)(floorf(y * q.inv) - (float)q.min_b[1]);
      const int i2 = (int)(floorf(z * q.inv) - (float)q.min_b[2]);
      key = (uint32_t)((int64_t)i0 + (int64_t)i1 * q.mul1 + (int64_t)i2 * q.mul2);
    }
    keys[i] = key;
  }
}

// Presorted check (second pass): vals = identity, and if every key is strictly above
// its predecessor the last block to finish sets nbits = 0, so the radix passes exit
// at once and the identity permutation stands -- the stable sort of sorted keys.
__global__ void __launch_bounds__(256) k_vg_sorted(const uint32_t* __restrict__ keys, const uint32_t* __restrict__ d_n,
                                                   VGParams* __restrict__ P, uint32_t* __restrict__ vals) {
  __shared__ uint32_t bad_sh;
  if (threadIdx.x == 0) bad_sh = 0;
  __syncthreads();
  const bool live = !P->overflow && P->nfinite != 0;
  const uint32_t n = *d_n;
  uint32_t bad = 0;
  if (live)
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
      vals[i] = i;
      if (i + 1 < n && !(keys[i] < keys[i + 1])) bad = 1;
    }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(&bad_sh, 1u);
  __syncthreads();
  if (threadIdx.x != 0) return;
  if (bad_sh) atomicOr(&P->unsorted, 1u);
  __threadfence();
  if (atomicAdd(&P->chk_done, 1u) == gridDim.x - 1) {
    __threadfence();
    if (live && atomicOr(&P->unsorted, 0u) == 0) P->nbits = 0;
  }
}

// One thread per leaf: Vector3f accumulation in ascending input index, then / n.
__global__ void __launch_bounds__(256) k_vg_centroid(const float* __restrict__ xyz, const uint32_t* __restrict__ d_n,
                                                     const VGParams* __restrict__ P, const uint32_t* __restrict__ vals,
                                                     const uint32_t* __restrict__ starts,
                                                     const uint32_t* __restrict__ d_nseg, float* __restrict__ out,
                                                     uint32_t* __restrict__ d_m) {
  const VGParams q = *P;
  const uint32_t n = *d_n;
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x, gsz = gridDim.x * 256;
  if (q.overflow) {  // "Integer indices would overflow": output = *input_
    for (uint32_t i = gid; i < n; i += gsz) {
      out[3 * i] = xyz[3 * i]; out[3 * i + 1] = xyz[3 * i + 1]; out[3 * i + 2] = xyz[3 * i + 2];
    }
    if (gid == 0) *d_m = n;
    return;
  }
  const uint32_t ns = q.nfinite ? *d_nseg : 0u;
  if (gid == 0) *d_m = ns;
  for (uint32_t s = gid; s < ns; s += gsz) {
    const uint32_t b = starts[s], e = starts[s + 1];
    float sx = 0.f, sy = 0.f, sz = 0.f;
    for (uint32_t k = b; k < e; ++k) {
      const uint32_t j = vals[k];
      sx += xyz[3 * j]; sy += xyz[3 * j + 1]; sz += xyz[3 * j + 2];
    }
    const float c = (float)(e - b);
    out[3 * s] = sx / c; out[3 * s + 1] = sy / c; out[3 * s + 2] = sz / c;
  }
}

inline uint32_t grid_for(uint32_t cap, uint32_t per = 256, uint32_t mx = 4096) {
  uint32_t g = (cap + per - 1) / per;
  return g < 1 ? 1 : (g > mx ? mx : g);
}

}  // namespace

void voxel_grid(const float* xyz, const uint32_t* d_n, uint32_t cap, float leaf, float* out, uint32_t* d_m, VGBufs b,
                hipStream_t st, bool presorted) {
  k_vg_bbox<<<VG_BBOX_BLOCKS, 256, 0, st>>>(xyz, d_n, b.part);
  k_vg_params<<<1, 64, 0, st>>>(b.part, VG_BBOX_BLOCKS, leaf, b.params);
  FCCF_LAUNCH("k_vg_keys", (d_n, 16.0), k_vg_keys, grid_for(cap), 256, 0, st, xyz, d_n, b.params, b.k0);
  if (presorted) k_vg_sorted<<<grid_for(cap, 1024, 1024), 256, 0, st>>>(b.k0, d_n, b.params, b.v0);
  // with nbits = 0 every pass exits and v0 keeps the identity written above
  radix_sort_u32(b.k0, b.v0, b.k1, b.v1, d_n, cap, &b.params->nbits, 32, !presorted, b.ss, st);
  segment_heads_u32(b.k0, d_n, cap, 0xFFFFFFFFu, b.starts, b.nseg, b.ss, st);
  FCCF_LAUNCH("k_vg_centroid", (d_n, 16.0, d_m, 12.0), k_vg_centroid, grid_for(cap), 256, 0, st, xyz, d_n, b.params, b.v0, b.starts, b.nseg, out, d_m);
}

}  // namespace fccf
