// voxelgrid.hip — K1: pcl::VoxelGrid<PointXYZ>::applyFilter on gfx950.
//
// Reference call sites: FCCF.cpp:1668-1678 (main, one pass per cloud) and
// :1377-1387 (driver, a second pass).  Semantics:
//   bbox over finite points -> int32 overflow guard (output = input) ->
//   idx = ijk0 + ijk1*div0 + ijk2*div0*div1 with ijk = int(floor(p*inv) - float(min_b))
//   -> sort (idx, index) -> one centroid per run, Vector3f sum / n, ascending idx.
// PCL sorts with libstdc++ std::sort (introsort, unstable); introsort.hip reproduces
// its order, so each leaf is summed in exactly the reference's order.
//
// HBM traffic per pass (algorithmic): read 12 B/pt, write 12 B/leaf; the sort adds
// its rounds and the owner pass (introsort.hip).
#define KT_TU 2  // ktrace.h source tag
#include "probe.h"
#include "kernels.h"
#include "group.h"
#include "ctx.h"

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
// The pass's entry kernel (VGEntry): block 0 also publishes the input pointer (and,
// with set_n, the count) and clears the pass's flags (keys' order check, the
// centroid kernel's non-finite flag) before any later kernel of the pass runs.
// Tag: 0 = a first pass (the patched entry node), 1 = a presorted second pass, so the
// two passes are distinct kernels when one graph holds both.
template <int Tag>
__global__ void __launch_bounds__(256) k_vg_bbox(B4<const float*> xyz2, B4<uint32_t*> d_n2, B4<uint32_t> n2,
                                                 int set_n, B4<float*> part2, B4<VGParams*> P2) {
  KT();
  __shared__ float sh[4][7];
  const int e = blockIdx.y;
  const float* __restrict__ xyz = xyz2[e];
  const uint32_t n = set_n ? n2[e] : *d_n2[e];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (Tag == 0) {
      P2[e]->t_main = __builtin_amdgcn_s_memrealtime();
      P2[e]->sort_err = 0;  // (the driver's pass adds its flags to main's)
    }
    P2[e]->unsorted = 0;
    P2[e]->redo = 0;
    P2[e]->chk_done = 0;
    P2[e]->nonfinite = 0;
    P2[e]->src = xyz;
    if (set_n) *d_n2[e] = n;
  }
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  uint32_t cnt = 0;
  auto add = [&](float x, float y, float z) {
    if (!finite3(x, y, z)) return;
    mn[0] = fminf(mn[0], x); mn[1] = fminf(mn[1], y); mn[2] = fminf(mn[2], z);
    mx[0] = fmaxf(mx[0], x); mx[1] = fmaxf(mx[1], y); mx[2] = fmaxf(mx[2], z);
    ++cnt;
  };
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x, gsz = gridDim.x * 256;
  const uint32_t nq = (((uintptr_t)xyz) & 15u) == 0 ? n / 4 : 0;  // four points per thread, 16-byte loads
  for (uint32_t qd = gid; qd < nq; qd += gsz) {
    const float4* v = reinterpret_cast<const float4*>(xyz) + 3 * (size_t)qd;
    const float4 a = v[0], b = v[1], c = v[2];
    add(a.x, a.y, a.z);
    add(a.w, b.x, b.y);
    add(b.z, b.w, c.x);
    add(c.y, c.z, c.w);
  }
  for (uint32_t i = 4 * nq + gid; i < n; i += gsz) add(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
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
    float* p = part2[e] + 8 * blockIdx.x;
    for (int a = 0; a < 6; ++a) p[a] = r[a];
    p[6] = __uint_as_float(c);
    p[7] = 0.f;
  }
}

// The pass's VoxelGrid parameters from the nparts bbox partials: leaf size, bounds,
// int32 overflow guard, index multipliers, radix width.  Every thread of the block
// calls it and gets the result (256 threads; min/max/count reductions are exact in
// any order, so every block computes the same bits).
__device__ VGParams vg_params_block(const float* __restrict__ part, int nparts, float leaf) {
  __shared__ float sh[4][7];
  __shared__ VGParams sq;
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  uint32_t cnt = 0;
  for (int b = threadIdx.x; b < nparts; b += blockDim.x) {
    const float* p = part + 8 * b;
    for (int a = 0; a < 3; ++a) { mn[a] = fminf(mn[a], p[a]); mx[a] = fmaxf(mx[a], p[3 + a]); }
    cnt += __float_as_uint(p[6]);
  }
  for (int a = 0; a < 3; ++a) { mn[a] = wave_min(mn[a]); mx[a] = wave_max(mx[a]); }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    for (int a = 0; a < 3; ++a) { sh[w][a] = mn[a]; sh[w][3 + a] = mx[a]; }
    sh[w][6] = __uint_as_float(cnt);
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    cnt = 0;
    for (int a = 0; a < 3; ++a) { mn[a] = INFINITY; mx[a] = -INFINITY; }
    for (int ww = 0; ww < (int)(blockDim.x >> 6); ++ww) {
      for (int a = 0; a < 3; ++a) { mn[a] = fminf(mn[a], sh[ww][a]); mx[a] = fmaxf(mx[a], sh[ww][3 + a]); }
      cnt += __float_as_uint(sh[ww][6]);
    }
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
    q.nonfinite = 0;
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
    sq = q;
  }
  __syncthreads();
  return sq;
}

// Block (0, e) publishes the parameters for the later kernels of the pass; the
// flags (unsorted, chk_done, nonfinite) were cleared by k_vg_bbox and are only
// ever set with atomics, so they are not part of that write.
__device__ void vg_params_publish(VGParams* P, const VGParams& q) {
  for (int a = 0; a < 3; ++a) {
    P->mn[a] = q.mn[a];
    P->mx[a] = q.mx[a];
    P->min_b[a] = q.min_b[a];
    P->div_b[a] = q.div_b[a];
  }
  P->inv = q.inv;
  P->nfinite = q.nfinite;
  P->mul1 = q.mul1;
  P->mul2 = q.mul2;
  P->overflow = q.overflow;
  P->nbits = q.nbits;
}

__device__ __forceinline__ uint32_t vg_key(const VGParams& q, float x, float y, float z) {
  if (!finite3(x, y, z)) return 0xFFFFFFFFu;
  const int i0 = (int)(floorf(x * q.inv) - (float)q.min_b[0]);
  const int i1 = (int)(floorf(y * q.inv) - (float)q.min_b[1]);
  const int i2 = (int)(floorf(z * q.inv) - (float)q.min_b[2]);
  return (uint32_t)((int64_t)i0 + (int64_t)i1 * q.mul1 + (int64_t)i2 * q.mul2);
}

// Leaf keys and vals = identity.  presorted (the driver's second pass): a key not
// strictly above its predecessor -- or any non-finite point -- sets P->unsorted;
// otherwise every leaf holds exactly one point and the pass is the identity (the
// sort tail, segmentation and centroid kernels take their shortcut).
__global__ void __launch_bounds__(256) k_vg_keys(B4<const uint32_t*> d_n2, B4<VGParams*> P2,
                                                 B4<uint32_t*> keys2, B4<uint32_t*> vals2, int presorted,
                                                 B4<const float*> part2, int nparts, float leaf) {
  KT();
  const int e = blockIdx.y;
  VGParams* P = P2[e];
  const VGParams q = vg_params_block(part2[e], nparts, leaf);  // every block, from the bbox partials
  if (blockIdx.x == 0 && threadIdx.x == 0) vg_params_publish(P, q);
  const uint32_t n = *d_n2[e];
  if (q.overflow) return;
  if (q.nfinite == 0) {
    if (presorted && n && blockIdx.x == 0 && threadIdx.x == 0) P->unsorted = 1u;
    return;
  }
  const float* __restrict__ xyz = P->src;
  uint32_t* __restrict__ keys = keys2[e];
  uint32_t* __restrict__ vals = vals2[e];
  bool bad = false;
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x, gsz = gridDim.x * 256;
  // four points per thread: three 16-byte loads, one 16-byte store of keys (and of
  // vals); the order check reads the next quad's first point
  const bool al = ((((uintptr_t)xyz) | ((uintptr_t)keys) | ((uintptr_t)vals)) & 15u) == 0;
  const uint32_t nq = al ? n / 4 : 0;
  for (uint32_t qd = gid; qd < nq; qd += gsz) {
    const float4* v = reinterpret_cast<const float4*>(xyz) + 3 * (size_t)qd;
    const float4 a = v[0], b = v[1], c = v[2];
    const uint32_t i0 = 4 * qd;
    uint4 k;
    k.x = vg_key(q, a.x, a.y, a.z);
    k.y = vg_key(q, a.w, b.x, b.y);
    k.z = vg_key(q, b.z, b.w, c.x);
    k.w = vg_key(q, c.y, c.z, c.w);
    reinterpret_cast<uint4*>(keys)[qd] = k;
    reinterpret_cast<uint4*>(vals)[qd] = make_uint4(i0, i0 + 1, i0 + 2, i0 + 3);
    if (presorted) {
      bad |= k.x == 0xFFFFFFFFu || k.y == 0xFFFFFFFFu || k.z == 0xFFFFFFFFu || k.w == 0xFFFFFFFFu;
      bad |= !(k.x < k.y) || !(k.y < k.z) || !(k.z < k.w);
      if (i0 + 4 < n && !(k.w < vg_key(q, xyz[3 * i0 + 12], xyz[3 * i0 + 13], xyz[3 * i0 + 14]))) bad = true;
    }
  }
  for (uint32_t i = 4 * nq + gid; i < n; i += gsz) {
    const uint32_t key = vg_key(q, xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
    keys[i] = key;
    vals[i] = i;
    if (presorted) {
      if (key == 0xFFFFFFFFu) bad = true;
      if (i + 1 < n && !(key < vg_key(q, xyz[3 * i + 3], xyz[3 * i + 4], xyz[3 * i + 5]))) bad = true;
    }
  }
  if (presorted && __ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(&P->unsorted, 1u);
}

// One thread per leaf: Vector3f accumulation in ascending input index, then / n.
// The first CL members' indices and points are loaded before any is summed (a
// leaf holds ~3 points: the loads of a thread overlap instead of forming a
// dependent chain); each block's 256 centroids are staged in LDS and written as
// coalesced 16-byte words.  The pass-through cases are flat 16-byte copies.
constexpr int CL = 4;
__global__ void __launch_bounds__(256) k_vg_centroid(B4<const uint32_t*> d_n2, B4<VGParams*> P2, B4<const uint32_t*> vals2,
                                                     B4<const uint32_t*> starts2, B4<const uint32_t*> d_nseg2,
                                                     B4<float*> out2, B4<uint32_t*> d_m2, int presorted,
                                                     B4<float*> copy2, B4<const uint32_t*> inject2,
                                                     B4<const float*> xyzs2) {
  KT();
  const int e = blockIdx.y;
  const VGParams q = *P2[e];
  float* __restrict__ cpy = copy2[e];
  bool bad = false;  // a non-finite output value (only tracked with a copy)
  const float* __restrict__ xyz = q.src;
  const uint32_t* __restrict__ vals = vals2[e];
  const uint32_t* __restrict__ starts = starts2[e];
  const uint32_t* __restrict__ d_nseg = d_nseg2[e];
  float* __restrict__ out = out2[e];
  uint32_t* __restrict__ d_m = d_m2[e];
  const uint32_t n = *d_n2[e];
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x, gsz = gridDim.x * 256;
  // VG_OPTIMISTIC: no sort or segmentation ran; an input out of leaf order is left to
  // the caller's redo (nothing is output, the flag goes to the cloud mailbox)
  if (presorted == VG_OPTIMISTIC && !q.overflow && n) {
    const uint32_t* inj = inject2[e];
    if (q.unsorted || (inj && ((*inj & VG_FORCE_REDO) || ((*inj & VG_FORCE_REDO_LATER) && e >= 2)))) {
      if (gid == 0) {
        *d_m = 0u;
        P2[e]->redo = 1u;
      }
      return;
    }
  }
  // "Integer indices would overflow": output = *input_; presorted with every leaf
  // holding one finite point: the centroid of one point is the point (p / 1.f == p)
  if (q.overflow || (presorted && q.unsorted == 0u && n && q.nfinite == n)) {
    const uint32_t nf = 3 * n;
    const bool al = ((((uintptr_t)xyz) | ((uintptr_t)out)) & 15u) == 0;
    const uint32_t n4 = al ? nf / 4 : 0;
    for (uint32_t i = gid; i < n4; i += gsz) {
      const float4 v = reinterpret_cast<const float4*>(xyz)[i];
      reinterpret_cast<float4*>(out)[i] = v;
      if (cpy) {
        reinterpret_cast<float4*>(cpy)[i] = v;
        bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
      }
    }
    for (uint32_t i = 4 * n4 + gid; i < nf; i += gsz) {
      out[i] = xyz[i];
      if (cpy) {
        cpy[i] = xyz[i];
        bad |= !isfinite(xyz[i]);
      }
    }
    if (gid == 0) *d_m = n;
    if (cpy && __ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(&P2[e]->nonfinite, 1u);
    return;
  }
  const uint32_t ns = q.nfinite ? *d_nseg : 0u;
  if (gid == 0) *d_m = ns;
  const float* __restrict__ xs = xyzs2[e];
  __shared__ __attribute__((aligned(16))) float so[3 * 256];
  const bool al = (((uintptr_t)out) & 15u) == 0;
  for (uint32_t s0 = blockIdx.x * 256; s0 < ns; s0 += gsz) {
    const uint32_t s = s0 + threadIdx.x;
    if (s < ns) {
      const uint32_t b = starts[s], e1 = starts[s + 1];
      float sx = 0.f, sy = 0.f, sz = 0.f;
      if (xs) {  // members in sorted order, contiguous
        for (uint32_t k0 = b; k0 < e1; k0 += CL) {
          float px[CL], py[CL], pz[CL];
#pragma unroll
          for (int c = 0; c < CL; ++c) {
            const size_t k = min(k0 + c, e1 - 1u);
            px[c] = xs[3 * k];
            py[c] = xs[3 * k + 1];
            pz[c] = xs[3 * k + 2];
          }
#pragma unroll
          for (int c = 0; c < CL; ++c)
            if (k0 + c < e1) { sx += px[c]; sy += py[c]; sz += pz[c]; }
        }
      }
      for (uint32_t k0 = b; !xs && k0 < e1; k0 += CL) {
        uint32_t j[CL];
        float px[CL], py[CL], pz[CL];
#pragma unroll
        for (int c = 0; c < CL; ++c) j[c] = vals[min(k0 + c, e1 - 1u)];
#pragma unroll
        for (int c = 0; c < CL; ++c) {
          px[c] = xyz[3 * (size_t)j[c]];
          py[c] = xyz[3 * (size_t)j[c] + 1];
          pz[c] = xyz[3 * (size_t)j[c] + 2];
        }
#pragma unroll
        for (int c = 0; c < CL; ++c)
          if (k0 + c < e1) { sx += px[c]; sy += py[c]; sz += pz[c]; }
      }
      const float cnt = (float)(e1 - b);
      so[3 * threadIdx.x] = sx / cnt;
      so[3 * threadIdx.x + 1] = sy / cnt;
      so[3 * threadIdx.x + 2] = sz / cnt;
      bad |= !finite3(so[3 * threadIdx.x], so[3 * threadIdx.x + 1], so[3 * threadIdx.x + 2]);
    }
    __syncthreads();
    const uint32_t m = min(256u, ns - s0);  // centroids of this block step
    float* dst = out + 3 * (size_t)s0;
    float* dcp = cpy ? cpy + 3 * (size_t)s0 : nullptr;
    if (al && m == 256u) {
      if (threadIdx.x < 192) {
        const float4 v = reinterpret_cast<const float4*>(so)[threadIdx.x];
        reinterpret_cast<float4*>(dst)[threadIdx.x] = v;
        if (dcp) reinterpret_cast<float4*>(dcp)[threadIdx.x] = v;
      }
    } else {
      for (uint32_t i = threadIdx.x; i < 3 * m; i += 256) {
        dst[i] = so[i];
        if (dcp) dcp[i] = so[i];
      }
    }
    __syncthreads();
  }
  if (cpy && __ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(&P2[e]->nonfinite, 1u);
}

inline uint32_t grid_for(uint32_t cap, uint32_t per = 256, uint32_t mx = 4096) {
  uint32_t g = (cap + per - 1) / per;
  return g < 1 ? 1 : (g > mx ? mx : g);
}

}  // namespace

const void* vg_entry_kernel() { return (const void*)k_vg_bbox<0>; }

void voxel_grid(B4<const float*> xyz, B4<uint32_t*> d_nw, uint32_t cap, float leaf, B4<float*> out,
                B4<uint32_t*> d_m, B4<VGBufs> b, hipStream_t st, int presorted, int nbatch, B4<float*> out_copy,
                const uint32_t* n_in, VGEntry* entry) {
  const B4<const uint32_t*> d_n(d_nw);
  // one field of every problem's buffers (entries past nbatch repeat the caller's last)
  auto F = [&](auto get) {
    B4<decltype(get(b[0]))> r;
    for (int e = 0; e < BMAX; ++e) r.v[e] = get(b[e]);
    return r;
  };
  const B4<VGParams*> P = F([](const VGBufs& v) { return v.params; });
  const B4<uint32_t*> k0 = F([](const VGBufs& v) { return v.k0; }), v0 = F([](const VGBufs& v) { return v.v0; });
  const B4<uint32_t*> k1 = F([](const VGBufs& v) { return v.k1; }), v1 = F([](const VGBufs& v) { return v.v1; });
  const B4<uint32_t*> starts = F([](const VGBufs& v) { return v.starts; }), nseg = F([](const VGBufs& v) { return v.nseg; });
  const B4<SortScratch> ss = F([](const VGBufs& v) { return v.ss; });

  VGEntry en;
  en.xyz = xyz;
  en.d_n = d_nw;
  en.n = B4<uint32_t>(0u);
  for (int e = 0; n_in && e < nbatch; ++e) en.n.v[e] = n_in[e];
  en.set_n = n_in ? 1 : 0;
  en.part = F([](const VGBufs& v) { return v.part; });
  en.P = P;
  en.bind();
  if (presorted)
    k_vg_bbox<1><<<dim3(VG_BBOX_BLOCKS, nbatch), 256, 0, st>>>(en.xyz, en.d_n, en.n, en.set_n, en.part, en.P);
  else
    k_vg_bbox<0><<<dim3(VG_BBOX_BLOCKS, nbatch), 256, 0, st>>>(en.xyz, en.d_n, en.n, en.set_n, en.part, en.P);
  if (entry) {
    *entry = en;
    entry->bind();
  }
  // probe: algorithmic bytes summed over the launch's clouds
  ProbeBytes pb_keys, pb_cen;
  for (int e = 0; e < nbatch; ++e) {
    pb_keys.add(d_n[e], 16.0);
    pb_cen.add(d_n[e], 16.0).add(d_m[e], 12.0);
  }
  const B4<const uint32_t*> unsorted = F([](const VGBufs& v) { return (const uint32_t*)&v.params->unsorted; });
  // the keys kernel also derives the parameters (k_vg_params folded in): each of its
  // VG_KEY_BLOCKS blocks reduces the bbox partials itself, so its grid is kept small
  const dim3 gk(std::min(grid_for(cap), (uint32_t)VG_KEY_BLOCKS), nbatch);
  FCCF_LAUNCH("k_vg_keys", (pb_keys), k_vg_keys, gk, 256, 0, st, d_n, P, k0, v0, presorted ? 1 : 0, F([](const VGBufs& v) { return (const float*)v.part; }), VG_BBOX_BLOCKS, leaf);
  // the first pass's sort also writes the points in sorted order (IsBufs::xyzs), so the
  // centroid reads each leaf's members contiguously; not for a sharded sort (each rank
  // finishes only its range, and the gather moves keys and values only)
  const bool sorted_pts = !presorted && b[0].is.shard_n <= 1;
  B4<IsBufs> isb = F([](const VGBufs& v) { return v.is; });
  if (sorted_pts) {
    for (int e = 0; e < BMAX; ++e) isb.v[e].xyzs = b[e].xyzs;
  }
  const B4<const float*> xyzs = sorted_pts ? F([](const VGBufs& v) { return (const float*)v.xyzs; })
                                           : B4<const float*>(nullptr);
  const B4<const VGParams*> Pc(P);
  if (!presorted) {
    introsort_u32(k0, v0, k1, v1, d_n, Pc, cap, isb, st, nbatch, false);
    if (b[0].is.shard_n > 1)  // row D: every rank's sorted slice of every cloud, gathered in rank order
      shard_gather_sorted((Group*)b[0].is.shard_group, k0, v0,
                          F([](const VGBufs& v) { return (const uint32_t*)v.is.bounds; }), nbatch, st);
    segment_heads_u32(B4<const uint32_t*>(k0), d_n, cap, 0xFFFFFFFFu, starts, nseg, ss, st, B4<uint32_t*>(nullptr),
                      nbatch);
  } else if (presorted == VG_PRESORTED) {  // usually already in leaf order: a sort and segmentation that run only if not
    introsort_u32(k0, v0, k1, v1, d_n, Pc, cap, isb, st, nbatch, true);
    segment_heads_u32(B4<const uint32_t*>(k0), d_n, cap, 0xFFFFFFFFu, starts, nseg, ss, st, B4<uint32_t*>(nullptr),
                      nbatch, unsorted);
  }
  const B4<const uint32_t*> inj = F([](const VGBufs& v) { return v.is.inject; });
  FCCF_LAUNCH("k_vg_centroid", (pb_cen), k_vg_centroid, dim3(grid_stream(cap, nbatch), nbatch), 256, 0, st, d_n, P, B4<const uint32_t*>(v0), B4<const uint32_t*>(starts), B4<const uint32_t*>(nseg), out, d_m, presorted, out_copy, inj, xyzs);
}

}  // namespace fccf
