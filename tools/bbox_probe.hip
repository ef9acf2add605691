// Dev probe (not product): why is k_vg_bbox ~20-30 us for 12 MB?  Times bbox-like
// reductions over a 1M-point xyz array with HIP events, in several variants:
//   A  the product's loop (3 x float4 per thread-quad, stride 48 B between lanes)
//   B  same, launched twice back to back (second = warm)
//   C  flat coalesced float4 reads of the array (no per-point decode)
//   D  A with 2048 blocks
// Build: hipcc --offload-arch=gfx950 -O3 tools/bbox_probe.hip -o /tmp/bbox_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>

__device__ __forceinline__ float wmin(float v) { for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64)); return v; }
__device__ __forceinline__ float wmax(float v) { for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64)); return v; }

__global__ void __launch_bounds__(256) kA(const float* __restrict__ xyz, uint32_t n, float* part) {
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  uint32_t cnt = 0;
  auto add = [&](float x, float y, float z) {
    if (!(isfinite(x) && isfinite(y) && isfinite(z))) return;
    mn[0] = fminf(mn[0], x); mn[1] = fminf(mn[1], y); mn[2] = fminf(mn[2], z);
    mx[0] = fmaxf(mx[0], x); mx[1] = fmaxf(mx[1], y); mx[2] = fmaxf(mx[2], z);
    ++cnt;
  };
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x, gsz = gridDim.x * 256, nq = n / 4;
  for (uint32_t qd = gid; qd < nq; qd += gsz) {
    const float4* v = reinterpret_cast<const float4*>(xyz) + 3 * (size_t)qd;
    const float4 a = v[0], b = v[1], c = v[2];
    add(a.x, a.y, a.z); add(a.w, b.x, b.y); add(b.z, b.w, c.x); add(c.y, c.z, c.w);
  }
  for (int a = 0; a < 3; ++a) { mn[a] = wmin(mn[a]); mx[a] = wmax(mx[a]); }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  __shared__ float sh[4][7];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { for (int a = 0; a < 3; ++a) { sh[w][a] = mn[a]; sh[w][3 + a] = mx[a]; } sh[w][6] = __uint_as_float(cnt); }
  __syncthreads();
  if (threadIdx.x == 0) {
    float r[6]; uint32_t c = 0;
    for (int a = 0; a < 6; ++a) r[a] = sh[0][a];
    for (int ww = 0; ww < 4; ++ww) { for (int a = 0; a < 3; ++a) { r[a] = fminf(r[a], sh[ww][a]); r[3 + a] = fmaxf(r[3 + a], sh[ww][3 + a]); } c += __float_as_uint(sh[ww][6]); }
    float* p = part + 8 * blockIdx.x;
    for (int a = 0; a < 6; ++a) p[a] = r[a];
    p[6] = __uint_as_float(c); p[7] = 0.f;
  }
}

template <class T>
struct B2 {
  T v[2];
  B2() = default;
  __host__ __device__ B2(T a) : v{a, a} {}
  __host__ __device__ B2(T a, T b) : v{a, b} {}
  __host__ __device__ T operator[](int i) const { return i ? v[1] : v[0]; }
};
struct VGP { float f[32]; uint32_t unsorted, chk_done, nonfinite; const float* src; };
// the product's signature: batch-indexed pointer pairs, block 0 publishing the input
template <int MODE>  // 0 product; 1 e = 0 (static index); 2 no block-0 publish; 3 select instead of index
__global__ void __launch_bounds__(256) kP(B2<const float*> xyz2, B2<uint32_t*> d_n2, B2<uint32_t> n2, int set_n,
                                          B2<float*> part2, B2<VGP*> P2) {
  const int e = MODE == 1 ? 0 : blockIdx.y;
  const float* __restrict__ xyz = MODE == 3 ? (e ? xyz2.v[1] : xyz2.v[0]) : xyz2[e];
  const uint32_t n = set_n ? n2[e] : *d_n2[e];
  if (MODE != 2 && blockIdx.x == 0 && threadIdx.x == 0) {
    P2[e]->unsorted = 0; P2[e]->chk_done = 0; P2[e]->nonfinite = 0; P2[e]->src = xyz;
    if (set_n) *d_n2[e] = n;
  }
  float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
  uint32_t cnt = 0;
  auto add = [&](float x, float y, float z) {
    if (!(isfinite(x) && isfinite(y) && isfinite(z))) return;
    mn[0] = fminf(mn[0], x); mn[1] = fminf(mn[1], y); mn[2] = fminf(mn[2], z);
    mx[0] = fmaxf(mx[0], x); mx[1] = fmaxf(mx[1], y); mx[2] = fmaxf(mx[2], z);
    ++cnt;
  };
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x, gsz = gridDim.x * 256;
  const uint32_t nq = (((uintptr_t)xyz) & 15u) == 0 ? n / 4 : 0;
  for (uint32_t qd = gid; qd < nq; qd += gsz) {
    const float4* v = reinterpret_cast<const float4*>(xyz) + 3 * (size_t)qd;
    const float4 a = v[0], b = v[1], c = v[2];
    add(a.x, a.y, a.z); add(a.w, b.x, b.y); add(b.z, b.w, c.x); add(c.y, c.z, c.w);
  }
  for (uint32_t i = 4 * nq + gid; i < n; i += gsz) add(xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]);
  for (int a = 0; a < 3; ++a) { mn[a] = wmin(mn[a]); mx[a] = wmax(mx[a]); }
  for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
  __shared__ float sh[4][7];
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { for (int a = 0; a < 3; ++a) { sh[w][a] = mn[a]; sh[w][3 + a] = mx[a]; } sh[w][6] = __uint_as_float(cnt); }
  __syncthreads();
  if (threadIdx.x == 0) {
    float r[6]; uint32_t c = 0;
    for (int a = 0; a < 6; ++a) r[a] = sh[0][a];
    for (int ww = 0; ww < 4; ++ww) { for (int a = 0; a < 3; ++a) { r[a] = fminf(r[a], sh[ww][a]); r[3 + a] = fmaxf(r[3 + a], sh[ww][3 + a]); } c += __float_as_uint(sh[ww][6]); }
    float* p = part2[e] + 8 * blockIdx.x;
    for (int a = 0; a < 6; ++a) p[a] = r[a];
    p[6] = __uint_as_float(c); p[7] = 0.f;
  }
}

__global__ void __launch_bounds__(256) kC(const float4* __restrict__ x, uint32_t n4, float* part) {
  float s = 0.f;
  const uint32_t gid = blockIdx.x * 256 + threadIdx.x, gsz = gridDim.x * 256;
  for (uint32_t i = gid; i < n4; i += gsz) { const float4 v = x[i]; s = fmaxf(s, fmaxf(fmaxf(v.x, v.y), fmaxf(v.z, v.w))); }
  s = wmax(s);
  if ((threadIdx.x & 63) == 0) part[blockIdx.x * 4 + (threadIdx.x >> 6)] = s;
}

int main() {
  const uint32_t n = 1000000;
  std::vector<float> h(3 * (size_t)n);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (float)((i * 2654435761u) % 10007) * 0.001f;
  float *d, *part, *big;
  hipMalloc(&d, 12 * (size_t)n);
  hipMalloc(&part, 8 * 4096 * 4);
  hipMalloc(&big, 512u << 20);
  hipMemcpy(d, h.data(), 12 * (size_t)n, hipMemcpyHostToDevice);
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto timeit = [&](const char* name, auto launch) {
    for (int rep = 0; rep < 3; ++rep) {
      hipMemset(big, rep, 512u << 20);  // evict caches between reps
      hipDeviceSynchronize();
      hipEventRecord(e0, 0);
      launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0; hipEventElapsedTime(&ms, e0, e1);
      std::printf("%-28s rep %d  %8.2f us\n", name, rep, ms * 1e3);
    }
  };
  timeit("A 512 blocks", [&] { kA<<<512, 256>>>(d, n, part); });
  timeit("B 512 blocks twice", [&] { kA<<<512, 256>>>(d, n, part); kA<<<512, 256>>>(d, n, part); });
  timeit("C flat float4 512 blocks", [&] { kC<<<512, 256>>>((const float4*)d, 3 * n / 4, part); });
  timeit("D 2048 blocks", [&] { kA<<<2048, 256>>>(d, n, part); });
  timeit("E 1024 blocks", [&] { kA<<<1024, 256>>>(d, n, part); });
  timeit("F C with 2048 blocks", [&] { kC<<<2048, 256>>>((const float4*)d, 3 * n / 4, part); });
  VGP* P;
  uint32_t* dn;
  hipMalloc(&P, 2 * sizeof(VGP));
  hipMalloc(&dn, 64);
  hipMemcpy(dn, &n, 4, hipMemcpyHostToDevice);
  timeit("P1 static e", [&] {
    kP<1><<<dim3(512, 1), 256>>>(B2<const float*>(d), B2<uint32_t*>(dn), B2<uint32_t>(n), 1, B2<float*>(part), B2<VGP*>(P));
  });
  timeit("P2 no publish", [&] {
    kP<2><<<dim3(512, 1), 256>>>(B2<const float*>(d), B2<uint32_t*>(dn), B2<uint32_t>(n), 1, B2<float*>(part), B2<VGP*>(P));
  });
  timeit("P3 select", [&] {
    kP<3><<<dim3(512, 1), 256>>>(B2<const float*>(d), B2<uint32_t*>(dn), B2<uint32_t>(n), 1, B2<float*>(part), B2<VGP*>(P));
  });
  timeit("P product sig, set_n", [&] {
    kP<0><<<dim3(512, 1), 256>>>(B2<const float*>(d), B2<uint32_t*>(dn), B2<uint32_t>(n), 1, B2<float*>(part), B2<VGP*>(P));
  });
  timeit("P product sig, d_n", [&] {
    kP<0><<<dim3(512, 1), 256>>>(B2<const float*>(d), B2<uint32_t*>(dn), B2<uint32_t>(n), 0, B2<float*>(part), B2<VGP*>(P));
  });
  timeit("P batch 2 (same cloud)", [&] {
    kP<0><<<dim3(512, 2), 256>>>(B2<const float*>(d), B2<uint32_t*>(dn), B2<uint32_t>(n), 1, B2<float*>(part, part + 4096 * 4), B2<VGP*>(P, P + 1));
  });
  hipFree(d); hipFree(part); hipFree(big);
  return 0;
}
