// pmc_calib.hip — calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the
// access patterns of K1's sort and VoxelGrid kernels.
// MI355X_MICROARCH.md ("HBM") calibrates only wide streaming reads (FETCH_SIZE = half
// the bytes); every other width is uncalibrated.  Each kernel below moves a KNOWN
// number of bytes in one pattern, so counter / algorithmic is that pattern's factor:
//   stream16_ld / stream4_ld / stream2_ld   coalesced loads, 16 / 4 / 2 B per lane
//   rand4_ld / rand12_ld / rand2_ld          independent random loads (4 B, 12 B as one
//                                            dwordx3, 2 B) over a 256 MiB table
//   stream16_st / stream4_st                 coalesced stores
//   scat4_st / scat12_st                     stores to a random permutation of positions
//                                            (every position written once)
//   part4_st                                 4-B stores scattered within 8 KiB windows
//                                            (a round scatter's partner writes)
// Every kernel reads or writes exactly the bytes it names (the random ones through an
// in-register hash, no index array).  Build: hipcc --offload-arch=gfx950 -O3
// tools/pmc_calib.hip -o tools/pmc_calib; run each PMC pass as its own process:
//   rocprofv3 --pmc FETCH_SIZE --kernel-trace -f csv -d DIR -- tools/pmc_calib
// and summarise with tools/pmc_calib.py.  Prints the algorithmic bytes per kernel.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

struct Pt3 {
  float x, y, z;
};

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

// a bijection of [0, 2^lg): odd multiplier, xor-shift, odd multiplier (mod 2^lg)
__device__ __forceinline__ uint32_t perm(uint32_t i, int lg) {
  const uint32_t m = (1u << lg) - 1u;
  uint32_t x = (i * 0x9E3779B1u) & m;
  x ^= x >> (lg / 2);
  return (x * 0x85EBCA77u) & m;
}

__global__ void stream16_ld(const float4* __restrict__ a, size_t n4, float* out) {
  float s = 0.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
    const float4 v = a[i];
    s += v.x + v.y + v.z + v.w;
  }
  if (s == 12345.f) out[0] = s;  // (never: keeps the loads)
}
__global__ void stream4_ld(const uint32_t* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 0x12345u) out[0] = s;
}
__global__ void stream2_ld(const uint16_t* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 0x12345u) out[0] = s;
}
// random loads: access i goes to line perm(i) of the table (2^21 lines of 128 B: every
// line touched once per launch, so no access can hit a line another one brought in)
__global__ void rand4_ld(const uint32_t* __restrict__ a, uint32_t m, uint32_t* out) {
  uint32_t s = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x)
    s += a[perm(i, 21) * 32u + (mix(i) & 31u)];
  if (s == 0x12345u) out[0] = s;
}
__global__ void rand2_ld(const uint16_t* __restrict__ a, uint32_t m, uint32_t* out) {
  uint32_t s = 0;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x)
    s += a[perm(i, 21) * 64u + (mix(i) & 63u)];
  if (s == 0x12345u) out[0] = s;
}
__global__ void rand12_ld(const char* __restrict__ a, uint32_t m, float* out) {
  float s = 0.f;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) {
    // a 12-byte point inside line perm(i) (4-byte aligned, never crossing the line)
    const Pt3 p = *(const Pt3*)(a + (size_t)perm(i, 21) * 128u + 4u * (mix(i) % 30u));
    s += p.x + p.y + p.z;
  }
  if (s == 12345.f) out[0] = s;
}
__global__ void stream16_st(float4* __restrict__ a, size_t n4) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}
__global__ void stream4_st(uint32_t* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = (uint32_t)i;
}
__global__ void scat4_st(uint32_t* __restrict__ a, int lg, uint32_t m) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x) a[perm(i, lg)] = i;
}
__global__ void scat12_st(Pt3* __restrict__ a, int lg, uint32_t m) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x)
    a[perm(i, lg)] = Pt3{(float)i, 1.f, 2.f};
}
// within each 2048-element window, the elements go to a permutation of the window
__global__ void part4_st(uint32_t* __restrict__ a, uint32_t m) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < m; i += gridDim.x * blockDim.x)
    a[(i & ~2047u) | perm(i & 2047u, 11)] = i;
}

int main() {
  const size_t bytes = 256ull << 20;  // 256 MiB tables: past the 32 MiB of L2 (MALL hits still count)
  void *A, *B;
  float* out;
  CK(hipMalloc(&A, bytes + 64));
  CK(hipMalloc(&B, bytes + 64));
  CK(hipMalloc((void**)&out, 64));
  CK(hipMemset(A, 0, bytes + 64));
  CK(hipMemset(B, 0, bytes + 64));
  const dim3 g(4096), b(256);
  const int reps = 3;
  const uint32_t m = 1u << 24;   // scattered stores per launch (16M: every position of the region once)
  const uint32_t mr = 1u << 21;  // random loads per launch (one per 128-B line of the table)
  std::printf("kernel algorithmic_bytes_per_launch\n");
  for (int r = 0; r < reps; ++r) {
    stream16_ld<<<g, b>>>((const float4*)A, bytes / 16, out);
    stream4_ld<<<g, b>>>((const uint32_t*)A, bytes / 4, (uint32_t*)out);
    stream2_ld<<<g, b>>>((const uint16_t*)A, bytes / 2, (uint32_t*)out);
    rand4_ld<<<g, b>>>((const uint32_t*)A, mr, (uint32_t*)out);
    rand2_ld<<<g, b>>>((const uint16_t*)A, mr, (uint32_t*)out);
    rand12_ld<<<g, b>>>((const char*)A, mr, out);
    stream16_st<<<g, b>>>((float4*)B, bytes / 16);
    stream4_st<<<g, b>>>((uint32_t*)B, bytes / 4);
    scat4_st<<<g, b>>>((uint32_t*)B, 24, m);     // 16M positions of 4 B (64 MiB region)
    scat12_st<<<g, b>>>((Pt3*)B, 24, m);         // 16M positions of 12 B (192 MiB region)
    part4_st<<<g, b>>>((uint32_t*)B, m);
    CK(hipGetLastError());
  }
  CK(hipDeviceSynchronize());
  std::printf("stream16_ld %zu\nstream4_ld %zu\nstream2_ld %zu\n", bytes, bytes, bytes);
  std::printf("rand4_ld %zu\nrand2_ld %zu\nrand12_ld %zu\n", (size_t)mr * 4, (size_t)mr * 2, (size_t)mr * 12);
  std::printf("stream16_st %zu\nstream4_st %zu\nscat4_st %zu\nscat12_st %zu\npart4_st %zu\n", bytes, bytes,
              (size_t)m * 4, (size_t)m * 12, (size_t)m * 4);
  return 0;
}
