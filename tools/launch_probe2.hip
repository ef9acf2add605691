// Development probe: what a kernel boundary costs inside a graph on gfx950, as a
// function of grid size and bytes written, and whether two streams' chains of
// dependent kernels overlap.  Prints us per kernel.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty() {}
__global__ void k_write(float* p, unsigned n) {
  for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = (float)i;
}

template <class F>
static double per_kernel(hipStream_t s0, hipStream_t s1, int nk, bool two, F launch) {
  hipGraph_t g;
  hipGraphExec_t ge;
  hipEvent_t f, j;
  hipEventCreateWithFlags(&f, hipEventDisableTiming);
  hipEventCreateWithFlags(&j, hipEventDisableTiming);
  hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal);
  if (two) {
    hipEventRecord(f, s0);
    hipStreamWaitEvent(s1, f, 0);
  }
  for (int i = 0; i < nk; ++i) {
    launch(s0, 0);
    if (two) launch(s1, 1);
  }
  if (two) {
    hipEventRecord(j, s1);
    hipStreamWaitEvent(s0, j, 0);
  }
  hipStreamEndCapture(s0, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s0);
  hipStreamSynchronize(s0);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, s0);
  hipGraphLaunch(ge, s0);
  hipEventRecord(b, s0);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  return ms * 1e3 / nk;
}

int main() {
  hipStream_t s0, s1;
  hipStreamCreateWithFlags(&s0, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  float* buf[2];
  hipMalloc(&buf[0], 64 << 20);
  hipMalloc(&buf[1], 64 << 20);
  const int NK = 100;
  for (int two = 0; two < 2; ++two) {
    printf("%s\n", two ? "two streams (per kernel pair):" : "one stream:");
    for (int blocks : {1, 64, 256, 1024, 4096}) {
      double t = per_kernel(s0, s1, NK, two, [&](hipStream_t s, int) { k_empty<<<blocks, 256, 0, s>>>(); });
      printf("  empty grid %5d x256: %.2f us\n", blocks, t);
    }
    for (unsigned mb : {0u, 1u, 4u, 16u}) {
      const unsigned n = mb ? (mb << 20) / 4 : 1024;
      double t = per_kernel(s0, s1, NK, two, [&](hipStream_t s, int k) { k_write<<<1024, 256, 0, s>>>(buf[k], n); });
      printf("  write %2u MB (1024x256): %.2f us  (%.0f GB/s)\n", mb, t, mb ? (mb << 20) / (t * 1e3) : 0.0);
    }
    for (int blocks : {244, 489}) {
      double t = per_kernel(s0, s1, NK, two, [&](hipStream_t s, int) { k_empty<<<blocks, 1024, 0, s>>>(); });
      printf("  empty grid %5d x1024: %.2f us\n", blocks, t);
    }
  }
  return 0;
}
