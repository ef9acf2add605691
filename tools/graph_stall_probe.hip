// Development probe: device-side timestamps (s_memrealtime, 100 MHz) of every
// kernel in a graph of N dependent kernels, to locate stalls between graph nodes
// without a profiler.  Each kernel reads and writes a word the previous one wrote.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void k_step(unsigned long long* ts, int i, unsigned* chain, unsigned n) {
  const unsigned long long t0 = wall_clock64();
  __shared__ unsigned v;
  if (threadIdx.x == 0) v = chain[0];
  __syncthreads();
  for (unsigned j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) chain[1 + j] = v + j;
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    chain[0] = v + 1;
    ts[2 * i] = t0;
    ts[2 * i + 1] = wall_clock64();
  }
}

struct Big {
  unsigned* p[48];
};
template <int K>
__global__ void k_stepv(unsigned long long* ts, int i, unsigned* chain, unsigned n, Big big) {
  const unsigned long long t0 = wall_clock64();
  __shared__ unsigned v;
  if (threadIdx.x == 0) v = chain[0] + (big.p[K] ? 0u : 1u);
  __syncthreads();
  for (unsigned j = blockIdx.x * blockDim.x + threadIdx.x; j < n; j += gridDim.x * blockDim.x) chain[1 + j] = v + j * K;
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    chain[0] = v + 1;
    ts[2 * i] = t0;
    ts[2 * i + 1] = wall_clock64();
  }
}

int main(int argc, char** argv) {
  const int N = argc > 1 ? atoi(argv[1]) : 48;
  const int blocks = argc > 2 ? atoi(argv[2]) : 64;
  const unsigned n = argc > 3 ? (unsigned)atoi(argv[3]) : 65536;
  unsigned long long* ts;
  unsigned* chain;
  hipMalloc(&ts, 16 * N);
  hipMalloc(&chain, 4 * (n + 1));
  hipMemset(chain, 0, 4 * (n + 1));
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  const int mode = argc > 4 ? atoi(argv[4]) : 0;
  Big big{};
  for (int i = 0; i < N; ++i) {
    if (mode == 0) k_step<<<blocks, 256, 0, s>>>(ts, i, chain, n);
    else if (i % 4 == 0) k_stepv<0><<<blocks, 256, 0, s>>>(ts, i, chain, n, big);
    else if (i % 4 == 1) k_stepv<1><<<blocks, 256, 0, s>>>(ts, i, chain, n, big);
    else if (i % 4 == 2) k_stepv<2><<<blocks, 256, 0, s>>>(ts, i, chain, n, big);
    else k_stepv<3><<<blocks, 256, 0, s>>>(ts, i, chain, n, big);
  }
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int rep = 0; rep < 3; ++rep) {
    hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
  }
  unsigned long long h[2 * 512];
  hipMemcpy(h, ts, 16 * N, hipMemcpyDeviceToHost);
  printf("N %d blocks %d n %u: start-to-start / duration (us)\n", N, blocks, n);
  for (int i = 0; i < N; ++i)
    printf("%3d %7.2f %6.2f%s", i, i ? (h[2 * i] - h[2 * i - 2]) / 100.0 : 0.0, (h[2 * i + 1] - h[2 * i]) / 100.0,
           (i % 6 == 5) ? "\n" : " |");
  printf("\ntotal %.1f us\n", (h[2 * N - 1] - h[0]) / 100.0);
  return 0;
}
