// Development probe: per-kernel cost of dependent tiny kernels (stream vs graph)
// and whether independent graph branches execute concurrently.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void tiny(int* p) { if (threadIdx.x == 0) p[blockIdx.x] += 1; }
__global__ void spin(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  int* d;
  hipMalloc(&d, 4096 * 4);
  hipStream_t s0, s1;
  hipStreamCreateWithFlags(&s0, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipEvent_t e0, e1, ef, ej;
  hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventCreateWithFlags(&ef, hipEventDisableTiming); hipEventCreateWithFlags(&ej, hipEventDisableTiming);
  const int N = 200;
  for (int rep = 0; rep < 3; ++rep) {
    // 1. stream launches
    hipDeviceSynchronize();
    double h0 = now_us();
    hipEventRecord(e0, s0);
    for (int i = 0; i < N; ++i) tiny<<<1, 64, 0, s0>>>(d);
    hipEventRecord(e1, s0);
    double h1 = now_us();
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("stream: %d tiny kernels: gpu %.1f us (%.2f us/kernel), host enqueue %.1f us\n", N, ms * 1e3, ms * 1e3 / N, h1 - h0);
    // 2. graph of the same chain
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < N; ++i) tiny<<<1, 64, 0, s0>>>(d);
    hipStreamEndCapture(s0, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s0);
    hipStreamSynchronize(s0);
    h0 = now_us();
    hipEventRecord(e0, s0);
    hipGraphLaunch(ge, s0);
    hipEventRecord(e1, s0);
    h1 = now_us();
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("graph : %d tiny kernels: gpu %.1f us (%.2f us/kernel), host launch %.1f us\n", N, ms * 1e3, ms * 1e3 / N, h1 - h0);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    // 3. two independent branches of 4 x 50 us spins each
    const long long cyc = 50LL * 2100;  // ~50 us at ~2.1 GHz
    hipStreamBeginCapture(s0, hipStreamCaptureModeThreadLocal);
    hipEventRecord(ef, s0);
    hipStreamWaitEvent(s1, ef, 0);
    for (int i = 0; i < 4; ++i) spin<<<1, 64, 0, s0>>>(cyc);
    for (int i = 0; i < 4; ++i) spin<<<1, 64, 0, s1>>>(cyc);
    hipEventRecord(ej, s1);
    hipStreamWaitEvent(s0, ej, 0);
    hipStreamEndCapture(s0, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s0);
    hipStreamSynchronize(s0);
    hipEventRecord(e0, s0);
    hipGraphLaunch(ge, s0);
    hipEventRecord(e1, s0);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("graph branches: 2 x 4 x ~50us spins: %.1f us (serial ~400, concurrent ~200)\n", ms * 1e3);
    hipGraphExecDestroy(ge);
    hipGraphDestroy(g);
    // 4. same two branches as plain streams
    hipEventRecord(e0, s0);
    hipEventRecord(ef, s0);
    hipStreamWaitEvent(s1, ef, 0);
    for (int i = 0; i < 4; ++i) spin<<<1, 64, 0, s0>>>(cyc);
    for (int i = 0; i < 4; ++i) spin<<<1, 64, 0, s1>>>(cyc);
    hipEventRecord(ej, s1);
    hipStreamWaitEvent(s0, ej, 0);
    hipEventRecord(e1, s0);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("streams branches: %.1f us\n", ms * 1e3);
  }
  return 0;
}
