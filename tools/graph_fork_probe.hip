// Development probe: does a captured hipGraph with two parallel branches (a fork to a
// second stream and a join back) run the branches concurrently on ROCm?  Each branch
// is one spin kernel of ~100 us on one workgroup; serial replays take ~200 us.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void spin(long long cycles) {
  const long long t0 = wall_clock64();
  while (wall_clock64() - t0 < cycles) {}
}

int main() {
  hipStream_t a, b;
  hipStreamCreateWithFlags(&a, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&b, hipStreamNonBlocking);
  hipEvent_t f, j;
  hipEventCreateWithFlags(&f, hipEventDisableTiming);
  hipEventCreateWithFlags(&j, hipEventDisableTiming);
  const long long cyc = 10000;  // wall_clock64 is 100 MHz: 100 us
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(a, hipStreamCaptureModeThreadLocal);
  hipEventRecord(f, a);
  hipStreamWaitEvent(b, f, 0);
  spin<<<1, 64, 0, a>>>(cyc);
  spin<<<1, 64, 0, b>>>(cyc);
  hipEventRecord(j, b);
  hipStreamWaitEvent(a, j, 0);
  hipError_t e = hipStreamEndCapture(a, &g);
  hipError_t e2 = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  size_t nn = 0;
  hipGraphGetNodes(g, nullptr, &nn);
  printf("capture %d instantiate %d nodes %zu\n", (int)e, (int)e2, nn);
  for (int it = 0; it < 5; ++it) {
    hipDeviceSynchronize();
    const auto t0 = std::chrono::steady_clock::now();
    hipGraphLaunch(ge, a);
    hipStreamSynchronize(a);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    printf("graph fork/join replay: %.1f us\n", us);
  }
  for (int it = 0; it < 3; ++it) {
    hipDeviceSynchronize();
    const auto t0 = std::chrono::steady_clock::now();
    hipEventRecord(f, a);
    hipStreamWaitEvent(b, f, 0);
    spin<<<1, 64, 0, a>>>(cyc);
    spin<<<1, 64, 0, b>>>(cyc);
    hipEventRecord(j, b);
    hipStreamWaitEvent(a, j, 0);
    hipStreamSynchronize(a);
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    printf("eager two streams: %.1f us\n", us);
  }
  return 0;
}
