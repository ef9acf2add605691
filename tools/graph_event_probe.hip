// Development probe: do timing events recorded inside a captured hipGraph give
// per-replay kernel durations (hipEventElapsedTime after each launch)?
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void spin(long long cycles) {
  const long long t0 = clock64();
  while (clock64() - t0 < cycles) {}
}

int main() {
  hipStream_t s;
  hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t a, b, o0, o1;
  hipEventCreate(&a); hipEventCreate(&b); hipEventCreate(&o0); hipEventCreate(&o1);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipError_t e1 = hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
  spin<<<1, 64, 0, s>>>(20000);
  hipError_t e2 = hipEventRecord(a, s);
  spin<<<1, 64, 0, s>>>(200000);  // the "probed" kernel
  hipError_t e3 = hipEventRecord(b, s);
  spin<<<1, 64, 0, s>>>(20000);
  hipError_t e4 = hipStreamEndCapture(s, &g);
  hipError_t e5 = hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  printf("capture %d record %d %d end %d inst %d\n", e1, e2, e3, e4, e5);
  for (int it = 0; it < 4; ++it) {
    hipEventRecord(o0, s);
    hipGraphLaunch(ge, s);
    hipEventRecord(o1, s);
    hipStreamSynchronize(s);
    float ms_in = -1, ms_out = -1;
    hipError_t r1 = hipEventElapsedTime(&ms_in, a, b);
    hipEventElapsedTime(&ms_out, o0, o1);
    printf("replay %d: inner %.2f us (rc %d), whole graph %.2f us\n", it, ms_in * 1e3, r1, ms_out * 1e3);
  }
  return 0;
}
