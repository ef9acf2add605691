// Dev: how late a host thread learns that a kernel has finished, by wait form.  A
// one-wave kernel spins for D us (s_memrealtime, 100 MHz), records an event and (form
// "flag") writes a sequence number to pinned host memory; the host waits with
//   sync   hipEventSynchronize
//   query  a hipEventQuery spin
//   flag   a spin on the pinned word (system-scope release store by the kernel)
// and the median of (return time - launch time - D) is the wake overhead.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/wake_probe tools/wake_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

__global__ void k_spin(unsigned long long ticks, unsigned* flag, unsigned seq) {
  if (threadIdx.x != 0) return;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
  if (flag) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main() {
  using clk = std::chrono::steady_clock;
  const double D_us = 200.0;
  const unsigned long long ticks = (unsigned long long)(D_us * 100.0);
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  unsigned* flag = nullptr;
  CK(hipHostMalloc((void**)&flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  *flag = 0;
  const char* names[3] = {"sync", "query", "flag"};
  std::vector<double> res[3];
  unsigned seq = 0;
  for (int rep = 0; rep < 60; ++rep)
    for (int form = 0; form < 3; ++form) {
      ++seq;
      const auto a = clk::now();
      k_spin<<<1, 64, 0, st>>>(ticks, form == 2 ? flag : nullptr, seq);
      CK(hipEventRecord(ev, st));
      if (form == 0) {
        CK(hipEventSynchronize(ev));
      } else if (form == 1) {
        hipError_t q;
        while ((q = hipEventQuery(ev)) == hipErrorNotReady) {
        }
        CK(q);
      } else {
        while (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != seq) {
        }
      }
      const double us = std::chrono::duration<double, std::micro>(clk::now() - a).count();
      if (rep >= 10) res[form].push_back(us - D_us);
      CK(hipStreamSynchronize(st));
    }
  for (int f = 0; f < 3; ++f) {
    std::sort(res[f].begin(), res[f].end());
    std::printf("%-6s wake overhead median %7.2f us  p10 %7.2f  p90 %7.2f\n", names[f], res[f][res[f].size() / 2],
                res[f][res[f].size() / 10], res[f][res[f].size() * 9 / 10]);
  }
  return 0;
}
