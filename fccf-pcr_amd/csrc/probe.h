// probe.h — per-kernel HIP-event timing for the roofline report (bench.py).
//
// A ctx may name one kernel to probe (fccf_ctx_set_probe).  Candidate kernels are
// launched through FCCF_LAUNCH(...): when the name matches, the launch goes through
// hipExtLaunchKernelGGL with a start and a stop event, which the runtime stamps
// from the kernel's own dispatch (the interval the profiler reports, without the
// queue latency that separate hipEventRecord markers would add).  HIP cannot time
// events inside a captured graph, so while a probe is on the device stages launch
// eagerly (CachedGraph::run).  After the call's streams are synchronised, each pair
// adds (elapsed time, algorithmic bytes) to the ctx totals.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace fccf {

struct ProbePair {
  hipEvent_t a = nullptr, b = nullptr;  // start / stop of the kernel's dispatch
  uint32_t* d_active = nullptr;         // device word: a kernel may clear it when it skipped its work
  const uint32_t* d_count = nullptr;   // device-resident unit counts (may be null)
  const uint32_t* d_count2 = nullptr;
  const uint32_t* d_count3 = nullptr;
  const uint32_t* d_count4 = nullptr;
  double per_unit = 0.0, per_unit2 = 0.0, fixed = 0.0, per_unit3 = 0.0, per_unit4 = 0.0;
  ~ProbePair() {
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    if (d_active) (void)hipFree(d_active);
  }
};

struct Probe {
  std::string target;                              // kernel name; empty = off
  std::vector<std::shared_ptr<ProbePair>> armed;   // pairs executed by the current call
  std::vector<std::shared_ptr<ProbePair>> spare;   // reusable pairs
  double total_ms = 0.0, total_bytes = 0.0;
  int64_t launches = 0;
  bool on() const { return !target.empty(); }
};

// The probe of the ctx whose call is running on this thread (null outside calls).
extern thread_local Probe* g_probe;

struct ProbeScope {
  std::shared_ptr<ProbePair> p;
  ProbeScope(const char* kernel, hipStream_t st, const uint32_t* d_count, double per_unit,
             const uint32_t* d_count2 = nullptr, double per_unit2 = 0.0, double fixed = 0.0,
             const uint32_t* d_count3 = nullptr, double per_unit3 = 0.0, const uint32_t* d_count4 = nullptr,
             double per_unit4 = 0.0);
  void end(hipStream_t st);
  // device word the probed kernel may set to 0 when it had nothing to do (the
  // launch is then left out of the totals); null when this launch is not probed
  uint32_t* active() const { return p ? p->d_active : nullptr; }
};

// algorithmic bytes of one launch = per_unit * *d_count + per_unit2 * *d_count2 + fixed
//   (+ per_unit3 * *d_count3 + per_unit4 * *d_count4: the second problem of a batched launch)
// Resolve armed pairs into totals (call after the streams are synchronised).
void probe_collect(Probe& pr);

}  // namespace fccf

// FCCF_LAUNCH(name, (d_count, per_unit[, d_count2, per_unit2, fixed]), kernel, grid, block, shmem, stream,
//             args...)  -- kernel<<<grid, block, shmem, stream>>>(args...), timed when probed.
// Arguments may use _probe.active() (null unless this launch is probed).
#define FCCF_LAUNCH(name, bytes, kernel, grid, block, shmem, st, ...)                               \
  do {                                                                                             \
    ::fccf::ProbeScope _probe(name, st, FCCF_UNPACK bytes);                                        \
    if (_probe.p)                                                                                  \
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, st, _probe.p->a, _probe.p->b, 0, __VA_ARGS__); \
    else                                                                                           \
      kernel<<<grid, block, shmem, st>>>(__VA_ARGS__);                                             \
    _probe.end(st);                                                                                \
  } while (0)
#define FCCF_UNPACK(...) __VA_ARGS__
