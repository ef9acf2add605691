// probe.h — per-kernel HIP-event timing for the roofline report (bench.py).
//
// A ctx may name one kernel to probe (fccf_ctx_set_probe).  Candidate kernels are
// launched through FCCF_LAUNCH(...): when the name matches, the launch goes through
// hipExtLaunchKernelGGL with a start and a stop event, which the runtime stamps
// from the kernel's own dispatch (the interval the profiler reports, without the
// queue latency that separate hipEventRecord markers would add).  HIP cannot time
// events inside a captured graph, so while a probe is on the device stages launch
// eagerly (CachedGraph::run).  After the call's streams are synchronised, each pair
// adds (elapsed time, algorithmic bytes) to the ctx totals, and to the totals of its
// launch width: the clouds one batched launch processes (grid.y of the cloud stage's
// kernels, 1..8), so a pipelined batch's eight-cloud launches are reported apart from
// a single registration's two-cloud ones.
#pragma once
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace fccf {

// Algorithmic bytes of one launch: fixed + sum of per[i] * *cnt[i] (device-resident
// unit counts, one term per problem of a batched launch).
struct ProbeBytes {
  static constexpr int MAXT = 32;  // (two terms per cloud at ten clouds per launch)
  const uint32_t* cnt[MAXT] = {};
  double per[MAXT] = {};
  int n = 0;
  double fixed = 0.0;
  ProbeBytes() = default;
  // the classic form: up to four (count, bytes per unit) terms and a fixed part
  ProbeBytes(const uint32_t* c1, double p1, const uint32_t* c2 = nullptr, double p2 = 0.0, double fx = 0.0,
             const uint32_t* c3 = nullptr, double p3 = 0.0, const uint32_t* c4 = nullptr, double p4 = 0.0)
      : fixed(fx) {
    add(c1, p1).add(c2, p2).add(c3, p3).add(c4, p4);
  }
  ProbeBytes& add(const uint32_t* c, double p) {
    if (c && n < MAXT) {
      cnt[n] = c;
      per[n] = p;
      ++n;
    }
    return *this;
  }
};

struct ProbePair {
  hipEvent_t a = nullptr, b = nullptr;  // start / stop of the kernel's dispatch
  uint32_t* d_active = nullptr;         // device word: a kernel may clear it when it skipped its work
  ProbeBytes bytes;
  int width = 1;  // problems (clouds) per launch: grid.y
  ~ProbePair() {
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    if (d_active) (void)hipFree(d_active);
  }
};

struct Probe {
  static constexpr int WMAX = 16;                  // widths 1..WMAX tallied apart
  std::string target;                              // kernel name; empty = off
  std::vector<std::shared_ptr<ProbePair>> armed;   // pairs executed by the current call
  std::vector<std::shared_ptr<ProbePair>> spare;   // reusable pairs
  double total_ms = 0.0, total_bytes = 0.0;
  int64_t launches = 0;
  double w_ms[WMAX + 1] = {}, w_bytes[WMAX + 1] = {};
  int64_t w_launches[WMAX + 1] = {};
  bool on() const { return !target.empty(); }
  void clear_totals() {
    total_ms = total_bytes = 0.0;
    launches = 0;
    for (int w = 0; w <= WMAX; ++w) {
      w_ms[w] = w_bytes[w] = 0.0;
      w_launches[w] = 0;
    }
  }
};

// The probe of the ctx whose call is running on this thread (null outside calls).
extern thread_local Probe* g_probe;

struct ProbeScope {
  std::shared_ptr<ProbePair> p;
  ProbeScope(const char* kernel, hipStream_t st, const ProbeBytes& bytes, int width);
  void end(hipStream_t st);
  // device word the probed kernel may set to 0 when it had nothing to do (the
  // launch is then left out of the totals); null when this launch is not probed
  uint32_t* active() const { return p ? p->d_active : nullptr; }
};

// Resolve armed pairs into totals (call after the streams are synchronised).
void probe_collect(Probe& pr);

}  // namespace fccf

// FCCF_LAUNCH(name, bytes, kernel, grid, block, shmem, stream, args...)
//   -- kernel<<<grid, block, shmem, stream>>>(args...), timed when probed.  bytes is a
// ProbeBytes, or a parenthesised list for its classic constructor:
// (d_count, per_unit[, d_count2, per_unit2, fixed[, d_count3, per_unit3, d_count4, per_unit4]]).
// Arguments may use _probe.active() (null unless this launch is probed).
#define FCCF_LAUNCH(name, bytes, kernel, grid, block, shmem, st, ...)                               \
  do {                                                                                             \
    ::fccf::ProbeScope _probe(name, st, ::fccf::ProbeBytes(FCCF_UNPACK bytes), (int)dim3(grid).y); \
    if (_probe.p)                                                                                  \
      hipExtLaunchKernelGGL(kernel, grid, block, shmem, st, _probe.p->a, _probe.p->b, 0, __VA_ARGS__); \
    else                                                                                           \
      kernel<<<grid, block, shmem, st>>>(__VA_ARGS__);                                             \
    _probe.end(st);                                                                                \
  } while (0)
#define FCCF_UNPACK(...) __VA_ARGS__
