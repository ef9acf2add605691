// probe.cpp — see probe.h.
#include "probe.h"

#include <algorithm>

#include "ctx.h"

namespace fccf {

thread_local Probe* g_probe = nullptr;

ProbeScope::ProbeScope(const char* kernel, hipStream_t st, const ProbeBytes& bytes, int width) {
  Probe* pr = g_probe;
  if (!pr || !pr->on() || pr->target != kernel) return;
  if (!pr->spare.empty()) {
    p = pr->spare.back();
    pr->spare.pop_back();
  } else {
    p = std::make_shared<ProbePair>();
    HIP_CHECK(hipEventCreate(&p->a));
    HIP_CHECK(hipEventCreate(&p->b));
    HIP_CHECK(hipMalloc((void**)&p->d_active, 4));
  }
  HIP_CHECK(hipMemsetAsync(p->d_active, 0xFF, 4, st));  // active unless the kernel says otherwise
  p->bytes = bytes;
  p->width = std::max(1, std::min(width, (int)Probe::WMAX));
}

void ProbeScope::end(hipStream_t st) {
  if (!p) return;
  (void)st;
  g_probe->armed.push_back(p);
}

void probe_collect(Probe& pr) {
  for (auto& p : pr.armed) {
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, p->a, p->b));
    uint32_t act = 1;
    HIP_CHECK(hipMemcpy(&act, p->d_active, 4, hipMemcpyDeviceToHost));
    pr.spare.push_back(p);
    if (!act) continue;  // the kernel skipped its work (e.g. a radix pass past the key width)
    double bytes = p->bytes.fixed;
    for (int i = 0; i < p->bytes.n; ++i) {
      uint32_t u = 0;
      HIP_CHECK(hipMemcpy(&u, p->bytes.cnt[i], 4, hipMemcpyDeviceToHost));
      bytes += p->bytes.per[i] * u;
    }
    pr.total_ms += ms;
    pr.total_bytes += bytes;
    ++pr.launches;
    pr.w_ms[p->width] += ms;
    pr.w_bytes[p->width] += bytes;
    ++pr.w_launches[p->width];
  }
  pr.armed.clear();
}

}  // namespace fccf
