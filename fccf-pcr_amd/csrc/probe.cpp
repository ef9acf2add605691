// probe.cpp — see probe.h.
#include "probe.h"

#include "ctx.h"

namespace fccf {

thread_local Probe* g_probe = nullptr;


ProbeScope::ProbeScope(const char* kernel, hipStream_t st, const uint32_t* d_count, double per_unit,
                       const uint32_t* d_count2, double per_unit2, double fixed, const uint32_t* d_count3,
                       double per_unit3, const uint32_t* d_count4, double per_unit4) {
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
  p->d_count = d_count;
  p->d_count2 = d_count2;
  p->per_unit = per_unit;
  p->per_unit2 = per_unit2;
  p->fixed = fixed;
  p->d_count3 = d_count3;
  p->d_count4 = d_count4;
  p->per_unit3 = per_unit3;
  p->per_unit4 = per_unit4;
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
    uint32_t act = 1, u1 = 0, u2 = 0, u3 = 0, u4 = 0;
    HIP_CHECK(hipMemcpy(&act, p->d_active, 4, hipMemcpyDeviceToHost));
    pr.spare.push_back(p);
    if (!act) continue;  // the kernel skipped its work (e.g. a radix pass past the key width)
    if (p->d_count) HIP_CHECK(hipMemcpy(&u1, p->d_count, 4, hipMemcpyDeviceToHost));
    if (p->d_count2) HIP_CHECK(hipMemcpy(&u2, p->d_count2, 4, hipMemcpyDeviceToHost));
    if (p->d_count3) HIP_CHECK(hipMemcpy(&u3, p->d_count3, 4, hipMemcpyDeviceToHost));
    if (p->d_count4) HIP_CHECK(hipMemcpy(&u4, p->d_count4, 4, hipMemcpyDeviceToHost));
    pr.total_ms += ms;
    pr.total_bytes += p->per_unit * u1 + p->per_unit2 * u2 + p->fixed + p->per_unit3 * u3 + p->per_unit4 * u4;
    ++pr.launches;
  }
  pr.armed.clear();
}

}  // namespace fccf
