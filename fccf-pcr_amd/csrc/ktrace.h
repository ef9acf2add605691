// ktrace.h — development-only device timestamps of kernel starts.
// `make KTRACE=1` builds an instrumented library into lib_kt/ (-DFCCF_KTRACE); the
// product build compiles KT() to nothing.  Every instrumented kernel records
// (source tag, line, s_memrealtime) for block (0, 0) into one device buffer whose
// word 0 is the shared record counter (tools/ktrace.py prints the timeline).
#pragma once
#ifndef KT_TU
#define KT_TU 0
#endif
#ifdef FCCF_KTRACE
#include <hip/hip_runtime.h>
namespace fccf {
static __device__ unsigned long long* g_kt = nullptr;
void ktrace_register(void (*setter)(unsigned long long*));
namespace {
struct KtReg {
  KtReg() {
    ktrace_register([](unsigned long long* p) { (void)hipMemcpyToSymbol(HIP_SYMBOL(g_kt), &p, sizeof p); });
  }
} kt_reg_;
}  // namespace
}  // namespace fccf
#define KT()                                                                                   \
  do {                                                                                         \
    if (::fccf::g_kt && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) {              \
      const unsigned long long i_ = atomicAdd(::fccf::g_kt, 1ull);                             \
      if (i_ < 8190) {                                                                         \
        ::fccf::g_kt[2 + 2 * i_] = ((unsigned long long)KT_TU << 32) | __LINE__;               \
        ::fccf::g_kt[3 + 2 * i_] = wall_clock64();                                             \
      }                                                                                        \
    }                                                                                          \
  } while (0)
#else
#define KT() ((void)0)
#endif
