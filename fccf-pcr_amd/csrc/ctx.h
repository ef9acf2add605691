// ctx.h — fccf_ctx internals: device, streams, workspace arena, debug store.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstring>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/fccf.h"
#include "pool.h"

namespace fccf {

struct Error : std::runtime_error {
  int code;
  Error(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

#define HIP_CHECK(x)                                                                          \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess)                                                                     \
      throw ::fccf::Error(FCCF_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_));        \
  } while (0)

// Bump allocator over one device allocation; reset per call, grown on demand.
struct Arena {
  char* base = nullptr;
  size_t cap = 0, off = 0, peak = 0;
  void reset() { off = 0; }
  void* take(size_t bytes) {
    size_t a = (off + 255) & ~size_t(255);
    if (a + bytes > cap) throw Error(FCCF_E_INTERNAL, "arena overflow");
    off = a + bytes;
    if (off > peak) peak = off;
    return base + a;
  }
  template <class T>
  T* take_n(size_t n) { return (T*)take(sizeof(T) * (n ? n : 1)); }
  void ensure(size_t bytes) {
    if (bytes <= cap) return;
    if (base) (void)hipFree(base);
    base = nullptr;
    cap = 0;
    if (hipMalloc((void**)&base, bytes) != hipSuccess) throw Error(FCCF_E_OOM, "hipMalloc arena");
    cap = bytes;
  }
  ~Arena() {
    if (base) (void)hipFree(base);
  }
};

struct PinnedBuf {
  void* p = nullptr;
  size_t cap = 0;
  void* get(size_t bytes) {
    if (bytes > cap) {
      if (p) (void)hipHostFree(p);
      p = nullptr;
      if (hipHostMalloc(&p, bytes) != hipSuccess) throw Error(FCCF_E_OOM, "hipHostMalloc");
      cap = bytes;
    }
    return p;
  }
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
};

}  // namespace fccf

struct fccf_ctx {
  int device = 0;
  hipStream_t st[4] = {nullptr, nullptr, nullptr, nullptr};  // [0,1] per-cloud main, [2,3] side
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  fccf::Arena arena;   // per-cloud buffers
  fccf::Arena arena2;  // matching
  fccf::Arena arena3;  // fine verify
  fccf::PinnedBuf pinned;
  fccf::Pool pool;
  bool debug = false;
  std::map<std::string, std::vector<uint8_t>> dbg;
  std::string last_error;

  template <class T>
  void dbg_put(const std::string& k, const T* p, size_t n) {
    if (!debug) return;
    auto& b = dbg[k];
    b.resize(sizeof(T) * n);
    if (n) std::memcpy(b.data(), p, b.size());
  }
  template <class T>
  void dbg_put(const std::string& k, const std::vector<T>& v) { dbg_put(k, v.data(), v.size()); }
};
