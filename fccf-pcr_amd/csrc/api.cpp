// api.cpp — C-ABI entry points of libfccf (context, errors, stage exports).
// The registration driver itself lives in pipeline.cpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "ctx.h"
#include "kernels.h"
#include "pipeline.h"

using namespace fccf;

extern "C" void fccf_params_default(fccf_params* p) {
  if (!p) return;
  // FCCF.cpp:126-175
  p->parameter_l1 = 0.5f; p->parameter_l2 = 1.0f; p->parameter_k1 = 5.0f; p->parameter_k2 = 2.0f;
  p->normal_vector_threshold1 = 5.0f; p->normal_vector_threshold2 = 8.0f;
  p->face_voxel_size = 1.0f;
  p->voxel_point_threshold = 5;
  p->curvature_threshold = 0.05f;
  p->select_plane_number = 15;
  p->quick_verify_angel_threshold = 10.0f; p->quick_verify_distance_threshold = 2.0f;
  p->required_optimize_plane = 4.0f;
  p->fine_verify_voxel_size = 0.5f; p->fine_verify_number = 4;
  p->included_angle_same_threshold = 5.0f; p->included_angle_min_threshold = 30.0f;
  p->included_angle_max_threshold = 150.0f;
  p->third_plane_threshold = 0.5f; p->third_plane_normal_threshold = 5.0f;
  p->cluster_number_threshold = 10; p->cluster_angel_threshold = 2.0f; p->cluster_distance_threshold = 0.8f;
  p->seclct_cluster_number = 200;
  p->rough_threshold_gl = 2;
}

extern "C" const char* fccf_strerror(int code) {
  switch (code) {
    case FCCF_OK: return "ok";
    case FCCF_E_ARG: return "invalid argument";
    case FCCF_E_HIP: return "HIP runtime error";
    case FCCF_E_RCCL: return "collective error";
    case FCCF_E_OOM: return "out of memory";
    case FCCF_E_IO: return "I/O error";
    case FCCF_E_INTERNAL: return "internal error";
    case FCCF_E_NODEVICE: return "no usable HIP device";
    default: return "unknown error";
  }
}

extern "C" int fccf_ctx_create(fccf_ctx** out, int device) {
  if (!out) return FCCF_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return FCCF_E_NODEVICE;
  if (device < 0 || device >= n) return FCCF_E_ARG;
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return FCCF_E_HIP;
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return FCCF_E_NODEVICE;  // code objects are gfx950-only
  fccf_ctx* c = new fccf_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) { delete c; return FCCF_E_HIP; }
  bool ok = true;
  for (auto& s : c->sa) ok = ok && hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess;
  ok = ok && hipStreamCreateWithFlags(&c->sb, hipStreamNonBlocking) == hipSuccess;
  for (auto& cs : c->cs)
    for (auto& e : cs.ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  if (!ok) {
    fccf_ctx_destroy(c);
    return FCCF_E_HIP;
  }
  *out = c;
  return FCCF_OK;
}

extern "C" int fccf_ctx_destroy(fccf_ctx* c) {
  if (!c) return FCCF_E_ARG;
  (void)hipSetDevice(c->device);
  (void)hipDeviceSynchronize();
  pipeline_release(c);
  for (auto& cs : c->cs) {
    for (auto& g : cs.g_seg) g.reset();
    cs.g_cen.reset();
    cs.g_rep.reset();
    cs.g_fine.reset();
    for (auto& e : cs.ev)
      if (e) (void)hipEventDestroy(e);
  }
  for (auto& s : c->sa)
    if (s) (void)hipStreamDestroy(s);
  if (c->sb) (void)hipStreamDestroy(c->sb);
  delete c;
  return FCCF_OK;
}

extern "C" int fccf_ctx_set_debug(fccf_ctx* c, int on) {
  if (!c) return FCCF_E_ARG;
  c->debug = on != 0;
  if (!c->debug) c->dbg.clear();
  return FCCF_OK;
}

extern "C" int fccf_ctx_set_probe(fccf_ctx* c, const char* kernel) {
  if (!c) return FCCF_E_ARG;
  c->probe.target = kernel ? kernel : "";
  c->probe.total_ms = c->probe.total_bytes = 0.0;
  c->probe.launches = 0;
  c->probe.armed.clear();
  return FCCF_OK;
}

extern "C" int fccf_probe_read(fccf_ctx* c, double* total_ms, int64_t* launches, double* total_bytes) {
  if (!c || !total_ms || !launches || !total_bytes) return FCCF_E_ARG;
  *total_ms = c->probe.total_ms;
  *launches = c->probe.launches;
  *total_bytes = c->probe.total_bytes;
  return FCCF_OK;
}

extern "C" int fccf_debug_get(fccf_ctx* c, const char* name, void* buf, int64_t cap, int64_t* nbytes) {
  if (!c || !name) return FCCF_E_ARG;
  auto it = c->dbg.find(name);
  if (it == c->dbg.end()) return FCCF_E_ARG;
  const int64_t n = (int64_t)it->second.size();
  if (nbytes) *nbytes = n;
  if (buf && cap > 0) std::memcpy(buf, it->second.data(), (size_t)std::min(n, cap));
  return FCCF_OK;
}

template <class F>
static int guarded(fccf_ctx* c, F&& f) {
  try {
    HIP_CHECK(hipSetDevice(c->device));
    f();
    return FCCF_OK;
  } catch (const Error& e) {
    c->last_error = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    return FCCF_E_OOM;
  } catch (...) {
    return FCCF_E_INTERNAL;
  }
}

extern "C" const char* fccf_ctx_last_error(fccf_ctx* c) { return c ? c->last_error.c_str() : ""; }

namespace {
int stage_downsample(fccf_ctx* c, const float* xyz, int64_t n, float leaf, float* out, int64_t* m, bool presorted) {
  if (!c || (!xyz && n) || !out || !m || n < 0 || n > (int64_t)0x7FFFFFFF || !(leaf > 0.f)) return FCCF_E_ARG;
  return guarded(c, [&] {
    hipStream_t st = c->sb;
    const uint32_t cap = (uint32_t)std::max<int64_t>(n, 1);
    c->arena2.ensure(voxel_grid_bytes(cap) + 12 * (size_t)cap * 2 + (1 << 20));
    c->arena2.reset();
    float* d_in = c->arena2.take_n<float>(3 * (size_t)cap);
    float* d_out = c->arena2.take_n<float>(3 * (size_t)cap);
    uint32_t* d_sc = c->arena2.take_n<uint32_t>(64);
    VGBufs b = voxel_grid_carve(c->arena2, cap);
    uint32_t hn = (uint32_t)n;
    HIP_CHECK(hipMemcpyAsync(d_in, xyz, 12 * (size_t)n, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_sc, &hn, 4, hipMemcpyHostToDevice, st));
    voxel_grid(d_in, d_sc, cap, leaf, d_out, d_sc + 1, b, st, presorted);
    HIP_CHECK(hipGetLastError());
    uint32_t hm = 0;
    HIP_CHECK(hipMemcpyAsync(&hm, d_sc + 1, 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    HIP_CHECK(hipMemcpyAsync(out, d_out, 12 * (size_t)hm, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    *m = hm;
  });
}

}  // namespace

extern "C" int fccf_stage_downsample(fccf_ctx* c, const float* xyz, int64_t n, float leaf, float* out, int64_t* m) {
  return stage_downsample(c, xyz, n, leaf, out, m, false);
}

extern "C" int fccf_stage_downsample_presorted(fccf_ctx* c, const float* xyz, int64_t n, float leaf, float* out,
                                               int64_t* m) {
  return stage_downsample(c, xyz, n, leaf, out, m, true);
}

namespace {
// Shared body of the sum stage exports: S-float elements, K components.
int stage_sum(fccf_ctx* c, const float* x, int64_t n, int S, bool divide, float* out) {
  if (!c || (!x && n) || !out || n < 0 || n > (int64_t)0x7FFFFFFF) return FCCF_E_ARG;
  return guarded(c, [&] {
    hipStream_t st = c->sb;
    const uint32_t cap = (uint32_t)std::max<int64_t>(n, 1);
    c->arena2.ensure(4 * (size_t)S * cap + exact_sum_bytes(S, cap) + (1 << 16));
    c->arena2.reset();
    float* d_in = c->arena2.take_n<float>((size_t)S * cap);
    uint32_t* d_sc = c->arena2.take_n<uint32_t>(64);
    float* d_out = c->arena2.take_n<float>(4);
    XsBufs xs = exact_sum_carve(c->arena2.take(exact_sum_bytes(S, cap)), S, cap);
    uint32_t hn = (uint32_t)n;
    if (n) HIP_CHECK(hipMemcpyAsync(d_in, x, 4 * (size_t)S * n, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_sc, &hn, 4, hipMemcpyHostToDevice, st));
    exact_sum(d_in, S, S, nullptr, d_sc, 1, d_out, divide, xs, st);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(out, d_out, 4 * (size_t)S, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
  });
}
}  // namespace

extern "C" int fccf_stage_centroid(fccf_ctx* c, const float* xyz, int64_t n, float out[4]) {
  if (!out) return FCCF_E_ARG;
  const int rc = stage_sum(c, xyz, n, 3, true, out);
  if (rc == FCCF_OK) out[3] = 1.f;
  return rc;
}

extern "C" int fccf_stage_seqsum(fccf_ctx* c, const float* x, int64_t n, float* out) {
  return stage_sum(c, x, n, 1, false, out);
}

extern "C" int fccf_device_upload(fccf_ctx* c, const float* xyz, int64_t n, float** d) {
  if (!c || !d || (!xyz && n) || n < 0) return FCCF_E_ARG;
  *d = nullptr;
  return guarded(c, [&] {
    float* p = nullptr;
    if (hipMalloc((void**)&p, 12 * (size_t)std::max<int64_t>(n, 1)) != hipSuccess) throw Error(FCCF_E_OOM, "hipMalloc");
    if (n) HIP_CHECK(hipMemcpy(p, xyz, 12 * (size_t)n, hipMemcpyHostToDevice));
    *d = p;
  });
}

extern "C" int fccf_device_free(fccf_ctx* c, float* d) {
  if (!c) return FCCF_E_ARG;
  return guarded(c, [&] {
    if (d) HIP_CHECK(hipFree(d));
  });
}

#ifdef FCCF_KTRACE
// ---------------------------------------------------------------- ktrace (development)
namespace fccf {
static std::vector<void (*)(unsigned long long*)>& kt_setters() {
  static std::vector<void (*)(unsigned long long*)> v;
  return v;
}
void ktrace_register(void (*setter)(unsigned long long*)) { kt_setters().push_back(setter); }
}  // namespace fccf

// Point every instrumented translation unit at buf (device, 16384 u64; word 0 =
// record count, reset here), or detach with NULL.
extern "C" int fccf_ktrace_arm(void* buf) {
  if (buf) (void)hipMemset(buf, 0, 8);
  for (auto f : fccf::kt_setters()) f((unsigned long long*)buf);
  return hipDeviceSynchronize() == hipSuccess ? FCCF_OK : FCCF_E_HIP;
}
#endif
