#include <chrono>
// api.cpp — C-ABI entry points of libfccf (context, errors, stage exports).
// The registration driver itself lives in pipeline.cpp.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <vector>
#include <atomic>
#include <thread>

#include "ctx.h"
#include "group.h"
#include "host_stages.h"
#include "kernels.h"
#include "match.h"
#include "mail.h"
#include "pipeline.h"

using namespace fccf;

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
  ok = ok && hipMalloc((void**)&c->d_flags, 256) == hipSuccess && hipMemset(c->d_flags, 0, 256) == hipSuccess;
  for (auto& e : c->ev_match) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
  for (auto& cs : c->cs) {
    for (auto& e : cs.ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    for (auto& e : cs.tev) ok = ok && hipEventCreate(&e) == hipSuccess;
    ok = ok && hipEventCreate(&cs.ev_in0) == hipSuccess && hipEventCreate(&cs.ev_in) == hipSuccess;
  }
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
  (void)device_sync_guarded();
  // a group still attached is detached, not destroyed: its handle stays the caller's,
  // and fccf_group_destroy then only releases the communicator
  if (c->group) {
    c->group->ctx = nullptr;
    c->group = nullptr;
  }
  pipeline_release(c);
  for (auto& cs : c->cs) {
    for (auto& g : cs.g_seg) g.reset();
    cs.g_fine.reset();
    for (auto& e : cs.ev)
      if (e) (void)hipEventDestroy(e);
    for (auto& e : cs.tev)
      if (e) (void)hipEventDestroy(e);
    if (cs.ev_in) (void)hipEventDestroy(cs.ev_in);
    if (cs.ev_in0) (void)hipEventDestroy(cs.ev_in0);
  }
  for (auto& s : c->sa)
    if (s) (void)hipStreamDestroy(s);
  if (c->sb) (void)hipStreamDestroy(c->sb);
  if (c->d_flags) (void)hipFree(c->d_flags);
  for (auto& e : c->ev_match)
    if (e) (void)hipEventDestroy(e);
  delete c;
  return FCCF_OK;
}

extern "C" int fccf_ctx_set_grow_device(fccf_ctx* c, int on) {
  if (!c) return FCCF_E_ARG;
  c->grow_device = on != 0;
  return FCCF_OK;
}

extern "C" int fccf_ctx_set_lm_device(fccf_ctx* c, int on) {
  if (!c) return FCCF_E_ARG;
  c->lm_device = on != 0;
  return FCCF_OK;
}

extern "C" int fccf_ctx_set_cluster_device(fccf_ctx* c, int on) {
  if (!c) return FCCF_E_ARG;
  c->cluster_device = on != 0;
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
  c->probe.clear_totals();
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

extern "C" int fccf_probe_read_widths(fccf_ctx* c, int max_width, double* ms, int64_t* launches, double* bytes) {
  if (!c || max_width < 1 || !ms || !launches || !bytes) return FCCF_E_ARG;
  for (int w = 1; w <= max_width; ++w) {
    const bool in = w <= fccf::Probe::WMAX;
    ms[w - 1] = in ? c->probe.w_ms[w] : 0.0;
    launches[w - 1] = in ? c->probe.w_launches[w] : 0;
    bytes[w - 1] = in ? c->probe.w_bytes[w] : 0.0;
  }
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

// The host-only stage exports (grow + selection + select_base, transform_cluster,
// fusion): the product's host code, which needs no device, so ctx may be null there
// (then no device form is selectable and no error message is kept).
template <class F>
static int host_guarded(fccf_ctx* c, F&& f) {
  if (c) return guarded(c, f);
  try {
    f();
    return FCCF_OK;
  } catch (const Error& e) {
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
    b.is.stats = 1;  // path counters for fccf_debug_sort_stats
    b.is.inject = c->d_flags;
    uint32_t hn = (uint32_t)n;
    HIP_CHECK(hipMemcpyAsync(d_in, xyz, 12 * (size_t)n, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_sc, &hn, 4, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemsetAsync(&b.params->sort_err, 0, 4, st));  // (a presorted pass alone does not clear it)
    voxel_grid(d_in, d_sc, cap, leaf, d_out, d_sc + 1, b, st, presorted);
    HIP_CHECK(hipGetLastError());
    uint32_t hm = 0, err = 0;
    HIP_CHECK(hipMemcpyAsync(&hm, d_sc + 1, 4, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(&err, &b.params->sort_err, 4, hipMemcpyDeviceToHost, st));
    // the first pass's sort path counters, for fccf_debug_sort_stats (the presorted pass
    // leaves them untouched unless it sorts)
    HIP_CHECK(hipMemcpyAsync(c->sort_stats, b.is.ctl, sizeof c->sort_stats, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (err) throw Error(FCCF_E_INTERNAL, "VoxelGrid: K1 sort invariant violated (flags " + std::to_string(err) + ")");
    HIP_CHECK(hipMemcpyAsync(out, d_out, 12 * (size_t)hm, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    *m = hm;
  });
}

}  // namespace

extern "C" int fccf_stage_downsample(fccf_ctx* c, const float* xyz, int64_t n, float leaf, float* out, int64_t* m) {
  return stage_downsample(c, xyz, n, leaf, out, m, false);
}

namespace {
__global__ void k_sortkeys_params(const uint32_t* keys, const uint32_t* d_n, VGParams* P) {
  __shared__ uint32_t cnt;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  uint32_t c = 0;
  for (uint32_t i = threadIdx.x; i < *d_n; i += blockDim.x) c += keys[i] != 0xFFFFFFFFu ? 1u : 0u;
  atomicAdd(&cnt, c);
  __syncthreads();
  if (threadIdx.x == 0) {
    P->overflow = 0;
    P->nfinite = cnt;
    P->unsorted = 1;
  }
}
}  // namespace

extern "C" int fccf_debug_sort_keys(fccf_ctx* c, const uint32_t* keys, int64_t n, int exact_gate, uint32_t* perm) {
  if (!c || (!keys && n) || (!perm && n) || n < 0 || n > (int64_t)0x7FFFFFFF) return FCCF_E_ARG;
  return guarded(c, [&] {
    hipStream_t st = c->sb;
    const uint32_t cap = (uint32_t)std::max<int64_t>(n, 1);
    c->arena2.ensure(voxel_grid_bytes(cap) + (1 << 20));
    c->arena2.reset();
    uint32_t* d_sc = c->arena2.take_n<uint32_t>(64);
    VGBufs b = voxel_grid_carve(c->arena2, cap);
    b.is.stats = 1;  // path counters for fccf_debug_sort_stats
    b.is.inject = c->d_flags;
    uint32_t hn = (uint32_t)n;
    HIP_CHECK(hipMemcpyAsync(d_sc, &hn, 4, hipMemcpyHostToDevice, st));
    if (n) HIP_CHECK(hipMemcpyAsync(b.k0, keys, 4 * (size_t)n, hipMemcpyHostToDevice, st));
    std::vector<uint32_t> iota((size_t)n);
    for (uint32_t i = 0; i < (uint32_t)n; ++i) iota[i] = i;
    if (n) HIP_CHECK(hipMemcpyAsync(b.v0, iota.data(), 4 * (size_t)n, hipMemcpyHostToDevice, st));
    k_sortkeys_params<<<1, 1024, 0, st>>>(b.k0, d_sc, b.params);
    // FCCF_IS_TRACE_OUT=<path> (dev): per block item / wave task timestamps (IsBufs::trace)
    static const char* tpath = std::getenv("FCCF_IS_TRACE_OUT");
    unsigned long long* dtr = nullptr;
    if (tpath) {
      HIP_CHECK(hipMalloc((void**)&dtr, 64 * (size_t)b.is.taskmax));
      HIP_CHECK(hipMemsetAsync(dtr, 0, 64 * (size_t)b.is.taskmax, st));
      b.is.trace = dtr;
    }
    // FCCF_SHARD_D_SIM=<r>/<N> (dev, row D): sort as rank r of N would -- its range only,
    // no gather (sort_stats[28..29] = the range); the other positions are left unsorted
    if (const char* sim = std::getenv("FCCF_SHARD_D_SIM")) {
      int r = 0, nr = 1;
      if (std::sscanf(sim, "%d/%d", &r, &nr) == 2 && nr > 1 && nr <= IS_SHARD_MAX && r >= 0 && r < nr) {
        b.is.shard_n = (uint32_t)nr;
        b.is.shard_rank = (uint32_t)r;
        b.is.shard_r0 = (uint32_t)shard_sort_r0(nr);
      }
    }
    const auto tsort = std::chrono::steady_clock::now();
    uint32_t sort_ns = 0;
    struct Ev {  // device time of the sort alone (sort_stats[31], ns); destroyed on every path
      hipEvent_t e = nullptr;
      ~Ev() {
        if (e) (void)hipEventDestroy(e);
      }
    } e0, e1;
    HIP_CHECK(hipEventCreate(&e0.e));
    HIP_CHECK(hipEventCreate(&e1.e));
    hipEvent_t ev0 = e0.e, ev1 = e1.e;
    HIP_CHECK(hipEventRecord(ev0, st));
    introsort_u32(b.k0, b.v0, b.k1, b.v1, B4<const uint32_t*>(d_sc), B4<const VGParams*>(b.params), cap, b.is, st, 1,
                  exact_gate != 0);
    HIP_CHECK(hipEventRecord(ev1, st));
    if (tpath) {
      std::vector<unsigned long long> h(8 * (size_t)b.is.taskmax);
      uint32_t ctl[32];
      HIP_CHECK(hipMemcpyAsync(h.data(), dtr, 64 * (size_t)b.is.taskmax, hipMemcpyDeviceToHost, st));
      HIP_CHECK(hipMemcpyAsync(ctl, b.is.ctl, sizeof ctl, hipMemcpyDeviceToHost, st));
      HIP_CHECK(hipStreamSynchronize(st));
      (void)tsort;
      if (FILE* f = std::fopen(tpath, "w")) {
        std::fprintf(f, "kind start end size who\n");
        for (uint32_t i = 0; i < std::min(ctl[24], b.is.taskmax); ++i)
          std::fprintf(f, "B %llu %llu %llu %llu\n", h[4 * i], h[4 * i + 1], h[4 * i + 2], h[4 * i + 3]);
        for (uint32_t i = 0; i < std::min(ctl[25], b.is.taskmax); ++i) {
          const unsigned long long* r = &h[4 * ((size_t)b.is.taskmax + i)];
          std::fprintf(f, "W %llu %llu %llu %llu\n", r[0], r[1], r[2], r[3]);
        }
        std::fclose(f);
      }
      (void)hipFree(dtr);
    }
    HIP_CHECK(hipGetLastError());
    if (n) HIP_CHECK(hipMemcpyAsync(perm, b.v0, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(c->sort_stats, b.is.ctl, sizeof c->sort_stats, hipMemcpyDeviceToHost, st));
    static_assert(sizeof c->sort_rounds == sizeof(IsRound) * IS_RMAX, "sort_rounds size");
    HIP_CHECK(hipMemcpyAsync(c->sort_rounds, b.is.rounds, sizeof c->sort_rounds, hipMemcpyDeviceToHost, st));
    {
      float ms = 0.f;
      HIP_CHECK(hipEventSynchronize(ev1));
      HIP_CHECK(hipEventElapsedTime(&ms, ev0, ev1));
      sort_ns = (uint32_t)std::min(4.0e9, (double)ms * 1e6);
    }
    HIP_CHECK(hipStreamSynchronize(st));
    c->sort_stats[31] = sort_ns;
    if (c->sort_stats[2] & IS_FAULT_MASK)
      throw Error(FCCF_E_INTERNAL, "K1 sort invariant violated (flags " + std::to_string(c->sort_stats[2]) + ")");
  });
}

namespace {
// the batched form's per-copy parameters (blockIdx.y = copy), and the point source the
// finish kernels gather sorted points from (null: no sorted points)
__global__ void k_sortkeys_params_batch(B4<const uint32_t*> keys2, B4<const uint32_t*> d_n2, B4<VGParams*> P2,
                                        const float* pts) {
  __shared__ uint32_t cnt;
  const int e = blockIdx.y;
  if (threadIdx.x == 0) cnt = 0;
  __syncthreads();
  uint32_t c = 0;
  const uint32_t* keys = keys2[e];
  for (uint32_t i = threadIdx.x; i < *d_n2[e]; i += blockDim.x) c += keys[i] != 0xFFFFFFFFu ? 1u : 0u;
  atomicAdd(&cnt, c);
  __syncthreads();
  if (threadIdx.x == 0) {
    VGParams* P = P2[e];
    P->overflow = 0;
    P->nfinite = cnt;
    P->unsorted = 1;
    P->src = pts;
  }
}
}  // namespace

// Dev / tests: K1's sort of `copies` copies of the same keys in one batched launch
// sequence (grid y = copies, as a pipelined stage group runs it), optionally writing the
// sorted points of xyz as VoxelGrid's first pass does.  perm: copy 0's order;
// dev_ms: the device span of the whole sort.
extern "C" int fccf_debug_sort_keys_batch(fccf_ctx* c, const uint32_t* keys, int64_t n, int copies, const float* xyz,
                                          uint32_t* perm, double* dev_ms) {
  if (!c || !keys || !perm || n < 1 || n > (int64_t)0x7FFFFFFF || copies < 1 || copies > BMAX) return FCCF_E_ARG;
  return guarded(c, [&] {
    hipStream_t st = c->sb;
    const uint32_t cap = (uint32_t)n;
    c->arena2.ensure((size_t)copies * (voxel_grid_bytes(cap) + 4096) + 12 * (size_t)n + (1 << 20));
    c->arena2.reset();
    VGBufs b[BMAX];
    uint32_t* d_sc[BMAX];
    for (int e = 0; e < copies; ++e) {
      d_sc[e] = c->arena2.take_n<uint32_t>(64);
      b[e] = voxel_grid_carve(c->arena2, cap);
    }
    float* pts = xyz ? c->arena2.take_n<float>(3 * (size_t)n) : nullptr;
    if (pts) HIP_CHECK(hipMemcpyAsync(pts, xyz, 12 * (size_t)n, hipMemcpyHostToDevice, st));
    std::vector<uint32_t> iota((size_t)n);
    for (uint32_t i = 0; i < (uint32_t)n; ++i) iota[i] = i;
    const uint32_t hn = (uint32_t)n;
    for (int e = 0; e < copies; ++e) {
      HIP_CHECK(hipMemcpyAsync(d_sc[e], &hn, 4, hipMemcpyHostToDevice, st));
      HIP_CHECK(hipMemcpyAsync(b[e].k0, keys, 4 * (size_t)n, hipMemcpyHostToDevice, st));
      HIP_CHECK(hipMemcpyAsync(b[e].v0, iota.data(), 4 * (size_t)n, hipMemcpyHostToDevice, st));
      b[e].is.xyzs = pts ? b[e].xyzs : nullptr;
    }
    auto all = [&](auto f) {
      using T = decltype(f(b[0]));
      T a[BMAX];
      for (int e = 0; e < copies; ++e) a[e] = f(b[e]);
      return B4<T>(a, copies);
    };
    k_sortkeys_params_batch<<<dim3(1, copies), 1024, 0, st>>>(all([](const VGBufs& x) { return (const uint32_t*)x.k0; }),
                                                              B4<const uint32_t*>((const uint32_t* const*)d_sc, copies),
                                                              all([](const VGBufs& x) { return x.params; }), pts);
    struct Ev {
      hipEvent_t e = nullptr;
      ~Ev() {
        if (e) (void)hipEventDestroy(e);
      }
    } e0, e1;
    HIP_CHECK(hipEventCreate(&e0.e));
    HIP_CHECK(hipEventCreate(&e1.e));
    HIP_CHECK(hipEventRecord(e0.e, st));
    introsort_u32(all([](const VGBufs& x) { return x.k0; }), all([](const VGBufs& x) { return x.v0; }),
                  all([](const VGBufs& x) { return x.k1; }), all([](const VGBufs& x) { return x.v1; }),
                  B4<const uint32_t*>((const uint32_t* const*)d_sc, copies),
                  all([](const VGBufs& x) { return (const VGParams*)x.params; }), cap,
                  all([](const VGBufs& x) { return x.is; }), st, copies, false);
    HIP_CHECK(hipEventRecord(e1.e, st));
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(perm, b[0].v0, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
    uint32_t ctl[BMAX][4];
    for (int e = 0; e < copies; ++e) HIP_CHECK(hipMemcpyAsync(ctl[e], b[e].is.ctl, 16, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    float ms = 0.f;
    HIP_CHECK(hipEventElapsedTime(&ms, e0.e, e1.e));
    if (dev_ms) *dev_ms = ms;
    for (int e = 0; e < copies; ++e)
      if (ctl[e][2] & IS_FAULT_MASK)
        throw Error(FCCF_E_INTERNAL, "K1 sort invariant violated (flags " + std::to_string(ctl[e][2]) + ")");
  });
}

extern "C" int fccf_debug_graph_mismatch(fccf_ctx* c) {
  if (!c) return FCCF_E_ARG;
  c->graph_mismatch = true;
  return FCCF_OK;
}

extern "C" int fccf_debug_inject_sort_fault(fccf_ctx* c, uint32_t bits) {
  if (!c || (bits & ~(IS_FAULT_MASK | VG_FORCE_REDO | VG_FORCE_REDO_LATER | IS_POISON_XYZS))) return FCCF_E_ARG;
  return guarded(c, [&] {
    HIP_CHECK(device_sync_guarded());  // no sort of this ctx in flight reads the word meanwhile
    HIP_CHECK(hipMemcpy(c->d_flags, &bits, 4, hipMemcpyHostToDevice));
  });
}

// Forces the interleaving behind the pipelined batch's capture lock (ctx.h
// capture_mutex): this thread captures a graph on stream X and, inside the
// capture, releases a second thread that waits on an event last recorded on X
// (as the batch's helper thread waits on ev[3]/ev[5]); the capture then holds
// for hold_ms.  guard = 1 waits through guarded_stream_wait (the product path),
// guard = 0 calls hipStreamWaitEvent directly (the pre-fix code).
// out[0] = ms the waiting thread spent in its wait call, out[1] = ms between the
// release and the end of the capture, out[2] = the wait's FCCF error (0 = ok),
// out[3] = 1 if the wait returned only after the capture had ended.
extern "C" int fccf_debug_capture_race(fccf_ctx* c, int hold_ms, int guard, double out[4]) {
  if (!c || !out || hold_ms < 0 || hold_ms > 10000) return FCCF_E_ARG;
  return guarded(c, [&] {
    using clk = std::chrono::steady_clock;
    hipStream_t X = nullptr, Y = nullptr;
    hipEvent_t E = nullptr;
    void* buf = nullptr;
    HIP_CHECK(hipStreamCreateWithFlags(&X, hipStreamNonBlocking));
    HIP_CHECK(hipStreamCreateWithFlags(&Y, hipStreamNonBlocking));
    HIP_CHECK(hipEventCreateWithFlags(&E, hipEventDisableTiming));
    HIP_CHECK(hipMalloc(&buf, 256));
    HIP_CHECK(hipEventRecord(E, X));
    HIP_CHECK(hipStreamSynchronize(X));
    std::atomic<int> released{0};
    std::atomic<int64_t> t_released{0}, t_cap_end{0};
    clk::time_point w0, w1;
    int werr = 0;
    std::thread waiter([&] {
      while (!released.load()) std::this_thread::yield();
      w0 = clk::now();
      try {
        if (guard) guarded_stream_wait(Y, E);
        else HIP_CHECK(hipStreamWaitEvent(Y, E, 0));
      } catch (const Error& e) {
        werr = e.code;
      }
      w1 = clk::now();
    });
    const auto base = clk::now();
    CachedGraph g;
    const uint8_t key = 1;
    try {
      g.run(&key, 1, X, [&] {
        HIP_CHECK(hipMemsetAsync(buf, 0, 256, X));
        t_released = (clk::now() - base).count();
        released = 1;
        std::this_thread::sleep_for(std::chrono::milliseconds(hold_ms));
        HIP_CHECK(hipMemsetAsync(buf, 1, 256, X));
        t_cap_end = (clk::now() - base).count();
      });
    } catch (...) {
      released = 1;
      waiter.join();
      throw;
    }
    waiter.join();
    HIP_CHECK(hipStreamSynchronize(X));
    (void)hipStreamSynchronize(Y);
    auto ms = [](clk::duration d) { return std::chrono::duration<double, std::milli>(d).count(); };
    out[0] = ms(w1 - w0);
    out[1] = ms(clk::duration(t_cap_end.load() - t_released.load()));
    out[2] = werr;
    out[3] = (w1 - base).count() >= t_cap_end.load() ? 1.0 : 0.0;
    (void)hipFree(buf);
    (void)hipEventDestroy(E);
    (void)hipStreamDestroy(Y);
    (void)hipStreamDestroy(X);
  });
}

extern "C" int fccf_debug_sort_stats(fccf_ctx* c, uint32_t out[32]) {
  if (!c || !out) return FCCF_E_ARG;
  std::memcpy(out, c->sort_stats, sizeof c->sort_stats);
  return FCCF_OK;
}

extern "C" int fccf_debug_sort_rounds(fccf_ctx* c, uint32_t out[96]) {
  if (!c || !out) return FCCF_E_ARG;
  std::memcpy(out, c->sort_rounds, sizeof c->sort_rounds);
  return FCCF_OK;
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

static_assert(sizeof(fccf_voxel) == sizeof(VoxRec) && sizeof(fccf_plane) == sizeof(Plane) &&
                  sizeof(fccf_base) == sizeof(Base), "record layouts");

// K2/K3 of one cloud (facefit.hip), as the pipeline runs them for each cloud of a pair.
extern "C" int fccf_stage_voxel_planes(fccf_ctx* c, const float* xyz, int64_t n, const fccf_params* params,
                                       fccf_voxel* planar, int64_t cap_planar, int64_t* n_planar, float* resid,
                                       int64_t cap_resid, int64_t* n_resid, float centroid[4]) {
  if (!c || (!xyz && n) || n < 0 || n > (int64_t)0x7FFFFFFF || !n_planar || !n_resid || cap_planar < 0 ||
      cap_resid < 0 || (cap_planar && !planar) || (cap_resid && !resid))
    return FCCF_E_ARG;
  fccf_params P;
  if (params) P = *params;
  else fccf_params_default(&P);
  if (n == 0) {  // no leaves: nothing to launch (compute3DCentroid of an empty cloud: zeros)
    *n_planar = *n_resid = 0;
    if (centroid) centroid[0] = centroid[1] = centroid[2] = 0.f, centroid[3] = 1.f;
    return FCCF_OK;
  }
  return guarded(c, [&] {
    hipStream_t st = c->sb;
    const uint32_t cap = (uint32_t)std::max<int64_t>(n, 1);
    c->arena2.ensure(12 * (size_t)cap * 2 + sizeof(VoxRec) * (size_t)cap + face_bufs_bytes(cap) +
                     exact_sum_bytes(3, cap) + (1 << 16));
    c->arena2.reset();
    float* d_in = c->arena2.take_n<float>(3 * (size_t)cap);
    float* d_res = c->arena2.take_n<float>(3 * (size_t)cap);
    VoxRec* d_pl = c->arena2.take_n<VoxRec>(cap);
    uint32_t* d_n = c->arena2.take_n<uint32_t>(16);
    float* d_cen = c->arena2.take_n<float>(4);
    XsBufs xs = exact_sum_carve(c->arena2.take(exact_sum_bytes(3, cap)), 3, cap);
    FaceBufs fb = face_bufs_carve(c->arena2, cap);
    fb.centroid = d_cen;
    const uint32_t hn = (uint32_t)n;
    if (n) HIP_CHECK(hipMemcpyAsync(d_in, xyz, 12 * (size_t)n, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d_n, &hn, 4, hipMemcpyHostToDevice, st));
    exact_sum(d_in, 3, 3, nullptr, d_n, 1, d_cen, true, xs, st);  // compute3DCentroid (:473)
    face_voxels_prepare(B4<const float*>(d_in), B4<const uint32_t*>(d_n), cap, (double)P.face_voxel_size,
                        B4<FaceBufs>(fb), st, 1);
    face_voxels_fit(B4<const uint32_t*>(d_n), cap, P.voxel_point_threshold, P.curvature_threshold, B4<float*>(d_res),
                    B4<FaceBufs>(fb), st, 1);
    face_voxels_orient(cap, B4<VoxRec*>(d_pl), B4<FaceBufs>(fb), st, 1);
    HIP_CHECK(hipGetLastError());
    uint32_t sc[4] = {0, 0, 0, 0};
    float cen[3] = {0.f, 0.f, 0.f};
    HIP_CHECK(hipMemcpyAsync(sc, fb.nleaf, 16, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(cen, d_cen, 12, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    *n_planar = n ? sc[2] : 0;
    *n_resid = n ? sc[3] : 0;
    const int64_t np = std::min(*n_planar, cap_planar), nr = std::min(*n_resid, cap_resid);
    if (np > 0) HIP_CHECK(hipMemcpyAsync(planar, d_pl, sizeof(VoxRec) * np, hipMemcpyDeviceToHost, st));
    if (nr > 0) HIP_CHECK(hipMemcpyAsync(resid, d_res, 12 * nr, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (centroid) {
      std::memcpy(centroid, cen, 12);
      centroid[3] = 1.f;
    }
  });
}

// Host stages (host_stages.cpp), exactly as the pipeline runs them per cloud.
extern "C" int fccf_stage_grow(fccf_ctx* c, const fccf_voxel* vox, int64_t nv, int side, const fccf_params* params,
                               fccf_plane* planes, int cap_planes, int* n_planes, double* theta, fccf_base* bases,
                               int cap_bases, int* n_bases) {
  if ((!vox && nv) || nv < 0 || nv > (int64_t)0x7FFFFFFF || (side != 1 && side != 2) || !n_planes ||
      !n_bases || cap_planes < 0 || cap_bases < 0 || (cap_planes && !planes) || (cap_bases && !bases))
    return FCCF_E_ARG;
  fccf_params P;
  if (params) P = *params;
  else fccf_params_default(&P);
  return host_guarded(c, [&] {
    std::vector<VoxRec> v((size_t)nv);
    if (nv) std::memcpy(v.data(), vox, sizeof(VoxRec) * (size_t)nv);
    GrowOut g;
    if (c && c->grow_device && nv <= (int64_t)GROW_CAP) {  // K4 on the device (grow.hip)
      hipStream_t st = c->sb;
      VoxRec* d = nullptr;
      if (hipMalloc((void**)&d, sizeof(VoxRec) * (size_t)std::max<int64_t>(nv, 1)) != hipSuccess)
        throw Error(FCCF_E_OOM, "hipMalloc");
      try {
        if (nv) HIP_CHECK(hipMemcpyAsync(d, v.data(), sizeof(VoxRec) * (size_t)nv, hipMemcpyHostToDevice, st));
        const VoxRec* dv[2] = {d, d};
        const uint32_t n2[2] = {(uint32_t)nv, 0u};
        std::vector<GroupOut> gg[2];
        grow_groups_device(c, dv, n2, P, st, gg);
        g = select_groups(gg[0], v.data(), P);
      } catch (...) {
        (void)hipFree(d);
        throw;
      }
      HIP_CHECK(hipFree(d));
    } else {
      g = grow_and_select(v.data(), (int)nv, P);
    }
    const std::vector<Base> b = select_base(g.planes, g.theta, P, side);
    *n_planes = (int)g.planes.size();
    *n_bases = (int)b.size();
    const int np = std::min(*n_planes, cap_planes), nb = std::min(*n_bases, cap_bases);
    if (np > 0) std::memcpy(planes, g.planes.data(), sizeof(Plane) * np);
    if (np > 0 && theta) std::memcpy(theta, g.theta.data(), sizeof(double) * np);
    if (nb > 0) std::memcpy(bases, b.data(), sizeof(Base) * nb);
  });
}

static_assert(sizeof(fccf_plane) == sizeof(MPlane) && sizeof(fccf_base) == sizeof(MBase), "table layouts");

extern "C" int fccf_debug_sincos(fccf_ctx* c, const double* x, int64_t n, double* s, double* co, uint32_t* ok) {
  if (!c || n < 0 || n > (1 << 24) || (n && (!x || !s || !co || !ok))) return FCCF_E_ARG;
  return guarded(c, [&] {
    if (!n) return;
    hipStream_t st = c->sb;
    c->arena2.ensure(28 * (size_t)n + 1024);
    c->arena2.reset();
    double* dx = c->arena2.take_n<double>(n);
    double* ds = c->arena2.take_n<double>(n);
    double* dc = c->arena2.take_n<double>(n);
    uint32_t* dk = c->arena2.take_n<uint32_t>(n);
    HIP_CHECK(hipMemcpyAsync(dx, x, 8 * (size_t)n, hipMemcpyHostToDevice, st));
    sincos_probe(dx, (int)n, ds, dc, dk, st);
    HIP_CHECK(hipGetLastError());
    HIP_CHECK(hipMemcpyAsync(s, ds, 8 * (size_t)n, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(co, dc, 8 * (size_t)n, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipMemcpyAsync(ok, dk, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
  });
}

extern "C" int fccf_stage_verify(fccf_ctx* c, const fccf_plane* F1, int nF1, const fccf_plane* F2, int nF2,
                                 const float* qt, int64_t n, const fccf_params* params, float* T_out, float* score,
                                 int32_t* npairs) {
  if (!c || nF1 < 0 || nF2 < 0 || nF1 > MAX_PLANES || nF2 > MAX_PLANES || (nF1 && !F1) || (nF2 && !F2) || n < 0 ||
      n > (1 << 24) || (n && (!qt || !T_out || !score || !npairs)))
    return FCCF_E_ARG;
  fccf_params P;
  if (params) P = *params;
  else fccf_params_default(&P);
  return guarded(c, [&] {
    std::vector<Plane> A((size_t)nF1), B((size_t)nF2);
    if (nF1) std::memcpy(A.data(), F1, sizeof(Plane) * (size_t)nF1);
    if (nF2) std::memcpy(B.data(), F2, sizeof(Plane) * (size_t)nF2);
    std::vector<QT> qs((size_t)n);
    for (int64_t k = 0; k < n; ++k) {
      const float* a = qt + 8 * k;
      qs[(size_t)k] = {a[0], a[1], a[2], a[3], a[4], a[5], a[6], a[7] != 0.f ? 1u : 0u};
    }
    std::vector<m44> T((size_t)n);
    std::vector<float> sc((size_t)n);
    std::vector<int> np((size_t)n);
    if (c->lm_device) {
      hipStream_t st = c->sb;
      MatchIn M;
      std::memset(&M, 0, sizeof M);
      if (nF1) std::memcpy(M.F1, F1, sizeof(MPlane) * nF1);
      if (nF2) std::memcpy(M.F2, F2, sizeof(MPlane) * nF2);
      M.nF1 = nF1;
      M.nF2 = nF2;
      c->arena2.ensure(sizeof(MatchIn) + 1024);
      c->arena2.reset();
      MatchIn* dM = c->arena2.take_n<MatchIn>(1);
      HIP_CHECK(hipMemcpyAsync(dM, &M, sizeof M, hipMemcpyHostToDevice, st));
      verify_items_device(c, qs, A, B, dM, P, st, T, sc, np);
    } else {
      c->pool.parallel_for((int)n, [&](int k) {
        T[(size_t)k] = T_from_qt(qs[(size_t)k]);
        sc[(size_t)k] = quick_verify(T[(size_t)k], A, B, P, &np[(size_t)k]);
      });
    }
    for (int64_t k = 0; k < n; ++k) {
      std::memcpy(T_out + 16 * k, &T[(size_t)k].m[0][0], 64);
      score[k] = sc[(size_t)k];
      npairs[k] = np[(size_t)k];
    }
  });
}

// K5 alone (match.hip) over the b1 range; the same kernels registration runs, without
// the pinned mailbox (K_pass is counted from the per-test candidate counts here).
namespace {
// fccf_stage_match, and with a group (G) the sharded search: G's block of source
// pairs, then the rank-ordered gather of every rank's lists (group.cpp).
int stage_match(fccf_ctx* c, const fccf_plane* F1, int nF1, const fccf_base* B1, int nB1, const fccf_plane* F2,
                int nF2, const fccf_base* B2, int nB2, int b1_lo, int b1_hi, const fccf_params* params,
                float* const cand[3], const int64_t cap[3], int64_t n_cand[3], int64_t* k_pass, Group* G) {
  if (!c || !n_cand || nF1 < 0 || nF2 < 0 || nB1 < 0 || nB2 < 0 || nF1 > MAX_PLANES || nF2 > MAX_PLANES ||
      nB1 > MAX_BASES || nB2 > MAX_BASES || (nF1 && !F1) || (nF2 && !F2) || (nB1 && !B1) || (nB2 && !B2))
    return FCCF_E_ARG;
  if (b1_hi < 0) b1_hi = nB1;
  if (G) shard_range(nB1, G->rank, G->n, &b1_lo, &b1_hi);
  if (b1_lo < 0 || b1_lo > b1_hi || b1_hi > nB1) return FCCF_E_ARG;
  // every pair must name planes of its own table: the kernels index F by i1, i2
  for (int i = 0; i < nB1; ++i)
    if (B1[i].i1 < 0 || B1[i].i1 >= nF1 || B1[i].i2 < 0 || B1[i].i2 >= nF1) return FCCF_E_ARG;
  for (int i = 0; i < nB2; ++i)
    if (B2[i].i1 < 0 || B2[i].i1 >= nF2 || B2[i].i2 < 0 || B2[i].i2 >= nF2) return FCCF_E_ARG;
  fccf_params P;
  if (params) P = *params;
  else fccf_params_default(&P);
  return guarded(c, [&] {
    hipStream_t st = c->sb;
    MatchIn M;
    std::memset(&M, 0, sizeof M);
    if (nF1) std::memcpy(M.F1, F1, sizeof(MPlane) * nF1);
    if (nF2) std::memcpy(M.F2, F2, sizeof(MPlane) * nF2);
    const int nb = b1_hi - b1_lo;  // the shard: b1-major order keeps each shard's lists contiguous
    if (nb) std::memcpy(M.B1, B1 + b1_lo, sizeof(MBase) * nb);
    if (nB2) std::memcpy(M.B2, B2, sizeof(MBase) * nB2);
    M.nF1 = nF1;
    M.nF2 = nF2;
    M.nB1 = nb;
    M.nB2 = nB2;
    M.ang_same = P.included_angle_same_threshold;
    M.third_thr = P.third_plane_threshold;
    M.third_cut = make_cut(P.third_plane_normal_threshold);
    const int K = nb * nB2, Kall = nB1 * nB2;
    const size_t per = (size_t)std::max(1, std::max(0, nF1 - 2) * std::max(0, nF2 - 2));
    const size_t ccap = std::max<size_t>(1, (size_t)(G ? Kall : K) * per);
    c->arena2.ensure(sizeof(MatchIn) + 3 * 4 * (size_t)std::max(K, 1) +
                     3 * ccap * (sizeof(MCand) + sizeof(QTd)) * (G ? 2 : 1) + (1 << 16));
    c->arena2.reset();
    MatchIn* dM = c->arena2.take_n<MatchIn>(1);
    uint32_t* dcnt = c->arena2.take_n<uint32_t>(std::max(K, 1));
    int32_t* dtype = c->arena2.take_n<int32_t>(std::max(K, 1));
    uint32_t* doff = c->arena2.take_n<uint32_t>(std::max(K, 1));
    uint32_t* dtot = c->arena2.take_n<uint32_t>(4);
    MCand* dc[3];
    QTd* dq[3];
    for (int t = 0; t < 3; ++t) {
      dc[t] = c->arena2.take_n<MCand>(ccap);
      dq[t] = c->arena2.take_n<QTd>(ccap);
    }
    HIP_CHECK(hipMemcpyAsync(dM, &M, sizeof M, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemsetAsync(dtot, 0, 16, st));
    match_candidates(dM, K, dcnt, dtype, doff, dtot, dc, dq, st, nullptr);
    HIP_CHECK(hipGetLastError());
    uint32_t tot[4] = {0, 0, 0, 0};
    std::vector<uint32_t> cnt((size_t)std::max(K, 1));
    HIP_CHECK(hipMemcpyAsync(tot, dtot, 16, hipMemcpyDeviceToHost, st));
    if (K) HIP_CHECK(hipMemcpyAsync(cnt.data(), dcnt, 4 * (size_t)K, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    int64_t kp = 0;
    for (int k = 0; k < K; ++k) kp += cnt[k] > 0;
    if (!K) tot[0] = tot[1] = tot[2] = 0;
    if (G) {
      MCand* ca[3];
      QTd* qa[3];
      for (int t = 0; t < 3; ++t) {
        ca[t] = c->arena2.take_n<MCand>(ccap);
        qa[t] = c->arena2.take_n<QTd>(ccap);
      }
      uint32_t* dta = c->arena2.take_n<uint32_t>(4);
      uint32_t tl[3] = {tot[0], tot[1], tot[2]};
      group_gather_candidates(G, dq, dc, tl, kp, qa, ca, ccap, tot, dta, &kp, st);
      for (int t = 0; t < 3; ++t) dc[t] = ca[t];
    }
    if (k_pass) *k_pass = kp;
    for (int t = 0; t < 3; ++t) {
      n_cand[t] = (G ? Kall : K) ? tot[t] : 0;
      const int64_t nc = std::min<int64_t>(n_cand[t], cand && cap && cand[t] ? cap[t] : 0);
      if (nc <= 0) continue;
      std::vector<MCand> v((size_t)nc);
      HIP_CHECK(hipMemcpyAsync(v.data(), dc[t], sizeof(MCand) * nc, hipMemcpyDeviceToHost, st));
      HIP_CHECK(hipStreamSynchronize(st));
      for (int64_t i = 0; i < nc; ++i) {  // [R | t; 0 0 0 1], row-major
        float* o = cand[t] + 16 * i;
        for (int r = 0; r < 3; ++r) {
          std::memcpy(o + 4 * r, v[i].R + 3 * r, 12);
          o[4 * r + 3] = v[i].t[r];
        }
        o[12] = o[13] = o[14] = 0.f;
        o[15] = 1.f;
      }
    }
  });
}
}  // namespace

extern "C" int fccf_stage_match(fccf_ctx* c, const fccf_plane* F1, int nF1, const fccf_base* B1, int nB1,
                                const fccf_plane* F2, int nF2, const fccf_base* B2, int nB2, int b1_lo, int b1_hi,
                                const fccf_params* params, float* const cand[3], const int64_t cap[3],
                                int64_t n_cand[3], int64_t* k_pass) {
  return stage_match(c, F1, nF1, B1, nB1, F2, nF2, B2, nB2, b1_lo, b1_hi, params, cand, cap, n_cand, k_pass, nullptr);
}

extern "C" int fccf_group_stage_match(fccf_group* g, const fccf_plane* F1, int nF1, const fccf_base* B1, int nB1,
                                      const fccf_plane* F2, int nF2, const fccf_base* B2, int nB2,
                                      const fccf_params* params, float* const cand[3], const int64_t cap[3],
                                      int64_t n_cand[3], int64_t* k_pass) {
  Group* G = group_of(g);
  if (!G) return FCCF_E_ARG;
  return stage_match(G->ctx, F1, nF1, B1, nB1, F2, nF2, B2, nB2, 0, -1, params, cand, cap, n_cand, k_pass, G);
}

extern "C" int fccf_stage_cluster(fccf_ctx* c, const float* cand, int64_t n, int cluster_num,
                                  const fccf_params* params, float* fine, int64_t cap, int64_t* n_fine,
                                  int64_t* n_clusters) {
  if ((!cand && n) || n < 0 || n > (int64_t)0x7FFFFFFF || cap < 0 || (cap && !fine) || !n_fine)
    return FCCF_E_ARG;
  fccf_params P;
  if (params) P = *params;
  else fccf_params_default(&P);
  return host_guarded(c, [&] {
    std::vector<QT> in((size_t)n), out;
    for (int64_t i = 0; i < n; ++i) {
      m44 T;
      std::memcpy(T.m, cand + 16 * i, sizeof T.m);
      in[i] = qt_from_T(T);
      in[i].alloc = 0;
    }
    int64_t ncl = 0;
    bool done = false;
    if (c && c->cluster_device && n > 0) {  // f3: radius search, seeds, sort and averaging on the device
      hipStream_t st = c->sb;
      MatchMail* mm = match_mail(c);
      const size_t nn = (size_t)n;
      c->arena2.ensure(sizeof(QTd) * nn + sizeof(uint64_t) * MatchMail::CB_CAP + 15 * 4 * nn + (1 << 16));
      c->arena2.reset();
      QTd* dq0 = c->arena2.take_n<QTd>(nn);
      uint32_t* dtot = c->arena2.take_n<uint32_t>(4);
      uint64_t* drows = c->arena2.take_n<uint64_t>(MatchMail::CB_CAP);
      QTd* const dq[3] = {dq0, dq0, dq0};
      uint8_t* h = (uint8_t*)c->pinned.get(sizeof(QTd) * nn + 16);
      QTd* hq = (QTd*)h;
      for (size_t i = 0; i < nn; ++i) hq[i] = {in[i].qw, in[i].qx, in[i].qy, in[i].qz, in[i].tx, in[i].ty, in[i].tz, 0u};
      uint32_t* ht = (uint32_t*)(h + sizeof(QTd) * nn);
      ht[0] = (uint32_t)n;
      ht[1] = ht[2] = ht[3] = 0;
      HIP_CHECK(hipMemcpyAsync(dq0, hq, sizeof(QTd) * nn, hipMemcpyHostToDevice, st));
      HIP_CHECK(hipMemcpyAsync(dtot, ht, 16, hipMemcpyHostToDevice, st));
      const float r2 = (float)((double)P.cluster_distance_threshold * (double)P.cluster_distance_threshold);
      cluster_bits(dq, dtot, r2, make_cut(P.cluster_angel_threshold), P.cluster_number_threshold, mm, st, drows);
      cluster_launch(c, dq, dtot, drows, nn, P, mm, st, &cluster_num);
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipStreamSynchronize(st));
      if (mm->cl_stat[0][0] == 0) {
        out = cluster_results(*mm, 0);
        ncl = (int64_t)mm->cl_stat[0][1];
        done = true;
      } else if (nn * ((nn + 63) / 64) <= MatchMail::CB_CAP && !((float)n <= P.cluster_number_threshold)) {
        transform_cluster(in, out, cluster_num, P, &ncl, &c->pool, mm->cbits);  // past the kernels' capacities
        done = true;
      }
    }
    if (!done) transform_cluster(in, out, cluster_num, P, &ncl, c ? &c->pool : nullptr, nullptr);
    *n_fine = (int64_t)out.size();
    if (n_clusters) *n_clusters = ncl;
    for (int64_t i = 0; i < std::min(*n_fine, cap); ++i) {
      const QT& q = out[i];
      const float a[8] = {q.qw, q.qx, q.qy, q.qz, q.tx, q.ty, q.tz, q.alloc ? 1.f : 0.f};
      std::memcpy(fine + 8 * i, a, sizeof a);
    }
  });
}

// Fusion (FCCF.cpp:1546-1606, host): the caller's ranked, verified candidates of the
// three types (18 floats each: row-major T, quick_verify score, fine_verify score).
extern "C" int fccf_stage_fuse(fccf_ctx* c, const float* const cand[3], const int64_t n[3], int analyse_max,
                               float T[16], float high[24]) {
  if (!cand || !n || !T || analyse_max < 0) return FCCF_E_ARG;
  for (int t = 0; t < 3; ++t)
    if (n[t] < 0 || (n[t] && !cand[t])) return FCCF_E_ARG;
  return host_guarded(c, [&] {
    std::vector<TS> ctv[3];
    for (int t = 0; t < 3; ++t)
      for (int64_t i = 0; i < n[t]; ++i) {
        TS x;
        const float* r = cand[t] + 18 * i;
        std::memcpy(x.T.m, r, sizeof x.T.m);
        x.score = r[16];
        x.score2 = r[17];
        ctv[t].push_back(x);
      }
    std::vector<High> tmp;
    const m44 R = fuse_types(ctv, analyse_max, &tmp);
    std::memcpy(T, R.m, sizeof R.m);
    if (high)
      for (int t = 0; t < 3; ++t) {
        const High& h = tmp[(size_t)t];
        const float a[8] = {h.qt.qw, h.qt.qx, h.qt.qy, h.qt.qz, h.qt.tx, h.qt.ty, h.qt.tz, h.score};
        std::memcpy(high + 8 * t, a, sizeof a);
      }
  });
}

// K7 alone (fine.hip): S1's octree bounds replayed, then the batched evaluation.
extern "C" int fccf_stage_fine_verify(fccf_ctx* c, const float* s1, int64_t n1, const float* s2, int64_t n2,
                                      const float* T, int E, float voxel, float* scores) {
  if (!c || !s1 || !s2 || !T || !scores || n1 < 1 || n2 < 1 || E < 1 || E > MAX_EVAL || !(voxel > 0.f) ||
      (int64_t)E * (n1 + n2) >= ((int64_t)1 << 31))
    return FCCF_E_ARG;
  return guarded(c, [&] {
    hipStream_t st = c->sb;
    const uint32_t u1 = (uint32_t)n1, u2 = (uint32_t)n2;
    const size_t nk = (size_t)E * (u1 + u2);
    const size_t af1 = aggr_floats(u1), af2 = aggr_floats(u2);
    const size_t need = 12 * ((size_t)u1 + u2) + 4 * af1 + 12 * (size_t)E * u2 + 4 * E * af2 +
                        sizeof(OctState) * (E + 2) + (3 * 8 + 3 * 4 + 4 + 8) * (nk + 1) + 64 * 5 +
                        sizeof(m44) * E + 64 + sort_scratch_bytes((uint32_t)nk) + 48 * 256 +
                        exact_sum_bytes(E, u1 + u2) + 256;
    c->arena2.ensure(need);
    c->arena2.reset();
    Arena& a = c->arena2;
    float* d1 = a.take_n<float>(3 * (size_t)u1);
    float* d2 = a.take_n<float>(3 * (size_t)u2);
    uint32_t* dn1 = a.take_n<uint32_t>(16);
    float* aggr1 = a.take_n<float>(af1);
    OctState* st1 = a.take_n<OctState>(1);
    FineBufs fb;
    fb.s2t = a.take_n<float>(3 * (size_t)E * u2);
    fb.aggr2 = a.take_n<float>((size_t)E * af2);
    fb.state = a.take_n<OctState>(E + 1);
    fb.k0 = a.take_n<uint64_t>(nk);
    fb.k1 = a.take_n<uint64_t>(nk);
    fb.k2 = a.take_n<uint64_t>(nk);
    fb.v0 = a.take_n<uint32_t>(nk);
    fb.v1 = a.take_n<uint32_t>(nk);
    fb.v2 = a.take_n<uint32_t>(nk);
    fb.pts = a.take_n<uint32_t>(MAX_EVAL);
    fb.starts = a.take_n<uint32_t>(nk + 1);
    fb.term = a.take_n<float>(nk + 1);
    fb.range = a.take_n<uint32_t>(2 * MAX_EVAL);
    fb.nseg_e = a.take_n<uint32_t>(2 * MAX_EVAL);
    fb.similar = a.take_n<float>(MAX_EVAL);
    fb.all = a.take_n<float>(MAX_EVAL);
    fb.scal = a.take_n<uint32_t>(16);
    fb.scores = a.take_n<float>(E);
    fb.T = a.take_n<m44>(E);
    fb.ss = sort_scratch_carve(a.take(sort_scratch_bytes((uint32_t)nk)), (uint32_t)nk);
    fb.xs = exact_sum_carve(a.take(exact_sum_bytes(E, u1 + u2)), E, u1 + u2);
    HIP_CHECK(hipMemcpyAsync(d1, s1, 12 * (size_t)u1, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(d2, s2, 12 * (size_t)u2, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(dn1, &u1, 4, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(fb.T, T, sizeof(m44) * E, hipMemcpyHostToDevice, st));
    octree_replay(d1, dn1, u1, (double)voxel, aggr1, st1, st);
    uint32_t err = 0;
    for (int mode = fine_mode_env(c->fine_sorted.load() ? 1 : 0);; mode = FV_LEAVES_SORTED) {
      fine_verify_batch(d1, u1, st1, d2, u2, E, (double)voxel, fb, st, nullptr, mode, fine_lds_cap_env());
      HIP_CHECK(hipGetLastError());
      HIP_CHECK(hipMemcpyAsync(scores, fb.scores, 4 * (size_t)E, hipMemcpyDeviceToHost, st));
      HIP_CHECK(hipMemcpyAsync(&err, fb.scal + 7, 4, hipMemcpyDeviceToHost, st));
      HIP_CHECK(hipStreamSynchronize(st));
      if (!(err & FV_ERR_LDS) || mode == FV_LEAVES_SORTED) break;  // (more leaves than the LDS form holds: sorted)
    }
    if (err) throw Error(FCCF_E_INTERNAL, "fine_verify: >= 2^24 points in one evaluation");
  });
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

extern "C" int fccf_device_download(fccf_ctx* c, const float* d, int64_t n, float* xyz) {
  if (!c || (!d && n) || (!xyz && n) || n < 0) return FCCF_E_ARG;
  return guarded(c, [&] {
    if (n) HIP_CHECK(hipMemcpy(xyz, d, 12 * (size_t)n, hipMemcpyDeviceToHost));
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
  return device_sync_guarded() == hipSuccess ? FCCF_OK : FCCF_E_HIP;
}
#endif
