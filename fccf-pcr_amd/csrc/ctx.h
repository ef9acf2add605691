// ctx.h — fccf_ctx internals: device, streams, workspace arena, debug store.
#pragma once
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <atomic>
#include <mutex>
#include <stdexcept>
#include <thread>
#include <string>
#include <type_traits>
#include <vector>

#include "../../include/fccf.h"
#include "error.h"
#include "ingest.h"
#include "pool.h"
#include "probe.h"

namespace fccf {

struct Group;

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
  void ensure(size_t bytes);
  ~Arena() {
    if (base) (void)hipFree(base);
  }
};

// Growing an arena frees and re-allocates device memory; a pipelined batch may be
// capturing the next pair's graphs on the helper thread meanwhile, so reallocation
// takes the capture lock too (capture_mutex below).
inline std::mutex& capture_mutex();

inline void Arena::ensure(size_t bytes) {
  if (bytes <= cap) return;
  std::lock_guard<std::mutex> lk(capture_mutex());
  {
    if (base) (void)hipFree(base);
    base = nullptr;
    cap = 0;
    if (hipMalloc((void**)&base, bytes) != hipSuccess) throw Error(FCCF_E_OOM, "hipMalloc arena");
    cap = bytes;
  }
}

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

// Pinned, host-mapped, coherent mailboxes (mail.h), allocated once per ctx.
struct MailBuf {
  void* p = nullptr;
  ~MailBuf() {
    if (p) (void)hipHostFree(p);
  }
};

// One captured hipGraph, re-captured whenever its key (the workspace layout and
// every launch argument that is not read from device memory) changes.  The
// pipeline's sizes live in device memory, so a graph replays for any input that
// fits the captured capacities.
// A pipelined batch enqueues the next pair's cloud stage from a helper thread
// while this thread waits on events of the current pair.  HIP rejects a wait on an
// event whose recording stream is being captured at that moment, so graph captures
// and the cross-thread event waits (pipeline.cpp) take this lock.  Captures happen
// only when a graph's key changes, so the steady state never contends.
inline std::mutex& capture_mutex() {
  static std::mutex m;
  return m;
}

// A device-wide synchronisation while another thread (the batch's helper, another
// phase-B chain, another virtual rank's ctx) may be capturing a graph: HIP may
// invalidate a capture that a concurrent device synchronisation meets.
inline hipError_t device_sync_guarded() {
  std::lock_guard<std::mutex> lk(capture_mutex());
  return hipDeviceSynchronize();
}

// A wait on an event that another thread's stream may be capturing right now.
inline void guarded_stream_wait(hipStream_t st, hipEvent_t ev) {
  std::lock_guard<std::mutex> lk(capture_mutex());
  HIP_CHECK(hipStreamWaitEvent(st, ev, 0));
}

// A host wait on an event whose stream another thread may be capturing (the fine stream
// sa[1], which every phase-B chain captures g_fine on): each query under the capture
// lock, the lock released between queries so that a capture can proceed.
inline void guarded_event_sync(hipEvent_t ev) {
  for (;;) {
    hipError_t e;
    {
      std::lock_guard<std::mutex> lk(capture_mutex());
      e = hipEventQuery(ev);
    }
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) HIP_CHECK(e);
    std::this_thread::sleep_for(std::chrono::microseconds(20));
  }
}

// A host wait on a pinned mailbox flag that a stage's last kernel sets after a
// system-scope fence (mail.h): polled for up to spin_us.  The runtime's event wait
// polls only briefly and then sleeps on an interrupt, and the thread woke 18-35 us
// after a ~1 ms cloud stage or a ~0.1 ms fine verification had ended (hipEventQuery
// polling did not shorten it; profiles/r05k, r05l).  Returns false when the flag was
// not seen in time (or FCCF_SPIN_US=0): the caller then waits on the stage's event.
// keep (optional) runs about every 200 us of polling: the caller keeps its pool's
// workers spinning for the parallel work that follows the wait.
template <class Keep = void (*)()>
inline bool mail_wait(const uint32_t* flag, double spin_us, Keep keep = nullptr) {
  const char* v = std::getenv("FCCF_SPIN_US");  // (read per wait: tests switch it)
  if (v && *v) spin_us = std::atof(v);
  if (spin_us <= 0.0) return false;
  const auto t0 = std::chrono::steady_clock::now();
  double next_keep = 200.0;
  for (uint32_t it = 0;; ++it) {
    if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != 0u) return true;
    if ((it & 63u) == 63u) {
      const double el = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (el > spin_us) return false;
      if (el > next_keep) {
        if constexpr (!std::is_pointer<Keep>::value) keep();
        next_keep = el + 200.0;
      }
    }
    for (int i = 0; i < 8; ++i) __builtin_ia32_pause();
  }
}

// The arguments of a patched kernel node that describe the workspace layout (every
// argument but the per-call inputs): their indices in kernelParams and their sizes.
struct PatchLayout {
  int n = 0;
  int idx[8] = {};
  size_t size[8] = {};
};

struct CachedGraph {
  std::vector<uint8_t> key;
  hipGraphExec_t exec = nullptr;
  int captures = 0;  // since the owner last cleared it
  // Patching: one kernel node (found by its function after the capture) whose
  // arguments are rewritten before every replay, so the graph can read inputs that
  // change from call to call (caller-owned clouds) without staging them.
  hipGraph_t graph = nullptr;
  hipGraphNode_t pnode = nullptr;
  hipKernelNodeParams pparams{};
  // Replay check: the layout arguments' bytes as captured.  A replay whose patch
  // carries other layout arguments -- a patch state shared by graphs of different
  // layouts, the bug class of a device fault in round 4 -- fails with FCCF_E_INTERNAL
  // before anything is launched (a memcmp of a few hundred bytes per replay).
  std::vector<uint8_t> layout_bytes;
  void reset() {
    if (exec) (void)hipGraphExecDestroy(exec);
    if (graph) (void)hipGraphDestroy(graph);
    exec = nullptr;
    graph = nullptr;
    pnode = nullptr;
    key.clear();
    layout_bytes.clear();
  }
  ~CachedGraph() { reset(); }
  // whether run() with this key would replay (not capture)
  bool replays(const void* k, size_t kn) const {
    return exec && key.size() == kn && std::memcmp(key.data(), k, kn) == 0;
  }
  static std::vector<uint8_t> layout_of(void** pargs, const PatchLayout* lay) {
    std::vector<uint8_t> b;
    for (int i = 0; lay && i < lay->n; ++i) {
      const uint8_t* a = (const uint8_t*)pargs[lay->idx[i]];
      b.insert(b.end(), a, a + lay->size[i]);
    }
    return b;
  }
  // body enqueues the work; pfunc/pargs (optional): the patched kernel and its
  // current arguments (kernelParams layout: one pointer per argument); lay: which of
  // them must equal the captured ones at every replay.
  // eager: launch the body directly this call (work with a host step inside, e.g. the
  // sharded sort's gather)
  template <class F>
  void run(const void* k, size_t kn, hipStream_t st, F body, const void* pfunc = nullptr, void** pargs = nullptr,
           bool eager = false, const PatchLayout* lay = nullptr) {
    if (eager || (g_probe && g_probe->on())) {  // probed calls launch eagerly (probe.h)
      body();
      return;
    }
    const uint8_t* kb = (const uint8_t*)k;
    if (!exec || key.size() != kn || std::memcmp(key.data(), kb, kn) != 0) {
      // no other thread may create a dependency on a stream while it is captured
      // (hipErrorStreamCaptureIsolation): see capture_mutex()
      std::lock_guard<std::mutex> lk(capture_mutex());
      reset();
      hipGraph_t g = nullptr;
      HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      try {
        body();
      } catch (...) {
        (void)hipStreamEndCapture(st, &g);
        if (g) (void)hipGraphDestroy(g);
        throw;
      }
      HIP_CHECK(hipStreamEndCapture(st, &g));
      const hipError_t e = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
      if (e != hipSuccess) {
        (void)hipGraphDestroy(g);
        exec = nullptr;
        throw Error(FCCF_E_HIP, std::string("hipGraphInstantiate: ") + hipGetErrorString(e));
      }
      graph = g;
      if (pfunc) find_node(pfunc);
      if (pfunc) layout_bytes = layout_of(pargs, lay);
      key.assign(kb, kb + kn);
      ++captures;
    } else if (pfunc) {
      if (layout_of(pargs, lay) != layout_bytes)
        throw Error(FCCF_E_INTERNAL, "graph replay: the patched entry arguments differ from the layout the graph "
                                     "was captured with");
      hipKernelNodeParams np = pparams;
      np.kernelParams = pargs;
      np.extra = nullptr;
      HIP_CHECK(hipGraphExecKernelNodeSetParams(exec, pnode, &np));
    }
    static const bool trace = std::getenv("FCCF_HOST_TRACE") != nullptr;
    const auto h0 = std::chrono::steady_clock::now();
    HIP_CHECK(hipGraphLaunch(exec, st));
    if (trace)
      std::fprintf(stderr, "graph launch host %.1f us\n",
                   std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - h0).count());
  }

 private:
  void find_node(const void* func) {
    size_t n = 0;
    HIP_CHECK(hipGraphGetNodes(graph, nullptr, &n));
    std::vector<hipGraphNode_t> nodes(n);
    if (n) HIP_CHECK(hipGraphGetNodes(graph, nodes.data(), &n));
    int found = 0;
    for (hipGraphNode_t nd : nodes) {
      hipGraphNodeType t;
      HIP_CHECK(hipGraphNodeGetType(nd, &t));
      if (t != hipGraphNodeTypeKernel) continue;
      hipKernelNodeParams p{};
      HIP_CHECK(hipGraphKernelNodeGetParams(nd, &p));
      if (p.func != func) continue;
      pnode = nd;
      pparams = p;
      ++found;
    }
    if (found != 1) {
      reset();
      throw Error(FCCF_E_HIP, "graph patch: the patched kernel must occur exactly once, found " +
                                  std::to_string(found));
    }
  }
};

}  // namespace fccf

struct fccf_ctx {
  int device = 0;
  // Pair slots.  A cloud stage (both VoxelGrid passes, centroid, face voxels) runs the
  // clouds of up to PAIRS_MAX = 5 pairs in the same launches (a pipelined batch groups
  // them: the sort's dependent rounds are paid once for ten clouds); stage group G
  // uses slots PAIRS_MAX * G + j (j < PAIRS_MAX), and the group's shared resources (arena
  // of its clouds, stage graphs, fork/join events) live in its first slot, PAIRS_MAX * G.
  // Two groups double-buffer, so a batch can
  // run the next group's clouds while this group's later stages run.  Two groups never
  // run their cloud stages at the same time, so they share streams: sa[0] the batched
  // cloud stage, sa[2] the centroid sums, sa[1] fine verification, and sb for matching
  // and everything else -- within the four hardware queues a process gets.
  struct CloudSet {
    fccf::Arena arena;
    fccf::Arena arena3;              // fine verification scratch of the pair on this set
    fccf::Arena inarena;             // staged host inputs of the pair on this set (copy stream)
    hipEvent_t ev_in0 = nullptr, ev_in = nullptr;  // their copies started / done (timing: fccf_stats h2d)
    hipEvent_t ev[8] = {};           // [0] inputs read (pass 1 done), [1] the stage's part A done (first slot
                                     // of a group), [3] fine verification done, [4] clouds done, [5] S1
                                     // replay done; [6]/[7] the centroid branch's fork/join inside part B
                                     // (capture-internal)
    hipEvent_t tev[6] = {};          // timing: [4] fine start, [5] fine done (fccf_stats::dev_ms[3]);
                                     // the cloud stage's spans are device stamps (CloudMail::stamp)
    fccf::CachedGraph g_seg[5];      // first slot of a group: its cloud stage of 1..PAIRS_MAX pairs, one graph
                                     // per pair count: part A (the VoxelGrid passes; with a group attached,
                                     // the whole stage)
    fccf::CachedGraph g_fine;        // fine-verify batch (K7) of the pair on this set: one graph per
                                     // set, so alternating pairs in a batch replay instead of re-capturing
    void* ws = nullptr;              // pipeline.cpp state of the registration in flight
  } cs[10];                           // two stage groups of up to PAIRS_MAX pair slots (pipeline.cpp)
  hipStream_t sa[4] = {};            // cloud stage streams: [0] part A, [2] part B, [3] B's centroid branch
                                     // (a capture fork; replays schedule it), [1] fine verification
  hipStream_t sb = nullptr;          // matching, copies, stage exports
  fccf::Arena arena2;  // matching (and the stage exports)
  fccf::PinnedBuf pinned;
  fccf::MailBuf mail;  // pipeline.cpp host_mail()
  fccf::Pool pool;
  fccf::AsyncTask enq;  // pipelined batch: enqueues the next pair's cloud stage
  // A pipelined batch runs the phase B of alternate pairs on two host threads ("chains",
  // pipeline.cpp): the calling thread and b1w, each with a pool of half the host threads
  // (bpool, created on first use), its own matching scratch (arena2 / arena2b), pinned
  // match mailbox (HostMail::match / match2) and completion event (ev_match).  The
  // fine-verification launches of both chains share sa[1] under fine_mutex.
  fccf::AsyncTask b1w;
  std::unique_ptr<fccf::Pool> bpool[5];
  fccf::Arena arena2b;
  hipEvent_t ev_match[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  // The batch's last stage group drains with a chain per pair: its third to fifth pairs
  // run phase B on b1w2 / b1w3 / b1w4 with pools of a quarter of the host threads
  // (bpool[2..4]), matching scratch arena2c / arena2d / arena2e and mailboxes
  // HostMail::match3 / match4 / match5.
  fccf::AsyncTask b1w2, b1w3, b1w4;
  fccf::Arena arena2c, arena2d, arena2e;
  std::mutex fine_mutex;
  fccf::Probe probe;
  fccf::Ingest ingest;  // pinned upload ring + copy stream (ingest.cpp)
  fccf::Group* group = nullptr;  // RCCL rank of a sharded registration (group.cpp), or none
  bool debug = false;
  // face-code radix passes (x 8 bits) the cloud stage launches: three until a scene's
  // 1 m octree needs a fourth digit (FACE_DEEP in a cloud's mailbox), then four
  std::atomic<int> face_fast_bits{24};
  // fine verification in the sorted leaf form (FV_LEAVES_SORTED): set once an evaluation
  // had more leaves than the LDS form holds (FV_ERR_LDS)
  std::atomic<bool> fine_sorted{false};
  bool grow_device = false;  // K4 region growing on the GPU (grow.hip) instead of the host
  bool lm_device = false;    // quick_verify + LM on the GPU (verify.hip) instead of the host pool
  bool cluster_device = false;  // transform_cluster's seeds, sort and averaging on the GPU (cluster.hip)
  fccf::Arena arena_v;       // device quick_verify batch (candidates in, refined T / scores out)
  uint32_t sort_stats[32] = {};  // IsBufs::ctl of the last fccf_debug_sort_keys
  uint32_t sort_rounds[4 * 24] = {};  // IsBufs::rounds (IS_RMAX records) of the last fccf_debug_sort_keys
  uint32_t* d_flags = nullptr;   // device words (zeroed at creation): [0] injected K1 sort faults (test hook)
  bool graph_mismatch = false;   // test hook: the next cloud-stage replay patches a wrong layout argument
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
