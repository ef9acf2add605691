// pipeline.cpp — fccf_register / fccf_register_device: the whole FCCF-PCR
// registration (FCCF.cpp main :1668-1683 + computer_transform_guess :1370-1608).
//
// Device (two HIP streams, one per cloud, no host round-trip inside a cloud):
//   K1 VoxelGrid x2 -> remove-NaN -> K2/K3 octree leaves + plane fit + compaction
// Host (round 1; <= a few thousand items): region growing / plane selection,
//   select_base, clustering, quick_verify + LM, score ranking, fusion.
// Device: K5 coplane-pair matching + closed-form transforms, K7 fine verify (batched).
//
// Cloud roles follow the reference's swapped call (FCCF.cpp:1683): driver
// "source" (index 0 here, F1/S1) is the TAR file, driver "target" (index 1, F2/S2)
// is the SRC file; the output T maps src-file points into the tar frame.
#define KT_TU 7  // ktrace.h source tag
#include <hip/hip_runtime.h>

#include <algorithm>
#include <condition_variable>
#include <exception>
#include <mutex>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "ctx.h"
#include "group.h"
#include "host_stages.h"
#include "kernels.h"
#include "match.h"
#include "mail.h"
#include "pipeline.h"

namespace fccf {

namespace {

using clk = std::chrono::steady_clock;
double ms_since(clk::time_point t0) { return std::chrono::duration<double, std::milli>(clk::now() - t0).count(); }

// ------------------------------------------------------------ remove-NaN (:1374-1375)
// The first VoxelGrid pass writes its output twice (ds1 for the record, ds1f for the
// second pass) and flags a non-finite output point.  Centroids of finite points are
// finite unless a leaf sum overflows, and the pass-through output (int32 index
// overflow) holds the input as is, so the flag is almost never set: then ds1f is
// already the NaN-free cloud and only its count is written.  Otherwise this single
// workgroup compacts ds1 into ds1f in order, 1024 points per step (slow, rare).
__global__ void __launch_bounds__(1024) k_finite_fix(B4<const float*> xyz2, B4<const uint32_t*> d_n2,
                                                     B4<const VGParams*> P2, B4<float*> out2, B4<uint32_t*> d_m2) {
  KT();
  const int e = blockIdx.y;
  if (threadIdx.x == 0) const_cast<VGParams*>(P2[e])->t_driver = __builtin_amdgcn_s_memrealtime();
  const uint32_t n = *d_n2[e];
  if (!P2[e]->nonfinite) {
    if (threadIdx.x == 0) *d_m2[e] = n;
    return;
  }
  const float* __restrict__ xyz = xyz2[e];
  float* __restrict__ out = out2[e];
  __shared__ uint32_t wsum[16];
  uint32_t base = 0;
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint32_t c0 = 0; c0 < n; c0 += 1024) {
    const uint32_t i = c0 + threadIdx.x;
    float x = 0.f, y = 0.f, z = 0.f;
    bool keep = false;
    if (i < n) {
      x = xyz[3 * i]; y = xyz[3 * i + 1]; z = xyz[3 * i + 2];
      keep = finite3(x, y, z);
    }
    const uint64_t m = __ballot(keep);
    if (lane == 0) wsum[w] = (uint32_t)__popcll(m);
    __syncthreads();
    uint32_t before = base, tot = 0;
    for (uint32_t k = 0; k < 16; ++k) {
      before += k < w ? wsum[k] : 0u;
      tot += wsum[k];
    }
    const uint32_t pos = before + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (keep) { out[3 * pos] = x; out[3 * pos + 1] = y; out[3 * pos + 2] = z; }
    base += tot;
    __syncthreads();
  }
  if (threadIdx.x == 0) *d_m2[e] = base;
}

inline uint32_t grid_for(uint32_t cap, uint32_t per = 256, uint32_t mx = 4096) {
  uint32_t g = (cap + per - 1) / per;
  return g < 1 ? 1 : (g > mx ? mx : g);
}

}  // namespace

namespace {

// Pairs per cloud stage: a stage group's clouds (2 per pair) share every launch of the
// stage (blockIdx.y), so PAIRS_MAX = BMAX / 2; two stage groups alternate, each with
// PAIRS_MAX slots (ctx CloudSets, mailboxes).  FCCF_PAIR_BATCH=1..PAIRS_MAX overrides
// the default.
constexpr int PAIRS_MAX = BMAX / 2;
constexpr int PAIRS_DEFAULT = 5;
static_assert(sizeof(((fccf_ctx*)nullptr)->cs) / sizeof(((fccf_ctx*)nullptr)->cs[0]) == 2 * PAIRS_MAX, "slots");
static_assert(sizeof(HostMail::clouds) / sizeof(CloudMail) == 2 * PAIRS_MAX, "cloud mailboxes");
static_assert(sizeof(HostMail::fine) / sizeof(FineMail) == 2 * PAIRS_MAX, "fine mailboxes");
static_assert(Group::SLOTS == 2 * PAIRS_MAX, "group fine buffers per slot");

// ------------------------------------------------------------ per-cloud device state
struct CloudWS {
  uint32_t cap = 0;
  uint32_t* sc = nullptr;  // [0] n_in, [1] m1, [2] m1 finite, [3] m2
  float *ds1 = nullptr, *ds1f = nullptr, *ds2 = nullptr;
  VGBufs vg;
  FaceBufs fb;
  VoxRec* planar = nullptr;
  float* resid = nullptr;
  float* faggr = nullptr;        // fine_verify S1 bounds replay (cloud 0 only)
  OctState* fstate = nullptr;
};

size_t cloud_bytes(uint32_t cap, bool) {
  const size_t N = cap;
  size_t b = 0;
  b += 12 * N * 3 + 64;                                        // ds1, ds1f, ds2
  b += voxel_grid_bytes(cap);                                  // K1
  b += 3 * 8 * N + 3 * 4 * N + 4 * (N + 1);                    // codes, vals (3 buffers), starts
  b += 4 * aggr_floats(cap) + 256;                             // aggregates, state, centroid
  b += sizeof(VoxRec) * N + 4 * 4 * N + 64;                    // leaf records, flags, offsets
  b += 12 * N + 4 * N;                                         // sorted points, leaf of point
  b += sizeof(VoxRec) * N + 12 * N;                            // planar out, residual out
  b += 4 * aggr_floats(cap) + 512;                             // fine-verify S1 bounds replay
  b += sort_scratch_bytes(cap) + 64 * 256;                     // sort scratch + alignment slack
  return b;
}

void carve_cloud(Arena& a, CloudWS& w, uint32_t cap, bool) {
  w.cap = cap;
  w.sc = a.take_n<uint32_t>(16);
  w.ds1 = a.take_n<float>(3 * (size_t)cap);
  w.ds1f = a.take_n<float>(3 * (size_t)cap);
  w.ds2 = a.take_n<float>(3 * (size_t)cap);
  w.vg = voxel_grid_carve(a, cap);
  w.fb = face_bufs_carve(a, cap);
  w.fb.vgp = w.vg.params;  // stage stamps (k_compact_planar -> CloudMail::stamp)
  w.planar = a.take_n<VoxRec>(cap);
  w.resid = a.take_n<float>(3 * (size_t)cap);
  w.faggr = a.take_n<float>(aggr_floats(cap));
  w.fstate = a.take_n<OctState>(1);
}

// Device part of the clouds of one or two pairs, batched (blockIdx.y = cloud, every
// cloud carved alike), nc = 2 * pairs clouds: pair j's clouds are 2j (the driver's
// source) and 2j + 1.  One graph on one stream:
//   A  both VoxelGrid passes with remove-NaN between them
//   F  octree leaves, per-leaf fit, residual cloud, after A
// plus, on the side stream after A, the sequential compute3DCentroid sums of every
// cloud (three rows each, one launch set), and the planar compaction, which orients
// normals towards the centroid, after F and the sums.
template <class T, class F>
B4<T> all_of(const CloudWS* w, int nc, F get) {
  T v[BMAX];
  for (int e = 0; e < BMAX; ++e) v[e] = get(w[e < nc ? e : nc - 1]);
  return B4<T>(v, BMAX);
}

// main's VoxelGrid pass (:1668-1678) over the inputs xin (n points each), its
// output also into ds1f; entry receives its entry kernel's arguments (graph patch)
void seg_pass1(CloudWS* w, int nc, const float* const* xin, const uint32_t* n, float leaf, hipStream_t st,
               VGEntry* entry) {
  const uint32_t cap = w[0].cap;
  auto sc = [&](int i) { return all_of<uint32_t*>(w, nc, [i](const CloudWS& c) { return c.sc + i; }); };
  const B4<VGBufs> vg = all_of<VGBufs>(w, nc, [](const CloudWS& c) { return c.vg; });
  const float* x[BMAX];
  for (int e = 0; e < BMAX; ++e) x[e] = xin[e < nc ? e : nc - 1];
  voxel_grid(B4<const float*>(x, BMAX), sc(0), cap, leaf,
             all_of<float*>(w, nc, [](const CloudWS& c) { return c.ds1; }), sc(1), vg, st, false, nc,
             all_of<float*>(w, nc, [](const CloudWS& c) { return c.ds1f; }), n, entry);
}
// the driver's remove-NaN and second VoxelGrid pass (:1374-1387); mode VG_OPTIMISTIC
// (the pipeline's default: no fallback sort launches, the host redoes a pass that was
// not in leaf order) or VG_PRESORTED (the redo)
void seg_downsample(CloudWS* w, int nc, float leaf, hipStream_t st, int mode) {
  const uint32_t cap = w[0].cap;
  auto sc = [&](int i) { return all_of<uint32_t*>(w, nc, [i](const CloudWS& c) { return c.sc + i; }); };
  const B4<VGBufs> vg = all_of<VGBufs>(w, nc, [](const CloudWS& c) { return c.vg; });
  const B4<float*> ds1 = all_of<float*>(w, nc, [](const CloudWS& c) { return c.ds1; });
  const B4<float*> ds1f = all_of<float*>(w, nc, [](const CloudWS& c) { return c.ds1f; });
  k_finite_fix<<<dim3(1, nc), 1024, 0, st>>>(B4<const float*>(ds1), sc(1),
                                             all_of<const VGParams*>(w, nc, [](const CloudWS& c) { return (const VGParams*)c.vg.params; }),
                                             ds1f, sc(2));  // driver :1374-1375
  voxel_grid(B4<const float*>(ds1f), sc(2), cap, leaf, all_of<float*>(w, nc, [](const CloudWS& c) { return c.ds2; }),
             sc(3), vg, st, mode, nc);  // driver :1377-1387
}
// PG: row P, the face stage sharded over a group's ranks by Morton range (group.cpp)
void seg_faces(CloudWS* w, int nc, const fccf_params& P, hipStream_t st, Group* PG = nullptr, int fast_bits = 32) {
  const uint32_t cap = w[0].cap;
  const B4<FaceBufs> fb = all_of<FaceBufs>(w, nc, [](const CloudWS& c) { return c.fb; });
  const B4<const uint32_t*> m2 = all_of<const uint32_t*>(w, nc, [](const CloudWS& c) { return (const uint32_t*)c.sc + 3; });
  if (PG) {
    face_voxels_sharded(PG, all_of<const float*>(w, nc, [](const CloudWS& c) { return (const float*)c.ds2; }), m2, cap,
                        (double)P.face_voxel_size, P.voxel_point_threshold, P.curvature_threshold,
                        all_of<float*>(w, nc, [](const CloudWS& c) { return c.resid; }), fb, st, nc);
    return;
  }
  face_voxels_prepare(all_of<const float*>(w, nc, [](const CloudWS& c) { return (const float*)c.ds2; }), m2, cap,
                      (double)P.face_voxel_size, fb, st, nc, fast_bits);
  face_voxels_fit(m2, cap, P.voxel_point_threshold, P.curvature_threshold,
                  all_of<float*>(w, nc, [](const CloudWS& c) { return c.resid; }), fb, st, nc);
}
// The residual cloud of the driver source is fine_verify's S1 (:788-805): its
// octree bounds do not depend on any candidate, so they are replayed after the
// clouds-done event, overlapping the host stages that produce the candidates.
// fine_verify's S1 octree bounds (cloud 0 of each pair) for the P pairs of a stage group
// in one batched launch pair (block aggregates, bounds replay): pair j's cloud 0 is
// w[2j], carved alike, so its fields sit at one byte stride from pair 0's
void seg_s1_replay(CloudWS* w, int P, const fccf_params& Pa, hipStream_t st) {
  SeqStrides sd;
  if (P > 1) {
    auto stride = [&](const void* a0, const void* a1) { return (size_t)((const char*)a1 - (const char*)a0); };
    sd.xyz = stride(w[0].resid, w[2].resid);
    sd.n = stride(w[0].fb.nresid, w[2].fb.nresid);
    sd.aggr = stride(w[0].faggr, w[2].faggr);
    sd.state = stride(w[0].fstate, w[2].fstate);
    for (int j = 2; j < P; ++j)
      if (stride(w[0].resid, w[2 * j].resid) != j * sd.xyz || stride(w[0].fb.nresid, w[2 * j].fb.nresid) != j * sd.n ||
          stride(w[0].faggr, w[2 * j].faggr) != j * sd.aggr || stride(w[0].fstate, w[2 * j].fstate) != j * sd.state)
        throw Error(FCCF_E_INTERNAL, "S1 replay: clouds not carved alike");
  }
  const double res = (double)Pa.fine_verify_voxel_size;
  block_aggr(w[0].resid, w[0].fb.nresid, w[0].cap, w[0].faggr, st, P, sd, w[0].fstate);  // (also resets the states)
  octree_sim(w[0].resid, w[0].fb.nresid, w[0].cap, res, w[0].faggr, w[0].fstate, st, P, sd);
}

// The ctx's pinned mailboxes (mail.h): allocated once, so graph-captured kernels may hold the pointer.
HostMail* host_mail(fccf_ctx* c) {
  if (!c->mail.p) {
    void* p = nullptr;
    if (hipHostMalloc(&p, sizeof(HostMail), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
      throw Error(FCCF_E_OOM, "hipHostMalloc mailbox");
    c->mail.p = p;
  }
  return (HostMail*)c->mail.p;
}

template <class T>
std::vector<T> d2h(const T* d, size_t n, hipStream_t st) {
  std::vector<T> v(n);
  if (n) HIP_CHECK(hipMemcpyAsync(v.data(), d, sizeof(T) * n, hipMemcpyDeviceToHost, st));
  return v;
}

void dump_planes(fccf_ctx* c, const std::string& k, const std::vector<Plane>& F) {
  if (!c->debug) return;
  std::vector<float> v;
  for (const Plane& p : F) {
    v.insert(v.end(), p.c, p.c + 3);
    v.insert(v.end(), p.n, p.n + 3);
    v.push_back(p.fps);
    v.push_back((float)p.nvox);
  }
  c->dbg_put(k, v);
}

}  // namespace

namespace {


// FCCF_HOST_TRACE=1 (development): host timestamps of phase B, microseconds since
// the pair's cloud stage was enqueued, printed to stderr when the pair finishes.
struct HostTrace {
  bool on = std::getenv("FCCF_HOST_TRACE") != nullptr;
  clk::time_point t0;
  std::string line;
  void mark(const char* what) {
    if (!on) return;
    char b[64];
    std::snprintf(b, sizeof b, " %s=%.0f", what, std::chrono::duration<double, std::micro>(clk::now() - t0).count());
    line += b;
  }
  void flush() {
    if (on) {
      // absolute start, for merging with a rocprofv3 kernel trace (tools/critical_path.py):
      // steady_clock is CLOCK_MONOTONIC; the BOOTTIME offset is printed beside it
      timespec m, b;
      clock_gettime(CLOCK_MONOTONIC, &m);
      clock_gettime(CLOCK_BOOTTIME, &b);
      const long long off = ((long long)b.tv_sec - m.tv_sec) * 1000000000LL + (b.tv_nsec - m.tv_nsec);
      std::fprintf(stderr, "host trace t0_mono_ns=%lld boot_minus_mono_ns=%lld:%s\n",
                   (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(t0.time_since_epoch()).count(), off,
                   line.c_str());
    }
    line.clear();
  }
};

// What the second half of phase B (fine scores -> fusion) takes over from the
// first half (growing ... fine-verify launch) of the same pair.
struct PhaseB {
  fccf_stats S;
  FineBufs fb{};  // this pair's fine-verification buffers and inputs (a rerun in the sorted form)
  struct {
    const float* s1;
    const OctState* s1_state;
    const float* s2;
    uint32_t n1, n2;
    float res;
  } fine_in{};
  std::vector<TS> ctv[3];
  std::vector<int64_t> counts;
  int E = 0, E_loc = 0, analyse_max = 0;  // E_loc: this rank's block of the E fine evaluations
  float* T_out = nullptr;
  fccf_stats* stats = nullptr;
  clk::time_point t_all, t_fine;
  HostTrace ht;
};

// A phase-B chain: what one pair's phase B1 uses exclusively.  A pipelined batch runs
// two chains on two host threads (alternate pairs), so two pairs' host stages (growth,
// clustering, the LM) overlap, and its last stage group drains with four (chains 2 and 3
// on two more threads, quarter pools); a single registration, or a batch whose ctx needs
// the one-chain form (group, probe, debug, the device growth/LM forms), uses chain 0.
// Chains 0 and 1 share the matching stream sb (each waits for its own work by its event)
// and the fine stream sa[1] (under fine_mutex).  The drain's chains 2 to 4 run after the
// batch's last cloud stage, when the cloud-stage streams sa[0], sa[2] and sa[3] are idle:
// each takes one of them for its matching and fine verification, so the drain's pairs
// spread over the hardware queues instead of queueing on two.
struct Chain {
  Pool* pool;
  Arena* arena2;     // matching scratch
  MatchMail* mm;     // pinned match mailbox
  hipEvent_t ev;     // this chain's matching work on its matching stream is complete
  bool may_redo;     // the stage redo (VG_REDO) runs in place (one chain only)
  hipStream_t sm = nullptr;  // matching stream (null: c->sb)
  hipStream_t sf = nullptr;  // fine-verification stream (null: c->sa[1], shared under fine_mutex)
};

struct BatchRestart {};  // two-chain batch: a stage needs its redo -> the batch again with one chain
struct WorkerAborted {};  // two-chain batch: the other worker failed first

// State of the registration whose clouds occupy CloudSet s.
struct PipeSet {
  PhaseB pb;
  CloudWS w[2];          // this pair's two clouds (inside its stage group's arena)
  int64_t nin[2] = {0, 0};
  uint32_t cap[2] = {1, 1};
  float* cen = nullptr;  // both cloud centroids: cloud k at cen[3k .. 3k+2]
  bool staged = false;   // host inputs copied by stage_inputs (ev_in0 .. ev_in time the H2D)
  clk::time_point t_enq;
  // the pair's device inputs and leaf, for a redo of the stage (VG_REDO)
  const float *in_src = nullptr, *in_tar = nullptr;
  int64_t in_nsrc = 0, in_ntar = 0;
  float leaf = 0.f;
  uint32_t sharded = 0;  // FCCF_SHARDED_* of the cloud stage (row D)
  bool redone = false;   // the stage (this pair's stage group) was redone (VG_REDO)
  // (a group's first slot, PAIRS_MAX * G, only) the stage group's last stage: how many pairs, the entry kernel's
  // arguments (patched into g_seg[P - 1] per call; one per graph, because the fields
  // other than the inputs are set only when that graph is captured) and the centroid
  // sums' scratch
  int group_pairs = 0;
  VGEntry entry[PAIRS_MAX];
  XsBufs xs;
};

PipeSet& pset(fccf_ctx* c, int s) {
  if (!c->cs[s].ws) c->cs[s].ws = new PipeSet();
  return *(PipeSet*)c->cs[s].ws;
}

// A stage group's events live on its first slot: one record per group at the stage's
// end instead of one per pair (every record and cross-stream wait is a packet the
// command processor handles between two stages' kernels).
// ev[0]: the group's inputs have been read; ev[4]: clouds done (records, counts, S1
// octree bounds); the slot's own ev[3] marks its fine verification.
hipEvent_t group_event(fccf_ctx* c, int s, int k) { return c->cs[PAIRS_MAX * (s / PAIRS_MAX)].ev[k]; }

// Host inputs of the pair for CloudSet s: both clouds copied into the set's input
// arena on the ctx's copy stream (ingest.h; the runtime's pageable path), after the
// previous pair on this set has finished reading it (its first pass, before ev[0]).
// ev_in marks the copies; clouds_enqueue makes st0 wait for it.  The pipelined batch
// stages pair i+1 while pair i's cloud stage still runs, so the host link is busy
// while the GPU computes instead of in front of the next cloud stage.
struct Staged {
  const float *src, *tar;
};
Staged stage_inputs(fccf_ctx* c, int s, const float* src, int64_t n_src, const float* tar, int64_t n_tar) {
  auto& cs = c->cs[s];
  c->ingest.init();
  cs.inarena.ensure(12 * (size_t)(n_src + n_tar) + 1024);  // (takes the capture lock to reallocate)
  cs.inarena.reset();
  float* dt = cs.inarena.take_n<float>(3 * (size_t)n_tar);
  float* ds = cs.inarena.take_n<float>(3 * (size_t)n_src);
  hipStream_t su = c->ingest.su;
  guarded_stream_wait(su, group_event(c, s, 0));
  HIP_CHECK(hipEventRecord(cs.ev_in0, su));
  if (n_tar) HIP_CHECK(hipMemcpyAsync(dt, tar, 12 * (size_t)n_tar, hipMemcpyHostToDevice, su));
  if (n_src) HIP_CHECK(hipMemcpyAsync(ds, src, 12 * (size_t)n_src, hipMemcpyHostToDevice, su));
  HIP_CHECK(hipEventRecord(cs.ev_in, su));
  return {ds, dt};
}

// Phase A: enqueue the cloud device stage of the pairs in[0 .. P) (1 <= P <= PAIRS_MAX)
// of stage group G, pair j on slot PAIRS_MAX * G + j (returns at once).  src/tar are device clouds
// (staged ones wait for their slot's ev_in).  Per pair: cloud 0 = driver source = TAR
// file; cloud 1 = driver target = SRC file (:1683).
// exact2: the driver's pass as VG_PRESORTED, eagerly (the redo of a stage whose
// optimistic second pass found its input out of leaf order; rare).
struct PairIn {
  const float *src, *tar;
  int64_t n_src, n_tar;
  bool staged;
};
void clouds_enqueue_group(fccf_ctx* c, int G, int P, const PairIn* in, float leaf, const fccf_params& Pa,
                          bool exact2 = false, bool batch = false) {
  if (P < 1 || P > PAIRS_MAX) throw Error(FCCF_E_INTERNAL, "cloud stage: 1 .. PAIRS_MAX pairs");
  const int S0 = PAIRS_MAX * G;  // the group's first slot
  auto& cg = c->cs[S0];          // the group's arena, stage graphs and fork/join events
  PipeSet& gs = pset(c, S0);
  const int nc = 2 * P;
  // (the centroid sums run on sa[2] beside the face stage, forked inside the stage)
  hipStream_t st0 = c->sa[0];
  hipStream_t sB = st0, ss = c->sa[2];
  // both clouds get the larger capacity (all clouds of a stage, in fact), so their
  // workspaces are laid out alike (batched launches address cloud e at a fixed offset)
  uint32_t capmax = 1;
  for (int j = 0; j < P; ++j)
    capmax = (uint32_t)std::max<int64_t>(capmax, std::max(in[j].n_src, in[j].n_tar));
  // the previous pairs on these slots may still be in fine verification, which reads
  // this workspace (residual clouds, S1 octree state): the stage waits for them
  // (recorded on the fine stream; a wait on an event already complete -- the steady
  // state, where those pairs finished long before -- is skipped: no packet)
  for (int j = 0; j < PAIRS_MAX; ++j) {
    std::lock_guard<std::mutex> lk(capture_mutex());
    if (hipEventQuery(c->cs[S0 + j].ev[3]) != hipSuccess) HIP_CHECK(hipStreamWaitEvent(st0, c->cs[S0 + j].ev[3], 0));
  }
  // (the centroid scratch is carved for BMAX clouds whatever the pair count, so slot
  // j's clouds sit at the same addresses in every stage form, and the per-slot graphs
  // keyed by those addresses -- the S1 replay, fine verification -- keep replaying when
  // a batch ends with a smaller group)
  cg.arena.ensure(nc * cloud_bytes(capmax, false) + exact_sum_bytes(3 * BMAX, capmax) + (1 << 20));
  cg.arena.reset();
  float* cen = cg.arena.take_n<float>(3 * BMAX + 4);
  gs.xs = exact_sum_carve(cg.arena.take(exact_sum_bytes(3 * BMAX, capmax)), 3 * BMAX, capmax);
  // Row D: with a group, large clouds shard their K1 sort after its first rounds
  // (introsort.hip, group.cpp); the stage then runs eagerly (a host step between the
  // sort and the gather of the sorted slices)
  Group* const DG = shard_sort_enabled(c->group, capmax, introsort_rounds(capmax)) ? c->group : nullptr;
  // Row P shards with row D
  Group* const PG = (DG && capmax >= 8192) ? DG : nullptr;
  CloudWS w[BMAX];
  const float* xin[BMAX] = {};
  uint32_t nv[BMAX] = {};
  for (int j = 0; j < P; ++j) {
    PipeSet& ps = pset(c, S0 + j);
    ps.t_enq = clk::now();
    ps.in_src = in[j].src;
    ps.in_tar = in[j].tar;
    ps.in_nsrc = in[j].n_src;
    ps.in_ntar = in[j].n_tar;
    ps.leaf = leaf;
    ps.staged = in[j].staged;
    ps.nin[0] = in[j].n_tar;
    ps.nin[1] = in[j].n_src;
    ps.cap[0] = ps.cap[1] = capmax;
    ps.cen = cen + 6 * j;
    ps.sharded = (DG ? FCCF_SHARDED_SORT : 0u) | (PG ? FCCF_SHARDED_FACES : 0u);
    ps.redone = exact2;
    const float* hin[2] = {in[j].tar, in[j].src};
    for (int k = 0; k < 2; ++k) {
      CloudWS& x = w[2 * j + k];
      x = CloudWS();
      carve_cloud(cg.arena, x, capmax, false);
      x.vg.is.inject = c->d_flags;  // (test hook; a constant pointer per ctx)
      if (DG) {
        x.vg.is.shard_n = (uint32_t)DG->n;
        x.vg.is.shard_rank = (uint32_t)DG->rank;
        x.vg.is.shard_r0 = (uint32_t)shard_sort_r0(DG->n);
        x.vg.is.shard_group = DG;
      }
      x.fb.centroid = cen + 3 * (2 * j + k);  // exact_sum_n writes cloud e's centroid to out[3e .. 3e+2]
      nv[2 * j + k] = (uint32_t)ps.nin[k];
      xin[2 * j + k] = hin[k];
      ps.w[k] = x;
    }
    // host inputs: staged by stage_inputs() into the slot's inarena on the copy stream
    if (in[j].staged) HIP_CHECK(hipStreamWaitEvent(st0, c->cs[S0 + j].ev_in, 0));
  }
  gs.group_pairs = P;
  // (graph keys are compared bytewise: no padding bytes, or their stack garbage forces
  // a re-capture -- about 10 ms -- on most calls)
  struct {
    const void* base;
    size_t acap;
    uint32_t cap;
    int32_t pairs;
    float leaf, fvs, vpt, ct, fine_res;
    int32_t face_bits;
  } key = {cg.arena.base, cg.arena.cap, capmax, P, leaf, Pa.face_voxel_size, Pa.voxel_point_threshold,
           Pa.curvature_threshold, Pa.fine_verify_voxel_size, c->face_fast_bits.load()};
  static_assert(sizeof key == 8 + 8 + 4 + 4 + 5 * 4 + 4, "graph key without padding");
  // The inputs (caller-owned device clouds, or the staged copies of host arrays) are
  // read in place: their pointers and counts are patched into pass 1's entry kernel
  // node.
  {
    const float* x[BMAX];
    uint32_t n[BMAX];
    for (int e = 0; e < BMAX; ++e) {
      x[e] = xin[e < nc ? e : nc - 1];
      n[e] = e < nc ? nv[e] : 0u;
    }
    gs.entry[P - 1].xyz = B4<const float*>(x, BMAX);
    gs.entry[P - 1].n = B4<uint32_t>(n, BMAX);
  }
  VGEntry& entry = gs.entry[P - 1];
  entry.bind();
  // The whole cloud stage is ONE graph: both VoxelGrid passes, then the centroid sums
  // forked onto ss beside the face voxels, joined before the orientation.  ROCm 7.2
  // runs the two branches of a replay concurrently (tools/graph_fork_probe.hip).  The
  // device spans come from s_memrealtime stamps the stage's kernels write (no timing
  // events, which would split the graph: four graphs with events between them were
  // 0.04 ms per registration slower).
  CloudMail* cmail = &host_mail(c)->clouds[S0];  // (the group's slots adjacent); never allocated inside the capture
  const XsBufs xs = gs.xs;
  PatchLayout lay;
  lay.n = VGEntry::LAYOUT_N;
  for (int i = 0; i < lay.n; ++i) {
    lay.idx[i] = VGEntry::layout_idx[i];
    lay.size[i] = VGEntry::layout_size[i];
  }
  // test hook (fccf_debug_graph_mismatch): a replay patched with another layout's
  // workspace pointer, which the replay check must refuse before anything runs
  // A pipelined batch launches its stages eagerly from the helper thread; a single
  // registration replays the graph.  A stage graph's launch holds the runtime for ~250 us
  // of host time (profiles/r05ab), while the two phase-B chains launch their matching
  // and fine kernels: in batches the eager stage read 0.664-0.671 against 0.706-0.716 ms
  // per registration, and single registrations were ~15 us faster with the graph
  // (profiles/r05ac).
  const bool eager = DG != nullptr || exact2 || batch;
  VGEntry wrong;
  void** pargs = entry.args;
  // (armed only for a call that replays: an eager stage checks no layout)
  if (c->graph_mismatch && !eager && cg.g_seg[P - 1].replays(&key, sizeof key)) {
    c->graph_mismatch = false;
    wrong = entry;
    wrong.part.v[0] += 64;
    wrong.bind();
    pargs = wrong.args;
  }
  auto part_b = [&] {
    HIP_CHECK(hipEventRecord(cg.ev[6], sB));
    HIP_CHECK(hipStreamWaitEvent(ss, cg.ev[6], 0));
    const float* d2[BMAX];
    const uint32_t* n2[BMAX];
    for (int e = 0; e < nc; ++e) {
      d2[e] = w[e].ds2;
      n2[e] = w[e].sc + 3;
    }
    exact_sum_n(d2, n2, nc, 3, 3, cen, true, xs, ss);  // compute3DCentroid (:473)
    HIP_CHECK(hipEventRecord(cg.ev[7], ss));
    seg_faces(w, nc, Pa, sB, PG, key.face_bits);
    HIP_CHECK(hipStreamWaitEvent(sB, cg.ev[7], 0));
    face_voxels_orient(capmax, all_of<VoxRec*>(w, nc, [](const CloudWS& x) { return x.planar; }),
                       all_of<FaceBufs>(w, nc, [](const CloudWS& x) { return x.fb; }), sB, nc, cmail,
                       all_of<const uint32_t*>(w, nc, [](const CloudWS& x) { return (const uint32_t*)x.sc; }));
    // fine verification's S1 octree bounds of every pair of the group: one batched replay
    // after k_mail_done, so phase B1 (which polls the mailbox flag) starts without it
    seg_s1_replay(w, P, Pa, sB);
  };
  for (int j = 0; j < P; ++j) __atomic_store_n(&cmail[j].done, 0u, __ATOMIC_RELAXED);  // (set by k_mail_done)
  cg.g_seg[P - 1].run(&key, sizeof key, st0, [&] {
    seg_pass1(w, nc, xin, nv, leaf, st0, &entry);
    seg_downsample(w, nc, leaf, st0, exact2 ? VG_PRESORTED : VG_OPTIMISTIC);
    part_b();
  }, vg_entry_kernel(), pargs, eager, &lay);
  HIP_CHECK(hipEventRecord(cg.ev[0], st0));  // external signal for stage_inputs (the group's inputs have been read)
  HIP_CHECK(hipEventRecord(cg.ev[4], sB));  // clouds done, S1 octree bounds replayed
  HIP_CHECK(hipGetLastError());
}

// One pair on slot s (a group's first slot)
void clouds_enqueue(fccf_ctx* c, int s, const float* src, int64_t n_src, const float* tar, int64_t n_tar,
                    bool staged, float leaf, const fccf_params& P, bool exact2 = false) {
  const PairIn in{src, tar, n_src, n_tar, staged};
  clouds_enqueue_group(c, s / PAIRS_MAX, 1, &in, leaf, P, exact2);
}

// The redo of slot s's stage group (VG_REDO): the same pairs, exact second pass
void clouds_redo(fccf_ctx* c, int s, const fccf_params& P) {
  const int G = s / PAIRS_MAX;
  const int S0 = PAIRS_MAX * G;
  const int np = pset(c, S0).group_pairs;
  PairIn in[PAIRS_MAX];
  for (int j = 0; j < np; ++j) {
    const PipeSet& ps = pset(c, S0 + j);
    in[j] = PairIn{ps.in_src, ps.in_tar, ps.in_nsrc, ps.in_ntar, ps.staged};
  }
  clouds_enqueue_group(c, G, np, in, pset(c, s).leaf, P, true);
}

// Phase B1: everything after the cloud stage of the pair on CloudSet s up to the
// launch of its fine verification (matching on c->sb, fine verification on
// c->sa[1]); phase_b2 collects the fine scores and fuses.  after_clouds() runs as
// soon as the cloud stage has completed (the batch driver enqueues the next pair's
// clouds there).  Between b1 and b2 of a pair the batch driver runs b1 of the next
// pair, so fine verification overlaps the next pair's host stages.
template <class AfterClouds>
void phase_b1(fccf_ctx* c, int s, const fccf_params& P, float T_out[16], fccf_stats* stats,
              AfterClouds&& after_clouds, const Chain& ch) {
  fccf_stats S;
  std::memset(&S, 0, sizeof S);
  PipeSet& ps = pset(c, s);
  CloudWS* w = ps.w;
  S.n_src = ps.nin[1];
  S.n_tar = ps.nin[0];
  if (c->debug) c->dbg.clear();
  const auto t_all = ps.t_enq;
  auto t0 = ps.t_enq;
  hipStream_t st0 = ch.sm ? ch.sm : c->sb;
  // counts and planar records of both clouds: written by k_compact_planar into
  // this set's pinned mailbox, visible once the clouds-done event has completed
  CloudMail& cm = host_mail(c)->clouds[s];
  // growing runs both clouds in parallel right after this wait: one worker besides this
  // thread (keeping more workers spinning slowed growth on the box)
  constexpr int warm_n = 1;
  ch.pool->warm(1000, warm_n);
  if (c->group) {
    // a sharded stage holds collectives: a bounded wait that aborts the group on a
    // peer's failure (group.h), polled under the capture lock
    group_wait_event(c->group, group_event(c, s, 4), true);
  } else {
    // (under the capture lock: with several pairs per stage, a later pair's B1 runs while
    // the helper thread may be capturing the next stage on the stream ev[4] was recorded
    // on, and HIP refuses to synchronize such an event; ev[4] is complete by then)
    if (!mail_wait(&cm.done, 5000.0, [&] { ch.pool->warm(400, warm_n); })) {
      std::lock_guard<std::mutex> lk(capture_mutex());
      HIP_CHECK(hipEventSynchronize(group_event(c, s, 4)));
    }
  }
  uint32_t sc[2][4], fsc[2][4];
  std::memcpy(sc, cm.sc, sizeof sc);
  std::memcpy(fsc, cm.fsc, sizeof fsc);
  if (((fsc[0][1] | fsc[1][1]) & VG_REDO) && !ch.may_redo) throw BatchRestart();
  if ((fsc[0][1] | fsc[1][1]) & VG_REDO) {
    // the driver's pass found main's output out of leaf order (optimistic mode ran no
    // sort): the stage again with the exact second pass.  When a later pair of a stage
    // group raises it, the first pair's B1 has already handed the next group's stage to
    // the helper thread: join that first, so the redo's eager launches cannot land in a
    // graph the helper is capturing (they queue behind that stage on sa[0]; rare)
    c->enq.wait();
    clouds_redo(c, s, P);
    if (c->group) {
      group_wait_event(c->group, group_event(c, s, 4), true);
    } else {
      std::lock_guard<std::mutex> lk(capture_mutex());
      HIP_CHECK(hipEventSynchronize(group_event(c, s, 4)));
    }
    std::memcpy(sc, cm.sc, sizeof sc);
    std::memcpy(fsc, cm.fsc, sizeof fsc);
  }
  // (also a later pair of the group, whose stage was redone with this one; a pair whose
  // B1 had finished before a later pair raised the redo keeps its count of 0)
  if (ps.redone) ++S.stage_redos;
  guarded_stream_wait(st0, group_event(c, s, 4));  // (cheap: the capture lock is free in the steady state)
  std::vector<VoxRec> vox[2];
  for (int k = 0; k < 2; ++k) {
    if (fsc[k][2] <= CloudMail::REC_CAP) vox[k].assign(cm.rec[k], cm.rec[k] + fsc[k][2]);
    else vox[k] = d2h(w[k].planar, fsc[k][2], st0);  // past the mailbox: copy from HBM
  }
  if (fsc[0][2] > CloudMail::REC_CAP || fsc[1][2] > CloudMail::REC_CAP) HIP_CHECK(hipStreamSynchronize(st0));
  // K1's sort checks its invariants on the device (IS_FAULT_*): a violation means the
  // VoxelGrid order may not be std::sort's, so no transform is returned
  if ((fsc[0][1] | fsc[1][1]) & FACE_DEEP) c->face_fast_bits = 32;  // (sticky: the next stages launch four passes)
  if ((fsc[0][1] | fsc[1][1]) & ~(VG_REDO | FACE_DEEP))
    throw Error(FCCF_E_INTERNAL, "VoxelGrid: K1 sort invariant violated (flags cloud 0: " + std::to_string(fsc[0][1]) +
                                     ", cloud 1: " + std::to_string(fsc[1][1]) + ")");
  {  // device spans of the cloud stage: its kernels' s_memrealtime stamps (100 MHz)
    float d[3] = {};
    for (int i = 0; i < 3; ++i)
      d[i] = cm.stamp[i + 1] > cm.stamp[i] ? (float)((double)(cm.stamp[i + 1] - cm.stamp[i]) * 1e-5) : 0.f;
    for (int i = 0; i < 3; ++i) S.dev_ms[i] = d[i];
    S.ms[FCCF_T_DOWNSAMPLE] = d[0] + d[1];
    S.ms[FCCF_T_VOXELFIT] = d[2];
    float h = 0.f;  // the staged host inputs' copy (complete before pass 1 started)
    if (ps.staged) {  // (the mailbox flag does not make the runtime see ev_in complete)
      HIP_CHECK(hipEventSynchronize(c->cs[s].ev_in));
      HIP_CHECK(hipEventElapsedTime(&h, c->cs[s].ev_in0, c->cs[s].ev_in));
    }
    S.ms[FCCF_T_H2D] = h;
  }
  S.m1_tar = sc[0][1];
  S.m1_src = sc[1][1];
  S.leaves1 = fsc[0][0];
  S.leaves2 = fsc[1][0];
  HostTrace ht;
  ht.t0 = ps.t_enq;
  ht.mark("clouds");
  after_clouds();
  ht.mark("next_enq");
  t0 = clk::now();
  S.m_tar = sc[0][3];
  S.m_src = sc[1][3];
  S.vox1 = fsc[0][2]; S.vox2 = fsc[1][2];
  S.res1 = fsc[0][3]; S.res2 = fsc[1][3];
  if (c->debug) {
    const char* dsn[2] = {"ds_tar", "ds_src"};
    for (int k = 0; k < 2; ++k) {
      const std::string s = std::to_string(k + 1);
      auto a = d2h(w[k].ds1, 3 * (size_t)sc[k][1], st0);
      auto b = d2h(w[k].ds2, 3 * (size_t)sc[k][3], st0);
      auto ce = d2h(w[k].fb.centroid, 4, st0);
      auto oc = d2h(w[k].fb.oct, 1, st0);
      auto recs = d2h(w[k].fb.recs, fsc[k][0], st0);
      auto pl = d2h(w[k].fb.flag_planar, fsc[k][0], st0);
      auto rc = d2h(w[k].fb.resid_cnt, fsc[k][0], st0);
      auto res = d2h(w[k].resid, 3 * (size_t)fsc[k][3], st0);
      HIP_CHECK(hipStreamSynchronize(st0));
      c->dbg_put(dsn[k], a);
      c->dbg_put("ds" + s, b);
      ce[3] = 1.f;  // Eigen::Vector4f centroid[3] (unused by the algorithm)
      c->dbg_put("centroid" + s, ce);
      std::vector<double> o = {oc[0].min[0], oc[0].min[1], oc[0].min[2], (double)oc[0].depth};
      c->dbg_put("oct" + s, o);
      std::vector<float> vv;
      for (const VoxRec& r : vox[k]) {
        vv.insert(vv.end(), r.c, r.c + 3);
        vv.insert(vv.end(), r.n, r.n + 3);
        vv.push_back((float)r.count);
        vv.push_back(0.f);
      }
      c->dbg_put("vox" + s, vv);
      std::vector<int32_t> vs;
      std::vector<float> vc;
      for (uint32_t i = 0; i < fsc[k][0]; ++i) {
        vs.push_back(recs[i].count);
        vs.push_back(pl[i] ? 1 : (rc[i] ? 2 : 0));
        vc.push_back(recs[i].curvature);
      }
      c->dbg_put("vstat" + s, vs);
      c->dbg_put("vcurv" + s, vc);
      c->dbg_put("res" + s, res);
    }
  }

  // ---------------- host: growing + selection + select_base
  GrowOut g[2];
  std::vector<Base> base[2];
  double sel_ms[2] = {0.0, 0.0};
  // K4 on the device (grow.hip) when the ctx asks for it and both clouds fit its LDS
  const bool gdev = c->grow_device && fsc[0][2] <= GROW_CAP && fsc[1][2] <= GROW_CAP;
  std::vector<GroupOut> gg[2];
  if (gdev) {
    const VoxRec* dv[2] = {w[0].planar, w[1].planar};
    const uint32_t nvv[2] = {fsc[0][2], fsc[1][2]};
    grow_groups_device(c, dv, nvv, P, st0, gg);
  }
  ch.pool->parallel_for(2, [&](int k) {  // the two clouds are independent
    g[k] = gdev ? select_groups(gg[k], vox[k].data(), P) : grow_and_select(vox[k].data(), (int)vox[k].size(), P);
    const auto tb = clk::now();
    base[k] = select_base(g[k].planes, g[k].theta, P, k + 1);
    sel_ms[k] = g[k].ms_select + ms_since(tb);
  });
  S.groups1 = (int64_t)g[0].groups.size();
  S.groups2 = (int64_t)g[1].groups.size();
  S.planes1 = (int64_t)g[0].planes.size();
  S.planes2 = (int64_t)g[1].planes.size();
  S.bases1 = (int64_t)base[0].size();
  S.bases2 = (int64_t)base[1].size();
  S.ms[FCCF_T_SELECT] = std::max(sel_ms[0], sel_ms[1]);  // range_face + selection + select_base
  S.ms[FCCF_T_GROW] = ms_since(t0) - S.ms[FCCF_T_SELECT];
  ht.mark("grow");
  if (c->debug)
    for (int k = 0; k < 2; ++k) {
      const std::string s = std::to_string(k + 1);
      dump_planes(c, "groups" + s, g[k].groups);
      dump_planes(c, "planes" + s, g[k].planes);
      c->dbg_put("theta" + s, g[k].theta);
      c->dbg_put("galloc" + s, g[k].galloc);
      std::vector<int32_t> bv;
      for (const Base& b : base[k]) {
        int32_t ab;
        std::memcpy(&ab, &b.angle, 4);
        bv.push_back(b.i1); bv.push_back(b.i2); bv.push_back(ab); bv.push_back(b.type < 0 ? -1 : b.type);
      }
      c->dbg_put("bases" + s, bv);
    }

  // ---------------- device: K5 matching + closed-form transforms
  t0 = clk::now();
  const int K = (int)(base[0].size() * base[1].size());
  S.K = K;
  if (g[0].planes.size() > (size_t)MAX_PLANES || g[1].planes.size() > (size_t)MAX_PLANES ||
      base[0].size() > (size_t)MAX_BASES || base[1].size() > (size_t)MAX_BASES)
    throw Error(FCCF_E_INTERNAL, "plane table capacity");
  MatchMail& mm = *ch.mm;
  MatchIn& M = mm.M;  // built in pinned memory: the H2D below is a true async copy
  std::memset(&M, 0, sizeof M);
  for (int k = 0; k < 2; ++k) {
    MPlane* dst = k == 0 ? M.F1 : M.F2;
    for (size_t i = 0; i < g[k].planes.size(); ++i) {
      const Plane& p = g[k].planes[i];
      std::memcpy(dst[i].c, p.c, 12);
      std::memcpy(dst[i].n, p.n, 12);
      dst[i].fps = p.fps;
      dst[i].nvox = p.nvox;
    }
    MBase* bd = k == 0 ? M.B1 : M.B2;
    for (size_t i = 0; i < base[k].size(); ++i) bd[i] = {base[k][i].i1, base[k][i].i2, base[k][i].angle, base[k][i].type};
  }
  M.nF1 = (int)g[0].planes.size();
  M.nF2 = (int)g[1].planes.size();
  M.nB1 = (int)base[0].size();
  M.nB2 = (int)base[1].size();
  M.ang_same = P.included_angle_same_threshold;
  M.third_thr = P.third_plane_threshold;
  M.third_cut = make_cut(P.third_plane_normal_threshold);
  // Sharded search (group.cpp): this rank tests its contiguous block of source pairs;
  // the lists of all ranks are gathered in rank order after the kernels.
  Group* G = c->group;
  if (G) {
    int lo = 0, hi = 0;
    shard_range(M.nB1, G->rank, G->n, &lo, &hi);
    if (lo) std::memmove(M.B1, M.B1 + lo, sizeof(MBase) * (size_t)(hi - lo));
    M.nB1 = hi - lo;
  }
  const int Kloc = M.nB1 * M.nB2;
  const size_t per = (size_t)std::max(1, std::max(0, M.nF1 - 2) * std::max(0, M.nF2 - 2));
  const size_t ccap = std::max<size_t>(1, (size_t)K * per);
  const size_t lists = 3 * ccap * (sizeof(MCand) + sizeof(QTd));
  // transform_cluster's radius search for all three lists on the device (k_cluster_bits)
  const char* cbe = std::getenv("FCCF_CLUSTER_BITS");  // "0": host radius search (tests both paths)
  const bool cbits_on = !(cbe && cbe[0] == '0');
  const bool cdev = c->cluster_device && cbits_on && K > 0;  // f3 on the device (cluster.hip)
  const size_t cl_bytes = cdev ? sizeof(uint64_t) * MatchMail::CB_CAP + 15 * 4 * ccap + 4096 : 0;
  Arena& a2 = *ch.arena2;
  a2.ensure(sizeof(MatchIn) + 3 * 4 * (size_t)std::max(K, 1) + lists * (G ? 2 : 1) + cl_bytes + (1 << 16));
  a2.reset();
  MatchIn* dM = a2.take_n<MatchIn>(1);
  uint32_t* dcnt = a2.take_n<uint32_t>(std::max(K, 1));
  int32_t* dtype = a2.take_n<int32_t>(std::max(K, 1));
  uint32_t* doff = a2.take_n<uint32_t>(std::max(K, 1));
  uint32_t* dtot = a2.take_n<uint32_t>(4);
  MCand* dc[3];
  QTd* dq[3];
  for (int t = 0; t < 3; ++t) {
    dc[t] = a2.take_n<MCand>(ccap);
    dq[t] = a2.take_n<QTd>(ccap);
  }
  uint32_t tot[4] = {0, 0, 0, 0};
  HIP_CHECK(hipMemcpyAsync(dM, &M, sizeof M, hipMemcpyHostToDevice, st0));
  // (k_match_scan writes the totals whenever there are tests: only an empty search
  // needs them zeroed -- one runtime fill kernel fewer on the dependent chain)
  if (Kloc <= 0) HIP_CHECK(hipMemsetAsync(dtot, 0, 16, st0));
  uint64_t* drows = cdev ? a2.take_n<uint64_t>(MatchMail::CB_CAP) : nullptr;
  match_candidates(dM, Kloc, dcnt, dtype, doff, dtot, dc, dq, st0, &mm);
  const float cr2 = (float)((double)P.cluster_distance_threshold * (double)P.cluster_distance_threshold);
  if (cbits_on && K > 0 && !G) {
    cluster_bits(dq, dtot, cr2, make_cut(P.cluster_angel_threshold), P.cluster_number_threshold, &mm, st0, drows);
    if (cdev) cluster_launch(c, dq, dtot, drows, ccap, P, &mm, st0, nullptr, &a2);
  }
  HIP_CHECK(hipGetLastError());
  // totals, K_pass and candidate lists are in the mailbox (sb may also carry the other
  // chain's matching: this chain waits for its own work)
  HIP_CHECK(hipEventRecord(ch.ev, st0));
  if (G) group_wait_event(G, ch.ev);
  else HIP_CHECK(hipEventSynchronize(ch.ev));
  std::vector<QTd> qraw[3];
  int64_t kpass = 0;
  if (G && K > 0) {
    uint32_t tl[3] = {0, 0, 0};
    int64_t kl = 0;
    if (Kloc > 0) {
      std::memcpy(tl, mm.tot, 12);
      kl = mm.kpass;
    }
    MCand* ca[3];
    QTd* qa[3];
    for (int t = 0; t < 3; ++t) {
      ca[t] = a2.take_n<MCand>(ccap);
      qa[t] = a2.take_n<QTd>(ccap);
    }
    uint32_t* dtot_all = a2.take_n<uint32_t>(4);
    group_gather_candidates(G, dq, dc, tl, kl, qa, ca, ccap, tot, dtot_all, &kpass, st0);
    for (int t = 0; t < 3; ++t) {
      dc[t] = ca[t];
      dq[t] = qa[t];
    }
    if (cbits_on) {
      cluster_bits(dq, dtot_all, cr2, make_cut(P.cluster_angel_threshold), P.cluster_number_threshold, &mm, st0,
                   drows);
      if (cdev) cluster_launch(c, dq, dtot_all, drows, ccap, P, &mm, st0, nullptr, &a2);
    }
    HIP_CHECK(hipGetLastError());
    for (int t = 0; t < 3; ++t) qraw[t] = d2h(dq[t], tot[t], st0);
    group_wait(G, st0);
  } else if (K > 0) {
    std::memcpy(tot, mm.tot, 12);
    kpass = mm.kpass;
    bool over = false;
    for (int t = 0; t < 3; ++t) {
      if (tot[t] <= MatchMail::Q_CAP) qraw[t].assign(mm.q[t], mm.q[t] + tot[t]);
      else { qraw[t] = d2h(dq[t], tot[t], st0); over = true; }  // past the mailbox: copy from HBM
    }
    if (over) HIP_CHECK(hipStreamSynchronize(st0));
  }
  S.K_pass = kpass;
  for (int t = 0; t < 3; ++t) S.cand[t] = tot[t];
  S.ms[FCCF_T_MATCH] = ms_since(t0);
  ht.mark("match");
  if (c->debug)
    for (int t = 0; t < 3; ++t) {
      auto cv = d2h(dc[t], tot[t], st0);
      HIP_CHECK(hipStreamSynchronize(st0));
      std::vector<float> v;
      for (const MCand& m : cv) {
        for (int i = 0; i < 3; ++i) {
          v.insert(v.end(), m.R + 3 * i, m.R + 3 * i + 3);
          v.push_back(m.t[i]);
        }
        v.insert(v.end(), {0.f, 0.f, 0.f, 1.f});
      }
      c->dbg_put("cand" + std::to_string(t), v);
    }

  // ---------------- host: clustering, quick_verify (LM), score ranking
  const int transformation_num = (int)(tot[0] + tot[1] + tot[2]);
  const int analyse_max = (int)P.fine_verify_number;
  std::vector<TS> ctv[3];
  std::vector<int64_t> counts = {(int64_t)K, kpass, (int64_t)tot[0], (int64_t)tot[1], (int64_t)tot[2]};
  // clustering of the three types (cheap: the neighbour sets come from the device),
  // then every type's quick_verify + LM in ONE parallel_for (the three lists are
  // independent), then score_range per type
  std::vector<QT> fine[3];
  auto tc = clk::now();
  for (int t = 0; t < 3; ++t) {
    std::vector<QT> qv(qraw[t].size());
    for (size_t i = 0; i < qv.size(); ++i) {
      const QTd& a = qraw[t][i];
      qv[i] = {a.qw, a.qx, a.qy, a.qz, a.tx, a.ty, a.tz, 0u};
    }
    const uint64_t* bits = nullptr;  // the device's neighbour rows, when they fit the mailbox
    if (cbits_on && K > 0) {
      uint64_t words = 0, off = 0;
      for (int u = 0; u < 3; ++u) {
        const uint64_t w = (uint64_t)tot[u] * ((tot[u] + 63) / 64);
        if (u < t) off += w;
        words += w;
      }
      if (words <= MatchMail::CB_CAP) bits = mm.cbits + off;
    }
    const int cluster_num =
        transformation_num ? (int)(P.seclct_cluster_number * (float)qv.size() / (float)transformation_num) : 0;
    if (cdev && mm.cl_stat[t][0] == 0) {  // clustered on the device (cluster_launch)
      if ((int)mm.cl_stat[t][3] != cluster_num) throw Error(FCCF_E_INTERNAL, "device cluster_num differs");
      fine[t] = cluster_results(mm, t);
      counts.push_back((int64_t)mm.cl_stat[t][1]);
      S.fine[t] = (int64_t)fine[t].size();
      continue;
    }
    int64_t ncl = 0;
    transform_cluster(qv, fine[t], cluster_num, P, &ncl, ch.pool, bits);
    counts.push_back(ncl);
    S.fine[t] = (int64_t)fine[t].size();
  }
  S.ms[FCCF_T_CLUSTER] = ms_since(tc);
  ht.mark("cluster");
  tc = clk::now();
  std::vector<std::pair<int, int>> items;  // (type, index) of every fine candidate
  std::vector<TS> res[3];
  std::vector<int> npairs[3];
  for (int t = 0; t < 3; ++t) {
    res[t].resize(fine[t].size());
    npairs[t].resize(fine[t].size());
    for (size_t i = 0; i < fine[t].size(); ++i) items.push_back({t, (int)i});
  }
  if (c->lm_device && !items.empty()) {  // f1: every candidate's quick_verify + LM on the device
    std::vector<QT> qs(items.size());
    for (size_t k = 0; k < items.size(); ++k) qs[k] = fine[items[k].first][(size_t)items[k].second];
    std::vector<m44> Ts(items.size());
    std::vector<float> scs(items.size());
    std::vector<int> nps(items.size());
    verify_items_device(c, qs, g[0].planes, g[1].planes, dM, P, st0, Ts, scs, nps);
    for (size_t k = 0; k < items.size(); ++k) {
      TS& r = res[items[k].first][(size_t)items[k].second];
      r.T = Ts[k];
      r.score = scs[k];
      r.score2 = 0.f;
      npairs[items[k].first][(size_t)items[k].second] = nps[k];
    }
  } else {
    // quick_verify (:680-783) in two parallel passes: every candidate's plane pairs and
    // its score, then the LMs.  The score is the pairs' importance sum under the
    // candidate's own T, before its LM (:778-782), and score_range (:1233-1251) ranks by
    // score alone; only the first analyse_max of each type are used afterwards (fine
    // verification and fusion, :1496-1606), so only their LM results can reach the
    // output: the LM runs for those (<= 3 x fine_verify_number), with T bit-identical
    // to refining every candidate.  A debug ctx refines every candidate (its qv0-2
    // intermediates hold every T).
    std::vector<std::vector<float>> qp(items.size());
    ch.pool->parallel_for((int)items.size(), [&](int k) {
      const int t = items[k].first, i = items[k].second;
      TS& r = res[t][i];
      r.T = T_from_qt(fine[t][i]);
      r.score = quick_verify_pairs(r.T, g[0].planes, g[1].planes, P, qp[(size_t)k], &npairs[t][i]);
      r.score2 = 0.f;
    });
    ht.mark("vpairs");
    std::vector<char> used(items.size(), c->debug ? 1 : 0);
    if (!c->debug) {
      size_t k0 = 0;  // items are type-major
      for (int t = 0; t < 3; ++t) {
        const size_t nt = fine[t].size();
        std::vector<int> ord(nt);
        for (size_t i = 0; i < nt; ++i) ord[i] = (int)i;
        for (size_t i = 0; i + 1 < nt && (int)i < analyse_max; ++i)  // score_range's exchange sort
          for (size_t j = i + 1; j < nt; ++j)
            if (res[t][(size_t)ord[i]].score < res[t][(size_t)ord[j]].score) std::swap(ord[i], ord[j]);
        for (size_t i = 0; i < nt && (int)i < analyse_max; ++i) used[k0 + (size_t)ord[i]] = 1;
        k0 += nt;
      }
    }
    std::vector<int> lm;  // candidates whose pairs reach required_optimize_plane and whose T is used
    for (size_t k = 0; k < items.size(); ++k)
      if (used[k] && (float)npairs[items[k].first][(size_t)items[k].second] >= P.required_optimize_plane)
        lm.push_back((int)k);
    // a thread per LM while the pool has threads for all of them; more LMs than threads:
    // lane groups (lm_solve_batch: SIMD across candidates, each lane bit-identical to
    // lm_solve), about one group per thread
    const int nth = std::max(1, ch.pool->size());
    const int lanes = (int)lm.size() > nth ? lm_batch_lanes() : 1;
    const int per = lanes > 1 ? std::max(1, std::min(lanes, ((int)lm.size() + nth - 1) / nth)) : 1;
    const int ngr = ((int)lm.size() + per - 1) / per;
    ch.pool->parallel_for(ngr, [&](int gi) {
      const int k0 = gi * per, cnt = std::min(per, (int)lm.size() - k0);
      const float* pf[8];
      int np[8];
      double best[8][7];
      for (int j = 0; j < cnt; ++j) {
        const int k = lm[(size_t)(k0 + j)];
        pf[j] = qp[(size_t)k].data();
        np[j] = npairs[items[k].first][(size_t)items[k].second];
      }
      lm_solve_batch(pf, np, cnt, best, lanes);
      for (int j = 0; j < cnt; ++j) {
        const int k = lm[(size_t)(k0 + j)];
        quick_verify_refine(res[items[k].first][(size_t)items[k].second].T, best[j]);
      }
    });
  }
  for (int t = 0; t < 3; ++t) {
    std::vector<float> fdump, qdump;
    for (size_t i = 0; i < fine[t].size(); ++i) {
      const QT& q = fine[t][i];
      const float a[8] = {q.qw, q.qx, q.qy, q.qz, q.tx, q.ty, q.tz, q.alloc ? 1.f : 0.f};
      fdump.insert(fdump.end(), a, a + 8);
      const TS& ts = res[t][i];
      if ((float)npairs[t][i] >= P.required_optimize_plane) ++S.lm_solves;
      ctv[t].push_back(ts);
      for (int a2 = 0; a2 < 4; ++a2)
        for (int b2 = 0; b2 < 4; ++b2) qdump.push_back(ts.T.m[a2][b2]);
      qdump.push_back(ts.score);
      qdump.push_back((float)npairs[t][i]);
    }
    // score_range (:1233-1251): exchange sort; only the first analyse_max positions matter
    auto& cv = ctv[t];
    for (size_t i = 0; i + 1 < cv.size() && (int)i < analyse_max; ++i)
      for (size_t j = i + 1; j < cv.size(); ++j)
        if (cv[i].score < cv[j].score) std::swap(cv[i], cv[j]);
    c->dbg_put("fine" + std::to_string(t), fdump);
    c->dbg_put("qv" + std::to_string(t), qdump);
  }
  S.ms[FCCF_T_VERIFY] = ms_since(tc);
  ht.mark("verify");

  // ---------------- device: K7 fine verify of the top analyse_max per type
  // (launched here on c->sa[1]; phase_b2 waits for it and fuses)
  PhaseB& pb = ps.pb;
  pb.t_fine = clk::now();
  std::vector<m44> evals;
  for (int t = 0; t < 3; ++t)
    for (int i = 0; i < (int)ctv[t].size() && i < analyse_max; ++i) evals.push_back(ctv[t][i].T);
  const int E = (int)evals.size();
  if (E > MAX_EVAL) throw Error(FCCF_E_INTERNAL, "too many fine-verify evaluations");
  // Sharded fine verification (group.cpp, row F): this rank scores its contiguous block
  // [flo, fhi) of the E evaluations; the blocks are all-gathered in rank order.
  Group* const FG = (c->group && c->group->n > 1) ? c->group : nullptr;
  int flo = 0, fhi = E;
  if (FG) shard_range(E, FG->rank, FG->n, &flo, &fhi);
  const int El = fhi - flo;
  hipStream_t sf = ch.sf ? ch.sf : c->sa[1];
  // the fine stream is shared by the chains: one chain's launch sequence (waits, graph
  // replay or capture, event records) at a time
  std::unique_lock<std::mutex> flk(c->fine_mutex);
  if (El > 0) {
    fccf::Arena& a3 = c->cs[s].arena3;
    const uint32_t n1 = (uint32_t)S.res1, n2 = (uint32_t)S.res2;
    const int E = El;  // this rank's evaluations: evals[flo, fhi)
    const size_t nk = (size_t)E * (n1 + n2);
    const size_t af2 = aggr_floats(n2);
    const size_t need = 12 * (size_t)E * n2 + 4 * E * af2 + sizeof(OctState) * (E + 1) +
                        (3 * 8 + 3 * 4 + 4 + 8) * (nk + 1) + 64 * 5 + sizeof(m44) * E + 64 +
                        sort_scratch_bytes((uint32_t)std::max<size_t>(nk, 1)) + 40 * 256 +
                        exact_sum_bytes(E, n1 + n2) + 256;
    a3.ensure(need);
    a3.reset();
    FineBufs fb;
    fb.s2t = a3.take_n<float>(3 * (size_t)E * n2);
    fb.aggr2 = a3.take_n<float>((size_t)E * af2);
    fb.state = a3.take_n<OctState>(E + 1);
    fb.k0 = a3.take_n<uint64_t>(nk);
    fb.k1 = a3.take_n<uint64_t>(nk);
    fb.k2 = a3.take_n<uint64_t>(nk);
    fb.v0 = a3.take_n<uint32_t>(nk);
    fb.v1 = a3.take_n<uint32_t>(nk);
    fb.v2 = a3.take_n<uint32_t>(nk);
    fb.pts = a3.take_n<uint32_t>(MAX_EVAL);
    fb.starts = a3.take_n<uint32_t>(nk + 1);
    fb.term = a3.take_n<float>(nk + 1);
    fb.range = a3.take_n<uint32_t>(2 * MAX_EVAL);
    fb.nseg_e = a3.take_n<uint32_t>(2 * MAX_EVAL);
    fb.similar = a3.take_n<float>(MAX_EVAL);
    fb.all = a3.take_n<float>(MAX_EVAL);
    fb.scal = a3.take_n<uint32_t>(16);
    fb.scores = a3.take_n<float>(E);
    fb.T = a3.take_n<m44>(E);
    fb.ss = sort_scratch_carve(a3.take(sort_scratch_bytes((uint32_t)std::max<size_t>(nk, 1))),
                               (uint32_t)std::max<size_t>(nk, 1));
    fb.xs = exact_sum_carve(a3.take(exact_sum_bytes(E, n1 + n2)), E, n1 + n2);
    FineMail& fm = host_mail(c)->fine[s];
    __atomic_store_n(&fm.done, 0u, __ATOMIC_RELAXED);  // (set by the launch's last kernel)
    fm.stamp[0] = fm.stamp[1] = 0;
    std::memcpy(fm.T, evals.data() + flo, sizeof(m44) * E);  // pinned staging: async H2D
    HIP_CHECK(hipMemcpyAsync(fb.T, fm.T, sizeof(m44) * E, hipMemcpyHostToDevice, sf));
    // the leaf form: LDS per evaluation unless the ctx met an evaluation with more leaves
    // than it holds (sticky), or the group's sharded gather reads the sorted form's words
    const int fmode = FG ? FV_LEAVES_SORTED : fine_mode_env(c->fine_sorted.load() ? 1 : 0);
    const uint32_t fcap = fine_lds_cap_env();
    struct {
      const void* base;
      size_t acap;
      const void *r1, *r2, *s1state;
      uint32_t n1, n2;
      int32_t E;
      float res;
      int32_t mode;
      uint32_t cap;
    } fkey = {a3.base, a3.cap, w[0].resid, w[1].resid, w[0].fstate, n1, n2, E, P.fine_verify_voxel_size, fmode, fcap};
    static_assert(sizeof fkey == 5 * 8 + 6 * 4, "graph key without padding");
    // what phase_b2 needs to rerun the batch in the sorted form (FV_ERR_LDS)
    pb.fb = fb;
    pb.fine_in = {w[0].resid, w[0].fstate, w[1].resid, n1, n2, P.fine_verify_voxel_size};
    ht.mark("fine_setup");
    // S1 octree bounds replayed (with the clouds); ev[4]'s stream may be capturing the next pair's clouds
    guarded_stream_wait(sf, group_event(c, s, 4));
    if (FG) HIP_CHECK(hipEventRecord(c->cs[s].tev[4], sf));  // (otherwise the mailbox stamps time it)
    c->cs[s].g_fine.run(&fkey, sizeof fkey, sf, [&] {
      fine_verify_batch(w[0].resid, n1, w[0].fstate, w[1].resid, n2, E, (double)P.fine_verify_voxel_size, fb, sf,
                        &fm, fmode, fcap);
    }, nullptr, nullptr, false);
    HIP_CHECK(hipGetLastError());
    if (FG) HIP_CHECK(hipEventRecord(c->cs[s].tev[5], sf));
    if (FG) group_fine_gather(FG, s, fb.scores, El, fb.scal + 7, sf);
    HIP_CHECK(hipEventRecord(c->cs[s].ev[3], sf));  // fine verification of this set's pair done
    ht.mark("fine_launched");
  } else if (E > 0 && FG) {  // no evaluation in this rank's block: it still takes part in the gather
    group_fine_gather(FG, s, nullptr, 0, nullptr, sf);
    HIP_CHECK(hipEventRecord(c->cs[s].ev[3], sf));
  }
  flk.unlock();
  pb.S = S;
  for (int t = 0; t < 3; ++t) pb.ctv[t] = std::move(ctv[t]);
  pb.counts = std::move(counts);
  pb.E = E;
  pb.E_loc = El;
  pb.analyse_max = analyse_max;
  pb.T_out = T_out;
  pb.stats = stats;
  pb.t_all = t_all;
  pb.ht = ht;
  pb.S.shard_ranks = c->group ? c->group->n : 1;
  pb.S.sharded = ps.sharded | (G && G->n > 1 && K > 0 ? FCCF_SHARDED_SEARCH : 0u) | (FG && E > 0 ? FCCF_SHARDED_FINE : 0u);
  if (c->group) b1_done(c->group);  // this pair's CH_MATCH / CH_FINE collectives are issued
}

// Phase B2: the fine scores of the pair on CloudSet s (launched by phase_b1), the
// score sums over all types and fusion (:1539-1606).
// batch: the pair is part of a pipelined batch, where the stage group's arena (the
// residual clouds and S1 octree state fine verification reads) may already be
// recycled by a later stage group when this runs.  An evaluation past the LDS form's
// capacity (FV_ERR_LDS) then cannot be rerun from that arena: phase_b2 returns true
// without a result, and the batch registers the pair again after its last pair
// (sorted form, sticky on the ctx).  A single registration reruns eagerly.
bool phase_b2(fccf_ctx* c, int s, bool batch = false) {
  PipeSet& ps = pset(c, s);
  PhaseB& pb = ps.pb;
  fccf_stats& S = pb.S;
  auto& ctv = pb.ctv;
  auto& counts = pb.counts;
  const int E = pb.E, analyse_max = pb.analyse_max;
  float* T_out = pb.T_out;
  std::vector<float> scores(E, 0.f);
  if (E > 0) {
    // scores and the error word are in the mailbox; with a group the fine stream holds the
    // score gather: a bounded wait.  ev[3] is recorded on the fine stream sa[1], which the
    // other phase-B chains capture g_fine on (a new capture whenever the pair sizes
    // change), so the event fallback queries under the capture lock, as phase_b1 does
    // for ev[4]
    if (c->group) group_wait_event(c->group, c->cs[s].ev[3]);
    else if (!mail_wait(&host_mail(c)->fine[s].done, 3000.0)) guarded_event_sync(c->cs[s].ev[3]);
    uint32_t err = 0;
    if (c->group && c->group->n > 1) {  // every rank's block, gathered in rank order
      group_fine_scores(c->group, s, E, scores.data(), &err);
    } else {
      FineMail& fm = host_mail(c)->fine[s];
      err = fm.err;
      if ((err & FV_ERR_LDS) && batch) {
        c->fine_sorted = true;
        pb.ht.flush();
        return true;
      }
      if (err & FV_ERR_LDS) {
        // an evaluation had more leaves than the LDS form holds: the batch again in the
        // sorted form, eagerly, and the ctx keeps that form (the scores are the same)
        c->fine_sorted = true;
        hipStream_t sf = c->sa[1];
        const auto& fi = pb.fine_in;
        fine_verify_batch(fi.s1, fi.n1, fi.s1_state, fi.s2, fi.n2, E, (double)fi.res, pb.fb, sf, &fm, FV_LEAVES_SORTED);
        HIP_CHECK(hipGetLastError());
        HIP_CHECK(hipStreamSynchronize(sf));
        err = fm.err;
        ++S.fine_reruns;
      }
      std::memcpy(scores.data(), fm.scores, 4 * (size_t)E);
    }
    if (err) throw Error(FCCF_E_INTERNAL, "fine_verify: >= 2^24 points in one evaluation");
    if (pb.E_loc > 0) {
      // the device span from the launch's own stamps (100 MHz; the timing events around
      // the launch only with a group, whose sharded gather follows it on the stream)
      const FineMail& fm = host_mail(c)->fine[s];
      float d = 0.f;
      if (!(c->group && c->group->n > 1)) {  // (the events are recorded with a sharded fine stage only)
        d = fm.stamp[0] && fm.stamp[1] >= fm.stamp[0] ? (float)((double)(fm.stamp[1] - fm.stamp[0]) * 1e-5) : 0.f;
      } else {
        guarded_event_sync(c->cs[s].tev[5]);  // (sa[1]: see ev[3] above)
        HIP_CHECK(hipEventElapsedTime(&d, c->cs[s].tev[4], c->cs[s].tev[5]));
      }
      S.dev_ms[3] = d;
    }
  }
  S.fine_evals = E;
  S.ms[FCCF_T_FINE] = ms_since(pb.t_fine);
  pb.ht.mark("fine");
  pb.ht.flush();

  // ---------------- host: score sums (over all types) and fusion (:1539-1606)
  auto t0 = clk::now();
  {
    int e = 0;
    for (int t = 0; t < 3; ++t) {
      std::vector<float> fv;
      for (int i = 0; i < (int)ctv[t].size() && i < analyse_max; ++i, ++e) {
        ctv[t][i].score2 = scores[e];
        for (int a = 0; a < 4; ++a)
          for (int b = 0; b < 4; ++b) fv.push_back(ctv[t][i].T.m[a][b]);
        fv.push_back(ctv[t][i].score);
        fv.push_back(ctv[t][i].score2);
      }
      c->dbg_put("fv" + std::to_string(t), fv);
    }
  }
  std::vector<High> tmp;
  const m44 T = fuse_types(ctv, analyse_max, &tmp);
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) T_out[4 * i + j] = T.m[i][j];
  S.ms[FCCF_T_FUSE] = ms_since(t0);
  S.ms_total = ms_since(pb.t_all);
  if (c->probe.on()) {
    HIP_CHECK(device_sync_guarded());
    probe_collect(c->probe);
  }
  S.graph_captures = c->cs[s].g_fine.captures;
  for (auto& g : c->cs[s].g_seg) S.graph_captures += g.captures;
  counts.push_back(S.lm_solves);
  counts.push_back(0);
  if (c->debug) {
    std::vector<float> hv;
    for (const High& h : tmp) {
      const float a[8] = {h.qt.qw, h.qt.qx, h.qt.qy, h.qt.qz, h.qt.tx, h.qt.ty, h.qt.tz, h.score};
      hv.insert(hv.end(), a, a + 8);
    }
    c->dbg_put("high", hv);
    c->dbg_put("T", T_out, 16);
    c->dbg_put("counts", counts);
  }
  if (pb.stats) *pb.stats = S;
  return false;
}

void reset_capture_counts(fccf_ctx* c) {
  for (auto& cs : c->cs) {
    for (auto& g : cs.g_seg) g.captures = 0;
    cs.g_fine.captures = 0;
  }
}

struct ProbeGuard {
  explicit ProbeGuard(Probe* p) {
    g_probe = p;
    p->armed.clear();
  }
  ~ProbeGuard() { g_probe = nullptr; }
};

}  // namespace

void grow_groups_device(fccf_ctx* c, const VoxRec* const dvox[2], const uint32_t nv[2], const fccf_params& P,
                        hipStream_t st, std::vector<GroupOut> out[2]) {
  // one contiguous block per cloud: the D2H of a block brings every output back
  const auto block_words = [](uint32_t n) { return (size_t)n * 22 + 64; };  // 4-byte words
  const size_t w0 = block_words(std::max(nv[0], 1u)), w1 = block_words(std::max(nv[1], 1u));
  c->arena2.ensure(4 * (w0 + w1) + 1024);
  c->arena2.reset();
  uint32_t* blk[2] = {c->arena2.take_n<uint32_t>(w0), c->arena2.take_n<uint32_t>(w1)};
  GrowIn in[2];
  GrowDev od[2];
  auto carve = [](uint32_t* b, uint32_t n, GrowDev& d) {
    n = std::max(n, 1u);
    d.gna = (double*)b;  // 8-byte aligned first
    uint32_t* q = b + 2 * (size_t)n;
    d.gac = (float*)q; q += 3 * (size_t)n;
    d.gan = (float*)q; q += 3 * (size_t)n;
    d.gfps = (float*)q; q += n;
    d.gsum = (float*)q; q += 7 * (size_t)n;
    d.ghead = q; q += n;
    d.gtail = q; q += n;
    d.gnmem = q; q += n;
    d.galloc = q; q += n;
    d.next = q; q += n;
    d.ng = q;
  };
  for (int k = 0; k < 2; ++k) {
    in[k] = {dvox[k], nv[k]};
    carve(blk[k], nv[k], od[k]);
  }
  GrowParams gp;
  gp.cut1 = make_cut(P.normal_vector_threshold1);
  gp.cut2 = make_cut(P.normal_vector_threshold2);
  gp.l1 = P.parameter_l1;
  gp.k1 = P.parameter_k1;
  gp.l2 = P.parameter_l2;
  gp.k2 = P.parameter_k2;
  grow_device(in, od, gp, st);
  HIP_CHECK(hipGetLastError());
  uint32_t* h = (uint32_t*)c->pinned.get(4 * (w0 + w1));
  HIP_CHECK(hipMemcpyAsync(h, blk[0], 4 * w0, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipMemcpyAsync(h + w0, blk[1], 4 * w1, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  for (int k = 0; k < 2; ++k) {
    GrowDev hd;
    carve(h + (k ? w0 : 0), nv[k], hd);
    const uint32_t G = nv[k] ? *hd.ng : 0u;
    if (G > nv[k]) throw Error(FCCF_E_INTERNAL, "k_grow: group count out of range");
    out[k].assign(G, GroupOut());
    for (uint32_t g = 0; g < G; ++g) {
      GroupOut& o = out[k][g];
      std::memcpy(o.ac, hd.gac + 3 * (size_t)g, 12);
      std::memcpy(o.an, hd.gan + 3 * (size_t)g, 12);
      o.fps = hd.gfps[g];
      o.alloc = hd.galloc[g] != 0;
      // a group's members are the first gnmem nodes of the list from its head: a group
      // merged into another keeps its tail, which the absorbing group extends later
      const uint32_t nm = hd.gnmem[g];
      if (nm == 0 || nm > nv[k]) throw Error(FCCF_E_INTERNAL, "k_grow: member count out of range");
      o.mem.resize(nm);
      uint32_t m = hd.ghead[g];
      for (uint32_t q = 0; q < nm; ++q) {
        if (m >= nv[k]) throw Error(FCCF_E_INTERNAL, "k_grow: member list corrupt");
        o.mem[q] = (int)m;
        m = hd.next[m];
      }
    }
  }
}

void verify_items_device(fccf_ctx* c, const std::vector<QT>& qs, const std::vector<Plane>& F1,
                         const std::vector<Plane>& F2, const MatchIn* dM, const fccf_params& P, hipStream_t st,
                         std::vector<m44>& T, std::vector<float>& score, std::vector<int>& npairs) {
  const int n = (int)qs.size();
  if (n == 0) return;
  const size_t in_b = sizeof(QTd) * (size_t)n, out_b = (16 * 4 + 4 + 4 + 4) * (size_t)n;
  c->arena_v.ensure(in_b + out_b + 8 * 256);  // (each take is 256-byte aligned)
  c->arena_v.reset();
  QTd* dq = c->arena_v.take_n<QTd>(n);
  VerifyOut o;
  o.T = c->arena_v.take_n<float>(16 * (size_t)n);
  o.score = c->arena_v.take_n<float>(n);
  o.npairs = c->arena_v.take_n<int32_t>(n);
  o.status = c->arena_v.take_n<uint32_t>(n);
  uint8_t* h = (uint8_t*)c->pinned.get(in_b + out_b);
  QTd* hq = (QTd*)h;
  for (int k = 0; k < n; ++k) hq[k] = {qs[k].qw, qs[k].qx, qs[k].qy, qs[k].qz, qs[k].tx, qs[k].ty, qs[k].tz, qs[k].alloc};
  HIP_CHECK(hipMemcpyAsync(dq, hq, in_b, hipMemcpyHostToDevice, st));
  // quick_verify's face-point sums (FCCF.cpp:688-697): float accumulation, int each step
  int fs1 = 0, fs2 = 0;
  for (const Plane& f : F1) fs1 = (int)((float)fs1 + f.fps);
  for (const Plane& f : F2) fs2 = (int)((float)fs2 + f.fps);
  VerifyIn in;
  in.q = dq;
  in.planes = dM;
  in.fs12 = fs1 + fs2;
  in.qcut = make_cut(P.quick_verify_angel_threshold);
  in.dist_thr = P.quick_verify_distance_threshold;
  in.required = P.required_optimize_plane;
  verify_device(in, n, o, st);
  HIP_CHECK(hipGetLastError());
  float* hT = (float*)(h + in_b);
  float* hs = hT + 16 * (size_t)n;
  int32_t* hn = (int32_t*)(hs + n);
  uint32_t* hst = (uint32_t*)(hn + n);
  HIP_CHECK(hipMemcpyAsync(hT, o.T, 64 * (size_t)n, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipMemcpyAsync(hs, o.score, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipMemcpyAsync(hn, o.npairs, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipMemcpyAsync(hst, o.status, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
  for (int k = 0; k < n; ++k) {
    if (hst[k]) {  // an argument beyond the device reduction: this candidate on the host
      T[k] = T_from_qt(qs[k]);
      score[k] = quick_verify(T[k], F1, F2, P, &npairs[k]);
      continue;
    }
    std::memcpy(&T[k].m[0][0], hT + 16 * (size_t)k, 64);
    score[k] = hs[k];
    npairs[k] = hn[k];
  }
}

void cluster_launch(fccf_ctx* c, QTd* const dq[3], const uint32_t* dtot, const uint64_t* drows, size_t ccap,
                    const fccf_params& P, MatchMail* mail, hipStream_t st, const int* cluster_num, Arena* scratch) {
  Arena& a2 = scratch ? *scratch : c->arena2;
  ClusterIn in{};
  ClusterOut out{};
  for (int t = 0; t < 3; ++t) {
    in.q[t] = dq[t];
    out.cseed[t] = a2.take_n<uint32_t>(ccap);
    out.csize[t] = a2.take_n<uint32_t>(ccap);
    out.bx[t] = a2.take_n<uint32_t>(ccap);
    out.bid[t] = a2.take_n<uint32_t>(ccap);
    out.emit[t] = a2.take_n<uint32_t>(ccap);
  }
  in.rows = drows;
  in.totals = dtot;
  in.cb_cap = MatchMail::CB_CAP;
  in.min_n = P.cluster_number_threshold;
  in.sel = P.seclct_cluster_number;
  if (cluster_num) {
    in.cnum_given = *cluster_num;
    in.has_cnum = 1;
  }
  out.cap = (uint32_t)std::min<size_t>(ccap, 0xFFFFFFFFu);
  out.stat = &mail->cl_stat[0][0];
  out.fine = &mail->cl_fine[0][0];
  out.fcap = MatchMail::CL_FCAP;
  // cluster_num <= sel (n <= total), so sel + 2 averaging waves per type cover the
  // emission loop (:1205-1229, at most cluster_num + 1); a type past them is the host's
  const double cmax = cluster_num ? (double)*cluster_num : (double)P.seclct_cluster_number;
  out.egrid = (uint32_t)std::clamp(cmax + 2.0, 2.0, (double)MatchMail::CL_FCAP);
  cluster_device(in, out, st);
}

MatchMail* match_mail(fccf_ctx* c) { return &host_mail(c)->match; }

std::vector<QT> cluster_results(const MatchMail& mm, int t) {
  std::vector<QT> f(mm.cl_stat[t][2]);
  for (size_t e = 0; e < f.size(); ++e) {
    const QTd& a = mm.cl_fine[t][e];
    f[e] = {a.qw, a.qx, a.qy, a.qz, a.tx, a.ty, a.tz, a.alloc};
  }
  return f;
}

void pipeline_release(fccf_ctx* c) {
  for (auto& cs : c->cs) {
    delete (PipeSet*)cs.ws;
    cs.ws = nullptr;
  }
}

// Chain k of nchains (see Chain).
Chain chain_of(fccf_ctx* c, int k, int nchains) {
  HostMail* hm = host_mail(c);
  if (nchains <= 1) return Chain{&c->pool, &c->arena2, &hm->match, c->ev_match[0], true};
  for (int i = 0; i < 5; ++i)
    if (!c->bpool[i]) c->bpool[i].reset(new Pool(std::max(1, c->pool.size() / (i < 2 ? 2 : 4))));
  switch (k) {
    case 0: return Chain{c->bpool[0].get(), &c->arena2, &hm->match, c->ev_match[0], false};
    case 1: return Chain{c->bpool[1].get(), &c->arena2b, &hm->match2, c->ev_match[1], false};
    case 2: return Chain{c->bpool[2].get(), &c->arena2c, &hm->match3, c->ev_match[2], false, c->sa[0], c->sa[0]};
    case 3: return Chain{c->bpool[3].get(), &c->arena2d, &hm->match4, c->ev_match[3], false, c->sa[2], c->sa[2]};
    default: return Chain{c->bpool[4].get(), &c->arena2e, &hm->match5, c->ev_match[4], false, c->sa[3], c->sa[3]};
  }
}

// Bytes this rank has received through its group's exchanges so far, per channel
// (fccf_stats.xch_bytes: the difference over a call).
void group_rx(const Group* g, int64_t rx[3]) {
  for (int k = 0; k < 3; ++k) rx[k] = g && g->tr ? g->tr->rx_bytes[k].load() : 0;
}
void put_xch_bytes(const Group* g, const int64_t rx0[3], fccf_stats* stats, int n) {
  if (!stats) return;
  int64_t rx1[3];
  group_rx(g, rx1);
  for (int i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) stats[i].xch_bytes[k] = rx1[k] - rx0[k];
}

void run_register(fccf_ctx* c, const float* src, int64_t n_src, const float* tar, int64_t n_tar, bool on_device,
                  float leaf, const fccf_params& P, float T_out[16], fccf_stats* stats) {
  group_check(c->group);
  int64_t rx0[3];
  group_rx(c->group, rx0);
  ProbeGuard probe_guard(&c->probe);
  reset_capture_counts(c);
  if (c->group) order_reset(c->group);
  if (!on_device) {
    const Staged in = stage_inputs(c, 0, src, n_src, tar, n_tar);
    src = in.src;
    tar = in.tar;
  }
  clouds_enqueue(c, 0, src, n_src, tar, n_tar, !on_device, leaf, P);
  phase_b1(c, 0, P, T_out, stats, [] {}, chain_of(c, 0, 1));
  phase_b2(c, 0);
  put_xch_bytes(c->group, rx0, stats, 1);
}

void run_register_batch(fccf_ctx* c, int n, const float* const* src, const int64_t* n_src, const float* const* tar,
                        const int64_t* n_tar, bool on_device, float leaf, const fccf_params& P, float* T_out,
                        fccf_stats* stats, int nchains) {
  if (n <= 0) return;
  group_check(c->group);
  ProbeGuard probe_guard(&c->probe);
  reset_capture_counts(c);
  // On an error (an exception out of a pair's phase B) the helper thread may still be
  // staging or enqueueing the next pair with references into this frame: join it, and
  // let the device finish what was enqueued, before the frame unwinds.
  struct JoinOnUnwind {
    fccf_ctx* c;
    bool armed = true;
    ~JoinOnUnwind() {
      if (!armed) return;
      // with a group, this rank will not finish the batch's collectives: abort the group
      // (its communicators end, so neither the helper thread's collectives nor the device
      // synchronisation below can wait for peers), and a helper thread waiting at the
      // collective-order gate throws instead of hanging (Group::om)
      if (c->group) group_abort(c->group, "a pipelined batch failed on this rank");
      try {
        c->enq.wait();
      } catch (...) {
      }
      (void)device_sync_guarded();
    }
  } join_guard{c};
  if (c->group) order_reset(c->group);
  // Pairs per cloud stage: five -- their ten clouds in the same launches, so the
  // sort's dependent rounds and the face stage's small launches are paid once for all
  // (DESIGN.md §12, §13); FCCF_PAIR_BATCH=1..5.  With a group the sharded stages gather
  // every cloud of the stage in one exchange (group.cpp); a probe keeps the batch's own
  // launch width (its byte counts sum over every cloud of a launch, probe.h).
  const char* pb_env = std::getenv("FCCF_PAIR_BATCH");
  const int pp_env = pb_env ? std::atoi(pb_env) : PAIRS_DEFAULT;
  const int PP = std::max(1, std::min(PAIRS_MAX, pp_env));
  const int ng = (n + PP - 1) / PP;  // stage groups; group g uses slots PAIRS_MAX (g & 1) + j
  auto cnt = [&](int g) { return std::min(PP, n - g * PP); };
  auto slot = [&](int i) { return PAIRS_MAX * ((i / PP) & 1) + i % PP; };
  // Host inputs: group g+1's clouds are staged on the copy stream at the start of
  // group g (from the helper thread: the pageable copy blocks its caller), so the host
  // link works while group g's cloud stage runs.
  std::vector<Staged> in(on_device ? 0 : n);
  auto dsrc = [&](int i) { return on_device ? src[i] : in[(size_t)i].src; };
  auto dtar = [&](int i) { return on_device ? tar[i] : in[(size_t)i].tar; };
  auto stage_group = [c, &in, src, n_src, tar, n_tar, cnt, slot, PP](int g) {
    HIP_CHECK(hipSetDevice(c->device));
    for (int j = 0; j < cnt(g); ++j) {
      const int i = g * PP + j;
      in[(size_t)i] = stage_inputs(c, slot(i), src[i], n_src[i], tar[i], n_tar[i]);
    }
  };
  auto enq_group = [c, n_src, n_tar, on_device, leaf, &P, dsrc, dtar, cnt, PP](int g) {
    HIP_CHECK(hipSetDevice(c->device));  // a no-op after the first call on the helper thread
    PairIn pin[PAIRS_MAX];
    for (int j = 0; j < cnt(g); ++j) {
      const int i = g * PP + j;
      pin[j] = PairIn{dsrc(i), dtar(i), n_src[i], n_tar[i], !on_device};
    }
    clouds_enqueue_group(c, g & 1, cnt(g), pin, leaf, P, false, true);
  };
  std::vector<int> redo;  // pairs to register again after the batch (phase_b2)
  if (!on_device) stage_group(0);
  enq_group(0);
  if (nchains <= 1) {
    const Chain ch = chain_of(c, 0, 1);
    // pair i: B1 (its clouds done -> the first pair of a group enqueues the next group's
    // clouds -> host stages -> launch fine verification), then B2 of pair i-1, whose fine
    // verification ran on the GPU during pair i's host stages
    for (int g = 0; g < ng; ++g) {
      c->enq.wait();  // this group's cloud stage is fully enqueued (its events recorded)
      if (!on_device && g + 1 < ng) {
        if (c->probe.on()) stage_group(g + 1);
        else c->enq.submit([stage_group, g] { stage_group(g + 1); });
      }
      for (int j = 0; j < cnt(g); ++j) {
        const int i = g * PP + j;
        phase_b1(c, slot(i), P, T_out + 16 * (size_t)i, stats ? stats + i : nullptr, [&] {
          if (j != 0 || g + 1 >= ng) return;
          // the next group's cloud stage is enqueued from a helper thread while this
          // thread runs the host stages (launches are ~60 us of host time); probed
          // runs stay on this thread (the probe's launch records are not shared)
          if (c->probe.on()) {
            enq_group(g + 1);
          } else {
            // with a group, the helper's gathers of the next stage (CH_CLOUD) wait until
            // every pair of this stage has issued its B1 collectives (CH_MATCH / CH_FINE):
            // one issue order on every rank
            if (c->group) order_need(c->group, (int64_t)g * PP + cnt(g));
            c->enq.submit([enq_group, g] { enq_group(g + 1); });  // (after the staging task, which submit() joins first)
          }
        }, ch);
        if (i > 0 && phase_b2(c, slot(i - 1), true)) redo.push_back(i - 1);
      }
    }
    c->enq.wait();
    if (phase_b2(c, slot(n - 1), true)) redo.push_back(n - 1);
  } else {
    // Two chains (four in the drain, below): pair i's phase B on worker i % 2 (this thread and c->b1w), each worker
    // running B1 of its next pair before B2 of its previous one (fine verification
    // overlaps).  The first pair of a group still enqueues the next group's stage, which
    // recycles the slots of the group before: it waits until every pair of that group has
    // finished B1 (B1 reads the slot's workspace; B2 does not).  The other worker's pairs
    // of a group wait until the group's stage is enqueued.
    struct Sync {
      std::mutex m;
      std::condition_variable cv;
      int submitted = 1;   // groups whose cloud-stage enqueue has been handed to the helper
      int ready = 0;       // groups whose cloud stage is fully enqueued
      std::vector<int> b1; // per group: pairs whose phase B1 has finished
      std::vector<char> b2;  // per pair: phase B2 has finished
      bool failed = false;
    } sy;
    sy.b1.assign((size_t)ng, 0);
    sy.b2.assign((size_t)n, 0);
    auto wait_until = [&sy](auto pred) {
      std::unique_lock<std::mutex> lk(sy.m);
      sy.cv.wait(lk, [&] { return sy.failed || pred(); });
      if (sy.failed) throw WorkerAborted();
    };
    auto update = [&sy](auto f) {
      {
        std::lock_guard<std::mutex> lk(sy.m);
        f();
      }
      sy.cv.notify_all();
    };
    const Chain chains[5] = {chain_of(c, 0, 2), chain_of(c, 1, 2), chain_of(c, 2, 5), chain_of(c, 3, 5),
                             chain_of(c, 4, 5)};
    // The last stage group drains with a chain per pair: after its stage nothing else is
    // left for the GPU, and its pairs' phase B would otherwise run two after two on each
    // chain (FCCF_DRAIN4=0: two chains throughout, tests)
    const char* d4e = std::getenv("FCCF_DRAIN4");  // (read per batch: tests switch it)
    const bool drain4_env = !(d4e && d4e[0] == '0');
    const int glast = ng - 1;
    const bool drain4 = drain4_env && ng >= 2 && cnt(glast) >= 3;
    const int nextra = drain4 ? cnt(glast) - 2 : 0;  // workers 2 .. 1 + nextra
    // pairs 2 to 4 of the last group go to workers 2 to 4
    auto drained = [&](int i) { return drain4 && i / PP == glast && i % PP >= 2; };
    auto worker = [&](int k) {
      HIP_CHECK(hipSetDevice(c->device));
      const Chain& ch = chains[k];
      int pending = -1;  // this worker's pair whose B2 is still to run
      if (k >= 2) {  // one pair of the last group: B1, then its B2
        const int i = glast * PP + k;
        if (i >= n) return;
        wait_until([&] { return sy.ready > glast; });
        // the slot's previous pair (two groups back) ran on worker 0 or 1: its B2 reads
        // the slot's phase-B state and fine mailbox, which this B1 rewrites
        if (i >= 2 * PP) wait_until([&] { return sy.b2[(size_t)(i - 2 * PP)] != 0; });
        phase_b1(c, slot(i), P, T_out + 16 * (size_t)i, stats ? stats + i : nullptr, [] {}, ch);
        update([&] { ++sy.b1[(size_t)glast]; });
        if (phase_b2(c, slot(i), true)) update([&] { redo.push_back(i); });
        return;
      }
      for (int i = k; i < n; i += 2) {
        if (drained(i)) continue;
        const int g = i / PP, j = i % PP;
        if (j == 0) {
          wait_until([&] { return sy.submitted > g; });
          c->enq.wait();  // group g's cloud stage is fully enqueued
          update([&] { sy.ready = g + 1; });
          if (!on_device && g + 1 < ng) {
            // staging group g+1 re-records the input events of group g-1's slots, which
            // that group's B1 reads (the H2D time): after it
            if (g >= 1) wait_until([&] { return sy.b1[(size_t)g - 1] >= cnt(g - 1); });
            c->enq.submit([stage_group, g] { stage_group(g + 1); });
          }
        } else {
          wait_until([&] { return sy.ready > g; });
        }
        phase_b1(c, slot(i), P, T_out + 16 * (size_t)i, stats ? stats + i : nullptr, [&] {
          if (j != 0 || g + 1 >= ng) return;
          if (g >= 1) wait_until([&] { return sy.b1[(size_t)g - 1] >= cnt(g - 1); });
          c->enq.submit([enq_group, g] { enq_group(g + 1); });
          update([&] { sy.submitted = g + 2; });
        }, ch);
        update([&] { ++sy.b1[(size_t)g]; });
        if (pending >= 0) {
          const bool rd = phase_b2(c, slot(pending), true);
          update([&] {
            if (rd) redo.push_back(pending);
            sy.b2[(size_t)pending] = 1;
          });
        }
        pending = i;
      }
      if (pending >= 0) {
        const bool rd = phase_b2(c, slot(pending), true);
        update([&] {
          if (rd) redo.push_back(pending);
          sy.b2[(size_t)pending] = 1;
        });
      }
    };
    auto guarded_worker = [&](int k) {
      try {
        worker(k);
      } catch (...) {
        update([&] { sy.failed = true; });
        throw;
      }
    };
    c->b1w.submit([&guarded_worker] { guarded_worker(1); });
    AsyncTask* helpers[4] = {&c->b1w, &c->b1w2, &c->b1w3, &c->b1w4};
    for (int k = 2; k < 2 + nextra; ++k) helpers[k - 1]->submit([&guarded_worker, k] { guarded_worker(k); });
    std::exception_ptr err[5];
    try {
      guarded_worker(0);
    } catch (...) {
      err[0] = std::current_exception();
    }
    for (int h = 0; h < 1 + nextra; ++h) {
      try {
        helpers[h]->wait();  // (always joined before this frame unwinds)
      } catch (...) {
        err[h + 1] = std::current_exception();
      }
    }
    // the first failure counts (a stage redo before anything else: the batch reruns with
    // one chain); the other worker's WorkerAborted only says it stopped
    bool restart = false;
    std::exception_ptr first;
    for (auto& e : err) {
      if (!e) continue;
      try {
        std::rethrow_exception(e);
      } catch (const BatchRestart&) {
        restart = true;
      } catch (const WorkerAborted&) {
      } catch (...) {
        if (!first) first = e;
      }
    }
    if (first) std::rethrow_exception(first);
    if (restart) throw BatchRestart();
    if (err[0] || err[1] || err[2] || err[3] || err[4]) throw Error(FCCF_E_INTERNAL, "pipelined batch: a phase-B worker stopped");
    c->enq.wait();
    std::sort(redo.begin(), redo.end());
  }
  join_guard.armed = false;
  if (c->group) order_reset(c->group);
  // pairs whose fine verification overflowed the LDS form (phase_b2): registered again
  // alone, now in the sorted form (the ctx keeps it), with the same result bits
  for (int i : redo) {
    fccf_stats* si = stats ? stats + i : nullptr;
    run_register(c, src[i], n_src[i], tar[i], n_tar[i], on_device, leaf, P, T_out + 16 * (size_t)i, si);
    if (si) ++si->fine_reruns;
  }
}

// The batch with two phase-B chains where the ctx allows it; a stage redo found by a two-chain batch (rare: an input out of leaf order after
// main's VoxelGrid) reruns the whole batch with one chain, whose redo runs in place.
void run_register_batch_any(fccf_ctx* c, int n, const float* const* src, const int64_t* n_src,
                            const float* const* tar, const int64_t* n_tar, bool on_device, float leaf,
                            const fccf_params& P, float* T_out, fccf_stats* stats) {
  const char* pb_env = std::getenv("FCCF_PAIR_BATCH");
  const int pp = pb_env ? std::atoi(pb_env) : PAIRS_DEFAULT;
  const bool two = pp >= 2 && n >= 2 && !c->group && !c->probe.on() && !c->debug &&
                   !c->grow_device && !c->lm_device;
  int64_t rx0[3];
  group_rx(c->group, rx0);
  if (two) {
    try {
      run_register_batch(c, n, src, n_src, tar, n_tar, on_device, leaf, P, T_out, stats, 2);
      put_xch_bytes(c->group, rx0, stats, n);
      return;
    } catch (const BatchRestart&) {
    }
  }
  run_register_batch(c, n, src, n_src, tar, n_tar, on_device, leaf, P, T_out, stats, 1);
  put_xch_bytes(c->group, rx0, stats, n);
}

}  // namespace fccf

using namespace fccf;

// With a group attached, a registration that fails on this rank leaves its peers in
// collectives it will not join: the group is aborted (group.h), so every rank returns
// an error within the group's time limit instead of hanging.
template <class F>
static int guarded2(fccf_ctx* c, F&& f) {
  try {
    HIP_CHECK(hipSetDevice(c->device));
    f();
    return FCCF_OK;
  } catch (const Error& e) {
    c->last_error = e.what();
    if (c->group) group_abort(c->group, e.what());
    return e.code;
  } catch (const std::bad_alloc&) {
    if (c->group) group_abort(c->group, "out of host memory");
    return FCCF_E_OOM;
  } catch (...) {
    if (c->group) group_abort(c->group, "internal error");
    return FCCF_E_INTERNAL;
  }
}

static int check_args(fccf_ctx* c, const float* s, int64_t ns, const float* t, int64_t nt, float leaf, float* T) {
  if (!c || !T || (!s && ns) || (!t && nt) || ns < 0 || nt < 0 || ns > 0x7FFFFFFF || nt > 0x7FFFFFFF ||
      !(leaf > 0.f) || !std::isfinite(leaf))
    return FCCF_E_ARG;
  return FCCF_OK;
}

extern "C" int fccf_register(fccf_ctx* c, const float* src, int64_t ns, const float* tar, int64_t nt, float leaf,
                             const fccf_params* params, float T[16], fccf_stats* stats) {
  if (int rc = check_args(c, src, ns, tar, nt, leaf, T)) return rc;
  fccf_params P;
  if (params) P = *params;
  else fccf_params_default(&P);
  return guarded2(c, [&] { run_register(c, src, ns, tar, nt, false, leaf, P, T, stats); });
}

extern "C" int fccf_register_device(fccf_ctx* c, const float* d_src, int64_t ns, const float* d_tar, int64_t nt,
                                    float leaf, const fccf_params* params, float T[16], fccf_stats* stats) {
  if (int rc = check_args(c, d_src, ns, d_tar, nt, leaf, T)) return rc;
  fccf_params P;
  if (params) P = *params;
  else fccf_params_default(&P);
  return guarded2(c, [&] { run_register(c, d_src, ns, d_tar, nt, true, leaf, P, T, stats); });
}

extern "C" int fccf_register_batch(fccf_ctx* c, int n, const float* const* src, const int64_t* ns,
                                   const float* const* tar, const int64_t* nt, int on_device, float leaf,
                                   const fccf_params* params, float* T, fccf_stats* stats) {
  if (!c || n < 0 || (n && (!src || !ns || !tar || !nt || !T))) return FCCF_E_ARG;
  for (int i = 0; i < n; ++i)
    if (int rc = check_args(c, src[i], ns[i], tar[i], nt[i], leaf, T + 16 * (size_t)i)) return rc;
  fccf_params P;
  if (params) P = *params;
  else fccf_params_default(&P);
  return guarded2(c, [&] { run_register_batch_any(c, n, src, ns, tar, nt, on_device != 0, leaf, P, T, stats); });
}
