// group.cpp — multi-GPU inside libfccf (SURVEY.md §8(b) fccf_group_create, §8(e)).
// One process per GPU; every rank holds communicators created from one
// ncclUniqueId that rank 0 made and the caller distributed out of band.
//
// What is sharded:
//  * K5, the coplane-pair correspondence search (FCCF.cpp:1410-1428): source pairs B1
//    in contiguous blocks (shard_range); each rank tests its block against all target
//    pairs on its GPU, then the per-type candidate lists are gathered in rank order:
//    the counts by one all-gather, the variable-length lists by an all-gather-v.  The
//    reference's loop is b1-major, so the concatenation is the unsharded list.
//  * F, fine_verify (:785-839): the <= 16 evaluations (the top fine_verify_number
//    candidates of each type) in contiguous blocks; each rank scores its block on
//    its GPU and the scores are all-gathered in rank order, so every rank fuses the
//    same scores in the same order.
//  * D, K1's std::sort (:1668-1678): after the replicated first rounds each rank
//    partitions and finishes only the segments in its range of the sort; the sorted
//    slices are all-gathered in rank order (shard_gather_sorted), every cloud of a
//    stage group in one exchange.
//  * P, the 1 m face stage (:470-534): each rank fits its Morton range of leaves; leaf
//    records, planar flags and residual points are all-gathered in rank order
//    (face_voxels_sharded).
// Everything else is replicated: growth, selection, clustering and the LM are
// sequential and deterministic, so every rank computes the same T with no further
// exchange.
//
// Transports: RCCL (RcclTransport: an exchange's all-gather-v ops are packed into one
// count-padded block per rank, moved by ONE ncclAllGather, and unpacked by one batched
// copy kernel -- Transport::allgatherv_multi), or virtual ranks (LocalTransport, test
// hook): n contexts
// of one process on one device exchange through a shared device staging buffer under
// host barriers -- the same gather logic with n > 1, where RCCL itself would refuse
// two ranks on one GPU.
//
// Failure handling (Group::aborted): every host wait that may depend on a peer is
// bounded and polls the transport's async error; a failing rank aborts its
// communicators (ncclCommAbort), and every rank returns FCCF_E_RCCL within the bound.
#include "group.h"

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ctx.h"
#include "kernels.h"

namespace fccf {

#define NCCL_CHECK(x)                                                                      \
  do {                                                                                     \
    ncclResult_t r_ = (x);                                                                 \
    if (r_ != ncclSuccess) throw ::fccf::Error(FCCF_E_RCCL, std::string(#x) + ": " + ncclGetErrorString(r_)); \
  } while (0)

// An open ncclGroupStart is always closed: a call that fails inside the group ends it
// (ncclGroupEnd) before the error propagates, so the communicator stays usable.
struct NcclGroup {
  bool open = false;
  NcclGroup() {
    NCCL_CHECK(ncclGroupStart());
    open = true;
  }
  void end() {
    open = false;
    NCCL_CHECK(ncclGroupEnd());
  }
  ~NcclGroup() {
    if (open) (void)ncclGroupEnd();
  }
};

// The communicators stay valid while a thread uses them: comm() is taken through a Use
// (per channel: the abort flag checked and a user count raised under the channel's
// mutex), and abort() frees a communicator (ncclCommAbort) only once no thread is
// inside an enqueue on it -- at once when idle, otherwise by the last user leaving.
// abort() never waits for a user, so it cannot hang behind an enqueue that waits for a
// peer.  (the helper thread could use a communicator that abort had freed.)
struct RcclTransport : Transport {
  Group* g;
  struct Chan {
    std::mutex m;
    int users = 0;
    bool pending = false;  // aborted while in use: the last user frees it
  } chan[CH_COUNT];
  std::atomic<bool> dead{false};
  explicit RcclTransport(Group* g_) : g(g_) {}
  struct Use {
    RcclTransport* t;
    int ch;
    ncclComm_t c;
    Use(RcclTransport* t_, int ch_) : t(t_), ch(ch_) {
      std::lock_guard<std::mutex> lk(t->chan[ch].m);
      c = t->g->comm[ch];
      if (t->dead || !c) throw Error(FCCF_E_RCCL, "group aborted: " + group_why(t->g));
      ++t->chan[ch].users;
    }
    ~Use() {
      std::lock_guard<std::mutex> lk(t->chan[ch].m);
      if (--t->chan[ch].users == 0 && t->chan[ch].pending) t->free_comm(ch);
    }
  };
  void free_comm(int ch) {  // (the channel's mutex held, no user)
    ncclComm_t& c = g->comm[ch];
    if (c) (void)ncclCommAbort(c);  // (also frees the communicator)
    c = nullptr;
    chan[ch].pending = false;
  }
  void allgatherv(int ch, const void* send, void* recv, const size_t* counts, const size_t* offs,
                  hipStream_t st) override {
    GatherOp op{send, recv, counts, offs};
    allgatherv_multi(ch, &op, 1, st);
  }
  void allgather(int ch, const void* send, void* recv, size_t bytes, hipStream_t st) override {
    Use u(this, ch);
    NCCL_CHECK(ncclAllGather(send, recv, bytes, ncclUint8, u.c, st));
    rx_bytes[ch] += (int64_t)bytes * (g->n - 1);
  }
  int async_error() override {
    for (int ch = 0; ch < CH_COUNT; ++ch) {
      std::lock_guard<std::mutex> lk(chan[ch].m);
      ncclComm_t c = g->comm[ch];
      if (!c || chan[ch].pending) continue;
      ncclResult_t r = ncclSuccess;
      if (ncclCommGetAsyncError(c, &r) != ncclSuccess) return (int)ncclInternalError;
      if (r != ncclSuccess && r != ncclInProgress) return (int)r;
    }
    return 0;
  }
  void abort() override {
    dead = true;
    for (int ch = 0; ch < CH_COUNT; ++ch) {
      std::lock_guard<std::mutex> lk(chan[ch].m);
      if (chan[ch].users == 0) free_comm(ch);
      else chan[ch].pending = true;
    }
  }
};

// Virtual ranks of one process on one device: every collective is host-synchronous.
// Each channel has its own barrier and staging (channels are driven from different
// host threads of a rank, like the separate communicators of the RCCL form).
struct LocalHub {
  int n;
  std::atomic<bool> aborted{false};
  struct Chan {
    std::mutex m;
    std::condition_variable cv;
    int arrived = 0;
    uint64_t gen = 0;
    char* stage = nullptr;
    size_t cap = 0, need = 0;
  } ch[CH_COUNT];
  explicit LocalHub(int n_) : n(n_) {}
  ~LocalHub() {
    for (Chan& c : ch)
      if (c.stage) (void)hipFree(c.stage);
  }
  void abort() {
    aborted = true;
    for (Chan& c : ch) {
      std::lock_guard<std::mutex> lk(c.m);
      c.cv.notify_all();
    }
  }
  // bounded: a rank that never arrives (its call failed without aborting, a dead
  // peer) ends the wait after timeout_s; an aborted hub ends it at once
  void barrier(int k, double timeout_s) {
    Chan& c = ch[k];
    std::unique_lock<std::mutex> lk(c.m);
    if (aborted) throw Error(FCCF_E_RCCL, "virtual-rank group aborted by a rank");
    const uint64_t my = c.gen;
    if (++c.arrived == n) {
      c.arrived = 0;
      ++c.gen;
      c.cv.notify_all();
      return;
    }
    const bool ok = c.cv.wait_for(lk, std::chrono::duration<double>(timeout_s),
                                  [&] { return c.gen != my || aborted.load(); });
    if (c.gen != my) return;
    if (aborted) throw Error(FCCF_E_RCCL, "virtual-rank group aborted by a rank");
    (void)ok;
    throw Error(FCCF_E_RCCL, "virtual-rank group: a rank did not reach the collective within the time limit");
  }
};

struct LocalTransport : Transport {
  Group* g;
  explicit LocalTransport(Group* g_) : g(g_) {}
  void allgatherv(int ch, const void* send, void* recv, const size_t* counts, const size_t* offs,
                  hipStream_t st) override {
    LocalHub::Chan& C = g->hub->ch[ch];
    size_t total = 0;
    for (int r = 0; r < g->n; ++r) total = std::max(total, offs[r] + counts[r]);
    HIP_CHECK(hipStreamSynchronize(st));  // this rank's send data is complete
    {
      std::lock_guard<std::mutex> lk(C.m);
      C.need = std::max(C.need, total);
    }
    g->hub->barrier(ch, g->timeout_s);
    if (g->rank == 0 && C.need > C.cap) {  // one rank grows the staging, between barriers
      // (hipFree synchronises the device: not while another rank's thread captures a graph)
      std::lock_guard<std::mutex> lk(capture_mutex());
      if (C.stage) HIP_CHECK(hipFree(C.stage));
      C.stage = nullptr;
      C.cap = 0;
      if (hipMalloc((void**)&C.stage, C.need) != hipSuccess) throw Error(FCCF_E_OOM, "virtual-rank staging");
      C.cap = C.need;
    }
    g->hub->barrier(ch, g->timeout_s);
    if (counts[g->rank]) {  // (on st: the legacy null stream would also wait for the other ranks' streams)
      HIP_CHECK(hipMemcpyAsync(C.stage + offs[g->rank], send, counts[g->rank], hipMemcpyDeviceToDevice, st));
      HIP_CHECK(hipStreamSynchronize(st));
    }
    g->hub->barrier(ch, g->timeout_s);
    // every rank's part except its own (in place: an all-gather-v may send from its recv buffer)
    for (int r = 0; r < g->n; ++r)
      if (r != g->rank && counts[r])
        HIP_CHECK(hipMemcpyAsync((char*)recv + offs[r], C.stage + offs[r], counts[r], hipMemcpyDeviceToDevice, st));
    if (counts[g->rank] && (const char*)send != (const char*)recv + offs[g->rank])
      HIP_CHECK(hipMemcpyAsync((char*)recv + offs[g->rank], send, counts[g->rank], hipMemcpyDeviceToDevice, st));
    HIP_CHECK(hipStreamSynchronize(st));
    g->hub->barrier(ch, g->timeout_s);  // (the staging is rewritten by the next collective)
    for (int r = 0; r < g->n; ++r)
      if (r != g->rank) rx_bytes[ch] += (int64_t)counts[r];
  }
  void allgather(int ch, const void* send, void* recv, size_t bytes, hipStream_t st) override {
    std::vector<size_t> counts((size_t)g->n, bytes), offs((size_t)g->n);
    for (int r = 0; r < g->n; ++r) offs[(size_t)r] = (size_t)r * bytes;
    allgatherv(ch, send, recv, counts.data(), offs.data(), st);
  }
  int async_error() override { return g->hub->aborted ? 1 : 0; }
  void abort() override { g->hub->abort(); }
};

// ------------------------------------------------------------ packed all-gather-v

namespace {
// Up to CP_MAX (src, dst, bytes) copies per launch, passed by value (kernel arguments):
// blockIdx.y = copy, the x blocks stride over it in 16-byte words when src, dst and the
// size allow, else in 4-byte words, else bytes (a uniform branch per copy).
constexpr int CP_MAX = 64;
struct CopyDesc {
  const char* src;
  char* dst;
  uint64_t bytes;
};
struct CopyBatch {
  int n;
  CopyDesc d[CP_MAX];
};

__global__ void __launch_bounds__(256) k_copy_batch(CopyBatch b) {
  if ((int)blockIdx.y >= b.n) return;
  const CopyDesc c = b.d[blockIdx.y];
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t al = (uint64_t)c.src | (uint64_t)c.dst | c.bytes;
  if ((al & 15u) == 0) {
    const uint4* s = (const uint4*)c.src;
    uint4* d = (uint4*)c.dst;
    for (uint64_t i = t; i < c.bytes / 16; i += stride) d[i] = s[i];
  } else if ((al & 3u) == 0) {
    const uint32_t* s = (const uint32_t*)c.src;
    uint32_t* d = (uint32_t*)c.dst;
    for (uint64_t i = t; i < c.bytes / 4; i += stride) d[i] = s[i];
  } else {
    for (uint64_t i = t; i < c.bytes; i += stride) c.dst[i] = c.src[i];
  }
}

void copy_batch(const std::vector<CopyDesc>& v, hipStream_t st) {
  for (size_t i = 0; i < v.size(); i += CP_MAX) {
    CopyBatch b;
    b.n = (int)std::min<size_t>(CP_MAX, v.size() - i);
    uint64_t mx = 0;
    for (int j = 0; j < b.n; ++j) {
      b.d[j] = v[i + (size_t)j];
      mx = std::max<uint64_t>(mx, b.d[j].bytes);
    }
    const unsigned gx = (unsigned)std::min<uint64_t>(64, std::max<uint64_t>(1, (mx / 16 + 4095) / 4096));
    k_copy_batch<<<dim3(gx, (unsigned)b.n), 256, 0, st>>>(b);
    HIP_CHECK(hipGetLastError());
  }
}

size_t pad16(size_t x) { return (x + 15) & ~size_t(15); }

// (the scratch of channel ch at >= the sizes; its previous use on st has finished first)
char* grow(char*& p, size_t& cap, size_t need, hipStream_t st) {
  if (need <= cap) return p;
  HIP_CHECK(hipStreamSynchronize(st));
  std::lock_guard<std::mutex> lk(capture_mutex());  // (hipFree may synchronise the device)
  if (p) (void)hipFree(p);
  p = nullptr;
  cap = 0;
  need = std::max(need, (size_t)1 << 20);
  if (hipMalloc((void**)&p, need) != hipSuccess) throw Error(FCCF_E_OOM, "hipMalloc (all-gather scratch)");
  cap = need;
  return p;
}
}  // namespace

Transport::~Transport() { free_scratch(); }

void Transport::free_scratch() {
  for (Scratch& s : scratch) {
    if (s.pack) (void)hipFree(s.pack);
    if (s.recv) (void)hipFree(s.recv);
    s = Scratch{};
  }
}

void Transport::allgatherv_multi(int ch, const GatherOp* ops, int nops, hipStream_t st) {
  const int n = n_ranks, me = my_rank;
  if (nops <= 0) return;
  // every rank's block: its parts of the ops, each 16-byte aligned; M = the largest block
  std::vector<size_t> inner((size_t)n * nops);
  size_t M = 0;
  for (int r = 0; r < n; ++r) {
    size_t o = 0;
    for (int i = 0; i < nops; ++i) {
      inner[(size_t)r * nops + i] = o;
      o += pad16(ops[i].counts[r]);
    }
    M = std::max(M, o);
  }
  if (M == 0) return;
  Scratch& S = scratch[ch];
  char* pack = grow(S.pack, S.cap_pack, M, st);
  char* recv = grow(S.recv, S.cap_recv, M * (size_t)n, st);
  std::vector<CopyDesc> cp;
  for (int i = 0; i < nops; ++i)
    if (ops[i].counts[me])
      cp.push_back(CopyDesc{(const char*)ops[i].send, pack + inner[(size_t)me * nops + i], ops[i].counts[me]});
  copy_batch(cp, st);
  allgather(ch, pack, recv, M, st);
  cp.clear();
  for (int i = 0; i < nops; ++i)
    for (int r = 0; r < n; ++r) {
      const size_t c = ops[i].counts[r];
      if (!c) continue;
      char* dst = (char*)ops[i].recv + ops[i].offs[r];
      if (r == me) {
        if ((const char*)ops[i].send != dst) cp.push_back(CopyDesc{(const char*)ops[i].send, dst, c});
      } else {
        cp.push_back(CopyDesc{recv + (size_t)r * M + inner[(size_t)r * nops + i], dst, c});
      }
    }
  copy_batch(cp, st);
}

// ------------------------------------------------------------ failure handling

void group_abort(Group* g, const std::string& why) {
  if (!g) return;
  {
    // the reason is written before the flag becomes visible: a reader that
    // sees `aborted` and then takes why_m finds it complete
    std::lock_guard<std::mutex> lk(g->why_m);
    if (g->aborted.load(std::memory_order_acquire)) return;
    g->abort_why = why;
    g->aborted.store(true, std::memory_order_release);
  }
  // a dead peer (the silent test hook) leaves its transport alone: the others find
  // out at their time limit
  if (!g->fail_silent && g->tr) g->tr->abort();
  order_abort(g);
}

std::string group_why(Group* g) {
  std::lock_guard<std::mutex> lk(g->why_m);
  return g->abort_why;
}

void group_check(Group* g) {
  if (g && g->aborted) throw Error(FCCF_E_RCCL, "group aborted (" + group_why(g) + "); destroy and recreate it");
}

namespace {
template <class Q>
void bounded_wait(Group* g, Q query, const char* what) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  for (uint64_t k = 0;; ++k) {
    const hipError_t e = query();
    if (e == hipSuccess) return;
    if (e != hipErrorNotReady) {
      const std::string m = std::string(what) + ": " + hipGetErrorString(e);
      group_abort(g, m);
      throw Error(FCCF_E_HIP, m);
    }
    if (g->aborted) throw Error(FCCF_E_RCCL, "group aborted (" + group_why(g) + ")");
    if ((k & 31) == 31) {
      if (const int ae = g->tr->async_error()) {
        const std::string m = std::string(what) + ": transport failed asynchronously (" + std::to_string(ae) + ")";
        group_abort(g, m);
        throw Error(FCCF_E_RCCL, m);
      }
      if (std::chrono::duration<double>(clk::now() - t0).count() > g->timeout_s) {
        const std::string m = std::string(what) + ": no completion within the group's time limit (" +
                              std::to_string(g->timeout_s) + " s)";
        group_abort(g, m);
        throw Error(FCCF_E_RCCL, m);
      }
    }
    // spin briefly (these waits are on the registration's critical path), then yield
    if (k < 4096) {
#if defined(__x86_64__)
      __builtin_ia32_pause();
#endif
    } else if (k < 65536) {
      std::this_thread::yield();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }
}
}  // namespace

void group_wait(Group* g, hipStream_t st) {
  bounded_wait(g, [st] { return hipStreamQuery(st); }, "group stream wait");
}

void group_wait_event(Group* g, hipEvent_t ev, bool capture_lock) {
  if (capture_lock)
    bounded_wait(g, [ev] {
      std::lock_guard<std::mutex> lk(capture_mutex());
      return hipEventQuery(ev);
    }, "group event wait");
  else
    bounded_wait(g, [ev] { return hipEventQuery(ev); }, "group event wait");
}

void group_fail_point(Group* g, int site) {
  if (!g || g->fail_at != site) return;
  g->fail_at = 0;
  throw Error(FCCF_E_RCCL, "injected failure at collective site " + std::to_string(site));
}

void shard_range(int n, int rank, int world, int* lo, int* hi) {
  const int q = n / world, r = n % world;
  *lo = rank * q + std::min(rank, r);
  *hi = *lo + q + (rank < r ? 1 : 0);
}

void group_gather_candidates(Group* g, QTd* const q_loc[3], MCand* const c_loc[3], const uint32_t tot_loc[3],
                             int64_t kpass_loc, QTd* const q_all[3], MCand* const c_all[3], size_t cap,
                             uint32_t tot_all[3], uint32_t* d_tot_all, int64_t* kpass_all, hipStream_t st) {
  const int n = g->n;
  group_fail_point(g, GROUP_FAIL_MATCH);
  uint32_t* h = g->h_cnt;  // pinned: [0..3] this rank's counts, [4 ..] every rank's
  h[0] = tot_loc[0];
  h[1] = tot_loc[1];
  h[2] = tot_loc[2];
  h[3] = (uint32_t)kpass_loc;
  HIP_CHECK(hipMemcpyAsync(g->d_cnt, h, 16, hipMemcpyHostToDevice, st));
  g->tr->allgather(CH_MATCH, g->d_cnt, g->d_cnt + 4, 16, st);
  HIP_CHECK(hipMemcpyAsync(h + 4, g->d_cnt + 4, 16 * (size_t)n, hipMemcpyDeviceToHost, st));
  group_wait(g, st);
  int64_t kp = 0;
  size_t off[3] = {0, 0, 0};
  std::vector<size_t> base((size_t)n * 3);
  for (int r = 0; r < n; ++r) {
    for (int t = 0; t < 3; ++t) {
      base[(size_t)r * 3 + t] = off[t];
      off[t] += h[4 + 4 * r + t];
    }
    kp += h[4 + 4 * r + 3];
  }
  for (int t = 0; t < 3; ++t) {
    if (off[t] > cap) throw Error(FCCF_E_INTERNAL, "sharded search: gathered candidates exceed capacity");
    tot_all[t] = (uint32_t)off[t];
  }
  *kpass_all = kp;
  // all-gather-v of each type's quaternion records and matrices, rank-ordered: the six
  // lists in one exchange
  std::vector<size_t> cnt((size_t)n * 6), offs((size_t)n * 6);
  GatherOp ops[6];
  for (int t = 0; t < 3; ++t) {
    size_t* cq = cnt.data() + (size_t)n * (2 * t);
    size_t* oq = offs.data() + (size_t)n * (2 * t);
    size_t* cc = cnt.data() + (size_t)n * (2 * t + 1);
    size_t* oc = offs.data() + (size_t)n * (2 * t + 1);
    for (int r = 0; r < n; ++r) {
      cq[r] = (size_t)h[4 + 4 * r + t] * sizeof(QTd);
      oq[r] = base[(size_t)r * 3 + t] * sizeof(QTd);
      cc[r] = (size_t)h[4 + 4 * r + t] * sizeof(MCand);
      oc[r] = base[(size_t)r * 3 + t] * sizeof(MCand);
    }
    ops[2 * t] = GatherOp{q_loc[t], q_all[t], cq, oq};
    ops[2 * t + 1] = GatherOp{c_loc[t], c_all[t], cc, oc};
  }
  g->tr->allgatherv_multi(CH_MATCH, ops, 6, st);
  h[0] = tot_all[0];
  h[1] = tot_all[1];
  h[2] = tot_all[2];
  h[3] = 0;
  HIP_CHECK(hipMemcpyAsync(d_tot_all, h, 16, hipMemcpyHostToDevice, st));
  group_wait(g, st);  // (h is reused by the next call)
}

void group_fine_gather(Group* g, int s, const float* d_scores, int E_loc, const uint32_t* d_err, hipStream_t st) {
  group_fail_point(g, GROUP_FAIL_FINE);
  float* snd = g->d_fsend[s];
  HIP_CHECK(hipMemsetAsync(snd, 0, sizeof(float) * Group::FE_BLK, st));
  if (E_loc > 0) {
    HIP_CHECK(hipMemcpyAsync(snd, d_scores, sizeof(float) * (size_t)E_loc, hipMemcpyDeviceToDevice, st));
    HIP_CHECK(hipMemcpyAsync(snd + MAX_EVAL, d_err, 4, hipMemcpyDeviceToDevice, st));  // the error word's bits
  }
  g->tr->allgather(CH_FINE, snd, g->d_frecv[s], sizeof(float) * Group::FE_BLK, st);
  HIP_CHECK(hipMemcpyAsync(g->h_frecv[s], g->d_frecv[s], sizeof(float) * Group::FE_BLK * (size_t)g->n,
                           hipMemcpyDeviceToHost, st));
}

void group_fine_scores(const Group* g, int s, int E, float* scores, uint32_t* err) {
  *err = 0;
  for (int r = 0; r < g->n; ++r) {
    int lo, hi;
    shard_range(E, r, g->n, &lo, &hi);
    const float* blk = g->h_frecv[s] + (size_t)r * Group::FE_BLK;
    for (int e = lo; e < hi; ++e) scores[e] = blk[e - lo];
    uint32_t w;
    std::memcpy(&w, blk + MAX_EVAL, 4);
    *err |= w;
  }
}

bool shard_sort_enabled(const Group* g, uint32_t cap, int rounds) {
  if (!g || g->n < 2 || g->n > IS_SHARD_MAX) return false;
  // FCCF_SHARD_D_MIN: the smallest cloud whose sort is sharded (default 2M points: below
  // it the sort is ~0.4 ms per cloud and the bounds read-back + gather do not pay)
  const char* e = std::getenv("FCCF_SHARD_D_MIN");
  const uint32_t mn = e ? (uint32_t)std::strtoul(e, nullptr, 10) : (1u << 21);
  return cap >= mn && rounds > shard_sort_r0(g->n);
}

int shard_sort_r0(int n_ranks) {
  // replicated rounds: enough that round r0's children (2^r0 at most) can split into
  // n_ranks blocks of similar size
  int lg = 0;
  while ((1 << lg) < n_ranks) ++lg;
  return lg + 3;
}

void cloud_gate(Group* g) {
  std::unique_lock<std::mutex> lk(g->om);
  const bool ok = g->ocv.wait_for(lk, std::chrono::duration<double>(g->timeout_s),
                                  [&] { return g->order_abort || g->b1_issued >= g->cloud_need; });
  if (g->order_abort) throw Error(FCCF_E_RCCL, "group: batch aborted before the cloud stage's gather");
  if (!ok) {
    lk.unlock();
    group_abort(g, "the cloud stage's gather waited past the time limit for the previous pairs' phase B1");
    throw Error(FCCF_E_RCCL, "group: order gate timed out");
  }
}

void b1_done(Group* g) {
  {
    std::lock_guard<std::mutex> lk(g->om);
    ++g->b1_issued;
  }
  g->ocv.notify_all();
}

void order_reset(Group* g) {
  std::lock_guard<std::mutex> lk(g->om);
  g->b1_issued = 0;
  g->cloud_need = 0;
  g->order_abort = false;
}

void order_need(Group* g, int64_t need) {
  std::lock_guard<std::mutex> lk(g->om);
  g->cloud_need = need;
}

void order_abort(Group* g) {
  {
    std::lock_guard<std::mutex> lk(g->om);
    g->order_abort = true;
  }
  g->ocv.notify_all();
}

void shard_gather_sorted(Group* g, const B4<uint32_t*>& k0, const B4<uint32_t*>& v0, const B4<const uint32_t*>& bounds,
                         int nbatch, hipStream_t st) {
  const int n = g->n;
  if (nbatch < 1 || nbatch > BMAX) throw Error(FCCF_E_INTERNAL, "sharded sort: 1 .. BMAX clouds per stage");
  for (int e = 0; e < nbatch; ++e)
    HIP_CHECK(hipMemcpyAsync(g->h_bounds + (size_t)e * (IS_SHARD_MAX + 1), bounds[e], 4 * (size_t)(n + 1),
                             hipMemcpyDeviceToHost, st));
  group_wait(g, st);
  cloud_gate(g);  // (the batch's helper thread: after the previous pairs' B1 collectives)
  group_fail_point(g, GROUP_FAIL_CLOUD);
  // every cloud's keys and values: one exchange of 2 x nbatch all-gather-v's
  std::vector<size_t> cnt((size_t)n * nbatch), off((size_t)n * nbatch);
  std::vector<GatherOp> ops;
  for (int e = 0; e < nbatch; ++e) {
    const uint32_t* b = g->h_bounds + (size_t)e * (IS_SHARD_MAX + 1);
    size_t* ce = cnt.data() + (size_t)n * e;
    size_t* oe = off.data() + (size_t)n * e;
    for (int r = 0; r < n; ++r) {
      if (b[r + 1] < b[r]) throw Error(FCCF_E_INTERNAL, "sharded sort: rank bounds out of order");
      ce[r] = 4 * (size_t)(b[r + 1] - b[r]);
      oe[r] = 4 * (size_t)b[r];
    }
    const size_t me = 4 * (size_t)b[g->rank];
    ops.push_back(GatherOp{(const char*)k0[e] + me, k0[e], ce, oe});
    ops.push_back(GatherOp{(const char*)v0[e] + me, v0[e], ce, oe});
  }
  g->tr->allgatherv_multi(CH_CLOUD, ops.data(), (int)ops.size(), st);
}

void face_voxels_sharded(Group* g, B4<const float*> xyz, B4<const uint32_t*> d_n, uint32_t cap, double res, float vpt,
                         float cthr, B4<float*> resid_out, B4<FaceBufs> b, hipStream_t st, int nbatch) {
  const int n = g->n;
  if (nbatch < 1 || nbatch > BMAX) throw Error(FCCF_E_INTERNAL, "sharded face stage: 1 .. BMAX clouds per stage");
  face_codes(xyz, d_n, cap, res, b, st, nbatch);  // replicated: the octree bounds depend on every point in order
  face_shard_select(d_n, cap, b, g->rank, n, st, nbatch);
  face_shard_sort(xyz, cap, b, st, nbatch);
  cloud_gate(g);  // (the batch's helper thread: after the previous pairs' B1 collectives)
  // the ranks' counts of every cloud (cnt(e) = scalar k of cloud e; BMAX words per
  // rank), all-gathered in one collective: every rank's base per cloud
  const size_t W = BMAX;
  auto gather_counts = [&](int k, std::vector<uint32_t>& base, uint32_t* tot) {
    for (int e = 0; e < nbatch; ++e)
      HIP_CHECK(hipMemcpyAsync(g->d_fcnt + e, b[e].nleaf + k, 4, hipMemcpyDeviceToDevice, st));
    g->tr->allgather(CH_CLOUD, g->d_fcnt, g->d_fcnt + W, 4 * W, st);
    HIP_CHECK(hipMemcpyAsync(g->h_fcnt, g->d_fcnt + W, 4 * W * (size_t)n, hipMemcpyDeviceToHost, st));
    group_wait(g, st);
    base.assign((size_t)nbatch * (n + 1), 0u);
    for (int e = 0; e < nbatch; ++e) {
      uint32_t run = 0;
      for (int r = 0; r < n; ++r) {
        base[(size_t)e * (n + 1) + r] = run;
        run += g->h_fcnt[W * r + e];
      }
      base[(size_t)e * (n + 1) + n] = run;
      tot[e] = run;
    }
  };
  std::vector<uint32_t> lb, rb;
  uint32_t ltot[BMAX] = {}, rtot[BMAX] = {};
  gather_counts(0, lb, ltot);  // leaves per rank
  // views of the full leaf arrays at this rank's first leaf
  B4<FaceBufs> bv = b;
  for (int e = 0; e < BMAX; ++e) {
    const uint32_t o = lb[(size_t)(e < nbatch ? e : 0) * (n + 1) + g->rank];
    bv.v[e].recs += o;
    bv.v[e].flag_planar += o;
    bv.v[e].resid_cnt += o;
    bv.v[e].resid_off += o;
  }
  face_shard_fit(cap, vpt, cthr, bv, st, nbatch);
  gather_counts(3, rb, rtot);  // residual points per rank
  B4<float*> rv = resid_out;
  for (int e = 0; e < BMAX; ++e) rv.v[e] += 3 * (size_t)rb[(size_t)(e < nbatch ? e : 0) * (n + 1) + g->rank];
  face_shard_resid(cap, bv, rv, st, nbatch);
  // rank-ordered all-gathers into the full arrays (in place: each rank's part is already
  // there), four per cloud, every cloud's in one exchange
  std::vector<size_t> cnt((size_t)n * 4 * nbatch), off((size_t)n * 4 * nbatch);
  std::vector<GatherOp> ops;
  auto allgv = [&](void* base, const std::vector<uint32_t>& bs, int e, size_t unit) {
    size_t* c = cnt.data() + (size_t)n * ops.size();
    size_t* o = off.data() + (size_t)n * ops.size();
    for (int r = 0; r < n; ++r) {
      const size_t i = (size_t)e * (n + 1) + r;
      c[r] = unit * (bs[i + 1] - bs[i]);
      o[r] = unit * bs[i];
    }
    ops.push_back(GatherOp{(const char*)base + o[g->rank], base, c, o});
  };
  for (int e = 0; e < nbatch; ++e) {
    allgv(b[e].recs, lb, e, sizeof(VoxRec));
    allgv(b[e].flag_planar, lb, e, 4);
    allgv(b[e].resid_cnt, lb, e, 4);  // (read only by the debug dumps: a leaf's residual flag)
    allgv(resid_out[e], rb, e, 12);
  }
  g->tr->allgatherv_multi(CH_CLOUD, ops.data(), (int)ops.size(), st);
  // the full counts where the unsharded stage leaves them: leaves (scalar 0), residual
  // points (3); then the planar offsets over every leaf (nplanar, scalar 2)
  uint32_t* h = g->h_fcnt + W * (size_t)n;
  for (int e = 0; e < nbatch; ++e) {
    h[2 * e] = ltot[e];
    h[2 * e + 1] = rtot[e];
    HIP_CHECK(hipMemcpyAsync(b[e].nleaf, h + 2 * e, 4, hipMemcpyHostToDevice, st));
    HIP_CHECK(hipMemcpyAsync(b[e].nresid, h + 2 * e + 1, 4, hipMemcpyHostToDevice, st));
  }
  face_planar_scan(cap, b, st, nbatch);
  group_wait(g, st);  // (h is reused by the next call)
}

}  // namespace fccf

using namespace fccf;

struct fccf_group {
  Group g;
};

Group* fccf::group_of(fccf_group* g) { return g ? &g->g : nullptr; }

namespace {

// the buffers of a group, after its transport exists
void group_alloc(Group& g) {
  const size_t n = (size_t)g.n;
  if (hipMalloc((void**)&g.d_cnt, 16 * (n + 1)) != hipSuccess) throw Error(FCCF_E_OOM, "hipMalloc");
  if (hipHostMalloc((void**)&g.h_cnt, 16 * (n + 1), hipHostMallocDefault) != hipSuccess)
    throw Error(FCCF_E_OOM, "hipHostMalloc");
  if (hipHostMalloc((void**)&g.h_bounds, 4 * BMAX * (IS_SHARD_MAX + 1), hipHostMallocDefault) != hipSuccess)
    throw Error(FCCF_E_OOM, "hipHostMalloc");
  if (hipMalloc((void**)&g.d_fcnt, 4 * BMAX * (n + 1)) != hipSuccess) throw Error(FCCF_E_OOM, "hipMalloc");
  if (hipHostMalloc((void**)&g.h_fcnt, 4 * BMAX * n + 4 * 2 * BMAX + 64, hipHostMallocDefault) != hipSuccess)
    throw Error(FCCF_E_OOM, "hipHostMalloc");
  const char* te = std::getenv("FCCF_GROUP_TIMEOUT_S");
  if (te && std::atof(te) > 0) g.timeout_s = std::atof(te);
  for (int s = 0; s < Group::SLOTS; ++s) {
    if (hipMalloc((void**)&g.d_fsend[s], sizeof(float) * Group::FE_BLK) != hipSuccess ||
        hipMalloc((void**)&g.d_frecv[s], sizeof(float) * Group::FE_BLK * n) != hipSuccess)
      throw Error(FCCF_E_OOM, "hipMalloc");
    if (hipHostMalloc((void**)&g.h_frecv[s], sizeof(float) * Group::FE_BLK * n, hipHostMallocDefault) != hipSuccess)
      throw Error(FCCF_E_OOM, "hipHostMalloc");
  }
}

void group_free(Group& g) {
  for (ncclComm_t& c : g.comm)
    if (c) {
      (void)ncclCommDestroy(c);
      c = nullptr;
    }
  if (g.d_cnt) (void)hipFree(g.d_cnt);
  if (g.h_cnt) (void)hipHostFree(g.h_cnt);
  for (int s = 0; s < Group::SLOTS; ++s) {
    if (g.d_fsend[s]) (void)hipFree(g.d_fsend[s]);
    if (g.d_frecv[s]) (void)hipFree(g.d_frecv[s]);
    if (g.h_frecv[s]) (void)hipHostFree(g.h_frecv[s]);
    g.d_fsend[s] = g.d_frecv[s] = g.h_frecv[s] = nullptr;
  }
  if (g.h_bounds) (void)hipHostFree(g.h_bounds);
  g.h_bounds = nullptr;
  if (g.d_fcnt) (void)hipFree(g.d_fcnt);
  if (g.h_fcnt) (void)hipHostFree(g.h_fcnt);
  g.d_fcnt = g.h_fcnt = nullptr;
  g.d_cnt = nullptr;
  g.h_cnt = nullptr;
  g.tr.reset();
  g.hub.reset();
}

}  // namespace

extern "C" int fccf_group_unique_id(uint8_t id[FCCF_GROUP_ID_BYTES]) {
  if (!id) return FCCF_E_ARG;
  static_assert(sizeof(ncclUniqueId) == FCCF_GROUP_ID_BYTES, "ncclUniqueId size");
  ncclUniqueId u;
  if (ncclGetUniqueId(&u) != ncclSuccess) return FCCF_E_RCCL;
  std::memcpy(id, &u, sizeof u);
  return FCCF_OK;
}

extern "C" int fccf_group_create(fccf_ctx* c, const uint8_t id[FCCF_GROUP_ID_BYTES], int n_ranks, int rank,
                                 fccf_group** out) {
  if (!c || !id || !out || n_ranks < 1 || rank < 0 || rank >= n_ranks || c->group) return FCCF_E_ARG;
  *out = nullptr;
  fccf_group* G = new fccf_group();
  try {
    HIP_CHECK(hipSetDevice(c->device));
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof u);
    NCCL_CHECK(ncclCommInitRank(&G->g.comm[CH_MATCH], n_ranks, u, rank));
    // the fine-verification channel: its own communicator, so collectives issued on the
    // matching and fine streams never interleave on one communicator
    NCCL_CHECK(ncclCommSplit(G->g.comm[CH_MATCH], 0, rank, &G->g.comm[CH_FINE], nullptr));
    NCCL_CHECK(ncclCommSplit(G->g.comm[CH_MATCH], 0, rank, &G->g.comm[CH_CLOUD], nullptr));
    G->g.ctx = c;
    G->g.n = n_ranks;
    G->g.rank = rank;
    G->g.tr.reset(new RcclTransport(&G->g));
    G->g.tr->n_ranks = n_ranks;
    G->g.tr->my_rank = rank;
    group_alloc(G->g);
    c->group = &G->g;
    *out = G;
    return FCCF_OK;
  } catch (const Error& e) {
    c->last_error = e.what();
    group_free(G->g);
    delete G;
    return e.code;
  } catch (...) {
    group_free(G->g);
    delete G;
    return FCCF_E_INTERNAL;
  }
}

extern "C" int fccf_group_create_local(fccf_ctx* const* ctxs, int n, fccf_group** out) {
  if (!ctxs || !out || n < 1) return FCCF_E_ARG;
  for (int r = 0; r < n; ++r)
    if (!ctxs[r] || ctxs[r]->group || ctxs[r]->device != ctxs[0]->device) return FCCF_E_ARG;
  for (int r = 0; r < n; ++r)
    for (int q = 0; q < r; ++q)
      if (ctxs[q] == ctxs[r]) return FCCF_E_ARG;
  auto hub = std::make_shared<LocalHub>(n);
  std::vector<fccf_group*> made;
  try {
    HIP_CHECK(hipSetDevice(ctxs[0]->device));
    for (int r = 0; r < n; ++r) {
      fccf_group* G = new fccf_group();
      made.push_back(G);
      G->g.ctx = ctxs[r];
      G->g.n = n;
      G->g.rank = r;
      G->g.hub = hub;
      G->g.tr.reset(new LocalTransport(&G->g));
      G->g.tr->n_ranks = n;
      G->g.tr->my_rank = r;
      group_alloc(G->g);
    }
  } catch (...) {
    for (fccf_group* G : made) {
      group_free(G->g);
      delete G;
    }
    return FCCF_E_OOM;
  }
  for (int r = 0; r < n; ++r) {
    ctxs[r]->group = &made[(size_t)r]->g;
    out[r] = made[(size_t)r];
  }
  return FCCF_OK;
}

extern "C" int fccf_group_destroy(fccf_group* G) {
  if (!G) return FCCF_E_ARG;
  if (G->g.ctx) {
    (void)hipSetDevice(G->g.ctx->device);
    (void)device_sync_guarded();
    if (G->g.ctx->group == &G->g) G->g.ctx->group = nullptr;
  }
  group_free(G->g);
  delete G;
  return FCCF_OK;
}

extern "C" int fccf_debug_group_fail(fccf_group* G, int site, int silent) {
  if (!G || site < 0 || site > GROUP_FAIL_CLOUD) return FCCF_E_ARG;
  G->g.fail_at = site;
  G->g.fail_silent = silent != 0;
  return FCCF_OK;
}

extern "C" int fccf_group_aborted(const fccf_group* G) {
  if (!G) return FCCF_E_ARG;
  return G->g.aborted ? 1 : 0;
}

extern "C" int fccf_group_bytes(const fccf_group* G, int64_t rx[3]) {
  if (!G || !rx) return FCCF_E_ARG;
  for (int c = 0; c < 3; ++c) rx[c] = G->g.tr ? G->g.tr->rx_bytes[c].load() : 0;
  return FCCF_OK;
}

extern "C" int fccf_group_info(const fccf_group* G, int* n_ranks, int* rank) {
  if (!G) return FCCF_E_ARG;
  if (n_ranks) *n_ranks = G->g.n;
  if (rank) *rank = G->g.rank;
  return FCCF_OK;
}
