// group.h — one rank of a multi-GPU registration group (one process per GPU) and
// the exchange steps of the sharded stages:
//   K5  the coplane-pair correspondence search (FCCF.cpp:1410-1428): source pairs in
//       contiguous blocks, the candidate lists gathered in rank order;
//   F   fine_verify (:785-839): the <= 16 evaluations in contiguous blocks, the
//       scores gathered in rank order.
// The collectives go through a Transport: RCCL over xGMI in the product (two
// communicators, one per stream that issues collectives, so the matching stream and
// the fine-verification stream never interleave operations on one communicator), or
// an in-process hub of virtual ranks on one device (fccf_group_create_local, a test
// hook that runs the same host-side exchange logic with n > 1 ranks on one GPU).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <atomic>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <memory>
#include <mutex>
#include <string>

#include "kernels.h"
#include "match.h"

struct fccf_ctx;
struct fccf_group;

namespace fccf {

// Collective channels: each is used from one stream only (stream order = issue order):
// CH_MATCH the candidate gather (phase B), CH_FINE the fine scores (fine stream),
// CH_CLOUD the sharded sort's slices (the cloud stage, possibly on the batch's helper
// thread).
enum { CH_MATCH = 0, CH_FINE = 1, CH_CLOUD = 2, CH_COUNT = 3 };

// One rank-ordered all-gather-v of a batch of them (Transport::allgatherv_multi).
struct GatherOp {
  const void* send;
  void* recv;
  const size_t* counts;  // n_ranks entries
  const size_t* offs;
};

struct Transport {
  virtual ~Transport();
  // Rank-ordered all-gather-v on channel ch, in the order of stream st: rank r's
  // counts[r] bytes (its `send`) land at recv + offs[r] on every rank.  Buffers are
  // device memory of the rank's device.
  virtual void allgatherv(int ch, const void* send, void* recv, const size_t* counts, const size_t* offs,
                          hipStream_t st) = 0;
  // Several all-gather-v's as one exchange.  The default (both transports) is ONE
  // all-gather of count-padded blocks: each rank packs its parts of every op into one
  // block (16-byte aligned parts), the blocks (the largest rank's size) are all-gathered,
  // and every rank's parts are copied to their places -- a pack and an unpack launch of
  // a descriptor copy kernel around one collective (group.cpp allgatherv_packed).
  virtual void allgatherv_multi(int ch, const GatherOp* ops, int nops, hipStream_t st);
  // The same with equal blocks of `bytes`, rank r's at recv + r * bytes.
  virtual void allgather(int ch, const void* send, void* recv, size_t bytes, hipStream_t st) = 0;
  // Bytes this rank received through collectives, per channel (fccf_stats.coll_bytes).
  std::atomic<int64_t> rx_bytes[3] = {{0}, {0}, {0}};
  // Device scratch of the packed all-gather-v, per channel (grown on demand; used only
  // from the channel's one stream).
  struct Scratch {
    char* pack = nullptr;
    char* recv = nullptr;
    size_t cap_pack = 0, cap_recv = 0;
  } scratch[3];
  void free_scratch();
  int n_ranks = 1, my_rank = 0;
  // A non-zero code once the transport has failed asynchronously (RCCL:
  // ncclCommGetAsyncError of any communicator; virtual ranks: the hub was aborted).
  virtual int async_error() { return 0; }
  // Ends every outstanding and future collective of this rank (RCCL: ncclCommAbort of
  // the communicators, which also releases the kernels waiting in them).
  virtual void abort() {}
};

struct LocalHub;  // group.cpp

struct Group {
  fccf_ctx* ctx = nullptr;
  int n = 1, rank = 0;
  ncclComm_t comm[CH_COUNT] = {nullptr, nullptr, nullptr};  // RCCL groups
  std::shared_ptr<LocalHub> hub;                   // virtual-rank groups
  std::unique_ptr<Transport> tr;
  uint32_t* d_cnt = nullptr;  // device: this rank's 4 counts, then all ranks' (n x 4)
  uint32_t* h_cnt = nullptr;  // pinned copy of all ranks' counts
  // sharded fine verification, per pair slot s (the pipelined batch overlaps pairs):
  // this rank's block of scores + its error word (FE_BLK floats), all ranks' blocks
  static constexpr int FE_BLK = MAX_EVAL + 1;
  static constexpr int SLOTS = 10;  // the ctx's pair slots (fccf_ctx::cs)
  float* d_fsend[SLOTS] = {};
  float* d_frecv[SLOTS] = {};  // n x FE_BLK
  float* h_frecv[SLOTS] = {};  // pinned copies
  uint32_t* h_bounds = nullptr;             // pinned: the sharded sort's rank bounds, per cloud (row D; BMAX clouds)
  uint32_t* d_fcnt = nullptr;               // row P: this rank's BMAX counts, then all ranks' (n x BMAX), device
  uint32_t* h_fcnt = nullptr;               // ... their pinned copy, then 2 x BMAX words of totals for the device
  // One issue order of collectives per rank.  Communicators that are used concurrently
  // must see their collectives issued in the same order on every rank, or their kernels
  // can wait on each other across ranks.  The pipelined batch issues CH_MATCH and CH_FINE
  // from phase B1 on the main thread and CH_CLOUD (row D) from the helper thread that
  // enqueues the next pair's cloud stage, so the cloud gather of pair i + 1 waits here
  // until the main thread has issued pair i's B1 collectives: order CLOUD(i), MATCH(i),
  // FINE(i), CLOUD(i + 1), ... on every rank (cloud_gate, b1_done).
  std::mutex om;
  std::condition_variable ocv;
  int64_t b1_issued = 0;   // pairs of the current batch whose phase-B1 collectives are issued
  int64_t cloud_need = 0;  // the next CH_CLOUD gather waits for b1_issued >= cloud_need
  bool order_abort = false;  // set on an error unwind: a waiting gather throws instead of hanging
  // Failure handling.  Every host wait that may depend on a peer (a stream or event
  // after a collective, the order gate, a virtual-rank barrier) is bounded by
  // timeout_s (FCCF_GROUP_TIMEOUT_S, default 30) and polls the transport's async error;
  // on an error, a timeout or any exception out of a registration with the group
  // attached, the rank aborts the group (group_abort): its communicators are aborted,
  // so kernels and waits of this rank end, and it returns FCCF_E_RCCL.  A peer blocked
  // in a collective with the failed rank ends at its own bound the same way.  An
  // aborted group fails every later call until it is destroyed (and recreated).
  std::atomic<bool> aborted{false};
  double timeout_s = 30.0;
  // why the group was aborted: written under why_m before `aborted` is set (group_abort),
  // read through group_why
  std::mutex why_m;
  std::string abort_why;
  // test hook (fccf_debug_group_fail): fail this rank at a collective site
  int fail_at = 0;          // GROUP_FAIL_* site, 0 = off
  bool fail_silent = false; // the failing rank does not abort its transport (a dead peer)
};
// Collective sites of the failure-injection hook.
enum { GROUP_FAIL_MATCH = 1, GROUP_FAIL_FINE = 2, GROUP_FAIL_CLOUD = 3 };
// Aborts the group (idempotent; see Group::aborted).  why: the reason recorded.
void group_abort(Group* g, const std::string& why);
// Throws FCCF_E_RCCL when the group is aborted.
void group_check(Group* g);
// The recorded abort reason (a copy taken under the group's why_m).
std::string group_why(Group* g);
// Bounded waits for a stream / an event that may depend on peers (see Group::aborted):
// return when complete; abort the group and throw FCCF_E_RCCL on an async transport
// error or after the group's time limit, FCCF_E_HIP on a device error.
// capture_lock: each poll under the pipeline's capture lock (ctx.h capture_mutex; an
// event whose stream another thread may be capturing).
void group_wait(Group* g, hipStream_t st);
void group_wait_event(Group* g, hipEvent_t ev, bool capture_lock = false);
// The failure-injection hook at site `site` (throws when armed for it).
void group_fail_point(Group* g, int site);
// The collective-order gate (see Group::om): blocks until b1_issued >= cloud_need, or
// throws FCCF_E_RCCL when the batch is unwinding after an error.
void cloud_gate(Group* g);
// Phase B1 of one more pair has issued its collectives (wakes a waiting cloud gather).
void b1_done(Group* g);
// Batch start / end: reset the gate; set the need of the next helper-issued cloud stage;
// abort a waiting gather (error unwind).
void order_reset(Group* g);
void order_need(Group* g, int64_t need);
void order_abort(Group* g);

// Row D (K1's sort sharded after its first rounds, introsort.hip): whether the cloud
// stage of clouds of cap points shards its sort over g, and the round it starts at.
bool shard_sort_enabled(const Group* g, uint32_t cap, int rounds);
int shard_sort_r0(int n_ranks);
// After a sharded sort: every rank's sorted slice [bounds[r], bounds[r+1]) of (k0, v0)
// of each of the nbatch clouds (up to BMAX: every pair of a stage group), gathered in
// rank order into every rank's arrays, all clouds in one exchange.  bounds[e]: the
// device copy of cloud e's bounds (IsBufs::bounds).  Synchronises st (the bounds).
void shard_gather_sorted(Group* g, const B4<uint32_t*>& k0, const B4<uint32_t*>& v0, const B4<const uint32_t*>& bounds,
                         int nbatch, hipStream_t st);

// Row P (FCCF.cpp:470-534): the face stage of the batch's clouds (the
// driver's downsampled clouds xyz, counts d_n) with each rank fitting only its Morton
// range of 1 m leaves; leaf records, planar flags and residual points are all-gathered
// in rank order into the same arrays (and counts) the unsharded stage fills.  Runs on
// st on the CH_CLOUD channel, synchronising st twice (the ranks' leaf and residual counts).
void face_voxels_sharded(Group* g, B4<const float*> xyz, B4<const uint32_t*> d_n, uint32_t cap, double res, float vpt,
                         float cthr, B4<float*> resid_out, B4<FaceBufs> b, hipStream_t st, int nbatch);

// the Group inside a C-ABI handle (null for null)
Group* group_of(fccf_group* g);

// Contiguous block [lo, hi) of n items for `rank` (sizes differ by at most one,
// lower ranks larger; shard.py's shard_range).
void shard_range(int n, int rank, int world, int* lo, int* hi);

// The rank-ordered concatenation of every rank's candidate lists (q: quaternion
// records, c: matrices) for the three types.  tot_loc/kpass_loc: this rank's counts.
// Writes the gathered lists to q_all/c_all (capacity cap each), the totals to tot_all
// (host) and d_tot_all (device, 4 words), and the summed K_pass.  Because the
// reference loop is b1-major and the blocks are contiguous, the result equals the
// unsharded lists element for element.  Synchronises st.
void group_gather_candidates(Group* g, QTd* const q_loc[3], MCand* const c_loc[3], const uint32_t tot_loc[3],
                             int64_t kpass_loc, QTd* const q_all[3], MCand* const c_all[3], size_t cap,
                             uint32_t tot_all[3], uint32_t* d_tot_all, int64_t* kpass_all, hipStream_t st);

// Sharded fine verification (row F): this rank evaluated the block [lo, hi) of the E
// transforms (shard_range), its E_loc = hi - lo scores at d_scores and its error word
// at d_err.  Enqueues on st (the fine stream): the block and the error word into the
// send slot of cloud set s, the all-gather, and the copy of every rank's block into
// g->h_frecv[s], complete when st reaches that point.
void group_fine_gather(Group* g, int s, const float* d_scores, int E_loc, const uint32_t* d_err, hipStream_t st);
// After st has passed group_fine_gather: the E scores in evaluation order and the
// OR of every rank's error word.
void group_fine_scores(const Group* g, int s, int E, float* scores, uint32_t* err);

}  // namespace fccf
