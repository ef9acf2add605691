// group.cpp — multi-GPU inside libfccf over RCCL (SURVEY.md §8(b) fccf_group_create,
// §8(e) row K5).  One process per GPU; every rank holds a communicator created from
// one ncclUniqueId that rank 0 made and the caller distributed out of band.
//
// What is sharded: the coplane-pair correspondence search (FCCF.cpp:1410-1428).
// Source pairs B1 are split into contiguous blocks (shard_range); each rank tests its
// block against all target pairs on its GPU, then the per-type candidate lists are
// gathered in rank order with RCCL over xGMI: the counts by one ncclAllGather, the
// variable-length lists by one group of per-root ncclBroadcasts (an all-gather-v).
// The reference's loop is b1-major, so the concatenation is the unsharded list.
// Everything else is replicated: every rank runs the cloud stage on the same inputs
// (the VoxelGrid's std::sort order spans the whole cloud), growth,
// selection, clustering and the LM are sequential and deterministic, so every rank
// computes the same T with no further exchange.
#include "group.h"

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "ctx.h"

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

void shard_range(int n, int rank, int world, int* lo, int* hi) {
  const int q = n / world, r = n % world;
  *lo = rank * q + std::min(rank, r);
  *hi = *lo + q + (rank < r ? 1 : 0);
}

void group_gather_candidates(Group* g, QTd* const q_loc[3], MCand* const c_loc[3], const uint32_t tot_loc[3],
                             int64_t kpass_loc, QTd* const q_all[3], MCand* const c_all[3], size_t cap,
                             uint32_t tot_all[3], uint32_t* d_tot_all, int64_t* kpass_all, hipStream_t st) {
  const int n = g->n;
  uint32_t* h = g->h_cnt;  // pinned: [0..3] this rank's counts, [4 ..] every rank's
  h[0] = tot_loc[0];
  h[1] = tot_loc[1];
  h[2] = tot_loc[2];
  h[3] = (uint32_t)kpass_loc;
  HIP_CHECK(hipMemcpyAsync(g->d_cnt, h, 16, hipMemcpyHostToDevice, st));
  NCCL_CHECK(ncclAllGather(g->d_cnt, g->d_cnt + 4, 4, ncclUint32, g->comm, st));
  HIP_CHECK(hipMemcpyAsync(h + 4, g->d_cnt + 4, 16 * (size_t)n, hipMemcpyDeviceToHost, st));
  HIP_CHECK(hipStreamSynchronize(st));
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
  // all-gather-v: one broadcast per (root, type) inside one group; empty blocks skipped
  {
    NcclGroup grp;
    for (int r = 0; r < n; ++r)
      for (int t = 0; t < 3; ++t) {
        const size_t cnt = h[4 + 4 * r + t];
        if (!cnt) continue;
        const size_t b = base[(size_t)r * 3 + t];
        NCCL_CHECK(ncclBroadcast(r == g->rank ? (const void*)q_loc[t] : (const void*)(q_all[t] + b), q_all[t] + b,
                                 cnt * sizeof(QTd), ncclUint8, r, g->comm, st));
        NCCL_CHECK(ncclBroadcast(r == g->rank ? (const void*)c_loc[t] : (const void*)(c_all[t] + b), c_all[t] + b,
                                 cnt * sizeof(MCand), ncclUint8, r, g->comm, st));
      }
    grp.end();
  }
  h[0] = tot_all[0];
  h[1] = tot_all[1];
  h[2] = tot_all[2];
  h[3] = 0;
  HIP_CHECK(hipMemcpyAsync(d_tot_all, h, 16, hipMemcpyHostToDevice, st));
  HIP_CHECK(hipStreamSynchronize(st));  // (h is reused by the next call)
}

}  // namespace fccf

using namespace fccf;

struct fccf_group {
  Group g;
};

Group* fccf::group_of(fccf_group* g) { return g ? &g->g : nullptr; }

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
    NCCL_CHECK(ncclCommInitRank(&G->g.comm, n_ranks, u, rank));
    G->g.ctx = c;
    G->g.n = n_ranks;
    G->g.rank = rank;
    if (hipMalloc((void**)&G->g.d_cnt, 16 * (size_t)(n_ranks + 1)) != hipSuccess) throw Error(FCCF_E_OOM, "hipMalloc");
    if (hipHostMalloc((void**)&G->g.h_cnt, 16 * (size_t)(n_ranks + 1), hipHostMallocDefault) != hipSuccess)
      throw Error(FCCF_E_OOM, "hipHostMalloc");
    c->group = &G->g;
    *out = G;
    return FCCF_OK;
  } catch (const Error& e) {
    c->last_error = e.what();
    if (G->g.comm) (void)ncclCommDestroy(G->g.comm);
    if (G->g.d_cnt) (void)hipFree(G->g.d_cnt);
    delete G;
    return e.code;
  }
}

extern "C" int fccf_group_destroy(fccf_group* G) {
  if (!G) return FCCF_E_ARG;
  if (G->g.ctx) {
    (void)hipSetDevice(G->g.ctx->device);
    (void)hipDeviceSynchronize();
    if (G->g.ctx->group == &G->g) G->g.ctx->group = nullptr;
  }
  if (G->g.comm) (void)ncclCommDestroy(G->g.comm);
  if (G->g.d_cnt) (void)hipFree(G->g.d_cnt);
  if (G->g.h_cnt) (void)hipHostFree(G->g.h_cnt);
  delete G;
  return FCCF_OK;
}

extern "C" int fccf_group_info(const fccf_group* G, int* n_ranks, int* rank) {
  if (!G) return FCCF_E_ARG;
  if (n_ranks) *n_ranks = G->g.n;
  if (rank) *rank = G->g.rank;
  return FCCF_OK;
}
