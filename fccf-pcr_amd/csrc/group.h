// group.h — RCCL communicator of one rank (one process per GPU) and the sharded
// correspondence search's candidate gather (FCCF.cpp:1410-1428).
#pragma once
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>

#include "match.h"

struct fccf_ctx;
struct fccf_group;

namespace fccf {

struct Group {
  fccf_ctx* ctx = nullptr;
  ncclComm_t comm = nullptr;
  int n = 1, rank = 0;
  uint32_t* d_cnt = nullptr;  // device: this rank's 4 counts, then all ranks' (n x 4)
  uint32_t* h_cnt = nullptr;  // pinned copy of all ranks' counts
};

// the Group inside a C-ABI handle (null for null)
Group* group_of(fccf_group* g);

// Contiguous block [lo, hi) of n source pairs for `rank` (sizes differ by at most
// one, lower ranks larger; shard.py's shard_range).
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

}  // namespace fccf
