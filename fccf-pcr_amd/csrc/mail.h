// mail.h — pinned, host-mapped mailboxes that the device stages write their
// phase-B outputs into, so the host reads them after ONE event/stream sync per
// stage instead of a chain of count-then-data device-to-host copies (each
// pageable copy is a blocking host round trip on ROCm).  Device kernels fill
// them as a side effect of a launch they already make (k_compact_planar,
// k_match_scan/k_match_emit, k_fv_score).  Anything past a mailbox capacity is
// still in its device buffer; the host copies that rare overflow explicitly.
#pragma once
#include <stdint.h>

#include "kernels.h"
#include "match.h"

namespace fccf {

struct CloudMail {                     // one per pair slot (fccf_ctx::cs)
  static constexpr uint32_t REC_CAP = 16384;   // planar 1 m voxels per cloud
  uint32_t sc[2][4];                   // per cloud: n_in, M1, M1 finite, M2
  uint32_t fsc[2][4];                  // per cloud: leaves, K1 sort fault flags (VGParams::sort_err),
                                       // planar leaves, residual points
  uint64_t stamp[4];                   // s_memrealtime (100 MHz) when main's pass, the driver's pass,
                                       // the face stage and its last kernel started (fccf_stats dev_ms)
  uint32_t done;                       // 1 once the stage's records and counts are in this mailbox
                                       // (k_mail_done; the host clears it before the stage's launch)
  uint32_t pad_[3];
  VoxRec rec[2][REC_CAP];              // oriented planar records, Morton order
};

struct MatchMail {
  static constexpr uint32_t Q_CAP = 65536;     // candidate transforms per type
  static constexpr uint32_t CB_CAP = 1u << 19; // neighbour bitmask words, all types
  MatchIn M;                           // host staging of the matching tables (H2D source)
  uint32_t tot[4];                     // candidates per type
  uint32_t kpass;                      // tests with >= 1 candidate
  uint32_t pad[3];
  QTd q[3][Q_CAP];
  // transform_cluster neighbour rows (k_cluster_bits): type t's n_t x W_t words
  // (W_t = ceil(n_t / 64)) at word offset sum_{t' < t} n_t' W_t'; written only when
  // all types fit CB_CAP and cbits_on.
  uint64_t cbits[CB_CAP];
  // device clustering (cluster.hip): per type status, clusters, emitted, cluster_num;
  // the averaged clusters in emission order
  static constexpr uint32_t CL_FCAP = 1024;
  uint32_t cl_stat[3][4];
  QTd cl_fine[3][CL_FCAP];
};

struct FineMail {
  m44 T[MAX_EVAL];                     // host staging of the evaluated transforms (H2D source)
  float scores[MAX_EVAL];
  uint32_t err;                        // fine_verify scal[7]
  uint32_t done;                       // 1 once scores and err are here (cleared before the launch)
  uint32_t pad_;
  uint64_t stamp[2];                   // s_memrealtime: the launch's first and last kernels started
};

struct HostMail {
  CloudMail clouds[10];  // per pair slot; a stage group's slots are adjacent (k_compact_planar)
  MatchMail match;      // phase-B chain 0 (pipeline.cpp Chain)
  MatchMail match2;     // chain 1: a pipelined batch's second host thread
  MatchMail match3;     // chains 2 to 4: the batch's last stage group (a chain per pair)
  MatchMail match4;
  MatchMail match5;
  FineMail fine[10];  // per pair slot: a pair's fine verification overlaps the next pair's phase B
};

}  // namespace fccf
