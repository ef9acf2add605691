// match.h — device-side tables of K5 (coplane-pair matching) and K7 (fine verify).
#pragma once
#include <stdint.h>

#include "devprim.h"
#include "fccf_math.h"

namespace fccf {

constexpr int MAX_PLANES = 17;   // select_plane_number + 1 planes are kept (:670)
constexpr int MAX_BASES = 136;   // C(17, 2)

struct MPlane { float c[3], n[3], fps; int32_t nvox; };
struct MBase { int32_t i1, i2; float angle; int32_t type; };

struct alignas(16) MatchIn {
  MPlane F1[MAX_PLANES], F2[MAX_PLANES];
  MBase B1[MAX_BASES], B2[MAX_BASES];
  int32_t nF1, nF2, nB1, nB2;
  float ang_same;    // included_angle_same_threshold
  float third_thr;   // third_plane_threshold
  AngleCut third_cut;  // theta < third_plane_normal_threshold
};

struct MCand { float R[9]; float t[3]; };
struct QTd { float qw, qx, qy, qz, tx, ty, tz; uint32_t alloc; };

// counts/types/offsets need K entries; totals 3; c[t]/q[t] sized by the caller.
struct MatchMail;
// mail (may be null): pinned mailbox receiving the totals, K_pass and the candidate lists (mail.h)
void match_candidates(const MatchIn* d_in, int K, uint32_t* cnt, int32_t* type, uint32_t* off, uint32_t* totals,
                      MCand* c[3], QTd* q[3], hipStream_t st, MatchMail* mail = nullptr);

// ------------------------------------------------ f3: transform_cluster on the device (cluster.hip)
// Everything is derived on the device from the totals, so the launches go into the
// match stage's stream before its one host sync.  Results land in the mailbox
// (MatchMail::cl_stat / cl_fine); a type whose status is not 0 is redone by the host.
struct ClusterIn {
  const QTd* q[3];           // candidates per type
  const uint64_t* rows;      // k_cluster_bits's neighbour rows in HBM (MatchMail::cbits layout)
  const uint32_t* totals;    // candidates per type
  uint32_t cb_cap;           // row words present only when all types fit (MatchMail::CB_CAP)
  float min_n;               // cluster_number_threshold: n <= min_n is not clustered (host)
  float sel;                 // seclct_cluster_number (cluster_num, :1458)
  int32_t cnum_given;        // has_cnum: every type's cluster_num is this instead (fccf_stage_cluster)
  uint32_t has_cnum;
};
struct ClusterOut {
  uint32_t *cseed[3], *csize[3];  // clusters in creation order
  uint32_t *bx[3], *bid[3];       // range_cluster's working array
  uint32_t* emit[3];              // averaged clusters in emission order
  uint32_t cap;                   // entries of each of those per type (>= the type's candidates)
  uint32_t* stat;                 // 4 per type: status, clusters, emitted, cluster_num
  QTd* fine;                      // fcap per type: the averages in emission order
  uint32_t fcap;
  uint32_t egrid;                 // averaging waves launched per type (<= fcap); cluster_num + 1 must fit
};
void cluster_device(const ClusterIn& in, const ClusterOut& out, hipStream_t st);

// ------------------------------------------------ f1: quick_verify + LM on the device (verify.hip)
struct VerifyIn {
  const QTd* q;           // candidate transforms as quaternion records, all types concatenated
  const MatchIn* planes;  // F1, F2 and their counts (the matching table)
  int32_t fs12;           // fs1 + fs2, quick_verify's face-point sums (FCCF.cpp:688-697)
  AngleCut qcut;          // quick_verify_angel_threshold
  float dist_thr;         // quick_verify_distance_threshold
  float required;         // required_optimize_plane
};
struct VerifyOut {
  float* T;          // 16 per candidate, row-major, refined
  float* score;
  int32_t* npairs;
  uint32_t* status;  // 1: a sin/cos argument outside the device reduction (host redoes it)
};
void verify_device(const VerifyIn& in, int n, const VerifyOut& out, hipStream_t st);
// test hook: the device's correctly rounded double sin/cos of x[0..n)
void sincos_probe(const double* x, int n, double* s, double* c, uint32_t* ok, hipStream_t st);

// ------------------------------------------------ K7: fine_verify (FCCF.cpp:785-839)
constexpr int MAX_EVAL = 16;
struct FineBufs {
  float* s2t;          // E * n2 * 3
  float* aggr2;        // E * blocks(n2) * 6
  OctState* state;     // E + 1 (slot E = after S1)
  uint64_t *k0, *k1, *k2;  // E * (n1 + n2): leaf entries' keys (three sort buffers)
  uint32_t *v0, *v1, *v2;  // their point counts (source | target << 16)
  uint32_t* pts;           // MAX_EVAL: finite points per evaluation (allinvec)
  uint32_t* starts;    // E * (n1 + n2) + 1
  float* term;         // per leaf similar_num term
  uint32_t* range;     // per evaluation: first leaf, end leaf (2 * MAX_EVAL)
  uint32_t* nseg_e;    // 2 * MAX_EVAL: leaf counts, then first leaves
  float* similar;      // MAX_EVAL
  float* all;          // MAX_EVAL
  uint32_t* scal;      // [0]=n keys, [1]=nbits, [2]=nseg, [3]=shift, [4]=n1, [5]=n2, [6]=E, [7]=error
  float* scores;       // E
  m44* T;              // E
  SortScratch ss;
  XsBufs xs;           // similar_num sum scratch (E rows, cap n1 + n2)
};
// s1_state: octree bounds after inserting S1 alone (octree_replay, run ahead of time).
// transform_cluster neighbour bitmasks of the three candidate lists into mail->cbits
// (layout in mail.h) and, when dev_rows is not null, the same words into dev_rows
// (device clustering); types with <= min_n candidates are skipped (not clustered).
void cluster_bits(QTd* const q[3], const uint32_t* totals, float r2, AngleCut ccut, float min_n, MatchMail* mail,
                  hipStream_t st, uint64_t* dev_rows = nullptr);

// mail (may be null): pinned mailbox receiving the E scores and the error word (mail.h)
// mode FV_LEAVES_LDS (default): one workgroup per evaluation merges its leaf entries
// in an LDS table of at most lds_cap leaves, sorts them in LDS and sums in leaf order;
// an evaluation with more leaves raises FV_ERR_LDS in the error word (scores invalid)
// and the caller reruns the batch in mode FV_LEAVES_SORTED (device-wide sort of the
// entries, exact_sum).  Both give the same scores bit for bit.
constexpr int FV_LEAVES_LDS = 0, FV_LEAVES_SORTED = 1;
constexpr uint32_t FV_ERR_POINTS = 1u, FV_ERR_LDS = 2u;  // error word bits (scal[7], FineMail::err)
constexpr uint32_t FV_LDS_MAX = 4096;                    // leaves per evaluation in the LDS form
struct FineMail;
void fine_verify_batch(const float* s1, uint32_t n1, const OctState* s1_state, const float* s2, uint32_t n2, int E,
                       double res, FineBufs b,
                       hipStream_t st, FineMail* mail = nullptr, int mode = FV_LEAVES_LDS,
                       uint32_t lds_cap = FV_LDS_MAX);
// the leaf-form for this call: FCCF_FINE_SORTED=1 forces the sorted form, FCCF_FINE_LDS_CAP
// lowers the LDS form's capacity (tests of the fallback)
int fine_mode_env(int sticky_sorted);
uint32_t fine_lds_cap_env();

}  // namespace fccf
