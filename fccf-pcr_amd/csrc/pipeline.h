// pipeline.h — workspace layout helpers shared by api.cpp and pipeline.cpp.
#pragma once
#include "ctx.h"
#include "host_stages.h"
#include "kernels.h"
#include "match.h"

namespace fccf {

inline size_t voxel_grid_bytes(uint32_t cap) {
  return 4 * sizeof(uint32_t) * (size_t)cap + sizeof(uint32_t) * ((size_t)cap + 1) + sizeof(float) * VG_BBOX_BLOCKS * 8 +
         sizeof(VGParams) + 64 + sort_scratch_bytes(cap) + introsort_bytes(cap) + 12 * (size_t)cap + 9 * 256;
}

inline VGBufs voxel_grid_carve(Arena& a, uint32_t cap) {
  VGBufs b;
  b.k0 = a.take_n<uint32_t>(cap);
  b.v0 = a.take_n<uint32_t>(cap);
  b.k1 = a.take_n<uint32_t>(cap);
  b.v1 = a.take_n<uint32_t>(cap);
  b.starts = a.take_n<uint32_t>((size_t)cap + 1);
  b.part = a.take_n<float>(VG_BBOX_BLOCKS * 8);
  b.params = a.take_n<VGParams>(1);
  b.nseg = a.take_n<uint32_t>(16);
  b.ss = sort_scratch_carve(a.take(sort_scratch_bytes(cap)), cap);
  b.is = introsort_carve(a.take(introsort_bytes(cap)), cap);
  b.is.err = &b.params->sort_err;
  b.is.vgp = b.params;
  b.xyzs = a.take_n<float>(3 * (size_t)cap);
  return b;
}

// Device buffers of the 1 m face-voxel stage of one cloud (K2/K3); centroid is left
// null for the caller to point at its compute3DCentroid output.
inline size_t face_bufs_bytes(uint32_t cap) {
  const size_t N = cap;
  return 3 * 8 * N + 3 * 4 * N + 4 * (N + 1) + 4 * aggr_floats(cap) + 256 + sizeof(VoxRec) * N + 4 * 4 * N + 64 +
         12 * N + 4 * N + sort_scratch_bytes(cap) + 24 * 256;
}

inline FaceBufs face_bufs_carve(Arena& a, uint32_t cap) {
  FaceBufs f;
  f.c0 = a.take_n<uint64_t>(cap);
  f.c1 = a.take_n<uint64_t>(cap);
  f.c2 = a.take_n<uint64_t>(cap);
  f.v0 = a.take_n<uint32_t>(cap);
  f.v1 = a.take_n<uint32_t>(cap);
  f.v2 = a.take_n<uint32_t>(cap);
  f.starts = a.take_n<uint32_t>((size_t)cap + 1);
  f.aggr = a.take_n<float>(aggr_floats(cap));
  f.oct = a.take_n<OctState>(1);
  f.centroid = nullptr;
  f.recs = a.take_n<VoxRec>(cap);
  f.flag_planar = a.take_n<uint32_t>(cap);
  f.resid_cnt = a.take_n<uint32_t>(cap);
  f.planar_off = a.take_n<uint32_t>(cap);
  f.resid_off = a.take_n<uint32_t>(cap);
  f.sp = a.take_n<float>(3 * (size_t)cap);
  f.seg_of = a.take_n<uint32_t>(cap);
  uint32_t* s = a.take_n<uint32_t>(16);
  f.nleaf = s;
  f.nbits = s + 1;
  f.nplanar = s + 2;
  f.nresid = s + 3;
  f.t_faces = reinterpret_cast<uint64_t*>(s + 4);
  f.vgp = nullptr;
  f.ss = sort_scratch_carve(a.take(sort_scratch_bytes(cap)), cap);
  return f;
}

// K4 (grow.hip): region growing stages 1-2 of both clouds on the device.  dvox: the
// clouds' planar voxel records in HBM, nv their counts (each <= GROW_CAP, else the
// caller grows on the host).  Uses arena2 and c->pinned; synchronises st.
void grow_groups_device(fccf_ctx* c, const VoxRec* const dvox[2], const uint32_t nv[2], const fccf_params& P,
                        hipStream_t st, std::vector<GroupOut> out[2]);

// f1 (verify.hip): quick_verify + LM of the candidates qs on the device; dM holds the
// F1/F2 tables (MatchIn, device).  Outputs per candidate: refined T, score, pairs.
// Uses arena_v and c->pinned; synchronises st.
// f3: transform_cluster after k_cluster_bits on the device (cluster.hip), the results
// into the mailbox (MatchMail::cl_stat/cl_fine); scratch from c->arena2.  cluster_num
// (may be null): one value for all types instead of the one derived from the totals.
struct MatchMail;
void cluster_launch(fccf_ctx* c, QTd* const dq[3], const uint32_t* dtot, const uint64_t* drows, size_t ccap,
                    const fccf_params& P, MatchMail* mail, hipStream_t st, const int* cluster_num = nullptr,
                    Arena* scratch = nullptr);
std::vector<QT> cluster_results(const MatchMail& mm, int t);  // type t's averages (status 0)
MatchMail* match_mail(fccf_ctx* c);
void verify_items_device(fccf_ctx* c, const std::vector<QT>& qs, const std::vector<Plane>& F1,
                         const std::vector<Plane>& F2, const MatchIn* dM, const fccf_params& P, hipStream_t st,
                         std::vector<m44>& T, std::vector<float>& score, std::vector<int>& npairs);

// Releases the per-CloudSet pipeline state (fccf_ctx_destroy).
void pipeline_release(fccf_ctx* c);

}  // namespace fccf
