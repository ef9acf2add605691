// pipeline.h — workspace layout helpers shared by api.cpp and pipeline.cpp.
#pragma once
#include "ctx.h"
#include "kernels.h"

namespace fccf {

inline size_t voxel_grid_bytes(uint32_t cap) {
  return 4 * sizeof(uint32_t) * (size_t)cap + sizeof(uint32_t) * ((size_t)cap + 1) + sizeof(float) * VG_BBOX_BLOCKS * 8 +
         sizeof(VGParams) + 64 + sort_scratch_bytes(cap) + 7 * 256;
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
  return b;
}

// Releases the per-CloudSet pipeline state (fccf_ctx_destroy).
void pipeline_release(fccf_ctx* c);

}  // namespace fccf
