// ingest.h — host -> HBM upload of the clouds: a ring of
// pinned staging slots on the ctx's copy stream.  Rows are converted into a slot
// by the ingest thread pool (PLY decode or a plain copy) while the slots filled
// before it are in flight over the host link, so parsing, staging and DMA overlap.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <memory>

#include "pool.h"

namespace fccf {

struct Ingest {
  static constexpr int NSLOT = 3;
  hipStream_t su = nullptr;                 // copy stream (created on first use)
  void* slot[NSLOT] = {};                   // pinned staging, rows_per_slot * 12 B each
  hipEvent_t ev[NSLOT] = {};                // the slot's last upload
  hipEvent_t done = nullptr;                // the last upload enqueued by upload_rows
  int64_t rows_per_slot = 0;
  std::unique_ptr<Pool> pool;               // not the ctx pool: the batch's helper thread uploads
                                            // while the caller's host stages use that one
  ~Ingest();
  void init();
  // Uploads rows [0, n) as float xyz to dst on su: fill(r0, nr, out) writes rows
  // [r0, r0 + nr) to out (3 * nr floats) and returns 0 or an error code; it runs on
  // the pool's threads in parallel pieces.  Records `done` after the last chunk.
  // Returns 0 or fill's first error (uploads already enqueued still complete).
  int upload_rows(float* dst, int64_t n, const std::function<int(int64_t, int64_t, float*)>& fill);
};

}  // namespace fccf
