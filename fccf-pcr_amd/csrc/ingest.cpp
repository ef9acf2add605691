// ingest.cpp — f2: PLY ingest and the host -> HBM upload of the
// clouds.  Reference: main loads both clouds with pcl::io::loadPLYFile<PointXYZ>
// (FCCF.cpp:1655-1665) before any compute; here the parse is chunked and every
// parsed chunk is uploaded while the next one is parsed (ingest.h), so the PLY -> HBM
// latency is max(parse, link) instead of their sum.  fccf_register's host arrays take
// the copy stream too (the runtime's pageable copy), which lets a pipelined batch
// upload pair i+1 while pair i computes.
#include "ingest.h"

#include <algorithm>
#include <atomic>
#include <cstring>
#include <thread>

#include "ctx.h"
#include "ply.h"

namespace fccf {

Ingest::~Ingest() {
  for (int i = 0; i < NSLOT; ++i) {
    if (ev[i]) (void)hipEventDestroy(ev[i]);
    if (slot[i]) (void)hipHostFree(slot[i]);
  }
  if (done) (void)hipEventDestroy(done);
  if (su) (void)hipStreamDestroy(su);
}

void Ingest::init() {
  if (su) return;
  rows_per_slot = 256 << 10;  // 3 MB of xyz per slot
  HIP_CHECK(hipStreamCreateWithFlags(&su, hipStreamNonBlocking));
  for (int i = 0; i < NSLOT; ++i) {
    if (hipHostMalloc(&slot[i], 12 * (size_t)rows_per_slot, hipHostMallocDefault) != hipSuccess)
      throw Error(FCCF_E_OOM, "hipHostMalloc ingest slot");
    HIP_CHECK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  }
  HIP_CHECK(hipEventCreateWithFlags(&done, hipEventDisableTiming));
  pool.reset(new Pool((int)std::min(16u, std::max(1u, std::thread::hardware_concurrency()))));
}

int Ingest::upload_rows(float* dst, int64_t n, const std::function<int(int64_t, int64_t, float*)>& fill) {
  init();
  const int P = pool->size();
  std::atomic<int> err{0};
  for (int64_t r0 = 0, k = 0; r0 < n; r0 += rows_per_slot, ++k) {
    const int s = (int)(k % NSLOT);
    const int64_t nr = std::min<int64_t>(rows_per_slot, n - r0);
    HIP_CHECK(hipEventSynchronize(ev[s]));  // the slot's previous upload has left the host
    float* out = (float*)slot[s];
    // pieces of >= 16k rows, at most one per thread
    const int parts = (int)std::max<int64_t>(1, std::min<int64_t>(P, nr / (16 << 10)));
    pool->parallel_for(parts, [&](int i) {
      const int64_t a = nr * i / parts, b = nr * (i + 1) / parts;
      if (const int rc = fill(r0 + a, b - a, out + 3 * a)) {
        int z = 0;
        err.compare_exchange_strong(z, rc);
      }
    });
    if (err.load()) break;
    HIP_CHECK(hipMemcpyAsync(dst + 3 * r0, out, 12 * (size_t)nr, hipMemcpyHostToDevice, su));
    HIP_CHECK(hipEventRecord(ev[s], su));
  }
  HIP_CHECK(hipEventRecord(done, su));
  return err.load();
}

}  // namespace fccf

using namespace fccf;

extern "C" int fccf_ply_load_device(fccf_ctx* c, const char* path, float** d_xyz, int64_t* n) {
  if (!c || !path || !d_xyz || !n) return FCCF_E_ARG;
  *d_xyz = nullptr;
  *n = 0;
  try {
    HIP_CHECK(hipSetDevice(c->device));
    c->ingest.init();
    ply::File f;
    if (int rc = ply::open(path, f, c->ingest.pool->size())) return rc;
    if (f.n > 0x7FFFFFFF) return FCCF_E_ARG;
    float* d = nullptr;
    if (hipMalloc((void**)&d, 12 * (size_t)std::max<int64_t>(f.n, 1)) != hipSuccess) return FCCF_E_OOM;
    int rc = FCCF_OK;
    if (ply::packed_xyz(f)) {
      // packed little-endian float rows: the mapped file is the upload's source (the
      // runtime's pageable path, 52 GB/s on the box, beats staging it ourselves)
      if (f.n) HIP_CHECK(hipMemcpyAsync(d, f.data + f.vbase, 12 * (size_t)f.n, hipMemcpyHostToDevice, c->ingest.su));
    } else {
      rc = c->ingest.upload_rows(d, f.n, [&f](int64_t r0, int64_t nr, float* out) {
        return ply::decode(f, r0, nr, out);
      });
    }
    // the buffer is complete (and the file's pages no longer read) before returning
    const hipError_t e = hipStreamSynchronize(c->ingest.su);
    if (rc || e != hipSuccess) {
      (void)hipFree(d);
      return rc ? rc : FCCF_E_HIP;
    }
    *d_xyz = d;
    *n = f.n;
    return FCCF_OK;
  } catch (const Error& e) {
    c->last_error = e.what();
    return e.code;
  } catch (const std::bad_alloc&) {
    return FCCF_E_OOM;
  } catch (...) {
    return FCCF_E_INTERNAL;
  }
}
