// Development microbenchmark: radix sort / scan primitives of devprim.hip in
// isolation, timed as graph replays (no profiler).  Prints us per call.
// Build: hipcc -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 tools/sort_bench.hip -o scratch/sort_bench
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../fccf-pcr_amd/csrc/devprim.hip"
#include "../fccf-pcr_amd/csrc/probe.cpp"

using namespace fccf;

template <class F>
static double time_graph(hipStream_t st, int reps, F body) {
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  for (int r = 0; r < reps; ++r) body();
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a, st);
  hipGraphLaunch(ge, st);
  hipEventRecord(b, st);
  hipEventSynchronize(b);
  float ms;
  hipEventElapsedTime(&ms, a, b);
  hipGraphExecDestroy(ge);
  hipGraphDestroy(g);
  return ms * 1e3 / reps;
}

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 1000000;
  const int bits = argc > 2 ? atoi(argv[2]) : 24;
  std::vector<uint32_t> hk(n);
  uint64_t s = 12345;
  for (uint32_t i = 0; i < n; ++i) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    hk[i] = (uint32_t)(s >> 33) & ((1u << bits) - 1u);
  }
  uint32_t *k0, *v0, *k1, *v1, *kin, *dn, *dbits, *dbits0, *starts, *dseg, *dtot;
  hipMalloc(&k0, 4 * n); hipMalloc(&v0, 4 * n); hipMalloc(&k1, 4 * n); hipMalloc(&v1, 4 * n); hipMalloc(&kin, 4 * n);
  hipMalloc(&starts, 4 * (size_t)n + 64); hipMalloc(&dseg, 4); hipMalloc(&dtot, 4);
  hipMalloc(&dn, 4); hipMalloc(&dbits, 4); hipMalloc(&dbits0, 4);
  hipMemcpy(kin, hk.data(), 4 * n, hipMemcpyHostToDevice);
  hipMemcpy(dn, &n, 4, hipMemcpyHostToDevice);
  hipMemcpy(dbits, &bits, 4, hipMemcpyHostToDevice);
  const uint32_t zero = 0;
  hipMemcpy(dbits0, &zero, 4, hipMemcpyHostToDevice);
  void* scr;
  hipMalloc(&scr, sort_scratch_bytes(n));
  SortScratch ss = sort_scratch_carve(scr, n);
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  const int R = 20;
  double t_copy = time_graph(st, R, [&] { hipMemcpyAsync(k0, kin, 4 * n, hipMemcpyDeviceToDevice, st); });
  double t_sort = time_graph(st, R, [&] {
    hipMemcpyAsync(k0, kin, 4 * n, hipMemcpyDeviceToDevice, st);
    radix_sort_u32(k0, v0, k1, v1, dn, n, dbits, 32, true, ss, st);
  });
  double t_skip = time_graph(st, R, [&] {
    hipMemcpyAsync(k0, kin, 4 * n, hipMemcpyDeviceToDevice, st);
    radix_sort_u32(k0, v0, k1, v1, dn, n, dbits0, 32, true, ss, st);
  });
  const uint32_t nb = sort_blocks(n);
  double t_hist = time_graph(st, R, [&] { k_rs_hist<uint32_t><<<nb, ST, 0, st>>>(kin, dn, dbits, 0, ss.hist, nb); });
  double t_hr = time_graph(st, R, [&] {  // idempotent pair: fresh counts, then their scan
    k_rs_hist<uint32_t><<<nb, ST, 0, st>>>(kin, dn, dbits, 0, ss.hist, nb);
    k_rs_rowscan<<<256, T, 0, st>>>(ss.hist, nb, ss.tot, dbits, 0);
  });
  // scatter alone: the offsets of kin's first digit, computed once (the scatter
  // only reads them)
  k_rs_hist<uint32_t><<<nb, ST, 0, st>>>(kin, dn, dbits, 0, ss.hist, nb);
  k_rs_rowscan<<<256, T, 0, st>>>(ss.hist, nb, ss.tot, dbits, 0);
  hipStreamSynchronize(st);
  double t_sc = time_graph(st, R, [&] {
    k_rs_scatter<uint32_t><<<nb, ST, 0, st>>>(kin, v0, k1, v1, dn, dbits, 0, ss.hist, ss.tot, nb, 1, nullptr);
  });
  double t_seg = time_graph(st, R, [&] { segment_heads_u32(k0, dn, n, 0xFFFFFFFFu, starts, dseg, ss, st); });
  double t_scan = time_graph(st, R, [&] { exclusive_scan_u32(kin, k1, dn, n, dtot, ss, st); });
  const double t_row = t_hr - t_hist;
  // check sortedness
  std::vector<uint32_t> out(n);
  hipMemcpy(k0, kin, 4 * n, hipMemcpyDeviceToDevice);
  radix_sort_u32(k0, v0, k1, v1, dn, n, dbits, 32, true, ss, st);
  hipStreamSynchronize(st);
  hipMemcpy(out.data(), k0, 4 * n, hipMemcpyDeviceToHost);
  bool ok = true;
  for (uint32_t i = 1; i < n; ++i) ok &= out[i - 1] <= out[i];
  printf("n %u bits %d sorted %d | copy %.1f sort(incl copy) %.1f skipped-sort(incl copy) %.1f | hist %.1f rowscan %.1f scatter %.1f | seg_heads %.1f excl_scan %.1f us\n",
         n, bits, (int)ok, t_copy, t_sort, t_skip, t_hist, t_row, t_sc, t_seg, t_scan);
  return 0;
}
