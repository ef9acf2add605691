// Development probe: device timestamps (ktrace.h) of the batched VoxelGrid pass as a
// graph, two clouds of N random points.  Shows where the time between kernels goes.
// Build: hipcc -DFCCF_KTRACE -O3 -std=c++17 -ffp-contract=off --offload-arch=gfx950 tools/vg_trace.hip -o scratch/vg_trace
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../fccf-pcr_amd/csrc/devprim.hip"
#include "../fccf-pcr_amd/csrc/voxelgrid.hip"
#include "../fccf-pcr_amd/csrc/probe.cpp"
#include "../fccf-pcr_amd/csrc/pipeline.h"

using namespace fccf;

int main(int argc, char** argv) {
  const uint32_t n = argc > 1 ? (uint32_t)atoi(argv[1]) : 2000;
  const int nbatch = argc > 2 ? atoi(argv[2]) : 2;
  std::vector<float> h(3 * (size_t)n);
  uint64_t s = 99;
  for (auto& v : h) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    v = (float)((s >> 40) % 100000) * 1e-4f * 20.f;
  }
  Arena a[2];
  VGBufs b[2];
  float *in[2], *out[2];
  uint32_t* sc[2];
  for (int k = 0; k < 2; ++k) {
    a[k].ensure(voxel_grid_bytes(n) + 24 * (size_t)n + (1 << 20));
    in[k] = a[k].take_n<float>(3 * (size_t)n);
    out[k] = a[k].take_n<float>(3 * (size_t)n);
    sc[k] = a[k].take_n<uint32_t>(64);
    b[k] = voxel_grid_carve(a[k], n);
    hipMemcpy(in[k], h.data(), 12 * (size_t)n, hipMemcpyHostToDevice);
    hipMemcpy(sc[k], &n, 4, hipMemcpyHostToDevice);
  }
  unsigned long long* kt;
  hipMalloc(&kt, 16 * 4096);
  hipMemcpyToSymbol(HIP_SYMBOL(g_kt), &kt, sizeof(kt));
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  voxel_grid(B2<const float*>(in[0], in[1]), B2<const uint32_t*>(sc[0], sc[1]), n, 0.05f, B2<float*>(out[0], out[1]),
             B2<uint32_t*>(sc[0] + 1, sc[1] + 1), B2<VGBufs>(b[0], b[1]), st, false, nbatch);
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int rep = 0; rep < 4; ++rep) {
    const unsigned z = 0;
    hipMemcpyToSymbol(HIP_SYMBOL(g_kt_n), &z, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, st);
    hipGraphLaunch(ge, st);
    hipEventRecord(e1, st);
    hipStreamSynchronize(st);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    unsigned cnt;
    hipMemcpyFromSymbol(&cnt, HIP_SYMBOL(g_kt_n), 4);
    std::vector<unsigned long long> t(2 * cnt);
    hipMemcpy(t.data(), kt, 16 * cnt, hipMemcpyDeviceToHost);
    if (rep < 3) continue;
    printf("n %u nbatch %d: graph %.1f us, %u kernels (id: start us)\n", n, nbatch, ms * 1e3, cnt);
    for (unsigned i = 0; i < cnt; ++i)
      printf("%2llu:%6.1f%s", t[2 * i], (t[2 * i + 1] - t[1]) / 100.0, (i % 8 == 7) ? "\n" : "  ");
    printf("\n");
  }
  return 0;
}
