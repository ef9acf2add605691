// Development probe for exactsum.hip: runs exact_sum on a raw float32 xyz file
// (e.g. a downsampled cloud dumped by the oracle) and prints kernel timings and
// chain counters.  Build: hipcc -DXS_PROBE -O3 --offload-arch=gfx950 ...
#include <chrono>
#include <cstdio>
#include <vector>

#include "../fccf-pcr_amd/csrc/exactsum.hip"

using namespace fccf;

int main(int argc, char** argv) {
  FILE* f = fopen(argv[1], "rb");
  std::vector<float> a(1 << 24);
  const size_t nf = fread(a.data(), 4, a.size(), f);
  fclose(f);
  const uint32_t n = (uint32_t)(nf / 3);
  float *d_x, *d_out;
  uint32_t* d_n;
  void* scratch;
  hipMalloc(&d_x, nf * 4);
  hipMalloc(&d_out, 64);
  hipMalloc(&d_n, 4);
  hipMalloc(&scratch, exact_sum_bytes(3, n));
  hipMemcpy(d_x, a.data(), nf * 4, hipMemcpyHostToDevice);
  hipMemcpy(d_n, &n, 4, hipMemcpyHostToDevice);
  XsBufs xs = exact_sum_carve(scratch, 3, n);
  hipStream_t st;
  hipStreamCreate(&st);
  float ref[3] = {0, 0, 0};
  for (uint32_t i = 0; i < n; ++i)
    for (int k = 0; k < 3; ++k) ref[k] += a[3 * i + k];
  for (int it = 0; it < 5; ++it) {
    unsigned long long z[8] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(xs_probe), z, sizeof(z));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0, st);
    exact_sum(d_x, 3, 3, nullptr, d_n, 1, d_out, false, xs, st);
    hipEventRecord(e1, st);
    hipStreamSynchronize(st);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    float out[3];
    hipMemcpy(out, d_out, 12, hipMemcpyDeviceToHost);
    hipMemcpyFromSymbol(z, HIP_SYMBOL(xs_probe), sizeof(z));
    printf("n %u total %.1f us exact %d%d%d scans %llu replays %llu dmiss %llu replay_clk %llu scan_clk %llu pf_miss %llu\n", n,
           ms * 1e3, out[0] == ref[0], out[1] == ref[1], out[2] == ref[2], z[0], z[1], z[2], z[3], z[4], z[5]);
  }
  return 0;
}
