// fccf_cli.cpp — drop-in for the reference CLI `./FCCF {src.ply} {tar.ply} {voxel}`
// (FCCF.cpp:1646-1689): same argv, same two stdout lines, same exit codes
// (a PLY load failure prints "Couldn't read file" on stderr and exits 0).
// Extra flags after the three positional arguments never change the default output:
//   --device N   HIP device ordinal (default 0)
//   --stats      print per-stage counters/timings to stderr
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <string>

#include "../../include/fccf.h"

// Eigen 3.3 operator<<(ostream, Matrix4f) with default IOFormat: every coefficient
// right-aligned to the widest printed coefficient (stream precision 6), separated
// by one space, rows by '\n', no trailing newline.
static void print_eigen(std::ostream& os, const float* T) {
  size_t width = 0;
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 4; ++i) {
      std::stringstream s;
      s.copyfmt(os);
      s << T[4 * i + j];
      width = std::max(width, s.str().size());
    }
  for (int i = 0; i < 4; ++i) {
    if (i) os << "\n";
    for (int j = 0; j < 4; ++j) {
      if (j) os << " ";
      os.width((std::streamsize)width);
      os << T[4 * i + j];
    }
  }
}

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: %s src.ply tar.ply voxel [--device N] [--stats]\n", argv[0]);
    return 1;  // the reference dereferences argv unchecked (FCCF.cpp:1648-1650)
  }
  const float leaf = (float)std::atof(argv[3]);
  int device = 0;
  bool stats = false;
  for (int i = 4; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--device") && i + 1 < argc) device = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--stats")) stats = true;
  }
  // The clouds are streamed from the files straight into HBM (fccf_ply_load_device:
  // chunked decode overlapped with the upload).  The ctx is created first, silently,
  // so the observable order stays the reference's: both loads (either failure prints
  // "Couldn't read file" and exits 0), then "Leaf size", then the registration.
  fccf_ctx* ctx = nullptr;
  const int crc = fccf_ctx_create(&ctx, device);
  float *src = nullptr, *tar = nullptr;
  int64_t ns = 0, nt = 0;
  const char* path[2] = {argv[1], argv[2]};
  float** dst[2] = {&src, &tar};
  int64_t* cnt[2] = {&ns, &nt};
  for (int k = 0; k < 2; ++k) {
    const int lrc = crc == FCCF_OK ? fccf_ply_load_device(ctx, path[k], dst[k], cnt[k])
                                   : fccf_ply_read(path[k], dst[k], cnt[k]);
    if (lrc != FCCF_OK) {
      if (lrc != FCCF_E_IO) {
        std::cerr << "fccf: " << fccf_strerror(lrc) << "\n";
        return 2;
      }
      std::cerr << "Couldn't read file \n";
      return 0;
    }
  }
  std::cout << "Leaf size : " << leaf << std::endl;
  if (crc != FCCF_OK) {
    std::cerr << "fccf: " << fccf_strerror(crc) << "\n";
    return 2;
  }
  float T[16];
  fccf_stats st;
  int rc = fccf_register_device(ctx, src, ns, tar, nt, leaf, nullptr, T, &st);
  if (rc != FCCF_OK) {
    std::cerr << "fccf: " << fccf_strerror(rc) << "\n";
    return 2;
  }
  std::cout << "Transformation: \n";
  print_eigen(std::cout, T);
  std::cout << std::endl;
  if (stats) {
    std::fprintf(stderr, "n=%lld/%lld m=%lld/%lld planes=%lld/%lld K=%lld K_pass=%lld cand=%lld/%lld/%lld total_ms=%.3f\n",
                 (long long)st.n_src, (long long)st.n_tar, (long long)st.m_src, (long long)st.m_tar,
                 (long long)st.planes1, (long long)st.planes2, (long long)st.K, (long long)st.K_pass,
                 (long long)st.cand[0], (long long)st.cand[1], (long long)st.cand[2], st.ms_total);
  }
  fccf_device_free(ctx, src);
  fccf_device_free(ctx, tar);
  fccf_ctx_destroy(ctx);
  return 0;
}
