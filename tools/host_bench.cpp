// host_bench.cpp — CPU timing of libfccf's host stages (transform_cluster,
// quick_verify + LM) on inputs dumped from the oracle (development tool; see
// tools/host_bench.py, which writes the inputs and builds/runs this).
#include <algorithm>
#include <chrono>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <thread>
#include <cstdlib>
#include <vector>

#include "../fccf-pcr_amd/csrc/host_stages.h"

using namespace fccf;
using clk = std::chrono::steady_clock;

static std::vector<float> rd(const char* p) {
  std::ifstream f(p, std::ios::binary);
  std::vector<char> b((std::istreambuf_iterator<char>(f)), {});
  std::vector<float> v(b.size() / 4);
  std::memcpy(v.data(), b.data(), b.size());
  return v;
}
static std::vector<Plane> planes(const std::vector<float>& v) {
  std::vector<Plane> F(v.size() / 8);
  for (size_t i = 0; i < F.size(); ++i) {
    std::memcpy(F[i].c, &v[8 * i], 12);
    std::memcpy(F[i].n, &v[8 * i + 3], 12);
    F[i].fps = v[8 * i + 6];
    F[i].nvox = (int32_t)v[8 * i + 7];
  }
  return F;
}

int main(int argc, char** argv) {
  const char* d = argc > 1 ? argv[1] : "scratch/hb";
  const int reps = argc > 2 ? atoi(argv[2]) : 20;
  const int nth = argc > 3 ? atoi(argv[3]) : 1;
  std::unique_ptr<Pool> pool(nth > 1 ? new Pool(nth) : nullptr);
  uint64_t chk = 0;
  fccf_params P;
  fccf_params_default(&P);
  std::string D(d);
  auto F1 = planes(rd((D + "/planes1.bin").c_str())), F2 = planes(rd((D + "/planes2.bin").c_str()));
  std::vector<std::vector<QT>> cand(3);
  size_t total = 0;
  for (int t = 0; t < 3; ++t) {
    auto v = rd((D + "/cand" + std::to_string(t) + ".bin").c_str());
    for (size_t i = 0; i + 16 <= v.size(); i += 16) {
      m44 T;
      for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) T.m[a][b] = v[i + 4 * a + b];
      cand[t].push_back(qt_from_T(T));
    }
    total += cand[t].size();
  }
  for (int k = 1; k <= 2; ++k) {  // region growing + selection per cloud
    auto v = rd((D + "/vox" + std::to_string(k) + ".bin").c_str());
    std::vector<VoxRec> vox(v.size() / 8);
    for (size_t i = 0; i < vox.size(); ++i) {
      std::memcpy(vox[i].c, &v[8 * i], 12);
      std::memcpy(vox[i].n, &v[8 * i + 3], 12);
      vox[i].count = (int32_t)v[8 * i + 6];
      vox[i].curvature = 0.f;
    }
    double tg = 0;
    size_t ng = 0;
    for (int r = 0; r < reps; ++r) {
      auto a = clk::now();
      GrowOut g = grow_and_select(vox.data(), (int)vox.size(), P);
      tg += std::chrono::duration<double, std::micro>(clk::now() - a).count();
      ng = g.groups.size();
    }
    std::printf("grow cloud %d: %zu voxels -> %zu groups: %.1f us\n", k, vox.size(), ng, tg / reps);
  }
  for (int k = 1; k <= 2; ++k) {  // region growing + selection per cloud
    auto v = rd((D + "/vox" + std::to_string(k) + ".bin").c_str());
    std::vector<VoxRec> vox(v.size() / 8);
    for (size_t i = 0; i < vox.size(); ++i) {
      std::memcpy(vox[i].c, &v[8 * i], 12);
      std::memcpy(vox[i].n, &v[8 * i + 3], 12);
      vox[i].count = (int32_t)v[8 * i + 6];
      vox[i].curvature = 0.f;
    }
    double tg = 0;
    size_t ng = 0;
    for (int r = 0; r < reps; ++r) {
      auto a = clk::now();
      GrowOut g = grow_and_select(vox.data(), (int)vox.size(), P);
      tg += std::chrono::duration<double, std::micro>(clk::now() - a).count();
      ng = g.groups.size();
      if (r == 0)
        for (const Plane& p : g.groups) {
          uint32_t b[8];
          std::memcpy(b, &p, 32);
          for (uint32_t x : b) chk = chk * 1000003u + x;
        }
    }
    std::printf("grow cloud %d: %zu voxels -> %zu groups: %.1f us\n", k, vox.size(), ng, tg / reps);
  }
  double tc = 0, tv = 0;
  size_t nfine = 0, nlm = 0;
  for (int r = 0; r < reps; ++r) {
    for (int t = 0; t < 3; ++t) {
      std::vector<QT> in = cand[t], fine;
      const int cn = total ? (int)(P.seclct_cluster_number * (float)in.size() / (float)total) : 0;
      int64_t ncl = 0;
      auto a = clk::now();
      transform_cluster(in, fine, cn, P, &ncl, pool.get());
      auto b = clk::now();
      std::vector<int> np(fine.size());
      std::vector<float> sc(fine.size());
      std::vector<double> dt(fine.size());
      auto one = [&](int i) {
        auto a0 = clk::now();
        m44 T = T_from_qt(fine[i]);
        sc[i] = quick_verify(T, F1, F2, P, &np[i]);
        dt[i] = std::chrono::duration<double, std::micro>(clk::now() - a0).count();
      };
      if (pool && std::getenv("HB_RAW")) {  // raw threads, static partition (pool-free reference)
        std::vector<std::thread> th;
        for (int t = 0; t < nth; ++t)
          th.emplace_back([&, t] { for (int i = t; i < (int)fine.size(); i += nth) one(i); });
        for (auto& x : th) x.join();
      } else if (pool) pool->parallel_for((int)fine.size(), one);
      else for (int i = 0; i < (int)fine.size(); ++i) one(i);
      for (size_t i = 0; r == 0 && i < fine.size(); ++i) {
        if ((float)np[i] >= P.required_optimize_plane) ++nlm;
        uint32_t b;
        std::memcpy(&b, &sc[i], 4);
        chk = chk * 1000003u + b;
        std::memcpy(&b, &fine[i].tx, 4);
        chk = chk * 1000003u + b;
      }
      auto c = clk::now();
      if (std::getenv("HB_ITEMS") && r == reps - 1 && t == 0) {
        double sum = 0;
        for (double x : dt) sum += x;
        std::vector<double> sd = dt;
        std::sort(sd.begin(), sd.end(), std::greater<double>());
        std::printf("  type0 items %zu: sum of item times %.1f us, wall %.1f us, slowest %.1f %.1f %.1f %.1f us\n",
                    dt.size(), sum, std::chrono::duration<double, std::micro>(c - b).count(), sd[0], sd[1], sd[2],
                    sd[3]);
      }
      tc += std::chrono::duration<double, std::micro>(b - a).count();
      tv += std::chrono::duration<double, std::micro>(c - b).count();
      if (r == 0) nfine += fine.size();
    }
  }
  std::printf("threads %d: candidates %zu -> fine %zu (LM solves %zu): cluster %.1f us, quick_verify %.1f us (%.2f us/call)"
              " checksum %016llx\n", nth, total, nfine, nlm, tc / reps, tv / reps, nfine ? tv / reps / nfine : 0.0,
              (unsigned long long)chk);
  return 0;
}
