// san_driver.cpp — TEST INFRASTRUCTURE: the host-only code of libfccf and the CPU
// oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5,
// "Race detection / sanitizers").  Built by tests/san/Makefile (host code only,
// no device code) and run by tests/test_sanitize.py:
//   san_driver ply <file>...   fccf_ply_read on each file (ply.cpp): "rc n checksum"
//   san_driver host            oracle registrations (fccf_oracle.cpp) of seeded scenes
//                              (synth.cpp), then libfccf's host stages (host_stages.cpp:
//                              growth + selection, select_base, transform_cluster,
//                              quick_verify + LM, fusion) on the oracle's inputs, each
//                              compared bit for bit with the oracle's outputs
// Any sanitizer report aborts the process (-fno-sanitize-recover).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../fccf-pcr_amd/csrc/host_stages.h"
#include "../../oracle/fccf_oracle.h"

using namespace fccf;

namespace {

int g_fail = 0;

template <class T>
std::vector<T> get(orc_ctx* h, const std::string& name) {
  const int64_t n = orc_get(h, name.c_str(), nullptr, 0);
  if (n < 0) {
    std::printf("missing oracle dump %s\n", name.c_str());
    ++g_fail;
    return {};
  }
  std::vector<T> v((size_t)n / sizeof(T));
  if (n) orc_get(h, name.c_str(), v.data(), n);
  return v;
}

void expect_bits(const std::string& what, const void* a, const void* b, size_t bytes, size_t na, size_t nb) {
  if (na != nb || std::memcmp(a, b, bytes) != 0) {
    std::printf("MISMATCH %s (%zu vs %zu items)\n", what.c_str(), na, nb);
    ++g_fail;
  }
}

std::vector<float> flat_planes(const std::vector<Plane>& F) {
  std::vector<float> v;
  for (const Plane& p : F) {
    v.insert(v.end(), p.c, p.c + 3);
    v.insert(v.end(), p.n, p.n + 3);
    v.push_back(p.fps);
    v.push_back((float)p.nvox);
  }
  return v;
}

// One oracle registration, then every host stage of libfccf on its inputs.
void host_case(int64_t n, double Lx, double Ly, double Lz, float leaf, int threads) {
  std::vector<float> src(3 * (size_t)n), tar(3 * (size_t)n);
  float Tgt[16];
  if (fccf_synth_pair(n, Lx, Ly, Lz, src.data(), tar.data(), Tgt) != FCCF_OK) {
    std::printf("synth failed\n");
    ++g_fail;
    return;
  }
  orc_ctx* h = orc_register(src.data(), n, tar.data(), n, leaf, ORC_ORDER_INTROSORT);
  if (!h) {
    std::printf("orc_register failed\n");
    ++g_fail;
    return;
  }
  fccf_params P;
  fccf_params_default(&P);
  std::vector<Plane> F[2];
  for (int k = 0; k < 2; ++k) {  // region growing + selection (FCCF.cpp:536-677), select_base (:429-468)
    const std::string s = std::to_string(k + 1);
    const std::vector<float> v = get<float>(h, "vox" + s);
    std::vector<VoxRec> vox(v.size() / 8);
    for (size_t i = 0; i < vox.size(); ++i) {
      std::memcpy(vox[i].c, &v[8 * i], 12);
      std::memcpy(vox[i].n, &v[8 * i + 3], 12);
      vox[i].count = (int32_t)v[8 * i + 6];
      vox[i].curvature = 0.f;
    }
    const GrowOut g = grow_and_select(vox.data(), (int)vox.size(), P);
    const std::vector<float> mine = flat_planes(g.planes), ref = get<float>(h, "planes" + s);
    expect_bits("planes" + s, mine.data(), ref.data(), 4 * std::min(mine.size(), ref.size()), mine.size(), ref.size());
    const std::vector<double> th = get<double>(h, "theta" + s);
    expect_bits("theta" + s, g.theta.data(), th.data(), 8 * std::min(th.size(), g.theta.size()), g.theta.size(),
                th.size());
    const std::vector<Base> B = select_base(g.planes, g.theta, P, k + 1);
    const std::vector<int32_t> rb = get<int32_t>(h, "bases" + s);
    expect_bits("bases" + s, B.data(), rb.data(), 16 * std::min(B.size(), rb.size() / 4), B.size(), rb.size() / 4);
    F[k] = g.planes;
  }
  std::vector<QT> cand[3];
  size_t total = 0;
  for (int t = 0; t < 3; ++t) {
    const std::vector<float> v = get<float>(h, "cand" + std::to_string(t));
    for (size_t i = 0; i + 16 <= v.size(); i += 16) {
      m44 T;
      for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) T.m[a][b] = v[i + 4 * a + b];
      cand[t].push_back(qt_from_T(T));
    }
    total += cand[t].size();
  }
  Pool pool(threads);
  for (int t = 0; t < 3; ++t) {  // transform_cluster (:1040-1231), quick_verify + LM (:680-783)
    const std::string s = std::to_string(t);
    std::vector<QT> in = cand[t], fine;
    const int cn = total ? (int)(P.seclct_cluster_number * (float)in.size() / (float)total) : 0;
    int64_t ncl = 0;
    transform_cluster(in, fine, cn, P, &ncl, threads > 1 ? &pool : nullptr);
    std::vector<float> fv;
    for (const QT& q : fine) {
      const float a[8] = {q.qw, q.qx, q.qy, q.qz, q.tx, q.ty, q.tz, q.alloc ? 1.f : 0.f};
      fv.insert(fv.end(), a, a + 8);
    }
    const std::vector<float> rf = get<float>(h, "fine" + s);
    expect_bits("fine" + s, fv.data(), rf.data(), 4 * std::min(fv.size(), rf.size()), fv.size(), rf.size());
    std::vector<float> qv(18 * fine.size());
    pool.parallel_for((int)fine.size(), [&](int i) {
      m44 T = T_from_qt(fine[(size_t)i]);
      int np = 0;
      const float sc = quick_verify(T, F[0], F[1], P, &np);
      for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) qv[18 * (size_t)i + 4 * a + b] = T.m[a][b];
      qv[18 * (size_t)i + 16] = sc;
      qv[18 * (size_t)i + 17] = (float)np;
    });
    const std::vector<float> rq = get<float>(h, "qv" + s);
    expect_bits("qv" + s, qv.data(), rq.data(), 4 * std::min(qv.size(), rq.size()), qv.size(), rq.size());
  }
  {  // fusion (:1546-1606) from the oracle's per-type best (high) records
    const std::vector<float> hv = get<float>(h, "high");
    std::vector<High> tmp;
    float best = 0.f;
    for (size_t i = 0; i + 8 <= hv.size(); i += 8) {
      High x;
      x.qt = {hv[i], hv[i + 1], hv[i + 2], hv[i + 3], hv[i + 4], hv[i + 5], hv[i + 6], 0u};
      x.score = hv[i + 7];
      tmp.push_back(x);
      if (best < x.score) best = x.score;
    }
    std::vector<High> hs;
    float sum = 0.f;
    for (const High& x : tmp)
      if (x.score > best * 0.8) {
        hs.push_back(x);
        sum += x.score;
      }
    const m44 T = fuse_answer(hs, sum);
    const std::vector<float> rt = get<float>(h, "T");
    float mine[16];
    for (int a = 0; a < 4; ++a)
      for (int b = 0; b < 4; ++b) mine[4 * a + b] = T.m[a][b];
    mine[12] = mine[13] = mine[14] = 0.f;
    mine[15] = 1.f;
    expect_bits("T", mine, rt.data(), 64, 16, rt.size());
  }
  orc_free(h);
  std::printf("host case n=%lld room=(%g,%g,%g) leaf=%g threads=%d: %s\n", (long long)n, Lx, Ly, Lz, leaf, threads,
              g_fail ? "MISMATCH" : "ok");
}

}  // namespace

int main(int argc, char** argv) {
  if (argc >= 2 && std::string(argv[1]) == "ply") {
    for (int i = 2; i < argc; ++i) {
      float* xyz = nullptr;
      int64_t n = 0;
      const int rc = fccf_ply_read(argv[i], &xyz, &n);
      uint64_t chk = 0;
      for (int64_t j = 0; rc == FCCF_OK && j < 3 * n; ++j) {
        uint32_t b;
        std::memcpy(&b, &xyz[j], 4);
        chk = chk * 1000003u + b;
      }
      std::printf("%s %d %lld %016llx\n", argv[i], rc, (long long)n, (unsigned long long)chk);
      fccf_free(xyz);
    }
    return 0;
  }
  if (argc >= 2 && std::string(argv[1]) == "host") {
    host_case(30000, 16.0, 12.0, 4.0, 0.1f, 1);
    host_case(60000, 20.0, 15.0, 4.0, 0.1f, 4);
    host_case(40000, 30.0, 24.0, 6.0, 0.1f, 3);
    return g_fail ? 1 : 0;
  }
  std::fprintf(stderr, "usage: san_driver ply <file>... | host\n");
  return 2;
}
