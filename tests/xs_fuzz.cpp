// Host-side fuzz of the exact parallel float-sum algorithm (fccf-pcr_amd/csrc/exactsum.h):
// the same chunk / group / chain structure as exactsum.hip, run serially, against
// the naive left-to-right float loop.  Prints "trials T mismatches M ..." .
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../fccf-pcr_amd/csrc/exactsum.h"
using namespace fccf;

struct Stats { long groups = 0, gfail = 0, chunks = 0, cfail = 0; };

static float naive(const std::vector<float>& x) {
  float s = 0.f;
  for (float v : x) s += v;
  return s;
}

static bool try_apply(float& s, const XsSum* tab, int Eb) {
  int E;
  int64_t M;
  if (Eb == XS_NOE || !xs_decompose(s, &E, &M)) return false;
  const int h = E - Eb;
  if (h < 0 || h >= XS_NE || !xs_valid(tab[h], M)) return false;
  s = xs_apply(tab[h], M, E);
  return true;
}

static float exact(const std::vector<float>& x, Stats& st) {
  const int n = (int)x.size(), nch = (n + XS_L - 1) / XS_L, ng = (nch + XS_G - 1) / XS_G;
  std::vector<double> pre(nch + 1, 0.0);
  for (int c = 0; c < nch; ++c) {
    double a = 0;
    for (int k = c * XS_L; k < std::min(n, (c + 1) * XS_L); ++k) a += x[k];
    pre[c + 1] = pre[c] + a;
  }
  std::vector<XsSum> ct((size_t)nch * XS_NE);
  std::vector<int> cE(nch);
  for (int c = 0; c < nch; ++c) {
    cE[c] = xs_predict(pre[c]);
    const int b = c * XS_L, m = std::min(XS_L, n - b);
    for (int h = 0; h < XS_NE; ++h)
      ct[(size_t)c * XS_NE + h] = cE[c] == XS_NOE ? xs_bad() : xs_run(&x[b], 1, m, cE[c] + h);
  }
  std::vector<XsSum> gt((size_t)ng * XS_NE);
  std::vector<int> gE(ng);
  for (int g = 0; g < ng; ++g) {
    gE[g] = xs_predict(pre[(size_t)g * XS_G]);
    for (int h = 0; h < XS_NE; ++h) {
      XsSum a = xs_identity();
      for (int c = g * XS_G; c < std::min(nch, (g + 1) * XS_G); ++c) {
        const int hc = gE[g] + h - cE[c];
        const bool have = gE[g] != XS_NOE && cE[c] != XS_NOE && hc >= 0 && hc < XS_NE;
        a = xs_compose(a, have ? ct[(size_t)c * XS_NE + hc] : xs_bad());
      }
      gt[(size_t)g * XS_NE + h] = a;
    }
  }
  float s = 0.f;
  for (int g = 0; g < ng; ++g) {
    ++st.groups;
    if (try_apply(s, &gt[(size_t)g * XS_NE], gE[g])) continue;
    ++st.gfail;
    for (int c = g * XS_G; c < std::min(nch, (g + 1) * XS_G); ++c) {
      ++st.chunks;
      if (try_apply(s, &ct[(size_t)c * XS_NE], cE[c])) continue;
      ++st.cfail;
      for (int k = c * XS_L; k < std::min(n, (c + 1) * XS_L); ++k) s += x[k];
    }
  }
  return s;
}

int main(int argc, char** argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 900;
  std::mt19937_64 g(argc > 2 ? atoll(argv[2]) : 7);
  int bad = 0;
  Stats st;
  std::normal_distribution<double> N(0, 1);
  std::uniform_real_distribution<double> U(0, 1);
  for (int trial = 0; trial < trials; ++trial) {
    const int n = (trial % 3 == 0) ? (int)(g() % 2000) : 1 + (int)(g() % 200000);
    std::vector<float> x(n);
    const int kind = trial % 9;
    for (int i = 0; i < n; ++i) {
      float& v = x[i];
      switch (kind) {
        case 0: v = (float)(10 + 5 * N(g)); break;                                 // growing sum
        case 1: v = (float)(5 * N(g)); break;                                      // random walk about 0
        case 2: v = (float)(-20 + 3 * N(g)); break;                                // negative
        case 3: v = (float)(std::round(N(g) * 8) / 2); break;                      // exact ties
        case 4: v = (float)(U(g) < 0.5 ? 1e-3 * N(g) : 1e3 * N(g)); break;         // mixed magnitudes
        case 5: v = (float)(U(g) * 1e-30); break;                                  // tiny (subnormal partials)
        case 6: v = (float)(std::ldexp(1.0, (int)(g() % 40) - 20) * (U(g) < .5 ? -1 : 1)); break;
        case 7: v = (i % 1000 == 7) ? (U(g) < .3 ? NAN : INFINITY) : (float)(3 + N(g)); break;
        default: v = (float)(0.37 + 0.001 * N(g)); break;                          // nearly constant
      }
    }
    const float a = naive(x), b = exact(x, st);
    uint32_t ua, ub;
    memcpy(&ua, &a, 4);
    memcpy(&ub, &b, 4);
    if (ua != ub) {
      ++bad;
      if (bad < 5) printf("MISMATCH kind %d n %d: %.9g vs %.9g\n", kind, n, a, b);
    }
  }
  printf("trials %d mismatches %d groups %ld gfail %ld chunks %ld cfail %ld\n", trials, bad, st.groups, st.gfail,
         st.chunks, st.cfail);
  return bad ? 1 : 0;
}
