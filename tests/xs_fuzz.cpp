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

struct Stats { long scans = 0, replays = 0; };

static float naive(const std::vector<float>& x) {
  float s = 0.f;
  for (float v : x) s += v;
  return s;
}

// Serial restatement of exactsum.hip's scan_jump: compose units cur.. under s's
// binade until the first prefix that does not validate, apply the prefix before
// it, hand that unit to `descend`, continue after it.
template <class Descend>
static void scan_jump(float& s, const std::vector<XsTab3>& T, int cnt, Stats& st, Descend descend) {
  int cur = 0;
  while (cur < cnt) {
    int E;
    int64_t M;
    if (!xs_decompose(s, &E, &M)) {
      descend(cur);
      ++cur;
      continue;
    }
    ++st.scans;
    XsSum a = xs_identity(), last = a;
    int f = cnt;
    for (int l = cur; l < cnt; ++l) {
      a = xs_compose(a, xs_pick(T[l], E));
      if (!xs_valid(a, M)) { f = l; break; }
      last = a;
    }
    if (f > cur) s = xs_apply(last, M, E);
    if (f >= cnt) break;
    descend(f);
    cur = f + 1;
  }
}

static float exact(const std::vector<float>& x, Stats& st) {
  const int n = (int)x.size(), nch = (n + XS_L - 1) / XS_L, ng = (nch + XS_G - 1) / XS_G;
  std::vector<double> pre(nch + 1, 0.0);
  for (int c = 0; c < nch; ++c) {
    double a = 0;
    for (int k = c * XS_L; k < std::min(n, (c + 1) * XS_L); ++k) a += x[k];
    pre[c + 1] = pre[c] + a;
  }
  std::vector<XsTab3> ct(nch);
  for (int c = 0; c < nch; ++c) {
    const int b = c * XS_L, m = std::min(XS_L, n - b);
    ct[c].Eb = xs_predict(pre[c]);
    XsSum* t[3] = {&ct[c].t0, &ct[c].t1, &ct[c].t2};
    for (int h = 0; h < XS_NE; ++h) *t[h] = ct[c].Eb == XS_NOE ? xs_bad() : xs_run(&x[b], 1, m, ct[c].Eb + h);
  }
  std::vector<XsTab3> gt(ng);
  for (int g = 0; g < ng; ++g) {
    gt[g].Eb = xs_predict(pre[(size_t)g * XS_G]);
    XsSum* t[3] = {&gt[g].t0, &gt[g].t1, &gt[g].t2};
    for (int h = 0; h < XS_NE; ++h) {
      XsSum a = xs_identity();
      for (int c = g * XS_G; c < std::min(nch, (g + 1) * XS_G); ++c)
        a = xs_compose(a, gt[g].Eb == XS_NOE ? xs_bad() : xs_pick(ct[c], gt[g].Eb + h));
      *t[h] = a;
    }
  }
  float s = 0.f;
  scan_jump(s, gt, ng, st, [&](int g) {
    const int c0 = g * XS_G, nc = std::min(XS_G, nch - c0);
    std::vector<XsTab3> sub(ct.begin() + c0, ct.begin() + c0 + nc);
    scan_jump(s, sub, nc, st, [&](int f) {
      ++st.replays;
      const int c = c0 + f;
      for (int k = c * XS_L; k < std::min(n, (c + 1) * XS_L); ++k) s += x[k];
    });
  });
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
  printf("trials %d mismatches %d scans %ld replays %ld\n", trials, bad, st.scans, st.replays);
  return bad ? 1 : 0;
}
