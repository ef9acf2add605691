// Host-side fuzz of key_div (fccf-pcr_amd/csrc/fccf_math.h): the octree key of a
// coordinate offset through a multiplication by 1/res, with the IEEE division near
// integers, against (uint32_t)(a / res).  Offsets near every multiple of res (a few ulps
// either side), random ones, powers of two.  Then morton_code's bit spreads against the
// per-level loop.  Prints "trials T mismatches M".
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <random>

#include "../fccf-pcr_amd/csrc/fccf_math.h"
using namespace fccf;

int main() {
  std::mt19937_64 rng(12345);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  const double fixed[] = {0.5, 1.0, 0.05, 0.1, 0.25, 0.3, 1.0 / 3.0, 0.7, 2.0, 0.01};
  long trials = 0, bad = 0;
  for (int r = 0; r < 60; ++r) {
    const double res = r < 10 ? fixed[r] : (double)(float)(0.005 + 2.0 * u(rng));  // (float-valued, as the params are)
    const double inv = 1.0 / res;
    auto check = [&](double a) {
      if (!(a >= 0.0) || a / res >= 4294967295.0) return;
      ++trials;
      if (key_div(a, res, inv) != (uint32_t)(a / res)) {
        if (++bad <= 10) std::printf("mismatch res %.17g a %.17g: %u vs %u\n", res, a, key_div(a, res, inv), (uint32_t)(a / res));
      }
    };
    for (int k = 0; k < 20000; ++k) {
      const double m = (double)(k < 4000 ? k : (uint64_t)(u(rng) * 2e6));
      const double c = m * res;
      double lo = c, hi = c;
      for (int s = 0; s < 6; ++s) {  // ulps either side of the multiple
        check(lo);
        check(hi);
        lo = std::nextafter(lo, 0.0);
        hi = std::nextafter(hi, 1e300);
      }
      check((double)(float)c);  // float coordinates minus a double minimum land near these too
      check(u(rng) * 512.0);
    }
    for (int e = -30; e < 30; ++e) check(std::ldexp(1.0, e));
  }
  // morton_code's bit spreads against the per-level loop it replaced (depth <= 21)
  for (int t = 0; t < 2000000; ++t) {
    const uint32_t depth = (uint32_t)(rng() % 22), kx = (uint32_t)rng(), ky = (uint32_t)rng(), kz = (uint32_t)rng();
    const uint32_t sx = t & 1 ? kx : kx & ((1u << (depth & 31)) - 1u);  // in range, and not
    uint64_t m = 0;
    for (int bit = (int)depth - 1; bit >= 0; --bit)
      m = (m << 3) | ((uint64_t)((sx >> bit) & 1u) << 2) | ((uint64_t)((ky >> bit) & 1u) << 1) | (uint64_t)((kz >> bit) & 1u);
    ++trials;
    if (morton_code(sx, ky, kz, depth) != m && ++bad <= 10) std::printf("morton mismatch depth %u\n", depth);
  }
  std::printf("trials %ld mismatches %ld\n", trials, bad);
  return bad ? 1 : 0;
}
