// Host-side check of hs_math.h's sincos_k (the rollout kernels' joint-value sines and cosines), compiled by
// tests/test_sincos_k.py: the same function runs on the host here (__host__ __device__), against the C
// library's sin and cos (the oracle's). Prints the largest ulp distance of each over seeded arguments in
// |x| < 64 (2e6 of them, a third placed within 1e-9 of a multiple of pi/2), the doubles nearest to every
// multiple of pi/2 below 2^20 and their neighbours, and the special cases.
#include <cinttypes>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>

#include "hs_math.h"

static int64_t ulps(double a, double b) {
  if (a == b) return 0;
  int64_t ia, ib;
  std::memcpy(&ia, &a, 8);
  std::memcpy(&ib, &b, 8);
  if (ia < 0) ia = INT64_MIN - ia;
  if (ib < 0) ib = INT64_MIN - ib;
  return ia > ib ? ia - ib : ib - ia;
}

int main() {
  uint64_t z = 0x9E3779B97F4A7C15ull;
  int64_t ms = 0, mc = 0;
  double worst_s = 0, worst_c = 0, max_abs = 0;
  for (int i = 0; i < 2000000; i++) {
    z = z * 6364136223846793005ull + 1442695040888963407ull;
    const double u = (double)(z >> 11) * (1.0 / 9007199254740992.0);
    double x = (u - 0.5) * 128;
    if (i % 3 == 0) x = std::nearbyint(x / 1.5707963267948966) * 1.5707963267948966 + (u - 0.5) * 2e-9;
    double s, c;
    hsd::sincos_k(x, &s, &c);
    const double S = std::sin(x), C = std::cos(x);
    const int64_t us = ulps(s, S), uc = ulps(c, C);
    if (us > ms) { ms = us; worst_s = x; }
    if (uc > mc) { mc = uc; worst_c = x; }
    max_abs = std::fmax(max_abs, std::fmax(std::fabs(s - S), std::fabs(c - C)));
  }
  // the hardest arguments of the range: the doubles nearest to n pi/2 (and their neighbours) for every
  // n with |n pi/2| < 2^20, where r = x - n pi/2 is a few ulps of x and any reduction error shows
  // (with a two-term pi/2 the error n * 1.5e-33 was thousands of ulps of r at |x| ~ 2^19)
  const long double pio2 = 1.570796326794896619231321691639751442L;
  for (int64_t n = 1; n * 1.5707963267948966 < 0x1p20; n++) {
    const double x0 = (double)((long double)n * pio2);
    for (int k = -1; k <= 1; k++) {
      const double x = k < 0 ? std::nextafter(x0, 0.0) : k > 0 ? std::nextafter(x0, 1e300) : x0;
      for (double xs : {x, -x}) {
        double s, c;
        hsd::sincos_k(xs, &s, &c);
        const int64_t us = ulps(s, std::sin(xs)), uc = ulps(c, std::cos(xs));
        if (us > ms) { ms = us; worst_s = xs; }
        if (uc > mc) { mc = uc; worst_c = xs; }
      }
    }
  }
  std::printf("max_ulp_sin %" PRId64 " at %.17g\n", ms, worst_s);
  std::printf("max_ulp_cos %" PRId64 " at %.17g\n", mc, worst_c);
  std::printf("max_abs %.3g\n", max_abs);
  const double special[] = {0.0, -0.0, 1.5707963267948966, -1.5707963267948966, 3.141592653589793,
                            -3.141592653589793, 6.283185307179586, 1e-300, 1e6, 1e300};
  for (double x : special) {
    double s, c;
    hsd::sincos_k(x, &s, &c);
    std::printf("special %.17g %" PRId64 " %" PRId64 " %d\n", x, ulps(s, std::sin(x)), ulps(c, std::cos(x)),
                std::signbit(s) == std::signbit(std::sin(x)) ? 1 : 0);
  }
  double s, c;
  hsd::sincos_k(NAN, &s, &c);
  const int nan_ok = std::isnan(s) && std::isnan(c);
  hsd::sincos_k(INFINITY, &s, &c);
  std::printf("nonfinite_nan %d\n", nan_ok && std::isnan(s) && std::isnan(c));
  return 0;
}
