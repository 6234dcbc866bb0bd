// Host-side check of hs_math.h's sincos_k (the rollout kernels' joint-value sines and cosines), compiled by
// tests/test_sincos_k.py: the same function runs on the host here (__host__ __device__), against the C
// library's sin and cos (the oracle's). Prints the largest ulp distance of each over seeded arguments in
// |x| < 64 (2e6 of them, a third placed within 1e-9 of a multiple of pi/2), and the special cases.
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
