// flopcount.h -- TEST INFRASTRUCTURE ONLY: a double that counts its arithmetic.
//
// hs_oracle_flops.cpp compiles the oracle with every `double` replaced by cdbl, so a run of the
// restatement counts the floating-point operations its algorithm performs (tools/flop_count.py ->
// profiles/flops.json, the algorithmic numerator of the bench's FP64 roofline). An operation is
// "trivial" when an operand makes it exact by construction: a product with an exact 0 or +-1, a sum
// with an exact 0, a quotient by 1. The reference's 4x4 affine products (matrix.cpp:78-97) are
// mostly such terms (the bottom row 0 0 0 1); the kernel's 3x4 form never issues them.
#pragma once
#include <cmath>
#include <cstdint>
#include <istream>
#include <ostream>
#include <type_traits>

struct hso_flop_counts {
  uint64_t add, mul, div, sqrt, trans, cmp, trivial;
};
extern hso_flop_counts g_hso_flops;  // single-threaded counting runs (hso_rollout)

struct cdbl {
  double v;
  cdbl() = default;
  constexpr cdbl(double x) : v(x) {}
  template <class T, class = typename std::enable_if<std::is_arithmetic<T>::value>::type>
  explicit constexpr operator T() const { return (T)v; }
  cdbl& operator+=(cdbl o);
  cdbl& operator-=(cdbl o);
  cdbl& operator*=(cdbl o);
  cdbl& operator/=(cdbl o);
};

inline bool hso_is_unit(double x) { return x == 1.0 || x == -1.0; }
inline cdbl operator+(cdbl a, cdbl b) {
  if (a.v == 0.0 || b.v == 0.0) g_hso_flops.trivial++; else g_hso_flops.add++;
  return cdbl(a.v + b.v);
}
inline cdbl operator-(cdbl a, cdbl b) {
  if (a.v == 0.0 || b.v == 0.0) g_hso_flops.trivial++; else g_hso_flops.add++;
  return cdbl(a.v - b.v);
}
inline cdbl operator*(cdbl a, cdbl b) {
  if (a.v == 0.0 || b.v == 0.0 || hso_is_unit(a.v) || hso_is_unit(b.v)) g_hso_flops.trivial++; else g_hso_flops.mul++;
  return cdbl(a.v * b.v);
}
inline cdbl operator/(cdbl a, cdbl b) {
  if (b.v == 1.0 || a.v == 0.0) g_hso_flops.trivial++; else g_hso_flops.div++;
  return cdbl(a.v / b.v);
}
inline cdbl operator-(cdbl a) { return cdbl(-a.v); }
inline cdbl operator+(cdbl a) { return a; }
inline cdbl& cdbl::operator+=(cdbl o) { return *this = *this + o; }
inline cdbl& cdbl::operator-=(cdbl o) { return *this = *this - o; }
inline cdbl& cdbl::operator*=(cdbl o) { return *this = *this * o; }
inline cdbl& cdbl::operator/=(cdbl o) { return *this = *this / o; }
inline bool operator<(cdbl a, cdbl b) { g_hso_flops.cmp++; return a.v < b.v; }
inline bool operator>(cdbl a, cdbl b) { g_hso_flops.cmp++; return a.v > b.v; }
inline bool operator<=(cdbl a, cdbl b) { g_hso_flops.cmp++; return a.v <= b.v; }
inline bool operator>=(cdbl a, cdbl b) { g_hso_flops.cmp++; return a.v >= b.v; }
inline bool operator==(cdbl a, cdbl b) { g_hso_flops.cmp++; return a.v == b.v; }
inline bool operator!=(cdbl a, cdbl b) { g_hso_flops.cmp++; return a.v != b.v; }

inline cdbl sqrt(cdbl a) { g_hso_flops.sqrt++; return cdbl(std::sqrt(a.v)); }
inline cdbl fabs(cdbl a) { return cdbl(std::fabs(a.v)); }
inline cdbl sin(cdbl a) { g_hso_flops.trans++; return cdbl(std::sin(a.v)); }
inline cdbl cos(cdbl a) { g_hso_flops.trans++; return cdbl(std::cos(a.v)); }
inline cdbl tan(cdbl a) { g_hso_flops.trans++; return cdbl(std::tan(a.v)); }
inline cdbl asin(cdbl a) { g_hso_flops.trans++; return cdbl(std::asin(a.v)); }
inline cdbl acos(cdbl a) { g_hso_flops.trans++; return cdbl(std::acos(a.v)); }
inline cdbl atan(cdbl a) { g_hso_flops.trans++; return cdbl(std::atan(a.v)); }
inline cdbl atan2(cdbl a, cdbl b) { g_hso_flops.trans++; return cdbl(std::atan2(a.v, b.v)); }
inline cdbl fmax(cdbl a, cdbl b) { g_hso_flops.cmp++; return cdbl(std::fmax(a.v, b.v)); }
inline cdbl fmin(cdbl a, cdbl b) { g_hso_flops.cmp++; return cdbl(std::fmin(a.v, b.v)); }
inline std::ostream& operator<<(std::ostream& o, cdbl a) { return o << a.v; }
inline std::istream& operator>>(std::istream& i, cdbl& a) { return i >> a.v; }
namespace std {
inline bool isnan(cdbl a) { return std::isnan(a.v); }
inline bool isfinite(cdbl a) { return std::isfinite(a.v); }
inline cdbl sqrt(cdbl a) { return ::sqrt(a); }
inline cdbl fabs(cdbl a) { return ::fabs(a); }
inline cdbl abs(cdbl a) { return ::fabs(a); }
}  // namespace std
