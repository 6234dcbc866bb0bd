// hs_math.h -- device math for the kinematic part of the path (gfx950).
//
// Rigid transforms are 3x4 column-major (hs_aff34); every product sums k = 0..2
// from an explicit 0 and adds the translation last, which is the rounding of
// the reference's 4x4 affine::mult (matrix.cpp:78-97) with its exact (0,0,0,1)
// bottom row. Its rounding follows the compiling file's contraction flag
// (hslabs_amd/build.py): hs_config.hip and hs_sim.hip (-ffp-contract=off) round
// like the reference's x86-64 -O2 build; the rollout kernels (fast) fuse a*b+c.
// `real` is double, or float for the fp32 build (hs_kernels_f32.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "hs_topo.h"

#ifndef HS_REAL
#define HS_REAL double
#endif

namespace hsd {
// one instantiation per precision (hs_kernels.hip: double, hs_kernels_f32.hip: float)
#if HS_REAL_IS_FLOAT
inline namespace f32 {
#else
inline namespace f64 {
#endif

using real = HS_REAL;
constexpr real kPi = (real)3.14159265358979323846;  // M_PI

struct A34 {
  real m[12];
  __device__ real operator()(int r, int c) const { return m[c * 3 + r]; }
  __device__ real& at(int r, int c) { return m[c * 3 + r]; }
};

__device__ inline A34 load34(const hs_aff34& s) {
  A34 a;
#pragma unroll
  for (int i = 0; i < 12; i++) a.m[i] = (real)s.m[i];
  return a;
}

// C = A * B (matrix.cpp:78-97 with bottom rows (0,0,0,1))
__device__ inline A34 mul(const A34& A, const A34& B) {
  A34 C;
#pragma unroll
  for (int c = 0; c < 4; c++)
#pragma unroll
    for (int r = 0; r < 3; r++) {
      real s = real(0);
      s = s + A(r, 0) * B(0, c);
      s = s + A(r, 1) * B(1, c);
      s = s + A(r, 2) * B(2, c);
      if (c == 3) s = s + A(r, 3);
      C.at(r, c) = s;
    }
  return C;
}

// u = A * (v, 1) (matrix.cpp:149-164)
__device__ inline void mulp(const A34& A, const real* v, real* u) {
#pragma unroll
  for (int r = 0; r < 3; r++) {
    real s = real(0);
    s = s + A(r, 0) * v[0];
    s = s + A(r, 1) * v[1];
    s = s + A(r, 2) * v[2];
    s = s + A(r, 3);
    u[r] = s;
  }
}

// affine::invert_rigidbody (matrix.cpp:182-193)
__device__ inline A34 invert(const A34& A) {
  A34 I;
  real t[3] = {-A(0, 3), -A(1, 3), -A(2, 3)};
#pragma unroll
  for (int r = 0; r < 3; r++)
#pragma unroll
    for (int c = 0; c < 3; c++) I.at(r, c) = A(c, r);
#pragma unroll
  for (int r = 0; r < 3; r++) {
    real s = real(0);
    s = s + I(r, 0) * t[0];
    s = s + I(r, 1) * t[1];
    s = s + I(r, 2) * t[2];
    I.at(r, 3) = real(0) + s;
  }
  return I;
}

// Values made opaque to the optimizer where hs_rollout_kernel passes them through LDS: there a product
// stored to LDS and loaded back is a rounded operand, here a register whose defining multiply the
// instruction selector would contract into the consuming add (-ffp-contract=fast), rounding once where
// hs_rollout_kernel rounds twice (f's torque = amr * inv added into particular_sub's cross term, g's
// force = mr * inv added into the subtree sums: 1e-14 differences). The asm emits nothing.
// hs_rollout_kernel's two-contact closed form fences its assembled system the same way (both kernels: the
// contraction across the assembly and the factorization depends on the surrounding code)
// (not volatile: a volatile asm is a scheduling boundary, and the step has dozens of these)
template <int N>
__device__ inline void opaque_vals(real* v) {
#pragma unroll
  for (int j = 0; j < N; j++) asm("" : "+v"(v[j]));
}

// sines / cosines of three Euler angles (one shared range reduction per angle:
// sincos is bitwise identical to sin and cos, tools/sincos_check.hip)
struct SC3 {
  real sphi, cphi, sth, cth, spsi, cpsi;
};

#if HS_REAL_IS_FLOAT
__device__ inline void sincos(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ inline void sincos_k(float x, float* s, float* c) { sincosf(x, s, c); }
__device__ inline void sincos_k_small(float x, float* s, float* c) { sincosf(x, s, c); }
#else
// sin and cos of an angle of moderate size (joint values, step phases: |x| < 2^20) for the rollout
// kernels: n = rint(x 2/pi), r = x - n pi/2 in three FMAs against pi/2 = P1 + P2 + P3 (+ 5.6e-50): the
// first is exact (r is a multiple of x's or P1's ulp and |r| <= pi/4 + 1), and the third term keeps r
// accurate where x lies within rounding of a multiple of pi/2 (two terms left an absolute error of
// n * 1.5e-33, thousands of ulps of r ~ 1e-16 at |x| ~ 2^19), then the fdlibm kernel
// polynomials on |r| <= pi/4 and the quadrant's swap and signs -- about half the instructions of the
// library's sincos (whose reduction carries a double-double tail and whose large-argument path shares
// the code), within 1 ulp (sin) / 2 ulp (cos) of the C library's (tests/test_sincos_k.py runs it on the
// host, near-multiples of pi/2 up to 2^20 included); sin(-0) comes out +0. Larger or non-finite x: the
// library's sincos.
// sincos_k's fast path alone (|x| < 2^20; larger or non-finite x give garbage): for callers that route
// such arguments elsewhere (the limb-lane kernel defers those steps), without the library's Payne-Hanek
// reduction inlined at every call site
__host__ __device__ inline void sincos_k_small(double x, double* s, double* c);
__host__ __device__ inline void sincos_k(double x, double* s, double* c) {
  if (!(fabs(x) < 0x1p20)) {
    ::sincos(x, s, c);
    return;
  }
  sincos_k_small(x, s, c);
}
__host__ __device__ inline void sincos_k_small(double x, double* s, double* c) {
  const double n = rint(x * 6.36619772367581382433e-01);  // 2/pi
  const double r = fma(-n, -0x1.f1976b7ed8fbcp-110,
                       fma(-n, 0x1.1a62633145c07p-54, fma(-n, 0x1.921fb54442d18p+0, x)));  // P3, P2, P1
  const double z = r * r;
  // __kernel_sin (S1..S6) and __kernel_cos (C1..C6) of fdlibm, tail argument 0
  const double ps = 8.33333333332248946124e-03 +
                    z * (-1.98412698298579493134e-04 +
                         z * (2.75573137070700676789e-06 + z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10)));
  const double sr = r + (z * r) * (-1.66666666666666324348e-01 + z * ps);
  const double pc = z * (4.16666666666666019037e-02 +
                         z * (-1.38888888888741095749e-03 +
                              z * (2.48015872894767294178e-05 +
                                   z * (-2.75573143513906633035e-07 +
                                        z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11)))));
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double cr = w + (((1.0 - w) - hz) + z * pc);
  const int q = (int)n;
  double ss = (q & 1) ? cr : sr, cc = (q & 1) ? sr : cr;
  if (q & 2) ss = -ss;
  if ((q + 1) & 2) cc = -cc;
  *s = ss;
  *c = cc;
}
#endif

__device__ inline SC3 sincos3(real phi, real theta, real psi) {
  SC3 t;
  sincos(phi, &t.sphi, &t.cphi);
  sincos(theta, &t.sth, &t.cth);
  sincos(psi, &t.spsi, &t.cpsi);
  return t;
}

// ODE dRFromEulerAngles transposed into affine layout (model.cpp:45, visualization.cpp:62-69)
__device__ inline A34 from_euler_sc(const real* pos, const SC3& t) {
  const real sphi = t.sphi, cphi = t.cphi, sth = t.sth, cth = t.cth, spsi = t.spsi, cpsi = t.cpsi;
  A34 A;
  // column c of the affine = row c of the ODE matrix
  A.at(0, 0) = cpsi * cth;
  A.at(1, 0) = spsi * cth;
  A.at(2, 0) = -sth;
  A.at(0, 1) = cpsi * sth * sphi - spsi * cphi;
  A.at(1, 1) = spsi * sth * sphi + cpsi * cphi;
  A.at(2, 1) = cth * sphi;
  A.at(0, 2) = cpsi * sth * cphi + spsi * sphi;
  A.at(1, 2) = spsi * sth * cphi - cpsi * sphi;
  A.at(2, 2) = cth * cphi;
  A.at(0, 3) = pos[0];
  A.at(1, 3) = pos[1];
  A.at(2, 3) = pos[2];
  return A;
}

__device__ inline A34 from_euler(const real* pos, real phi, real theta, real psi) {
  return from_euler_sc(pos, sincos3(phi, theta, psi));
}

// free joint transformation: set_rotation then translate (model.cpp:37-49); t = sincos3 of q6[3..5]
__device__ inline A34 free_joint_sc(const real* q6, const SC3& t) {
  A34 A = from_euler_sc(q6, t);
#pragma unroll
  for (int r = 0; r < 3; r++) A.at(r, 3) = real(0) + q6[r];
  return A;
}

__device__ inline A34 free_joint(const real* q6) { return free_joint_sc(q6, sincos3(q6[3], q6[4], q6[5])); }

// hinge transformation Rz(q) (model.cpp:50-57)
// mul(A, hinge_joint(q)) given (cos q, sin q), without the products by the hinge's zeros and
// one: column 0 = A0 c + A1 s, column 1 = A0 (-s) + A1 c (mul's sums with the zero terms
// dropped, which add exact zeros), columns 2 and 3 copied
__device__ inline A34 mul_hinge(const A34& A, real c, real s) {
  A34 C;
#pragma unroll
  for (int r = 0; r < 3; r++) {
    C.at(r, 0) = fma(A(r, 1), s, A(r, 0) * c);
    C.at(r, 1) = fma(A(r, 1), c, A(r, 0) * (-1 * s));
    C.at(r, 2) = A(r, 2);
    C.at(r, 3) = A(r, 3);
  }
  return C;
}

__device__ inline A34 hinge_joint(real q) {
  real c, s;
  sincos(q, &s, &c);
  A34 A;
#pragma unroll
  for (int i = 0; i < 12; i++) A.m[i] = real(0);
  A.at(2, 2) = real(1);
  A.at(0, 0) = c;
  A.at(0, 1) = -1 * s;
  A.at(1, 1) = c;
  A.at(1, 0) = 1 * s;
  return A;
}

// euler_angles_from_affine (visualization.cpp:81-101)
__device__ inline void euler_from(const A34& A, real* ang) {
  real r11 = A(0, 0), r21 = A(1, 0), r31 = A(2, 0), r32 = A(2, 1), r33 = A(2, 2);
  real th1 = -asin(r31);
  real ct1 = cos(th1);
  ang[0] = atan2(r32 / ct1, r33 / ct1);
  ang[1] = th1;
  ang[2] = atan2(r21 / ct1, r11 / ct1);
}

__device__ inline real norm3(const real* v) {
  real s = real(0);
  s = s + v[0] * v[0];
  s = s + v[1] * v[1];
  s = s + v[2] * v[2];
  return sqrt(s);
}

// limb_solver_yxx (lik.cpp:151-184) and limb_solver_zxx (lik.cpp:189-223), bend = true, as one
// straight-line sequence (kind only picks constants, so the independent atan2 and acos chains share
// a basic block the scheduler can interleave); every operation is the solvers' own:
//   yxx: d = p - (0, 0, s0 l0), c = (p2 - s0 l0) / l, theta = acos c + (1 - s0) pi/2,
//        beta = s0 acos(.), gamma = s0 acos(.)
//   zxx: d = p + (0, 0, l0),    c = (p2 + l0) / l,    theta = acos c - s0 pi/2,
//        beta = acos(.),    gamma = acos(.)
// (x - (-l0) = x + l0 and the angle offsets are exact). mod_twopi (visualization.cpp:73-79): atan2
// is already in [-pi, pi], and theta in [0, 2 pi] (yxx) or [-pi/2, 3 pi/2] (zxx) needs at most one
// subtraction of 2 pi.
__device__ inline void limb_ik(int kind, const real* ls, int ysign, const real* p, real* ja, bool ignore_reach,
                               bool& unreach, bool& fail) {
  const real l0 = ls[0], l1 = ls[1], l2 = ls[2];
  const int s0 = ysign;
  const bool yxx = kind == HS_LIK_YXX;
  const real z0 = yxx ? s0 * l0 : -l0;
  real d[3];
  d[0] = p[0] - real(0); d[1] = p[1] - real(0); d[2] = p[2] - z0;
  real l = norm3(d);
  const bool out = l1 + l2 - l < 0;
  if (out) {
    if (ignore_reach) unreach = true;
    else fail = true;
  }
  l = (out && ignore_reach) ? l1 + l2 : l;
  const real phi = atan2(p[0], p[1]);
  const real c = (p[2] - z0) / l;
  const real toff = yxx ? (s0 > 0 ? real(0) : kPi) : (s0 > 0 ? -kPi / 2 : kPi / 2);
  real theta = acos(c) + toff;
  theta = (theta > kPi) ? theta - 2 * kPi : theta;
  const real ll = l * l;
  const real del = l2 * l2 - l1 * l1;
  const real sb = yxx ? real(s0) : real(1);  // s1 s0 (yxx) or s1 (zxx), s1 = 1 (bend)
  const real beta = sb * acos((ll - del) / (2 * l1 * l));
  const real gamma = sb * acos((ll + del) / (2 * l2 * l));
  ja[0] = -phi;
  ja[1] = -theta + beta;
  ja[2] = -(beta + gamma);
}

}  // inline namespace
}  // namespace hsd
