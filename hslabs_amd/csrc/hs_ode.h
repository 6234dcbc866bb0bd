// hs_ode.h -- the ODE rigid-body formulas the closed-loop simulation needs,
// restated for host (model load) and device (hs_sim.hip); templates on the real type
// (double everywhere the reference computes, float for the single-precision simulation).
//
// Conventions follow ODE 0.13 (the reference links an unpinned -lode built in
// double precision, makefile:7-9): dMatrix3 is row-major 3x4 (R[i*4+j]),
// quaternions are (w, x, y, z). Sums run left to right like ODE's
// dCalcVectorDot3 helpers.
#pragma once
#include <hip/hip_runtime.h>

#include <math.h>

namespace hsode {

#define HSODE_FN __host__ __device__ __attribute__((always_inline)) inline

template <class T>
HSODE_FN T dot3(const T* a, const T* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <class T>
HSODE_FN T dot3_41(const T* a, const T* b) { return a[0] * b[0] + a[4] * b[1] + a[8] * b[2]; }
template <class T>
HSODE_FN T dot3_14(const T* a, const T* b) { return a[0] * b[0] + a[1] * b[4] + a[2] * b[8]; }
template <class T>
HSODE_FN void cross3(T* r, const T* a, const T* b) {
  T r0 = a[1] * b[2] - a[2] * b[1], r1 = a[2] * b[0] - a[0] * b[2], r2 = a[0] * b[1] - a[1] * b[0];
  r[0] = r0; r[1] = r1; r[2] = r2;
}
// r = B c, B a dMatrix3 (dMultiply0_331)
template <class T>
HSODE_FN void mul0_331(T* r, const T* B, const T* c) {
  T r0 = dot3(B, c), r1 = dot3(B + 4, c), r2 = dot3(B + 8, c);
  r[0] = r0; r[1] = r1; r[2] = r2;
}
// r = B c, B 3x3 row-major (the same sums as mul0_331 on a compact matrix)
template <class T>
HSODE_FN void mul0_33(T* r, const T* B, const T* c) {
  T r0 = dot3(B, c), r1 = dot3(B + 3, c), r2 = dot3(B + 6, c);
  r[0] = r0; r[1] = r1; r[2] = r2;
}
// r = B^T c (dMultiply1_331)
template <class T>
HSODE_FN void mul1_331(T* r, const T* B, const T* c) {
  T r0 = dot3_41(B, c), r1 = dot3_41(B + 1, c), r2 = dot3_41(B + 2, c);
  r[0] = r0; r[1] = r1; r[2] = r2;
}

// rotation.cpp dQtoR
template <class T>
HSODE_FN void q_to_R(const T* q, T* R) {
  T qq1 = 2 * q[1] * q[1], qq2 = 2 * q[2] * q[2], qq3 = 2 * q[3] * q[3];
  R[0] = 1 - qq2 - qq3; R[1] = 2 * (q[1] * q[2] - q[0] * q[3]); R[2] = 2 * (q[1] * q[3] + q[0] * q[2]); R[3] = 0;
  R[4] = 2 * (q[1] * q[2] + q[0] * q[3]); R[5] = 1 - qq1 - qq3; R[6] = 2 * (q[2] * q[3] - q[0] * q[1]); R[7] = 0;
  R[8] = 2 * (q[1] * q[3] - q[0] * q[2]); R[9] = 2 * (q[2] * q[3] + q[0] * q[1]); R[10] = 1 - qq1 - qq2; R[11] = 0;
}

// rotation.cpp dQfromR
template <class T>
HSODE_FN void q_from_R(T* q, const T* R) {
#define HSODE_R(i, j) R[(i) * 4 + (j)]
  T tr = HSODE_R(0, 0) + HSODE_R(1, 1) + HSODE_R(2, 2), s;
  if (tr >= 0) {
    s = sqrt(tr + 1);
    q[0] = T(0.5) * s;
    s = T(0.5) * (T(1) / s);
    q[1] = (HSODE_R(2, 1) - HSODE_R(1, 2)) * s;
    q[2] = (HSODE_R(0, 2) - HSODE_R(2, 0)) * s;
    q[3] = (HSODE_R(1, 0) - HSODE_R(0, 1)) * s;
    return;
  }
  int c;
  if (HSODE_R(1, 1) > HSODE_R(0, 0)) c = (HSODE_R(2, 2) > HSODE_R(1, 1)) ? 2 : 1;
  else c = (HSODE_R(2, 2) > HSODE_R(0, 0)) ? 2 : 0;
  if (c == 0) {
    s = sqrt((HSODE_R(0, 0) - (HSODE_R(1, 1) + HSODE_R(2, 2))) + 1);
    q[1] = T(0.5) * s;
    s = T(0.5) * (T(1) / s);
    q[2] = (HSODE_R(0, 1) + HSODE_R(1, 0)) * s;
    q[3] = (HSODE_R(2, 0) + HSODE_R(0, 2)) * s;
    q[0] = (HSODE_R(2, 1) - HSODE_R(1, 2)) * s;
  } else if (c == 1) {
    s = sqrt((HSODE_R(1, 1) - (HSODE_R(2, 2) + HSODE_R(0, 0))) + 1);
    q[2] = T(0.5) * s;
    s = T(0.5) * (T(1) / s);
    q[3] = (HSODE_R(1, 2) + HSODE_R(2, 1)) * s;
    q[1] = (HSODE_R(0, 1) + HSODE_R(1, 0)) * s;
    q[0] = (HSODE_R(0, 2) - HSODE_R(2, 0)) * s;
  } else {
    s = sqrt((HSODE_R(2, 2) - (HSODE_R(0, 0) + HSODE_R(1, 1))) + 1);
    q[3] = T(0.5) * s;
    s = T(0.5) * (T(1) / s);
    q[1] = (HSODE_R(2, 0) + HSODE_R(0, 2)) * s;
    q[2] = (HSODE_R(1, 2) + HSODE_R(2, 1)) * s;
    q[0] = (HSODE_R(1, 0) - HSODE_R(0, 1)) * s;
  }
#undef HSODE_R
}

// odemath.cpp dSafeNormalize4
template <class T>
HSODE_FN void normalize4(T* a) {
  T l = a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
  if (l > 0) {
    l = T(1) / sqrt(l);
    a[0] *= l; a[1] *= l; a[2] *= l; a[3] *= l;
  } else {
    a[0] = 1; a[1] = a[2] = a[3] = 0;
  }
}

// odemath.cpp dSafeNormalize3 (scale by the largest magnitude first)
template <class T>
HSODE_FN void normalize3(T* a) {
  T aa0 = fabs(a[0]), aa1 = fabs(a[1]), aa2 = fabs(a[2]), l;
  if (aa1 > aa0) l = (aa2 > aa1) ? aa2 : aa1;
  else if (aa2 > aa0) l = aa2;
  else {
    if (aa0 <= 0) { a[0] = 1; a[1] = a[2] = 0; return; }
    l = aa0;
  }
  a[0] /= l; a[1] /= l; a[2] /= l;
  l = T(1) / sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  a[0] *= l; a[1] *= l; a[2] *= l;
}

// dQMultiply1: qa = conj(qb) qc
template <class T>
HSODE_FN void qmul1(T* qa, const T* qb, const T* qc) {
  T a0 = qb[0] * qc[0] + qb[1] * qc[1] + qb[2] * qc[2] + qb[3] * qc[3];
  T a1 = qb[0] * qc[1] - qb[1] * qc[0] - qb[2] * qc[3] + qb[3] * qc[2];
  T a2 = qb[0] * qc[2] - qb[2] * qc[0] - qb[3] * qc[1] + qb[1] * qc[3];
  T a3 = qb[0] * qc[3] - qb[3] * qc[0] - qb[1] * qc[2] + qb[2] * qc[1];
  qa[0] = a0; qa[1] = a1; qa[2] = a2; qa[3] = a3;
}
// dQMultiply2: qa = qb conj(qc)
template <class T>
HSODE_FN void qmul2(T* qa, const T* qb, const T* qc) {
  T a0 = qb[0] * qc[0] + qb[1] * qc[1] + qb[2] * qc[2] + qb[3] * qc[3];
  T a1 = -qb[0] * qc[1] + qb[1] * qc[0] - qb[2] * qc[3] + qb[3] * qc[2];
  T a2 = -qb[0] * qc[2] + qb[2] * qc[0] - qb[3] * qc[1] + qb[1] * qc[3];
  T a3 = -qb[0] * qc[3] + qb[3] * qc[0] - qb[1] * qc[2] + qb[2] * qc[1];
  qa[0] = a0; qa[1] = a1; qa[2] = a2; qa[3] = a3;
}

// odemath.cpp dPlaneSpace
template <class T>
HSODE_FN void plane_space(const T* n, T* p, T* q) {
  if (fabs(n[2]) > T(M_SQRT1_2)) {
    T a = n[1] * n[1] + n[2] * n[2];
    T k = T(1) / sqrt(a);
    p[0] = 0; p[1] = -n[2] * k; p[2] = n[1] * k;
    q[0] = a * k; q[1] = -n[0] * p[2]; q[2] = n[0] * p[1];
  } else {
    T a = n[0] * n[0] + n[1] * n[1];
    T k = T(1) / sqrt(a);
    p[0] = -n[1] * k; p[1] = n[0] * k; p[2] = 0;
    q[0] = -n[2] * p[1]; q[1] = n[2] * p[0]; q[2] = a * k;
  }
}

// misc.cpp dRandInt (ODE >= 0.11) given the dRand output r: low-bit folding for small n, r mod n
HSODE_FN int rand_int_from(uint32_t r, int n) {
  uint32_t un = (uint32_t)n;
  if (un <= 0x00010000u) {
    r ^= (r >> 16);
    if (un <= 0x00000100u) {
      r ^= (r >> 8);
      if (un <= 0x00000010u) {
        r ^= (r >> 4);
        if (un <= 0x00000004u) {
          r ^= (r >> 2);
          if (un <= 0x00000002u) r ^= (r >> 1);
        }
      }
    }
  }
  return (int)(r % un);
}
// dRand (32-bit LCG) then dRandInt
HSODE_FN int rand_int(uint32_t& seed, int n) {
  seed = (uint32_t)((1664525ull * seed + 1013904223ull) & 0xffffffffull);
  return rand_int_from(seed, n);
}

#undef HSODE_FN
}  // namespace hsode
