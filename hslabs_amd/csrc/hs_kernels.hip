// hs_kernels.hip -- the batched control-loop hot path on gfx950 (MI355X).
//
// Two rollouts per wavefront (one 64-thread workgroup), 32 lanes each. Per
// rollout the half-wave
//   S  sets up the gait (pgssweeper::setup_pergen, pergen.cpp:453-507),
//   K  samples the trajectory: lane = (sample, limb) runs pergen set_rec
//      (pergen.cpp:225-239), the torso/body chain FK, limb IK (lik.cpp:151-223,
//      316-347) and the limb FK (model.cpp:183-201), and writes the dynamic
//      features of the parts it owns (dynrec.cpp:134-155) to LDS,
//   D  lane = part: 5-point finite differences (dynrec.cpp:175-224),
//   S1 lane = part, leaves -> root: particular solution of B0 x = f
//      (replaces the SparseQR solve of ftsolver.cpp:107-113 by the tree
//      back-substitution B0's block-triangular structure allows),
//   S3 the lexicographic least squares of ftsolver.cpp:185-236 in closed form
//      (one lane per contact + a 6x6 Schur complement); a conditioning guard
//      sends the step to the out-of-line Eigen-style FullPivLU/ColPivQR path
//      (tree-built null basis, Gram matrices in a global-memory workspace),
//   S4 motor torques, contact forces and positive work (periodic.cpp:261-343).
//
// LDS layout: a launch solves one step per rollout, so the five stencil
// samples keep only what that step reads -- pos/ust at t-2dt, t, t+2dt, R at
// t+-dt, q at t-dt..t+dt, joint/foot features at t -- and the stencil-only
// block is reused by the fast solve once D has consumed it (9.5 KB per
// hexapod rollout). A horizon H > 1 is H launches (hs_capi.cpp): the sampler
// is latency-bound, so recomputing the window on 30 lanes costs about what a
// sliding window's one new sample on 6 lanes would, at twice the occupancy.
//
// Every floating-point operation sequence matches oracle/hs_oracle.cpp
// (compiled with -ffp-contract=off), so the only expected differences against
// it are ULP differences of the device sin/cos/atan2/acos/asin.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>
#include <type_traits>

#include "hs_internal.h"
#include "hs_math.h"

namespace {

using namespace hsd;

constexpr int WAVE = 64;
constexpr int HALF = 32;     // lanes per rollout: two rollouts per wavefront
constexpr int NS = 5;        // samples in the derivative stencil (periodic.cpp:192-202)
static_assert(NS * HS_LMAX <= HALF && 6 + HS_NMAX <= HALF && HS_KMAX <= HALF, "a rollout's lane maps exceed 32");
#ifndef HS_MIN_WAVES
#define HS_MIN_WAVES 2  // waves per SIMD the H = 1 register budget allows (8 workgroups/CU at 19.5 KB LDS)
#endif

// ---------------------------------------------------------------------------
// LDS layouts
// ---------------------------------------------------------------------------
// NM = part capacity of the LDS layouts (the host picks the smallest instantiation >= n,
// so LDS per rollout follows the model: hexapod 9.5 KB).

struct SchurL {  // per-contact Schur complement (all D_c invertible)
  double Dinv[HS_LMAX][9], S[HS_LMAX][36], h[HS_LMAX][6];
  double lam[6];
};

struct AugL {  // augmented system K = D + rho A^T A (a singular D_c)
  double K[HS_KMAX * HS_KMAX], X[HS_KMAX * 7], St[36], lam[6];
  int ok;
};

struct FastL {  // blocks of the closed-form solve
  double A[HS_LMAX][18], D[HS_LMAX][9], g[HS_LMAX][3];
  int ok[HS_LMAX];
  union {
    SchurL sc;
    AugL ag;
  };
};

struct WorkL {  // per-joint positive work of the step (outputs phase; FastL is dead by then)
  double wd[HS_NMAX];
};

// Workspace of the general path (k x k matrices, leading dimension LD >= k).
// SHARED: in LDS (the dead stencil block, k <= 12: any 4-legged model, up to 4
// contacts of a 6-legged one); otherwise one global-memory slot per rollout.
template <int LD_, bool SHARED_>
struct GenMats {
  static constexpr int LD = LD_;
  static constexpr bool SHARED = SHARED_;
  double ntn0[LD * LD], lu[LD * LD], Ny[LD * LD], qr[LD * LD];
  double n1[LD / 3][9];  // 3x3 diagonal blocks of the first-order Gram (column-major)
  double ntx0[LD], ntx1[LD], y0[LD], b[LD], z[LD], c[LD], hc[LD], nu[LD], nd[LD];
  int8_t rowsT[LD], colsT[LD], q[LD], piv[LD], rycol[LD], cperm[LD];
};
using GenLDS = GenMats<12, true>;
using GenWS = GenMats<HS_KMAX, false>;

template <int NM>
struct StencilL {  // fields only the finite differences read
  double pos[2][NM][3];  // t-2dt, t+2dt
  double ust[3][NM][3];  // t-2dt, t, t+2dt
  double rot[2][NM][9];  // t-dt, t+dt
};

template <int NM>
struct CentreL {  // fields read after D
  double pos[NM][3], jpos[NM][3], jz[NM][3], fpos[HS_LMAX][3];
  double q[3][6 + NM];  // t-dt, t, t+dt
  int contact[HS_LMAX];
  int unreach[HS_LMAX];
};

struct ForceL {  // solve_forces: W = I + G G^T, later the normal matrix; L^-1 [C | d]
  double W[(6 + HS_KMAX) * (6 + HS_KMAX)];
  double Ct[(6 + HS_KMAX) * (HS_KMAX + 1)];
  double y[HS_KMAX];
};

template <int NM, bool FORCES>
struct OneStore {
  union {
    StencilL<NM> sten;
    FastL fl;  // written only after D has consumed the stencil
    GenLDS gl;  // general path, k <= 12 (fast solve declined)
    WorkL wk;
    typename std::conditional<FORCES, ForceL, WorkL>::type fr;  // forces-given-torques mode
  };
  CentreL<NM> c;
};

struct SetupL {
  double pos0[HS_LMAX][3];  // default foot positions, pergen order
  double ts[HS_LMAX], xs[HS_LMAX];
  double t_step, max_radius, v, dt;
};

template <int NM>
struct SolveL {
  union {  // particular() overwrites each part's f with its x in place
    double f[6 * NM];
    double x[6 * NM];
  };
  double y[HS_KMAX];
  int cfoot[HS_LMAX];
};

template <int NM, bool FORCES>
struct Smem {
  OneStore<NM, FORCES> d;
  SetupL st;
  SolveL<NM> sv;
};

// Cross-lane exchange through LDS inside the single wave of a workgroup: an
// LDS-only workgroup fence (lgkmcnt, no vmcnt, so HBM stores stay in flight).
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// The general path with a global workspace also needs its HBM stores performed.
template <class G>
__device__ inline void gsync() {
  if constexpr (G::SHARED) wave_sync();
  else __syncthreads();
}

#ifdef HS_STAMPS
// diagnostic build only: per-phase shader-clock stamps of the first 4096 rollouts
__device__ unsigned long long g_stamps[4096][16];
#define STAMP(slot)                                                                                    \
  do {                                                                                                 \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_stamps[blockIdx.x][slot] = __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define STAMP(slot) do {} while (0)
#endif

// ballot over the 32 lanes of this rollout (bit l = sub-lane l)
__device__ inline uint32_t half_ballot(bool pred) {
  return (uint32_t)(__ballot(pred) >> (threadIdx.x & HALF));
}

__device__ inline A34 node_joint_parent(const hs_topo* T, int v) { return load34(T->node[v].J_A_parent); }
__device__ inline A34 node_pj(const hs_topo* T, int v) { return load34(T->node[v].A_pj_body); }

// ---------------------------------------------------------------------------
// Sample views. k = offset from the step's centre sample (-2..2).
// ---------------------------------------------------------------------------
template <int NM, bool FORCES>
struct OneWin {
  OneStore<NM, FORCES>* d;
  __device__ bool want_pos(int k) const { return (k & 1) == 0; }
  __device__ bool want_ust(int k) const { return (k & 1) == 0; }
  __device__ bool want_rot(int k) const { return (k & 1) != 0; }
  __device__ bool want_q(int k) const { return k >= -1 && k <= 1; }
  __device__ bool want_centre(int k) const { return k == 0; }
  __device__ double* pos(int k, int v) const { return k == 0 ? d->c.pos[v] : d->sten.pos[k > 0][v]; }
  __device__ double* ust(int k, int v) const { return d->sten.ust[(k + 2) >> 1][v]; }
  __device__ double* rot(int k, int v) const { return d->sten.rot[k > 0][v]; }
  __device__ double* q(int k) const { return d->c.q[k + 1]; }
  __device__ double* jpos(int, int v) const { return d->c.jpos[v]; }
  __device__ double* jz(int, int v) const { return d->c.jz[v]; }
  __device__ double* fpos(int, int f) const { return d->c.fpos[f]; }
  __device__ int& contact(int, int f) const { return d->c.contact[f]; }
  __device__ int& unreach(int, int L) const { return d->c.unreach[L]; }
};

// ---------------------------------------------------------------------------
// S: gait setup, lanes L < n_limbs (pergen.cpp:453-507, 30-51, 143-153)
// ---------------------------------------------------------------------------
__device__ void gait_setup(const hs_topo* T, const hs_gait_params& g, int n_t, SetupL& st, int lane) {
  const int nl = T->n_limbs;
  if (lane < nl) {
    const int L = lane;
    double q6[6] = {g.torso_pos[0], g.torso_pos[1], g.torso_pos[2],
                    g.torso_angles[0], g.torso_angles[1], g.torso_angles[2]};
    A34 A0 = mul(mul(node_joint_parent(T, 0), free_joint(q6)), node_pj(T, 0));  // orient_torso
    A34 A = A0;
    for (int k = 1; k < T->limb_chain_len[L]; k++) A = mul(A, node_pj(T, T->limb_chain[L][k]));
    int c = T->limb_child[L];
    A34 Ac = mul(mul(mul(A, node_joint_parent(T, c)), hinge_joint(0.0)), node_pj(T, c));
    double pos[3] = {Ac(0, 3), Ac(1, 3), Ac(2, 3)};  // get_limb_hip_pos
    if (g.foot_shift_type == 0) {                   // setup_foot_shift / shift_pos0
      double sh[3] = {0.0, g.foot_shift, 0.0}, ls[3];
      mulp(A0, sh, ls);
      if (L % 2) for (int i = 0; i < 3; i++) ls[i] *= -1;
      for (int i = 0; i < 3; i++) pos[i] += ls[i];
    } else if (g.foot_shift_type == 1) {
      double x = pos[0], y = pos[1];
      double f = g.foot_shift / sqrt(x * x + y * y);
      double d[3] = {x * f, y * f, 0.0};
      for (int i = 0; i < 3; i++) pos[i] += d[i];
    }
    int j = T->limb_pergen[L];
    st.pos0[j][0] = pos[0];
    st.pos0[j][1] = pos[1];
    st.pos0[j][2] = T->rcap;  // set_limb_poss
  }
  if (lane == 0) {  // periodicgenerator::set_step_duration
    double f = g.step_duration;
    int n = nl;
    double t_step = f * (1. / 2 - 1. / n) + 1. / n;
    for (int i = 0; i < 2; i++) {
      int jmax = n / 2;
      int z = (jmax == 1) ? 1 : jmax - 1;
      for (int jj = 0; jj < jmax; jj++) {
        int k = jj + i * jmax;
        double ts = jj * (1. / 2 - t_step) / z + double(i) / 2;
        st.ts[k] = ts;
        st.xs[k] = ts + t_step / 2 - 1. / 2;
      }
    }
    st.t_step = t_step;
    st.v = g.step_length / g.period;  // pergensetup::set_TLh
    st.dt = g.period / n_t;           // record_trajectory
  }
  wave_sync();
  if (lane == 0) {  // compute_max_radius
    double mr = 0;
    if (g.curvature != 0) {
      double cy = 1. / g.curvature;
      for (int j = 0; j < nl; j++) {
        double d0 = st.pos0[j][0] - 0.0, d1 = st.pos0[j][1] - cy, d2 = st.pos0[j][2] - 0.0;
        double s = 0;
        s += d0 * d0;
        s += d1 * d1;
        s += d2 * d2;
        double rad = sqrt(s);
        if (rad > mr) mr = rad;
      }
    }
    st.max_radius = mr;
  }
  wave_sync();
}

// ---------------------------------------------------------------------------
// K: one (sample, limb) pair per lane
// ---------------------------------------------------------------------------
__device__ inline double stepx(double t) { return (1 - cos(kPi * t)) / 2; }
__device__ inline double stepz(double t) { double a = sin(kPi * t); return a * a; }

template <class W>
__device__ void node_features(const hs_topo* T, int v, const A34& A, const A34* J, const W& w, int k) {
  const hs_node& nd = T->node[v];
  if (w.want_pos(k)) {
    double com[3] = {nd.com[0], nd.com[1], nd.com[2]}, p[3];
    mulp(A, com, p);
    double* P = w.pos(k, v);
    for (int i = 0; i < 3; i++) P[i] = p[i];
  }
  if (w.want_ust(k)) {
    double* U = w.ust(k, v);
    U[0] = (A(2, 1) - A(1, 2)) / 2;
    U[1] = (A(0, 2) - A(2, 0)) / 2;
    U[2] = (A(1, 0) - A(0, 1)) / 2;
  }
  if (w.want_rot(k)) {
    double* R = w.rot(k, v);
    for (int c = 0; c < 3; c++)
      for (int r = 0; r < 3; r++) R[c * 3 + r] = A(r, c);
  }
  if (w.want_centre(k)) {
    double* Jp = w.jpos(k, v);
    double* Jz = w.jz(k, v);
    for (int i = 0; i < 3; i++) Jp[i] = J ? (*J)(i, 3) : A(i, 3);
    for (int i = 0; i < 3; i++) Jz[i] = J ? (*J)(i, 2) : 0.0;
    if (nd.foot >= 0) {
      double cap[3] = {nd.cap[0], nd.cap[1], nd.cap[2]}, fp[3];
      mulp(A, cap, fp);
      double* F = w.fpos(k, nd.foot);
      for (int i = 0; i < 3; i++) F[i] = fp[i];
      w.contact(k, nd.foot) = fp[2] < T->rcap + 1e-4;
    }
  }
}

template <class W>
__device__ void kin_sample(const hs_topo* T, const hs_gait_params& g, const SetupL& st, int isample, int L,
                           bool ignore_reach, const W& w, int k) {
  double t = 0;  // t accumulates dt (periodic.cpp:171-181)
  for (int i = 0; i < isample; i++) t += st.dt;
  // pergensetup::set_rec -> turn_torso (pergen.cpp:386-397)
  double o0[3] = {g.torso_pos[0], g.torso_pos[1], g.torso_pos[2]};
  double o1[3] = {g.torso_angles[0], g.torso_angles[1], g.torso_angles[2]};
  double tv = t * st.v;
  bool turned = false;
  double psi = 0;
  if (g.curvature != 0) {
    int s = (g.curvature > 0) ? 1 : -1;
    psi = s * tv / st.max_radius;
    turned = psi != 0;
  }
  if (!turned) {
    o0[0] += tv;
  } else {
    double rc = 1. / g.curvature;
    double tp[3] = {rc * sin(psi), rc * (1 - cos(psi)), 0};
    A34 At = from_euler(tp, 0.0, 0.0, psi);
    A34 A0 = from_euler(o0, o1[0], o1[1], o1[2]);
    A34 A1 = mul(At, A0);
    o0[0] = A1(0, 3); o0[1] = A1(1, 3); o0[2] = A1(2, 3);
    euler_from(A1, o1);
  }
  // periodicgenerator::limb_positions for this limb's pergen index (pergen.cpp:82-94)
  int j = T->limb_pergen[L];
  double target[3];
  {
    double tt = t / g.period;
    int t_int = int(tt);
    double t_frac = tt - t_int;
    double t_lift = st.ts[j], stepf;
    if (t_frac < t_lift) stepf = 0;
    else if (t_frac < t_lift + st.t_step) stepf = (t_frac - t_lift) / st.t_step;
    else stepf = 1;
    double dx = (t_int + st.xs[j] + stepx(stepf)) * g.step_length;
    double dy = 0;
    double dz = stepz(stepf) * g.step_height;
    if (g.curvature != 0) {  // turn_position (pergen.cpp:160-183)
      int s = (g.curvature > 0) ? 1 : -1;
      double x0 = st.pos0[j][0], y0 = st.pos0[j][1];
      double rc = 1. / g.curvature;
      double rx = x0, ry = y0 - rc;
      double r = sqrt(rx * rx + ry * ry);
      double alpha = atan2(ry, rx);
      double beta = -s * dx / st.max_radius;
      double gamma = alpha - beta / 2;
      double sb = 2 * sin(beta / 2);
      dx = r * sin(gamma) * sb;
      dy += -r * cos(gamma) * sb;
    }
    target[0] = dx + st.pos0[j][0];
    target[1] = dy + st.pos0[j][1];
    target[2] = dz + st.pos0[j][2];
  }
  // set_jvalues_with_lik: torso + body chain FK, then limb IK (model.cpp:354-359, lik.cpp:89-99)
  double q6[6] = {o0[0], o0[1], o0[2], o1[0], o1[1], o1[2]};
  A34 A0 = mul(mul(node_joint_parent(T, 0), free_joint(q6)), node_pj(T, 0));
  const bool wq = w.want_q(k);
  if (L == 0) {
    if (wq) for (int i = 0; i < 6; i++) w.q(k)[i] = q6[i];
    A34 J0 = node_joint_parent(T, 0);  // torso joint frame J = I * J_A_parent
    node_features(T, 0, A0, &J0, w, k);
  }
  A34 A = A0;
  for (int kk = 1; kk < T->limb_chain_len[L]; kk++) {
    int v = T->limb_chain[L][kk];
    A = mul(A, node_pj(T, v));
    if (T->node[v].owner_limb == L) node_features(T, v, A, nullptr, w, k);
  }
  int c = T->limb_child[L];
  A34 J = mul(A, node_joint_parent(T, c));  // poslimb (lik.cpp:341-347)
  A34 Jinv = invert(J);
  double pl[3], ja[3];
  mulp(Jinv, target, pl);
  bool unreach = false, fail = false;
  limb_ik(T->lik_kind, T->ls, T->limb_ysign[L], pl, ja, ignore_reach, unreach, fail);
  if (w.want_centre(k)) w.unreach(k, L) = (unreach || fail) ? 1 : 0;
  // limb FK with the new joint values (compute_dynrecs' recompute_modelnodes)
  int v = c;
  for (int kk = 0; kk < 3; kk++) {
    const hs_node& nd = T->node[v];
    A34 Jv = (kk == 0) ? J : mul(A, node_joint_parent(T, v));
    A = mul(mul(Jv, hinge_joint(ja[kk])), node_pj(T, v));
    if (wq) w.q(k)[6 + nd.hinge] = ja[kk];
    node_features(T, v, A, &Jv, w, k);
    if (kk < 2) v = nd.kids[0];
  }
}

// ---------------------------------------------------------------------------
// D: finite differences at the centre sample, lane = part (dynrec.cpp:175-224)
// ---------------------------------------------------------------------------
template <class W, class SV>
__device__ void dynamics(const hs_topo* T, const SetupL& st, SV& sv, const W& w, int lane) {
  const int n = T->n;
  if (lane < n) {
    const int i = lane;
    const double inv = 1. / (2 * st.dt);
    const double m = T->mass[i];
    const double *Pp = w.pos(2, i), *P0 = w.pos(0, i), *Pm = w.pos(-2, i);
    const double *Up = w.ust(2, i), *U0 = w.ust(0, i), *Um = w.ust(-2, i);
    double vp[3], vm[3], mr[3], wp[3], wm[3], amp[3], amm[3], amr[3];
    for (int j = 0; j < 3; j++) {
      vp[j] = Pp[j] - P0[j];
      vp[j] *= inv;
      vm[j] = P0[j] - Pm[j];
      vm[j] *= inv;
      double mp = vp[j] * m, mm = vm[j] * m;
      mr[j] = mp - mm;
      mr[j] *= inv;
      wp[j] = Up[j] - U0[j];
      wp[j] *= inv;
      wm[j] = U0[j] - Um[j];
      wm[j] *= inv;
    }
    // ang_mom = R (I (R^T w)), I = identity (compute_ang_mom, dynrec.cpp:205-216)
    const double* Rp = w.rot(1, i);
    const double* Rm = w.rot(-1, i);
    double up[3], um[3];
    for (int r = 0; r < 3; r++) {
      double s = 0.0, t = 0.0;
      for (int k = 0; k < 3; k++) { s = s + Rp[r * 3 + k] * wp[k]; t = t + Rm[r * 3 + k] * wm[k]; }
      up[r] = s;
      um[r] = t;
    }
    for (int r = 0; r < 3; r++) {
      double s = 0.0, t = 0.0;
      for (int k = 0; k < 3; k++) { s = s + Rp[k * 3 + r] * up[k]; t = t + Rm[k * 3 + r] * um[k]; }
      amp[r] = s;
      amm[r] = t;
    }
    for (int j = 0; j < 3; j++) {
      amr[j] = amp[j] - amm[j];
      amr[j] *= inv;
    }
    for (int j = 0; j < 3; j++) {
      sv.f[3 * i + j] = mr[j];
      sv.f[3 * (n + i) + j] = amr[j];
    }
    sv.f[3 * i + 2] += m * 1.0;  // gravity, g = 1 (dynrec.cpp:291-295)
  }
  wave_sync();
}

// ---------------------------------------------------------------------------
// S1: tree back-substitution B0 x = f, level by level (deepest first)
// ---------------------------------------------------------------------------
template <class W, class SV>
__device__ void particular(const hs_topo* T, SV& sv, const W& w, int lane) {
  const int n = T->n;
  for (int level = T->max_depth; level >= 0; level--) {
    if (lane < n && T->node[lane].depth == level) {
      const int i = lane;
      const hs_node& nd = T->node[i];
      const double* Pi = w.pos(0, i);
      double F[3], Tq[3];
      for (int j = 0; j < 3; j++) { F[j] = sv.f[3 * i + j]; Tq[j] = sv.f[3 * (n + i) + j]; }
      for (int kk = 0; kk < nd.nkids; kk++) {
        int c = nd.kids[kk];
        const double* Jc = w.jpos(0, c);
        for (int j = 0; j < 3; j++) F[j] += sv.x[3 * c + j];
        double r[3];
        for (int j = 0; j < 3; j++) r[j] = Pi[j] - Jc[j];
        const double* Fc = &sv.x[3 * c];
        Tq[0] -= r[1] * Fc[2] - r[2] * Fc[1];
        Tq[1] -= r[2] * Fc[0] - r[0] * Fc[2];
        Tq[2] -= r[0] * Fc[1] - r[1] * Fc[0];
        for (int j = 0; j < 3; j++) Tq[j] += sv.x[3 * (n + c) + j];
      }
      for (int j = 0; j < 3; j++) sv.x[3 * i + j] = F[j];
      if (nd.parent >= 0) {
        const double* Ji = w.jpos(0, i);
        double r[3];
        for (int j = 0; j < 3; j++) r[j] = Ji[j] - Pi[j];
        Tq[0] -= r[1] * F[2] - r[2] * F[1];
        Tq[1] -= r[2] * F[0] - r[0] * F[2];
        Tq[2] -= r[0] * F[1] - r[1] * F[0];
      }
      for (int j = 0; j < 3; j++) sv.x[3 * (n + i) + j] = Tq[j];
    }
    wave_sync();
  }
}

// Tree-basis null-space entry for a torque row: (arm x e_jj)[row], arm = ref - fpos
__device__ inline double cross_e(const double* d, int jj, int row) {
  // d x e0 = (0, d2, -d1); d x e1 = (-d2, 0, d0); d x e2 = (d1, -d0, 0)
  if (jj == 0) return row == 0 ? 0.0 : (row == 1 ? d[2] : -d[1]);
  if (jj == 1) return row == 0 ? -d[2] : (row == 1 ? 0.0 : d[0]);
  return row == 0 ? d[1] : (row == 1 ? -d[0] : 0.0);
}

// ===========================================================================
// General path (rare: the fast solve's guard tripped): Gram matrices of the
// tree-built null basis and the Eigen 3.3 FullPivLU / ColPivHouseholderQR rank
// loop of ftsolver.cpp:185-303 (oracle/hs_oracle.cpp tree mode, same
// operation order). G is the LDS or the global workspace (GenMats).
// ===========================================================================

// S2: Gram matrices of the masked, penalty-weighted null basis (ftsolver.cpp:185-207)
template <class W, class SV, class G>
__device__ void build_grams(const hs_topo* T, const SV& sv, G& g, const W& w, int k, int lane) {
  constexpr int LD = G::LD;
  const int n = T->n;
  const int nc = k / 3;
  const double* P0 = w.pos(0, 0);
  // zeroth order: rows {0,1,2} = -I, rows {3n..3n+2} = (pos_0 - fpos) x e_jj, weight 1
  for (int e = lane; e < k * k; e += HALF) {
    int ci = e % k, cj = e / k;
    const double* fa = w.fpos(0, sv.cfoot[ci / 3]);
    const double* fb = w.fpos(0, sv.cfoot[cj / 3]);
    int ja = ci % 3, jb = cj % 3;
    double da[3], db[3];
    for (int r = 0; r < 3; r++) { da[r] = P0[r] - fa[r]; db[r] = P0[r] - fb[r]; }
    double s = 0.0;
    for (int r = 0; r < 3; r++) {
      double na = (r == ja) ? -1.0 : 0.0, nb = (r == jb) ? -1.0 : 0.0;
      s = s + na * nb;
    }
    for (int r = 0; r < 3; r++) s = s + cross_e(da, ja, r) * cross_e(db, jb, r);
    g.ntn0[ci + cj * LD] = s;
  }
  if (lane < k) {
    int ci = lane, ja = ci % 3;
    const double* fa = w.fpos(0, sv.cfoot[ci / 3]);
    double da[3];
    for (int r = 0; r < 3; r++) da[r] = P0[r] - fa[r];
    double s = 0.0;
    for (int r = 0; r < 3; r++) s = s + ((r == ja) ? -1.0 : 0.0) * (1.0 * sv.x[r]);
    for (int r = 0; r < 3; r++) s = s + cross_e(da, ja, r) * (1.0 * sv.x[3 * n + r]);
    g.ntx0[ci] = s;
  }
  // first order: torque rows of the non-root ancestors of each contact foot,
  // weighted by the joint-axis components (set_action_penalties, ftsolver.cpp:239-246)
  for (int e = lane; e < nc * 9 + k; e += HALF) {
    bool is_vec = e >= nc * 9;
    int cc = is_vec ? (e - nc * 9) / 3 : e / 9;
    int a_col = is_vec ? (e - nc * 9) % 3 : (e % 9) % 3;
    int b_col = is_vec ? 0 : (e % 9) / 3;
    int foot = T->footis[sv.cfoot[cc]];
    const double* fp = w.fpos(0, sv.cfoot[cc]);
    // ancestors of foot below the root, in ascending part order (top of the chain first)
    int chain[HS_NMAX], len = 0;
    for (int a = foot; a >= 0 && T->node[a].parent >= 0; a = T->node[a].parent) chain[len++] = a;
    double s = 0.0;
    for (int t = len - 1; t >= 0; t--) {
      int a = chain[t];
      const double* Ja = w.jpos(0, a);
      const double* Za = w.jz(0, a);
      double d[3];
      for (int r = 0; r < 3; r++) d[r] = Ja[r] - fp[r];
      for (int r = 0; r < 3; r++) {
        double wz = Za[r];
        double na = wz * cross_e(d, a_col, r);
        double nb = is_vec ? wz * sv.x[3 * n + 3 * a + r] : wz * cross_e(d, b_col, r);
        s = s + na * nb;
      }
    }
    if (is_vec) g.ntx1[3 * cc + a_col] = s;
    else g.n1[cc][b_col * 3 + a_col] = s;
  }
  gsync<G>();
}

// first-order Gram entry (block diagonal)
template <class G>
__device__ inline double ntn1_at(const G& g, int i, int j) {
  return (i / 3 == j / 3) ? g.n1[i / 3][(j % 3) * 3 + (i % 3)] : 0.0;
}

// half-wave argmax with first-index tie break
__device__ inline void wave_argmax(double& v, int& idx) {
  for (int off = HALF / 2; off >= 1; off >>= 1) {
    double ov = __shfl_xor(v, off);
    int oi = __shfl_xor(idx, off);
    if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
  }
}

struct LUInfo {
  int nz;          // nonzero pivots
  double maxpivot;
};

// Eigen FullPivLU::computeInPlace of ntn0 into g.lu (k x k)
template <class G>
__device__ LUInfo fullpiv_lu(G& g, int k, int lane) {
  constexpr int LD = G::LD;
  for (int e = lane; e < k * k; e += HALF) {
    int i = e % k, j = e / k;
    g.lu[i + j * LD] = g.ntn0[i + j * LD];
  }
  gsync<G>();
  LUInfo info{k, 0.0};
  for (int p = 0; p < k; p++) {
    const int m = k - p;
    double best = -1.0;
    int bidx = 1 << 30;
    for (int e = lane; e < m * m; e += HALF) {
      double a = fabs(g.lu[(p + e % m) + (p + e / m) * LD]);
      if (a > best || (a == best && e < bidx)) { best = a; bidx = e; }
    }
    wave_argmax(best, bidx);
    if (best == 0) {
      info.nz = p;
      for (int i = p + lane; i < k; i += HALF) { g.rowsT[i] = i; g.colsT[i] = i; }
      break;
    }
    if (best > info.maxpivot) info.maxpivot = best;
    const int bi = p + bidx % m, bj = p + bidx / m;
    if (lane == 0) { g.rowsT[p] = bi; g.colsT[p] = bj; }
    if (bi != p && lane < k) {
      double t = g.lu[p + lane * LD];
      g.lu[p + lane * LD] = g.lu[bi + lane * LD];
      g.lu[bi + lane * LD] = t;
    }
    gsync<G>();
    if (bj != p && lane < k) {
      double t = g.lu[lane + p * LD];
      g.lu[lane + p * LD] = g.lu[lane + bj * LD];
      g.lu[lane + bj * LD] = t;
    }
    gsync<G>();
    if (p < k - 1) {
      double piv = g.lu[p + p * LD];
      if (lane > p && lane < k) g.lu[lane + p * LD] /= piv;
      gsync<G>();
      const int mm = k - p - 1;
      for (int e = lane; e < mm * mm; e += HALF) {
        int i = p + 1 + e % mm, j = p + 1 + e / mm;
        g.lu[i + j * LD] -= g.lu[i + p * LD] * g.lu[p + j * LD];
      }
      gsync<G>();
    }
  }
  if (lane == 0) {
    for (int i = 0; i < k; i++) g.q[i] = i;
    for (int p = 0; p < k; p++) { int t = g.q[p]; g.q[p] = g.q[g.colsT[p]]; g.q[g.colsT[p]] = t; }
  }
  gsync<G>();
  return info;
}

template <class G>
__device__ inline int lu_rank(const G& g, const LUInfo& info, double thr) {
  constexpr int LD = G::LD;
  double pt = fabs(info.maxpivot) * thr;
  int r = 0;
  for (int i = 0; i < info.nz; i++) r += fabs(g.lu[i + i * LD]) > pt;
  return r;
}

// column-oriented upper-triangular solve of vec[0..r) against U (ld LD), all lanes
template <class G>
__device__ void upper_solve_shared(const double* U, double* vec, int r, int lane) {
  constexpr int LD = G::LD;
  for (int i = r - 1; i >= 0; i--) {
    double ci = vec[i];
    if (ci != 0) {
      double xi = ci / U[i + i * LD];
      if (lane < i) vec[lane] -= xi * U[lane + i * LD];
      if (lane == i) vec[i] = xi;
    }
    gsync<G>();
  }
}

// FullPivLU::solve(-ntx0) -> g.y0
template <class G>
__device__ void lu_solve(G& g, const LUInfo& info, int k, int r, int lane) {
  constexpr int LD = G::LD;
  if (lane == 0) {
    for (int i = 0; i < k; i++) g.c[i] = -g.ntx0[i];
    for (int p = 0; p < k; p++) { double t = g.c[p]; g.c[p] = g.c[g.rowsT[p]]; g.c[g.rowsT[p]] = t; }
  }
  if (lane < k) g.y0[lane] = 0.0;
  gsync<G>();
  if (r == 0) return;
  for (int j = 0; j < k; j++) {  // unit lower
    double cj = g.c[j];
    if (lane > j && lane < k) g.c[lane] -= cj * g.lu[lane + j * LD];
    gsync<G>();
  }
  upper_solve_shared<G>(g.lu, g.c, r, lane);
  if (lane < r) g.y0[g.q[lane]] = g.c[lane];
  gsync<G>();
}

// FullPivLU::kernel() -> g.Ny (k x dimker); uses g.qr as scratch; g.piv/rycol set
template <class G>
__device__ void lu_kernel_image(G& g, const LUInfo& info, int k, int r, double thr, int lane) {
  constexpr int LD = G::LD;
  if (lane == 0) {
    double pt = info.maxpivot * thr;
    int p = 0;
    for (int i = 0; i < info.nz; i++)
      if (fabs(g.lu[i + i * LD]) > pt) g.piv[p++] = i;
    for (int i = 0; i < r; i++) g.rycol[i] = g.q[g.piv[i]];  // image columns
  }
  gsync<G>();
  const int dimker = k - r;
  if (dimker == 0) return;
  double* mm = g.qr;  // r x k trapezoid
  for (int e = lane; e < r * k; e += HALF) {
    int i = e % r, j = e / r;
    mm[i + j * LD] = (j >= i) ? g.lu[g.piv[i] + j * LD] : 0.0;
  }
  gsync<G>();
  if (lane < r) {  // bring non-negligible pivots to the front (rows own a column swap each)
    for (int i = 0; i < r; i++) {
      int pc = g.piv[i];
      if (pc != i) { double t = mm[lane + i * LD]; mm[lane + i * LD] = mm[lane + pc * LD]; mm[lane + pc * LD] = t; }
    }
  }
  gsync<G>();
  if (lane < dimker) {  // solve U11 X = U12, one right-hand column per lane
    double* col = &mm[(r + lane) * LD];
    for (int i = r - 1; i >= 0; i--) {
      if (col[i] != 0) {
        col[i] /= mm[i + i * LD];
        for (int rr = 0; rr < i; rr++) col[rr] -= col[i] * mm[rr + i * LD];
      }
    }
  }
  gsync<G>();
  if (lane < r) {
    for (int i = r - 1; i >= 0; i--) {
      int pc = g.piv[i];
      if (pc != i) { double t = mm[lane + i * LD]; mm[lane + i * LD] = mm[lane + pc * LD]; mm[lane + pc * LD] = t; }
    }
  }
  gsync<G>();
  for (int e = lane; e < k * dimker; e += HALF) {
    int i = e % k, kk = e / k;
    int row = g.q[i];
    double v;
    if (i < r) v = -mm[i + (r + kk) * LD];
    else v = (i == r + kk) ? 1.0 : 0.0;
    g.Ny[row + kk * LD] = v;
  }
  gsync<G>();
}

// entry (i, j) of m = [ntn1 Ny, ntn0 Ry] (ftsolver.cpp:222-226), evaluated where needed
template <class G>
__device__ inline double m_at(const G& g, int k, int dimker, int i, int j) {
  constexpr int LD = G::LD;
  double s = 0.0;
  if (j < dimker) {
    int b0 = (i / 3) * 3;
    for (int kk = b0; kk < b0 + 3; kk++) s = s + ntn1_at(g, i, kk) * g.Ny[kk + j * LD];
  } else {
    int col = g.rycol[j - dimker];
    for (int kk = 0; kk < k; kk++) s = s + g.ntn0[i + kk * LD] * g.ntn0[kk + col * LD];
  }
  return s;
}

// Eigen 3.3 ColPivHouseholderQR on g.qr (k x k, holding m); returns nonzero pivots
template <class G>
__device__ int colpiv_qr(G& g, int k, int lane) {
  constexpr int LD = G::LD;
  if (lane < k) {
    double s = 0;
    for (int i = 0; i < k; i++) s += g.qr[i + lane * LD] * g.qr[i + lane * LD];
    g.nd[lane] = sqrt(s);
    g.nu[lane] = g.nd[lane];
  }
  gsync<G>();
  double mx = 0;
  for (int j = 0; j < k; j++) mx = fmax(mx, g.nu[j]);
  const double th = mx * DBL_EPSILON;
  const double threshold_helper = th * th / (double)k;
  const double ndt = sqrt(DBL_EPSILON);
  int np = k;
  for (int p = 0; p < k; p++) {
    int bi = p;
    double bv = g.nu[p];
    for (int j = p + 1; j < k; j++)
      if (g.nu[j] > bv) { bv = g.nu[j]; bi = j; }
    if (np == k && bv * bv < threshold_helper * (double)(k - p)) np = p;
    gsync<G>();
    if (lane == 0) g.cperm[p] = bi;
    if (bi != p) {
      if (lane < k) {
        double t = g.qr[lane + p * LD];
        g.qr[lane + p * LD] = g.qr[lane + bi * LD];
        g.qr[lane + bi * LD] = t;
      }
      if (lane == 0) {
        double t = g.nu[p]; g.nu[p] = g.nu[bi]; g.nu[bi] = t;
        t = g.nd[p]; g.nd[p] = g.nd[bi]; g.nd[bi] = t;
      }
    }
    gsync<G>();
    // makeHouseholderInPlace on column p, rows p..k-1
    const int len = k - p;
    double c0 = g.qr[p + p * LD];
    double tail = 0;
    for (int i = 1; i < len; i++) tail += g.qr[p + i + p * LD] * g.qr[p + i + p * LD];
    double tau, beta;
    if (len == 1 || tail <= DBL_MIN) {
      tau = 0;
      beta = c0;
      if (lane >= 1 && lane < len) g.qr[p + lane + p * LD] = 0;
    } else {
      beta = sqrt(c0 * c0 + tail);
      if (c0 >= 0) beta = -beta;
      double den = c0 - beta;
      if (lane >= 1 && lane < len) g.qr[p + lane + p * LD] /= den;
      tau = (beta - c0) / beta;
    }
    gsync<G>();
    if (lane == 0) { g.qr[p + p * LD] = beta; g.hc[p] = tau; }
    // apply to columns p+1..k-1, then downdate their norms (one column per lane)
    const int j = lane;
    if (j > p && j < k) {
      if (len == 1) {
        g.qr[p + j * LD] *= (1 - tau);
      } else if (tau != 0) {
        double tmp = 0;
        for (int i = 1; i < len; i++) tmp += g.qr[p + i + p * LD] * g.qr[p + i + j * LD];
        tmp += g.qr[p + j * LD];
        g.qr[p + j * LD] -= tau * tmp;
        for (int i = 1; i < len; i++) g.qr[p + i + j * LD] -= tau * g.qr[p + i + p * LD] * tmp;
      }
      if (g.nu[j] != 0) {
        double temp = fabs(g.qr[p + j * LD]) / g.nu[j];
        temp = (1 + temp) * (1 - temp);
        temp = temp < 0 ? 0 : temp;
        double ratio = g.nu[j] / g.nd[j];
        double temp2 = temp * (ratio * ratio);
        if (temp2 <= ndt) {
          double s = 0;
          for (int i = p + 1; i < k; i++) s += g.qr[i + j * LD] * g.qr[i + j * LD];
          g.nd[j] = sqrt(s);
          g.nu[j] = g.nd[j];
        } else {
          g.nu[j] *= sqrt(temp);
        }
      }
    }
    gsync<G>();
  }
  return np;
}

// QR solve m z = b (least squares, basic solution) -> g.z
template <class G>
__device__ void qr_solve(G& g, int k, int np, int lane) {
  constexpr int LD = G::LD;
  if (lane < k) { g.c[lane] = g.b[lane]; g.z[lane] = 0.0; }
  gsync<G>();
  if (np == 0) return;
  for (int p = 0; p < np; p++) {
    const int len = k - p;
    const double tau = g.hc[p];
    if (len == 1) {
      if (lane == p) g.c[p] *= (1 - tau);
    } else if (tau != 0) {
      double tmp = 0;
      for (int i = 1; i < len; i++) tmp += g.qr[p + i + p * LD] * g.c[p + i];
      tmp += g.c[p];
      gsync<G>();
      if (lane == 0) g.c[p] -= tau * tmp;
      if (lane >= 1 && lane < len) g.c[p + lane] -= tau * g.qr[p + lane + p * LD] * tmp;
    }
    gsync<G>();
  }
  upper_solve_shared<G>(g.qr, g.c, np, lane);
  if (lane == 0) {
    int perm[HS_KMAX];
    for (int i = 0; i < k; i++) perm[i] = i;
    for (int p = 0; p < k; p++) { int t = perm[p]; perm[p] = perm[g.cperm[p]]; perm[g.cperm[p]] = t; }
    for (int i = 0; i < np; i++) g.z[perm[i]] = g.c[i];
  }
  gsync<G>();
}

// S3 general: adaptive-rank two-stage least squares (ftsolver.cpp:277-303) -> sv.y.
// The reference re-runs FullPivLU on the same zeroth-order Gram every pass; it
// is factorized once here (identical factors), only the rank threshold moves.
template <class SV, class G>
__device__ uint32_t contact_solve(SV& sv, G& g, int k, int lane) {
  constexpr int LD = G::LD;
  uint32_t flags = 0;
  if (k == 0) return HS_FLAG_NO_CONTACT;
  const LUInfo info = fullpiv_lu(g, k, lane);
  STAMP(10);
  int rank0 = k;
  int iters = 0;
  double rel_error = 0;
  do {
    iters++;
    double thr = DBL_EPSILON * (double)k;
    int r = lu_rank(g, info, thr);
    for (int guard = 0; guard < 2100 && r > rank0; guard++) {  // setThreshold doubling
      thr = 2 * thr;
      r = lu_rank(g, info, thr);
    }
    lu_solve(g, info, k, r, lane);
    lu_kernel_image(g, info, k, r, thr, lane);
    STAMP(11);
    if (r == k) flags |= HS_FLAG_FULL_RANK;
    rank0 = r;
    const int dimker = k - r;
    // b = -(ntx1 + ntn1 y0)
    if (lane < k) {
      int i = lane, b0 = (i / 3) * 3;
      double t = 0.0;
      for (int kk = b0; kk < b0 + 3; kk++) t = t + ntn1_at(g, i, kk) * g.y0[kk];
      g.b[i] = -(g.ntx1[i] + t);
    }
    for (int e = lane; e < k * k; e += HALF) {  // m, built straight into the QR buffer
      int i = e % k, j = e / k;
      g.qr[i + j * LD] = m_at(g, k, dimker, i, j);
    }
    gsync<G>();
    STAMP(12);
    int np = colpiv_qr(g, k, lane);
    STAMP(13);
    qr_solve(g, k, np, lane);
    STAMP(14);
    // rel_error = |m z - b| / |b|
    if (lane < k) {
      double s = 0.0;
      for (int j = 0; j < k; j++) s = s + m_at(g, k, dimker, lane, j) * g.z[j];
      g.c[lane] = s - g.b[lane];
    }
    gsync<G>();
    double rn = 0, bn = 0;
    for (int i = 0; i < k; i++) { rn += g.c[i] * g.c[i]; bn += g.b[i] * g.b[i]; }
    rel_error = sqrt(rn) / sqrt(bn);
    rank0--;
    if (lane < k) {
      double s = 0.0;
      for (int j = 0; j < dimker; j++) s = s + g.Ny[lane + j * LD] * g.z[j];
      sv.y[lane] = g.y0[lane] + s;
    }
    gsync<G>();
    if (rel_error > 1e-6 && rank0 <= 0) { flags |= HS_FLAG_LOOP_EXHAUST; break; }
  } while (rel_error > 1e-6 && iters <= HS_KMAX + 1);
  if (iters > 1) flags |= HS_FLAG_RANK_RETRY;
  return flags;
}

template <class W, class SV, class G>
__device__ __attribute__((always_inline)) inline uint32_t general_solve(const hs_topo* T, SV& sv, G& g, const W& w,
                                                                        int k, int lane) {
  build_grams(T, sv, g, w, k, lane);
  STAMP(9);
  return contact_solve(sv, g, k, lane);
}

// ---------------------------------------------------------------------------
// S3 fast path: closed form of the same lexicographic least squares
// (oracle/hs_oracle.cpp fast_contact_solve, identical operation order).
// One lane per contact builds A_c, D_c, g_c; >= 3 contacts: 6x6 Schur
// complement of the zeroth-order constraints; 1 contact: unique LS; 2 contacts:
// rank-5 kernel along the feet line. Returns false (wave-uniform) when a
// Cholesky pivot falls under the guard -> general path.
// ---------------------------------------------------------------------------
constexpr double kFastPivotGuard = 1e-10;

template <int N>
__device__ inline bool chol_n(double* a, double guard) {  // row-major, in place
  double mx = 0;
#pragma unroll
  for (int i = 0; i < N; i++) mx = fmax(mx, a[i * N + i]);
#pragma unroll
  for (int j = 0; j < N; j++) {
    double s = a[j * N + j];
#pragma unroll
    for (int k = 0; k < j; k++) s -= a[j * N + k] * a[j * N + k];
    if (!(s > guard * mx)) return false;
    double l = sqrt(s);
    a[j * N + j] = l;
#pragma unroll
    for (int i = j + 1; i < N; i++) {
      double t = a[i * N + j];
#pragma unroll
      for (int k = 0; k < j; k++) t -= a[i * N + k] * a[j * N + k];
      a[i * N + j] = t / l;
    }
  }
  return true;
}

template <int N>
__device__ inline void chol_solve_n(const double* L, double* b) {
#pragma unroll
  for (int i = 0; i < N; i++) {
    double s = b[i];
#pragma unroll
    for (int k = 0; k < i; k++) s -= L[i * N + k] * b[k];
    b[i] = s / L[i * N + i];
  }
#pragma unroll
  for (int i = N - 1; i >= 0; i--) {
    double s = b[i];
#pragma unroll
    for (int k = i + 1; k < N; k++) s -= L[k * N + i] * b[k];
    b[i] = s / L[i * N + i];
  }
}

__device__ inline void cross_rows(const double* d, double v[3][3]) {
  v[0][0] = 0;     v[0][1] = -d[2]; v[0][2] = d[1];
  v[1][0] = d[2];  v[1][1] = 0;     v[1][2] = -d[0];
  v[2][0] = -d[1]; v[2][1] = d[0];  v[2][2] = 0;
}

// In-place Cholesky of a k x k SPD matrix (row-major, lower triangle used) by
// the half-wave, right-looking: element (i, j) gets its products subtracted in
// increasing order, exactly like the oracle's left-looking chol(). False (wave-
// uniform) when a pivot falls to guard * (max original diagonal) or below.
__device__ bool chol_half(double* K, int k, double guard, int lane) {
  double mx = 0;
  for (int i = 0; i < k; i++) mx = fmax(mx, K[i * k + i]);
  for (int j = 0; j < k; j++) {
    const double s = K[j * k + j];
    if (!(s > guard * mx)) return false;
    const double l = sqrt(s);
    if (lane == 0) K[j * k + j] = l;
    for (int i = j + 1 + lane; i < k; i += HALF) K[i * k + j] = K[i * k + j] / l;
    wave_sync();
    const int m = k - 1 - j;
    for (int e = lane; e < m * m; e += HALF) {
      const int i = j + 1 + e / m, c2 = j + 1 + e % m;
      if (c2 <= i) K[i * k + c2] -= K[i * k + j] * K[c2 * k + j];
    }
    wave_sync();
  }
  return true;
}

// nc >= 3 with a singular D_c (straight, IK-clamped leg) or Schur complement:
// augmented system K = D + rho A^T A, w = -K^-1 (g~ + A^T lam),
// (A K^-1 A^T) lam = a - A K^-1 g~ (oracle aug_solve, same operation order; the
// half-wave right-looking Cholesky subtracts in the oracle's left-looking order).
// False when the minimizer is not unique (a pivot under the guard).
template <class SV>
__device__ bool aug_solve(FastL& fl, SV& sv, const double* a, int nc, int lane) {
  AugL& ag = fl.ag;
  const int k = 3 * nc;
  auto Aat = [&](int r, int i) { return fl.A[i / 3][r * 3 + i % 3]; };  // A (6 x k)
  double md = 0, ma = 0;
  for (int c = 0; c < nc; c++)
    for (int i = 0; i < 3; i++) {
      md = fmax(md, fl.D[c][4 * i]);
      double s = 0;
      for (int r = 0; r < 6; r++) s += Aat(r, 3 * c + i) * Aat(r, 3 * c + i);
      ma = fmax(ma, s);
    }
  const double rho = (md > 0 && ma > 0) ? md / ma : 1.0;
  for (int e = lane; e < k * k; e += HALF) {
    const int i = e / k, j = e % k;
    double s = 0;
    for (int r = 0; r < 6; r++) s += Aat(r, i) * Aat(r, j);
    ag.K[i * k + j] = ((i / 3 == j / 3) ? fl.D[i / 3][3 * (i % 3) + j % 3] : 0.0) + rho * s;
  }
  for (int e = lane; e < k * 7; e += HALF) {
    const int i = e / 7, q = e % 7;
    double v;
    if (q < 6) {
      v = Aat(q, i);
    } else {
      double s = 0;
      for (int r = 0; r < 6; r++) s += Aat(r, i) * a[r];
      v = fl.g[i / 3][i % 3] + rho * s;
    }
    ag.X[i * 7 + q] = v;
  }
  wave_sync();
  if (!chol_half(ag.K, k, kFastPivotGuard, lane)) return false;
  if (lane < 7) {  // K X = [A^T | g~], one right-hand column per lane
    const int q = lane;
    for (int i = 0; i < k; i++) {
      double s = ag.X[i * 7 + q];
      for (int m = 0; m < i; m++) s -= ag.K[i * k + m] * ag.X[m * 7 + q];
      ag.X[i * 7 + q] = s / ag.K[i * k + i];
    }
    for (int i = k - 1; i >= 0; i--) {
      double s = ag.X[i * 7 + q];
      for (int m = i + 1; m < k; m++) s -= ag.K[m * k + i] * ag.X[m * 7 + q];
      ag.X[i * 7 + q] = s / ag.K[i * k + i];
    }
  }
  wave_sync();
  for (int e = lane; e < 42; e += HALF) {
    const int r = e / 7, q = e % 7;
    double s = 0;
    for (int i = 0; i < k; i++) s += Aat(r, i) * ag.X[i * 7 + q];
    if (q < 6) ag.St[6 * r + q] = s;
    else ag.lam[r] = a[r] - s;
  }
  wave_sync();
  if (lane == 0) {
    double St[36], lam[6];
    for (int i = 0; i < 36; i++) St[i] = ag.St[i];
    for (int i = 0; i < 6; i++) lam[i] = ag.lam[i];
    int ok = chol_n<6>(St, kFastPivotGuard);
    if (ok) {
      chol_solve_n<6>(St, lam);
      for (int i = 0; i < 6; i++) ag.lam[i] = lam[i];
    }
    ag.ok = ok;
  }
  wave_sync();
  if (!ag.ok) return false;
  for (int i = lane; i < k; i += HALF) {
    double s = ag.X[i * 7 + 6];
    for (int r = 0; r < 6; r++) s += ag.X[i * 7 + r] * ag.lam[r];
    sv.y[i] = -s;
  }
  wave_sync();
  return true;
}

template <class W, class SV>
__device__ bool fast_solve(const hs_topo* T, SV& sv, FastL& fl, const W& w, int nc, int lane) {
  const int n = T->n;
  if (nc == 0) return true;
  const double* P0 = w.pos(0, 0);
  if (lane < nc) {  // A_c, D_c, g_c for contact c = lane
    const int c = lane, fi = sv.cfoot[c];
    const double* fp = w.fpos(0, fi);
    double d0[3], v[3][3];
    for (int r = 0; r < 3; r++) d0[r] = P0[r] - fp[r];
    cross_rows(d0, v);
    double Ac[18];
    for (int r = 0; r < 3; r++)
      for (int j = 0; j < 3; j++) { Ac[r * 3 + j] = (r == j) ? -1.0 : 0.0; Ac[(3 + r) * 3 + j] = v[r][j]; }
    for (int i = 0; i < 18; i++) fl.A[c][i] = Ac[i];
    double D[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
    for (int p = T->footis[fi]; p >= 0 && T->node[p].parent >= 0; p = T->node[p].parent) {
      const double* Jp = w.jpos(0, p);
      const double* Jz = w.jz(0, p);
      double da[3], va[3][3];
      for (int r = 0; r < 3; r++) da[r] = Jp[r] - fp[r];
      cross_rows(da, va);
      for (int r = 0; r < 3; r++) {
        double w2 = Jz[r] * Jz[r];
        if (w2 == 0) continue;
        for (int i = 0; i < 3; i++) {
          for (int j = 0; j < 3; j++) D[3 * i + j] += w2 * va[r][i] * va[r][j];
          g[i] += w2 * va[r][i] * sv.x[3 * n + 3 * p + r];
        }
      }
    }
    for (int i = 0; i < 9; i++) fl.D[c][i] = D[i];
    for (int i = 0; i < 3; i++) fl.g[c][i] = g[i];
    int ok = 1;
    if (nc >= 3) {
      double L[9];
      for (int i = 0; i < 9; i++) L[i] = D[i];
      ok = chol_n<3>(L, kFastPivotGuard);
      if (ok) {
        double Dinv[9];
        for (int j = 0; j < 3; j++) {
          double e[3] = {0, 0, 0};
          e[j] = 1;
          chol_solve_n<3>(L, e);
          for (int i = 0; i < 3; i++) Dinv[3 * i + j] = e[i];
        }
        double E[18];
        for (int r = 0; r < 6; r++)
          for (int j = 0; j < 3; j++) {
            double s = 0;
            for (int i = 0; i < 3; i++) s += Ac[r * 3 + i] * Dinv[3 * i + j];
            E[r * 3 + j] = s;
          }
        for (int r = 0; r < 6; r++) {
          for (int q = 0; q < 6; q++) {
            double s = 0;
            for (int j = 0; j < 3; j++) s += E[r * 3 + j] * Ac[q * 3 + j];
            fl.sc.S[c][6 * r + q] = s;
          }
          double s = 0;
          for (int j = 0; j < 3; j++) s += E[r * 3 + j] * g[j];
          fl.sc.h[c][r] = s;
        }
        for (int i = 0; i < 9; i++) fl.sc.Dinv[c][i] = Dinv[i];
      }
    }
    fl.ok[c] = ok;
  }
  wave_sync();
  const double a[6] = {sv.x[0], sv.x[1], sv.x[2], sv.x[3 * n], sv.x[3 * n + 1], sv.x[3 * n + 2]};
  for (int c = 0; c < nc; c++)
    if (!fl.ok[c]) return aug_solve(fl, sv, a, nc, lane);  // only nc >= 3 factors D_c
  int ok = 1;
  if (nc == 1) {  // unique least-squares solution (A^T A) w = -A^T a
    if (lane == 0) {
      double M[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
      const double* A = fl.A[0];
      for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++)
          for (int r = 0; r < 6; r++) M[3 * i + j] += A[r * 3 + i] * A[r * 3 + j];
        for (int r = 0; r < 6; r++) b[i] -= A[r * 3 + i] * a[r];
      }
      ok = chol_n<3>(M, kFastPivotGuard);
      if (ok) {
        chol_solve_n<3>(M, b);
        for (int i = 0; i < 3; i++) sv.y[i] = b[i];
      }
      fl.ok[0] = ok;
    }
  } else if (nc == 2) {  // rank 5: kernel n = (u,-u)/sqrt2 along the line between the feet
    if (lane == 0) {
      const double* f0 = w.fpos(0, sv.cfoot[0]);
      const double* f1 = w.fpos(0, sv.cfoot[1]);
      double u[3], un = 0;
      for (int r = 0; r < 3; r++) { u[r] = f0[r] - f1[r]; un += u[r] * u[r]; }
      un = sqrt(un);
      ok = un > 1e-12;
      double nv[6], M[36], b[6];
      if (ok) {
        for (int r = 0; r < 3; r++) { nv[r] = u[r] / un / sqrt(2.0); nv[3 + r] = -nv[r]; }
        for (int i = 0; i < 6; i++) {
          const double* Ai = fl.A[i / 3];
          for (int j = 0; j < 6; j++) {
            const double* Aj = fl.A[j / 3];
            double s = 0;
            for (int r = 0; r < 6; r++) s += Ai[r * 3 + i % 3] * Aj[r * 3 + j % 3];
            M[6 * i + j] = s + nv[i] * nv[j];
          }
          double s = 0;
          for (int r = 0; r < 6; r++) s += Ai[r * 3 + i % 3] * a[r];
          b[i] = -s;
        }
        ok = chol_n<6>(M, kFastPivotGuard);
      }
      if (ok) {
        chol_solve_n<6>(M, b);
        double nDn = 0, nr = 0;
        for (int c = 0; c < 2; c++)
          for (int i = 0; i < 3; i++) {
            double Dw = 0, Dn = 0;
            for (int j = 0; j < 3; j++) { Dw += fl.D[c][3 * i + j] * b[3 * c + j]; Dn += fl.D[c][3 * i + j] * nv[3 * c + j]; }
            nr += nv[3 * c + i] * (Dw + fl.g[c][i]);
            nDn += nv[3 * c + i] * Dn;
          }
        ok = nDn > 0;
        if (ok) {
          double t = -nr / nDn;
          for (int i = 0; i < 6; i++) sv.y[i] = b[i] + t * nv[i];
        }
      }
      fl.ok[0] = ok;
    }
  } else {  // Schur complement of the 6 zeroth-order constraints
    if (lane == 0) {
      double Sm[36], h[6];
      for (int i = 0; i < 36; i++) Sm[i] = 0;
      for (int i = 0; i < 6; i++) h[i] = 0;
      for (int c = 0; c < nc; c++) {
        for (int i = 0; i < 36; i++) Sm[i] += fl.sc.S[c][i];
        for (int i = 0; i < 6; i++) h[i] += fl.sc.h[c][i];
      }
      double lam[6];
      for (int r = 0; r < 6; r++) lam[r] = a[r] - h[r];
      ok = chol_n<6>(Sm, kFastPivotGuard);
      if (ok) {
        chol_solve_n<6>(Sm, lam);
        for (int r = 0; r < 6; r++) fl.sc.lam[r] = lam[r];
      }
      fl.ok[0] = ok;
    }
    wave_sync();
    if (!fl.ok[0]) return aug_solve(fl, sv, a, nc, lane);
    if (lane < nc) {
      const int c = lane;
      const double* Ac = fl.A[c];
      double t[3];
      for (int i = 0; i < 3; i++) {
        double s = fl.g[c][i];
        for (int r = 0; r < 6; r++) s += Ac[r * 3 + i] * fl.sc.lam[r];
        t[i] = s;
      }
      for (int i = 0; i < 3; i++) {
        double s = 0;
        for (int j = 0; j < 3; j++) s += fl.sc.Dinv[c][3 * i + j] * t[j];
        sv.y[3 * c + i] = -s;
      }
    }
  }
  wave_sync();
  return fl.ok[0] != 0;
}

__device__ inline uint64_t best_key(double cot, int64_t id) {
  float c = (float)cot;
  uint32_t bits = __float_as_uint(c);
  uint32_t ord = (c != c) ? 0xFFFFFFFFu : ((bits & 0x80000000u) ? ~bits : (bits | 0x80000000u));
  return ((uint64_t)ord << 32) | (uint32_t)id;
}

// ---------------------------------------------------------------------------
// One control-loop step at centre sample i (row = b * H + h of the outputs)
// ---------------------------------------------------------------------------
template <class W, class SV>
__device__ void step(const hs_topo* T, const hs_run_args& a, const hs::launch_map& mp, const SetupL& st, SV& sv,
                     FastL& fl, GenLDS& gl, WorkL& wk, const W& w, GenWS* G, int b, bool live, int h,
                     double& work, int lane) {
  const int n = T->n, nmj = T->nmj, nf = T->nf, cfg = T->cfg, nl = T->n_limbs;
  STAMP(3);
  dynamics(T, st, sv, w, lane);
  STAMP(4);
  particular(T, sv, w, lane);
  STAMP(5);
  // contact list in foot order (ftsolver contact columns)
  const uint32_t cmask = half_ballot(lane < nf && w.contact(0, lane));
  const int nc = __popc(cmask);
  if (lane < nf && ((cmask >> lane) & 1)) sv.cfoot[__popc(cmask & ((1u << lane) - 1))] = lane;
  wave_sync();
  int k = 3 * nc;
  uint32_t flags = 0;
  STAMP(6);
  if (fast_solve(T, sv, fl, w, nc, lane)) {
    if (nc == 0) flags |= HS_FLAG_NO_CONTACT;
    if (nc == 1) flags |= HS_FLAG_FULL_RANK;
  } else if (k <= GenLDS::LD) {
    flags = general_solve(T, sv, gl, w, k, lane) | HS_FLAG_GENERAL;
  } else {
    flags = general_solve(T, sv, *G, w, k, lane) | HS_FLAG_GENERAL;
  }
  STAMP(7);

  // S4: x = x_part + N y for the hinge torque rows, motor torques (periodic.cpp:328-343),
  // and the step's positive work (compute_vel_traj + work_over_period, periodic.cpp:261-307)
  const size_t row = (size_t)b * a.horizon + h;
  double tq = 0.0;
  if (lane < nmj) {
    int h_id = T->hinge_ids[lane];
    int fi = T->node[h_id].limb_below;
    int cc = -1;
    for (int c = 0; c < nc; c++) if (sv.cfoot[c] == fi) cc = c;
    const double* Jp = w.jpos(0, h_id);
    const double* Jz = w.jz(0, h_id);
    double d[3];
    if (cc >= 0) {
      const double* fp = w.fpos(0, fi);
      for (int rr = 0; rr < 3; rr++) d[rr] = Jp[rr] - fp[rr];
    }
    for (int r = 0; r < 3; r++) {
      double s = 0.0;
      if (cc >= 0)
        for (int jj = 0; jj < 3; jj++) s = s + cross_e(d, jj, r) * sv.y[3 * cc + jj];
      double xr = sv.x[3 * n + 3 * h_id + r] + s;
      tq = tq + Jz[r] * xr;
    }
    double dd = w.q(1)[6 + lane] - w.q(-1)[6 + lane];
    if (dd > kPi) dd -= 2 * kPi;
    else if (dd < -kPi) dd += 2 * kPi;
    double jvel = dd / (2 * st.dt);
    double dw = tq * jvel;
    wk.wd[lane] = (dw > 0) ? dw : 0;
    if (mp.pd_tau && live) {  // linear_feedback_control (player.cpp:417-432), target = get_motor_adas
      const size_t o = row * mp.st_tau + lane;
      const double q0 = w.q(0)[6 + lane];
      double a1 = mp.pd_q[o] - q0;
      if (a1 > kPi) a1 -= 2 * kPi;  // arrayops::modulus(., 2 pi) (core.cpp:122-131)
      else if (a1 <= -kPi) a1 += 2 * kPi;
      a1 *= mp.pd_k1;
      double a2 = mp.pd_dq[o] - jvel;
      a2 *= mp.pd_k2;
      a1 += a2;
      mp.pd_tau[o] = tq + a1;
      if (mp.pd_q0) mp.pd_q0[o] = q0;
      if (mp.pd_dq0) mp.pd_dq0[o] = jvel;
    }
  }
  if (live && a.tau && lane < mp.st_tau) a.tau[row * mp.st_tau + lane] = tq;  // 0 past nmj
  if (half_ballot(lane < nmj && tq != tq) || half_ballot(lane < k && sv.y[lane] != sv.y[lane])) flags |= HS_FLAG_NAN;
  if (half_ballot(lane < nl && w.unreach(0, lane))) flags |= HS_FLAG_UNREACH;
  // contact forces z = -N_cont y (ftsolver.cpp:91, 276-284)
  if (live && a.cf && lane < mp.st_cf) {
    int fi = lane / 3, j = lane % 3;
    double zv = (lane < 3 * nf) ? -0.0 : 0.0;
    for (int c = 0; c < nc; c++) if (sv.cfoot[c] == fi) zv = -(0.0 + (-1.0) * sv.y[3 * c + j]);
    a.cf[row * mp.st_cf + lane] = zv;
  }
  if (live && a.x) {  // full joint force/torque vector x += N y
    for (int rI = lane; rI < 6 * n; rI += HALF) {
      int part = (rI < 3 * n) ? rI / 3 : (rI - 3 * n) / 3, comp = rI % 3;
      double s = 0.0;
      for (int c = 0; c < nc; c++) {
        int foot = T->footis[sv.cfoot[c]];
        bool anc = false;
        for (int aa = foot; aa >= 0; aa = T->node[aa].parent) anc |= (aa == part);
        if (!anc) continue;
        if (rI < 3 * n) {
          s = s + (-1.0) * sv.y[3 * c + comp];
        } else {
          const double* ref = (T->node[part].parent >= 0) ? w.jpos(0, part) : w.pos(0, part);
          const double* fp = w.fpos(0, sv.cfoot[c]);
          double d[3];
          for (int rr = 0; rr < 3; rr++) d[rr] = ref[rr] - fp[rr];
          for (int jj = 0; jj < 3; jj++) s = s + cross_e(d, jj, comp) * sv.y[3 * c + jj];
        }
      }
      a.x[row * mp.st_x + rI] = sv.x[rI] + s;
    }
    for (int rI = 6 * n + lane; rI < mp.st_x; rI += HALF) a.x[row * mp.st_x + rI] = 0.0;
  }
  if (live && a.q && lane < mp.st_q) a.q[row * mp.st_q + lane] = (lane < cfg) ? w.q(0)[lane] : 0.0;
  if (live && a.dq && lane < mp.st_q) {  // compute_vel_traj (periodic.cpp:261-282)
    double v = 0.0;
    if (lane < cfg) {
      double d = w.q(1)[lane] - w.q(-1)[lane];
      if (d > kPi) d -= 2 * kPi;
      else if (d < -kPi) d += 2 * kPi;
      v = d / (2 * st.dt);
    }
    a.dq[row * mp.st_q + lane] = v;
  }
  if (live && a.flags && lane == 0) a.flags[row] = flags;
  wave_sync();
  double work_dt = 0;  // summed in joint order like work_over_period
  for (int jj = 0; jj < nmj; jj++) work_dt += wk.wd[jj];
  work_dt *= st.dt;
  work += work_dt;
  STAMP(8);
}

// ---------------------------------------------------------------------------
// Contact forces given motor torques: forcetorquesolver::solve_forces
// (ftsolver.cpp:331-378; oracle solve_forces). Least squares over the tree
// rows, the torso rows (torso force/torque forced to zero) and the torque rows
// jz_h . x_h = z_h, unknowns = non-root joint wrenches + forces of ALL feet.
// The tree rows' coefficient block is unit triangular, so eliminating the
// joint wrenches exactly leaves (Woodbury)
//   y = argmin (C y - d)^T (I + G G^T)^-1 (C y - d)
// over m = 6 + nmj rows: G = (torso, torque) rows composed with the tree
// inverse -- T_i = -[[I, 0], [[p_i - p_0]x, I]] for the torso, (u_hi, jz_h) with
// u_hi = (jpos_h - pos_i) x jz_h on the subtree of hinge h -- C = [I; [fpos -
// p_0]x] and jz_h . [(jpos_h - fpos)x] (the tree basis seen by those rows),
// d = (torso part of x_part, z - jz . x_part). Rank-deficient normal matrix
// (a straight leg): HS_FLAG_GENERAL, Tikhonov 1e-12 of its largest diagonal.
// ---------------------------------------------------------------------------
__device__ inline bool in_subtree(const hs_topo* T, int i, int h) {
  for (int a = i; a >= 0; a = T->node[a].parent)
    if (a == h) return true;
  return false;
}

__device__ inline void cross3(const double* a, const double* b, double* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

template <class W, class SV>
__device__ uint32_t forces_solve(const hs_topo* T, const SV& sv, ForceL& fr, const W& w, const double* z, int lane) {
  const int n = T->n, nj = T->nmj, nf = T->nf, m = 6 + nj, nq = 3 * nf, ld = nq + 1;
  const double* P0 = w.pos(0, 0);
  for (int e = lane; e < m * m; e += HALF) {  // I + G G^T, lower triangle
    const int r = e / m, c = e % m;
    if (c > r) continue;
    double s = 0.0;
    if (r < 6) {
      for (int i = 1; i < n; i++) {
        const double* Pi = w.pos(0, i);
        double ri[3], Sr[3] = {0, 0, 0}, Sc[3] = {0, 0, 0};
        for (int t = 0; t < 3; t++) ri[t] = Pi[t] - P0[t];
        // T_i row a = -(e_a, 0) for a < 3, -([r_i]x row a-3, e_{a-3}) for a >= 3
        if (r >= 3) for (int t = 0; t < 3; t++) Sr[t] = cross_e(ri, t, r - 3);
        if (c >= 3) for (int t = 0; t < 3; t++) Sc[t] = cross_e(ri, t, c - 3);
        double v;
        if (r < 3 && c < 3) v = (r == c) ? 1.0 : 0.0;
        else if (c < 3) v = Sr[c];
        else v = Sr[0] * Sc[0] + Sr[1] * Sc[1] + Sr[2] * Sc[2] + ((r == c) ? 1.0 : 0.0);
        s += v;
      }
    } else {
      const int h = T->hinge_ids[r - 6];
      const double* Jh = w.jpos(0, h);
      const double* Zh = w.jz(0, h);
      const int h2 = (c >= 6) ? T->hinge_ids[c - 6] : -1;
      for (int i = 1; i < n; i++) {
        if (!in_subtree(T, i, h) || (h2 >= 0 && !in_subtree(T, i, h2))) continue;
        const double* Pi = w.pos(0, i);
        double a3[3], u[3];
        for (int t = 0; t < 3; t++) a3[t] = Jh[t] - Pi[t];
        cross3(a3, Zh, u);
        if (c < 6) {  // T_i row c . (u, jz_h)
          if (c < 3) {
            s += -u[c];
          } else {
            double ri[3], ru[3];
            for (int t = 0; t < 3; t++) ri[t] = Pi[t] - P0[t];
            cross3(ri, u, ru);
            s += -(ru[c - 3] + Zh[c - 3]);
          }
        } else {
          const double* J2 = w.jpos(0, h2);
          const double* Z2 = w.jz(0, h2);
          double b3[3], u2[3];
          for (int t = 0; t < 3; t++) b3[t] = J2[t] - Pi[t];
          cross3(b3, Z2, u2);
          s += u[0] * u2[0] + u[1] * u2[1] + u[2] * u2[2] + (Zh[0] * Z2[0] + Zh[1] * Z2[1] + Zh[2] * Z2[2]);
        }
      }
    }
    fr.W[r * m + c] = ((r == c) ? 1.0 : 0.0) + s;
  }
  for (int e = lane; e < m * ld; e += HALF) {  // [C | d]
    const int r = e / ld, q = e % ld;
    double v = 0.0;
    if (q < nq) {
      const int fi = q / 3, jj = q % 3;
      const double* fp = w.fpos(0, fi);
      if (r < 3) {
        v = (r == jj) ? 1.0 : 0.0;
      } else if (r < 6) {
        double d[3];
        for (int t = 0; t < 3; t++) d[t] = fp[t] - P0[t];
        v = cross_e(d, jj, r - 3);
      } else {
        const int h = T->hinge_ids[r - 6];
        if (in_subtree(T, T->footis[fi], h)) {
          const double* Jh = w.jpos(0, h);
          const double* Zh = w.jz(0, h);
          double d[3];
          for (int t = 0; t < 3; t++) d[t] = Jh[t] - fp[t];
          for (int t = 0; t < 3; t++) v += Zh[t] * cross_e(d, jj, t);
        }
      }
    } else if (r < 3) {
      v = sv.x[r];
    } else if (r < 6) {
      v = sv.x[3 * n + r - 3];
    } else {
      const int h = T->hinge_ids[r - 6];
      const double* Zh = w.jz(0, h);
      double t = 0;
      for (int j = 0; j < 3; j++) t += Zh[j] * sv.x[3 * n + 3 * h + j];
      v = z[r - 6] - t;
    }
    fr.Ct[r * ld + q] = v;
  }
  wave_sync();
  chol_half(fr.W, m, 0.0, lane);  // I + G G^T: eigenvalues >= 1
  if (lane < ld) {                // L^-1 [C | d], one column per lane
    for (int i = 0; i < m; i++) {
      double s = fr.Ct[i * ld + lane];
      for (int t = 0; t < i; t++) s -= fr.W[i * m + t] * fr.Ct[t * ld + lane];
      fr.Ct[i * ld + lane] = s / fr.W[i * m + i];
    }
  }
  wave_sync();
  uint32_t flags = 0;
  for (int pass = 0; pass < 2; pass++) {  // normal equations; second pass regularized
    double eps = 0;
    if (pass == 1) {
      for (int p = 0; p < nq; p++) {
        double s = 0;
        for (int i = 0; i < m; i++) s += fr.Ct[i * ld + p] * fr.Ct[i * ld + p];
        eps = fmax(eps, s);
      }
      eps *= 1e-12;
    }
    for (int e = lane; e < nq * ld; e += HALF) {
      const int p = e / ld, q = e % ld;
      if (q < nq && q > p) continue;
      double s = 0;
      for (int i = 0; i < m; i++) s += fr.Ct[i * ld + p] * fr.Ct[i * ld + q];
      if (q < nq) fr.W[p * nq + q] = s + ((p == q) ? eps : 0.0);
      else fr.y[p] = s;
    }
    wave_sync();
    if (chol_half(fr.W, nq, pass == 0 ? kFastPivotGuard : 0.0, lane)) break;
    flags = HS_FLAG_GENERAL;  // least squares not unique
  }
  if (lane == 0) {
    for (int i = 0; i < nq; i++) {
      double s = fr.y[i];
      for (int k = 0; k < i; k++) s -= fr.W[i * nq + k] * fr.y[k];
      fr.y[i] = s / fr.W[i * nq + i];
    }
    for (int i = nq - 1; i >= 0; i--) {
      double s = fr.y[i];
      for (int k = i + 1; k < nq; k++) s -= fr.W[k * nq + i] * fr.y[k];
      fr.y[i] = s / fr.W[i * nq + i];
    }
  }
  wave_sync();
  return flags;
}

template <class W, class SV>
__device__ void forces_step(const hs_topo* T, const hs_run_args& a, const hs::launch_map& mp, const SetupL& st,
                            SV& sv, ForceL& fr, const W& w, int b, bool live, int h, int lane) {
  const int nf = T->nf, cfg = T->cfg, nl = T->n_limbs, nq = 3 * nf;
  dynamics(T, st, sv, w, lane);
  particular(T, sv, w, lane);
  const size_t row = (size_t)b * a.horizon + h;
  const double* z = mp.tau_in + (live ? row : 0) * mp.st_tau;
  uint32_t flags = forces_solve(T, sv, fr, w, z, lane);
  if (half_ballot(lane < nq && fr.y[lane] != fr.y[lane])) flags |= HS_FLAG_NAN;
  if (half_ballot(lane < nl && w.unreach(0, lane))) flags |= HS_FLAG_UNREACH;
  if (live && a.cf && lane < mp.st_cf) a.cf[row * mp.st_cf + lane] = (lane < nq) ? fr.y[lane] : 0.0;
  if (live && a.q && lane < mp.st_q) a.q[row * mp.st_q + lane] = (lane < cfg) ? w.q(0)[lane] : 0.0;
  if (live && a.flags && lane == 0) a.flags[row] = flags;
}

template <int NM, bool FORCES>
__global__ __launch_bounds__(WAVE, HS_MIN_WAVES) void hs_rollout_kernel(const hs_topo* __restrict__ T0,
                                                                                 hs_run_args a, GenWS* __restrict__ gws,
                                                                                 hs::launch_map mp) {
  __shared__ Smem<NM, FORCES> smem[2];
  const int sub = threadIdx.x / HALF;  // rollout slot within the wave
  const int lane = threadIdx.x % HALF; // lane within the rollout
  // one model per wavefront: the topology pointer stays wave-uniform (scalar loads)
  const hs_topo* __restrict__ T = mp.topos ? mp.topos[mp.wave_model[blockIdx.x]] : T0;
  int b, bb;
  bool live;  // an idle half (odd group) computes a copy of its neighbour and stores nothing
  if (mp.wave_rollouts) {
    b = mp.wave_rollouts[2 * blockIdx.x + sub];
    live = b >= 0;
    bb = live ? b : mp.wave_rollouts[2 * blockIdx.x];
  } else {
    b = blockIdx.x * 2 + sub;
    live = b < a.n_rollouts;
    bb = live ? b : a.n_rollouts - 1;
  }
  GenWS* G = gws + (live ? b : a.n_rollouts);
  Smem<NM, FORCES>& sm = smem[sub];
  double work = (live && a.accumulate && a.work_cot) ? a.work_cot[2 * (size_t)b] : 0.0;
  const hs_gait_params g = a.params[bb];
  const int nl = T->n_limbs;
  const bool ignore_reach = a.ignore_reach != 0;

  STAMP(0);
  gait_setup(T, g, a.n_t, sm.st, lane);
  STAMP(1);

  // K: the five-sample window, lane = (sample, limb)
  const int i = a.k0 + 2;  // centre sample of this launch's step
  {
    const int sl = lane / nl, L = lane % nl;
    if (sl < NS) kin_sample(T, g, sm.st, i - 2 + sl, L, ignore_reach, OneWin<NM, FORCES>{&sm.d}, sl - 2);
    wave_sync();
  }
  STAMP(2);
  if constexpr (FORCES) {
    forces_step(T, a, mp, sm.st, sm.sv, sm.d.fr, OneWin<NM, FORCES>{&sm.d}, b, live, mp.h_row, lane);
    return;
  } else {
    step(T, a, mp, sm.st, sm.sv, sm.d.fl, sm.d.gl, sm.d.wk, OneWin<NM, FORCES>{&sm.d}, G, b, live, mp.h_row, work,
         lane);
  }
  if (lane == 0 && live) {
    double cot = work / (T->total_mass * g.step_length);
    if (a.work_cot) {
      a.work_cot[2 * (size_t)b] = work;
      a.work_cot[2 * (size_t)b + 1] = cot;
    }
    if (a.best_key) atomicMin((unsigned long long*)a.best_key, (unsigned long long)best_key(cot, a.rollout_id_base + b));
  }
}

}  // namespace

#ifdef HS_STAMPS
extern "C" int hs_debug_read_stamps(unsigned long long* out, int n_rows) {
  if (n_rows > 4096) n_rows = 4096;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 16 * n_rows, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int hs_debug_clear_stamps() {
  static unsigned long long zero[4096][16];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
#endif

namespace hs {

size_t general_workspace_bytes() { return sizeof(GenWS); }

launch_map single_model_map(const hs_topo& t, int32_t n_rollouts) {
  launch_map mp{};
  mp.n_waves = (n_rollouts + 1) / 2;  // two rollouts per wavefront
  mp.max_parts = t.n;
  mp.st_tau = t.nmj;
  mp.st_cf = 3 * t.nf;
  mp.st_q = t.cfg;
  mp.st_x = 6 * t.n;
  return mp;
}

template <int NM>
void launch_nm(const hs_topo* d_topo, const hs_run_args& a, GenWS* ws, const launch_map& mp, hipStream_t st) {
  if (mp.tau_in)
    hipLaunchKernelGGL((hs_rollout_kernel<NM, true>), dim3(mp.n_waves), dim3(WAVE), 0, st, d_topo, a, ws, mp);
  else
    hipLaunchKernelGGL((hs_rollout_kernel<NM, false>), dim3(mp.n_waves), dim3(WAVE), 0, st, d_topo, a, ws, mp);
}

int launch_rollouts(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp) {
  if (a.n_rollouts <= 0 || mp.n_waves <= 0) return 0;
  hipStream_t st = (hipStream_t)a.stream;
  GenWS* ws = (GenWS*)workspace;
  // one launch per step of the horizon: step h writes output row h, work accumulates in
  // step order (periodic.cpp:291-304), the best key is taken after the last step
  for (int h = 0; h < a.horizon; h++) {
    hs_run_args ah = a;
    launch_map mh = mp;
    ah.k0 = a.k0 + h;
    ah.accumulate = (h == 0) ? a.accumulate : 1;
    if (h + 1 < a.horizon) ah.best_key = nullptr;
    mh.h_row = h;
    // smallest LDS layout that holds the (largest) model's parts: myant 17, spider 19, hexapod 22
    if (mp.max_parts <= 18) launch_nm<18>(d_topo, ah, ws, mh, st);
    else if (mp.max_parts <= 22) launch_nm<22>(d_topo, ah, ws, mh, st);
    else launch_nm<HS_NMAX>(d_topo, ah, ws, mh, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}

}  // namespace hs
