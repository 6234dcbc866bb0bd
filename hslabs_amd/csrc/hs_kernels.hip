// hs_kernels.hip -- the batched control-loop hot path on gfx950 (MI355X).
//
// One wavefront (one 64-thread workgroup) per rollout. Per rollout the wave
//   S  sets up the gait (pgssweeper::setup_pergen, pergen.cpp:453-507),
//   K  samples the trajectory: lane = (sample, limb) runs pergen set_rec
//      (pergen.cpp:225-239), the torso/body chain FK, limb IK (lik.cpp:151-223,
//      316-347) and the limb FK (model.cpp:183-201), and writes the dynamic
//      features of the parts it owns (dynrec.cpp:134-155) to an LDS ring of
//      five samples,
//   D  lane = part: 5-point finite differences (dynrec.cpp:175-224),
//   S1 lane = part, leaves -> root: particular solution of B0 x = f
//      (replaces the SparseQR solve of ftsolver.cpp:107-113 by the tree
//      back-substitution B0's block-triangular structure allows),
//   S2 zeroth/first-order Gram matrices in the tree-built null basis
//      [-B0^-1 Bc; I] (replaces SparseQR(B^T)'s Q, ftsolver.cpp:116-146),
//   S3 the adaptive-rank FullPivLU / ColPivHouseholderQR loop of
//      ftsolver.cpp:185-236 with Eigen 3.3 semantics, all 64 lanes on the
//      k x k (k <= 18) matrices held in LDS,
//   S4 motor torques, contact forces and positive work (periodic.cpp:261-343).
// Every floating-point operation sequence matches oracle/hs_oracle.cpp's tree
// mode (compiled with -ffp-contract=off), so the only expected differences
// against it are ULP differences of the device sin/cos/atan2/acos/asin.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>

#include "hs_internal.h"
#include "hs_math.h"

namespace {

using namespace hsd;

constexpr int WAVE = 64;
constexpr int NS = 5;        // samples in the derivative stencil (periodic.cpp:192-202)
constexpr int LD = HS_KMAX;  // leading dimension of k x k matrices in LDS

struct SampleL {
  double pos[HS_NMAX][3], jpos[HS_NMAX][3], ust[HS_NMAX][3], rot[HS_NMAX][9], jz[HS_NMAX][3];
  double fpos[HS_LMAX][3];
  double q[6 + HS_NMAX];
  int contact[HS_LMAX];
  int unreach[HS_LMAX];
};

struct SetupL {
  double pos0[HS_LMAX][3];  // default foot positions, pergen order
  double ts[HS_LMAX], xs[HS_LMAX];
  double t_step, max_radius, v, dt;
};

struct FastL {  // per-contact blocks exchanged through LDS
  double A[HS_LMAX][18], D[HS_LMAX][9], g[HS_LMAX][3], Dinv[HS_LMAX][9], S[HS_LMAX][36], h[HS_LMAX][6];
  double lam[6];
  int ok[HS_LMAX];
};

struct GenMats {  // k x k matrices of the Eigen-style general path
  double ntn0[HS_KMAX * LD], lu[HS_KMAX * LD], Ny[HS_KMAX * LD], M[HS_KMAX * LD], qr[HS_KMAX * LD];
};

struct SolveL {
  double f[6 * HS_NMAX], x[6 * HS_NMAX];
  union {
    GenMats gm;  // general path
    FastL fl;    // fast path (dead once the general path starts)
  };
  double n1[HS_LMAX][9];  // 3x3 diagonal blocks of the first-order Gram (column-major)
  double ntx0[HS_KMAX], ntx1[HS_KMAX], y0[HS_KMAX], b[HS_KMAX], z[HS_KMAX], y[HS_KMAX], c[HS_KMAX];
  double hc[HS_KMAX], nu[HS_KMAX], nd[HS_KMAX], tau[HS_NMAX];
  int rowsT[HS_KMAX], colsT[HS_KMAX], q[HS_KMAX], piv[HS_KMAX], rycol[HS_KMAX], cperm[HS_KMAX];
  int cfoot[HS_LMAX];
};

struct Smem {
  SampleL s[NS];
  SetupL st;
  SolveL sv;
};

__device__ inline void wave_sync() { __syncthreads(); }

#ifdef HS_STAMPS
// diagnostic build only: per-phase shader-clock stamps of the first 4096 rollouts
__device__ unsigned long long g_stamps[4096][16];
#define STAMP(slot)                                                                  \
  do {                                                                               \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_stamps[blockIdx.x][slot] += __builtin_amdgcn_s_memtime(); \
  } while (0)
#else
#define STAMP(slot) do {} while (0)
#endif

__device__ inline A34 node_joint_parent(const hs_topo* T, int v) { return load34(T->node[v].J_A_parent); }
__device__ inline A34 node_pj(const hs_topo* T, int v) { return load34(T->node[v].A_pj_body); }

// ---------------------------------------------------------------------------
// S: gait setup, lanes L < n_limbs (pergen.cpp:453-507, 30-51, 143-153)
// ---------------------------------------------------------------------------
__device__ void gait_setup(const hs_topo* T, const hs_gait_params& g, int n_t, Smem& sm, int lane) {
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
    sm.st.pos0[j][0] = pos[0];
    sm.st.pos0[j][1] = pos[1];
    sm.st.pos0[j][2] = T->rcap;  // set_limb_poss
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
        sm.st.ts[k] = ts;
        sm.st.xs[k] = ts + t_step / 2 - 1. / 2;
      }
    }
    sm.st.t_step = t_step;
    sm.st.v = g.step_length / g.period;  // pergensetup::set_TLh
    sm.st.dt = g.period / n_t;           // record_trajectory
  }
  wave_sync();
  if (lane == 0) {  // compute_max_radius
    double mr = 0;
    if (g.curvature != 0) {
      double cy = 1. / g.curvature;
      for (int j = 0; j < nl; j++) {
        double d0 = sm.st.pos0[j][0] - 0.0, d1 = sm.st.pos0[j][1] - cy, d2 = sm.st.pos0[j][2] - 0.0;
        double s = 0;
        s += d0 * d0;
        s += d1 * d1;
        s += d2 * d2;
        double rad = sqrt(s);
        if (rad > mr) mr = rad;
      }
    }
    sm.st.max_radius = mr;
  }
  wave_sync();
}

// ---------------------------------------------------------------------------
// K: one (sample, limb) pair per lane
// ---------------------------------------------------------------------------
__device__ inline double stepx(double t) { return (1 - cos(kPi * t)) / 2; }
__device__ inline double stepz(double t) { double a = sin(kPi * t); return a * a; }

__device__ void node_features(const hs_topo* T, int v, const A34& A, const A34* J, SampleL& S) {
  const hs_node& nd = T->node[v];
  double com[3] = {nd.com[0], nd.com[1], nd.com[2]}, p[3];
  mulp(A, com, p);
  for (int i = 0; i < 3; i++) S.pos[v][i] = p[i];
  for (int i = 0; i < 3; i++) S.jpos[v][i] = J ? (*J)(i, 3) : A(i, 3);
  S.ust[v][0] = (A(2, 1) - A(1, 2)) / 2;
  S.ust[v][1] = (A(0, 2) - A(2, 0)) / 2;
  S.ust[v][2] = (A(1, 0) - A(0, 1)) / 2;
  for (int c = 0; c < 3; c++)
    for (int r = 0; r < 3; r++) S.rot[v][c * 3 + r] = A(r, c);
  for (int i = 0; i < 3; i++) S.jz[v][i] = J ? (*J)(i, 2) : 0.0;
  if (nd.foot >= 0) {
    double cap[3] = {nd.cap[0], nd.cap[1], nd.cap[2]}, fp[3];
    mulp(A, cap, fp);
    for (int i = 0; i < 3; i++) S.fpos[nd.foot][i] = fp[i];
    S.contact[nd.foot] = fp[2] < T->rcap + 1e-4;
  }
}

__device__ void kin_sample(const hs_topo* T, const hs_gait_params& g, const SetupL& st, int isample, int L,
                           bool ignore_reach, SampleL& S) {
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
  if (L == 0) {
    for (int i = 0; i < 6; i++) S.q[i] = q6[i];
    A34 J0 = node_joint_parent(T, 0);  // torso joint frame J = I * J_A_parent
    node_features(T, 0, A0, &J0, S);
  }
  A34 A = A0;
  for (int k = 1; k < T->limb_chain_len[L]; k++) {
    int v = T->limb_chain[L][k];
    A = mul(A, node_pj(T, v));
    if (T->node[v].owner_limb == L) node_features(T, v, A, nullptr, S);
  }
  int c = T->limb_child[L];
  A34 J = mul(A, node_joint_parent(T, c));  // poslimb (lik.cpp:341-347)
  A34 Jinv = invert(J);
  double pl[3], ja[3];
  mulp(Jinv, target, pl);
  bool unreach = false, fail = false;
  limb_ik(T->lik_kind, T->ls, T->limb_ysign[L], pl, ja, ignore_reach, unreach, fail);
  S.unreach[L] = (unreach || fail) ? 1 : 0;
  // limb FK with the new joint values (compute_dynrecs' recompute_modelnodes)
  int v = c;
  for (int k = 0; k < 3; k++) {
    const hs_node& nd = T->node[v];
    A34 Jv = (k == 0) ? J : mul(A, node_joint_parent(T, v));
    A = mul(mul(Jv, hinge_joint(ja[k])), node_pj(T, v));
    S.q[6 + nd.hinge] = ja[k];
    node_features(T, v, A, &Jv, S);
    if (k < 2) v = nd.kids[0];
  }
}

// ---------------------------------------------------------------------------
// D: finite differences at the centre sample, lane = part (dynrec.cpp:175-224)
// ---------------------------------------------------------------------------
__device__ void dynamics(const hs_topo* T, Smem& sm, int im2, int im1, int i0, int ip1, int ip2, int lane) {
  const int n = T->n;
  if (lane < n) {
    const int i = lane;
    const double inv = 1. / (2 * sm.st.dt);
    const double m = T->mass[i];
    double vp[3], vm[3], mr[3], wp[3], wm[3], amp[3], amm[3], amr[3];
    for (int j = 0; j < 3; j++) {
      vp[j] = sm.s[ip2].pos[i][j] - sm.s[i0].pos[i][j];
      vp[j] *= inv;
      vm[j] = sm.s[i0].pos[i][j] - sm.s[im2].pos[i][j];
      vm[j] *= inv;
      double mp = vp[j] * m, mm = vm[j] * m;
      mr[j] = mp - mm;
      mr[j] *= inv;
      wp[j] = sm.s[ip2].ust[i][j] - sm.s[i0].ust[i][j];
      wp[j] *= inv;
      wm[j] = sm.s[i0].ust[i][j] - sm.s[im2].ust[i][j];
      wm[j] *= inv;
    }
    // ang_mom = R (I (R^T w)), I = identity (compute_ang_mom, dynrec.cpp:205-216)
    const double* Rp = sm.s[ip1].rot[i];
    const double* Rm = sm.s[im1].rot[i];
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
      sm.sv.f[3 * i + j] = mr[j];
      sm.sv.f[3 * (n + i) + j] = amr[j];
    }
    sm.sv.f[3 * i + 2] += m * 1.0;  // gravity, g = 1 (dynrec.cpp:291-295)
  }
  wave_sync();
}

// ---------------------------------------------------------------------------
// S1: tree back-substitution B0 x = f, level by level (deepest first)
// ---------------------------------------------------------------------------
__device__ void particular(const hs_topo* T, Smem& sm, const SampleL& S, int lane) {
  const int n = T->n;
  for (int level = T->max_depth; level >= 0; level--) {
    if (lane < n && T->node[lane].depth == level) {
      const int i = lane;
      const hs_node& nd = T->node[i];
      double F[3], Tq[3];
      for (int j = 0; j < 3; j++) { F[j] = sm.sv.f[3 * i + j]; Tq[j] = sm.sv.f[3 * (n + i) + j]; }
      for (int kk = 0; kk < nd.nkids; kk++) {
        int c = nd.kids[kk];
        for (int j = 0; j < 3; j++) F[j] += sm.sv.x[3 * c + j];
        double r[3];
        for (int j = 0; j < 3; j++) r[j] = S.pos[i][j] - S.jpos[c][j];
        const double* Fc = &sm.sv.x[3 * c];
        Tq[0] -= r[1] * Fc[2] - r[2] * Fc[1];
        Tq[1] -= r[2] * Fc[0] - r[0] * Fc[2];
        Tq[2] -= r[0] * Fc[1] - r[1] * Fc[0];
        for (int j = 0; j < 3; j++) Tq[j] += sm.sv.x[3 * (n + c) + j];
      }
      for (int j = 0; j < 3; j++) sm.sv.x[3 * i + j] = F[j];
      if (nd.parent >= 0) {
        double r[3];
        for (int j = 0; j < 3; j++) r[j] = S.jpos[i][j] - S.pos[i][j];
        Tq[0] -= r[1] * F[2] - r[2] * F[1];
        Tq[1] -= r[2] * F[0] - r[0] * F[2];
        Tq[2] -= r[0] * F[1] - r[1] * F[0];
      }
      for (int j = 0; j < 3; j++) sm.sv.x[3 * (n + i) + j] = Tq[j];
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

// ---------------------------------------------------------------------------
// S2: Gram matrices of the masked, penalty-weighted null basis (ftsolver.cpp:185-207)
// ---------------------------------------------------------------------------
__device__ int build_grams(const hs_topo* T, Smem& sm, const SampleL& S, int lane) {
  const int n = T->n, nf = T->nf;
  int nc = 0;
  for (int fi = 0; fi < nf; fi++) {
    if (S.contact[fi]) {
      if (lane == 0) sm.sv.cfoot[nc] = fi;
      nc++;
    }
  }
  const int k = 3 * nc;
  wave_sync();
  // zeroth order: rows {0,1,2} = -I, rows {3n..3n+2} = (pos_0 - fpos) x e_jj, weight 1
  for (int e = lane; e < k * k; e += WAVE) {
    int ci = e % k, cj = e / k;
    int fa = sm.sv.cfoot[ci / 3], fb = sm.sv.cfoot[cj / 3];
    int ja = ci % 3, jb = cj % 3;
    double da[3], db[3];
    for (int r = 0; r < 3; r++) { da[r] = S.pos[0][r] - S.fpos[fa][r]; db[r] = S.pos[0][r] - S.fpos[fb][r]; }
    double s = 0.0;
    for (int r = 0; r < 3; r++) {
      double na = (r == ja) ? -1.0 : 0.0, nb = (r == jb) ? -1.0 : 0.0;
      s = s + na * nb;
    }
    for (int r = 0; r < 3; r++) s = s + cross_e(da, ja, r) * cross_e(db, jb, r);
    sm.sv.gm.ntn0[ci + cj * LD] = s;
  }
  if (lane < k) {
    int ci = lane, fa = sm.sv.cfoot[ci / 3], ja = ci % 3;
    double da[3];
    for (int r = 0; r < 3; r++) da[r] = S.pos[0][r] - S.fpos[fa][r];
    double s = 0.0;
    for (int r = 0; r < 3; r++) s = s + ((r == ja) ? -1.0 : 0.0) * (1.0 * sm.sv.x[r]);
    for (int r = 0; r < 3; r++) s = s + cross_e(da, ja, r) * (1.0 * sm.sv.x[3 * n + r]);
    sm.sv.ntx0[ci] = s;
  }
  // first order: torque rows of the non-root ancestors of each contact foot,
  // weighted by the joint-axis components (set_action_penalties, ftsolver.cpp:239-246)
  for (int e = lane; e < nc * 9 + k; e += WAVE) {
    bool is_vec = e >= nc * 9;
    int cc = is_vec ? (e - nc * 9) / 3 : e / 9;
    int a_col = is_vec ? (e - nc * 9) % 3 : (e % 9) % 3;
    int b_col = is_vec ? 0 : (e % 9) / 3;
    int foot = T->footis[sm.sv.cfoot[cc]];
    // ancestors of foot below the root, in ascending part order (top of the chain first)
    int chain[HS_NMAX], len = 0;
    for (int a = foot; a >= 0 && T->node[a].parent >= 0; a = T->node[a].parent) chain[len++] = a;
    double s = 0.0;
    for (int t = len - 1; t >= 0; t--) {
      int a = chain[t];
      double d[3];
      for (int r = 0; r < 3; r++) d[r] = S.jpos[a][r] - S.fpos[sm.sv.cfoot[cc]][r];
      for (int r = 0; r < 3; r++) {
        double w = S.jz[a][r];
        double na = w * cross_e(d, a_col, r);
        double nb = is_vec ? w * sm.sv.x[3 * n + 3 * a + r] : w * cross_e(d, b_col, r);
        s = s + na * nb;
      }
    }
    if (is_vec) sm.sv.ntx1[3 * cc + a_col] = s;
    else sm.sv.n1[cc][b_col * 3 + a_col] = s;
  }
  wave_sync();
  return k;
}

// first-order Gram entry (block diagonal)
__device__ inline double ntn1_at(const SolveL& sv, int i, int j) {
  return (i / 3 == j / 3) ? sv.n1[i / 3][(j % 3) * 3 + (i % 3)] : 0.0;
}

// wave-wide argmax with first-index tie break
__device__ inline void wave_argmax(double& v, int& idx) {
  for (int off = 32; off >= 1; off >>= 1) {
    double ov = __shfl_xor(v, off);
    int oi = __shfl_xor(idx, off);
    if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
  }
}

struct LUInfo {
  int nz;          // nonzero pivots
  double maxpivot;
};

// Eigen FullPivLU::computeInPlace on sv.gm.lu (k x k)
__device__ LUInfo fullpiv_lu(SolveL& sv, int k, int lane) {
  for (int e = lane; e < k * k; e += WAVE) {
    int i = e % k, j = e / k;
    sv.gm.lu[i + j * LD] = sv.gm.ntn0[i + j * LD];
  }
  wave_sync();
  LUInfo info{k, 0.0};
  for (int p = 0; p < k; p++) {
    const int m = k - p;
    double best = -1.0;
    int bidx = 1 << 30;
    for (int e = lane; e < m * m; e += WAVE) {
      double a = fabs(sv.gm.lu[(p + e % m) + (p + e / m) * LD]);
      if (a > best || (a == best && e < bidx)) { best = a; bidx = e; }
    }
    wave_argmax(best, bidx);
    if (best == 0) {
      info.nz = p;
      for (int i = p + lane; i < k; i += WAVE) { sv.rowsT[i] = i; sv.colsT[i] = i; }
      break;
    }
    if (best > info.maxpivot) info.maxpivot = best;
    const int bi = p + bidx % m, bj = p + bidx / m;
    if (lane == 0) { sv.rowsT[p] = bi; sv.colsT[p] = bj; }
    if (bi != p && lane < k) {
      double t = sv.gm.lu[p + lane * LD];
      sv.gm.lu[p + lane * LD] = sv.gm.lu[bi + lane * LD];
      sv.gm.lu[bi + lane * LD] = t;
    }
    wave_sync();
    if (bj != p && lane < k) {
      double t = sv.gm.lu[lane + p * LD];
      sv.gm.lu[lane + p * LD] = sv.gm.lu[lane + bj * LD];
      sv.gm.lu[lane + bj * LD] = t;
    }
    wave_sync();
    if (p < k - 1) {
      double piv = sv.gm.lu[p + p * LD];
      if (lane > p && lane < k) sv.gm.lu[lane + p * LD] /= piv;
      wave_sync();
      const int mm = k - p - 1;
      for (int e = lane; e < mm * mm; e += WAVE) {
        int i = p + 1 + e % mm, j = p + 1 + e / mm;
        sv.gm.lu[i + j * LD] -= sv.gm.lu[i + p * LD] * sv.gm.lu[p + j * LD];
      }
      wave_sync();
    }
  }
  if (lane == 0) {
    for (int i = 0; i < k; i++) sv.q[i] = i;
    for (int p = 0; p < k; p++) { int t = sv.q[p]; sv.q[p] = sv.q[sv.colsT[p]]; sv.q[sv.colsT[p]] = t; }
  }
  wave_sync();
  return info;
}

__device__ inline int lu_rank(const SolveL& sv, const LUInfo& info, double thr) {
  double pt = fabs(info.maxpivot) * thr;
  int r = 0;
  for (int i = 0; i < info.nz; i++) r += fabs(sv.gm.lu[i + i * LD]) > pt;
  return r;
}

// column-oriented upper-triangular solve of vec[0..r) against U = mat (ld LD), all lanes
__device__ void upper_solve_shared(const double* U, double* vec, int r, int lane) {
  for (int i = r - 1; i >= 0; i--) {
    double ci = vec[i];
    if (ci != 0) {
      double xi = ci / U[i + i * LD];
      if (lane < i) vec[lane] -= xi * U[lane + i * LD];
      if (lane == i) vec[i] = xi;
    }
    wave_sync();
  }
}

// FullPivLU::solve(-ntx0) -> sv.y0
__device__ void lu_solve(SolveL& sv, const LUInfo& info, int k, int r, int lane) {
  if (lane == 0) {
    for (int i = 0; i < k; i++) sv.c[i] = -sv.ntx0[i];
    for (int p = 0; p < k; p++) { double t = sv.c[p]; sv.c[p] = sv.c[sv.rowsT[p]]; sv.c[sv.rowsT[p]] = t; }
  }
  if (lane < k) sv.y0[lane] = 0.0;
  wave_sync();
  if (r == 0) return;
  for (int j = 0; j < k; j++) {  // unit lower
    double cj = sv.c[j];
    if (lane > j && lane < k) sv.c[lane] -= cj * sv.gm.lu[lane + j * LD];
    wave_sync();
  }
  upper_solve_shared(sv.gm.lu, sv.c, r, lane);
  if (lane < r) sv.y0[sv.q[lane]] = sv.c[lane];
  wave_sync();
}

// FullPivLU::kernel() -> sv.gm.Ny (k x dimker); uses sv.gm.qr as scratch; sv.piv/rycol set
__device__ void lu_kernel_image(SolveL& sv, const LUInfo& info, int k, int r, double thr, int lane) {
  if (lane == 0) {
    double pt = info.maxpivot * thr;
    int p = 0;
    for (int i = 0; i < info.nz; i++)
      if (fabs(sv.gm.lu[i + i * LD]) > pt) sv.piv[p++] = i;
    for (int i = 0; i < r; i++) sv.rycol[i] = sv.q[sv.piv[i]];  // image columns
  }
  wave_sync();
  const int dimker = k - r;
  if (dimker == 0) return;
  double* mm = sv.gm.qr;  // r x k trapezoid
  for (int e = lane; e < r * k; e += WAVE) {
    int i = e % r, j = e / r;
    mm[i + j * LD] = (j >= i) ? sv.gm.lu[sv.piv[i] + j * LD] : 0.0;
  }
  wave_sync();
  if (lane < r) {  // bring non-negligible pivots to the front (rows own a column swap each)
    for (int i = 0; i < r; i++) {
      int pc = sv.piv[i];
      if (pc != i) { double t = mm[lane + i * LD]; mm[lane + i * LD] = mm[lane + pc * LD]; mm[lane + pc * LD] = t; }
    }
  }
  wave_sync();
  if (lane < dimker) {  // solve U11 X = U12, one right-hand column per lane
    double* col = &mm[(r + lane) * LD];
    for (int i = r - 1; i >= 0; i--) {
      if (col[i] != 0) {
        col[i] /= mm[i + i * LD];
        for (int rr = 0; rr < i; rr++) col[rr] -= col[i] * mm[rr + i * LD];
      }
    }
  }
  wave_sync();
  if (lane < r) {
    for (int i = r - 1; i >= 0; i--) {
      int pc = sv.piv[i];
      if (pc != i) { double t = mm[lane + i * LD]; mm[lane + i * LD] = mm[lane + pc * LD]; mm[lane + pc * LD] = t; }
    }
  }
  wave_sync();
  for (int e = lane; e < k * dimker; e += WAVE) {
    int i = e % k, kk = e / k;
    int row = sv.q[i];
    double v;
    if (i < r) v = -mm[i + (r + kk) * LD];
    else v = (i == r + kk) ? 1.0 : 0.0;
    sv.gm.Ny[row + kk * LD] = v;
  }
  wave_sync();
}

// Eigen 3.3 ColPivHouseholderQR on sv.gm.qr (k x k, copy of M); returns nonzero pivots
__device__ int colpiv_qr(SolveL& sv, int k, int lane) {
  for (int e = lane; e < k * k; e += WAVE) {
    int i = e % k, j = e / k;
    sv.gm.qr[i + j * LD] = sv.gm.M[i + j * LD];
  }
  wave_sync();
  if (lane < k) {
    double s = 0;
    for (int i = 0; i < k; i++) s += sv.gm.qr[i + lane * LD] * sv.gm.qr[i + lane * LD];
    sv.nd[lane] = sqrt(s);
    sv.nu[lane] = sv.nd[lane];
  }
  wave_sync();
  double mx = 0;
  for (int j = 0; j < k; j++) mx = fmax(mx, sv.nu[j]);
  const double th = mx * DBL_EPSILON;
  const double threshold_helper = th * th / (double)k;
  const double ndt = sqrt(DBL_EPSILON);
  int np = k;
  for (int p = 0; p < k; p++) {
    int bi = p;
    double bv = sv.nu[p];
    for (int j = p + 1; j < k; j++)
      if (sv.nu[j] > bv) { bv = sv.nu[j]; bi = j; }
    if (np == k && bv * bv < threshold_helper * (double)(k - p)) np = p;
    wave_sync();
    if (lane == 0) sv.cperm[p] = bi;
    if (bi != p) {
      if (lane < k) {
        double t = sv.gm.qr[lane + p * LD];
        sv.gm.qr[lane + p * LD] = sv.gm.qr[lane + bi * LD];
        sv.gm.qr[lane + bi * LD] = t;
      }
      if (lane == 0) {
        double t = sv.nu[p]; sv.nu[p] = sv.nu[bi]; sv.nu[bi] = t;
        t = sv.nd[p]; sv.nd[p] = sv.nd[bi]; sv.nd[bi] = t;
      }
    }
    wave_sync();
    // makeHouseholderInPlace on column p, rows p..k-1
    const int len = k - p;
    double c0 = sv.gm.qr[p + p * LD];
    double tail = 0;
    for (int i = 1; i < len; i++) tail += sv.gm.qr[p + i + p * LD] * sv.gm.qr[p + i + p * LD];
    double tau, beta;
    if (len == 1 || tail <= DBL_MIN) {
      tau = 0;
      beta = c0;
      if (lane >= 1 && lane < len) sv.gm.qr[p + lane + p * LD] = 0;
    } else {
      beta = sqrt(c0 * c0 + tail);
      if (c0 >= 0) beta = -beta;
      double den = c0 - beta;
      if (lane >= 1 && lane < len) sv.gm.qr[p + lane + p * LD] /= den;
      tau = (beta - c0) / beta;
    }
    wave_sync();
    if (lane == 0) { sv.gm.qr[p + p * LD] = beta; sv.hc[p] = tau; }
    // apply to columns p+1..k-1, then downdate their norms (one column per lane)
    const int j = lane;
    if (j > p && j < k) {
      if (len == 1) {
        sv.gm.qr[p + j * LD] *= (1 - tau);
      } else if (tau != 0) {
        double tmp = 0;
        for (int i = 1; i < len; i++) tmp += sv.gm.qr[p + i + p * LD] * sv.gm.qr[p + i + j * LD];
        tmp += sv.gm.qr[p + j * LD];
        sv.gm.qr[p + j * LD] -= tau * tmp;
        for (int i = 1; i < len; i++) sv.gm.qr[p + i + j * LD] -= tau * sv.gm.qr[p + i + p * LD] * tmp;
      }
      if (sv.nu[j] != 0) {
        double temp = fabs(sv.gm.qr[p + j * LD]) / sv.nu[j];
        temp = (1 + temp) * (1 - temp);
        temp = temp < 0 ? 0 : temp;
        double ratio = sv.nu[j] / sv.nd[j];
        double temp2 = temp * (ratio * ratio);
        if (temp2 <= ndt) {
          double s = 0;
          for (int i = p + 1; i < k; i++) s += sv.gm.qr[i + j * LD] * sv.gm.qr[i + j * LD];
          sv.nd[j] = sqrt(s);
          sv.nu[j] = sv.nd[j];
        } else {
          sv.nu[j] *= sqrt(temp);
        }
      }
    }
    wave_sync();
  }
  return np;
}

// QR solve M z = b (least squares, basic solution) -> sv.z
__device__ void qr_solve(SolveL& sv, int k, int np, int lane) {
  if (lane < k) { sv.c[lane] = sv.b[lane]; sv.z[lane] = 0.0; }
  wave_sync();
  if (np == 0) return;
  for (int p = 0; p < np; p++) {
    const int len = k - p;
    const double tau = sv.hc[p];
    if (len == 1) {
      if (lane == p) sv.c[p] *= (1 - tau);
    } else if (tau != 0) {
      double tmp = 0;
      for (int i = 1; i < len; i++) tmp += sv.gm.qr[p + i + p * LD] * sv.c[p + i];
      tmp += sv.c[p];
      if (lane == 0) sv.c[p] -= tau * tmp;
      if (lane >= 1 && lane < len) sv.c[p + lane] -= tau * sv.gm.qr[p + lane + p * LD] * tmp;
    }
    wave_sync();
  }
  upper_solve_shared(sv.gm.qr, sv.c, np, lane);
  if (lane == 0) {
    int perm[HS_KMAX];
    for (int i = 0; i < k; i++) perm[i] = i;
    for (int p = 0; p < k; p++) { int t = perm[p]; perm[p] = perm[sv.cperm[p]]; perm[sv.cperm[p]] = t; }
    for (int i = 0; i < np; i++) sv.z[perm[i]] = sv.c[i];
  }
  wave_sync();
}

struct StepResult {
  uint32_t flags;
};

// S3: adaptive-rank two-stage least squares (ftsolver.cpp:277-303) -> sv.y
__device__ uint32_t contact_solve(SolveL& sv, int k, int lane) {
  uint32_t flags = 0;
  if (k == 0) return HS_FLAG_NO_CONTACT;
  int rank0 = k;
  int iters = 0;
  double rel_error = 0;
  do {
    iters++;
    STAMP(9);
    LUInfo info = fullpiv_lu(sv, k, lane);
    STAMP(10);
    double thr = DBL_EPSILON * (double)k;
    int r = lu_rank(sv, info, thr);
    for (int guard = 0; guard < 2100 && r > rank0; guard++) {  // setThreshold doubling
      thr = 2 * thr;
      r = lu_rank(sv, info, thr);
    }
    lu_solve(sv, info, k, r, lane);
    lu_kernel_image(sv, info, k, r, thr, lane);
    STAMP(11);
    if (r == k) flags |= HS_FLAG_FULL_RANK;
    rank0 = r;
    const int dimker = k - r;
    // b = -(ntx1 + ntn1 y0)
    if (lane < k) {
      int i = lane, b0 = (i / 3) * 3;
      double t = 0.0;
      for (int kk = b0; kk < b0 + 3; kk++) t = t + ntn1_at(sv, i, kk) * sv.y0[kk];
      sv.b[i] = -(sv.ntx1[i] + t);
    }
    // M = [ntn1 Ny, ntn0 Ry]
    for (int e = lane; e < k * k; e += WAVE) {
      int i = e % k, j = e / k;
      double s = 0.0;
      if (j < dimker) {
        int b0 = (i / 3) * 3;
        for (int kk = b0; kk < b0 + 3; kk++) s = s + ntn1_at(sv, i, kk) * sv.gm.Ny[kk + j * LD];
      } else {
        int col = sv.rycol[j - dimker];
        for (int kk = 0; kk < k; kk++) s = s + sv.gm.ntn0[i + kk * LD] * sv.gm.ntn0[kk + col * LD];
      }
      sv.gm.M[i + j * LD] = s;
    }
    wave_sync();
    STAMP(12);
    int np = colpiv_qr(sv, k, lane);
    STAMP(13);
    qr_solve(sv, k, np, lane);
    STAMP(14);
    // rel_error = |M z - b| / |b|
    if (lane < k) {
      double s = 0.0;
      for (int j = 0; j < k; j++) s = s + sv.gm.M[lane + j * LD] * sv.z[j];
      sv.c[lane] = s - sv.b[lane];
    }
    wave_sync();
    double rn = 0, bn = 0;
    for (int i = 0; i < k; i++) { rn += sv.c[i] * sv.c[i]; bn += sv.b[i] * sv.b[i]; }
    rel_error = sqrt(rn) / sqrt(bn);
    rank0--;
    if (lane < k) {
      double s = 0.0;
      for (int j = 0; j < dimker; j++) s = s + sv.gm.Ny[lane + j * LD] * sv.z[j];
      sv.y[lane] = sv.y0[lane] + s;
    }
    wave_sync();
    if (rel_error > 1e-6 && rank0 <= 0) { flags |= HS_FLAG_LOOP_EXHAUST; break; }
  } while (rel_error > 1e-6 && iters <= HS_KMAX + 1);
  if (iters > 1) flags |= HS_FLAG_RANK_RETRY;
  return flags;
}

// ---------------------------------------------------------------------------
// S3 fast path: closed form of the same lexicographic least squares
// (oracle/hs_oracle.cpp fast_contact_solve, identical operation order).
// One lane per contact builds A_c, D_c, g_c; >= 3 contacts: 6x6 Schur
// complement of the zeroth-order constraints; 1 contact: unique LS; 2 contacts:
// rank-5 kernel along the feet line. Returns false (wave-uniform) when a
// Cholesky pivot falls under the guard -> Eigen-style path.
// ---------------------------------------------------------------------------
constexpr double kFastPivotGuard = 1e-10;

__device__ inline bool chol_n(double* a, int n, double guard) {  // row-major, in place
  double mx = 0;
  for (int i = 0; i < n; i++) mx = fmax(mx, a[i * n + i]);
  for (int j = 0; j < n; j++) {
    double s = a[j * n + j];
    for (int k = 0; k < j; k++) s -= a[j * n + k] * a[j * n + k];
    if (!(s > guard * mx)) return false;
    double l = sqrt(s);
    a[j * n + j] = l;
    for (int i = j + 1; i < n; i++) {
      double t = a[i * n + j];
      for (int k = 0; k < j; k++) t -= a[i * n + k] * a[j * n + k];
      a[i * n + j] = t / l;
    }
  }
  return true;
}

__device__ inline void chol_solve_n(const double* L, int n, double* b) {
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * b[k];
    b[i] = s / L[i * n + i];
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = b[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * b[k];
    b[i] = s / L[i * n + i];
  }
}

__device__ inline void cross_rows(const double* d, double v[3][3]) {
  v[0][0] = 0;     v[0][1] = -d[2]; v[0][2] = d[1];
  v[1][0] = d[2];  v[1][1] = 0;     v[1][2] = -d[0];
  v[2][0] = -d[1]; v[2][1] = d[0];  v[2][2] = 0;
}



__device__ bool fast_solve(const hs_topo* T, SolveL& sv, FastL& fl, const SampleL& S, int nc, int lane) {
  const int n = T->n;
  if (nc == 0) return true;
  if (lane < nc) {  // A_c, D_c, g_c for contact c = lane
    const int c = lane, fi = sv.cfoot[c];
    const double* fp = S.fpos[fi];
    double d0[3], v[3][3];
    for (int r = 0; r < 3; r++) d0[r] = S.pos[0][r] - fp[r];
    cross_rows(d0, v);
    double* Ac = fl.A[c];
    for (int r = 0; r < 3; r++)
      for (int j = 0; j < 3; j++) { Ac[r * 3 + j] = (r == j) ? -1.0 : 0.0; Ac[(3 + r) * 3 + j] = v[r][j]; }
    double D[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
    for (int p = T->footis[fi]; p >= 0 && T->node[p].parent >= 0; p = T->node[p].parent) {
      double da[3], va[3][3];
      for (int r = 0; r < 3; r++) da[r] = S.jpos[p][r] - fp[r];
      cross_rows(da, va);
      for (int r = 0; r < 3; r++) {
        double w2 = S.jz[p][r] * S.jz[p][r];
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
      ok = chol_n(L, 3, kFastPivotGuard);
      if (ok) {
        double Dinv[9];
        for (int j = 0; j < 3; j++) {
          double e[3] = {0, 0, 0};
          e[j] = 1;
          chol_solve_n(L, 3, e);
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
            fl.S[c][6 * r + q] = s;
          }
          double s = 0;
          for (int j = 0; j < 3; j++) s += E[r * 3 + j] * g[j];
          fl.h[c][r] = s;
        }
        for (int i = 0; i < 9; i++) fl.Dinv[c][i] = Dinv[i];
      }
    }
    fl.ok[c] = ok;
  }
  wave_sync();
  for (int c = 0; c < nc; c++)
    if (!fl.ok[c]) return false;
  const double a[6] = {sv.x[0], sv.x[1], sv.x[2], sv.x[3 * n], sv.x[3 * n + 1], sv.x[3 * n + 2]};
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
      ok = chol_n(M, 3, kFastPivotGuard);
      if (ok) {
        chol_solve_n(M, 3, b);
        for (int i = 0; i < 3; i++) sv.y[i] = b[i];
      }
      fl.ok[0] = ok;
    }
  } else if (nc == 2) {  // rank 5: kernel n = (u,-u)/sqrt2 along the line between the feet
    if (lane == 0) {
      const double* f0 = S.fpos[sv.cfoot[0]];
      const double* f1 = S.fpos[sv.cfoot[1]];
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
        ok = chol_n(M, 6, kFastPivotGuard);
      }
      if (ok) {
        chol_solve_n(M, 6, b);
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
        for (int i = 0; i < 36; i++) Sm[i] += fl.S[c][i];
        for (int i = 0; i < 6; i++) h[i] += fl.h[c][i];
      }
      double lam[6];
      for (int r = 0; r < 6; r++) lam[r] = a[r] - h[r];
      ok = chol_n(Sm, 6, kFastPivotGuard);
      if (ok) {
        chol_solve_n(Sm, 6, lam);
        for (int r = 0; r < 6; r++) fl.lam[r] = lam[r];
      }
      fl.ok[0] = ok;
    }
    wave_sync();
    if (fl.ok[0] && lane < nc) {
      const int c = lane;
      const double* Ac = fl.A[c];
      double t[3];
      for (int i = 0; i < 3; i++) {
        double s = fl.g[c][i];
        for (int r = 0; r < 6; r++) s += Ac[r * 3 + i] * fl.lam[r];
        t[i] = s;
      }
      for (int i = 0; i < 3; i++) {
        double s = 0;
        for (int j = 0; j < 3; j++) s += fl.Dinv[c][3 * i + j] * t[j];
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

__global__ __launch_bounds__(WAVE) void hs_rollout_kernel(const hs_topo* __restrict__ T, hs_run_args a) {
  __shared__ Smem sm;
  const int lane = threadIdx.x;
  const int b = blockIdx.x;
  if (b >= a.n_rollouts) return;
  const hs_gait_params g = a.params[b];
  const int n = T->n, nmj = T->nmj, nf = T->nf, cfg = T->cfg, nl = T->n_limbs;
  const bool ignore_reach = a.ignore_reach != 0;

  STAMP(0);
  gait_setup(T, g, a.n_t, sm, lane);
  STAMP(1);

  // initial window: samples k0 .. k0+4, lane = (sample, limb)
  {
    int sl = lane / nl, L = lane % nl;
    if (sl < NS) {
      int i = a.k0 + sl;
      kin_sample(T, g, sm.st, i, L, ignore_reach, sm.s[i % NS]);
    }
  }
  wave_sync();
  STAMP(2);

  double work = (a.accumulate && a.work_cot) ? a.work_cot[2 * (size_t)b] : 0.0;
  for (int h = 0; h < a.horizon; h++) {
    const int i = a.k0 + h + 2;
    if (h > 0) {
      if (lane < nl) kin_sample(T, g, sm.st, i + 2, lane, ignore_reach, sm.s[(i + 2) % NS]);
      wave_sync();
    }
    const int s0 = i % NS;
    const SampleL& S = sm.s[s0];
    STAMP(3);
    dynamics(T, sm, (i - 2) % NS, (i - 1) % NS, s0, (i + 1) % NS, (i + 2) % NS, lane);
    STAMP(4);
    particular(T, sm, S, lane);
    STAMP(5);
    int nc = 0;
    for (int fi = 0; fi < nf; fi++) {
      if (S.contact[fi]) {
        if (lane == 0) sm.sv.cfoot[nc] = fi;
        nc++;
      }
    }
    wave_sync();
    int k = 3 * nc;
    uint32_t flags = 0;
    STAMP(6);
    if (fast_solve(T, sm.sv, sm.sv.fl, S, nc, lane)) {
      if (nc == 0) flags |= HS_FLAG_NO_CONTACT;
      if (nc == 1) flags |= HS_FLAG_FULL_RANK;
    } else {
      k = build_grams(T, sm, S, lane);
      flags = contact_solve(sm.sv, k, lane) | HS_FLAG_GENERAL;
    }
    STAMP(7);

    // S4: x = x_part + N y for the hinge torque rows, motor torques (periodic.cpp:328-343)
    if (lane < nmj) {
      int h_id = T->hinge_ids[lane];
      int fi = T->node[h_id].limb_below;
      int cc = -1;
      for (int c = 0; c < k / 3; c++) if (sm.sv.cfoot[c] == fi) cc = c;
      double tq = 0.0;
      for (int r = 0; r < 3; r++) {
        double s = 0.0;
        if (cc >= 0) {
          double d[3];
          for (int rr = 0; rr < 3; rr++) d[rr] = S.jpos[h_id][rr] - S.fpos[fi][rr];
          for (int jj = 0; jj < 3; jj++) s = s + cross_e(d, jj, r) * sm.sv.y[3 * cc + jj];
        }
        double xr = sm.sv.x[3 * n + 3 * h_id + r] + s;
        tq = tq + S.jz[h_id][r] * xr;
      }
      sm.sv.tau[lane] = tq;
    }
    wave_sync();
    // contact forces z = -N_cont y (ftsolver.cpp:91, 276-284)
    if (a.cf && lane < 3 * nf) {
      int fi = lane / 3, j = lane % 3;
      double zv = -0.0;
      for (int c = 0; c < k / 3; c++) if (sm.sv.cfoot[c] == fi) zv = -(0.0 + (-1.0) * sm.sv.y[3 * c + j]);
      a.cf[((size_t)b * a.horizon + h) * 3 * nf + lane] = zv;
    }
    if (a.x) {  // full joint force/torque vector x += N y
      for (int rI = lane; rI < 6 * n; rI += WAVE) {
        int part = (rI < 3 * n) ? rI / 3 : (rI - 3 * n) / 3, comp = rI % 3;
        double s = 0.0;
        for (int c = 0; c < k / 3; c++) {
          int foot = T->footis[sm.sv.cfoot[c]];
          bool anc = false;
          for (int aa = foot; aa >= 0; aa = T->node[aa].parent) anc |= (aa == part);
          if (!anc) continue;
          if (rI < 3 * n) {
            s = s + (-1.0) * sm.sv.y[3 * c + comp];
          } else {
            const double* ref = (T->node[part].parent >= 0) ? S.jpos[part] : S.pos[part];
            double d[3];
            for (int rr = 0; rr < 3; rr++) d[rr] = ref[rr] - S.fpos[sm.sv.cfoot[c]][rr];
            for (int jj = 0; jj < 3; jj++) s = s + cross_e(d, jj, comp) * sm.sv.y[3 * c + jj];
          }
        }
        a.x[((size_t)b * a.horizon + h) * 6 * n + rI] = sm.sv.x[rI] + s;
      }
    }
    if (a.tau && lane < nmj) a.tau[((size_t)b * a.horizon + h) * nmj + lane] = sm.sv.tau[lane];
    if (a.q && lane < cfg) a.q[((size_t)b * a.horizon + h) * cfg + lane] = S.q[lane];
    // positive work over this step (compute_vel_traj + work_over_period)
    {
      const SampleL& Sp = sm.s[(i + 1) % NS];
      const SampleL& Sm = sm.s[(i - 1) % NS];
      double work_dt = 0;
      for (int jj = 0; jj < nmj; jj++) {
        double dd = Sp.q[6 + jj] - Sm.q[6 + jj];
        if (dd > kPi) dd -= 2 * kPi;
        else if (dd < -kPi) dd += 2 * kPi;
        double jvel = dd / (2 * sm.st.dt);
        double dw = sm.sv.tau[jj] * jvel;
        dw = (dw > 0) ? dw : 0;
        work_dt += dw;
      }
      work_dt *= sm.st.dt;
      work += work_dt;
      for (int jj = 0; jj < nmj; jj++) {
        double v = sm.sv.tau[jj];
        if (v != v) flags |= HS_FLAG_NAN;
      }
      for (int c = 0; c < 3 * (k / 3); c++) if (sm.sv.y[c] != sm.sv.y[c]) flags |= HS_FLAG_NAN;
      for (int L = 0; L < nl; L++) if (S.unreach[L]) flags |= HS_FLAG_UNREACH;
    }
    if (a.flags && lane == 0) a.flags[(size_t)b * a.horizon + h] = flags;
    wave_sync();
    STAMP(8);
  }
  if (lane == 0) {
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

int launch_rollouts(const hs_topo* d_topo, const hs_topo& h_topo, const hs_run_args& a) {
  (void)h_topo;
  if (a.n_rollouts <= 0) return 0;
  hipStream_t st = (hipStream_t)a.stream;
  hipLaunchKernelGGL(hs_rollout_kernel, dim3(a.n_rollouts), dim3(WAVE), 0, st, d_topo, a);
  return (int)hipGetLastError();
}

}  // namespace hs
