// hs_sim.hip -- the reference's closed-loop simulation step on gfx950: position
// control -> motor torques -> plane collisions -> ODE QuickStep (projected
// Gauss-Seidel / SOR-LCP), for a batch of independent robots.
//
// One rollout per wavefront (a 64-thread workgroup); the whole ODE world of the
// rollout lives in LDS for all n_steps steps of a launch (bodies, the constraint
// rows, the SOR state), so HBM sees only the controller tables and the outputs.
// Per step:
//   P  lane = motor: hinge angle / rate (dJointGetHingeAngle/Rate), PD torque
//      (player.cpp:388-432);
//   B  lane = body: dJointAddHingeTorque sums in motor order, collision with the
//      z = 0 plane (dCollideCapsulePlane / dCollideSpherePlane), world inverse
//      inertia, gyroscopic torque, gravity, v/h + M^-1 f;
//   R  lane = joint (hinges, fixed joints, then this step's contacts): getInfo2
//      rows at the offsets of ODE's island order (dxProcessIslands);
//   A  lane = row: rhs = c/h - J (v/h + M^-1 f), CFM/h, Ad = w / (J M^-1 J^T + cfm);
//   G  SOR_LCP sweeps. The row order is ODE's: identity, reshuffled by dRandInt
//      every 8 sweeps. Gauss-Seidel is sequential, but consecutive rows that touch
//      disjoint bodies commute exactly (each reads and writes only its bodies'
//      constraint accelerations fc), so after each reshuffle the order is cut into
//      maximal runs of body-disjoint rows and a run is solved by one lane per row:
//      the sequential semantics (and ODE's per-row operation order) are kept;
//   U  lane = body: velocity update and dxStepBody.
// M^-1 J^T (ODE's iMJ) and the Ad-scaled J are recomputed from J where they are
// used (same single roundings as ODE's stored copies), which keeps the row storage
// at one J: LDS per hexapod rollout ~ 35 KB, 4 rollouts per CU.
//
// Every formula follows oracle/hs_oracle_sim.cpp (the CPU restatement, test
// infrastructure) in the same operation order, and this file is compiled
// with -ffp-contract=off (hslabs_amd/build.py) like the oracle and the
// reference's x86-64 build: a contact exists when a capsule end's depth is
// >= 0, and a stance foot planned at z = rcap sits within rounding of that
// threshold, so a fused multiply-add would flip contact sets against the CPU
// restatement. The remaining differences are the device atan2 (hinge angle)
// versus glibc.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hs_internal.h"
#include "hs_math.h"
#include "hs_ode.h"

namespace {

using namespace hsode;
constexpr int WAVE = 64;

__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

enum { ROW_BILATERAL = 0, ROW_NORMAL = 1, ROW_FRICTION = 2 };

// Diagnostic build (-DHS_SIM_STAMPS, tools/sim_stamps.py): shader-clock cycles per phase,
// summed over the steps of a launch, per wavefront.
#ifdef HS_SIM_STAMPS
__device__ unsigned long long g_sim_stamps[4096][16];
#define SIM_ACC(slot)                                                                 \
  do {                                                                                \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime();                     \
    if (threadIdx.x == 0 && blockIdx.x < 4096) g_sim_stamps[blockIdx.x][slot] += now_ - t_last; \
    t_last = now_;                                                                    \
  } while (0)
#else
#define SIM_ACC(slot) do {} while (0)
#endif

// the run's parameters in the kernel's precision (k1, k2 as player.cpp:393-394 forms them)
template <class real>
struct SimP {
  real dt, h1, k, k1, k2, sor_w, erp, cfm, gravity, bounce, bounce_vel, soft_cfm, mu;
  int iterations;
  __device__ explicit SimP(const hs_sim_params& p)
      : dt((real)p.dt), h1(real(1) / (real)p.dt), k((real)p.k), k1(-(real)p.k),
        k2(real(-2) * sqrt((real)p.k)), sor_w((real)p.sor_w), erp((real)p.erp), cfm((real)p.cfm),
        gravity((real)p.gravity), bounce((real)p.bounce), bounce_vel((real)p.bounce_vel),
        soft_cfm((real)p.soft_cfm), mu((real)p.mu), iterations(p.iterations) {}
};

template <int NM, int MM, class Real>
struct SimL {
  static_assert(MM < 256, "row ids, positions and levels are stored in bytes");
  using real = Real;
  // bodies (part ids index everything; ODE's island numbering does not change any arithmetic)
  // (no rotation matrices: R = dQtoR(q) is formed where it is read, from the same q)
  real pos[NM][3], q[NM][4], lvel[NM][3], avel[NM][3], tacc[NM][3];
  real invI[NM][9];      // world inverse inertia, 3x3 row-major
  real invm[NM];         // 1 / mass, kept on chip: the SOR rows read it for every update
  real fc[NM][6];        // v/h + M^-1 f while the rows are built (ODE's tmp1), then SOR's fc
  // constraint rows
  real J[MM][9];         // Jacobian rows, unscaled, as J1l | J1a | J2a: every two-body row here has
                           // J2l = -J1l (ball, fixed and hinge-axis rows), and contacts have no body2
  real rhs[MM];          // c, then rhs, then rhs * Ad
  real cfm[MM];          // cfm, then cfm / h, then Ad * cfm
  real Ad[MM];
  real lambda[MM];
  int8_t rb1[MM], rb2[MM], rtype[MM];
  // LDS shared by lifetime: the step's setup scratch (torques, contact points) is dead once the
  // rows are built, the sweep scheduling exists only during the sweeps (row ids, positions and
  // levels are < MM <= 216 and fit a byte)
  union {
    struct {
      real cpos[NM][3], cdepth[NM];
      real tau[NM];
    };
    struct {
      uint8_t order[MM];     // row at each sweep position (ODE's order)
      uint8_t swp[MM];       // Fisher-Yates swap targets s_i of a reshuffle
      uint8_t sched[MM];     // rows grouped by level
      uint8_t lv[MM];        // level of each position
      uint16_t run_se[MM];   // levels: start in sched | length << 8
      union {
        uint64_t bmask[NM][4];  // positions touching each body (dead once the levels are known)
        int32_t cnt[MM];        // rows per level
      };
    };
  };
  int16_t joff[HS_SIM_JMAX], coff[NM];
  int8_t contact[NM];
  int32_t m, nc, nruns;
  uint32_t seed;
};

// hinge.cpp getHingeAngle (body1 = part, body2 = parent; no dJOINT_REVERSE)
template <class L>
__device__ inline typename L::real hinge_angle(const L& s, const hs_simjoint_t<typename L::real>& J) {
  using real = typename L::real;
  real qq[4], qr[4];
  qmul1(qq, s.q[J.b1], s.q[J.b2]);
  qmul2(qr, qq, J.qrel);
  real cost2 = qr[0];
  real sint2 = sqrt(qr[1] * qr[1] + qr[2] * qr[2] + qr[3] * qr[3]);
  real theta = (dot3(qr + 1, J.axis1) >= 0) ? (2 * atan2(sint2, cost2)) : (2 * atan2(sint2, -cost2));
  if (theta > real(M_PI)) theta -= real(2 * M_PI);
  return -theta;
}

template <class L>
__device__ inline void put_row(L& s, int r, const typename L::real* j12) {
#pragma unroll
  for (int j = 0; j < 6; j++) s.J[r][j] = j12[j];
#pragma unroll
  for (int j = 0; j < 3; j++) s.J[r][6 + j] = j12[9 + j];
}
template <class L>
__device__ inline void get_row(const L& s, int r, typename L::real* j12) {
#pragma unroll
  for (int j = 0; j < 6; j++) j12[j] = s.J[r][j];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    j12[6 + j] = -j12[j];
    j12[9 + j] = s.J[r][6 + j];
  }
}

template <class L>
__device__ inline void set_ball(L& s, const hs_simjoint_t<typename L::real>& J, typename L::real k, int r0,
                                const typename L::real* R1, const typename L::real* R2) {
  using real = typename L::real;
  real a1[3], a2[3];
  mul0_331(a1, R1, J.anchor1);
  mul0_331(a2, R2, J.anchor2);
  // J1l = I, J1a = -[a1]x, J2l = -I, J2a = [a2]x
  const real rows[3][12] = {
      {1, 0, 0, 0, a1[2], -a1[1], -1, 0, 0, 0, -a2[2], a2[1]},
      {0, 1, 0, -a1[2], 0, a1[0], 0, -1, 0, a2[2], 0, -a2[0]},
      {0, 0, 1, a1[1], -a1[0], 0, 0, 0, -1, -a2[1], a2[0], 0}};
  for (int r = 0; r < 3; r++) {
    put_row(s, r0 + r, rows[r]);
    s.rhs[r0 + r] = k * (a2[r] + s.pos[J.b2][r] - a1[r] - s.pos[J.b1][r]);
  }
}

template <class L>
__device__ inline void hinge_rows(L& s, const hs_simjoint_t<typename L::real>& J, typename L::real fps, typename L::real erp, typename L::real cfm, int r0) {
  using real = typename L::real;
  const real k = fps * erp;
  real R1[12], R2[12];
  q_to_R(s.q[J.b1], R1);
  q_to_R(s.q[J.b2], R2);
  set_ball(s, J, k, r0, R1, R2);
  real ax1[3], p[3], qv[3], ax2[3], b[3];
  mul0_331(ax1, R1, J.axis1);
  plane_space(ax1, p, qv);
  mul0_331(ax2, R2, J.axis2);
  cross3(b, ax1, ax2);
  const real r3[12] = {0, 0, 0, p[0], p[1], p[2], 0, 0, 0, -p[0], -p[1], -p[2]};
  const real r4[12] = {0, 0, 0, qv[0], qv[1], qv[2], 0, 0, 0, -qv[0], -qv[1], -qv[2]};
  put_row(s, r0 + 3, r3);
  put_row(s, r0 + 4, r4);
  s.rhs[r0 + 3] = k * dot3(b, p);
  s.rhs[r0 + 4] = k * dot3(b, qv);
  for (int r = 0; r < 5; r++) {
    s.cfm[r0 + r] = cfm;
    s.rtype[r0 + r] = ROW_BILATERAL;
    s.rb1[r0 + r] = (int8_t)J.b1;
    s.rb2[r0 + r] = (int8_t)J.b2;
  }
}

template <class L>
__device__ inline void fixed_rows(L& s, const hs_simjoint_t<typename L::real>& J, typename L::real fps, typename L::real erp, typename L::real cfm, int r0) {
  using real = typename L::real;
  const real k = fps * erp;
  // three linear rows: J1l = I, J1a = [ofs]x, J2l = -I
  real ofs[3], R1[12];
  q_to_R(s.q[J.b1], R1);
  mul0_331(ofs, R1, J.offset);
  const real rows[3][12] = {
      {1, 0, 0, 0, -ofs[2], ofs[1], -1, 0, 0, 0, 0, 0},
      {0, 1, 0, ofs[2], 0, -ofs[0], 0, -1, 0, 0, 0, 0},
      {0, 0, 1, -ofs[1], ofs[0], 0, 0, 0, -1, 0, 0, 0}};
  for (int r = 0; r < 3; r++) {
    put_row(s, r0 + r, rows[r]);
    s.rhs[r0 + r] = k * (s.pos[J.b2][r] - s.pos[J.b1][r] + ofs[r]);
  }
  // setFixedOrientation: rows 3..5, J1a = I, J2a = -I
  real qq[4], qerr[4], e[3];
  qmul1(qq, s.q[J.b1], s.q[J.b2]);
  qmul2(qerr, qq, J.qrel);
  if (qerr[0] < 0) { qerr[1] = -qerr[1]; qerr[2] = -qerr[2]; qerr[3] = -qerr[3]; }
  mul0_331(e, R1, qerr + 1);
  for (int r = 0; r < 3; r++) {
    real row[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    row[3 + r] = 1;
    row[9 + r] = -1;
    put_row(s, r0 + 3 + r, row);
    s.rhs[r0 + 3 + r] = 2 * k * e[r];
  }
  for (int r = 0; r < 6; r++) {
    s.cfm[r0 + r] = cfm;
    s.rtype[r0 + r] = ROW_BILATERAL;
    s.rb1[r0 + r] = (int8_t)J.b1;
    s.rb2[r0 + r] = (int8_t)J.b2;
  }
}

// contact.cpp getInfo2: body1 = the geom's body, body2 = the environment, normal (0,0,1)
template <class L>
__device__ inline void contact_rows(L& s, int b, const SimP<typename L::real>& P, typename L::real fps, int r0) {
  using real = typename L::real;
  const real normal[3] = {0, 0, 1};
  real c1[3];
  for (int i = 0; i < 3; i++) c1[i] = s.cpos[b][i] - s.pos[b][i];
  real jn[3], t1[3], t2[3], j1[3], j2[3];
  cross3(jn, c1, normal);
  plane_space(normal, t1, t2);
  cross3(j1, c1, t1);
  cross3(j2, c1, t2);
  for (int j = 0; j < 3; j++) {
    s.J[r0][j] = normal[j]; s.J[r0][3 + j] = jn[j]; s.J[r0][6 + j] = 0;
    s.J[r0 + 1][j] = t1[j]; s.J[r0 + 1][3 + j] = j1[j]; s.J[r0 + 1][6 + j] = 0;
    s.J[r0 + 2][j] = t2[j]; s.J[r0 + 2][3 + j] = j2[j]; s.J[r0 + 2][6 + j] = 0;
  }
  const real k = fps * P.erp;
  real depth = s.cdepth[b];
  if (depth < 0) depth = 0;
  real c = k * depth;
  real outgoing = dot3(normal, s.lvel[b]) + dot3(jn, s.avel[b]);
  if (P.bounce_vel >= 0 && (-outgoing) > P.bounce_vel) {
    real newc = -P.bounce * outgoing;
    if (newc > c) c = newc;
  }
  s.rhs[r0] = c;
  s.rhs[r0 + 1] = 0;
  s.rhs[r0 + 2] = 0;
  s.cfm[r0] = P.soft_cfm;
  s.cfm[r0 + 1] = P.cfm;
  s.cfm[r0 + 2] = P.cfm;
  s.rtype[r0] = ROW_NORMAL;
  s.rtype[r0 + 1] = ROW_FRICTION;
  s.rtype[r0 + 2] = ROW_FRICTION;
  for (int r = 0; r < 3; r++) {
    s.rb1[r0 + r] = (int8_t)b;
    s.rb2[r0 + r] = -1;
  }
}

// iMJ block of one body: linear invMass * J, angular invI * J (compute_invM_JT)
template <class L>
__device__ inline void imj_block(const L& s, const hs_simtopo_t<typename L::real>& T, int b, const typename L::real* Jb, typename L::real* out) {
  using real = typename L::real;
  const real k1 = s.invm[b];
  for (int j = 0; j < 3; j++) out[j] = k1 * Jb[j];
  mul0_33(out + 3, s.invI[b], Jb + 3);
}

__device__ inline double swap_pair(double v) {  // value of the other lane of the pair (DPP quad_perm 1,0,3,2)
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0xB1, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0xB1, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ inline float swap_pair(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
}

// What one lane of a row's lane pair needs of the row: its body block of the scaled J and of
// iMJ (half 0: body1 columns 0..5, half 1: body2 columns 6..11); the even lane also the row's
// scalars. Nothing here changes during the sweeps, so it is loaded one run ahead of use.
template <class real>
struct RowData {
  real Js[6], iM[6], rhs, adcfm;
  int body, b2, rt;
};

template <class L>
__device__ inline RowData<typename L::real> load_row(const L& s, int row, int half) {
  using real = typename L::real;
  RowData<real> r;
  const int rr = row < 0 ? 0 : row;
  const int b1 = s.rb1[rr], b2 = s.rb2[rr];
  r.body = row < 0 ? -1 : (half ? b2 : b1);
  r.b2 = b2;
  r.rt = s.rtype[rr];
  const int bb = r.body < 0 ? 0 : r.body;
  real Jb[6];
#pragma unroll
  for (int j = 0; j < 3; j++) {
    const real l = s.J[rr][j];
    Jb[j] = half ? -l : l;                 // J2l = -J1l
    Jb[3 + j] = s.J[rr][3 + 3 * half + j];  // J1a | J2a
  }
  const real ad = s.Ad[rr];
#pragma unroll
  for (int j = 0; j < 6; j++) r.Js[j] = Jb[j] * ad;  // SOR_LCP: J *= Ad
  // compute_invM_JT: invMass J (linear), invI J (angular)
  const real k1 = s.invm[bb];
  for (int j = 0; j < 3; j++) r.iM[j] = k1 * Jb[j];
  mul0_33(r.iM + 3, s.invI[bb], Jb + 3);
  r.rhs = s.rhs[rr];
  r.adcfm = s.cfm[rr];
  return r;
}

// One SOR row update (SOR_LCP inner loop) on a lane pair, in ODE's order of operations:
// delta = (b - lambda Ad) - sum_body1 - sum_body2, each sum f0 J0 + f1 J1 + ... left to right;
// the two sums are computed by the two lanes and exchanged. The multiply-adds of the sums and
// of the fc update are fused here (explicit fma; the file is otherwise unfused), which moves
// lambda by ulps against the unfused restatement and never decides a contact.
template <class L>
__device__ inline void sor_pair(L& s, const RowData<typename L::real>& r, int row, int half, typename L::real mu) {
  using real = typename L::real;
  const bool act = row >= 0 && r.body >= 0;
  const real* f = s.fc[act ? r.body : 0];
  const real f0 = f[0], f1 = f[1], f2 = f[2], f3 = f[3], f4 = f[4], f5 = f[5];
  const real lam = s.lambda[row < 0 ? 0 : row];
  real sum = f0 * r.Js[0];
  sum = fma(f1, r.Js[1], sum);
  sum = fma(f2, r.Js[2], sum);
  sum = fma(f3, r.Js[3], sum);
  sum = fma(f4, r.Js[4], sum);
  sum = fma(f5, r.Js[5], sum);
  if (!act) sum = 0;
  const real other = swap_pair(sum);  // the body2 sum, on the even lane
  real delta = r.rhs - lam * r.adcfm;
  delta -= sum;
  delta -= (r.b2 >= 0) ? other : real(0);  // x - 0 == x
  const real lo = (r.rt == ROW_BILATERAL) ? real(-INFINITY) : (r.rt == ROW_NORMAL ? real(0) : -mu);
  const real hi = (r.rt == ROW_BILATERAL) ? real(INFINITY) : mu;
  const real nl = lam + delta;
  const bool below = nl < lo, above = !below && nl > hi;
  const real newl = below ? lo : (above ? hi : nl);
  delta = (below || above) ? newl - lam : delta;
  if (row >= 0 && half == 0) s.lambda[row] = newl;
  const real d2 = swap_pair(delta);
  if (half) delta = d2;
  if (act) {
    real* g = s.fc[r.body];
    g[0] = fma(delta, r.iM[0], f0);
    g[1] = fma(delta, r.iM[1], f1);
    g[2] = fma(delta, r.iM[2], f2);
    g[3] = fma(delta, r.iM[3], f3);
    g[4] = fma(delta, r.iM[4], f4);
    g[5] = fma(delta, r.iM[5], f5);
  }
}

template <class L>
__device__ inline int run_row(const L& s, int se, int pair) {  // row of a lane pair in a level, -1 = idle
  return pair < (se >> 8) ? s.sched[(se & 0xFF) + pair] : -1;
}

// MINW: waves per SIMD the register budget is built for. 1 leaves every kernel its 256 VGPRs
// (2 waves/SIMD); the fp32 kernel also exists at 3 (168 VGPRs, 32 B of spills), which fits 11
// instead of 8 rollouts per CU but runs each ~20 % slower (launch_class picks per batch).
template <int NM, int MM, class Real, int MINW>
__global__ __launch_bounds__(WAVE, MINW) void hs_sim_kernel(const hs_topo* __restrict__ T0,
                                                         const hs_simtopo_t<Real>* __restrict__ S, hs_sim_args a) {
  using real = Real;
  __shared__ SimL<NM, MM, Real> s;
  const int lane = threadIdx.x;
  const int b = blockIdx.x;
  if (b >= a.n_rollouts) return;
  const hs_simtopo_t<Real>& T = *S;
  const int n = T.n, nmj = T.nmj, nj = T.nj, cfg = T0->cfg;
  const SimP<real> P(a.params);
  const real h = P.dt, h1 = P.h1;
  // the ABI's arrays are double*; in the single-precision build they hold floats
  const real* q_tab = reinterpret_cast<const real*>(a.q_tab);
  const real* dq_tab = reinterpret_cast<const real*>(a.dq_tab);
  const real* tau_tab = reinterpret_cast<const real*>(a.tau_tab);
  real* o_tau = reinterpret_cast<real*>(a.tau_cmd);
  real* o_q = reinterpret_cast<real*>(a.q_meas);
  real* o_torso = reinterpret_cast<real*>(a.torso);
  real* o_fn = reinterpret_cast<real*>(a.normal_force);
#ifdef HS_SIM_STAMPS
  unsigned long long t_last = __builtin_amdgcn_s_memtime();
#endif
  real* gbody = reinterpret_cast<real*>(a.body) + (size_t)b * n * HS_SIM_BODY;
  // load the world
  for (int e = lane; e < n * HS_SIM_BODY; e += WAVE) {
    const int p = e / HS_SIM_BODY, c = e % HS_SIM_BODY;
    const real v = gbody[e];
    if (c < 3) s.pos[p][c] = v;
    else if (c < 7) s.q[p][c - 3] = v;
    else if (c < 10) s.lvel[p][c - 7] = v;
    else s.avel[p][c - 10] = v;
  }
  if (lane == 0) s.seed = a.seed[b];
  int tsi = a.tsi[b];
  wave_sync();
  if (lane < n) s.invm[lane] = real(1) / T.mass[lane];
  wave_sync();

  SIM_ACC(0);
  for (int step = 0; step < a.n_steps; step++) {
    const size_t orow = (size_t)b * a.n_steps + step;
    // ---- P: position control (set_position_control_torques, player.cpp:388-409)
    if (lane < nmj) {
      const hs_simjoint_t<real>& J = T.joint[T.motor_joint[lane]];
      const real qm = hinge_angle(s, J);
      real tq = 0;
      if (P.k > 0) {
        real ax[3], R1[12];
        q_to_R(s.q[J.b1], R1);
        mul0_331(ax, R1, J.axis1);
        const real rate = dot3(ax, s.avel[J.b1]) - dot3(ax, s.avel[J.b2]);
        const int t = tsi % a.n_t;
        const int hrow = (t + a.n_t - 2) % a.n_t;
        const size_t tb = (size_t)b * a.n_t + hrow;
        real a1 = qm - q_tab[tb * cfg + 6 + lane];
        real a2 = rate - dq_tab[tb * cfg + 6 + lane];
        if (a1 > real(M_PI)) a1 -= real(2 * M_PI);  // arrayops::modulus (core.cpp:122-131)
        else if (a1 <= -real(M_PI)) a1 += real(2 * M_PI);
        a1 *= P.k1;
        a2 *= P.k2;
        a1 += a2;
        tq = tau_tab[tb * nmj + lane] + a1;
      }
      s.tau[lane] = tq;
      if (o_q) o_q[orow * nmj + lane] = qm;
      if (o_tau) o_tau[orow * nmj + lane] = tq;
    }
    wave_sync();
    SIM_ACC(1);
    // ---- B: per body accumulators, collision, inertia, v/h + M^-1 f
    if (lane < n) {
      const int p = lane;
      real tq[3] = {0, 0, 0};
      if (P.k > 0) {
        for (int c = 0; c < T.tq_n[p]; c++) {  // dJointAddHingeTorque in motor order
          const int j = T.tq_motor[p][c];
          const hs_simjoint_t<real>& J = T.joint[T.motor_joint[j]];
          real ax[3], R1[12];
          q_to_R(s.q[J.b1], R1);
          mul0_331(ax, R1, J.axis1);
          for (int i = 0; i < 3; i++) ax[i] *= s.tau[j];
          if (T.tq_sign[p][c] > 0)
            for (int i = 0; i < 3; i++) tq[i] += ax[i];
          else
            for (int i = 0; i < 3; i++) tq[i] += -ax[i];
        }
      }
      // collision with the plane (0,0,1,0)
      bool hit = false;
      real R[12];
      q_to_R(s.q[p], R);
      if (T.gtype[p] == HS_GEOM_CAPSULE) {
        const real sign = (R[10] > 0) ? real(-1) : real(1);  // dCalcVectorDot3_14(plane normal, R + 2)
        real pp[3];
        pp[0] = s.pos[p][0] + R[2] * T.glen[p] * real(0.5) * sign;
        pp[1] = s.pos[p][1] + R[6] * T.glen[p] * real(0.5) * sign;
        pp[2] = s.pos[p][2] + R[10] * T.glen[p] * real(0.5) * sign;
        const real depth = 0 - (pp[0] * real(0) + pp[1] * real(0) + pp[2] * real(1)) + T.gr[p];
        if (depth >= 0) {
          hit = true;
          s.cpos[p][0] = pp[0] - real(0) * T.gr[p];
          s.cpos[p][1] = pp[1] - real(0) * T.gr[p];
          s.cpos[p][2] = pp[2] - real(1) * T.gr[p];
          s.cdepth[p] = depth;
        }
      } else if (T.gtype[p] == HS_GEOM_SPHERE) {
        const real depth = 0 - (s.pos[p][0] * real(0) + s.pos[p][1] * real(0) + s.pos[p][2] * real(1)) + T.gr[p];
        if (depth >= 0) {
          hit = true;
          s.cpos[p][0] = s.pos[p][0] - real(0) * T.gr[p];
          s.cpos[p][1] = s.pos[p][1] - real(0) * T.gr[p];
          s.cpos[p][2] = s.pos[p][2] - real(1) * T.gr[p];
          s.cdepth[p] = depth;
        }
      }
      s.contact[p] = hit ? 1 : 0;
      // world inverse inertia R invI_b R^T, gyroscopic torque, gravity (dxQuickStepper)
      real Ib[12], iIb[12], tmp[12], I[12];
      for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) { Ib[r * 4 + c] = T.inertia[p][r * 3 + c]; iIb[r * 4 + c] = T.inv_inertia[p][r * 3 + c]; }
        Ib[r * 4 + 3] = iIb[r * 4 + 3] = 0;
      }
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) tmp[r * 4 + c] = dot3(iIb + r * 4, R + c * 4);
      for (int r = 0; r < 3; r++) {
        for (int c = 0; c < 3; c++) s.invI[p][r * 3 + c] = dot3_14(R + r * 4, tmp + c);
      }
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) tmp[r * 4 + c] = dot3(Ib + r * 4, R + c * 4);
      for (int r = 0; r < 3; r++)
        for (int c = 0; c < 3; c++) I[r * 4 + c] = dot3_14(R + r * 4, tmp + c);
      real t3[3];
      const real* w = s.avel[p];
      mul0_331(t3, I, w);
      tq[0] -= w[1] * t3[2] - w[2] * t3[1];
      tq[1] -= w[2] * t3[0] - w[0] * t3[2];
      tq[2] -= w[0] * t3[1] - w[1] * t3[0];
      real fa[3] = {0, 0, 0};
      if (P.gravity != 0) fa[2] += T.mass[p] * (-P.gravity);
      const real im = s.invm[p];
      for (int i = 0; i < 3; i++) {
        s.tacc[p][i] = tq[i];
        s.fc[p][i] = fa[i] * im + s.lvel[p][i] * h1;  // tmp1
      }
      real it[3];
      mul0_33(it, s.invI[p], tq);
      for (int i = 0; i < 3; i++) s.fc[p][3 + i] = it[i] + w[i] * h1;
    }
    wave_sync();
    SIM_ACC(2);
    // ---- row offsets in island order (dxProcessIslands: per visited body, its contact
    // first -- the newest joint in its list -- then the static joints first reached from it)
    if (lane == 0) {
      int off = 0, nc = 0;
      for (int v = 0; v < n; v++) {
        const int bv = T.border[v];
        if (s.contact[bv]) { s.coff[bv] = (int16_t)off; off += (P.mu > 0) ? 3 : 1; nc++; }
        for (int k = T.jseq_start[v]; k < T.jseq_start[v + 1]; k++) {
          const int jid = T.jseq[k];
          s.joff[jid] = (int16_t)off;
          off += (T.joint[jid].type == HS_SJ_HINGE) ? 5 : 6;
        }
      }
      s.m = off;
      s.nc = nc;
    }
    wave_sync();
    SIM_ACC(3);
    const int m = s.m;
    // ---- R: getInfo2 of every joint
    if (lane < nj) {
      const hs_simjoint_t<real>& J = T.joint[lane];
      if (J.type == HS_SJ_HINGE) hinge_rows(s, J, h1, P.erp, P.cfm, s.joff[lane]);
      else fixed_rows(s, J, h1, P.erp, P.cfm, s.joff[lane]);
    } else if (lane < nj + n) {
      const int p = lane - nj;
      if (s.contact[p]) contact_rows(s, p, P, h1, s.coff[p]);
    }
    wave_sync();
    SIM_ACC(4);
    // ---- A: rhs, CFM / h, Ad (SOR_LCP prologue)
    for (int i = lane; i < m; i += WAVE) {
      const int b1 = s.rb1[i], b2 = s.rb2[i];
      real Jr[12];
      get_row(s, i, Jr);
      real sum = 0;
      for (int j = 0; j < 6; j++) sum += Jr[j] * s.fc[b1][j];  // fc holds tmp1 here
      if (b2 >= 0)
        for (int j = 0; j < 6; j++) sum += Jr[6 + j] * s.fc[b2][j];
      const real rhs = s.rhs[i] * h1 - sum;
      const real cfm = s.cfm[i] * h1;
      real iM[6], dsum = 0;
      imj_block(s, T, b1, Jr, iM);
      for (int j = 0; j < 6; j++) dsum += iM[j] * Jr[j];
      if (b2 >= 0) {
        imj_block(s, T, b2, Jr + 6, iM);
        for (int j = 0; j < 6; j++) dsum += iM[j] * Jr[6 + j];
      }
      const real ad = P.sor_w / (dsum + cfm);
      s.Ad[i] = ad;
      s.rhs[i] = rhs * ad;
      s.cfm[i] = ad * cfm;
      s.lambda[i] = 0;
    }
    wave_sync();
    for (int e = lane; e < n * 6; e += WAVE) s.fc[e / 6][e % 6] = 0;  // SOR_LCP: fc = 0 (no warm start)
    wave_sync();
    SIM_ACC(5);
    // ---- G: SOR sweeps
    {
      const int pair = lane >> 1, half = lane & 1;
      for (int i = lane; i < m; i += WAVE) s.order[i] = (uint8_t)i;  // findex all -1: identity order
      uint32_t seed = __builtin_amdgcn_readfirstlane(s.seed);
      for (int it0 = 0; it0 < P.iterations; it0 += 8) {
        // RANDOMLY_REORDER_CONSTRAINTS: Fisher-Yates with dRandInt over the current order, i.e.
        // order' = order o t_1 o ... o t_{m-1} with t_i the transposition (i, s_i). The draws s_i are
        // independent given the jump-ahead tables; the composition is traced backwards from every
        // position at once (lane-parallel), so no swap chain runs through LDS.
        const int nblk = (m + 63) >> 6;  // position blocks in use (uniform)
        int src[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int p = lane + 64 * k;
          if (p >= 1 && p < m) s.swp[p] = (uint8_t)rand_int_from(T.lcg_a[p] * seed + T.lcg_c[p], p + 1);
          src[k] = p;
        }
        if (m > 1) seed = T.lcg_a[m - 1] * seed + T.lcg_c[m - 1];
        wave_sync();
        // s_i are read as LDS broadcasts (VGPR operands: no v_readlane -> SGPR hazards)
#pragma unroll 4
        for (int i = m - 1; i >= 1; i--) {
          const int si = s.swp[i];
#pragma unroll
          for (int k = 0; k < 4; k++)
            if (k < nblk) src[k] = (src[k] == i) ? si : ((src[k] == si) ? i : src[k]);
        }
        SIM_ACC(11);
        int ordr[4];
#pragma unroll
        for (int k = 0; k < 4; k++) ordr[k] = (lane + 64 * k < m) ? s.order[src[k]] : 0;
        wave_sync();
        // Dependency levels. Rows sharing a body must keep ODE's order; rows that share none
        // commute exactly. level(p) = 1 + the level of the latest earlier position sharing a body
        // with p, so one level is a set of body-disjoint rows whose earlier neighbours all sit in
        // lower levels: solving the levels in turn, each in parallel, is Gauss-Seidel in ODE's order.
        int pb1[4], pb2[4], pv1[4], pv2[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const int p = lane + 64 * k;
          if (p < m) s.order[p] = (uint8_t)ordr[k];
          pb1[k] = (p < m) ? s.rb1[ordr[k]] : -2;
          pb2[k] = (p < m) ? s.rb2[ordr[k]] : -2;
        }
        // positions touching each body, as 4 x 64-bit masks
        for (int bd = 0; bd < n; bd++) {
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const uint64_t bm = (k < nblk) ? __ballot(pb1[k] == bd || pb2[k] == bd) : 0ull;
            if (lane == k) s.bmask[bd][k] = bm;
          }
        }
        wave_sync();
        // latest earlier position touching the same body (-1: none)
#pragma unroll
        for (int k = 0; k < 4; k++) {
          pv1[k] = pv2[k] = -1;
          for (int e = 0; e < 2; e++) {
            const int bd = e ? pb2[k] : pb1[k];
            int pv = -1;
            if (bd >= 0) {
              const uint64_t below = (lane == 0) ? 0ull : (s.bmask[bd][k] & ((1ull << lane) - 1ull));
              if (below) pv = 64 * k + 63 - __clzll(below);
              else
                for (int kk = k - 1; kk >= 0; kk--) {
                  const uint64_t w = s.bmask[bd][kk];
                  if (w) { pv = 64 * kk + 63 - __clzll(w); break; }
                }
            }
            if (e) pv2[k] = pv; else pv1[k] = pv;
          }
        }
        SIM_ACC(12);
        // longest paths by relaxation (converges after the number of levels)
#pragma unroll
        for (int k = 0; k < 4; k++) if (lane + 64 * k < m) s.lv[lane + 64 * k] = 0;
        wave_sync();
        int lvr[4] = {0, 0, 0, 0};
        for (;;) {
          bool changed = false;
          int nl[4];
#pragma unroll
          for (int k = 0; k < 4; k++) {
            nl[k] = 0;
            if (k < nblk) {
              const int a1 = pv1[k] >= 0 ? s.lv[pv1[k]] + 1 : 0;
              const int a2 = pv2[k] >= 0 ? s.lv[pv2[k]] + 1 : 0;
              nl[k] = a1 > a2 ? a1 : a2;
              changed |= (lane + 64 * k < m) && nl[k] != lvr[k];
            }
          }
          wave_sync();
          if (!__any(changed)) break;
#pragma unroll
          for (int k = 0; k < 4; k++) {
            lvr[k] = nl[k];
            if (k < nblk && lane + 64 * k < m) s.lv[lane + 64 * k] = (uint8_t)nl[k];
          }
          wave_sync();
        }
        SIM_ACC(13);
        int nlev = 0;
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (lane + 64 * k < m) nlev = max(nlev, lvr[k] + 1);
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) nlev = max(nlev, __shfl_xor(nlev, off));
        // level sizes and ranks (any order inside a level: its rows are body-disjoint)
#pragma unroll
        for (int k = 0; k < 4; k++) if (lane + 64 * k < m) s.cnt[lane + 64 * k] = 0;
        wave_sync();
        int rank[4];
#pragma unroll
        for (int k = 0; k < 4; k++) rank[k] = (lane + 64 * k < m) ? atomicAdd(&s.cnt[lvr[k]], 1) : 0;
        wave_sync();
        {
          int base = 0;
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const int l = lane + 64 * k;
            const int size = (l < nlev) ? s.cnt[l] : 0;
            int incl = size;
#pragma unroll
            for (int off = 1; off < 64; off <<= 1) {
              const int up = __shfl_up(incl, off);
              if (lane >= off) incl += up;
            }
            if (l < nlev) s.run_se[l] = (uint16_t)((base + incl - size) | (size << 8));
            base += __shfl(incl, 63);
          }
          wave_sync();
#pragma unroll
          for (int k = 0; k < 4; k++) {
            const int p = lane + 64 * k;
            if (p < m) s.sched[(s.run_se[lvr[k]] & 0xFF) + rank[k]] = (uint8_t)ordr[k];
          }
          if (lane == 0) s.nruns = nlev;
        }
        wave_sync();
        SIM_ACC(6);
        // sweeps it0 .. it0+7 over the same runs, software-pipelined: while run t is solved, the
        // row data of run t+1, the rows of run t+2 and the bounds of run t+3 are loaded
        const int nb = __builtin_amdgcn_readfirstlane(s.nruns);
        const int total = min(8, P.iterations - it0) * nb;
        int k2 = (2 % nb), k3 = (3 % nb);
        int se2 = __builtin_amdgcn_readfirstlane(s.run_se[k2]);
        int row0 = run_row(s, __builtin_amdgcn_readfirstlane(s.run_se[0]), pair);
        int row1 = run_row(s, __builtin_amdgcn_readfirstlane(s.run_se[1 % nb]), pair);
        RowData d0 = load_row(s, row0, half);
        for (int t = 0; t < total; t++) {
          const RowData d1 = load_row(s, row1, half);
          const int row2 = run_row(s, se2, pair);
          const int se3 = __builtin_amdgcn_readfirstlane(s.run_se[k3]);
          sor_pair(s, d0, row0, half, P.mu);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
          d0 = d1;
          row0 = row1;
          row1 = row2;
          se2 = se3;
          k3 = (k3 + 1 == nb) ? 0 : k3 + 1;
        }
        wave_sync();
        SIM_ACC(7);
#ifdef HS_SIM_STAMPS
        if (lane == 0 && blockIdx.x < 4096) g_sim_stamps[blockIdx.x][9] += nb;
#endif
      }
      if (lane == 0) s.seed = seed;
    }
    // ---- U: velocities (constraint part, then external forces) and dxStepBody
    if (lane < n) {
      const int p = lane;
      for (int j = 0; j < 3; j++) s.lvel[p][j] += h * s.fc[p][j];
      for (int j = 0; j < 3; j++) s.avel[p][j] += h * s.fc[p][3 + j];
      const real hm = h * s.invm[p];
      real fa[3] = {0, 0, 0};  // facc: gravity only (the motors add torques)
      if (P.gravity != 0) fa[2] += T.mass[p] * (-P.gravity);
      real ta[3];
      for (int j = 0; j < 3; j++) {
        s.lvel[p][j] += hm * fa[j];
        ta[j] = s.tacc[p][j] * h;
      }
      real t3[3];
      mul0_33(t3, s.invI[p], ta);
      for (int j = 0; j < 3; j++) s.avel[p][j] += t3[j];
      for (int j = 0; j < 3; j++) s.pos[p][j] += h * s.lvel[p][j];
      const real* w = s.avel[p];
      real* qv = s.q[p];
      real dq[4];
      dq[0] = real(0.5) * (-w[0] * qv[1] - w[1] * qv[2] - w[2] * qv[3]);
      dq[1] = real(0.5) * (w[0] * qv[0] + w[1] * qv[3] - w[2] * qv[2]);
      dq[2] = real(0.5) * (-w[0] * qv[3] + w[1] * qv[0] + w[2] * qv[1]);
      dq[3] = real(0.5) * (w[0] * qv[2] - w[1] * qv[1] + w[2] * qv[0]);
      for (int j = 0; j < 4; j++) qv[j] += h * dq[j];
      normalize4(qv);
    }
    if (lane == 0) {
      if (a.n_contacts) a.n_contacts[orow] = s.nc;
      if (a.normal_force) {
        real fsum = 0;
        for (int v = 0; v < n; v++) {
          const int bv = T.border[v];
          if (s.contact[bv]) fsum += s.lambda[s.coff[bv]];
        }
        o_fn[orow] = fsum;
      }
    }
    wave_sync();
    if (o_torso && lane < 3) o_torso[orow * 3 + lane] = s.pos[0][lane];
    tsi++;
    SIM_ACC(8);
#ifdef HS_SIM_STAMPS
    if (lane == 0 && blockIdx.x < 4096) g_sim_stamps[blockIdx.x][10] += m;
#endif
  }
  // store the world
  for (int e = lane; e < n * HS_SIM_BODY; e += WAVE) {
    const int p = e / HS_SIM_BODY, c = e % HS_SIM_BODY;
    real v;
    if (c < 3) v = s.pos[p][c];
    else if (c < 7) v = s.q[p][c - 3];
    else if (c < 10) v = s.lvel[p][c - 7];
    else v = s.avel[p][c - 10];
    gbody[e] = v;
  }
  if (lane == 0) {
    a.seed[b] = s.seed;
    a.tsi[b] = tsi;
  }
}

// init_play_config + orient_odebodys: lane = part, A_ground by walking the chain from the root
// (each product in the reference's order: J_A_ground = A_parent J_A_parent, then * E(q) * A_pj_body).
// IO = the precision of the configuration and body arrays; the pose is built in double and
// rounded once into a float state for the single-precision simulation.
template <class IO>
__global__ __launch_bounds__(WAVE) void hs_sim_reset_kernel(const hs_topo* __restrict__ T, const hs_simtopo* __restrict__ S,
                                                             int32_t n_rollouts, const IO* __restrict__ config,
                                                             int32_t stride, IO* __restrict__ body) {
  using namespace hsd;
  const int b = blockIdx.x, p = threadIdx.x;
  if (b >= n_rollouts || p >= T->n) return;
  double cf[6 + HS_NMAX];
  for (int i = 0; i < T->cfg; i++) cf[i] = (double)config[(size_t)b * stride + i];
  int chain[HS_NMAX], len = 0;
  for (int a = p; a >= 0; a = T->node[a].parent) chain[len++] = a;
  A34 A;
  for (int i = 0; i < 12; i++) A.m[i] = (i % 4 == 0) ? 1.0 : 0.0;  // unity (columns 0..2 of I, zero translation)
  for (int k = len - 1; k >= 0; k--) {
    const hs_node& nd = T->node[chain[k]];
    if (nd.jtype == HS_J_FREE) {
      A34 JA = mul(A, load34(nd.J_A_parent));
      A = mul(mul(JA, free_joint(cf)), load34(nd.A_pj_body));
    } else if (nd.jtype == HS_J_HINGE) {
      A34 JA = mul(A, load34(nd.J_A_parent));
      A = mul(mul(JA, hinge_joint(cf[6 + nd.hinge])), load34(nd.A_pj_body));
    } else {
      A = mul(A, load34(nd.A_pj_body));
    }
  }
  A34 G = mul(A, load34(S->body_geom[p]));
  double Rin[12], q[4], R[12];
  for (int r = 0; r < 3; r++) {
    for (int c = 0; c < 3; c++) Rin[r * 4 + c] = G(r, c);
    Rin[r * 4 + 3] = 0;
  }
  q_from_R(q, Rin);
  normalize4(q);
  IO* o = body + ((size_t)b * T->n + p) * HS_SIM_BODY;
  for (int i = 0; i < 3; i++) o[i] = (IO)G(i, 3);
  for (int i = 0; i < 4; i++) o[3 + i] = (IO)q[i];
  for (int i = 7; i < 13; i++) o[i] = 0;
  (void)R;
}

}  // namespace

#ifdef HS_SIM_STAMPS
extern "C" int hs_debug_read_sim_stamps(unsigned long long* out, int n_rows) {
  if (n_rows > 4096) n_rows = 4096;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_sim_stamps), sizeof(unsigned long long) * 16 * n_rows, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int hs_debug_clear_sim_stamps() {
  static unsigned long long zero[4096][16];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_sim_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
#endif

namespace hs {

int launch_sim_reset(const hs_topo* d_topo, const hs_simtopo* d_sim, int32_t n_rollouts, const double* config,
                     int32_t config_stride, double* body, int32_t precision, void* stream) {
  if (n_rollouts <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (precision == HS_PREC_F32)
    hipLaunchKernelGGL(hs_sim_reset_kernel<float>, dim3(n_rollouts), dim3(WAVE), 0, st, d_topo, d_sim, n_rollouts,
                       reinterpret_cast<const float*>(config), config_stride, reinterpret_cast<float*>(body));
  else
    hipLaunchKernelGGL(hs_sim_reset_kernel<double>, dim3(n_rollouts), dim3(WAVE), 0, st, d_topo, d_sim, n_rollouts,
                       config, config_stride, body);
  return (int)hipGetLastError();
}

// rounds of resident rollouts a batch needs with kernel k (every rollout runs a whole launch)
static long sim_rounds(const void* k, long B) {
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, WAVE, 0) != hipSuccess || per_cu <= 0) return -1;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return -1;
  const long slots = (long)per_cu * cus;
  return (B + slots - 1) / slots;
}

template <int NM, int MM, class R, class S>
static void launch_class(const hs_topo* d_topo, const S* d_sim, const hs_sim_args& a, hipStream_t st) {
  if constexpr (sizeof(R) == 4) {
    // the 3-waves/SIMD build when it saves more than its per-rollout slowdown in rounds
    // (measured: spider B = 16384, 8 -> 6 rounds, +8 %; hexapod B = 4096, 2 -> 2 rounds, -9 %)
    const long r2 = sim_rounds((const void*)hs_sim_kernel<NM, MM, R, 1>, a.n_rollouts);
    const long r3 = sim_rounds((const void*)hs_sim_kernel<NM, MM, R, 3>, a.n_rollouts);
    if (r2 > 0 && r3 > 0 && 5 * r3 < 4 * r2) {
      hipLaunchKernelGGL((hs_sim_kernel<NM, MM, R, 3>), dim3(a.n_rollouts), dim3(WAVE), 0, st, d_topo, d_sim, a);
      return;
    }
  }
  hipLaunchKernelGGL((hs_sim_kernel<NM, MM, R, 1>), dim3(a.n_rollouts), dim3(WAVE), 0, st, d_topo, d_sim, a);
}

template <class R, class S>
static int launch_sim_typed(const hs_topo* d_topo, const S* d_sim, const hs_simtopo& hs, const hs_sim_args& a) {
  hipStream_t st = (hipStream_t)a.stream;
  // smallest LDS layout holding the model: parts and rows (6 per fixed, 5 per hinge, 3 per contact)
  if (hs.n <= 18 && hs.m_max <= 144)
    launch_class<18, 144, R>(d_topo, d_sim, a, st);
  else if (hs.n <= 22 && hs.m_max <= 176)
    launch_class<22, 176, R>(d_topo, d_sim, a, st);
  else if (hs.n <= HS_NMAX && hs.m_max <= 9 * HS_NMAX)
    launch_class<HS_NMAX, 9 * HS_NMAX, R>(d_topo, d_sim, a, st);
  else
    return (int)hipErrorInvalidValue;
  return (int)hipGetLastError();
}

int launch_sim_steps(const hs_topo* d_topo, const hs_simtopo* d_sim, const hs_simtopo_t<float>* d_sim_f32,
                     const hs_simtopo& hs, const hs_sim_args& a) {
  if (a.n_rollouts <= 0 || a.n_steps <= 0) return 0;
  if (a.precision == HS_PREC_F32) return launch_sim_typed<float>(d_topo, d_sim_f32, hs, a);
  return launch_sim_typed<double>(d_topo, d_sim, hs, a);
}

}  // namespace hs
