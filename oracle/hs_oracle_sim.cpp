// hs_oracle_sim.cpp -- TEST INFRASTRUCTURE ONLY. Included at the end of
// hs_oracle.cpp (one translation unit: it uses the restated affine/model code).
//
// CPU restatement of the reference's closed-loop simulation step,
// modelplayer::simulate_ode with position control (player.cpp:325-339):
//   set_position_control_torques (player.cpp:388-432)
//   -> dJointAddHingeTorque per motor (visualization.cpp:350-356)
//   -> dSpaceCollide + nearCallback: capsule/sphere vs the z = 0 plane,
//      surface mode Bounce|SoftCFM, mu = inf, bounce .5, bounce_vel .1,
//      soft_cfm .001 (visualization.cpp:296-326)
//   -> dWorldQuickStep (visualization.cpp:333-337): world ERP .8, gravity
//      (0,0,-1), CFM left at ODE's double default, 20 SOR iterations, w 1.3.
//
// ODE itself is not in this image, so its algorithms are
// restated from ODE 0.13 (the reference's makefile:7 links an unpinned
// -lode, built in double precision, makefile:9):
//   ode.cpp          dBodyCreate defaults (mass 1, I = identity, gyroscopic
//                    term on), dBodySetRotation (R -> q, normalize, q -> R)
//   util.cpp         dxProcessIslands: body / joint order of the island
//                    (world body list newest first, per-body joint lists
//                    newest first, depth-first from the newest body)
//   quickstep.cpp    dxQuickStepper + SOR_LCP: WARM_STARTING off,
//                    RANDOMLY_REORDER_CONSTRAINTS on (dRandInt reshuffle every
//                    8 iterations), REORDER_CONSTRAINTS off
//   joints/*.cpp     hinge (setBall + 2 rotational rows, no limit/motor row),
//                    fixed (3 linear + setFixedOrientation rows), contact
//                    (normal + 2 friction rows, dPlaneSpace tangents, bounce)
//   collision        dCollideCapsulePlane / dCollideSpherePlane (1 contact)
//   rotation.cpp     dQfromR, dQtoR, dDQfromW, dQMultiply0..2; odemath.cpp
//                    dSafeNormalize3/4, dPlaneSpace; misc.cpp dRand/dRandInt
//   step.cpp         dxStepBody (infinitesimal rotation, no damping / caps)
//
// Parity against ODE itself is unpinned (no ODE here): this restatement is
// pinned by physical known-answer tests in tests/test_sim_oracle.py (free fall,
// hinge angle of an oriented configuration, static stance force balance,
// linear momentum without gravity/contacts, LCP residuals at many iterations).

namespace {

// dMatrix3 = row-major 3x4 (R[i*4+j]), dQuaternion = (w, x, y, z)
inline double dot3(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
inline double dot3_41(const double* a, const double* b) { return a[0] * b[0] + a[4] * b[1] + a[8] * b[2]; }
inline double dot3_14(const double* a, const double* b) { return a[0] * b[0] + a[1] * b[4] + a[2] * b[8]; }
inline void cross3(double* r, const double* a, const double* b) {
  r[0] = a[1] * b[2] - a[2] * b[1];
  r[1] = a[2] * b[0] - a[0] * b[2];
  r[2] = a[0] * b[1] - a[1] * b[0];
}
inline void mul0_331(double* r, const double* B, const double* c) {  // r = B c
  double r0 = dot3(B, c), r1 = dot3(B + 4, c), r2 = dot3(B + 8, c);
  r[0] = r0; r[1] = r1; r[2] = r2;
}
inline void mul1_331(double* r, const double* B, const double* c) {  // r = B^T c
  double r0 = dot3_41(B, c), r1 = dot3_41(B + 1, c), r2 = dot3_41(B + 2, c);
  r[0] = r0; r[1] = r1; r[2] = r2;
}
inline void mul0_333(double* A, const double* B, const double* C) {  // A = B C
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) A[i * 4 + j] = dot3_14(B + i * 4, C + j);
    A[i * 4 + 3] = 0;
  }
}
inline void mul2_333(double* A, const double* B, const double* C) {  // A = B C^T
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) A[i * 4 + j] = dot3(B + i * 4, C + j * 4);
    A[i * 4 + 3] = 0;
  }
}

void dQtoR(const double* q, double* R) {  // rotation.cpp dQtoR
  double qq1 = 2 * q[1] * q[1], qq2 = 2 * q[2] * q[2], qq3 = 2 * q[3] * q[3];
  R[0] = 1 - qq2 - qq3;            R[1] = 2 * (q[1] * q[2] - q[0] * q[3]); R[2] = 2 * (q[1] * q[3] + q[0] * q[2]); R[3] = 0;
  R[4] = 2 * (q[1] * q[2] + q[0] * q[3]); R[5] = 1 - qq1 - qq3;     R[6] = 2 * (q[2] * q[3] - q[0] * q[1]); R[7] = 0;
  R[8] = 2 * (q[1] * q[3] - q[0] * q[2]); R[9] = 2 * (q[2] * q[3] + q[0] * q[1]); R[10] = 1 - qq1 - qq2;   R[11] = 0;
}

void dQfromR(double* q, const double* R) {  // rotation.cpp dQfromR
  auto r = [&](int i, int j) { return R[i * 4 + j]; };
  double tr = r(0, 0) + r(1, 1) + r(2, 2), s;
  if (tr >= 0) {
    s = sqrt(tr + 1);
    q[0] = 0.5 * s;
    s = 0.5 * (1.0 / s);
    q[1] = (r(2, 1) - r(1, 2)) * s;
    q[2] = (r(0, 2) - r(2, 0)) * s;
    q[3] = (r(1, 0) - r(0, 1)) * s;
    return;
  }
  int c;
  if (r(1, 1) > r(0, 0)) c = (r(2, 2) > r(1, 1)) ? 2 : 1;
  else c = (r(2, 2) > r(0, 0)) ? 2 : 0;
  if (c == 0) {
    s = sqrt((r(0, 0) - (r(1, 1) + r(2, 2))) + 1);
    q[1] = 0.5 * s;
    s = 0.5 * (1.0 / s);
    q[2] = (r(0, 1) + r(1, 0)) * s;
    q[3] = (r(2, 0) + r(0, 2)) * s;
    q[0] = (r(2, 1) - r(1, 2)) * s;
  } else if (c == 1) {
    s = sqrt((r(1, 1) - (r(2, 2) + r(0, 0))) + 1);
    q[2] = 0.5 * s;
    s = 0.5 * (1.0 / s);
    q[3] = (r(1, 2) + r(2, 1)) * s;
    q[1] = (r(0, 1) + r(1, 0)) * s;
    q[0] = (r(0, 2) - r(2, 0)) * s;
  } else {
    s = sqrt((r(2, 2) - (r(0, 0) + r(1, 1))) + 1);
    q[3] = 0.5 * s;
    s = 0.5 * (1.0 / s);
    q[1] = (r(2, 0) + r(0, 2)) * s;
    q[2] = (r(1, 2) + r(2, 1)) * s;
    q[0] = (r(1, 0) - r(0, 1)) * s;
  }
}

void dNormalize4(double* a) {  // odemath.cpp dSafeNormalize4
  double l = a[0] * a[0] + a[1] * a[1] + a[2] * a[2] + a[3] * a[3];
  if (l > 0) {
    l = 1.0 / sqrt(l);
    a[0] *= l; a[1] *= l; a[2] *= l; a[3] *= l;
  } else {
    a[0] = 1; a[1] = a[2] = a[3] = 0;
  }
}

void dNormalize3(double* a) {  // odemath.cpp dSafeNormalize3
  double aa0 = fabs(a[0]), aa1 = fabs(a[1]), aa2 = fabs(a[2]), l;
  if (aa1 > aa0) l = (aa2 > aa1) ? aa2 : aa1;
  else if (aa2 > aa0) l = aa2;
  else {
    if (aa0 <= 0) { a[0] = 1; a[1] = a[2] = 0; return; }
    l = aa0;
  }
  a[0] /= l; a[1] /= l; a[2] /= l;
  l = 1.0 / sqrt(a[0] * a[0] + a[1] * a[1] + a[2] * a[2]);
  a[0] *= l; a[1] *= l; a[2] *= l;
}

void dQMultiply1(double* qa, const double* qb, const double* qc) {  // qa = conj(qb) qc
  qa[0] = qb[0] * qc[0] + qb[1] * qc[1] + qb[2] * qc[2] + qb[3] * qc[3];
  qa[1] = qb[0] * qc[1] - qb[1] * qc[0] - qb[2] * qc[3] + qb[3] * qc[2];
  qa[2] = qb[0] * qc[2] - qb[2] * qc[0] - qb[3] * qc[1] + qb[1] * qc[3];
  qa[3] = qb[0] * qc[3] - qb[3] * qc[0] - qb[1] * qc[2] + qb[2] * qc[1];
}
void dQMultiply2(double* qa, const double* qb, const double* qc) {  // qa = qb conj(qc)
  qa[0] = qb[0] * qc[0] + qb[1] * qc[1] + qb[2] * qc[2] + qb[3] * qc[3];
  qa[1] = -qb[0] * qc[1] + qb[1] * qc[0] - qb[2] * qc[3] + qb[3] * qc[2];
  qa[2] = -qb[0] * qc[2] + qb[2] * qc[0] - qb[3] * qc[1] + qb[1] * qc[3];
  qa[3] = -qb[0] * qc[3] + qb[3] * qc[0] - qb[1] * qc[2] + qb[2] * qc[1];
}

void dPlaneSpace(const double* n, double* p, double* q) {  // odemath.cpp
  if (fabs(n[2]) > M_SQRT1_2) {
    double a = n[1] * n[1] + n[2] * n[2];
    double k = 1.0 / sqrt(a);
    p[0] = 0; p[1] = -n[2] * k; p[2] = n[1] * k;
    q[0] = a * k; q[1] = -n[0] * p[2]; q[2] = n[0] * p[1];
  } else {
    double a = n[0] * n[0] + n[1] * n[1];
    double k = 1.0 / sqrt(a);
    p[0] = -n[1] * k; p[1] = n[0] * k; p[2] = 0;
    q[0] = -n[2] * p[1]; q[1] = n[2] * p[0]; q[2] = a * k;
  }
}

uint32_t dRand(uint32_t& seed) {  // misc.cpp: 32-bit LCG
  seed = (uint32_t)((1664525ull * seed + 1013904223ull) & 0xffffffffull);
  return seed;
}
int dRandInt(uint32_t& seed, int n) {  // misc.cpp (ODE >= 0.11)
  uint32_t un = (uint32_t)n, r = dRand(seed);
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

enum { SJ_HINGE = 0, SJ_FIXED = 1, SJ_CONTACT = 2 };

struct SimJoint {
  int type = SJ_HINGE;
  int b1 = -1, b2 = -1;  // node[0].body, node[1].body (part ids; -1 = static environment)
  double anchor1[3] = {0, 0, 0}, anchor2[3] = {0, 0, 0}, axis1[3] = {0, 0, 0}, axis2[3] = {0, 0, 0};
  double qrel[4] = {1, 0, 0, 0}, offset[3] = {0, 0, 0};
  // contact
  double cpos[3] = {0, 0, 0}, normal[3] = {0, 0, 1}, depth = 0;
};

struct SimTopo {
  int n = 0, nmj = 0;
  std::vector<SimJoint> joints;           // creation order (kinematicmodel::set_ode_joints, model.cpp:375-400)
  std::vector<int> motors;                // motor j -> joint id (visualizer::add_motor order)
  std::vector<std::vector<int>> blist;    // per body: static joint ids, newest first
};

// a body state row: pos[3], q[4], lvel[3], avel[3]
constexpr int SB = 13;

void part_odebody_pose(const Node& nd, double* pos, double* q, double* R) {
  // odepart::get_odebody_posrot_from_body (visualization.cpp:520-527) + dBodySetPosition/Rotation
  Aff A;
  nd.A_ground.mult(nd.A_body_geom, A);
  double Rin[12];
  for (int i = 0; i < 3; i++) {
    for (int j = 0; j < 3; j++) Rin[i * 4 + j] = A.get_a(i, j);  // transpose_odematrix of the affine data
    Rin[i * 4 + 3] = 0;
    pos[i] = A.a[12 + i];
  }
  dQfromR(q, Rin);
  dNormalize4(q);
  dQtoR(q, R);
}

SimTopo sim_topo(const hso_model* m0) {
  // bodies oriented at the loaded configuration (modelplayer::load_model: orient_odebodys,
  // then set_ode_joints; player.cpp:46-51), joint frames fixed there
  hso_model mm = *m0;
  hso_model* m = &mm;
  for (int i = 0; i < m->cfg; i++) jv(m, i) = 0;
  recompute_modelnodes(m);
  SimTopo t;
  t.n = m->n;
  t.nmj = m->nmj;
  std::vector<double> pos(3 * m->n), q(4 * m->n), R(12 * m->n);
  for (int p = 0; p < m->n; p++) part_odebody_pose(m->nodes[p], &pos[3 * p], &q[4 * p], &R[12 * p]);
  t.blist.assign(m->n, {});
  for (int p = 0; p < m->n; p++) {
    const Node& nd = m->nodes[p];
    if (nd.parent < 0) continue;
    SimJoint J;
    if (nd.jtype == J_HINGE) {  // odepart::make_hinge_joint (visualization.cpp:583-603)
      J.type = SJ_HINGE;
      J.b1 = p;
      J.b2 = nd.parent;
      double anc[3], ax[4];
      for (int i = 0; i < 3; i++) { anc[i] = nd.J_A_ground.a[12 + i]; ax[i] = nd.J_A_ground.a[8 + i]; }
      double d1[3], d2[3];  // setAnchors (joint.cpp)
      for (int i = 0; i < 3; i++) { d1[i] = anc[i] - pos[3 * J.b1 + i]; d2[i] = anc[i] - pos[3 * J.b2 + i]; }
      mul1_331(J.anchor1, &R[12 * J.b1], d1);
      mul1_331(J.anchor2, &R[12 * J.b2], d2);
      dNormalize3(ax);  // setAxes
      mul1_331(J.axis1, &R[12 * J.b1], ax);
      mul1_331(J.axis2, &R[12 * J.b2], ax);
      dQMultiply1(J.qrel, &q[4 * J.b1], &q[4 * J.b2]);  // computeInitialRelativeRotation
      t.motors.push_back((int)t.joints.size());
    } else if (nd.jtype == J_NONE) {  // odepart::make_fixed_joint (visualization.cpp:572-579)
      J.type = SJ_FIXED;
      J.b1 = nd.parent;
      J.b2 = p;
      dQMultiply1(J.qrel, &q[4 * J.b1], &q[4 * J.b2]);  // dJointSetFixed
      double ofs[3];
      for (int i = 0; i < 3; i++) ofs[i] = pos[3 * J.b1 + i] - pos[3 * J.b2 + i];
      mul1_331(J.offset, &R[12 * J.b1], ofs);
    } else {
      continue;
    }
    int id = (int)t.joints.size();
    t.joints.push_back(J);
    // addJointReferencesToBodies: front insertion into both bodies' lists
    t.blist[J.b1].insert(t.blist[J.b1].begin(), id);
    t.blist[J.b2].insert(t.blist[J.b2].begin(), id);
  }
  return t;
}

struct SimBody {
  double pos[3], q[4], R[12], lvel[3], avel[3], facc[3], tacc[3];
  double mass, invMass, I[12], invI[12];
};

void load_bodies(int n, const double* st, std::vector<SimBody>& B) {
  B.resize(n);
  for (int p = 0; p < n; p++) {
    SimBody& b = B[p];
    const double* s = st + SB * p;
    for (int i = 0; i < 3; i++) { b.pos[i] = s[i]; b.lvel[i] = s[7 + i]; b.avel[i] = s[10 + i]; b.facc[i] = b.tacc[i] = 0; }
    for (int i = 0; i < 4; i++) b.q[i] = s[3 + i];
    dQtoR(b.q, b.R);
    // dBodyCreate: dMassSetParameters(1, 0,0,0, 1,1,1, 0,0,0); invI = inverse of the identity
    b.mass = 1;
    b.invMass = 1.0 / b.mass;
    for (int i = 0; i < 12; i++) b.I[i] = b.invI[i] = 0;
    for (int i = 0; i < 3; i++) b.I[i * 5] = b.invI[i * 5] = 1;
  }
}

void store_bodies(const std::vector<SimBody>& B, double* st) {
  for (size_t p = 0; p < B.size(); p++) {
    const SimBody& b = B[p];
    double* s = st + SB * p;
    for (int i = 0; i < 3; i++) { s[i] = b.pos[i]; s[7 + i] = b.lvel[i]; s[10 + i] = b.avel[i]; }
    for (int i = 0; i < 4; i++) s[3 + i] = b.q[i];
  }
}

// hinge.cpp getHingeAngle / getHingeAngleFromRelativeQuat, dJointGetHingeAngle(Rate)
double hinge_angle(const SimJoint& J, const std::vector<SimBody>& B) {
  double qq[4], qrel[4];
  dQMultiply1(qq, B[J.b1].q, B[J.b2].q);
  dQMultiply2(qrel, qq, J.qrel);
  double cost2 = qrel[0];
  double sint2 = sqrt(qrel[1] * qrel[1] + qrel[2] * qrel[2] + qrel[3] * qrel[3]);
  double theta = (dot3(qrel + 1, J.axis1) >= 0) ? (2 * atan2(sint2, cost2)) : (2 * atan2(sint2, -cost2));
  if (theta > M_PI) theta -= 2 * M_PI;
  return -theta;
}
double hinge_rate(const SimJoint& J, const std::vector<SimBody>& B) {
  double ax[3];
  mul0_331(ax, B[J.b1].R, J.axis1);
  double rate = dot3(ax, B[J.b1].avel);
  rate -= dot3(ax, B[J.b2].avel);
  return rate;
}

struct SimParams {
  double dt, k, sor_w, erp, cfm, gravity, bounce, bounce_vel, soft_cfm, mu;
  int iterations;
};

// Jacobian rows of one joint (getInfo2), written into the m x 12 block at row r0
struct Rows {
  std::vector<double> J, c, cfm, lo, hi;
  std::vector<int> jb;
  void resize(int m, double gcfm) {
    J.assign(12 * m, 0.0);
    c.assign(m, 0.0);
    cfm.assign(m, gcfm);
    lo.assign(m, -INFINITY);
    hi.assign(m, INFINITY);
    jb.assign(2 * m, -1);
  }
};

void set_ball(const SimJoint& J, const std::vector<SimBody>& B, double fps, double erp, Rows& w, int r0) {
  double* J1 = &w.J[12 * r0];
  for (int i = 0; i < 3; i++) J1[12 * i + i] = 1;  // J1l
  double a1[3], a2[3];
  mul0_331(a1, B[J.b1].R, J.anchor1);
  // dSetCrossMatrixMinus(J1a, a1): row i of -[a1]x
  J1[3 + 0 * 12 + 1] = a1[2];  J1[3 + 0 * 12 + 2] = -a1[1];
  J1[3 + 1 * 12 + 0] = -a1[2]; J1[3 + 1 * 12 + 2] = a1[0];
  J1[3 + 2 * 12 + 0] = a1[1];  J1[3 + 2 * 12 + 1] = -a1[0];
  for (int i = 0; i < 3; i++) J1[12 * i + 6 + i] = -1;  // J2l
  mul0_331(a2, B[J.b2].R, J.anchor2);
  // dSetCrossMatrixPlus(J2a, a2): row i of [a2]x
  J1[9 + 0 * 12 + 1] = -a2[2]; J1[9 + 0 * 12 + 2] = a2[1];
  J1[9 + 1 * 12 + 0] = a2[2];  J1[9 + 1 * 12 + 2] = -a2[0];
  J1[9 + 2 * 12 + 0] = -a2[1]; J1[9 + 2 * 12 + 1] = a2[0];
  double k = fps * erp;
  for (int j = 0; j < 3; j++) w.c[r0 + j] = k * (a2[j] + B[J.b2].pos[j] - a1[j] - B[J.b1].pos[j]);
}

void hinge_info2(const SimJoint& J, const std::vector<SimBody>& B, double fps, double erp, Rows& w, int r0) {
  set_ball(J, B, fps, erp, w, r0);
  double ax1[3], p[3], q[3];
  mul0_331(ax1, B[J.b1].R, J.axis1);
  dPlaneSpace(ax1, p, q);
  double* J3 = &w.J[12 * (r0 + 3)];
  double* J4 = &w.J[12 * (r0 + 4)];
  for (int i = 0; i < 3; i++) {
    J3[3 + i] = p[i]; J4[3 + i] = q[i];
    J3[9 + i] = -p[i]; J4[9 + i] = -q[i];
  }
  double ax2[3], b[3];
  mul0_331(ax2, B[J.b2].R, J.axis2);
  cross3(b, ax1, ax2);
  double k = fps * erp;
  w.c[r0 + 3] = k * dot3(b, p);
  w.c[r0 + 4] = k * dot3(b, q);
}

void fixed_info2(const SimJoint& J, const std::vector<SimBody>& B, double fps, double erp, double cfm, Rows& w, int r0) {
  // setFixedOrientation(joint, info, qrel, 3) (joint.cpp)
  for (int i = 0; i < 3; i++) {
    w.J[12 * (r0 + 3 + i) + 3 + i] = 1;
    w.J[12 * (r0 + 3 + i) + 9 + i] = -1;
  }
  double qq[4], qerr[4], e[3];
  dQMultiply1(qq, B[J.b1].q, B[J.b2].q);
  dQMultiply2(qerr, qq, J.qrel);
  if (qerr[0] < 0) { qerr[1] = -qerr[1]; qerr[2] = -qerr[2]; qerr[3] = -qerr[3]; }
  mul0_331(e, B[J.b1].R, qerr + 1);
  double k = fps * erp;  // correcting angular velocity (erp fps) 2 v, v = vector part of qerr
  w.c[r0 + 3] = 2 * k * e[0];
  w.c[r0 + 4] = 2 * k * e[1];
  w.c[r0 + 5] = 2 * k * e[2];
  // three linear rows (fixed.cpp getInfo2); the joint's erp/cfm are the world's at creation
  double* J0 = &w.J[12 * r0];
  for (int i = 0; i < 3; i++) { J0[12 * i + i] = 1; J0[12 * i + 6 + i] = -1; w.cfm[r0 + i] = cfm; }
  double ofs[3];
  mul0_331(ofs, B[J.b1].R, J.offset);
  // dSetCrossMatrixPlus(J1a, ofs)
  J0[3 + 0 * 12 + 1] = -ofs[2]; J0[3 + 0 * 12 + 2] = ofs[1];
  J0[3 + 1 * 12 + 0] = ofs[2];  J0[3 + 1 * 12 + 2] = -ofs[0];
  J0[3 + 2 * 12 + 0] = -ofs[1]; J0[3 + 2 * 12 + 1] = ofs[0];
  for (int j = 0; j < 3; j++) w.c[r0 + j] = k * (B[J.b2].pos[j] - B[J.b1].pos[j] + ofs[j]);
}

void contact_info2(const SimJoint& J, const std::vector<SimBody>& B, const SimParams& P, double fps, Rows& w, int r0) {
  // contact.cpp getInfo2; body1 = the geom's body, body2 = none (dJointAttach(c, b, 0))
  const double* normal = J.normal;
  double c1[3];
  for (int i = 0; i < 3; i++) c1[i] = J.cpos[i] - B[J.b1].pos[i];
  double* J0 = &w.J[12 * r0];
  for (int i = 0; i < 3; i++) J0[i] = normal[i];
  cross3(J0 + 3, c1, normal);
  double k = fps * P.erp;
  double depth = J.depth - 0.0;  // world->contactp.min_depth = 0
  if (depth < 0) depth = 0;
  w.cfm[r0] = P.soft_cfm;  // dContactSoftCFM
  double pushout = k * depth + 0.0;
  w.c[r0] = pushout;
  if (w.c[r0] > INFINITY) w.c[r0] = INFINITY;  // contactp.max_vel = dInfinity
  // dContactBounce
  double outgoing = dot3(J0, B[J.b1].lvel) + dot3(J0 + 3, B[J.b1].avel);
  outgoing -= 0.0;
  if (P.bounce_vel >= 0 && (-outgoing) > P.bounce_vel) {
    double newc = -P.bounce * outgoing + 0.0;
    if (newc > w.c[r0]) w.c[r0] = newc;
  }
  w.lo[r0] = 0;
  w.hi[r0] = INFINITY;
  double t1[3], t2[3];
  dPlaneSpace(normal, t1, t2);
  double* J1 = J0 + 12;
  double* J2 = J0 + 24;
  for (int i = 0; i < 3; i++) { J1[i] = t1[i]; J2[i] = t2[i]; }
  cross3(J1 + 3, c1, t1);
  cross3(J2 + 3, c1, t2);
  w.lo[r0 + 1] = -P.mu; w.hi[r0 + 1] = P.mu;
  w.lo[r0 + 2] = -P.mu; w.hi[r0 + 2] = P.mu;
}

// dCollideCapsulePlane / dCollideSpherePlane against the plane (0,0,1,0); 1 contact
bool collide_plane(const Node& nd, const SimBody& b, double* cpos, double* depth) {
  const double n[3] = {0, 0, 1};
  if (nd.gtype == 2) {
    double sign = (dot3_14(n, b.R + 2) > 0) ? -1.0 : 1.0;
    double p[3];
    p[0] = b.pos[0] + b.R[2] * nd.glen * 0.5 * sign;
    p[1] = b.pos[1] + b.R[6] * nd.glen * 0.5 * sign;
    p[2] = b.pos[2] + b.R[10] * nd.glen * 0.5 * sign;
    double k = dot3(p, n);
    double d = 0 - k + nd.gr;
    if (d < 0) return false;
    for (int i = 0; i < 3; i++) cpos[i] = p[i] - n[i] * nd.gr;
    *depth = d;
    return true;
  }
  if (nd.gtype == 1) {
    double k = dot3(b.pos, n);
    double d = 0 - k + nd.gr;
    if (d >= 0) {
      for (int i = 0; i < 3; i++) cpos[i] = b.pos[i] - n[i] * nd.gr;
      *depth = d;
      return true;
    }
  }
  return false;
}

struct StepOut {
  int n_contacts = 0;
  double normal_force = 0;  // sum of the contact normal lambdas
};

// dxQuickStepper over the robot's island (quickstep.cpp)
void quickstep(const hso_model* m, const SimTopo& T, const SimParams& P, std::vector<SimBody>& B,
               std::vector<SimJoint>& contacts, uint32_t& seed, StepOut& so) {
  const int n = T.n;
  const double h = P.dt, h1 = 1.0 / h;
  // dxProcessIslands: body order and joint order
  std::vector<int> contact_of(n, -1);
  for (size_t c = 0; c < contacts.size(); c++) contact_of[contacts[c].b1] = (int)c;
  std::vector<char> btag(n, 0), jtag(T.joints.size(), 0), ctag(contacts.size(), 0);
  std::vector<int> border, jorder;  // jorder: >= 0 static joint id, < 0: -(contact index)-1
  std::vector<int> stack;
  for (int bb = n - 1; bb >= 0; bb--) {  // world body list: newest first
    if (btag[bb]) continue;
    btag[bb] = 1;
    stack.push_back(bb);
    while (!stack.empty()) {
      int b = stack.back();
      stack.pop_back();
      border.push_back(b);
      // per-body joint list newest first: this step's contact, then the static joints
      if (contact_of[b] >= 0 && !ctag[contact_of[b]]) {
        ctag[contact_of[b]] = 1;
        jorder.push_back(-contact_of[b] - 1);
      }
      for (int jid : T.blist[b]) {
        if (jtag[jid]) continue;
        jtag[jid] = 1;
        jorder.push_back(jid);
        const SimJoint& J = T.joints[jid];
        int other = (J.b1 == b) ? J.b2 : J.b1;
        if (other >= 0 && !btag[other]) { btag[other] = 1; stack.push_back(other); }
      }
    }
  }
  std::vector<int> tag(n);
  for (int i = 0; i < n; i++) tag[border[i]] = i;
  const int nb = n;
  // inverse inertia in the world frame; gyroscopic torque
  std::vector<double> invI(12 * nb);
  for (int i = 0; i < nb; i++) {
    SimBody& b = B[border[i]];
    double tmp[12];
    mul2_333(tmp, b.invI, b.R);
    mul0_333(&invI[12 * i], b.R, tmp);
    double I[12], t3[3];
    mul2_333(tmp, b.I, b.R);
    mul0_333(I, b.R, tmp);
    mul0_331(t3, I, b.avel);
    b.tacc[0] -= b.avel[1] * t3[2] - b.avel[2] * t3[1];
    b.tacc[1] -= b.avel[2] * t3[0] - b.avel[0] * t3[2];
    b.tacc[2] -= b.avel[0] * t3[1] - b.avel[1] * t3[0];
  }
  if (P.gravity != 0)
    for (int i = 0; i < nb; i++) B[border[i]].facc[2] += B[border[i]].mass * (-P.gravity);
  // rows
  std::vector<int> ofs(jorder.size()), jm(jorder.size());
  int mrows = 0;
  for (size_t j = 0; j < jorder.size(); j++) {
    int id = jorder[j];
    int mj = (id < 0) ? (P.mu > 0 ? 3 : 1) : (T.joints[id].type == SJ_HINGE ? 5 : 6);
    ofs[j] = mrows;
    jm[j] = mj;
    mrows += mj;
  }
  const int mr = mrows;
  Rows w;
  w.resize(mr, P.cfm);
  for (size_t j = 0; j < jorder.size(); j++) {
    int id = jorder[j];
    const SimJoint& J = (id < 0) ? contacts[-id - 1] : T.joints[id];
    if (J.type == SJ_HINGE) hinge_info2(J, B, h1, P.erp, w, ofs[j]);
    else if (J.type == SJ_FIXED) fixed_info2(J, B, h1, P.erp, P.cfm, w, ofs[j]);
    else contact_info2(J, B, P, h1, w, ofs[j]);
    int b1 = (J.b1 >= 0) ? tag[J.b1] : -1, b2 = (J.b2 >= 0) ? tag[J.b2] : -1;
    for (int r = 0; r < jm[j]; r++) { w.jb[2 * (ofs[j] + r)] = b1; w.jb[2 * (ofs[j] + r) + 1] = b2; }
  }
  // rhs = c/h - J (v/h + invM fe)
  std::vector<double> tmp1(6 * nb);
  for (int i = 0; i < nb; i++) {
    const SimBody& b = B[border[i]];
    for (int j = 0; j < 3; j++) tmp1[6 * i + j] = b.facc[j] * b.invMass + b.lvel[j] * h1;
    mul0_331(&tmp1[6 * i + 3], &invI[12 * i], b.tacc);
    for (int j = 0; j < 3; j++) tmp1[6 * i + 3 + j] += b.avel[j] * h1;
  }
  std::vector<double> rhs(mr);
  for (int i = 0; i < mr; i++) {
    int b1 = w.jb[2 * i], b2 = w.jb[2 * i + 1];
    const double* Jr = &w.J[12 * i];
    double sum = 0;
    for (int j = 0; j < 6; j++) sum += Jr[j] * tmp1[6 * b1 + j];
    if (b2 >= 0)
      for (int j = 0; j < 6; j++) sum += Jr[6 + j] * tmp1[6 * b2 + j];
    rhs[i] = sum;
  }
  for (int i = 0; i < mr; i++) rhs[i] = w.c[i] * h1 - rhs[i];
  for (int i = 0; i < mr; i++) w.cfm[i] *= h1;
  // SOR_LCP (WARM_STARTING off: lambda = 0, fc = 0)
  std::vector<double> lambda(mr, 0.0), fc(6 * nb, 0.0), iMJ(12 * mr, 0.0), Ad(mr);
  for (int i = 0; i < mr; i++) {  // compute_invM_JT
    int b1 = w.jb[2 * i], b2 = w.jb[2 * i + 1];
    const double* Jr = &w.J[12 * i];
    double* iM = &iMJ[12 * i];
    double k1 = B[border[b1]].invMass;
    for (int j = 0; j < 3; j++) iM[j] = k1 * Jr[j];
    mul0_331(iM + 3, &invI[12 * b1], Jr + 3);
    if (b2 >= 0) {
      double k2 = B[border[b2]].invMass;
      for (int j = 0; j < 3; j++) iM[6 + j] = k2 * Jr[6 + j];
      mul0_331(iM + 9, &invI[12 * b2], Jr + 9);
    }
  }
  for (int i = 0; i < mr; i++) {
    const double* Jr = &w.J[12 * i];
    const double* iM = &iMJ[12 * i];
    double sum = 0;
    for (int j = 0; j < 6; j++) sum += iM[j] * Jr[j];
    if (w.jb[2 * i + 1] >= 0)
      for (int j = 6; j < 12; j++) sum += iM[j] * Jr[j];
    Ad[i] = P.sor_w / (sum + w.cfm[i]);
  }
  for (int i = 0; i < mr; i++) {
    for (int j = 0; j < 12; j++) w.J[12 * i + j] *= Ad[i];
    rhs[i] *= Ad[i];
    Ad[i] *= w.cfm[i];
  }
  std::vector<int> order(mr);
  for (int i = 0; i < mr; i++) order[i] = i;  // every findex is -1: identity order
  for (int it = 0; it < P.iterations; it++) {
    if ((it & 7) == 0) {
      for (int i = 1; i < mr; i++) {
        int swapi = dRandInt(seed, i + 1);
        std::swap(order[i], order[swapi]);
      }
    }
    for (int i = 0; i < mr; i++) {
      int index = order[i];
      const double* Jr = &w.J[12 * index];
      const double* iM = &iMJ[12 * index];
      int b1 = w.jb[2 * index], b2 = w.jb[2 * index + 1];
      double delta = rhs[index] - lambda[index] * Ad[index];
      double* f = &fc[6 * b1];
      delta -= f[0] * Jr[0] + f[1] * Jr[1] + f[2] * Jr[2] + f[3] * Jr[3] + f[4] * Jr[4] + f[5] * Jr[5];
      if (b2 >= 0) {
        f = &fc[6 * b2];
        delta -= f[0] * Jr[6] + f[1] * Jr[7] + f[2] * Jr[8] + f[3] * Jr[9] + f[4] * Jr[10] + f[5] * Jr[11];
      }
      double new_lambda = lambda[index] + delta;
      if (new_lambda < w.lo[index]) {
        delta = w.lo[index] - lambda[index];
        lambda[index] = w.lo[index];
      } else if (new_lambda > w.hi[index]) {
        delta = w.hi[index] - lambda[index];
        lambda[index] = w.hi[index];
      } else {
        lambda[index] = new_lambda;
      }
      f = &fc[6 * b1];
      for (int j = 0; j < 6; j++) f[j] += delta * iM[j];
      if (b2 >= 0) {
        f = &fc[6 * b2];
        for (int j = 0; j < 6; j++) f[j] += delta * iM[6 + j];
      }
    }
  }
  so.n_contacts = (int)contacts.size();
  so.normal_force = 0;
  for (size_t j = 0; j < jorder.size(); j++)
    if (jorder[j] < 0) so.normal_force += lambda[ofs[j]];
  // velocities: constraint part, then external forces
  for (int i = 0; i < nb; i++) {
    SimBody& b = B[border[i]];
    for (int j = 0; j < 3; j++) b.lvel[j] += h * fc[6 * i + j];
    for (int j = 0; j < 3; j++) b.avel[j] += h * fc[6 * i + 3 + j];
  }
  for (int i = 0; i < nb; i++) {
    SimBody& b = B[border[i]];
    double hm = h * b.invMass;
    for (int j = 0; j < 3; j++) {
      b.lvel[j] += hm * b.facc[j];
      b.tacc[j] *= h;
    }
    double t3[3];
    mul0_331(t3, &invI[12 * i], b.tacc);
    for (int j = 0; j < 3; j++) b.avel[j] += t3[j];
  }
  // dxStepBody
  for (int i = 0; i < nb; i++) {
    SimBody& b = B[border[i]];
    for (int j = 0; j < 3; j++) b.pos[j] += h * b.lvel[j];
    double dq[4];
    const double* wv = b.avel;
    const double* q = b.q;
    dq[0] = 0.5 * (-wv[0] * q[1] - wv[1] * q[2] - wv[2] * q[3]);
    dq[1] = 0.5 * (wv[0] * q[0] + wv[1] * q[3] - wv[2] * q[2]);
    dq[2] = 0.5 * (-wv[0] * q[3] + wv[1] * q[0] + wv[2] * q[1]);
    dq[3] = 0.5 * (wv[0] * q[2] - wv[1] * q[1] + wv[2] * q[0]);
    for (int j = 0; j < 4; j++) b.q[j] += h * dq[j];
    dNormalize4(b.q);
    dQtoR(b.q, b.R);
    for (int j = 0; j < 3; j++) b.facc[j] = b.tacc[j] = 0;
  }
}

}  // namespace

extern "C" {

int hso_sim_reset(const hso_model* m0, const double* config, double* body) {
  // init_play_config (player.cpp:351-356): joint values -> FK -> orient_odebodys, zero velocities
  hso_model mm = *m0;
  hso_model* m = &mm;
  for (int i = 0; i < m->cfg; i++) jv(m, i) = config[i];
  recompute_modelnodes(m);
  for (int p = 0; p < m->n; p++) {
    double R[12];
    double* s = body + SB * p;
    part_odebody_pose(m->nodes[p], s, s + 3, R);
    for (int i = 7; i < 13; i++) s[i] = 0;
  }
  return 0;
}

int hso_sim_hinges(const hso_model* m, const double* body, double* q, double* dq) {
  SimTopo T = sim_topo(m);
  std::vector<SimBody> B;
  load_bodies(T.n, body, B);
  for (int j = 0; j < T.nmj; j++) {
    const SimJoint& J = T.joints[T.motors[j]];
    if (q) q[j] = hinge_angle(J, B);
    if (dq) dq[j] = hinge_rate(J, B);
  }
  return 0;
}

/* p: dt, k, sor_w, erp, cfm, gravity, bounce, bounce_vel, soft_cfm, mu (10 doubles) */
int hso_sim_run(const hso_model* m, const double* p10, int iterations, int n_t, const double* q_tab,
                const double* dq_tab, const double* tau_tab, double* body, uint32_t* seed, int32_t* tsi,
                int n_steps, double* tau_cmd, double* q_meas, double* torso, int32_t* n_contacts,
                double* normal_force) {
  SimParams P{p10[0], p10[1], p10[2], p10[3], p10[4], p10[5], p10[6], p10[7], p10[8], p10[9], iterations};
  SimTopo T = sim_topo(m);
  const int n = T.n, nmj = T.nmj, cfg = m->cfg;
  std::vector<SimBody> B;
  load_bodies(n, body, B);
  std::vector<double> tau(nmj), qm(nmj), dqm(nmj);
  for (int s = 0; s < n_steps; s++) {
    // set_position_control_torques (player.cpp:388-409)
    if (P.k > 0) {
      double k1 = -P.k, k2 = -2 * sqrt(P.k);
      int t = *tsi % n_t;  // get_motor_adas / get_computed_torques index (periodic.cpp:394-399)
      int hrow = (t + n_t - 2) % n_t;  // hs_run output row holding sample t (t < 2: t + n_t)
      for (int j = 0; j < nmj; j++) {
        const SimJoint& J = T.joints[T.motors[j]];
        qm[j] = hinge_angle(J, B);
        dqm[j] = hinge_rate(J, B);
        double a1 = qm[j] - q_tab[(size_t)hrow * cfg + 6 + j];
        double a2 = dqm[j] - dq_tab[(size_t)hrow * cfg + 6 + j];
        if (a1 > M_PI) a1 -= 2 * M_PI;  // arrayops::modulus (core.cpp:122-131)
        else if (a1 <= -M_PI) a1 += 2 * M_PI;
        a1 *= k1;
        a2 *= k2;
        a1 += a2;
        tau[j] = tau_tab[(size_t)hrow * nmj + j] + a1;
      }
      // dJointAddHingeTorque (hinge.cpp): +tau axis on body1, -tau axis on body2
      for (int j = 0; j < nmj; j++) {
        const SimJoint& J = T.joints[T.motors[j]];
        double ax[3];
        mul0_331(ax, B[J.b1].R, J.axis1);
        for (int i = 0; i < 3; i++) ax[i] *= tau[j];
        for (int i = 0; i < 3; i++) B[J.b1].tacc[i] += ax[i];
        for (int i = 0; i < 3; i++) B[J.b2].tacc[i] += -ax[i];
      }
    } else {
      for (int j = 0; j < nmj; j++) {
        tau[j] = 0;
        qm[j] = hinge_angle(T.joints[T.motors[j]], B);
      }
    }
    // dSpaceCollide + nearCallback
    std::vector<SimJoint> contacts;
    for (int p = 0; p < n; p++) {
      SimJoint C;
      if (collide_plane(m->nodes[p], B[p], C.cpos, &C.depth)) {
        C.type = SJ_CONTACT;
        C.b1 = p;
        C.b2 = -1;
        contacts.push_back(C);
      }
    }
    StepOut so;
    quickstep(m, T, P, B, contacts, *seed, so);
    *tsi += 1;  // play_t += play_dt
    if (tau_cmd) for (int j = 0; j < nmj; j++) tau_cmd[(size_t)s * nmj + j] = tau[j];
    if (q_meas) for (int j = 0; j < nmj; j++) q_meas[(size_t)s * nmj + j] = qm[j];
    if (torso) for (int i = 0; i < 3; i++) torso[3 * s + i] = B[0].pos[i];
    if (n_contacts) n_contacts[s] = so.n_contacts;
    if (normal_force) normal_force[s] = so.normal_force;
  }
  store_bodies(B, body);
  return 0;
}

/* B rollouts on n_threads std::threads (bench.py's cpu_baseline leg): tables [B][n_t][...],
 * body [B][n][13], seed/tsi [B]; per-step outputs are not kept. */
int hso_sim_batch(const hso_model* m, const double* p10, int iterations, int n_t, int B, const double* q_tab,
                  const double* dq_tab, const double* tau_tab, double* body, uint32_t* seed, int32_t* tsi,
                  int n_steps, int n_threads) {
  const size_t cfg = m->cfg, nmj = m->nmj, nb = (size_t)m->n * SB;
  std::vector<std::thread> th;
  if (n_threads < 1) n_threads = 1;
  for (int t = 0; t < n_threads; t++)
    th.emplace_back([=]() {
      for (int b = t; b < B; b += n_threads)
        hso_sim_run(m, p10, iterations, n_t, q_tab + (size_t)b * n_t * cfg, dq_tab + (size_t)b * n_t * cfg,
                    tau_tab + (size_t)b * n_t * nmj, body + (size_t)b * nb, seed + b, tsi + b, n_steps, nullptr,
                    nullptr, nullptr, nullptr, nullptr);
    });
  for (auto& x : th) x.join();
  return 0;
}

}  // extern "C"
