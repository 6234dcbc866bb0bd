// hs_simtopo.h -- device-resident description of a model's ODE world, for the
// closed-loop simulation kernels (hs_sim.hip).
//
// Built by hs_model_load() from the same XML as hs_topo: one ODE body per part
// (odepart::make, visualization.cpp:441-504: default mass 1, identity inertia,
// geom at the body origin), one joint per non-root part created in preorder by
// kinematicmodel::set_ode_joints (model.cpp:375-400): a hinge
// (odepart::make_hinge_joint, visualization.cpp:583-603: body1 = part,
// body2 = parent) or a fixed joint (make_fixed_joint, visualization.cpp:572-579:
// body1 = parent, body2 = part), with anchors, axes and relative rotations fixed
// at the loaded configuration (modelplayer::load_model orients the bodies first,
// player.cpp:46-51). The island order of ODE's dxProcessIslands is static here
// (contacts attach to the environment, so they never add bodies): the body
// visitation order and, per visited body, the static joints first reached from it.
#pragma once
#include <stdint.h>

#include "hs_topo.h"

#define HS_SIM_JMAX (HS_NMAX - 1)  // static joints: one per non-root part
#define HS_SIM_BODY 13             // body state row: pos[3], q[4] (w,x,y,z), lvel[3], avel[3]
#define HS_SIM_TQMAX 6             // motor torque terms per body (own hinge + child hinges)
#define HS_SIM_LCG 256             // > rows of any model (9 HS_NMAX - 6)

enum { HS_SJ_HINGE = 0, HS_SJ_FIXED = 1 };
enum { HS_GEOM_NONE = 0, HS_GEOM_SPHERE = 1, HS_GEOM_CAPSULE = 2, HS_GEOM_CYLINDER = 3 };

// real = double (built on the host, as the reference computes) or float (a rounded copy for
// the single-precision simulation kernel)
template <class real>
struct hs_simjoint_t {
  int32_t type;    // HS_SJ_*
  int32_t b1, b2;  // node[0].body, node[1].body (part ids)
  int32_t motor;   // motor index (visualizer::add_motor order) or -1
  real anchor1[3], anchor2[3];  // setAnchors: anchor in body1 / body2 frames
  real axis1[3], axis2[3];      // setAxes: hinge axis in body1 / body2 frames
  real qrel[4];                 // conj(q1) q2 at creation (hinge angle zero / fixed orientation)
  real offset[3];               // fixed: R1^T (pos1 - pos2)
};

template <class real>
struct hs_simtopo_t {
  int32_t n, nmj, nj, m_max;  // parts, motors, static joints, rows bound (6 nj + 3 n_collidable)
  int32_t n_coll, pad0, pad1, pad2;
  // geometry per part: class, radius, cylinder length (dCreateSphere / dCreateCapsule), and the
  // geom frame in the part frame (odepart::A_body_geom, 3x4 column-major like hs_aff34)
  int32_t gtype[HS_NMAX];
  real gr[HS_NMAX], glen[HS_NMAX];
  hs_aff34 body_geom[HS_NMAX];  // (double: used by the reset, which builds states in double)
  real mass[HS_NMAX];
  real inertia[HS_NMAX][9];   // body-frame inertia (row-major), dBodyCreate default: identity
  real inv_inertia[HS_NMAX][9];
  // island order (dxProcessIslands): visitation order of the parts, and for the body visited
  // at position v the static joints first reached from it: jseq[jseq_start[v] .. jseq_start[v+1])
  int32_t border[HS_NMAX];
  int32_t jseq_start[HS_NMAX + 1];
  int32_t jseq[HS_SIM_JMAX];
  int32_t motor_joint[HS_NMAX];  // motor j -> joint id
  // dJointAddHingeTorque terms per body, in motor order: motor index, sign (+1 body1, -1 body2)
  int32_t tq_n[HS_NMAX];
  int32_t tq_motor[HS_NMAX][HS_SIM_TQMAX];
  int32_t tq_sign[HS_NMAX][HS_SIM_TQMAX];
  hs_simjoint_t<real> joint[HS_SIM_JMAX];
  // ODE's dRand LCG (seed' = a seed + c mod 2^32) jumped i steps: seed_i = lcg_a[i] seed + lcg_c[i],
  // so the dRandInt draws of one SOR reshuffle can be made by all lanes at once
  uint32_t lcg_a[HS_SIM_LCG], lcg_c[HS_SIM_LCG];
};

using hs_simjoint = hs_simjoint_t<double>;
using hs_simtopo = hs_simtopo_t<double>;

// the single-precision copy: every real rounded, everything else as is
inline void hs_simtopo_round(hs_simtopo_t<float>& d, const hs_simtopo& s) {
  d.n = s.n; d.nmj = s.nmj; d.nj = s.nj; d.m_max = s.m_max;
  d.n_coll = s.n_coll; d.pad0 = s.pad0; d.pad1 = s.pad1; d.pad2 = s.pad2;
  for (int i = 0; i < HS_NMAX; i++) {
    d.gtype[i] = s.gtype[i];
    d.gr[i] = (float)s.gr[i];
    d.glen[i] = (float)s.glen[i];
    d.body_geom[i] = s.body_geom[i];
    d.mass[i] = (float)s.mass[i];
    for (int k = 0; k < 9; k++) {
      d.inertia[i][k] = (float)s.inertia[i][k];
      d.inv_inertia[i][k] = (float)s.inv_inertia[i][k];
    }
    d.border[i] = s.border[i];
    d.motor_joint[i] = s.motor_joint[i];
    d.tq_n[i] = s.tq_n[i];
    for (int k = 0; k < HS_SIM_TQMAX; k++) { d.tq_motor[i][k] = s.tq_motor[i][k]; d.tq_sign[i][k] = s.tq_sign[i][k]; }
  }
  for (int i = 0; i <= HS_NMAX; i++) d.jseq_start[i] = s.jseq_start[i];
  for (int i = 0; i < HS_SIM_JMAX; i++) {
    d.jseq[i] = s.jseq[i];
    const hs_simjoint& a = s.joint[i];
    hs_simjoint_t<float>& b = d.joint[i];
    b.type = a.type; b.b1 = a.b1; b.b2 = a.b2; b.motor = a.motor;
    for (int k = 0; k < 3; k++) {
      b.anchor1[k] = (float)a.anchor1[k]; b.anchor2[k] = (float)a.anchor2[k];
      b.axis1[k] = (float)a.axis1[k]; b.axis2[k] = (float)a.axis2[k];
      b.offset[k] = (float)a.offset[k];
    }
    for (int k = 0; k < 4; k++) b.qrel[k] = (float)a.qrel[k];
  }
  for (int i = 0; i < HS_SIM_LCG; i++) { d.lcg_a[i] = s.lcg_a[i]; d.lcg_c[i] = s.lcg_c[i]; }
}
