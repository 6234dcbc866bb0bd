// hs_model.cpp -- host side of the boundary: MuJoCo-subset XML -> hs_topo.
//
// Replaces kinematicmodel::load_fromxml / mnode_from_xnode / make_joint
// (model.cpp:224-289, 119-174), the odepart geometry (visualization.cpp:441-504),
// liksolver::set_limbs (lik.cpp:44-78) and periodic::set_dynparts
// (periodic.cpp:34-58), without ODE, rapidxml or pointer-linked trees. The
// constant transforms are built with the same operation sequence as the
// reference (ODE rotation formulas restated) so the device tables hold the
// values the reference model would hold.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "hs_internal.h"
#include "hs_ode.h"

namespace hs {

namespace {

// 4x4 column-major rigid transform used only while building tables.
struct M4 {
  double a[16];
  static M4 unity() { M4 m; for (int i = 0; i < 16; i++) m.a[i] = (i % 5 == 0) ? 1.0 : 0.0; return m; }
  static M4 translation(const double* p) { M4 m = unity(); m.a[12] = p[0]; m.a[13] = p[1]; m.a[14] = p[2]; return m; }
  M4 operator*(const M4& b) const {  // sum over k = 0..3 from zero (matrix.cpp:78-97)
    M4 c;
    for (int i = 0; i < 4; i++)
      for (int j = 0; j < 4; j++) {
        double s = 0;
        for (int k = 0; k < 4; k++) s += a[k * 4 + j] * b.a[i * 4 + k];
        c.a[i * 4 + j] = s;
      }
    return c;
  }
  void set_rotation12(const double* r) { for (int i = 0; i < 12; i++) a[i] = r[i]; a[12] = a[13] = a[14] = 0; a[15] = 1; }
  void translate(const double* t) { for (int i = 0; i < 3; i++) a[12 + i] += t[i]; }
  M4 transposed() const { M4 t; for (int i = 0; i < 4; i++) for (int j = 0; j < 4; j++) t.a[i * 4 + j] = a[j * 4 + i]; return t; }
  void invert_rigid() {  // matrix.cpp:182-193
    double t[4] = {-a[12], -a[13], -a[14], 1.0};
    a[12] = a[13] = a[14] = 0;
    *this = transposed();
    double t1[4];
    for (int i = 0; i < 4; i++) {
      double s = 0;
      for (int j = 0; j < 4; j++) s += a[j * 4 + i] * t[j];
      t1[i] = s;
    }
    translate(t1);
  }
  hs_aff34 to34() const { hs_aff34 r; for (int c = 0; c < 4; c++) for (int i = 0; i < 3; i++) r.m[c * 3 + i] = a[c * 4 + i]; return r; }
};

// ODE dRFromAxisAndAngle = dQFromAxisAndAngle + dQtoR (row-major 3x4)
void ode_axis_angle(double* R, double ax, double ay, double az, double angle) {
  double q0, q1, q2, q3;
  double l = ax * ax + ay * ay + az * az;
  if (l > 0.0) {
    angle *= 0.5;
    q0 = cos(angle);
    l = sin(angle) * (1.0 / sqrt(l));
    q1 = ax * l; q2 = ay * l; q3 = az * l;
  } else {
    q0 = 1; q1 = q2 = q3 = 0;
  }
  double qq1 = 2 * q1 * q1, qq2 = 2 * q2 * q2, qq3 = 2 * q3 * q3;
  const double r[12] = {1 - qq2 - qq3, 2 * (q1 * q2 - q0 * q3), 2 * (q1 * q3 + q0 * q2), 0,
                        2 * (q1 * q2 + q0 * q3), 1 - qq1 - qq3, 2 * (q2 * q3 - q0 * q1), 0,
                        2 * (q1 * q3 - q0 * q2), 2 * (q2 * q3 + q0 * q1), 1 - qq1 - qq2, 0};
  memcpy(R, r, sizeof(r));
}

// rot_ztov (visualization.cpp:11-25): rotation taking z to v, stored as ODE rows.
void rot_z_to(double* R, const double* v) {
  double x1 = v[0], y1 = v[1], z1 = v[2];
  double a[3] = {y1 * 1.0 - z1 * 0.0, z1 * 0.0 - x1 * 1.0, x1 * 0.0 - y1 * 0.0};  // v x (0,0,1)
  double an = 0;
  for (int i = 0; i < 3; i++) an += a[i] * a[i];
  an = sqrt(an);
  if (an < 1e-10) { a[0] = 0; a[1] = 1; a[2] = 0; }
  double vn = 0;
  for (int i = 0; i < 3; i++) vn += v[i] * v[i];
  vn = sqrt(vn);
  double angle = asin(an / vn);
  double vz = 0;
  vz += v[0] * 0.0; vz += v[1] * 0.0; vz += v[2] * 1.0;
  if (vz < 0) angle = M_PI - angle;
  ode_axis_angle(R, a[0], a[1], a[2], angle);
}

struct XEl {
  std::string tag;
  std::vector<std::pair<std::string, std::string>> at;
  std::vector<int> kids;
};

struct XDoc {
  std::vector<XEl> el;
  const char* attr(int e, const char* k) const {
    for (auto& p : el[e].at) if (p.first == k) return p.second.c_str();
    return nullptr;
  }
  int child(int e, const char* tag) const {
    for (int k : el[e].kids) if (el[k].tag == tag) return k;
    return -1;
  }
};

bool xml_parse(const std::string& s, XDoc& d) {
  d.el.clear();
  d.el.push_back(XEl{"#doc", {}, {}});
  std::vector<int> open{0};
  size_t i = 0;
  while ((i = s.find('<', i)) != std::string::npos) {
    if (!s.compare(i, 4, "<!--")) { size_t e = s.find("-->", i); if (e == std::string::npos) return false; i = e + 3; continue; }
    if (!s.compare(i, 2, "<?") || !s.compare(i, 2, "<!")) { size_t e = s.find('>', i); if (e == std::string::npos) return false; i = e + 1; continue; }
    if (!s.compare(i, 2, "</")) {
      size_t e = s.find('>', i);
      if (e == std::string::npos || open.size() < 2) return false;
      open.pop_back();
      i = e + 1;
      continue;
    }
    size_t j = i + 1;
    while (j < s.size() && !isspace((unsigned char)s[j]) && s[j] != '>' && s[j] != '/') j++;
    XEl el;
    el.tag = s.substr(i + 1, j - i - 1);
    bool closed = false;
    for (;;) {
      while (j < s.size() && isspace((unsigned char)s[j])) j++;
      if (j >= s.size()) return false;
      if (s[j] == '/') { closed = true; j++; continue; }
      if (s[j] == '>') { j++; break; }
      size_t k = s.find('=', j);
      if (k == std::string::npos) return false;
      std::string key = s.substr(j, k - j);
      while (!key.empty() && isspace((unsigned char)key.back())) key.pop_back();
      size_t q = s.find_first_of("\"'", k);
      if (q == std::string::npos) return false;
      size_t qe = s.find(s[q], q + 1);
      if (qe == std::string::npos) return false;
      el.at.emplace_back(key, s.substr(q + 1, qe - q - 1));
      j = qe + 1;
    }
    int id = (int)d.el.size();
    d.el.push_back(el);
    d.el[open.back()].kids.push_back(id);
    if (!closed) open.push_back(id);
    i = j;
  }
  return open.size() == 1;
}

int parse_vals(const char* s, double* v, int n) {  // core.cpp:8-12 (stream extraction)
  if (!s) return 0;
  std::istringstream ss(s);
  int k = 0;
  while (k < n && (ss >> v[k])) k++;
  return k;
}

struct Build {
  const XDoc* d;
  hs_topo* t;
  std::vector<M4> Apj, JAp;
  std::vector<double> rcap;
  std::vector<M4> geomA;          // odepart::A_body_geom
  std::vector<int> gtype;         // HS_GEOM_*
  std::vector<double> gr, glen;   // radius, cylinder length
  std::vector<int> jtype, parent;
  std::vector<std::vector<int>> kids;
  int cfg = 0, nhinge = 0;
  std::vector<int> hinge_of;
  std::string err;

  int body(int e, int par) {
    int id = (int)Apj.size();
    if (id >= HS_NMAX) { err = "too many bodies"; return -1; }
    double pos[3] = {0, 0, 0};
    parse_vals(d->attr(e, "pos"), pos, 3);
    Apj.push_back(M4::translation(pos));
    JAp.push_back(M4::unity());
    rcap.push_back(0);
    gtype.push_back(HS_GEOM_NONE);
    gr.push_back(0);
    glen.push_back(0);
    jtype.push_back(HS_J_NONE);
    parent.push_back(par);
    kids.emplace_back();
    hinge_of.push_back(-1);
    hs_node& nd = t->node[id];
    memset(&nd, 0, sizeof(nd));
    nd.parent = par;
    nd.foot = -1;
    nd.hinge = -1;
    nd.owner_limb = -1;
    nd.limb_below = -1;
    M4 geom = M4::unity();
    double cap[3] = {0, 0, 0};
    int g = d->child(e, "geom");
    if (g >= 0) {
      const char* ty = d->attr(g, "type");
      std::string type = ty ? ty : "";
      if (type == "sphere") {
        double gp[3] = {0, 0, 0};
        parse_vals(d->attr(g, "pos"), gp, 3);
        geom = M4::translation(gp);
        gtype[id] = HS_GEOM_SPHERE;
        parse_vals(d->attr(g, "size"), &gr[id], 1);
      } else if (type == "capsule" || type == "cylinder") {
        double r = 0, ft[6] = {0, 0, 0, 0, 0, 0};
        parse_vals(d->attr(g, "size"), &r, 1);
        parse_vals(d->attr(g, "fromto"), ft, 6);
        double mid[3], dir[4];
        for (int i = 0; i < 3; i++) mid[i] = (ft[i] + ft[i + 3]) / 2.;
        for (int i = 0; i < 3; i++) dir[i] = ft[i + 3] - ft[i];
        double R[12];
        rot_z_to(R, dir);
        geom.set_rotation12(R);
        for (int i = 0; i < 3; i++) geom.a[12 + i] = mid[i];
        for (int i = 0; i < 3; i++) cap[i] = ft[i + 3];
        if (type == "capsule") rcap[id] = r;
        gtype[id] = (type == "capsule") ? HS_GEOM_CAPSULE : HS_GEOM_CYLINDER;
        gr[id] = r;
        double l2 = 0;  // extvec::norm of fromto[3:] - fromto[:3] (visualization.cpp:495-499)
        for (int i = 0; i < 3; i++) l2 += dir[i] * dir[i];
        glen[id] = sqrt(l2);
      }
    }
    geomA.push_back(geom);
    for (int i = 0; i < 3; i++) { nd.com[i] = geom.a[12 + i]; nd.cap[i] = cap[i]; }
    int j = d->child(e, "joint");
    if (j >= 0) {
      const char* ty = d->attr(j, "type");
      std::string type = ty ? ty : "";
      double jp[3] = {0, 0, 0};
      parse_vals(d->attr(j, "pos"), jp, 3);
      if (type == "free") {
        if (par >= 0) { err = "free joint below the root"; return -1; }
        M4 J = Apj[id];
        J.translate(jp);
        JAp[id] = J;
        double mj[3] = {-jp[0], -jp[1], -jp[2]};
        M4 P = M4::unity();
        P.translate(mj);
        Apj[id] = P;
        jtype[id] = HS_J_FREE;
        cfg += 6;
      } else if (type == "hinge") {
        double ax[3] = {0, 0, 1};
        parse_vals(d->attr(j, "axis"), ax, 3);
        double R[12];
        rot_z_to(R, ax);
        M4 A1;
        A1.set_rotation12(R);
        M4 J = Apj[id] * A1;
        J.translate(jp);
        JAp[id] = J;
        M4 P;
        P.set_rotation12(R);
        for (int i = 0; i < 3; i++) P.a[12 + i] = jp[i];
        P.invert_rigid();
        Apj[id] = P;
        jtype[id] = HS_J_HINGE;
        hinge_of[id] = nhinge++;
        cfg += 1;
      } else {
        err = "unsupported joint type " + type;
        return -1;
      }
    }
    for (int k : d->el[e].kids) {
      if (d->el[k].tag != "body") continue;
      int c = body(k, id);
      if (c < 0) return -1;
      kids[id].push_back(c);
    }
    return id;
  }
};

// The ODE world of the model (hs_simtopo.h): bodies oriented at the loaded configuration
// (all joint values 0), joints created in preorder, the static island order.
void build_sim(const Build& b, const hs_topo& t, hs_simtopo* s) {
  memset(s, 0, sizeof(*s));
  const int n = t.n;
  s->n = n;
  s->nmj = t.nmj;
  // A_ground at joint values 0 (model.cpp:183-201; E(0) is the identity, so A * E is exact)
  std::vector<M4> Ag(n), JAg(n);
  for (int i = 0; i < n; i++) {
    M4 A = (b.parent[i] < 0) ? M4::unity() : Ag[b.parent[i]];
    if (b.jtype[i] != HS_J_NONE) {
      JAg[i] = A * b.JAp[i];
      Ag[i] = JAg[i] * b.Apj[i];
    } else {
      Ag[i] = A * b.Apj[i];
    }
  }
  // orient_odebodys (model.cpp:295-305): pose of A_ground * A_body_geom, dBodySetRotation
  std::vector<double> pos(3 * n), q(4 * n), R(12 * n);
  for (int i = 0; i < n; i++) {
    M4 A = Ag[i] * b.geomA[i];
    double Rin[12];
    for (int r = 0; r < 3; r++) {
      for (int c = 0; c < 3; c++) Rin[r * 4 + c] = A.a[c * 4 + r];
      Rin[r * 4 + 3] = 0;
      pos[3 * i + r] = A.a[12 + r];
    }
    hsode::q_from_R(&q[4 * i], Rin);
    hsode::normalize4(&q[4 * i]);
    hsode::q_to_R(&q[4 * i], &R[12 * i]);
    s->gtype[i] = b.gtype[i];
    s->gr[i] = b.gr[i];
    s->glen[i] = b.glen[i];
    s->body_geom[i] = b.geomA[i].to34();
    s->mass[i] = 1.0;  // dBodyCreate: dMassSetParameters(1, 0,0,0, 1,1,1, 0,0,0)
    for (int k = 0; k < 3; k++) s->inertia[i][4 * k] = s->inv_inertia[i][4 * k] = 1.0;
    if (b.gtype[i] == HS_GEOM_SPHERE || b.gtype[i] == HS_GEOM_CAPSULE) s->n_coll++;
  }
  // kinematicmodel::set_ode_joints (model.cpp:375-400); per-body joint lists newest first
  std::vector<std::vector<int>> blist(n);
  int nj = 0, rows = 0;
  for (int p = 0; p < n; p++) {
    if (b.parent[p] < 0 || b.jtype[p] == HS_J_FREE) continue;
    hs_simjoint& J = s->joint[nj];
    J.motor = -1;
    if (b.jtype[p] == HS_J_HINGE) {  // odepart::make_hinge_joint (visualization.cpp:583-603)
      J.type = HS_SJ_HINGE;
      J.b1 = p;
      J.b2 = b.parent[p];
      double anc[3], ax[3], d1[3], d2[3];
      for (int i = 0; i < 3; i++) { anc[i] = JAg[p].a[12 + i]; ax[i] = JAg[p].a[8 + i]; }
      for (int i = 0; i < 3; i++) { d1[i] = anc[i] - pos[3 * J.b1 + i]; d2[i] = anc[i] - pos[3 * J.b2 + i]; }
      hsode::mul1_331(J.anchor1, &R[12 * J.b1], d1);  // setAnchors
      hsode::mul1_331(J.anchor2, &R[12 * J.b2], d2);
      hsode::normalize3(ax);  // setAxes
      hsode::mul1_331(J.axis1, &R[12 * J.b1], ax);
      hsode::mul1_331(J.axis2, &R[12 * J.b2], ax);
      hsode::qmul1(J.qrel, &q[4 * J.b1], &q[4 * J.b2]);
      J.motor = t.node[p].hinge;
      s->motor_joint[J.motor] = nj;
      rows += 5;
    } else {  // odepart::make_fixed_joint (visualization.cpp:572-579) + dJointSetFixed
      J.type = HS_SJ_FIXED;
      J.b1 = b.parent[p];
      J.b2 = p;
      hsode::qmul1(J.qrel, &q[4 * J.b1], &q[4 * J.b2]);
      double ofs[3];
      for (int i = 0; i < 3; i++) ofs[i] = pos[3 * J.b1 + i] - pos[3 * J.b2 + i];
      hsode::mul1_331(J.offset, &R[12 * J.b1], ofs);
      rows += 6;
    }
    blist[J.b1].insert(blist[J.b1].begin(), nj);  // addJointReferencesToBodies
    blist[J.b2].insert(blist[J.b2].begin(), nj);
    nj++;
  }
  s->nj = nj;
  s->m_max = rows + 3 * s->n_coll;
  // dxProcessIslands from the newest body (world body list is newest first); contacts attach to
  // the environment, so the visitation order is static
  std::vector<char> btag(n, 0), jtag(nj, 0);
  std::vector<int> stack;
  int nv = 0, ns = 0;
  for (int bb = n - 1; bb >= 0; bb--) {
    if (btag[bb]) continue;
    btag[bb] = 1;
    stack.push_back(bb);
    while (!stack.empty()) {
      int v = stack.back();
      stack.pop_back();
      s->jseq_start[nv] = ns;
      s->border[nv++] = v;
      for (int jid : blist[v]) {
        if (jtag[jid]) continue;
        jtag[jid] = 1;
        s->jseq[ns++] = jid;
        const hs_simjoint& J = s->joint[jid];
        int other = (J.b1 == v) ? J.b2 : J.b1;
        if (other >= 0 && !btag[other]) { btag[other] = 1; stack.push_back(other); }
      }
    }
  }
  s->jseq_start[nv] = ns;
  // dRand jump-ahead tables (misc.cpp: seed' = 1664525 seed + 1013904223 mod 2^32)
  s->lcg_a[0] = 1;
  s->lcg_c[0] = 0;
  for (int i = 1; i < HS_SIM_LCG; i++) {
    s->lcg_a[i] = s->lcg_a[i - 1] * 1664525u;
    s->lcg_c[i] = s->lcg_c[i - 1] * 1664525u + 1013904223u;
  }
  // dJointAddHingeTorque terms per body in motor order
  for (int j = 0; j < t.nmj; j++) {
    const hs_simjoint& J = s->joint[s->motor_joint[j]];
    for (int k = 0; k < 2; k++) {
      int bd = k == 0 ? J.b1 : J.b2;
      int c = s->tq_n[bd]++;
      s->tq_motor[bd][c] = j;
      s->tq_sign[bd][c] = k == 0 ? 1 : -1;
    }
  }
}

}  // namespace

int load_model_file(const char* path, int lik_variant, hs_topo* t, std::string& err, hs_simtopo* sim) {
  std::ifstream f(path);
  if (!f) { err = std::string("cannot open ") + path; return HS_E_IO; }
  std::stringstream ss;
  ss << f.rdbuf();
  XDoc d;
  if (!xml_parse(ss.str(), d)) { err = "malformed XML"; return HS_E_PARSE; }
  int mj = d.child(0, "mujoco");
  if (mj < 0) { err = "not a mujoco file"; return HS_E_PARSE; }
  int wb = d.child(mj, "worldbody");
  int root = wb >= 0 ? d.child(wb, "body") : -1;
  if (root < 0) { err = "no worldbody/body"; return HS_E_PARSE; }
  memset(t, 0, sizeof(*t));
  Build b;
  b.d = &d;
  b.t = t;
  if (b.body(root, -1) < 0) { err = b.err; return HS_E_TOPOLOGY; }
  int n = (int)b.Apj.size();
  if (b.jtype[0] != HS_J_FREE) { err = "root body needs a free joint"; return HS_E_TOPOLOGY; }

  // IK variant (lik.cpp:7-20, 44-78, 226-245)
  if (lik_variant < 0) {
    std::string p(path);
    size_t s = p.find_last_of('/');
    std::string base = s == std::string::npos ? p : p.substr(s + 1);
    if (base == "myant.xml") lik_variant = 0;
    else if (base == "hexapod.xml") lik_variant = 1;
    else if (base == "spider.xml") lik_variant = 2;
    else { err = "no limb IK solver for " + base; return HS_E_NOLIK; }
  }
  std::vector<int> tops;
  if (lik_variant == 0) tops = {2, 6, 10, 14};
  else if (lik_variant == 1) tops = {2, 5, 9, 12, 16, 19};
  else if (lik_variant == 2) tops = {1, 4, 7, 10, 13, 16};
  else { err = "bad lik variant"; return HS_E_NOLIK; }
  const double ls_yxx[3] = {.05, .4, .4}, ls_zxx[3] = {.1, .4, .4};
  t->lik_kind = lik_variant == 2 ? HS_LIK_ZXX : HS_LIK_YXX;
  memcpy(t->ls, lik_variant == 2 ? ls_zxx : ls_yxx, sizeof(t->ls));
  int nl = (int)tops.size();
  t->n_limbs = nl;
  t->torso_mask = 3;  // switch_torso_penalty(1,1), player.cpp:263
  static const int map4[4] = {0, 3, 1, 2}, map6[6] = {0, 3, 4, 1, 2, 5};  // pergen.cpp:243-262
  for (int L = 0; L < nl; L++) {
    int c = tops[L];
    if (c >= n) { err = "limb node out of range"; return HS_E_TOPOLOGY; }
    int v = c;
    for (int j = 0; j < 3; j++) {
      if (b.jtype[v] != HS_J_HINGE) { err = "limb link without hinge"; return HS_E_TOPOLOGY; }
      t->limb_node[L][j] = v;
      if (j < 2) {
        if (b.kids[v].empty()) { err = "limb too short"; return HS_E_TOPOLOGY; }
        v = b.kids[v][0];
      }
    }
    t->limb_child[L] = c;
    t->limb_parent[L] = b.parent[c];
    t->limb_foot[L] = v;
    t->limb_ysign[L] = (lik_variant == 0) ? (L < 2 ? 1 : -1) : (L % 2 == 0 ? 1 : -1);
    t->limb_pergen[L] = nl == 4 ? map4[L] : map6[L];
    if (nl != 4 && nl != 6) { err = "pergen needs 4 or 6 limbs"; return HS_E_TOPOLOGY; }
    std::vector<int> chain;
    for (int a = b.parent[c]; a >= 0; a = b.parent[a]) chain.insert(chain.begin(), a);
    for (size_t k = 1; k < chain.size(); k++)
      if (b.jtype[chain[k]] != HS_J_NONE) { err = "jointed body above a limb"; return HS_E_TOPOLOGY; }
    t->limb_chain_len[L] = (int)chain.size();
    for (size_t k = 0; k < chain.size(); k++) t->limb_chain[L][k] = chain[k];
    t->rcap = b.rcap[c + 2];  // lik.cpp:132-140 reads part (top + 2)
  }
  // ownership: which limb lane computes each node's kinematics
  for (int L = 0; L < nl; L++) {
    for (int k = 0; k < t->limb_chain_len[L]; k++) {
      int a = t->limb_chain[L][k];
      if (t->node[a].owner_limb < 0) t->node[a].owner_limb = L;
    }
    int v = t->limb_child[L];
    for (int j = 0; j < 3; j++) {
      if (t->node[v].owner_limb >= 0) { err = "limbs share a link"; return HS_E_TOPOLOGY; }
      t->node[v].owner_limb = L;
      if (j < 2) v = b.kids[v][0];
    }
  }
  for (int i = 0; i < n; i++)
    if (t->node[i].owner_limb < 0) { err = "body not on any limb chain"; return HS_E_TOPOLOGY; }

  // dynparts (periodic.cpp:34-58), feet in preorder
  t->n = n;
  t->cfg = b.cfg;
  t->nmj = b.cfg - 6;
  int nf = 0, nh = 0;
  t->total_mass = 0;
  for (int i = 0; i < n; i++) {
    hs_node& nd = t->node[i];
    nd.J_A_parent = b.JAp[i].to34();
    nd.A_pj_body = b.Apj[i].to34();
    nd.jtype = b.jtype[i];
    nd.nkids = (int)b.kids[i].size();
    if (nd.nkids > HS_CMAX) { err = "too many children"; return HS_E_TOPOLOGY; }
    for (int k = 0; k < nd.nkids; k++) nd.kids[k] = b.kids[i][k];
    nd.depth = nd.parent < 0 ? 0 : t->node[nd.parent].depth + 1;
    if (nd.depth > t->max_depth) t->max_depth = nd.depth;
    t->mass[i] = 1.0;  // dBodyCreate default mass (visualization.cpp:458, 485)
    t->total_mass += t->mass[i];
    for (int L = 0; L < nl; L++)
      if (t->limb_foot[L] == i) { nd.foot = nf; t->footis[nf++] = i; }
    if (nd.jtype == HS_J_HINGE) { nd.hinge = nh; t->hinge_ids[nh++] = i; }
  }
  t->nf = nf;
  // subtree sizes; the table is in preorder (every subtree one contiguous range), which the
  // rollout kernel's back-substitution relies on
  for (int i = n - 1; i >= 0; i--) {
    hs_node& nd = t->node[i];
    nd.size = 1;
    int next = i + 1;
    for (int k = 0; k < nd.nkids; k++) {
      if (nd.kids[k] != next) { err = "node table not in preorder"; return HS_E_TOPOLOGY; }
      nd.size += t->node[nd.kids[k]].size;
      next += t->node[nd.kids[k]].size;
    }
  }
  if (n > 0 && t->node[0].size != n) { err = "node table not one tree"; return HS_E_TOPOLOGY; }
  for (int j = 0; j < t->nmj; j++) {  // motor j's subtree as one packed range [h, h + size)
    const int h = t->hinge_ids[j];
    t->hinge_range[j] = h | ((h + t->node[h].size) << 8);
  }
  // the per-limb kinematics plan (hs_topo::limb_own*, link): the products in double, like every
  // topology entry (3x4 products summed as the kernels' mul, translation last)
  auto mul34 = [](const hs_aff34& A, const hs_aff34& B) {
    hs_aff34 C;
    for (int c = 0; c < 4; c++)
      for (int r = 0; r < 3; r++) {
        double s = 0;
        for (int k = 0; k < 3; k++) s = s + A.m[k * 3 + r] * B.m[c * 3 + k];
        if (c == 3) s = s + A.m[9 + r];
        C.m[c * 3 + r] = s;
      }
    return C;
  };
  auto mulp3 = [](const hs_aff34& A, const double* v, double* u) {
    for (int r = 0; r < 3; r++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s = s + A.m[k * 3 + r] * v[k];
      u[r] = s + A.m[9 + r];
    }
  };
  for (int L = 0; L < nl; L++) {
    int m = 0;
    hs_aff34 Q;  // pj of the chain bodies below the torso, multiplied in chain order
    for (int i = 0; i < 12; i++) Q.m[i] = (i % 4 == 0 && i < 9) ? 1.0 : 0.0;
    for (int k = 1; k < t->limb_chain_len[L]; k++) {
      const int v = t->limb_chain[L][k];
      Q = k == 1 ? t->node[v].A_pj_body : mul34(Q, t->node[v].A_pj_body);
      if (t->node[v].owner_limb != L) continue;
      if (m == HS_OWN_MAX) { err = "too many chain bodies on one limb"; return HS_E_TOPOLOGY; }
      if (t->node[v].foot >= 0) { err = "foot on a limb chain"; return HS_E_TOPOLOGY; }
      t->limb_own[L][m] = v;
      t->limb_own_rel[L][m] = Q;
      for (int i = 0; i < 3; i++) t->limb_own_com[L][m][i] = t->node[v].com[i];
      m++;
    }
    t->limb_own_n[L] = m;
    const hs_node& child = t->node[t->limb_child[L]];
    t->limb_hip_rel[L] = t->limb_chain_len[L] > 1 ? mul34(Q, child.J_A_parent) : child.J_A_parent;
    for (int i = 0; i < 3; i++) t->limb_child_t[L][i] = child.A_pj_body.m[9 + i];
    for (int k = 0; k < 3; k++) {
      const hs_node& nd = t->node[t->limb_node[L][k]];
      hs_link& lk = t->link[L][k];
      lk.P = k > 0 ? mul34(t->node[t->limb_node[L][k - 1]].A_pj_body, nd.J_A_parent) : hs_aff34{};
      for (int i = 0; i < 9; i++) lk.Rpj[i] = nd.A_pj_body.m[i];
      mulp3(nd.A_pj_body, nd.com, lk.com);
      mulp3(nd.A_pj_body, nd.cap, lk.cap);
      lk.foot = nd.foot;
      lk.hinge = nd.hinge;
    }
  }
  // each hinge may carry at most one foot below it (keeps the 1st-order Gram block diagonal)
  for (int fi = 0; fi < nf; fi++)
    for (int a = t->footis[fi]; a >= 0; a = t->node[a].parent) {
      hs_node& nd = t->node[a];
      if (nd.parent < 0) break;
      if (nd.limb_below == -1) nd.limb_below = fi;
      else if (nd.limb_below != fi) {
        if (nd.jtype == HS_J_HINGE) { err = "hinge above two feet"; return HS_E_TOPOLOGY; }
        nd.limb_below = -2;
      }
    }
  if (nf != nl) { err = "foot count"; return HS_E_TOPOLOGY; }
  for (int fi = 0; fi < nf; fi++) {
    int m = 0;
    for (int a = t->footis[fi]; a >= 0 && t->node[a].parent >= 0; a = t->node[a].parent) {
      if (m == HS_CHAIN_MAX) { err = "limb chain too long"; return HS_E_TOPOLOGY; }
      t->foot_chain[fi][m++] = a;
    }
    t->foot_chain_len[fi] = m;
    uint8_t b[8] = {(uint8_t)m, 0, 0, 0, 0, 0, 0, 0};
    for (int k = 0; k < m; k++) b[1 + k] = (uint8_t)t->foot_chain[fi][k];
    for (int w = 0; w < 2; w++)
      t->foot_chain8[fi][w] = (uint32_t)b[4 * w] | (uint32_t)b[4 * w + 1] << 8 | (uint32_t)b[4 * w + 2] << 16 |
                              (uint32_t)b[4 * w + 3] << 24;
  }
  for (int j = 0; j < nh; j++) t->hinge_foot[j] = t->node[t->hinge_ids[j]].limb_below;
  {  // hs_topo::limb_lane_ok
    bool ok = nl >= 1 && nl <= 7 && nf == nl && t->nmj == 3 * nl;
    uint32_t feet = 0;
    for (int L = 0; ok && L < nl; L++) {
      const int v0 = t->limb_node[L][0], f = t->node[t->limb_node[L][2]].foot;
      for (int k = 0; k < 3; k++) {
        const hs_node& nd = t->node[t->limb_node[L][k]];
        ok = ok && t->limb_node[L][k] == v0 + k && nd.size == 3 - k && nd.hinge >= 0 && nd.limb_below == f;
        ok = ok && ((k == 2) ? nd.foot >= 0 : nd.foot < 0);
      }
      ok = ok && f >= 0 && f < 32 && !((feet >> f) & 1) && t->limb_own_n[L] <= 1;
      if (ok) feet |= 1u << f;
    }
    t->limb_lane_ok = ok ? 1 : 0;
  }
  if (sim) {
    for (int i = 0; i < n; i++) {
      int nt = 0;
      for (int j = 0; j < t->nmj; j++) {
        int p = t->hinge_ids[j];
        if (p == i || b.parent[p] == i) nt++;
      }
      if (nt > HS_SIM_TQMAX) { err = "too many hinges on one body for the simulation tables"; return HS_E_TOPOLOGY; }
    }
    build_sim(b, *t, sim);
  }
  return HS_OK;
}

int read_pgs_config(const char* path, int setup_id, hs_gait_params* out, std::string& xml, std::string& err) {
  std::ifstream f(path);
  if (!f) { err = std::string("cannot open ") + path; return HS_E_IO; }
  std::string line;
  while (std::getline(f, line)) {  // modelplayer::get_rec_str (player.cpp:230-244)
    std::istringstream ls(line);
    int id;
    if (!(ls >> id) || id != setup_id) continue;
    memset(out, 0, sizeof(*out));
    out->foot_shift_type = -1;
    std::string key;
    while (ls >> key) {  // get_pgs_config_params (player.cpp:170-208)
      if (key == "xml_file") ls >> xml;
      else if (key == "torso_pos") ls >> out->torso_pos[0] >> out->torso_pos[1] >> out->torso_pos[2];
      else if (key == "torso_angles") ls >> out->torso_angles[0] >> out->torso_angles[1] >> out->torso_angles[2];
      else if (key == "step_duration") ls >> out->step_duration;
      else if (key == "period") ls >> out->period;
      else if (key == "step_length") ls >> out->step_length;
      else if (key == "step_height") ls >> out->step_height;
      else if (key == "curvature") ls >> out->curvature;
      else if (key == "lateral_foot_shift") { out->foot_shift_type = 0; ls >> out->foot_shift; }
      else if (key == "radial_foot_shift") { out->foot_shift_type = 1; ls >> out->foot_shift; }
      else { err = "unknown key " + key; return HS_E_PARSE; }
    }
    return HS_OK;
  }
  err = "no string with rec_id = " + std::to_string(setup_id);
  return HS_E_NOTFOUND;
}

}  // namespace hs
