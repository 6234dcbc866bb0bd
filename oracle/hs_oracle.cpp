// hs_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see hs_oracle.h).
//
// Line-by-line CPU restatement of the reference hot path, written without
// ODE, Eigen or rapidxml. Every function cites the reference file:line it
// restates; operation order follows the reference wherever it is observable
// in fp64 rounding (e.g. affine::mult sums k=0..3 from s=0, derivatives
// multiply by 1./(2*dt)).
//
// Third-party semantics restated (unpinned versions):
//   ODE  dRFromEulerAngles, dRFromAxisAndAngle (= dQFromAxisAndAngle + dQtoR),
//        default body mass (dMassSetParameters(1, 0,0,0, 1,1,1, 0,0,0)).
//   Eigen 3.3 FullPivLU (rank/threshold/solve/kernel/image), ColPivHouseholderQR
//        (nonzero-pivot rule, norm downdate, solve), Householder QR for the
//        SparseQR particular solve and null space (orthonormal basis).
#include "hs_oracle.h"

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <limits>
#include <map>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace {

// ---------------------------------------------------------------------------
// matrix.h / matrix.cpp restated: affine (4x4 column-major), extvec (4-vector)
// ---------------------------------------------------------------------------
struct Vec {  // extvec, matrix.h:61-88; default ctor sets w=1 (matrix.h:64)
  double v[4];
  Vec() { v[0] = v[1] = v[2] = 0; v[3] = 1; }
  Vec(double x, double y, double z) { v[0] = x; v[1] = y; v[2] = z; v[3] = 1; }
  void set(double x, double y, double z) { v[0] = x; v[1] = y; v[2] = z; }
  void set(const double* a) { for (int i = 0; i < 3; i++) v[i] = a[i]; }
  void set_zeros() { for (int i = 0; i < 3; i++) v[i] = 0; }
  void subtract(const Vec& u) { for (int i = 0; i < 4; i++) v[i] -= u.v[i]; }  // matrix.cpp:250-254
  void add(const Vec& u) { for (int i = 0; i < 3; i++) v[i] += u.v[i]; }       // matrix.cpp:318-323
  void times(double f) { for (int i = 0; i < 3; i++) v[i] *= f; }              // matrix.cpp:290-294
  double norm() const {  // matrix.cpp:256-261
    double s = 0;
    for (int i = 0; i < 3; i++) s += v[i] * v[i];
    return sqrt(s);
  }
  double dot(const Vec& u) const {  // matrix.cpp:303-309
    double s = 0;
    for (int i = 0; i < 3; i++) s += v[i] * u.v[i];
    return s;
  }
  void cross(const Vec& u, Vec& w) const {  // matrix.cpp:275-281
    double x1 = v[0], y1 = v[1], z1 = v[2], x2 = u.v[0], y2 = u.v[1], z2 = u.v[2];
    w.set(y1 * z2 - z1 * y2, z1 * x2 - x1 * z2, x1 * y2 - y1 * x2);
  }
  void normalize() {
    double len = norm();
    for (int i = 0; i < 3; i++) v[i] /= len;
  }
};

struct Aff {  // affine, matrix.h:27-55; a[j*4+i] = A(i,j)
  double a[16];
  void set_zeros() { for (int i = 0; i < 16; i++) a[i] = 0; }
  void set_unity() {  // matrix.cpp:12-19
    set_zeros();
    for (int i = 0; i < 4; i++) a[i * 5] = 1;
  }
  void set_translation(double x, double y, double z) {  // matrix.cpp:22-28
    set_unity();
    a[12] = x; a[13] = y; a[14] = z;
  }
  void set_translation(const double* v) { set_translation(v[0], v[1], v[2]); }
  void copy_transposed(const Aff& b) {  // matrix.cpp:65-75
    double* p = a;
    for (int i = 0; i < 4; i++) {
      const double* p1 = b.a + i;
      for (int j = 0; j < 4; j++) { *p++ = *p1; p1 += 4; }
    }
  }
  void mult(const Aff& b) {  // a *= b, matrix.cpp:78-97
    Aff c;
    c.copy_transposed(*this);
    double* p = a;
    const double* pb = b.a;
    for (int i = 0; i < 4; i++) {
      const double* pc = c.a;
      for (int j = 0; j < 4; j++) {
        double s = 0;
        const double* p1 = pc;
        const double* p2 = pb;
        for (int k = 0; k < 4; k++) s += (*p1++) * (*p2++);
        *p++ = s;
        pc += 4;
      }
      pb += 4;
    }
  }
  void mult(const Aff& b, Aff& c) const { c = *this; c.mult(b); }  // matrix.cpp:100-104
  void set_rotation(const double* rot12) {  // matrix.cpp:107-113 (dMatrix3 or affine)
    for (int i = 0; i < 12; i++) a[i] = rot12[i];
    for (int i = 12; i < 15; i++) a[i] = 0;
    a[15] = 1;
  }
  void translate(const Vec& t) { for (int i = 0; i < 3; i++) a[12 + i] += t.v[i]; }  // matrix.cpp:124-128
  void transpose() { Aff A; A.copy_transposed(*this); *this = A; }
  void set_a(int i, int j, double val) { a[j * 4 + i] = val; }
  double get_a(int i, int j) const { return a[j * 4 + i]; }
  void mult(const Vec& v, Vec& u) const {  // matrix.cpp:149-164, uses all 4 components
    for (int i = 0; i < 4; i++) {
      const double* p = a + i;
      double s = 0;
      for (int j = 0; j < 4; j++) { s += (*p) * v.v[j]; p += 4; }
      u.v[i] = s;
    }
  }
  void invert_rigidbody() {  // matrix.cpp:182-193
    Vec t, t1;
    for (int i = 0; i < 3; i++) { t.v[i] = -a[12 + i]; a[12 + i] = 0; }
    transpose();
    mult(t, t1);
    translate(t1);
  }
  void get_translation(Vec& t) const { for (int i = 0; i < 3; i++) t.v[i] = a[12 + i]; }
};

// ---------------------------------------------------------------------------
// ODE restated (rotation.cpp of ODE; double precision build assumed, makefile:9)
// dMatrix3 is row-major 3x4: R[i*4+j].
// ---------------------------------------------------------------------------
void dRFromEulerAngles(double* R, double phi, double theta, double psi) {
  double sphi = sin(phi), cphi = cos(phi), stheta = sin(theta), ctheta = cos(theta);
  double spsi = sin(psi), cpsi = cos(psi);
  R[0] = cpsi * ctheta;  R[1] = spsi * ctheta;  R[2] = -stheta; R[3] = 0;
  R[4] = cpsi * stheta * sphi - spsi * cphi;
  R[5] = spsi * stheta * sphi + cpsi * cphi;
  R[6] = ctheta * sphi;  R[7] = 0;
  R[8] = cpsi * stheta * cphi + spsi * sphi;
  R[9] = spsi * stheta * cphi - cpsi * sphi;
  R[10] = ctheta * cphi; R[11] = 0;
}

void dRFromAxisAndAngle(double* R, double ax, double ay, double az, double angle) {
  double q[4];
  double l = ax * ax + ay * ay + az * az;  // dQFromAxisAndAngle
  if (l > 0.0) {
    angle *= 0.5;
    q[0] = cos(angle);
    l = sin(angle) * (1.0 / sqrt(l));
    q[1] = ax * l; q[2] = ay * l; q[3] = az * l;
  } else {
    q[0] = 1; q[1] = q[2] = q[3] = 0;
  }
  double qq1 = 2 * q[1] * q[1], qq2 = 2 * q[2] * q[2], qq3 = 2 * q[3] * q[3];  // dQtoR
  R[0] = 1 - qq2 - qq3;          R[1] = 2 * (q[1] * q[2] - q[0] * q[3]);
  R[2] = 2 * (q[1] * q[3] + q[0] * q[2]); R[3] = 0;
  R[4] = 2 * (q[1] * q[2] + q[0] * q[3]); R[5] = 1 - qq1 - qq3;
  R[6] = 2 * (q[2] * q[3] - q[0] * q[1]); R[7] = 0;
  R[8] = 2 * (q[1] * q[3] - q[0] * q[2]); R[9] = 2 * (q[2] * q[3] + q[0] * q[1]);
  R[10] = 1 - qq1 - qq2;          R[11] = 0;
}

// visualization.cpp:11-25
void rot_ztov(double* rot, const Vec& v) {
  const Vec z(0, 0, 1);
  Vec a;
  v.cross(z, a);
  double anorm = a.norm();
  if (anorm < 1e-10) a.set(0, 1, 0);
  double angle = asin(anorm / v.norm());
  if (v.dot(z) < 0) angle = M_PI - angle;
  dRFromAxisAndAngle(rot, a.v[0], a.v[1], a.v[2], angle);
}

// visualization.cpp:54-60
void affine_from_posrot(Aff& A, const double* pos, const double* rot) {
  for (int i = 0; i < 12; i++) A.a[i] = rot[i];
  for (int i = 0; i < 3; i++) A.a[12 + i] = pos[i];
  A.a[15] = 1;
}

// visualization.cpp:62-69
void affine_from_orientation(Aff& A, const Vec* orientation) {
  double pos[4] = {orientation[0].v[0], orientation[0].v[1], orientation[0].v[2], 0};
  double rot[12];
  dRFromEulerAngles(rot, orientation[1].v[0], orientation[1].v[1], orientation[1].v[2]);
  affine_from_posrot(A, pos, rot);
}

// visualization.cpp:73-79
void mod_twopi(double& a) {
  if (a < -M_PI) {
    while (a < -M_PI) a += 2 * M_PI;
  } else if (a > M_PI) {
    while (a > M_PI) a -= 2 * M_PI;
  }
}

// visualization.cpp:81-101
void euler_angles_from_affine(const Aff& A, double* angles) {
  const double* p = A.a;
  double r11 = p[0], r21 = p[1], r31 = p[2], r32 = p[6], r33 = p[10];
  double th1 = -asin(r31);
  double ct1 = cos(th1);
  double ps1 = atan2(r32 / ct1, r33 / ct1);
  double ph1 = atan2(r21 / ct1, r11 / ct1);
  angles[0] = ps1; angles[1] = th1; angles[2] = ph1;
}

// ---------------------------------------------------------------------------
// Minimal XML reader for the MuJoCo subset (replaces rapidxml parse<0>:
// comments/declarations skipped, elements + attributes only).
// ---------------------------------------------------------------------------
struct XNode {
  std::string name;
  std::vector<std::pair<std::string, std::string>> attrs;
  std::vector<XNode*> kids;
  ~XNode() { for (auto* k : kids) delete k; }
  const char* attr(const char* n) const {
    for (auto& a : attrs) if (a.first == n) return a.second.c_str();
    return nullptr;
  }
  XNode* first(const char* n) const {
    for (auto* k : kids) if (k->name == n) return k;
    return nullptr;
  }
};

bool parse_xml(const std::string& s, XNode* root, std::string& err) {
  std::vector<XNode*> stack{root};
  size_t i = 0, n = s.size();
  while (i < n) {
    if (s[i] != '<') { i++; continue; }
    if (s.compare(i, 4, "<!--") == 0) {
      size_t e = s.find("-->", i + 4);
      if (e == std::string::npos) { err = "unterminated comment"; return false; }
      i = e + 3; continue;
    }
    if (s.compare(i, 2, "<?") == 0 || s.compare(i, 2, "<!") == 0) {
      size_t e = s.find('>', i);
      if (e == std::string::npos) { err = "bad declaration"; return false; }
      i = e + 1; continue;
    }
    if (s.compare(i, 2, "</") == 0) {
      size_t e = s.find('>', i);
      if (e == std::string::npos || stack.size() < 2) { err = "bad close tag"; return false; }
      stack.pop_back();
      i = e + 1; continue;
    }
    size_t j = i + 1;
    while (j < n && !isspace((unsigned char)s[j]) && s[j] != '>' && s[j] != '/') j++;
    XNode* node = new XNode;
    node->name = s.substr(i + 1, j - i - 1);
    stack.back()->kids.push_back(node);
    bool selfclose = false;
    while (j < n) {
      while (j < n && isspace((unsigned char)s[j])) j++;
      if (j >= n) { err = "eof in tag"; return false; }
      if (s[j] == '/') { selfclose = true; j++; continue; }
      if (s[j] == '>') { j++; break; }
      size_t k = j;
      while (k < n && s[k] != '=' && !isspace((unsigned char)s[k])) k++;
      std::string key = s.substr(j, k - j);
      while (k < n && s[k] != '"' && s[k] != '\'') k++;
      if (k >= n) { err = "bad attribute"; return false; }
      char q = s[k];
      size_t e = s.find(q, k + 1);
      if (e == std::string::npos) { err = "unterminated attribute"; return false; }
      node->attrs.emplace_back(key, s.substr(k + 1, e - k - 1));
      j = e + 1;
    }
    if (!selfclose) stack.push_back(node);
    i = j;
  }
  return true;
}

// core.cpp:8-12 (stringstream >> double until failure)
int str_to_vals(const char* str, double* val, int maxn) {
  std::stringstream ss;
  ss << str;
  int k = 0;
  double d;
  while (k < maxn && (ss >> d)) val[k++] = d;
  return k;
}

// ---------------------------------------------------------------------------
// model.h / model.cpp + odepart geometry (visualization.cpp:441-568)
// ---------------------------------------------------------------------------
enum { J_NONE = -1, J_FREE = 0, J_HINGE = 1 };

struct Node {
  Aff A_pj_body, A_ground;
  int parent = -1;
  std::vector<int> kids;
  int jtype = J_NONE;
  Aff J_A_parent, J_A_ground;
  double jval[6] = {0, 0, 0, 0, 0, 0};
  // odepart
  Aff A_body_geom;
  Vec capsule_to_pos;
  double rcap = 0;
  int gtype = 0;          // dGeomGetClass of the part's geom: 0 none, 1 sphere, 2 capsule, 3 cylinder
  double gr = 0, glen = 0;  // radius, cylinder length (dCreateSphere / dCreateCapsule, visualization.cpp:459,486)
  std::string name;
};

struct Limb {
  int child, parent;  // top-link node and its parent (lik.cpp:384-390)
  int vnode[3];       // nodes holding the three joint values (lik.cpp:393-400)
  int foot;           // child->first->first (lik.cpp:453-455)
  int ysign;
};

}  // namespace

struct hso_model {
  std::vector<Node> nodes;                // preorder = mnodes = odeparts order
  std::vector<std::pair<int, int>> jvals;  // (node, slot) in joint_values order
  std::string fname;                      // basename, keys the lik variant (lik.cpp:9-11)
  int lik_index = -1;
  std::vector<Limb> limbs;
  double rcap = 0;
  const double* ls = nullptr;
  // periodic::set_dynparts (periodic.cpp:34-58)
  std::vector<int> parentis, footis, hinge_ids;
  std::vector<double> masses;
  int n = 0, nf = 0, nmj = 0, cfg = 0;
  // forcetorquesolver::switch_torso_penalty (ftsolver.cpp:262-273): bit 0 = torso force rows, bit 1 =
  // torso torque rows in the zeroth-order stage (penal_mask0); the reference's only call is (1,1)
  // (player.cpp:263), main.cpp:87 passes (1, 0+1)
  int torso_mask = 3;
};

namespace {

const double limb_ls[] = {.05, .4, .4};   // lik.cpp:226
const double limb_ls1[] = {.1, .4, .4};   // lik.cpp:227

// modeljoint::transformation, model.cpp:37-62
void joint_transformation(const Node& nd, Aff& A) {
  if (nd.jtype == J_FREE) {
    Vec pos;
    pos.set(nd.jval);
    double rot[12];
    dRFromEulerAngles(rot, nd.jval[3], nd.jval[4], nd.jval[5]);
    A.set_rotation(rot);
    A.translate(pos);
  } else {
    double val = nd.jval[0];
    double c = cos(val), s = sin(val);
    A.set_unity();
    for (int i = 0; i < 2; i++) {
      A.set_a(i, i, c);
      A.set_a(i, 1 - i, (2 * i - 1) * s);
    }
  }
}

// modelnode::recompute_A_ground, model.cpp:183-201
void recompute_node(hso_model* m, int id, const Aff& A) {
  Node& nd = m->nodes[id];
  if (nd.jtype != J_NONE) {
    A.mult(nd.J_A_parent, nd.J_A_ground);
    nd.A_ground = nd.J_A_ground;
    Aff E;
    joint_transformation(nd, E);
    nd.A_ground.mult(E);
    nd.A_ground.mult(nd.A_pj_body);
  } else {
    nd.A_ground = A;
    nd.A_ground.mult(nd.A_pj_body);
  }
  for (int c : nd.kids) recompute_node(m, c, nd.A_ground);
}

// kinematicmodel::recompute_modelnodes, model.cpp:314-318
void recompute_modelnodes(hso_model* m) {
  Aff A;
  A.set_unity();
  recompute_node(m, 0, A);
}

double& jv(hso_model* m, int i) { return m->nodes[m->jvals[i].first].jval[m->jvals[i].second]; }

// odepart::capsule_lenposrot_from_fromto + make_ccylinder, visualization.cpp:475-504
void make_ccylinder(Node& nd, const XNode* g, bool capped) {
  double r = 0, fromto[6] = {0};
  if (const char* s = g->attr("size")) str_to_vals(s, &r, 1);
  if (const char* s = g->attr("fromto")) str_to_vals(s, fromto, 6);
  double pos[4];
  for (int i = 0; i < 3; i++) pos[i] = (fromto[i] + fromto[i + 3]) / 2.;
  Vec r1, r2;
  r1.set(fromto);
  r2.set(fromto + 3);
  r2.subtract(r1);
  double rot[12];
  rot_ztov(rot, r2);
  nd.capsule_to_pos.set(fromto + 3);
  affine_from_posrot(nd.A_body_geom, pos, rot);
  if (capped) nd.rcap = r;
  nd.gtype = capped ? 2 : 3;
  nd.gr = r;
  nd.glen = r2.norm();
}

// kinematicmodel::mnode_from_xnode, model.cpp:246-260 (+ make_odepart 264-271, make_joint 272-289)
int mnode_from_xnode(hso_model* m, const XNode* x, const Aff& A, int parent) {
  double pos[3] = {0, 0, 0};
  if (const char* s = x->attr("pos")) str_to_vals(s, pos, 3);
  int id = (int)m->nodes.size();
  m->nodes.emplace_back();
  {
    Node& nd = m->nodes[id];
    nd.A_pj_body.set_translation(pos);  // modelnode ctor, model.cpp:81-86
    nd.A_ground = A;
    nd.A_ground.mult(nd.A_pj_body);
    nd.parent = parent;
    if (const char* s = x->attr("name")) nd.name = s;
    nd.A_body_geom.set_unity();
    // make_odepart (visualization.cpp:442-470)
    const XNode* g = x->first("geom");
    if (g) {
      const char* t = g->attr("type");
      std::string type = t ? t : "";
      if (type == "sphere") {
        double r = 0, gp[3] = {0, 0, 0};
        if (const char* s = g->attr("size")) str_to_vals(s, &r, 1);
        if (const char* s = g->attr("pos")) str_to_vals(s, gp, 3);
        nd.A_body_geom.set_translation(gp);
        nd.gtype = 1;
        nd.gr = r;
      } else if (type == "capsule") {
        make_ccylinder(nd, g, true);
      } else if (type == "cylinder") {
        make_ccylinder(nd, g, false);
      }
    }
    // make_joint (model.cpp:272-289, 119-174)
    const XNode* j = x->first("joint");
    if (j) {
      const char* t = j->attr("type");
      std::string type = t ? t : "";
      double jp[3] = {0, 0, 0}, axis[3] = {0, 0, 1};
      if (const char* s = j->attr("pos")) str_to_vals(s, jp, 3);
      if (type == "free") {
        Vec p;
        p.set(jp);
        Aff J = nd.A_pj_body;
        J.translate(p);
        nd.J_A_parent = J;
        nd.jtype = J_FREE;
        J.set_unity();
        p.times(-1);
        J.translate(p);
        nd.A_pj_body = J;
        for (int k = 0; k < 6; k++) m->jvals.emplace_back(id, k);
      } else if (type == "hinge") {
        if (const char* s = j->attr("axis")) str_to_vals(s, axis, 3);
        Vec p, v;
        p.set(jp);
        v.set(axis);
        double rot[12];
        rot_ztov(rot, v);
        Aff A1;
        A1.set_rotation(rot);
        Aff J = nd.A_pj_body;
        J.mult(A1);
        J.translate(p);
        nd.J_A_parent = J;
        nd.jtype = J_HINGE;
        double pd[3] = {p.v[0], p.v[1], p.v[2]};
        affine_from_posrot(nd.A_pj_body, pd, rot);
        nd.A_pj_body.invert_rigidbody();
        m->jvals.emplace_back(id, 0);
      }
    }
  }
  Aff myA = m->nodes[id].A_ground;
  for (const XNode* c : x->kids) {
    if (c->name != "body") continue;
    int cid = mnode_from_xnode(m, c, myA, id);
    m->nodes[id].kids.push_back(cid);
  }
  return id;
}

// ---------------------------------------------------------------------------
// lik.cpp restated
// ---------------------------------------------------------------------------
// lik.cpp:142 global ignore_reach_flag -> per-thread flag
thread_local bool tl_ignore_reach = false;
thread_local bool tl_unreach = false;

// lik.cpp:151-184
bool limb_solver_yxx(const Vec& pos_limb, Vec& ja, const double* ls, int ysign, bool bend) {
  double l0 = ls[0], l1 = ls[1], l2 = ls[2];
  int s0 = ysign;
  int s1 = 2 * int(bend) - 1;
  Vec pos0(0, 0, s0 * l0);
  Vec pos1 = pos_limb;
  pos1.subtract(pos0);
  double l = pos1.norm();
  if (l1 + l2 - l < 0) {
    if (tl_ignore_reach) { l = l1 + l2; tl_unreach = true; }
    else return false;
  }
  double x1 = pos_limb.v[0], y1 = pos_limb.v[1], z1 = pos_limb.v[2];
  double c = (z1 - s0 * l0) / l;
  double phi = atan2(x1, y1);
  double theta = acos(c) + (1 - s0) * M_PI / 2;
  mod_twopi(phi);
  mod_twopi(theta);
  double ll = l * l;
  double del = l2 * l2 - l1 * l1;
  double beta = s1 * s0 * acos((ll - del) / (2 * l1 * l));
  double gamma = s1 * s0 * acos((ll + del) / (2 * l2 * l));
  ja.set(-phi, -theta + beta, -(beta + gamma));
  return true;
}

// lik.cpp:189-223
bool limb_solver_zxx(const Vec& pos_limb, Vec& ja, const double* ls, int ysign, bool bend) {
  double l0 = ls[0], l1 = ls[1], l2 = ls[2];
  int s0 = ysign;
  int s1 = 2 * int(bend) - 1;
  Vec pos0(0, 0, l0);
  Vec pos1 = pos_limb;
  pos1.add(pos0);
  double l = pos1.norm();
  if (l1 + l2 - l < 0) {
    if (tl_ignore_reach) { l = l1 + l2; tl_unreach = true; }
    else return false;
  }
  double x = pos_limb.v[0], y = pos_limb.v[1], z = pos_limb.v[2];
  double c = (z + l0) / l;
  double phi = atan2(x, y);
  double theta = acos(c) - s0 * M_PI / 2;
  mod_twopi(phi);
  mod_twopi(theta);
  double ll = l * l;
  double del = l2 * l2 - l1 * l1;
  double beta = s1 * acos((ll - del) / (2 * l1 * l));
  double gamma = s1 * acos((ll + del) / (2 * l2 * l));
  ja.set(-phi, -theta + beta, -(beta + gamma));
  return true;
}

// bend_solver_yxx, lik.cpp:248-272 (used only by the round-trip KAT)
bool bend_solver_yxx(Vec& pos, const Vec& angles, const double* ls, int ysign) {
  int s0 = ysign;
  double alpha0 = angles.v[0], alpha1 = angles.v[1], alpha2 = angles.v[2];
  double l0 = ls[0], l1 = ls[1], l2 = ls[2];
  int s1 = (alpha2 < 0) ? 1 : -1;
  double ca = cos(alpha2);
  double l = sqrt(l1 * l1 + l2 * l2 + 2 * l1 * l2 * ca);
  double theta = s1 * acos((l1 + l2 * ca) / l) - alpha1 + (1 - s0) * M_PI / 2;
  double phi = -alpha0;
  double stl = sin(theta) * l;
  pos.set(stl * sin(phi), stl * cos(phi), s0 * l0 + cos(theta) * l);
  return (alpha2 * s0 < 0);
}

bool limb_solve(const hso_model* m, int limbi, const Vec& pos_limb, Vec& ja, bool bend) {
  const Limb& L = m->limbs[limbi];
  if (m->lik_index == 2) return limb_solver_zxx(pos_limb, ja, m->ls, L.ysign, bend);
  return limb_solver_yxx(pos_limb, ja, m->ls, L.ysign, bend);
}

// liklimb::place_limb + poslimb, lik.cpp:316-347
bool place_limb(hso_model* m, int limbi, const Vec& pos_ground) {
  const Limb& L = m->limbs[limbi];
  Node& child = m->nodes[L.child];
  m->nodes[L.parent].A_ground.mult(child.J_A_parent, child.J_A_ground);  // joint->compute_A_ground
  Aff A = child.J_A_ground;
  A.invert_rigidbody();
  Vec pos_limb;
  A.mult(pos_ground, pos_limb);
  Vec ja;
  if (!limb_solve(m, limbi, pos_limb, ja, true)) return false;
  for (int i = 0; i < 3; i++) m->nodes[L.vnode[i]].jval[0] = ja.v[i];
  return true;
}

// kinematicmodel::set_jvalues_with_lik, model.cpp:354-359 -> liksolver::place_limbs lik.cpp:89-99
bool set_jvalues_with_lik(hso_model* m, const double* rec) {
  for (int i = 0; i < 6; i++) jv(m, i) = rec[i];
  recompute_modelnodes(m);
  const double* p = rec + 6;
  for (size_t i = 0; i < m->limbs.size(); i++) {
    Vec pg;
    pg.set(p);
    if (!place_limb(m, (int)i, pg)) return false;
    p += 3;
  }
  return true;
}

// ---------------------------------------------------------------------------
// pergen.cpp restated
// ---------------------------------------------------------------------------
struct PerGen {  // periodicgenerator, pergen.h:27-58
  int n = 0;
  double t_step = 0;
  std::vector<double> ts, xs;
  double period = 0, step_length = 0, step_height = 0;
  std::vector<Vec> limb_pos0s;
  double step_duration = 0, curvature = 0, max_radius = 0;

  void init(int n_) { n = n_; ts.assign(n, 0); xs.assign(n, 0); curvature = 0; }
  void set_step_duration(double f) {  // pergen.cpp:30-51
    t_step = f * (1. / 2 - 1. / n) + 1. / n;
    for (int i = 0; i < 2; i++) {
      int jmax = n / 2;
      int z = (jmax == 1) ? 1 : jmax - 1;
      for (int j = 0; j < jmax; j++) {
        int k = j + i * jmax;
        ts[k] = j * (1. / 2 - t_step) / z + double(i) / 2;
        xs[k] = ts[k] + t_step / 2 - 1. / 2;
      }
    }
    step_duration = f;
  }
  static double stepx(double t) { return (1 - cos(M_PI * t)) / 2; }  // pergen.cpp:62-64
  static double stepz(double t) { double a = sin(M_PI * t); return a * a; }  // pergen.cpp:68-71
  double step_frac(int limbi, double t) const {  // pergen.cpp:74-79
    double t_lift = ts[limbi];
    if (t < t_lift) return 0;
    else if (t < t_lift + t_step) return (t - t_lift) / t_step;
    else return 1;
  }
  void compute_max_radius() {  // pergen.cpp:143-153
    if (curvature == 0) return;
    Vec center(0, 1. / curvature, 0);
    max_radius = 0;
    for (auto& p : limb_pos0s) {
      double tmp[3];
      for (int i = 0; i < 3; i++) tmp[i] = p.v[i];
      for (int i = 0; i < 3; i++) tmp[i] -= center.v[i];
      double s = 0;
      for (int i = 0; i < 3; i++) s += tmp[i] * tmp[i];
      double rad = sqrt(s);
      if (rad > max_radius) max_radius = rad;
    }
  }
  void turn_position(const Vec& pos0, const Vec& delpos, Vec& pos) const {  // pergen.cpp:160-183
    double dx = delpos.v[0], dy = delpos.v[1], dz = delpos.v[2];
    if (curvature != 0) {
      int s = (curvature > 0) ? 1 : -1;
      double x0 = pos0.v[0], y0 = pos0.v[1];
      double rc = 1. / curvature;
      double rx = x0, ry = y0 - rc;
      double r = sqrt(rx * rx + ry * ry);
      double alpha = atan2(ry, rx);
      double beta = -s * dx / max_radius;
      double gamma = alpha - beta / 2;
      double sb = 2 * sin(beta / 2);
      dx = r * sin(gamma) * sb;
      dy += -r * cos(gamma) * sb;
    }
    Vec delpos1(dx, dy, dz);
    delpos1.add(pos0);
    pos = delpos1;
  }
  void limb_positions(double time, std::vector<Vec>& limb_poss) const {  // pergen.cpp:82-94
    double t = time / period;
    int t_int = int(t);
    double t_frac = t - t_int;
    for (int i = 0; i < n; i++) {
      double stepf = step_frac(i, t_frac);
      double delx = (t_int + xs[i] + stepx(stepf)) * step_length;
      double delz = stepz(stepf) * step_height;
      Vec delpos(delx, 0, delz);
      turn_position(limb_pos0s[i], delpos, limb_poss[i]);
    }
  }
  void get_turn_orientation(double dx, Vec* o) const {  // pergen.cpp:187-198
    if (curvature != 0) {
      int s = (curvature > 0) ? 1 : -1;
      double psi = s * dx / max_radius;
      double rc = 1. / curvature;
      o[0].set(rc * sin(psi), rc * (1 - cos(psi)), 0);
      o[1].set(0, 0, psi);
    } else {
      o[0].set(dx, 0, 0);
      o[1].set(0, 0, 0);
    }
  }
};

struct PGS {  // pergensetup, pergen.h:68-108
  int n = 0;
  PerGen pergen;
  std::vector<int> likpergen;
  std::vector<Vec> limb_poss;
  double v = 0;
  Vec torso_pos0, euler_angles;
  Aff rec_transform;              // pergen.h:75, set_unity at construction (pergen.cpp:206)
  bool rec_transform_flag = false;

  void init(int n_) {  // pergen.cpp:201-208, 243-262
    n = n_;
    rec_transform.set_unity();
    rec_transform_flag = false;
    pergen.init(n);
    limb_poss.assign(n, Vec());
    if (n == 4) likpergen = {0, 3, 1, 2};
    else if (n == 6) likpergen = {0, 3, 4, 1, 2, 5};
    else likpergen.clear();
  }
  void set_TLh(double T, double L, double h) {  // pergen.cpp:214-217
    pergen.period = T; pergen.step_length = L; pergen.step_height = h;
    v = L / T;
  }
  static void transform_orientation(const Aff& A, Vec* o) {  // pergen.cpp:377-383
    Aff A0, A1;
    affine_from_orientation(A0, o);
    A.mult(A0, A1);
    A1.get_translation(o[0]);
    euler_angles_from_affine(A1, o[1].v);
  }
  void turn_torso(double t, Vec* o) const {  // pergen.cpp:386-397
    double tv = t * v;
    Vec to[2];
    pergen.get_turn_orientation(tv, to);
    if (to[1].v[2] == 0) {
      o[0].v[0] += tv;
    } else {
      Aff A;
      affine_from_orientation(A, to);
      transform_orientation(A, o);
    }
  }
  void set_rec_transform(const Vec& rec_transl, const Vec& rec_eas) {  // pergen.cpp:316-320
    const Vec o[2] = {rec_transl, rec_eas};
    affine_from_orientation(rec_transform, o);
    rec_transform_flag = true;
  }
  void transform_rec(double* rec) const {  // pergen.cpp:323-335
    Vec o[2];
    o[0].set(rec);  // rec_to_orientation, pergen.cpp:365-368
    o[1].set(rec + 3);
    transform_orientation(rec_transform, o);
    for (int i = 0; i < 3; i++) { rec[i] = o[0].v[i]; rec[3 + i] = o[1].v[i]; }  // orientation_to_rec
    for (int i = 0; i < n; i++) {
      Vec pos0, pos;
      double* p = rec + 6 + i * 3;
      pos0.set(p);
      rec_transform.mult(pos0, pos);
      for (int c = 0; c < 3; c++) p[c] = pos.v[c];
    }
  }
  void set_rec(double* rec, double t) {  // pergen.cpp:225-239
    Vec o[2] = {torso_pos0, euler_angles};
    turn_torso(t, o);
    for (int i = 0; i < 3; i++) { rec[i] = o[0].v[i]; rec[3 + i] = o[1].v[i]; }
    pergen.limb_positions(t, limb_poss);
    for (int i = 0; i < n; i++) {
      int j = likpergen[i];
      for (int c = 0; c < 3; c++) rec[6 + i * 3 + c] = limb_poss[j].v[c];
    }
    if (rec_transform_flag) transform_rec(rec);
  }
};

// pgssweeper::setup_pergen / partial_setup_pergen / setup_foot_shift / shift_pos0,
// pergen.cpp:453-507 (kinematicmodel::orient_torso model.cpp:394-400)
void setup_pergen(hso_model* m, PGS& pgs, const hso_gait* g) {
  pgs.init((int)m->limbs.size());
  Vec orientation[2];
  orientation[0].set(g->torso_pos);
  orientation[1].set(g->torso_angles);
  for (int i = 0; i < 2; i++)
    for (int j = 0; j < 3; j++) jv(m, j + i * 3) = orientation[i].v[j];
  recompute_modelnodes(m);
  pgs.pergen.set_step_duration(g->step_duration);
  double rcap = m->rcap;
  int shift_type = g->foot_shift_type;
  Vec lat_shift;
  double rad_shift = 0;
  if (shift_type == 0) {
    Vec shift(0, g->foot_shift, 0);
    m->nodes[0].A_ground.mult(shift, lat_shift);
  } else if (shift_type == 1) {
    rad_shift = g->foot_shift;
  }
  for (int i = 0; i < pgs.n; i++) {
    Vec pos;
    m->nodes[m->limbs[i].child].A_ground.get_translation(pos);  // get_limb_hip_pos
    if (shift_type >= 0) {
      Vec delpos;
      if (shift_type == 0) {
        delpos = lat_shift;
        if (i % 2) delpos.times(-1);
      } else if (shift_type == 1) {
        double x = pos.v[0], y = pos.v[1];
        double f = rad_shift / sqrt(x * x + y * y);
        delpos.set(x * f, y * f, 0);
      }
      pos.add(delpos);
    }
    Vec pos0 = pos;  // set_limb_poss, pergen.cpp:268-275
    pos0.v[2] = rcap;
    pgs.limb_poss[pgs.likpergen[i]] = pos0;
  }
  pgs.pergen.limb_pos0s = pgs.limb_poss;  // set_pos0s
  pgs.pergen.compute_max_radius();
  pgs.torso_pos0 = orientation[0];
  pgs.euler_angles = orientation[1];
  pgs.set_TLh(g->period, g->step_length, g->step_height);
  pgs.pergen.curvature = g->curvature;  // set_curvature
  pgs.pergen.compute_max_radius();
  // the gait's record transform (set_rec_transform / set_rec_rotation, pergen.cpp:309-320; a sweep
  // copies it from the swept setup, copy_rec_transform, pergen.cpp:338-342, 446)
  if (g->rec_transform_flag)
    pgs.set_rec_transform(Vec(g->rec_transl[0], g->rec_transl[1], g->rec_transl[2]),
                          Vec(g->rec_eas[0], g->rec_eas[1], g->rec_eas[2]));
}

// ---------------------------------------------------------------------------
// dynrec.cpp restated
// ---------------------------------------------------------------------------
struct DynRec {  // dynrecord, dynrec.h:76-106
  int n = 0, nf = 0;
  std::vector<Vec> pos, jpos, vel, mom, mom_rate, acc, ust, ang_vel, ang_mom, ang_mom_rate, fpos, jzaxis;
  std::vector<Aff> rot;
  std::vector<char> contacts;
  void init(int n_, int nf_) {
    n = n_; nf = nf_;
    for (auto* v : {&pos, &jpos, &vel, &mom, &mom_rate, &acc, &ust, &ang_vel, &ang_mom, &ang_mom_rate, &jzaxis})
      v->assign(n, Vec());
    fpos.assign(nf, Vec());
    rot.assign(n, Aff());
    contacts.assign(nf, 0);
  }
  int ncontacts() const { int s = 0; for (char c : contacts) s += c; return s; }
};

// dynpart::recompute + dynrecord::initialize, dynrec.cpp:31-51, 79-93, 134-155
void dynrec_initialize(hso_model* m, DynRec& d, double rcap) {
  int fi = 0;
  for (int i = 0; i < m->n; i++) {
    const Node& nd = m->nodes[i];
    Vec jpos, com, pos_body;
    if (nd.jtype != J_NONE) nd.J_A_ground.get_translation(jpos);
    else nd.A_ground.get_translation(jpos);
    nd.A_body_geom.get_translation(pos_body);
    nd.A_ground.mult(pos_body, com);
    d.pos[i] = com;
    d.jpos[i] = jpos;
    const Aff& A = nd.A_ground;
    double x = (A.get_a(2, 1) - A.get_a(1, 2)) / 2;
    double y = (A.get_a(0, 2) - A.get_a(2, 0)) / 2;
    double z = (A.get_a(1, 0) - A.get_a(0, 1)) / 2;
    d.ust[i].set(x, y, z);
    d.rot[i].set_rotation(A.a);
    if (fi < m->nf && m->footis[fi] == i) {
      Vec fp;
      nd.A_ground.mult(nd.capsule_to_pos, fp);
      d.fpos[fi] = fp;
      d.contacts[fi] = (fp.v[2] < rcap + 1e-4);
      fi++;
    }
    if (nd.jtype != J_NONE) d.jzaxis[i].set(nd.J_A_ground.a + 8);
    else d.jzaxis[i].set_zeros();
  }
}

// dynrec.cpp:193-203
void compute_ders_field(int n, std::vector<Vec>& der, const std::vector<Vec>& prev, const std::vector<Vec>& next, double dt) {
  for (int i = 0; i < n; i++) {
    der[i] = next[i];
    der[i].subtract(prev[i]);
    der[i].times(1. / (2 * dt));
  }
}

// dynrec.cpp:175-189, 205-224
void compute_ders(hso_model* m, DynRec& d, int stage, const DynRec& prev, const DynRec& next, double dt) {
  if (stage == 0) {
    compute_ders_field(d.n, d.vel, prev.pos, next.pos, dt);
    compute_ders_field(d.n, d.ang_vel, prev.ust, next.ust, dt);
    for (int i = 0; i < d.n; i++) { d.mom[i] = d.vel[i]; d.mom[i].times(m->masses[i]); }
    Aff A_I;  // dBodyGetMass default: I = identity (dMassSetParameters(1,0,0,0,1,1,1,0,0,0))
    double I12[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
    A_I.set_rotation(I12);
    for (int i = 0; i < d.n; i++) {
      Vec v, u;
      Aff rot_tr;
      rot_tr.copy_transposed(d.rot[i]);
      rot_tr.mult(d.ang_vel[i], v);
      A_I.mult(v, u);
      d.rot[i].mult(u, d.ang_mom[i]);
    }
  } else {
    compute_ders_field(d.n, d.mom_rate, prev.mom, next.mom, dt);
    compute_ders_field(d.n, d.acc, prev.vel, next.vel, dt);
    compute_ders_field(d.n, d.ang_mom_rate, prev.ang_mom, next.ang_mom, dt);
  }
}

// ---------------------------------------------------------------------------
// Dense linear algebra with Eigen 3.3 semantics
// Column-major storage: M[i + j*ld].
// ---------------------------------------------------------------------------
struct Mat {
  int r = 0, c = 0;
  std::vector<double> d;
  Mat() {}
  Mat(int r_, int c_) : r(r_), c(c_), d((size_t)r_ * c_, 0.0) {}
  double& operator()(int i, int j) { return d[(size_t)i + (size_t)j * r]; }
  double operator()(int i, int j) const { return d[(size_t)i + (size_t)j * r]; }
  const double* ptr(int i, int j) const { return &d[(size_t)i + (size_t)j * r]; }
};

Mat matmul(const Mat& A, const Mat& B) {
  Mat C(A.r, B.c);
  for (int j = 0; j < B.c; j++)
    for (int k = 0; k < A.c; k++) {
      double b = B(k, j);
      for (int i = 0; i < A.r; i++) C(i, j) += A(i, k) * b;
    }
  return C;
}
std::vector<double> matvec(const Mat& A, const std::vector<double>& x) {
  std::vector<double> y(A.r, 0.0);
  for (int k = 0; k < A.c; k++)
    for (int i = 0; i < A.r; i++) y[i] += A(i, k) * x[k];
  return y;
}
Mat transpose(const Mat& A) {
  Mat T(A.c, A.r);
  for (int i = 0; i < A.r; i++)
    for (int j = 0; j < A.c; j++) T(j, i) = A(i, j);
  return T;
}
double vnorm(const std::vector<double>& v) {
  double s = 0;
  for (double x : v) s += x * x;
  return sqrt(s);
}

// Householder reflector (Eigen MatrixBase::makeHouseholder, Householder.h)
void make_householder(double* col, int len, int stride, double& tau, double& beta) {
  double c0 = col[0];
  double tail = 0;
  for (int i = 1; i < len; i++) tail += col[i * stride] * col[i * stride];
  if (len == 1 || tail <= DBL_MIN) {
    tau = 0; beta = c0;
    for (int i = 1; i < len; i++) col[i * stride] = 0;
  } else {
    beta = sqrt(c0 * c0 + tail);
    if (c0 >= 0) beta = -beta;
    double den = c0 - beta;
    for (int i = 1; i < len; i++) col[i * stride] /= den;
    tau = (beta - c0) / beta;
  }
}

// Apply H = I - tau v v^T (v = [1; ess]) on the left of rows k.. of columns [c0,c1) of M.
void apply_householder_left(Mat& M, int k, const double* ess, double tau, int c0, int c1) {
  int rows = M.r - k;
  if (rows == 1) {
    for (int j = c0; j < c1; j++) M(k, j) *= (1 - tau);
    return;
  }
  if (tau == 0) return;
  for (int j = c0; j < c1; j++) {
    double tmp = 0;
    for (int i = 1; i < rows; i++) tmp += ess[i - 1] * M(k + i, j);
    tmp += M(k, j);
    M(k, j) -= tau * tmp;
    for (int i = 1; i < rows; i++) M(k + i, j) -= tau * ess[i - 1] * tmp;
  }
}

// Unpivoted Householder QR in place (A = Q R); hcoeffs stored; essential parts below diag.
struct HQR {
  Mat qr;
  std::vector<double> tau;
  void compute(const Mat& A) {
    qr = A;
    int size = std::min(qr.r, qr.c);
    tau.assign(size, 0);
    std::vector<double> ess;
    for (int k = 0; k < size; k++) {
      double beta;
      make_householder(&qr(k, k), qr.r - k, 1, tau[k], beta);
      qr(k, k) = beta;
      ess.assign(&qr(k, k) + 1, &qr(k, k) + (qr.r - k));
      apply_householder_left(qr, k, ess.data(), tau[k], k + 1, qr.c);
    }
  }
  // Q * e (apply H_{size-1} ... H_0 in reverse order)
  std::vector<double> apply_Q(std::vector<double> e) const {
    int size = (int)tau.size();
    Mat col(qr.r, 1);
    for (int i = 0; i < qr.r; i++) col(i, 0) = e[i];
    for (int k = size - 1; k >= 0; k--)
      apply_householder_left(col, k, qr.ptr(k, k) + 1, tau[k], 0, 1);
    for (int i = 0; i < qr.r; i++) e[i] = col(i, 0);
    return e;
  }
  std::vector<double> apply_Qt(std::vector<double> b) const {
    int size = (int)tau.size();
    Mat col(qr.r, 1);
    for (int i = 0; i < qr.r; i++) col(i, 0) = b[i];
    for (int k = 0; k < size; k++) apply_householder_left(col, k, qr.ptr(k, k) + 1, tau[k], 0, 1);
    for (int i = 0; i < qr.r; i++) b[i] = col(i, 0);
    return b;
  }
  // solve square full-rank system via R^{-1} Q^T b
  std::vector<double> solve(const std::vector<double>& b) const {
    std::vector<double> c = apply_Qt(b);
    int n = qr.c;
    for (int i = n - 1; i >= 0; i--) {
      c[i] /= qr(i, i);
      for (int r = 0; r < i; r++) c[r] -= c[i] * qr(r, i);
    }
    c.resize(n);
    return c;
  }
};

// upper-triangular solve in place, column-oriented (Eigen triangular_solve_vector, Upper)
void upper_solve_inplace(const Mat& U, int n, double* x) {
  for (int i = n - 1; i >= 0; i--) {
    if (x[i] != 0) {
      x[i] /= U(i, i);
      for (int r = 0; r < i; r++) x[r] -= x[i] * U(r, i);
    }
  }
}

// Decisions taken within rounding of a threshold (hard part 2:
// such samples are flagged, not silently compared). Each decision the solve takes against a
// threshold reports its margin: |log(value / threshold)| / log(band), so a margin <= 1 means the
// value lies within the decision's band of its threshold, where another rounding (another basis,
// FMA contraction, single precision) may decide the other way:
//   FullPivLU rank (ftsolver.cpp:208-214, Eigen's |u_ii| > maxpivot * thr): every pivot, band 4
//   threshold doubled (ftsolver.cpp:212-214: setThreshold(2 thr) while rank > rank0): margin 0
//   rel_error > 1e-6 (ftsolver.cpp:228-232): band 10, i.e. rel_error in [1e-7, 1e-5]
//   ColPivHouseholderQR nonzero pivots (|col|^2 < threshold_helper (rows - k)): band 16 on the squares
//   the closed form's routing: the collinearity guard (band 4) and its pivot guards (band 4)
// and one conditioning test: the second stage's system (the last pass's m, ftsolver.cpp:222-227) with a
// kept ColPivQR pivot under kCondQR of its first (a condition number above 1e7: a rounding-level change
// of the inputs -- another basis, FMA contraction -- moves the answer by more than the parity bound;
// the reference's own SparseQR and tree bases disagree there, tests/test_oracle.py).
// The step then carries HSO_FLAG_NEAR_RANK (the kernel computes the same margins, HS_FLAG_NEAR_RANK).
constexpr double kNearBand = 4.0, kNearBandRel = 10.0, kNearBandQR = 16.0, kCondQR = 1e-7;
struct NearTrack {
  double margin = INFINITY;
  int cat = 0;  // the decision closest to its threshold: HSO_NEAR_*
  double lu_kept = INFINITY, qr_kept = INFINITY;  // conditioning of the last pass: smallest kept pivot ratios
  bool ill = false;                               // the last pass's qr_kept < kCondQR
#ifndef HSO_FLOPCOUNT
  void note(double ratio, double band, int c) {
    if (!(ratio > 0)) return;  // exact zeros are structural, not near anything
    const double m = fabs(log(ratio)) / log(band);
    if (m < margin) { margin = m; cat = c; }
  }
#endif
  bool near() const { return margin <= 1.0 || ill; }
};
thread_local NearTrack tl_near;
// diagnostics, not arithmetic of the path: the FLOP-counting build (hs_oracle_flops.cpp) leaves them out
#ifdef HSO_FLOPCOUNT
#define NEAR_NOTE(ratio, band, cat) ((void)0)
#else
#define NEAR_NOTE(ratio, band, cat) tl_near.note((ratio), (band), (cat))
#endif
enum { HSO_NEAR_LU = 1, HSO_NEAR_DOUBLED = 2, HSO_NEAR_REL = 3, HSO_NEAR_QR = 4, HSO_NEAR_COLLINEAR = 5,
       HSO_NEAR_PIVOT = 6, HSO_NEAR_COND = 7 };

// Eigen FullPivLU (FullPivLU.h), restated.
struct FPLU {
  int n = 0;
  Mat lu;
  std::vector<int> rowsT, colsT, q;
  int nonzero_pivots = 0;
  double maxpivot = 0;
  bool prescribed = false;
  double prescribed_thr = 0;
  void compute(const Mat& A) {
    n = A.r;
    lu = A;
    rowsT.assign(n, 0);
    colsT.assign(n, 0);
    nonzero_pivots = n;
    maxpivot = 0;
    for (int k = 0; k < n; k++) {
      int bi = k, bj = k;
      double best = fabs(lu(k, k));
      for (int j = k; j < n; j++)
        for (int i = k; i < n; i++) {
          double s = fabs(lu(i, j));
          if (s > best) { best = s; bi = i; bj = j; }
        }
      if (best == 0) {
        nonzero_pivots = k;
        for (int i = k; i < n; i++) { rowsT[i] = i; colsT[i] = i; }
        break;
      }
      if (best > maxpivot) maxpivot = best;
      rowsT[k] = bi;
      colsT[k] = bj;
      if (k != bi) for (int j = 0; j < n; j++) std::swap(lu(k, j), lu(bi, j));
      if (k != bj) for (int i = 0; i < n; i++) std::swap(lu(i, k), lu(i, bj));
      if (k < n - 1) {
        double p = lu(k, k);
        for (int i = k + 1; i < n; i++) lu(i, k) /= p;
        for (int j = k + 1; j < n; j++)
          for (int i = k + 1; i < n; i++) lu(i, j) -= lu(i, k) * lu(k, j);
      }
    }
    q.resize(n);
    for (int i = 0; i < n; i++) q[i] = i;
    for (int k = 0; k < n; k++) std::swap(q[k], q[colsT[k]]);
  }
  double threshold() const { return prescribed ? prescribed_thr : DBL_EPSILON * (double)n; }
  void set_threshold(double t) { prescribed = true; prescribed_thr = t; }
  int rank() const {
    double thr = fabs(maxpivot) * threshold();
    int r = 0;
    for (int i = 0; i < nonzero_pivots; i++) r += (fabs(lu(i, i)) > thr);
    return r;
  }
  std::vector<int> pivots() const {
    double thr = maxpivot * threshold();
    std::vector<int> p;
    for (int i = 0; i < nonzero_pivots; i++)
      if (fabs(lu(i, i)) > thr) p.push_back(i);
    return p;
  }
  std::vector<double> solve(const std::vector<double>& rhs) const {
    int r = rank();
    std::vector<double> dst(n, 0.0);
    if (r == 0) return dst;
    std::vector<double> c = rhs;
    for (int k = 0; k < n; k++) std::swap(c[k], c[rowsT[k]]);  // P * rhs
    for (int j = 0; j < n; j++)  // unit lower solve (column oriented)
      for (int i = j + 1; i < n; i++) c[i] -= c[j] * lu(i, j);
    upper_solve_inplace(lu, r, c.data());
    for (int i = 0; i < r; i++) dst[q[i]] = c[i];
    return dst;
  }
  // kernel: n x (n-r) basis; 0 columns when full rank (the reference would get one zero column)
  Mat kernel() const {
    int r = rank();
    int dimker = n - r;
    Mat dst(n, dimker);
    if (dimker == 0) return dst;
    std::vector<int> piv = pivots();
    Mat mm(r, n);
    for (int i = 0; i < r; i++)
      for (int j = i; j < n; j++) mm(i, j) = lu(piv[i], j);
    for (int i = 0; i < r; i++)
      if (piv[i] != i) for (int row = 0; row < r; row++) std::swap(mm(row, i), mm(row, piv[i]));
    for (int col = r; col < n; col++) {
      std::vector<double> x(r);
      for (int i = 0; i < r; i++) x[i] = mm(i, col);
      upper_solve_inplace(mm, r, x.data());
      for (int i = 0; i < r; i++) mm(i, col) = x[i];
    }
    for (int i = r - 1; i >= 0; i--)
      if (piv[i] != i) for (int row = 0; row < r; row++) std::swap(mm(row, i), mm(row, piv[i]));
    for (int i = 0; i < r; i++)
      for (int k = 0; k < dimker; k++) dst(q[i], k) = -mm(i, r + k);
    for (int i = r; i < n; i++) for (int k = 0; k < dimker; k++) dst(q[i], k) = 0;
    for (int k = 0; k < dimker; k++) dst(q[r + k], k) = 1;
    return dst;
  }
  // image: columns of the original matrix at the pivot columns
  Mat image(const Mat& orig) const {
    int r = rank();
    Mat dst(n, r);
    std::vector<int> piv = pivots();
    for (int i = 0; i < r; i++)
      for (int row = 0; row < n; row++) dst(row, i) = orig(row, q[piv[i]]);
    return dst;
  }
};

// Eigen 3.3 ColPivHouseholderQR (ColPivHouseholderQR.h), restated.
struct CPQR {
  Mat qr;
  std::vector<double> hc;
  std::vector<int> perm;
  int nonzero_pivots = 0;
  void compute(const Mat& A) {
    qr = A;
    int rows = qr.r, cols = qr.c, size = std::min(rows, cols);
    hc.assign(size, 0);
    std::vector<int> colsT(cols, 0);
    std::vector<double> nu(cols), nd(cols);
    for (int k = 0; k < cols; k++) {
      double s = 0;
      for (int i = 0; i < rows; i++) s += qr(i, k) * qr(i, k);
      nd[k] = sqrt(s);
      nu[k] = nd[k];
    }
    double mx = 0;
    for (int k = 0; k < cols; k++) mx = std::max(mx, nu[k]);
    double th = mx * DBL_EPSILON;
    double threshold_helper = th * th / (double)rows;
    double norm_downdate_threshold = sqrt(DBL_EPSILON);
    nonzero_pivots = size;
    std::vector<double> ess;
    for (int k = 0; k < size; k++) {
      int bi = k;
      double bv = nu[k];
      for (int j = k + 1; j < cols; j++)
        if (nu[j] > bv) { bv = nu[j]; bi = j; }
      double bsq = bv * bv;
      if (nonzero_pivots == size) NEAR_NOTE(bsq / (threshold_helper * (double)(rows - k)), kNearBandQR, HSO_NEAR_QR);
      if (nonzero_pivots == size && bsq < threshold_helper * (double)(rows - k)) nonzero_pivots = k;
      colsT[k] = bi;
      if (k != bi) {
        for (int i = 0; i < rows; i++) std::swap(qr(i, k), qr(i, bi));
        std::swap(nu[k], nu[bi]);
        std::swap(nd[k], nd[bi]);
      }
      double beta;
      make_householder(&qr(k, k), rows - k, 1, hc[k], beta);
      qr(k, k) = beta;
      ess.assign(&qr(k, k) + 1, &qr(k, k) + (rows - k));
      apply_householder_left(qr, k, ess.data(), hc[k], k + 1, cols);
      for (int j = k + 1; j < cols; j++) {
        if (nu[j] != 0) {
          double temp = fabs(qr(k, j)) / nu[j];
          temp = (1 + temp) * (1 - temp);
          temp = temp < 0 ? 0 : temp;
          double ratio = nu[j] / nd[j];
          double temp2 = temp * (ratio * ratio);  // temp * abs2(nu/nd)
          if (temp2 <= norm_downdate_threshold) {
            double s = 0;
            for (int i = k + 1; i < rows; i++) s += qr(i, j) * qr(i, j);
            nd[j] = sqrt(s);
            nu[j] = nd[j];
          } else {
            nu[j] *= sqrt(temp);
          }
        }
      }
    }
    perm.resize(cols);
    for (int i = 0; i < cols; i++) perm[i] = i;
    for (int k = 0; k < size; k++) std::swap(perm[k], perm[colsT[k]]);
  }
  std::vector<double> solve(const std::vector<double>& b) const {
    int cols = qr.c, np = nonzero_pivots;
    std::vector<double> dst(cols, 0.0);
    if (np == 0) return dst;
    Mat c(qr.r, 1);
    for (int i = 0; i < qr.r; i++) c(i, 0) = b[i];
    for (int k = 0; k < np; k++) apply_householder_left(c, k, qr.ptr(k, k) + 1, hc[k], 0, 1);
    std::vector<double> x(np);
    for (int i = 0; i < np; i++) x[i] = c(i, 0);
    upper_solve_inplace(qr, np, x.data());
    for (int i = 0; i < np; i++) dst[perm[i]] = x[i];
    return dst;
  }
};

// ---------------------------------------------------------------------------
// ftsolver.cpp restated
// ---------------------------------------------------------------------------
struct FTOut {
  std::vector<double> x, z;  // x [6n], z [3 nf]
  uint32_t flags = 0;
  int k = 0, rank0 = 0, iters = 0;
  double rel_error = 0;
  double near_margin = INFINITY;  // the decision closest to its threshold (NearTrack)
  int near_cat = 0;
  double lu_kept = INFINITY, qr_kept = INFINITY;
};

// dynrecord::set_forcetorque_system (dynrec.cpp:227-297) as dense B0 (6n x 6n) and f
void build_B0_f(const hso_model* m, const DynRec& d, Mat& B0, std::vector<double>& f) {
  int n = m->n;
  B0 = Mat(6 * n, 6 * n);
  f.assign(6 * n, 0.0);
  auto cross_elems = [&](int i, int j, const Vec& r) {  // dynrec.cpp:253-262
    int k = 3 * (n + i), k1 = 3 * j;
    for (int l = 0; l < 3; l++) {
      int dk[3];
      for (int l1 = 0; l1 < 3; l1++) dk[l1] = (l + l1) % 3;
      B0(k + dk[0], k1 + dk[1]) = -r.v[dk[2]];
      B0(k + dk[1], k1 + dk[0]) = r.v[dk[2]];
    }
  };
  for (int i = 0; i < n; i++) {
    int pi = m->parentis[i];
    for (int j = 0; j < 3; j++) {  // ftsys_forces
      B0(3 * i + j, 3 * i + j) = 1;
      if (pi >= 0) B0(3 * pi + j, 3 * i + j) = -1;
      f[3 * i + j] = d.mom_rate[i].v[j];
    }
    for (int j = 0; j < 3; j++) {  // ftsys_torques
      B0(3 * (n + i) + j, 3 * (n + i) + j) = 1;
      if (pi >= 0) B0(3 * (n + pi) + j, 3 * (n + i) + j) = -1;
    }
    if (pi >= 0) {
      Vec r = d.jpos[i];
      r.subtract(d.pos[i]);
      cross_elems(i, i, r);
      r = d.pos[pi];
      r.subtract(d.jpos[i]);
      cross_elems(pi, i, r);
    }
    for (int j = 0; j < 3; j++) f[3 * (n + i) + j] = d.ang_mom_rate[i].v[j];
    f[3 * i + 2] += m->masses[i] * 1.0;  // ftsys_gravity, g = 1
  }
}

// contact columns (dynrec.cpp:313-344) appended to B (6n x (6n+k))
Mat build_B_contacts(const hso_model* m, const DynRec& d, const Mat& B0) {
  int n = m->n, k = 3 * d.ncontacts();
  Mat B(6 * n, 6 * n + k);
  for (int j = 0; j < 6 * n; j++)
    for (int i = 0; i < 6 * n; i++) B(i, j) = B0(i, j);
  int ci = 0;
  for (int fi = 0; fi < m->nf; fi++) {
    if (!d.contacts[fi]) continue;
    int i = m->footis[fi];
    for (int j = 0; j < 3; j++) B(3 * i + j, 3 * (2 * n + ci) + j) = 1;
    Vec r = d.fpos[fi];
    r.subtract(d.pos[i]);
    int kk = 3 * (n + i), k1 = 3 * (2 * n + ci);
    for (int l = 0; l < 3; l++) {
      int dk[3];
      for (int l1 = 0; l1 < 3; l1++) dk[l1] = (l + l1) % 3;
      B(kk + dk[0], k1 + dk[1]) = -r.v[dk[2]];
      B(kk + dk[1], k1 + dk[0]) = r.v[dk[2]];
    }
    ci++;
  }
  return B;
}

// Tree particular solution of B0 x = f (leaves -> root; parents precede children in preorder).
std::vector<double> tree_particular(const hso_model* m, const DynRec& d, const std::vector<double>& f) {
  int n = m->n;
  std::vector<double> x(6 * n, 0.0);
  for (int i = n - 1; i >= 0; i--) {
    double F[3], T[3];
    for (int j = 0; j < 3; j++) { F[j] = f[3 * i + j]; T[j] = f[3 * (n + i) + j]; }
    for (int c : m->nodes[i].kids) {
      for (int j = 0; j < 3; j++) F[j] += x[3 * c + j];
      double r[3];  // (pos_i - jpos_c) x F_c moved to the rhs
      for (int j = 0; j < 3; j++) r[j] = d.pos[i].v[j] - d.jpos[c].v[j];
      const double* Fc = &x[3 * c];
      T[0] -= r[1] * Fc[2] - r[2] * Fc[1];
      T[1] -= r[2] * Fc[0] - r[0] * Fc[2];
      T[2] -= r[0] * Fc[1] - r[1] * Fc[0];
      for (int j = 0; j < 3; j++) T[j] += x[3 * (n + c) + j];
    }
    for (int j = 0; j < 3; j++) x[3 * i + j] = F[j];
    if (m->parentis[i] >= 0) {
      double r[3];
      for (int j = 0; j < 3; j++) r[j] = d.jpos[i].v[j] - d.pos[i].v[j];
      T[0] -= r[1] * F[2] - r[2] * F[1];
      T[1] -= r[2] * F[0] - r[0] * F[2];
      T[2] -= r[0] * F[1] - r[1] * F[0];
    }
    for (int j = 0; j < 3; j++) x[3 * (n + i) + j] = T[j];
  }
  return x;
}

// Tree-built null basis N (6n x k): column (ci, j) = force rows of every ancestor a of
// the contact foot: -e_j; torque rows: (jpos_a - fpos) x e_j  (derivation: DESIGN.md).
Mat tree_null_basis(const hso_model* m, const DynRec& d) {
  int n = m->n, k = 3 * d.ncontacts();
  Mat N(6 * n, k);
  int ci = 0;
  for (int fi = 0; fi < m->nf; fi++) {
    if (!d.contacts[fi]) continue;
    for (int a = m->footis[fi]; a >= 0; a = m->parentis[a]) {
      // moment arm from the contact point to part a's joint; the root has no joint
      // cross term in B (dynrec.cpp:291: only pi >= 0), so its arm is to its COM
      const Vec& ref = (m->parentis[a] >= 0) ? d.jpos[a] : d.pos[a];
      double dd[3];
      for (int j = 0; j < 3; j++) dd[j] = ref.v[j] - d.fpos[fi].v[j];
      for (int j = 0; j < 3; j++) N(3 * a + j, 3 * ci + j) = -1;
      // d x e0 = (0, d2, -d1); d x e1 = (-d2, 0, d0); d x e2 = (d1, -d0, 0)
      int r0 = 3 * (n + a);
      N(r0 + 1, 3 * ci + 0) = dd[2];  N(r0 + 2, 3 * ci + 0) = -dd[1];
      N(r0 + 0, 3 * ci + 1) = -dd[2]; N(r0 + 2, 3 * ci + 1) = dd[0];
      N(r0 + 0, 3 * ci + 2) = dd[1];  N(r0 + 1, 3 * ci + 2) = -dd[0];
    }
    ci++;
  }
  return N;
}

// forcetorquesolver::solve_contact_forces, ftsolver.cpp:185-236 (+ set_action_penalties 239-246,
// masks 262-303: switch_torso_penalty(f, t) -> mask0 = {(0,3) if f, (3n,3n+3) if t}, mask1 = the
// complement in ascending row order, set_penal_mask1 291-303)
void solve_contact_forces(const hso_model* m, const std::vector<double>& jz, const std::vector<double>& x,
                          const Mat& N, std::vector<double>& y, FTOut& out) {
  int n = m->n, k = N.c;
  std::vector<double> c(6 * n, 1.0);
  for (int i = 3; i < 3 * n; i++) c[i] = 0;
  for (int i = 3; i < 3 * n; i++) c[3 * n + i] = jz[i];
  // rows of mask0 and mask1 (mask1 = complement)
  std::vector<int> r0, r1;
  std::vector<char> in0(6 * n, 0);
  if (m->torso_mask & 1) in0[0] = in0[1] = in0[2] = 1;
  if (m->torso_mask & 2) in0[3 * n] = in0[3 * n + 1] = in0[3 * n + 2] = 1;
  for (int i = 0; i < 6 * n; i++) (in0[i] ? r0 : r1).push_back(i);
  Mat N0((int)r0.size(), k), N1((int)r1.size(), k);
  std::vector<double> x0(r0.size()), x1(r1.size());
  for (size_t a = 0; a < r0.size(); a++) {
    for (int j = 0; j < k; j++) N0((int)a, j) = c[r0[a]] * N(r0[a], j);
    x0[a] = c[r0[a]] * x[r0[a]];
  }
  for (size_t a = 0; a < r1.size(); a++) {
    for (int j = 0; j < k; j++) N1((int)a, j) = c[r1[a]] * N(r1[a], j);
    x1[a] = c[r1[a]] * x[r1[a]];
  }
  Mat N0t = transpose(N0), N1t = transpose(N1);
  std::vector<double> ntx0 = matvec(N0t, x0), ntx1 = matvec(N1t, x1);
  Mat ntn0 = matmul(N0t, N0), ntn1 = matmul(N1t, N1);

  out.k = k;
  y.assign(k, 0.0);
  if (k == 0) { out.flags |= HSO_FLAG_NO_CONTACT; out.iters = 1; out.rel_error = NAN; return; }
  double rel_error;
  int rank0 = k;
  int iters = 0;
  do {
    iters++;
    FPLU lu;
    lu.compute(ntn0);
    while (lu.rank() > rank0) {
      lu.set_threshold(2 * lu.threshold());
      NEAR_NOTE(1.0, kNearBand, HSO_NEAR_DOUBLED);
    }
    for (int i = 0; i < lu.nonzero_pivots; i++)
      NEAR_NOTE(fabs(lu.lu(i, i)) / (fabs(lu.maxpivot) * lu.threshold()), kNearBand, HSO_NEAR_LU);
#ifndef HSO_FLOPCOUNT
    tl_near.lu_kept = INFINITY;
    for (int i = 0; i < lu.nonzero_pivots; i++) {
      const double rr = fabs(lu.lu(i, i)) / fabs(lu.maxpivot);
      if (rr > lu.threshold() && rr < tl_near.lu_kept) tl_near.lu_kept = rr;
    }
#endif
    std::vector<double> mntx0(k);
    for (int i = 0; i < k; i++) mntx0[i] = -ntx0[i];
    std::vector<double> y0 = lu.solve(mntx0);
    Mat Ny = lu.kernel();
    Mat Ry = lu.image(ntn0);
    int r = lu.rank();
    if (r == k) out.flags |= HSO_FLAG_FULL_RANK;
    rank0 = r;
    std::vector<double> t = matvec(ntn1, y0);
    std::vector<double> b(k);
    for (int i = 0; i < k; i++) b[i] = -(ntx1[i] + t[i]);
    Mat A = matmul(ntn1, Ny), Bm = matmul(ntn0, Ry);
    Mat M(k, k);
    for (int j = 0; j < A.c; j++) for (int i = 0; i < k; i++) M(i, j) = A(i, j);
    for (int j = 0; j < Bm.c; j++) for (int i = 0; i < k; i++) M(i, A.c + j) = Bm(i, j);
    CPQR qr;
    qr.compute(M);
#ifndef HSO_FLOPCOUNT
    tl_near.qr_kept = INFINITY;
    for (int i = 0; i < qr.nonzero_pivots; i++) tl_near.qr_kept = std::min(tl_near.qr_kept, fabs(qr.qr(i, i)) / fabs(qr.qr(0, 0)));
    tl_near.ill = tl_near.qr_kept < kCondQR;
#endif
    std::vector<double> z = qr.solve(b);
    std::vector<double> mz = matvec(M, z);
    for (int i = 0; i < k; i++) mz[i] -= b[i];
    rel_error = vnorm(mz) / vnorm(b);
    NEAR_NOTE(rel_error / 1e-6, kNearBandRel, HSO_NEAR_REL);
    rank0--;
    std::vector<double> zh(z.begin(), z.begin() + Ny.c);
    std::vector<double> nyz = matvec(Ny, zh);
    for (int i = 0; i < k; i++) y[i] = y0[i] + nyz[i];
    if (rel_error > 1e-6 && rank0 <= 0) { out.flags |= HSO_FLAG_LOOP_EXHAUST; break; }
  } while (rel_error > 1e-6);
  if (iters > 1) out.flags |= HSO_FLAG_RANK_RETRY;
  out.iters = iters;
  out.rank0 = rank0 + 1;
  out.rel_error = rel_error;
}

// ---------------------------------------------------------------------------
// Closed-form restatement of the two-stage least squares (the HIP kernel's fast
// path). With the tree basis, y = w = contact forces, the zeroth-order rows are
// A_c = [-I; [d0_c]x] (d0_c = pos_0 - fpos_c) and the first-order Gram is
// block-diagonal, D_c = sum_a [d_a]x^T diag(jz_a^2) [d_a]x, g_c likewise with
// the particular torques. When A has full row rank 6 (>= 3 non-collinear feet)
// the zeroth-order minimizers are {A w = -a} and the first-order minimizer is
// w_c = -D_c^-1 (g_c + A_c^T lam), (sum_c A_c D_c^-1 A_c^T) lam = a - sum_c A_c D_c^-1 g_c.
// One foot: unique LS solution. Two feet: rank 5, kernel (u,-u) along the feet
// line, t from the 1-D first-order problem. Returns false (caller falls back to
// the Eigen-style path) when a pivot is below the conditioning guard.
// ---------------------------------------------------------------------------
constexpr double kFastPivotGuard = 1e-10;

// in-place Cholesky of an n x n SPD matrix (row-major a[i*n+j]); false if a pivot
// falls below guard * max diagonal (a guarded pivot's distance to it goes to tl_near)
bool chol(double* a, int n, double guard) {
  double mx = 0;
  for (int i = 0; i < n; i++) mx = std::max(mx, a[i * n + i]);
  for (int j = 0; j < n; j++) {
    double s = a[j * n + j];
    for (int k = 0; k < j; k++) s -= a[j * n + k] * a[j * n + k];
    if (guard > 0) NEAR_NOTE(s / (guard * mx), kNearBand, HSO_NEAR_PIVOT);
    if (!(s > guard * mx)) return false;
    double l = sqrt(s), rl = 1.0 / l;  // one division per pivot, as the kernel
    a[j * n + j] = l;
    for (int i = j + 1; i < n; i++) {
      double t = a[i * n + j];
      for (int k = 0; k < j; k++) t -= a[i * n + k] * a[j * n + k];
      a[i * n + j] = t * rl;
    }
  }
  return true;
}
void chol_solve(const double* L, int n, double* b) {
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * b[k];
    b[i] = s * (1.0 / L[i * n + i]);
  }
  for (int i = n - 1; i >= 0; i--) {
    double s = b[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * b[k];
    b[i] = s * (1.0 / L[i * n + i]);
  }
}

// LDL^T (the kernel's ldl_n): unit-lower L below the diagonal, d on it; pivot guard as chol's
bool ldl(double* a, int n, double guard) {
  double mx = 0;
  for (int i = 0; i < n; i++) mx = std::max(mx, a[i * n + i]);
  double v[18];
  for (int j = 0; j < n; j++) {
    for (int k = 0; k < j; k++) v[k] = a[j * n + k] * a[k * n + k];
    double dj = a[j * n + j];
    for (int k = 0; k < j; k++) dj -= a[j * n + k] * v[k];
    if (guard > 0) NEAR_NOTE(dj / (guard * mx), kNearBand, HSO_NEAR_PIVOT);
    if (!(dj > guard * mx)) return false;
    const double r = 1.0 / dj;
    a[j * n + j] = dj;
    for (int i = j + 1; i < n; i++) {
      double t = a[i * n + j];
      for (int k = 0; k < j; k++) t -= a[i * n + k] * v[k];
      a[i * n + j] = t * r;
    }
  }
  return true;
}
void ldl_solve(const double* L, int n, double* b) {
  for (int i = 0; i < n; i++) {
    double s = b[i];
    for (int k = 0; k < i; k++) s -= L[i * n + k] * b[k];
    b[i] = s;
  }
  for (int i = 0; i < n; i++) b[i] *= 1.0 / L[i * n + i];
  for (int i = n - 1; i >= 0; i--) {
    double s = b[i];
    for (int k = i + 1; k < n; k++) s -= L[k * n + i] * b[k];
    b[i] = s;
  }
}

// rows of [d]x: ([d]x w)_r = v_r . w
inline void cross_rows(const double* d, double v[3][3]) {
  v[0][0] = 0;     v[0][1] = -d[2]; v[0][2] = d[1];
  v[1][0] = d[2];  v[1][1] = 0;     v[1][2] = -d[0];
  v[2][0] = -d[1]; v[2][1] = d[0];  v[2][2] = 0;
}

// nc >= 3 when a block D_c is singular (a straight, IK-clamped leg: no joint
// torque resists a force along it) or the per-contact Schur complement is. The
// equality-constrained minimizer is still unique when D is positive definite on
// null(A), and then K = D + rho A^T A is positive definite and
//   w = -K^-1 (g~ + A^T lam),  (A K^-1 A^T) lam = a - A K^-1 g~,  g~ = g + rho A^T a
// gives it independently of rho (rho balances the two terms' scales). A pivot
// under the guard means the minimizer is not unique: the Eigen-style path decides.
bool aug_solve(int nc, const std::vector<double>& A, const std::vector<double>& D, const std::vector<double>& g,
               const double* a, std::vector<double>& y) {
  const int k = 3 * nc;
  auto Aat = [&](int r, int i) { return A[18 * (i / 3) + r * 3 + i % 3]; };  // A (6 x k)
  double md = 0, ma = 0;
  for (int c = 0; c < nc; c++)
    for (int i = 0; i < 3; i++) {
      md = std::max(md, D[9 * c + 4 * i]);
      double s = 0;
      for (int r = 0; r < 6; r++) s += Aat(r, 3 * c + i) * Aat(r, 3 * c + i);
      ma = std::max(ma, s);
    }
  const double rho = (md > 0 && ma > 0) ? md / ma : 1.0;
  std::vector<double> K(k * k), X(k * 7);
  for (int i = 0; i < k; i++) {
    for (int j = 0; j < k; j++) {
      double s = 0;
      for (int r = 0; r < 6; r++) s += Aat(r, i) * Aat(r, j);
      K[i * k + j] = ((i / 3 == j / 3) ? D[9 * (i / 3) + 3 * (i % 3) + j % 3] : 0.0) + rho * s;
    }
    double s = 0;
    for (int r = 0; r < 6; r++) s += Aat(r, i) * a[r];
    X[i * 7 + 6] = g[i] + rho * s;
    for (int q = 0; q < 6; q++) X[i * 7 + q] = Aat(q, i);
  }
  if (!chol(K.data(), k, kFastPivotGuard)) return false;
  std::vector<double> col(k);
  for (int q = 0; q < 7; q++) {
    for (int i = 0; i < k; i++) col[i] = X[i * 7 + q];
    chol_solve(K.data(), k, col.data());
    for (int i = 0; i < k; i++) X[i * 7 + q] = col[i];
  }
  double St[36], lam[6];
  for (int r = 0; r < 6; r++) {
    for (int q = 0; q < 7; q++) {
      double s = 0;
      for (int i = 0; i < k; i++) s += Aat(r, i) * X[i * 7 + q];
      if (q < 6) St[6 * r + q] = s;
      else lam[r] = a[r] - s;
    }
  }
  if (!chol(St, 6, kFastPivotGuard)) return false;
  chol_solve(St, 6, lam);
  for (int i = 0; i < k; i++) {
    double s = X[i * 7 + 6];
    for (int r = 0; r < 6; r++) s += X[i * 7 + r] * lam[r];
    y[i] = -s;
  }
  return true;
}

// Nearly collinear contact feet (nc >= 3) make G = A A^T (zeroth-order rows) close to rank 5; the
// reference's loop (ftsolver.cpp:205-232) then finds rel_error > 1e-6 on its first pass (ntn0 * Ry
// carries G's conditioning squared) and retries at lower ranks, so the closed form's exact minimizer
// is not its answer. Accepted when c2(C) / (tr(C) maxdiag(G)) >= 1e-3, C = sum_c e_c e_c^T,
// e_c = d0_c - mean d0 (c2(C) / tr(C) is G's smallest eigenvalue mu2 + mu3 within 4x); the ratio
// follows the reference's 6th FullPivLU pivot ratio within ~2x, and every retry measured in tree mode
// had it below 2.5e-5 (tests/test_oracle.py::test_zeroth_guard_*). The kernel's division-free form
// (zeroth_well_posed in hs_kernels.hip): C' = nc Q - s s^T (s = sum d0_c, Q = sum d0_c d0_c^T),
// c2(C') >= 1e-3 * nc * tr(C') * maxdiag(G).
constexpr double kZerothGuard = 1e-3;
bool zeroth_well_posed(const DynRec& d, const std::vector<int>& cf) {
  const int nc = (int)cf.size();
  double s0 = 0, s1 = 0, s2 = 0, q00 = 0, q11 = 0, q22 = 0, q01 = 0, q02 = 0, q12 = 0;
  for (int c = 0; c < nc; c++) {
    const Vec& fp = d.fpos[cf[c]];
    const double d0 = d.pos[0].v[0] - fp.v[0], d1 = d.pos[0].v[1] - fp.v[1], d2 = d.pos[0].v[2] - fp.v[2];
    s0 += d0; s1 += d1; s2 += d2;
    q00 += d0 * d0; q11 += d1 * d1; q22 += d2 * d2;
    q01 += d0 * d1; q02 += d0 * d2; q12 += d1 * d2;
  }
  const double k = nc;
  const double c00 = k * q00 - s0 * s0, c11 = k * q11 - s1 * s1, c22 = k * q22 - s2 * s2;
  const double c01 = k * q01 - s0 * s1, c02 = k * q02 - s0 * s2, c12 = k * q12 - s1 * s2;
  const double c2 = (c00 * c11 - c01 * c01) + (c00 * c22 - c02 * c02) + (c11 * c22 - c12 * c12);
  const double tq = q00 + q11 + q22;
  const double md = std::max(k, std::max(tq - q00, std::max(tq - q11, tq - q22)));
  NEAR_NOTE(c2 / (kZerothGuard * k * (c00 + c11 + c22) * md), kNearBand, HSO_NEAR_COLLINEAR);
  return c2 >= kZerothGuard * k * (c00 + c11 + c22) * md;
}

bool fast_contact_solve(const hso_model* m, const DynRec& d, const std::vector<double>& x, std::vector<double>& y) {
  const int n = m->n;
  std::vector<int> cf;  // contact -> foot index
  for (int fi = 0; fi < m->nf; fi++)
    if (d.contacts[fi]) cf.push_back(fi);
  const int nc = (int)cf.size(), k = 3 * nc;
  y.assign(k, 0.0);
  if (nc == 0) return true;
  double a[6] = {x[0], x[1], x[2], x[3 * n], x[3 * n + 1], x[3 * n + 2]};
  // A_c (6x3), D_c (3x3), g_c (3)
  std::vector<double> A(6 * 3 * nc), D(9 * nc, 0.0), g(3 * nc, 0.0);
  for (int c = 0; c < nc; c++) {
    const Vec& fp = d.fpos[cf[c]];
    double d0[3];
    for (int r = 0; r < 3; r++) d0[r] = d.pos[0].v[r] - fp.v[r];
    double v[3][3];
    cross_rows(d0, v);
    double* Ac = &A[18 * c];  // row-major 6x3
    for (int r = 0; r < 3; r++)
      for (int j = 0; j < 3; j++) { Ac[r * 3 + j] = (r == j) ? -1.0 : 0.0; Ac[(3 + r) * 3 + j] = v[r][j]; }
    for (int p = m->footis[cf[c]]; p >= 0 && m->parentis[p] >= 0; p = m->parentis[p]) {
      double da[3];
      for (int r = 0; r < 3; r++) da[r] = d.jpos[p].v[r] - fp.v[r];
      double va[3][3];
      cross_rows(da, va);
      for (int r = 0; r < 3; r++) {
        double w2 = d.jzaxis[p].v[r] * d.jzaxis[p].v[r];
        if (w2 == 0) continue;
        for (int i = 0; i < 3; i++) {
          for (int j = 0; j < 3; j++) D[9 * c + 3 * i + j] += w2 * va[r][i] * va[r][j];
          g[3 * c + i] += w2 * va[r][i] * x[3 * n + 3 * p + r];
        }
      }
    }
  }
  if (nc == 1) {  // rank 3 = k: unique least-squares solution (A^T A) w = -A^T a
    double M[9] = {0}, b[3] = {0};
    for (int i = 0; i < 3; i++) {
      for (int j = 0; j < 3; j++)
        for (int r = 0; r < 6; r++) M[3 * i + j] += A[r * 3 + i] * A[r * 3 + j];
      for (int r = 0; r < 6; r++) b[i] -= A[r * 3 + i] * a[r];
    }
    if (!chol(M, 3, kFastPivotGuard)) return false;
    chol_solve(M, 3, b);
    for (int i = 0; i < 3; i++) y[i] = b[i];
    return true;
  }
  if (nc == 2) {  // rank 5: kernel n = (u, -u)/sqrt2, u along the line between the feet
    double u[3], un = 0;
    for (int r = 0; r < 3; r++) { u[r] = d.fpos[cf[0]].v[r] - d.fpos[cf[1]].v[r]; un += u[r] * u[r]; }
    un = sqrt(un);
    if (!(un > 1e-12)) return false;
    double nv[6];
    for (int r = 0; r < 3; r++) { nv[r] = u[r] / un / sqrt(2.0); nv[3 + r] = -nv[r]; }
    double M[36] = {0}, b[6] = {0};
    for (int i = 0; i < 6; i++) {
      for (int j = 0; j < 6; j++) {
        double s = 0;
        for (int r = 0; r < 6; r++) s += A[18 * (i / 3) + r * 3 + i % 3] * A[18 * (j / 3) + r * 3 + j % 3];
        M[6 * i + j] = s + nv[i] * nv[j];
      }
      double s = 0;
      for (int r = 0; r < 6; r++) s += A[18 * (i / 3) + r * 3 + i % 3] * a[r];
      b[i] = -s;
    }
    if (!chol(M, 6, kFastPivotGuard)) return false;
    chol_solve(M, 6, b);
    double nDn = 0, nr = 0;
    for (int c = 0; c < 2; c++)
      for (int i = 0; i < 3; i++) {
        double Dw = 0, Dn = 0;
        for (int j = 0; j < 3; j++) { Dw += D[9 * c + 3 * i + j] * b[3 * c + j]; Dn += D[9 * c + 3 * i + j] * nv[3 * c + j]; }
        nr += nv[3 * c + i] * (Dw + g[3 * c + i]);
        nDn += nv[3 * c + i] * Dn;
      }
    if (!(nDn > 0)) return false;
    double t = -nr / nDn;
    for (int i = 0; i < 6; i++) y[i] = b[i] + t * nv[i];
    return true;
  }
  // nc >= 3: nearly collinear feet leave it to the Eigen-style path (the kernel's zeroth_well_posed)
  if (!zeroth_well_posed(d, cf)) return false;
  // Schur complement on the 6 zeroth-order constraints
  // per-contact blocks, summed over the contacts pairwise as the kernel's lanes do
  // (((c3 + c2) + (c1 + c0)) + ((c7 + c6) + (c5 + c4)), absent contacts 0: hs_kernels.hip fast_solve_lanes)
  double Sc[8][36] = {}, hc[8][6] = {};
  std::vector<double> Dinv(9 * nc);
  for (int c = 0; c < nc; c++) {
    double L[9];
    for (int i = 0; i < 9; i++) L[i] = D[9 * c + i];
    if (!ldl(L, 3, kFastPivotGuard)) return aug_solve(nc, A, D, g, a, y);
    for (int j = 0; j < 3; j++) {  // Dinv columns
      double e[3] = {0, 0, 0};
      e[j] = 1;
      ldl_solve(L, 3, e);
      for (int i = 0; i < 3; i++) Dinv[9 * c + 3 * i + j] = e[i];
    }
    const double* Ac = &A[18 * c];
    double E[18];  // A_c Dinv_c (6x3)
    for (int r = 0; r < 6; r++)
      for (int j = 0; j < 3; j++) {
        double s = 0;
        for (int i = 0; i < 3; i++) s += Ac[r * 3 + i] * Dinv[9 * c + 3 * i + j];
        E[r * 3 + j] = s;
      }
    for (int r = 0; r < 6; r++) {
      for (int q = 0; q < 6; q++) {
        double s = 0;
        for (int j = 0; j < 3; j++) s += E[r * 3 + j] * Ac[q * 3 + j];
        Sc[c][6 * r + q] = s;
      }
      double s = 0;
      for (int j = 0; j < 3; j++) s += E[r * 3 + j] * g[3 * c + j];
      hc[c][r] = s;
    }
  }
  auto pairwise = [](const double* v) { return ((v[3] + v[2]) + (v[1] + v[0])) + ((v[7] + v[6]) + (v[5] + v[4])); };
  double S[36], h[6];
  for (int e = 0; e < 36; e++) {
    double v[8];
    for (int c = 0; c < 8; c++) v[c] = Sc[c][e];
    S[e] = pairwise(v);
  }
  for (int r = 0; r < 6; r++) {
    double v[8];
    for (int c = 0; c < 8; c++) v[c] = hc[c][r];
    h[r] = pairwise(v);
  }
  double lam[6];
  for (int r = 0; r < 6; r++) lam[r] = a[r] - h[r];
  if (!ldl(S, 6, kFastPivotGuard)) return aug_solve(nc, A, D, g, a, y);
  ldl_solve(S, 6, lam);
  for (int c = 0; c < nc; c++) {
    const double* Ac = &A[18 * c];
    double t[3];
    for (int i = 0; i < 3; i++) {
      double s = g[3 * c + i];
      for (int r = 0; r < 6; r++) s += Ac[r * 3 + i] * lam[r];
      t[i] = s;
    }
    for (int i = 0; i < 3; i++) {
      double s = 0;
      for (int j = 0; j < 3; j++) s += Dinv[9 * c + 3 * i + j] * t[j];
      y[3 * c + i] = -s;
    }
  }
  return true;
}

// forcetorquesolver::solve_forces (ftsolver.cpp:331-378): contact forces of ALL feet
// (set_forcetorque_system_contacts with contact_feet_flag = false, dynrec.cpp:313-325)
// realising the motor torques z, torso force/torque columns zeroed, least squares
// over [B0 Bc_all; jz-rows] [x; y] = [f; z] (add_torque_constraints_to_B, 359-378).
// SparseQR's basic solution leaves the zero torso columns at 0; the other columns are
// factorized here by a column-by-column Householder QR in their natural order (the
// joint wrenches, then the feet's force components). A force column whose pivot r_jj^2
// falls to 1e-10 of the largest force column's squared norm after the wrenches' reflections
// (the reduced normal matrix's largest diagonal; the kernel's chol_packed guard on the same
// quantity) is dependent: it is dropped and its force component set to 0, the basic
// solution of the rank-deficient least squares (a straight leg's torques cannot fix its
// foot force along the leg). Returns false when a column was dropped.
// rule HSO_FORCES_SPARSEQR instead restates SparseQR's own rank rule (Eigen 3.3 SparseQR::factorize,
// the solver ftsolver.cpp:349-353 calls, default threshold): every column of the literal system, the
// zeroed torso columns included, is kept iff its Householder |beta| (its norm on the rows not yet
// eliminated) is at least 20 (rows + cols) eps max_j |A_j|; a dropped column's unknown is 0
// (_solve_impl's basic solution). The column order stays natural: the COLAMD pre-ordering
// (COLAMDOrdering<int>, ftsolver.h:17) is not restated, so which of several dependent columns
// SparseQR drops is not pinned. On full-rank systems both rules give the least-squares solution.
bool solve_forces(const hso_model* m, const DynRec& d, const double* z, std::vector<double>& y,
                  int rule = HSO_FORCES_KERNEL) {
  const int n = m->n, nf = m->nf, nmj = m->nmj;
  Mat B0;
  std::vector<double> f;
  build_B0_f(m, d, B0, f);
  const int rows = 6 * n + nmj, cols = 6 * n - 6 + 3 * nf;
  std::vector<int> keep;  // B0 columns without the torso force / torque
  for (int c = 0; c < 6 * n; c++)
    if (!(c < 3 || (c >= 3 * n && c < 3 * n + 3))) keep.push_back(c);
  Mat A(rows, cols);
  for (int j = 0; j < (int)keep.size(); j++)
    for (int i = 0; i < 6 * n; i++) A(i, j) = B0(i, keep[j]);
  const int y0 = (int)keep.size();
  for (int fi = 0; fi < nf; fi++) {  // all feet
    int i = m->footis[fi];
    for (int j = 0; j < 3; j++) A(3 * i + j, y0 + 3 * fi + j) = 1;
    Vec r = d.fpos[fi];
    r.subtract(d.pos[i]);
    int kk = 3 * (n + i), k1 = y0 + 3 * fi;
    for (int l = 0; l < 3; l++) {
      int dk[3];
      for (int l1 = 0; l1 < 3; l1++) dk[l1] = (l + l1) % 3;
      A(kk + dk[0], k1 + dk[1]) = -r.v[dk[2]];
      A(kk + dk[1], k1 + dk[0]) = r.v[dk[2]];
    }
  }
  std::vector<double> b(f);
  b.resize(rows);
  for (int jj = 0; jj < nmj; jj++) {  // torque constraint rows
    int h = m->hinge_ids[jj];
    for (int j = 0; j < 3; j++) {
      int col = -1;
      for (int q = 0; q < (int)keep.size(); q++)
        if (keep[q] == 3 * n + 3 * h + j) col = q;
      A(6 * n + jj, col) = d.jzaxis[h].v[j];
    }
    b[6 * n + jj] = z[jj];
  }
  const double kRankGuard = 1e-10;  // the kernel's kFastPivotGuard on the reduced normal matrix
  if (rule == HSO_FORCES_SPARSEQR) {
    // the literal matrix: the torso force / torque columns present and zero (ftsolver.cpp:349)
    const int cf = 6 * n + 3 * nf;
    Mat F(rows, cf);
    for (int j = 0; j < (int)keep.size(); j++)
      for (int i = 0; i < rows; i++) F(i, keep[j]) = A(i, j);
    for (int j = y0; j < cols; j++)
      for (int i = 0; i < rows; i++) F(i, 6 * n + (j - y0)) = A(i, j);
    double mx = 0;
    for (int j = 0; j < cf; j++) {
      double s2 = 0;
      for (int i = 0; i < rows; i++) s2 += F(i, j) * F(i, j);
      mx = std::max(mx, std::sqrt(s2));
    }
    if (mx == 0) mx = 1;
    const double thr = 20.0 * (rows + cf) * mx * std::numeric_limits<double>::epsilon();
    Mat bq(rows, 1);
    for (int i = 0; i < rows; i++) bq(i, 0) = b[i];
    std::vector<int> kept;
    bool fullq = true;
    std::vector<double> essq;
    for (int j = 0; j < cf; j++) {
      const int k = (int)kept.size();
      if (k >= std::min(rows, cf)) { fullq = false; continue; }
      double s2 = 0;  // |beta|^2: the column's norm on rows k.. (c0^2 + sqrNorm)
      for (int i = k; i < rows; i++) s2 += F(i, j) * F(i, j);
      if (!(std::sqrt(s2) >= thr)) {  // SparseQR: a zero pivot, the column moved to the end
        if (!(j < 3 || (j >= 3 * n && j < 3 * n + 3))) fullq = false;  // the zero torso columns always drop
        continue;
      }
      double tau, beta;
      make_householder(&F(k, j), rows - k, 1, tau, beta);
      F(k, j) = beta;
      essq.assign(&F(k, j) + 1, &F(k, j) + (rows - k));
      apply_householder_left(F, k, essq.data(), tau, j + 1, cf);
      apply_householder_left(bq, k, essq.data(), tau, 0, 1);
      kept.push_back(j);
    }
    std::vector<double> uq(cf, 0.0);
    for (int t = (int)kept.size() - 1; t >= 0; t--) {
      double v = bq(t, 0);
      for (int t2 = t + 1; t2 < (int)kept.size(); t2++) v -= F(t, kept[t2]) * uq[kept[t2]];
      uq[kept[t]] = v / F(t, kept[t]);
    }
    y.assign(uq.begin() + 6 * n, uq.end());
    return fullq;
  }
  Mat R = A, bm(rows, 1);
  for (int i = 0; i < rows; i++) bm(i, 0) = b[i];
  std::vector<int> piv;  // kept columns in order (R's row t belongs to piv[t])
  bool full = true;
  double mxd = 0;
  std::vector<double> ess;
  for (int j = 0; j < cols; j++) {
    const int k = (int)piv.size();
    if (j == y0)  // the force columns' squared norms after the wrenches' reflections
      for (int jj = y0; jj < cols; jj++) {
        double s2 = 0;
        for (int i = k; i < rows; i++) s2 += R(i, jj) * R(i, jj);
        mxd = std::max(mxd, s2);
      }
    if (j >= y0) {
      double s2 = 0;  // r_jj^2 if kept: the column's squared norm on the rows not yet eliminated
      for (int i = k; i < rows; i++) s2 += R(i, j) * R(i, j);
      NEAR_NOTE(s2 / (kRankGuard * mxd), kNearBand, HSO_NEAR_PIVOT);
      if (!(s2 > kRankGuard * mxd)) { full = false; continue; }
    }
    double tau, beta;
    make_householder(&R(k, j), rows - k, 1, tau, beta);
    R(k, j) = beta;
    ess.assign(&R(k, j) + 1, &R(k, j) + (rows - k));
    apply_householder_left(R, k, ess.data(), tau, j + 1, cols);
    apply_householder_left(bm, k, ess.data(), tau, 0, 1);
    piv.push_back(j);
  }
  std::vector<double> u(cols, 0.0);  // dropped columns stay 0
  for (int t = (int)piv.size() - 1; t >= 0; t--) {
    double v = bm(t, 0);
    for (int t2 = t + 1; t2 < (int)piv.size(); t2++) v -= R(t, piv[t2]) * u[piv[t2]];
    u[piv[t]] = v / R(t, piv[t]);
  }
  y.assign(u.begin() + y0, u.begin() + y0 + 3 * nf);
  return full;
}

// forcetorquesolver::solve_forcetorques, ftsolver.cpp:78-102
void solve_forcetorques(const hso_model* m, const DynRec& d, int basis, FTOut& out) {
  int n = m->n;
  tl_near = NearTrack();
  std::vector<double> jz(3 * n);
  for (int i = 0; i < n; i++) for (int j = 0; j < 3; j++) jz[3 * i + j] = d.jzaxis[i].v[j];
  Mat B0;
  std::vector<double> f;
  build_B0_f(m, d, B0, f);
  std::vector<double> x;
  Mat N;
  if (basis == HSO_BASIS_ORTHO) {
    HQR qr0;  // SparseQR particular solution (ftsolver.cpp:107-113)
    qr0.compute(B0);
    x = qr0.solve(f);
    // SparseQR(B^T) null space (ftsolver.cpp:116-146): B resized square, last k cols of Q
    Mat B = build_B_contacts(m, d, B0);
    int k = B.c - 6 * n, mm = B.c;
    Mat Bsq(mm, mm);
    for (int j = 0; j < mm; j++) for (int i = 0; i < 6 * n; i++) Bsq(i, j) = B(i, j);
    HQR qr1;
    qr1.compute(transpose(Bsq));
    N = Mat(6 * n, k);
    for (int i = 0; i < k; i++) {
      std::vector<double> e(mm, 0.0);
      e[mm - 1 - i] = 1;
      std::vector<double> col = qr1.apply_Q(e);
      for (int r = 0; r < 6 * n; r++) N(r, i) = col[r];  // conservativeResize to 6n rows
    }
  } else {
    x = tree_particular(m, d, f);
    N = tree_null_basis(m, d);
  }
  std::vector<double> y;
  // the closed form is the (1,1) penalty's; other masks take the Eigen-style path
  if (basis == HSO_BASIS_FAST && m->torso_mask == 3 && fast_contact_solve(m, d, x, y)) {
    out.k = N.c;
    out.iters = 1;
    out.rank0 = -1;
    if (N.c == 0) out.flags |= HSO_FLAG_NO_CONTACT;
    if (N.c == 3) out.flags |= HSO_FLAG_FULL_RANK;
  } else {
    if (basis == HSO_BASIS_FAST) out.flags |= HSO_FLAG_GENERAL;
    solve_contact_forces(m, jz, x, N, y, out);
  }
  int k = N.c;
  // z = -N_cont y over all feet (ftsolver.cpp:276-284, 91)
  out.z.assign(3 * m->nf, 0.0);
  for (int fi = 0; fi < m->nf; fi++)
    for (int j = 0; j < 3; j++) {
      double s = 0;
      for (int c = 0; c < k; c++) s += N(3 * m->footis[fi] + j, c) * y[c];
      out.z[3 * fi + j] = -s;
    }
  for (int r = 0; r < 6 * n; r++) {
    double s = 0;
    for (int c = 0; c < k; c++) s += N(r, c) * y[c];
    x[r] += s;
  }
  out.x = x;
  out.near_margin = tl_near.margin;
  out.near_cat = (tl_near.ill && !(tl_near.margin <= 1.0)) ? HSO_NEAR_COND : tl_near.cat;
  out.lu_kept = tl_near.lu_kept;
  out.qr_kept = tl_near.qr_kept;
  if (tl_near.near()) out.flags |= HSO_FLAG_NEAR_RANK;
}

int load_model(const char* path, hso_model** out) {
  std::ifstream fs(path);
  if (!fs) return -1;
  std::stringstream ss;
  ss << fs.rdbuf();
  XNode root;
  std::string err;
  if (!parse_xml(ss.str(), &root, err)) return -2;
  XNode* mj = root.first("mujoco");
  if (!mj) return -3;
  XNode* wb = mj->first("worldbody");
  if (!wb) return -3;
  XNode* body = wb->first("body");
  if (!body) return -3;
  hso_model* m = new hso_model;
  Aff A;
  A.set_unity();
  mnode_from_xnode(m, body, A, -1);
  std::string p(path);
  size_t sl = p.find_last_of('/');
  m->fname = (sl == std::string::npos) ? p : p.substr(sl + 1);
  // liksolver ctor / set_limbs, lik.cpp:7-78
  std::vector<int> inds;
  if (m->fname == "myant.xml") { m->lik_index = 0; inds = {2, 6, 10, 14}; m->ls = limb_ls; }
  else if (m->fname == "hexapod.xml") { m->lik_index = 1; inds = {2, 5, 9, 12, 16, 19}; m->ls = limb_ls; }
  else if (m->fname == "spider.xml") { m->lik_index = 2; inds = {1, 4, 7, 10, 13, 16}; m->ls = limb_ls1; }
  else { delete m; return -4; }
  for (size_t i = 0; i < inds.size(); i++) {
    Limb L;
    L.child = inds[i];
    L.parent = m->nodes[L.child].parent;
    int nd = L.child;
    for (int j = 0; j < 3; j++) { L.vnode[j] = nd; if (j < 2) nd = m->nodes[nd].kids.front(); }
    L.foot = m->nodes[m->nodes[L.child].kids.front()].kids.front();
    if (m->lik_index == 0) L.ysign = ((int)i < 2) ? 1 : -1;
    else L.ysign = (i % 2 == 0) ? 1 : -1;
    m->limbs.push_back(L);
    double r1 = m->nodes[inds[i] + 2].rcap;  // lik.cpp:132-140
    m->rcap = r1;
  }
  recompute_modelnodes(m);
  // periodic::set_dynparts
  m->n = (int)m->nodes.size();
  std::vector<char> isfoot(m->n, 0);
  for (auto& L : m->limbs) isfoot[L.foot] = 1;
  for (int i = 0; i < m->n; i++) {
    m->parentis.push_back(m->nodes[i].parent);
    m->masses.push_back(1.0);  // dBodyCreate default mass (visualization.cpp:458,485)
    if (isfoot[i]) m->footis.push_back(i);
    if (m->nodes[i].jtype == J_HINGE) m->hinge_ids.push_back(i);
  }
  m->nf = (int)m->footis.size();
  m->cfg = (int)m->jvals.size();
  m->nmj = m->cfg - 6;
  *out = m;
  return 0;
}

// One rollout (periodic.cpp:77-96, 149-160, 192-202, 261-307, 328-343, 377-391)
int run_rollout(const hso_model* m0, const hso_gait* g, int n_t, int k0, int H, int basis, int ignore_reach,
                double* q, double* tau, double* cf, double* xo, uint32_t* flags, double* work_cot, double* diag,
                double* nearv = nullptr) {
  hso_model mm = *m0;  // private model state (joint values live in the tree, model.h:38)
  hso_model* m = &mm;
  tl_ignore_reach = ignore_reach != 0;
  PGS pgs;
  setup_pergen(m, pgs, g);
  int n = m->n, cfg = m->cfg, nmj = m->nmj, nf = m->nf;
  int nsamp = k0 + H + 4;
  double dt = pgs.pergen.period / n_t;
  std::vector<double> traj((size_t)nsamp * cfg);
  std::vector<char> unreach(nsamp, 0);
  std::vector<double> rec(cfg);
  double t = 0;
  for (int i = 0; i < nsamp; i++) {  // record_trajectory
    tl_unreach = false;
    pgs.set_rec(rec.data(), t);
    if (!set_jvalues_with_lik(m, rec.data())) return -10;
    unreach[i] = tl_unreach;
    for (int j = 0; j < cfg; j++) traj[(size_t)i * cfg + j] = jv(m, j);
    t += dt;
  }
  if (q) std::copy(traj.begin(), traj.end(), q);
  // compute_dynrecs: only samples k0 .. k0+H+3 are needed
  std::vector<DynRec> dr(nsamp);
  for (int i = k0; i < nsamp; i++) {
    dr[i].init(n, nf);
    for (int j = 0; j < cfg; j++) jv(m, j) = traj[(size_t)i * cfg + j];
    recompute_modelnodes(m);
    dynrec_initialize(m, dr[i], m->rcap);
  }
  // compute_dynrec_ders: stage 0 on k0+1..nsamp-2, stage 1 on k0+2..nsamp-3
  for (int i = k0 + 1; i <= nsamp - 2; i++) compute_ders(m, dr[i], 0, dr[i - 1], dr[i + 1], dt);
  for (int i = k0 + 2; i <= nsamp - 3; i++) compute_ders(m, dr[i], 1, dr[i - 1], dr[i + 1], dt);
  double work = 0;
  for (int h = 0; h < H; h++) {
    int i = k0 + h + 2;
    FTOut ft;
    solve_forcetorques(m, dr[i], basis, ft);
    // get_motor_torques: tau_j = jz_p . x[3n+3p..]
    std::vector<double> mt(nmj);
    for (int jj = 0; jj < nmj; jj++) {
      int kk = 3 * m->hinge_ids[jj], k1 = 3 * n + kk;
      double s = 0;
      for (int j = 0; j < 3; j++) s += dr[i].jzaxis[m->hinge_ids[jj]].v[j] * ft.x[k1 + j];
      mt[jj] = s;
    }
    uint32_t fl = ft.flags;
    if (unreach[i]) fl |= HSO_FLAG_UNREACH;
    for (double v : mt) if (std::isnan(v)) fl |= HSO_FLAG_NAN;
    for (double v : ft.z) if (std::isnan(v)) fl |= HSO_FLAG_NAN;
    if (tau) std::copy(mt.begin(), mt.end(), tau + (size_t)h * nmj);
    if (cf) std::copy(ft.z.begin(), ft.z.end(), cf + (size_t)h * 3 * nf);
    if (xo) std::copy(ft.x.begin(), ft.x.end(), xo + (size_t)h * 6 * n);
    if (flags) flags[h] = fl;
    if (diag) {
      diag[4 * h + 0] = ft.k; diag[4 * h + 1] = ft.rank0;
      diag[4 * h + 2] = ft.iters; diag[4 * h + 3] = ft.rel_error;
    }
    if (nearv) { nearv[4 * h] = ft.near_margin; nearv[4 * h + 1] = ft.near_cat; nearv[4 * h + 2] = ft.lu_kept; nearv[4 * h + 3] = ft.qr_kept; }
    // compute_vel_traj (periodic.cpp:261-282) + work_over_period (285-307)
    double work_dt = 0;
    for (int jj = 0; jj < nmj; jj++) {
      int j = 6 + jj;
      double dd = traj[(size_t)(i + 1) * cfg + j] - traj[(size_t)(i - 1) * cfg + j];
      if (dd > M_PI) dd -= 2 * M_PI;
      else if (dd < -M_PI) dd += 2 * M_PI;
      double jvel = dd / (2 * dt);
      double dw = mt[jj] * jvel;
      dw = (dw > 0) ? dw : 0;
      work_dt += dw;
    }
    work_dt *= dt;
    work += work_dt;
  }
  if (work_cot) {
    double weight = 0;
    for (int i = 0; i < n; i++) weight += m->masses[i];
    work_cot[0] = work;
    work_cot[1] = work / (weight * g->step_length);
  }
  return 0;
}

// periodic::solve_contforces_given_torques (periodic.cpp:368-374) over steps
// k0 .. k0+H-1 of one rollout; tau_in [H][nmj] -> cf [H][3 nf]
int run_forces(const hso_model* m0, const hso_gait* g, int n_t, int k0, int H, int ignore_reach, int rule,
               const double* tau_in, double* cf, uint32_t* flags) {
  hso_model mm = *m0;
  hso_model* m = &mm;
  tl_ignore_reach = ignore_reach != 0;
  PGS pgs;
  setup_pergen(m, pgs, g);
  int n = m->n, cfg = m->cfg, nf = m->nf, nmj = m->nmj;
  int nsamp = k0 + H + 4;
  double dt = pgs.pergen.period / n_t;
  std::vector<double> traj((size_t)nsamp * cfg);
  std::vector<char> unreach(nsamp, 0);
  std::vector<double> rec(cfg);
  double t = 0;
  for (int i = 0; i < nsamp; i++) {
    tl_unreach = false;
    pgs.set_rec(rec.data(), t);
    if (!set_jvalues_with_lik(m, rec.data())) return -10;
    unreach[i] = tl_unreach;
    for (int j = 0; j < cfg; j++) traj[(size_t)i * cfg + j] = jv(m, j);
    t += dt;
  }
  std::vector<DynRec> dr(nsamp);
  for (int i = k0; i < nsamp; i++) {
    dr[i].init(n, nf);
    for (int j = 0; j < cfg; j++) jv(m, j) = traj[(size_t)i * cfg + j];
    recompute_modelnodes(m);
    dynrec_initialize(m, dr[i], m->rcap);
  }
  for (int i = k0 + 1; i <= nsamp - 2; i++) compute_ders(m, dr[i], 0, dr[i - 1], dr[i + 1], dt);
  for (int i = k0 + 2; i <= nsamp - 3; i++) compute_ders(m, dr[i], 1, dr[i - 1], dr[i + 1], dt);
  for (int h = 0; h < H; h++) {
    int i = k0 + h + 2;
    std::vector<double> y;
    tl_near = NearTrack();
    uint32_t fl = solve_forces(m, dr[i], tau_in + (size_t)h * nmj, y, rule) ? 0u : (HSO_FLAG_GENERAL | HSO_FLAG_DEPENDENT);
    if (tl_near.near()) fl |= HSO_FLAG_NEAR_RANK;
    if (unreach[i]) fl |= HSO_FLAG_UNREACH;
    for (double v : y) if (std::isnan(v)) fl |= HSO_FLAG_NAN;
    if (cf) std::copy(y.begin(), y.end(), cf + (size_t)h * 3 * nf);
    if (flags) flags[h] = fl;
  }
  return 0;
}

}  // namespace

extern "C" {

int hso_model_load(const char* xml_path, hso_model** out) { return load_model(xml_path, out); }
void hso_model_free(hso_model* m) { delete m; }
void hso_model_dims(const hso_model* m, int* d) {
  d[0] = m->n; d[1] = m->nmj; d[2] = m->nf; d[3] = m->cfg; d[4] = m->lik_index; d[5] = (int)m->limbs.size();
}

int hso_model_set_torso_penalty(hso_model* m, int force, int torque) {
  if (!m) return -1;
  if (!force && !torque) return -2;  // mask_l0 == 0: the reference exits ("mask0 not set", ftsolver.cpp:245)
  m->torso_mask = (force ? 1 : 0) | (torque ? 2 : 0);
  return 0;
}

int hso_rollout(const hso_model* m, const hso_gait* g, int n_t, int k0, int H, int basis, int ignore_reach,
                double* q, double* tau, double* cf, double* x, uint32_t* flags, double* work_cot, double* diag) {
  if (!m || !g || n_t <= 0 || k0 < 0 || H <= 0) return -1;
  return run_rollout(m, g, n_t, k0, H, basis, ignore_reach, q, tau, cf, x, flags, work_cot, diag);
}

int hso_forces(const hso_model* m, const hso_gait* g, int n_t, int k0, int H, int ignore_reach, const double* tau_in,
               double* cf, uint32_t* flags) {
  if (!m || !g || !tau_in || n_t <= 0 || k0 < 0 || H <= 0) return -1;
  return run_forces(m, g, n_t, k0, H, ignore_reach, HSO_FORCES_KERNEL, tau_in, cf, flags);
}

int hso_forces_rule(const hso_model* m, const hso_gait* g, int n_t, int k0, int H, int ignore_reach, int rule,
                    const double* tau_in, double* cf, uint32_t* flags) {
  if (!m || !g || !tau_in || n_t <= 0 || k0 < 0 || H <= 0) return -1;
  if (rule != HSO_FORCES_KERNEL && rule != HSO_FORCES_SPARSEQR) return -2;
  return run_forces(m, g, n_t, k0, H, ignore_reach, rule, tau_in, cf, flags);
}

int hso_batch_near(const hso_model* m, const hso_gait* params, int B, int n_t, int k0, int H, int basis,
                   int ignore_reach, int n_threads, double* tau, double* cf, double* work_cot, uint32_t* flags,
                   double* nearv) {
  if (n_threads < 1) n_threads = 1;
  std::vector<int> rc(n_threads, 0);
  auto worker = [&](int tid) {
    for (int b = tid; b < B; b += n_threads) {
      int r = run_rollout(m, &params[b], n_t, k0, H, basis, ignore_reach, nullptr,
                          tau ? tau + (size_t)b * H * m->nmj : nullptr,
                          cf ? cf + (size_t)b * H * 3 * m->nf : nullptr, nullptr,
                          flags ? flags + (size_t)b * H : nullptr,
                          work_cot ? work_cot + 2 * (size_t)b : nullptr, nullptr,
                          nearv ? nearv + 4 * (size_t)b * H : nullptr);
      if (r) rc[tid] = r;
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < n_threads; t++) th.emplace_back(worker, t);
  worker(0);
  for (auto& t : th) t.join();
  for (int r : rc) if (r) return r;
  return 0;
}

int hso_forces_batch(const hso_model* m, const hso_gait* params, int B, int n_t, int k0, int H, int ignore_reach,
                     int n_threads, const double* tau_in, double* cf, uint32_t* flags) {
  if (!m || !params || !tau_in || n_t <= 0 || k0 < 0 || H <= 0) return -1;
  if (n_threads < 1) n_threads = 1;
  std::vector<int> rc(n_threads, 0);
  auto worker = [&](int tid) {
    for (int b = tid; b < B; b += n_threads) {
      int r = run_forces(m, &params[b], n_t, k0, H, ignore_reach, HSO_FORCES_KERNEL, tau_in + (size_t)b * H * m->nmj,
                         cf ? cf + (size_t)b * H * 3 * m->nf : nullptr, flags ? flags + (size_t)b * H : nullptr);
      if (r) rc[tid] = r;
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < n_threads; t++) th.emplace_back(worker, t);
  worker(0);
  for (auto& t : th) t.join();
  for (int r : rc) if (r) return r;
  return 0;
}

int hso_batch(const hso_model* m, const hso_gait* params, int B, int n_t, int k0, int H, int basis,
              int ignore_reach, int n_threads, double* tau, double* cf, double* work_cot, uint32_t* flags) {
  return hso_batch_near(m, params, B, n_t, k0, H, basis, ignore_reach, n_threads, tau, cf, work_cot, flags, nullptr);
}

double hso_lik_roundtrip(const hso_model* m, int n, uint64_t seed) {
  // liklimb::solver_test_yxx (lik.cpp:371-404), m = 1 branch; uses splitmix64 instead of rand()
  if (m->lik_index == 2) return 0;  // bend_solver2 unfinished in the reference (lik.cpp:289-291)
  double worst = 0;
  uint64_t s = seed;
  auto rnd = [&]() {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * (1.0 / 9007199254740992.0);
  };
  tl_ignore_reach = false;
  for (size_t L = 0; L < m->limbs.size(); L++) {
    for (int i = 0; i < n; i++) {
      Vec a0, pos, a1;
      for (int j = 0; j < 3; j++) a0.v[j] = (2 * rnd() - 1) * M_PI;
      bool bend = bend_solver_yxx(pos, a0, m->ls, m->limbs[L].ysign);
      limb_solver_yxx(pos, a1, m->ls, m->limbs[L].ysign, bend);
      a1.subtract(a0);
      for (int j = 0; j < 3; j++) mod_twopi(a1.v[j]);
      double d = a1.v[0] - M_PI;
      mod_twopi(d);
      if (fabs(d) < 1e-3) continue;  // phi+pi branch ignored (lik.cpp:390)
      double e = a1.norm();
      if (e > worst) worst = e;
    }
  }
  return worst;
}

void hso_euler_roundtrip(const double* ang, double* out) {
  Vec o[2];
  o[0].set(0, 0, 0);
  o[1].set(ang);
  Aff A;
  affine_from_orientation(A, o);
  euler_angles_from_affine(A, out);
}

void hso_rot_ztov(const double* v3, double* R9) {
  Vec v;
  v.set(v3);
  double rot[12];
  rot_ztov(rot, v);
  Aff A;
  A.set_rotation(rot);
  for (int j = 0; j < 3; j++) for (int i = 0; i < 3; i++) R9[j * 3 + i] = A.a[j * 4 + i];
}

int hso_pergen_rec(const hso_model* m0, const hso_gait* g, double t, double* rec) {
  hso_model mm = *m0;
  hso_model* m = &mm;
  PGS pgs;
  setup_pergen(m, pgs, g);
  pgs.set_rec(rec, t);
  return 0;
}

int hso_lik(const hso_model* m0, const double* rec, int ignore_reach, double* config, int* unreach) {
  hso_model mm = *m0;
  hso_model* m = &mm;
  for (int j = 0; j < m->cfg; j++) jv(m, j) = config[j];
  tl_ignore_reach = ignore_reach != 0;
  tl_unreach = false;
  const bool ok = set_jvalues_with_lik(m, rec);
  for (int j = 0; j < m->cfg; j++) config[j] = jv(m, j);
  if (unreach) *unreach = tl_unreach ? 1 : 0;
  return ok ? 0 : -10;
}

int hso_fk(const hso_model* m0, const double* config, double* a_ground, double* a_joint) {
  hso_model mm = *m0;
  hso_model* m = &mm;
  for (int j = 0; j < m->cfg; j++) jv(m, j) = config[j];  // kinematicmodel::set_jvalues
  recompute_modelnodes(m);
  for (int i = 0; i < m->n; i++) {
    const Node& nd = m->nodes[i];
    for (int c = 0; c < 4; c++)
      for (int r = 0; r < 3; r++) {
        a_ground[12 * i + 3 * c + r] = nd.A_ground.a[4 * c + r];
        if (a_joint) a_joint[12 * i + 3 * c + r] = nd.jtype != J_NONE ? nd.J_A_ground.a[4 * c + r] : 0.0;
      }
  }
  return 0;
}

double hso_fk_ik_check(const hso_model* m0, const hso_gait* g, double t, int ignore_reach) {
  hso_model mm = *m0;
  hso_model* m = &mm;
  tl_ignore_reach = ignore_reach != 0;
  PGS pgs;
  setup_pergen(m, pgs, g);
  std::vector<double> rec(m->cfg);
  pgs.set_rec(rec.data(), t);
  if (!set_jvalues_with_lik(m, rec.data())) return -1;
  recompute_modelnodes(m);
  double worst = 0;
  for (size_t L = 0; L < m->limbs.size(); L++) {
    Vec fp;
    const Node& ft = m->nodes[m->limbs[L].foot];
    ft.A_ground.mult(ft.capsule_to_pos, fp);
    for (int j = 0; j < 3; j++) worst = std::max(worst, fabs(fp.v[j] - rec[6 + 3 * L + j]));
  }
  return worst;
}

int hso_dynrec_dump(const hso_model* m0, const hso_gait* g, int n_t, int step, double* pos, double* jpos,
                    double* jz, double* mom_rate, double* amr, double* fpos, int32_t* contacts,
                    int32_t* parents, int32_t* footis, int32_t* hinge_ids) {
  hso_model mm = *m0;
  hso_model* m = &mm;
  tl_ignore_reach = true;
  PGS pgs;
  setup_pergen(m, pgs, g);
  int nsamp = step + 5;
  double dt = pgs.pergen.period / n_t;
  std::vector<DynRec> dr(nsamp);
  std::vector<double> rec(m->cfg);
  std::vector<std::vector<double>> traj(nsamp);
  double t = 0;
  for (int i = 0; i < nsamp; i++) {
    pgs.set_rec(rec.data(), t);
    if (!set_jvalues_with_lik(m, rec.data())) return -10;
    traj[i].resize(m->cfg);
    for (int j = 0; j < m->cfg; j++) traj[i][j] = jv(m, j);
    t += dt;
  }
  for (int i = step; i < nsamp; i++) {
    dr[i].init(m->n, m->nf);
    for (int j = 0; j < m->cfg; j++) jv(m, j) = traj[i][j];
    recompute_modelnodes(m);
    dynrec_initialize(m, dr[i], m->rcap);
  }
  for (int i = step + 1; i <= nsamp - 2; i++) compute_ders(m, dr[i], 0, dr[i - 1], dr[i + 1], dt);
  compute_ders(m, dr[step + 2], 1, dr[step + 1], dr[step + 3], dt);
  const DynRec& d = dr[step + 2];
  for (int i = 0; i < m->n; i++)
    for (int j = 0; j < 3; j++) {
      pos[3 * i + j] = d.pos[i].v[j];
      jpos[3 * i + j] = d.jpos[i].v[j];
      jz[3 * i + j] = d.jzaxis[i].v[j];
      mom_rate[3 * i + j] = d.mom_rate[i].v[j];
      amr[3 * i + j] = d.ang_mom_rate[i].v[j];
    }
  for (int f = 0; f < m->nf; f++) {
    for (int j = 0; j < 3; j++) fpos[3 * f + j] = d.fpos[f].v[j];
    contacts[f] = d.contacts[f];
    footis[f] = m->footis[f];
  }
  for (int i = 0; i < m->n; i++) parents[i] = m->parentis[i];
  for (int i = 0; i < m->nmj; i++) hinge_ids[i] = m->hinge_ids[i];
  return 3 * d.ncontacts();
}

int hso_residuals(const hso_model* m0, const hso_gait* g, int n_t, int step, int basis, double* out2) {
  hso_model mm = *m0;
  hso_model* m = &mm;
  tl_ignore_reach = true;
  PGS pgs;
  setup_pergen(m, pgs, g);
  int nsamp = step + 5;
  double dt = pgs.pergen.period / n_t;
  std::vector<DynRec> dr(nsamp);
  std::vector<double> rec(m->cfg);
  double t = 0;
  std::vector<std::vector<double>> traj(nsamp);
  for (int i = 0; i < nsamp; i++) {
    pgs.set_rec(rec.data(), t);
    if (!set_jvalues_with_lik(m, rec.data())) return -10;
    traj[i].resize(m->cfg);
    for (int j = 0; j < m->cfg; j++) traj[i][j] = jv(m, j);
    t += dt;
  }
  for (int i = 0; i < nsamp; i++) {
    dr[i].init(m->n, m->nf);
    for (int j = 0; j < m->cfg; j++) jv(m, j) = traj[i][j];
    recompute_modelnodes(m);
    dynrec_initialize(m, dr[i], m->rcap);
  }
  for (int i = 1; i <= nsamp - 2; i++) compute_ders(m, dr[i], 0, dr[i - 1], dr[i + 1], dt);
  for (int i = 2; i <= nsamp - 3; i++) compute_ders(m, dr[i], 1, dr[i - 1], dr[i + 1], dt);
  const DynRec& d = dr[step + 2];
  Mat B0;
  std::vector<double> f;
  build_B0_f(m, d, B0, f);
  std::vector<double> x;
  Mat N;
  if (basis == HSO_BASIS_ORTHO) {
    HQR qr0;
    qr0.compute(B0);
    x = qr0.solve(f);
  } else {
    x = tree_particular(m, d, f);
  }
  std::vector<double> r = matvec(B0, x);
  double e0 = 0;
  for (size_t i = 0; i < r.size(); i++) e0 = std::max(e0, fabs(r[i] - f[i]));
  Mat B = build_B_contacts(m, d, B0);
  int k = B.c - 6 * m->n;
  if (basis == HSO_BASIS_ORTHO) {
    int mmn = B.c;
    Mat Bsq(mmn, mmn);
    for (int j = 0; j < mmn; j++) for (int i = 0; i < 6 * m->n; i++) Bsq(i, j) = B(i, j);
    HQR qr1;
    qr1.compute(transpose(Bsq));
    N = Mat(mmn, k);
    for (int i = 0; i < k; i++) {
      std::vector<double> e(mmn, 0.0);
      e[mmn - 1 - i] = 1;
      std::vector<double> col = qr1.apply_Q(e);
      for (int rr = 0; rr < mmn; rr++) N(rr, i) = col[rr];
    }
  } else {
    Mat Nt = tree_null_basis(m, d);
    N = Mat(6 * m->n + k, k);
    for (int j = 0; j < k; j++) {
      for (int i = 0; i < 6 * m->n; i++) N(i, j) = Nt(i, j);
      N(6 * m->n + j, j) = 1;
    }
  }
  Mat BN = matmul(B, N);
  double e1 = 0;
  for (double v : BN.d) e1 = std::max(e1, fabs(v));
  out2[0] = e0;
  out2[1] = e1;
  return k;
}

}  // extern "C"

// closed-loop simulation restatement (same translation unit: uses the model code above)
#ifndef HSO_FLOPCOUNT
#include "hs_oracle_sim.cpp"
#endif
