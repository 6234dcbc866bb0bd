// hslabs.hpp -- C++ shim over include/hslabs.h that keeps the reference's
// call shapes for the hot path, so player.cpp-style callers switch by changing
// includes. Header-only; link with -lhslabs.
//
//   kinematicmodel::load_fromxml / get_config_dim / number_of_motor_joints /
//            get_mnode / get_joint_values / get_lik / recompute_modelnodes /
//            set_jvalues_with_lik / set_jvalues / get_jvalues / orient_torso /
//            get_foot_mnodes                                               (model.h:96-137)
//   modelnode / modeljoint (read side), affine / extvec (read side)        (model.h:34-86, matrix.h)
//   liksolver::place_limbs / place_limb / get_limb_hip_pos /
//            set_ignore_reach_flag / get_number_of_limbs                   (lik.h, lik.cpp:82-146)
//   pergensetup::set_rec                                                   (pergen.cpp:225-239)
//   arrayops, str_to_val                                                   (core.h:13, 27-48)
//   pgsconfigparams                                                        (pergen.h:137-146)
//   pergensetup (setup parameters of one gait)                             (pergen.h:68-108)
//   periodic::record_trajectory / compute_dynrecs / compute_dynrec_ders /
//            switch_torso_penalty / compute_torques_over_period /
//            get_computed_torques / work_over_period / get_total_mass /
//            get_contforce_stat / get_motor_torques /
//            solve_contforces_given_torques / get_complete_traj /
//            get_motor_adas                                                (periodic.h:27-87)
//   modelplayer::make_pergensu / measure_cot / measure_cot_sweep /
//            record_per_traj / test_dynamics                               (player.cpp:147-321,
//                                                                           617-629; playerexperim.cpp:95-121)
//   modelplayer::setup_per_controller / simulate_ode / get_ode_motor_adas /
//            torso position, fall_check                                    (player.cpp:325-382, 669-681;
//                                                                           visualization.cpp:366-374)
//   new_2d_array / delete_2d_array / save_2d_array                         (core.h:11-14)
//
// Differences from the reference: errors throw hslabs::error instead of
// exit(1); the whole cycle is computed on the GPU by compute_torques_over_period
// (record_trajectory / compute_dynrecs / compute_dynrec_ders only record their
// arguments; switch_torso_penalty sets the model's solver mask, as the reference's
// ftsolver holds it); measure_cot_sweep runs all
// sweep values in one batched launch.
#ifndef HSLABS_HPP
#define HSLABS_HPP

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <iostream>
#include <set>
#include <sstream>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "hslabs.h"

namespace hslabs {

struct error : std::runtime_error {
  int code;
  error(int c, const std::string& what) : std::runtime_error(what), code(c) {}
};

inline void check(int rc, const char* what) {
  if (rc != HS_OK) throw error(rc, std::string(what) + ": " + hs_last_error());
}

// core.h:11-14
inline double** new_2d_array(int n, int m) {
  double** a = new double*[n];
  for (int i = 0; i < n; i++) a[i] = new double[m];
  return a;
}
inline void delete_2d_array(double** a, int n) {
  if (!a) return;
  for (int i = 0; i < n; i++) delete[] a[i];
  delete[] a;
}
inline void save_2d_array(double** a, int n, int m, const std::string& fname, bool append) {
  std::ofstream f(fname.c_str(), append ? std::ios_base::app : std::ios_base::out);
  for (int i = 0; i < n; i++) {
    for (int j = 0; j < m; j++) f << (j ? " " : "") << a[i][j];
    f << "\n";
  }
}

// core.h:13 (core.cpp:8-12): reads whitespace-separated doubles from str into val until one
// fails to parse
inline void str_to_val(const char* str, double* val) {
  std::istringstream in(str ? str : "");
  double d;
  while (in >> d) *val++ = d;
}

// core.h:27-48: arithmetic on double arrays of length n
class arrayops {
  int n_ = 0;
  std::vector<double> tmp_;

 public:
  arrayops() {}
  explicit arrayops(int n) : n_(n) {}
  void set_n(int n) { n_ = n; tmp_.clear(); }
  void print(const double* a) const {
    for (int i = 0; i < n_; i++) std::cout << (i ? " " : "") << a[i];
    std::cout << std::endl;
  }
  void assign(double* a, const double* a1) const { std::copy(a1, a1 + n_, a); }
  double* add(double* a, const double* a1) const { for (int i = 0; i < n_; i++) a[i] += a1[i]; return a; }
  double* subtract(double* a, const double* a1) const { for (int i = 0; i < n_; i++) a[i] -= a1[i]; return a; }
  double* times(double* a, double b) const { for (int i = 0; i < n_; i++) a[i] *= b; return a; }
  // period-b wrap into (-b/2, b/2] of arguments in (-3b/2, 3b/2] (core.cpp:120-131)
  double* modulus(double* a, double b) const {
    const double bh = b / 2;
    for (int i = 0; i < n_; i++) {
      if (a[i] > bh) a[i] -= b;
      else if (a[i] <= -bh) a[i] += b;
    }
    return a;
  }
  double dot(const double* a, const double* a1) const {
    double s = 0;
    for (int i = 0; i < n_; i++) s += a[i] * a1[i];
    return s;
  }
  double norm(const double* a) const { return std::sqrt(dot(a, a)); }
  double distance(const double* a, const double* a1) {
    tmp_.assign(a, a + n_);
    subtract(tmp_.data(), a1);
    return norm(tmp_.data());
  }
  void assign_scalar(double* a, double b) const { std::fill(a, a + n_, b); }
  double l1_norm(const double* a) const {
    double s = 0;
    for (int i = 0; i < n_; i++) s += std::fabs(a[i]);
    return s;
  }
  double** new_2d_array(int m) const { return hslabs::new_2d_array(m, n_); }
  void delete_2d_array(double** a, int m) const { hslabs::delete_2d_array(a, m); }
};

// matrix.h:57-88 (the part callers of the kinematic model use): a point (x, y, z, 1)
class extvec {
  double v_[4] = {0, 0, 0, 1};

 public:
  extvec() {}
  extvec(double x, double y, double z) { set(x, y, z); }
  void set(double x, double y, double z) { v_[0] = x; v_[1] = y; v_[2] = z; }
  void set(const double* a) { set(a[0], a[1], a[2]); }
  void set_v(int i, double val) { v_[i] = val; }
  double get_v(int i) const { return v_[i]; }
  double* get_data() { return v_; }
  const double* get_data() const { return v_; }
  void get_components(double& x, double& y, double& z) const { x = v_[0]; y = v_[1]; z = v_[2]; }
  void get_components(double* p) const { std::copy(v_, v_ + 3, p); }
  void print() const { std::cout << v_[0] << " " << v_[1] << " " << v_[2] << std::endl; }
};

// matrix.h:16-55 (read side): a rigid transform [rot, transl; 0 0 0 1], stored column-wise in 16
// doubles like the reference, so get_data() + 8 is the z axis (dynrec.cpp:84-93)
class affine {
  double a_[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};

 public:
  double* get_data() { return a_; }
  const double* get_data() const { return a_; }
  double get_a(int i, int j) const { return a_[4 * j + i]; }
  void get_translation(extvec& t) const { t.set(a_[12], a_[13], a_[14]); }
  // u = A (v, 1) (matrix.cpp:149-164)
  void mult(const extvec& v, extvec& u) const {
    double r[3];
    for (int i = 0; i < 3; i++) {
      double s = 0;
      for (int k = 0; k < 3; k++) s += a_[4 * k + i] * v.get_v(k);
      r[i] = s + a_[12 + i];
    }
    u.set(r);
  }
  // from the ABI's 3x4 column-major block ([c * 3 + r])
  void set_from34(const double* m) {
    for (int c = 0; c < 4; c++) {
      for (int r = 0; r < 3; r++) a_[4 * c + r] = m[3 * c + r];
      a_[4 * c + 3] = (c == 3) ? 1.0 : 0.0;
    }
  }
  void print() const {
    for (int i = 0; i < 4; i++) {
      for (int j = 0; j < 4; j++) std::cout << (j ? " " : "") << get_a(i, j);
      std::cout << std::endl;
    }
  }
};

enum joint_type { free6, hinge, slider };  // model.h:26

class kinematicmodel;

// model.h:34-51 (read side): the joint of a model node, its values and ground frame
class modeljoint {
  friend class kinematicmodel;
  joint_type type_ = hinge;
  affine A_ground_;
  double* values_ = nullptr;

 public:
  double* get_values() { return values_; }
  affine* get_A_ground() { return &A_ground_; }
  joint_type get_type() const { return type_; }
};

// model.h:64-86 (read side)
class modelnode {
  friend class kinematicmodel;
  affine A_ground_;
  modeljoint joint_;
  bool has_joint_ = false;
  modelnode* parent_ = nullptr;
  std::vector<modelnode*> kids_;
  hs_node_info info_{};

 public:
  const affine* get_A_ground() const { return &A_ground_; }
  modeljoint* get_joint() const { return has_joint_ ? const_cast<modeljoint*>(&joint_) : nullptr; }
  modelnode* get_first_child() const { return kids_.empty() ? nullptr : kids_.front(); }
  modelnode* get_parent() const { return parent_; }
  const std::vector<modelnode*>& get_child_nodes() const { return kids_; }
  // hs_node_info: odepart positions (com, foot capsule end), mass, foot / limb / motor indices
  const hs_node_info& info() const { return info_; }
};

// lik.cpp:142: one process-wide flag, like the reference's global ignore_reach_flag
inline bool& lik_ignore_reach_flag() {
  static bool flag = false;
  return flag;
}

class liksolver;

// kinematicmodel (model.h:96-137): the per-configuration API runs on the GPU through hs_model_lik /
// hs_model_fk (one configuration per call here; the ABI takes batches)
class kinematicmodel {
  hs_model_t h_ = nullptr;
  hs_model_dims d_{};
  std::string xmlfname_;
  mutable std::vector<double> jv_;       // joint_values (model.h:100), get_jvalues order
  std::vector<double*> jv_ptrs_;
  mutable std::vector<modelnode> nodes_;  // mnodes, XML preorder
  liksolver* lik_ = nullptr;

 public:
  explicit kinematicmodel(bool /*vis_flag*/ = false) {}
  ~kinematicmodel();
  kinematicmodel(const kinematicmodel&) = delete;
  kinematicmodel& operator=(const kinematicmodel&) = delete;
  // model.cpp:224-242: load, build the node tree, recompute_modelnodes
  void load_fromxml(const std::string& fname, int lik_variant = -1);
  bool if_loaded() const { return h_ != nullptr; }
  std::string get_xmlfname() const { return xmlfname_; }
  int get_config_dim() const { return d_.config_dim; }
  int number_of_motor_joints() const { return d_.nmj; }
  int number_of_parts() const { return d_.n_parts; }
  int number_of_feet() const { return d_.nfeet; }
  double total_mass() const { return d_.total_mass; }
  hs_model_t handle() const { return h_; }
  // model.h:108-111
  const modelnode* get_mnode(int i) const { return &nodes_.at((size_t)i); }
  std::vector<double*>* get_joint_values() { return &jv_ptrs_; }
  const liksolver* get_lik() const { return lik_; }
  // model.cpp:314-318: every node's A_ground (and its joint's) from the current joint values
  void recompute_modelnodes() const {
    std::vector<double> ag((size_t)d_.n_parts * 12), aj((size_t)d_.n_parts * 12);
    check(hs_model_fk_host(h_, 1, jv_.data(), d_.config_dim, ag.data(), aj.data()), "recompute_modelnodes");
    for (size_t i = 0; i < nodes_.size(); i++) {
      nodes_[i].A_ground_.set_from34(&ag[12 * i]);
      nodes_[i].joint_.A_ground_.set_from34(&aj[12 * i]);
    }
  }
  // model.cpp:354-359: torso values from rec, recompute_modelnodes, then liksolver::place_limbs
  // (lik.cpp:89-99) with the foot positions rec[6 ..]; throws where the reference exits
  // (lik.cpp:321-330)
  void set_jvalues_with_lik(const double* rec) const {
    std::copy(rec, rec + 6, jv_.begin());
    recompute_modelnodes();
    place_limbs(rec + 6);
  }
  // model.cpp:361-372
  void set_jvalues(const double* values) const { std::copy(values, values + d_.config_dim, jv_.begin()); }
  void get_jvalues(double* values) const { std::copy(jv_.begin(), jv_.end(), values); }
  // model.cpp:403-409
  void orient_torso(const extvec* orientation) const {
    for (int i = 0; i < 2; i++)
      for (int j = 0; j < 3; j++) jv_[(size_t)(3 * i + j)] = orientation[i].get_v(j);
    recompute_modelnodes();
  }
  // model.cpp:411-420: the feet's model nodes
  void get_foot_mnodes(std::set<modelnode*>& foot_set) const {
    for (modelnode& n : nodes_)
      if (n.info_.foot >= 0) foot_set.insert(&n);
  }
  // liksolver::place_limbs on this model: the limb values for foot positions feet[3 * n_limbs]
  // in the ground frame, from the torso's current values (rows of hs_model_lik). only_limb >= 0
  // sets that limb's values alone (liksolver::place_limb, lik.cpp:82-85; the other rows of feet
  // are then ignored). A target out of reach throws unless lik_ignore_reach_flag() (where the
  // reference prints the limb and exits, lik.cpp:321-330).
  void place_limbs(const double* feet, int only_limb = -1) const {
    std::vector<double> rec(6 + 3 * (size_t)d_.n_limbs), q(jv_);
    std::copy(jv_.begin(), jv_.begin() + 6, rec.begin());
    std::copy(feet, feet + 3 * d_.n_limbs, rec.begin() + 6);
    uint32_t status = 0;
    check(hs_model_lik_host(h_, 1, rec.data(), 1, q.data(), &status), "place_limbs");
    for (int L = 0; L < d_.n_limbs; L++) {
      if (only_limb >= 0 && L != only_limb) continue;
      if ((status & HS_LIK_LIMB_BIT(L)) && !lik_ignore_reach_flag())
        throw error(HS_E_ARG, "place_limbs: the target of limb " + std::to_string(L) + " is out of reach");
    }
    if (only_limb < 0) {
      jv_ = q;
      return;
    }
    const modelnode* n = nullptr;
    for (const modelnode& c : nodes_)
      if (c.info_.limb == only_limb) n = &c;
    for (int k = 0; k < 3 && n; k++, n = n->get_first_child()) jv_[6 + (size_t)n->info_.hinge] = q[6 + (size_t)n->info_.hinge];
  }
};

// liksolver (lik.h:27-58, the caller-facing part), over its kinematicmodel
class liksolver {
  const kinematicmodel* model_;
  std::vector<const modelnode*> limb_child_;

 public:
  explicit liksolver(const kinematicmodel* model) : model_(model) {
    for (int i = 0; i < model->number_of_parts(); i++)
      if (model->get_mnode(i)->info().limb >= 0) {
        const int L = model->get_mnode(i)->info().limb;
        if ((int)limb_child_.size() <= L) limb_child_.resize((size_t)L + 1);
        limb_child_[(size_t)L] = model->get_mnode(i);
      }
  }
  int get_number_of_limbs() const { return (int)limb_child_.size(); }
  void set_ignore_reach_flag(bool value) const { lik_ignore_reach_flag() = value; }  // lik.cpp:144-146
  void place_limbs(const double* feet) const { model_->place_limbs(feet); }        // lik.cpp:89-99
  // lik.cpp:82-85: one limb, the others kept
  void place_limb(int limbi, double x, double y, double z) const {
    std::vector<double> feet(3 * (size_t)get_number_of_limbs());
    for (int L = 0; L < get_number_of_limbs(); L++) {  // every row the target (only limbi's is kept)
      feet[3 * (size_t)L] = x;
      feet[3 * (size_t)L + 1] = y;
      feet[3 * (size_t)L + 2] = z;
    }
    model_->place_limbs(feet.data(), limbi);
  }
  // lik.cpp:104-106, 358-361: the limb's top-link body position
  void get_limb_hip_pos(int limbi, extvec& pos) const { limb_child_.at((size_t)limbi)->get_A_ground()->get_translation(pos); }
  // lik.cpp:364-366: child -> first child -> first child
  const modelnode* get_foot(int limbi) const {
    return limb_child_.at((size_t)limbi)->get_first_child()->get_first_child();
  }
};

inline kinematicmodel::~kinematicmodel() {
  delete lik_;
  hs_model_free(h_);
}

inline void kinematicmodel::load_fromxml(const std::string& fname, int lik_variant) {
  delete lik_;
  lik_ = nullptr;
  hs_model_free(h_);
  h_ = nullptr;
  check(hs_model_load_ex(fname.c_str(), lik_variant, &h_), "load_fromxml");
  check(hs_model_get_dims(h_, &d_), "hs_model_get_dims");
  xmlfname_ = fname;
  jv_.assign((size_t)d_.config_dim, 0.0);
  jv_ptrs_.clear();
  for (double& v : jv_) jv_ptrs_.push_back(&v);
  nodes_.assign((size_t)d_.n_parts, modelnode());
  for (int i = 0; i < d_.n_parts; i++) {
    modelnode& n = nodes_[(size_t)i];
    check(hs_model_get_node(h_, i, &n.info_), "hs_model_get_node");
    n.parent_ = n.info_.parent >= 0 ? &nodes_[(size_t)n.info_.parent] : nullptr;
    for (int k = 0; k < n.info_.n_kids; k++) n.kids_.push_back(&nodes_[(size_t)n.info_.kids[k]]);
    n.has_joint_ = n.info_.jtype >= 0;
    n.joint_.type_ = n.info_.jtype == 0 ? free6 : hinge;
    n.joint_.values_ = n.info_.jtype == 0 ? &jv_[0] : (n.info_.hinge >= 0 ? &jv_[6 + (size_t)n.info_.hinge] : nullptr);
  }
  lik_ = new liksolver(this);
  recompute_modelnodes();
}

struct pgsconfigparams {
  std::string fname;
  double orientation[2][3] = {{0, 0, 0}, {0, 0, 0}};
  double step_duration = 0;
  double TLh[3] = {0, 0, 0};
  double curvature = 0;
  std::pair<int, double> foot_shift{-1, 0.0};
  void set_TLh(double period, double step_length, double step_height) {
    TLh[0] = period; TLh[1] = step_length; TLh[2] = step_height;
  }
  hs_gait_params to_c() const {
    hs_gait_params g;
    std::memset(&g, 0, sizeof(g));
    for (int i = 0; i < 3; i++) { g.torso_pos[i] = orientation[0][i]; g.torso_angles[i] = orientation[1][i]; }
    g.step_duration = step_duration;
    g.period = TLh[0]; g.step_length = TLh[1]; g.step_height = TLh[2];
    g.curvature = curvature;
    g.foot_shift_type = foot_shift.first;
    g.foot_shift = foot_shift.second;
    return g;
  }
  static pgsconfigparams from_c(const hs_gait_params& g, const std::string& fname) {
    pgsconfigparams p;
    p.fname = fname;
    for (int i = 0; i < 3; i++) { p.orientation[0][i] = g.torso_pos[i]; p.orientation[1][i] = g.torso_angles[i]; }
    p.step_duration = g.step_duration;
    p.set_TLh(g.period, g.step_length, g.step_height);
    p.curvature = g.curvature;
    p.foot_shift = std::make_pair((int)g.foot_shift_type, g.foot_shift);
    return p;
  }
};

class pergensetup;

// The periodicgenerator of a pergensetup (pergen.h:27-58), the accessors callers read through
// pergensetup::get_pergen() (player.cpp:274 measure_cot: pgs->get_pergen()->get_step_length())
class periodicgenerator {
  const pgsconfigparams* pcp_;

 public:
  explicit periodicgenerator(const pgsconfigparams* pcp) : pcp_(pcp) {}
  double get_period() const { return pcp_->TLh[0]; }
  double get_step_length() const { return pcp_->TLh[1]; }
  double get_step_duration() const { return pcp_->step_duration; }
  double get_curvature() const { return pcp_->curvature; }
  void get_TLh(double TLh[3]) const { std::copy(pcp_->TLh, pcp_->TLh + 3, TLh); }
};

// The gait of one rollout (pergensetup, pergen.h:68-108): its pgsconfigparams, the record
// transform (pergen.h:75-76) and accessors.
class pergensetup {
  pgsconfigparams pcp_;
  int n_;
  const kinematicmodel* model_;
  periodicgenerator pergen_{&pcp_};
  bool rec_transform_flag_ = false;  // pergen.cpp:207
  double rec_transl_[3] = {0, 0, 0}, rec_eas_[3] = {0, 0, 0};

 public:
  pergensetup(int n_limbs, const pgsconfigparams& pcp, const kinematicmodel* model = nullptr)
      : pcp_(pcp), n_(n_limbs), model_(model) {}
  pergensetup(const pergensetup& o)
      : pcp_(o.pcp_), n_(o.n_), model_(o.model_), rec_transform_flag_(o.rec_transform_flag_) {
    std::copy(o.rec_transl_, o.rec_transl_ + 3, rec_transl_);
    std::copy(o.rec_eas_, o.rec_eas_ + 3, rec_eas_);
  }
  pergensetup& operator=(const pergensetup&) = delete;
  // pergen.cpp:225-239: torso position and angles, then the feet in lik order, at time t, transformed
  // by the record transform when set (needs the model the gait was set up for: make_pergensu passes it)
  void set_rec(double* rec, double t) const {
    if (!model_) throw error(HS_E_ARG, "pergensetup without a model");
    hs_gait_params g = to_c();
    check(hs_pergen_rec_host(model_->handle(), &g, 1, &t, 1, rec), "set_rec");
  }
  int get_limb_number() const { return n_; }
  int get_config_dim() const { return 6 + 3 * n_; }
  double get_period() const { return pcp_.TLh[0]; }
  double get_step_length() const { return pcp_.TLh[1]; }
  const periodicgenerator* get_pergen() const { return &pergen_; }  // pergen.h:81
  const kinematicmodel* get_model() const { return model_; }
  void get_config_params(pgsconfigparams* pcp) const { *pcp = pcp_; }
  const pgsconfigparams& params() const { return pcp_; }
  void set_TLh(double T, double L, double h) { pcp_.set_TLh(T, L, h); }
  void set_TLh(const double TLh[3]) { pcp_.set_TLh(TLh[0], TLh[1], TLh[2]); }
  // pergen.cpp:316-320: rec_transform = affine_from_orientation({rec_transl, rec_eas}), flag on
  void set_rec_transform(const extvec& rec_transl, const extvec& rec_eas) {
    rec_transl.get_components(rec_transl_);
    rec_eas.get_components(rec_eas_);
    rec_transform_flag_ = true;
  }
  // pergen.cpp:309-313: the rotation by Euler angles, the transform's translation kept
  void set_rec_rotation(const extvec& rec_eas) {
    extvec t(rec_transl_[0], rec_transl_[1], rec_transl_[2]);
    set_rec_transform(t, rec_eas);
  }
  // pergen.cpp:338-342 (pgssweeper::next, pergen.cpp:446)
  void copy_rec_transform(const pergensetup* pgs) {
    rec_transform_flag_ = pgs->rec_transform_flag_;
    std::copy(pgs->rec_transl_, pgs->rec_transl_ + 3, rec_transl_);
    std::copy(pgs->rec_eas_, pgs->rec_eas_ + 3, rec_eas_);
  }
  bool get_rec_transform_flag() const { return rec_transform_flag_; }
  // the ABI record of this gait: pgsconfigparams plus the record transform
  hs_gait_params to_c() const {
    hs_gait_params g = pcp_.to_c();
    g.rec_transform_flag = rec_transform_flag_ ? 1 : 0;
    for (int i = 0; i < 3; i++) { g.rec_transl[i] = rec_transl_[i]; g.rec_eas[i] = rec_eas_[i]; }
    return g;
  }
};

// pgssweeper (pergen.h:110-134; pergen.cpp:400-449): iterates over gaits made from pgs0 by
// sweeping one parameter, each with pgs0's record transform (next, pergen.cpp:433-449)
class pgssweeper {
  const pergensetup* pgs0_;
  pergensetup* pgs_ = nullptr;
  int parami_ = -1, n_val_ = 0, vali_ = 0;
  double val0_ = 0, delval_ = 0, val_ = 0;

 public:
  pgssweeper(const pergensetup* pgs, const kinematicmodel* /*model*/ = nullptr) : pgs0_(pgs) {}
  ~pgssweeper() { delete pgs_; }
  pgssweeper(const pgssweeper&) = delete;
  pgssweeper& operator=(const pgssweeper&) = delete;
  pergensetup* get_pgs() const { return pgs_; }
  double get_val() const { return val_; }
  // pergen.cpp:417-430; throws where the reference exits (unknown parameter)
  void sweep(const std::string& param_name, double val0, double val1, int n_val) {
    val0_ = val0;
    n_val_ = n_val;
    delval_ = (val1 - val0) / n_val;
    vali_ = 0;
    const char* names[] = {"step_duration", "period", "step_length", "step_height"};
    parami_ = -1;
    for (int i = 0; i < 4; i++)
      if (param_name == names[i]) parami_ = i;
    if (parami_ < 0) throw error(HS_E_ARG, "cannot sweep over " + param_name);
    std::cout << "sweeping over " << param_name << ":" << std::endl;
  }
  // pergen.cpp:433-449
  bool next() {
    if (vali_ > n_val_) {
      vali_ = 0;
      return false;
    }
    val_ = val0_ + vali_ * delval_;
    vali_++;
    delete pgs_;
    pgs_ = nullptr;
    pgsconfigparams pcp;
    pgs0_->get_config_params(&pcp);
    if (parami_ == 0) pcp.step_duration = val_;
    else if (parami_ > 0 && parami_ < 4) pcp.TLh[parami_ - 1] = val_;
    pgs_ = new pergensetup(pgs0_->get_limb_number(), pcp, pgs0_->get_model());
    pgs_->copy_rec_transform(pgs0_);
    return true;
  }
};

class periodic {
  const kinematicmodel* model_;
  const pergensetup* pgs_ = nullptr;
  int n_t_ = 0;
  mutable std::vector<double> tau_;  // computed_torques: row h = trajectory sample h + 2 (periodic.cpp:387)
  std::vector<double> cf_, x_, wc_;
  std::vector<uint32_t> flags_;
  std::vector<double> rec_;       // get_complete_traj records
  std::vector<double> last_tau_;  // motor torques of the solver's last solve (get_motor_torques)
  mutable std::vector<double> masses_;
  mutable std::vector<int> parentis_, footis_;
  double min_cfz_ = 1e10, max_mu_ = -1e10;

  hs_gait_params gait() const {
    if (!pgs_) throw error(HS_E_ARG, "record_trajectory first");
    return pgs_->to_c();
  }
  // dynrecs[i] exists with its derivatives for samples i = 2 .. n_t + 2 (traj_size = n_t + 5,
  // periodic.cpp:79, 192-202); the reference reads out of bounds elsewhere, this throws
  int step_of(int i) const {
    if (!pgs_) throw error(HS_E_ARG, "record_trajectory first");
    if (i < 2 || i > n_t_ + 2) throw error(HS_E_ARG, "trajectory sample " + std::to_string(i) + " has no dynamics record");
    return i - 2;
  }

 public:
  // periodic.cpp:10-58 (set_dynparts): masses, parent ids and foot part ids in preorder
  explicit periodic(const kinematicmodel* model) : model_(model) {
    for (int i = 0; i < model->number_of_parts(); i++) {
      const hs_node_info& nd = model->get_mnode(i)->info();
      masses_.push_back(nd.mass);
      parentis_.push_back(nd.parent);
      if (nd.foot >= 0) footis_.push_back(i);
    }
  }
  // periodic.h:43-48
  int get_number_of_dynparts() const { return (int)masses_.size(); }
  double* get_masses() const { return masses_.data(); }
  int* get_parentis() const { return parentis_.data(); }
  int* get_footis() const { return footis_.data(); }
  void record_trajectory(const pergensetup* pgs, int n_t) {
    pgs_ = pgs;
    n_t_ = n_t;
    tau_.clear();
    rec_.clear();
    last_tau_.clear();
  }
  void compute_dynrecs() {}
  void compute_dynrec_ders() {}
  // ftsolver.cpp:262-273 through periodic.cpp:205-207: a setting of the model's solver, used by every
  // later solve on it (hs_model_set_torso_penalty); (0,0) throws where the reference exits
  void switch_torso_penalty(bool force, bool torque) {
    check(hs_model_set_torso_penalty(model_->handle(), force ? 1 : 0, torque ? 1 : 0), "switch_torso_penalty");
  }
  int get_nt() const { return n_t_; }
  int get_nfeet() const { return model_->number_of_feet(); }
  double get_total_mass() const { return model_->total_mass(); }
  // periodic.cpp:377-391 (+ analyze_contforces 347-357)
  void compute_torques_over_period() {
    const int nmj = model_->number_of_motor_joints(), nf = model_->number_of_feet();
    const int n = model_->number_of_parts(), cfg = model_->get_config_dim();
    hs_gait_params g = gait();
    tau_.assign((size_t)n_t_ * nmj, 0);
    cf_.assign((size_t)n_t_ * 3 * nf, 0);
    x_.assign((size_t)n_t_ * 6 * n, 0);
    wc_.assign(2, 0);
    flags_.assign(n_t_, 0);
    std::vector<double> q((size_t)n_t_ * cfg);
    check(hs_run_host(model_->handle(), &g, 1, n_t_, 0, n_t_, 1, q.data(), tau_.data(), cf_.data(), x_.data(),
                      flags_.data(), wc_.data()),
          "compute_torques_over_period");
    min_cfz_ = 1e10;
    max_mu_ = -1e10;
    for (int h = 0; h < n_t_; h++)
      for (int f = 0; f < nf; f++) {
        const double* c = &cf_[((size_t)h * nf + f) * 3];
        if (c[2] < min_cfz_) min_cfz_ = c[2];
        double mu = std::sqrt(c[0] * c[0] + c[1] * c[1]) / c[2];
        if (mu > max_mu_) max_mu_ = mu;
      }
    last_tau_.assign(tau_.end() - nmj, tau_.end());  // the loop's last solve: sample n_t + 1
  }
  // periodic.h:51: computed_torques[i % n_t] holds the torques of trajectory sample i
  double* get_computed_torques(int i) const {
    if (tau_.empty()) throw error(HS_E_ARG, "compute_torques_over_period first");
    int h = ((i - 2) % n_t_ + n_t_) % n_t_;
    return &tau_[(size_t)h * model_->number_of_motor_joints()];
  }
  const double* get_contact_forces(int i) const {
    int h = ((i - 2) % n_t_ + n_t_) % n_t_;
    return &cf_[(size_t)h * 3 * model_->number_of_feet()];
  }
  uint32_t get_flags(int i) const { return flags_[((i - 2) % n_t_ + n_t_) % n_t_]; }
  void get_contforce_stat(double* stat) const { stat[0] = min_cfz_; stat[1] = max_mu_; }
  // periodic.cpp:328-343: the motor torques of the force/torque solver's last solve (the last sample
  // of compute_torques_over_period, or solve_torques_contforces' sample)
  void get_motor_torques(double* motor_torques) const {
    if (last_tau_.empty()) throw error(HS_E_ARG, "no force/torque solve yet");
    std::copy(last_tau_.begin(), last_tau_.end(), motor_torques);
  }
  // periodic.cpp:361-366: motor torques and contact forces (3 nfeet, airborne feet 0) of sample i
  void solve_torques_contforces(int i, double* torques, double* contforces) {
    hs_gait_params g = gait();
    const int k0 = step_of(i), nmj = model_->number_of_motor_joints();
    std::vector<double> t((size_t)nmj);
    check(hs_run_host(model_->handle(), &g, 1, n_t_, k0, 1, 1, nullptr, t.data(), contforces, nullptr, nullptr,
                      nullptr),
          "solve_torques_contforces");
    std::copy(t.begin(), t.end(), torques);
    last_tau_ = t;
  }
  // periodic.cpp:368-374 (forcetorquesolver::solve_forces): forces of all feet for sample i
  void solve_contforces_given_torques(int i, double* contforces, const double* torques) const {
    hs_gait_params g = gait();
    const int k0 = step_of(i);
    check(hs_run_forces_host(model_->handle(), &g, 1, n_t_, k0, 1, 1, torques, contforces, nullptr),
          "solve_contforces_given_torques");
  }
  // periodic.cpp:406-426: n_t records of (q, dq, torques) = 2 config_dim + nmj
  void get_complete_traj(double** complete_traj) {
    const int len = 2 * model_->get_config_dim() + model_->number_of_motor_joints();
    ensure_complete_traj();
    for (int i = 0; i < n_t_; i++) std::copy(&rec_[(size_t)i * len], &rec_[(size_t)i * len] + len, complete_traj[i]);
  }
  // periodic.cpp:408-417: the record of time step tsi < n_t (tsi < 2 read at tsi + n_t)
  void get_complete_traj_rec(int tsi, double* rec) {
    if (tsi >= n_t_) throw error(HS_E_ARG, "time step must be < n_t");  // the reference exits
    if (tsi < 0) throw error(HS_E_ARG, "time step must be >= 0");
    const int len = 2 * model_->get_config_dim() + model_->number_of_motor_joints();
    ensure_complete_traj();
    std::copy(&rec_[(size_t)tsi * len], &rec_[(size_t)tsi * len] + len, rec);
  }
  // periodic.cpp:394-404: motor angles and rates of trajectory sample tsi
  void get_motor_adas(int tsi, double* as, double* das) {
    const int cfg = model_->get_config_dim(), len = 2 * cfg + model_->number_of_motor_joints();
    ensure_complete_traj();
    const double* r = &rec_[(size_t)(((tsi % n_t_) + n_t_) % n_t_) * len];  // records are indexed by tsi mod n_t
    std::copy(r + 6, r + cfg, as);
    std::copy(r + cfg + 6, r + 2 * cfg, das);
  }
  // periodic.cpp:285-307
  double work_over_period() {
    if (tau_.empty()) compute_torques_over_period();
    return wc_[0];
  }

 private:
  void ensure_complete_traj() {
    if (!rec_.empty()) return;
    hs_gait_params g = gait();
    const int len = 2 * model_->get_config_dim() + model_->number_of_motor_joints();
    rec_.assign((size_t)n_t_ * len, 0);
    check(hs_complete_traj(model_->handle(), &g, 1, n_t_, 1, rec_.data()), "get_complete_traj");
  }
};

// hs_batch_*: rollouts sharded over the devices of device_mask (bit d = HIP device d), host
// parameters in, host outputs out, best-rollout reduce across the devices
class batch {
  hs_batch_t h_ = nullptr;

 public:
  batch(const kinematicmodel& m, int n_rollouts, int horizon, int n_t, uint32_t device_mask = 1u,
        int precision = HS_PREC_F64) {
    check(hs_batch_create(m.handle(), n_rollouts, horizon, n_t, precision, device_mask, &h_), "hs_batch_create");
  }
  ~batch() { hs_batch_free(h_); }
  batch(const batch&) = delete;
  batch& operator=(const batch&) = delete;
  void set_params(const std::vector<hs_gait_params>& p) { check(hs_batch_set_params(h_, p.data()), "hs_batch_set_params"); }
  void run(int k0, const hs_batch_outputs& out, bool ignore_reach = true) {
    check(hs_batch_run(h_, k0, ignore_reach ? 1 : 0, &out), "hs_batch_run");
  }
  std::pair<float, int64_t> select_best() {
    float c = 0;
    int64_t id = -1;
    check(hs_select_best(h_, &c, &id), "hs_select_best");
    return {c, id};
  }
  // across the ranks of an RCCL communicator (hs_select_best_comm): one all-reduce(MIN) of 8 bytes
  std::pair<float, int64_t> select_best(hs_comm_t comm) {
    float c = 0;
    int64_t id = -1;
    check(hs_select_best_comm(h_, comm, &c, &id), "hs_select_best_comm");
    return {c, id};
  }
  hs_batch_t handle() const { return h_; }
};

class modelplayer {
  kinematicmodel model_;
  bool contact_force_flag_ = false;
  uint32_t device_mask_ = 1u;  // devices a sweep is sharded over (hs_batch_create)
  hs_sim_t sim_ = nullptr;  // the ODE world of setup_per_controller (one rollout)
  double play_t_ = 0, play_dt_ = 0.01;
  std::string traj_fname_ = "traj.txt";
  std::vector<double> last_tau_, last_q_;

 public:
  modelplayer() {}
  ~modelplayer() { unset_per_controller(); }
  modelplayer(const modelplayer&) = delete;
  modelplayer& operator=(const modelplayer&) = delete;
  // player.cpp:370-382: controller tables over one cycle of n_t = int(T/play_dt+.5) samples, the
  // world at the trajectory sample of t0, at rest; position control on (step_mode 6)
  void setup_per_controller(const pergensetup* pgs, double t0) {
    unset_per_controller();
    hs_gait_params g = pgs->to_c();
    hs_sim_params sp;
    hs_sim_default_params(&sp);
    sp.dt = play_dt_;
    check(hs_sim_create(model_.handle(), &g, 1, &sp, t0, &sim_), "setup_per_controller");
    play_t_ = int(t0 / play_dt_ + .5) * play_dt_;
    last_tau_.assign(model_.number_of_motor_joints(), 0);
    last_q_.assign(model_.number_of_motor_joints(), 0);
  }
  void unset_per_controller() {
    if (sim_) hs_sim_free(sim_);
    sim_ = nullptr;
  }
  // player.cpp:325-339 (position control): PD torques, dJointAddHingeTorque, collide, QuickStep
  void simulate_ode(int n_steps = 1) {
    if (!sim_) throw error(HS_E_ARG, "setup_per_controller first");
    const int nmj = model_.number_of_motor_joints();
    std::vector<double> tau((size_t)n_steps * nmj), q((size_t)n_steps * nmj);
    check(hs_sim_advance(sim_, n_steps, tau.data(), q.data(), nullptr, nullptr, nullptr), "simulate_ode");
    std::copy(tau.end() - nmj, tau.end(), last_tau_.begin());
    std::copy(q.end() - nmj, q.end(), last_q_.begin());
    play_t_ += n_steps * play_dt_;
  }
  double get_play_t() const { return play_t_; }
  void set_play_dt(double dt) { play_dt_ = dt; }
  // motor torques applied in the last step (set_ode_motor_torques) and the angles they saw
  const double* get_last_motor_torques() const { return last_tau_.data(); }
  const double* get_last_motor_angles() const { return last_q_.data(); }
  // body state of part i: pos[3], quaternion[4], lvel[3], avel[3] (dBodyGetPosition etc.)
  void get_ode_body(int part, double* state13) const {
    if (!sim_) throw error(HS_E_ARG, "setup_per_controller first");
    std::vector<double> b((size_t)model_.number_of_parts() * HS_SIM_BODY_STRIDE);
    check(hs_sim_get_state(sim_, b.data(), nullptr), "get_ode_body");
    std::copy(&b[(size_t)part * HS_SIM_BODY_STRIDE], &b[(size_t)part * HS_SIM_BODY_STRIDE] + HS_SIM_BODY_STRIDE,
              state13);
  }
  // dBodyGetPosition(get_torso_odebody()) (player.cpp:664-674)
  void get_torso_pos(double* pos) const {
    double st[HS_SIM_BODY_STRIDE];
    get_ode_body(0, st);
    std::copy(st, st + 3, pos);
  }
  // player.cpp:669-681 without exit(1): true when the torso is below hc
  bool fall_check(double hc) const {
    double p[3];
    get_torso_pos(p);
    return p[2] < hc;
  }
  kinematicmodel* get_model() { return &model_; }
  void set_flag(const std::string& name, bool v) {
    if (name == "contact_force") contact_force_flag_ = v;
    else throw error(HS_E_ARG, "unknown flag " + name);
  }
  // player.cpp:147-166
  pergensetup* make_pergensu(const std::string& config_fname, int setup_id, const std::string& model_dir = "") {
    hs_gait_params g;
    char xml[256];
    check(hs_pgs_config_read(config_fname.c_str(), setup_id, &g, xml, sizeof(xml)), "make_pergensu");
    pgsconfigparams pcp = pgsconfigparams::from_c(g, xml);
    std::string path = model_dir.empty() ? pcp.fname : model_dir + "/" + pcp.fname;
    if (!model_.if_loaded()) model_.load_fromxml(path);
    else if (model_.get_xmlfname() != path) throw error(HS_E_ARG, "model not from " + pcp.fname);
    int n_limbs = (model_.get_config_dim() - 6) / 3;
    return new pergensetup(n_limbs, pcp, &model_);
  }
  // measure_cot's own periodic solves with switch_torso_penalty(1,1) (player.cpp:263); the model's
  // setting (another periodic's, in the reference) is restored afterwards
  struct penalty_11 {
    hs_model_t m;
    int32_t f = 1, t = 1;
    explicit penalty_11(hs_model_t m_) : m(m_) {
      check(hs_model_get_torso_penalty(m, &f, &t), "hs_model_get_torso_penalty");
      if (!f || !t) check(hs_model_set_torso_penalty(m, 1, 1), "switch_torso_penalty");
    }
    ~penalty_11() {
      if (!f || !t) (void)hs_model_set_torso_penalty(m, f, t);
    }
  };
  // player.cpp:259-285
  double measure_cot(const pergensetup* pgs, int n_t) {
    penalty_11 pen(model_.handle());
    periodic per(&model_);
    per.record_trajectory(pgs, n_t);
    per.compute_torques_over_period();
    double work = per.work_over_period();
    double cot = work / (per.get_total_mass() * pgs->get_pergen()->get_step_length());
    if (contact_force_flag_) {
      double stat[2];
      per.get_contforce_stat(stat);
      std::cout << "min cfz = " << stat[0] << ", max mu = " << stat[1] << std::endl;
    }
    return cot;
  }
  // player.cpp:311-321 with pgssweeper::sweep/next (pergen.cpp:417-449, each value with the swept
  // gait's record transform), one launch for all values
  std::vector<std::pair<double, double>> measure_cot_sweep(const pergensetup* pgs, int n_t,
                                                           const std::string& param_name, double val0,
                                                           double val1, int n_val, bool print = true) {
    std::vector<hs_gait_params> params;
    std::vector<double> vals;
    {
      pgssweeper sweeper(pgs, &model_);
      std::streambuf* quiet = print ? nullptr : std::cout.rdbuf(nullptr);  // sweep() announces itself
      try {
        sweeper.sweep(param_name, val0, val1, n_val);
      } catch (...) {
        if (quiet) std::cout.rdbuf(quiet);
        throw;
      }
      if (quiet) std::cout.rdbuf(quiet);
      while (sweeper.next()) {
        params.push_back(sweeper.get_pgs()->to_c());
        vals.push_back(sweeper.get_val());
      }
    }
    std::vector<double> cot(params.size());
    penalty_11 pen(model_.handle());
    batch b(model_, (int)params.size(), n_t, n_t, device_mask_);
    b.set_params(params);
    hs_batch_outputs o;
    std::memset(&o, 0, sizeof(o));
    o.cot = cot.data();
    b.run(0, o);
    std::vector<std::pair<double, double>> out;
    for (size_t i = 0; i < vals.size(); i++) {
      out.emplace_back(vals[i], cot[i]);
      if (print) std::cout << "val = " << vals[i] << " COT = " << cot[i] << std::endl;
    }
    return out;
  }
  // devices measure_cot_sweep shards its rollouts over (bit d = HIP device d)
  void set_device_mask(uint32_t mask) { device_mask_ = mask; }
  // one cycle's complete trajectory records of n_t samples to fname (player.cpp:617-629 with n_t given)
  void record_per_traj(const pergensetup* pgs, int n_t, const std::string& fname) {
    const int len = 2 * model_.get_config_dim() + model_.number_of_motor_joints();
    penalty_11 pen(model_.handle());  // prepare_per_traj_dyn (player.cpp:263)
    double** traj = new_2d_array(n_t, len);
    periodic per(&model_);
    per.record_trajectory(pgs, n_t);
    per.get_complete_traj(traj);
    save_2d_array(traj, n_t, len, fname, false);
    delete_2d_array(traj, n_t);
  }
  // player.cpp:619-630: n_t = int(T / play_dt + .5) records of one cycle to traj.txt
  void record_per_traj(const pergensetup* pgs) {
    record_per_traj(pgs, int(pgs->get_period() / play_dt_ + .5), traj_fname_);
  }
  // player.cpp:634-655: every sweep value's cycle appended to traj.txt, n_t from the UNSWEPT period
  // (the reference's), all values in one batched launch
  void record_per_traj_sweep(const pergensetup* pgs, const std::string& param_name, double val0, double val1,
                             int n_val) {
    const int n_t = int(pgs->get_period() / play_dt_ + .5);
    const int len = 2 * model_.get_config_dim() + model_.number_of_motor_joints();
    std::vector<hs_gait_params> params;
    pgssweeper sweeper(pgs, &model_);
    sweeper.sweep(param_name, val0, val1, n_val);
    while (sweeper.next()) params.push_back(sweeper.get_pgs()->to_c());
    penalty_11 pen(model_.handle());
    std::vector<double> rec(params.size() * (size_t)n_t * len);
    check(hs_complete_traj(model_.handle(), params.data(), (int)params.size(), n_t, 1, rec.data()),
          "record_per_traj_sweep");
    std::vector<double*> rows((size_t)n_t);
    for (size_t v = 0; v < params.size(); v++) {
      for (int i = 0; i < n_t; i++) rows[(size_t)i] = &rec[(v * n_t + i) * (size_t)len];
      save_2d_array(rows.data(), n_t, len, traj_fname_, v > 0);
    }
  }
  // where record_per_traj[_sweep](pgs) write ("traj.txt" in the working directory, like the reference)
  void set_traj_fname(const std::string& f) { traj_fname_ = f; }
  // playerexperim.cpp:95-121: contact forces recovered from the computed torques; returns the
  // distance s the reference prints
  double test_dynamics(const pergensetup* pgs, int n_t = 20, int tsi = 2) {
    periodic per(&model_);
    per.record_trajectory(pgs, n_t);
    per.compute_torques_over_period();
    const int nf = per.get_nfeet();
    std::vector<double> cf1(3 * nf);
    per.solve_contforces_given_torques(tsi, cf1.data(), per.get_computed_torques(tsi));
    const double* cf = per.get_contact_forces(tsi);
    double s = 0;
    for (int i = 0; i < 3 * nf; i++) {
      double d = cf[i] - cf1[i];
      s += d * d;
    }
    std::cout << "s = " << std::sqrt(s) << std::endl;
    return std::sqrt(s);
  }
};

}  // namespace hslabs

#endif
