// hslabs.hpp -- C++ shim over include/hslabs.h that keeps the reference's
// call shapes for the hot path, so player.cpp-style callers switch by changing
// includes. Header-only; link with -lhslabs.
//
//   kinematicmodel::load_fromxml / get_config_dim / number_of_motor_joints  (model.h:96-137)
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
// (record_trajectory / compute_dynrecs / compute_dynrec_ders /
// switch_torso_penalty only record their arguments); measure_cot_sweep runs all
// sweep values in one batched launch.
#ifndef HSLABS_HPP
#define HSLABS_HPP

#include <cmath>
#include <cstring>
#include <fstream>
#include <iostream>
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

class kinematicmodel {
  hs_model_t h_ = nullptr;
  hs_model_dims d_{};
  std::string xmlfname_;

 public:
  explicit kinematicmodel(bool /*vis_flag*/ = false) {}
  ~kinematicmodel() { hs_model_free(h_); }
  kinematicmodel(const kinematicmodel&) = delete;
  kinematicmodel& operator=(const kinematicmodel&) = delete;
  void load_fromxml(const std::string& fname, int lik_variant = -1) {
    hs_model_free(h_);
    h_ = nullptr;
    check(hs_model_load_ex(fname.c_str(), lik_variant, &h_), "load_fromxml");
    check(hs_model_get_dims(h_, &d_), "hs_model_get_dims");
    xmlfname_ = fname;
  }
  bool if_loaded() const { return h_ != nullptr; }
  std::string get_xmlfname() const { return xmlfname_; }
  int get_config_dim() const { return d_.config_dim; }
  int number_of_motor_joints() const { return d_.nmj; }
  int number_of_parts() const { return d_.n_parts; }
  int number_of_feet() const { return d_.nfeet; }
  double total_mass() const { return d_.total_mass; }
  hs_model_t handle() const { return h_; }
};

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

// The gait of one rollout (pergensetup): its pgsconfigparams plus accessors.
class pergensetup {
  pgsconfigparams pcp_;
  int n_;

 public:
  pergensetup(int n_limbs, const pgsconfigparams& pcp) : pcp_(pcp), n_(n_limbs) {}
  int get_limb_number() const { return n_; }
  int get_config_dim() const { return 6 + 3 * n_; }
  double get_period() const { return pcp_.TLh[0]; }
  double get_step_length() const { return pcp_.TLh[1]; }
  void get_config_params(pgsconfigparams* pcp) const { *pcp = pcp_; }
  const pgsconfigparams& params() const { return pcp_; }
  void set_TLh(double T, double L, double h) { pcp_.set_TLh(T, L, h); }
};

class periodic {
  const kinematicmodel* model_;
  const pergensetup* pgs_ = nullptr;
  int n_t_ = 0;
  bool force_pen_ = true, torque_pen_ = true;
  std::vector<double> tau_, cf_, x_, wc_;
  std::vector<uint32_t> flags_;
  std::vector<double> rec_;  // get_complete_traj records
  double min_cfz_ = 1e10, max_mu_ = -1e10;

 public:
  explicit periodic(const kinematicmodel* model) : model_(model) {}
  void record_trajectory(const pergensetup* pgs, int n_t) { pgs_ = pgs; n_t_ = n_t; tau_.clear(); rec_.clear(); }
  void compute_dynrecs() {}
  void compute_dynrec_ders() {}
  void switch_torso_penalty(bool force, bool torque) {
    if (!force || !torque) throw error(HS_E_ARG, "only switch_torso_penalty(1,1) is on the GPU path");
    force_pen_ = force; torque_pen_ = torque;
  }
  int get_nt() const { return n_t_; }
  int get_nfeet() const { return model_->number_of_feet(); }
  double get_total_mass() const { return model_->total_mass(); }
  // periodic.cpp:377-391 (+ analyze_contforces 347-357)
  void compute_torques_over_period() {
    if (!pgs_) throw error(HS_E_ARG, "record_trajectory first");
    const int nmj = model_->number_of_motor_joints(), nf = model_->number_of_feet();
    const int n = model_->number_of_parts(), cfg = model_->get_config_dim();
    hs_gait_params g = pgs_->params().to_c();
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
  }
  // computed_torques[i % n_t] holds the torques of trajectory sample i (periodic.cpp:387)
  const double* get_computed_torques(int i) const {
    int h = ((i - 2) % n_t_ + n_t_) % n_t_;
    return &tau_[(size_t)h * model_->number_of_motor_joints()];
  }
  const double* get_contact_forces(int i) const {
    int h = ((i - 2) % n_t_ + n_t_) % n_t_;
    return &cf_[(size_t)h * 3 * model_->number_of_feet()];
  }
  uint32_t get_flags(int i) const { return flags_[((i - 2) % n_t_ + n_t_) % n_t_]; }
  void get_contforce_stat(double* stat) const { stat[0] = min_cfz_; stat[1] = max_mu_; }
  // periodic.cpp:368-374 (forcetorquesolver::solve_forces): forces of all feet for step i
  void solve_contforces_given_torques(int i, double* contforces, const double* torques) const {
    if (!pgs_) throw error(HS_E_ARG, "record_trajectory first");
    hs_gait_params g = pgs_->params().to_c();
    int k0 = ((i - 2) % n_t_ + n_t_) % n_t_;
    check(hs_run_forces_host(model_->handle(), &g, 1, n_t_, k0, 1, 1, torques, contforces, nullptr),
          "solve_contforces_given_torques");
  }
  // periodic.cpp:406-426: n_t records of (q, dq, torques) = 2 config_dim + nmj
  void get_complete_traj(double** complete_traj) {
    if (!pgs_) throw error(HS_E_ARG, "record_trajectory first");
    const int len = 2 * model_->get_config_dim() + model_->number_of_motor_joints();
    if (rec_.empty()) {
      hs_gait_params g = pgs_->params().to_c();
      rec_.assign((size_t)n_t_ * len, 0);
      check(hs_complete_traj(model_->handle(), &g, 1, n_t_, 1, rec_.data()), "get_complete_traj");
    }
    for (int i = 0; i < n_t_; i++) std::copy(&rec_[(size_t)i * len], &rec_[(size_t)i * len] + len, complete_traj[i]);
  }
  // periodic.cpp:394-404: motor angles and rates of trajectory sample tsi
  void get_motor_adas(int tsi, double* as, double* das) {
    const int cfg = model_->get_config_dim(), len = 2 * cfg + model_->number_of_motor_joints();
    std::vector<double*> rows((size_t)n_t_);
    std::vector<double> buf((size_t)n_t_ * len);
    for (int i = 0; i < n_t_; i++) rows[i] = &buf[(size_t)i * len];
    get_complete_traj(rows.data());
    const double* r = rows[((tsi % n_t_) + n_t_) % n_t_];  // records are indexed by tsi mod n_t
    std::copy(r + 6, r + cfg, as);
    std::copy(r + cfg + 6, r + 2 * cfg, das);
  }
  // periodic.cpp:285-307
  double work_over_period() {
    if (tau_.empty()) compute_torques_over_period();
    return wc_[0];
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
};

class modelplayer {
  kinematicmodel model_;
  bool contact_force_flag_ = false;
  uint32_t device_mask_ = 1u;  // devices a sweep is sharded over (hs_batch_create)
  hs_sim_t sim_ = nullptr;  // the ODE world of setup_per_controller (one rollout)
  double play_t_ = 0, play_dt_ = 0.01;
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
    hs_gait_params g = pgs->params().to_c();
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
    return new pergensetup(n_limbs, pcp);
  }
  // player.cpp:269-285
  double measure_cot(const pergensetup* pgs, int n_t) {
    periodic per(&model_);
    per.record_trajectory(pgs, n_t);
    per.compute_torques_over_period();
    double work = per.work_over_period();
    double cot = work / (per.get_total_mass() * pgs->get_step_length());
    if (contact_force_flag_) {
      double stat[2];
      per.get_contforce_stat(stat);
      std::cout << "min cfz = " << stat[0] << ", max mu = " << stat[1] << std::endl;
    }
    return cot;
  }
  // player.cpp:311-321 with pgssweeper::sweep/next (pergen.cpp:417-449), one launch for all values
  std::vector<std::pair<double, double>> measure_cot_sweep(const pergensetup* pgs, int n_t,
                                                           const std::string& param_name, double val0,
                                                           double val1, int n_val, bool print = true) {
    const char* names[] = {"step_duration", "period", "step_length", "step_height"};
    int parami = -1;
    for (int i = 0; i < 4; i++)
      if (param_name == names[i]) parami = i;
    if (parami < 0) throw error(HS_E_ARG, "cannot sweep over " + param_name);
    double delval = (val1 - val0) / n_val;
    std::vector<hs_gait_params> params;
    std::vector<double> vals;
    for (int vali = 0; vali <= n_val; vali++) {
      double val = val0 + vali * delval;
      pgsconfigparams p = pgs->params();
      if (parami == 0) p.step_duration = val;
      else p.TLh[parami - 1] = val;
      params.push_back(p.to_c());
      vals.push_back(val);
    }
    std::vector<double> cot(params.size());
    batch b(model_, (int)params.size(), n_t, n_t, device_mask_);
    b.set_params(params);
    hs_batch_outputs o;
    std::memset(&o, 0, sizeof(o));
    o.cot = cot.data();
    b.run(0, o);
    std::vector<std::pair<double, double>> out;
    if (print) std::cout << "sweeping over " << param_name << ":" << std::endl;
    for (size_t i = 0; i < vals.size(); i++) {
      out.emplace_back(vals[i], cot[i]);
      if (print) std::cout << "val = " << vals[i] << " COT = " << cot[i] << std::endl;
    }
    return out;
  }
  // devices measure_cot_sweep shards its rollouts over (bit d = HIP device d)
  void set_device_mask(uint32_t mask) { device_mask_ = mask; }
  // player.cpp:617-629: one cycle's complete trajectory records to traj.txt
  void record_per_traj(const pergensetup* pgs, int n_t, const std::string& fname = "traj.txt") {
    const int len = 2 * model_.get_config_dim() + model_.number_of_motor_joints();
    double** traj = new_2d_array(n_t, len);
    periodic per(&model_);
    per.record_trajectory(pgs, n_t);
    per.get_complete_traj(traj);
    save_2d_array(traj, n_t, len, fname, false);
    delete_2d_array(traj, n_t);
  }
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
