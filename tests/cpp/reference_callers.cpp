// The reference's own callers of the hot path, compiled against the C++ shim (include/hslabs.hpp)
// with plain g++: the member-function bodies below are those of player.cpp:259-285 (measure_cot,
// prepare_per_traj_dyn), 311-321 (measure_cot_sweep), 393-432 (set_position_control_torques,
// linear_feedback_control), 619-655 (record_per_traj[_sweep]), playerexperim.cpp:95-121
// (test_dynamics) and cpc.cpp:51-63 (set_target_points_by_per), unchanged. What they reach outside
// the path is stubbed here and says so: get_vis()->get_ode_motor_adas (ODE joint state) returns
// the targets shifted by a fixed offset, set_ode_motor_torques records the command, and
// cpccontroller's apply_mask keeps the record (CPC itself is out of scope).
//
// Output lines "<key> <values>" are checked by tests/test_cpp_shim.py against the Python binding
// and the oracle.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "hslabs.hpp"

using namespace hslabs;
using std::cout;
using std::endl;
using std::string;

struct odestub {  // visualizer::get_ode_motor_adas (visualization.cpp:367-374), no ODE world here
  const periodic* per = nullptr;
  int nmj = 0;
  double dq = 0.01, ddq = -0.2;
  mutable std::vector<double> q0, dq0;
  void get_ode_motor_adas(double* as, double* das) const {
    for (int i = 0; i < nmj; i++) {
      as[i] = q0[i] + dq * (i + 1);
      das[i] = dq0[i] + ddq;
    }
  }
};

class refplayer {  // the members of modelplayer (player.h:45-55) these bodies use
 public:
  kinematicmodel* model;
  double play_t, play_dt;
  int config_dim, nmj;
  bool contact_force_flag, ghost_walking_flag;
  periodic* play_per;
  odestub vis;
  std::vector<double> last_cmd;
  struct ghoststub {
    void get_motor_adas(double*, double*) {}
  } ghost_, *ghost = &ghost_;

  explicit refplayer(kinematicmodel* m)
      : model(m), play_t(0), play_dt(0.02), config_dim(m->get_config_dim()), nmj(m->number_of_motor_joints()),
        contact_force_flag(true), ghost_walking_flag(false), play_per(nullptr) {}
  const odestub* get_vis() const { return &vis; }
  void set_ode_motor_torques(const double* t) { last_cmd.assign(t, t + nmj); }

  // ---- player.cpp:259-264
  void prepare_per_traj_dyn(periodic& per, pergensetup* pgs, int n_t){
    per.record_trajectory(pgs,n_t);
    per.compute_dynrecs();
    per.compute_dynrec_ders();
    per.switch_torso_penalty(1,1);
  }

  // ---- player.cpp:269-285
  double measure_cot(pergensetup* pgs, int n_t){
    periodic per (model);
    prepare_per_traj_dyn(per,pgs,n_t);
    double work = per.work_over_period();
    double weight = per.get_total_mass();
    double step_length = pgs->get_pergen()->get_step_length();
    double cot = work/(weight*step_length);
    //cout << "COT = " << cot << endl;
    if(contact_force_flag){
      double stat[2];
      per.get_contforce_stat(stat);
      cout << "min cfz = " << stat[0];
      cout << ", max mu = " << stat[1] << endl;
    }

    return cot;
  }

  // ---- player.cpp:311-321
  void measure_cot_sweep(pergensetup* pgs, int n_t, string param_name, double val0, double val1, int n_val){

    pgssweeper sweeper (pgs, model);
    sweeper.sweep(param_name, val0, val1, n_val);
    while(sweeper.next()){
      pergensetup* pgs1 = sweeper.get_pgs();
      double cot = measure_cot(pgs1, n_t);
      double val = sweeper.get_val();
      cout << "val = " << val << " COT = " << cot << endl;
    }
  }

  // ---- player.cpp:393-412 (get_vis() / ghost: the stubs above)
  void set_position_control_torques(){
    double k = 100;
    double k1 = -k, k2 = -2*sqrt(k);
    int an = 5;
    double** a = new_2d_array(an,nmj);
    double *q0 = a[0], *dq0 = a[1], *q = a[2], *dq = a[3];
    double *motor_torques = a[4];
    int tsi = int(play_t/play_dt+.5);
    play_per->get_motor_adas(tsi,q0,dq0);
    vis.q0.assign(q0, q0 + nmj); vis.dq0.assign(dq0, dq0 + nmj);  // (stub: the measured state)
    get_vis()->get_ode_motor_adas(q,dq);
    if(ghost_walking_flag){ghost->get_motor_adas(q,dq);}
    double *p = play_per->get_computed_torques(tsi);
    std::copy(p,p+nmj,motor_torques);
    double *x0[2] = {q0,dq0}, *x[2] = {q,dq};
    linear_feedback_control(motor_torques,x0,x,k1,k2);
    //arrayops ao (nmj); cout << ao.norm(p) << " " << ao.norm(motor_torques) << " " << ao.distance(motor_torques,p) << endl;
    //arrayops ao (nmj); cout << ao.norm(motor_torques)<<endl;
    set_ode_motor_torques(motor_torques);
    delete_2d_array(a,an);
  }

  // ---- player.cpp:416-432
  void linear_feedback_control(double* torques, double** x0, double** x, double k1, double k2){
    double *q0 = x0[0], *dq0 = x0[1], *q = x[0], *dq = x[1];
    double* a1 = new double [2*nmj];
    double* a2 = a1 + nmj;
    arrayops ao (nmj);
    ao.assign(a1,q);
    ao.assign(a2,dq);
    //ao.assign_scalar(torques,0); // temp, test
    //ao.print(torques);ao.print(q0);ao.print(dq0);
    ao.modulus(ao.subtract(a1,q0),2*M_PI);
    ao.subtract(a2,dq0);
    //cout<<ao.l1_norm(a1)+ao.l1_norm(a2)*0<<endl;
    ao.add(ao.times(a1,k1),ao.times(a2,k2));
    ao.add(torques,a1);
    //ao.print(torques); cout<<endl;
    delete [] a1;
  }

  // ---- player.cpp:619-630
  void record_per_traj(pergensetup* pgs){
    double T = pgs->get_period();
    int n_t = int(T/play_dt+.5);
    int rec_len = 2*config_dim+nmj;
    double** traj = new_2d_array(n_t,rec_len);
    periodic* per = new periodic (model);
    prepare_per_traj_dyn(*per,pgs,n_t);
    per->get_complete_traj(traj);
    save_2d_array(traj,n_t,rec_len,"traj.txt",false);
    delete per;
    delete_2d_array(traj,n_t);
  }

  // ---- player.cpp:634-655
  void record_per_traj_sweep(pergensetup* pgs, string param_name, double val0, double val1, int n_val){
    double T = pgs->get_period();
    int n_t = int(T/play_dt+.5);
    int rec_len = 2*config_dim+nmj;
    double** traj = new_2d_array(n_t,rec_len);

    pgssweeper sweeper (pgs, model);
    sweeper.sweep(param_name, val0, val1, n_val);
    bool flag = false;
    while(sweeper.next()){
      pergensetup* pgs1 = sweeper.get_pgs();
      //cout<<"val = "<<sweeper.get_val()<<endl;
      periodic* per = new periodic (model);
      prepare_per_traj_dyn(*per,pgs1,n_t);
      per->get_complete_traj(traj);
      save_2d_array(traj,n_t,rec_len,"traj.txt",flag);
      delete per;
      if(!flag){flag = true;}
    }

    delete_2d_array(traj,n_t);
  }

  // ---- playerexperim.cpp:95-121
  void test_dynamics(pergensetup* pgs){
    // preparing per
    periodic per (model);
    prepare_per_traj_dyn(per,pgs,20);

    int nf = per.get_nfeet();
    double* torques = new double [nmj];
    double* contforces = new double [3*nf];
    double* contforces1 = new double [3*nf];
    int tsi = 2; // time step
    // obtaining torques for a given time step tsi
    per.solve_torques_contforces(tsi,torques,contforces);

    for(int i=0;i<nf;i++){cout<<contforces[3*i+2]<<" ";}cout<<endl;
    //for(int i=0;i<nmj;i++){cout<<torques[i]<<" ";}cout<<endl;

    // computing contact forces for a given tsi and torques
    per.solve_contforces_given_torques(tsi,contforces1,torques);
    //for(int i=0;i<nf;i++){cout<<contforces1[3*i+2]<<" ";}cout<<endl;

    // verifying correctness of cfs
    double s=0;for(int i=0;i<3*nf;i++){double d = contforces[i]-contforces1[i];s+=d*d;}cout<<"s = "<<sqrt(s)<<endl;

    delete [] torques;
    delete [] contforces;
    delete [] contforces1;
  }
};

class refcpc {  // the cpccontroller members set_target_points_by_per uses (cpc.h)
 public:
  int q_dim, chi_dim, tps_size;
  double** target_points;
  explicit refcpc(const kinematicmodel* model)
      : q_dim(model->get_config_dim()), chi_dim(model->number_of_motor_joints()), tps_size(0),
        target_points(NULL) {}
  void apply_mask(double*) {}  // (stub: CPC's coordinate mask is out of scope)

  // ---- cpc.cpp:51-63
  void set_target_points_by_per(periodic* per){
    //per->print();exit(1);
    if(target_points){cout<<"ERROR: target points are present"<<endl;exit(1);}
    int nt = per->get_nt();
    int rec_len = 2*q_dim + chi_dim;
    target_points = new_2d_array(nt,rec_len);
    for(int i=0;i<nt;i++){
      per->get_complete_traj_rec(i,target_points[i]);
      apply_mask(target_points[i]);
    }
    tps_size = nt;
    //print_target_points();exit(1);
  }
};

static void print_row(const char* key, const double* v, int n) {
  std::printf("%s", key);
  for (int i = 0; i < n; i++) std::printf(" %.17g", v[i]);
  std::printf("\n");
}

int main(int argc, char** argv) {
  std::string models = argc > 1 ? argv[1] : "models";
  modelplayer shim;
  pergensetup* pgs = shim.make_pergensu(models + "/pgs_config.txt", 8, models);  // main.cpp:35
  refplayer player0(shim.get_model());
  player0.play_dt = .02;  // main.cpp:31

  // measure_cot / measure_cot_sweep, the reference's bodies
  double cot = player0.measure_cot(pgs, 20);
  std::printf("cot %.17g\n", cot);
  std::fflush(stdout);
  player0.contact_force_flag = false;
  player0.measure_cot_sweep(pgs, 20, "period", 3, 18, 15);  // main.cpp:69
  std::cout.flush();

  // test_dynamics, and the periodic accessors of periodic.h:43-51
  player0.test_dynamics(pgs);
  std::cout.flush();
  {
    periodic per(player0.model);
    player0.prepare_per_traj_dyn(per, pgs, 20);
    per.compute_torques_over_period();
    const int n = per.get_number_of_dynparts();
    std::vector<double> m(per.get_masses(), per.get_masses() + n);
    std::vector<double> pi(per.get_parentis(), per.get_parentis() + n);
    std::vector<double> fi(per.get_footis(), per.get_footis() + per.get_nfeet());
    print_row("masses", m.data(), n);
    print_row("parentis", pi.data(), n);
    print_row("footis", fi.data(), per.get_nfeet());
    std::vector<double> mt(player0.nmj), tq(player0.nmj), cf(3 * per.get_nfeet());
    per.get_motor_torques(mt.data());  // the loop's last solve: sample n_t + 1
    print_row("motor_torques_last", mt.data(), player0.nmj);
    per.solve_torques_contforces(7, tq.data(), cf.data());
    per.get_motor_torques(mt.data());
    print_row("solve7_tau", tq.data(), player0.nmj);
    print_row("solve7_cf", cf.data(), 3 * per.get_nfeet());
    print_row("motor_torques_7", mt.data(), player0.nmj);
    double* ct = per.get_computed_torques(7);  // periodic.h:51: a writable pointer, as player.cpp:404 binds it
    print_row("computed_7", ct, player0.nmj);
  }

  // the position controller's command (set_position_control_torques / linear_feedback_control)
  {
    periodic per(player0.model);
    player0.prepare_per_traj_dyn(per, pgs, 150);  // setup_per_controller: n_t = int(T / play_dt + .5)
    per.compute_torques_over_period();
    player0.play_per = &per;
    player0.vis.nmj = player0.nmj;
    for (double t : {0.0, 0.02, 1.0, 2.98}) {
      player0.play_t = t;
      player0.set_position_control_torques();
      std::printf("tsi %d\n", int(t / player0.play_dt + .5));
      print_row("cmd", player0.last_cmd.data(), player0.nmj);
      print_row("ff", per.get_computed_torques(int(t / player0.play_dt + .5)), player0.nmj);
      print_row("q0", player0.vis.q0.data(), player0.nmj);
      print_row("dq0", player0.vis.dq0.data(), player0.nmj);
    }
    player0.play_per = nullptr;

    // cpc.cpp:51-63 on the same periodic
    refcpc cpc(player0.model);
    cpc.set_target_points_by_per(&per);
    print_row("tp0", cpc.target_points[0], 2 * cpc.q_dim + cpc.chi_dim);
    print_row("tp77", cpc.target_points[77], 2 * cpc.q_dim + cpc.chi_dim);
    std::printf("tps_size %d\n", cpc.tps_size);
    delete_2d_array(cpc.target_points, cpc.tps_size);
  }

  // record_per_traj / record_per_traj_sweep: traj.txt in the working directory
  player0.record_per_traj(pgs);
  std::rename("traj.txt", "traj_one.txt");
  pgs->set_rec_rotation(extvec(0, 0, -1.571));  // main.cpp:38
  player0.record_per_traj_sweep(pgs, "step_length", -.5, .5, 1);  // main.cpp:56
  std::rename("traj.txt", "traj_sweep.txt");
  double cot_rot = player0.measure_cot(pgs, 20);
  std::printf("cot_rotated %.17g\n", cot_rot);
  delete pgs;
  return 0;
}
