// The model.h / core.h surface of include/hslabs.hpp, used the way the reference's callers use
// it (periodic.cpp:85-96 record_trajectory, player.cpp:114-124 set_config, pergen.cpp:450-456):
//   model_api <models_dir> <pgs_config.txt> <setup_id>...
// For each setup: pergensetup::set_rec at a few times, kinematicmodel::set_jvalues_with_lik,
// get_jvalues (printed for the oracle comparison), recompute_modelnodes and the FK-after-IK check
// of hso_fk_ik_check (feet on their targets), then orient_torso / get_limb_hip_pos, and the
// arrayops / str_to_val helpers of core.h.
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <memory>
#include <set>
#include <string>
#include <vector>

#include "hslabs.hpp"

using namespace hslabs;

int main(int argc, char** argv) {
  if (argc < 4) {
    std::cerr << "usage: model_api <models_dir> <pgs_config.txt> <setup_id>...\n";
    return 2;
  }
  const std::string dir = argv[1], cfg = argv[2];
  std::cout.precision(17);
  const double times[] = {0.0, 0.37, 1.25, 2.9};
  for (int a = 3; a < argc; a++) {
    const int id = std::atoi(argv[a]);
    modelplayer player;
    std::unique_ptr<pergensetup> pgs(player.make_pergensu(cfg, id, dir));
    kinematicmodel* model = player.get_model();
    const liksolver* lik = model->get_lik();
    lik->set_ignore_reach_flag(true);  // main.cpp:41
    const int cd = model->get_config_dim(), nl = lik->get_number_of_limbs();
    std::vector<double> rec(6 + 3 * nl), q(cd);
    for (double t : times) {
      pgs->set_rec(rec.data(), t);
      model->set_jvalues_with_lik(rec.data());
      model->get_jvalues(q.data());
      std::cout << "q " << id << " " << t;
      for (double v : q) std::cout << " " << v;
      std::cout << "\n";
      model->recompute_modelnodes();
      double worst = 0;
      for (int L = 0; L < nl; L++) {
        const modelnode* foot = lik->get_foot(L);
        const double* fp = foot->info().foot_pos;
        extvec local(fp[0], fp[1], fp[2]), ground;
        foot->get_A_ground()->mult(local, ground);
        for (int j = 0; j < 3; j++) worst = std::max(worst, std::fabs(ground.get_v(j) - rec[6 + 3 * L + j]));
      }
      std::cout << "fkik " << id << " " << t << " " << worst << "\n";
      // joint z axes: get_data() + 8 of the joint frame (dynrec.cpp:84-93) is a unit vector
      double zerr = 0;
      for (int i = 0; i < model->number_of_parts(); i++) {
        modeljoint* j = model->get_mnode(i)->get_joint();
        if (!j) continue;
        const double* z = j->get_A_ground()->get_data() + 8;
        zerr = std::max(zerr, std::fabs(z[0] * z[0] + z[1] * z[1] + z[2] * z[2] - 1));
      }
      std::cout << "zaxis " << id << " " << t << " " << zerr << "\n";
    }
    // set_jvalues / get_jvalues round trip and the joint-values pointers (model.h:110)
    std::vector<double> q2(cd);
    for (int i = 0; i < cd; i++) q2[i] = 0.01 * i;
    model->set_jvalues(q2.data());
    std::vector<double*>* jp = model->get_joint_values();
    double jerr = 0;
    for (int i = 0; i < cd; i++) jerr = std::max(jerr, std::fabs(*(*jp)[i] - q2[i]));
    std::cout << "jvalues " << id << " " << jerr << "\n";
    // orient_torso (model.cpp:403-409) moves every hip by the torso translation
    extvec hip0, hip1;
    model->recompute_modelnodes();
    lik->get_limb_hip_pos(0, hip0);
    extvec orientation[2];
    orientation[0].set(q2[0] + 0.5, q2[1] - 0.25, q2[2] + 1.0);
    orientation[1].set(q2[3], q2[4], q2[5]);
    model->orient_torso(orientation);
    lik->get_limb_hip_pos(0, hip1);
    std::cout << "orient " << id << " " << hip1.get_v(0) - hip0.get_v(0) << " " << hip1.get_v(1) - hip0.get_v(1) << " "
              << hip1.get_v(2) - hip0.get_v(2) << "\n";
    std::set<modelnode*> feet;
    model->get_foot_mnodes(feet);
    std::cout << "feet " << id << " " << feet.size() << "\n";
    // an unreachable foot without ignore_reach throws where the reference exits (lik.cpp:321-330)
    lik->set_ignore_reach_flag(false);
    bool threw = false;
    try {
      lik->place_limb(0, 100.0, 100.0, 100.0);
    } catch (const error&) {
      threw = true;
    }
    std::cout << "unreach_throws " << id << " " << threw << "\n";
  }
  // core.h helpers
  double v[3] = {0, 0, 0};
  str_to_val("1.5 -2 3e-1", v);
  arrayops ao(3);
  double a[3] = {4, -4, 1}, b[3] = {1, 1, 1};
  ao.modulus(a, 2 * M_PI);
  std::cout << "str_to_val " << v[0] << " " << v[1] << " " << v[2] << "\n";
  std::cout << "modulus " << a[0] << " " << a[1] << " " << a[2] << "\n";
  std::cout << "dot " << ao.dot(v, b) << " norm " << ao.norm(b) << " distance " << ao.distance(v, b) << "\n";
  return 0;
}
