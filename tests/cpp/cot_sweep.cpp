// Reference-shaped caller of the C++ shim: the hot-path part of main.cpp:33-89
// (make_pergensu(8) -> measure_cot_sweep(period 3..18) -> periodic work_over_period).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "hslabs.hpp"

using namespace hslabs;

int main(int argc, char** argv) {
  std::string models = argc > 1 ? argv[1] : "models";
  modelplayer player0;
  pergensetup* pgs = player0.make_pergensu(models + "/pgs_config.txt", 8, models);  // main.cpp:35
  double cot = player0.measure_cot(pgs, 20);                                         // main.cpp:72
  std::printf("COT = %.12f\n", cot);
  auto sweep = player0.measure_cot_sweep(pgs, 20, "period", 3, 18, 15, false);        // main.cpp:69
  for (auto& vc : sweep) std::printf("val = %g COT = %.12f\n", vc.first, vc.second);
  {  // the same sweep as a device-sharded batch and its best-rollout reduce
    std::vector<hs_gait_params> ps;
    for (size_t i = 0; i < sweep.size(); i++) {
      pgsconfigparams p = pgs->params();
      p.TLh[0] = sweep[i].first;  // period
      ps.push_back(p.to_c());
    }
    batch b(*player0.get_model(), (int)ps.size(), 20, 20);
    b.set_params(ps);
    std::vector<double> cot_b(ps.size());
    hs_batch_outputs o;
    std::memset(&o, 0, sizeof(o));
    o.cot = cot_b.data();
    b.run(0, o);
    auto best = b.select_best();
    size_t imin = 0;
    for (size_t i = 0; i < cot_b.size(); i++) {
      if (cot_b[i] != sweep[i].second) return 4;
      if ((float)cot_b[i] < (float)cot_b[imin]) imin = i;
    }
    std::printf("best = %.9g id %lld\n", (double)best.first, (long long)best.second);
    if (best.second != (int64_t)imin || best.first != (float)cot_b[imin]) return 5;
  }
  periodic per(player0.get_model());                                                  // main.cpp:81-89
  per.record_trajectory(pgs, 20);
  per.compute_dynrecs();
  per.compute_dynrec_ders();
  per.switch_torso_penalty(1, 1);
  double work = per.work_over_period();
  std::printf("work = %.12f\n", work);
  const double* tau = per.get_computed_torques(2);
  std::printf("tau[2][0] = %.12f\n", tau[0]);
  double as[18], das[18];
  per.get_motor_adas(2, as, das);
  std::printf("adas[2][0] = %.12f %.12f\n", as[0], das[0]);
  double s = player0.test_dynamics(pgs);                      // playerexperim.cpp:95-121
  player0.record_per_traj(pgs, 20, argc > 2 ? argv[2] : "traj.txt");  // player.cpp:617-629
  if (!(s < 1e-9)) return 3;
  try {
    player0.measure_cot_sweep(pgs, 20, "curvature", 0, 1, 2, false);
    return 2;
  } catch (const error& e) {
    std::printf("error ok: %s\n", e.what());
  }
  delete pgs;
  return (std::isfinite(cot) && std::fabs(cot - sweep[0].second) < 1e-12) ? 0 : 1;
}
