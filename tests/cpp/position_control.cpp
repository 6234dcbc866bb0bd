// Reference-shaped caller of the closed-loop simulation through the C++ shim:
// modelplayer::position_control_test (player.cpp:356-362) without the drawing
// loop -- make_pergensu(8), setup_per_controller(pgs, 0), then simulate_ode
// every play_dt for two gait periods (the visualizer's step loop, player.cpp:55-62).
#include <cmath>
#include <cstdio>
#include <string>

#include "hslabs.hpp"

using namespace hslabs;

int main(int argc, char** argv) {
  std::string models = argc > 1 ? argv[1] : "models";
  modelplayer player;
  pergensetup* pgs = player.make_pergensu(models + "/pgs_config.txt", 8, models);
  player.setup_per_controller(pgs, 0.0);
  double p0[3], p1[3];
  player.get_torso_pos(p0);
  for (int i = 0; i < 600; i++) player.simulate_ode();  // 2 periods of T = 3 at play_dt = .01
  player.get_torso_pos(p1);
  std::printf("play_t = %.4f\n", player.get_play_t());
  std::printf("torso0 = %.9f %.9f %.9f\n", p0[0], p0[1], p0[2]);
  std::printf("torso1 = %.9f %.9f %.9f\n", p1[0], p1[1], p1[2]);
  std::printf("tau_last[0] = %.9f\n", player.get_last_motor_torques()[0]);
  std::printf("fallen = %d\n", player.fall_check(0.4) ? 1 : 0);
  delete pgs;
  return std::isfinite(p1[0]) ? 0 : 1;
}
