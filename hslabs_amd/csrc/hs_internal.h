// hs_internal.h -- declarations shared by the host-side translation units.
#pragma once
#include <cstddef>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hslabs.h"
#include "hs_topo.h"

namespace hs {

int load_model_file(const char* path, int lik_variant, hs_topo* t, std::string& err);
int read_pgs_config(const char* path, int setup_id, hs_gait_params* out, std::string& xml, std::string& err);

// Kernel launcher (hs_kernels.hip). `workspace` holds general_workspace_bytes()
// per rollout (global-memory scratch of the conditioning fallback). Returns a
// hipError_t value.
size_t general_workspace_bytes();
int launch_rollouts(const hs_topo* d_topo, const hs_topo& h_topo, const hs_run_args& a, void* workspace);

}  // namespace hs

constexpr int HS_MAX_DEVICES = 64;

struct hs_model_s {
  hs_topo host;
  hs_topo* dev[HS_MAX_DEVICES];  // per-device topology copy, created lazily
  void* ws[HS_MAX_DEVICES];      // per-device fallback workspace
  size_t ws_rollouts[HS_MAX_DEVICES];
  std::vector<std::pair<int, void*>> retired;  // outgrown workspaces (in-flight kernels may use them)
  std::mutex mu;
};
