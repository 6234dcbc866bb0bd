// hs_internal.h -- declarations shared by the host-side translation units.
#pragma once
#include <string>

#include "../../include/hslabs.h"
#include "hs_topo.h"

namespace hs {

int load_model_file(const char* path, int lik_variant, hs_topo* t, std::string& err);
int read_pgs_config(const char* path, int setup_id, hs_gait_params* out, std::string& xml, std::string& err);

// Kernel launcher (hs_kernels.hip). Returns a hipError_t value.
int launch_rollouts(const hs_topo* d_topo, const hs_topo& h_topo, const hs_run_args& a);

}  // namespace hs

struct hs_model_s {
  hs_topo host;
  hs_topo* dev[64];  // per-device copy, created lazily
};
