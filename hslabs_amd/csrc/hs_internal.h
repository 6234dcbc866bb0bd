// hs_internal.h -- declarations shared by the host-side translation units.
#pragma once
#include <cstddef>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/hslabs.h"
#include "hs_simtopo.h"
#include "hs_topo.h"

namespace hs {

// records msg for hs_last_error() (thread-local) and returns code
int set_error(int code, const std::string& msg);
// the best-key all-reduce of hs_comm.cpp (ncclMin over ncclUint64, in place, async on stream)
int comm_reduce_min(hs_comm_t comm, uint64_t* key, void* stream);
int comm_device(hs_comm_t comm);
uint64_t* comm_scratch(hs_comm_t comm);  // 8 B on the comm's device

int load_model_file(const char* path, int lik_variant, hs_topo* t, std::string& err, hs_simtopo* sim = nullptr);
int read_pgs_config(const char* path, int setup_id, hs_gait_params* out, std::string& xml, std::string& err);

// Gait setup (pergensetup::setup_pergen, once per rollout in the reference) across the
// launches of one call: the first launch computes and stores it per rollout, the rest load it.
enum { SETUP_COMPUTE = 0, SETUP_STORE = 1, SETUP_LOAD = 2 };
// Steps the closed form declines, in fused launches (hs_run_calls, HS_SOLVE_AUTO): the step launch
// (FIX_DEFER) appends (local step, 2 * wavefront + half) items to fix_items and counts them in
// *fix_count instead of calling the general path; the fixup launch after it (FIX_SOLVE, the
// instantiation with the general path) recomputes those steps and stores their outputs and work
// (after the call's last step launch, together with the work reduce).
enum { FIX_NONE = 0, FIX_DEFER = 1, FIX_SOLVE = 2 };

// Which rollouts a launch's wavefronts run and where their output rows go.
struct launch_map {
  const int32_t* wave_model;     // mixed: model of each wavefront, an index into the launch's
                                 // contiguous topology array (null: one model)
  const int32_t* wave_rollouts;  // mixed: [2 * n_waves] rollout ids, -1 = idle half
  int32_t n_waves;
  int32_t max_parts;             // LDS layout class (largest model)
  int32_t h_row;                 // output row of this launch's step within the horizon
  int32_t setup_io;              // SETUP_*: gait setup computed here, also stored, or loaded
  const double* tau_in;          // forces-given-torques mode: motor torques [B][H][st_tau] (else null)
  // position control (hs_run_pd; null pd_tau = off): rows [B][H][st_tau]
  const double *pd_q, *pd_dq;
  double pd_k1, pd_k2;
  double *pd_tau, *pd_q0, *pd_dq0;
  int32_t st_tau, st_cf, st_q, st_x;  // output row strides (mixed: maxima over the models)
  // fused steps (hs_run_calls): one launch runs fused_n steps x fused_w wavefronts, wavefront
  // blockIdx -> (local step, batch wavefront) by groups of batch wavefronts (fused_coords in
  // hs_kernels.hip: a group's steps in order, its wavefronts fastest); global step s = fused_s0 + local step is
  // call s / fused_h, step s % fused_h of that call, output row s; the step's work goes to
  // fused_work[s][b] (summed in order afterwards), the general-path scratch to
  // fused_gen[local step][b]. setup_only: store the gait setup and return.
  int32_t fused_w, fused_s0, fused_n, fused_h;
  void* fused_work;
  void* fused_gen;
  int32_t setup_only;
  int32_t fix_mode;     // FIX_*
  int32_t* fix_count;   // items appended by the step launch (the setup pass zeroes the call's counters)
  int32_t* fix_items;   // [2 * item]: local step, 2 * wavefront + half
  int32_t fix_n_counts; // setup pass: zero fix_count[0 .. fix_n_counts)
  // FIX_SOLVE with fix_reduce: the call's last fixup and the work reduce in one launch (a workgroup per
  // 64 rollouts fixes their items, then sums their work); red_*: the reduce's own arguments
  int32_t fix_reduce, red_key_steps, red_n_steps;
  // fix_reduce with fix_barrier (a counter zeroed by the setup pass; null when the reduce grid is too large to
  // be resident at once): the items are spread over all the launch's workgroups, which meet at a grid
  // barrier before the reduce (a rollout's items may sit on another workgroup); otherwise each workgroup
  // fixes its own rollouts' items in turn
  int32_t* fix_barrier;
  double red_total_mass;
  const double* red_rollout_mass;
  uint64_t* red_best_key;
  // the call's preparation pass (hs_prep_kernel) stores the sample times of samples [ktab_lo,
  // ktab_lo + ttab_n) and, when ktab_n > 0, the limb IK (and for turning or transformed gaits the torso
  // record) of samples [ktab_lo, ktab_lo + ktab_n) per rollout (ktab_range); the step launches read them. ktab_nl: limb lanes per
  // rollout the pass enumerates (the launch's largest model)
  int32_t ktab_n, ktab_lo, ktab_nl, ttab_n;
  // the preparation pass's XCD units: rollouts [u * prep_unit, (u + 1) * prep_unit) are written on XCD
  // u % 8, where the step launches read them (0 or 2: hs_rollout_kernel's two rollouts per wavefront; 8:
  // the limb-lane kernel's eight)
  int32_t prep_unit;
  // the limb-lane kernel over a mixed plan: wavefront w runs model limb_model[w] for the rollouts
  // limb_rollouts[8 w .. 8 w + 7] (-1: an idle group), whose slots in hs_rollout_kernel's layout (the fixup's
  // items) are limb_slots[...]; limb_waves wavefronts per step (null: one model, rollouts 8 w + group)
  const int32_t *limb_model, *limb_rollouts, *limb_slots;
  int32_t limb_waves;
};

// Kernel launcher (hs_kernels.hip). `workspace` holds general_workspace_bytes()
// per rollout + 1 (global-memory scratch of the conditioning fallback; the
// extra slot serves idle half-waves). Returns a hipError_t value.
size_t general_workspace_bytes();
// one fused step's general-path scratch per rollout (fused_gen holds [steps in a launch][B + 1] of them)
size_t solve_workspace_bytes();
// the samples n_calls calls of `horizon` steps from k0 read: [lo, lo + n); the IK table holds all of
// them (n_table = n) when they fit it, else none (n_table = 0); the sample-time table the first
// n_ttab = min(n, its capacity)
void ktab_range(int32_t k0, int32_t n_t, int32_t horizon, int64_t n_calls, int32_t* lo, int32_t* n_table,
                int32_t* n_ttab);
int launch_rollouts(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp);
// single precision build of the same kernels (hs_kernels_f32.hip): outputs are float
size_t general_workspace_bytes_f32();
int launch_rollouts_f32(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp);
launch_map single_model_map(const hs_topo& t, int32_t n_rollouts);
// one launch of mp.fused_n fused steps (or the setup-only pass when mp.setup_only)
int launch_fused(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp);
int launch_fused_f32(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp);
// the same fused step launch by the limb-lane kernel (hs_limb.h): lane = (rollout, limb), 8 rollouts per
// wavefront; the steps it does not take are deferred to the FIX_SOLVE launch like the fused launch's
int launch_limb(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp);
int launch_limb_f32(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp);
// work_cot[b] = (w, w / (total_mass * step_length)) with w = (accumulate ? work_cot[b][0] : 0) + the steps'
// work in step order, then the best key
// (rollout_mass: per-rollout total mass of a mixed plan, else null and total_mass)
int launch_fused_reduce(const hs_run_args& a, double total_mass, const double* rollout_mass, const void* work_steps,
                        int32_t n_steps);
int launch_fused_reduce_f32(const hs_run_args& a, double total_mass, const double* rollout_mass,
                            const void* work_steps, int32_t n_steps);

// pergensetup::set_rec for n_rollouts x n_times items (hs_kernels.hip), rec [B][n_times][6 + 3 n_limbs]
int launch_pergen_rec(const hs_topo* d_topo, const hs_gait_params* params, int32_t n_rollouts, const double* times,
                      int32_t n_times, double* rec, void* stream);
// per-configuration kinematics (hs_config.hip): recompute_modelnodes and set_jvalues_with_lik
int launch_fk(const hs_topo* d_topo, int32_t n_parts, int32_t n_cfg, const double* config, int32_t stride,
              double* a_ground, double* a_joint, void* stream);
int launch_lik(const hs_topo* d_topo, int32_t n_cfg, const double* rec, int32_t ignore_reach, double* config,
               uint32_t* status, void* stream);

// closed-loop simulation kernels (hs_sim.hip); return hipError_t values
int launch_sim_reset(const hs_topo* d_topo, const hs_simtopo* d_sim, int32_t n_rollouts, const double* config,
                     int32_t config_stride, double* body, int32_t precision, void* stream);
int launch_sim_steps(const hs_topo* d_topo, const hs_simtopo* d_sim, const hs_simtopo_t<float>* d_sim_f32,
                     const hs_simtopo& host_sim, const hs_sim_args& a);

}  // namespace hs

constexpr int HS_MAX_DEVICES = 64;

// Per-rollout device workspaces (general-path scratch, the setup record, the IK table), one per
// (device, stream): launches on one stream run in order, so a call's setup pass hands the record
// to its step launches, and calls on different streams never share one.
struct ws_pool {
  struct slot {
    int dev;
    void* stream;
    void* ptr;
    size_t n;
  };
  std::vector<slot> live;
  std::vector<std::pair<int, void*>> retired;  // outgrown: kernels still queued may use them
  // workspace of >= n rollouts for (current device, stream); returns a hipError_t value
  int get(void* stream, size_t n, void** out);
  void release();
};

struct hs_model_s {
  hs_topo host;
  hs_topo* dev[HS_MAX_DEVICES];  // per-device topology copy, created lazily
  hs_simtopo sim;                // ODE world of the model (closed-loop simulation)
  hs_simtopo* sim_dev[HS_MAX_DEVICES];
  hs_simtopo_t<float>* sim_dev_f32[HS_MAX_DEVICES];  // rounded copy for the single-precision kernel
  ws_pool ws;
  ws_pool fused_gen, fused_work;  // hs_run_calls: general-path scratch per (step in a launch, rollout), step work
  ws_pool fused_fix;              // hs_run_calls: fixup counters and items
  std::mutex mu;
};
