// hs_capi.cpp -- implementation of include/hslabs.h (host side, HIP runtime).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <mutex>
#include <string>
#include <vector>

#include "hs_internal.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

}  // namespace

int hs::set_error(int code, const std::string& msg) { return fail(code, msg); }

namespace {

int hip_fail(hipError_t e, const char* what) {
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return HS_E_DEVICE;
}

void free_on_device(int dev, void* p) {
  int cur = 0;
  if (hipGetDevice(&cur) == hipSuccess && hipSetDevice(dev) == hipSuccess) {
    (void)hipFree(p);
    (void)hipSetDevice(cur);
  }
}

}  // namespace

// one rollout's workspace slot: either precision's RolloutWS (the fp32 build's general path computes
// in double, so its slot is not simply half the fp64 one)
static size_t ws_slot_bytes() {
  const size_t a = hs::general_workspace_bytes(), b = hs::general_workspace_bytes_f32();
  return a > b ? a : b;
}

int ws_pool::get(void* stream, size_t n, void** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  for (slot& s : live) {
    if (s.dev != dev || s.stream != stream) continue;
    if (s.n < n) {
      void* w = nullptr;
      e = hipMalloc(&w, n * ws_slot_bytes());
      if (e != hipSuccess) return (int)e;
      retired.emplace_back(dev, s.ptr);
      s.ptr = w;
      s.n = n;
    }
    *out = s.ptr;
    return 0;
  }
  void* w = nullptr;
  e = hipMalloc(&w, n * ws_slot_bytes());
  if (e != hipSuccess) return (int)e;
  live.push_back({dev, stream, w, n});
  *out = w;
  return 0;
}

void ws_pool::release() {
  for (slot& s : live) free_on_device(s.dev, s.ptr);
  for (auto& r : retired) free_on_device(r.first, r.second);
  live.clear();
  retired.clear();
}

namespace {

// Device copy of the topology for the current device (created once per device)
// and the rollout workspace of (device, stream) for at least n_rollouts rollouts.
int device_state(hs_model_t m, int n_rollouts, void* stream, const hs_topo** topo, void** ws) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  if (dev < 0 || dev >= HS_MAX_DEVICES) return fail(HS_E_DEVICE, "device index out of range");
  std::lock_guard<std::mutex> lk(m->mu);
  if (!m->dev[dev]) {
    hs_topo* d = nullptr;
    e = hipMalloc(&d, sizeof(hs_topo));
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(topo)");
    e = hipMemcpy(d, &m->host, sizeof(hs_topo), hipMemcpyHostToDevice);
    if (e != hipSuccess) { (void)hipFree(d); return hip_fail(e, "hipMemcpy(topo)"); }
    m->dev[dev] = d;
  }
  if (ws) {  // null: topology only
    e = (hipError_t)m->ws.get(stream, (size_t)n_rollouts, ws);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(workspace)");
  }
  *topo = m->dev[dev];
  return HS_OK;
}

// Device copies of the topology and the ODE world description for the current device.
int sim_device_state(hs_model_t m, const hs_topo** topo, const hs_simtopo** sim,
                     const hs_simtopo_t<float>** sim_f32 = nullptr) {
  int rc = device_state(m, 0, nullptr, topo, nullptr);
  if (rc != HS_OK) return rc;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  std::lock_guard<std::mutex> lk(m->mu);
  if (!m->sim_dev[dev]) {
    hs_simtopo* d = nullptr;
    e = hipMalloc(&d, sizeof(hs_simtopo));
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(simtopo)");
    e = hipMemcpy(d, &m->sim, sizeof(hs_simtopo), hipMemcpyHostToDevice);
    if (e != hipSuccess) { (void)hipFree(d); return hip_fail(e, "hipMemcpy(simtopo)"); }
    m->sim_dev[dev] = d;
  }
  if (sim_f32 && !m->sim_dev_f32[dev]) {
    hs_simtopo_t<float> h;
    hs_simtopo_round(h, m->sim);
    hs_simtopo_t<float>* d = nullptr;
    e = hipMalloc(&d, sizeof(h));
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(simtopo f32)");
    e = hipMemcpy(d, &h, sizeof(h), hipMemcpyHostToDevice);
    if (e != hipSuccess) { (void)hipFree(d); return hip_fail(e, "hipMemcpy(simtopo f32)"); }
    m->sim_dev_f32[dev] = d;
  }
  *sim = m->sim_dev[dev];
  if (sim_f32) *sim_f32 = m->sim_dev_f32[dev];
  return HS_OK;
}

// n_calls launches, k0 marching through the cycle (hs_run_steps semantics). total_mass / rollout_mass:
// the model's, or a mixed plan's per-rollout masses (the best key's selection COT)
int launch_steps(const hs_topo* d, const hs_run_args& a, void* ws, const hs::launch_map& mp, int32_t n_calls,
                 void* const* kernel_events, double total_mass, const double* rollout_mass) {
  hs_run_args c = a;
  hipStream_t st = (hipStream_t)a.stream;
  // the best key covers the work of all n_calls calls: taken after the last one only
  if (c.key_steps == 0) c.key_steps = (int32_t)std::min<int64_t>((int64_t)n_calls * a.horizon, INT32_MAX);
  // With the work in work_cot the key is taken by the work reduce kernel after the last launch (n_steps
  // = 0: it re-reads the accumulated work, writes the same values back and min-reduces each workgroup's
  // 64 keys before its one atomic): taken in the step launch, every wavefront's atomic on the one key
  // address queued behind the others' and the call's last launch ran 26-39 us instead of 19.6 us
  // (profiles/r05_t1_steps_trace_tail.txt)
  const bool key_reduce = a.best_key && a.work_cot && !mp.tau_in;
  // one gait setup per rollout per call: the preparation pass of the fused path (hs_prep_kernel: the
  // setup record, sample times, IK table and torso record) stores it and every launch loads it, so the
  // kinematics of these launches and of hs_run_calls' fused launches come from the same kernels
  hs::launch_map base = mp;
  base.setup_only = 1;
  base.setup_io = hs::SETUP_STORE;
  base.fix_n_counts = 0;
  hs::ktab_range(a.k0, a.n_t, a.horizon, n_calls, &base.ktab_lo, &base.ktab_n, &base.ttab_n);
  const int le0 = (a.precision == HS_PREC_F32) ? hs::launch_fused_f32(d, c, ws, base) : hs::launch_fused(d, c, ws, base);
  if (le0 != 0) return hip_fail((hipError_t)le0, "kernel launch (setup pass)");
  base.setup_only = 0;
  for (int32_t i = 0; i < n_calls; i++) {
    c.k0 = (int32_t)(((int64_t)a.k0 + (int64_t)i * a.horizon) % a.n_t);
    c.best_key = (i + 1 == n_calls && !key_reduce) ? a.best_key : nullptr;
    hs::launch_map mi = base;
    mi.setup_io = hs::SETUP_LOAD;
    hipError_t e = hipSuccess;
    if (kernel_events) e = hipEventRecord((hipEvent_t)kernel_events[2 * i], st);
    if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
    int le = (a.precision == HS_PREC_F32) ? hs::launch_rollouts_f32(d, c, ws, mi) : hs::launch_rollouts(d, c, ws, mi);
    if (le != 0) return hip_fail((hipError_t)le, "kernel launch");
    if (kernel_events) e = hipEventRecord((hipEvent_t)kernel_events[2 * i + 1], st);
    if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
  }
  if (key_reduce) {
    hs_run_args r = c;
    r.best_key = a.best_key;
    r.accumulate = 1;  // the work the launches accumulated; no step terms added
    const int le = (a.precision == HS_PREC_F32) ? hs::launch_fused_reduce_f32(r, total_mass, rollout_mass, nullptr, 0)
                                                : hs::launch_fused_reduce(r, total_mass, rollout_mass, nullptr, 0);
    if (le != 0) return hip_fail((hipError_t)le, "kernel launch (best key)");
  }
  return HS_OK;
}


// switch_torso_penalty other than (1,1): the closed form solves the (1,1) problem, so every step of
// the call takes the Eigen-style path (HS_SOLVE_REFERENCE routing, the launches sized for it)
hs_run_args routed(const hs_run_args& a, int32_t torso_mask) {
  hs_run_args c = a;
  if (torso_mask != 3) c.solve_mode = HS_SOLVE_REFERENCE;
  return c;
}

int check_args(const hs_model_s* m, const hs_run_args* a) {
  if (!m || !a) return fail(HS_E_ARG, "null model or args");
  if (a->n_rollouts < 0) return fail(HS_E_ARG, "n_rollouts < 0");
  if (a->horizon < 1) return fail(HS_E_ARG, "horizon must be >= 1");
  if (a->k0 < 0) return fail(HS_E_ARG, "k0 must be >= 0");
  if (a->precision != HS_PREC_F64 && a->precision != HS_PREC_F32) return fail(HS_E_ARG, "unknown precision");
  if (a->n_t < 1) return fail(HS_E_ARG, "n_t must be >= 1");
  if (a->n_rollouts > 0 && !a->params) return fail(HS_E_ARG, "params is null");
  if (a->n_rollouts > (1 << 30)) return fail(HS_E_ARG, "too many rollouts");
  if (a->solve_mode != HS_SOLVE_AUTO && a->solve_mode != HS_SOLVE_REFERENCE) return fail(HS_E_ARG, "unknown solve_mode");
  if (a->key_steps < 0) return fail(HS_E_ARG, "key_steps < 0");
  if (a->best_key && !a->work_cot) return fail(HS_E_ARG, "best_key needs work_cot (the key is the work's COT)");
  return HS_OK;
}

// hs_run_calls / hs_run_mixed_calls: a setup-only pass, launches of CHUNK steps over (step, wavefront),
// the in-order work reduce. Each step in flight in a launch has its own general-path scratch.
// The limb-lane kernel (hs_limb.h) takes the fused step launches of a call when the model is of its class
// (hs_topo::limb_lane_ok), the call solves in HS_SOLVE_AUTO and asks for no x, q or dq rows (the kernel
// writes tau, cf, flags and the work terms), and the preparation pass holds the IK table (the kernel reads
// its rows); HS_LIMB=0 in the environment keeps hs_rollout_kernel's fused step launch (A/B, tests)
std::atomic<int64_t> g_limb_launches{0};
// hs_run_steps' calls up to this horizon take the limb-lane kernel (a launch per call holds the call's
// horizon steps; longer calls keep hs_rollout_kernel's launch)
#define HS_ONLINE_MAX_H 64

bool limb_kernel_wanted() {
  const char* e = getenv("HS_LIMB");  // read per call: a test switches kernels within one process
  return !(e && e[0] == '0');
}
bool limb_online_wanted() {
  const char* e = getenv("HS_LIMB_ONLINE");
  return e && e[0] == '1';
}
bool limb_f32_wanted() {
  const char* e = getenv("HS_LIMB_F32");
  return !(e && e[0] == '0');
}
bool limb_eligible(const hs_topo& host, const hs_run_args& a) {
  // fp32: within the single-precision build's bound of hs_rollout_kernel's float results, not bitwise
  // (float contraction differs by context: ~1e-6 relative); HS_LIMB_F32=0 keeps hs_rollout_kernel there
  return limb_kernel_wanted() && host.limb_lane_ok && a.solve_mode == HS_SOLVE_AUTO && !a.x && !a.q && !a.dq &&
         (a.precision == HS_PREC_F64 || limb_f32_wanted());
}

// online (hs_run_steps through the limb-lane kernel): a launch per call over its horizon steps, each call
// writing output rows [0, horizon) like hs_run_steps' launches, its declined steps fixed and its work
// added to work_cot (in step order, the reduce's two roundings) by one fixup + reduce launch before the
// next call's launch, the best key by the last call's reduce
int run_fused(const hs_topo* d, const hs_run_args& a, void* ws, hs::launch_map mp, ws_pool& gen_pool,
              ws_pool& work_pool, ws_pool& fix_pool, std::mutex& mu, double total_mass, const double* rollout_mass,
              int32_t n_calls, bool limb = false, bool online = false, void* const* kernel_events = nullptr) {
  const int64_t S = online ? a.horizon : (int64_t)n_calls * a.horizon;  // output rows per rollout
  if (S > (1 << 24) || (int64_t)n_calls * a.horizon > INT32_MAX) return fail(HS_E_ARG, "too many steps");
  // steps per launch: the launch refills the SIMDs from its queue of wavefronts (the batch's last
  // wavefronts no longer end every step). Up to 512k wavefronts per launch (256 rounds of a full
  // MI355X at 2 per SIMD; measured B = 4096, 200 steps, interleaved A/B: 16 steps -2.5 %, 32 steps
  // -0.5 % against 64; 128 steps +0.5 %, 256 steps +1.2 % against 64), and each step in flight
  // holds general-path scratch for its rollouts (~13 GB at 512k wavefronts, of 288 GB HBM).
#ifndef HS_FUSED_WAVES
#define HS_FUSED_WAVES 524288
#endif
#ifndef HS_FUSED_MAX_STEPS
#define HS_FUSED_MAX_STEPS 256
#endif
#ifndef HS_FUSED_RESERVE_STEPS
#define HS_FUSED_RESERVE_STEPS 1024
#endif
  const int32_t B = a.n_rollouts;
  const int32_t CHUNK = online ? a.horizon
                               : std::max(1, std::min(HS_FUSED_MAX_STEPS, HS_FUSED_WAVES / std::max(1, mp.n_waves)));
  const int32_t n_chunks = online ? n_calls : (int32_t)((S + CHUNK - 1) / CHUNK);
  const size_t gwb = ws_slot_bytes();
  // steps the closed form declines (every step in HS_SOLVE_REFERENCE) are deferred to a fixup launch
  // after each step launch, so the step kernel carries no call to the general path; one counter per
  // launch (zeroed by the setup pass), then the items
  // (then as many grid-barrier counters for the fixup + reduce launches, hs_internal.h fix_barrier)
  const size_t fix_counts_bytes = ((size_t)2 * n_chunks * sizeof(int32_t) + 255) / 256 * 256;
  const size_t fix_bytes = fix_counts_bytes + (size_t)CHUNK * mp.n_waves * 2 * 2 * sizeof(int32_t);
  void *gen = nullptr, *work = nullptr, *fix = nullptr;
  {
    std::lock_guard<std::mutex> lk(mu);
    // the general-path scratch of every step in flight: [CHUNK][B + 1] SolveWS (in workspace units)
    hipError_t e = (hipError_t)gen_pool.get(
        a.stream, ((size_t)CHUNK * (B + 1) * hs::solve_workspace_bytes() + gwb - 1) / gwb, &gen);
    // the [step][rollout] work buffer is reserved for at least HS_FUSED_RESERVE_STEPS steps (at most
    // 512 MB) on first use, so a caller growing its call length (a short warmup, then the real run)
    // does not hit a hipMalloc between its launches
    const size_t need = (size_t)S * B * sizeof(double);
    const size_t want =
        std::max(need, std::min((size_t)HS_FUSED_RESERVE_STEPS * B * sizeof(double), (size_t)512 << 20));
    if (e == hipSuccess) e = (hipError_t)work_pool.get(a.stream, (want + gwb - 1) / gwb, &work);
    if (e == hipSuccess) e = (hipError_t)fix_pool.get(a.stream, (fix_bytes + gwb - 1) / gwb, &fix);
    if (e != hipSuccess) return hip_fail(e, "hipMalloc(fused workspace)");
  }
  int32_t* fix_counts = (int32_t*)fix;
  int32_t* fix_items = (int32_t*)((char*)fix + fix_counts_bytes);
  const bool f32 = a.precision == HS_PREC_F32;
  hs_run_args c = a;
  c.horizon = (int32_t)S;  // output rows per rollout
  c.best_key = nullptr;    // taken by the reduce, after the last step
  hs_run_args r = a;       // the reduce: its key covers the call's steps unless told otherwise
  if (r.key_steps == 0) r.key_steps = (int32_t)((int64_t)n_calls * a.horizon);
  mp.fused_h = a.horizon;
  mp.fused_work = work;
  mp.fused_gen = gen;
  mp.setup_only = 1;  // gait setup once per rollout, stored for every step
  mp.setup_io = hs::SETUP_STORE;
  mp.fix_count = fix_counts;
  mp.fix_n_counts = 2 * n_chunks;  // the fixup counters and the barrier counters
  // the fixup + reduce launch's grid barrier: its ceil(B / 64) workgroups must be resident together
  const char* fb = getenv("HS_FIX_BARRIER");  // 0: each workgroup fixes its own rollouts' items (A/B)
  const bool barrier_ok = (B + 63) / 64 <= 1024 && !(fb && fb[0] == '0');
  hs::ktab_range(a.k0, a.n_t, a.horizon, n_calls, &mp.ktab_lo, &mp.ktab_n, &mp.ttab_n);  // the preparation pass's rows
  limb = limb && mp.ktab_n > 0 && (!mp.wave_rollouts || mp.limb_rollouts);
  mp.prep_unit = limb ? 8 : 2;  // the rollouts' records written on the XCD whose step launches read them
  int le = f32 ? hs::launch_fused_f32(d, c, ws, mp) : hs::launch_fused(d, c, ws, mp);
  mp.setup_only = 0;
  mp.setup_io = hs::SETUP_LOAD;
  mp.fix_n_counts = 0;
  mp.fix_items = fix_items;
  bool reduced = false;
  if (online) {
    hipStream_t st = (hipStream_t)a.stream;
    for (int32_t i = 0; le == 0 && i < n_calls; i++) {
      c.k0 = (int32_t)(((int64_t)a.k0 + (int64_t)i * a.horizon) % a.n_t);
      mp.fused_s0 = 0;
      mp.fused_n = a.horizon;
      mp.fix_mode = hs::FIX_DEFER;
      mp.fix_count = fix_counts + i;
      mp.fix_reduce = 0;
      hipError_t e = kernel_events ? hipEventRecord((hipEvent_t)kernel_events[2 * i], st) : hipSuccess;
      if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
      if (limb) {  // (no IK table for the call: hs_rollout_kernel's fused step launch, the same shape)
        le = f32 ? hs::launch_limb_f32(d, c, ws, mp) : hs::launch_limb(d, c, ws, mp);
        g_limb_launches++;
      } else {
        le = f32 ? hs::launch_fused_f32(d, c, ws, mp) : hs::launch_fused(d, c, ws, mp);
      }
      if (le != 0) break;
      mp.fix_mode = hs::FIX_SOLVE;
      mp.fix_reduce = a.work_cot != nullptr;
      mp.fix_barrier = barrier_ok ? fix_counts + n_chunks + i : nullptr;
      if (mp.fix_reduce) {
        mp.red_total_mass = total_mass;
        mp.red_rollout_mass = rollout_mass;
        mp.red_n_steps = a.horizon;
        mp.red_key_steps = r.key_steps;
        mp.red_best_key = i + 1 == n_calls ? r.best_key : nullptr;
      }
      le = f32 ? hs::launch_fused_f32(d, c, ws, mp) : hs::launch_fused(d, c, ws, mp);
      if (le == 0 && kernel_events) e = hipEventRecord((hipEvent_t)kernel_events[2 * i + 1], st);
      if (e != hipSuccess) return hip_fail(e, "hipEventRecord");
    }
    if (le != 0) return hip_fail((hipError_t)le, "kernel launch");
    return HS_OK;
  }
  for (int64_t s0 = 0, ci = 0; le == 0 && s0 < S; s0 += CHUNK, ci++) {
    mp.fused_s0 = (int32_t)s0;
    mp.fused_n = (int32_t)std::min<int64_t>(CHUNK, S - s0);
    mp.fix_mode = hs::FIX_DEFER;
    mp.fix_count = fix_counts + ci;
    if (limb) {
      le = f32 ? hs::launch_limb_f32(d, c, ws, mp) : hs::launch_limb(d, c, ws, mp);
      g_limb_launches++;
    }
    else le = f32 ? hs::launch_fused_f32(d, c, ws, mp) : hs::launch_fused(d, c, ws, mp);
    if (le != 0) break;
    // the same steps' declined (step, rollout) items, with the general path; after the last step
    // launch of an HS_SOLVE_AUTO call (few items, if any) together with the work reduce
    mp.fix_mode = hs::FIX_SOLVE;
    mp.fix_reduce = s0 + CHUNK >= S && a.solve_mode == HS_SOLVE_AUTO && a.work_cot;
    mp.fix_barrier = barrier_ok ? fix_counts + n_chunks + ci : nullptr;
    if (mp.fix_reduce) {
      mp.red_total_mass = total_mass;
      mp.red_rollout_mass = rollout_mass;
      mp.red_n_steps = (int32_t)S;
      mp.red_key_steps = r.key_steps;
      mp.red_best_key = r.best_key;
      reduced = true;
    }
    le = f32 ? hs::launch_fused_f32(d, c, ws, mp) : hs::launch_fused(d, c, ws, mp);
  }
  if (le == 0 && !reduced)
    le = f32 ? hs::launch_fused_reduce_f32(r, total_mass, rollout_mass, work, (int32_t)S)
             : hs::launch_fused_reduce(r, total_mass, rollout_mass, work, (int32_t)S);
  if (le != 0) return hip_fail((hipError_t)le, "kernel launch");
  return HS_OK;
}

}  // namespace

namespace hs {

launch_map single_model_map(const hs_topo& t, int32_t n_rollouts) {
  launch_map mp{};
  mp.n_waves = (n_rollouts + 1) / 2;  // two rollouts per wavefront
  mp.max_parts = t.n;
  mp.ktab_nl = t.n_limbs;
  mp.st_tau = t.nmj;
  mp.st_cf = 3 * t.nf;
  mp.st_q = t.cfg;
  mp.st_x = 6 * t.n;
  return mp;
}

}  // namespace hs

struct hs_mixed_s {
  int dev = 0;
  int32_t n_rollouts = 0, n_waves = 0;
  std::vector<hs_model_t> models;
  hs_model_dims max_dims;
  int32_t st_tau = 0, st_cf = 0, st_q = 0, st_x = 0;
  hs_topo* d_topos = nullptr;  // the models' topologies, contiguous (wave_model indexes it)
  int32_t* d_wave_model = nullptr;
  int32_t* d_wave_rollouts = nullptr;
  // the limb-lane kernel's layout (every model of the plan of its class): 8 rollouts of one model per
  // wavefront, [model], [8 * wave] rollout ids (-1 idle) and their hs_rollout_kernel slots
  int32_t limb_waves = 0;
  int32_t *d_limb_model = nullptr, *d_limb_rollouts = nullptr;
  double* d_rollout_mass = nullptr;  // total mass of each rollout's model (the fused reduce's COT)
  int32_t torso_mask = 3;            // 3 unless a model's switch_torso_penalty (at plan creation) differs
  ws_pool ws;
  ws_pool fused_gen, fused_work, fused_fix;
  std::mutex mu;
};

extern "C" {

int hs_abi_version(void) { return HSLABS_ABI_VERSION; }

int hs_model_limb_lane(hs_model_t m, int32_t* ok) {
  if (!m || !ok) return fail(HS_E_ARG, "null argument");
  *ok = m->host.limb_lane_ok;
  return HS_OK;
}

int64_t hs_limb_launches(void) { return g_limb_launches.load(); }

extern "C" int hs_limb_deferred_f64(unsigned long long* out);
extern "C" int hs_limb_deferred_f32(unsigned long long* out);

int hs_limb_stats(int64_t* launches, int64_t* deferred) {
  if (launches) *launches = g_limb_launches.load();
  if (deferred) {
    unsigned long long a = 0, b = 0;
    hipError_t e = (hipError_t)hs_limb_deferred_f64(&a);
    if (e == hipSuccess) e = (hipError_t)hs_limb_deferred_f32(&b);
    if (e != hipSuccess) return hip_fail(e, "hs_limb_stats");
    *deferred = (int64_t)(a + b);
  }
  return HS_OK;
}

const char* hs_last_error(void) { return g_err.c_str(); }

int hs_model_load_ex(const char* xml_path, int lik_variant, hs_model_t* out) {
  if (!xml_path || !out) return fail(HS_E_ARG, "null argument");
  hs_model_s* m = new hs_model_s;
  memset(m->dev, 0, sizeof(m->dev));
  memset(m->sim_dev, 0, sizeof(m->sim_dev));
  memset(m->sim_dev_f32, 0, sizeof(m->sim_dev_f32));
  std::string err;
  int rc = hs::load_model_file(xml_path, lik_variant, &m->host, err, &m->sim);
  if (rc != HS_OK) {
    delete m;
    return fail(rc, err);
  }
  *out = m;
  return HS_OK;
}

int hs_model_load(const char* xml_path, hs_model_t* out) { return hs_model_load_ex(xml_path, -1, out); }

void hs_model_free(hs_model_t m) {
  if (!m) return;
  for (int d = 0; d < HS_MAX_DEVICES; d++) {
    if (m->dev[d]) free_on_device(d, m->dev[d]);
    if (m->sim_dev[d]) free_on_device(d, m->sim_dev[d]);
    if (m->sim_dev_f32[d]) free_on_device(d, m->sim_dev_f32[d]);
  }
  m->ws.release();
  m->fused_gen.release();
  m->fused_work.release();
  m->fused_fix.release();
  delete m;
}

int hs_model_get_dims(hs_model_t m, hs_model_dims* o) {
  if (!m || !o) return fail(HS_E_ARG, "null argument");
  const hs_topo& t = m->host;
  o->n_parts = t.n;
  o->nmj = t.nmj;
  o->nfeet = t.nf;
  o->config_dim = t.cfg;
  o->n_limbs = t.n_limbs;
  o->lik_kind = t.lik_kind;
  o->total_mass = t.total_mass;
  o->rcap = t.rcap;
  return HS_OK;
}

int hs_model_set_torso_penalty(hs_model_t m, int32_t force, int32_t torque) {
  if (!m) return fail(HS_E_ARG, "null model");
  if (!force && !torque) return fail(HS_E_ARG, "switch_torso_penalty(0,0): mask0 not set (ftsolver.cpp:245)");
  const int32_t mask = (force ? 1 : 0) | (torque ? 2 : 0);
  std::lock_guard<std::mutex> lk(m->mu);
  m->host.torso_mask = mask;
  bool uploaded = false;
  for (int dev = 0; dev < HS_MAX_DEVICES; dev++) uploaded |= m->dev[dev] != nullptr;
  if (!uploaded) return HS_OK;  // the first call uploads the host copy
  int cur = 0;
  hipError_t e = hipGetDevice(&cur);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  for (int dev = 0; dev < HS_MAX_DEVICES && e == hipSuccess; dev++) {
    if (!m->dev[dev]) continue;
    // later calls only: the device copy changes once the work queued before is done
    e = hipSetDevice(dev);
    if (e == hipSuccess) e = hipDeviceSynchronize();
    if (e == hipSuccess)
      e = hipMemcpy(&m->dev[dev]->torso_mask, &mask, sizeof(mask), hipMemcpyHostToDevice);
  }
  (void)hipSetDevice(cur);
  if (e != hipSuccess) return hip_fail(e, "hs_model_set_torso_penalty");
  return HS_OK;
}

int hs_model_get_torso_penalty(hs_model_t m, int32_t* force, int32_t* torque) {
  if (!m || !force || !torque) return fail(HS_E_ARG, "null argument");
  *force = (m->host.torso_mask & 1) ? 1 : 0;
  *torque = (m->host.torso_mask & 2) ? 1 : 0;
  return HS_OK;
}

int hs_model_get_node(hs_model_t m, int32_t i, hs_node_info* o) {
  if (!m || !o) return fail(HS_E_ARG, "null argument");
  const hs_topo& t = m->host;
  if (i < 0 || i >= t.n) return fail(HS_E_ARG, "node index out of range");
  const hs_node& nd = t.node[i];
  memset(o, 0, sizeof(*o));
  o->parent = nd.parent;
  o->jtype = nd.jtype;
  o->hinge = nd.hinge;
  o->foot = nd.foot;
  o->limb = -1;
  for (int L = 0; L < t.n_limbs; L++)
    if (t.limb_child[L] == i) o->limb = L;
  o->n_kids = nd.nkids;
  for (int k = 0; k < nd.nkids && k < HS_NODE_MAX_KIDS; k++) o->kids[k] = nd.kids[k];
  for (int r = 0; r < 3; r++) {
    o->com[r] = nd.com[r];
    o->foot_pos[r] = nd.foot >= 0 ? nd.cap[r] : 0.0;
  }
  o->mass = t.mass[i];
  return HS_OK;
}

int hs_pgs_config_read(const char* path, int setup_id, hs_gait_params* out, char* xml_file, int32_t xml_file_len) {
  if (!path || !out) return fail(HS_E_ARG, "null argument");
  std::string xml, err;
  int rc = hs::read_pgs_config(path, setup_id, out, xml, err);
  if (rc != HS_OK) return fail(rc, err);
  if (xml_file && xml_file_len > 0) {
    snprintf(xml_file, (size_t)xml_file_len, "%s", xml.c_str());
  }
  return HS_OK;
}

int hs_run(hs_model_t m, const hs_run_args* a) { return hs_run_steps(m, a, 1, nullptr); }

int hs_run_steps(hs_model_t m, const hs_run_args* a, int32_t n_calls, void* const* kernel_events) {
  int rc = check_args(m, a);
  if (rc != HS_OK) return rc;
  if (n_calls < 0) return fail(HS_E_ARG, "n_calls < 0");
  if (a->n_rollouts == 0 || n_calls == 0) return HS_OK;
  const hs_topo* d = nullptr;
  void* ws = nullptr;
  rc = device_state(m, a->n_rollouts + 1, a->stream, &d, &ws);  // + the idle half-wave of an odd batch
  if (rc != HS_OK) return rc;
  const hs_run_args r = routed(*a, m->host.torso_mask);
  // HS_LIMB_ONLINE=1, the limb-lane kernel's class: a launch per call and a fixup + reduce launch after it
  // (run_fused's online shape, the same outputs, work and key bitwise). Not the default: its launch of
  // B / 8 wavefronts lasts one wavefront's life, 18.2-18.7 us at B = 4096 (the limb lanes' dependent
  // chain), and the fixup + reduce adds 4.7-5.2 us: 155 M steps/s against hs_rollout_kernel's launch per
  // call with the general path inline, 20 us at 32 lanes per rollout (profiles/r06_t7_steps_trace_tail.txt)
  if (limb_online_wanted() && limb_eligible(m->host, r) && a->horizon <= HS_ONLINE_MAX_H)
    return run_fused(d, r, ws, hs::single_model_map(m->host, a->n_rollouts), m->fused_gen, m->fused_work,
                     m->fused_fix, m->mu, m->host.total_mass, nullptr, n_calls, true, true, kernel_events);
  // HS_ONLINE_DEFER=1: the same online shape on hs_rollout_kernel's fused instantiation (FIX_DEFER, 4
  // waves/SIMD, no general-path call) and its fixup + reduce per call (VERDICT r05 item 4's variant;
  // measured)
  const char* od = getenv("HS_ONLINE_DEFER");
  if (od && od[0] == '1' && r.solve_mode == HS_SOLVE_AUTO && a->horizon <= HS_ONLINE_MAX_H)
    return run_fused(d, r, ws, hs::single_model_map(m->host, a->n_rollouts), m->fused_gen, m->fused_work,
                     m->fused_fix, m->mu, m->host.total_mass, nullptr, n_calls, false, true, kernel_events);
  return launch_steps(d, r, ws, hs::single_model_map(m->host, a->n_rollouts), n_calls, kernel_events,
                      m->host.total_mass, nullptr);
}

int hs_run_calls(hs_model_t m, const hs_run_args* a, int32_t n_calls) {
  int rc = check_args(m, a);
  if (rc != HS_OK) return rc;
  if (n_calls < 0) return fail(HS_E_ARG, "n_calls < 0");
  if (a->n_rollouts == 0 || n_calls == 0) return HS_OK;
  const hs_topo* d = nullptr;
  void* ws = nullptr;
  rc = device_state(m, a->n_rollouts + 1, a->stream, &d, &ws);
  if (rc != HS_OK) return rc;
  const hs_run_args r = routed(*a, m->host.torso_mask);
  return run_fused(d, r, ws, hs::single_model_map(m->host, a->n_rollouts), m->fused_gen, m->fused_work, m->fused_fix,
                   m->mu, m->host.total_mass, nullptr, n_calls, limb_eligible(m->host, r));
}

int hs_run_pd(hs_model_t m, const hs_run_args* a, const hs_pd_args* pd) {
  int rc = check_args(m, a);
  if (rc != HS_OK) return rc;
  if (!pd || (a->n_rollouts > 0 && (!pd->q_meas || !pd->dq_meas || !pd->tau_cmd)))
    return fail(HS_E_ARG, "pd: q_meas, dq_meas and tau_cmd are required");
  if (!(pd->k >= 0)) return fail(HS_E_ARG, "pd: k must be >= 0");
  if (a->n_rollouts == 0) return HS_OK;
  const hs_topo* d = nullptr;
  void* ws = nullptr;
  rc = device_state(m, a->n_rollouts + 1, a->stream, &d, &ws);
  if (rc != HS_OK) return rc;
  hs::launch_map mp = hs::single_model_map(m->host, a->n_rollouts);
  mp.pd_q = pd->q_meas;
  mp.pd_dq = pd->dq_meas;
  mp.pd_k1 = -pd->k;                 // player.cpp:394
  mp.pd_k2 = -2 * std::sqrt(pd->k);
  mp.pd_tau = pd->tau_cmd;
  mp.pd_q0 = pd->q_target;
  mp.pd_dq0 = pd->dq_target;
  return launch_steps(d, routed(*a, m->host.torso_mask), ws, mp, 1, nullptr, m->host.total_mass, nullptr);
}

int hs_run_forces(hs_model_t m, const hs_run_args* a, const double* tau_in) {
  int rc = check_args(m, a);
  if (rc != HS_OK) return rc;
  if (a->n_rollouts > 0 && !tau_in) return fail(HS_E_ARG, "tau_in is null");
  if (a->n_rollouts == 0) return HS_OK;
  const hs_topo* d = nullptr;
  void* ws = nullptr;
  rc = device_state(m, a->n_rollouts + 1, a->stream, &d, &ws);
  if (rc != HS_OK) return rc;
  hs::launch_map mp = hs::single_model_map(m->host, a->n_rollouts);
  mp.tau_in = tau_in;
  return launch_steps(d, *a, ws, mp, 1, nullptr, m->host.total_mass, nullptr);
}

int hs_run_forces_calls(hs_model_t m, const hs_run_args* a, int32_t n_calls, const double* tau_in) {
  int rc = check_args(m, a);
  if (rc != HS_OK) return rc;
  if (n_calls < 0) return fail(HS_E_ARG, "n_calls < 0");
  if (a->n_rollouts > 0 && n_calls > 0 && !tau_in) return fail(HS_E_ARG, "tau_in is null");
  if (a->n_rollouts == 0 || n_calls == 0) return HS_OK;
  const int64_t S = (int64_t)n_calls * a->horizon;  // steps, one row each
  if (S > (1 << 24)) return fail(HS_E_ARG, "too many steps");
  const hs_topo* d = nullptr;
  void* ws = nullptr;
  rc = device_state(m, a->n_rollouts + 1, a->stream, &d, &ws);
  if (rc != HS_OK) return rc;
  hs::launch_map mp = hs::single_model_map(m->host, a->n_rollouts);
  mp.tau_in = tau_in;
  hs_run_args c = *a;
  c.horizon = (int32_t)S;  // output (and tau_in) rows per rollout
  c.tau = c.x = c.work_cot = nullptr;
  c.best_key = nullptr;
  // the run_fused scheme without the work reduce: hs_rollout_kernel's forces mode solves every step
  // itself (its LDS layout runs 3 wavefronts / SIMD). The limb-lane kernel's forces mode (the model of
  // its class, HS_SOLVE_AUTO, no q rows, fp64, the preparation pass's table) takes forces_solve's fast
  // path and defers a step whose foot block B_f is near singular (the dense normal equations) to a
  // fixup launch of hs_rollout_kernel's forces mode after each step launch
  const int32_t CHUNK = std::max(1, std::min(HS_FUSED_MAX_STEPS, HS_FUSED_WAVES / std::max(1, mp.n_waves)));
  const int32_t n_chunks = (int32_t)((S + CHUNK - 1) / CHUNK);
  const bool f32 = a->precision == HS_PREC_F32;
  mp.fused_h = a->horizon;
  mp.setup_only = 1;
  mp.setup_io = hs::SETUP_STORE;
  hs::ktab_range(a->k0, a->n_t, a->horizon, n_calls, &mp.ktab_lo, &mp.ktab_n, &mp.ttab_n);
  const bool limb = limb_kernel_wanted() && m->host.limb_lane_ok && a->solve_mode == HS_SOLVE_AUTO && !a->q &&
                    !f32 && mp.ktab_n > 0;
  int32_t* fix_counts = nullptr;
  if (limb) {
    const size_t counts_bytes = ((size_t)n_chunks * sizeof(int32_t) + 255) / 256 * 256;
    const size_t bytes = counts_bytes + (size_t)CHUNK * mp.n_waves * 2 * 2 * sizeof(int32_t);
    const size_t gwb = ws_slot_bytes();
    void* fix = nullptr;
    {
      std::lock_guard<std::mutex> lk(m->mu);
      const hipError_t e = (hipError_t)m->fused_fix.get(a->stream, (bytes + gwb - 1) / gwb, &fix);
      if (e != hipSuccess) return hip_fail(e, "hipMalloc(forces fixup items)");
    }
    fix_counts = (int32_t*)fix;
    mp.fix_count = fix_counts;
    mp.fix_n_counts = n_chunks;
    mp.fix_items = (int32_t*)((char*)fix + counts_bytes);
    mp.prep_unit = 8;
  }
  int le = f32 ? hs::launch_fused_f32(d, c, ws, mp) : hs::launch_fused(d, c, ws, mp);
  mp.setup_only = 0;
  mp.setup_io = hs::SETUP_LOAD;
  mp.fix_n_counts = 0;
  for (int64_t s0 = 0, ci = 0; le == 0 && s0 < S; s0 += CHUNK, ci++) {
    mp.fused_s0 = (int32_t)s0;
    mp.fused_n = (int32_t)std::min<int64_t>(CHUNK, S - s0);
    if (limb) {
      mp.fix_count = fix_counts + ci;
      mp.fix_mode = hs::FIX_DEFER;
      le = hs::launch_limb(d, c, ws, mp);
      g_limb_launches++;
      if (le != 0) break;
      mp.fix_mode = hs::FIX_SOLVE;
      mp.fix_reduce = 0;
      le = hs::launch_fused(d, c, ws, mp);
      mp.fix_mode = hs::FIX_NONE;
    } else {
      le = f32 ? hs::launch_fused_f32(d, c, ws, mp) : hs::launch_fused(d, c, ws, mp);
    }
  }
  if (le != 0) return hip_fail((hipError_t)le, "kernel launch");
  return HS_OK;
}

int hs_mixed_create(const hs_model_t* models, int32_t n_models, const int32_t* model_index, int32_t n_rollouts,
                    hs_mixed_t* out) {
  if (!models || !out || (n_rollouts > 0 && !model_index)) return fail(HS_E_ARG, "null argument");
  if (n_models < 1 || n_models > 64) return fail(HS_E_ARG, "n_models must be in [1, 64]");
  if (n_rollouts < 0 || n_rollouts > (1 << 30)) return fail(HS_E_ARG, "bad n_rollouts");
  std::vector<std::vector<int32_t>> groups((size_t)n_models);
  for (int32_t b = 0; b < n_rollouts; b++) {
    int32_t k = model_index[b];
    if (k < 0 || k >= n_models) return fail(HS_E_ARG, "model_index out of range");
    groups[(size_t)k].push_back(b);
  }
  hs_mixed_s* p = new hs_mixed_s;
  p->n_rollouts = n_rollouts;
  p->models.assign(models, models + n_models);
  std::vector<hs_topo> topos;
  std::vector<int32_t> wave_model, wave_rollouts;
  std::vector<int32_t> limb_model, limb_rollouts, limb_slots;
  bool limb_ok = true;
  hs_model_dims& md = p->max_dims;
  memset(&md, 0, sizeof(md));
  int32_t max_cf = 0, max_x = 0;
  for (int k = 0; k < n_models; k++) {
    if (!models[k]) { delete p; return fail(HS_E_ARG, "null model"); }
    const hs_topo& t = models[k]->host;
    topos.push_back(t);
    if (t.torso_mask != 3) p->torso_mask = t.torso_mask;  // routes the plan's calls (each wave reads its own)
    if (t.n > md.n_parts) {
      hs_model_get_dims(models[k], &md);  // the model with the most parts, maxima patched below
    }
    max_cf = std::max(max_cf, 3 * t.nf);
    max_x = std::max(max_x, 6 * t.n);
    p->st_tau = std::max(p->st_tau, t.nmj);
    p->st_q = std::max(p->st_q, t.cfg);
    const std::vector<int32_t>& g = groups[(size_t)k];
    const int32_t slot0 = (int32_t)wave_rollouts.size();
    for (size_t i = 0; i < g.size(); i += 2) {  // two rollouts of one model per wavefront
      wave_model.push_back(k);
      wave_rollouts.push_back(g[i]);
      wave_rollouts.push_back(i + 1 < g.size() ? g[i + 1] : -1);
    }
    limb_ok = limb_ok && t.limb_lane_ok;
    for (size_t i = 0; i < g.size(); i += 8) {  // the limb-lane kernel: eight per wavefront, the same order
      limb_model.push_back(k);
      for (size_t j = i; j < i + 8; j++) {
        limb_rollouts.push_back(j < g.size() ? g[j] : -1);
        limb_slots.push_back(j < g.size() ? slot0 + (int32_t)j : -1);
      }
    }
  }
  md.nmj = p->st_tau;
  md.nfeet = max_cf / 3;
  md.config_dim = p->st_q;
  p->st_cf = max_cf;
  p->st_x = max_x;
  p->n_waves = (int32_t)wave_model.size();
  hipError_t e = hipGetDevice(&p->dev);
  size_t nt = topos.size() * sizeof(hs_topo), nw = wave_model.size() * sizeof(int32_t);
  if (e == hipSuccess) e = hipMalloc(&p->d_topos, nt);
  if (e == hipSuccess && nw) e = hipMalloc(&p->d_wave_model, nw);
  if (e == hipSuccess && nw) e = hipMalloc(&p->d_wave_rollouts, 2 * nw);
  if (e == hipSuccess) e = hipMemcpy(p->d_topos, topos.data(), nt, hipMemcpyHostToDevice);
  if (e == hipSuccess && nw) e = hipMemcpy(p->d_wave_model, wave_model.data(), nw, hipMemcpyHostToDevice);
  if (e == hipSuccess && nw) e = hipMemcpy(p->d_wave_rollouts, wave_rollouts.data(), 2 * nw, hipMemcpyHostToDevice);
  if (e == hipSuccess && limb_ok && !limb_model.empty()) {
    // [model][rollouts][slots] in one allocation
    const size_t nl = limb_model.size();
    e = hipMalloc(&p->d_limb_model, (nl + 16 * nl) * sizeof(int32_t));
    p->limb_waves = (int32_t)nl;
    p->d_limb_rollouts = p->d_limb_model + nl;
    if (e == hipSuccess) e = hipMemcpy(p->d_limb_model, limb_model.data(), nl * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(p->d_limb_rollouts, limb_rollouts.data(), 8 * nl * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e == hipSuccess)
      e = hipMemcpy(p->d_limb_rollouts + 8 * nl, limb_slots.data(), 8 * nl * sizeof(int32_t), hipMemcpyHostToDevice);
  }
  if (e == hipSuccess && n_rollouts > 0) {
    std::vector<double> mass((size_t)n_rollouts);
    for (int32_t r = 0; r < n_rollouts; r++) mass[(size_t)r] = models[model_index[r]]->host.total_mass;
    e = hipMalloc(&p->d_rollout_mass, mass.size() * sizeof(double));
    if (e == hipSuccess) e = hipMemcpy(p->d_rollout_mass, mass.data(), mass.size() * sizeof(double), hipMemcpyHostToDevice);
  }
  if (e != hipSuccess) {
    hs_mixed_free(p);
    return hip_fail(e, "mixed plan upload");
  }
  *out = p;
  return HS_OK;
}

void hs_mixed_free(hs_mixed_t p) {
  if (!p) return;
  if (p->d_topos) free_on_device(p->dev, p->d_topos);
  if (p->d_wave_model) free_on_device(p->dev, p->d_wave_model);
  if (p->d_wave_rollouts) free_on_device(p->dev, p->d_wave_rollouts);
  if (p->d_limb_model) free_on_device(p->dev, p->d_limb_model);
  if (p->d_rollout_mass) free_on_device(p->dev, p->d_rollout_mass);
  p->ws.release();
  p->fused_gen.release();
  p->fused_work.release();
  p->fused_fix.release();
  delete p;
}

int hs_mixed_get_dims(hs_mixed_t p, hs_model_dims* out) {
  if (!p || !out) return fail(HS_E_ARG, "null argument");
  *out = p->max_dims;
  return HS_OK;
}

int hs_run_mixed(hs_mixed_t p, const hs_run_args* a) { return hs_run_mixed_steps(p, a, 1, nullptr); }

int hs_run_mixed_steps(hs_mixed_t p, const hs_run_args* a, int32_t n_calls, void* const* kernel_events) {
  if (!p) return fail(HS_E_ARG, "null plan");
  int rc = check_args(p->models[0], a);
  if (rc != HS_OK) return rc;
  if (a->n_rollouts != p->n_rollouts) return fail(HS_E_ARG, "n_rollouts differs from the plan's");
  if (n_calls < 0) return fail(HS_E_ARG, "n_calls < 0");
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  if (dev != p->dev) return fail(HS_E_DEVICE, "plan was created on another device");
  if (a->n_rollouts == 0 || n_calls == 0) return HS_OK;
  hs::launch_map mp{};
  mp.wave_model = p->d_wave_model;
  mp.wave_rollouts = p->d_wave_rollouts;
  mp.n_waves = p->n_waves;
  mp.max_parts = p->max_dims.n_parts;
  mp.st_tau = p->st_tau;
  mp.st_cf = p->st_cf;
  mp.st_q = p->st_q;
  mp.st_x = p->st_x;
  void* ws = nullptr;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    e = (hipError_t)p->ws.get(a->stream, (size_t)p->n_rollouts + 1, &ws);
  }
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(workspace)");
  return launch_steps(p->d_topos, routed(*a, p->torso_mask), ws, mp, n_calls, kernel_events, 0.0, p->d_rollout_mass);
}

int hs_run_mixed_calls(hs_mixed_t p, const hs_run_args* a, int32_t n_calls) {
  if (!p) return fail(HS_E_ARG, "null plan");
  int rc = check_args(p->models[0], a);
  if (rc != HS_OK) return rc;
  if (a->n_rollouts != p->n_rollouts) return fail(HS_E_ARG, "n_rollouts differs from the plan's");
  if (n_calls < 0) return fail(HS_E_ARG, "n_calls < 0");
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  if (dev != p->dev) return fail(HS_E_DEVICE, "plan was created on another device");
  if (a->n_rollouts == 0 || n_calls == 0) return HS_OK;
  hs::launch_map mp{};
  mp.wave_model = p->d_wave_model;
  mp.wave_rollouts = p->d_wave_rollouts;
  mp.n_waves = p->n_waves;
  mp.max_parts = p->max_dims.n_parts;
  mp.st_tau = p->st_tau;
  mp.st_cf = p->st_cf;
  mp.st_q = p->st_q;
  mp.st_x = p->st_x;
  void* ws = nullptr;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    e = (hipError_t)p->ws.get(a->stream, (size_t)p->n_rollouts + 1, &ws);
  }
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(workspace)");
  const hs_run_args r = routed(*a, p->torso_mask);
  bool limb = false;
  if (p->d_limb_model) {  // every model of the plan is of the limb-lane kernel's class
    mp.limb_model = p->d_limb_model;
    mp.limb_rollouts = p->d_limb_rollouts;
    mp.limb_slots = p->d_limb_rollouts + 8 * (size_t)p->limb_waves;
    mp.limb_waves = p->limb_waves;
    limb = limb_eligible(p->models[0]->host, r);
  }
  return run_fused(p->d_topos, r, ws, mp, p->fused_gen, p->fused_work, p->fused_fix, p->mu, 0.0, p->d_rollout_mass,
                   n_calls, limb);
}

int hs_complete_traj(hs_model_t m, const hs_gait_params* params, int32_t B, int32_t n_t, int32_t ignore_reach,
                     double* rec) {
  if (!m || (B > 0 && (!params || !rec))) return fail(HS_E_ARG, "null argument");
  if (B <= 0 || n_t < 2) return fail(HS_E_ARG, "empty batch or n_t < 2");
  const hs_topo& t = m->host;
  const size_t rows = (size_t)B * n_t, cfg = (size_t)t.cfg, nmj = (size_t)t.nmj;
  hs_gait_params* dp = nullptr;
  double *dq = nullptr, *ddq = nullptr, *dtau = nullptr;
  hipError_t e = hipMalloc(&dp, (size_t)B * sizeof(hs_gait_params));
  if (e == hipSuccess) e = hipMalloc(&dq, rows * cfg * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&ddq, rows * cfg * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&dtau, rows * nmj * sizeof(double));
  if (e == hipSuccess) e = hipMemcpy(dp, params, (size_t)B * sizeof(hs_gait_params), hipMemcpyHostToDevice);
  int rc = HS_OK;
  if (e != hipSuccess) {
    rc = hip_fail(e, "alloc/copy");
  } else {
    hs_run_args a;
    memset(&a, 0, sizeof(a));
    a.n_rollouts = B;
    a.horizon = n_t;  // compute_torques_over_period: steps i = 2 .. n_t + 1
    a.n_t = n_t;
    a.ignore_reach = ignore_reach;
    a.params = dp;
    a.q = dq;
    a.dq = ddq;
    a.tau = dtau;
    rc = hs_run(m, &a);
    std::vector<double> q(rows * cfg), v(rows * cfg), tau(rows * nmj);
    if (rc == HS_OK) e = hipDeviceSynchronize();
    if (rc == HS_OK && e == hipSuccess) e = hipMemcpy(q.data(), dq, q.size() * sizeof(double), hipMemcpyDeviceToHost);
    if (rc == HS_OK && e == hipSuccess) e = hipMemcpy(v.data(), ddq, v.size() * sizeof(double), hipMemcpyDeviceToHost);
    if (rc == HS_OK && e == hipSuccess)
      e = hipMemcpy(tau.data(), dtau, tau.size() * sizeof(double), hipMemcpyDeviceToHost);
    if (rc == HS_OK && e != hipSuccess) rc = hip_fail(e, "run/copy back");
    if (rc == HS_OK) {
      const size_t len = 2 * cfg + nmj;
      for (int32_t b = 0; b < B; b++)
        for (int32_t tsi = 0; tsi < n_t; tsi++) {  // get_complete_traj_rec: tsi < 2 -> tsi + n_t
          const int32_t i = (tsi < 2) ? tsi + n_t : tsi;
          const size_t src = (size_t)b * n_t + (size_t)(i - 2);
          double* r = rec + ((size_t)b * n_t + tsi) * len;
          std::copy(&q[src * cfg], &q[src * cfg] + cfg, r);
          std::copy(&v[src * cfg], &v[src * cfg] + cfg, r + cfg);
          std::copy(&tau[src * nmj], &tau[src * nmj] + nmj, r + 2 * cfg);
        }
    }
  }
  (void)hipFree(dp);
  (void)hipFree(dq);
  (void)hipFree(ddq);
  (void)hipFree(dtau);
  return rc;
}

int hs_run_forces_host(hs_model_t m, const hs_gait_params* params, int32_t B, int32_t n_t, int32_t k0, int32_t H,
                       int32_t ignore_reach, const double* tau_in, double* cf, uint32_t* flags) {
  if (!m || (B > 0 && (!params || !tau_in))) return fail(HS_E_ARG, "null argument");
  if (B <= 0 || H <= 0) return fail(HS_E_ARG, "empty batch");
  const hs_topo& t = m->host;
  const size_t rows = (size_t)B * H, nmj = (size_t)t.nmj, ncf = 3 * (size_t)t.nf;
  hs_gait_params* dp = nullptr;
  double *dtau = nullptr, *dcf = nullptr;
  uint32_t* dfl = nullptr;
  hipError_t e = hipMalloc(&dp, (size_t)B * sizeof(hs_gait_params));
  if (e == hipSuccess) e = hipMalloc(&dtau, rows * nmj * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&dcf, rows * ncf * sizeof(double));
  if (e == hipSuccess) e = hipMalloc(&dfl, rows * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemcpy(dp, params, (size_t)B * sizeof(hs_gait_params), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dtau, tau_in, rows * nmj * sizeof(double), hipMemcpyHostToDevice);
  int rc = HS_OK;
  if (e != hipSuccess) {
    rc = hip_fail(e, "alloc/copy");
  } else {
    hs_run_args a;
    memset(&a, 0, sizeof(a));
    a.n_rollouts = B;
    a.horizon = H;
    a.k0 = k0;
    a.n_t = n_t;
    a.ignore_reach = ignore_reach;
    a.params = dp;
    a.cf = dcf;
    a.flags = dfl;
    rc = hs_run_forces(m, &a, dtau);
    if (rc == HS_OK) e = hipDeviceSynchronize();
    if (rc == HS_OK && e == hipSuccess && cf) e = hipMemcpy(cf, dcf, rows * ncf * sizeof(double), hipMemcpyDeviceToHost);
    if (rc == HS_OK && e == hipSuccess && flags)
      e = hipMemcpy(flags, dfl, rows * sizeof(uint32_t), hipMemcpyDeviceToHost);
    if (rc == HS_OK && e != hipSuccess) rc = hip_fail(e, "run/copy back");
  }
  (void)hipFree(dp);
  (void)hipFree(dtau);
  (void)hipFree(dcf);
  (void)hipFree(dfl);
  return rc;
}

int hs_traj_save(const char* path, const double* rec, int32_t n_rows, int32_t rec_len, int32_t append) {
  if (!path || (n_rows > 0 && !rec) || n_rows < 0 || rec_len < 0) return fail(HS_E_ARG, "bad argument");
  std::ofstream file(path, append ? std::ios_base::app : std::ios_base::out);
  if (!file) return fail(HS_E_IO, std::string("cannot open ") + path);
  for (int32_t i = 0; i < n_rows; i++) {
    for (int32_t j = 0; j < rec_len; j++) {
      if (j) file << " ";
      file << rec[(size_t)i * rec_len + j];
    }
    file << std::endl;
  }
  return file ? HS_OK : fail(HS_E_IO, std::string("write failed: ") + path);
}

int hs_run_host(hs_model_t m, const hs_gait_params* params, int32_t B, int32_t n_t, int32_t k0, int32_t H,
                int32_t ignore_reach, double* q, double* tau, double* cf, double* x, uint32_t* flags,
                double* work_cot) {
  if (!m || (B > 0 && !params)) return fail(HS_E_ARG, "null argument");
  if (B <= 0 || H <= 0) return fail(HS_E_ARG, "empty batch");
  const hs_topo& t = m->host;
  size_t nq = (size_t)B * H * t.cfg, ntau = (size_t)B * H * t.nmj, ncf = (size_t)B * H * 3 * t.nf;
  size_t nx = (size_t)B * H * 6 * t.n, nfl = (size_t)B * H, nwc = (size_t)B * 2;
  hs_gait_params* dp = nullptr;
  double *dq = nullptr, *dtau = nullptr, *dcf = nullptr, *dx = nullptr, *dwc = nullptr;
  uint32_t* dfl = nullptr;
  hipError_t e = hipSuccess;
  int rc = HS_OK;
#define HS_ALLOC(ptr, n, T)                                   \
  if (e == hipSuccess) e = hipMalloc(&ptr, (n) * sizeof(T));
  HS_ALLOC(dp, (size_t)B, hs_gait_params);
  if (q) HS_ALLOC(dq, nq, double);
  if (tau) HS_ALLOC(dtau, ntau, double);
  if (cf) HS_ALLOC(dcf, ncf, double);
  if (x) HS_ALLOC(dx, nx, double);
  if (flags) HS_ALLOC(dfl, nfl, uint32_t);
  if (work_cot) HS_ALLOC(dwc, nwc, double);
#undef HS_ALLOC
  if (e == hipSuccess) e = hipMemcpy(dp, params, (size_t)B * sizeof(hs_gait_params), hipMemcpyHostToDevice);
  if (e != hipSuccess) {
    rc = hip_fail(e, "alloc/copy");
  } else {
    hs_run_args a;
    memset(&a, 0, sizeof(a));
    a.n_rollouts = B;
    a.horizon = H;
    a.k0 = k0;
    a.n_t = n_t;
    a.ignore_reach = ignore_reach;
    a.params = dp;
    a.q = dq;
    a.tau = dtau;
    a.cf = dcf;
    a.x = dx;
    a.flags = dfl;
    a.work_cot = dwc;
    rc = hs_run(m, &a);
    if (rc == HS_OK) {
      e = hipDeviceSynchronize();
      if (e == hipSuccess && q) e = hipMemcpy(q, dq, nq * sizeof(double), hipMemcpyDeviceToHost);
      if (e == hipSuccess && tau) e = hipMemcpy(tau, dtau, ntau * sizeof(double), hipMemcpyDeviceToHost);
      if (e == hipSuccess && cf) e = hipMemcpy(cf, dcf, ncf * sizeof(double), hipMemcpyDeviceToHost);
      if (e == hipSuccess && x) e = hipMemcpy(x, dx, nx * sizeof(double), hipMemcpyDeviceToHost);
      if (e == hipSuccess && flags) e = hipMemcpy(flags, dfl, nfl * sizeof(uint32_t), hipMemcpyDeviceToHost);
      if (e == hipSuccess && work_cot) e = hipMemcpy(work_cot, dwc, nwc * sizeof(double), hipMemcpyDeviceToHost);
      if (e != hipSuccess) rc = hip_fail(e, "run/copy back");
    }
  }
  (void)hipFree(dp);
  (void)hipFree(dq);
  (void)hipFree(dtau);
  (void)hipFree(dcf);
  (void)hipFree(dx);
  (void)hipFree(dfl);
  (void)hipFree(dwc);
  return rc;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// per-configuration kinematics (hs_config.hip, hs_kernels.hip)
// ---------------------------------------------------------------------------
namespace {

// device scratch of a synchronous host-buffer call: freed on scope exit
struct dev_buf {
  void* p = nullptr;
  hipError_t alloc(size_t bytes) { return bytes ? hipMalloc(&p, bytes) : hipSuccess; }
  ~dev_buf() { (void)hipFree(p); }
  template <class T>
  T* as() const { return static_cast<T*>(p); }
};

}  // namespace

extern "C" {

int hs_pergen_rec(hs_model_t m, const hs_gait_params* params, int32_t B, const double* times, int32_t n_times,
                  double* rec, void* stream) {
  if (!m) return fail(HS_E_ARG, "null model");
  if (B < 0 || n_times < 0 || (int64_t)B * n_times > (int64_t(1) << 31)) return fail(HS_E_ARG, "bad batch size");
  if ((int64_t)B * n_times == 0) return HS_OK;
  if (!params || !times || !rec) return fail(HS_E_ARG, "null params, times or rec");
  const hs_topo* d = nullptr;
  int rc = device_state(m, 0, nullptr, &d, nullptr);
  if (rc != HS_OK) return rc;
  int e = hs::launch_pergen_rec(d, params, B, times, n_times, rec, stream);
  return e ? hip_fail((hipError_t)e, "hs_pergen_rec launch") : HS_OK;
}

int hs_pergen_rec_host(hs_model_t m, const hs_gait_params* params, int32_t B, const double* times, int32_t n_times,
                       double* rec) {
  if (!m) return fail(HS_E_ARG, "null model");
  if (B < 0 || n_times < 0 || (int64_t)B * n_times > (int64_t(1) << 31)) return fail(HS_E_ARG, "bad batch size");
  if ((int64_t)B * n_times == 0) return HS_OK;
  if (!params || !times || !rec) return fail(HS_E_ARG, "null params, times or rec");
  const size_t len = 6 + 3 * (size_t)m->host.n_limbs, nrec = (size_t)B * n_times * len;
  dev_buf dp, dt, dr;
  hipError_t e = dp.alloc((size_t)B * sizeof(hs_gait_params));
  if (e == hipSuccess) e = dt.alloc((size_t)n_times * sizeof(double));
  if (e == hipSuccess) e = dr.alloc(nrec * sizeof(double));
  if (e == hipSuccess) e = hipMemcpy(dp.p, params, (size_t)B * sizeof(hs_gait_params), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dt.p, times, (size_t)n_times * sizeof(double), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "alloc/copy");
  int rc = hs_pergen_rec(m, dp.as<hs_gait_params>(), B, dt.as<double>(), n_times, dr.as<double>(), nullptr);
  if (rc != HS_OK) return rc;
  e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(rec, dr.p, nrec * sizeof(double), hipMemcpyDeviceToHost);
  return e == hipSuccess ? HS_OK : hip_fail(e, "run/copy back");
}

int hs_model_lik(hs_model_t m, int32_t n, const double* rec, int32_t ignore_reach, double* config, uint32_t* status,
                 void* stream) {
  if (!m) return fail(HS_E_ARG, "null model");
  if (n < 0 || n > (1 << 30)) return fail(HS_E_ARG, "bad n");
  if (n == 0) return HS_OK;
  if (!rec || !config) return fail(HS_E_ARG, "null rec or config");
  const hs_topo* d = nullptr;
  int rc = device_state(m, 0, nullptr, &d, nullptr);
  if (rc != HS_OK) return rc;
  int e = hs::launch_lik(d, n, rec, ignore_reach, config, status, stream);
  return e ? hip_fail((hipError_t)e, "hs_model_lik launch") : HS_OK;
}

int hs_model_lik_host(hs_model_t m, int32_t n, const double* rec, int32_t ignore_reach, double* config,
                      uint32_t* status) {
  if (!m) return fail(HS_E_ARG, "null model");
  if (n < 0 || n > (1 << 30)) return fail(HS_E_ARG, "bad n");
  if (n == 0) return HS_OK;
  if (!rec || !config) return fail(HS_E_ARG, "null rec or config");
  const size_t nrec = (size_t)n * (6 + 3 * (size_t)m->host.n_limbs), ncfg = (size_t)n * m->host.cfg;
  dev_buf dr, dc, ds;
  hipError_t e = dr.alloc(nrec * sizeof(double));
  if (e == hipSuccess) e = dc.alloc(ncfg * sizeof(double));
  if (e == hipSuccess) e = ds.alloc((size_t)n * sizeof(uint32_t));
  if (e == hipSuccess) e = hipMemcpy(dr.p, rec, nrec * sizeof(double), hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(dc.p, config, ncfg * sizeof(double), hipMemcpyHostToDevice);  // kept entries
  if (e != hipSuccess) return hip_fail(e, "alloc/copy");
  int rc = hs_model_lik(m, n, dr.as<double>(), ignore_reach, dc.as<double>(), ds.as<uint32_t>(), nullptr);
  if (rc != HS_OK) return rc;
  std::vector<uint32_t> st((size_t)n);
  e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(config, dc.p, ncfg * sizeof(double), hipMemcpyDeviceToHost);
  if (e == hipSuccess) e = hipMemcpy(st.data(), ds.p, (size_t)n * sizeof(uint32_t), hipMemcpyDeviceToHost);
  if (e != hipSuccess) return hip_fail(e, "run/copy back");
  if (status) std::copy(st.begin(), st.end(), status);
  for (int32_t i = 0; i < n; i++)
    if (st[i] & HS_FLAG_LIK_FAILED)
      return fail(HS_E_ARG, "limb target out of reach in configuration " + std::to_string(i) +
                                " (lik.cpp:321-330; set ignore_reach to clamp it)");
  return HS_OK;
}

int hs_model_fk(hs_model_t m, int32_t n, const double* config, int32_t stride, double* a_ground, double* a_joint,
                void* stream) {
  if (!m) return fail(HS_E_ARG, "null model");
  if (n < 0 || n > (1 << 26)) return fail(HS_E_ARG, "bad n");
  if (n == 0) return HS_OK;
  if (!config || !a_ground) return fail(HS_E_ARG, "null config or a_ground");
  if (stride < m->host.cfg) return fail(HS_E_ARG, "config_stride < config_dim");
  const hs_topo* d = nullptr;
  int rc = device_state(m, 0, nullptr, &d, nullptr);
  if (rc != HS_OK) return rc;
  int e = hs::launch_fk(d, m->host.n, n, config, stride, a_ground, a_joint, stream);
  return e ? hip_fail((hipError_t)e, "hs_model_fk launch") : HS_OK;
}

int hs_model_fk_host(hs_model_t m, int32_t n, const double* config, int32_t stride, double* a_ground,
                     double* a_joint) {
  if (!m) return fail(HS_E_ARG, "null model");
  if (n < 0 || n > (1 << 26)) return fail(HS_E_ARG, "bad n");
  if (n == 0) return HS_OK;
  if (!config || !a_ground) return fail(HS_E_ARG, "null config or a_ground");
  if (stride < m->host.cfg) return fail(HS_E_ARG, "config_stride < config_dim");
  const size_t ncfg = (size_t)n * stride, na = (size_t)n * m->host.n * 12;
  dev_buf dc, dg, dj;
  hipError_t e = dc.alloc(ncfg * sizeof(double));
  if (e == hipSuccess) e = dg.alloc(na * sizeof(double));
  if (e == hipSuccess && a_joint) e = dj.alloc(na * sizeof(double));
  if (e == hipSuccess) e = hipMemcpy(dc.p, config, ncfg * sizeof(double), hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_fail(e, "alloc/copy");
  int rc = hs_model_fk(m, n, dc.as<double>(), stride, dg.as<double>(), dj.as<double>(), nullptr);
  if (rc != HS_OK) return rc;
  e = hipDeviceSynchronize();
  if (e == hipSuccess) e = hipMemcpy(a_ground, dg.p, na * sizeof(double), hipMemcpyDeviceToHost);
  if (e == hipSuccess && a_joint) e = hipMemcpy(a_joint, dj.p, na * sizeof(double), hipMemcpyDeviceToHost);
  return e == hipSuccess ? HS_OK : hip_fail(e, "run/copy back");
}

double hs_best_key_cot(double work, double total_mass, double step_length, int32_t n_t, int32_t steps) {
  const double aL = std::fabs(step_length);  // the device computes the same expression (key_cot)
  if (!(aL >= HS_KEY_MIN_STEP_LENGTH) || n_t < 1 || steps < 1) return NAN;
  return work * ((double)n_t / (double)steps) / (total_mass * aL);
}

uint64_t hs_best_key_encode(double cot, int64_t id) {
  float c = (float)cot;
  uint32_t bits;
  memcpy(&bits, &c, 4);
  uint32_t ord = std::isnan(c) ? 0xFFFFFFFFu : ((bits & 0x80000000u) ? ~bits : (bits | 0x80000000u));
  return ((uint64_t)ord << 32) | (uint32_t)id;
}

void hs_best_key_decode(uint64_t key, float* cot, int64_t* id) {
  uint32_t ord = (uint32_t)(key >> 32);
  uint32_t bits = (ord & 0x80000000u) ? (ord & 0x7FFFFFFFu) : ~ord;
  float c;
  memcpy(&c, &bits, 4);
  if (ord == 0xFFFFFFFFu) c = NAN;
  if (cot) *cot = c;
  if (id) *id = (int64_t)(uint32_t)key;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// closed-loop simulation (hs_sim.hip)
// ---------------------------------------------------------------------------
extern "C" {

void hs_sim_default_params(hs_sim_params* p) {
  if (!p) return;
  memset(p, 0, sizeof(*p));
  p->dt = 0.01;          // modelplayer::play_dt (player.cpp:23)
  p->k = 100;            // set_position_control_torques (player.cpp:393)
  p->sor_w = 1.3;        // ODE dWorldSetQuickStepW default
  p->erp = 0.8;          // visualization.cpp:146
  p->cfm = 1e-10;        // ODE global CFM default (double precision); visualization.cpp:147 leaves it
  p->gravity = 1;        // visualization.cpp:144
  p->bounce = 0.5;       // nearCallback (visualization.cpp:310-320)
  p->bounce_vel = 0.1;
  p->soft_cfm = 0.001;
  p->mu = INFINITY;      // dInfinity
  p->iterations = 20;    // ODE dWorldSetQuickStepNumIterations default
}

int hs_sim_reset(hs_model_t m, int32_t n_rollouts, const double* config, int32_t config_stride, double* body,
                 int32_t precision, void* stream) {
  if (!m) return fail(HS_E_ARG, "null model");
  if (n_rollouts < 0 || n_rollouts > (1 << 30)) return fail(HS_E_ARG, "bad n_rollouts");
  if (n_rollouts == 0) return HS_OK;
  if (!config || !body) return fail(HS_E_ARG, "null config or body");
  if (config_stride < m->host.cfg) return fail(HS_E_ARG, "config_stride < config_dim");
  if (precision != HS_PREC_F64 && precision != HS_PREC_F32) return fail(HS_E_ARG, "unknown precision");
  const hs_topo* d = nullptr;
  const hs_simtopo* ds = nullptr;
  int rc = sim_device_state(m, &d, &ds);
  if (rc != HS_OK) return rc;
  int e = hs::launch_sim_reset(d, ds, n_rollouts, config, config_stride, body, precision, stream);
  if (e != 0) return hip_fail((hipError_t)e, "hs_sim_reset launch");
  return HS_OK;
}

int hs_sim_step(hs_model_t m, const hs_sim_args* a) {
  if (!m || !a) return fail(HS_E_ARG, "null model or args");
  if (a->n_rollouts < 0 || a->n_rollouts > (1 << 30)) return fail(HS_E_ARG, "bad n_rollouts");
  if (a->n_steps < 0) return fail(HS_E_ARG, "n_steps < 0");
  if (a->n_rollouts == 0 || a->n_steps == 0) return HS_OK;
  if (!a->body || !a->seed || !a->tsi) return fail(HS_E_ARG, "body, seed and tsi are required");
  const hs_sim_params& P = a->params;
  if (!(P.dt > 0)) return fail(HS_E_ARG, "dt must be > 0");
  if (P.iterations < 0) return fail(HS_E_ARG, "iterations < 0");
  if (!(P.mu > 0)) return fail(HS_E_ARG, "mu must be > 0 (the reference uses dInfinity: 3 rows per contact)");
  if (P.k > 0) {
    if (a->n_t < 1) return fail(HS_E_ARG, "n_t must be >= 1 with position control");
    if (!a->q_tab || !a->dq_tab || !a->tau_tab) return fail(HS_E_ARG, "controller tables are required when k > 0");
  }
  if (m->sim.m_max > 9 * HS_NMAX) return fail(HS_E_TOPOLOGY, "too many constraint rows for the simulation kernel");
  if (a->precision != HS_PREC_F64 && a->precision != HS_PREC_F32) return fail(HS_E_ARG, "unknown precision");
  const hs_topo* d = nullptr;
  const hs_simtopo* ds = nullptr;
  const hs_simtopo_t<float>* dsf = nullptr;
  int rc = sim_device_state(m, &d, &ds, a->precision == HS_PREC_F32 ? &dsf : nullptr);
  if (rc != HS_OK) return rc;
  hs_sim_args c = *a;
  if (c.n_t < 1) c.n_t = 1;
  int e = hs::launch_sim_steps(d, ds, dsf, m->sim, c);
  if (e != 0) return hip_fail((hipError_t)e, "hs_sim_step launch");
  return HS_OK;
}

struct hs_sim_s {
  hs_model_t model;
  int dev;
  hipStream_t stream;
  int32_t B, n_t;
  hs_sim_params params;
  void *params_d, *q, *dq, *tau, *body, *seed, *tsi;
  void* out[5];
  size_t out_steps;
};

void hs_sim_free(hs_sim_t s) {
  if (!s) return;
  int cur = 0;
  (void)hipGetDevice(&cur);
  (void)hipSetDevice(s->dev);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  for (void* p : {s->params_d, s->q, s->dq, s->tau, s->body, s->seed, s->tsi}) (void)hipFree(p);
  for (void* p : s->out) (void)hipFree(p);
  if (s->stream) (void)hipStreamDestroy(s->stream);
  (void)hipSetDevice(cur);
  delete s;
}

int hs_sim_create(hs_model_t m, const hs_gait_params* params, int32_t B, const hs_sim_params* sp, double t0,
                  hs_sim_t* out) {
  if (!m || !params || !out || B < 1) return fail(HS_E_ARG, "hs_sim_create: null argument or B < 1");
  hs_sim_params P;
  if (sp) P = *sp;
  else hs_sim_default_params(&P);
  if (!(P.dt > 0)) return fail(HS_E_ARG, "dt must be > 0");
  const int n_t = (int)(params[0].period / P.dt + .5);  // setup_per_controller (player.cpp:376)
  for (int b = 1; b < B; b++)
    if ((int)(params[b].period / P.dt + .5) != n_t) return fail(HS_E_ARG, "rollouts need one n_t = int(T/dt+.5)");
  if (n_t < 2) return fail(HS_E_ARG, "period shorter than two simulation steps");
  hs_sim_s* s = new hs_sim_s();
  s->model = m;
  s->B = B;
  s->n_t = n_t;
  s->params = P;
  const hs_topo& t = m->host;
  hipError_t e = hipGetDevice(&s->dev);
  if (e == hipSuccess) e = hipStreamCreate(&s->stream);
  const size_t nb = (size_t)B;
  auto alloc = [&](void** p, size_t bytes) {
    if (e == hipSuccess) e = hipMalloc(p, bytes);
  };
  alloc(&s->params_d, nb * sizeof(hs_gait_params));
  alloc(&s->q, nb * n_t * t.cfg * sizeof(double));
  alloc(&s->dq, nb * n_t * t.cfg * sizeof(double));
  alloc(&s->tau, nb * n_t * t.nmj * sizeof(double));
  alloc(&s->body, nb * t.n * HS_SIM_BODY_STRIDE * sizeof(double));
  alloc(&s->seed, nb * sizeof(uint32_t));
  alloc(&s->tsi, nb * sizeof(int32_t));
  if (e == hipSuccess) e = hipMemcpyAsync(s->params_d, params, nb * sizeof(hs_gait_params), hipMemcpyHostToDevice, s->stream);
  if (e != hipSuccess) {
    hs_sim_free(s);
    return hip_fail(e, "hs_sim_create");
  }
  hs_run_args a;
  memset(&a, 0, sizeof(a));
  a.n_rollouts = B;
  a.horizon = n_t;
  a.k0 = 0;
  a.n_t = n_t;
  a.ignore_reach = 1;
  a.params = (const hs_gait_params*)s->params_d;
  a.q = (double*)s->q;
  a.dq = (double*)s->dq;
  a.tau = (double*)s->tau;
  a.stream = s->stream;
  int rc = hs_run(m, &a);
  const int tsi0 = (int)(t0 / P.dt + .5);  // play_t = int(t0/play_dt+.5)*play_dt
  const int h0 = ((tsi0 % n_t) + n_t - 2) % n_t;
  if (rc == HS_OK)
    rc = hs_sim_reset(m, B, (const double*)s->q + (size_t)h0 * t.cfg, n_t * t.cfg, (double*)s->body, HS_PREC_F64,
                      s->stream);
  std::vector<int32_t> tsi(nb, tsi0);
  if (rc == HS_OK) {
    e = hipMemsetAsync(s->seed, 0, nb * sizeof(uint32_t), s->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(s->tsi, tsi.data(), nb * sizeof(int32_t), hipMemcpyHostToDevice, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    if (e != hipSuccess) rc = hip_fail(e, "hs_sim_create");
  }
  if (rc != HS_OK) {
    std::string keep = g_err;
    hs_sim_free(s);
    g_err = keep;
    return rc;
  }
  *out = s;
  return HS_OK;
}

int hs_sim_advance(hs_sim_t s, int32_t n_steps, double* tau_cmd, double* q_meas, double* torso, int32_t* n_contacts,
                   double* normal_force) {
  if (!s || n_steps < 0) return fail(HS_E_ARG, "hs_sim_advance: bad argument");
  if (n_steps == 0) return HS_OK;
  const hs_topo& t = s->model->host;
  const size_t rows = (size_t)s->B * n_steps;
  const size_t bytes[5] = {rows * t.nmj * sizeof(double), rows * t.nmj * sizeof(double), rows * 3 * sizeof(double),
                           rows * sizeof(int32_t), rows * sizeof(double)};
  void* host[5] = {tau_cmd, q_meas, torso, n_contacts, normal_force};
  hipError_t e = hipSetDevice(s->dev);
  if (e == hipSuccess && (size_t)n_steps > s->out_steps) {
    for (void*& p : s->out) {
      (void)hipFree(p);
      p = nullptr;
    }
    s->out_steps = 0;
    for (int i = 0; i < 5 && e == hipSuccess; i++) e = hipMalloc(&s->out[i], bytes[i]);
    if (e == hipSuccess) s->out_steps = (size_t)n_steps;
  }
  if (e != hipSuccess) return hip_fail(e, "hs_sim_advance");
  hs_sim_args a;
  memset(&a, 0, sizeof(a));
  a.n_rollouts = s->B;
  a.n_steps = n_steps;
  a.n_t = s->n_t;
  a.params = s->params;
  a.body = (double*)s->body;
  a.seed = (uint32_t*)s->seed;
  a.tsi = (int32_t*)s->tsi;
  a.q_tab = (const double*)s->q;
  a.dq_tab = (const double*)s->dq;
  a.tau_tab = (const double*)s->tau;
  a.tau_cmd = tau_cmd ? (double*)s->out[0] : nullptr;
  a.q_meas = q_meas ? (double*)s->out[1] : nullptr;
  a.torso = torso ? (double*)s->out[2] : nullptr;
  a.n_contacts = n_contacts ? (int32_t*)s->out[3] : nullptr;
  a.normal_force = normal_force ? (double*)s->out[4] : nullptr;
  a.stream = s->stream;
  int rc = hs_sim_step(s->model, &a);
  if (rc != HS_OK) return rc;
  for (int i = 0; i < 5 && e == hipSuccess; i++)
    if (host[i]) e = hipMemcpyAsync(host[i], s->out[i], bytes[i], hipMemcpyDeviceToHost, s->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  if (e != hipSuccess) return hip_fail(e, "hs_sim_advance");
  return HS_OK;
}

int hs_sim_get_state(hs_sim_t s, double* body, int32_t* tsi) {
  if (!s) return fail(HS_E_ARG, "null sim");
  const hs_topo& t = s->model->host;
  hipError_t e = hipSetDevice(s->dev);
  if (e == hipSuccess && body)
    e = hipMemcpyAsync(body, s->body, (size_t)s->B * t.n * HS_SIM_BODY_STRIDE * sizeof(double), hipMemcpyDeviceToHost,
                       s->stream);
  if (e == hipSuccess && tsi)
    e = hipMemcpyAsync(tsi, s->tsi, (size_t)s->B * sizeof(int32_t), hipMemcpyDeviceToHost, s->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
  if (e != hipSuccess) return hip_fail(e, "hs_sim_get_state");
  return HS_OK;
}

}  // extern "C"

// ---- batch handle sharded over the devices of one process -------------------------------------
struct hs_batch_s {
  struct shard {
    int dev = 0;
    int32_t id0 = 0, count = 0;  // contiguous rollout range (hslabs_amd/dist.py shard)
    hipStream_t stream = nullptr;
    hs_gait_params* params = nullptr;
    void *q = nullptr, *tau = nullptr, *cf = nullptr, *x = nullptr, *work_cot = nullptr;
    uint32_t* flags = nullptr;
    uint64_t* best_key = nullptr;
  };
  hs_model_t model = nullptr;
  int32_t B = 0, H = 0, n_t = 0, precision = HS_PREC_F64;
  bool have_params = false, ran = false;
  std::vector<shard> shards;
};

namespace {

// restores the caller's current device when a batch call returns
struct device_guard {
  int cur = 0;
  bool ok = false;
  device_guard() { ok = hipGetDevice(&cur) == hipSuccess; }
  ~device_guard() {
    if (ok) (void)hipSetDevice(cur);
  }
};

void batch_release(hs_batch_s* b) {
  for (auto& sh : b->shards) {
    if (hipSetDevice(sh.dev) != hipSuccess) continue;
    for (void* p : {(void*)sh.params, sh.q, sh.tau, sh.cf, sh.x, sh.work_cot, (void*)sh.flags, (void*)sh.best_key})
      if (p) (void)hipFree(p);
    if (sh.stream) (void)hipStreamDestroy(sh.stream);
  }
  b->shards.clear();
}

}  // namespace

extern "C" {

int hs_batch_create(hs_model_t m, int32_t B, int32_t H, int32_t n_t, int32_t precision, uint32_t mask,
                    hs_batch_t* out) {
  if (!m || !out) return fail(HS_E_ARG, "null argument");
  *out = nullptr;
  if (B <= 0 || H <= 0 || n_t <= 0) return fail(HS_E_ARG, "empty batch");
  if (precision != HS_PREC_F64 && precision != HS_PREC_F32) return fail(HS_E_ARG, "unknown precision");
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDeviceCount");
  std::vector<int> devs;
  for (int d = 0; d < 32; d++)
    if (mask & (1u << d)) {
      if (d >= ndev || d >= HS_MAX_DEVICES) return fail(HS_E_DEVICE, "device_mask names a missing device");
      devs.push_back(d);
    }
  if (devs.empty()) return fail(HS_E_ARG, "empty device_mask");
  device_guard guard;
  auto* b = new hs_batch_s;
  b->model = m;
  b->B = B;
  b->H = H;
  b->n_t = n_t;
  b->precision = precision;
  const hs_topo& t = m->host;
  const size_t w = precision == HS_PREC_F32 ? sizeof(float) : sizeof(double);
  const int n = (int)devs.size();
  const int32_t base = B / n, rem = B % n;
  for (int r = 0; r < n; r++) {
    hs_batch_s::shard sh;
    sh.dev = devs[r];
    sh.count = base + (r < rem ? 1 : 0);
    sh.id0 = r * base + std::min<int32_t>(r, rem);
    b->shards.push_back(sh);
  }
  for (auto& sh : b->shards) {
    const size_t rows = (size_t)std::max(sh.count, 1) * H;
    e = hipSetDevice(sh.dev);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&sh.stream, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipMalloc(&sh.params, (size_t)std::max(sh.count, 1) * sizeof(hs_gait_params));
    if (e == hipSuccess) e = hipMalloc(&sh.q, rows * t.cfg * w);
    if (e == hipSuccess) e = hipMalloc(&sh.tau, rows * t.nmj * w);
    if (e == hipSuccess) e = hipMalloc(&sh.cf, rows * 3 * t.nf * w);
    if (e == hipSuccess) e = hipMalloc(&sh.x, rows * 6 * t.n * w);
    if (e == hipSuccess) e = hipMalloc(&sh.flags, rows * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&sh.work_cot, (size_t)std::max(sh.count, 1) * 2 * w);
    if (e == hipSuccess) e = hipMalloc(&sh.best_key, sizeof(uint64_t));
    if (e != hipSuccess) {
      batch_release(b);
      delete b;
      return hip_fail(e, "hs_batch_create");
    }
  }
  *out = b;
  return HS_OK;
}

int hs_batch_set_params(hs_batch_t b, const hs_gait_params* params) {
  if (!b || !params) return fail(HS_E_ARG, "null argument");
  device_guard guard;
  hipError_t e = hipSuccess;
  for (auto& sh : b->shards) {
    if (sh.count == 0) continue;
    e = hipSetDevice(sh.dev);
    if (e == hipSuccess)
      e = hipMemcpyAsync(sh.params, params + sh.id0, (size_t)sh.count * sizeof(hs_gait_params),
                         hipMemcpyHostToDevice, sh.stream);
    if (e != hipSuccess) return hip_fail(e, "hs_batch_set_params");
  }
  for (auto& sh : b->shards) {
    e = hipSetDevice(sh.dev);
    if (e == hipSuccess) e = hipStreamSynchronize(sh.stream);
    if (e != hipSuccess) return hip_fail(e, "hs_batch_set_params");
  }
  b->have_params = true;
  return HS_OK;
}

}  // extern "C"

namespace {

// hs_batch_run (host outputs) and hs_batch_run_device (device outputs, any device of the process:
// the copies go through unified addressing, peer-to-peer where the buffer is on another GPU)
int batch_run(hs_batch_t b, int32_t k0, int32_t ignore_reach, const hs_batch_outputs* out, bool device_out) {
  if (!b) return fail(HS_E_ARG, "null batch");
  if (!b->have_params) return fail(HS_E_ARG, "hs_batch_set_params not called");
  if (k0 < 0) return fail(HS_E_ARG, "k0 < 0");
  device_guard guard;
  const hs_topo& t = b->model->host;
  const size_t w = b->precision == HS_PREC_F32 ? sizeof(float) : sizeof(double);
  const uint64_t init = ~0ull;
  hipError_t e = hipSuccess;
  // launch every shard, then collect: the devices run concurrently
  for (auto& sh : b->shards) {
    if (sh.count == 0) continue;
    e = hipSetDevice(sh.dev);
    if (e == hipSuccess) e = hipMemcpyAsync(sh.best_key, &init, sizeof(init), hipMemcpyHostToDevice, sh.stream);
    if (e != hipSuccess) return hip_fail(e, "hs_batch_run");
    hs_run_args a;
    memset(&a, 0, sizeof(a));
    a.n_rollouts = sh.count;
    a.horizon = b->H;
    a.k0 = k0;
    a.n_t = b->n_t;
    a.ignore_reach = ignore_reach;
    a.params = sh.params;
    a.q = (out && out->q) ? (double*)sh.q : nullptr;
    a.tau = (double*)sh.tau;
    a.cf = (double*)sh.cf;
    a.x = (out && out->x) ? (double*)sh.x : nullptr;
    a.flags = sh.flags;
    a.work_cot = (double*)sh.work_cot;
    a.best_key = sh.best_key;
    a.rollout_id_base = sh.id0;
    a.stream = sh.stream;
    a.precision = b->precision;
    int rc = hs_run(b->model, &a);
    if (rc != HS_OK) return rc;
  }
  for (auto& sh : b->shards) {
    if (sh.count == 0) continue;
    e = hipSetDevice(sh.dev);
    const size_t rows = (size_t)sh.count * b->H, row0 = (size_t)sh.id0 * b->H;
    const hipMemcpyKind kind = device_out ? hipMemcpyDefault : hipMemcpyDeviceToHost;
    auto copy = [&](void* host, const void* dev, size_t per_row, size_t elem, size_t host_row0) {
      if (e == hipSuccess && host)
        e = hipMemcpyAsync((char*)host + host_row0 * per_row * elem, dev, rows * per_row * elem, kind, sh.stream);
    };
    if (out) {
      copy(out->q, sh.q, t.cfg, w, row0);
      copy(out->tau, sh.tau, t.nmj, w, row0);
      copy(out->cf, sh.cf, 3 * t.nf, w, row0);
      copy(out->x, sh.x, 6 * t.n, w, row0);
      copy(out->flags, sh.flags, 1, sizeof(uint32_t), row0);
    }
    if (device_out && out) {  // work / cot: the columns of work_cot [B][2], strided copies
      for (int col = 0; col < 2; col++) {
        void* dst = col == 0 ? (void*)out->work : (void*)out->cot;
        if (e == hipSuccess && dst)
          e = hipMemcpy2DAsync((char*)dst + (size_t)sh.id0 * w, w, (const char*)sh.work_cot + col * w, 2 * w, w,
                               (size_t)sh.count, hipMemcpyDefault, sh.stream);
      }
    }
    if (e == hipSuccess) e = hipStreamSynchronize(sh.stream);
    if (e == hipSuccess && !device_out && out && (out->work || out->cot)) {
      std::vector<char> wc((size_t)sh.count * 2 * w);
      e = hipMemcpy(wc.data(), sh.work_cot, wc.size(), hipMemcpyDeviceToHost);
      for (int32_t i = 0; e == hipSuccess && i < sh.count; i++) {
        double wk, ct;
        if (w == sizeof(float)) {
          wk = ((const float*)wc.data())[2 * i];
          ct = ((const float*)wc.data())[2 * i + 1];
        } else {
          wk = ((const double*)wc.data())[2 * i];
          ct = ((const double*)wc.data())[2 * i + 1];
        }
        const size_t gi = (size_t)sh.id0 + i;
        if (w == sizeof(float)) {
          if (out->work) ((float*)out->work)[gi] = (float)wk;
          if (out->cot) ((float*)out->cot)[gi] = (float)ct;
        } else {
          if (out->work) out->work[gi] = wk;
          if (out->cot) out->cot[gi] = ct;
        }
      }
    }
    if (e != hipSuccess) return hip_fail(e, "hs_batch_run");
  }
  b->ran = true;
  return HS_OK;
}

int local_best(hs_batch_t b, uint64_t* best) {
  if (!b) return fail(HS_E_ARG, "null batch");
  if (!b->ran) return fail(HS_E_ARG, "hs_batch_run not called");
  device_guard guard;
  *best = ~0ull;
  for (auto& sh : b->shards) {
    if (sh.count == 0) continue;
    uint64_t k = ~0ull;
    hipError_t e = hipSetDevice(sh.dev);
    if (e == hipSuccess) e = hipMemcpy(&k, sh.best_key, sizeof(k), hipMemcpyDeviceToHost);
    if (e != hipSuccess) return hip_fail(e, "hs_select_best");
    *best = std::min(*best, k);
  }
  return HS_OK;
}

}  // namespace

extern "C" {

int hs_batch_run(hs_batch_t b, int32_t k0, int32_t ignore_reach, const hs_batch_outputs* out) {
  return batch_run(b, k0, ignore_reach, out, false);
}

int hs_batch_run_device(hs_batch_t b, int32_t k0, int32_t ignore_reach, const hs_batch_outputs* out) {
  return batch_run(b, k0, ignore_reach, out, true);
}

int hs_select_best(hs_batch_t b, float* cot, int64_t* rollout_id) {
  uint64_t best = ~0ull;
  int rc = local_best(b, &best);
  if (rc != HS_OK) return rc;
  hs_best_key_decode(best, cot, rollout_id);
  return HS_OK;
}

int hs_select_best_comm(hs_batch_t b, hs_comm_t comm, float* cot, int64_t* rollout_id) {
  if (!comm) return fail(HS_E_ARG, "null comm");
  // the local minimum, or the error that prevents it; either way this rank then takes part in the
  // all-reduce (contributing UINT64_MAX on an error), so its peers are never left waiting in it
  uint64_t best = ~0ull;
  int rc = (cot && rollout_id) ? local_best(b, &best) : fail(HS_E_ARG, "null cot or rollout_id");
  if (rc == HS_OK)
    for (auto& sh : b->shards)
      if (sh.dev != hs::comm_device(comm)) {
        rc = fail(HS_E_ARG, "the batch runs on a device the comm does not");
        best = ~0ull;
      }
  if (rc != HS_OK) best = ~0ull;  // local_best may have failed after a partial minimum
  std::string err = rc != HS_OK ? std::string(hs_last_error()) : std::string();
  device_guard guard;
  hipStream_t st = nullptr;  // the comm device's null stream: the reduce does not use the batch's key
  uint64_t* key = hs::comm_scratch(comm);
  hipError_t e = hipSetDevice(hs::comm_device(comm));
  if (e == hipSuccess) e = hipMemcpyAsync(key, &best, sizeof(best), hipMemcpyHostToDevice, st);
  if (e != hipSuccess) return hip_fail(e, "hs_select_best_comm");
  int rr = hs::comm_reduce_min(comm, key, st);
  if (rr != HS_OK) return rr;
  e = hipMemcpyAsync(&best, key, sizeof(best), hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e != hipSuccess) return hip_fail(e, "hs_select_best_comm");
  if (rc != HS_OK) return fail(rc, err);
  hs_best_key_decode(best, cot, rollout_id);
  return HS_OK;
}

uint64_t* hs_batch_best_key_device(hs_batch_t b, int32_t i) {
  if (!b || i < 0 || i >= (int32_t)b->shards.size()) {
    fail(HS_E_ARG, "no such device in the batch");
    return nullptr;
  }
  return b->shards[i].best_key;
}

void hs_batch_free(hs_batch_t b) {
  if (!b) return;
  device_guard guard;
  batch_release(b);
  delete b;
}

}  // extern "C"
