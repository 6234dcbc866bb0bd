// hs_config.hip -- the per-configuration kinematics of the kinematicmodel API (model.h:96-137) for
// batches of configurations on gfx950: forward kinematics (recompute_modelnodes) and the limb
// inverse kinematics (set_jvalues_with_lik). These are the model.h / core.h entry points every
// caller outside periodic binds (player.cpp:69, 122, 354; ghost.cpp:53-54; periodic.cpp:89-90).
//
// Built with -ffp-contract=off (hslabs_amd/build.py): every product rounds like the reference's
// affine::mult (matrix.cpp:78-97), so the only differences from the CPU restatement are ULPs of
// the device sin / cos / atan2 / acos.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "hs_internal.h"
#include "hs_math.h"

namespace {

using namespace hsd;

constexpr int WAVE = 64;

__device__ inline A34 unity34() {
  A34 A;
#pragma unroll
  for (int i = 0; i < 12; i++) A.m[i] = (i % 4 == 0) ? 1.0 : 0.0;  // columns 0..2 of I, zero translation
  return A;
}

__device__ inline void store34(double* o, const A34& A) {
#pragma unroll
  for (int i = 0; i < 12; i++) o[i] = A.m[i];
}

// kinematicmodel::recompute_modelnodes (model.cpp:314-318): lane = (configuration, node), the
// node's A_ground by walking its chain from the root in modelnode::recompute_A_ground's order
// (model.cpp:183-201): a jointed node's J_A_ground = A_parent J_A_parent (modeljoint::
// compute_A_ground, model.cpp:65-67), then * transformation(values) * A_pj_body.
__global__ __launch_bounds__(WAVE) void hs_fk_kernel(const hs_topo* __restrict__ T, int32_t n_cfg,
                                                     const double* __restrict__ config, int32_t stride,
                                                     double* __restrict__ a_ground, double* __restrict__ a_joint) {
  const int n = T->n;
  const int64_t g = (int64_t)blockIdx.x * WAVE + threadIdx.x;
  if (g >= (int64_t)n_cfg * n) return;
  const int64_t b = g / n;
  const int p = (int)(g % n);
  const double* q = config + b * stride;
  int chain[HS_NMAX], len = 0;
  for (int a = p; a >= 0 && len < HS_NMAX; a = T->node[a].parent) chain[len++] = a;
  A34 A = unity34(), J = unity34();
  bool jointed = false;
  for (int k = len - 1; k >= 0; k--) {
    const hs_node& nd = T->node[chain[k]];
    jointed = nd.jtype == HS_J_FREE || nd.jtype == HS_J_HINGE;
    if (jointed) {
      J = mul(A, load34(nd.J_A_parent));
      const A34 E = (nd.jtype == HS_J_FREE) ? free_joint(q) : hinge_joint(q[6 + nd.hinge]);
      A = mul(mul(J, E), load34(nd.A_pj_body));
    } else {
      A = mul(A, load34(nd.A_pj_body));
    }
  }
  store34(a_ground + g * 12, A);
  if (a_joint) {
    if (!jointed)
#pragma unroll
      for (int i = 0; i < 12; i++) J.m[i] = 0.0;
    store34(a_joint + g * 12, J);
  }
}

// kinematicmodel::set_jvalues_with_lik (model.cpp:354-359): the torso's six values from rec, the
// limbs' parents' frames from the recomputed torso (the chain from the root to a limb's parent is
// jointless, so no limb value enters), then liksolver::place_limbs (lik.cpp:89-99) in lik order:
// poslimb (lik.cpp:341-347) and the closed-form limb solver (lik.cpp:151-223, bend = true).
// Lane = configuration. status: HS_FLAG_UNREACH when a target was clamped (ignore_reach), and
// HS_FLAG_LIK_FAILED when one was out of reach without it (the reference prints and exits,
// lik.cpp:321-330; the row then holds the solver's NaN angles).
__global__ __launch_bounds__(WAVE) void hs_lik_kernel(const hs_topo* __restrict__ T, int32_t n_cfg,
                                                      const double* __restrict__ rec, int32_t ignore_reach,
                                                      double* __restrict__ config, uint32_t* __restrict__ status) {
  const int64_t b = (int64_t)blockIdx.x * WAVE + threadIdx.x;
  if (b >= n_cfg) return;
  const int nl = T->n_limbs, cfg = T->cfg;
  const double* r = rec + b * (6 + 3 * nl);
  double* q = config + b * cfg;
  double q6[6];
  for (int i = 0; i < 6; i++) q6[i] = q[i] = r[i];
  const A34 A0 = mul(mul(mul(unity34(), load34(T->node[0].J_A_parent)), free_joint(q6)), load34(T->node[0].A_pj_body));
  const double ls[3] = {T->ls[0], T->ls[1], T->ls[2]};
  uint32_t st = 0;
  for (int L = 0; L < nl; L++) {
    A34 A = A0;
    for (int k = 1; k < T->limb_chain_len[L]; k++) A = mul(A, load34(T->node[T->limb_chain[L][k]].A_pj_body));
    const int c = T->limb_child[L];
    const A34 Jinv = invert(mul(A, load34(T->node[c].J_A_parent)));
    double pl[3], ja[3];
    mulp(Jinv, r + 6 + 3 * L, pl);
    bool unreach = false, fail = false;
    limb_ik(T->lik_kind, ls, T->limb_ysign[L], pl, ja, ignore_reach != 0, unreach, fail);
    if (unreach) st |= HS_FLAG_UNREACH;
    if (fail) st |= HS_FLAG_LIK_FAILED;
    if (unreach || fail) st |= HS_LIK_LIMB_BIT(L);
    for (int kk = 0; kk < 3; kk++) q[6 + T->node[T->limb_node[L][kk]].hinge] = ja[kk];
  }
  if (status) status[b] = st;
}

}  // namespace

namespace hs {

int launch_fk(const hs_topo* d_topo, int32_t n_parts, int32_t n_cfg, const double* config, int32_t stride,
              double* a_ground, double* a_joint, void* stream) {
  const int64_t lanes = (int64_t)n_cfg * n_parts;
  if (lanes <= 0) return 0;
  hipLaunchKernelGGL(hs_fk_kernel, dim3((unsigned)((lanes + WAVE - 1) / WAVE)), dim3(WAVE), 0, (hipStream_t)stream,
                     d_topo, n_cfg, config, stride, a_ground, a_joint);
  return (int)hipGetLastError();
}

int launch_lik(const hs_topo* d_topo, int32_t n_cfg, const double* rec, int32_t ignore_reach, double* config,
               uint32_t* status, void* stream) {
  if (n_cfg <= 0) return 0;
  hipLaunchKernelGGL(hs_lik_kernel, dim3((unsigned)((n_cfg + WAVE - 1) / WAVE)), dim3(WAVE), 0, (hipStream_t)stream,
                     d_topo, n_cfg, rec, ignore_reach, config, status);
  return (int)hipGetLastError();
}

}  // namespace hs
