// hs_kernels.hip -- the batched control-loop hot path on gfx950 (MI355X).
//
// Two rollouts per wavefront (one 64-thread workgroup), 32 lanes each. Per
// rollout the half-wave
//   S  sets up the gait (pgssweeper::setup_pergen, pergen.cpp:453-507),
//   K  samples the trajectory: lane = (sample, limb) runs pergen set_rec
//      (pergen.cpp:225-239), the torso/body chain FK, limb IK (lik.cpp:151-223,
//      316-347) and the limb FK (model.cpp:183-201), and writes the dynamic
//      features of the parts it owns (dynrec.cpp:134-155) to LDS,
//   D  lane = part: 5-point finite differences (dynrec.cpp:175-224),
//   S1 lane = part, leaves -> root: particular solution of B0 x = f
//      (replaces the SparseQR solve of ftsolver.cpp:107-113 by the tree
//      back-substitution B0's block-triangular structure allows),
//   S3 the lexicographic least squares of ftsolver.cpp:185-236 in closed form
//      (one lane per contact + a 6x6 Schur complement); a conditioning guard
//      sends the step to the out-of-line Eigen-style FullPivLU/ColPivQR path
//      (tree-built null basis, Gram matrices in a global-memory workspace),
//   S4 motor torques, contact forces and positive work (periodic.cpp:261-343).
//
// LDS layout (PostL, round 5): a launch solves one step per rollout, so the
// five stencil samples keep only what that step reads -- pos/ust at t-2dt, t,
// t+2dt, q at t-dt..t+dt, joint/foot features at t -- and once D has consumed
// the stencil, the particular solution x, the closed-form blocks and the forces
// y live in its place: 5.1 KB per hexapod rollout, 10.1 KB per workgroup, 16
// workgroups per CU = 4 waves/SIMD for the fused step launch. A horizon H > 1
// is H steps (hs_capi.cpp), each recomputing its window on 30 lanes: the
// sampler is latency-bound, and a ring of five full samples (26 KB per
// rollout) measured half the throughput.
//
// The floating-point operation sequences follow oracle/hs_oracle.cpp's fast mode
// (built with -ffp-contract=off like the reference's x86-64 g++ -O2), but this
// file is compiled with -ffp-contract=fast-honor-pragmas (hslabs_amd/build.py):
// a*b+c is one FMA except where `#pragma clang fp contract(off)` says otherwise
// (work_add: work_over_period's two roundings), so results differ from the
// oracle by FMA roundings (<= 2.3e-12 on the per-joint torques,
// profiles/r01_parity_report.txt) and by ULPs of the device
// sin/cos/atan2/acos/asin.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cstdint>
#include <type_traits>

#ifndef HS_REAL_IS_FLOAT
#define HS_REAL_IS_FLOAT 0
#endif
#include "hs_internal.h"
#include "hs_math.h"

namespace {

using namespace hsd;

// Measured per precision (interleaved A/B, one box): fp32 configs[2] (spider, curved synthetic gaits)
// 370 -> 383 M steps/s with both; fp64 hexapod -5 % with the LDS copy (straight waves included),
// -0.8 % at K = 200 without the preload
#ifndef HS_CURVED_LDS
#define HS_CURVED_LDS HS_REAL_IS_FLOAT  // waves with a turning gait copy the setup record to LDS
#endif
#ifndef HS_PRELOAD
#define HS_PRELOAD (!HS_REAL_IS_FLOAT)  // straight_preload at wave start (0: inside the straight branch)
#endif
#ifndef HS_KTE_PRELOAD
// the IK table row loaded at wave start, before the gait is known to be straight (fp64: +1.3 % at
// K = 200 on hexapod); in the fp32 build inside the straight branch (spider, whose synthetic gaits are
// curved, 346 -> 370 M steps/s: the row's registers stay out of the turning path)
#define HS_KTE_PRELOAD (!HS_REAL_IS_FLOAT)
#endif

constexpr int WAVE = 64;
constexpr int HALF = 32;     // lanes per rollout: two rollouts per wavefront
constexpr int NS = 5;        // samples in the derivative stencil (periodic.cpp:192-202)
static_assert(NS * HS_LMAX <= HALF && 6 + HS_NMAX <= HALF && HS_KMAX <= HALF, "a rollout's lane maps exceed 32");
#ifndef HS_MIN_WAVES
// fp64: <= 168 VGPRs: the per-step launch (its general path called out of line, scratch frame) and the
// fixup launch; 4 waves/SIMD measured 7-10 % slower for the per-step launch (profiles/r05_s4_ab.txt)
#define HS_MIN_WAVES 3
#endif
#ifndef HS_MIN_WAVES_DEFER
// the fused step launch (FIX_DEFER: no general-path call) at 4 waves/SIMD: 128 VGPRs, its spills (52 B)
// all in the two-contact 6 x 6 system (tools/spill_lines.py; the entry's 108 B of round 5's first 4-wave
// build were removed, DESIGN.md section 4 Registers); the PostL layout's 10.1 KB of LDS per hexapod
// workgroup fits 16 workgroups/CU. Same box, interleaved: driver command 286.4 -> 296.2 M steps/s,
// K = 200 365.8 -> 381.9 M (profiles/r05_s4_ab.txt)
#define HS_MIN_WAVES_DEFER 4
#endif
#ifndef HS_MIN_WAVES_FORCES
#define HS_MIN_WAVES_FORCES 3  // solve_forces mode (hs_run_forces): the control step's LDS layout
#endif
#ifndef HS_MIN_WAVES_F32
#define HS_MIN_WAVES_F32 4  // fp32: 5.5 KB LDS per hexapod workgroup; the per-step and fixup launches 128 VGPRs
#endif
#ifndef HS_MIN_WAVES_F32_DEFER
// fp32's fused step launch at 5 waves/SIMD: 95 VGPRs, its 84 B of spills in the two-contact path only
// (tools/spill_lines.py --file hs_kernels_f32.hip); same box against 4: configs[2] 551 -> 606 M steps/s,
// hexapod fp32 K = 200 522 -> 570 M (profiles/r05_s11_ab.txt). At 6 (80 VGPRs) the entry and the outputs
// spill and it is no faster
#define HS_MIN_WAVES_F32_DEFER 5
#endif

// ---------------------------------------------------------------------------
// LDS layouts
// ---------------------------------------------------------------------------
// NM = part capacity of the LDS layouts (the host picks the smallest instantiation >= n,
// so LDS per rollout follows the model: hexapod 5.1 KB in the PostL layout).

// packed per-contact Schur entries: the lower triangle of S_c row by row (r (r + 1) / 2 + q), then h_c
constexpr int SCH_H = 21, SCH_N = 27;
__host__ __device__ constexpr int sch_lower(int r, int q) { return r * (r + 1) / 2 + q; }

struct SchurL {  // Schur complement of the contacts (all D_c invertible)
  real Dinv[HS_LMAX][9];
  real Ssum[SCH_N];  // sum over contacts of the packed [S_c | h_c] (summed across the contact lanes)
  real lam[6];
};

// augmented system K = D + rho A^T A (tier 2: a singular D_c); rare, so it lives in the rollout's
// global workspace (aliasing the general path's, which runs only after it declines)
struct AugL {
  real K[HS_KMAX * HS_KMAX], X[HS_KMAX * 7], St[36], lam[6], rdiag[HS_KMAX];
  int ok;
};

struct FastL {  // blocks of the closed-form solve
  real d0[HS_LMAX][3];  // A_c = [-I; [d0_c]x] (d0_c = torso COM - contact foot), kept as d0_c
  real D[HS_LMAX][9], g[HS_LMAX][3];
  int ok[HS_LMAX];
  SchurL sc;
};

struct WorkL {  // per-joint positive work of the step (outputs phase; FastL is dead by then)
  real wd[HS_NMAX];
};

// Workspace of the general path (k x k matrices, leading dimension LD >= k).
// SHARED: in LDS; otherwise (GenWS, the only instance) one global-memory slot per rollout.
// The path computes in double in both builds (greal): in single precision FullPivLU's rank test
// (pivots against eps * k) and ColPivQR's nonzero-pivot rule would decide on float rounding of the
// Grams -- a third of the fp32 hexapod steps sat within the HS_FLAG_NEAR_RANK band (round 4) --
// while the Grams of float inputs formed in double keep the exact rank structure (A^T A of a 6 x k A
// has rank <= 6 to double rounding), so the decisions are the fp64 path's. Only the inputs (positions,
// axes, the particular solution) are float there, and the forces are rounded to float once.
using greal = double;
// Eigen's epsilon / min and ftsolver.cpp:228-232's loop tolerance
constexpr greal gEps = DBL_EPSILON;
constexpr greal gTiny = DBL_MIN;
constexpr greal gRelTol = 1e-6;
// the conditioning test: the last pass's second-stage system with a kept ColPivQR pivot under gCondQR of
// its first (condition above 1e7): rounding-level changes of the inputs move the answer by more than the
// parity bound there (oracle NearTrack::ill)
constexpr greal gCondQR = 1e-7;
template <int LD_, bool SHARED_>
struct GenMats {
  static constexpr int LD = LD_;
  static constexpr bool SHARED = SHARED_;
  greal ntn0[LD * LD], lu[LD * LD], Ny[LD * LD], qr[LD * LD];
  greal n1[LD / 3][9];  // 3x3 diagonal blocks of the first-order Gram (column-major)
  greal ntx0[LD], ntx1[LD], y0[LD], b[LD], z[LD], c[LD], hc[LD], nu[LD], nd[LD];
  greal u1[3][LD];  // torso rows of N in the first-order stage (switch_torso_penalty other than (1,1))
  int coupled;     // u1 is set: the first-order Gram couples the contacts
  int8_t rowsT[LD], colsT[LD], q[LD], piv[LD], rycol[LD], cperm[LD];
};
using GenWS = GenMats<HS_KMAX, false>;
// A rollout's global solve workspace: tier 2's augmented system (fast_solve) or the Eigen-style path's
// matrices. Tier 2 runs first and the general path only after it declined; each writes every entry it
// reads before reading it, so the members never carry values from one to the other.
union SolveWS {
  GenWS gen;
  AugL aug;
};

template <int NM>
struct StencilL {  // fields only the finite differences read
  real pos[2][NM][3];  // t-2dt, t+2dt
  real ust[3][NM][3];  // t-2dt, t, t+2dt
};

template <int NM>
struct CentreL {  // fields read after D
  real pos[NM][3], jpos[NM][3], jz[NM][3], fpos[HS_LMAX][3];
  real q[3][6 + 3 * HS_LMAX];  // t-dt, t, t+dt (every hinge is a limb hinge: config_dim <= 24)
  int contact[HS_LMAX];
  int unreach[HS_LMAX];
};

struct ForceL {  // solve_forces by limbs (forces_solve): per limb S_l and e_l (a), per foot K_f and q_f
                 // (b); the dense fallback reuses the space from a[0][27] on (336 reals in all)
  real a[HS_LMAX][27];
  real b[HS_LMAX][27];
  real spare[12];
};

// What the control step keeps once D has consumed the stencil, in the stencil's place: D writes each
// part's f rows over that part's own stencil rows (every lane reads its rows before it writes, one
// wavefront in program order), the particular solution x overwrites f in place, the closed form's
// blocks and the forces y follow it (round 5: the layout that brought the step to 10 KB of LDS per
// workgroup, 4 waves per SIMD)
template <int NM>
struct PostL {
  union {
    real f[6 * NM];
    real x[6 * NM];
  };
  FastL fl;
  real y[HS_KMAX];
};

template <int NM, bool FORCES>
struct OneStore {
  union {
    StencilL<NM> sten;
    // forces-given-torques mode: its blocks (x and y stay in SolveL, which forces_solve reads with them)
    typename std::conditional<FORCES, ForceL, PostL<NM>>::type post;
  };
  CentreL<NM> c;
};

struct SetupL {
  real pos0[HS_LMAX][3];  // default foot positions, pergen order
  real ts[HS_LMAX], xs[HS_LMAX];
  real t_step, max_radius, v, dt;
  SC3 tsc;  // sin / cos of the configured torso angles (every sample of a straight gait)
};

// Straight, untransformed gaits (curvature 0, no record transform): the torso keeps its configured
// angles and moves by tv = t v along x (pergen.cpp:386-397 without the turn), and every body above
// the limbs is jointless (the loader's topology check), so the torso frame, the chain's body frames
// and each limb's hip joint frame (poslimb, lik.cpp:341-347) are a constant rotation with a
// translation affine in tv: A(t) = [R | c + tv u], u = column 0 of the torso's J_A_parent. The gait
// setup keeps them at tv = 0 (the products kin_sample forms, once per rollout instead of per sample):
// the hip frames whole, and for the torso and the chain bodies the features themselves -- a body's
// position A(t) com = (R com + c) + tv u, its rotation's skew part (constant) and its frame origin
// c + tv u -- so a sample adds tv u to two points.
// IK table entry (RolloutWS::ktab): the joint values of a limb at a sample; its unreachable-or-failed
// flag is a byte of RolloutWS::kbad (24 B entries in fp64: the table is written and read once per call)
constexpr int KT_W = 3;
// torso record row (RolloutWS::ktor), turning or transformed gaits: the torso's q6 (set_rec's position and
// Euler angles) and its frame A0 = J_A_parent free_joint(q6) A_pj_body at a sample
constexpr int KR_W = 18;
constexpr int BF_W = 9;  // a body's features at tv = 0: position R com + c, skew part of R (ust), origin c
struct KinFrames {
  real J0[HS_LMAX][12];                 // each limb's hip joint frame
  real own[HS_LMAX][HS_OWN_MAX][BF_W];  // the chain bodies each limb computes (hs_topo::limb_own)
  real torso[6];                        // the torso (node 0): position and ust (its joint frame is J_A_parent)
};
// the features of a body with frame A (node_features' pos and ust; the origin for a jointless body's jpos)
__device__ inline void store_body(const A34& A, const real* com, real* bf, int n) {
  real p[3];
  mulp(A, com, p);
  for (int i = 0; i < 3; i++) bf[i] = p[i];
  bf[3] = (A(2, 1) - A(1, 2)) / 2;
  bf[4] = (A(0, 2) - A(2, 0)) / 2;
  bf[5] = (A(1, 0) - A(0, 1)) / 2;
  if (n > 6)
    for (int i = 0; i < 3; i++) bf[6 + i] = A(i, 3);
}

template <int NM>
struct SolveXY {
  union {  // particular() overwrites each part's f with its x in place
    real f[6 * NM];
    real x[6 * NM];
  };
  real y[HS_KMAX];
};
struct SolveNone {};
template <int NM, bool FORCES>
struct SolveL {
  typename std::conditional<FORCES, SolveXY<NM>, SolveNone>::type xy;  // the control step keeps them in PostL
  int cfoot[HS_LMAX];
  uint32_t fch[HS_LMAX][2];  // hs_topo::foot_chain8, copied at the wave's start (the contact blocks' chains)
};
// The solve's LDS arrays as the phases see them (sv.f, sv.x, sv.y, sv.cfoot, sv.fch)
struct SolveRef {
  real* f;
  real* x;
  real* y;
  int* cfoot;
  uint32_t (*fch)[2];
};

template <int NM, bool FORCES>
struct Smem {
  OneStore<NM, FORCES> d;
  SolveL<NM, FORCES> sv;
#if HS_CURVED_LDS
  SetupL st;  // the setup pass's record, copied per step in waves with a curved gait
#endif
};

// Cross-lane exchange through LDS inside the single wave of a workgroup: an
// LDS-only workgroup fence (lgkmcnt, no vmcnt, so HBM stores stay in flight).
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}
// HS_FLAG_NEAR_RANK bands (include/hslabs.h; oracle/hs_oracle.cpp NearTrack): a decision whose value lies
// within kNearBand of its threshold (rel_error: within 10x of gRelTol; ColPivQR's squared column norms:
// within kNearBand^2) is flagged, since another rounding may take it the other way
constexpr real kNearBand = real(4);
// v is within `band` of threshold t (both positive; a NaN is not)
template <class T>
__device__ inline bool near_thr(T v, T t, T band) { return v >= t / band && v <= t * band; }

// The ABI's arrays are double*; in the fp32 build they hold floats.
__device__ inline real* outp(double* p) { return reinterpret_cast<real*>(p); }
__device__ inline const real* inp(const double* p) { return reinterpret_cast<const real*>(p); }

// The general path with a global workspace also needs its HBM stores performed.
template <class G>
__device__ inline void gsync() {
  if constexpr (G::SHARED) wave_sync();
  else __syncthreads();
}

#ifdef HS_STAMPS
// diagnostic build only: per-phase shader-clock stamps of the first 4096 rollouts
// (slots 16, 17: the constant 100 MHz clock at wave entry and exit, comparable across CUs)
__device__ unsigned long long g_stamps[4096][32];  // slots 24..31: hs_prep_kernel's
__device__ unsigned int g_stamp_base;  // row r holds block g_stamp_base + r (hs_debug_set_stamp_base)
#define STAMP(slot)                                                                                    \
  do {                                                                                                 \
    const unsigned r_ = blockIdx.x - g_stamp_base;                                                     \
    if (threadIdx.x == 0 && r_ < 4096u) g_stamps[r_][slot] = __builtin_amdgcn_s_memtime();             \
  } while (0)
#define RSTAMP(slot)                                                                                   \
  do {                                                                                                 \
    const unsigned r_ = blockIdx.x - g_stamp_base;                                                     \
    if (threadIdx.x == 0 && r_ < 4096u) g_stamps[r_][slot] = __builtin_amdgcn_s_memrealtime();         \
  } while (0)
#else
#define STAMP(slot) do {} while (0)
#define RSTAMP(slot) do {} while (0)
#endif

// HS_DBG = n (diagnostic variant builds only): intermediate value n of every part written to g_dbg[row][slot]
// by both step kernels (the limb-lane kernel's bitwise check, tests/test_gpu_limb.py)
#ifdef HS_DBG
__device__ double g_dbg[1 << 22];
__device__ inline int* dbg_rows() {
  __shared__ int r[8];
  return r;
}
#define DBG(slot, val, n)                                                        \
  do {                                                                           \
    if (HS_DBG == (n)) {                                                         \
      const int r_ = dbg_rows()[threadIdx.x / HALF];                             \
      if (r_ >= 0 && (size_t)r_ * 32 + (slot) < (1u << 22)) g_dbg[(size_t)r_ * 32 + (slot)] = (double)(val); \
    }                                                                            \
  } while (0)
#else
#define DBG(slot, val, n) do {} while (0)
#endif

// ballot over the 32 lanes of this rollout (bit l = sub-lane l)
__device__ inline uint32_t half_ballot(bool pred) {
  return (uint32_t)(__ballot(pred) >> (threadIdx.x & HALF));
}

__device__ inline A34 node_joint_parent(const hs_topo* T, int v) { return load34(T->node[v].J_A_parent); }
__device__ inline A34 node_pj(const hs_topo* T, int v) { return load34(T->node[v].A_pj_body); }

// ---------------------------------------------------------------------------
// Sample views. k = offset from the step's centre sample (-2..2).
// ---------------------------------------------------------------------------
template <int NM, bool FORCES>
struct OneWin {
  OneStore<NM, FORCES>* d;
  __device__ bool want_pos(int k) const { return (k & 1) == 0; }
  __device__ bool want_ust(int k) const { return (k & 1) == 0; }
  __device__ bool want_q(int k) const { return k >= -1 && k <= 1; }
  __device__ bool want_centre(int k) const { return k == 0; }
  __device__ real* pos(int k, int v) const { return k == 0 ? d->c.pos[v] : d->sten.pos[k > 0][v]; }
  __device__ real* ust(int k, int v) const { return d->sten.ust[(k + 2) >> 1][v]; }
  __device__ real* q(int k) const { return d->c.q[k + 1]; }
  __device__ real* jpos(int, int v) const { return d->c.jpos[v]; }
  __device__ real* jz(int, int v) const { return d->c.jz[v]; }
  __device__ real* fpos(int, int f) const { return d->c.fpos[f]; }
  __device__ int& contact(int, int f) const { return d->c.contact[f]; }
  __device__ int& unreach(int, int L) const { return d->c.unreach[L]; }
};

// gait parameters of one rollout in the working precision (hs_gait_params, pergen.h:137-146)
struct GaitR {
  real torso_pos[3], torso_angles[3];
  real step_duration, period, step_length, step_height, curvature, foot_shift;
  int foot_shift_type;
  int rec_xf;  // rec_transform_flag: the transform itself is read where it applies (gait_record)
};

__device__ inline GaitR load_gait(const hs_gait_params& p) {
  GaitR g;
  for (int i = 0; i < 3; i++) {
    g.torso_pos[i] = (real)p.torso_pos[i];
    g.torso_angles[i] = (real)p.torso_angles[i];
  }
  g.step_duration = (real)p.step_duration;
  g.period = (real)p.period;
  g.step_length = (real)p.step_length;
  g.step_height = (real)p.step_height;
  g.curvature = (real)p.curvature;
  g.foot_shift = (real)p.foot_shift;
  g.foot_shift_type = p.foot_shift_type;
  g.rec_xf = p.rec_transform_flag;
  return g;
}

// pergensetup::transform_rec (pergen.cpp:323-335) with rec_transform = affine_from_orientation(
// {rec_transl, rec_eas}) (set_rec_transform, pergen.cpp:316-320): the torso by transform_orientation
// (pergen.cpp:377-383: A1 = rec_transform A0, then its translation and Euler angles), the foot target
// by rec_transform.mult with w = 1
__device__ inline void transform_rec(const hs_gait_params& p, real* o0, real* o1, real* target) {
  const real tr[3] = {(real)p.rec_transl[0], (real)p.rec_transl[1], (real)p.rec_transl[2]};
  const A34 R = from_euler(tr, (real)p.rec_eas[0], (real)p.rec_eas[1], (real)p.rec_eas[2]);
  const A34 A1 = mul(R, from_euler(o0, o1[0], o1[1], o1[2]));
  o0[0] = A1(0, 3); o0[1] = A1(1, 3); o0[2] = A1(2, 3);
  euler_from(A1, o1);
  real t[3];
  mulp(R, target, t);
  target[0] = t[0]; target[1] = t[1]; target[2] = t[2];
}

// the straight gait's frame at tv = t v: [R | c + tv u] (KinFrames)
__device__ inline A34 frame_at(A34 A, const real* u, real tv) {
#pragma unroll
  for (int r = 0; r < 3; r++) A.at(r, 3) = fma(tv, u[r], A(r, 3));
  return A;
}
__device__ inline A34 load34r(const real* m) {
  A34 a;
#pragma unroll
  for (int i = 0; i < 12; i++) a.m[i] = m[i];
  return a;
}
__device__ inline void store34r(const A34& a, real* m) {
#pragma unroll
  for (int i = 0; i < 12; i++) m[i] = a.m[i];
}

// ---------------------------------------------------------------------------
// S: gait setup, lanes L < n_limbs (pergen.cpp:453-507, 30-51, 143-153)
// ---------------------------------------------------------------------------
// periodicgenerator::set_step_duration (pergen.cpp:30-51) for n limbs: the stepping fraction t_step and
// pergen index j's lift-off time ts and shift xs (the loop's entry k = j = jj + i jmax)
__device__ inline real step_fraction(const GaitR& g, int n) {
  const real f = g.step_duration;
  return f * (real(1) / 2 - real(1) / n) + real(1) / n;
}
__device__ inline void lift_off(int n, int j, real t_step, real& ts, real& xs) {
  const int jmax = n / 2;
  const int z = (jmax == 1) ? 1 : jmax - 1;
  const int i = j / jmax, jj = j % jmax;
  ts = jj * (real(1) / 2 - t_step) / z + real(i) / 2;
  xs = ts + t_step / 2 - real(1) / 2;
}

// the torso frame at the configured pose (orient_torso); tsc: sincos3 of the configured angles
__device__ inline A34 torso_frame(const hs_topo* T, const GaitR& g, const SC3& tsc) {
  const real q6[6] = {g.torso_pos[0], g.torso_pos[1], g.torso_pos[2],
                      g.torso_angles[0], g.torso_angles[1], g.torso_angles[2]};
  return mul(mul(node_joint_parent(T, 0), free_joint_sc(q6, tsc)), node_pj(T, 0));
}

// Limb L's part of the gait setup from the torso frame A0: the hip joint frame J0 (poslimb,
// lik.cpp:341-347) and the default foot position of its pergen index (get_limb_hip_pos, the foot
// shift, set_limb_poss; pergen.cpp:453-507). kf (optional): store the chain body frames this limb owns
// and its hip frame (KinFrames, the straight gaits' frames at tv = 0)
// The chain's products come precombined from the loader (hs_topo::limb_own_rel, limb_hip_rel): one product
// per frame, every load indexed by the limb alone
// A limb's setup constants (hs_topo::limb_*), loaded before the gait parameters they do not depend on
struct LimbPlan {
  A34 hip, own0;  // limb_hip_rel, limb_own_rel[0] (limb_own_n > 0)
  real ct[3], com0[3];
  int own_n, ysign;  // ysign: limb_ysign, read by the table rows' IK
};
__device__ __attribute__((always_inline)) inline LimbPlan load_plan(const hs_topo* T, int L) {
  LimbPlan p;
  p.own_n = T->limb_own_n[L];
  p.ysign = T->limb_ysign[L];
  p.hip = load34(T->limb_hip_rel[L]);
  p.own0 = load34(T->limb_own_rel[L][0]);
  for (int i = 0; i < 3; i++) {
    p.ct[i] = (real)T->limb_child_t[L][i];
    p.com0[i] = (real)T->limb_own_com[L][0][i];
  }
  return p;
}
__device__ __attribute__((always_inline)) inline void limb_setup(const hs_topo* T, const GaitR& g, const A34& A0, int L,
                                                                 const LimbPlan& pl, A34& J0, real* pos0,
                                                                 KinFrames* kf = nullptr) {
  if (kf)
    for (int m = 0; m < pl.own_n; m++) {
      real com[3];
      for (int i = 0; i < 3; i++) com[i] = m == 0 ? pl.com0[i] : (real)T->limb_own_com[L][m][i];
      store_body(mul(A0, m == 0 ? pl.own0 : load34(T->limb_own_rel[L][m])), com, kf->own[L][m], BF_W);
    }
  J0 = mul(A0, pl.hip);
  if (kf) store34r(J0, kf->J0[L]);
  // get_limb_hip_pos: the child's frame J0 Rz(0) pj_child (Rz(0) = I) at its translation
  real pos[3];
  mulp(J0, pl.ct, pos);
  if (g.foot_shift_type == 0) {                   // setup_foot_shift / shift_pos0
    real sh[3] = {real(0), g.foot_shift, real(0)}, ls[3];
    mulp(A0, sh, ls);
    if (L % 2) for (int i = 0; i < 3; i++) ls[i] *= -1;
    for (int i = 0; i < 3; i++) pos[i] += ls[i];
  } else if (g.foot_shift_type == 1) {
    real x = pos[0], y = pos[1];
    real f = g.foot_shift / sqrt(x * x + y * y);
    real d[3] = {x * f, y * f, real(0)};
    for (int i = 0; i < 3; i++) pos[i] += d[i];
  }
  pos0[0] = pos[0];
  pos0[1] = pos[1];
  pos0[2] = (real)T->rcap;  // set_limb_poss
}

// compute_max_radius's distance of one default foot position from the turning centre (0, 1 / curvature)
__device__ inline real turn_radius(const real* pos0, real curvature) {
  const real cy = real(1) / curvature;
  const real d0 = pos0[0] - real(0), d1 = pos0[1] - cy, d2 = pos0[2] - real(0);
  real s = 0;
  s += d0 * d0;
  s += d1 * d1;
  s += d2 * d2;
  return sqrt(s);
}

// The whole setup on a half-wave (hs_pergen_rec_kernel), lanes L < n_limbs: SetupL in LDS
__device__ __attribute__((always_inline)) inline void gait_setup(const hs_topo* T, const GaitR& g, int n_t, SetupL& st,
                                                                 int lane) {
  const int nl = T->n_limbs;
  const real t_step = step_fraction(g, nl);
  if (lane < nl) {
    const int L = lane;
    const SC3 tsc = sincos3(g.torso_angles[0], g.torso_angles[1], g.torso_angles[2]);
    if (L == 0) st.tsc = tsc;
    A34 J0;
    const int j = T->limb_pergen[L];
    limb_setup(T, g, torso_frame(T, g, tsc), L, load_plan(T, L), J0, st.pos0[j]);
    lift_off(nl, j, t_step, st.ts[j], st.xs[j]);
  }
  if (lane == 0) {
    st.t_step = t_step;
    st.v = g.step_length / g.period;  // pergensetup::set_TLh
    st.dt = g.period / n_t;           // record_trajectory
  }
  wave_sync();
  if (lane == 0) {  // compute_max_radius
    real mr = 0;
    if (g.curvature != 0)
      for (int j = 0; j < nl; j++) {
        const real rad = turn_radius(st.pos0[j], g.curvature);
        if (rad > mr) mr = rad;
      }
    st.max_radius = mr;
  }
  wave_sync();
}

// ---------------------------------------------------------------------------
// K: one (sample, limb) pair per lane
// ---------------------------------------------------------------------------
// pergen.cpp:143-153 step profiles: stepx(t) = (1 - cos(pi t)) / 2, stepz(t) = sin(pi t)^2, from one sincos
__device__ inline void step_profiles(real t, real& sx, real& sz) {
  real s, c;
  sincos(kPi * t, &s, &c);
  sx = (1 - c) / 2;
  sz = s * s;
}

// What the kinematics reads of one node, fetched in one batch of independent loads instead of
// one round trip per branch that consumes it (fetching earlier measured slower: the values
// stay live across the gait record and their waits land on its loads, vmcnt being in order).
struct NodeK {
  A34 Jp, pj;  // J_A_parent, A_pj_body
  real com[3], cap[3];
  int foot, hinge, owner;
};
__device__ __attribute__((always_inline)) inline NodeK load_nodek(const hs_topo* T, int v) {
  const hs_node& nd = T->node[v];
  NodeK r;
  r.Jp = load34(nd.J_A_parent);
  r.pj = load34(nd.A_pj_body);
#pragma unroll
  for (int i = 0; i < 3; i++) {
    r.com[i] = (real)nd.com[i];
    r.cap[i] = (real)nd.cap[i];
  }
  r.foot = nd.foot;
  r.hinge = nd.hinge;
  r.owner = nd.owner_limb;
  return r;
}

template <class W>
__device__ __attribute__((always_inline)) inline void node_features(const hs_topo* T, int v, const NodeK& nd, const A34& A, const A34* J, const W& w, int k) {
  if (w.want_pos(k)) {
    real p[3];
    mulp(A, nd.com, p);
    real* P = w.pos(k, v);
    for (int i = 0; i < 3; i++) P[i] = p[i];
  }
  if (w.want_ust(k)) {
    real* U = w.ust(k, v);
    U[0] = (A(2, 1) - A(1, 2)) / 2;
    U[1] = (A(0, 2) - A(2, 0)) / 2;
    U[2] = (A(1, 0) - A(0, 1)) / 2;
  }
  if (w.want_centre(k)) {
    real* Jp = w.jpos(k, v);
    real* Jz = w.jz(k, v);
    for (int i = 0; i < 3; i++) Jp[i] = J ? (*J)(i, 3) : A(i, 3);
    for (int i = 0; i < 3; i++) Jz[i] = J ? (*J)(i, 2) : real(0);
    if (nd.foot >= 0) {
      real fp[3];
      mulp(A, nd.cap, fp);
      real* F = w.fpos(k, nd.foot);
      for (int i = 0; i < 3; i++) F[i] = fp[i];
      w.contact(k, nd.foot) = fp[2] < (real)(T->rcap + 1e-4);
    }
  }
}

// periodicgenerator::limb_positions' step of one pergen index at time t (pergen.cpp:82-94): the
// forward shift dx and lift dz of its foot, t_lift / xs its lift-off entries, t_step the stepping fraction
__device__ inline void limb_step(const GaitR& g, real t, real t_lift, real xs, real t_step, real& dx, real& dz) {
  const real tt = t / g.period;
  const int t_int = int(tt);
  const real t_frac = tt - t_int;
  real stepf;
  if (t_frac < t_lift) stepf = 0;
  else if (t_frac < t_lift + t_step) stepf = (t_frac - t_lift) / t_step;
  else stepf = 1;
  real sx, sz;
  step_profiles(stepf, sx, sz);
  dx = (t_int + xs + sx) * g.step_length;
  dz = sz * g.step_height;
}

// What gait_record reads of the gait setup for one pergen index j: the rollout's entries and j's
// (from the setup record, limb_rec, or from the preparation pass's registers)
struct LimbRec {
  real v, t_step, max_radius, ts, xs, pos0[3];
  SC3 tsc;
};
__device__ __attribute__((always_inline)) inline LimbRec limb_rec(const SetupL& st, int j) {
  LimbRec r;
  r.v = st.v;
  r.t_step = st.t_step;
  r.max_radius = st.max_radius;
  r.ts = st.ts[j];
  r.xs = st.xs[j];
  for (int i = 0; i < 3; i++) r.pos0[i] = st.pos0[j][i];
  r.tsc = st.tsc;
  return r;
}

// pergensetup::set_rec at time t for lik limb L (pergen.cpp:225-239): torso position o0 and Euler
// angles o1 (turn_torso, pergen.cpp:386-397; `turned` when the torso frame was rotated), and the
// limb's foot target (limb_positions of its pergen index, pergen.cpp:82-94, 160-183); st: that
// index's LimbRec
// STRAIGHT: the caller knows curvature == 0 (a wave of straight gaits), so the turning code is left
// out and the record is one basic block the scheduler can interleave with the torso FK
template <bool STRAIGHT = false>
__device__ __attribute__((always_inline)) inline void gait_record(const GaitR& g, const hs_gait_params& gp,
                                                                  const LimbRec& st, real t, real* o0, real* o1,
                                                                  bool& turned, real* target) {
  o0[0] = g.torso_pos[0]; o0[1] = g.torso_pos[1]; o0[2] = g.torso_pos[2];
  o1[0] = g.torso_angles[0]; o1[1] = g.torso_angles[1]; o1[2] = g.torso_angles[2];
  real tv = t * st.v;
  turned = false;
  real psi = 0;
  if (!STRAIGHT && g.curvature != 0) {
    int s = (g.curvature > 0) ? 1 : -1;
    psi = s * tv / st.max_radius;
    turned = psi != 0;
  }
  if (!turned) {
    o0[0] += tv;
  } else {
    real rc = real(1) / g.curvature;
    real sp, cp;
    sincos(psi, &sp, &cp);
    real tp[3] = {rc * sp, rc * (1 - cp), 0};
    A34 At = from_euler_sc(tp, SC3{real(0), real(1), real(0), real(1), sp, cp});  // sin 0 = 0, cos 0 = 1
    A34 A0 = from_euler_sc(o0, st.tsc);
    A34 A1 = mul(At, A0);
    o0[0] = A1(0, 3); o0[1] = A1(1, 3); o0[2] = A1(2, 3);
    euler_from(A1, o1);
  }
  // periodicgenerator::limb_positions for this limb's pergen index (pergen.cpp:82-94)
  real dx, dz;
  limb_step(g, t, st.ts, st.xs, st.t_step, dx, dz);
  real dy = 0;
  if (!STRAIGHT && g.curvature != 0) {  // turn_position (pergen.cpp:160-183)
    int s = (g.curvature > 0) ? 1 : -1;
    real x0 = st.pos0[0], y0 = st.pos0[1];
    real rc = real(1) / g.curvature;
    real rx = x0, ry = y0 - rc;
    real r = sqrt(rx * rx + ry * ry);
    real alpha = atan2(ry, rx);
    real beta = -s * dx / st.max_radius;
    real gamma = alpha - beta / 2;
    real sb = 2 * sin(beta / 2);
    real sg, cg;
    sincos(gamma, &sg, &cg);
    dx = r * sg * sb;
    dy += -r * cg * sb;
  }
  target[0] = dx + st.pos0[0];
  target[1] = dy + st.pos0[1];
  target[2] = dz + st.pos0[2];
  if (!STRAIGHT && g.rec_xf) {  // set_rec's last step (pergen.cpp:238)
    transform_rec(gp, o0, o1, target);
    turned = true;  // the torso angles are no longer the configured ones
  }
}

// sample times t_i = dt + dt + ... (i terms, periodic.cpp:171-181), stored once per rollout by the
// call's preparation pass (the same additions in the same order) for the samples its steps read:
// t_tab[r] = t_(lo + r), r < ttab_n
__device__ inline real sample_time_sum(real dt, int isample) {
  real t = 0;
  for (int i = 0; i < isample; i++) t += dt;
  return t;
}
__device__ inline real sample_time(const SetupL& st, const real* t_tab, int isample, int lo, int ttab_n) {
  const int r = isample - lo;
  if (t_tab && r >= 0 && r < ttab_n) return t_tab[r];
  return sample_time_sum(st.dt, isample);
}

// limb FK with the new joint values (compute_dynrecs' recompute_modelnodes, model.cpp:183-201) from the
// hip joint frame J, and the dynamic features of the links (dynrec.cpp:134-155), on the limb's
// precombined plan (hs_topo::link): per link k the hinge frame H = J_k Rz(q_k) (mul_hinge), its body frame
// A_k = H pj_k seen through the products the features need -- pos = H (pj_k com), the rotation skew of
// A_k (ust) from H's and pj_k's rotations, the foot H (pj_2 cap) -- and the next joint frame J_(k+1) =
// H (pj_k Jp_(k+1)): one 3 x 4 product per link where the node-by-node form takes two
// (sq, cq: sin and cos of the joint values ja)
template <class W>
__device__ __attribute__((always_inline)) inline void limb_fk(const hs_topo* T, int L, const A34& J, const real* ja,
                                                              const real* sq, const real* cq, bool wq, const W& w,
                                                              int k) {
  const int lv[3] = {T->limb_node[L][0], T->limb_node[L][1], T->limb_node[L][2]};
  A34 Jv = J, H;
#pragma unroll
  for (int kk = 0; kk < 3; kk++) {  // limb_child, its first kid, that one's first kid
    const hs_link& lk = T->link[L][kk];
    if (kk > 0) Jv = mul(H, load34(lk.P));
    H = mul_hinge(Jv, cq[kk], sq[kk]);
    if (wq) w.q(k)[6 + lk.hinge] = ja[kk];
    const int v = lv[kk];
    if (w.want_pos(k)) {
      const real c[3] = {(real)lk.com[0], (real)lk.com[1], (real)lk.com[2]};
      real p[3];
      mulp(H, c, p);
      real* P = w.pos(k, v);
      for (int i = 0; i < 3; i++) P[i] = p[i];
      if (k == 0) DBG(v, p[0], 1);
      if (k == -2) DBG(v, p[0], 12);
    }
    if (w.want_ust(k)) {  // (A(2,1) - A(1,2)) / 2 etc. of A = H pj: (r, c) = sum_m H(r, m) pj(m, c)
      real R[9];
#pragma unroll
      for (int i = 0; i < 9; i++) R[i] = (real)lk.Rpj[i];
      auto a_rc = [&](int r, int c) { return H(r, 0) * R[c * 3 + 0] + H(r, 1) * R[c * 3 + 1] + H(r, 2) * R[c * 3 + 2]; };
      real* U = w.ust(k, v);
      U[0] = (a_rc(2, 1) - a_rc(1, 2)) / 2;
      U[1] = (a_rc(0, 2) - a_rc(2, 0)) / 2;
      U[2] = (a_rc(1, 0) - a_rc(0, 1)) / 2;
      if (k == 0) DBG(v, U[0], 5);
      if (k == -2) DBG(v, U[0], 9);
      if (k == 2) DBG(v, U[0], 11);
    }
    if (w.want_centre(k)) {
      real* Jp = w.jpos(k, v);
      real* Jz = w.jz(k, v);
      for (int i = 0; i < 3; i++) Jp[i] = Jv(i, 3);
      for (int i = 0; i < 3; i++) Jz[i] = Jv(i, 2);
      if (lk.foot >= 0) {
        const real c[3] = {(real)lk.cap[0], (real)lk.cap[1], (real)lk.cap[2]};
        real fp[3];
        mulp(H, c, fp);
        real* F = w.fpos(k, lk.foot);
        for (int i = 0; i < 3; i++) F[i] = fp[i];
        if (k == 0) DBG(24 + lk.foot, fp[2], 25);
        w.contact(k, lk.foot) = fp[2] < (real)(T->rcap + 1e-4);
      }
    }
  }
}

template <bool STRAIGHT, class W>
__device__ __attribute__((always_inline)) inline void kin_sample(const hs_topo* T, const GaitR& g, const hs_gait_params& gp,
                                                                 const SetupL& st, int isample, int L, bool ignore_reach,
                                                                 const W& w, int k, const real* t_tab, int tlo,
                                                                 int ttab_n) {
  const int j = T->limb_pergen[L];
  const int ysign = T->limb_ysign[L];
  const int clen = T->limb_chain_len[L];
  const int lv[3] = {T->limb_node[L][0], T->limb_node[L][1], T->limb_node[L][2]};
  const real t = sample_time(st, t_tab, isample, tlo, ttab_n);  // t accumulates dt (periodic.cpp:171-181)
  real o0[3], o1[3], target[3];
  bool turned;
  gait_record<STRAIGHT>(g, gp, limb_rec(st, j), t, o0, o1, turned, target);
  STAMP(20);
  // set_jvalues_with_lik: torso + body chain FK, then limb IK (model.cpp:354-359, lik.cpp:89-99)
  real q6[6] = {o0[0], o0[1], o0[2], o1[0], o1[1], o1[2]};
  const A34 F = (!STRAIGHT && turned) ? free_joint(q6) : free_joint_sc(q6, st.tsc);  // straight: angles fixed
  const NodeK n0 = load_nodek(T, 0);  // the torso
  A34 A0 = mul(mul(n0.Jp, F), n0.pj);
  const bool wq = w.want_q(k);
  if (L == 0) {
    if (wq) for (int i = 0; i < 6; i++) w.q(k)[i] = q6[i];
    node_features(T, 0, n0, A0, &n0.Jp, w, k);  // torso joint frame J = I * J_A_parent
  }
  A34 A = A0;
  for (int kk = 1; kk < clen; kk++) {
    const int v = T->limb_chain[L][kk];
    const NodeK nc = load_nodek(T, v);
    A = mul(A, nc.pj);
    if (nc.owner == L) node_features(T, v, nc, A, nullptr, w, k);
  }
  NodeK nk = load_nodek(T, lv[0]);  // limb_child
  A34 J = mul(A, nk.Jp);  // poslimb (lik.cpp:341-347)
  A34 Jinv = invert(J);
  STAMP(21);
  real pl[3], ja[3];
  mulp(Jinv, target, pl);
  bool unreach = false, fail = false;
  const real ls[3] = {(real)T->ls[0], (real)T->ls[1], (real)T->ls[2]};
  limb_ik(T->lik_kind, ls, ysign, pl, ja, ignore_reach, unreach, fail);
  if (w.want_centre(k)) w.unreach(k, L) = (unreach || fail) ? 1 : 0;
  STAMP(22);
  real sq[3], cq[3];
#pragma unroll
  for (int kk = 0; kk < 3; kk++) sincos_k(ja[kk], &sq[kk], &cq[kk]);
  limb_fk(T, L, J, ja, sq, cq, wq, w, k);
}

// set_rec's foot target of limb L at time t and the limb IK from the hip frame J (kin_sample's
// sequence from the gait record on); bad = unreachable (ignore_reach) or failed
// the limb IK of limb L for a foot target, from its hip joint frame J (lik.cpp:341-347, 151-223)
// (kind, ls, ysign: the model's IK variant, link lengths and the limb's side, read by the caller)
__device__ __attribute__((always_inline)) inline void hip_ik_k(const A34& J, const real* target, int kind,
                                                               const real* ls, int ysign, bool ignore_reach, real* ja,
                                                               bool& bad) {
  const A34 Jinv = invert(J);
  real pl[3];
  mulp(Jinv, target, pl);
  bool unreach = false, fail = false;
  limb_ik(kind, ls, ysign, pl, ja, ignore_reach, unreach, fail);
  bad = unreach || fail;
}
__device__ __attribute__((always_inline)) inline void hip_ik(const hs_topo* T, int L, const A34& J, const real* target,
                                                             bool ignore_reach, real* ja, bool& bad) {
  const real ls[3] = {(real)T->ls[0], (real)T->ls[1], (real)T->ls[2]};
  hip_ik_k(J, target, T->lik_kind, ls, T->limb_ysign[L], ignore_reach, ja, bad);
}

__device__ __attribute__((always_inline)) inline void straight_ik(const hs_topo* T, const GaitR& g,
                                                                  const hs_gait_params& gp, const SetupL& st, real t,
                                                                  int L, const A34& J, bool ignore_reach, real* ja,
                                                                  bool& bad) {
  real o0[3], o1[3], target[3];
  bool turned;
  gait_record<true>(g, gp, limb_rec(st, T->limb_pergen[L]), t, o0, o1, turned, target);
  hip_ik(T, L, J, target, ignore_reach, ja, bad);
}

// What kin_sample_straight loads that no computed value feeds (the sample time, the torso speed, the
// hip frame, the IK table row): loaded at the wave's start, before the gait record decides the path,
// so these latencies overlap the gait parameters' instead of following them
struct StraightPre {
  real t, v;
  A34 J0;
  real kte[KT_W];
  bool bad;
  real own0[BF_W];  // the limb's first chain body (limb_own_n > 0), and the torso (lane L = 0)
  real tor[6];
};
// (kt: the table, whose row r holds sample lo + r)
__device__ __attribute__((always_inline)) inline StraightPre straight_preload(const SetupL& st, const real* t_tab,
                                                                             const KinFrames& kf, const real* kt,
                                                                             const uint8_t* kb, int isample, int lo,
                                                                             int ttab_n, int L) {
  StraightPre p;
  p.t = sample_time(st, t_tab, isample, lo, ttab_n);
  p.v = st.v;
  p.J0 = load34r(kf.J0[L]);
#pragma unroll
  for (int i = 0; i < BF_W; i++) p.own0[i] = kf.own[L][0][i];
#pragma unroll
  for (int i = 0; i < 6; i++) p.tor[i] = kf.torso[i];
  if (kt) {
    const real* e = kt + ((size_t)(isample - lo) * HS_LMAX + L) * KT_W;
#pragma unroll
    for (int i = 0; i < KT_W; i++) p.kte[i] = e[i];
    p.bad = kb[(isample - lo) * HS_LMAX + L] != 0;
  }
  return p;
}

// kin_sample for a straight, untransformed gait: the frames from kf (the gait setup's), the joint
// values from the IK table kt (null: solved here, with the table kernel's straight_ik); pre: the
// preloaded values (straight_preload)
template <class W>
__device__ __attribute__((always_inline)) inline void kin_sample_straight(
    const hs_topo* T, const hs_gait_params& gp, const SetupL& st, int isample, int L,
    bool ignore_reach, const W& w, int k, const StraightPre& pre, const KinFrames& kf, const real* kt,
    const uint8_t* kb, int ktab_lo) {
  const real t = pre.t;
  const real tv = t * pre.v;  // gait_record's torso advance
  const bool wq = w.want_q(k);
  const NodeK n0 = load_nodek(T, 0);
  const real u[3] = {n0.Jp(0, 0), n0.Jp(1, 0), n0.Jp(2, 0)};
  A34 J = pre.J0;
#if HS_KTE_PRELOAD
  const real* kte = pre.kte;
  const bool kbad = pre.bad;
#else
  real kte[KT_W];  // the table row, loaded once the gait is known to be straight
  bool kbad = false;
  if (kt) {
    const real* e = kt + ((size_t)(isample - ktab_lo) * HS_LMAX + L) * KT_W;
#pragma unroll
    for (int i = 0; i < KT_W; i++) kte[i] = e[i];
    kbad = kb[(isample - ktab_lo) * HS_LMAX + L] != 0;
  }
#endif
  for (int m = 0; m < T->limb_own_n[L]; m++) {  // the chain bodies this limb computes (never a foot)
    const int v = T->limb_own[L][m];
    real bf[BF_W];
#pragma unroll
    for (int i = 0; i < BF_W; i++) bf[i] = m == 0 ? pre.own0[i] : kf.own[L][m][i];
    if (w.want_pos(k)) {
      real* P = w.pos(k, v);
      for (int i = 0; i < 3; i++) P[i] = fma(tv, u[i], bf[i]);
    }
    if (w.want_ust(k)) {
      real* U = w.ust(k, v);
      for (int i = 0; i < 3; i++) U[i] = bf[3 + i];
    }
    if (w.want_centre(k)) {  // a body without a joint: J = its frame, no axis (node_features with J = null)
      real* Jp = w.jpos(k, v);
      real* Jz = w.jz(k, v);
      for (int i = 0; i < 3; i++) Jp[i] = fma(tv, u[i], bf[6 + i]);
      for (int i = 0; i < 3; i++) Jz[i] = real(0);
    }
  }
  if (L == 0) {
    if (wq) {
      real* q = w.q(k);
      q[0] = (real)gp.torso_pos[0] + tv;
      q[1] = (real)gp.torso_pos[1];
      q[2] = (real)gp.torso_pos[2];
      for (int i = 0; i < 3; i++) q[3 + i] = (real)gp.torso_angles[i];
    }
    // node_features of the torso: its joint frame J = I * J_A_parent, not a foot
    if (w.want_pos(k)) {
      real* P = w.pos(k, 0);
      for (int i = 0; i < 3; i++) P[i] = fma(tv, u[i], pre.tor[i]);
    }
    if (w.want_ust(k)) {
      real* U = w.ust(k, 0);
      for (int i = 0; i < 3; i++) U[i] = pre.tor[3 + i];
    }
    if (w.want_centre(k)) {
      real* Jp = w.jpos(k, 0);
      real* Jz = w.jz(k, 0);
      for (int i = 0; i < 3; i++) Jp[i] = n0.Jp(i, 3);
      for (int i = 0; i < 3; i++) Jz[i] = n0.Jp(i, 2);
    }
  }
  STAMP(20);
  J = frame_at(J, u, tv);
  real ja[3], sq[3], cq[3];
  bool bad;
  if (kt) {
#pragma unroll
    for (int kk = 0; kk < 3; kk++) {
      ja[kk] = kte[kk];
      sincos_k(ja[kk], &sq[kk], &cq[kk]);
    }
    bad = kbad;
    STAMP(21);
  } else {
    straight_ik(T, load_gait(gp), gp, st, t, L, J, ignore_reach, ja, bad);  // untabulated calls only
#pragma unroll
    for (int kk = 0; kk < 3; kk++) sincos_k(ja[kk], &sq[kk], &cq[kk]);
  }
  if (w.want_centre(k)) w.unreach(k, L) = bad ? 1 : 0;
  STAMP(22);
  limb_fk(T, L, J, ja, sq, cq, wq, w, k);
}

// kin_sample for a turning or transformed gait from the preparation pass's rows: the torso's q6 and frame
// at the sample (tor, a RolloutWS::ktor row: the gait record and torso FK kin_sample forms) and the limb's
// joint values (kte, its ktab entry); the chain bodies and the hip frame from the torso frame as in
// kin_sample, then the limb FK
template <class W>
__device__ __attribute__((always_inline)) inline void kin_sample_tab(const hs_topo* T, int L, const W& w, int k,
                                                                     const real* tor, const real* kte, bool bad) {
  const int clen = T->limb_chain_len[L];
  const bool wq = w.want_q(k);
  const NodeK n0 = load_nodek(T, 0);
  const A34 A0 = load34r(tor + 6);
  if (L == 0) {
    if (wq) for (int i = 0; i < 6; i++) w.q(k)[i] = tor[i];
    node_features(T, 0, n0, A0, &n0.Jp, w, k);  // torso joint frame J = I * J_A_parent
  }
  A34 A = A0;
  for (int kk = 1; kk < clen; kk++) {
    const int v = T->limb_chain[L][kk];
    const NodeK nc = load_nodek(T, v);
    A = mul(A, nc.pj);
    if (nc.owner == L) node_features(T, v, nc, A, nullptr, w, k);
  }
  const A34 J = mul(A, node_joint_parent(T, T->limb_child[L]));  // poslimb (lik.cpp:341-347)
  STAMP(20);
  real ja[3], sq[3], cq[3];
#pragma unroll
  for (int kk = 0; kk < 3; kk++) {
    ja[kk] = kte[kk];
    sincos_k(ja[kk], &sq[kk], &cq[kk]);
  }
  if (w.want_centre(k)) w.unreach(k, L) = bad ? 1 : 0;
  STAMP(21);
  STAMP(22);
  limb_fk(T, L, J, ja, sq, cq, wq, w, k);
}

// ---------------------------------------------------------------------------
// D: finite differences at the centre sample, lane = part (dynrec.cpp:175-224)
// ---------------------------------------------------------------------------
// SYNC = false: the caller's next phase reads only this lane's rows (particular_sub's first stage)
template <bool SYNC = true, class W, class SV>
// dt: the sample spacing (SetupL::dt, read once at the wave's start)
__device__ __attribute__((always_inline)) inline void dynamics(const hs_topo* T, real dt, SV& sv, const W& w, int lane) {
  const int n = T->n;
  const int i = lane;
  const real m = (real)T->mass[lane < n ? lane : 0];
  real mr[3], amr[3];
  if (lane < n) {
    const real inv = real(1) / (2 * dt);
    const real *Pp = w.pos(2, i), *P0 = w.pos(0, i), *Pm = w.pos(-2, i);
    const real *Up = w.ust(2, i), *U0 = w.ust(0, i), *Um = w.ust(-2, i);
    real vp[3], vm[3], wp[3], wm[3];
    for (int j = 0; j < 3; j++) {
      vp[j] = Pp[j] - P0[j];
      vp[j] *= inv;
      vm[j] = P0[j] - Pm[j];
      vm[j] *= inv;
      real mp = vp[j] * m, mm = vm[j] * m;
      mr[j] = mp - mm;
      mr[j] *= inv;
      wp[j] = Up[j] - U0[j];
      wp[j] *= inv;
      wm[j] = U0[j] - Um[j];
      wm[j] *= inv;
    }
    // ang_mom = R (I (R^T w)) (compute_ang_mom, dynrec.cpp:205-216) with I the identity: every
    // inertia is ODE's default dMass (dBodyCreate; the reference sets no other, dynrec.cpp:62-68),
    // so R R^T w = w exactly in exact arithmetic and the two rotations (9 + 9 products and the
    // t +- dt rotations kept for them, 3.2 KB of LDS per hexapod rollout) are skipped: this rounds
    // ang_mom once instead of through R^T and R (a few ULPs of |w|, ~1e-15 relative)
    for (int j = 0; j < 3; j++) {
      amr[j] = wp[j] - wm[j];
      amr[j] *= inv;
    }
  }
  // PostL: f overlays the stencil, and lane i's f rows can land on another lane's stencil rows
  // (pos[1][n + i - NM]). Every lane's reads above happen before any lane's writes below only because
  // the wavefront executes them in program order: this wavefront-scope fence keeps the compiler from
  // moving a write above another lane's read; it emits no instruction
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane < n) {
    for (int j = 0; j < 3; j++) {
      sv.f[3 * i + j] = mr[j];
      sv.f[3 * (n + i) + j] = amr[j];
    }
    sv.f[3 * i + 2] += m * real(1);  // gravity, g = 1 (dynrec.cpp:291-295)
    DBG(i, mr[0], 2);
    DBG(i, amr[0], 10);
    DBG(i, sv.f[3 * i + 1], 13);
    DBG(i, sv.f[3 * i + 2], 14);
    DBG(i, sv.f[3 * (n + i) + 1], 16);
  }
  if (SYNC) wave_sync();
}

// ---------------------------------------------------------------------------
// S1: tree back-substitution B0 x = f, level by level (deepest first)
// ---------------------------------------------------------------------------
template <class W, class SV>
__device__ __attribute__((always_inline)) inline void particular(const hs_topo* T, SV& sv, const W& w, int lane) {
  const int n = T->n;
  // this lane's node links, loaded once (independent loads, not one L2 round trip per level)
  const hs_node& nd = T->node[lane < n ? lane : 0];
  const int depth = lane < n ? nd.depth : -1, parent = nd.parent, nk = nd.nkids;
  int kids[HS_CMAX];
#pragma unroll
  for (int kk = 0; kk < HS_CMAX; kk++) kids[kk] = nd.kids[kk];
  for (int level = T->max_depth; level >= 0; level--) {
    if (depth == level) {
      const int i = lane;
      const real* Pi = w.pos(0, i);
      real F[3], Tq[3];
      for (int j = 0; j < 3; j++) { F[j] = sv.f[3 * i + j]; Tq[j] = sv.f[3 * (n + i) + j]; }
#pragma unroll
      for (int kk = 0; kk < HS_CMAX; kk++) {
        if (kk >= nk) break;
        const int c = kids[kk];
        const real* Jc = w.jpos(0, c);
        for (int j = 0; j < 3; j++) F[j] += sv.x[3 * c + j];
        real r[3];
        for (int j = 0; j < 3; j++) r[j] = Pi[j] - Jc[j];
        const real* Fc = &sv.x[3 * c];
        Tq[0] -= r[1] * Fc[2] - r[2] * Fc[1];
        Tq[1] -= r[2] * Fc[0] - r[0] * Fc[2];
        Tq[2] -= r[0] * Fc[1] - r[1] * Fc[0];
        for (int j = 0; j < 3; j++) Tq[j] += sv.x[3 * (n + c) + j];
      }
      for (int j = 0; j < 3; j++) sv.x[3 * i + j] = F[j];
      if (parent >= 0) {
        const real* Ji = w.jpos(0, i);
        real r[3];
        for (int j = 0; j < 3; j++) r[j] = Ji[j] - Pi[j];
        Tq[0] -= r[1] * F[2] - r[2] * F[1];
        Tq[1] -= r[2] * F[0] - r[0] * F[2];
        Tq[2] -= r[0] * F[1] - r[1] * F[0];
      }
      for (int j = 0; j < 3; j++) sv.x[3 * (n + i) + j] = Tq[j];
    }
    wave_sync();
  }
}

// S1 as subtree sums: the recursion above, unrolled. With the torso COM p0 as the
// origin, x_i = (F_i, V_i - (J_i - p0) x F_i) (the root: (F_0, V_0)), where over i's subtree
// F_i = sum f_k and V_i = sum (t_k + (P_k - p0) x f_k) -- the same equations (B0 x = f), summed in
// another order. The node table is in preorder, so every subtree is the contiguous range
// [i, i + size_i): a non-root node sums its range directly (a body segment's, the longest, is 7
// parts on the hexapod), the root adds its children's sums; three wavefront syncs instead of one
// per tree level.
template <class W, class SV>
__device__ __attribute__((always_inline)) inline void particular_sub(const hs_topo* T, SV& sv, const W& w, int lane) {
  const int n = T->n;
  const bool on = lane < n;
  const hs_node& nd = T->node[on ? lane : 0];
  const int sz = on ? nd.size : 0, parent = nd.parent, nk = nd.nkids;
  int kids[HS_CMAX];
#pragma unroll
  for (int kk = 0; kk < HS_CMAX; kk++) kids[kk] = nd.kids[kk];
  const real* P0 = w.pos(0, 0);
  const real o[3] = {P0[0], P0[1], P0[2]};
  if (lane == 0) DBG(31, o[0], 15);
  if (lane == 0) DBG(30, o[1], 15);
  if (on) {  // g_i = (f_i, t_i + (P_i - p0) x f_i), the torque part in place
    const int i = lane;
    const real* Pi = w.pos(0, i);
    real f[3], t[3], d[3];
    for (int j = 0; j < 3; j++) { f[j] = sv.f[3 * i + j]; t[j] = sv.f[3 * (n + i) + j]; d[j] = Pi[j] - o[j]; }
    t[0] += d[1] * f[2] - d[2] * f[1];
    t[1] += d[2] * f[0] - d[0] * f[2];
    t[2] += d[0] * f[1] - d[1] * f[0];
    for (int j = 0; j < 3; j++) sv.x[3 * (n + i) + j] = t[j];
    DBG(i, t[0], 3);
  }
  wave_sync();
  real F[3] = {0, 0, 0}, V[3] = {0, 0, 0};
  const bool leafward = on && parent >= 0;
  if (leafward) {  // the subtree's range, in preorder
    for (int m = 0; m < sz; m++) {
      const int kx = lane + m;
      for (int j = 0; j < 3; j++) { F[j] += sv.x[3 * kx + j]; V[j] += sv.x[3 * (n + kx) + j]; }
    }
  }
  if (leafward)  // every lane's reads above precede these writes (one wavefront, in order)
    for (int j = 0; j < 3; j++) { sv.x[3 * lane + j] = F[j]; sv.x[3 * (n + lane) + j] = V[j]; }
  wave_sync();
  if (on && parent < 0) {  // the root: its own g plus its children's sums
    for (int j = 0; j < 3; j++) { F[j] = sv.x[3 * lane + j]; V[j] = sv.x[3 * (n + lane) + j]; }
#pragma unroll
    for (int kk = 0; kk < HS_CMAX; kk++) {
      if (kk >= nk) break;
      const int c = kids[kk];
      for (int j = 0; j < 3; j++) { F[j] += sv.x[3 * c + j]; V[j] += sv.x[3 * (n + c) + j]; }
    }
  }
  if (on) {  // x_i; the root's reads above precede these writes
    real d[3] = {0, 0, 0};
    if (parent >= 0) {
      const real* Ji = w.jpos(0, lane);
      for (int j = 0; j < 3; j++) d[j] = Ji[j] - o[j];
    }
    V[0] -= d[1] * F[2] - d[2] * F[1];
    V[1] -= d[2] * F[0] - d[0] * F[2];
    V[2] -= d[0] * F[1] - d[1] * F[0];
    for (int j = 0; j < 3; j++) { sv.x[3 * lane + j] = F[j]; sv.x[3 * (n + lane) + j] = V[j]; }
    DBG(lane, V[0], 4);
    DBG(lane, F[0], 18);
    DBG(lane, d[0], 17);
  }
  // no trailing sync: the caller's contact list ends with one before x is read across lanes
}

// Tree-basis null-space entry for a torque row: (arm x e_jj)[row], arm = ref - fpos
template <class T>
__device__ inline T cross_e(const T* d, int jj, int row) {
  // d x e0 = (0, d2, -d1); d x e1 = (-d2, 0, d0); d x e2 = (d1, -d0, 0)
  if (jj == 0) return row == 0 ? T(0) : (row == 1 ? d[2] : -d[1]);
  if (jj == 1) return row == 0 ? -d[2] : (row == 1 ? T(0) : d[0]);
  return row == 0 ? d[1] : (row == 1 ? -d[0] : T(0));
}

// ===========================================================================
// General path (rare: the fast solve's guard tripped): Gram matrices of the
// tree-built null basis and the Eigen 3.3 FullPivLU / ColPivHouseholderQR rank
// loop of ftsolver.cpp:185-303 (oracle/hs_oracle.cpp tree mode, same
// operation order). G is the LDS or the global workspace (GenMats).
// ===========================================================================

// S2: Gram matrices of the masked, penalty-weighted null basis (ftsolver.cpp:185-207)
template <class W, class SV, class G>
__device__ void build_grams(const hs_topo* T, const SV& sv, G& g, const W& w, int k, int lane) {
  constexpr int LD = G::LD;
  const int n = T->n;
  const int nc = k / 3;
  const real* P0 = w.pos(0, 0);
  // switch_torso_penalty (ftsolver.cpp:262-273): the torso rows of mask0 (bit 0: force rows, bit 1:
  // torque rows; the reference's (1,1) is 3). Rows outside mask0 belong to mask1 with weight 1, ahead
  // of the joint torque rows in row order (set_penal_mask1, ftsolver.cpp:291-303)
  const int tm = T->torso_mask;
  const bool t_force0 = (tm & 1) != 0, t_torque0 = (tm & 2) != 0;
  // zeroth order: rows {0,1,2} = -I, rows {3n..3n+2} = (pos_0 - fpos) x e_jj, weight 1
  for (int e = lane; e < k * k; e += HALF) {
    int ci = e % k, cj = e / k;
    const real* fa = w.fpos(0, sv.cfoot[ci / 3]);
    const real* fb = w.fpos(0, sv.cfoot[cj / 3]);
    int ja = ci % 3, jb = cj % 3;
    greal da[3], db[3];
    for (int r = 0; r < 3; r++) { da[r] = P0[r] - fa[r]; db[r] = P0[r] - fb[r]; }
    greal s = greal(0);
    if (t_force0)
      for (int r = 0; r < 3; r++) {
        greal na = (r == ja) ? greal(-1) : greal(0), nb = (r == jb) ? greal(-1) : greal(0);
        s = s + na * nb;
      }
    if (t_torque0)
      for (int r = 0; r < 3; r++) s = s + cross_e(da, ja, r) * cross_e(db, jb, r);
    g.ntn0[ci + cj * LD] = s;
  }
  if (lane < k) {
    int ci = lane, ja = ci % 3;
    const real* fa = w.fpos(0, sv.cfoot[ci / 3]);
    greal da[3];
    for (int r = 0; r < 3; r++) da[r] = P0[r] - fa[r];
    greal s = greal(0);
    if (t_force0)
      for (int r = 0; r < 3; r++) s = s + ((r == ja) ? greal(-1) : greal(0)) * (greal(1) * sv.x[r]);
    if (t_torque0)
      for (int r = 0; r < 3; r++) s = s + cross_e(da, ja, r) * (greal(1) * sv.x[3 * n + r]);
    g.ntx0[ci] = s;
    // the first-order torso rows (one group at most: mask0 is never empty), for the coupling terms
    for (int r = 0; r < 3; r++)
      g.u1[r][ci] = !t_force0 ? ((r == ja) ? greal(-1) : greal(0)) : (!t_torque0 ? cross_e(da, ja, r) : greal(0));
  }
  if (lane == 0) g.coupled = tm != 3;
  // first order: torque rows of the non-root ancestors of each contact foot,
  // weighted by the joint-axis components (set_action_penalties, ftsolver.cpp:239-246),
  // after the torso rows mask0 leaves out
  for (int e = lane; e < nc * 9 + k; e += HALF) {
    bool is_vec = e >= nc * 9;
    int cc = is_vec ? (e - nc * 9) / 3 : e / 9;
    int a_col = is_vec ? (e - nc * 9) % 3 : (e % 9) % 3;
    int b_col = is_vec ? 0 : (e % 9) / 3;
    int foot = T->footis[sv.cfoot[cc]];
    const real* fp = w.fpos(0, sv.cfoot[cc]);
    // ancestors of foot below the root, in ascending part order (top of the chain first)
    int chain[HS_NMAX], len = 0;
    for (int a = foot; a >= 0 && T->node[a].parent >= 0; a = T->node[a].parent) chain[len++] = a;
    greal s = greal(0);
    if (!t_force0)  // torso force rows 0..2: N = -I per contact, x1 = x
      for (int r = 0; r < 3; r++) {
        greal na = (r == a_col) ? greal(-1) : greal(0);
        greal nb = is_vec ? greal(1) * sv.x[r] : ((r == b_col) ? greal(-1) : greal(0));
        s = s + na * nb;
      }
    if (!t_torque0) {  // torso torque rows 3n..3n+2: N = [pos_0 - fpos]x
      greal d0[3];
      for (int r = 0; r < 3; r++) d0[r] = P0[r] - fp[r];
      for (int r = 0; r < 3; r++) {
        greal na = cross_e(d0, a_col, r);
        greal nb = is_vec ? greal(1) * sv.x[3 * n + r] : cross_e(d0, b_col, r);
        s = s + na * nb;
      }
    }
    for (int t = len - 1; t >= 0; t--) {
      int a = chain[t];
      const real* Ja = w.jpos(0, a);
      const real* Za = w.jz(0, a);
      greal d[3];
      for (int r = 0; r < 3; r++) d[r] = Ja[r] - fp[r];
      for (int r = 0; r < 3; r++) {
        greal wz = Za[r];
        greal na = wz * cross_e(d, a_col, r);
        greal nb = is_vec ? wz * sv.x[3 * n + 3 * a + r] : wz * cross_e(d, b_col, r);
        s = s + na * nb;
      }
    }
    if (is_vec) g.ntx1[3 * cc + a_col] = s;
    else g.n1[cc][b_col * 3 + a_col] = s;
  }
  gsync<G>();
}

// first-order Gram entry (block diagonal)
template <class G>
__device__ inline greal ntn1_at(const G& g, int i, int j) {
  return (i / 3 == j / 3) ? g.n1[i / 3][(j % 3) * 3 + (i % 3)] : greal(0);
}
// with torso rows in the first order (g.coupled): the off-block entries are their products, summed
// in row order (the blocks already start with them)
template <class G>
__device__ inline greal ntn1_full(const G& g, int i, int j) {
  if (i / 3 == j / 3) return g.n1[i / 3][(j % 3) * 3 + (i % 3)];
  greal s = greal(0);
  for (int r = 0; r < 3; r++) s = s + g.u1[r][i] * g.u1[r][j];
  return s;
}

// half-wave argmax with first-index tie break
__device__ inline void wave_argmax(greal& v, int& idx) {
  for (int off = HALF / 2; off >= 1; off >>= 1) {
    greal ov = __shfl_xor(v, off);
    int oi = __shfl_xor(idx, off);
    if (ov > v || (ov == v && oi < idx)) { v = ov; idx = oi; }
  }
}

struct LUInfo {
  int nz;          // nonzero pivots
  greal maxpivot;
};

// Eigen FullPivLU::computeInPlace of ntn0 into g.lu (k x k)
template <class G>
__device__ LUInfo fullpiv_lu(G& g, int k, int lane) {
  constexpr int LD = G::LD;
  for (int e = lane; e < k * k; e += HALF) {
    int i = e % k, j = e / k;
    g.lu[i + j * LD] = g.ntn0[i + j * LD];
  }
  gsync<G>();
  LUInfo info{k, greal(0)};
  for (int p = 0; p < k; p++) {
    const int m = k - p;
    greal best = greal(-1);
    int bidx = 1 << 30;
    for (int e = lane; e < m * m; e += HALF) {
      greal a = fabs(g.lu[(p + e % m) + (p + e / m) * LD]);
      if (a > best || (a == best && e < bidx)) { best = a; bidx = e; }
    }
    wave_argmax(best, bidx);
    if (best == 0) {
      info.nz = p;
      for (int i = p + lane; i < k; i += HALF) { g.rowsT[i] = i; g.colsT[i] = i; }
      break;
    }
    if (best > info.maxpivot) info.maxpivot = best;
    const int bi = p + bidx % m, bj = p + bidx / m;
    if (lane == 0) { g.rowsT[p] = bi; g.colsT[p] = bj; }
    if (bi != p && lane < k) {
      greal t = g.lu[p + lane * LD];
      g.lu[p + lane * LD] = g.lu[bi + lane * LD];
      g.lu[bi + lane * LD] = t;
    }
    gsync<G>();
    if (bj != p && lane < k) {
      greal t = g.lu[lane + p * LD];
      g.lu[lane + p * LD] = g.lu[lane + bj * LD];
      g.lu[lane + bj * LD] = t;
    }
    gsync<G>();
    if (p < k - 1) {
      greal piv = g.lu[p + p * LD];
      if (lane > p && lane < k) g.lu[lane + p * LD] /= piv;
      gsync<G>();
      const int mm = k - p - 1;
      for (int e = lane; e < mm * mm; e += HALF) {
        int i = p + 1 + e % mm, j = p + 1 + e / mm;
        g.lu[i + j * LD] -= g.lu[i + p * LD] * g.lu[p + j * LD];
      }
      gsync<G>();
    }
  }
  if (lane == 0) {
    for (int i = 0; i < k; i++) g.q[i] = i;
    for (int p = 0; p < k; p++) { int t = g.q[p]; g.q[p] = g.q[g.colsT[p]]; g.q[g.colsT[p]] = t; }
  }
  gsync<G>();
  return info;
}

// any nonzero pivot within kNearBand of the rank threshold maxpivot * thr (the decisions lu_rank takes)
template <class G>
__device__ inline bool lu_near(const G& g, const LUInfo& info, greal thr) {
  constexpr int LD = G::LD;
  const greal pt = fabs(info.maxpivot) * thr;
  bool nr = false;
  for (int i = 0; i < info.nz; i++) nr |= near_thr(fabs(g.lu[i + i * LD]), pt, greal(kNearBand));
  return nr;
}

template <class G>
__device__ inline int lu_rank(const G& g, const LUInfo& info, greal thr) {
  constexpr int LD = G::LD;
  greal pt = fabs(info.maxpivot) * thr;
  int r = 0;
  for (int i = 0; i < info.nz; i++) r += fabs(g.lu[i + i * LD]) > pt;
  return r;
}

// column-oriented upper-triangular solve of vec[0..r) against U (ld LD), all lanes
template <class G>
__device__ void upper_solve_shared(const greal* U, greal* vec, int r, int lane) {
  constexpr int LD = G::LD;
  for (int i = r - 1; i >= 0; i--) {
    greal ci = vec[i];
    if (ci != 0) {
      greal xi = ci / U[i + i * LD];
      if (lane < i) vec[lane] -= xi * U[lane + i * LD];
      if (lane == i) vec[i] = xi;
    }
    gsync<G>();
  }
}

// FullPivLU::solve(-ntx0) -> g.y0
template <class G>
__device__ void lu_solve(G& g, const LUInfo& info, int k, int r, int lane) {
  constexpr int LD = G::LD;
  if (lane == 0) {
    for (int i = 0; i < k; i++) g.c[i] = -g.ntx0[i];
    for (int p = 0; p < k; p++) { greal t = g.c[p]; g.c[p] = g.c[g.rowsT[p]]; g.c[g.rowsT[p]] = t; }
  }
  if (lane < k) g.y0[lane] = greal(0);
  gsync<G>();
  if (r == 0) return;
  for (int j = 0; j < k; j++) {  // unit lower
    greal cj = g.c[j];
    if (lane > j && lane < k) g.c[lane] -= cj * g.lu[lane + j * LD];
    gsync<G>();
  }
  upper_solve_shared<G>(g.lu, g.c, r, lane);
  if (lane < r) g.y0[g.q[lane]] = g.c[lane];
  gsync<G>();
}

// FullPivLU::kernel() -> g.Ny (k x dimker); uses g.qr as scratch; g.piv/rycol set
template <class G>
__device__ void lu_kernel_image(G& g, const LUInfo& info, int k, int r, greal thr, int lane) {
  constexpr int LD = G::LD;
  if (lane == 0) {
    greal pt = info.maxpivot * thr;
    int p = 0;
    for (int i = 0; i < info.nz; i++)
      if (fabs(g.lu[i + i * LD]) > pt) g.piv[p++] = i;
    for (int i = 0; i < r; i++) g.rycol[i] = g.q[g.piv[i]];  // image columns
  }
  gsync<G>();
  const int dimker = k - r;
  if (dimker == 0) return;
  greal* mm = g.qr;  // r x k trapezoid
  for (int e = lane; e < r * k; e += HALF) {
    int i = e % r, j = e / r;
    mm[i + j * LD] = (j >= i) ? g.lu[g.piv[i] + j * LD] : greal(0);
  }
  gsync<G>();
  if (lane < r) {  // bring non-negligible pivots to the front (rows own a column swap each)
    for (int i = 0; i < r; i++) {
      int pc = g.piv[i];
      if (pc != i) { greal t = mm[lane + i * LD]; mm[lane + i * LD] = mm[lane + pc * LD]; mm[lane + pc * LD] = t; }
    }
  }
  gsync<G>();
  if (lane < dimker) {  // solve U11 X = U12, one right-hand column per lane
    greal* col = &mm[(r + lane) * LD];
    for (int i = r - 1; i >= 0; i--) {
      if (col[i] != 0) {
        col[i] /= mm[i + i * LD];
        for (int rr = 0; rr < i; rr++) col[rr] -= col[i] * mm[rr + i * LD];
      }
    }
  }
  gsync<G>();
  if (lane < r) {
    for (int i = r - 1; i >= 0; i--) {
      int pc = g.piv[i];
      if (pc != i) { greal t = mm[lane + i * LD]; mm[lane + i * LD] = mm[lane + pc * LD]; mm[lane + pc * LD] = t; }
    }
  }
  gsync<G>();
  for (int e = lane; e < k * dimker; e += HALF) {
    int i = e % k, kk = e / k;
    int row = g.q[i];
    greal v;
    if (i < r) v = -mm[i + (r + kk) * LD];
    else v = (i == r + kk) ? greal(1) : greal(0);
    g.Ny[row + kk * LD] = v;
  }
  gsync<G>();
}

// entry (i, j) of m = [ntn1 Ny, ntn0 Ry] (ftsolver.cpp:222-226), evaluated where needed
template <class G>
__device__ inline greal m_at(const G& g, int k, int dimker, int i, int j) {
  constexpr int LD = G::LD;
  greal s = greal(0);
  if (j < dimker) {
    if (g.coupled) {
      for (int kk = 0; kk < k; kk++) s = s + ntn1_full(g, i, kk) * g.Ny[kk + j * LD];
    } else {
      int b0 = (i / 3) * 3;
      for (int kk = b0; kk < b0 + 3; kk++) s = s + ntn1_at(g, i, kk) * g.Ny[kk + j * LD];
    }
  } else {
    int col = g.rycol[j - dimker];
    for (int kk = 0; kk < k; kk++) s = s + g.ntn0[i + kk * LD] * g.ntn0[kk + col * LD];
  }
  return s;
}

// Eigen 3.3 ColPivHouseholderQR on g.qr (k x k, holding m); returns nonzero pivots
// near: a nonzero-pivot decision (Eigen's |col|^2 < threshold_helper (k - p)) within kNearBand^2
template <class G>
__device__ int colpiv_qr(G& g, int k, int lane, bool& near) {
  constexpr int LD = G::LD;
  if (lane < k) {
    greal s = 0;
    for (int i = 0; i < k; i++) s += g.qr[i + lane * LD] * g.qr[i + lane * LD];
    g.nd[lane] = sqrt(s);
    g.nu[lane] = g.nd[lane];
  }
  gsync<G>();
  greal mx = 0;
  for (int j = 0; j < k; j++) mx = fmax(mx, g.nu[j]);
  const greal th = mx * gEps;
  const greal threshold_helper = th * th / (greal)k;
  const greal ndt = sqrt(gEps);
  int np = k;
  for (int p = 0; p < k; p++) {
    int bi = p;
    greal bv = g.nu[p];
    for (int j = p + 1; j < k; j++)
      if (g.nu[j] > bv) { bv = g.nu[j]; bi = j; }
    if (np == k) near |= near_thr(bv * bv, threshold_helper * (greal)(k - p), greal(kNearBand) * greal(kNearBand));
    if (np == k && bv * bv < threshold_helper * (greal)(k - p)) np = p;
    gsync<G>();
    if (lane == 0) g.cperm[p] = bi;
    if (bi != p) {
      if (lane < k) {
        greal t = g.qr[lane + p * LD];
        g.qr[lane + p * LD] = g.qr[lane + bi * LD];
        g.qr[lane + bi * LD] = t;
      }
      if (lane == 0) {
        greal t = g.nu[p]; g.nu[p] = g.nu[bi]; g.nu[bi] = t;
        t = g.nd[p]; g.nd[p] = g.nd[bi]; g.nd[bi] = t;
      }
    }
    gsync<G>();
    // makeHouseholderInPlace on column p, rows p..k-1
    const int len = k - p;
    greal c0 = g.qr[p + p * LD];
    greal tail = 0;
    for (int i = 1; i < len; i++) tail += g.qr[p + i + p * LD] * g.qr[p + i + p * LD];
    greal tau, beta;
    if (len == 1 || tail <= gTiny) {
      tau = 0;
      beta = c0;
      if (lane >= 1 && lane < len) g.qr[p + lane + p * LD] = 0;
    } else {
      beta = sqrt(c0 * c0 + tail);
      if (c0 >= 0) beta = -beta;
      greal den = c0 - beta;
      if (lane >= 1 && lane < len) g.qr[p + lane + p * LD] /= den;
      tau = (beta - c0) / beta;
    }
    gsync<G>();
    if (lane == 0) { g.qr[p + p * LD] = beta; g.hc[p] = tau; }
    // apply to columns p+1..k-1, then downdate their norms (one column per lane)
    const int j = lane;
    if (j > p && j < k) {
      if (len == 1) {
        g.qr[p + j * LD] *= (1 - tau);
      } else if (tau != 0) {
        greal tmp = 0;
        for (int i = 1; i < len; i++) tmp += g.qr[p + i + p * LD] * g.qr[p + i + j * LD];
        tmp += g.qr[p + j * LD];
        g.qr[p + j * LD] -= tau * tmp;
        for (int i = 1; i < len; i++) g.qr[p + i + j * LD] -= tau * g.qr[p + i + p * LD] * tmp;
      }
      if (g.nu[j] != 0) {
        greal temp = fabs(g.qr[p + j * LD]) / g.nu[j];
        temp = (1 + temp) * (1 - temp);
        temp = temp < 0 ? 0 : temp;
        greal ratio = g.nu[j] / g.nd[j];
        greal temp2 = temp * (ratio * ratio);
        if (temp2 <= ndt) {
          greal s = 0;
          for (int i = p + 1; i < k; i++) s += g.qr[i + j * LD] * g.qr[i + j * LD];
          g.nd[j] = sqrt(s);
          g.nu[j] = g.nd[j];
        } else {
          g.nu[j] *= sqrt(temp);
        }
      }
    }
    gsync<G>();
  }
  return np;
}

// QR solve m z = b (least squares, basic solution) -> g.z
template <class G>
__device__ void qr_solve(G& g, int k, int np, int lane) {
  constexpr int LD = G::LD;
  if (lane < k) { g.c[lane] = g.b[lane]; g.z[lane] = greal(0); }
  gsync<G>();
  if (np == 0) return;
  for (int p = 0; p < np; p++) {
    const int len = k - p;
    const greal tau = g.hc[p];
    if (len == 1) {
      if (lane == p) g.c[p] *= (1 - tau);
    } else if (tau != 0) {
      greal tmp = 0;
      for (int i = 1; i < len; i++) tmp += g.qr[p + i + p * LD] * g.c[p + i];
      tmp += g.c[p];
      gsync<G>();
      if (lane == 0) g.c[p] -= tau * tmp;
      if (lane >= 1 && lane < len) g.c[p + lane] -= tau * g.qr[p + lane + p * LD] * tmp;
    }
    gsync<G>();
  }
  upper_solve_shared<G>(g.qr, g.c, np, lane);
  if (lane == 0) {
    int perm[HS_KMAX];
    for (int i = 0; i < k; i++) perm[i] = i;
    for (int p = 0; p < k; p++) { int t = perm[p]; perm[p] = perm[g.cperm[p]]; perm[g.cperm[p]] = t; }
    for (int i = 0; i < np; i++) g.z[perm[i]] = g.c[i];
  }
  gsync<G>();
}

// S3 general: adaptive-rank two-stage least squares (ftsolver.cpp:185-236) -> sv.y.
// The reference re-runs FullPivLU on the same zeroth-order Gram every pass; it
// is factorized once here (identical factors), only the rank threshold moves.
template <class SV, class G>
__device__ uint32_t contact_solve(SV& sv, G& g, int k, int lane) {
  constexpr int LD = G::LD;
  uint32_t flags = 0;
  if (k == 0) return HS_FLAG_NO_CONTACT;
  const LUInfo info = fullpiv_lu(g, k, lane);
  STAMP(10);
  int rank0 = k;
  int iters = 0;
  greal rel_error = 0;
  bool ill = false;  // the last pass's second stage ill-conditioned (gCondQR)
  do {
    iters++;
    greal thr = gEps * (greal)k;
    int r = lu_rank(g, info, thr);
    for (int guard = 0; guard < 2100 && r > rank0; guard++) {  // setThreshold doubling
      thr = 2 * thr;
      r = lu_rank(g, info, thr);
      flags |= HS_FLAG_NEAR_RANK;  // the threshold now sits within 2x of a pivot by construction
    }
    if (lu_near(g, info, thr)) flags |= HS_FLAG_NEAR_RANK;
    lu_solve(g, info, k, r, lane);
    lu_kernel_image(g, info, k, r, thr, lane);
    STAMP(11);
    if (r == k) flags |= HS_FLAG_FULL_RANK;
    rank0 = r;
    const int dimker = k - r;
    // b = -(ntx1 + ntn1 y0)
    if (lane < k) {
      int i = lane, b0 = (i / 3) * 3;
      greal t = greal(0);
      if (g.coupled)
        for (int kk = 0; kk < k; kk++) t = t + ntn1_full(g, i, kk) * g.y0[kk];
      else
        for (int kk = b0; kk < b0 + 3; kk++) t = t + ntn1_at(g, i, kk) * g.y0[kk];
      g.b[i] = -(g.ntx1[i] + t);
    }
    for (int e = lane; e < k * k; e += HALF) {  // m, built straight into the QR buffer
      int i = e % k, j = e / k;
      g.qr[i + j * LD] = m_at(g, k, dimker, i, j);
    }
    gsync<G>();
    STAMP(12);
    bool qr_near = false;
    int np = colpiv_qr(g, k, lane, qr_near);
    if (qr_near) flags |= HS_FLAG_NEAR_RANK;
    {  // the smallest kept pivot of this pass (the last pass's decides)
      greal rmin = greal(INFINITY);
      for (int i = 0; i < np; i++) rmin = fmin(rmin, fabs(g.qr[i + i * LD]));
      ill = np > 0 && rmin < gCondQR * fabs(g.qr[0]);
    }
    STAMP(13);
    qr_solve(g, k, np, lane);
    STAMP(14);
    // rel_error = |m z - b| / |b|
    if (lane < k) {
      greal s = greal(0);
      for (int j = 0; j < k; j++) s = s + m_at(g, k, dimker, lane, j) * g.z[j];
      g.c[lane] = s - g.b[lane];
    }
    gsync<G>();
    greal rn = 0, bn = 0;
    for (int i = 0; i < k; i++) { rn += g.c[i] * g.c[i]; bn += g.b[i] * g.b[i]; }
    rel_error = sqrt(rn) / sqrt(bn);
    if (near_thr(rel_error, gRelTol, greal(10))) flags |= HS_FLAG_NEAR_RANK;
    rank0--;
    if (lane < k) {
      greal s = greal(0);
      for (int j = 0; j < dimker; j++) s = s + g.Ny[lane + j * LD] * g.z[j];
      sv.y[lane] = g.y0[lane] + s;
    }
    gsync<G>();
    if (rel_error > gRelTol && rank0 <= 0) { flags |= HS_FLAG_LOOP_EXHAUST; break; }
  } while (rel_error > gRelTol && iters <= HS_KMAX + 1);
  if (iters > 1) flags |= HS_FLAG_RANK_RETRY;
  if (ill) flags |= HS_FLAG_NEAR_RANK;
  return flags;
}

// The general path is an out-of-line call: it keeps its own register allocation apart from the
// kernel body's 168-VGPR budget (3 waves/SIMD). Inlined at that budget (the former HS_GENERAL_INLINE
// build) hipcc of ROCm 7.2 spills 7 VGPRs in the block that fullpiv_lu's lane-0 permutation loop
// falls through to when its last lane leaves -- before that block restores EXEC, so the spill stores
// run with EXEC == 0 and write nothing, and their reloads return stale scratch: wrong forces on every
// HS_SOLVE_REFERENCE step. tools/isa_check.py finds the pattern in the built
// library and hslabs_amd/build.py refuses a library that has it. The call costs only the steps that
// take it (stack frame in scratch, 288 B per lane).
#ifdef HS_GENERAL_INLINE
#error "HS_GENERAL_INLINE: the inlined general path is miscompiled at 3 waves/SIMD (VGPR spills at EXEC == 0)"
#endif
#define HS_GENERAL_ATTR __attribute__((noinline))
template <class W, class SV, class G>
__device__ HS_GENERAL_ATTR uint32_t general_solve(const hs_topo* T, SV& sv, G& g, const W& w, int k, int lane) {
  build_grams(T, sv, g, w, k, lane);
  STAMP(9);
  return contact_solve(sv, g, k, lane);
}

// ---------------------------------------------------------------------------
// S3 fast path: closed form of the same lexicographic least squares
// (oracle/hs_oracle.cpp fast_contact_solve, identical operation order).
// One lane per contact builds A_c, D_c, g_c; >= 3 contacts: 6x6 Schur
// complement of the zeroth-order constraints; 1 contact: unique LS; 2 contacts:
// rank-5 kernel along the feet line. Returns false (wave-uniform) when a
// Cholesky pivot falls under the guard -> general path.
// ---------------------------------------------------------------------------
// conditioning guard of the closed-form Cholesky pivots (relative to the largest diagonal)
constexpr real kFastPivotGuard = HS_REAL_IS_FLOAT ? real(1e-4) : real(1e-10);

// Nearly collinear contact feet (nc >= 3): the zeroth-order Gram G = A A^T = sum_c A_c A_c^T is
// close to rank 5. The reference's loop (ftsolver.cpp:205-232) then sees a rank-deficient first-order
// system (its ntn0 * Ry columns carry G's conditioning squared), finds rel_error > 1e-6 and retries at
// lower ranks, landing on a different answer from the closed form's exact minimizer. G's smallest
// eigenvalue is that of J = sum_c [e_c]x [e_c]x^T = tr(C) I - C (the Schur complement of its
// translation block; e_c = d0_c - mean d0, C = sum_c e_c e_c^T), i.e. mu2 + mu3 for C's eigenvalues
// mu1 >= mu2 >= mu3, which c2(C) / tr(C) gives to within a factor of 4 (c2 = the sum of C's principal
// 2x2 minors). The closed form is taken only when c2(C) / (tr(C) maxdiag(G)) >= kZerothGuard; the
// ratio follows the reference's 6th FullPivLU pivot ratio to within ~2x. Over the oracle's tree mode on
// 120k transformed steps every retry had it below 2.5e-5; plain synthetic gaits stay
// above 1e-2. Steps under the guard take the Eigen-style path, which restates the reference's loop.
// No division: with s = sum d0_c and Q = sum d0_c d0_c^T, C' = nc Q - s s^T = nc C, so the test reads
// c2(C') >= kZerothGuard * nc * tr(C') * maxdiag(G), maxdiag(G) = max(nc, tr Q - Q_ii). A heuristic
// with a 40x margin on each side, so it runs in single precision: contact lane c holds d0_c, the nine
// moments are summed over the 8-lane group by DPP (quad xor 1, xor 2, half-row mirror), and lanes past
// nc add zeros. Every lane of the half-wave calls it; the verdict is the same on lanes 0 .. 7.
constexpr float kZerothGuard = 1e-3f;

template <int CTRL>
__device__ inline float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ inline float group8_sum(float v) {
  v += dpp_f<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_f<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_f<0x141>(v);  // row_half_mirror: lane i <- 7 - i, the other quad's sum
  return v;
}

// a real moved across lanes by DPP control CTRL (a double as two 32-bit moves)
template <int CTRL>
__device__ inline real dpp_r(real x) {
#if HS_REAL_IS_FLOAT
  return dpp_f<CTRL>(x);
#else
  const long long u = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_mov_dpp((int)u, CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(u >> 32), CTRL, 0xF, 0xF, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
#endif
}
// sum over the 4-lane quad (DPP quad_perm xor 1, xor 2): every lane of the quad gets the same value
// (each addition is commutative in its two operands)
__device__ inline real quad_sum(real v) {
  v += dpp_r<0xB1>(v);
  v += dpp_r<0x4E>(v);
  return v;
}

// bit 0: well posed (take the closed form); bit 1: the ratio lies within kNearBand of the guard
// (HS_FLAG_NEAR_RANK: another rounding may route the step the other way)
template <class W, class SV>
__device__ inline int zeroth_well_posed(const real* P0, const W& w, const SV& sv, int nc, int lane) {
  float d0 = 0.f, d1 = 0.f, d2 = 0.f;
  if (lane < nc) {
    const real* fp = w.fpos(0, sv.cfoot[lane]);
    d0 = float(P0[0] - fp[0]); d1 = float(P0[1] - fp[1]); d2 = float(P0[2] - fp[2]);
  }
  const float s0 = group8_sum(d0), s1 = group8_sum(d1), s2 = group8_sum(d2);
  const float q00 = group8_sum(d0 * d0), q11 = group8_sum(d1 * d1), q22 = group8_sum(d2 * d2);
  const float q01 = group8_sum(d0 * d1), q02 = group8_sum(d0 * d2), q12 = group8_sum(d1 * d2);
  const float k = float(nc);
  const float c00 = k * q00 - s0 * s0, c11 = k * q11 - s1 * s1, c22 = k * q22 - s2 * s2;
  const float c01 = k * q01 - s0 * s1, c02 = k * q02 - s0 * s2, c12 = k * q12 - s1 * s2;
  const float c2 = (c00 * c11 - c01 * c01) + (c00 * c22 - c02 * c02) + (c11 * c22 - c12 * c12);
  const float tq = q00 + q11 + q22;
  const float md = fmaxf(k, fmaxf(tq - q00, fmaxf(tq - q11, tq - q22)));
  const float t = kZerothGuard * k * (c00 + c11 + c22) * md;
  return (c2 >= t ? 1 : 0) | (c2 >= t / float(kNearBand) && c2 <= t * float(kNearBand) ? 2 : 0);  // 0 on NaN
}

// rl (N): receives 1 / L_jj, the reciprocal each pivot's column was scaled by, for chol_solve_n
// near: set when a pivot lies within kNearBand of the guard (HS_FLAG_NEAR_RANK)
template <int N>
__device__ inline bool chol_n(real* a, real guard, real* rl_out, bool& near) {  // row-major, in place
  real mx = 0;
#pragma unroll
  for (int i = 0; i < N; i++) mx = fmax(mx, a[i * N + i]);
#pragma unroll
  for (int j = 0; j < N; j++) {
    real s = a[j * N + j];
#pragma unroll
    for (int k = 0; k < j; k++) s -= a[j * N + k] * a[j * N + k];
    near |= near_thr(s, guard * mx, kNearBand);
    if (!(s > guard * mx)) return false;
    const real l = sqrt(s), rl = real(1) / l;  // one division per pivot (oracle chol)
    a[j * N + j] = l;
    rl_out[j] = rl;
#pragma unroll
    for (int i = j + 1; i < N; i++) {
      real t = a[i * N + j];
#pragma unroll
      for (int k = 0; k < j; k++) t -= a[i * N + k] * a[j * N + k];
      a[i * N + j] = t * rl;
    }
  }
  return true;
}

// rl: chol_n's reciprocals of the pivots (1 / L_ii, the same divisions, not recomputed)
template <int N>
__device__ inline void chol_solve_n(const real* L, const real* rl, real* b) {
#pragma unroll
  for (int i = 0; i < N; i++) {
    real s = b[i];
#pragma unroll
    for (int k = 0; k < i; k++) s -= L[i * N + k] * b[k];
    b[i] = s * rl[i];
  }
#pragma unroll
  for (int i = N - 1; i >= 0; i--) {
    real s = b[i];
#pragma unroll
    for (int k = i + 1; k < N; k++) s -= L[k * N + i] * b[k];
    b[i] = s * rl[i];
  }
}

// LDL^T of an N x N SPD matrix in place (row-major; lower part: unit-lower L, diagonal: d), no
// square roots: pivot d_j = a_jj - sum_k L_jk (L_jk d_k), the Cholesky pivot in exact arithmetic, so
// the guard (d_j > guard * max diagonal) decides like chol_n's. rd: 1 / d_j. False: a pivot under it.
// 1 / x for a positive normal pivot: v_rcp_f64 refined by two Newton steps (within an ulp of the
// correctly rounded quotient), five instructions instead of the IEEE division's scale / fixup sequence
__device__ inline real pivot_rcp(real x) {
#if !HS_REAL_IS_FLOAT
  real r = __builtin_amdgcn_rcp(x);
  real e = fma(-x, r, real(1));
  r = fma(r, e, r);
  e = fma(-x, r, real(1));
  return fma(r, e, r);
#else
  return real(1) / x;
#endif
}

// near (guarded factorizations): set when a pivot lies within kNearBand of the guard
template <int N>
__device__ inline bool ldl_n(real* a, real guard, real* rd, bool& near) {
  real mx = 0;
#pragma unroll
  for (int i = 0; i < N; i++) mx = fmax(mx, a[i * N + i]);
#pragma unroll
  for (int j = 0; j < N; j++) {
    real v[N];  // L_jk d_k
#pragma unroll
    for (int k = 0; k < j; k++) v[k] = a[j * N + k] * a[k * N + k];
    real dj = a[j * N + j];
#pragma unroll
    for (int k = 0; k < j; k++) dj -= a[j * N + k] * v[k];
    near |= near_thr(dj, guard * mx, kNearBand);
    if (!(dj > guard * mx)) return false;
    const real r = pivot_rcp(dj);
    a[j * N + j] = dj;
    rd[j] = r;
#pragma unroll
    for (int i = j + 1; i < N; i++) {
      real t = a[i * N + j];
#pragma unroll
      for (int k = 0; k < j; k++) t -= a[i * N + k] * v[k];
      a[i * N + j] = t * r;
    }
  }
  return true;
}

// unguarded (guard 0: SPD by construction, no decision taken)
template <int N>
__device__ inline bool ldl_n(real* a, real guard, real* rd) {
  bool unused = false;
  return ldl_n<N>(a, guard, rd, unused);
}

// solve L D L^T x = b in place with ldl_n's factors
template <int N>
__device__ inline void ldl_solve_n(const real* L, const real* rd, real* b) {
#pragma unroll
  for (int i = 0; i < N; i++) {
    real s = b[i];
#pragma unroll
    for (int k = 0; k < i; k++) s -= L[i * N + k] * b[k];
    b[i] = s;
  }
#pragma unroll
  for (int i = 0; i < N; i++) b[i] *= rd[i];
#pragma unroll
  for (int i = N - 1; i >= 0; i--) {
    real s = b[i];
#pragma unroll
    for (int k = i + 1; k < N; k++) s -= L[k * N + i] * b[k];
    b[i] = s;
  }
}

__device__ inline void cross_rows(const real* d, real v[3][3]) {
  v[0][0] = 0;     v[0][1] = -d[2]; v[0][2] = d[1];
  v[1][0] = d[2];  v[1][1] = 0;     v[1][2] = -d[0];
  v[2][0] = -d[1]; v[2][1] = d[0];  v[2][2] = 0;
}

// entry (r, j) of A_c = [-I; [d0]x] (the values cross_rows lays out)
__device__ inline real a_entry(const real* d0, int r, int j) {
  if (r < 3) return (r == j) ? real(-1) : real(0);
  const int i = r - 3;
  if (i == j) return real(0);
  const real v = d0[3 - i - j];
  return ((j - i + 3) % 3 == 1) ? -v : v;
}

// In-place Cholesky of a k x k SPD matrix (row-major, lower triangle used) by
// the half-wave, right-looking: element (i, j) gets its products subtracted in
// increasing order, exactly like the oracle's left-looking chol(). False (wave-
// uniform) when a pivot falls to guard * (max original diagonal) or below.
// rdiag (optional) receives 1 / L_jj.
// (GLOBAL: K lives in global memory, so the exchanges need the workgroup's global-memory fences)
template <bool GLOBAL>
__device__ inline void ws_sync() {
  if constexpr (GLOBAL) __syncthreads();
  else wave_sync();
}

// Lane-strided walks over matrix entries without integer divisions (a 32-bit division by a
// runtime size is ~40 VALU instructions) or per-step loops. TriWalk: the packed lower triangle row
// by row ((0,0), (1,0), (1,1), (2,0), ...) with rows of r + 1 + EXTRA entries, entries p = lane,
// lane + 32, ...: the row from a single-precision square root (exact for p < 2^20), corrected by
// one step either way
template <int EXTRA = 0>
struct TriWalk {
  int p, r, c;
  __device__ explicit TriWalk(int p_) : p(p_) { locate(); }
  // first index of row r: r (r + 1) / 2 + EXTRA r = r (r + 1 + 2 EXTRA) / 2
  __device__ static int row0(int r) { return r * (r + 1 + 2 * EXTRA) / 2; }
  __device__ void locate() {
    const float b = 1.0f + 2.0f * EXTRA;  // r^2 + b r - 2 p = 0
    r = (int)((sqrtf(b * b + 8.0f * (float)p) - b) * 0.5f);
    if (row0(r + 1) <= p) r++;
    if (row0(r) > p) r--;
    c = p - row0(r);
  }
  __device__ void next() {
    p += HALF;
    locate();
  }
};
// RectWalk: row-major entries of an (any) x ld rectangle
struct RectWalk {
  int r, c, ld;
  __device__ RectWalk(int p, int ld_) : r(0), c(p), ld(ld_) { settle(); }
  __device__ void settle() {
    while (c >= ld) { c -= ld; r++; }
  }
  __device__ void next() { c += HALF; settle(); }
};

template <bool GLOBAL>
__device__ __attribute__((always_inline)) inline bool chol_half(real* K, int k, real guard, int lane, bool& near,
                                                                 real* rdiag = nullptr) {
  real mx = 0;
  for (int i = 0; i < k; i++) mx = fmax(mx, K[i * k + i]);
  for (int j = 0; j < k; j++) {
    const real s = K[j * k + j];
    near |= near_thr(s, guard * mx, kNearBand);
    if (!(s > guard * mx)) return false;
    const real l = sqrt(s), rl = real(1) / l;
    if (lane == 0) {
      K[j * k + j] = l;
      if (rdiag) rdiag[j] = rl;
    }
    for (int i = j + 1 + lane; i < k; i += HALF) K[i * k + j] = K[i * k + j] * rl;
    ws_sync<GLOBAL>();
    const int m = k - 1 - j;
    for (int e = lane; e < m * m; e += HALF) {
      const int i = j + 1 + e / m, c2 = j + 1 + e % m;
      if (c2 <= i) K[i * k + c2] -= K[i * k + j] * K[c2 * k + j];
    }
    ws_sync<GLOBAL>();
  }
  return true;
}

// packed lower-triangle index (row-major: row r holds r + 1 entries)
__device__ inline int pk(int r, int c) { return r * (r + 1) / 2 + c; }

// chol_half's right-looking Cholesky on a packed lower triangle in LDS (solve_forces: its normal
// matrix), the same operations per entry; the trailing update walks the packed entries. A pivot at or
// under guard * (largest diagonal) drops its variable (returned in the mask): its column is zeroed, so
// the later pivots are those of the system without it, and the caller's solves leave it at 0 -- the
// basic solution of a rank-deficient least squares (SparseQR's, ftsolver.cpp:349-353, in the natural
// column order). near: a pivot within kNearBand of the guard (HS_FLAG_NEAR_RANK).
__device__ __attribute__((always_inline)) inline uint32_t chol_packed(real* K, int k, real guard, int lane,
                                                                      bool& near) {
  real mx = 0;
  for (int i = 0; i < k; i++) mx = fmax(mx, K[pk(i, i)]);
  uint32_t dropped = 0;
  // one pivot's column: scaled by 1 / L_jj, or zeroed when the pivot is dropped (L_jj = 1 then)
  auto pivot = [&](int j) {
    const real s = K[pk(j, j)];
    near |= near_thr(s, guard * mx, kNearBand);
    const bool keep = s > guard * mx;  // false on NaN
    const real l = keep ? sqrt(s) : real(1), rl = keep ? real(1) / l : real(0);
    if (!keep) dropped |= 1u << j;
    if (lane == 0) K[pk(j, j)] = l;
    for (int i = j + 1 + lane; i < k; i += HALF) K[pk(i, j)] = K[pk(i, j)] * rl;
    wave_sync();
  };
  // two pivots per trailing pass: pivot j, column j + 1 updated by it, pivot j + 1, then every
  // entry right of both takes pivot j's product and pivot j + 1's in that order -- each entry sees
  // the operations of one pivot at a time, in pivot order, as in chol_half
  for (int j = 0; j < k; j += 2) {
    const bool two = j + 1 < k;
    pivot(j);
    if (two) {
      for (int i = j + 1 + lane; i < k; i += HALF) K[pk(i, j + 1)] -= K[pk(i, j)] * K[pk(j + 1, j)];
      wave_sync();
      pivot(j + 1);
    }
    const int j1 = two ? j + 2 : j + 1, m = k - j1;
    for (TriWalk<> t(lane); t.r < m; t.next()) {  // the trailing lower triangle, entry by entry
      const int i = j1 + t.r, c2 = j1 + t.c;
      real v = K[pk(i, c2)];
      v -= K[pk(i, j)] * K[pk(c2, j)];
      if (two) v -= K[pk(i, j + 1)] * K[pk(c2, j + 1)];
      K[pk(i, c2)] = v;
    }
    wave_sync();
  }
  return dropped;
}

// nc >= 3 with a singular D_c (straight, IK-clamped leg) or Schur complement:
// augmented system K = D + rho A^T A, w = -K^-1 (g~ + A^T lam),
// (A K^-1 A^T) lam = a - A K^-1 g~ (oracle aug_solve, same operation order; the
// half-wave right-looking Cholesky subtracts in the oracle's left-looking order).
// False when the minimizer is not unique (a pivot under the guard).
template <class SV>
__device__ __attribute__((always_inline)) inline bool aug_solve(FastL& fl, AugL& ag, SV& sv, const real* a, int nc,
                                                                int lane, bool& near) {
  const int k = 3 * nc;
  auto Aat = [&](int r, int i) { return a_entry(fl.d0[i / 3], r, i % 3); };  // A (6 x k)
  real md = 0, ma = 0;
  for (int c = 0; c < nc; c++)
    for (int i = 0; i < 3; i++) {
      md = fmax(md, fl.D[c][4 * i]);
      real s = 0;
      for (int r = 0; r < 6; r++) s += Aat(r, 3 * c + i) * Aat(r, 3 * c + i);
      ma = fmax(ma, s);
    }
  const real rho = (md > 0 && ma > 0) ? md / ma : real(1);
  for (int e = lane; e < k * k; e += HALF) {
    const int i = e / k, j = e % k;
    real s = 0;
    for (int r = 0; r < 6; r++) s += Aat(r, i) * Aat(r, j);
    ag.K[i * k + j] = ((i / 3 == j / 3) ? fl.D[i / 3][3 * (i % 3) + j % 3] : real(0)) + rho * s;
  }
  for (int e = lane; e < k * 7; e += HALF) {
    const int i = e / 7, q = e % 7;
    real v;
    if (q < 6) {
      v = Aat(q, i);
    } else {
      real s = 0;
      for (int r = 0; r < 6; r++) s += Aat(r, i) * a[r];
      v = fl.g[i / 3][i % 3] + rho * s;
    }
    ag.X[i * 7 + q] = v;
  }
  __syncthreads();
  if (!chol_half<true>(ag.K, k, kFastPivotGuard, lane, near, ag.rdiag)) return false;
  __syncthreads();
  if (lane < 7) {  // K X = [A^T | g~], one right-hand column per lane
    const int q = lane;
    for (int i = 0; i < k; i++) {
      real s = ag.X[i * 7 + q];
      for (int m = 0; m < i; m++) s -= ag.K[i * k + m] * ag.X[m * 7 + q];
      ag.X[i * 7 + q] = s * ag.rdiag[i];
    }
    for (int i = k - 1; i >= 0; i--) {
      real s = ag.X[i * 7 + q];
      for (int m = i + 1; m < k; m++) s -= ag.K[m * k + i] * ag.X[m * 7 + q];
      ag.X[i * 7 + q] = s * ag.rdiag[i];
    }
  }
  __syncthreads();
  for (int e = lane; e < 42; e += HALF) {
    const int r = e / 7, q = e % 7;
    real s = 0;
    for (int i = 0; i < k; i++) s += Aat(r, i) * ag.X[i * 7 + q];
    if (q < 6) ag.St[6 * r + q] = s;
    else ag.lam[r] = a[r] - s;
  }
  __syncthreads();
  if (lane == 0) {
    real St[36], lam[6];
    for (int i = 0; i < 36; i++) St[i] = ag.St[i];
    for (int i = 0; i < 6; i++) lam[i] = ag.lam[i];
    real rl[6];
    int ok = chol_n<6>(St, kFastPivotGuard, rl, near);
    if (ok) {
      chol_solve_n<6>(St, rl, lam);
      for (int i = 0; i < 6; i++) ag.lam[i] = lam[i];
    }
    ag.ok = ok;
  }
  __syncthreads();
  if (!ag.ok) return false;
  for (int i = lane; i < k; i += HALF) {
    real s = ag.X[i * 7 + 6];
    for (int r = 0; r < 6; r++) s += ag.X[i * 7 + r] * ag.lam[r];
    sv.y[i] = -s;
  }
  __syncthreads();
  return true;
}

// aug_ok = false (the fixup launch's idle half, which stores nothing): decline instead of using the
// augmented system, whose global workspace is the idle slot every fixup wavefront shares
// lnear: this lane saw a routing decision within kNearBand of its guard (fast_solve ballots it)
template <class W, class SV>
__device__ __attribute__((always_inline)) inline bool fast_solve_lanes(const hs_topo* T, SV& sv, FastL& fl, AugL& ag,
                                                                       const W& w, int nc, bool aug_ok, int lane,
                                                                       bool& lnear) {
  const int n = T->n;
  if (nc == 0) return true;
  const real* P0 = w.pos(0, 0);
  const int zw = nc >= 3 ? zeroth_well_posed(P0, w, sv, nc, lane) : 1;
  const int coll = (zw & 1) ? 0 : 2;
  lnear |= (zw & 2) != 0 && lane < 8;  // the group of lanes 0 .. 7 holds the contacts' sums
  // four lanes per contact (lane = 4 c + s): lane s sums the D_c / g_c terms of the foot chain's
  // joints s, s + 4, the quad adds them (DPP), every lane of the quad factorizes D_c, and the Schur
  // block's rows are split {s, 5 - s} (seven packed entries and two of h per lane; lane 3 repeats
  // lane 2's rows and stores D_c, g_c, d0_c and D_c^-1 instead) -- one instruction stream, the lanes
  // differing only in data. The blocks are summed over the contacts across the lanes (sch below)
  real sch[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};  // this lane's 7 packed entries and 2 of h; 0 past nc
  {
    const int c = lane >> 2, s4 = lane & 3;
    if (c < nc) {
      const int fi = sv.cfoot[c];
      const real* fp = w.fpos(0, fi);
      real d0[3];
      for (int r = 0; r < 3; r++) d0[r] = P0[r] - fp[r];
      real Dp[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};  // packed lower 00 10 11 20 21 22
      const uint8_t* fch = reinterpret_cast<const uint8_t*>(sv.fch[fi]);
      const int nch = fch[0];
      for (int m = s4; m < nch; m += 4) {
        const int p = fch[1 + m];
        const real* Jp = w.jpos(0, p);
        const real* Jz = w.jz(0, p);
        real da[3], va[3][3];
        for (int r = 0; r < 3; r++) da[r] = Jp[r] - fp[r];
        cross_rows(da, va);
#pragma unroll
        for (int r = 0; r < 3; r++) {
          const real w2 = Jz[r] * Jz[r];
#pragma unroll
          for (int i = 0; i < 3; i++) {
            if (i == r) continue;
#pragma unroll
            for (int j = 0; j <= i; j++)
              if (j != r) Dp[i * (i + 1) / 2 + j] += w2 * va[r][i] * va[r][j];
            g[i] += w2 * va[r][i] * sv.x[3 * n + 3 * p + r];
          }
        }
      }
#pragma unroll
      for (int e = 0; e < 6; e++) Dp[e] = quad_sum(Dp[e]);
#pragma unroll
      for (int i = 0; i < 3; i++) g[i] = quad_sum(g[i]);
      const real D[9] = {Dp[0], Dp[1], Dp[3], Dp[1], Dp[2], Dp[4], Dp[3], Dp[4], Dp[5]};
      if (s4 == 0) DBG(24 + fi, Dp[0], 6);
      if (s4 == 0) DBG(24 + fi, g[0], 7);
      if (s4 == 3) {
        for (int r = 0; r < 3; r++) fl.d0[c][r] = d0[r];
        for (int i = 0; i < 9; i++) fl.D[c][i] = D[i];
        for (int i = 0; i < 3; i++) fl.g[c][i] = g[i];
      }
      int ok = 1;
      if (nc >= 3) {
        real L[9];
        for (int i = 0; i < 9; i++) L[i] = D[i];
        real rl[3];
        ok = ldl_n<3>(L, kFastPivotGuard, rl, lnear);
        if (ok) {
          real Dinv[9];
          for (int j = 0; j < 3; j++) {
            real e[3] = {0, 0, 0};
            e[j] = 1;
            ldl_solve_n<3>(L, rl, e);
            for (int i = 0; i < 3; i++) Dinv[3 * i + j] = e[i];
          }
          if (s4 == 3)
            for (int i = 0; i < 9; i++) fl.sc.Dinv[c][i] = Dinv[i];
          const int sr = s4 < 3 ? s4 : 2, r0 = sr, r1 = 5 - sr;
          real E0[3], E1[3];  // rows r0, r1 of E = A_c D_c^-1
#pragma unroll
          for (int j = 0; j < 3; j++) {
            real a = 0, b = 0;
#pragma unroll
            for (int i = 0; i < 3; i++) {
              a += a_entry(d0, r0, i) * Dinv[3 * i + j];
              b += a_entry(d0, r1, i) * Dinv[3 * i + j];
            }
            E0[j] = a;
            E1[j] = b;
          }
#pragma unroll
          for (int t = 0; t < 7; t++) {  // row r0's r0 + 1 entries, then row r1's
            const bool first = t <= r0;  // entry (r0, t) or (r1, t - r0 - 1)
            const int q = first ? t : t - r0 - 1;
            real v = 0;
#pragma unroll
            for (int j = 0; j < 3; j++) v += (first ? E0[j] : E1[j]) * a_entry(d0, q, j);
            if (s4 < 3) sch[t] = v;
          }
          real h0 = 0, h1 = 0;
          for (int j = 0; j < 3; j++) {
            h0 += E0[j] * g[j];
            h1 += E1[j] * g[j];
          }
          if (s4 < 3) {
            sch[7] = h0;
            sch[8] = h1;
          }
        }
      }
      if (s4 == 0) fl.ok[c] = ok | coll;
    }
  }
  // sum over the contacts c = 0 .. 7 of lanes 4 c + s: within each 16-lane row by DPP (row_shr 4, then
  // 8: lane 12 + s holds its row's four contacts), then the two rows (xor 16). Lanes 12 .. 14 store the
  // packed [S | h] (a pairwise order, not the contacts' sequence: ULPs of the Schur complement)
#pragma unroll
  for (int e = 0; e < 9; e++) {
    real v = sch[e];
    v += dpp_r<0x114>(v);
    v += dpp_r<0x118>(v);
    sch[e] = v + __shfl_xor(v, 16);
  }
  {
    const int s4 = lane & 3, r0 = s4, r1 = 5 - s4;
    if ((lane & ~3) == 12 && s4 < 3) {
#pragma unroll
      for (int t = 0; t < 7; t++) {
        const bool first = t <= r0;
        fl.sc.Ssum[first ? sch_lower(r0, t) : sch_lower(r1, t - r0 - 1)] = sch[t];
      }
      fl.sc.Ssum[SCH_H + r0] = sch[7];
      fl.sc.Ssum[SCH_H + r1] = sch[8];
    }
  }
  wave_sync();
  STAMP(18);
  const real a[6] = {sv.x[0], sv.x[1], sv.x[2], sv.x[3 * n], sv.x[3 * n + 1], sv.x[3 * n + 2]};
  if (nc >= 3 && (fl.ok[0] & 2)) return false;  // nearly collinear contacts: the Eigen-style path
  for (int c = 0; c < nc; c++)
    if (!(fl.ok[c] & 1)) return aug_ok ? aug_solve(fl, ag, sv, a, nc, lane, lnear) : false;  // only nc >= 3 factors D_c
  int ok = 1;
  if (nc == 1) {  // unique least-squares solution (A^T A) w = -A^T a
    if (lane == 0) {
      real M[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, b[3] = {0, 0, 0};
      const real* d0 = fl.d0[0];
      for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++)
          for (int r = 0; r < 6; r++) M[3 * i + j] += a_entry(d0, r, i) * a_entry(d0, r, j);
        for (int r = 0; r < 6; r++) b[i] -= a_entry(d0, r, i) * a[r];
      }
      real rl[3];
      DBG(24 + sv.cfoot[0], M[4], 19);
      DBG(24 + sv.cfoot[0], b[1], 20);
      ok = chol_n<3>(M, kFastPivotGuard, rl, lnear);
      if (ok) {
        chol_solve_n<3>(M, rl, b);
        for (int i = 0; i < 3; i++) sv.y[i] = b[i];
        DBG(24 + sv.cfoot[0], b[0], 21);
      }
      fl.ok[0] = ok;
    }
  } else if (nc == 2) {  // rank 5: kernel n = (u,-u)/sqrt2 along the line between the feet
    if (lane == 0) {
      const real* f0 = w.fpos(0, sv.cfoot[0]);
      const real* f1 = w.fpos(0, sv.cfoot[1]);
      real u[3], un = 0;
      for (int r = 0; r < 3; r++) { u[r] = f0[r] - f1[r]; un += u[r] * u[r]; }
      un = sqrt(un);
      ok = un > real(1e-12);
      real nv[6], M[36], b[6], rl[6];
      if (ok) {
        for (int r = 0; r < 3; r++) { nv[r] = u[r] / un / sqrt(real(2)); nv[3 + r] = -nv[r]; }
        DBG(24 + sv.cfoot[0], nv[2], 26);
        for (int i = 0; i < 6; i++) {
          const real* di = fl.d0[i / 3];
          for (int j = 0; j < 6; j++) {
            const real* dj = fl.d0[j / 3];
            real s = 0;
            for (int r = 0; r < 6; r++) s += a_entry(di, r, i % 3) * a_entry(dj, r, j % 3);
            M[6 * i + j] = s + nv[i] * nv[j];
          }
          real s = 0;
          for (int r = 0; r < 6; r++) s += a_entry(di, r, i % 3) * a[r];
          b[i] = -s;
        }
        DBG(24 + sv.cfoot[0], M[5], 27);
        opaque_vals<36>(M);  // the assembled system (hs_limb_kernel fences the same values)
        opaque_vals<6>(b);
        opaque_vals<6>(nv);
        ok = chol_n<6>(M, kFastPivotGuard, rl, lnear);
      }
      if (ok) {
        chol_solve_n<6>(M, rl, b);
        opaque_vals<6>(b);
        real nDn = 0, nr = 0;
        for (int c = 0; c < 2; c++)
          for (int i = 0; i < 3; i++) {
            real Dw = 0, Dn = 0;
            for (int j = 0; j < 3; j++) { Dw += fl.D[c][3 * i + j] * b[3 * c + j]; Dn += fl.D[c][3 * i + j] * nv[3 * c + j]; }
            nr += nv[3 * c + i] * (Dw + fl.g[c][i]);
            nDn += nv[3 * c + i] * Dn;
          }
        ok = nDn > 0;
        if (ok) {
          real t = -nr / nDn;
          for (int i = 0; i < 6; i++) sv.y[i] = b[i] + t * nv[i];
          DBG(24 + sv.cfoot[0], sv.y[0], 22);
          DBG(24 + sv.cfoot[0], b[0], 23);
          DBG(24 + sv.cfoot[0], t, 24);
        }
      }
      fl.ok[0] = ok;
    }
  } else {  // Schur complement of the 6 zeroth-order constraints (its entries summed above)
    if (lane == 0) {
      real Sm[36], h[6];
#pragma unroll
      for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) Sm[6 * i + j] = (j <= i) ? fl.sc.Ssum[sch_lower(i, j)] : real(0);  // upper: unread
      for (int i = 0; i < 6; i++) h[i] = fl.sc.Ssum[SCH_H + i];
      real lam[6], rl[6];
      for (int r = 0; r < 6; r++) lam[r] = a[r] - h[r];
      ok = ldl_n<6>(Sm, kFastPivotGuard, rl, lnear);
      if (ok) {
        ldl_solve_n<6>(Sm, rl, lam);
        for (int r = 0; r < 6; r++) fl.sc.lam[r] = lam[r];
      }
      fl.ok[0] = ok;
    }
    wave_sync();
    STAMP(19);
    if (!fl.ok[0]) return aug_ok ? aug_solve(fl, ag, sv, a, nc, lane, lnear) : false;
    if (lane < nc) {
      const int c = lane;
      const real* d0 = fl.d0[c];
      real t[3];
#pragma unroll
      for (int i = 0; i < 3; i++) {  // g + A_c^T lam, A_c's zero entries skipped (exact zeros)
        real s = fl.g[c][i];
#pragma unroll
        for (int r = 0; r < 6; r++) {
          if (r < 3 && r != i) continue;
          if (r >= 3 && r - 3 == i) continue;
          s += a_entry(d0, r, i) * fl.sc.lam[r];
        }
        t[i] = s;
      }
      for (int i = 0; i < 3; i++) {
        real s = 0;
        for (int j = 0; j < 3; j++) s += fl.sc.Dinv[c][3 * i + j] * t[j];
        sv.y[3 * c + i] = -s;
      }
      DBG(24 + sv.cfoot[c], sv.y[3 * c], 8);
    }
  }
  wave_sync();
  return fl.ok[0] != 0;
}

// near (uniform over the half-wave): a routing decision of the closed form lay within kNearBand of its
// guard on some lane (HS_FLAG_NEAR_RANK)
template <class W, class SV>
__device__ __attribute__((always_inline)) inline bool fast_solve(const hs_topo* T, SV& sv, FastL& fl, AugL& ag, const W& w,
                                                                 int nc, bool aug_ok, int lane, bool& near) {
  bool lnear = false;
  const bool ok = fast_solve_lanes(T, sv, fl, ag, w, nc, aug_ok, lane, lnear);
  near = half_ballot(lnear) != 0;
  return ok;
}

// work_over_period's accumulation (periodic.cpp:301-302): work_dt *= dt_traj; work_period += work_dt --
// two roundings, as the reference's x86-64 build performs them (this file is otherwise contracted)
__device__ inline real work_add(real work, real work_dt, real dt) {
#pragma clang fp contract(off)
  const real wdt = work_dt * dt;
  return work + wdt;
}

// selection COT of the best-rollout key (hs_best_key_cot, include/hslabs.h): one cycle's work over
// sum m * |L|; |L| under HS_KEY_MIN_STEP_LENGTH gives NaN (never selected)
__device__ inline real key_cot(real work, real mass, real L, int n_t, int steps) {
  const real aL = fabs(L);
  if (!(aL >= (real)HS_KEY_MIN_STEP_LENGTH) || steps < 1) return (real)NAN;
  return work * ((real)n_t / (real)steps) / (mass * aL);
}

__device__ inline uint64_t best_key(real cot, int64_t id) {
  float c = (float)cot;
  uint32_t bits = __float_as_uint(c);
  uint32_t ord = (c != c) ? 0xFFFFFFFFu : ((bits & 0x80000000u) ? ~bits : (bits | 0x80000000u));
  return ((uint64_t)ord << 32) | (uint32_t)id;
}

// The work reduce of a fused call for rollouts blockIdx.x * 64 + lane (one wavefront per workgroup):
// work_cot[b] = (w, w / (total mass * step length)) with w = (accumulate ? work_cot[b][0] : 0) + the
// steps' joint work sums times dt in step order, then the best key
__device__ inline void reduce_rollouts(const hs_run_args& a, real total_mass, const double* __restrict__ rollout_mass,
                                       const real* __restrict__ ws, int n_steps, uint64_t* best_key_out,
                                       int key_steps) {
  const int b0 = blockIdx.x * blockDim.x + threadIdx.x;
  const bool live = b0 < a.n_rollouts;
  const int b = live ? b0 : a.n_rollouts - 1;  // dead lanes load a valid row and store nothing
  if (rollout_mass) total_mass = (real)rollout_mass[b];  // a mixed plan: the rollout's model
  real w = a.accumulate ? outp(a.work_cot)[2 * (size_t)b] : real(0);
  const real dt = (real)a.params[b].period / a.n_t;  // gait_setup's st.dt
  // periodic.cpp:302-303, in step order; the loads of up to 32 steps issue together ahead of their
  // FMAs (a 20-step job: one round trip)
  for (int s = 0; s < n_steps; s += 32) {
    real v[32];
#pragma unroll
    for (int j = 0; j < 32; j++) v[j] = s + j < n_steps ? ws[(size_t)(s + j) * a.n_rollouts + b] : real(0);
#pragma unroll
    for (int j = 0; j < 32; j++)
      if (s + j < n_steps) w = work_add(w, v[j], dt);
  }
  const real L = (real)a.params[b].step_length;
  const real cot = w / (total_mass * L);
  if (live) {
    outp(a.work_cot)[2 * (size_t)b] = w;
    outp(a.work_cot)[2 * (size_t)b + 1] = cot;
  }
  if (best_key_out) {  // the wave's minimum first: one atomic per wave, not one per rollout on one address
    const real kc = key_cot(w, total_mass, L, a.n_t, key_steps);
    unsigned long long k = live ? (unsigned long long)best_key(kc, a.rollout_id_base + b) : ~0ull;
#pragma unroll
    for (int off = WAVE / 2; off >= 1; off >>= 1) {
      const unsigned long long o = __shfl_xor(k, off);
      k = o < k ? o : k;
    }
    if (threadIdx.x == 0) atomicMin((unsigned long long*)best_key_out, k);
  }
}

// ---------------------------------------------------------------------------
// One control-loop step at centre sample i (row = b * H + h of the outputs)
// ---------------------------------------------------------------------------
// DEFER: a step the closed form declines is not solved here but handed to the fixup launch (the
// step's half-wave stores nothing and `deferred` is set), so this instantiation has no call to the
// out-of-line general path: the call alone costs the whole kernel SGPRs (spills in the hot solve
// region) and 2.4 % of the step time
// dt (SetupL::dt) is loaded at the wave's start (a value read from the setup record later would be read
// again after every output store, which may alias it)
template <bool DEFER, class W, class SV>
__device__ __attribute__((always_inline)) inline void step(const hs_topo* T, const hs_run_args& a, const hs::launch_map& mp, real dt, SV& sv,
                     FastL& fl, const W& w, SolveWS* G, int b, bool live, int h,
                     real& work, bool& deferred, bool may_general, int lane) {
  const int n = T->n, nmj = T->nmj, nf = T->nf, cfg = T->cfg, nl = T->n_limbs;
  STAMP(3);
  // D writes, and S1's first stage reads, part i's rows on lane i only: no sync between them
  dynamics<false>(T, dt, sv, w, lane);
  STAMP(4);
  particular_sub(T, sv, w, lane);
  STAMP(5);
  // contact list in foot order (ftsolver contact columns)
  const uint32_t cmask = half_ballot(lane < nf && w.contact(0, lane));
  const int nc = __popc(cmask);
  if (lane < nf && ((cmask >> lane) & 1)) sv.cfoot[__popc(cmask & ((1u << lane) - 1))] = lane;
  wave_sync();
  int k = 3 * nc;
  uint32_t flags = 0;
  STAMP(6);
  // tier 2 (aug_solve) and the general path share the rollout's global workspace (SolveWS): the
  // general path runs only after tier 2 declined. may_general = false (the fixup's idle half) skips both
  bool fast_near = false;
  if (a.solve_mode == HS_SOLVE_AUTO && fast_solve(T, sv, fl, G->aug, w, nc, may_general, lane, fast_near)) {
    if (nc == 0) flags |= HS_FLAG_NO_CONTACT;
    if (nc == 1) flags |= HS_FLAG_FULL_RANK;
  } else {
    if constexpr (DEFER) {
      deferred = true;  // uniform over the half-wave: its outputs come from the fixup launch
      live = false;
    } else if (may_general) {
      flags = general_solve(T, sv, G->gen, w, k, lane) | HS_FLAG_GENERAL;
    }
  }
  if (fast_near) flags |= HS_FLAG_NEAR_RANK;  // the closed form's routing itself was a near decision
  STAMP(7);

  // S4: x = x_part + N y for the hinge torque rows, motor torques (periodic.cpp:328-343),
  // and the step's positive work (compute_vel_traj + work_over_period, periodic.cpp:261-307)
  const size_t row = (size_t)b * a.horizon + h;
  real tq = real(0);
  real* const wd = reinterpret_cast<WorkL&>(fl).wd;  // FastL is dead once y is known
  if (lane < nmj) {
    const int h_id = T->hinge_ids[lane], fi = T->hinge_foot[lane];  // this lane's motor's part and foot
    // contact index of foot fi: its rank among the feet down (the contact list's order)
    const int cc = (fi >= 0 && ((cmask >> fi) & 1)) ? __popc(cmask & ((1u << fi) - 1)) : -1;
    const real* Jp = w.jpos(0, h_id);
    const real* Jz = w.jz(0, h_id);
    // every operand read in one batch, without branches (a hinge with no foot in contact takes y = 0:
    // its terms are exact zeros, s stays +0 as when they were skipped)
    const real* fp = w.fpos(0, fi >= 0 ? fi : 0);
    const int yb = cc >= 0 ? 3 * cc : 0;
    real d[3], y3[3];
#pragma unroll
    for (int rr = 0; rr < 3; rr++) {
      d[rr] = Jp[rr] - fp[rr];
      const real yv = sv.y[yb + rr];
      y3[rr] = cc >= 0 ? yv : real(0);
    }
#pragma unroll
    for (int r = 0; r < 3; r++) {
      real s = real(0);
#pragma unroll
      for (int jj = 0; jj < 3; jj++)
        if (jj != r) s = s + cross_e(d, jj, r) * y3[jj];  // (d x e_r)[r] = 0: skipped
      real xr = sv.x[3 * n + 3 * h_id + r] + s;
      tq = tq + Jz[r] * xr;
    }
    real dd = w.q(1)[6 + lane] - w.q(-1)[6 + lane];
    if (dd > kPi) dd -= 2 * kPi;
    else if (dd < -kPi) dd += 2 * kPi;
    real jvel = dd / (2 * dt);
    real dw = tq * jvel;
    wd[lane] = (dw > 0) ? dw : 0;
    if (mp.pd_tau && live) {  // linear_feedback_control (player.cpp:417-432), target = get_motor_adas
      const size_t o = row * mp.st_tau + lane;
      const real q0 = w.q(0)[6 + lane];
      real a1 = inp(mp.pd_q)[o] - q0;
      if (a1 > kPi) a1 -= 2 * kPi;  // arrayops::modulus(., 2 pi) (core.cpp:122-131)
      else if (a1 <= -kPi) a1 += 2 * kPi;
      a1 *= mp.pd_k1;
      real a2 = inp(mp.pd_dq)[o] - jvel;
      a2 *= mp.pd_k2;
      a1 += a2;
      outp(mp.pd_tau)[o] = tq + a1;
      if (mp.pd_q0) outp(mp.pd_q0)[o] = q0;
      if (mp.pd_dq0) outp(mp.pd_dq0)[o] = jvel;
    }
  }
  if (live && a.tau && lane < mp.st_tau) outp(a.tau)[row * mp.st_tau + lane] = tq;  // 0 past nmj
  if (half_ballot(lane < nmj && tq != tq) || half_ballot(lane < k && sv.y[lane] != sv.y[lane])) flags |= HS_FLAG_NAN;
  if (half_ballot(lane < nl && w.unreach(0, lane))) flags |= HS_FLAG_UNREACH;
  // contact forces z = -N_cont y (ftsolver.cpp:91, 276-284)
  if (live && a.cf && lane < mp.st_cf) {
    const int fi = lane / 3, j = lane % 3;
    real zv = (lane < 3 * nf) ? -real(0) : real(0);
    if (lane < 3 * nf && ((cmask >> fi) & 1)) zv = -(real(0) + (real(-1)) * sv.y[3 * __popc(cmask & ((1u << fi) - 1)) + j]);
    outp(a.cf)[row * mp.st_cf + lane] = zv;
  }
  if (live && a.x) {  // full joint force/torque vector x += N y
    for (int rI = lane; rI < 6 * n; rI += HALF) {
      int part = (rI < 3 * n) ? rI / 3 : (rI - 3 * n) / 3, comp = rI % 3;
      real s = real(0);
      for (int c = 0; c < nc; c++) {
        int foot = T->footis[sv.cfoot[c]];
        bool anc = false;
        for (int aa = foot; aa >= 0; aa = T->node[aa].parent) anc |= (aa == part);
        if (!anc) continue;
        if (rI < 3 * n) {
          s = s + (real(-1)) * sv.y[3 * c + comp];
        } else {
          const real* ref = (T->node[part].parent >= 0) ? w.jpos(0, part) : w.pos(0, part);
          const real* fp = w.fpos(0, sv.cfoot[c]);
          real d[3];
          for (int rr = 0; rr < 3; rr++) d[rr] = ref[rr] - fp[rr];
          for (int jj = 0; jj < 3; jj++) s = s + cross_e(d, jj, comp) * sv.y[3 * c + jj];
        }
      }
      outp(a.x)[row * mp.st_x + rI] = sv.x[rI] + s;
    }
    for (int rI = 6 * n + lane; rI < mp.st_x; rI += HALF) outp(a.x)[row * mp.st_x + rI] = real(0);
  }
  if (live && a.q && lane < mp.st_q) outp(a.q)[row * mp.st_q + lane] = (lane < cfg) ? w.q(0)[lane] : real(0);
  if (live && a.dq && lane < mp.st_q) {  // compute_vel_traj (periodic.cpp:261-282)
    real v = real(0);
    if (lane < cfg) {
      real d = w.q(1)[lane] - w.q(-1)[lane];
      if (d > kPi) d -= 2 * kPi;
      else if (d < -kPi) d += 2 * kPi;
      v = d / (2 * dt);
    }
    outp(a.dq)[row * mp.st_q + lane] = v;
  }
  if (live && a.flags && lane == 0) a.flags[row] = flags;
  // the joints' positive work summed in joint order, as work_over_period's loop does (periodic.cpp:
  // 294-300; a DPP tree sum rounds differently, which can reorder near-tied rollouts' COTs)
  wave_sync();
  real work_dt = real(0);
  for (int jj = 0; jj < nmj; jj++) work_dt += wd[jj];
  // work_over_period: work_dt *= dt; work += work_dt (two roundings, periodic.cpp:301-302); fused steps
  // hand back the joint sum itself and the reduce performs the same two operations in step order
  if (mp.fused_w) work = work_dt;
  else work = work_add(work, work_dt, dt);
  STAMP(8);
  RSTAMP(17);
}

// ---------------------------------------------------------------------------
// Contact forces given motor torques: forcetorquesolver::solve_forces
// (ftsolver.cpp:331-378; oracle solve_forces). Least squares over the tree
// rows, the torso rows (torso force/torque forced to zero) and the torque rows
// jz_h . x_h = z_h, unknowns = non-root joint wrenches + forces of ALL feet.
// The tree rows' coefficient block is unit triangular, so eliminating the
// joint wrenches exactly leaves (Woodbury)
//   y = argmin (C y - d)^T (I + G G^T)^-1 (C y - d)
// over m = 6 + nmj rows: G = (torso, torque) rows composed with the tree
// inverse -- T_i = -[[I, 0], [[p_i - p_0]x, I]] for the torso, (u_hi, jz_h) with
// u_hi = (jpos_h - pos_i) x jz_h on the subtree of hinge h -- C = [I; [fpos -
// p_0]x] and jz_h . [(jpos_h - fpos)x] (the tree basis seen by those rows),
// d = (torso part of x_part, z - jz . x_part). Rank-deficient normal matrix
// (a straight leg): HS_FLAG_GENERAL and the basic solution (the dependent
// forces, in foot order, at 0: SparseQR's kind of answer, ftsolver.cpp:349-353).
// ---------------------------------------------------------------------------

__device__ inline void cross3(const real* a, const real* b, real* c) {
  c[0] = a[1] * b[2] - a[2] * b[1];
  c[1] = a[2] * b[0] - a[0] * b[2];
  c[2] = a[0] * b[1] - a[1] * b[0];
}

// Block elimination by limbs. Every hinge is a limb link and a limb's three links are its own
// subtree (the loader's topology class), so W = I + G G^T couples motors of one limb only: ordered
// (motors, torso) it is W = [[M, W_mt], [W_tm, W_tt]] with M = diag(M_l), 3 x 3 per limb, and C's motor
// rows touch only their limb's foot. With S = W_tt - W_tm M^-1 W_mt (>= I), C~ = C_t - W_tm M^-1 C_m,
// d~ = d_t - W_tm M^-1 d_m and, per foot, B_f = C_mf^T M_l^-1 C_mf, r_f = C_mf^T M_l^-1 d_m, the normal
// equations are N y = r with N = diag(B_f) + C~^T S^-1 C~, r = r_b + C~^T S^-1 d~ (the same N as
// (L^-1 C)^T (L^-1 C) for W = L L^T). When every B_f is well conditioned (LDL^T pivots above
// kForcesBlockGuard of its diagonal), the Schur complement of diag(B_f) in the KKT system gives
//   (S + sum_f C~_f B_f^-1 C~_f^T) lam = sum_f C~_f B_f^-1 r_f - d~,   y_f = B_f^-1 (r_f - C~_f^T lam),
// a 6 x 6 system (>= I); otherwise (a straight leg: B_f singular) N is formed and factorized as a
// dense 3 nf x 3 nf Cholesky, pivot guard kFastPivotGuard: a pivot under it drops its force component
// (HS_FLAG_GENERAL, the basic solution; chol_packed). Lanes: one per limb for the limb's blocks (M_l = L D L^T: every product Y_a^T D^-1 Y_b,
// Y = L^-1 [W_mt | C_m | d_m]), one per packed entry for the sums over limbs (in limb order).
constexpr real kForcesBlockGuard = HS_REAL_IS_FLOAT ? real(1e-3) : real(1e-6);
constexpr int FSUM = 27;  // packed 6 x 6 lower triangle (21) + a 6-vector

// entry e < 21 of W_tt = I + sum_{i >= 1} T_i T_i^T from s = sum r_i, Q = sum r_i r_i^T (r_i = p_i - p_0;
// T_i's torso block [[I, 0], [[r_i]x, I]]): n I; [s]x rows; (n + tr Q) I - Q
__device__ inline real wtt_entry(int e, const real* ts, int n) {
  const TriWalk<> t(e);
  const int r = t.r, c = t.c;
  if (r < 3) return (r == c) ? real(n) : real(0);
  if (c < 3) return cross_e(ts, c, r - 3);
  const int a = r - 3, b = c - 3;
  const real* q = ts + 3;  // Q00 Q11 Q22 Q01 Q02 Q12
  const real qab = (a == b) ? q[a] : q[a + b + 2];
  return ((a == b) ? real(n) + q[0] + q[1] + q[2] : real(0)) - qab;
}

// One limb's blocks of forces_solve (lane = limb), in stages both kernels share: the raw rows and M's
// LDL^T (forces_rows), the foot's C~_f / B_f / r_f (forces_foot), B_f's factor and V = L_B^-1 [C~^T | r_f]
// (forces_v). J, Z, P: the limb's three links' joint positions, axes and part positions at the centre
// sample, fp its foot, P0 the torso's position, X the links' x torque rows, zz the motors' torques.
// After forces_rows, prod(a, b) = (L^-1 R)_a^T D^-1 (L^-1 R)_b: S_l (packed lower) and e_l are prod(r, c)
// and prod(r, 9); after forces_v, vprod(a, b): K_f and q_f.
struct ForcesRows {
  real R[3][10], rdM[3];
  __device__ real prod(int a, int b) const {
    return R[0][a] * rdM[0] * R[0][b] + R[1][a] * rdM[1] * R[1][b] + R[2][a] * rdM[2] * R[2][b];
  }
};
struct ForcesV {
  real V[3][7], rdB[3];
  __device__ real vprod(int a, int b) const {
    return V[0][a] * rdB[0] * V[0][b] + V[1][a] * rdB[1] * V[1][b] + V[2][a] * rdB[2] * V[2][b];
  }
};
__device__ __attribute__((always_inline)) inline void forces_rows(ForcesRows& F, const real (&J)[3][3],
                                                                  const real (&Z)[3][3], const real (&P)[3][3],
                                                                  const real* fp, const real* P0,
                                                                  const real (&X)[3][3], const real* zz) {
  // raw rows of motor k: R[k] = (W_mt row (6), C_m row vs foot f (3), d_m (1)); M lower (k' <= k)
  real M[9];
  auto& R = F.R;
  for (int k = 0; k < 3; k++) {
    for (int c = 0; c < 10; c++) R[k][c] = 0;
    for (int c = 0; c < 3; c++) M[3 * k + c] = (c == k) ? real(1) : real(0);
  }
#pragma unroll
  for (int i = 0; i < 3; i++) {  // part p[i] lies in the subtrees of motors 0 .. i
    real ri[3], u[3][3];
    for (int t = 0; t < 3; t++) ri[t] = P[i][t] - P0[t];
#pragma unroll
    for (int k = 0; k <= i; k++) {
      real a3[3], ru[3];
      for (int t = 0; t < 3; t++) a3[t] = J[k][t] - P[i][t];
      cross3(a3, Z[k], u[k]);
      cross3(ri, u[k], ru);
      for (int c = 0; c < 3; c++) R[k][c] += -u[k][c];
      for (int c = 0; c < 3; c++) R[k][3 + c] += -(ru[c] + Z[k][c]);
#pragma unroll
      for (int k2 = 0; k2 <= k; k2++)
        M[3 * k + k2] += (u[k][0] * u[k2][0] + u[k][1] * u[k2][1] + u[k][2] * u[k2][2]) +
                         (Z[k][0] * Z[k2][0] + Z[k][1] * Z[k2][1] + Z[k][2] * Z[k2][2]);
    }
  }
#pragma unroll
  for (int k = 0; k < 3; k++) {
    real dd[3];
    for (int t = 0; t < 3; t++) dd[t] = J[k][t] - fp[t];
    for (int jj = 0; jj < 3; jj++) {
      real v = 0;
      for (int t = 0; t < 3; t++) v += Z[k][t] * cross_e(dd, jj, t);
      R[k][6 + jj] = v;
    }
    real t0 = 0;
    for (int t = 0; t < 3; t++) t0 += Z[k][t] * X[k][t];
    R[k][9] = zz[k] - t0;
  }
  ldl_n<3>(M, real(0), F.rdM);  // M >= I
#pragma unroll
  for (int c = 0; c < 10; c++) {  // Y = L^-1 R
    R[1][c] -= M[3] * R[0][c];
    R[2][c] -= M[6] * R[0][c] + M[7] * R[1][c];
  }
}
// C~_f (Ct), B_f raw (Bd) and its LDL^T (Bl / rdB), r_f (rb); returns whether B_f factors
__device__ __attribute__((always_inline)) inline bool forces_foot(const ForcesRows& F, const real* fp, const real* P0,
                                                                  real* Ct, real* Bd, real* Bl, real* rdB, real* rb) {
  real d[3];
  for (int t = 0; t < 3; t++) d[t] = fp[t] - P0[t];
#pragma unroll
  for (int r = 0; r < 6; r++)
#pragma unroll
    for (int jj = 0; jj < 3; jj++) {
      const real ct = (r < 3) ? ((r == jj) ? real(1) : real(0)) : cross_e(d, jj, r - 3);
      Ct[3 * r + jj] = ct - F.prod(r, 6 + jj);
    }
  Bd[0] = F.prod(6, 6); Bd[1] = F.prod(7, 6); Bd[2] = F.prod(7, 7);
  Bd[3] = F.prod(8, 6); Bd[4] = F.prod(8, 7); Bd[5] = F.prod(8, 8);
  for (int jj = 0; jj < 3; jj++) rb[jj] = F.prod(6 + jj, 9);
  Bl[0] = Bd[0]; Bl[3] = Bd[1]; Bl[4] = Bd[2]; Bl[6] = Bd[3]; Bl[7] = Bd[4]; Bl[8] = Bd[5];
  return ldl_n<3>(Bl, kForcesBlockGuard, rdB);
}
// K_f = C~ B^-1 C~^T, q_f = C~ B^-1 r_f, through V = L_B^-1 [C~^T | r_f]
__device__ __attribute__((always_inline)) inline void forces_v(ForcesV& G, const real* Ct, const real* Bl,
                                                               const real* rdB, const real* rb) {
  auto& V = G.V;
  for (int c = 0; c < 6; c++)
    for (int k = 0; k < 3; k++) V[k][c] = Ct[3 * c + k];
  for (int k = 0; k < 3; k++) V[k][6] = rb[k];
#pragma unroll
  for (int c = 0; c < 7; c++) {
    V[1][c] -= Bl[3] * V[0][c];
    V[2][c] -= Bl[6] * V[0][c] + Bl[7] * V[1][c];
  }
  for (int k = 0; k < 3; k++) G.rdB[k] = rdB[k];
}
// hs_rollout_kernel's form: S_l / e_l to fa, K_f / q_f to fb (its LDS ForceL rows)
__device__ __attribute__((always_inline)) inline bool forces_limb_block(const real (&J)[3][3], const real (&Z)[3][3],
                                                                        const real (&P)[3][3], const real* fp,
                                                                        const real* P0, const real (&X)[3][3],
                                                                        const real* zz, real* fa, real* fb, real* Ct,
                                                                        real* Bd, real* Bl, real* rdB, real* rb,
                                                                        real* dbgv = nullptr) {
  ForcesRows F;
  forces_rows(F, J, Z, P, fp, P0, X, zz);
  if (dbgv) { dbgv[0] = zz[0] - F.R[0][9]; dbgv[1] = zz[0]; dbgv[2] = X[0][0]; dbgv[3] = Z[0][0]; }
#pragma unroll
  for (int e = 0; e < 21; e++) {  // S_l = W_tm M^-1 W_mt (packed lower)
    const TriWalk<> t(e);
    fa[e] = F.prod(t.r, t.c);
  }
#pragma unroll
  for (int r = 0; r < 6; r++) fa[21 + r] = F.prod(r, 9);  // e_l = W_tm M^-1 d_m
  const bool okB = forces_foot(F, fp, P0, Ct, Bd, Bl, rdB, rb);
  if (okB) {
    ForcesV G;
    forces_v(G, Ct, Bl, rdB, rb);
#pragma unroll
    for (int e = 0; e < 21; e++) {
      const TriWalk<> t(e);
      fb[e] = G.vprod(t.r, t.c);
    }
#pragma unroll
    for (int r = 0; r < 6; r++) fb[21 + r] = G.vprod(r, 6);
  }
  return okB;
}

template <class W, class SV>
__device__ __attribute__((always_inline)) inline uint32_t forces_solve(const hs_topo* T, SV& sv, ForceL& fr, const W& w,
                                                                       const real* z, bool dense, int lane) {
  const int n = T->n, nl = T->n_limbs, nq = 3 * T->nf;
  const real* P0 = w.pos(0, 0);
  real* ts = sv.y;  // the 9 part sums until y is written
  if (lane < 9) {   // s (3), Q (6)
    const int a = lane < 3 ? lane : (lane < 6 ? lane - 3 : (lane == 6 ? 0 : (lane == 7 ? 0 : 1)));
    const int b = lane < 6 ? (lane < 3 ? -1 : lane - 3) : (lane == 6 ? 1 : 2);
    real s = 0;
    for (int i = 1; i < n; i++) {
      const real* Pi = w.pos(0, i);
      const real ra = Pi[a] - P0[a];
      s += (b < 0) ? ra : ra * (Pi[b] - P0[b]);
    }
    ts[lane] = s;
    if (lane == 3) DBG(0, s, 30);
  }
  // per limb: C~_f (6 x 3), B_f (raw and LDL^T), r_f stay in registers to the end
  real Ct[18], Bd[6], Bl[9], rdB[3], rb[3];
  int f = 0;
  bool okB = true;
  if (lane < nl) {
    const int L = lane;
    int p[3];
    for (int k = 0; k < 3; k++) p[k] = T->limb_node[L][k];
    f = T->node[p[2]].foot;
    real J[3][3], Z[3][3], P[3][3], X[3][3], zz[3];
    for (int k = 0; k < 3; k++) {
      for (int t = 0; t < 3; t++) {
        J[k][t] = w.jpos(0, p[k])[t];
        Z[k][t] = w.jz(0, p[k])[t];
        P[k][t] = w.pos(0, p[k])[t];
        X[k][t] = sv.x[3 * n + 3 * p[k] + t];
      }
      zz[k] = z[T->node[p[k]].hinge];
    }
#ifdef HS_DBG
    real dbgv[4] = {0, 0, 0, 0};
    okB = forces_limb_block(J, Z, P, w.fpos(0, f), P0, X, zz, fr.a[L], fr.b[L], Ct, Bd, Bl, rdB, rb, dbgv);
    DBG(24 + f, dbgv[0], 40);
    DBG(24 + f, dbgv[1], 41);
    DBG(24 + f, dbgv[2], 42);
    DBG(24 + f, dbgv[3], 43);
#else
    okB = forces_limb_block(J, Z, P, w.fpos(0, f), P0, X, zz, fr.a[L], fr.b[L], Ct, Bd, Bl, rdB, rb);
#endif
    DBG(24 + f, fr.a[L][0], 31);
    DBG(24 + f, fr.b[L][0], 32);
    DBG(24 + f, Ct[0], 36);
    DBG(24 + f, rb[0], 37);
    DBG(24 + f, fr.a[L][21], 38);
  }
  const bool fast = !dense && half_ballot(lane < nl && !okB) == 0;
  wave_sync();
  STAMP(4);
  if (lane < FSUM) {  // sums over the limbs, in limb order; W_tt and the torso part of d added
    real s = 0;
    for (int L = 0; L < nl; L++) s += fast ? ((lane < 21) ? fr.b[L][lane] - fr.a[L][lane] : fr.b[L][lane] + fr.a[L][lane])
                                          : fr.a[L][lane];
    const real dt = (lane < 21) ? real(0) : (lane < 24 ? sv.x[lane - 21] : sv.x[3 * n + lane - 24]);
    // fast: K = W_tt - sum S_l + sum K_f, rhs = sum (q_f + e_l) - d_t; else S = W_tt - sum S_l, d~ = d_t - sum e_l
    const real v = (lane < 21) ? (fast ? wtt_entry(lane, ts, n) + s : wtt_entry(lane, ts, n) - s)
                               : (fast ? s - dt : dt - s);
    fr.a[0][lane] = v;  // lane reads column `lane` only, so slot 0 takes the sums in place
    if (lane == 0) DBG(1, v, 33);
  }
  wave_sync();
  STAMP(5);
  uint32_t flags = 0;
  if (fast) {
    real K[36], rd[6], lam[6];
#pragma unroll
    for (int r = 0; r < 6; r++) {
#pragma unroll
      for (int c = 0; c < 6; c++) K[6 * r + c] = (c <= r) ? fr.a[0][pk(r, c)] : real(0);
      lam[r] = fr.a[0][21 + r];
    }
    ldl_n<6>(K, real(0), rd);  // >= I
    ldl_solve_n<6>(K, rd, lam);
    if (lane == 0) DBG(2, lam[0], 34);
    if (lane < nl) {  // y_f = B_f^-1 (r_f - C~_f^T lam)
      real t[3];
      for (int k = 0; k < 3; k++) {
        real s = rb[k];
        for (int r = 0; r < 6; r++) s -= Ct[3 * r + k] * lam[r];
        t[k] = s;
      }
      ldl_solve_n<3>(Bl, rdB, t);
      DBG(24 + f, t[0], 35);
      for (int k = 0; k < 3; k++) sv.y[3 * f + k] = t[k];
    }
    wave_sync();
    STAMP(9);
    return flags;
  }
  // dense normal equations over the feet (a B_f near singular): N = diag(B_f) + V^T D_S^-1 V with
  // S = L_S D_S L_S^T, V = L_S^-1 C~, r = r_b + V^T D_S^-1 L_S^-1 d~
  real* const base = &fr.a[0][0];
  real* const Vm = base + FSUM;       // [6][HS_KMAX]
  real* const vv = Vm + 6 * HS_KMAX;  // 6
  real* const rdS = vv + 6;           // 6
  real* const N = rdS + 6;            // packed lower, nq x nq
  real* const rr = N + HS_KMAX * (HS_KMAX + 1) / 2;
  {
    real S[36], rd[6], v6[6];
#pragma unroll
    for (int r = 0; r < 6; r++) {
#pragma unroll
      for (int c = 0; c < 6; c++) S[6 * r + c] = (c <= r) ? base[pk(r, c)] : real(0);
      v6[r] = base[21 + r];
    }
    ldl_n<6>(S, real(0), rd);  // >= I
    for (int i = 0; i < 6; i++) {
      real s = v6[i];
      for (int k = 0; k < i; k++) s -= S[6 * i + k] * v6[k];
      v6[i] = s;
    }
    if (lane < nl) {
      for (int jj = 0; jj < 3; jj++) {
        real col[6];
        for (int i = 0; i < 6; i++) {
          real s = Ct[3 * i + jj];
          for (int k = 0; k < i; k++) s -= S[6 * i + k] * col[k];
          col[i] = s;
        }
        for (int i = 0; i < 6; i++) Vm[i * HS_KMAX + 3 * f + jj] = col[i];
      }
    }
    if (lane == 0)
      for (int i = 0; i < 6; i++) {
        vv[i] = v6[i];
        rdS[i] = rd[i];
      }
  }
  wave_sync();
  for (TriWalk<1> t(lane); t.r < nq; t.next()) {  // V^T D^-1 V and its rhs, entry by entry
    const int p = t.r, q = (t.c == p + 1) ? nq : t.c;
    real s = 0;
    for (int k = 0; k < 6; k++) s += Vm[k * HS_KMAX + p] * rdS[k] * ((q < nq) ? Vm[k * HS_KMAX + q] : vv[k]);
    if (q < nq) N[pk(p, q)] = s;
    else rr[p] = s;
  }
  wave_sync();
  if (lane < nl) {  // + the feet's own blocks
    const int q0 = 3 * f;
    N[pk(q0, q0)] += Bd[0];
    N[pk(q0 + 1, q0)] += Bd[1];
    N[pk(q0 + 1, q0 + 1)] += Bd[2];
    N[pk(q0 + 2, q0)] += Bd[3];
    N[pk(q0 + 2, q0 + 1)] += Bd[4];
    N[pk(q0 + 2, q0 + 2)] += Bd[5];
    for (int k = 0; k < 3; k++) rr[q0 + k] += rb[k];
  }
  wave_sync();
  bool rank_near = false;  // a rank decision within kNearBand of the guard (HS_FLAG_NEAR_RANK)
  const uint32_t dropped = chol_packed(N, nq, kFastPivotGuard, lane, rank_near);
  if (dropped) flags = HS_FLAG_GENERAL | HS_FLAG_DEPENDENT;  // least squares not unique: its basic solution
  if (rank_near) flags |= HS_FLAG_NEAR_RANK;
  STAMP(8);
  if (lane == 0) {  // the two triangular solves with y in registers (nq <= HS_KMAX)
    real yv[HS_KMAX];
#pragma unroll
    for (int i = 0; i < HS_KMAX; i++) yv[i] = (i < nq) ? rr[i] : real(0);
#pragma unroll
    for (int i = 0; i < HS_KMAX; i++) {
      if (i < nq) {
        real s = yv[i];
#pragma unroll
        for (int k = 0; k < i; k++) s -= N[pk(i, k)] * yv[k];
        yv[i] = ((dropped >> i) & 1) ? real(0) : s / N[pk(i, i)];
      }
    }
#pragma unroll
    for (int i = HS_KMAX - 1; i >= 0; i--) {
      if (i < nq) {
        real s = yv[i];
#pragma unroll
        for (int k = i + 1; k < HS_KMAX; k++)
          if (k < nq) s -= N[pk(k, i)] * yv[k];
        yv[i] = ((dropped >> i) & 1) ? real(0) : s / N[pk(i, i)];
      }
    }
#pragma unroll
    for (int i = 0; i < HS_KMAX; i++)
      if (i < nq) sv.y[i] = yv[i];
  }
  wave_sync();
  STAMP(9);
  return flags;
}

template <class W, class SV>
__device__ __attribute__((always_inline)) inline void forces_step(const hs_topo* T, const hs_run_args& a, const hs::launch_map& mp, real dt,
                            SV& sv, ForceL& fr, const W& w, int b, bool live, int h, int lane) {
  const int nf = T->nf, cfg = T->cfg, nl = T->n_limbs, nq = 3 * nf;
  dynamics(T, dt, sv, w, lane);
  // the control step's subtree sums (round 6: the level-by-level recursion summed x in another order,
  // so the forces mode's x differed from the control step's -- and the limb-lane kernel's -- by rounding)
  particular_sub(T, sv, w, lane);
  wave_sync();  // particular_sub leaves x unsynchronised across lanes; forces_solve reads it across lanes
  STAMP(10);
  const size_t row = (size_t)b * a.horizon + h;
  const real* z = inp(mp.tau_in) + (live ? row : 0) * mp.st_tau;
  uint32_t flags = forces_solve(T, sv, fr, w, z, a.solve_mode == HS_SOLVE_REFERENCE, lane);
  if (half_ballot(lane < nq && sv.y[lane] != sv.y[lane])) flags |= HS_FLAG_NAN;
  if (half_ballot(lane < nl && w.unreach(0, lane))) flags |= HS_FLAG_UNREACH;
  if (live && a.cf && lane < mp.st_cf) outp(a.cf)[row * mp.st_cf + lane] = (lane < nq) ? sv.y[lane] : real(0);
  if (live && a.q && lane < mp.st_q) outp(a.q)[row * mp.st_q + lane] = (lane < cfg) ? w.q(0)[lane] : real(0);
  if (live && a.flags && lane == 0) a.flags[row] = flags;
  STAMP(11);
}

// Global per-rollout workspace: the general path's scratch, and the call's gait setup record, sample
// times, straight-gait frames and IK table, stored by the call's preparation pass (hs_prep_kernel) for
// every step launch of the call.
#ifndef HS_KTAB
#define HS_KTAB 64  // table rows: the samples [ktab_lo, ktab_lo + n) a call's steps read (hs::ktab_range)
#endif
struct RolloutWS {
  SolveWS sol;
  SetupL st;
  real t_tab[HS_KTAB];  // sample times of the call's rows (sample_time): t_tab[r] = t_(ktab_lo + r)
  KinFrames kf;         // a straight gait's frames
  real ktab[HS_KTAB][HS_LMAX][KT_W];  // limb L's joint values at sample ktab_lo + r
  real ktor[HS_KTAB][KR_W];           // turning or transformed gaits: the torso at sample ktab_lo + r
  uint8_t kbad[HS_KTAB][HS_LMAX];     // 1: ktab[r][L]'s limb IK unreachable or failed
};
static_assert(sizeof(SetupL) % sizeof(real) == 0, "SetupL is copied as reals");

// ---------------------------------------------------------------------------
// The call's preparation pass (hs_prep_kernel): the gait setup of every rollout (pergensetup::
// setup_pergen, pergen.cpp:453-507), its sample times (periodic.cpp:171-181) and the IK table of the
// samples the call's steps read (with, for turning or transformed gaits, the torso record) -- in one launch.
//
// Lane = (rollout, limb L, chunk of HS_PREP_ROWS table rows). Every lane runs its limb's setup (torso
// frame, chain, hip frame J0, default foot position, lift-off entries) itself -- the lanes of one
// wavefront do it in the same instructions, so the repetition costs one pass per wavefront -- and then
// the rows of its chunk: the sample time, and for a straight gait J = J0 advanced by t v along the
// torso's x and the limb IK at the foot target (straight_ik's operations); for a turning or transformed
// gait kin_sample's record, torso FK, chain and limb IK, the torso's q6 and frame stored per row
// (RolloutWS::ktor, lane L = 0). The chunk-0 lanes store the
// setup record; max_radius (compute_max_radius, curved gaits) is the maximum over a rollout's limb
// lanes, exchanged in LDS. A rollout's limb lanes form a group that never crosses a wavefront (groups of
// nli lanes, floor(64 / nli) per wavefront). XCD-aware: block 8 jb + x runs groups of batch wavefronts
// w = x (mod 8), whose step launches run on XCD x (blocks are dealt round-robin over the 8 XCDs,
// MI355X_MICROARCH.md), so the record and rows are written into the L2 the steps read them from.
// ---------------------------------------------------------------------------
#ifndef HS_PREP_ROWS
#define HS_PREP_ROWS 5  // table rows per lane (round 4, B = 4096, 24 rows: 3, 4, 5, 6, 8 rows give 24.1, 25.0, 23.4, 24.9, 29.7 us)
#endif
#ifndef HS_PREP_WAVES
#define HS_PREP_WAVES 2  // waves per SIMD (251 VGPRs, 255 mixed, no scratch; at 3, 168 VGPRs and 336 B of spills: tools/isa_stats.py)
#endif
#ifndef HS_PREP_WPB
#define HS_PREP_WPB 4  // wavefronts per workgroup (each a group of lanes of its own: only wave-local exchanges);
                       // 4: the pass's wavefronts start sooner, 22.9 -> 20.5 us per driver job (r05_ab_t2.txt)
#endif
// an exchange through LDS among the lanes of one wavefront: LDS operations of a wavefront complete in
// order, so only the compiler must not move the accesses across it (no s_barrier: with several
// wavefronts per workgroup they take different paths)
__device__ inline void wave_lds_sync() {
#if HS_PREP_WPB == 1
  wave_sync();
#else
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
#endif
}
__device__ inline int ktab_lanes(const hs::launch_map& mp) { return mp.ktab_nl > 0 ? mp.ktab_nl : HS_LMAX; }
__host__ __device__ inline int prep_chunks(int ttab_n) { return (ttab_n > 0 ? ttab_n + HS_PREP_ROWS - 1 : HS_PREP_ROWS) / HS_PREP_ROWS; }
// XCD units of the pass: prep_unit rollouts each (2: hs_rollout_kernel's wavefronts, 8: the limb kernel's)
__host__ __device__ inline int prep_units(const hs::launch_map& mp, int n_rollouts, int& R) {
  R = mp.prep_unit > 2 && !mp.wave_rollouts ? mp.prep_unit : 2;
  return R == 2 ? mp.n_waves : (n_rollouts + R - 1) / R;
}
__host__ __device__ inline int64_t prep_blocks(int n_units, int R, int ttab_n, int nli) {
  const int64_t groups_per_xcd = R * (int64_t)prep_chunks(ttab_n) * ((n_units + 7) / 8);
  const int gpw = WAVE / nli;
  const int64_t waves_per_xcd = (groups_per_xcd + gpw - 1) / gpw;
  return 8 * ((waves_per_xcd + HS_PREP_WPB - 1) / HS_PREP_WPB);
}

// MIXED: a mixed-topology launch (launch_map::wave_model), whose lane groups of one wavefront may hold
// different models; otherwise the topology pointer is the kernel argument itself, wave-uniform, so its
// rollout-independent entries come through the scalar cache
template <bool MIXED>
__global__ __launch_bounds__(WAVE * HS_PREP_WPB, HS_PREP_WAVES) void hs_prep_kernel(const hs_topo* __restrict__ T0,
                                                                   hs_run_args a, RolloutWS* __restrict__ rws,
                                                                   hs::launch_map mp) {
  __shared__ real rad_s[HS_PREP_WPB][WAVE];
  __shared__ real q6s_s[HS_PREP_WPB][HS_PREP_ROWS][6][WAVE / 4];  // turning rows: [row][q6 entry][group] (>= 4 limbs)
  __shared__ real tgs_s[HS_PREP_WPB][HS_PREP_ROWS][3][WAVE];      // [row][target entry][lane]
  const int wv = (int)threadIdx.x / WAVE, tl = (int)threadIdx.x % WAVE;  // wavefront in the block, its lane
  real(&rad)[WAVE] = rad_s[wv];
  real(&q6s)[HS_PREP_ROWS][6][WAVE / 4] = q6s_s[wv];
  real(&tgs)[HS_PREP_ROWS][3][WAVE] = tgs_s[wv];
  RSTAMP(29);
  STAMP(24);
  if (blockIdx.x == 0)  // the call's fixup counters, before its step launches append to them
    for (int i = threadIdx.x; i < mp.fix_n_counts; i += blockDim.x) mp.fix_count[i] = 0;
  const int nli = ktab_lanes(mp), gpw = WAVE / nli;
  const int C = prep_chunks(mp.ttab_n);
  const int gl = tl / nli, L = tl % nli;
  // group (q, sub, chunk) in XCD x's sequence (x = blockIdx.x % 8: the block's XCD)
  const int gi = ((int)(blockIdx.x / 8) * HS_PREP_WPB + wv) * gpw + gl;
  int R;
  const int n_units = prep_units(mp, a.n_rollouts, R);
  const int chunk = gi % C, sub = (gi / C) % R, w = 8 * (gi / (R * C)) + (int)(blockIdx.x % 8);
  bool on = gl < gpw && w < n_units;
  int b = 0;
  const hs_topo* __restrict__ T = T0;
  if (on) {
    b = mp.wave_rollouts ? mp.wave_rollouts[2 * w + sub] : R * w + sub;
    if (MIXED) T = T0 + mp.wave_model[w];
    on = b >= 0 && b < a.n_rollouts && L < T->n_limbs;
  }
  GaitR g;
  A34 J0;
  real pos0[3], ts = 0, xs = 0, t_step = 0, dt = 0, v = 0;
  bool straight = false;
  real my_rad = 0;
  SC3 tsc;
  RolloutWS* __restrict__ ws = rws + b;
  LimbPlan plan;
  if (on) {
    plan = load_plan(T, L);  // issued before the gait parameters: its waits do not queue behind them
    g = load_gait(a.params[b]);
    straight = g.curvature == 0 && !g.rec_xf;  // kin_sample's turning / record-transform test
    const int nl = T->n_limbs, j = T->limb_pergen[L];
    tsc = sincos3(g.torso_angles[0], g.torso_angles[1], g.torso_angles[2]);
    const A34 A0 = torso_frame(T, g, tsc);
    limb_setup(T, g, A0, L, plan, J0, pos0, chunk == 0 ? &ws->kf : nullptr);
    t_step = step_fraction(g, nl);
    lift_off(nl, j, t_step, ts, xs);
    v = g.step_length / g.period;  // pergensetup::set_TLh
    dt = g.period / a.n_t;         // record_trajectory
    if (chunk == 0) {
      SetupL& st = ws->st;
      for (int i = 0; i < 3; i++) st.pos0[j][i] = pos0[i];
      st.ts[j] = ts;
      st.xs[j] = xs;
      if (L == 0) {
        st.t_step = t_step;
        st.v = v;
        st.dt = dt;
        st.tsc = tsc;
        const real com0[3] = {(real)T->node[0].com[0], (real)T->node[0].com[1], (real)T->node[0].com[2]};
        store_body(A0, com0, ws->kf.torso, 6);
      }
    }
    if (g.curvature != 0) my_rad = turn_radius(pos0, g.curvature);
  }
  STAMP(25);
  rad[tl] = my_rad;
  wave_lds_sync();
  real mr = 0;  // compute_max_radius over the rollout's limbs (every lane: turning rows read it)
  if (on && g.curvature != 0)
    for (int l = 0; l < T->n_limbs; l++) {
      const real r = rad[tl - L + l];
      if (r > mr) mr = r;
    }
  if (on && chunk == 0 && L == 0) ws->st.max_radius = mr;
  STAMP(26);
  if (!on) return;
  const int r0 = chunk * HS_PREP_ROWS, r1 = min(r0 + HS_PREP_ROWS, mp.ttab_n);
  if (r0 >= r1) return;
  const bool table = mp.ktab_n > 0;
  const hs_aff34& Jp0 = T->node[0].J_A_parent;
  const real u[3] = {(real)Jp0.m[0], (real)Jp0.m[1], (real)Jp0.m[2]};
  const real ls[3] = {(real)T->ls[0], (real)T->ls[1], (real)T->ls[2]};
  const int kind = T->lik_kind;
  const bool ir = a.ignore_reach != 0;
  auto store_row = [&](int r, const real* ja, bool bad) {
    real* e = ws->ktab[r][L];
#pragma unroll
    for (int kk = 0; kk < 3; kk++) e[kk] = ja[kk];
    ws->kbad[r][L] = bad ? 1 : 0;
  };
  real t = sample_time_sum(dt, mp.ktab_lo + r0);
  // kin_sample's foot target, hip frame and limb IK at samples ktab_lo + r, one loop per kind of gait
  // (a lane's kind is fixed: the other loop's values are not live in this one)
  if (!table || straight) {
#pragma unroll 1
    for (int r = r0; r < r1; r++) {
      if (r > r0) t += dt;  // the loop's next addition
      if (L == 0) ws->t_tab[r] = t;
      if (table) {  // straight_ik's: J = J0 advanced by t v
        real dx, dz;
        limb_step(g, t, ts, xs, t_step, dx, dz);
        const real target[3] = {dx + pos0[0], real(0) + pos0[1], dz + pos0[2]};
        real ja[3];
        bool bad;
        hip_ik_k(frame_at(J0, u, t * v), target, kind, ls, plan.ysign, ir, ja, bad);
        store_row(r, ja, bad);
      }
      if (r == r0) STAMP(27);
    }
  } else {
    // turning or transformed gaits (kin_sample's sequence), in two passes over the rows so that the gait
    // record's values and the FK + IK's are not live together: (1) the record: the torso's q6 (lane L = 0,
    // per group) and the foot targets to LDS; (2) the torso FK (free_joint: sincos of the configured
    // angles when not turned, as free_joint_sc with the setup's), the chain, the hip frame, the limb IK
    const LimbRec rl{v, t_step, mr, ts, xs, {pos0[0], pos0[1], pos0[2]}, tsc};
    const hs_gait_params& gp = a.params[b];
#pragma unroll 1
    for (int r = r0; r < r1; r++) {
      if (r > r0) t += dt;
      if (L == 0) ws->t_tab[r] = t;
      real o0[3], o1[3], target[3];
      bool turned;
      gait_record<false>(g, gp, rl, t, o0, o1, turned, target);
      if (L == 0) {
        const real q6[6] = {o0[0], o0[1], o0[2], o1[0], o1[1], o1[2]};
        for (int i = 0; i < 6; i++) q6s[r - r0][i][gl] = q6[i];
      }
      for (int i = 0; i < 3; i++) tgs[r - r0][i][tl] = target[i];
    }
    wave_lds_sync();
#pragma unroll 1
    for (int r = r0; r < r1; r++) {
      real q6[6], target[3];
      for (int i = 0; i < 6; i++) q6[i] = q6s[r - r0][i][gl];
      for (int i = 0; i < 3; i++) target[i] = tgs[r - r0][i][tl];
      const A34 A0 = mul(mul(node_joint_parent(T, 0), free_joint(q6)), node_pj(T, 0));
      if (L == 0) {  // the torso record the step launches read (kin_sample_tab)
        real* tr = ws->ktor[r];
        for (int i = 0; i < 6; i++) tr[i] = q6[i];
        store34r(A0, tr + 6);
      }
      A34 A = A0;
      for (int k = 1; k < T->limb_chain_len[L]; k++) A = mul(A, node_pj(T, T->limb_chain[L][k]));
      real ja[3];
      bool bad;
      hip_ik(T, L, mul(A, node_joint_parent(T, T->limb_child[L])), target, ir, ja, bad);
      store_row(r, ja, bad);
      if (r == r0) STAMP(27);
    }
  }
  STAMP(28);
  RSTAMP(30);
}

// One wavefront's step: fused step fstep (0 outside fused launches) of batch wavefront wid. only_sub
// >= 0 (the fixup launch): only that half stores, the other computes a copy and stores nothing.
template <int NM, bool FORCES, bool DEFER>
__device__ __attribute__((always_inline)) inline void rollout_wave(const hs_topo* __restrict__ T0, const hs_run_args& a,
                                                                   RolloutWS* __restrict__ rws, const hs::launch_map& mp,
                                                                   Smem<NM, FORCES>* smem, int fstep, int wid,
                                                                   int only_sub) {
  const int sub = threadIdx.x / HALF;  // rollout slot within the wave
  const int lane = threadIdx.x % HALF; // lane within the rollout
  // one model per wavefront: the topology pointer stays wave-uniform (scalar loads)
  // (indexing the kernel argument keeps T a known-global pointer: global_load, not flat_load)
  const hs_topo* __restrict__ T = mp.wave_model ? T0 + mp.wave_model[wid] : T0;
  int b, bb;
  bool live;  // an idle half (odd group) computes a copy of its neighbour and stores nothing
  if (mp.wave_rollouts) {
    b = mp.wave_rollouts[2 * wid + sub];
    live = b >= 0;
    bb = live ? b : mp.wave_rollouts[2 * wid];
  } else {
    b = wid * 2 + sub;
    live = b < a.n_rollouts;
    bb = live ? b : a.n_rollouts - 1;
  }
  // fixup: the neighbour's step is already stored; that half runs along without storing and without
  // the general path, whose workspace (the idle slot) the fixup's other wavefronts would share
  const bool fix_idle = only_sub >= 0 && sub != only_sub;
  if (fix_idle) {
    bb = live ? b : bb;
    live = false;
  }
  SolveWS* G = mp.fused_gen ? &((SolveWS*)mp.fused_gen)[(size_t)fstep * (a.n_rollouts + 1) + (live ? b : a.n_rollouts)]
                            : &rws[live ? b : a.n_rollouts].sol;
  Smem<NM, FORCES>& sm = smem[sub];
  SolveRef sv;
  if constexpr (FORCES) {
    sv.f = sm.sv.xy.f;
    sv.x = sm.sv.xy.x;
    sv.y = sm.sv.xy.y;
  } else {
    sv.f = sm.d.post.f;
    sv.x = sm.d.post.x;
    sv.y = sm.d.post.y;
  }
  sv.cfoot = sm.sv.cfoot;
  sv.fch = sm.sv.fch;
  real work = (live && a.accumulate && a.work_cot && !mp.fused_w) ? outp(a.work_cot)[2 * (size_t)b] : real(0);
  int k0 = a.k0, h_row = mp.h_row;
  if (mp.fused_w) {
    const int s = mp.fused_s0 + fstep, c = s / mp.fused_h;
    k0 = (int)(((int64_t)a.k0 + (int64_t)c * mp.fused_h) % a.n_t) + s % mp.fused_h;
    h_row = s;
  }
#ifdef HS_DBG
  if (lane == 0) dbg_rows()[sub] = live ? b * a.horizon + h_row : -1;
  wave_sync();
#endif
  const int nl = T->n_limbs;
  // the gait setup of the rollout, stored by the call's preparation pass (hs_prep_kernel;
  // the idle half reads its neighbour's): read from global memory where it is used
  const SetupL& st = rws[bb].st;
  const int i = k0 + 2;  // centre sample of this launch's step
  const int sl = lane / nl, L = lane % nl;
  const real* kt = mp.ktab_n > 0 ? &rws[bb].ktab[0][0][0] : nullptr;
  const uint8_t* kb = &rws[bb].kbad[0][0];
#if HS_PRELOAD
  const StraightPre pre = straight_preload(st, rws[bb].t_tab, rws[bb].kf, HS_KTE_PRELOAD ? kt : nullptr, kb,
                                           i - 2 + (sl < NS ? sl : 0), mp.ktab_lo, mp.ttab_n, L);
#endif
  const real dt = st.dt;
  // the gait's kind from two of its parameters; the whole record (GaitR) is loaded only on the paths that
  // read it, so that it is not held in registers (at 4 waves/SIMD: spilled) across the step
  const hs_gait_params& gp = a.params[bb];
  const bool ignore_reach = a.ignore_reach != 0;
  const bool straight = (real)gp.curvature == 0 && !gp.rec_transform_flag;
#if HS_CURVED_LDS
  // a wave with a turning or transformed gait: the record in LDS for the turning path's many reads
  if (!kt && __ballot(!straight)) {
    constexpr int NW = sizeof(SetupL) / sizeof(real);
    const real* cache = reinterpret_cast<const real*>(&rws[bb].st);
    real* lds = reinterpret_cast<real*>(&smem[sub].st);
    for (int e = lane; e < NW; e += HALF) lds[e] = cache[e];
    wave_sync();
  }
  const SetupL& st_curved = smem[sub].st;
#else
  const SetupL& st_curved = st;
#endif

  STAMP(0);
  STAMP(1);

  // K: the five-sample window, lane = (sample, limb)
  {
    const real* t_tab = rws[bb].t_tab;
    // a straight, untransformed gait (the common case): its frames from the setup pass, its joint
    // values from the call's IK table when there is one (kin_sample_straight)
    if (sl < NS) {
      if (straight) {
#if !HS_PRELOAD
        const StraightPre pre = straight_preload(st, t_tab, rws[bb].kf, HS_KTE_PRELOAD ? kt : nullptr, kb,
                                                 i - 2 + sl, mp.ktab_lo, mp.ttab_n, L);
#endif
        kin_sample_straight(T, gp, st, i - 2 + sl, L, ignore_reach, OneWin<NM, FORCES>{&sm.d}, sl - 2,
                            pre, rws[bb].kf, kt, kb, mp.ktab_lo);
      } else if (kt) {  // a turning or transformed gait with the call's tables
        const int r = i - 2 + sl - mp.ktab_lo;
#if HS_PRELOAD && HS_KTE_PRELOAD
        const real* kte = pre.kte;
        const bool kbad = pre.bad;
#else
        const real* kte = kt + ((size_t)r * HS_LMAX + L) * KT_W;
        const bool kbad = kb[r * HS_LMAX + L] != 0;
#endif
        kin_sample_tab(T, L, OneWin<NM, FORCES>{&sm.d}, sl - 2, rws[bb].ktor[r], kte, kbad);
      } else {
        kin_sample<false>(T, load_gait(gp), gp, st_curved, i - 2 + sl, L, ignore_reach, OneWin<NM, FORCES>{&sm.d},
                          sl - 2, t_tab, mp.ktab_lo, mp.ttab_n);
      }
    }
    // the foot chains (hs_topo::foot_chain8), to LDS with the kinematics' stores: the contact blocks then
    // read them there instead of through two dependent global loads
    if (!FORCES && lane < 2 * HS_LMAX) (&sv.fch[0][0])[lane] = (&T->foot_chain8[0][0])[lane];
    wave_sync();
  }
  STAMP(2);
  if constexpr (FORCES) {
    forces_step(T, a, mp, dt, sv, sm.d.post, OneWin<NM, FORCES>{&sm.d}, b, live, h_row, lane);
    return;
  } else {
    bool deferred = false;
    step<DEFER>(T, a, mp, dt, sv, sm.d.post.fl, OneWin<NM, FORCES>{&sm.d}, G, b, live, h_row, work,
                deferred, !fix_idle, lane);
    if (DEFER && deferred) {  // the fixup launch solves this (step, rollout) with the general path
      if (lane == 0 && live) {
        const int it = atomicAdd(mp.fix_count, 1);
        mp.fix_items[2 * it] = fstep;
        mp.fix_items[2 * it + 1] = 2 * wid + sub;
      }
      return;
    }
  }
  if (DEFER || mp.fused_w) {  // this step's joint sum of positive work, summed over the steps in order by the reduce
    if (lane == 0 && live)
      reinterpret_cast<real*>(mp.fused_work)[(size_t)(mp.fused_s0 + fstep) * a.n_rollouts + b] = work;
    return;
  }
  const bool out = lane == 0 && live;
  if (out && a.work_cot) {
    real cot = work / ((real)T->total_mass * (real)gp.step_length);
    outp(a.work_cot)[2 * (size_t)b] = work;
    outp(a.work_cot)[2 * (size_t)b + 1] = cot;
  }
  if (a.best_key) {
    unsigned long long key = ~0ull;
    if (out) key = best_key(key_cot(work, (real)T->total_mass, (real)gp.step_length, a.n_t, a.key_steps), a.rollout_id_base + b);
    if constexpr (!DEFER) {  // both rollouts of the wave are here: their minimum first
      const unsigned long long o = __shfl_xor(key, HALF);
      key = o < key ? o : key;
    }
    // The key only decreases, so any value read from it bounds the final minimum from above: a key not
    // below it cannot win, and skipping its atomic keeps the last launch from queueing one atomic per
    // wave on a single address (~20 us per call at B = 4096)
    if ((DEFER ? lane : (int)threadIdx.x) == 0 && key != ~0ull &&
        key < __hip_atomic_load((unsigned long long*)a.best_key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
      atomicMin((unsigned long long*)a.best_key, key);
  }
}

// A fused launch's block -> (local step, batch wavefront): groups of HS_FUSED_GROUP batch wavefronts
// (a multiple of 8, so a wavefront's steps stay on its XCD, block % 8), each group's steps in order,
// the group's wavefronts fastest. A rollout's steps then run close together in time, and its setup
// record, frames and table rows, read by every step, are fetched into the XCD's L2 once per call
// instead of once per sweep of the whole batch over a step (whose output stores evict them).
// Exception: the last group, gw = W - g0 wavefronts, is narrower when W is not a multiple of
// HS_FUSED_GROUP, and when gw is not a multiple of 8 either its wavefronts change XCD from step to step
// (a locality loss only; every step is independent, outputs are unaffected). The BASELINE shapes have
// none: W = 2048 (configs[1], [4]), 8192 (configs[2]), 16384 (configs[3]'s shard)
#ifndef HS_FUSED_GROUP
#define HS_FUSED_GROUP 256
#endif
template <int GROUP = HS_FUSED_GROUP>
__device__ inline void fused_coords(int blk, int W, int n, int& fstep, int& wid) {
  if constexpr (GROUP > 0) {
    const int q = blk / (GROUP * n), g0 = q * GROUP;
    const int gw = W - g0 < GROUP ? W - g0 : GROUP;  // the last group may be narrower
    const int r = blk - g0 * n;
    fstep = r / gw;
    wid = g0 + r % gw;
  } else {
    fstep = blk / W;
    wid = blk % W;
  }
}

// MODE (hs::FIX_*): NONE, the step with the general path out of line; DEFER, the fused step launch
// without it; SOLVE, the fixup launch over the deferred items (its own instantiation, so the loop
// costs the other two nothing)
template <int NM, bool FORCES, int MODE>
__global__ __launch_bounds__(WAVE, FORCES ? HS_MIN_WAVES_FORCES
                                                 : (HS_REAL_IS_FLOAT ? (MODE == hs::FIX_DEFER ? HS_MIN_WAVES_F32_DEFER : HS_MIN_WAVES_F32)
                                                                     : (MODE == hs::FIX_DEFER ? HS_MIN_WAVES_DEFER : HS_MIN_WAVES))) void hs_rollout_kernel(const hs_topo* __restrict__ T0,
                                                                                 hs_run_args a, RolloutWS* __restrict__ rws,
                                                                                 hs::launch_map mp) {
  __shared__ Smem<NM, FORCES> smem[2];
  RSTAMP(16);
  STAMP(15);
  if constexpr (MODE == hs::FIX_SOLVE) {  // the deferred (step, rollout) items
    const int n = *mp.fix_count;           // written by the previous launch on this stream
    if (mp.fix_reduce) {  // workgroup w: the work reduce of rollouts 64 w .. 64 w + 63 after the items
      // fix_barrier: the items over every workgroup (a rollout whose legs stay straight defers many of its
      // steps: one workgroup fixing them in turn ran 200 us, configs[4]), then a grid barrier: the launch's
      // ceil(B / 64) <= 1024 one-wavefront workgroups are resident together (the host passes no barrier
      // otherwise); n is the same for all, so every workgroup arrives. Otherwise each workgroup fixes its
      // own rollouts' items in turn. (One call site of the step: a second inlined copy doubled the code.)
      const bool spread = mp.fix_barrier != nullptr;
      for (int it = spread ? (int)blockIdx.x : 0; it < n; it += spread ? (int)gridDim.x : 1) {
        const int fstep = mp.fix_items[2 * it], ws = mp.fix_items[2 * it + 1];
        const int rb = mp.wave_rollouts ? mp.wave_rollouts[ws] : ws;
        if (!spread && rb / WAVE != (int)blockIdx.x) continue;
        rollout_wave<NM, FORCES, false>(T0, a, rws, mp, smem, fstep, ws >> 1, ws & 1);
        wave_sync();
      }
      if (n > 0) __threadfence();  // the fixed steps' rows and work terms, before this workgroup's arrival
      if (spread && n > 0 && threadIdx.x == 0) {
        atomicAdd(mp.fix_barrier, 1);
        // bounded (~2^24 polls): a barrier that never fills ends the wait instead of hanging the device
        for (int spin = 0; spin < (1 << 24); spin++) {
          if (__hip_atomic_load(mp.fix_barrier, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= (int)gridDim.x) break;
          __builtin_amdgcn_s_sleep(2);
        }
      }
      __syncthreads();
      if (spread && n > 0) __threadfence();
      reduce_rollouts(a, (real)mp.red_total_mass, mp.red_rollout_mass, reinterpret_cast<const real*>(mp.fused_work),
                      mp.red_n_steps, mp.red_best_key, mp.red_key_steps);
      return;
    }
    for (int it = blockIdx.x; it < n; it += gridDim.x) {  // one item per wavefront
      const int fstep = mp.fix_items[2 * it], ws = mp.fix_items[2 * it + 1];
      rollout_wave<NM, FORCES, false>(T0, a, rws, mp, smem, fstep, ws >> 1, ws & 1);
      wave_sync();
    }
  } else {
    // fused steps: this wavefront's step and its wavefront within the batch
    int fstep = 0, wid = (int)blockIdx.x;
    if (mp.fused_w) fused_coords((int)blockIdx.x, mp.fused_w, mp.fused_n, fstep, wid);
    rollout_wave<NM, FORCES, MODE == hs::FIX_DEFER>(T0, a, rws, mp, smem, fstep, wid, -1);
  }
}

#include "hs_limb.h"

#if !HS_REAL_IS_FLOAT
// pergensetup::set_rec (pergen.cpp:225-239) after setup_pergen (pergen.cpp:453-507), for
// n_rollouts x n_times (rollout, time) items, two per wavefront: the gait setup of the item's
// rollout on its half-wave, then lane L < n_limbs writes lik limb L's foot target, lane 0 the
// torso position and angles. rec rows: [torso_pos(3), torso_angles(3), foot targets (3 n_limbs)].
__global__ __launch_bounds__(WAVE) void hs_pergen_rec_kernel(const hs_topo* __restrict__ T,
                                                             const hs_gait_params* __restrict__ params,
                                                             int32_t n_rollouts, const double* __restrict__ times,
                                                             int32_t n_times, double* __restrict__ rec) {
  __shared__ SetupL st[2];
  const int sub = threadIdx.x / HALF, lane = threadIdx.x % HALF;
  const int64_t n_items = (int64_t)n_rollouts * n_times;
  const int64_t item = (int64_t)blockIdx.x * 2 + sub;
  const bool live = item < n_items;
  const int64_t it = live ? item : n_items - 1;  // an idle half computes its neighbour's item, stores nothing
  const int b = (int)(it / n_times), ti = (int)(it % n_times);
  const GaitR g = load_gait(params[b]);
  gait_setup(T, g, 1, st[sub], lane);  // every lane of the wave takes part (wave_sync inside)
  const int nl = T->n_limbs;
  if (live && lane < nl) {
    real o0[3], o1[3], target[3];
    bool turned;
    gait_record<false>(g, params[b], limb_rec(st[sub], T->limb_pergen[lane]), (real)times[ti], o0, o1, turned, target);
    double* r = rec + it * (6 + 3 * nl);
    if (lane == 0)
      for (int i = 0; i < 3; i++) { r[i] = o0[i]; r[3 + i] = o1[i]; }
    for (int i = 0; i < 3; i++) r[6 + 3 * lane + i] = target[i];
  }
}
#endif

}  // namespace

#if HS_REAL_IS_FLOAT
extern "C" int hs_limb_deferred_f32(unsigned long long* out) {
#else
extern "C" int hs_limb_deferred_f64(unsigned long long* out) {
#endif
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_limb_deferred), sizeof(unsigned long long), 0,
                                  hipMemcpyDeviceToHost);
}

#if defined(HS_DBG) && !HS_REAL_IS_FLOAT
extern "C" int hs_debug_read_dbg(double* out, int n) {
  if (n > (1 << 22)) n = 1 << 22;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_dbg), sizeof(double) * n, 0, hipMemcpyDeviceToHost);
}
#endif

#if defined(HS_STAMPS) && !HS_REAL_IS_FLOAT
extern "C" int hs_debug_read_stamps(unsigned long long* out, int n_rows) {
  if (n_rows > 4096) n_rows = 4096;
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * 32 * n_rows, 0,
                                  hipMemcpyDeviceToHost);
}
extern "C" int hs_debug_set_stamp_base(unsigned int base) {
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_base), &base, sizeof(base), 0, hipMemcpyHostToDevice);
}
extern "C" int hs_debug_clear_stamps() {
  static unsigned long long zero[4096][32];
  return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), zero, sizeof(zero), 0, hipMemcpyHostToDevice);
}
#endif

namespace hs {

#if HS_REAL_IS_FLOAT
size_t general_workspace_bytes_f32() { return sizeof(RolloutWS); }
#else
size_t general_workspace_bytes() { return sizeof(RolloutWS); }
size_t solve_workspace_bytes() { return sizeof(SolveWS); }  // >= the fp32 build's

void ktab_range(int32_t k0, int32_t n_t, int32_t horizon, int64_t n_calls, int32_t* lo_out, int32_t* n_out,
                int32_t* ttab_out) {
  // call c starts at centre sample (k0 + c horizon) % n_t + 2 (the fused and the per-step paths
  // alike) and its steps read that first k0 + [0, horizon + NS - 1); the first k0s repeat with a
  // period dividing n_t
  int64_t lo = INT64_MAX, hi = 0;
  const int64_t nc = n_calls < n_t ? n_calls : n_t;
  for (int64_t c = 0; c < nc; c++) {
    const int64_t f = ((int64_t)k0 + c * horizon) % n_t;
    lo = f < lo ? f : lo;
    hi = f + horizon + NS - 1 > hi ? f + horizon + NS - 1 : hi;
  }
  const int64_t n = nc > 0 ? hi - lo : 0;
  *lo_out = nc > 0 ? (int32_t)lo : 0;
  *n_out = n <= HS_KTAB ? (int32_t)n : 0;                // the IK table: every sample, or none
  *ttab_out = (int32_t)(n < HS_KTAB ? n : HS_KTAB);      // sample times: the first HS_KTAB samples
}

int launch_pergen_rec(const hs_topo* d_topo, const hs_gait_params* params, int32_t n_rollouts, const double* times,
                      int32_t n_times, double* rec, void* stream) {
  const int64_t items = (int64_t)n_rollouts * n_times;
  if (items <= 0) return 0;
  hipLaunchKernelGGL(hs_pergen_rec_kernel, dim3((unsigned)((items + 1) / 2)), dim3(WAVE), 0, (hipStream_t)stream,
                     d_topo, params, n_rollouts, times, n_times, rec);
  return (int)hipGetLastError();
}
#endif

template <int NM>
void launch_nm(const hs_topo* d_topo, const hs_run_args& a, RolloutWS* ws, const launch_map& mp, hipStream_t st) {
  if (mp.tau_in && mp.fix_mode == FIX_SOLVE)  // the limb-lane forces launch's deferred items
    hipLaunchKernelGGL((hs_rollout_kernel<NM, true, FIX_SOLVE>), dim3(mp.n_waves), dim3(WAVE), 0, st, d_topo, a, ws, mp);
  else if (mp.tau_in)
    hipLaunchKernelGGL((hs_rollout_kernel<NM, true, FIX_NONE>), dim3(mp.n_waves), dim3(WAVE), 0, st, d_topo, a, ws, mp);
  else if (mp.fix_mode == FIX_DEFER)
    hipLaunchKernelGGL((hs_rollout_kernel<NM, false, FIX_DEFER>), dim3(mp.n_waves), dim3(WAVE), 0, st, d_topo, a, ws, mp);
  else if (mp.fix_mode == FIX_SOLVE)
    hipLaunchKernelGGL((hs_rollout_kernel<NM, false, FIX_SOLVE>), dim3(mp.n_waves), dim3(WAVE), 0, st, d_topo, a, ws, mp);
  else
    hipLaunchKernelGGL((hs_rollout_kernel<NM, false, FIX_NONE>), dim3(mp.n_waves), dim3(WAVE), 0, st, d_topo, a, ws, mp);
}

#if HS_REAL_IS_FLOAT
int launch_rollouts_f32(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp) {
#else
int launch_rollouts(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp) {
#endif
  if (a.n_rollouts <= 0 || mp.n_waves <= 0) return 0;
  hipStream_t st = (hipStream_t)a.stream;
  RolloutWS* ws = (RolloutWS*)workspace;
  // one launch per step of the horizon: step h writes output row h, work accumulates in
  // step order (periodic.cpp:291-304), the best key is taken after the last step
  for (int h = 0; h < a.horizon; h++) {
    hs_run_args ah = a;
    launch_map mh = mp;
    ah.k0 = a.k0 + h;
    ah.accumulate = (h == 0) ? a.accumulate : 1;
    if (h + 1 < a.horizon) ah.best_key = nullptr;
    mh.h_row = h;
    if (h > 0 && mp.setup_io != SETUP_COMPUTE) mh.setup_io = SETUP_LOAD;
    // smallest LDS layout that holds the (largest) model's parts: myant 17, spider 19, hexapod 22
    if (mp.max_parts <= 18) launch_nm<18>(d_topo, ah, ws, mh, st);
    else if (mp.max_parts <= 22) launch_nm<22>(d_topo, ah, ws, mh, st);
    else launch_nm<HS_NMAX>(d_topo, ah, ws, mh, st);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return (int)e;
  }
  return 0;
}


#if HS_REAL_IS_FLOAT
int launch_fused_f32(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp) {
#else
int launch_fused(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp) {
#endif
  if (a.n_rollouts <= 0 || mp.n_waves <= 0) return 0;
  hipStream_t st = (hipStream_t)a.stream;
  RolloutWS* ws = (RolloutWS*)workspace;
  if (mp.setup_only) {  // the call's preparation pass: setup record, sample times, IK table
    int R;
    const int units = prep_units(mp, a.n_rollouts, R);
    const int64_t blocks = prep_blocks(units, R, mp.ttab_n, mp.ktab_nl > 0 ? mp.ktab_nl : HS_LMAX);
    if (mp.wave_model)
      hipLaunchKernelGGL(hs_prep_kernel<true>, dim3((unsigned)blocks), dim3(WAVE * HS_PREP_WPB), 0, st, d_topo, a, ws, mp);
    else
      hipLaunchKernelGGL(hs_prep_kernel<false>, dim3((unsigned)blocks), dim3(WAVE * HS_PREP_WPB), 0, st, d_topo, a, ws, mp);
    return (int)hipGetLastError();
  }
  launch_map m = mp;
  m.fused_w = mp.setup_only ? 0 : mp.n_waves;
  m.n_waves = mp.setup_only ? mp.n_waves : mp.n_waves * mp.fused_n;  // the grid
  // the fixup launch: in HS_SOLVE_AUTO a few wavefronts loop over the deferred items (usually none:
  // they exit at once); in HS_SOLVE_REFERENCE every step is an item, one wavefront each
  if (mp.fix_mode == FIX_SOLVE) m.n_waves = a.solve_mode != HS_SOLVE_AUTO ? 2 * m.n_waves : (m.n_waves < 256 ? m.n_waves : 256);
  if (mp.fix_mode == FIX_SOLVE && mp.fix_reduce) m.n_waves = (a.n_rollouts + WAVE - 1) / WAVE;  // 64 rollouts each
  if (mp.max_parts <= 18) launch_nm<18>(d_topo, a, ws, m, st);
  else if (mp.max_parts <= 22) launch_nm<22>(d_topo, a, ws, m, st);
  else launch_nm<HS_NMAX>(d_topo, a, ws, m, st);
  return (int)hipGetLastError();
}

#if HS_REAL_IS_FLOAT
int launch_limb_f32(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp) {
#else
int launch_limb(const hs_topo* d_topo, const hs_run_args& a, void* workspace, const launch_map& mp) {
#endif
  if (a.n_rollouts <= 0 || mp.fused_n <= 0) return 0;
  hipStream_t st = (hipStream_t)a.stream;
  RolloutWS* ws = (RolloutWS*)workspace;
  launch_map m = mp;
  m.fused_w = mp.limb_rollouts ? mp.limb_waves : (a.n_rollouts + LGR - 1) / LGR;  // wavefronts per step: 8 rollouts each
  const dim3 grid((unsigned)((int64_t)m.fused_w * mp.fused_n));
  if (mp.tau_in) {  // solve_forces (hs_run_forces_calls)
    if (mp.max_parts <= 18) hipLaunchKernelGGL((hs_limb_kernel<18, true>), grid, dim3(WAVE), 0, st, d_topo, a, ws, m);
    else if (mp.max_parts <= 22) hipLaunchKernelGGL((hs_limb_kernel<22, true>), grid, dim3(WAVE), 0, st, d_topo, a, ws, m);
    else hipLaunchKernelGGL((hs_limb_kernel<HS_NMAX, true>), grid, dim3(WAVE), 0, st, d_topo, a, ws, m);
  } else {
    if (mp.max_parts <= 18) hipLaunchKernelGGL((hs_limb_kernel<18, false>), grid, dim3(WAVE), 0, st, d_topo, a, ws, m);
    else if (mp.max_parts <= 22) hipLaunchKernelGGL((hs_limb_kernel<22, false>), grid, dim3(WAVE), 0, st, d_topo, a, ws, m);
    else hipLaunchKernelGGL((hs_limb_kernel<HS_NMAX, false>), grid, dim3(WAVE), 0, st, d_topo, a, ws, m);
  }
  return (int)hipGetLastError();
}

__global__ void hs_fused_reduce_kernel(hs_run_args a, real total_mass, const double* __restrict__ rollout_mass,
                                       const real* __restrict__ ws, int n_steps) {
  reduce_rollouts(a, total_mass, rollout_mass, ws, n_steps, reinterpret_cast<uint64_t*>(a.best_key), a.key_steps);
}

#if HS_REAL_IS_FLOAT
int launch_fused_reduce_f32(const hs_run_args& a, double total_mass, const double* rollout_mass,
                            const void* work_steps, int32_t n_steps) {
#else
int launch_fused_reduce(const hs_run_args& a, double total_mass, const double* rollout_mass, const void* work_steps,
                        int32_t n_steps) {
#endif
  if (a.n_rollouts <= 0 || !a.work_cot) return 0;
  // one wavefront per workgroup: B = 4096 spreads over 64 CUs instead of 16
  hipLaunchKernelGGL(hs_fused_reduce_kernel, dim3((a.n_rollouts + 63) / 64), dim3(64), 0, (hipStream_t)a.stream, a,
                     (real)total_mass, rollout_mass, (const real*)work_steps, n_steps);
  return (int)hipGetLastError();
}

}  // namespace hs
