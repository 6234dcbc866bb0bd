// hs_limb.h -- the limb-lane step kernel (round 6), included by hs_kernels.hip inside its anonymous
// namespace (both precisions).
//
// hs_rollout_kernel maps a rollout to 32 lanes and each phase to the lanes it can use: kinematics 30
// (sample, limb) lanes, dynamics and the particular solution one lane per part, the contact blocks four
// lanes per contact, the 6 x 6 Schur system one lane -- 16 % of the issued FP64 lane operations are
// useful. This kernel maps a rollout to a group of 8 lanes, one per limb (the torso
// on lane 7), and keeps a limb's whole step in its lane's registers: the limb FK at the stencil's three
// pos / ust samples, the finite differences of its parts, its links' subtree sums, its contact's blocks
// and its motors' torques -- the work of every phase is per limb, so 6 of 8 lanes are busy in every
// phase, and 8 rollouts share a wavefront. Cross-limb exchanges: the chain bodies' subtree sums and the
// root's through LDS, the contact blocks' Schur entries moved to lane = contact rank (ds_bpermute) and
// summed by DPP in fast_solve_lanes' pairwise order, the motors' work summed in joint order from LDS.
//
// Every value is computed by the same operations in the same order as hs_rollout_kernel's fused step
// (the same helpers, the same expressions), so the outputs are bitwise those of that kernel
// (tests/test_gpu_limb.py). The kernel takes the common case: a call with the preparation pass's IK
// table, a model of the limb-lane class (hs_topo::limb_lane_ok), HS_SOLVE_AUTO, no x / q / dq outputs,
// a step the closed form's tier 1 solves (0 to 6 contacts; a guard near its threshold sets
// HS_FLAG_NEAR_RANK as fast_solve does). Every other step -- a singular contact block (tier 2), nearly
// collinear feet (the Eigen-style path), a joint value past sincos_k_small's range -- is deferred to the
// fixup launch (hs_rollout_kernel FIX_SOLVE), which computes it with hs_rollout_kernel's whole machinery:
// the same (step, rollout) items the fused step launch defers. A mixed plan of limb-lane models runs
// eight rollouts of one model per wavefront (launch_map::limb_model / limb_rollouts).

#ifndef HS_LIMB_ROOT_BRANCHFREE
#define HS_LIMB_ROOT_BRANCHFREE 0
#endif
#ifndef HS_LIMB_WORK_UNROLL
#define HS_LIMB_WORK_UNROLL 0
#endif
#ifndef HS_LIMB_SAMPLE_BARRIER
#define HS_LIMB_SAMPLE_BARRIER 1  // scheduling barriers between the stencil's samples (register pressure)
#endif
#ifndef HS_LIMB_LINK_BARRIER
#define HS_LIMB_LINK_BARRIER 0  // 1: within noise at the driver command, 3 % slower at K = 200 (r06_t5)
#endif
#ifndef HS_LIMB_PAD
#define HS_LIMB_PAD 1
#endif
#ifndef HS_LIMB_NEAR_DEFER
#define HS_LIMB_NEAR_DEFER 0
#endif
#ifndef HS_LIMB_WORK_DPP
#define HS_LIMB_WORK_DPP 0  // the joint-order work sum as a DPP chain across the limb lanes (A/B)
#endif
#ifndef HS_LIMB_KID_LANES
#define HS_LIMB_KID_LANES 1  // the root's kids' range sums on lanes 0 .. nk - 1 (K = 200 +4 %, r06_t32)
#endif
#ifndef HS_LIMB_GROUP
// the fused launch's block order for the limb kernel (fused_coords): groups of this many batch wavefronts
// (8 rollouts each), each group's steps in order
#define HS_LIMB_GROUP HS_FUSED_GROUP
#endif
#ifndef HS_LIMB_NC12
#define HS_LIMB_NC12 1  // one and two contacts solved here (0: deferred, A/B)
#endif
#ifndef HS_LIMB_EARLY_LOADS
#define HS_LIMB_EARLY_LOADS 0
#endif
#ifndef HS_LIMB_MIXED_T
#define HS_LIMB_MIXED_T 1
#endif
#ifndef HS_LIMB_WAVES
#define HS_LIMB_WAVES 2  // waves per SIMD the limb kernel is built for
#endif
#ifndef HS_LIMB_WAVES_F32
#define HS_LIMB_WAVES_F32 HS_LIMB_WAVES  // the single-precision build's (140 VGPRs, 10.9 KB: 3 fit)
#endif

constexpr int LG = 8;           // lanes per rollout group
constexpr int LGR = WAVE / LG;  // rollouts per wavefront

// steps this process's limb-lane launches deferred to the fixup launch (hs_limb_stats; one atomic per
// deferred step, rare)
__device__ unsigned long long g_limb_deferred;

template <int NM, bool FORCES = false>
struct LimbLds {
  real g[NM][6];     // per part g_i = (f_i, t_i + (P_i - p0) x f_i); a root kid's slot then its subtree sums
  real a[6];         // the root's x (torso force, torque): the zeroth-order right-hand side
  real wd[HS_NMAX];  // the motors' positive work of the step, in joint order
  real p[FORCES ? NM : 1][3];  // forces mode: the parts' positions at the centre sample (forces_solve's s, Q sums)
};

// a value of lane `src` of this lane's group (ds_bpermute)
__device__ inline real grp_get(real v, int src) { return __shfl(v, src); }
__device__ inline float grp_getf(float v, int src) { return __shfl(v, src); }
// any lane of the 8-lane group
__device__ inline bool grp_any(bool p, int gbase) { return ((__ballot(p) >> gbase) & 0xFFull) != 0; }
__device__ inline uint32_t grp_or(uint32_t v) {
  v |= (uint32_t)__shfl_xor((int)v, 1);
  v |= (uint32_t)__shfl_xor((int)v, 2);
  v |= (uint32_t)__shfl_xor((int)v, 4);
  return v;
}
// sum over the group's lanes 0..7 holding per-contact values by rank (0 past nc): ((v3 + v2) + (v1 + v0)) +
// ((v4 + v5) + (v6 + v7)) -- fast_solve_lanes' pairwise order over its contact lanes (row_shr 4, row_shr 8,
// xor 16: (v3 + v2) + (v1 + v0) and (v7 + v6) + (v5 + v4), then their sum); every lane gets the total
__device__ inline real rank8_sum(real v) {
  v += dpp_r<0xB1>(v);   // quad_perm [1, 0, 3, 2]
  v += dpp_r<0x4E>(v);   // quad_perm [2, 3, 0, 1]
  v += dpp_r<0x141>(v);  // row_half_mirror: lane i <- 7 - i, the other quad's sum
  return v;
}

// opaque_vals (hs_math.h): values made opaque where hs_rollout_kernel passes them through LDS

// The same pointer, opaque to the optimizer: the three samples' FK read the same topology entries (a
// limb's link products, rotations, COMs: 80 reals) and frames, and merged loads would keep them live
// across all three -- 160 VGPRs on top of the samples' results. Loads through a fresh opaque pointer per
// sample are issued again (L1 hits) where that sample uses them.
// (through an address-space-1 pointer: a generic one would turn the topology reads into flat loads)
__device__ inline const hs_topo* opaque_s(const hs_topo* p) {
  using gptr = const __attribute__((address_space(1))) hs_topo*;
  gptr q = (gptr)p;
  asm volatile("" : "+s"(q));
  return (const hs_topo*)q;
}

// One link of limb_fk (its operations): the next joint frame Jv (from the previous link's hinge frame H),
// the hinge frame H, the link's pos and ust, and at the centre sample its joint position and axis and
// (the foot link) the foot
template <bool CENTRE>
__device__ __attribute__((always_inline)) inline void fk_link(const hs_topo* T, const hs_link& lk, int kk, A34& Jv,
                                                              A34& H, real s, real c, real* P, real* U, real* Jp,
                                                              real* Jz, real* fp, bool& contact) {
#if HS_LIMB_LINK_BARRIER
  // (a scheduling barrier per link: the machine scheduler hoists the three links' constant loads, 80 reals,
  // to the top of the sample's block for latency, and the register allocator then spills them)
  __builtin_amdgcn_sched_barrier(0);
#endif
  if (kk > 0) Jv = mul(H, load34(lk.P));
  H = mul_hinge(Jv, c, s);
  {
    const real cm[3] = {(real)lk.com[0], (real)lk.com[1], (real)lk.com[2]};
    mulp(H, cm, P);
  }
  {
    real R[9];
#pragma unroll
    for (int i = 0; i < 9; i++) R[i] = (real)lk.Rpj[i];
    auto a_rc = [&](int r, int c) { return H(r, 0) * R[c * 3 + 0] + H(r, 1) * R[c * 3 + 1] + H(r, 2) * R[c * 3 + 2]; };
    U[0] = (a_rc(2, 1) - a_rc(1, 2)) / 2;
    U[1] = (a_rc(0, 2) - a_rc(2, 0)) / 2;
    U[2] = (a_rc(1, 0) - a_rc(0, 1)) / 2;
  }
  if (CENTRE) {
#pragma unroll
    for (int i = 0; i < 3; i++) Jp[i] = Jv(i, 3);
#pragma unroll
    for (int i = 0; i < 3; i++) Jz[i] = Jv(i, 2);
    if (kk == 2) {  // the foot link (hs_topo::limb_lane_ok)
      const real cp[3] = {(real)lk.cap[0], (real)lk.cap[1], (real)lk.cap[2]};
      mulp(H, cp, fp);
      contact = fp[2] < (real)(T->rcap + 1e-4);
    }
  }
}

// dynamics()' finite differences of one part (dynrec.cpp:175-224) from its pos / ust at t - 2dt, t, t + 2dt
__device__ inline void part_dyn(real m, real inv, const real* Pm, const real* P0, const real* Pp, const real* Um,
                                const real* U0, const real* Up, real* f) {
  real vp[3], vm[3], mr[3], wp[3], wm[3], amr[3];
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
  for (int j = 0; j < 3; j++) {
    amr[j] = wp[j] - wm[j];
    amr[j] *= inv;
  }
  for (int j = 0; j < 3; j++) {
    f[j] = mr[j];
    f[3 + j] = amr[j];
  }
  opaque_vals<6>(f);    // dynamics() stores f and adds gravity to the stored value
  f[2] += m * real(1);  // gravity, g = 1 (dynrec.cpp:291-295)
}

// particular_sub's first stage for one part: g = (f, t + (P - o) x f)
__device__ inline void part_g(const real* P, const real* o, real* f) {
  opaque_vals<6>(f);  // f as dynamics() stores it (LDS), then g as particular_sub stores it
  real d[3];
  for (int j = 0; j < 3; j++) d[j] = P[j] - o[j];
  f[3] += d[1] * f[2] - d[2] * f[1];
  f[4] += d[2] * f[0] - d[0] * f[2];
  f[5] += d[0] * f[1] - d[1] * f[0];
  opaque_vals<6>(f);
}

// pos and ust of a jointless chain body or of the torso at one sample: straight gaits from the setup's
// features at tv = 0 (kin_sample_straight), turning ones from the body frame A (node_features)
struct BodyS {
  real P[3], U[3];
};
__device__ inline BodyS body_straight(const real* bf, const real* u, real tv) {
  BodyS s;
  for (int i = 0; i < 3; i++) s.P[i] = fma(tv, u[i], bf[i]);
  for (int i = 0; i < 3; i++) s.U[i] = bf[3 + i];
  return s;
}
__device__ inline BodyS body_frame(const A34& A, const real* com) {
  BodyS s;
  mulp(A, com, s.P);
  s.U[0] = (A(2, 1) - A(1, 2)) / 2;
  s.U[1] = (A(0, 2) - A(2, 0)) / 2;
  s.U[2] = (A(1, 0) - A(0, 1)) / 2;
  return s;
}

// Limb L's hip joint frame J at one sample and its chain body's pos / ust (limb_own_n <= 1, hs_topo::
// limb_lane_ok): straight gaits from KinFrames at tv, turning ones from the torso record's frame and the
// chain products (kin_sample_tab)
__device__ __attribute__((always_inline)) inline A34 limb_frame(const hs_topo* T, int L, bool straight, const bool own,
                                                                const RolloutWS& W, int row, const real* u, real tv,
                                                                BodyS& ob) {
#ifdef HS_LIMB_EXP_STRAIGHT
  straight = true;
#endif
  if (straight) {
    if (own) ob = body_straight(W.kf.own[L][0], u, tv);
    return frame_at(load34r(W.kf.J0[L]), u, tv);
  }
  A34 A = load34r(W.ktor[row] + 6);
  const int clen = T->limb_chain_len[L];
  for (int kk = 1; kk < clen; kk++) {
    const int v = T->limb_chain[L][kk];
    A = mul(A, node_pj(T, v));
    if (T->node[v].owner_limb == L) {
      const real com[3] = {(real)T->node[v].com[0], (real)T->node[v].com[1], (real)T->node[v].com[2]};
      ob = body_frame(A, com);
    }
  }
  return mul(A, node_joint_parent(T, T->limb_child[L]));
}

// the links' pos and ust at an outer sample of the stencil (the limb FK without the centre's features)
// (big: a joint value sincos_k_small does not take, |x| >= 2^20 or not finite: the step is deferred)
__device__ inline bool sincos_big(real x) { return !(fabs(x) < (real)0x1p20); }
__device__ __attribute__((always_inline)) inline void limb_outer(const hs_topo* T, const hs_link (&LK)[3], const A34& J,
                                                                 const real* ja, real (&P)[3][3], real (&U)[3][3],
                                                                 bool& big) {
  real sq[3], cq[3];
#pragma unroll
  for (int kk = 0; kk < 3; kk++) {
    big |= sincos_big(ja[kk]);
    sincos_k_small(ja[kk], &sq[kk], &cq[kk]);
  }
  A34 Jv = J, H;
  real nul[3];
  bool nc = false;
#pragma unroll
  for (int kk = 0; kk < 3; kk++) fk_link<false>(T, LK[kk], kk, Jv, H, sq[kk], cq[kk], P[kk], U[kk], nul, nul, nul, nc);
}

// A contact's first-order block D_c (packed lower: 00 10 11 20 21 22) and g_c on its limb lane
// (fast_solve_lanes: joint m of the foot's chain, foot link first, on lane m of a quad, summed
// ((m0 + m1) + (m2 + m3)); the chain's jointless bodies add exact zeros)
__device__ __attribute__((always_inline)) inline void contact_block(const real (&Jp)[3][3], const real (&Jz)[3][3],
                                                                    const real (&xt)[3][3], const real* fp, real* Dp6,
                                                                    real* gc) {
  real tD[3][6], tg[3][3];
#pragma unroll
  for (int m = 0; m < 3; m++) {
    const int p = 2 - m;
    real Dp[6] = {0, 0, 0, 0, 0, 0}, g[3] = {0, 0, 0};
    real da[3], va[3][3];
    for (int r = 0; r < 3; r++) da[r] = Jp[p][r] - fp[r];
    cross_rows(da, va);
#pragma unroll
    for (int r = 0; r < 3; r++) {
      const real w2 = Jz[p][r] * Jz[p][r];
#pragma unroll
      for (int i = 0; i < 3; i++) {
        if (i == r) continue;
#pragma unroll
        for (int j = 0; j <= i; j++)
          if (j != r) Dp[i * (i + 1) / 2 + j] += w2 * va[r][i] * va[r][j];
        g[i] += w2 * va[r][i] * xt[p][r];
      }
    }
    for (int e = 0; e < 6; e++) tD[m][e] = Dp[e];
    for (int i = 0; i < 3; i++) tg[m][i] = g[i];
  }
#pragma unroll
  for (int e = 0; e < 6; e++) Dp6[e] = (tD[0][e] + tD[1][e]) + (tD[2][e] + real(0));
#pragma unroll
  for (int i = 0; i < 3; i++) gc[i] = (tg[0][i] + tg[1][i]) + (tg[2][i] + real(0));
}

// hs_limb_kernel's forces mode after S1 (forces_solve's fast path, every value by its operations in its
// order): the parts' s, Q sums over nodes 1 .. n - 1 in node order (every lane of the group), the limb's
// blocks on its lane (forces_limb_block), the sums over the limbs in limb order (a DPP chain: lane l adds
// its term to lane l - 1's partial sum, the total on lane nl - 1), the 6 x 6 system on every lane, each
// limb's foot forces on its lane
template <int NM>
__device__ __attribute__((always_inline)) inline void limb_forces(const hs_topo* T, const hs_run_args& a,
                                                                  const hs::launch_map& mp, LimbLds<NM, true>& S, bool limb,
                                                                  int l, int L, int gbase, int nl, bool live, int b,
                                                                  int fstep, int s_glob, const real* o,
                                                                  const real (&Jp)[3][3], const real (&Jz)[3][3],
                                                                  const real (&Pc)[3][3], const real* fp,
                                                                  const real (&xt)[3][3], bool bad, bool big) {
  const int n = T->n;
#ifdef HS_DBG
  const int dbg_r = live ? b * a.horizon + s_glob : -1;
#define FDBG(slot, val, n_)                                                                                      \
  do {                                                                                                           \
    if (HS_DBG == (n_) && dbg_r >= 0 && (size_t)dbg_r * 32 + (slot) < (1u << 22)) g_dbg[(size_t)dbg_r * 32 + (slot)] = (double)(val); \
  } while (0)
#else
#define FDBG(slot, val, n_) do {} while (0)
#endif
  real ts[9];
#pragma unroll
  for (int q = 0; q < 9; q++) ts[q] = 0;
  for (int i = 1; i < n; i++) {
    real r[3];
    for (int t = 0; t < 3; t++) r[t] = S.p[i][t] - o[t];
    // forces_solve's lanes select between r_a and the product r_a r_b before adding (a lane-dependent
    // select): the product is rounded, then added -- not one FMA
    real q[6] = {r[0] * r[0], r[1] * r[1], r[2] * r[2], r[0] * r[1], r[0] * r[2], r[1] * r[2]};
    opaque_vals<6>(q);
    ts[0] += r[0];
    ts[1] += r[1];
    ts[2] += r[2];
    for (int j = 0; j < 6; j++) ts[3 + j] += q[j];
  }
  opaque_vals<9>(ts);  // forces_solve keeps them in LDS (sv.y)
  const int dbg_f = T->link[L][2].foot;
  (void)dbg_f;
  if (l == 0) FDBG(0, ts[3], 30);
  const size_t orow = (size_t)b * a.horizon + s_glob;
  // the limb's blocks (forces_solve's stages), its 27 terms of the sums over the limbs formed as soon as
  // both factors exist: K_f - S_l (packed lower), q_f + e_l -- forces_solve's fr.b - fr.a / fr.b + fr.a,
  // each product rounded as its LDS rows hold it (the two 27-entry blocks are never live together)
  real Ct[18], Bd[6], Bl[9], rdB[3], rb[3], vl[27];
  bool okB = true;
  if (limb) {
    const real* z = inp(mp.tau_in) + (live ? orow : 0) * mp.st_tau;
    real zz[3];
    for (int kk = 0; kk < 3; kk++) zz[kk] = z[T->node[T->limb_node[L][kk]].hinge];
    ForcesRows F;
    forces_rows(F, Jp, Jz, Pc, fp, o, xt, zz);
    okB = forces_foot(F, fp, o, Ct, Bd, Bl, rdB, rb);
    FDBG(24 + dbg_f, Ct[0], 36);
    FDBG(24 + dbg_f, rb[0], 37);
    if (okB) {
      ForcesV G;
      forces_v(G, Ct, Bl, rdB, rb);
#pragma unroll
      for (int e = 0; e < 27; e++) {
        const TriWalk<> t(e < 21 ? e : 0);
        real pa = e < 21 ? F.prod(t.r, t.c) : F.prod(e - 21, 9);
        real pb = e < 21 ? G.vprod(t.r, t.c) : G.vprod(e - 21, 6);
        opaque_vals<1>(&pa);  // fr.a / fr.b (LDS)
        opaque_vals<1>(&pb);
        vl[e] = (e < 21) ? pb - pa : pb + pa;
      }
    }
  }
  const bool fast = !grp_any(limb && !okB, gbase);
  if (!fast || grp_any(big, gbase)) {  // the dense normal equations: the forces fixup's (forces_solve)
    if (l == 0 && live) {
      atomicAdd(&g_limb_deferred, 1ull);
      const int it = atomicAdd(mp.fix_count, 1);
      mp.fix_items[2 * it] = fstep;
      mp.fix_items[2 * it + 1] = b;  // 2 * wavefront + half of hs_rollout_kernel's layout
    }
    return;
  }
  // K = W_tt - sum S_l + sum K_f, rhs = sum (q_f + e_l) - d_t
  real kv[27];
#pragma unroll
  for (int e = 0; e < 27; e++) {
    const real v = limb ? vl[e] : real(0);
    real s = real(0) + v;
    for (int k = 1; k < nl; k++) {
      const real prev = dpp_r<0x111>(s);  // row_shr 1: lane l - 1's partial sum
      if (l >= 1) s = prev + v;
    }
    const real tot = grp_get(s, gbase + nl - 1);
    const real dtv = (e < 21) ? real(0) : (e < 24 ? S.a[e - 21] : S.a[e - 21]);
    kv[e] = (e < 21) ? wtt_entry(e, ts, n) + tot : tot - dtv;
  }
  opaque_vals<27>(kv);  // fr.a[0] (LDS)
  if (l == 0) FDBG(1, kv[0], 33);
  real K[36], rd[6], lam[6];
#pragma unroll
  for (int r = 0; r < 6; r++) {
#pragma unroll
    for (int c = 0; c < 6; c++) K[6 * r + c] = (c <= r) ? kv[pk(r, c)] : real(0);
    lam[r] = kv[21 + r];
  }
  ldl_n<6>(K, real(0), rd);  // >= I
  ldl_solve_n<6>(K, rd, lam);
  if (l == 0) FDBG(2, lam[0], 34);
  bool nan = false;
  real t[3] = {0, 0, 0};
  if (limb) {  // y_f = B_f^-1 (r_f - C~_f^T lam)
    for (int k = 0; k < 3; k++) {
      real s = rb[k];
      for (int r = 0; r < 6; r++) s -= Ct[3 * r + k] * lam[r];
      t[k] = s;
    }
    ldl_solve_n<3>(Bl, rdB, t);
    FDBG(24 + dbg_f, t[0], 35);
    for (int k = 0; k < 3; k++) nan |= t[k] != t[k];
    const int f = T->link[L][2].foot;
    if (live && a.cf)
      for (int k = 0; k < 3; k++) outp(a.cf)[orow * mp.st_cf + 3 * f + k] = t[k];
  }
  if (live && a.cf)  // a mixed plan's columns past this model's feet
    for (int c = 3 * T->nf + l; c < mp.st_cf; c += LG) outp(a.cf)[orow * mp.st_cf + c] = real(0);
  const bool any_nan = grp_any(nan, gbase), any_bad = grp_any(limb && bad, gbase);
  if (l == 0 && live && a.flags) a.flags[orow] = (any_nan ? HS_FLAG_NAN : 0u) | (any_bad ? HS_FLAG_UNREACH : 0u);
}
#undef FDBG

// FORCES: hs_run_forces_calls' solve_forces step (contact forces given motor torques, forces_solve's fast
// path: a limb's blocks on its lane, the sums over the limbs in limb order by a DPP chain, the 6 x 6 on
// every lane of the group; a B_f near singular defers the step to the forces fixup launch)
template <int NM, bool FORCES>
__global__ __launch_bounds__(WAVE, HS_REAL_IS_FLOAT ? HS_LIMB_WAVES_F32 : HS_LIMB_WAVES) void hs_limb_kernel(const hs_topo* __restrict__ T0, hs_run_args a,
                                                                      RolloutWS* __restrict__ rws, hs::launch_map mp) {
  // the outer samples' pos / ust of every lane's links (kinematics), then the groups' exchange arrays:
  // 18 KB per wavefront, 8 per CU at 2 waves / SIMD
  // kinematics: the outer samples' pos / ust of every limb lane's links and the limbs' link records (read
  // by every sample's FK: from LDS, not through three rounds of L1/L2 latency per sample), then the
  // groups' exchange arrays: 17.4 KB per wavefront, 8 per CU at 2 waves / SIMD
  __shared__ union {
    struct {
      real outer[36][LGR * HS_LMAX];  // [Pm, Um, Pp, Up][link][component][limb lane]: one conflict-free row per value
      hs_link links[HS_LMAX][3];
    } k;
    LimbLds<NM, FORCES> g[LGR];
  } sh;
  LimbLds<NM, FORCES>* lds = sh.g;
  int fstep = 0, q = (int)blockIdx.x;
  fused_coords<HS_LIMB_GROUP>((int)blockIdx.x, mp.fused_w, mp.fused_n, fstep, q);
#if HS_LIMB_MIXED_T
  const hs_topo* __restrict__ T = mp.limb_model ? T0 + mp.limb_model[q] : T0;  // a mixed plan's wavefront model
#else
  const hs_topo* __restrict__ T = T0;
#endif
#if HS_LIMB_EARLY_LOADS
  // the rollout's first loads (its records, sample times, torso) issued before the link records' copy and
  // its barrier, so their latency overlaps the copy
  RSTAMP(16);
  STAMP(15);
  const int lane = (int)threadIdx.x, grp = lane >> 3, l = lane & 7, gbase = lane & ~7;
  const int b = mp.limb_rollouts ? mp.limb_rollouts[q * LGR + grp] : q * LGR + grp;
  const bool live = b >= 0 && b < a.n_rollouts;
  // an idle group computes a copy of a rollout of its wavefront's model and stores nothing
  const int bb = live ? b : (mp.limb_rollouts ? mp.limb_rollouts[q * LGR] : a.n_rollouts - 1);
  LimbLds<NM, FORCES>& S = lds[grp];
  const int ol = grp * HS_LMAX + (l < HS_LMAX ? l : 0);  // this limb lane's column of sh.k.outer
  const int s_glob = mp.fused_s0 + fstep, call = s_glob / mp.fused_h;
  const int k0 = (int)(((int64_t)a.k0 + (int64_t)call * mp.fused_h) % a.n_t) + s_glob % mp.fused_h;
  const int row0 = k0 - mp.ktab_lo;  // table row of sample i - 2 (centre i = k0 + 2)
  const int nl = T->n_limbs, nmj = T->nmj;
  const bool limb = l < nl, tlane = l == LG - 1;
  const int L = limb ? l : 0;
  const RolloutWS& W = rws[bb];
  const hs_gait_params& gp = a.params[bb];
  const bool straight = (real)gp.curvature == 0 && !gp.rec_transform_flag;
  const real dt = W.st.dt;
  const real v = W.st.v;
  const NodeK n0 = load_nodek(T, 0);
  const real u[3] = {n0.Jp(0, 0), n0.Jp(1, 0), n0.Jp(2, 0)};
  real tv[5];
#pragma unroll
  for (int k = 0; k < 5; k += 2) tv[k] = W.t_tab[row0 + k] * v;  // gait_record's torso advance
  // the torso COM at the centre sample (particular_sub's origin o = pos(0, 0)), on every lane
  real o[3];
  if (straight) {
    for (int i = 0; i < 3; i++) o[i] = fma(tv[2], u[i], W.kf.torso[i]);
  } else {
    mulp(load34r(W.ktor[row0 + 2] + 6), n0.com, o);
  }
  const real inv = real(1) / (2 * dt);
  {  // the link records, 8 bytes per lane and load
    const uint64_t* src = reinterpret_cast<const uint64_t*>(&T->link[0][0]);
    uint64_t* dst = reinterpret_cast<uint64_t*>(&sh.k.links[0][0]);
    constexpr int NW = sizeof(sh.k.links) / sizeof(uint64_t);
    for (int e = (int)threadIdx.x; e < NW; e += WAVE) dst[e] = src[e];
    wave_sync();
  }
#else
  {  // the link records, 8 bytes per lane and load
    const uint64_t* src = reinterpret_cast<const uint64_t*>(&T->link[0][0]);
    uint64_t* dst = reinterpret_cast<uint64_t*>(&sh.k.links[0][0]);
    constexpr int NW = sizeof(sh.k.links) / sizeof(uint64_t);
    for (int e = (int)threadIdx.x; e < NW; e += WAVE) dst[e] = src[e];
    wave_sync();
  }
  RSTAMP(16);
  STAMP(15);
  const int lane = (int)threadIdx.x, grp = lane >> 3, l = lane & 7, gbase = lane & ~7;
  const int b = mp.limb_rollouts ? mp.limb_rollouts[q * LGR + grp] : q * LGR + grp;
  const bool live = b >= 0 && b < a.n_rollouts;
  // an idle group computes a copy of a rollout of its wavefront's model and stores nothing
  const int bb = live ? b : (mp.limb_rollouts ? mp.limb_rollouts[q * LGR] : a.n_rollouts - 1);
  LimbLds<NM, FORCES>& S = lds[grp];
  const int ol = grp * HS_LMAX + (l < HS_LMAX ? l : 0);  // this limb lane's column of sh.k.outer
  const int s_glob = mp.fused_s0 + fstep, call = s_glob / mp.fused_h;
  const int k0 = (int)(((int64_t)a.k0 + (int64_t)call * mp.fused_h) % a.n_t) + s_glob % mp.fused_h;
  const int row0 = k0 - mp.ktab_lo;  // table row of sample i - 2 (centre i = k0 + 2)
  const int nl = T->n_limbs, nmj = T->nmj;
  const bool limb = l < nl, tlane = l == LG - 1;
  const int L = limb ? l : 0;
  const RolloutWS& W = rws[bb];
  const hs_gait_params& gp = a.params[bb];
  const bool straight = (real)gp.curvature == 0 && !gp.rec_transform_flag;
  const real dt = W.st.dt;
  const real v = W.st.v;
  const NodeK n0 = load_nodek(T, 0);
  const real u[3] = {n0.Jp(0, 0), n0.Jp(1, 0), n0.Jp(2, 0)};
  real tv[5];
#pragma unroll
  for (int k = 0; k < 5; k += 2) tv[k] = W.t_tab[row0 + k] * v;  // gait_record's torso advance
  // the torso COM at the centre sample (particular_sub's origin o = pos(0, 0)), on every lane
  real o[3];
  if (straight) {
    for (int i = 0; i < 3; i++) o[i] = fma(tv[2], u[i], W.kf.torso[i]);
  } else {
    mulp(load34r(W.ktor[row0 + 2] + 6), n0.com, o);
  }
  const real inv = real(1) / (2 * dt);
#endif
#ifdef HS_DBG
  const int dbg_r = live ? b * a.horizon + s_glob : -1;
#define LDBG(slot, val, n)                                                                                       \
  do {                                                                                                           \
    if (HS_DBG == (n) && dbg_r >= 0 && (size_t)dbg_r * 32 + (slot) < (1u << 22)) g_dbg[(size_t)dbg_r * 32 + (slot)] = (double)(val); \
  } while (0)
#else
#define LDBG(slot, val, n) do {} while (0)
#endif

  // the torso's g (node 0; its joint frame J = I * J_A_parent, node_features), on every lane: its loads and
  // arithmetic overlap the limbs' (a torso-lane branch after them would expose its load latency)
  real g0[6];
  {
    BodyS tb[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
      if (straight) tb[k] = body_straight(W.kf.torso, u, tv[2 * k]);
      else tb[k] = body_frame(load34r(W.ktor[row0 + 2 * k] + 6), n0.com);
    }
    part_dyn((real)T->mass[0], inv, tb[0].P, tb[1].P, tb[2].P, tb[0].U, tb[1].U, tb[2].U, g0);
    part_g(tb[1].P, o, g0);
  }
  STAMP(0);
  // ---- K and D: the limb's links and its chain body (limb lanes), the torso (lane 7) ----
  // Liveness drives the order (the step's peak registers are here): the outer samples' pos / ust first,
  // then the centre link by link, each link's finite differences as soon as its centre values exist
  real g3[3][6];  // the links' g (f, then f's torque part moved about o)
  real Jp[3][3], Jz[3][3], fp[3];
  bool contact = false;
  bool own = false;  // this limb computes a chain body (limb_own_n = 1)
  real gown[6];
  real jvel[3];
  real Pc[3][3], Pown[3];  // forces mode: the links' and the chain body's positions at the centre
  bool bad = false, big = false;
  const hs_topo* const T_ = T;
  if (limb) {
    const int row = row0;
    own = T->limb_own_n[L] > 0;
    // the outer samples (t - 2dt, t + 2dt): the links' pos / ust to LDS (36 reals; held in registers across
    // the centre's FK they pushed the kernel past 256 VGPRs), the chain body's pos / ust kept
    BodyS om, op, oc;
    {
      real P[3][3], U[3][3];
      const hs_topo* Ts = opaque_s(T);
      limb_outer(Ts, sh.k.links[L], limb_frame(Ts, L, straight, own, W, row, u, tv[0], om), W.ktab[row][L], P, U, big);
#pragma unroll
      for (int kk = 0; kk < 3; kk++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
          sh.k.outer[3 * kk + j][ol] = P[kk][j];
          sh.k.outer[9 + 3 * kk + j][ol] = U[kk][j];
        }
    }
    STAMP(1);
    // (sched_barrier: the machine scheduler would interleave the independent samples for ILP, holding
    // two samples' FK working sets at once)
#if HS_LIMB_SAMPLE_BARRIER
    __builtin_amdgcn_sched_barrier(0);
#endif
    {
      real P[3][3], U[3][3];
      const hs_topo* Ts = opaque_s(T);
      limb_outer(Ts, sh.k.links[L], limb_frame(Ts, L, straight, own, W, row + 4, u, tv[4], op), W.ktab[row + 4][L], P, U,
                 big);
#pragma unroll
      for (int kk = 0; kk < 3; kk++)
#pragma unroll
        for (int j = 0; j < 3; j++) {
          sh.k.outer[18 + 3 * kk + j][ol] = P[kk][j];
          sh.k.outer[27 + 3 * kk + j][ol] = U[kk][j];
        }
    }
#if HS_LIMB_SAMPLE_BARRIER
    __builtin_amdgcn_sched_barrier(0);
#endif
    STAMP(2);
    {
      const hs_topo* T = opaque_s(T_);
      const A34 J = limb_frame(T, L, straight, own, W, row + 2, u, tv[2], oc);
      if (own) {  // the chain body's differences first: its three samples are dead before the links' FK
        part_dyn((real)T->mass[T->limb_own[L][0]], inv, om.P, oc.P, op.P, om.U, oc.U, op.U, gown);
        part_g(oc.P, o, gown);
        if constexpr (FORCES)
          for (int j = 0; j < 3; j++) Pown[j] = oc.P[j];
      }
      const real* ja = W.ktab[row + 2][L];
      real sq[3], cq[3];
#pragma unroll
      for (int kk = 0; kk < 3; kk++) {
        big |= sincos_big(ja[kk]);
        sincos_k_small(ja[kk], &sq[kk], &cq[kk]);
      }
      A34 Jv = J, H;
#pragma unroll
      for (int kk = 0; kk < 3; kk++) {
        real P0[3], U0[3];
        fk_link<true>(T, sh.k.links[L][kk], kk, Jv, H, sq[kk], cq[kk], P0, U0, Jp[kk], Jz[kk], fp, contact);
        opaque_vals<3>(P0);  // the features as hs_rollout_kernel's later phases read them (LDS)
        if constexpr (FORCES)
          for (int j = 0; j < 3; j++) Pc[kk][j] = P0[j];
        opaque_vals<3>(U0);
        opaque_vals<3>(Jp[kk]);
        opaque_vals<3>(Jz[kk]);
        if (kk == 2) opaque_vals<3>(fp);
        real Pm[3], Um[3], Pp[3], Up[3];
#if HS_LIMB_SAMPLE_BARRIER
        __builtin_amdgcn_sched_barrier(0);  // the link's outer values read here, not hoisted above its FK
#endif
#pragma unroll
        for (int j = 0; j < 3; j++) {
          Pm[j] = sh.k.outer[3 * kk + j][ol];
          Um[j] = sh.k.outer[9 + 3 * kk + j][ol];
          Pp[j] = sh.k.outer[18 + 3 * kk + j][ol];
          Up[j] = sh.k.outer[27 + 3 * kk + j][ol];
        }
        part_dyn((real)T->mass[T->limb_node[L][kk]], inv, Pm, P0, Pp, Um, U0, Up, g3[kk]);
        LDBG(T->limb_node[L][kk], P0[0], 1);
        LDBG(T->limb_node[L][kk], U0[0], 5);
        LDBG(T->limb_node[L][kk], g3[kk][0], 2);
        LDBG(T->limb_node[L][kk], g3[kk][3], 10);
        LDBG(T->limb_node[L][kk], g3[kk][1], 13);
        LDBG(T->limb_node[L][kk], g3[kk][2], 14);
        LDBG(T->limb_node[L][kk], g3[kk][4], 16);
        if (l == 0) LDBG(31, o[0], 15);
        if (l == 0) LDBG(30, o[1], 15);
        LDBG(T->limb_node[L][kk], Um[0], 9);
        LDBG(T->limb_node[L][kk], Up[0], 11);
        LDBG(T->limb_node[L][kk], Pm[0], 12);
        part_g(P0, o, g3[kk]);
        LDBG(T->limb_node[L][kk], g3[kk][3], 3);
      }
    }
    bad = W.kbad[row + 2][L] != 0;
    // the motors' joint rates at the centre (compute_vel_traj's wrapped difference of q at t +- dt)
#pragma unroll
    for (int kk = 0; kk < 3; kk++) {
      if constexpr (FORCES) break;
      real dd = W.ktab[row + 3][L][kk] - W.ktab[row + 1][L][kk];
      if (dd > kPi) dd -= 2 * kPi;
      else if (dd < -kPi) dd += 2 * kPi;
      jvel[kk] = dd / (2 * dt);
    }
  }
  STAMP(3);
  wave_sync();  // S.g overlays sh.k: every lane's outer and link reads first
  if (limb) {
    // g to LDS (the chain bodies' and the root's subtree sums read them)
#pragma unroll
    for (int kk = 0; kk < 3; kk++)
      for (int j = 0; j < 6; j++) S.g[T->limb_node[L][kk]][j] = g3[kk][j];
    if (own)
      for (int j = 0; j < 6; j++) S.g[T->limb_own[L][0]][j] = gown[j];
    if constexpr (FORCES) {
#pragma unroll
      for (int kk = 0; kk < 3; kk++)
        for (int j = 0; j < 3; j++) S.p[T->limb_node[L][kk]][j] = Pc[kk][j];
      if (own)
        for (int j = 0; j < 3; j++) S.p[T->limb_own[L][0]][j] = Pown[j];
    }
  } else if (tlane) {
    for (int j = 0; j < 6; j++) S.g[0][j] = g0[j];
  }
  wave_sync();

  STAMP(4);
  // ---- S1: subtree sums (particular_sub's stage 2) ----
  // links: their own range in registers (the limb's links are consecutive in preorder, sizes 3, 2, 1); the
  // root on the torso lane: its own g plus each kid's subtree sum (the kid's preorder range, in order),
  // particular_sub's two levels of sums
  real xt[3][3];  // the links' x torque rows
  if (limb) {
#pragma unroll
    for (int kk = 0; kk < 3; kk++) {
      real F[3] = {0, 0, 0}, V[3] = {0, 0, 0};
#pragma unroll
      for (int m = kk; m < 3; m++)
        for (int j = 0; j < 3; j++) { F[j] += g3[m][j]; V[j] += g3[m][3 + j]; }
      // particular_sub applies stage 3 in a block of its own (after a wavefront barrier): F, V enter it
      // as opaque values
      opaque_vals<3>(F);
      opaque_vals<3>(V);
      real d[3];
      for (int j = 0; j < 3; j++) d[j] = Jp[kk][j] - o[j];
      V[0] -= d[1] * F[2] - d[2] * F[1];
      V[1] -= d[2] * F[0] - d[0] * F[2];
      V[2] -= d[0] * F[1] - d[1] * F[0];
      for (int j = 0; j < 3; j++) xt[kk][j] = V[j];
      opaque_vals<3>(xt[kk]);  // x as the later phases read it (LDS)
      LDBG(T->limb_node[L][kk], V[0], 4);
      LDBG(T->limb_node[L][kk], F[0], 18);
      LDBG(T->limb_node[L][kk], d[0], 17);
    }
  }
#if HS_LIMB_KID_LANES
  // the root's kids' range sums on lanes 0 .. nk - 1 of the group, in parallel (each range in preorder, as
  // the torso lane would sum it), into the kid's own slot (ranges are disjoint: no lane reads another's)
  {
    const int nk = T->node[0].nkids;
    if (l < nk && l < HS_CMAX) {
      const int c = T->node[0].kids[l], sz = T->node[c].size;
      real Fk[3] = {0, 0, 0}, Vk[3] = {0, 0, 0};
#pragma unroll
      for (int r = 0; r < 8; r++)
        if (r < sz)
          for (int j = 0; j < 3; j++) { Fk[j] += S.g[c + r][j]; Vk[j] += S.g[c + r][3 + j]; }
      for (int r = 8; r < sz; r++)
        for (int j = 0; j < 3; j++) { Fk[j] += S.g[c + r][j]; Vk[j] += S.g[c + r][3 + j]; }
      for (int j = 0; j < 3; j++) { S.g[c][j] = Fk[j]; S.g[c][3 + j] = Vk[j]; }
    }
  }
  wave_sync();
  if (tlane) {  // x_0 = (F, V - 0 x F): its own g plus the kids' sums, in kid order
    real F[3], V[3];
    for (int j = 0; j < 3; j++) { F[j] = S.g[0][j]; V[j] = S.g[0][3 + j]; }
    const int nk = T->node[0].nkids;
    for (int kk = 0; kk < HS_CMAX; kk++) {
      if (kk >= nk) break;
      const int c = T->node[0].kids[kk];
      for (int j = 0; j < 3; j++) { F[j] += S.g[c][j]; V[j] += S.g[c][3 + j]; }
    }
    const real d[3] = {0, 0, 0};
    V[0] -= d[1] * F[2] - d[2] * F[1];
    V[1] -= d[2] * F[0] - d[0] * F[2];
    V[2] -= d[0] * F[1] - d[1] * F[0];
    for (int j = 0; j < 3; j++) { S.a[j] = F[j]; S.a[3 + j] = V[j]; }
  }
#else
  if (tlane) {  // x_0 = (F, V - 0 x F)
    real F[3], V[3];
    for (int j = 0; j < 3; j++) { F[j] = S.g[0][j]; V[j] = S.g[0][3 + j]; }
    const int nk = T->node[0].nkids;
    for (int kk = 0; kk < HS_CMAX; kk++) {
      if (kk >= nk) break;
      const int c = T->node[0].kids[kk], sz = T->node[c].size;
      real Fk[3] = {0, 0, 0}, Vk[3] = {0, 0, 0};
#if HS_LIMB_ROOT_BRANCHFREE
      // the range's loads issued together, without a branch per part (ranges of up to 8 parts unrolled:
      // hexapod 7, spider 3, myant 4; a part past the range is loaded from a valid row and not added)
#pragma unroll
      for (int r = 0; r < 8; r++) {
        const int rr = c + r < NM ? c + r : NM - 1;
        real gv[6];
        for (int j = 0; j < 6; j++) gv[j] = S.g[rr][j];
        for (int j = 0; j < 3; j++) {
          Fk[j] = r < sz ? Fk[j] + gv[j] : Fk[j];
          Vk[j] = r < sz ? Vk[j] + gv[3 + j] : Vk[j];
        }
      }
#else
      // ranges of up to 8 parts unrolled (hexapod 7, spider 3, myant 4)
#pragma unroll
      for (int r = 0; r < 8; r++)
        if (r < sz)
          for (int j = 0; j < 3; j++) { Fk[j] += S.g[c + r][j]; Vk[j] += S.g[c + r][3 + j]; }
#endif
      for (int r = 8; r < sz; r++)
        for (int j = 0; j < 3; j++) { Fk[j] += S.g[c + r][j]; Vk[j] += S.g[c + r][3 + j]; }
      for (int j = 0; j < 3; j++) { F[j] += Fk[j]; V[j] += Vk[j]; }
    }
    const real d[3] = {0, 0, 0};
    V[0] -= d[1] * F[2] - d[2] * F[1];
    V[1] -= d[2] * F[0] - d[0] * F[2];
    V[2] -= d[0] * F[1] - d[1] * F[0];
    for (int j = 0; j < 3; j++) { S.a[j] = F[j]; S.a[3 + j] = V[j]; }
  }
#endif
  wave_sync();  // S.a before the Schur system reads it

  STAMP(5);
  if constexpr (FORCES) {
    limb_forces<NM>(T, a, mp, S, limb, l, L, gbase, nl, live, b, fstep, s_glob, o, Jp, Jz, Pc, fp, xt, bad, big);
    return;
  }
  // ---- contact list in foot order (ftsolver's contact columns) ----
  const int fiL = T->link[L][2].foot;
  const uint32_t cm = grp_or((limb && contact) ? 1u << fiL : 0u);
  const int nc = __popc(cm);
  const bool mine = limb && contact;
  if (limb) LDBG(24 + fiL, fp[2], 25);
  // the limb lane holding contact rank l (lane l < nc of the group gathers that contact's values)
  int src = 0;
  for (int L2 = 0; L2 < nl; L2++) {
    const int f2 = T->link[L2][2].foot;
    if (((cm >> f2) & 1) && __popc(cm & ((1u << f2) - 1)) == l) src = L2;
  }
  src += gbase;
  const bool slot = l < nc;
  // joint values outside sincos_k_small's range: the fixup's
  bool defer = grp_any(big, gbase);
  // a routing decision within kNearBand of its guard: HS_FLAG_NEAR_RANK, as fast_solve sets it (the values
  // are hs_rollout_kernel's bitwise, so the decisions are its own)
  bool nearf = false;
  real y3[3] = {0, 0, 0};
  real d0[3] = {0, 0, 0}, Dinv[9], gc[3], Dp6[6];
  if (mine)
    for (int r = 0; r < 3; r++) d0[r] = o[r] - fp[r];  // A_c = [-I; [d0_c]x]
  if (mine && nc >= (HS_LIMB_NC12 ? 2 : 3)) contact_block(Jp, Jz, xt, fp, Dp6, gc);
#ifdef HS_LIMB_EXP_NOSOLVE
  defer |= nc >= 3;
  if (false) {
#else
  if (nc >= 3) {
#endif
    // zeroth_well_posed: the feet's scatter, in single precision, the contacts' d0 on lanes 0 .. nc - 1
    float e0 = grp_getf(float(o[0] - fp[0]), src), e1 = grp_getf(float(o[1] - fp[1]), src),
          e2 = grp_getf(float(o[2] - fp[2]), src);
    if (!slot) e0 = e1 = e2 = 0.f;
    {
      const float s0 = group8_sum(e0), s1 = group8_sum(e1), s2 = group8_sum(e2);
      const float q00 = group8_sum(e0 * e0), q11 = group8_sum(e1 * e1), q22 = group8_sum(e2 * e2);
      const float q01 = group8_sum(e0 * e1), q02 = group8_sum(e0 * e2), q12 = group8_sum(e1 * e2);
      const float k = float(nc);
      const float c00 = k * q00 - s0 * s0, c11 = k * q11 - s1 * s1, c22 = k * q22 - s2 * s2;
      const float c01 = k * q01 - s0 * s1, c02 = k * q02 - s0 * s2, c12 = k * q12 - s1 * s2;
      const float c2 = (c00 * c11 - c01 * c01) + (c00 * c22 - c02 * c02) + (c11 * c22 - c12 * c12);
      const float tq = q00 + q11 + q22;
      const float md = fmaxf(k, fmaxf(tq - q00, fmaxf(tq - q11, tq - q22)));
      const float t = kZerothGuard * k * (c00 + c11 + c22) * md;
      const bool well = c2 >= t;
      const bool nearz = c2 >= t / float(kNearBand) && c2 <= t * float(kNearBand);
      defer |= !well;  // the same on every lane of the group (group8_sum)
      nearf |= nearz;
    }
    STAMP(6);
    // the contact's Schur block of its first-order block D_c (contact_block)
    real sch[27];
#pragma unroll
    for (int e = 0; e < 27; e++) sch[e] = 0;
    bool lnear = false, ok = true;
    if (mine) {
      const real* Dp = Dp6;
      opaque_vals<3>(d0);
      const real D[9] = {Dp[0], Dp[1], Dp[3], Dp[1], Dp[2], Dp[4], Dp[3], Dp[4], Dp[5]};
      LDBG(24 + fiL, Dp[0], 6);
      LDBG(24 + fiL, gc[0], 7);
      real Lm[9];
      for (int i = 0; i < 9; i++) Lm[i] = D[i];
      real rl[3];
      ok = ldl_n<3>(Lm, kFastPivotGuard, rl, lnear);
      if (ok) {
        for (int j = 0; j < 3; j++) {
          real e[3] = {0, 0, 0};
          e[j] = 1;
          ldl_solve_n<3>(Lm, rl, e);
          for (int i = 0; i < 3; i++) Dinv[3 * i + j] = e[i];
        }
        // the block's Schur entries: row r of E = A_c D_c^-1, then (E A_c^T)(r, q) for q <= r, and h_r
#pragma unroll
        for (int r = 0; r < 6; r++) {
          real E[3];
#pragma unroll
          for (int j = 0; j < 3; j++) {
            real acc = 0;
#pragma unroll
            for (int i = 0; i < 3; i++) acc += a_entry(d0, r, i) * Dinv[3 * i + j];
            E[j] = acc;
          }
#pragma unroll
          for (int qq = 0; qq <= r; qq++) {
            real vv = 0;
#pragma unroll
            for (int j = 0; j < 3; j++) vv += E[j] * a_entry(d0, qq, j);
            sch[sch_lower(r, qq)] = vv;
          }
          real hh = 0;
          for (int j = 0; j < 3; j++) hh += E[j] * gc[j];
          sch[SCH_H + r] = hh;
        }
      }
    }
    defer |= grp_any(mine && !ok, gbase);  // a singular D_c: tier 2's
    nearf |= grp_any(mine && lnear, gbase);
    // what fast_solve_lanes stores in FastL and reads back for y (LDS): g_c, d0_c, D_c^-1
    opaque_vals<3>(gc);
    opaque_vals<9>(Dinv);
    // the blocks summed over the contacts by rank
    real Ssum[27];
#pragma unroll
    for (int e = 0; e < 27; e++) {
      real vv = grp_get(sch[e], src);
      Ssum[e] = rank8_sum(slot ? vv : real(0));
    }
    STAMP(7);
    // the 6 x 6 Schur complement system (every lane of the group: the same values)
    real lam[6];
    {
      opaque_vals<27>(Ssum);  // FastL::sc.Ssum
      real Sm[36], rl6[6];
#pragma unroll
      for (int i = 0; i < 6; i++)
#pragma unroll
        for (int j = 0; j < 6; j++) Sm[6 * i + j] = (j <= i) ? Ssum[sch_lower(i, j)] : real(0);
      for (int r = 0; r < 6; r++) lam[r] = S.a[r] - Ssum[SCH_H + r];
      bool near6 = false;
      const bool ok6 = ldl_n<6>(Sm, kFastPivotGuard, rl6, near6);
      defer |= !ok6;
      nearf |= near6;
      if (ok6) ldl_solve_n<6>(Sm, rl6, lam);
      opaque_vals<6>(lam);  // FastL::sc.lam
    }
    if (mine) {  // y_c = -D_c^-1 (g_c + A_c^T lam)
      real t[3];
#pragma unroll
      for (int i = 0; i < 3; i++) {
        real s = gc[i];
#pragma unroll
        for (int r = 0; r < 6; r++) {
          if (r < 3 && r != i) continue;
          if (r >= 3 && r - 3 == i) continue;
          s += a_entry(d0, r, i) * lam[r];
        }
        t[i] = s;
      }
      for (int i = 0; i < 3; i++) {
        real s = 0;
        for (int j = 0; j < 3; j++) s += Dinv[3 * i + j] * t[j];
        y3[i] = -s;
      }
      LDBG(24 + fiL, y3[0], 8);
      opaque_vals<3>(y3);  // sv.y
    }
  }
#if !HS_LIMB_NC12
  defer |= nc == 1 || nc == 2;  // (A/B: one and two contacts to the fixup launch)
  if (false) {
#else
  if (nc == 1 || nc == 2) {
#endif
    // fast_solve_lanes' one- and two-contact closed forms (its lane 0, from FastL): here on every lane of
    // the group, the contacts' values gathered from their limb lanes
    int s0 = 0, s1 = 0;
    for (int L2 = 0; L2 < nl; L2++) {
      const int f2 = T->link[L2][2].foot;
      if ((cm >> f2) & 1) {
        const int r2 = __popc(cm & ((1u << f2) - 1));
        if (r2 == 0) s0 = L2;
        if (r2 == 1) s1 = L2;
      }
    }
    s0 += gbase;
    s1 += gbase;
    const real a[6] = {S.a[0], S.a[1], S.a[2], S.a[3], S.a[4], S.a[5]};
    bool lnear = false, ok;
    real y[6];
    if (nc == 1) {  // unique least-squares solution (A^T A) w = -A^T a
      real dd[3];
      for (int r = 0; r < 3; r++) dd[r] = grp_get(d0[r], s0);
      real M[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, bv[3] = {0, 0, 0};
      for (int i = 0; i < 3; i++) {
        for (int j = 0; j < 3; j++)
          for (int r = 0; r < 6; r++) M[3 * i + j] += a_entry(dd, r, i) * a_entry(dd, r, j);
        for (int r = 0; r < 6; r++) bv[i] -= a_entry(dd, r, i) * a[r];
      }
      real rl[3];
      if (mine) LDBG(24 + fiL, M[4], 19);
      if (mine) LDBG(24 + fiL, bv[1], 20);
      ok = chol_n<3>(M, kFastPivotGuard, rl, lnear);
      if (ok) chol_solve_n<3>(M, rl, bv);
      for (int i = 0; i < 3; i++) y[i] = bv[i];
      if (mine && ok) LDBG(24 + fiL, bv[0], 21);
    } else {  // rank 5: kernel n = (u,-u)/sqrt2 along the line between the feet
      real f0[3], f1[3], dA[2][3], Dc[2][6], gg[2][3];
      for (int r = 0; r < 3; r++) {
        f0[r] = grp_get(fp[r], s0);
        f1[r] = grp_get(fp[r], s1);
        dA[0][r] = grp_get(d0[r], s0);
        dA[1][r] = grp_get(d0[r], s1);
        gg[0][r] = grp_get(gc[r], s0);
        gg[1][r] = grp_get(gc[r], s1);
      }
      for (int e = 0; e < 6; e++) {
        Dc[0][e] = grp_get(Dp6[e], s0);
        Dc[1][e] = grp_get(Dp6[e], s1);
      }
      const real Dm[2][9] = {{Dc[0][0], Dc[0][1], Dc[0][3], Dc[0][1], Dc[0][2], Dc[0][4], Dc[0][3], Dc[0][4], Dc[0][5]},
                             {Dc[1][0], Dc[1][1], Dc[1][3], Dc[1][1], Dc[1][2], Dc[1][4], Dc[1][3], Dc[1][4], Dc[1][5]}};
      real u[3], un = 0;
      for (int r = 0; r < 3; r++) { u[r] = f0[r] - f1[r]; un += u[r] * u[r]; }
      un = sqrt(un);
      ok = un > real(1e-12);
      real nv[6], M[36], bv[6], rl[6];
      if (ok) {
        for (int r = 0; r < 3; r++) { nv[r] = u[r] / un / sqrt(real(2)); nv[3 + r] = -nv[r]; }
        const bool first = mine && __popc(cm & ((1u << fiL) - 1)) == 0;
        if (first) LDBG(24 + fiL, nv[2], 26);
        for (int i = 0; i < 6; i++) {
          const real* di = dA[i / 3];
          for (int j = 0; j < 6; j++) {
            const real* dj = dA[j / 3];
            real sv = 0;
            for (int r = 0; r < 6; r++) sv += a_entry(di, r, i % 3) * a_entry(dj, r, j % 3);
            M[6 * i + j] = sv + nv[i] * nv[j];
          }
          real sv = 0;
          for (int r = 0; r < 6; r++) sv += a_entry(di, r, i % 3) * a[r];
          bv[i] = -sv;
        }
        if (first) LDBG(24 + fiL, M[5], 27);
        opaque_vals<36>(M);  // as hs_rollout_kernel's fast_solve_lanes fences them
        opaque_vals<6>(bv);
        opaque_vals<6>(nv);
        ok = chol_n<6>(M, kFastPivotGuard, rl, lnear);
      }
      if (ok) {
        chol_solve_n<6>(M, rl, bv);
        opaque_vals<6>(bv);
        real nDn = 0, nr = 0;
        for (int c = 0; c < 2; c++)
          for (int i = 0; i < 3; i++) {
            real Dw = 0, Dn = 0;
            for (int j = 0; j < 3; j++) { Dw += Dm[c][3 * i + j] * bv[3 * c + j]; Dn += Dm[c][3 * i + j] * nv[3 * c + j]; }
            nr += nv[3 * c + i] * (Dw + gg[c][i]);
            nDn += nv[3 * c + i] * Dn;
          }
        ok = nDn > 0;
        if (ok) {
          real t = -nr / nDn;
          for (int i = 0; i < 6; i++) y[i] = bv[i] + t * nv[i];
          if (mine && __popc(cm & ((1u << fiL) - 1)) == 0) {
            LDBG(24 + fiL, y[0], 22);
            LDBG(24 + fiL, bv[0], 23);
            LDBG(24 + fiL, t, 24);
          }
        }
      }
    }
    defer |= !ok;  // the same on every lane of the group
    nearf |= lnear;
    if (mine && ok) {
      const int rk = __popc(cm & ((1u << fiL) - 1));
      for (int i = 0; i < 3; i++) y3[i] = rk == 0 ? y[i] : y[3 + i];
      opaque_vals<3>(y3);  // sv.y
    }
  }
  STAMP(8);
#if HS_LIMB_NEAR_DEFER
  defer |= nearf;
#endif
  if (defer) {  // the whole step to the fixup launch (hs_rollout_kernel FIX_SOLVE)
    if (l == 0 && live) {
      atomicAdd(&g_limb_deferred, 1ull);  // hs_limb_stats
      const int it = atomicAdd(mp.fix_count, 1);
      mp.fix_items[2 * it] = fstep;
      mp.fix_items[2 * it + 1] = mp.limb_slots ? mp.limb_slots[q * LGR + grp] : b;  // 2 * wavefront + half of hs_rollout_kernel's layout
    }
    return;
  }

  // ---- S4: motor torques, contact forces, work (step()'s outputs) ----
  const size_t orow = (size_t)b * a.horizon + s_glob;
  bool nan = false;
  real wl[3] = {0, 0, 0};  // this limb's three work terms, its motors in link order
  bool lm = true;          // its motors are joints 3 L, 3 L + 1, 3 L + 2 (limb-major joint order)
  if (limb) {
#pragma unroll
    for (int kk = 0; kk < 3; kk++) {
      const int hh = T->link[L][kk].hinge;
      real d[3], yy[3];
#pragma unroll
      for (int rr = 0; rr < 3; rr++) {
        d[rr] = Jp[kk][rr] - fp[rr];
        yy[rr] = mine ? y3[rr] : real(0);
      }
      real tq = real(0);
#pragma unroll
      for (int r = 0; r < 3; r++) {
        real s = real(0);
#pragma unroll
        for (int jj = 0; jj < 3; jj++)
          if (jj != r) s = s + cross_e(d, jj, r) * yy[jj];
        real xr = xt[kk][r] + s;
        tq = tq + Jz[kk][r] * xr;
      }
      real dw = tq * jvel[kk];
      S.wd[hh] = (dw > 0) ? dw : 0;
      wl[kk] = (dw > 0) ? dw : 0;
      lm &= hh == 3 * L + kk;
      nan |= tq != tq;
      if (live && a.tau) outp(a.tau)[orow * mp.st_tau + hh] = tq;
    }
    if (mine)
      for (int j = 0; j < 3; j++) nan |= y3[j] != y3[j];
    if (live && a.cf)
      for (int j = 0; j < 3; j++) {
        real zv = -real(0);
        if (mine) zv = -(real(0) + (real(-1)) * y3[j]);
        outp(a.cf)[orow * mp.st_cf + 3 * fiL + j] = zv;
      }
  }
  // a mixed plan's rows past this model's joints and feet (hs_rollout_kernel writes them 0; a single model's
  // rows have none: the loops' code is kept off its path, ~1 % at K = 200, r06_t17)
  if (HS_LIMB_PAD && live && mp.limb_rollouts) {
    if (a.tau)
      for (int c = nmj + l; c < mp.st_tau; c += LG) outp(a.tau)[orow * mp.st_tau + c] = real(0);
    if (a.cf)
      for (int c = 3 * T->nf + l; c < mp.st_cf; c += LG) outp(a.cf)[orow * mp.st_cf + c] = real(0);
  }
  const bool any_nan = grp_any(nan, gbase), any_bad = grp_any(limb && bad, gbase);
#if HS_LIMB_WORK_DPP
  // the joint-order sum work_over_period takes, as a chain across the limb lanes when the joints are
  // limb-major (lane l adds its three terms, in order, to lane l - 1's partial sum: the same additions in
  // the same order as the loop over S.wd), else the loop
  const bool chain = !grp_any(limb && !lm, gbase) && nmj == 3 * nl;
  real wsum = 0;
  if (chain) {
    real sacc = ((real(0) + wl[0]) + wl[1]) + wl[2];
    for (int k = 1; k < nl; k++) {
      const real prev = dpp_r<0x111>(sacc);  // row_shr 1: lane l - 1's partial sum
      if (l >= 1) sacc = ((prev + wl[0]) + wl[1]) + wl[2];
    }
    wsum = grp_get(sacc, gbase + nl - 1);
  }
#endif
  wave_sync();
  if (l == 0 && live) {
    uint32_t flags = 0;
    if (nc == 0) flags |= HS_FLAG_NO_CONTACT;
    if (nc == 1) flags |= HS_FLAG_FULL_RANK;
    if (nearf) flags |= HS_FLAG_NEAR_RANK;
    if (any_nan) flags |= HS_FLAG_NAN;
    if (any_bad) flags |= HS_FLAG_UNREACH;
    if (a.flags) a.flags[orow] = flags;
    // the joints' positive work in joint order (work_over_period's loop, periodic.cpp:294-300), summed over
    // the steps in order by the reduce
    real work_dt = real(0);
#if HS_LIMB_WORK_UNROLL
    real wdv[HS_NMAX];
#pragma unroll
    for (int jj = 0; jj < HS_NMAX; jj++) wdv[jj] = S.wd[jj];  // issued together; only the nmj terms summed
#pragma unroll
    for (int jj = 0; jj < HS_NMAX; jj++) work_dt = jj < nmj ? work_dt + wdv[jj] : work_dt;
#elif HS_LIMB_WORK_DPP
    if (chain) work_dt = wsum;
    else
      for (int jj = 0; jj < nmj; jj++) work_dt += S.wd[jj];
#else
    for (int jj = 0; jj < nmj; jj++) work_dt += S.wd[jj];
#endif
    reinterpret_cast<real*>(mp.fused_work)[(size_t)s_glob * a.n_rollouts + b] = work_dt;
  }
  STAMP(9);
  RSTAMP(17);
}
