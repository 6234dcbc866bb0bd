// hs_topo.h -- flat, device-resident description of one robot model.
//
// Built once on the host by hs_model_load() (hs_model.cpp) from the MuJoCo-style
// XML and copied to HBM; every wavefront reads it through the scalar cache
// (all addresses are wave-uniform). It replaces the pointer-linked tree of
// reference model.h:34-137 (modelnode/modeljoint), the odepart geometry of
// visualization.h:93-120 and the liksolver tables of lik.cpp:7-78.
#pragma once
#include <stdint.h>

#define HS_NMAX 24  // parts (hexapod 22, spider 19, myant 17)
#define HS_LMAX 6   // limbs / feet
#define HS_KMAX 18  // 3 * contacts
#define HS_CMAX 6   // children per node
#define HS_CHAIN_MAX 6  // ancestors of a foot below the root (hexapod 4)

enum { HS_J_NONE = -1, HS_J_FREE = 0, HS_J_HINGE = 1 };
enum { HS_LIK_YXX = 0, HS_LIK_ZXX = 1 };

// 3x4 rigid transform, column-major: m[c*3 + r], c = 0..3 (c = 3 is translation).
// The implicit bottom row is (0,0,0,1): the reference's 4x4 product
// (matrix.cpp:78-97) adds A(j,3)*B(3,i) = A(j,3)*0 for i < 3 and A(j,3)*1 for
// i = 3, both exact, so the 3x4 product rounds identically.
struct hs_aff34 { double m[12]; };

struct hs_node {
  hs_aff34 J_A_parent;  // modeljoint::A_parent (model.cpp:119-174)
  hs_aff34 A_pj_body;   // modelnode::A_pj_body
  double com[3];        // odepart::A_body_geom translation (get_com_pos, visualization.cpp:541-545)
  double cap[3];        // odepart::capsule_to_pos (get_foot_pos, visualization.cpp:553-568)
  int32_t parent, jtype, depth, nkids;
  int32_t kids[HS_CMAX];
  int32_t foot;         // foot index (preorder) or -1
  int32_t hinge;        // motor index (0..nmj-1) or -1
  int32_t owner_limb;   // limb lane that computes this node's FK/features
  int32_t limb_below;   // limb whose foot is at/below this node, -1 if none or several
  int32_t size;         // nodes in this node's subtree (preorder table: the subtree is [i, i + size))
};

#define HS_OWN_MAX 2  // chain bodies one limb lane computes

// one limb link for the rollout kernels' limb FK (hs_topo::link)
struct hs_link {
  hs_aff34 P;      // A_pj_body of the previous link times this link's J_A_parent (unused for link 0)
  double Rpj[9];   // rotation of this link's A_pj_body, column-major [c * 3 + r]
  double com[3];   // A_pj_body * com
  double cap[3];   // A_pj_body * cap (the foot link)
  int32_t foot, hinge;  // node[] foot / hinge of the link
};

struct hs_topo {
  int32_t n, nf, nmj, cfg;
  int32_t n_limbs, lik_kind, max_depth;
  int32_t torso_mask;      // switch_torso_penalty (ftsolver.cpp:262-273): bit 0 force, bit 1 torque rows in stage 0 (default 3)
  double ls[3];            // link lengths (lik.cpp:226-227)
  double rcap;             // foot capsule radius (lik.cpp:132-140)
  double total_mass;       // sum of part masses (periodic.cpp:320-325)
  double mass[HS_NMAX];    // dBodyGetMass default = 1 (dynrec.cpp:62-68)
  int32_t footis[HS_LMAX];       // foot part ids, preorder (periodic.cpp:34-58)
  int32_t hinge_ids[HS_NMAX];    // hinge part ids, preorder (periodic.cpp:311-319)
  int32_t limb_child[HS_LMAX];   // limb top-link node (lik.cpp:50-63)
  int32_t limb_parent[HS_LMAX];
  int32_t limb_foot[HS_LMAX];    // foot node of each limb (lik.cpp:453-455)
  int32_t limb_ysign[HS_LMAX];   // lik.cpp:230-245
  int32_t limb_pergen[HS_LMAX];  // likpergen_map (pergen.cpp:243-262)
  int32_t limb_node[HS_LMAX][3];        // the limb's three hinged links, top first
  int32_t limb_chain_len[HS_LMAX];      // nodes from root to limb parent (inclusive)
  int32_t limb_chain[HS_LMAX][HS_NMAX]; // root ... limb parent
  // index tables that turn pointer chases into independent loads:
  int32_t foot_chain_len[HS_LMAX];      // ancestors of foot fi with a parent (foot part first)
  int32_t foot_chain[HS_LMAX][HS_NMAX];
  int32_t hinge_foot[HS_NMAX];          // node[hinge_ids[j]].limb_below by motor index j
  hs_node node[HS_NMAX];
  // (after node[], so the fields above keep their offsets) motor j's subtree in the preorder
  // table: hinge_ids[j] | (hinge_ids[j] + its size) << 8, one load for solve_forces' subtree tests
  int32_t hinge_range[HS_NMAX];
  // Per-limb kinematics plan: everything a limb lane of the rollout kernels reads, at addresses that
  // depend on the limb alone (no node-id chase). Chain bodies the limb computes (owner_limb == L, the
  // root aside; never a foot), in chain order:
  int32_t limb_own_n[HS_LMAX];
  int32_t limb_own[HS_LMAX][HS_OWN_MAX];
  double limb_own_com[HS_LMAX][HS_OWN_MAX][3];
  // its three links precombined (limb_fk): with H_k = J_k Rz(q_k) the link's hinge frame and pj_k its
  // A_pj_body, the body frame is A_k = H_k pj_k and the next joint frame J_(k+1) = H_k (pj_k Jp_(k+1)),
  // one product per link; the features come from H_k: pos = H_k (pj_k com_k), the foot H_2 (pj_2 cap)
  struct hs_link link[HS_LMAX][3];
  // the gait setup's chain products from the torso's body frame A0 (limb_setup, one product per frame):
  // its owned bodies' frames A0 own_rel[m], its hip joint frame J0 = A0 hip_rel (poslimb, lik.cpp:341-347),
  // and the limb child's A_pj_body translation (get_limb_hip_pos: J0 Rz(0) pj_child's column 3)
  hs_aff34 limb_own_rel[HS_LMAX][HS_OWN_MAX];
  hs_aff34 limb_hip_rel[HS_LMAX];
  double limb_child_t[HS_LMAX][3];
  // foot_chain packed for the rollout kernels' LDS copy: foot fi's bytes [len, chain[0], ..., chain[len - 1]]
  // (len <= HS_CHAIN_MAX < 8, node ids < 256) in two little-endian words
  uint32_t foot_chain8[HS_LMAX][2];
  // the limb-lane step kernel's topology class (hs_limb.h; set by the loader): every limb's three links
  // consecutive in preorder with subtree sizes 3, 2, 1, its foot on the third link only, one limb per
  // foot, every motor a limb link, at most one chain body per limb (limb_own_n <= 1), at most 7 limbs
  // (lane 7 of a rollout's group is the torso's)
  int32_t limb_lane_ok;
};
