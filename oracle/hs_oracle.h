/*
 * hs_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement ("oracle") of the HSLabs control-loop hot path
 * (pergen -> lik -> FK -> dynrec -> ftsolver -> motor torques), used as the
 * parity checker for the HIP product path and as the bench's cpu_baseline leg.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline may load it.
 * The product (hslabs_amd/, include/hslabs.h) never links or calls this code.
 *
 * Parity status: the reference (ODE + Eigen + rapidxml)
 * cannot be built in this image, so this restatement is pinned by the
 * reference's own self-checks restated as known-answer tests (IK round trip
 * lik.cpp:371-404, rot_ztov check visualization.cpp:24, Euler round trip
 * pergen.cpp:377-383, rank-loop residual ftsolver.cpp:228-232, static-stance
 * force balance) and by an independent numpy/scipy formulation in tests/.
 * Against the reference binary itself: "parity unpinned".
 */
#ifndef HS_ORACLE_H
#define HS_ORACLE_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* Gait setup parameters: the fields of pgsconfigparams (pergen.h:137-146),
 * same meaning as a pgs_config.txt line (player.cpp:170-208). */
typedef struct {
  double torso_pos[3];
  double torso_angles[3];
  double step_duration;
  double period, step_length, step_height;
  double curvature;
  double foot_shift;       /* value of lateral/radial foot shift */
  int32_t foot_shift_type; /* -1 none, 0 lateral, 1 radial (pergen.h:143) */
  int32_t rec_transform_flag; /* pergensetup::rec_transform_flag (pergen.h:76) */
  double rec_transl[3], rec_eas[3]; /* set_rec_transform (pergen.cpp:316-320) */
} hso_gait;

/* null-space basis modes */
enum { HSO_BASIS_ORTHO = 0, /* reference-faithful: orthonormal Q of QR(B^T) (ftsolver.cpp:187-202) */
       HSO_BASIS_TREE = 1,  /* tree-built basis [-B0^-1 Bc; I], Eigen-style LU/QR loop */
       HSO_BASIS_FAST = 2   /* tree basis + closed-form Schur solve (the HIP kernel's fast path),
                               falling back to the TREE path when ill-conditioned */ };

/* flag bits per step (also used by the product, see include/hslabs.h) */
#define HSO_FLAG_RANK_RETRY   1u  /* adaptive-rank loop ran more than once (ftsolver.cpp:207-232) */
#define HSO_FLAG_FULL_RANK    2u  /* zeroth-order Gram full rank: reference would assert in comma init */
#define HSO_FLAG_LOOP_EXHAUST 4u  /* rank loop reached rank 0 without converging */
#define HSO_FLAG_NAN          8u  /* NaN in torques / contact forces */
#define HSO_FLAG_UNREACH     16u  /* an IK target was clamped (ignore_reach, lik.cpp:250-253) */
#define HSO_FLAG_NO_CONTACT  32u  /* k == 0 */
#define HSO_FLAG_GENERAL     64u  /* FAST mode: closed form declined, Eigen-style path used */
#define HSO_FLAG_DEPENDENT  512u  /* solve_forces: a column dropped as dependent, the basic solution returned
                                     (with HSO_FLAG_GENERAL; one point of a non-unique solution set) */
#define HSO_FLAG_NEAR_RANK  256u  /* a rank / routing decision within rounding of its threshold (NearTrack):
                                     another rounding may decide it the other way (HS_FLAG_NEAR_RANK) */

typedef struct hso_model hso_model;

int hso_model_load(const char* xml_path, hso_model** out);
void hso_model_free(hso_model* m);
/* n_parts, nmj, nfeet, config_dim, lik variant, n_limbs */
void hso_model_dims(const hso_model* m, int* dims6);
/* periodic::switch_torso_penalty -> forcetorquesolver::switch_torso_penalty (ftsolver.cpp:262-273):
 * which torso rows (force, torque) form the zeroth-order stage of every later solve of this model
 * (default (1,1), player.cpp:263). (0,0) returns -2: the reference exits (ftsolver.cpp:245). */
int hso_model_set_torso_penalty(hso_model* m, int force, int torque);

/*
 * One rollout, processing steps k = k0 .. k0+H-1, i.e. trajectory samples
 * i = k+2 (periodic.cpp:377-391 uses i in [2, n_t+2) with k0=0, H=n_t).
 * Outputs (any pointer may be NULL):
 *   q    [(k0+H+4) x config_dim]  trajectory records (periodic.cpp:166-185)
 *   tau  [H x nmj]                motor torques (periodic.cpp:328-343)
 *   cf   [H x 3*nfeet]            contact forces z (ftsolver.cpp:163)
 *   x    [H x 6n]                 joint force/torque vector (ftsolver.cpp:166)
 *   flags[H]
 *   work_cot[2]                   positive work over the processed steps and
 *                                 work/(sum m * step_length) (player.cpp:269-285)
 *   diag [H x 4]                  k, final rank0, loop iterations, rel_error
 * ignore_reach: lik.cpp:142 global (main.cpp:41 sets it).
 */
int hso_rollout(const hso_model* m, const hso_gait* g, int n_t, int k0, int H, int basis,
                int ignore_reach, double* q, double* tau, double* cf, double* x,
                uint32_t* flags, double* work_cot, double* diag);

/* Batched CPU baseline: B rollouts (params[B]), same k0/H for all, tree basis,
 * n_threads std::threads over rollouts. Outputs tau[B][H][nmj], cf[B][H][3nf],
 * work_cot[B][2]. Returns 0 on success. */
/* forcetorquesolver::solve_forces via periodic::solve_contforces_given_torques
 * (ftsolver.cpp:331-378, periodic.cpp:368-374): tau_in [H][nmj] -> cf [H][3 nf]
 * for ALL feet; flags HSO_FLAG_GENERAL when the least squares is rank deficient. */
int hso_forces(const hso_model* m, const hso_gait* g, int n_t, int k0, int H, int ignore_reach, const double* tau_in,
               double* cf, uint32_t* flags);
/* hso_forces under a chosen rank rule for the (numerically) rank-deficient least squares:
 * HSO_FORCES_KERNEL (hso_forces: the kernel's pivot guard, 1e-10 of the reduced normal matrix's largest
 * diagonal, force columns in natural order) or HSO_FORCES_SPARSEQR (Eigen SparseQR's default threshold,
 * 20 (rows + cols) eps max column norm on |r_kk|, every column in natural order; COLAMD not restated).
 * A dropped column sets HSO_FLAG_GENERAL | HSO_FLAG_DEPENDENT. */
#define HSO_FORCES_KERNEL 0
#define HSO_FORCES_SPARSEQR 1
int hso_forces_rule(const hso_model* m, const hso_gait* g, int n_t, int k0, int H, int ignore_reach, int rule,
                    const double* tau_in, double* cf, uint32_t* flags);
/* hso_forces for B rollouts on n_threads threads: tau_in [B][H][nmj] -> cf [B][H][3 nf], flags [B][H] */
int hso_forces_batch(const hso_model* m, const hso_gait* params, int B, int n_t, int k0, int H, int ignore_reach,
                     int n_threads, const double* tau_in, double* cf, uint32_t* flags);
int hso_batch(const hso_model* m, const hso_gait* params, int B, int n_t, int k0, int H,
              int basis, int ignore_reach, int n_threads, double* tau, double* cf,
              double* work_cot, uint32_t* flags);
/* hso_batch plus, per step, the margin of the decision closest to its threshold and its kind
 * (nearv [B][H][2]: margin, HSO_NEAR_* category; margin <= 1 sets HSO_FLAG_NEAR_RANK) */
int hso_batch_near(const hso_model* m, const hso_gait* params, int B, int n_t, int k0, int H,
                   int basis, int ignore_reach, int n_threads, double* tau, double* cf,
                   double* work_cot, uint32_t* flags, double* nearv);

/* Known-answer helpers (restated reference self-checks). */
/* lik.cpp:371-404: bend_solver o limb_solver round trip; returns max error over n tries */
double hso_lik_roundtrip(const hso_model* m, int n, uint64_t seed);
/* visualization.cpp:62-101: affine_from_orientation o euler_angles_from_affine */
void hso_euler_roundtrip(const double* angles3, double* out3);
/* rot_ztov (visualization.cpp:11-25): R (affine column-major 3x3 part, 9 doubles) */
void hso_rot_ztov(const double* v3, double* R9);
/* FK after IK: foot positions vs pergen targets for record at time t; out: max |err| */
double hso_fk_ik_check(const hso_model* m, const hso_gait* g, double t, int ignore_reach);
/* per-configuration kinematics (the product's hs_pergen_rec / hs_model_lik / hs_model_fk):
 * pergensetup::set_rec at time t (pergen.cpp:225-239) after setup_pergen: rec [6 + 3 n_limbs] */
int hso_pergen_rec(const hso_model* m, const hso_gait* g, double t, double* rec);
/* kinematicmodel::set_jvalues_with_lik (model.cpp:354-359) on a copy of the model holding config
 * (in/out, [config_dim]); returns 0, or -10 when a target is out of reach without ignore_reach
 * (lik.cpp:321-330); *unreach = 1 when a target was clamped */
int hso_lik(const hso_model* m, const double* rec, int ignore_reach, double* config, int* unreach);
/* kinematicmodel::set_jvalues + recompute_modelnodes (model.cpp:314-318, 361-366): A_ground of every
 * node and of its joint (zeros without one), 3x4 column-major (12 doubles, [c*3 + r]) per node */
int hso_fk(const hso_model* m, const double* config, double* a_ground, double* a_joint);
/* static residual checks for one step: |B0 x0 - f|, |[B0 Bc] N| (both bases) */
int hso_residuals(const hso_model* m, const hso_gait* g, int n_t, int step, int basis, double* out2);

/* Dynamics record of one step (sample i = step+2) for independent cross-checks:
 * pos/jpos/jz/mom_rate/ang_mom_rate [n*3], fpos [nf*3], contacts [nf], parents [n], footis [nf],
 * hinge_ids [nmj]. Returns k = 3 * #contacts. */
int hso_dynrec_dump(const hso_model* m, const hso_gait* g, int n_t, int step, double* pos, double* jpos,
                    double* jz, double* mom_rate, double* amr, double* fpos, int32_t* contacts,
                    int32_t* parents, int32_t* footis, int32_t* hinge_ids);

/* ---- closed-loop simulation (hs_oracle_sim.cpp): modelplayer::simulate_ode with position
 * control on a restated ODE 0.13 dWorldQuickStep (player.cpp:325-339, visualization.cpp:296-337).
 * Body state rows: pos[3], quaternion (w,x,y,z)[4], lvel[3], avel[3] per part (preorder). */
/* init_play_config (player.cpp:351-356): configuration -> body states (zero velocities) */
int hso_sim_reset(const hso_model* m, const double* config, double* body);
/* dJointGetHingeAngle / Rate of every motor for a body state */
int hso_sim_hinges(const hso_model* m, const double* body, double* q, double* dq);
/* n_steps simulation steps of one rollout. p10 = dt, k, sor_w, erp, cfm, gravity, bounce,
 * bounce_vel, soft_cfm, mu. Tables as hs_run writes them with k0 = 0, H = n_t:
 * q_tab/dq_tab [n_t][config_dim], tau_tab [n_t][nmj] (row h = trajectory sample h + 2).
 * seed: dRand state, tsi: play step index; both advanced. Outputs per step (may be NULL):
 * tau_cmd/q_meas [n_steps][nmj], torso [n_steps][3], n_contacts [n_steps], normal_force [n_steps]. */
int hso_sim_run(const hso_model* m, const double* p10, int iterations, int n_t, const double* q_tab,
                const double* dq_tab, const double* tau_tab, double* body, uint32_t* seed, int32_t* tsi,
                int n_steps, double* tau_cmd, double* q_meas, double* torso, int32_t* n_contacts,
                double* normal_force);

#ifdef __cplusplus
}
#endif
#endif
