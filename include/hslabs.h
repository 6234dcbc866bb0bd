/*
 * hslabs.h -- C ABI of the MI355X-native HSLabs control-loop path.
 *
 * Drop-in boundary for the reference's pergen -> lik -> FK -> dynrec ->
 * ftsolver -> motor-torque path. The reference exposes this path only as C++
 * classes (no FFI); each entry point below names the reference interface it
 * replaces (file:line in underactuated/HSLabs). Plain pointers and sizes only;
 * no HIP or torch types. All functions return 0 on success and a negative
 * HS_E* code on failure (never exit(), unlike lik.cpp:321-330 / pergen.cpp:12);
 * hs_last_error() returns a thread-local message for the last failure.
 *
 * Threading: a model handle is immutable after load and may be shared by
 * threads; hs_run() calls on distinct streams are independent.
 */
#ifndef HSLABS_H
#define HSLABS_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define HSLABS_ABI_VERSION 15

enum {
  HS_OK = 0,
  HS_E_ARG = -1,        /* bad argument / size */
  HS_E_IO = -2,         /* file not found / unreadable */
  HS_E_PARSE = -3,      /* malformed XML or config line (model.cpp:224-244, player.cpp:170-208) */
  HS_E_TOPOLOGY = -4,   /* model outside the supported topology class */
  HS_E_NOLIK = -5,      /* no limb IK variant for this model (lik.cpp:7-20) */
  HS_E_DEVICE = -6,     /* HIP runtime error */
  HS_E_NOTFOUND = -7    /* config id not present (player.cpp:243) */
};

/* Per-step flag bits (hs_run_args.flags). */
#define HS_FLAG_RANK_RETRY   1u  /* adaptive-rank loop iterated (ftsolver.cpp:208-232) */
#define HS_FLAG_FULL_RANK    2u  /* zeroth-order Gram full rank (reference asserts in its comma initializer) */
#define HS_FLAG_LOOP_EXHAUST 4u  /* rank loop reached rank 0 without converging */
#define HS_FLAG_NAN          8u  /* NaN in torques or contact forces */
#define HS_FLAG_UNREACH     16u  /* an IK target was clamped (ignore_reach, lik.cpp:250-253) */
#define HS_FLAG_NO_CONTACT  32u  /* no foot in contact (k = 0) */
#define HS_FLAG_GENERAL     64u  /* closed-form solve declined (conditioning guard): Eigen-style
                                    FullPivLU/ColPivQR path used (informational) */
#define HS_FLAG_NEAR_RANK  256u  /* a rank or routing decision of the step lay within rounding of its
                                    threshold, so another rounding (another basis, FMA contraction,
                                    the other precision) may decide it the other way: a FullPivLU pivot
                                    within 4x of the rank threshold in use (ftsolver.cpp:208-214), the
                                    threshold doubled (:212-214), rel_error in [1e-7, 1e-5] against the
                                    loop's 1e-6 (:228-232), a ColPivQR column norm within 4x of its
                                    nonzero-pivot threshold, the closed form's collinearity guard or
                                    pivot guards within 4x of theirs; the Eigen-style path's second
                                    stage ill-conditioned (a kept ColPivQR pivot under 1e-7 of the first,
                                    the parity bound); solve_forces: a normal-matrix pivot within 4x of
                                    its rank guard (ftsolver.cpp:349-353). The
                                    step's outputs are the path's answer; equality with another
                                    implementation is only expected where neither side sets this, or
                                    where the answer does not depend on the decision. */
#define HS_FLAG_DEPENDENT  512u  /* solve_forces only (hs_run_forces*), with HS_FLAG_GENERAL: the least
                                    squares is numerically rank deficient under the kernel's guard (a
                                    reduced normal-matrix pivot under 1e-10 of its largest diagonal) and
                                    the dropped force components are 0 -- the basic solution, one point
                                    of a non-unique solution set. The reference's SparseQR
                                    (ftsolver.cpp:349-353) drops a column only under
                                    20 (rows + cols) eps max |column| (~1e-12 relative, its COLAMD
                                    order), so on such steps it may keep the column and return the
                                    ill-conditioned full solution: parity is not claimed here. */

/* Gait setup of one rollout: the fields of pgsconfigparams (pergen.h:137-146),
 * same meaning and units as a pgs_config.txt line (player.cpp:170-208), plus
 * pergensetup's record transform (pergen.h:75-76). 192 bytes; the kernels read
 * the first 104 and the transform only where rec_transform_flag is set. */
typedef struct {
  double torso_pos[3];     /* "torso_pos" */
  double torso_angles[3];  /* "torso_angles" (Euler phi, theta, psi; model.cpp:45) */
  double step_duration;    /* in [0,1] (pergen.cpp:30-51) */
  double period;           /* T */
  double step_length;      /* L */
  double step_height;      /* h */
  double curvature;        /* 0 = straight (pergen.cpp:160-198) */
  double foot_shift;       /* lateral_foot_shift / radial_foot_shift value */
  int32_t foot_shift_type; /* -1 none, 0 lateral, 1 radial */
  int32_t rec_transform_flag; /* pergensetup::rec_transform_flag (pergen.cpp:206, 319): 1 = every
                                 record is transformed by rec_transform (set_rec, pergen.cpp:238) */
  double rec_transl[3];    /* rec_transform = affine_from_orientation({rec_transl, rec_eas})   */
  double rec_eas[3];       /* (set_rec_transform / set_rec_rotation, pergen.cpp:309-320)       */
  double reserved[5];
} hs_gait_params;

typedef struct hs_model_s* hs_model_t;

typedef struct {
  int32_t n_parts;     /* dynparts / model nodes (periodic.h:45) */
  int32_t nmj;         /* motor joints (model.h:114 number_of_motor_joints) */
  int32_t nfeet;       /* periodic.h:48 get_nfeet */
  int32_t config_dim;  /* model.h:125 get_config_dim */
  int32_t n_limbs;     /* liksolver::get_number_of_limbs (lik.h:48) */
  int32_t lik_kind;    /* 0 = y-x-x legs (lik.cpp:151), 1 = z-x-x legs (lik.cpp:189) */
  double total_mass;   /* periodic::get_total_mass (periodic.cpp:320) */
  double rcap;         /* liksolver::get_rcap (lik.h:50) */
} hs_model_dims;

/* Replaces kinematicmodel::load_fromxml (model.cpp:224-244) + liksolver ctor
 * (lik.cpp:7-20) + periodic::set_dynparts (periodic.cpp:34-58). The IK variant
 * is chosen by basename like lik.cpp:9-11 ("myant.xml", "hexapod.xml",
 * "spider.xml"); hs_model_load_ex(lik_variant >= 0) selects it explicitly
 * (0 = myant, 1 = hexapod, 2 = spider tables). */
int hs_model_load(const char* xml_path, hs_model_t* out);
int hs_model_load_ex(const char* xml_path, int lik_variant, hs_model_t* out);
void hs_model_free(hs_model_t model);
int hs_model_get_dims(hs_model_t model, hs_model_dims* out);

/* periodic::switch_torso_penalty -> forcetorquesolver::switch_torso_penalty (ftsolver.cpp:262-273):
 * which torso rows form the zeroth-order stage of the contact solve (penal_mask0: the torso force
 * rows with `force`, the torso torque rows with `torque`); the other torso rows join the first-order
 * stage with weight 1 (set_penal_mask1, ftsolver.cpp:291-303; set_action_penalties 239-246). Applies
 * to every later call on this model (hs_run*, hs_batch_*, and mixed plans created afterwards).
 * The default is the reference's only call, (1,1) (player.cpp:263); with another mask every step
 * takes the Eigen-style path (the closed form is the (1,1) problem's; flags carry HS_FLAG_GENERAL).
 * (0,0) is HS_E_ARG: the reference exits with "mask0 not set" (ftsolver.cpp:245). Waits for the
 * work queued on the devices that hold the model. Not concurrent with hs_run* on the same model
 * (like the reference's solver state, the setting belongs to the model): a launch issued by another
 * thread while this call runs may see the old mask on the device and the new one on the host. */
int hs_model_set_torso_penalty(hs_model_t model, int32_t force, int32_t torque);
int hs_model_get_torso_penalty(hs_model_t model, int32_t* force, int32_t* torque);

/* One model node (modelnode, model.h:64-86; kinematicmodel::get_mnode, model.h:108), nodes in XML
 * preorder (the order of mnodes, odeparts and dynparts). */
#define HS_NODE_MAX_KIDS 6
typedef struct {
  int32_t parent;     /* get_parent() index, -1 for the root */
  int32_t jtype;      /* get_joint()->get_type(): -1 no joint (ODE fixed joint), 0 free6, 1 hinge (model.h:26) */
  int32_t hinge;      /* hinge: motor index, its value at configuration index 6 + hinge; else -1 */
  int32_t foot;       /* foot index (periodic::get_nfeet order, periodic.cpp:34-58), else -1 */
  int32_t limb;       /* lik limb whose top link this node is (liklimb::child, lik.cpp:295-301), else -1 */
  int32_t n_kids;
  int32_t kids[HS_NODE_MAX_KIDS]; /* child_nodes in order (get_first_child = kids[0]) */
  double com[3];      /* odepart body position in the node frame (A_body_geom translation,
                         visualization.cpp:541-545) */
  double foot_pos[3]; /* foot: capsule end in the node frame (odepart::get_foot_pos,
                         visualization.cpp:553-568); else 0 */
  double mass;        /* dBodyGetMass (dynpart::set_inertial_params, dynrec.cpp:62-68) */
} hs_node_info;
int hs_model_get_node(hs_model_t model, int32_t i, hs_node_info* out);

/* Replaces modelplayer::get_rec_str + get_pgs_config_params (player.cpp:170-244):
 * reads line `setup_id` of a pgs_config.txt. xml_file receives the model name. */
int hs_pgs_config_read(const char* path, int setup_id, hs_gait_params* out, char* xml_file, int32_t xml_file_len);

/*
 * One batched pass of the hot path. Rollout b (0 <= b < n_rollouts) runs the
 * gait setup (pgssweeper::setup_pergen, pergen.cpp:453-507), samples the
 * trajectory at t_i = i * (period / n_t) for i = k0 .. k0+H+3 (record_trajectory,
 * periodic.cpp:77-96: pergen set_rec + lik + FK), builds dynamics records
 * (periodic.cpp:149-202, dynrec.cpp:134-224) and solves steps
 * i = k0+2 .. k0+H+1 (compute_torques_over_period, periodic.cpp:377-391).
 * With k0 = 0 and H = n_t this is exactly one reference cycle and work_cot[1]
 * is the reference COT (player.cpp:269-285).
 *
 * All arrays are DEVICE pointers on the current HIP device, row-major. Outputs
 * may be NULL. The call is asynchronous on `stream` (a hipStream_t, NULL =
 * default stream).
 */
typedef struct {
  int32_t n_rollouts;
  int32_t horizon;        /* H >= 1 */
  int32_t k0;             /* first step index (0 = reference i = 2) */
  int32_t n_t;            /* samples per period (measure_cot n_t, main.cpp:69) */
  int32_t ignore_reach;   /* liksolver::set_ignore_reach_flag (lik.cpp:142-147) */
  int32_t accumulate;     /* 1: add this call's work to work_cot[b][0] (successive H-step calls
                             then sum work in the reference's step order, periodic.cpp:291-304) */
  const hs_gait_params* params; /* [n_rollouts] */
  double* q;              /* [B][H][config_dim]: configuration at each solved sample */
  double* tau;            /* [B][H][nmj]: motor torques (periodic.cpp:328-343) */
  double* cf;             /* [B][H][3*nfeet]: contact forces (ftsolver.cpp:163) */
  double* x;              /* [B][H][6*n_parts]: joint forces/torques (ftsolver.cpp:166) */
  uint32_t* flags;        /* [B][H] */
  double* work_cot;       /* [B][2]: positive work, work/(sum m * step_length) */
  uint64_t* best_key;     /* scalar; atomically min-reduced with the rollouts' keys after the LAST
                             step of the call (hs_best_key_encode of hs_best_key_cot; needs work_cot) */
  int64_t rollout_id_base;/* global id of rollout 0 (shard offset) */
  void* stream;           /* hipStream_t */
  double* dq;             /* [B][H][config_dim]: rates at each solved sample (compute_vel_traj,
                             periodic.cpp:261-282: wrapped central difference / 2 dt) */
  int32_t precision;      /* HS_PREC_F64 (0) or HS_PREC_F32 (1, BASELINE configs[2]): with F32 the
                             arithmetic is single precision and every floating-point array of the
                             call (q, dq, tau, cf, x, work_cot; hs_pd_args; hs_run_forces' tau_in)
                             holds float (the pointer types stay double*). params stay double. */
  int32_t solve_mode;     /* HS_SOLVE_AUTO (0): the contact solve's closed form, the Eigen-style
                             path only where the minimizer is not unique; HS_SOLVE_REFERENCE (1):
                             every step through the Eigen-style FullPivLU / ColPivHouseholderQR
                             adaptive-rank loop of ftsolver.cpp:185-236 (same results where the
                             minimizer is unique; much slower; flags carry HS_FLAG_GENERAL). In
                             hs_run_forces[_calls]: every step through the dense normal equations
                             over the feet instead of the 6 x 6 system (same results) */
  int32_t key_steps;      /* control steps whose work the best key covers (0: the steps of this
                             call, i.e. H for hs_run, n_calls * H for hs_run_steps / hs_run_calls);
                             callers that accumulate work over several calls pass the total */
} hs_run_args;

#define HS_PREC_F64 0
#define HS_PREC_F32 1
#define HS_SOLVE_AUTO 0
#define HS_SOLVE_REFERENCE 1

int hs_run(hs_model_t model, const hs_run_args* args);

/* n_calls successive hs_run launches on args->stream: call c solves steps
 * k0_c = (args->k0 + c * horizon) mod n_t .. k0_c + horizon - 1, i.e. the
 * control loop marching through the gait cycle (compute_torques_over_period's
 * step order, periodic.cpp:377-391, wrapped); outputs are overwritten per call
 * and work_cot accumulates when args->accumulate is set. The best key (if
 * args->best_key) is taken once, after the last call, over the accumulated work
 * (key_steps 0 = n_calls * horizon steps). kernel_events, if not
 * NULL, holds 2 * n_calls caller-created hipEvent_t recorded immediately before
 * and after each launch (per-launch kernel timing on the launch stream). Every call
 * (hs_run, hs_run_steps, hs_run_calls, the forces and PD forms) first runs the setup
 * pass: each rollout's gait setup, a straight gait's frames and, when the steps read
 * more samples than it holds, the limb IK of those samples (before the events). */
int hs_run_steps(hs_model_t model, const hs_run_args* args, int32_t n_calls, void* const* kernel_events);

/* Position control (modelplayer::set_position_control_torques +
 * linear_feedback_control, player.cpp:388-432): for each solved step, with the
 * target state of periodic::get_motor_adas (periodic.cpp:394-404: motor angles
 * of the centre sample, rates by the wrapped central difference of
 * compute_vel_traj, periodic.cpp:261-282) and the step's computed torques as
 * feedforward (get_computed_torques),
 *   tau_cmd = tau_ff + (k1 * mod2pi(q - q0) + k2 * (dq - dq0)),
 *   k1 = -k, k2 = -2 sqrt(k), mod2pi into (-pi, pi] (arrayops::modulus).
 * The reference's step index tsi (mod n_t, lifted to [2, n_t + 1]) is the
 * centre sample: args->k0 = tsi - 2. All arrays DEVICE, [B][H][nmj]. */
typedef struct {
  const double* q_meas;   /* measured motor angles (get_ode_motor_adas) */
  const double* dq_meas;  /* measured motor rates */
  double k;               /* position gain (player.cpp:393: 100) */
  double* tau_cmd;        /* out: feedforward + feedback */
  double* q_target;       /* out, optional: get_motor_adas angles */
  double* dq_target;      /* out, optional: get_motor_adas rates */
} hs_pd_args;
/* The n_calls control steps of hs_run_steps (call c solves steps k0_c .. k0_c + H - 1 with
 * k0_c = (k0 + c H) mod n_t) fused into few launches over (step, rollout), so the SIMDs are
 * refilled from one queue of wavefronts instead of each step ending on its batch's slowest ones.
 * Every step keeps its own output rows: q, dq, tau, cf, x, flags are [B][n_calls * H][...]
 * (row c H + h). work_cot receives the same work (summed in step order, bitwise equal to
 * hs_run_steps with accumulate) and COT; the best key is taken once, after the last step
 * (needs work_cot). Asynchronous on args->stream like hs_run. */
int hs_run_calls(hs_model_t model, const hs_run_args* args, int32_t n_calls);

int hs_run_pd(hs_model_t model, const hs_run_args* args, const hs_pd_args* pd);

/* Contact forces given motor torques: forcetorquesolver::solve_forces via
 * periodic::solve_contforces_given_torques (ftsolver.cpp:331-378,
 * periodic.cpp:368-374) for steps k0 .. k0+H-1 of every rollout. tau_in is a
 * DEVICE array [B][H][nmj]; args->cf receives the least-squares forces of ALL
 * feet (airborne ones included, contact_feet_flag = false), torso force and
 * torque forced to zero; args->q and args->flags as in hs_run (HS_FLAG_GENERAL
 * = the least squares is rank deficient, e.g. a straight leg; then the
 * Tikhonov-regularized solution is returned). tau, x, work_cot and best_key are
 * not written. */
int hs_run_forces(hs_model_t model, const hs_run_args* args, const double* tau_in);
/* n_calls calls of hs_run_forces (call horizon args->horizon, k0 marching by it), fused like
 * hs_run_calls: a setup pass stores each rollout's gait setup once, then launches of up to 512k
 * wavefronts over (step, rollout); every step S = n_calls * horizon keeps its own row. tau_in is a
 * DEVICE array [B][S][nmj], args->cf / q / flags have S rows per rollout. Outputs are bitwise those
 * of hs_run_forces with horizon S. (periodic::solve_contforces_given_torques over a trajectory,
 * periodic.cpp:368-374, as called per sample by modelplayer::test_dynamics,
 * playerexperim.cpp:95-121.) */
int hs_run_forces_calls(hs_model_t model, const hs_run_args* args, int32_t n_calls, const double* tau_in);
/* Host-buffer, synchronous form: tau_in [B][H][nmj] -> cf [B][H][3*nfeet], flags [B][H] (may be NULL). */
int hs_run_forces_host(hs_model_t model, const hs_gait_params* params, int32_t n_rollouts, int32_t n_t, int32_t k0,
                       int32_t horizon, int32_t ignore_reach, const double* tau_in, double* cf, uint32_t* flags);

/* Mixed-topology batches (BASELINE configs[4], e.g. myant + hexapod interleaved):
 * rollout b runs models[model_index[b]]. The reference runs one kinematicmodel
 * per periodic object (periodic.cpp:34-58); a plan batches several in one
 * launch. It groups each model's rollouts two per wavefront, so topology reads
 * stay wave-uniform, and is reusable across calls on the device current at
 * creation. Models must outlive the plan. model_index is a HOST array. */
typedef struct hs_mixed_s* hs_mixed_t;
int hs_mixed_create(const hs_model_t* models, int32_t n_models, const int32_t* model_index, int32_t n_rollouts,
                    hs_mixed_t* out);
void hs_mixed_free(hs_mixed_t plan);
/* Output row strides of the plan's batches = the maxima over its models:
 * tau rows hold max nmj, cf 3 * max nfeet, q max config_dim, x 6 * max n_parts
 * (the other fields of *out are those of the model with the most parts).
 * Entries past a rollout's own dimensions are written as 0. */
int hs_mixed_get_dims(hs_mixed_t plan, hs_model_dims* out);
/* hs_run / hs_run_steps over a plan (args->n_rollouts must equal the plan's). */
int hs_run_mixed(hs_mixed_t plan, const hs_run_args* args);
int hs_run_mixed_steps(hs_mixed_t plan, const hs_run_args* args, int32_t n_calls, void* const* kernel_events);
/* hs_run_calls for a mixed plan (rows with the plan's strides) */
int hs_run_mixed_calls(hs_mixed_t plan, const hs_run_args* args, int32_t n_calls);

/* Host-buffer convenience wrapper of hs_run (copies in/out, synchronous).
 * Replaces periodic::compute_torques_over_period + get_motor_torques +
 * work_over_period for a batch of rollouts. Output pointers may be NULL. */
int hs_run_host(hs_model_t model, const hs_gait_params* params, int32_t n_rollouts, int32_t n_t,
                int32_t k0, int32_t horizon, int32_t ignore_reach, double* q, double* tau, double* cf,
                double* x, uint32_t* flags, double* work_cot);

/* periodic::get_complete_traj (periodic.cpp:406-426) for a batch of rollouts
 * (synchronous, host buffers): rec[b][tsi] for tsi = 0 .. n_t-1 (tsi < 2 read
 * at tsi + n_t, like get_complete_traj_rec) = [configuration (config_dim),
 * rates (config_dim), computed torques (nmj)] -- the records
 * modelplayer::record_per_traj writes to traj.txt (player.cpp:619-629).
 * rec holds n_rollouts * n_t * (2 * config_dim + nmj) doubles. */
int hs_complete_traj(hs_model_t model, const hs_gait_params* params, int32_t n_rollouts, int32_t n_t,
                     int32_t ignore_reach, double* rec);

/* save_2d_array (core.cpp:46-61): n_rows rows of rec_len doubles, space
 * separated, default ostream formatting, appended when append != 0. */
int hs_traj_save(const char* path, const double* rec, int32_t n_rows, int32_t rec_len, int32_t append);

/*
 * Per-configuration kinematics: the kinematicmodel / pergensetup entry points every caller
 * outside periodic binds (model.h:122-130, pergen.h:68-108; player.cpp:69, 122, 354,
 * ghost.cpp:53-54, periodic.cpp:89-90), for batches of n configurations. DEVICE arrays on the
 * current HIP device, asynchronous on stream (a hipStream_t, NULL = default stream); the _host
 * forms take host arrays and are synchronous. fp64 only.
 */
/* Row length of a trajectory record: torso position and Euler angles, then the foot position of
 * every limb in lik order (liksolver::place_limbs, lik.cpp:87-99; pergensetup::set_rec,
 * pergen.cpp:220-239). = 6 + 3 * n_limbs = config_dim for the shipped models. */
#define HS_REC_LEN(dims) (6 + 3 * (dims).n_limbs)

/* pergensetup::set_rec (pergen.cpp:225-239) after pgssweeper::setup_pergen (pergen.cpp:453-507):
 * rec[b][i] = the record of rollout b's gait at time times[i] (t in the units of period), for
 * n_rollouts x n_times items. params [n_rollouts], times [n_times], rec [B][n_times][rec_len]. */
int hs_pergen_rec(hs_model_t model, const hs_gait_params* params, int32_t n_rollouts, const double* times,
                  int32_t n_times, double* rec, void* stream);
int hs_pergen_rec_host(hs_model_t model, const hs_gait_params* params, int32_t n_rollouts, const double* times,
                       int32_t n_times, double* rec);

#define HS_FLAG_LIK_FAILED 128u /* hs_model_lik status: a foot target out of reach with ignore_reach = 0
                                   (the reference prints the limb and exits, lik.cpp:321-330); the
                                   limb's angles are then NaN */
#define HS_LIK_LIMB_BIT(L) (1u << (16 + (L))) /* hs_model_lik status: limb L's target was out of reach */
/* kinematicmodel::set_jvalues_with_lik (model.cpp:354-359 -> liksolver::place_limbs,
 * lik.cpp:89-99, liklimb::place_limb / poslimb, lik.cpp:316-347): rec [n][rec_len] -> config
 * [n][config_dim] (joint values in get_jvalues order, model.cpp:368-372). Only the torso's six
 * values and the limbs' hinge values are written; other entries keep what config held (the
 * reference leaves the other joint values as they were). ignore_reach as
 * liksolver::set_ignore_reach_flag (lik.cpp:142-147): a target beyond reach is clamped to the
 * stretched limb (status HS_FLAG_UNREACH); without it status gets HS_FLAG_LIK_FAILED; either way
 * HS_LIK_LIMB_BIT(L) names the limb. status [n] may be NULL. The host form returns HS_E_ARG when any row failed (after writing all rows). */
int hs_model_lik(hs_model_t model, int32_t n, const double* rec, int32_t ignore_reach, double* config,
                 uint32_t* status, void* stream);
int hs_model_lik_host(hs_model_t model, int32_t n, const double* rec, int32_t ignore_reach, double* config,
                      uint32_t* status);

/* kinematicmodel::recompute_modelnodes (model.cpp:314-318; modelnode::recompute_A_ground,
 * model.cpp:183-201) for n configurations config [n][config_stride] (config_stride >=
 * config_dim): the ground transform of every model node, get_mnode(i)->get_A_ground()
 * (model.h:73, 108), into a_ground [n][n_parts][12], and of every node's joint,
 * get_joint()->get_A_ground() (model.h:45), into a_joint [n][n_parts][12] (may be NULL; zeros
 * for a node without a joint). Each transform is the 3x4 top of the reference's column-major 4x4
 * affine (matrix.h:27-28): element (row r, column c) at [c * 3 + r], c = 3 the translation. Node
 * order = model nodes in XML preorder (kinematicmodel::mnodes). */
int hs_model_fk(hs_model_t model, int32_t n, const double* config, int32_t config_stride, double* a_ground,
                double* a_joint, void* stream);
int hs_model_fk_host(hs_model_t model, int32_t n, const double* config, int32_t config_stride, double* a_ground,
                     double* a_joint);

/* Best-rollout key: (order-preserving bits of (float)c) << 32 | (uint32)rollout id, where c is
 * the selection COT of hs_best_key_cot. NaN maps to the largest key (never selected); ties go to
 * the lowest id. Initial value for a reduction: UINT64_MAX.
 *
 * Selection COT (a deliberate deviation from the signed COT player.cpp:269-285 prints, which
 * work_cot[1] keeps): the cost of transport of ONE gait cycle of forward or backward walking,
 *   c = work * (n_t / steps) / (total_mass * |step_length|),
 * steps = the control steps the accumulated work covers (hs_run_args.key_steps), so a key taken
 * after K != n_t steps ranks rollouts like measure_cot over one cycle would; |step_length| <
 * HS_KEY_MIN_STEP_LENGTH gives NaN (a gait that does not travel has no meaningful COT). The
 * reference only prints per-setup COTs of its sweep (player.cpp:311-321) and never selects. */
#define HS_KEY_MIN_STEP_LENGTH 1e-3
double hs_best_key_cot(double work, double total_mass, double step_length, int32_t n_t, int32_t steps);
uint64_t hs_best_key_encode(double cot, int64_t rollout_id);
void hs_best_key_decode(uint64_t key, float* cot, int64_t* rollout_id);

/*
 * Batch handle sharded over the devices of one process (SURVEY.md 8b exports 2-5): the
 * in-process counterpart of one process per GPU. Rollouts split into contiguous ranges, one per
 * device set in device_mask (bit d = HIP device d; the same ranges as hslabs_amd/dist.py shard),
 * each range run on its device's own stream with rollout_id_base = its first id. Parameters and
 * outputs live on the devices; hs_batch_run copies the requested outputs to caller-owned HOST
 * arrays laid out for the whole batch. Replaces the loop of pgssweeper::setup_pergen +
 * modelplayer::measure_cot over a parameter sweep (player.cpp:259-321).
 */
typedef struct hs_batch_s* hs_batch_t;

typedef struct {         /* host arrays, any may be NULL; float instead of double with HS_PREC_F32 */
  double* q;             /* [B][H][config_dim] */
  double* tau;           /* [B][H][nmj] */
  double* cf;            /* [B][H][3*nfeet] */
  double* x;             /* [B][H][6*n_parts] */
  uint32_t* flags;       /* [B][H] */
  double* work;          /* [B]: positive work of the run's steps (work_over_period) */
  double* cot;           /* [B]: work / (sum m * step_length) (player.cpp:269-285) */
} hs_batch_outputs;

int hs_batch_create(hs_model_t model, int32_t n_rollouts, int32_t horizon, int32_t n_t, int32_t precision,
                    uint32_t device_mask, hs_batch_t* out);
/* host params[n_rollouts] (pgsconfigparams fields, pergen.h:137-146) -> the devices' shards */
int hs_batch_set_params(hs_batch_t batch, const hs_gait_params* params);
/* steps k0 .. k0+H-1 of every rollout (hs_run semantics), synchronous; resets and refills the
 * per-device best keys */
int hs_batch_run(hs_batch_t batch, int32_t k0, int32_t ignore_reach, const hs_batch_outputs* out);
/* hs_batch_run into caller-owned DEVICE buffers (same [B] layouts; each may be on any device of the
 * process: a shard's rows are copied device-to-device, peer-to-peer when the buffer is on another
 * GPU; float arrays with HS_PREC_F32), synchronous. periodic::get_motor_torques and
 * solve_torques_contforces write caller-allocated arrays the same way (periodic.cpp:328-343). */
int hs_batch_run_device(hs_batch_t batch, int32_t k0, int32_t ignore_reach, const hs_batch_outputs* out);
/* The best-rollout reduce inside one process: minimum of the per-device keys of the last run
 * (lowest selection COT, ties to the lowest id), by host reads of the devices' 8-byte keys. */
int hs_select_best(hs_batch_t batch, float* cot, int64_t* rollout_id);
/* device pointer of the uint64 best key of the i-th device of the batch (in mask order) */
uint64_t* hs_batch_best_key_device(hs_batch_t batch, int32_t i);
void hs_batch_free(hs_batch_t batch);

/*
 * One process per GPU: the path's single collective, the best-rollout reduce, as
 * ONE RCCL all-reduce (ncclUint64, ncclMin) of the 8-byte key over xGMI. It replaces the serial
 * sweep whose minimum a caller of player.cpp:311-321 would take. The communicator spans the ranks
 * of the job, one HIP device each: rank 0 creates the id with hs_comm_unique_id, the caller
 * broadcasts its HS_COMM_ID_BYTES bytes (MPI, torch.distributed, a file ...), every rank calls
 * hs_comm_init with the device it runs on current. Rollouts are sharded in contiguous id ranges
 * (rollout_id_base), so the reduced key names the global winner.
 */
#define HS_COMM_ID_BYTES 128
typedef struct hs_comm_s* hs_comm_t;
int hs_comm_unique_id(char id[HS_COMM_ID_BYTES]);
int hs_comm_init(int32_t n_ranks, int32_t rank, const char id[HS_COMM_ID_BYTES], hs_comm_t* out);
void hs_comm_free(hs_comm_t comm);
int hs_comm_size(hs_comm_t comm, int32_t* n_ranks, int32_t* rank);
/* in-place all-reduce(MIN) of the uint64 key at key (DEVICE pointer, the comm's device), async
 * on stream (a hipStream_t, NULL = default stream) */
int hs_comm_reduce_best(hs_comm_t comm, uint64_t* key, void* stream);
/* hs_select_best across the ranks: this process's minimum over its batch's devices (the batch
 * must run on the comm's device only), all-reduced over the communicator, decoded on every rank.
 * The reduce runs in the comm's own 8-byte device buffer: the batch's per-device keys keep their
 * local values (a later hs_select_best still returns this process's minimum). Collective: every
 * rank must call it. A rank whose batch fails the checks (not run, another device, null outputs) or
 * whose local keys cannot be read back still takes part, contributing the largest key, and then
 * returns the error, so its peers complete (with the minimum over the other ranks). Two failures
 * return before the collective and leave the peers waiting: a null comm, and a HIP runtime error on
 * the comm's own device while staging the key (the communicator is unusable then). */
int hs_select_best_comm(hs_batch_t batch, hs_comm_t comm, float* cot, int64_t* rollout_id);

/*
 * Closed-loop simulation: modelplayer::simulate_ode with position control
 * (player.cpp:325-339) for a batch of independent robots, each in its own ODE
 * world as the reference sets it up (visualization.cpp:140-150: gravity 1,
 * ERP .8, a z = 0 plane; one body per part with ODE's default mass, hinge and
 * fixed joints from kinematicmodel::set_ode_joints, model.cpp:375-400). One
 * step is
 *   set_position_control_torques (player.cpp:388-432): targets and
 *     feedforward torques of the controller tables at tsi, measured hinge
 *     angles / rates (dJointGetHingeAngle/Rate), k1 = -k, k2 = -2 sqrt(k);
 *   dJointAddHingeTorque for every motor (visualization.cpp:350-356);
 *   dSpaceCollide + nearCallback (visualization.cpp:296-326): one contact per
 *     capsule / sphere touching the plane, Bounce|SoftCFM, mu = inf;
 *   dWorldQuickStep (visualization.cpp:333-337): the projected Gauss-Seidel
 *     (SOR-LCP) constraint solve, `iterations` sweeps with ODE's random
 *     reordering every 8 sweeps, then the semi-implicit body update;
 *   tsi += 1 (play_t += play_dt).
 * The ODE formulas are restated from ODE 0.13 (the reference links an
 * unpinned -lode); see DESIGN.md.
 */
#define HS_SIM_BODY_STRIDE 13 /* per part: pos[3], quaternion (w,x,y,z)[4], lvel[3], avel[3] */

typedef struct {
  double dt;          /* play_dt (player.cpp:23: 0.01) */
  double k;           /* position gain (player.cpp:393: 100); <= 0: no position control */
  double sor_w;       /* dWorldSetQuickStepW (ODE default 1.3) */
  double erp;         /* dWorldSetERP (visualization.cpp:146: 0.8) */
  double cfm;         /* global CFM (ODE double-precision default 1e-10) */
  double gravity;     /* visualization.cpp:144: 1 */
  double bounce;      /* nearCallback surface (visualization.cpp:310-320): .5 */
  double bounce_vel;  /* .1 */
  double soft_cfm;    /* .001 */
  double mu;          /* dInfinity */
  int32_t iterations; /* dWorldSetQuickStepNumIterations (ODE default 20) */
  int32_t reserved;
} hs_sim_params;

/* The reference's values (above). */
void hs_sim_default_params(hs_sim_params* p);

/* init_play_config (player.cpp:351-356) + orient_odebodys (model.cpp:295-305):
 * body states of B configurations (joint values, config [B][config_stride],
 * DEVICE), zero velocities. body: DEVICE [B][n_parts][HS_SIM_BODY_STRIDE].
 * precision HS_PREC_F32: config and body hold floats (the pose is built in
 * double and rounded once). */
int hs_sim_reset(hs_model_t model, int32_t n_rollouts, const double* config, int32_t config_stride, double* body,
                 int32_t precision, void* stream);

typedef struct {
  int32_t n_rollouts;
  int32_t n_steps;         /* simulation steps of this call (one launch runs them all) */
  int32_t n_t;             /* controller table rows (setup_per_controller: int(T / play_dt + .5)) */
  int32_t precision;       /* HS_PREC_F64, or HS_PREC_F32 (BASELINE configs[2]): single-precision
                              arithmetic; body, the tables and the outputs hold floats (pointer types
                              stay double*, like hs_run_args); seed/tsi/n_contacts unchanged */
  hs_sim_params params;
  /* per-rollout state, DEVICE, read and advanced */
  double* body;            /* [B][n_parts][HS_SIM_BODY_STRIDE] */
  uint32_t* seed;          /* [B] ODE dRand state (dRandInt reshuffles of the SOR rows) */
  int32_t* tsi;            /* [B] play step index, int(play_t / play_dt + .5) */
  /* controller tables, DEVICE: exactly what hs_run writes with k0 = 0, H = n_t (row h = trajectory
     sample h + 2; get_motor_adas / get_computed_torques of tsi read row (tsi mod n_t + n_t - 2) mod n_t) */
  const double* q_tab;     /* [B][n_t][config_dim] (hs_run_args.q) */
  const double* dq_tab;    /* [B][n_t][config_dim] (hs_run_args.dq) */
  const double* tau_tab;   /* [B][n_t][nmj] (hs_run_args.tau) */
  /* optional per-step outputs, DEVICE (NULL to skip) */
  double* tau_cmd;         /* [B][n_steps][nmj] motor torques applied */
  double* q_meas;          /* [B][n_steps][nmj] hinge angles at the start of the step */
  double* torso;           /* [B][n_steps][3] root body position after the step */
  int32_t* n_contacts;     /* [B][n_steps] */
  double* normal_force;    /* [B][n_steps] sum of the contact normal constraint forces */
  void* stream;            /* hipStream_t */
} hs_sim_args;

/* n_steps closed-loop steps of every rollout, one launch (state stays on chip between steps). */
int hs_sim_step(hs_model_t model, const hs_sim_args* args);

/* Host-side handle over the calls above, for callers without device memory of their own
 * (the C++ shim's modelplayer): owns the device tables and state of B rollouts.
 * hs_sim_create = modelplayer::setup_per_controller (player.cpp:370-382) for every rollout:
 * n_t = int(period / params->dt + .5) controller rows from hs_run (same n_t for the whole
 * batch, else HS_E_ARG), play_t = int(t0 / dt + .5) dt, bodies at that trajectory sample
 * at rest (init_play_config). params is HOST memory; sim_params NULL = hs_sim_default_params. */
typedef struct hs_sim_s* hs_sim_t;
int hs_sim_create(hs_model_t model, const hs_gait_params* params, int32_t n_rollouts, const hs_sim_params* sim_params,
                  double t0, hs_sim_t* out);
/* n_steps of simulate_ode (synchronous); HOST outputs as in hs_sim_args, each may be NULL. */
int hs_sim_advance(hs_sim_t sim, int32_t n_steps, double* tau_cmd, double* q_meas, double* torso, int32_t* n_contacts,
                   double* normal_force);
/* HOST copies of the state: body [B][n_parts][HS_SIM_BODY_STRIDE], tsi [B] (either may be NULL). */
int hs_sim_get_state(hs_sim_t sim, double* body, int32_t* tsi);
void hs_sim_free(hs_sim_t sim);

/* The fused step launches' kernel (ABI 15). hs_run_calls takes the limb-lane kernel (lane = (rollout,
 * limb), eight rollouts per wavefront) for a model of its class (*ok = 1: every shipped
 * model), HS_SOLVE_AUTO, no x / q / dq rows, and calls whose samples fit the IK table; its outputs are
 * bitwise hs_rollout_kernel's (the steps it does not take go to the same fixup launch). HS_LIMB=0 in the
 * environment keeps hs_rollout_kernel. hs_limb_launches: the limb-lane launches this process has made. */
int hs_model_limb_lane(hs_model_t model, int32_t* ok);
int64_t hs_limb_launches(void);
/* Diagnostics of the limb-lane kernel: its launches and the steps it deferred to the fixup launch (one,
 * two contacts, guards near their thresholds, ...) in this process; *deferred is read from the device
 * (synchronous on the current device). Either pointer may be NULL. */
int hs_limb_stats(int64_t* launches, int64_t* deferred);

const char* hs_last_error(void);
int hs_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif
