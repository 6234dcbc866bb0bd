"""ctypes binding of include/hslabs.h (the C-ABI boundary).

This module is the Python mirror of the reference-side binding a maintainer
would write. It never falls back to a CPU path: if the
in-tree gfx950 library is missing, loading fails loudly.
"""
from __future__ import annotations

import ctypes
import hashlib
import os

from . import build as _build

ABI_VERSION = 15

HS_OK = 0
HS_FLAG_RANK_RETRY = 1
HS_FLAG_FULL_RANK = 2
HS_FLAG_LOOP_EXHAUST = 4
HS_FLAG_NAN = 8
HS_FLAG_UNREACH = 16
HS_FLAG_NO_CONTACT = 32
HS_FLAG_GENERAL = 64
HS_FLAG_NEAR_RANK = 256  # a rank / routing decision within rounding of its threshold (include/hslabs.h)
HS_FLAG_DEPENDENT = 512  # solve_forces: a dependent force component dropped, the basic solution (include/hslabs.h)
HS_PREC_F64 = 0
HS_PREC_F32 = 1
HS_SOLVE_AUTO = 0
HS_SOLVE_REFERENCE = 1
KEY_MIN_STEP_LENGTH = 1e-3
COMM_ID_BYTES = 128

# every symbol declared in include/hslabs.h
EXPORTS = [
    "hs_model_load", "hs_model_load_ex", "hs_model_free", "hs_model_get_dims", "hs_pgs_config_read",
    "hs_run", "hs_run_steps", "hs_run_calls", "hs_run_pd", "hs_run_forces", "hs_run_forces_calls", "hs_mixed_create", "hs_mixed_free",
    "hs_mixed_get_dims", "hs_complete_traj", "hs_traj_save", "hs_run_forces_host",
    "hs_run_mixed", "hs_run_mixed_steps", "hs_run_mixed_calls", "hs_run_host", "hs_best_key_cot", "hs_best_key_encode",
    "hs_best_key_decode", "hs_last_error", "hs_abi_version",
    "hs_sim_default_params", "hs_sim_reset", "hs_sim_step", "hs_sim_create", "hs_sim_advance", "hs_sim_get_state",
    "hs_sim_free", "hs_batch_create", "hs_batch_set_params", "hs_batch_run", "hs_batch_run_device", "hs_select_best",
    "hs_batch_best_key_device", "hs_batch_free", "hs_comm_unique_id", "hs_comm_init", "hs_comm_free", "hs_comm_size",
    "hs_comm_reduce_best", "hs_select_best_comm", "hs_pergen_rec", "hs_pergen_rec_host", "hs_model_lik",
    "hs_model_lik_host", "hs_model_fk", "hs_model_fk_host", "hs_model_get_node", "hs_model_set_torso_penalty",
    "hs_model_get_torso_penalty", "hs_model_limb_lane", "hs_limb_launches", "hs_limb_stats",
]
HS_FLAG_LIK_FAILED = 128
SIM_BODY_STRIDE = 13


class GaitParamsC(ctypes.Structure):
    """hs_gait_params (192 bytes)."""

    _fields_ = [
        ("torso_pos", ctypes.c_double * 3),
        ("torso_angles", ctypes.c_double * 3),
        ("step_duration", ctypes.c_double),
        ("period", ctypes.c_double),
        ("step_length", ctypes.c_double),
        ("step_height", ctypes.c_double),
        ("curvature", ctypes.c_double),
        ("foot_shift", ctypes.c_double),
        ("foot_shift_type", ctypes.c_int32),
        ("rec_transform_flag", ctypes.c_int32),
        ("rec_transl", ctypes.c_double * 3),
        ("rec_eas", ctypes.c_double * 3),
        ("reserved", ctypes.c_double * 5),
    ]


assert ctypes.sizeof(GaitParamsC) == 192


class BatchOutputsC(ctypes.Structure):
    """hs_batch_outputs: host arrays (NULL = not wanted)."""

    _fields_ = [(f, ctypes.c_void_p) for f in ("q", "tau", "cf", "x", "flags", "work", "cot")]


class ModelDimsC(ctypes.Structure):
    _fields_ = [
        ("n_parts", ctypes.c_int32), ("nmj", ctypes.c_int32), ("nfeet", ctypes.c_int32),
        ("config_dim", ctypes.c_int32), ("n_limbs", ctypes.c_int32), ("lik_kind", ctypes.c_int32),
        ("total_mass", ctypes.c_double), ("rcap", ctypes.c_double),
    ]


class NodeInfoC(ctypes.Structure):
    """hs_node_info."""
    _fields_ = [(f, ctypes.c_int32) for f in ("parent", "jtype", "hinge", "foot", "limb", "n_kids")] + \
               [("kids", ctypes.c_int32 * 6), ("com", ctypes.c_double * 3), ("foot_pos", ctypes.c_double * 3),
                ("mass", ctypes.c_double)]


class PdArgsC(ctypes.Structure):
    """hs_pd_args."""
    _fields_ = [("q_meas", ctypes.c_void_p), ("dq_meas", ctypes.c_void_p), ("k", ctypes.c_double),
                ("tau_cmd", ctypes.c_void_p), ("q_target", ctypes.c_void_p), ("dq_target", ctypes.c_void_p)]


class RunArgsC(ctypes.Structure):
    _fields_ = [
        ("n_rollouts", ctypes.c_int32), ("horizon", ctypes.c_int32), ("k0", ctypes.c_int32),
        ("n_t", ctypes.c_int32), ("ignore_reach", ctypes.c_int32), ("accumulate", ctypes.c_int32),
        ("params", ctypes.c_void_p), ("q", ctypes.c_void_p), ("tau", ctypes.c_void_p),
        ("cf", ctypes.c_void_p), ("x", ctypes.c_void_p), ("flags", ctypes.c_void_p),
        ("work_cot", ctypes.c_void_p), ("best_key", ctypes.c_void_p),
        ("rollout_id_base", ctypes.c_int64), ("stream", ctypes.c_void_p), ("dq", ctypes.c_void_p),
        ("precision", ctypes.c_int32), ("solve_mode", ctypes.c_int32), ("key_steps", ctypes.c_int32),
    ]


class SimParamsC(ctypes.Structure):
    """hs_sim_params."""
    _fields_ = [(f, ctypes.c_double) for f in ("dt", "k", "sor_w", "erp", "cfm", "gravity", "bounce", "bounce_vel",
                                               "soft_cfm", "mu")] + [("iterations", ctypes.c_int32),
                                                                     ("reserved", ctypes.c_int32)]


class SimArgsC(ctypes.Structure):
    """hs_sim_args."""
    _fields_ = [("n_rollouts", ctypes.c_int32), ("n_steps", ctypes.c_int32), ("n_t", ctypes.c_int32),
                ("precision", ctypes.c_int32), ("params", SimParamsC)] + \
               [(f, ctypes.c_void_p) for f in ("body", "seed", "tsi", "q_tab", "dq_tab", "tau_tab", "tau_cmd", "q_meas",
                                               "torso", "n_contacts", "normal_force", "stream")]


class HSError(RuntimeError):
    pass


_lib = None
LOADED = None  # {"path", "sha256"} of the library load() mapped


def lib_path() -> str:
    return _build.LIB


def load(build_if_missing: bool = True) -> ctypes.CDLL:
    """Load the in-tree libhslabs.so (building it first if allowed)."""
    global _lib
    if _lib is not None:
        return _lib
    # One HIP runtime per process. torch ships its own libamdhip64 (SONAME libamdhip64.so.7) and
    # its libraries NEED it by the unversioned name, so if libhslabs.so pulled /opt/rocm's copy in
    # first, a later `import torch` would load a second runtime and libhslabs' runtime would then
    # see no device (measured on the MI355X box). Importing torch first makes libhslabs bind to the
    # runtime already in the process.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    path = _build.LIB
    variant = os.environ.get("HSLABS_VARIANT")  # an A/B tuning build (build.build_variant), by name only
    if variant:
        if not variant.replace("_", "").isalnum():
            raise HSError(f"bad HSLABS_VARIANT {variant!r}")
        path = os.path.join(_build.VARIANT_DIR, f"libhslabs_{variant}.so")
        if not os.path.exists(path):
            raise HSError(f"HSLABS_VARIANT={variant}: {path} not built")
    if not os.path.exists(path):
        if not build_if_missing:
            raise HSError(f"libhslabs.so not built ({path}); run `python -m hslabs_amd.build`")
        _build.build()
    L = ctypes.CDLL(path)
    global LOADED
    with open(path, "rb") as f:
        LOADED = {"path": os.path.relpath(path, os.path.dirname(_build.HERE)),
                  "sha256": hashlib.sha256(f.read()).hexdigest()[:16]}
    dp = ctypes.POINTER(ctypes.c_double)
    vp = ctypes.c_void_p
    L.hs_model_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(vp)]
    L.hs_model_load_ex.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(vp)]
    L.hs_model_free.argtypes = [vp]
    L.hs_model_free.restype = None
    L.hs_model_get_dims.argtypes = [vp, ctypes.POINTER(ModelDimsC)]
    L.hs_model_set_torso_penalty.argtypes = [vp, ctypes.c_int32, ctypes.c_int32]
    L.hs_model_get_torso_penalty.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
    L.hs_pgs_config_read.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.POINTER(GaitParamsC),
                                     ctypes.c_char_p, ctypes.c_int32]
    L.hs_run.argtypes = [vp, ctypes.POINTER(RunArgsC)]
    L.hs_run_steps.argtypes = [vp, ctypes.POINTER(RunArgsC), ctypes.c_int32, ctypes.POINTER(vp)]
    L.hs_run_calls.argtypes = [vp, ctypes.POINTER(RunArgsC), ctypes.c_int32]
    L.hs_run_mixed_calls.argtypes = [vp, ctypes.POINTER(RunArgsC), ctypes.c_int32]
    L.hs_run_forces.argtypes = [vp, ctypes.POINTER(RunArgsC), vp]
    L.hs_run_forces_calls.argtypes = [vp, ctypes.POINTER(RunArgsC), ctypes.c_int32, vp]
    L.hs_run_forces_host.argtypes = [vp, ctypes.POINTER(GaitParamsC), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                     ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_double),
                                     ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
    L.hs_run_pd.argtypes = [vp, ctypes.POINTER(RunArgsC), ctypes.POINTER(PdArgsC)]
    L.hs_complete_traj.argtypes = [vp, ctypes.POINTER(GaitParamsC), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                                   ctypes.POINTER(ctypes.c_double)]
    L.hs_traj_save.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_double), ctypes.c_int32, ctypes.c_int32,
                               ctypes.c_int32]
    L.hs_mixed_create.argtypes = [ctypes.POINTER(vp), ctypes.c_int32, ctypes.POINTER(ctypes.c_int32), ctypes.c_int32,
                                  ctypes.POINTER(vp)]
    L.hs_mixed_free.argtypes = [vp]
    L.hs_mixed_free.restype = None
    L.hs_mixed_get_dims.argtypes = [vp, ctypes.POINTER(ModelDimsC)]
    L.hs_run_mixed.argtypes = [vp, ctypes.POINTER(RunArgsC)]
    L.hs_run_mixed_steps.argtypes = [vp, ctypes.POINTER(RunArgsC), ctypes.c_int32, ctypes.POINTER(vp)]
    L.hs_run_host.argtypes = [vp, ctypes.POINTER(GaitParamsC), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                              ctypes.c_int32, ctypes.c_int32, dp, dp, dp, dp, ctypes.POINTER(ctypes.c_uint32), dp]
    L.hs_best_key_cot.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int32, ctypes.c_int32]
    L.hs_best_key_cot.restype = ctypes.c_double
    L.hs_best_key_encode.argtypes = [ctypes.c_double, ctypes.c_int64]
    L.hs_best_key_encode.restype = ctypes.c_uint64
    L.hs_best_key_decode.argtypes = [ctypes.c_uint64, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int64)]
    L.hs_best_key_decode.restype = None
    L.hs_sim_default_params.argtypes = [ctypes.POINTER(SimParamsC)]
    L.hs_sim_default_params.restype = None
    L.hs_sim_reset.argtypes = [vp, ctypes.c_int32, vp, ctypes.c_int32, vp, ctypes.c_int32, vp]
    L.hs_sim_step.argtypes = [vp, ctypes.POINTER(SimArgsC)]
    L.hs_sim_create.argtypes = [vp, ctypes.POINTER(GaitParamsC), ctypes.c_int32, ctypes.POINTER(SimParamsC),
                                ctypes.c_double, ctypes.POINTER(vp)]
    L.hs_sim_advance.argtypes = [vp, ctypes.c_int32, dp, dp, dp, ctypes.POINTER(ctypes.c_int32), dp]
    L.hs_sim_get_state.argtypes = [vp, dp, ctypes.POINTER(ctypes.c_int32)]
    L.hs_sim_free.argtypes = [vp]
    L.hs_sim_free.restype = None
    L.hs_batch_create.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_uint32,
                                  ctypes.POINTER(vp)]
    L.hs_batch_set_params.argtypes = [vp, ctypes.POINTER(GaitParamsC)]
    L.hs_batch_run.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(BatchOutputsC)]
    L.hs_batch_run_device.argtypes = [vp, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(BatchOutputsC)]
    L.hs_select_best.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int64)]
    L.hs_select_best_comm.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int64)]
    L.hs_comm_unique_id.argtypes = [ctypes.c_char_p]
    L.hs_comm_init.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_char_p, ctypes.POINTER(vp)]
    L.hs_comm_free.argtypes = [vp]
    L.hs_comm_free.restype = None
    L.hs_comm_size.argtypes = [vp, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]
    L.hs_comm_reduce_best.argtypes = [vp, vp, vp]
    L.hs_batch_best_key_device.argtypes = [vp, ctypes.c_int32]
    L.hs_batch_best_key_device.restype = vp
    L.hs_batch_free.argtypes = [vp]
    L.hs_batch_free.restype = None
    u32p = ctypes.POINTER(ctypes.c_uint32)
    L.hs_pergen_rec.argtypes = [vp, vp, ctypes.c_int32, vp, ctypes.c_int32, vp, vp]
    L.hs_pergen_rec_host.argtypes = [vp, ctypes.POINTER(GaitParamsC), ctypes.c_int32, dp, ctypes.c_int32, dp]
    L.hs_model_lik.argtypes = [vp, ctypes.c_int32, vp, ctypes.c_int32, vp, vp, vp]
    L.hs_model_lik_host.argtypes = [vp, ctypes.c_int32, dp, ctypes.c_int32, dp, u32p]
    L.hs_model_fk.argtypes = [vp, ctypes.c_int32, vp, ctypes.c_int32, vp, vp, vp]
    L.hs_model_fk_host.argtypes = [vp, ctypes.c_int32, dp, ctypes.c_int32, dp, dp]
    L.hs_model_get_node.argtypes = [vp, ctypes.c_int32, ctypes.POINTER(NodeInfoC)]
    L.hs_last_error.argtypes = []
    L.hs_last_error.restype = ctypes.c_char_p
    L.hs_model_limb_lane.argtypes = [vp, ctypes.POINTER(ctypes.c_int32)]
    L.hs_limb_launches.argtypes = []
    L.hs_limb_launches.restype = ctypes.c_int64
    L.hs_limb_stats.argtypes = [ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    L.hs_abi_version.argtypes = []
    L.hs_abi_version.restype = ctypes.c_int
    if L.hs_abi_version() != ABI_VERSION:
        raise HSError("libhslabs ABI version mismatch")
    _lib = L
    return L


def check(rc: int, what: str = "") -> None:
    if rc != HS_OK:
        msg = load().hs_last_error().decode(errors="replace")
        raise HSError(f"{what}: {msg} (rc={rc})")
