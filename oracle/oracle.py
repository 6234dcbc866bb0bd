"""ctypes wrapper around the oracle (TEST INFRASTRUCTURE ONLY).

The oracle is the CPU restatement of the HSLabs hot path (see hs_oracle.h for
what it restates and how parity is pinned). Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module; the product package
``hslabs_amd`` never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from dataclasses import dataclass, field

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libhs_oracle.so")

BASIS_ORTHO = 0
BASIS_TREE = 1

FLAG_RANK_RETRY = 1
FLAG_FULL_RANK = 2
FLAG_LOOP_EXHAUST = 4
FLAG_NAN = 8
FLAG_UNREACH = 16
FLAG_NO_CONTACT = 32
FLAG_GENERAL = 64
FLAG_NEAR_RANK = 256  # a rank / routing decision within rounding of its threshold (hs_oracle.cpp NearTrack)
FLAG_DEPENDENT = 512  # solve_forces: a column dropped as dependent, the basic solution returned
FORCES_KERNEL = 0     # solve_forces' rank rules (hso_forces_rule): the kernel's pivot guard
FORCES_SPARSEQR = 1   # Eigen SparseQR's default threshold (COLAMD order not restated)
NEAR_KINDS = {0: "none", 1: "LU pivot", 2: "threshold doubled", 3: "rel_error", 4: "QR pivot", 5: "collinear guard",
              6: "pivot guard", 7: "ill-conditioned second stage"}
BASIS_FAST = 2


class Gait(ctypes.Structure):
    """pgsconfigparams (pergen.h:137-146)."""

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
    ]


@dataclass
class GaitParams:
    xml_file: str = "hexapod.xml"
    torso_pos: tuple = (0.0, 0.0, 0.0)
    torso_angles: tuple = (0.0, 0.0, 0.0)
    step_duration: float = 1.0
    period: float = 3.0
    step_length: float = 0.5
    step_height: float = 0.1
    curvature: float = 0.0
    foot_shift_type: int = -1
    foot_shift: float = 0.0
    rec_transform: tuple | None = None  # (rec_transl, rec_eas): pergensetup::set_rec_transform

    def to_c(self) -> Gait:
        g = Gait()
        for i in range(3):
            g.torso_pos[i] = self.torso_pos[i]
            g.torso_angles[i] = self.torso_angles[i]
        g.step_duration = self.step_duration
        g.period = self.period
        g.step_length = self.step_length
        g.step_height = self.step_height
        g.curvature = self.curvature
        g.foot_shift = self.foot_shift
        g.foot_shift_type = self.foot_shift_type
        if self.rec_transform is not None:
            g.rec_transform_flag = 1
            for i in range(3):
                g.rec_transl[i] = self.rec_transform[0][i]
                g.rec_eas[i] = self.rec_transform[1][i]
        return g


def parse_pgs_line(rest: str) -> GaitParams:
    """modelplayer::get_pgs_config_params (player.cpp:170-208)."""
    toks = rest.split()
    p = GaitParams()
    i = 0
    while i < len(toks):
        key = toks[i]
        i += 1
        if key == "xml_file":
            p.xml_file = toks[i]; i += 1
        elif key == "torso_pos":
            p.torso_pos = tuple(float(t) for t in toks[i:i + 3]); i += 3
        elif key == "torso_angles":
            p.torso_angles = tuple(float(t) for t in toks[i:i + 3]); i += 3
        elif key == "step_duration":
            p.step_duration = float(toks[i]); i += 1
        elif key == "period":
            p.period = float(toks[i]); i += 1
        elif key == "step_length":
            p.step_length = float(toks[i]); i += 1
        elif key == "step_height":
            p.step_height = float(toks[i]); i += 1
        elif key == "curvature":
            p.curvature = float(toks[i]); i += 1
        elif key == "lateral_foot_shift":
            p.foot_shift_type, p.foot_shift = 0, float(toks[i]); i += 1
        elif key == "radial_foot_shift":
            p.foot_shift_type, p.foot_shift = 1, float(toks[i]); i += 1
        else:
            raise ValueError(f"unknown key {key}")
    return p


def load_pgs_config(path: str, setup_id: int) -> GaitParams:
    """modelplayer::get_rec_str (player.cpp:230-244) + get_pgs_config_params."""
    with open(path) as f:
        for line in f:
            parts = line.split(None, 1)
            if parts and parts[0].lstrip("-").isdigit() and int(parts[0]) == setup_id:
                return parse_pgs_line(parts[1] if len(parts) > 1 else "")
    raise KeyError(f"no string with rec_id = {setup_id}")


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None
_perf = {}


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = _bind(LIB_PATH)
    return _lib


def perf_lib(tag: str, timeout: float = 180.0):
    """The CPU-baseline build (-O3 -march=native) for this machine's CPU (tag), built on first use
    (bench.py cpu_baseline only; the parity checker is lib()). Returns (CDLL, path) or raises."""
    if tag not in _perf:
        safe = "".join(c if c.isalnum() else "_" for c in tag)[:48]
        subprocess.run(["make", "-s", "-C", HERE, "perf", f"PERF_TAG={safe}"], check=True, timeout=timeout)
        path = os.path.join(HERE, "_build", f"perf_{safe}", "libhs_oracle.so")
        _perf[tag] = (_bind(path), path)
    return _perf[tag]


def _bind(path):
    L = ctypes.CDLL(path)
    dp = ctypes.POINTER(ctypes.c_double)
    L.hso_model_load.argtypes = [ctypes.c_char_p, ctypes.POINTER(ctypes.c_void_p)]
    L.hso_model_free.argtypes = [ctypes.c_void_p]
    L.hso_model_dims.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    L.hso_model_set_torso_penalty.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    L.hso_rollout.argtypes = [ctypes.c_void_p, ctypes.POINTER(Gait), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                              ctypes.c_int, ctypes.c_int, dp, dp, dp, dp,
                              ctypes.POINTER(ctypes.c_uint32), dp, dp]
    L.hso_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(Gait), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, dp, dp, dp,
                            ctypes.POINTER(ctypes.c_uint32)]
    L.hso_batch_near.argtypes = [ctypes.c_void_p, ctypes.POINTER(Gait), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                 ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, dp, dp, dp,
                                 ctypes.POINTER(ctypes.c_uint32), dp]
    L.hso_forces.argtypes = [ctypes.c_void_p, ctypes.POINTER(Gait), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                             ctypes.c_int, dp, dp, ctypes.POINTER(ctypes.c_uint32)]
    L.hso_forces_rule.argtypes = [ctypes.c_void_p, ctypes.POINTER(Gait), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                  ctypes.c_int, ctypes.c_int, dp, dp, ctypes.POINTER(ctypes.c_uint32)]
    L.hso_forces_batch.argtypes = [ctypes.c_void_p, ctypes.POINTER(Gait), ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, dp, dp, ctypes.POINTER(ctypes.c_uint32)]
    L.hso_lik_roundtrip.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64]
    L.hso_lik_roundtrip.restype = ctypes.c_double
    L.hso_euler_roundtrip.argtypes = [dp, dp]
    L.hso_rot_ztov.argtypes = [dp, dp]
    L.hso_fk_ik_check.argtypes = [ctypes.c_void_p, ctypes.POINTER(Gait), ctypes.c_double, ctypes.c_int]
    L.hso_fk_ik_check.restype = ctypes.c_double
    L.hso_residuals.argtypes = [ctypes.c_void_p, ctypes.POINTER(Gait), ctypes.c_int, ctypes.c_int,
                                ctypes.c_int, dp]
    L.hso_pergen_rec.argtypes = [ctypes.c_void_p, ctypes.POINTER(Gait), ctypes.c_double, dp]
    L.hso_lik.argtypes = [ctypes.c_void_p, dp, ctypes.c_int, dp, ctypes.POINTER(ctypes.c_int)]
    L.hso_fk.argtypes = [ctypes.c_void_p, dp, dp, dp]
    ip = ctypes.POINTER(ctypes.c_int32)
    L.hso_dynrec_dump.argtypes = [ctypes.c_void_p, ctypes.POINTER(Gait), ctypes.c_int, ctypes.c_int,
                                  dp, dp, dp, dp, dp, dp, ip, ip, ip, ip]
    up = ctypes.POINTER(ctypes.c_uint32)
    if not hasattr(L, "hso_sim_reset"):  # the FLOP-counting build has no simulation part
        return L
    L.hso_sim_reset.argtypes = [ctypes.c_void_p, dp, dp]
    L.hso_sim_hinges.argtypes = [ctypes.c_void_p, dp, dp, dp]
    L.hso_sim_run.argtypes = [ctypes.c_void_p, dp, ctypes.c_int, ctypes.c_int, dp, dp, dp, dp, up, ip,
                              ctypes.c_int, dp, dp, dp, ip, dp]
    L.hso_sim_batch.argtypes = [ctypes.c_void_p, dp, ctypes.c_int, ctypes.c_int, ctypes.c_int, dp, dp, dp, dp,
                                up, ip, ctypes.c_int, ctypes.c_int]
    return L


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


@dataclass
class Model:
    path: str
    handle: ctypes.c_void_p = field(default=None)
    n: int = 0
    nmj: int = 0
    nf: int = 0
    cfg: int = 0
    lik_index: int = -1
    n_limbs: int = 0
    L: object = field(default=None, repr=False)  # the build that owns the handle (default lib())

    def __post_init__(self):
        self.L = self.L or lib()
        h = ctypes.c_void_p()
        rc = self.L.hso_model_load(self.path.encode(), ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"oracle: cannot load {self.path} (rc={rc})")
        self.handle = h
        d = (ctypes.c_int * 6)()
        self.L.hso_model_dims(h, d)
        self.n, self.nmj, self.nf, self.cfg, self.lik_index, self.n_limbs = list(d)

    def switch_torso_penalty(self, force: bool, torque: bool):
        """periodic::switch_torso_penalty (ftsolver.cpp:262-273) for every later solve of this model;
        (False, False) raises: the reference exits (ftsolver.cpp:245)"""
        rc = self.L.hso_model_set_torso_penalty(self.handle, int(bool(force)), int(bool(torque)))
        if rc != 0:
            raise ValueError(f"oracle: switch_torso_penalty({force}, {torque}) rejected (rc={rc})")

    def __del__(self):
        try:
            if self.handle:
                self.L.hso_model_free(self.handle)
        except Exception:
            pass


def rollout(model: Model, gait: GaitParams, n_t: int = 20, k0: int = 0, H: int | None = None,
            basis: int = BASIS_ORTHO, ignore_reach: bool = True) -> dict:
    """One rollout through the oracle: returns q, tau, cf, x, flags, work, cot, diag."""
    if H is None:
        H = n_t
    ns = k0 + H + 4
    q = np.zeros((ns, model.cfg))
    tau = np.zeros((H, model.nmj))
    cf = np.zeros((H, 3 * model.nf))
    x = np.zeros((H, 6 * model.n))
    flags = np.zeros(H, dtype=np.uint32)
    wc = np.zeros(2)
    diag = np.zeros((H, 4))
    g = gait.to_c()
    rc = lib().hso_rollout(model.handle, ctypes.byref(g), n_t, k0, H, basis, int(ignore_reach),
                           _ptr(q), _ptr(tau), _ptr(cf), _ptr(x),
                           flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), _ptr(wc), _ptr(diag))
    if rc != 0:
        raise RuntimeError(f"oracle rollout failed rc={rc}")
    return dict(q=q, tau=tau, cf=cf, x=x, flags=flags, work=wc[0], cot=wc[1], diag=diag)


def motor_adas(model: Model, gait: GaitParams, tsi: int, n_t: int = 20, ignore_reach: bool = True):
    """periodic::get_motor_adas (periodic.cpp:394-404): motor angles of trajectory sample tsi
    (mod n_t, lifted to [2, n_t + 1]) and their rates from compute_vel_traj (periodic.cpp:261-282:
    central difference, +-pi wrap, / 2 dt); also that step's computed torques
    (get_computed_torques(tsi), periodic.h:51). -> (q0, dq0, tau_ff), each [nmj]."""
    tsi %= n_t
    if tsi < 2:
        tsi += n_t
    r = rollout(model, gait, n_t, k0=tsi - 2, H=1, basis=BASIS_FAST, ignore_reach=ignore_reach)
    q = r["q"]
    d = q[tsi + 1] - q[tsi - 1]
    d = np.where(d > np.pi, d - 2 * np.pi, np.where(d < -np.pi, d + 2 * np.pi, d))
    dt = gait.period / n_t
    return q[tsi, 6:].copy(), (d / (2 * dt))[6:], r["tau"][0]


def pd_torques(model: Model, gait: GaitParams, tsi: int, q, dq, k: float = 100.0, n_t: int = 20,
               ignore_reach: bool = True):
    """modelplayer::set_position_control_torques + linear_feedback_control (player.cpp:388-432):
    tau = tau_ff + (k1 * modulus(q - q0, 2 pi) + k2 * (dq - dq0)), k1 = -k, k2 = -2 sqrt(k);
    arrayops::modulus maps into (-pi, pi] (core.cpp:122-131). -> (tau_cmd, q0, dq0)."""
    q0, dq0, tau_ff = motor_adas(model, gait, tsi, n_t, ignore_reach)
    k1, k2 = -k, -2 * np.sqrt(k)
    a1 = np.asarray(q, dtype=np.float64) - q0
    a1 = np.where(a1 > np.pi, a1 - 2 * np.pi, np.where(a1 <= -np.pi, a1 + 2 * np.pi, a1))
    a1 = a1 * k1
    a2 = (np.asarray(dq, dtype=np.float64) - dq0) * k2
    a1 = a1 + a2
    return tau_ff + a1, q0, dq0


def forces(model: Model, gait: GaitParams, tau_in, n_t: int = 20, k0: int = 0, ignore_reach: bool = True,
           rule: int = FORCES_KERNEL) -> dict:
    """Contact forces of all feet given motor torques tau_in [H][nmj] (ftsolver.cpp:331-378); rule: the
    rank rule of a (numerically) rank-deficient least squares (FORCES_KERNEL or FORCES_SPARSEQR)."""
    tau_in = np.ascontiguousarray(tau_in, dtype=np.float64)
    H = tau_in.shape[0]
    cf = np.zeros((H, 3 * model.nf))
    flags = np.zeros(H, dtype=np.uint32)
    g = gait.to_c()
    rc = lib().hso_forces_rule(model.handle, ctypes.byref(g), n_t, k0, H, int(ignore_reach), rule, _ptr(tau_in),
                               _ptr(cf), flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    if rc != 0:
        raise RuntimeError(f"oracle forces failed rc={rc}")
    return dict(cf=cf, flags=flags)


def forces_batch(model: Model, gaits: list, tau_in, n_t: int = 20, k0: int = 0, ignore_reach: bool = True,
                 n_threads: int = 1, L=None) -> dict:
    """forces() for B rollouts on n_threads threads: tau_in [B][H][nmj] -> cf [B][H][3 nf], flags [B][H]."""
    L = L or lib()
    tau_in = np.ascontiguousarray(tau_in, dtype=np.float64)
    B, H = tau_in.shape[:2]
    arr = (Gait * B)(*[g.to_c() for g in gaits])
    cf = np.zeros((B, H, 3 * model.nf))
    flags = np.zeros((B, H), dtype=np.uint32)
    rc = L.hso_forces_batch(model.handle, arr, B, n_t, k0, H, int(ignore_reach), n_threads, _ptr(tau_in), _ptr(cf),
                            flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)))
    if rc != 0:
        raise RuntimeError(f"oracle forces_batch failed rc={rc}")
    return dict(cf=cf, flags=flags)


def batch(model: Model, gaits: list, n_t: int, k0: int, H: int, basis: int = BASIS_TREE,
          ignore_reach: bool = True, n_threads: int = 1, L=None) -> dict:
    """B rollouts on n_threads threads. L: another build of the same restatement (perf_lib) whose
    hso_model the Model was loaded with (Model(path, L=...)). near_margin / near_kind: per step, the
    decision closest to its threshold (margin <= 1 sets FLAG_NEAR_RANK; NEAR_KINDS)."""
    L = L or lib()
    B = len(gaits)
    arr = (Gait * B)(*[g.to_c() for g in gaits])
    tau = np.zeros((B, H, model.nmj))
    cf = np.zeros((B, H, 3 * model.nf))
    wc = np.zeros((B, 2))
    flags = np.zeros((B, H), dtype=np.uint32)
    near = np.zeros((B, H, 4))
    rc = L.hso_batch_near(model.handle, arr, B, n_t, k0, H, basis, int(ignore_reach), n_threads,
                          _ptr(tau), _ptr(cf), _ptr(wc), flags.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                          _ptr(near))
    if rc != 0:
        raise RuntimeError(f"oracle batch failed rc={rc}")
    return dict(tau=tau, cf=cf, work=wc[:, 0], cot=wc[:, 1], flags=flags, near_margin=near[..., 0],
                near_kind=near[..., 1].astype(np.int32), lu_kept=near[..., 2], qr_kept=near[..., 3])


def lik_roundtrip(model: Model, n: int = 1000, seed: int = 1) -> float:
    return lib().hso_lik_roundtrip(model.handle, n, seed)


def euler_roundtrip(angles) -> np.ndarray:
    a = np.ascontiguousarray(angles, dtype=np.float64)
    out = np.zeros(3)
    lib().hso_euler_roundtrip(_ptr(a), _ptr(out))
    return out


def rot_ztov(v) -> np.ndarray:
    a = np.ascontiguousarray(v, dtype=np.float64)
    out = np.zeros(9)
    lib().hso_rot_ztov(_ptr(a), _ptr(out))
    return out.reshape(3, 3).T  # stored column-major


def fk_ik_check(model: Model, gait: GaitParams, t: float, ignore_reach: bool = True) -> float:
    g = gait.to_c()
    return lib().hso_fk_ik_check(model.handle, ctypes.byref(g), t, int(ignore_reach))


def pergen_rec(model: Model, gait: GaitParams, t: float) -> np.ndarray:
    """pergensetup::set_rec (pergen.cpp:225-239): [6 + 3 n_limbs]."""
    g = gait.to_c()
    rec = np.zeros(6 + 3 * model.n_limbs)
    lib().hso_pergen_rec(model.handle, ctypes.byref(g), t, _ptr(rec))
    return rec


def set_jvalues_with_lik(model: Model, rec, ignore_reach: bool = False, config=None):
    """kinematicmodel::set_jvalues_with_lik (model.cpp:354-359) -> (config, ok, unreach)."""
    r = np.ascontiguousarray(rec, dtype=np.float64)
    q = np.zeros(model.cfg) if config is None else np.array(config, dtype=np.float64)
    u = ctypes.c_int(0)
    rc = lib().hso_lik(model.handle, _ptr(r), int(ignore_reach), _ptr(q), ctypes.byref(u))
    return q, rc == 0, bool(u.value)


def recompute_modelnodes(model: Model, config):
    """set_jvalues + recompute_modelnodes (model.cpp:314-318, 361-366): (A_ground, joint A_ground) of
    every node as [n][3][4] (zeros for a node without a joint)."""
    q = np.ascontiguousarray(config, dtype=np.float64)
    ag, aj = np.zeros(model.n * 12), np.zeros(model.n * 12)
    lib().hso_fk(model.handle, _ptr(q), _ptr(ag), _ptr(aj))
    return (ag.reshape(model.n, 4, 3).transpose(0, 2, 1).copy(), aj.reshape(model.n, 4, 3).transpose(0, 2, 1).copy())


def residuals(model: Model, gait: GaitParams, n_t: int, step: int, basis: int):
    g = gait.to_c()
    out = np.zeros(2)
    k = lib().hso_residuals(model.handle, ctypes.byref(g), n_t, step, basis, _ptr(out))
    return k, out[0], out[1]


def dynrec_dump(model: Model, gait: GaitParams, n_t: int, step: int) -> dict:
    """Dynamics record of step `step` (sample step+2): the inputs of ftsolver."""
    n, nf = model.n, model.nf
    out = {k: np.zeros((n, 3)) for k in ("pos", "jpos", "jz", "mom_rate", "amr")}
    out["fpos"] = np.zeros((nf, 3))
    out["contacts"] = np.zeros(nf, np.int32)
    out["parents"] = np.zeros(n, np.int32)
    out["footis"] = np.zeros(nf, np.int32)
    out["hinge_ids"] = np.zeros(model.nmj, np.int32)
    ip = ctypes.POINTER(ctypes.c_int32)
    g = gait.to_c()
    k = lib().hso_dynrec_dump(model.handle, ctypes.byref(g), n_t, step, *[_ptr(out[k]) for k in
                              ("pos", "jpos", "jz", "mom_rate", "amr", "fpos")],
                              *[out[k].ctypes.data_as(ip) for k in ("contacts", "parents", "footis", "hinge_ids")])
    if k < 0:
        raise RuntimeError("dynrec_dump failed")
    out["k"] = k
    return out


# ---------------------------------------------------------------------------
# closed-loop simulation (hs_oracle_sim.cpp): simulate_ode with position control on a
# restated ODE 0.13 QuickStep (player.cpp:325-339, visualization.cpp:140-150, 296-337)
# ---------------------------------------------------------------------------
SIM_BODY = 13  # pos[3], quaternion[4], lvel[3], avel[3]


@dataclass
class SimParams:
    dt: float = 0.01           # modelplayer::play_dt (player.cpp:23)
    k: float = 100.0           # set_position_control_torques (player.cpp:393)
    sor_w: float = 1.3         # ODE default dWorldSetQuickStepW
    erp: float = 0.8           # dWorldSetERP (visualization.cpp:146)
    cfm: float = 1e-10         # ODE dDOUBLE default global CFM (visualization.cpp:147 leaves it)
    gravity: float = 1.0       # visualization.cpp:144
    bounce: float = 0.5        # nearCallback surface (visualization.cpp:310-320)
    bounce_vel: float = 0.1
    soft_cfm: float = 0.001
    mu: float = float("inf")
    iterations: int = 20       # ODE default dWorldSetQuickStepNumIterations

    def p10(self) -> np.ndarray:
        return np.array([self.dt, self.k, self.sor_w, self.erp, self.cfm, self.gravity, self.bounce,
                         self.bounce_vel, self.soft_cfm, self.mu], dtype=np.float64)


def sim_reset(model: Model, config) -> np.ndarray:
    """init_play_config (player.cpp:351-356): body states [n][13] of a configuration."""
    c = np.ascontiguousarray(config, dtype=np.float64)
    body = np.zeros((model.n, SIM_BODY))
    lib().hso_sim_reset(model.handle, _ptr(c), _ptr(body))
    return body


def sim_hinges(model: Model, body):
    b = np.ascontiguousarray(body, dtype=np.float64)
    q = np.zeros(model.nmj)
    dq = np.zeros(model.nmj)
    lib().hso_sim_hinges(model.handle, _ptr(b), _ptr(q), _ptr(dq))
    return q, dq


def controller_tables(model: Model, gait: GaitParams, n_t: int, ignore_reach: bool = True):
    """setup_per_controller tables (player.cpp:370-382) in hs_run's layout (k0 = 0, H = n_t):
    q_tab/dq_tab [n_t][cfg] = trajectory sample h + 2 and its compute_vel_traj rates, tau_tab [n_t][nmj]."""
    r = rollout(model, gait, n_t, k0=0, H=n_t, basis=BASIS_FAST, ignore_reach=ignore_reach)
    q = r["q"]
    d = q[3:n_t + 3] - q[1:n_t + 1]
    d = np.where(d > np.pi, d - 2 * np.pi, np.where(d < -np.pi, d + 2 * np.pi, d))
    dt = gait.period / n_t
    return q[2:n_t + 2].copy(), d / (2 * dt), r["tau"].copy()


def sim_run(model: Model, params: SimParams, n_t: int, q_tab, dq_tab, tau_tab, body, seed: int, tsi: int,
            n_steps: int) -> dict:
    """n_steps of modelplayer::simulate_ode for one rollout. Returns the new state and per-step outputs."""
    body = np.array(body, dtype=np.float64, copy=True)
    q_tab = np.ascontiguousarray(q_tab, dtype=np.float64)
    dq_tab = np.ascontiguousarray(dq_tab, dtype=np.float64)
    tau_tab = np.ascontiguousarray(tau_tab, dtype=np.float64)
    sd = np.array([seed], dtype=np.uint32)
    ts = np.array([tsi], dtype=np.int32)
    out = dict(tau_cmd=np.zeros((n_steps, model.nmj)), q_meas=np.zeros((n_steps, model.nmj)),
               torso=np.zeros((n_steps, 3)), n_contacts=np.zeros(n_steps, np.int32),
               normal_force=np.zeros(n_steps))
    p10 = params.p10()
    ip = ctypes.POINTER(ctypes.c_int32)
    rc = lib().hso_sim_run(model.handle, _ptr(p10), params.iterations, n_t, _ptr(q_tab), _ptr(dq_tab),
                           _ptr(tau_tab), _ptr(body), sd.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                           ts.ctypes.data_as(ip), n_steps, _ptr(out["tau_cmd"]), _ptr(out["q_meas"]),
                           _ptr(out["torso"]), out["n_contacts"].ctypes.data_as(ip), _ptr(out["normal_force"]))
    if rc != 0:
        raise RuntimeError(f"oracle sim_run failed rc={rc}")
    out.update(body=body, seed=int(sd[0]), tsi=int(ts[0]))
    return out


def sim_batch(model: Model, params: SimParams, n_t: int, q_tab, dq_tab, tau_tab, body, seed, tsi, n_steps: int,
              n_threads: int = 1) -> None:
    """B rollouts of sim_run in place (body [B][n][13], seed/tsi [B] advanced), n_threads threads."""
    B = body.shape[0]
    for a in (q_tab, dq_tab, tau_tab, body):
        assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    p10 = params.p10()
    rc = lib().hso_sim_batch(model.handle, _ptr(p10), params.iterations, n_t, B, _ptr(q_tab), _ptr(dq_tab),
                             _ptr(tau_tab), _ptr(body), seed.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                             tsi.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n_steps, n_threads)
    if rc != 0:
        raise RuntimeError(f"oracle sim_batch failed rc={rc}")
