"""Python host mirror of the reference's interface for the hot path.

Names follow the reference classes so caller code reads the same:
``KinematicModel`` (kinematicmodel, model.h:96-137), ``PgsConfigParams``
(pgsconfigparams, pergen.h:137-146), ``Periodic`` (periodic, periodic.h:27-87),
``ModelPlayer.measure_cot`` / ``measure_cot_sweep`` (player.cpp:269-321).
Everything runs through the C ABI (include/hslabs.h) on the GPU; there is no
CPU fallback. Errors raise ``HSError`` instead of exit(1).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np

from . import capi

# numpy view of hs_gait_params (192 bytes)
GAIT_DTYPE = np.dtype([
    ("torso_pos", "<f8", (3,)), ("torso_angles", "<f8", (3,)), ("step_duration", "<f8"),
    ("period", "<f8"), ("step_length", "<f8"), ("step_height", "<f8"), ("curvature", "<f8"),
    ("foot_shift", "<f8"), ("foot_shift_type", "<i4"), ("rec_transform_flag", "<i4"),
    ("rec_transl", "<f8", (3,)), ("rec_eas", "<f8", (3,)), ("reserved", "<f8", (5,)),
])
assert GAIT_DTYPE.itemsize == 192


def _require(ok: bool, msg: str) -> None:
    """argument check that survives python -O (the native call would read past a short tensor)"""
    if not ok:
        raise ValueError(msg)

SWEEP_NAMES = ("step_duration", "period", "step_length", "step_height")  # pergen.cpp:423


@dataclass
class PgsConfigParams:
    """pgsconfigparams (pergen.h:137-146)."""

    fname: str = ""
    torso_pos: tuple = (0.0, 0.0, 0.0)
    torso_angles: tuple = (0.0, 0.0, 0.0)
    step_duration: float = 1.0
    period: float = 3.0
    step_length: float = 0.5
    step_height: float = 0.1
    curvature: float = 0.0
    foot_shift: tuple = (-1, 0.0)  # (type, value): -1 none, 0 lateral, 1 radial
    # pergensetup's record transform (pergen.h:75-76; set_rec_transform, pergen.cpp:316-320):
    # None, or (rec_transl, rec_eas) -- every record is then transformed (transform_rec, pergen.cpp:238)
    rec_transform: tuple | None = None

    def set_rec_rotation(self, rec_eas) -> None:
        """pergensetup::set_rec_rotation (pergen.cpp:309-313): the rotation by Euler angles, the
        transform's translation kept (zero unless set before)."""
        transl = (0.0, 0.0, 0.0) if self.rec_transform is None else tuple(self.rec_transform[0])
        self.rec_transform = (transl, tuple(float(v) for v in rec_eas))

    def set_rec_transform(self, rec_transl, rec_eas) -> None:
        """pergensetup::set_rec_transform (pergen.cpp:316-320)."""
        self.rec_transform = (tuple(float(v) for v in rec_transl), tuple(float(v) for v in rec_eas))

    def to_record(self) -> np.ndarray:
        r = np.zeros((), GAIT_DTYPE)
        r["torso_pos"] = self.torso_pos
        r["torso_angles"] = self.torso_angles
        r["step_duration"] = self.step_duration
        r["period"] = self.period
        r["step_length"] = self.step_length
        r["step_height"] = self.step_height
        r["curvature"] = self.curvature
        r["foot_shift_type"] = self.foot_shift[0]
        r["foot_shift"] = self.foot_shift[1]
        if self.rec_transform is not None:
            r["rec_transform_flag"] = 1
            r["rec_transl"] = self.rec_transform[0]
            r["rec_eas"] = self.rec_transform[1]
        return r

    @staticmethod
    def from_record(r) -> "PgsConfigParams":
        return PgsConfigParams(
            torso_pos=tuple(float(v) for v in r["torso_pos"]),
            torso_angles=tuple(float(v) for v in r["torso_angles"]),
            step_duration=float(r["step_duration"]), period=float(r["period"]),
            step_length=float(r["step_length"]), step_height=float(r["step_height"]),
            curvature=float(r["curvature"]), foot_shift=(int(r["foot_shift_type"]), float(r["foot_shift"])),
            rec_transform=((tuple(float(v) for v in r["rec_transl"]), tuple(float(v) for v in r["rec_eas"]))
                           if int(r["rec_transform_flag"]) else None))


def read_pgs_config(path: str, setup_id: int) -> PgsConfigParams:
    """modelplayer::get_rec_str + get_pgs_config_params (player.cpp:170-244)."""
    L = capi.load()
    c = capi.GaitParamsC()
    buf = ctypes.create_string_buffer(256)
    capi.check(L.hs_pgs_config_read(path.encode(), setup_id, ctypes.byref(c), buf, 256), "hs_pgs_config_read")
    rec = np.frombuffer(bytes(c), dtype=GAIT_DTYPE)[0]
    p = PgsConfigParams.from_record(rec)
    p.fname = buf.value.decode()
    return p


@dataclass
class KinematicModel:
    """kinematicmodel (model.h:96-137) backed by hs_model_t."""

    xml_path: str
    lik_variant: int = -1
    handle: ctypes.c_void_p = field(default=None, repr=False)

    def __post_init__(self):
        L = capi.load()
        h = ctypes.c_void_p()
        capi.check(L.hs_model_load_ex(self.xml_path.encode(), self.lik_variant, ctypes.byref(h)),
                   f"hs_model_load({self.xml_path})")
        self.handle = h
        d = capi.ModelDimsC()
        capi.check(L.hs_model_get_dims(h, ctypes.byref(d)), "hs_model_get_dims")
        self.n_parts, self.nmj, self.nfeet = d.n_parts, d.nmj, d.nfeet
        self.config_dim, self.n_limbs, self.lik_kind = d.config_dim, d.n_limbs, d.lik_kind
        self.total_mass, self.rcap = d.total_mass, d.rcap
        ok = ctypes.c_int32()
        capi.check(L.hs_model_limb_lane(h, ctypes.byref(ok)), "hs_model_limb_lane")
        self.limb_lane_ok = bool(ok.value)  # hs_run_calls' limb-lane kernel takes this model (ABI 15)

    def get_config_dim(self) -> int:
        return self.config_dim

    def switch_torso_penalty(self, force: bool, torque: bool):
        """periodic::switch_torso_penalty (ftsolver.cpp:262-273) for every later solve on this model
        (hs_model_set_torso_penalty); (False, False) raises HSError like the reference's exit."""
        capi.check(capi.load().hs_model_set_torso_penalty(self.handle, int(bool(force)), int(bool(torque))),
                   "hs_model_set_torso_penalty")

    def torso_penalty(self) -> tuple:
        f, t = ctypes.c_int32(), ctypes.c_int32()
        capi.check(capi.load().hs_model_get_torso_penalty(self.handle, ctypes.byref(f), ctypes.byref(t)),
                   "hs_model_get_torso_penalty")
        return bool(f.value), bool(t.value)

    def number_of_motor_joints(self) -> int:
        return self.nmj

    def get_mnode(self, i: int) -> dict:
        """kinematicmodel::get_mnode (model.h:108) as the node's topology record (hs_node_info)."""
        c = capi.NodeInfoC()
        capi.check(capi.load().hs_model_get_node(self.handle, i, ctypes.byref(c)), "hs_model_get_node")
        return {"parent": c.parent, "jtype": c.jtype, "hinge": c.hinge, "foot": c.foot, "limb": c.limb,
                "kids": list(c.kids[:c.n_kids]), "com": np.array(c.com), "foot_pos": np.array(c.foot_pos),
                "mass": c.mass}

    # batched per-configuration kinematics (hs_pergen_rec / hs_model_lik / hs_model_fk, host buffers)
    def pergen_rec(self, params, times) -> np.ndarray:
        """pergensetup::set_rec (pergen.cpp:225-239) of every gait at every time: [B][n_times][6 + 3 n_limbs]."""
        arr = params_array(params)
        t = np.ascontiguousarray(times, dtype=np.float64).reshape(-1)
        rec = np.zeros((len(arr), len(t), 6 + 3 * self.n_limbs))
        dp = ctypes.POINTER(ctypes.c_double)
        capi.check(capi.load().hs_pergen_rec_host(self.handle, arr.ctypes.data_as(ctypes.POINTER(capi.GaitParamsC)),
                                                  len(arr), t.ctypes.data_as(dp), len(t), rec.ctypes.data_as(dp)),
                   "hs_pergen_rec_host")
        return rec

    def set_jvalues_with_lik(self, rec, ignore_reach: bool = False, config=None):
        """kinematicmodel::set_jvalues_with_lik (model.cpp:354-359) for rows rec [n][6 + 3 n_limbs]:
        returns (config [n][config_dim], status [n]); raises HSError when a target is out of reach
        and ignore_reach is off (lik.cpp:321-330)."""
        r = np.ascontiguousarray(rec, dtype=np.float64).reshape(-1, 6 + 3 * self.n_limbs)
        n = len(r)
        q = np.zeros((n, self.config_dim)) if config is None else np.array(config, np.float64).reshape(n, -1)
        st = np.zeros(n, np.uint32)
        dp = ctypes.POINTER(ctypes.c_double)
        capi.check(capi.load().hs_model_lik_host(self.handle, n, r.ctypes.data_as(dp), int(ignore_reach),
                                                 q.ctypes.data_as(dp), st.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32))),
                   "hs_model_lik_host")
        return q, st

    def recompute_modelnodes(self, config, joints: bool = False):
        """kinematicmodel::recompute_modelnodes (model.cpp:314-318) for configurations [n][config_dim]:
        A_ground of every model node as [n][n_parts][3][4] (and the joints' A_ground if joints)."""
        q = np.ascontiguousarray(config, dtype=np.float64).reshape(-1, self.config_dim)
        n = len(q)
        ag = np.zeros((n, self.n_parts, 12))
        aj = np.zeros((n, self.n_parts, 12)) if joints else None
        dp = ctypes.POINTER(ctypes.c_double)
        capi.check(capi.load().hs_model_fk_host(self.handle, n, q.ctypes.data_as(dp), self.config_dim,
                                                ag.ctypes.data_as(dp), None if aj is None else aj.ctypes.data_as(dp)),
                   "hs_model_fk_host")

        def rows(a):  # [c * 3 + r] -> [r][c]
            return a.reshape(n, self.n_parts, 4, 3).transpose(0, 1, 3, 2).copy()
        return (rows(ag), rows(aj)) if joints else rows(ag)

    def __del__(self):
        try:
            if self.handle:
                capi.load().hs_model_free(self.handle)
                self.handle = None
        except Exception:
            pass


def limb_launches() -> int:
    """fused step launches this process made with the limb-lane kernel (hs_limb_launches)"""
    return int(capi.load().hs_limb_launches())


def limb_deferred() -> int:
    """steps the limb-lane kernel deferred to the fixup launch in this process (hs_limb_stats; synchronous)"""
    d = ctypes.c_int64()
    capi.check(capi.load().hs_limb_stats(None, ctypes.byref(d)), "hs_limb_stats")
    return int(d.value)


def params_array(params) -> np.ndarray:
    """list[PgsConfigParams] | structured array -> contiguous GAIT_DTYPE array."""
    if isinstance(params, np.ndarray) and params.dtype == GAIT_DTYPE:
        return np.ascontiguousarray(params)
    arr = np.zeros(len(params), GAIT_DTYPE)
    for i, p in enumerate(params):
        arr[i] = p.to_record()
    return arr


def run_host(model: KinematicModel, params, n_t: int = 20, k0: int = 0, horizon: int | None = None,
             ignore_reach: bool = True, want=("q", "tau", "cf", "x", "flags", "work_cot")) -> dict:
    """Synchronous host-buffer run of the batched path (hs_run_host)."""
    arr = params_array(params)
    B = len(arr)
    H = n_t if horizon is None else horizon
    out = {
        "q": np.zeros((B, H, model.config_dim)) if "q" in want else None,
        "tau": np.zeros((B, H, model.nmj)) if "tau" in want else None,
        "cf": np.zeros((B, H, 3 * model.nfeet)) if "cf" in want else None,
        "x": np.zeros((B, H, 6 * model.n_parts)) if "x" in want else None,
        "flags": np.zeros((B, H), np.uint32) if "flags" in want else None,
        "work_cot": np.zeros((B, 2)) if "work_cot" in want else None,
    }
    dp = ctypes.POINTER(ctypes.c_double)

    def P(a, t=dp):
        return None if a is None else a.ctypes.data_as(t)

    L = capi.load()
    rc = L.hs_run_host(model.handle, arr.ctypes.data_as(ctypes.POINTER(capi.GaitParamsC)), B, n_t, k0, H,
                       int(ignore_reach), P(out["q"]), P(out["tau"]), P(out["cf"]), P(out["x"]),
                       P(out["flags"], ctypes.POINTER(ctypes.c_uint32)), P(out["work_cot"]))
    capi.check(rc, "hs_run_host")
    return out


class ShardedBatch:
    """hs_batch_*: a batch sharded over the devices of this process (device_mask bit d = HIP
    device d), host parameters in, host outputs out, and the best-rollout reduce
    (hs_select_best). The in-process counterpart of one process per GPU (dist.py)."""

    def __init__(self, model: KinematicModel, params, horizon: int = 1, n_t: int = 20, fp32: bool = False,
                 device_mask: int = 1):
        self.model = model
        self.params = params_array(params)
        self.B, self.H, self.n_t = len(self.params), horizon, n_t
        self.dtype = np.float32 if fp32 else np.float64
        L = capi.load()
        h = ctypes.c_void_p()
        capi.check(L.hs_batch_create(model.handle, self.B, horizon, n_t, capi.HS_PREC_F32 if fp32 else capi.HS_PREC_F64,
                                     device_mask, ctypes.byref(h)), "hs_batch_create")
        self.handle = h
        capi.check(L.hs_batch_set_params(h, self.params.ctypes.data_as(ctypes.POINTER(capi.GaitParamsC))),
                   "hs_batch_set_params")

    def _shapes(self) -> dict:
        m, B, H = self.model, self.B, self.H
        return {"q": (B, H, m.config_dim), "tau": (B, H, m.nmj), "cf": (B, H, 3 * m.nfeet),
                "x": (B, H, 6 * m.n_parts), "flags": (B, H), "work": (B,), "cot": (B,)}

    def run(self, k0: int = 0, ignore_reach: bool = True, want=("tau", "cf", "flags", "work", "cot")) -> dict:
        shapes = self._shapes()
        out = {k: np.zeros(shapes[k], np.uint32 if k == "flags" else self.dtype) for k in want}
        o = capi.BatchOutputsC(**{k: v.ctypes.data for k, v in out.items()})
        capi.check(capi.load().hs_batch_run(self.handle, k0, int(ignore_reach), ctypes.byref(o)), "hs_batch_run")
        return out

    def run_device(self, out: dict, k0: int = 0, ignore_reach: bool = True) -> None:
        """hs_batch_run_device: the requested outputs into caller-owned device tensors (any device of
        the process; keys as in run(), whole-batch layouts). Every tensor is checked first: a known
        key, the shape run() uses, the batch's float dtype (flags int32/uint32), contiguous and on a
        GPU -- the native call copies raw bytes sized by the batch and cannot check any of that."""
        import torch

        shapes = self._shapes()
        fdt = torch.float32 if self.dtype == np.float32 else torch.float64
        for k, v in out.items():
            if k not in shapes:
                raise ValueError(f"run_device: unknown output {k!r} (expected one of {sorted(shapes)})")
            if not isinstance(v, torch.Tensor) or not v.is_cuda:
                raise ValueError(f"run_device: {k} must be a GPU tensor")
            want = (torch.int32, torch.uint32) if k == "flags" else (fdt,)
            if v.dtype not in want:
                raise ValueError(f"run_device: {k} has dtype {v.dtype}, expected {' or '.join(map(str, want))}")
            if tuple(v.shape) != shapes[k]:
                raise ValueError(f"run_device: {k} has shape {tuple(v.shape)}, expected {shapes[k]}")
            if not v.is_contiguous():
                raise ValueError(f"run_device: {k} must be contiguous")
        o = capi.BatchOutputsC(**{k: v.data_ptr() for k, v in out.items()})
        capi.check(capi.load().hs_batch_run_device(self.handle, k0, int(ignore_reach), ctypes.byref(o)),
                   "hs_batch_run_device")

    def select_best(self, comm: "Comm | None" = None):
        """(selection cot as float32, rollout id) of the last run's best rollout; with a Comm, the
        best over all ranks (hs_select_best_comm, one RCCL all-reduce)."""
        c, i = ctypes.c_float(), ctypes.c_int64()
        L = capi.load()
        if comm is None:
            capi.check(L.hs_select_best(self.handle, ctypes.byref(c), ctypes.byref(i)), "hs_select_best")
        else:
            capi.check(L.hs_select_best_comm(self.handle, comm.handle, ctypes.byref(c), ctypes.byref(i)),
                       "hs_select_best_comm")
        return c.value, i.value

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and capi._lib is not None:
            capi._lib.hs_batch_free(h)
            self.handle = None


class Comm:
    """hs_comm_t: the RCCL communicator of the best-rollout reduce, one process per GPU
    (SURVEY.md 8e). Rank 0 makes the id (``unique_id``), the caller broadcasts it, every rank
    constructs a Comm with its device current."""

    def __init__(self, n_ranks: int, rank: int, uid: bytes):
        _require(len(uid) == capi.COMM_ID_BYTES, f"a comm id is {capi.COMM_ID_BYTES} bytes")
        h = ctypes.c_void_p()
        capi.check(capi.load().hs_comm_init(n_ranks, rank, uid, ctypes.byref(h)), "hs_comm_init")
        self.handle, self.n_ranks, self.rank = h, n_ranks, rank

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(capi.COMM_ID_BYTES)
        capi.check(capi.load().hs_comm_unique_id(buf), "hs_comm_unique_id")
        return buf.raw

    def reduce_best(self, key, stream=None) -> None:
        """In-place all-reduce(MIN) of a device key tensor (int64 [1] holding the uint64 bits)."""
        import torch

        st = stream if stream is not None else torch.cuda.current_stream(key.device)
        capi.check(capi.load().hs_comm_reduce_best(self.handle, key.data_ptr(), st.cuda_stream), "hs_comm_reduce_best")

    def free(self) -> None:
        if self.handle:
            capi.load().hs_comm_free(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


class DeviceBatch:
    """Device-resident batch (torch tensors on the current HIP device) for hs_run.

    The gait parameter records and every output buffer live in HBM; ``run``
    only enqueues the kernel on the current torch stream.
    """

    def __init__(self, model: KinematicModel, params, n_t: int = 20, k0: int = 0, horizon: int = 1,
                 ignore_reach: bool = True, outputs=("tau", "cf", "work_cot", "flags"), device=None,
                 rollout_id_base: int = 0, dtype=None):
        import torch

        self.torch = torch
        self.model = model
        self._alloc(model, params, n_t, k0, horizon, ignore_reach, outputs, device, rollout_id_base, dtype)

    def _alloc(self, dims, params, n_t, k0, horizon, ignore_reach, outputs, device, rollout_id_base, dtype=None):
        """dtype: torch.float64 (default) or torch.float32 (HS_PREC_F32: single-precision
        arithmetic and outputs, BASELINE configs[2])."""
        torch = self.torch
        arr = params_array(params)
        self.B, self.H, self.n_t, self.k0 = len(arr), horizon, n_t, k0
        self.ignore_reach = ignore_reach
        self.rollout_id_base = rollout_id_base
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.dtype = dtype or torch.float64
        assert self.dtype in (torch.float64, torch.float32)
        self.precision = capi.HS_PREC_F32 if self.dtype == torch.float32 else capi.HS_PREC_F64
        self.params = torch.from_numpy(arr.view(np.uint8).copy()).to(dev)
        f64 = dict(dtype=self.dtype, device=dev)
        B, H = self.B, self.H
        self.q = torch.empty((B, H, dims.config_dim), **f64) if "q" in outputs else None
        self.dq = torch.empty((B, H, dims.config_dim), **f64) if "dq" in outputs else None
        self.tau = torch.empty((B, H, dims.nmj), **f64) if "tau" in outputs else None
        self.cf = torch.empty((B, H, 3 * dims.nfeet), **f64) if "cf" in outputs else None
        self.x = torch.empty((B, H, 6 * dims.n_parts), **f64) if "x" in outputs else None
        self.flags = torch.empty((B, H), dtype=torch.int32, device=dev) if "flags" in outputs else None
        self.work_cot = torch.empty((B, 2), **f64) if "work_cot" in outputs else None
        self.best_key = torch.full((1,), -1, dtype=torch.int64, device=dev)  # UINT64_MAX bit pattern
        self.solve_mode = capi.HS_SOLVE_AUTO  # HS_SOLVE_REFERENCE: every step through the Eigen-style path
        self.key_steps = 0  # steps the best key's work covers (0: those of the call)

    def reset_best(self):
        self.best_key.fill_(-1)

    def _args(self, stream, best: bool, accumulate: bool):
        torch = self.torch
        a = capi.RunArgsC()
        a.n_rollouts, a.horizon, a.k0, a.n_t = self.B, self.H, self.k0, self.n_t
        a.ignore_reach = int(self.ignore_reach)
        a.accumulate = int(accumulate)

        def ptr(t):
            return None if t is None else t.data_ptr()

        a.params = ptr(self.params)
        a.q, a.tau, a.cf, a.x = ptr(self.q), ptr(self.tau), ptr(self.cf), ptr(self.x)
        a.flags, a.work_cot, a.dq = ptr(self.flags), ptr(self.work_cot), ptr(self.dq)
        a.best_key = ptr(self.best_key) if best else None
        a.rollout_id_base = self.rollout_id_base
        a.precision = self.precision
        a.solve_mode = self.solve_mode
        a.key_steps = self.key_steps
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        a.stream = st.cuda_stream
        return a

    def _launch(self, a, n_calls, ev):
        capi.check(capi.load().hs_run_steps(self.model.handle, ctypes.byref(a), n_calls, ev), "hs_run_steps")

    def run(self, stream=None, best: bool = True, accumulate: bool = False) -> None:
        self._launch(self._args(stream, best, accumulate), 1, None)

    def run_pd(self, q_meas, dq_meas, k: float = 100.0, stream=None, targets: bool = False):
        """Position control (hs_run_pd, player.cpp:388-432): motor torque commands for the
        measured motor angles / rates [B][H][nmj] (device tensors) around this batch's
        trajectory; also runs the step (tau = feedforward). Returns tau_cmd, or
        (tau_cmd, q_target, dq_target) with ``targets``."""
        torch = self.torch
        f64 = dict(dtype=self.dtype, device=self.device)
        q = q_meas.to(**f64).contiguous()
        dq = dq_meas.to(**f64).contiguous()
        shape = (self.B, self.H, self.model.nmj)
        _require(q.shape == shape and dq.shape == shape, f"q_meas / dq_meas must be {shape}")
        out = torch.empty(shape, **f64)
        q0 = torch.empty(shape, **f64) if targets else None
        dq0 = torch.empty(shape, **f64) if targets else None
        pd = capi.PdArgsC(q.data_ptr(), dq.data_ptr(), float(k), out.data_ptr(),
                          q0.data_ptr() if targets else None, dq0.data_ptr() if targets else None)
        a = self._args(stream, False, False)
        capi.check(capi.load().hs_run_pd(self.model.handle, ctypes.byref(a), ctypes.byref(pd)), "hs_run_pd")
        self._pd_in = (q, dq)  # keep alive until the stream has consumed them
        return (out, q0, dq0) if targets else out

    def run_forces(self, tau_in, stream=None) -> None:
        """Contact forces of all feet given motor torques (hs_run_forces,
        forcetorquesolver::solve_forces): tau_in is a device tensor [B][H][nmj]; writes
        self.cf (and q / flags if allocated)."""
        t = tau_in.to(dtype=self.dtype, device=self.device).contiguous()
        _require(t.shape == (self.B, self.H, self.model.nmj), f"tau_in must be {(self.B, self.H, self.model.nmj)}")
        a = self._args(stream, False, False)
        a.tau = a.x = a.work_cot = None
        capi.check(capi.load().hs_run_forces(self.model.handle, ctypes.byref(a), t.data_ptr()), "hs_run_forces")
        self._tau_in = t  # keep alive until the stream has consumed it

    def run_forces_calls(self, tau_in, n_calls: int, call_horizon: int = 1, stream=None) -> None:
        """n_calls calls of run_forces with call horizon ``call_horizon`` fused into few launches
        (hs_run_forces_calls): tau_in is a device tensor [B][S][nmj] with S = n_calls *
        call_horizon = this batch's horizon; every step writes its own row of cf (and q / flags)."""
        S = n_calls * call_horizon
        _require(self.H == S, "the batch's horizon must equal n_calls * call_horizon (one row per step)")
        t = tau_in.to(dtype=self.dtype, device=self.device).contiguous()
        _require(t.shape == (self.B, S, self.model.nmj), f"tau_in must be {(self.B, S, self.model.nmj)}")
        a = self._args(stream, False, False)
        a.tau = a.x = a.work_cot = None
        a.horizon = call_horizon
        capi.check(capi.load().hs_run_forces_calls(self.model.handle, ctypes.byref(a), n_calls, t.data_ptr()),
                   "hs_run_forces_calls")
        self._tau_in = t

    def forces_launcher(self, tau_in, n_calls: int, call_horizon: int = 1, stream=None):
        """run_forces_calls(...) with its arguments resolved once: a no-argument callable that only
        enqueues the fused launches (bench.py --forces' timed loop)."""
        S = n_calls * call_horizon
        _require(self.H == S, "the batch's horizon must equal n_calls * call_horizon (one row per step)")
        t = tau_in.to(dtype=self.dtype, device=self.device).contiguous()
        _require(t.shape == (self.B, S, self.model.nmj), f"tau_in must be {(self.B, S, self.model.nmj)}")
        a = self._args(stream, False, False)
        a.tau = a.x = a.work_cot = None
        a.horizon = call_horizon
        L = capi.load()
        ref, h, ptr = ctypes.byref(a), self.model.handle, t.data_ptr()

        def launch():
            rc = L.hs_run_forces_calls(h, ref, n_calls, ptr)
            if rc != capi.HS_OK:
                capi.check(rc, "hs_run_forces_calls")
        launch.args, launch.tau_in = a, t  # keep the struct and the torques alive with the callable
        return launch

    def run_steps(self, n_calls: int, stream=None, best: bool = False, accumulate: bool = True,
                  events=None) -> None:
        """n_calls launches marching k0 through the cycle (hs_run_steps); the launch loop is
        native; the best key (``best``) is taken after the last launch. ``events``: 2*n_calls
        torch.cuda.Event(enable_timing=True), recorded around each launch."""
        a = self._args(stream, best, accumulate)
        ev = None
        if events is not None:
            _require(len(events) == 2 * n_calls, "events must hold 2 * n_calls events")
            st = stream if stream is not None else self.torch.cuda.current_stream(self.device)
            for e in events:  # torch creates the HIP event on first record
                if not e.cuda_event:
                    e.record(st)
            ev = (ctypes.c_void_p * len(events))(*[e.cuda_event for e in events])
        self._launch(a, n_calls, ev)


    def calls_launcher(self, n_calls: int, call_horizon: int = 1, stream=None, best: bool = False,
                       accumulate: bool = True):
        """run_calls(...) with its arguments resolved once: returns a no-argument callable that only
        enqueues the fused launches (for timed loops: no per-call pointer lookups in Python)."""
        _require(self.H >= n_calls * call_horizon, "outputs need one row per fused step")
        a = self._args(stream, best, accumulate)
        a.horizon = call_horizon
        L = capi.load()
        ref = ctypes.byref(a)
        if isinstance(self, MixedBatch):
            fn, h, what = L.hs_run_mixed_calls, self.plan, "hs_run_mixed_calls"
        else:
            fn, h, what = L.hs_run_calls, self.model.handle, "hs_run_calls"

        def launch():
            rc = fn(h, ref, n_calls)
            if rc != capi.HS_OK:
                capi.check(rc, what)
        launch.args = a  # keeps the struct alive with the callable
        return launch

    def run_calls(self, n_calls: int, call_horizon: int = 1, stream=None, best: bool = False,
                  accumulate: bool = True) -> None:
        """The n_calls control steps of run_steps(n_calls) with call horizon ``call_horizon``
        fused into few launches (hs_run_calls): every step keeps its own output row, rows packed
        per rollout with stride n_calls * call_horizon, so this batch's horizon must be at least
        that (equal: the [B][H] views hold the steps in order)."""
        _require(self.H >= n_calls * call_horizon, "outputs need one row per fused step")
        a = self._args(stream, best, accumulate)
        a.horizon = call_horizon
        L = capi.load()
        if isinstance(self, MixedBatch):
            capi.check(L.hs_run_mixed_calls(self.plan, ctypes.byref(a), n_calls), "hs_run_mixed_calls")
        else:
            capi.check(L.hs_run_calls(self.model.handle, ctypes.byref(a), n_calls), "hs_run_calls")


class SimBatch:
    """Closed-loop simulation of a batch of robots (hs_sim_reset / hs_sim_step).

    modelplayer::setup_per_controller (player.cpp:370-382) for every rollout:
    the controller tables come from hs_run over one cycle sampled at
    n_t = int(T / play_dt + .5) (k0 = 0, H = n_t: trajectory, compute_vel_traj
    rates, computed torques), the initial state is the configuration of
    trajectory sample tsi0 with zero velocities (init_play_config); then each
    ``step(n)`` runs n times modelplayer::simulate_ode with position control
    (player.cpp:325-339) in one launch. n_t must be the same for the whole batch
    (group rollouts by period otherwise). All state lives in HBM as torch tensors.
    """

    def __init__(self, model: KinematicModel, params, dt: float = 0.01, tsi0: int = 2, device=None,
                 ignore_reach: bool = True, dtype=None, **sim_overrides):
        """dtype: torch.float64 (default) or torch.float32 (HS_PREC_F32: single-precision tables,
        state and arithmetic, BASELINE configs[2])."""
        import torch

        self.torch = torch
        self.model = model
        arr = params_array(params)
        n_ts = {int(float(T) / dt + .5) for T in arr["period"]}
        if len(n_ts) != 1:
            raise ValueError(f"rollouts need one table length n_t = int(T / dt + .5); got {sorted(n_ts)}")
        self.n_t = n_ts.pop()
        if self.n_t < 2:
            raise ValueError("period shorter than two simulation steps")
        self.B = len(arr)
        self.params = SimBatch.default_params()
        self.params.dt = dt
        for k, v in sim_overrides.items():
            if not hasattr(self.params, k):
                raise TypeError(f"unknown simulation parameter {k}")
            setattr(self.params, k, v)
        dev = device or torch.device("cuda", torch.cuda.current_device())
        self.device = dev
        self.dtype = dtype or torch.float64
        assert self.dtype in (torch.float64, torch.float32)
        self.precision = capi.HS_PREC_F32 if self.dtype == torch.float32 else capi.HS_PREC_F64
        self.tables = DeviceBatch(model, arr, n_t=self.n_t, k0=0, horizon=self.n_t, ignore_reach=ignore_reach,
                                  outputs=("q", "dq", "tau"), device=dev, dtype=self.dtype)
        self.tables.run(best=False)
        self.body = torch.empty((self.B, model.n_parts, capi.SIM_BODY_STRIDE), dtype=self.dtype, device=dev)
        self.seed = torch.zeros(self.B, dtype=torch.int32, device=dev)
        self.tsi = torch.full((self.B,), int(tsi0), dtype=torch.int32, device=dev)
        self.reset(tsi0)

    @staticmethod
    def default_params() -> "capi.SimParamsC":
        p = capi.SimParamsC()
        capi.load().hs_sim_default_params(ctypes.byref(p))
        return p

    def table_row(self, tsi: int) -> int:
        """hs_run output row holding trajectory sample tsi (get_motor_adas lifts tsi < 2 by n_t)."""
        return (tsi % self.n_t + self.n_t - 2) % self.n_t

    def reset(self, tsi0: int = 2, stream=None) -> None:
        """init_play_config (player.cpp:351-356): bodies at trajectory sample tsi0, at rest."""
        torch = self.torch
        config = self.tables.q[:, self.table_row(tsi0), :].contiguous()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        capi.check(capi.load().hs_sim_reset(self.model.handle, self.B, config.data_ptr(), config.shape[1],
                                            self.body.data_ptr(), self.precision, st.cuda_stream), "hs_sim_reset")
        self._config = config
        self.seed.zero_()
        self.tsi.fill_(int(tsi0))

    def step(self, n_steps: int = 1, stream=None, outputs=("tau_cmd", "q_meas", "torso", "n_contacts",
                                                           "normal_force")) -> dict:
        """n_steps of simulate_ode for every rollout (one launch). Returns the requested
        per-step outputs as device tensors [B][n_steps][...]."""
        torch = self.torch
        B, nmj = self.B, self.model.nmj
        f64 = dict(dtype=self.dtype, device=self.device)
        out = {}
        if "tau_cmd" in outputs:
            out["tau_cmd"] = torch.empty((B, n_steps, nmj), **f64)
        if "q_meas" in outputs:
            out["q_meas"] = torch.empty((B, n_steps, nmj), **f64)
        if "torso" in outputs:
            out["torso"] = torch.empty((B, n_steps, 3), **f64)
        if "n_contacts" in outputs:
            out["n_contacts"] = torch.empty((B, n_steps), dtype=torch.int32, device=self.device)
        if "normal_force" in outputs:
            out["normal_force"] = torch.empty((B, n_steps), **f64)
        a = capi.SimArgsC()
        a.n_rollouts, a.n_steps, a.n_t = B, n_steps, self.n_t
        a.precision = self.precision
        a.params = self.params
        a.body, a.seed, a.tsi = self.body.data_ptr(), self.seed.data_ptr(), self.tsi.data_ptr()
        a.q_tab, a.dq_tab, a.tau_tab = self.tables.q.data_ptr(), self.tables.dq.data_ptr(), self.tables.tau.data_ptr()
        for k in ("tau_cmd", "q_meas", "torso", "n_contacts", "normal_force"):
            setattr(a, k, out[k].data_ptr() if k in out else None)
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        a.stream = st.cuda_stream
        capi.check(capi.load().hs_sim_step(self.model.handle, ctypes.byref(a)), "hs_sim_step")
        return out


class MixedBatch(DeviceBatch):
    """Mixed-topology batch (BASELINE configs[4]): rollout b runs models[model_index[b]]
    through one hs_mixed plan. Output rows use the maxima over the models
    (``dims``); entries past a rollout's own dimensions are 0."""

    def __init__(self, models, model_index, params, n_t: int = 20, k0: int = 0, horizon: int = 1,
                 ignore_reach: bool = True, outputs=("tau", "cf", "work_cot", "flags"), device=None,
                 rollout_id_base: int = 0, dtype=None):
        import torch

        self.torch = torch
        self.models = list(models)
        self.model_index = np.ascontiguousarray(model_index, dtype=np.int32)
        L = capi.load()
        if device is not None:
            torch.cuda.set_device(device)
        hs = (ctypes.c_void_p * len(self.models))(*[m.handle for m in self.models])
        plan = ctypes.c_void_p()
        capi.check(L.hs_mixed_create(hs, len(self.models),
                                     self.model_index.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                     len(self.model_index), ctypes.byref(plan)), "hs_mixed_create")
        self.plan = plan
        d = capi.ModelDimsC()
        capi.check(L.hs_mixed_get_dims(plan, ctypes.byref(d)), "hs_mixed_get_dims")
        self.dims = d
        self.model = self.models[0]
        _require(len(params_array(params)) == len(self.model_index), "one parameter record per rollout of the plan")
        self._alloc(d, params, n_t, k0, horizon, ignore_reach, outputs, device, rollout_id_base, dtype)

    def _launch(self, a, n_calls, ev):
        capi.check(capi.load().hs_run_mixed_steps(self.plan, ctypes.byref(a), n_calls, ev), "hs_run_mixed_steps")

    def __del__(self):
        plan = getattr(self, "plan", None)
        if plan:
            try:
                capi.load().hs_mixed_free(plan)
            except Exception:
                pass
            self.plan = None


def complete_traj(model: KinematicModel, params, n_t: int = 20, ignore_reach: bool = True) -> np.ndarray:
    """periodic::get_complete_traj (periodic.cpp:406-426) for a batch (hs_complete_traj):
    [B][n_t][2 * config_dim + nmj] = (configuration, rates, computed torques) per tsi."""
    arr = params_array(params)
    B = len(arr)
    rec = np.zeros((B, n_t, 2 * model.config_dim + model.nmj))
    L = capi.load()
    rc = L.hs_complete_traj(model.handle, arr.ctypes.data_as(ctypes.POINTER(capi.GaitParamsC)), B, n_t,
                            int(ignore_reach), rec.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    capi.check(rc, "hs_complete_traj")
    return rec


def save_2d_array(path: str, rec, append: bool = False) -> None:
    """save_2d_array (core.cpp:46-61) through hs_traj_save: the traj.txt format."""
    a = np.ascontiguousarray(np.asarray(rec, dtype=np.float64).reshape(-1, np.shape(rec)[-1]))
    rc = capi.load().hs_traj_save(path.encode(), a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)), a.shape[0],
                                  a.shape[1], int(append))
    capi.check(rc, "hs_traj_save")


def decode_best_key(key: int):
    """-> (cot as float32, global rollout id)"""
    L = capi.load()
    c = ctypes.c_float()
    i = ctypes.c_int64()
    L.hs_best_key_decode(ctypes.c_uint64(key & 0xFFFFFFFFFFFFFFFF), ctypes.byref(c), ctypes.byref(i))
    return c.value, i.value


class Periodic:
    """periodic (periodic.h:27-87) for one gait setup, computed on the GPU."""

    def __init__(self, model: KinematicModel):
        self.model = model
        self.n_t = 0
        self._res = None

    def record_trajectory(self, pgs: PgsConfigParams, n_t: int) -> None:  # periodic.cpp:77-96
        self.pgs, self.n_t = pgs, n_t
        self._res = None

    def compute_torques_over_period(self) -> None:  # periodic.cpp:377-391
        self._res = run_host(self.model, [self.pgs], n_t=self.n_t, k0=0, horizon=self.n_t)

    def _ensure(self):
        if self._res is None:
            self.compute_torques_over_period()
        return self._res

    def get_computed_torques(self, i: int) -> np.ndarray:  # periodic.h:51 (computed_torques[i % n_t])
        # step h solves sample h+2, stored by the reference at (h+2) % n_t
        h = (i - 2) % self.n_t
        return self._ensure()["tau"][0, h]

    def work_over_period(self) -> float:  # periodic.cpp:285-307
        return float(self._ensure()["work_cot"][0, 0])

    def get_total_mass(self) -> float:
        return self.model.total_mass

    def switch_torso_penalty(self, force: bool, torque: bool) -> None:  # periodic.cpp:205-207
        self.model.switch_torso_penalty(force, torque)
        self._res = None


class _Penalty11:
    """measure_cot's own periodic solves with switch_torso_penalty(1,1) (player.cpp:263); the model's
    setting (another periodic's, in the reference) is restored afterwards"""

    def __init__(self, model: KinematicModel):
        self.model = model

    def __enter__(self):
        self.saved = self.model.torso_penalty()
        if self.saved != (True, True):
            self.model.switch_torso_penalty(True, True)

    def __exit__(self, *exc):
        if self.saved != (True, True):
            self.model.switch_torso_penalty(*self.saved)


class ModelPlayer:
    """The hot-path-facing part of modelplayer (player.cpp:259-321)."""

    def __init__(self, model: KinematicModel):
        self.model = model

    def measure_cot(self, pgs: PgsConfigParams, n_t: int) -> float:  # player.cpp:269-285
        with _Penalty11(self.model):
            r = run_host(self.model, [pgs], n_t=n_t, k0=0, horizon=n_t, want=("work_cot",))
        return float(r["work_cot"][0, 1])

    @staticmethod
    def sweep_params(pgs: PgsConfigParams, param_name: str, val0: float, val1: float, n_val: int):
        """pgssweeper::sweep/next (pergen.cpp:417-449): n_val+1 values."""
        if param_name not in SWEEP_NAMES:
            raise capi.HSError(f"cannot sweep over {param_name}")
        delval = (val1 - val0) / n_val
        out = []
        for vali in range(n_val + 1):
            val = val0 + vali * delval
            p = PgsConfigParams(**{k: getattr(pgs, k) for k in pgs.__dataclass_fields__})
            setattr(p, param_name, val)
            out.append((val, p))
        return out

    def measure_cot_sweep(self, pgs: PgsConfigParams, n_t: int, param_name: str, val0: float, val1: float,
                          n_val: int):
        """All sweep values in one batched launch; returns [(val, cot)] (player.cpp:311-321)."""
        sw = self.sweep_params(pgs, param_name, val0, val1, n_val)
        with _Penalty11(self.model):
            r = run_host(self.model, [p for _, p in sw], n_t=n_t, k0=0, horizon=n_t, want=("work_cot",))
        return [(v, float(r["work_cot"][i, 1])) for i, (v, _) in enumerate(sw)]

    def record_per_traj(self, pgs: PgsConfigParams, n_t: int, path: str = "traj.txt") -> np.ndarray:
        """modelplayer::record_per_traj (player.cpp:617-629): the complete trajectory records of
        one cycle written to traj.txt (n_t rows of 2 * config_dim + nmj)."""
        rec = complete_traj(self.model, [pgs], n_t)[0]
        save_2d_array(path, rec, append=False)
        return rec

    def record_per_traj_sweep(self, pgs: PgsConfigParams, n_t: int, param_name: str, val0: float, val1: float,
                              n_val: int, path: str = "traj.txt") -> np.ndarray:
        """modelplayer::record_per_traj_sweep (player.cpp:631-653): every sweep value's cycle,
        appended one after another; all values in one batched launch."""
        sw = self.sweep_params(pgs, param_name, val0, val1, n_val)
        rec = complete_traj(self.model, [p for _, p in sw], n_t)
        for i in range(len(sw)):
            save_2d_array(path, rec[i], append=i > 0)
        return rec
