"""The limb-lane step kernel (hslabs_amd/csrc/hs_limb.h, round 6) against hs_rollout_kernel's fused step.

hs_run_calls takes the limb-lane kernel for its fused step launches when the model is of its class
(hs_topo::limb_lane_ok: hexapod, spider, myant), the call solves in HS_SOLVE_AUTO with the IK table and
asks for no x / q / dq rows; HS_LIMB=0 in the environment keeps hs_rollout_kernel. The limb-lane kernel
computes every value with the same operations in the same order (0 to 6 contacts; a guard near its
threshold flagged HS_FLAG_NEAR_RANK as the old kernel flags it), and defers to the fixup launch (the
old kernel's general machinery) every step it does not take -- tier 2, the Eigen-style path, a joint
value past sincos_k_small's range -- so the two kernels' fp64 outputs are BITWISE equal: torques,
contact forces, flags, the accumulated work and COT, and the best key (mixed plans included). The fp32
build and solve_forces' forces mode are held to stated tolerances instead. Parity with the oracle then
follows from tests/test_gpu_parity.py, which runs the default (limb-lane) path.
"""
import os

import numpy as np
import pytest

from conftest import MODELS, transformed

pytestmark = pytest.mark.gpu

OUTS = ("tau", "cf", "flags", "work_cot")


@pytest.fixture(scope="module")
def gpu(product):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return product


@pytest.fixture(scope="module")
def hmodels(gpu):
    return {n: gpu.KinematicModel(os.path.join(MODELS, f"{n}.xml")) for n in ("hexapod", "spider", "myant")}


def run(gpu, model, params, limb, K=20, Hc=1, k0=0, best=True, dtype=None, rollout_id_base=0, steps=False,
        accumulate=True):
    """K calls of Hc steps: fused (hs_run_calls, K * Hc output rows) or steps=True (hs_run_steps, a launch
    per call, each call writing rows [0, Hc); limb: its opt-in online shape, HS_LIMB_ONLINE=1)"""
    import torch

    old = os.environ.get("HS_LIMB")
    os.environ["HS_LIMB"] = "1" if limb else "0"
    os.environ["HS_LIMB_ONLINE"] = "1" if limb and steps else "0"
    try:
        b = gpu.DeviceBatch(model, params, n_t=20, k0=k0, horizon=Hc if steps else K * Hc, outputs=OUTS, dtype=dtype,
                            rollout_id_base=rollout_id_base)
        b.key_steps = K * Hc
        b.work_cot.zero_()
        b.reset_best()
        if steps:
            b.run_steps(K, best=best, accumulate=accumulate)
        else:
            b.run_calls(K, call_horizon=Hc, best=best, accumulate=accumulate)
        torch.cuda.synchronize()
        out = {k: getattr(b, k).cpu().numpy() for k in OUTS}
        out["best_key"] = int(b.best_key.item())
        return out
    finally:
        os.environ.pop("HS_LIMB_ONLINE")
        if old is None:
            os.environ.pop("HS_LIMB")
        else:
            os.environ["HS_LIMB"] = old


def same(a, b, what):
    for k in ("tau", "cf", "flags", "work_cot"):
        assert np.array_equal(a[k], b[k], equal_nan=True), \
            f"{what}: {k} differs on {int((a[k] != b[k]).sum())} entries (max {np.nanmax(np.abs(a[k].astype(float) - b[k].astype(float))):.3e})"
    assert a["best_key"] == b["best_key"], what


def test_models_are_of_the_limb_lane_class(gpu, hmodels):
    for n, m in hmodels.items():
        assert m.limb_lane_ok, n


@pytest.mark.parametrize("name,curved,B", [("hexapod", False, 4096), ("hexapod", True, 1003), ("spider", True, 2048),
                                            ("myant", False, 1024), ("spider", False, 517)])
def test_limb_kernel_bitwise_equals_rollout_kernel(gpu, hmodels, name, curved, B):
    """configs[1]'s shape (K = 20 calls of H = 1) and odd batches (idle lanes in the last wavefront):
    straight and turning gaits (the torso record's frames), myant's one- and two-contact steps (solved in
    the limb kernel by fast_solve_lanes' closed forms)"""
    from hslabs_amd import synth

    p = synth.gen_params(B, name, id0=4321, curved=curved)
    n0, d0 = gpu.api.limb_launches(), gpu.api.limb_deferred()
    a = run(gpu, hmodels[name], p, True)
    n1, d1 = gpu.api.limb_launches(), gpu.api.limb_deferred()
    # the share of steps the limb-lane kernel hands to the fixup launch (guards near their thresholds,
    # tier 2, the Eigen-style path): none on the synthetic gaits, 0 to 6 contacts
    share = (d1 - d0) / (B * 20)
    print(f"{name} curved={curved}: {d1 - d0} of {B * 20} steps deferred ({100 * share:.2f} %)")
    assert share <= 0.002
    b = run(gpu, hmodels[name], p, False)
    assert n1 > n0 and gpu.api.limb_launches() == n1  # the limb-lane kernel ran in the first run only
    same(a, b, f"{name} curved={curved} B={B}")
    assert np.isfinite(a["tau"]).all()


def test_limb_kernel_transformed_records(gpu, hmodels):
    """record transforms (tilted, lifted: ill-posed steps the closed form declines, deferred) mixed with
    plain gaits in one wavefront"""
    from hslabs_amd import synth

    rng = np.random.default_rng(17)
    p, _ = transformed(synth.gen_params(512, "hexapod", id0=900, curved=True), rng, tilt=0.05)
    same(run(gpu, hmodels["hexapod"], p, True), run(gpu, hmodels["hexapod"], p, False), "transformed hexapod")


@pytest.mark.parametrize("K,Hc,k0", [(7, 3, 5), (45, 1, 13), (300, 1, 0)])
def test_limb_kernel_call_shapes(gpu, hmodels, K, Hc, k0):
    """calls of H > 1, k0 wrapping mod n_t, and more steps than one launch (256 per launch: two launches
    and their fixups)"""
    from hslabs_amd import synth

    p = synth.gen_params(640, "hexapod", id0=77)
    same(run(gpu, hmodels["hexapod"], p, True, K=K, Hc=Hc, k0=k0),
         run(gpu, hmodels["hexapod"], p, False, K=K, Hc=Hc, k0=k0), f"K={K} H={Hc} k0={k0}")


def test_limb_kernel_configs3_shard(gpu, hmodels):
    """configs[3]'s per-rank shard (32,768 rollouts from id 229,376) with the best key"""
    from hslabs_amd import synth

    p = synth.gen_params(32768, "hexapod", id0=229376)
    same(run(gpu, hmodels["hexapod"], p, True, rollout_id_base=229376),
         run(gpu, hmodels["hexapod"], p, False, rollout_id_base=229376), "configs[3] shard")


@pytest.mark.parametrize("B,K,Hc,dtype", [(4096, 20, 1, "f64"), (1001, 3, 7, "f64"), (2048, 2, 32, "f32")])
def test_limb_kernel_mixed_plan(gpu, hmodels, B, K, Hc, dtype):
    """configs[4]'s mixed plan (myant + hexapod interleaved, one launch: eight rollouts of one model per
    wavefront, the fixup's items in hs_rollout_kernel's slots): fp64 bitwise, fp32 within the bound; the
    rows past myant's joints and feet written 0 (the output buffers start as NaN here)"""
    import torch
    from hslabs_amd import synth

    params, idx = synth.gen_mixed(B)
    ms = [hmodels[n] for n in synth.MIXED_MODELS]
    f32 = dtype == "f32"

    def go(limb):
        old = os.environ.get("HS_LIMB")
        os.environ["HS_LIMB"] = "1" if limb else "0"
        try:
            mb = gpu.MixedBatch(ms, idx, params, n_t=20, k0=0, horizon=K * Hc, outputs=OUTS,
                                dtype=torch.float32 if f32 else None)
            for k in ("tau", "cf"):
                getattr(mb, k).fill_(float("nan"))
            mb.key_steps = K * Hc
            mb.work_cot.zero_()
            mb.reset_best()
            mb.run_calls(K, call_horizon=Hc, best=True, accumulate=True)
            torch.cuda.synchronize()
            out = {k: getattr(mb, k).cpu().numpy() for k in OUTS}
            out["best_key"] = int(mb.best_key.item())
            return out
        finally:
            if old is None:
                os.environ.pop("HS_LIMB")
            else:
                os.environ["HS_LIMB"] = old

    n0 = gpu.api.limb_launches()
    a = go(True)
    assert gpu.api.limb_launches() > n0
    b = go(False)
    assert np.isfinite(a["tau"]).all() and np.isfinite(a["cf"]).all()
    if not f32:
        same(a, b, f"mixed B={B} K={K} H={Hc}")
    else:
        assert (a["flags"] == b["flags"]).mean() > 0.999
        err = np.abs(a["tau"].astype(np.float64) - b["tau"]) / np.maximum(1.0, np.abs(b["tau"].astype(np.float64)))
        assert err.max() < 1e-3


@pytest.mark.parametrize("name,B,K,Hc,curved,straight_legs", [("hexapod", 4096, 20, 1, False, False),
                                                               ("spider", 1003, 4, 5, True, False),
                                                               ("myant", 640, 20, 1, False, False),
                                                               ("hexapod", 512, 10, 1, False, True)])
def test_limb_kernel_forces_bitwise(gpu, hmodels, name, B, K, Hc, curved, straight_legs):
    """solve_forces (hs_run_forces_calls, bench.py --forces' shape first) through the limb-lane kernel's
    forces mode against hs_rollout_kernel's: flags and contact forces bitwise on straight gaits (both take
    the control step's subtree sums for x), within 1e-13 relative on turning gaits; the steps whose foot
    block is near singular (straight legs: the dense normal equations) deferred to the forces fixup"""
    import torch
    from hslabs_amd import synth

    m = hmodels[name]
    p = synth.gen_params(B, name, id0=11, curved=curved)
    if straight_legs:  # long steps and a high torso: legs stretched to the IK's reach
        p["step_length"] *= 2.5
    ctl = gpu.DeviceBatch(m, p, n_t=20, k0=0, horizon=K * Hc, outputs=("tau",))
    ctl.run_calls(K, call_horizon=Hc)
    i = torch.arange(K * Hc, device=ctl.tau.device)[None, :, None]
    j = torch.arange(m.nmj, device=ctl.tau.device)[None, None, :]
    tau = ctl.tau + 0.2 * torch.sin(0.7 * i + 1.3 * j)

    def go(limb):
        old = os.environ.get("HS_LIMB")
        os.environ["HS_LIMB"] = "1" if limb else "0"
        try:
            fb = gpu.DeviceBatch(m, p, n_t=20, k0=0, horizon=K * Hc, outputs=("cf", "flags"))
            fb.cf.fill_(float("nan"))
            fb.forces_launcher(tau, K, call_horizon=Hc)()
            torch.cuda.synchronize()
            return fb.cf.cpu().numpy(), fb.flags.cpu().numpy()
        finally:
            if old is None:
                os.environ.pop("HS_LIMB")
            else:
                os.environ["HS_LIMB"] = old

    n0, d0 = gpu.api.limb_launches(), gpu.api.limb_deferred()
    ca, fa = go(True)
    n1, d1 = gpu.api.limb_launches(), gpu.api.limb_deferred()
    cb, fb_ = go(False)
    assert n1 > n0
    print(f"forces {name}: {d1 - d0} of {B * K * Hc} steps deferred to the forces fixup")
    assert np.array_equal(fa, fb_), f"flags differ on {int((fa != fb_).sum())} steps"
    assert np.isfinite(ca).all()
    err = np.abs(ca - cb) / np.maximum(1.0, np.abs(cb))
    print(f"forces {name}: {int((ca != cb).sum())} of {ca.size} entries differ, max relative {err.max():.2e}")
    if curved:  # turning gaits: ULP-level differences remain on some steps
        assert err.max() < 1e-13
    else:
        assert np.array_equal(ca, cb), f"forces differ on {int((ca != cb).sum())} entries (max relative {err.max():.2e})"


@pytest.mark.parametrize("name,K,Hc,k0,acc", [("hexapod", 20, 1, 0, True), ("hexapod", 6, 4, 17, True),
                                               ("myant", 9, 1, 3, False), ("spider", 1, 20, 0, True)])
def test_limb_kernel_online_calls(gpu, hmodels, name, K, Hc, k0, acc):
    """hs_run_steps through the limb-lane kernel (HS_LIMB_ONLINE=1: a launch per call, then its fixup + work
    reduce; opt-in, slower than the default at B = 4096, hs_capi.cpp hs_run_steps): the call's rows,
    the accumulated (or last call's) work and COT, and the key after the last call, bitwise equal to
    hs_rollout_kernel's launch per call with the general path inline"""
    from hslabs_amd import synth

    p = synth.gen_params(1000, name, id0=31, curved=True)
    n0 = gpu.api.limb_launches()
    a = run(gpu, hmodels[name], p, True, K=K, Hc=Hc, k0=k0, steps=True, accumulate=acc)
    assert gpu.api.limb_launches() == n0 + K
    b = run(gpu, hmodels[name], p, False, K=K, Hc=Hc, k0=k0, steps=True, accumulate=acc)
    same(a, b, f"online {name} K={K} H={Hc}")


@pytest.mark.parametrize("K,Hc,acc", [(20, 1, True), (5, 3, False)])
def test_online_defer_variant_bitwise(gpu, hmodels, K, Hc, acc):
    """HS_ONLINE_DEFER=1 (hs_run_steps on hs_rollout_kernel's fused FIX_DEFER instantiation, a launch per
    call and its fixup + reduce): bitwise the default launch per call with the general path inline"""
    import torch
    from hslabs_amd import synth

    m = hmodels["hexapod"]
    p = synth.gen_params(777, "hexapod", id0=3, curved=True)

    def go(defer):
        os.environ["HS_ONLINE_DEFER"] = "1" if defer else "0"
        try:
            return run(gpu, m, p, False, K=K, Hc=Hc, steps=True, accumulate=acc)
        finally:
            os.environ.pop("HS_ONLINE_DEFER")

    same(go(True), go(False), f"online defer K={K} H={Hc}")


@pytest.mark.parametrize("name,B,K,Hc,curved", [("spider", 16384, 2, 32, False), ("hexapod", 2048, 20, 1, True),
                                                 ("myant", 1024, 20, 1, False)])
def test_limb_kernel_fp32_close_to_rollout_kernel(gpu, hmodels, name, B, K, Hc, curved):
    """the single-precision build (configs[2]'s shape first) takes the limb-lane kernel too; float contraction
    differs by context, so its results are within the fp32 build's stated bound of hs_rollout_kernel's
    float results, not bitwise: the same flags on all but a few near-threshold steps, and torques within
    FP32_TOL (tests/test_gpu.py) relative wherever the flags agree"""
    import torch
    from hslabs_amd import synth

    p = synth.gen_params(B, name, id0=5, curved=curved)
    n0 = gpu.api.limb_launches()
    a = run(gpu, hmodels[name], p, True, K=K, Hc=Hc, dtype=torch.float32)
    assert gpu.api.limb_launches() > n0
    b = run(gpu, hmodels[name], p, False, K=K, Hc=Hc, dtype=torch.float32)
    same_flags = a["flags"] == b["flags"]
    ok = same_flags[..., None] & np.isfinite(a["tau"]) & np.isfinite(b["tau"])
    err = np.abs(a["tau"].astype(np.float64) - b["tau"]) / np.maximum(1.0, np.abs(b["tau"].astype(np.float64)))
    print(f"{name} fp32: flags differ on {int((~same_flags).sum())} of {same_flags.size} steps, "
          f"max rel torque difference {err[ok].max():.2e}")
    assert same_flags.mean() > 0.999
    assert err[ok].max() < 1e-3
    wa, wb = a["work_cot"][:, 0].astype(np.float64), b["work_cot"][:, 0].astype(np.float64)
    assert np.allclose(wa, wb, rtol=1e-3, atol=1e-6)
