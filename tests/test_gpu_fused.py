"""Fused control steps (hs_run_calls): the steps of hs_run_steps in few launches over
(step, rollout), every step with its own output rows. Bitwise equality with the launch-per-step
path is expected: the same kernel code per step, the gait setup stored by a setup-only pass
(the same values the first launch of hs_run_steps stores), the work summed in step order.
"""
import os

import numpy as np
import pytest

from conftest import MODELS

pytestmark = pytest.mark.gpu

OUTS = ("q", "dq", "tau", "cf", "x", "flags", "work_cot")


@pytest.fixture(scope="module")
def gpu(product):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return product


@pytest.fixture(scope="module")
def hmodels(gpu):
    return {n: gpu.KinematicModel(os.path.join(MODELS, f"{n}.xml")) for n in ("hexapod", "spider", "myant")}


def npy(t):
    return None if t is None else t.cpu().numpy()


@pytest.mark.parametrize("name,B", [("hexapod", 1000), ("spider", 3), ("myant", 257)])
def test_fused_cycle_equals_horizon_run(gpu, hmodels, name, B):
    """n_t calls of H = 1 from k0 = 0 are the rows of one hs_run with H = n_t."""
    import torch
    from hslabs_amd import synth

    m = hmodels[name]
    p = synth.gen_params(B, name)
    ref = gpu.DeviceBatch(m, p, n_t=20, horizon=20, outputs=OUTS)
    ref.run(best=True)
    fz = gpu.DeviceBatch(m, p, n_t=20, horizon=20, outputs=OUTS)
    fz.work_cot.zero_()
    fz.run_calls(20, call_horizon=1, best=True, accumulate=False)
    torch.cuda.synchronize()
    for k in ("q", "dq", "tau", "cf", "x", "flags", "work_cot", "best_key"):
        assert np.array_equal(npy(getattr(ref, k)), npy(getattr(fz, k)), equal_nan=True), k


def test_fused_wraps_like_run_steps(gpu, hmodels):
    """45 calls (more than a cycle, k0 wrapping mod n_t) of H = 3 with accumulated work equal the
    launch-per-call loop, call by call."""
    import torch
    from hslabs_amd import synth

    m = hmodels["hexapod"]
    p = synth.gen_params(129, "hexapod", curved=True)
    n_calls, Hc = 45, 3
    seq = gpu.DeviceBatch(m, p, n_t=20, k0=5, horizon=Hc, outputs=OUTS)
    seq.work_cot.zero_()
    rows = {k: [] for k in ("q", "tau", "cf", "x", "flags")}
    for c in range(n_calls):
        seq.k0 = (5 + c * Hc) % 20
        seq.run(best=False, accumulate=True)
        for k in rows:
            rows[k].append(npy(getattr(seq, k)))
    fz = gpu.DeviceBatch(m, p, n_t=20, k0=5, horizon=n_calls * Hc, outputs=OUTS)
    fz.work_cot.zero_()
    fz.run_calls(n_calls, call_horizon=Hc, accumulate=True)
    torch.cuda.synchronize()
    for k in rows:
        want = np.concatenate(rows[k], axis=1)
        assert np.array_equal(want, npy(getattr(fz, k)), equal_nan=True), k
    assert np.array_equal(npy(seq.work_cot), npy(fz.work_cot))


def test_fused_fp32_equals_fp32_steps(gpu, hmodels):
    import torch
    from hslabs_amd import synth

    m = hmodels["spider"]
    p = synth.gen_params(512, "spider")
    ref = gpu.DeviceBatch(m, p, n_t=20, horizon=32, outputs=OUTS, dtype=torch.float32)
    ref.run(best=True)
    fz = gpu.DeviceBatch(m, p, n_t=20, horizon=32, outputs=OUTS, dtype=torch.float32)
    fz.work_cot.zero_()
    fz.run_calls(1, call_horizon=32, best=True, accumulate=False)
    torch.cuda.synchronize()
    for k in ("tau", "cf", "x", "flags", "work_cot", "best_key"):
        assert np.array_equal(npy(getattr(ref, k)), npy(getattr(fz, k)), equal_nan=True), k


def test_fused_argument_errors(gpu, hmodels):
    import ctypes

    from hslabs_amd import capi, synth

    b = gpu.DeviceBatch(hmodels["hexapod"], synth.gen_params(4, "hexapod"), horizon=2)
    a = b._args(None, False, True)
    L = capi.load()
    assert L.hs_run_calls(hmodels["hexapod"].handle, ctypes.byref(a), -1) != 0
    assert L.hs_run_calls(hmodels["hexapod"].handle, ctypes.byref(a), 0) == 0
    a.horizon = 0
    assert L.hs_run_calls(hmodels["hexapod"].handle, ctypes.byref(a), 2) != 0


def test_fused_mixed_plan_equals_steps(gpu, hmodels):
    """configs[4]'s plan (myant + hexapod interleaved): fused calls = one launch per call."""
    import torch
    from hslabs_amd import synth

    models = [hmodels[n] for n in synth.MIXED_MODELS]
    params, midx = synth.gen_mixed(301)
    n_calls = 25
    seq = gpu.MixedBatch(models, midx, params, n_t=20, k0=0, horizon=1, outputs=("tau", "cf", "flags", "work_cot"))
    seq.work_cot.zero_()
    rows = {k: [] for k in ("tau", "cf", "flags")}
    for c in range(n_calls):
        seq.k0 = c % 20
        seq.run(best=False, accumulate=True)
        for k in rows:
            rows[k].append(npy(getattr(seq, k)))
    fz = gpu.MixedBatch(models, midx, params, n_t=20, k0=0, horizon=n_calls,
                        outputs=("tau", "cf", "flags", "work_cot"))
    fz.work_cot.zero_()
    fz.run_calls(n_calls, call_horizon=1, accumulate=True, best=True)
    torch.cuda.synchronize()
    for k in rows:
        assert np.array_equal(np.concatenate(rows[k], axis=1), npy(getattr(fz, k)), equal_nan=True), k
    assert np.array_equal(npy(seq.work_cot), npy(fz.work_cot))
    key = npy(fz.best_key).view(np.uint64)[0]
    from hslabs_amd import capi

    L = capi.load()
    want = min(L.hs_best_key_encode(float(c), i) for i, c in enumerate(npy(fz.work_cot)[:, 1]))
    assert int(key) == want
