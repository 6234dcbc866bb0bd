"""GPU parity of the closed-loop simulation (hs_sim_reset / hs_sim_step, hs_sim.hip)
against the CPU restatement of ODE's QuickStep (oracle/hs_oracle_sim.cpp).

Both sides start from the same body states (the GPU reset, itself checked
against the oracle's) and read the same controller tables (hs_run output), so
the comparison isolates the simulation step. The kernel keeps the oracle's
operation order except for fused multiply-adds inside the SOR sweeps and the
device atan2 (hinge angles): body states agree to ~1e-13 after 100 steps on the
seeded batches below. Tolerances: body state 1e-10, torques / angles 1e-9,
normal force 1e-8 relative; contact counts identical.
"""
import os

import numpy as np
import pytest

from conftest import MODELS

pytestmark = pytest.mark.gpu

BODY_TOL = 1e-10


@pytest.fixture(scope="module")
def gpu(product):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return product


@pytest.fixture(scope="module")
def hmodels(gpu):
    return {n: gpu.KinematicModel(os.path.join(MODELS, f"{n}.xml")) for n in ("hexapod", "spider", "myant")}


def tables(sb):
    return sb.tables.q.cpu().numpy(), sb.tables.dq.cpu().numpy(), sb.tables.tau.cpu().numpy()


def make_batch(gpu, model, name, B, period=3.0, **kw):
    from hslabs_amd import synth

    return gpu.SimBatch(model, synth.gen_sim_params(B, name, period=period), **kw)


@pytest.mark.parametrize("name", ["hexapod", "spider", "myant"])
def test_reset_matches_oracle(gpu, hmodels, oracle_mod, omodels, name):
    sb = make_batch(gpu, hmodels[name], name, 8)
    body = sb.body.cpu().numpy()
    qt, _, _ = tables(sb)
    for b in range(8):
        ob = oracle_mod.sim_reset(omodels[name], qt[b, sb.table_row(2)])
        assert np.abs(ob - body[b]).max() < 1e-12
        q, dq = oracle_mod.sim_hinges(omodels[name], body[b])
        d = (q - qt[b, sb.table_row(2), 6:] + np.pi) % (2 * np.pi) - np.pi
        assert np.abs(d).max() < 1e-12 and np.abs(dq).max() == 0


@pytest.mark.parametrize("name,B,steps", [("hexapod", 24, 100), ("spider", 8, 60), ("myant", 8, 60)])
def test_steps_match_oracle(gpu, hmodels, oracle_mod, omodels, name, B, steps):
    import torch

    sb = make_batch(gpu, hmodels[name], name, B)
    body0 = sb.body.cpu().numpy()
    qt, dqt, tt = tables(sb)
    out = sb.step(steps)
    torch.cuda.synchronize()
    body = sb.body.cpu().numpy()
    o = {k: v.cpu().numpy() for k, v in out.items()}
    P = oracle_mod.SimParams()
    for b in range(B):
        r = oracle_mod.sim_run(omodels[name], P, sb.n_t, qt[b], dqt[b], tt[b], body0[b], 0, 2, steps)
        assert (r["n_contacts"] == o["n_contacts"][b]).all()
        assert np.abs(r["body"] - body[b]).max() < BODY_TOL
        assert np.abs(r["tau_cmd"] - o["tau_cmd"][b]).max() < 1e-9 * max(1, np.abs(r["tau_cmd"]).max())
        assert np.abs(r["q_meas"] - o["q_meas"][b]).max() < 1e-9
        assert np.abs(r["torso"] - o["torso"][b]).max() < BODY_TOL
        assert np.abs(r["normal_force"] - o["normal_force"][b]).max() < 1e-8 * max(1, r["normal_force"].max())
    assert (sb.tsi.cpu().numpy() == 2 + steps).all()
    assert (sb.seed.cpu().numpy() != 0).all()


def test_launch_split_is_bitwise(gpu, hmodels):
    """State (bodies, dRand seed, tsi) fully describes a rollout: 3 launches of 10 steps
    equal one launch of 30, bit for bit."""
    import torch

    a = make_batch(gpu, hmodels["hexapod"], "hexapod", 64)
    b = make_batch(gpu, hmodels["hexapod"], "hexapod", 64)
    oa = a.step(30)
    parts = [b.step(10) for _ in range(3)]
    torch.cuda.synchronize()
    assert torch.equal(a.body, b.body) and torch.equal(a.seed, b.seed) and torch.equal(a.tsi, b.tsi)
    assert torch.equal(oa["tau_cmd"], torch.cat([p["tau_cmd"] for p in parts], dim=1))


def test_rollouts_are_independent(gpu, hmodels):
    """A rollout's trajectory does not depend on its batch neighbours or batch size."""
    import torch
    from hslabs_amd import synth

    params = synth.gen_sim_params(37, "hexapod")
    big = gpu.SimBatch(hmodels["hexapod"], params)
    big.step(40)
    for i in (0, 17, 36):
        one = gpu.SimBatch(hmodels["hexapod"], params[i:i + 1])
        one.step(40)
        torch.cuda.synchronize()
        assert torch.equal(one.body[0], big.body[i])


def test_free_fall_on_gpu(gpu, hmodels):
    """No control, high above the plane: v_z = -n h g for every body, no contacts."""
    import torch

    sb = make_batch(gpu, hmodels["hexapod"], "hexapod", 16, k=0.0)
    sb.body[:, :, 2] += 10.0
    n = 40
    out = sb.step(n)
    torch.cuda.synchronize()
    b = sb.body.cpu().numpy()
    assert np.abs(b[:, :, 9] + n * 0.01).max() < 1e-12
    assert (out["n_contacts"].cpu().numpy() == 0).all()


def test_full_batch_one_period(gpu, hmodels):
    """BASELINE-size batch (4096 hexapods) over one gait period (300 steps): finite states,
    upright torsos, the weight carried on average."""
    import torch

    sb = make_batch(gpu, hmodels["hexapod"], "hexapod", 4096)
    z0 = sb.body[:, 0, 2].clone()
    out = sb.step(300, outputs=("torso", "normal_force", "n_contacts"))
    torch.cuda.synchronize()
    body = sb.body.cpu().numpy()
    assert np.isfinite(body).all()
    z = out["torso"][:, :, 2].cpu().numpy()
    assert (z > 0).all()
    assert np.median(np.abs(z[:, -1] - z0.cpu().numpy())) < 0.1
    fn = out["normal_force"].cpu().numpy()[:, 100:]
    assert abs(np.median(fn.mean(axis=1)) - 22.0) < 0.25 * 22.0  # 22 unit masses, g = 1


def test_bad_arguments_fail_loudly(gpu, hmodels):
    import ctypes

    from hslabs_amd import capi

    sb = make_batch(gpu, hmodels["hexapod"], "hexapod", 2)
    a = capi.SimArgsC()
    a.n_rollouts, a.n_steps, a.n_t = 2, 1, sb.n_t
    a.params = sb.params
    a.params.mu = 0.0
    a.body, a.seed, a.tsi = sb.body.data_ptr(), sb.seed.data_ptr(), sb.tsi.data_ptr()
    a.q_tab, a.dq_tab, a.tau_tab = sb.tables.q.data_ptr(), sb.tables.dq.data_ptr(), sb.tables.tau.data_ptr()
    L = capi.load()
    assert L.hs_sim_step(hmodels["hexapod"].handle, ctypes.byref(a)) == -1
    a.params.mu = float("inf")
    a.q_tab = None
    assert L.hs_sim_step(hmodels["hexapod"].handle, ctypes.byref(a)) == -1
    assert b"tables" in L.hs_last_error()


@pytest.mark.parametrize("name", ["hexapod", "spider", "myant"])
def test_every_part_in_contact(gpu, hmodels, oracle_mod, omodels, name):
    """Maximum row count: the robot pushed into the plane so every capsule and sphere touches it
    (hexapod: 108 joint rows + 22 contacts x 3 = 174 of the 176-row layout), 5 steps vs the oracle."""
    import torch

    sb = make_batch(gpu, hmodels[name], name, 4)
    sb.body[:, :, 2] = 0.0  # every body centre on the plane: every capsule and sphere penetrates it
    body0 = sb.body.cpu().numpy()
    qt, dqt, tt = tables(sb)
    out = sb.step(5)
    torch.cuda.synchronize()
    body = sb.body.cpu().numpy()
    nc = out["n_contacts"].cpu().numpy()
    import xml.etree.ElementTree as ET

    bodies = ET.parse(os.path.join(MODELS, f"{name}.xml")).getroot().iter("body")
    ncoll = sum(1 for bd in bodies if bd.find("geom") is not None and bd.find("geom").get("type") in ("capsule", "sphere"))
    assert nc[:, 0].max() == ncoll
    P = oracle_mod.SimParams()
    for b in range(4):
        r = oracle_mod.sim_run(omodels[name], P, sb.n_t, qt[b], dqt[b], tt[b], body0[b], 0, 2, 5)
        assert (r["n_contacts"] == nc[b]).all()
        assert np.abs(r["body"] - body[b]).max() < 1e-9 * max(1.0, np.abs(r["body"]).max())


# ---- single precision (HS_PREC_F32, BASELINE configs[2] "fp32"): same algorithm in float.
# Floats cannot follow the double trajectories bit for bit, so these check the reset against
# the oracle to float rounding, closed-form physics, the fp32 path's own determinism, and that
# its trajectories stay near the fp64 ones over configs[2]'s 32-step horizon.

@pytest.mark.parametrize("name", ["hexapod", "spider", "myant"])
def test_f32_reset_matches_oracle(gpu, hmodels, oracle_mod, omodels, name):
    import torch

    sb = make_batch(gpu, hmodels[name], name, 8, dtype=torch.float32)
    assert sb.body.dtype == torch.float32
    body = sb.body.cpu().numpy().astype(np.float64)
    qt = sb.tables.q.cpu().numpy().astype(np.float64)
    for b in range(8):
        ob = oracle_mod.sim_reset(omodels[name], qt[b, sb.table_row(2)])
        assert np.abs(ob - body[b]).max() < 1e-5 * max(1.0, np.abs(ob).max())


def test_f32_free_fall(gpu, hmodels):
    import torch

    sb = make_batch(gpu, hmodels["hexapod"], "hexapod", 16, k=0.0, dtype=torch.float32)
    sb.body[:, :, 2] += 10.0
    n = 40
    out = sb.step(n)
    torch.cuda.synchronize()
    b = sb.body.cpu().numpy().astype(np.float64)
    # the joints are internal forces: the mean body velocity (all masses 1) falls freely to float
    # rounding; single bodies carry the ERP corrections of float-sized joint drift (~1e-4)
    assert np.abs(b[:, :, 9].mean(axis=1) + n * 0.01).max() < 1e-5
    assert np.abs(b[:, :, 9] + n * 0.01).max() < 1e-3
    assert (out["n_contacts"].cpu().numpy() == 0).all()


def test_f32_launch_split_is_bitwise(gpu, hmodels):
    import torch

    a = make_batch(gpu, hmodels["spider"], "spider", 64, dtype=torch.float32)
    b = make_batch(gpu, hmodels["spider"], "spider", 64, dtype=torch.float32)
    oa = a.step(30)
    parts = [b.step(10) for _ in range(3)]
    torch.cuda.synchronize()
    assert torch.equal(a.body, b.body) and torch.equal(a.seed, b.seed) and torch.equal(a.tsi, b.tsi)
    assert torch.equal(oa["tau_cmd"], torch.cat([p["tau_cmd"] for p in parts], dim=1))


@pytest.mark.parametrize("name", ["hexapod", "spider", "myant"])
def test_f32_follows_f64_over_horizon(gpu, hmodels, name):
    """configs[2]'s horizon (32 steps): fp32 torsos within 1e-2 of the fp64 ones (median 5e-4),
    joint angles within 5e-2, the mean normal force within 1 % (median). Measured on MI355X
    (tools/sim_f32_check.py, 256 rollouts): torso median 3e-5..1.1e-4, max 1.4e-3..2.4e-3;
    angles max 3e-3..7e-3; force median 1.5e-4..3.8e-4; 6-8 % of contact counts differ (contacts
    made or broken a step apart at depth ~0)."""
    import torch
    from hslabs_amd import synth

    p = synth.gen_sim_params(256, name)
    a = gpu.SimBatch(hmodels[name], p, dtype=torch.float64)
    b = gpu.SimBatch(hmodels[name], p, dtype=torch.float32)
    outs = ("torso", "q_meas", "normal_force")
    oa, ob = a.step(32, outputs=outs), b.step(32, outputs=outs)
    torch.cuda.synchronize()
    assert torch.isfinite(b.body).all()
    dt = (oa["torso"] - ob["torso"].double()).abs().amax(dim=(1, 2)).cpu().numpy()
    assert np.median(dt) < 5e-4 and dt.max() < 1e-2
    dq = oa["q_meas"] - ob["q_meas"].double()
    dq = ((dq + np.pi) % (2 * np.pi) - np.pi).abs().max().item()
    assert dq < 5e-2
    fa, fb = oa["normal_force"].mean(dim=1), ob["normal_force"].double().mean(dim=1)
    assert np.median(((fa - fb).abs() / fa.abs().clamp(min=1)).cpu().numpy()) < 1e-2


def test_f32_full_batch_one_period(gpu, hmodels):
    """4096 hexapods in fp32 over one gait period: the physics of the fp64 test holds."""
    import torch

    sb = make_batch(gpu, hmodels["hexapod"], "hexapod", 4096, dtype=torch.float32)
    z0 = sb.body[:, 0, 2].clone()
    out = sb.step(300, outputs=("torso", "normal_force", "n_contacts"))
    torch.cuda.synchronize()
    assert torch.isfinite(sb.body).all()
    z = out["torso"][:, :, 2].cpu().numpy()
    assert (z > 0).all()
    assert np.median(np.abs(z[:, -1] - z0.cpu().numpy())) < 0.1
    fn = out["normal_force"].cpu().numpy()[:, 100:]
    assert abs(np.median(fn.mean(axis=1)) - 22.0) < 0.25 * 22.0


def test_f32_configs2_shape(gpu, hmodels):
    """BASELINE configs[2] shape: 16384 spiders x 32 steps in one launch, finite and on the ground."""
    import torch

    sb = make_batch(gpu, hmodels["spider"], "spider", 16384, dtype=torch.float32)
    out = sb.step(32, outputs=("torso", "n_contacts"))
    torch.cuda.synchronize()
    assert torch.isfinite(sb.body).all()
    assert (out["torso"][:, :, 2] > 0).all()
    assert (out["n_contacts"][:, -1] > 0).float().mean().item() > 0.99


def test_f32_occupancy_builds_agree(gpu, hmodels):
    """A 16384-spider fp32 batch runs the 3-waves/SIMD build of the kernel (more rollouts per CU),
    a small one the default build: the same rollouts come out bit for bit."""
    import torch
    from hslabs_amd import synth

    params = synth.gen_sim_params(16384, "spider")
    big = gpu.SimBatch(hmodels["spider"], params, dtype=torch.float32)
    big.step(32, outputs=())
    idx = [0, 5000, 16383]
    small = gpu.SimBatch(hmodels["spider"], params[idx], dtype=torch.float32)
    small.step(32, outputs=())
    torch.cuda.synchronize()
    for k, i in enumerate(idx):
        assert torch.equal(small.body[k], big.body[i])
        assert small.seed[k].item() == big.seed[i].item()
