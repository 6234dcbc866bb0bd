"""switch_torso_penalty(force, torque) other than the reference's (1,1) (ftsolver.cpp:262-273, through
periodic.cpp:205-207; main.cpp:87 passes (1, 0+1)) on the GPU, against the oracle with the same mask.

mask0 holds the chosen torso rows, mask1 the rest in row order (set_penal_mask1, ftsolver.cpp:291-303),
so the torso rows left out of mask0 join the first-order stage with weight 1 ahead of the joint torque
rows and couple every pair of contacts. The kernel routes every step of such a model through its
Eigen-style path (the closed form is the (1,1) problem's), whose first-order Gram gains those rows.
The oracle's masks are pinned on CPU by the independent scipy formulation
(tests/test_oracle.py::test_torso_penalty_masks). Tolerances are test_gpu_parity.py's.
"""
import os

import numpy as np
import pytest

from conftest import MODELS, PGS_CONFIG, PGS_IDS, record_to_oracle_gait, to_oracle_gait
from test_gpu_parity import GEN, as_batch, compare, fused_cycle, npy, threads

pytestmark = pytest.mark.gpu

MASKS = [(True, False), (False, True)]


@pytest.fixture(scope="module")
def gpu(product):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return product


def masked_models(gpu, oracle_mod, name, force, torque):
    """fresh models (the setting persists on a model, so never the shared fixtures)"""
    path = os.path.join(MODELS, f"{name}.xml")
    hm = gpu.KinematicModel(path)
    hm.switch_torso_penalty(force, torque)
    om = oracle_mod.Model(path)
    om.switch_torso_penalty(force, torque)
    return hm, om


@pytest.mark.parametrize("force,torque", MASKS)
@pytest.mark.parametrize("sid", PGS_IDS)
def test_pgs_setups(gpu, oracle_mod, sid, force, torque):
    import torch

    p = gpu.read_pgs_config(PGS_CONFIG, sid)
    name = p.fname.replace(".xml", "")
    hm, om = masked_models(gpu, oracle_mod, name, force, torque)
    b = gpu.DeviceBatch(hm, [p], n_t=20, k0=0, horizon=20, outputs=("tau", "cf", "flags", "work_cot"))
    b.run(best=False)
    torch.cuda.synchronize()
    og = to_oracle_gait(oracle_mod, p)
    r = as_batch(oracle_mod.rollout(om, og, 20, basis=oracle_mod.BASIS_TREE))
    g = {k: npy(getattr(b, k)) for k in ("tau", "cf", "flags", "work_cot")}
    g["flags"] = g["flags"].astype(np.uint32)
    assert ((g["flags"] & GEN) != 0).all(), "every step of a masked model takes the Eigen-style path"
    compare(f"pgs {sid} torso penalty ({force:d},{torque:d})", g, r, oracle_mod, om, [og], oracle_mod.BASIS_TREE,
            min_work=1.0)


@pytest.mark.parametrize("force,torque", MASKS)
@pytest.mark.parametrize("name,curved", [("hexapod", False), ("hexapod", True), ("myant", False)])
def test_synthetic(gpu, oracle_mod, name, curved, force, torque):
    """256 rollouts x one cycle through the fused path (hs_run_calls: every step deferred by the step
    launch, solved by the fixup launch), against the oracle and bitwise against one launch per call"""
    import torch

    from hslabs_amd import synth

    hm, om = masked_models(gpu, oracle_mod, name, force, torque)
    params = synth.gen_params(256, name, id0=4242, curved=curved)
    g = fused_cycle(gpu, hm, params)
    gaits = [record_to_oracle_gait(oracle_mod, r) for r in params]
    r = oracle_mod.batch(om, gaits, 20, 0, 20, basis=oracle_mod.BASIS_TREE, n_threads=threads())
    assert ((g["flags"] & GEN) != 0).all()
    compare(f"{name} torso penalty ({force:d},{torque:d})", g, r, oracle_mod, om, gaits, oracle_mod.BASIS_TREE,
            min_work=0.95)
    seq = gpu.DeviceBatch(hm, params, n_t=20, k0=0, horizon=20, outputs=("tau", "cf", "flags"))
    seq.run(best=False)
    torch.cuda.synchronize()
    assert np.array_equal(npy(seq.tau), g["tau"]) and np.array_equal(npy(seq.cf), g["cf"])


def test_switching_back_restores_the_closed_form(gpu, oracle_mod):
    """(1,0), then (1,1) again on the same model (its device copy updated between calls): the
    results equal a fresh model's bitwise, closed form included; the masked call differed"""
    import torch

    from hslabs_amd import synth

    params = synth.gen_params(128, "hexapod", id0=99)
    fresh = gpu.KinematicModel(os.path.join(MODELS, "hexapod.xml"))
    ref = fused_cycle(gpu, fresh, params)
    m = gpu.KinematicModel(os.path.join(MODELS, "hexapod.xml"))
    base = fused_cycle(gpu, m, params)  # uploads the model's device copy with (1,1)
    m.switch_torso_penalty(True, False)
    masked = fused_cycle(gpu, m, params)
    m.switch_torso_penalty(True, True)
    back = fused_cycle(gpu, m, params)
    torch.cuda.synchronize()
    for k in ("tau", "cf", "flags", "work_cot"):
        assert np.array_equal(base[k], ref[k]) and np.array_equal(back[k], ref[k]), k
    assert not (back["flags"] & GEN).any()
    assert np.abs(masked["tau"] - ref["tau"]).max() > 1e-6


def test_shim_measure_cot_uses_11(gpu, oracle_mod):
    """modelplayer::measure_cot solves with its own periodic's switch_torso_penalty(1,1)
    (player.cpp:259-285): a masked model still measures the (1,1) COT, and keeps its mask"""
    p = gpu.read_pgs_config(PGS_CONFIG, 8)
    m = gpu.KinematicModel(os.path.join(MODELS, "hexapod.xml"))
    player = gpu.ModelPlayer(m)
    cot11 = player.measure_cot(p, 20)
    m.switch_torso_penalty(False, True)
    assert player.measure_cot(p, 20) == cot11
    assert m.torso_penalty() == (False, True)
    r = oracle_mod.rollout(oracle_mod.Model(os.path.join(MODELS, "hexapod.xml")), to_oracle_gait(oracle_mod, p), 20)
    assert cot11 == pytest.approx(r["cot"], rel=1e-9)
