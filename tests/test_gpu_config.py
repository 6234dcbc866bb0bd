"""GPU parity of the per-configuration kinematics (the model.h / pergen.h entry points outside
periodic): hs_pergen_rec (pergensetup::set_rec, pergen.cpp:225-239), hs_model_lik
(kinematicmodel::set_jvalues_with_lik, model.cpp:354-359 + lik.cpp:89-99, 316-347) and
hs_model_fk (recompute_modelnodes, model.cpp:183-201, 314-318), against the oracle's restatement
of the same functions. hs_config.hip is built without FMA contraction, so the only differences
are ULPs of the device sin / cos / atan2 / acos: the bound is 1e-12 absolute on records, angles
and transforms of unit-scale models."""
import os

import numpy as np
import pytest

from conftest import MODELS, PGS_CONFIG, PGS_IDS, record_to_oracle_gait, to_oracle_gait

pytestmark = pytest.mark.gpu

TOL = 1e-12
TIMES = (0.0, 0.37, 1.25, 2.9, 4.4)


@pytest.fixture(scope="module")
def gpu(product):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return product


@pytest.fixture(scope="module")
def pmodels(gpu):
    return {n: gpu.KinematicModel(os.path.join(MODELS, f"{n}.xml")) for n in ("hexapod", "spider", "myant")}


def _setups(gpu):
    for i in PGS_IDS:
        p = gpu.read_pgs_config(PGS_CONFIG, i)
        yield i, p, p.fname.split(".")[0]


def test_pergen_rec_all_setups(gpu, pmodels, omodels, oracle_mod):
    O = oracle_mod
    for i, p, name in _setups(gpu):
        rec = pmodels[name].pergen_rec([p], TIMES)[0]
        for k, t in enumerate(TIMES):
            ref = O.pergen_rec(omodels[name], to_oracle_gait(O, p), t)
            assert np.abs(rec[k] - ref).max() < TOL, (i, t)


def test_pergen_rec_synthetic_batches(gpu, pmodels, omodels, oracle_mod):
    from hslabs_amd import synth

    O = oracle_mod
    rng = np.random.default_rng(5)
    for name in ("hexapod", "spider", "myant"):
        params = synth.gen_params(96, name, curved=True)
        times = rng.uniform(0, 6, 7)
        rec = pmodels[name].pergen_rec(params, times)
        assert rec.shape == (96, 7, 6 + 3 * pmodels[name].n_limbs)
        for b in range(0, 96, 7):
            g = record_to_oracle_gait(O, params[b])
            for k, t in enumerate(times):
                assert np.abs(rec[b, k] - O.pergen_rec(omodels[name], g, t)).max() < TOL, (name, b, t)


def test_lik_matches_oracle(gpu, pmodels, omodels, oracle_mod):
    """set_jvalues_with_lik on every pgs setup's records (ignore_reach as main.cpp:41 sets it)."""
    O = oracle_mod
    for i, p, name in _setups(gpu):
        m, om = pmodels[name], omodels[name]
        recs = np.stack([O.pergen_rec(om, to_oracle_gait(O, p), t) for t in TIMES])
        q, st = m.set_jvalues_with_lik(recs, ignore_reach=True)
        for k in range(len(TIMES)):
            qr, ok, unreach = O.set_jvalues_with_lik(om, recs[k], ignore_reach=True)
            assert ok
            assert np.abs(q[k] - qr).max() < TOL, (i, TIMES[k])
            assert bool(st[k] & gpu.capi.HS_FLAG_UNREACH) == unreach, (i, TIMES[k])


def test_lik_keeps_other_joint_values_and_reach(gpu, pmodels, omodels, oracle_mod):
    """Out-of-reach targets: clamped with ignore_reach (HS_FLAG_UNREACH + the limb's bit, the
    oracle's clamped angles), an error without it (the reference exits, lik.cpp:321-330)."""
    O = oracle_mod
    m, om = pmodels["hexapod"], omodels["hexapod"]
    p = gpu.read_pgs_config(PGS_CONFIG, 8)
    rec = O.pergen_rec(om, to_oracle_gait(O, p), 0.5)
    far = rec.copy()
    far[6 + 3 * 2 + 2] -= 5.0  # limb 2's foot 5 m below its hip
    q, st = m.set_jvalues_with_lik(far[None], ignore_reach=True)
    qr, ok, unreach = O.set_jvalues_with_lik(om, far, ignore_reach=True)
    assert ok and unreach
    assert st[0] & gpu.capi.HS_FLAG_UNREACH and st[0] & (1 << (16 + 2))
    assert not st[0] & (1 << (16 + 1))
    assert np.abs(q[0] - qr).max() < TOL
    with pytest.raises(gpu.capi.HSError, match="out of reach"):
        m.set_jvalues_with_lik(far[None], ignore_reach=False)
    _, ok, _ = O.set_jvalues_with_lik(om, far, ignore_reach=False)
    assert not ok


def test_fk_matches_oracle(gpu, pmodels, omodels, oracle_mod):
    """recompute_modelnodes on random configurations: every node's A_ground and its joint's."""
    O = oracle_mod
    rng = np.random.default_rng(11)
    for name, m in pmodels.items():
        om = omodels[name]
        q = rng.uniform(-np.pi, np.pi, (64, m.config_dim))
        q[:, :3] = rng.uniform(-1, 1, (64, 3))
        ag, aj = m.recompute_modelnodes(q, joints=True)
        assert ag.shape == (64, m.n_parts, 3, 4)
        for b in range(64):
            rg, rj = O.recompute_modelnodes(om, q[b])
            assert np.abs(ag[b] - rg).max() < TOL, (name, b)
            assert np.abs(aj[b] - rj).max() < TOL, (name, b)


def test_fk_after_ik_puts_feet_on_targets(gpu, pmodels, omodels, oracle_mod):
    """hso_fk_ik_check (the reference's FK-after-IK consistency) through the product: set_rec ->
    set_jvalues_with_lik -> recompute_modelnodes, feet = A_ground(foot) * capsule end."""
    O = oracle_mod
    for i, p, name in _setups(gpu):
        m = pmodels[name]
        nodes = [m.get_mnode(v) for v in range(m.n_parts)]
        feet = {nd["foot"]: (v, nd["foot_pos"]) for v, nd in enumerate(nodes) if nd["foot"] >= 0}
        limb_foot = []
        for v, nd in enumerate(nodes):  # lik.cpp:364-366: child -> first -> first
            if nd["limb"] >= 0:
                f = nodes[nodes[v]["kids"][0]]["kids"][0]
                limb_foot.append((nd["limb"], f, nodes[f]["foot_pos"]))
        assert len(limb_foot) == m.n_limbs and len(feet) == m.nfeet
        rec = m.pergen_rec([p], TIMES)[0]
        q, _ = m.set_jvalues_with_lik(rec, ignore_reach=True)
        ag = m.recompute_modelnodes(q)
        for k, t in enumerate(TIMES):
            worst = 0.0
            for L, f, fp in limb_foot:
                g = ag[k, f, :, :3] @ fp + ag[k, f, :, 3]
                worst = max(worst, np.abs(g - rec[k, 6 + 3 * L:9 + 3 * L]).max())
            ref = O.fk_ik_check(omodels[name], to_oracle_gait(O, p), t)
            assert ref < 1e-12 and worst < 1e-12, (i, t, worst, ref)


def test_device_batches_agree_with_host_forms(gpu, pmodels):
    """The DEVICE forms on 65536 configurations (async on a torch stream) equal the host forms."""
    import ctypes

    import torch

    from hslabs_amd import synth

    m = pmodels["hexapod"]
    L = gpu.capi.load()
    params = synth.gen_params(8192, "hexapod", curved=True)
    times = np.linspace(0.0, 3.0, 8)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    P = torch.from_numpy(params.view(np.uint8).copy()).to(dev)
    T = torch.from_numpy(times).to(dev)
    R = torch.zeros((8192, 8, 6 + 3 * m.n_limbs), dtype=torch.float64, device=dev)
    n = 8192 * 8
    Q = torch.zeros((n, m.config_dim), dtype=torch.float64, device=dev)
    S = torch.zeros(n, dtype=torch.int32, device=dev)
    A = torch.zeros((n, m.n_parts, 12), dtype=torch.float64, device=dev)
    vp = ctypes.c_void_p
    sp = vp(stream.cuda_stream)
    gpu.capi.check(L.hs_pergen_rec(m.handle, vp(P.data_ptr()), 8192, vp(T.data_ptr()), 8, vp(R.data_ptr()), sp), "rec")
    gpu.capi.check(L.hs_model_lik(m.handle, n, vp(R.data_ptr()), 1, vp(Q.data_ptr()), vp(S.data_ptr()), sp), "lik")
    gpu.capi.check(L.hs_model_fk(m.handle, n, vp(Q.data_ptr()), m.config_dim, vp(A.data_ptr()), None, sp), "fk")
    torch.cuda.synchronize()
    sel = np.arange(0, 8192, 257)
    rec_h = m.pergen_rec(params[sel], times)
    assert np.array_equal(R.cpu().numpy()[sel], rec_h)
    q_h, _ = m.set_jvalues_with_lik(rec_h.reshape(-1, rec_h.shape[-1]), ignore_reach=True)
    qd = Q.cpu().numpy().reshape(8192, 8, -1)[sel].reshape(-1, m.config_dim)
    assert np.array_equal(qd, q_h)
    a_h = m.recompute_modelnodes(q_h)
    ad = A.cpu().numpy().reshape(8192, 8, m.n_parts, 4, 3).transpose(0, 1, 2, 4, 3)[sel].reshape(a_h.shape)
    assert np.array_equal(ad, a_h)


def test_lik_matches_the_rollout_kernel_configurations(gpu, pmodels):
    """hs_run's q output (the configuration of every solved sample: record_trajectory's
    set_jvalues_with_lik + get_jvalues, periodic.cpp:85-96) against hs_pergen_rec + hs_model_lik at
    the same sample times (t accumulated by += dt like periodic.cpp:171-181). The rollout kernel
    contracts a*b+c into FMAs, so the two agree to rounding, not bitwise."""
    from hslabs_amd import synth

    m = pmodels["hexapod"]
    params = synth.gen_params(64, "hexapod", curved=True)
    out = gpu.run_host(m, params, n_t=20, k0=0, horizon=20, want=("q",))
    for b in range(0, 64, 9):
        dt = params[b]["period"] / 20
        t, times = 0.0, []
        for i in range(22):
            times.append(t)
            t += dt
        rec = m.pergen_rec(params[b:b + 1], times[2:])[0]
        q, _ = m.set_jvalues_with_lik(rec, ignore_reach=True)
        assert np.abs(q - out["q"][b]).max() < 1e-11, b
