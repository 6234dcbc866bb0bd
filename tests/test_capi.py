"""C-ABI boundary (CPU): the library loads, exports every symbol of include/hslabs.h,
loads models / configs like the reference, reports errors instead of exit(1).
No compute calls here (no GPU in this container)."""
import ctypes
import os
import re
import shutil

import numpy as np
import pytest

from conftest import MODELS, PGS_CONFIG, ROOT


def header_functions():
    src = open(os.path.join(ROOT, "include", "hslabs.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hs_[a-z_0-9]+)\s*\(", src)))


def test_exports_every_declared_symbol(product):
    L = product.capi.load()
    declared = header_functions()
    assert declared, "no functions parsed from include/hslabs.h"
    for name in declared:
        assert hasattr(L, name), f"missing export {name}"
    assert sorted(product.capi.EXPORTS) == declared
    assert L.hs_abi_version() == product.capi.ABI_VERSION


def test_library_is_gfx950(product):
    data = open(product.capi.lib_path(), "rb").read()
    assert b"gfx950" in data


@pytest.mark.parametrize("name,n,nmj,nf,cfg", [("hexapod", 22, 18, 6, 24), ("spider", 19, 18, 6, 24),
                                               ("myant", 17, 12, 4, 18)])
def test_model_dims(product, omodels, name, n, nmj, nf, cfg):
    m = product.KinematicModel(os.path.join(MODELS, f"{name}.xml"))
    assert (m.n_parts, m.nmj, m.nfeet, m.config_dim) == (n, nmj, nf, cfg)
    assert m.total_mass == float(n)  # dBodyCreate default mass 1 per part
    assert m.rcap == 0.08
    o = omodels[name]
    assert (o.n, o.nmj, o.nf, o.cfg) == (n, nmj, nf, cfg)


def test_torso_penalty_setting(product):
    """periodic::switch_torso_penalty (ftsolver.cpp:262-273): (1,1) by default (player.cpp:263), any
    mask with at least one torso group, (0,0) refused where the reference exits (ftsolver.cpp:245)"""
    m = product.KinematicModel(os.path.join(MODELS, "hexapod.xml"))
    assert m.torso_penalty() == (True, True)
    m.switch_torso_penalty(True, False)
    assert m.torso_penalty() == (True, False)
    m.switch_torso_penalty(False, True)
    assert m.torso_penalty() == (False, True)
    with pytest.raises(product.HSError, match="mask0 not set"):
        m.switch_torso_penalty(False, False)
    assert m.torso_penalty() == (False, True)  # unchanged by the refused call
    per = product.Periodic(m)
    per.switch_torso_penalty(True, True)
    assert m.torso_penalty() == (True, True)


def test_model_errors(product, tmp_path):
    with pytest.raises(product.HSError, match="cannot open"):
        product.KinematicModel(str(tmp_path / "nope.xml"))
    bad = tmp_path / "hexapod.xml"
    bad.write_text("<mujoco><worldbody><body pos='0 0 1'>")
    with pytest.raises(product.HSError):
        product.KinematicModel(str(bad))
    # lik.cpp:9-11 keys the IK solver on the file name
    renamed = tmp_path / "robot.xml"
    shutil.copy(os.path.join(MODELS, "hexapod.xml"), renamed)
    with pytest.raises(product.HSError, match="no limb IK solver"):
        product.KinematicModel(str(renamed))
    m = product.KinematicModel(str(renamed), lik_variant=1)  # explicit variant
    assert m.n_parts == 22


def test_pgs_config_matches_oracle_parser(product, oracle_mod):
    for sid in range(33):
        p = product.read_pgs_config(PGS_CONFIG, sid)
        o = oracle_mod.load_pgs_config(PGS_CONFIG, sid)
        assert p.fname == o.xml_file
        assert p.torso_pos == pytest.approx(o.torso_pos) and p.torso_angles == pytest.approx(o.torso_angles)
        assert (p.step_duration, p.period, p.step_length, p.step_height, p.curvature) == \
            (o.step_duration, o.period, o.step_length, o.step_height, o.curvature)
        assert p.foot_shift == (o.foot_shift_type, o.foot_shift)
    with pytest.raises(product.HSError, match="no string with rec_id"):
        product.read_pgs_config(PGS_CONFIG, 99)


def test_best_key_encoding_orders_like_cot(product):
    L = product.capi.load()
    cots = [-3.5, -1e-3, -0.0, 0.0, 1e-30, 0.25, 0.5917, 3.0, float("inf"), float("nan")]
    keys = [L.hs_best_key_encode(c, i) for i, c in enumerate(cots)]
    assert keys == sorted(keys)
    for i, c in enumerate(cots):
        cot, rid = product.decode_best_key(keys[i])
        assert rid == i
        if np.isnan(c):
            assert np.isnan(cot)
        else:
            assert cot == np.float32(c)


def test_torch_key_matches_c_encoding(product):
    import torch

    from hslabs_amd import dist as hdist

    L = product.capi.load()
    cot = torch.tensor([0.7, -2.0, 0.3, float("nan"), 0.3], dtype=torch.float64)
    key = hdist.best_key(cot, 1000)
    c, rid = hdist.decode(key)
    assert rid == 1001 and c == np.float32(-2.0)
    u = (int(key.item()) ^ (-(2 ** 63))) & 0xFFFFFFFFFFFFFFFF
    assert u == L.hs_best_key_encode(-2.0, 1001)


def test_selection_cot_is_per_cycle_with_abs_step_length(product):
    """hs_best_key_cot (include/hslabs.h) and its torch twin (dist.select_cot) agree bitwise:
    one cycle's work over sum m * |L|, NaN for gaits under 1e-3 of travel per cycle."""
    import torch

    from hslabs_amd import dist as hdist

    L = product.capi.load()
    assert L.hs_best_key_cot(2.0, 22.0, 0.5, 20, 20) == 2.0 / (22.0 * 0.5)
    assert L.hs_best_key_cot(2.0, 22.0, -0.5, 20, 20) == 2.0 / (22.0 * 0.5)
    assert L.hs_best_key_cot(20.0, 22.0, 0.5, 20, 200) == 20.0 * (20 / 200) / (22.0 * 0.5)
    assert np.isnan(L.hs_best_key_cot(2.0, 22.0, 0.0009, 20, 20))
    assert np.isnan(L.hs_best_key_cot(2.0, 22.0, -0.0009, 20, 20))
    rng = np.random.default_rng(3)
    work = rng.uniform(0, 50, 64)
    sl = rng.uniform(-0.5, 0.5, 64)
    for steps in (1, 20, 37, 200):
        got = hdist.select_cot(torch.from_numpy(work), torch.from_numpy(sl), 22.0, 20, steps).numpy()
        want = np.array([L.hs_best_key_cot(w, 22.0, s, 20, steps) for w, s in zip(work, sl)])
        assert np.array_equal(got, want, equal_nan=True)
        got32 = hdist.select_cot(torch.from_numpy(work.astype(np.float32)), torch.from_numpy(sl), 22.0, 20, steps)
        assert got32.dtype == torch.float32


def test_run_argument_validation(product):
    L = product.capi.load()
    m = product.KinematicModel(os.path.join(MODELS, "hexapod.xml"))
    a = product.capi.RunArgsC()
    a.n_rollouts, a.horizon, a.n_t = 4, 0, 20
    assert L.hs_run(m.handle, ctypes.byref(a)) == -1  # horizon < 1
    a.horizon, a.k0 = 1, -1
    assert L.hs_run(m.handle, ctypes.byref(a)) == -1
    a.k0, a.params = 0, None
    assert L.hs_run(m.handle, ctypes.byref(a)) == -1  # params null
    assert b"params" in L.hs_last_error()
    a.n_rollouts = 0
    assert L.hs_run(m.handle, ctypes.byref(a)) == 0  # empty batch is a no-op
    assert L.hs_run(None, ctypes.byref(a)) == -1


def test_gait_record_layout(product):
    from hslabs_amd import GAIT_DTYPE, PgsConfigParams

    assert GAIT_DTYPE.itemsize == 192 == ctypes.sizeof(product.capi.GaitParamsC)
    p = PgsConfigParams(torso_pos=(1, 2, 3), torso_angles=(4, 5, 6), step_duration=0.5, period=7, step_length=8,
                        step_height=9, curvature=10, foot_shift=(1, 11))
    rec = p.to_record()
    c = product.capi.GaitParamsC.from_buffer_copy(rec.tobytes())
    assert list(c.torso_pos) == [1, 2, 3] and list(c.torso_angles) == [4, 5, 6]
    assert (c.step_duration, c.period, c.step_length, c.step_height, c.curvature, c.foot_shift,
            c.foot_shift_type) == (0.5, 7, 8, 9, 10, 11, 1)
    assert PgsConfigParams.from_record(rec) == p
    assert c.rec_transform_flag == 0
    p.set_rec_rotation((0, 0, -1.571))  # main.cpp:38
    p.set_rec_transform((0.5, -0.25, 0.0), (0.1, 0.2, 0.3))
    c = product.capi.GaitParamsC.from_buffer_copy(p.to_record().tobytes())
    assert c.rec_transform_flag == 1 and list(c.rec_transl) == [0.5, -0.25, 0.0]
    assert list(c.rec_eas) == [0.1, 0.2, 0.3]
    assert PgsConfigParams.from_record(p.to_record()) == p


def test_sweep_values_follow_pgssweeper(product):
    # pergen.cpp:417-449: n_val+1 values val0 + vali*(val1-val0)/n_val
    sw = product.ModelPlayer.sweep_params(product.PgsConfigParams(), "period", 3, 18, 15)
    vals = [v for v, _ in sw]
    assert len(vals) == 16 and vals[0] == 3 and vals[-1] == 18
    assert all(p.period == v for v, p in sw)
    with pytest.raises(product.HSError):
        product.ModelPlayer.sweep_params(product.PgsConfigParams(), "curvature", 0, 1, 2)


def test_synthetic_params_reproducible_and_in_range(product):
    from hslabs_amd import synth

    a = synth.gen_params(1000, "hexapod")
    b = synth.gen_params(500, "hexapod", id0=500)
    assert a[500:].tobytes() == b.tobytes()  # counter-based: shards regenerate identically
    assert (a["period"] >= 3).all() and (a["period"] < 18).all()
    assert (np.abs(a["step_length"]) <= 0.5).all()
    assert (a["step_duration"] >= 0).all() and (a["step_duration"] <= 1).all()
    assert (a["torso_pos"][:, 2] >= -0.47).all() and (a["torso_pos"][:, 2] < -0.05).all()
    assert (a["foot_shift_type"] == -1).all() and (a["curvature"] == 0).all()
    c = synth.gen_params(100, "hexapod", curved=True)
    assert (c["curvature"] >= -0.15).all() and (c["curvature"] < 0.5).all()


def test_shard_ranges_cover_batch():
    from hslabs_amd import dist as hdist

    for n, w in [(262144, 8), (10, 3), (5, 8)]:
        ranges = [hdist.shard(n, w, r) for r in range(w)]
        assert sum(c for _, c in ranges) == n
        ids = [i for s, c in ranges for i in range(s, s + c)]
        assert ids == list(range(n))


def test_mixed_plan_argument_validation(product):
    """hs_mixed_create checks its host-side arguments before touching a device."""
    L = product.capi.load()
    ms = [product.KinematicModel(os.path.join(MODELS, f"{n}.xml")) for n in ("myant", "hexapod")]
    hs = (ctypes.c_void_p * 2)(*[m.handle for m in ms])
    plan = ctypes.c_void_p()
    idx = np.array([0, 1, 2, 1], dtype=np.int32)  # 2 is out of range
    p32 = ctypes.POINTER(ctypes.c_int32)
    assert L.hs_mixed_create(hs, 2, idx.ctypes.data_as(p32), 4, ctypes.byref(plan)) == -1
    assert b"model_index" in L.hs_last_error()
    assert L.hs_mixed_create(hs, 0, idx.ctypes.data_as(p32), 4, ctypes.byref(plan)) == -1
    assert L.hs_mixed_create(None, 2, idx.ctypes.data_as(p32), 4, ctypes.byref(plan)) == -1
    assert L.hs_run_mixed(None, None) == -1
    assert L.hs_mixed_get_dims(None, None) == -1
    L.hs_mixed_free(None)  # no-op


def test_mixed_synthetic_batch_layout(product):
    from hslabs_amd import synth

    p, idx = synth.gen_mixed(64, id0=10)
    assert (idx == (np.arange(10, 74) % 2)).all() and idx.mean() == 0.5
    a = synth.gen_params(64, "myant", id0=10)
    h = synth.gen_params(64, "hexapod", id0=10)
    assert (p[idx == 0] == a[idx == 0]).all() and (p[idx == 1] == h[idx == 1]).all()


def test_traj_save_format(product, tmp_path):
    """save_2d_array (core.cpp:46-61): space-separated rows, default ostream formatting
    (6 significant digits, %g), append mode for sweeps."""
    rec = np.array([[0.1, -2.5e-7, 123456789.0, 0.0], [-0.0, 1.0 / 3.0, 1e-5, 42.0]])
    path = str(tmp_path / "traj.txt")
    product.save_2d_array(path, rec)
    product.save_2d_array(path, rec[:1], append=True)
    lines = open(path).read().splitlines()
    want = [" ".join("%g" % v for v in row) for row in rec] + [" ".join("%g" % v for v in rec[0])]
    assert lines == want
    assert lines[0] == "0.1 -2.5e-07 1.23457e+08 0"


def test_batch_handle_without_device_fails_loudly(product):
    """hs_batch_create reports an error code and message (no GPU in this container), never
    a CPU fallback; invalid arguments are rejected before any device call."""
    import ctypes

    L = product.capi.load()
    m = product.KinematicModel(os.path.join(MODELS, "hexapod.xml"))
    h = ctypes.c_void_p()
    assert L.hs_batch_create(m.handle, 0, 1, 20, 0, 1, ctypes.byref(h)) != 0
    assert b"empty batch" in L.hs_last_error()
    assert L.hs_batch_create(m.handle, 16, 1, 20, 9, 1, ctypes.byref(h)) != 0
    rc = L.hs_batch_create(m.handle, 16, 1, 20, 0, 1, ctypes.byref(h))
    if rc == 0:  # a GPU is present after all
        L.hs_batch_free(h)
    else:
        assert h.value is None and L.hs_last_error()
    c, i = ctypes.c_float(), ctypes.c_int64()
    assert L.hs_select_best(None, ctypes.byref(c), ctypes.byref(i)) != 0
    assert L.hs_batch_best_key_device(None, 0) is None
