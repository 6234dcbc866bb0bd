"""The C++ shim (include/hslabs.hpp) keeps the reference's call shapes: a main.cpp-like
program compiles with plain g++ against libhslabs.so (CPU) and runs on the GPU."""
import os
import subprocess

import numpy as np
import pytest

from conftest import MODELS, PGS_CONFIG, ROOT


def compile_prog(product, out, src="cot_sweep.cpp"):
    libdir = os.path.dirname(product.capi.lib_path())
    cmd = ["g++", "-O2", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", src), "-L", libdir, "-lhslabs",
           f"-Wl,-rpath,{libdir}", "-o", str(out)]
    subprocess.run(cmd, check=True)
    return out


def test_shim_compiles_and_links(product, tmp_path):
    exe = compile_prog(product, tmp_path / "cot_sweep")
    assert os.path.exists(exe)
    assert os.path.exists(compile_prog(product, tmp_path / "position_control", "position_control.cpp"))
    assert os.path.exists(compile_prog(product, tmp_path / "model_api", "model_api.cpp"))
    assert os.path.exists(compile_prog(product, tmp_path / "reference_callers", "reference_callers.cpp"))
    # the C header alone is valid C (no C++ or HIP types leak through the boundary)
    src = tmp_path / "c_only.c"
    src.write_text('#include "hslabs.h"\nint main(void){return hs_abi_version()==HSLABS_ABI_VERSION?0:1;}\n')
    libdir = os.path.dirname(product.capi.lib_path())
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-L",
                    libdir, "-lhslabs", f"-Wl,-rpath,{libdir}", "-o", str(tmp_path / "c_only")], check=True)
    assert subprocess.run([str(tmp_path / "c_only")]).returncode == 0


@pytest.mark.gpu
def test_shim_runs_reference_shaped_main(product, tmp_path):
    exe = compile_prog(product, tmp_path / "cot_sweep")
    traj = tmp_path / "traj.txt"
    out = subprocess.run([str(exe), MODELS, str(traj)], check=True, capture_output=True, text=True,
                         timeout=300).stdout
    s = float([ln for ln in out.splitlines() if ln.startswith("s = ")][0].split("=")[1])
    assert s < 1e-9  # test_dynamics: forces from the computed torques == computed forces
    rec = np.loadtxt(traj)
    assert rec.shape == (20, 2 * 24 + 18)
    lines = out.splitlines()
    cot = float(lines[0].split("=")[1])
    p = product.read_pgs_config(PGS_CONFIG, 8)
    m = product.KinematicModel(os.path.join(MODELS, "hexapod.xml"))
    ref = product.run_host(m, [p], n_t=20, horizon=20)
    assert cot == pytest.approx(ref["work_cot"][0, 1], rel=1e-14)
    sweep = [ln for ln in lines if ln.startswith("val =")]
    assert len(sweep) == 16
    work = float([ln for ln in lines if ln.startswith("work =")][0].split("=")[1])
    assert work == pytest.approx(ref["work_cot"][0, 0], rel=1e-14)
    tau0 = float([ln for ln in lines if ln.startswith("tau[2][0]")][0].split("=")[1])
    assert tau0 == pytest.approx(ref["tau"][0, 0, 0], rel=1e-12)
    assert "error ok" in out


@pytest.mark.gpu
def test_shim_position_control_walks(product, tmp_path):
    """setup_per_controller + 600 x simulate_ode through the shim: the hexapod of pgs id 8 walks two
    step lengths (2 x 0.5); the run equals the Python binding's (oracle parity: tests/test_gpu_sim.py)."""
    exe = compile_prog(product, tmp_path / "position_control", "position_control.cpp")
    out = subprocess.run([str(exe), MODELS], check=True, capture_output=True, text=True, timeout=300).stdout
    vals = {ln.split("=")[0].strip(): [float(v) for v in ln.split("=")[1].split()] for ln in out.splitlines()}
    t0, t1 = np.array(vals["torso0"]), np.array(vals["torso1"])
    assert vals["play_t"][0] == pytest.approx(6.0)
    assert abs((t1[0] - t0[0]) - 1.0) < 0.2
    assert vals["fallen"][0] == 0
    # the same run through the Python binding (same kernels, same tables): identical to print precision
    import torch

    p = product.read_pgs_config(PGS_CONFIG, 8)
    m = product.KinematicModel(os.path.join(MODELS, "hexapod.xml"))
    sb = product.SimBatch(m, [p], tsi0=0)
    out = sb.step(600, outputs=("torso",))
    torch.cuda.synchronize()
    assert np.abs(out["torso"][0, -1].cpu().numpy() - t1).max() < 2e-9


@pytest.mark.gpu
def test_shim_model_api(product, oracle_mod, omodels, tmp_path):
    """model.h / core.h through the shim (set_rec -> set_jvalues_with_lik -> get_jvalues ->
    recompute_modelnodes -> feet, orient_torso, get_limb_hip_pos, arrayops, str_to_val) reproduces
    the oracle's configurations and its FK-after-IK check to 1e-12."""
    from conftest import to_oracle_gait

    O = oracle_mod
    exe = compile_prog(product, tmp_path / "model_api", "model_api.cpp")
    ids = [0, 8, 10, 17, 24, 25]  # myant, hexapod, turned hexapod, myant, spider x2
    out = subprocess.run([str(exe), MODELS, PGS_CONFIG, *map(str, ids)], check=True, capture_output=True, text=True,
                         timeout=300).stdout
    rows = [ln.split() for ln in out.splitlines()]
    n_q = 0
    for r in rows:
        if r[0] == "q":
            i, t, q = int(r[1]), float(r[2]), np.array([float(v) for v in r[3:]])
            p = product.read_pgs_config(PGS_CONFIG, i)
            om = omodels[p.fname.split(".")[0]]
            rec = O.pergen_rec(om, to_oracle_gait(O, p), t)
            qr, ok, _ = O.set_jvalues_with_lik(om, rec, ignore_reach=True)
            assert ok and np.abs(q - qr).max() < 1e-12, (i, t)
            n_q += 1
        elif r[0] == "fkik":
            assert float(r[3]) < 1e-12, r
        elif r[0] == "zaxis":
            assert float(r[3]) < 1e-14, r
        elif r[0] == "jvalues":
            assert float(r[2]) == 0.0, r
        elif r[0] == "orient":
            assert np.allclose([float(v) for v in r[2:5]], [0.5, -0.25, 1.0], atol=1e-12), r
        elif r[0] == "feet":
            assert int(r[2]) in (4, 6), r
        elif r[0] == "unreach_throws":
            assert r[2] == "1", r
    assert n_q == 4 * len(ids)
    kv = {r[0]: r[1:] for r in rows}
    assert [float(v) for v in kv["str_to_val"]] == [1.5, -2.0, 0.3]
    assert np.allclose([float(v) for v in kv["modulus"]], [4 - 2 * np.pi, -4 + 2 * np.pi, 1.0], atol=1e-15)
    assert float(kv["dot"][0]) == pytest.approx(-0.2)


@pytest.mark.gpu
def test_shim_runs_the_reference_callers(product, oracle_mod, omodels, tmp_path):
    """tests/cpp/reference_callers.cpp: the reference's own bodies of measure_cot (player.cpp:269-285),
    measure_cot_sweep (311-321), set_position_control_torques + linear_feedback_control (393-432),
    record_per_traj[_sweep] (619-655), test_dynamics (playerexperim.cpp:95-121) and cpc.cpp:51-63's
    target-point loop, compiled against the shim, give the Python binding's numbers (the same
    kernels) and the oracle's COT."""
    from conftest import to_oracle_gait

    exe = compile_prog(product, tmp_path / "reference_callers", "reference_callers.cpp")
    out = subprocess.run([str(exe), MODELS], check=True, capture_output=True, text=True, timeout=300,
                         cwd=str(tmp_path)).stdout
    lines = out.splitlines()
    rows = {}
    for ln in lines:
        k, *v = ln.split()
        try:
            rows.setdefault(k, []).append(np.array([float(x) for x in v]))
        except ValueError:
            pass
    H = product
    p = H.read_pgs_config(PGS_CONFIG, 8)
    m = H.KinematicModel(os.path.join(MODELS, "hexapod.xml"))
    ref = H.run_host(m, [p], n_t=20, horizon=20)
    # measure_cot: the shim's numbers and the oracle's COT (reference-faithful basis)
    cot = rows["cot"][0][0]
    assert cot == pytest.approx(ref["work_cot"][0, 1], rel=1e-14)
    assert cot == pytest.approx(oracle_mod.rollout(omodels["hexapod"], to_oracle_gait(oracle_mod, p), 20,
                                                   basis=oracle_mod.BASIS_ORTHO)["cot"], rel=1e-9)
    assert any(ln.startswith("min cfz = ") for ln in lines)
    # measure_cot_sweep: pgssweeper's 16 values, printed with cout's 6 digits
    sweep = [ln for ln in lines if ln.startswith("val = ")]
    assert len(sweep) == 16 and "sweeping over period:" in out
    py = H.ModelPlayer(m).measure_cot_sweep(p, 20, "period", 3, 18, 15)
    for ln, (v, c) in zip(sweep, py):
        toks = ln.split()
        assert float(toks[2]) == pytest.approx(v, rel=1e-5) and float(toks[5]) == pytest.approx(c, rel=1e-5)
    # test_dynamics: torques -> forces round trip
    s = float([ln for ln in lines if ln.startswith("s = ")][0].split("=")[1])
    assert s < 1e-9
    # periodic.h:43-51 accessors
    assert np.all(rows["masses"][0] == 1) and len(rows["masses"][0]) == m.n_parts
    assert list(rows["parentis"][0]) == [m.get_mnode(i)["parent"] for i in range(m.n_parts)]
    assert list(rows["footis"][0]) == [4, 7, 11, 14, 18, 21]
    assert np.array_equal(rows["motor_torques_last"][0], ref["tau"][0, 19])  # sample n_t + 1
    assert np.array_equal(rows["solve7_tau"][0], ref["tau"][0, 5])           # sample 7 = step 5
    assert np.array_equal(rows["solve7_cf"][0], ref["cf"][0, 5])
    assert np.array_equal(rows["motor_torques_7"][0], ref["tau"][0, 5])
    assert np.array_equal(rows["computed_7"][0], ref["tau"][0, 5])
    # the position controller: tau_ff + k1 mod(q - q0) + k2 (dq - dq0) with the stub's offsets
    r150 = H.run_host(m, [p], n_t=150, horizon=150)
    ct = H.complete_traj(m, [p], 150)[0]
    for j, tsi in enumerate(int(v[0]) for v in rows["tsi"]):
        ff = r150["tau"][0, (tsi - 2) % 150]
        assert np.array_equal(rows["ff"][j], ff)
        assert np.array_equal(rows["q0"][j], ct[tsi % 150, 6:24])
        assert np.array_equal(rows["dq0"][j], ct[tsi % 150, 30:48])
        want = ff + (-100.0) * 0.01 * np.arange(1, 19) + (-20.0) * (-0.2)
        assert np.abs(rows["cmd"][j] - want).max() < 1e-12
    # cpc.cpp:51-63: get_complete_traj_rec rows
    assert np.array_equal(rows["tp0"][0], ct[0]) and np.array_equal(rows["tp77"][0], ct[77])
    assert rows["tps_size"][0][0] == 150
    # record_per_traj: n_t = int(T / play_dt + .5) = 150 rows of traj.txt (ostream's 6 digits)
    one = np.loadtxt(tmp_path / "traj_one.txt")
    assert one.shape == (150, 66) and np.allclose(one, ct, rtol=1e-5, atol=1e-6)
    # record_per_traj_sweep with main.cpp:38's rotation: 2 values appended, n_t from the unswept period
    sw = np.loadtxt(tmp_path / "traj_sweep.txt")
    assert sw.shape == (300, 66)
    gaits = []
    for L in (-0.5, 0.5):
        g = H.read_pgs_config(PGS_CONFIG, 8)
        g.step_length = L
        g.set_rec_rotation((0, 0, -1.571))
        gaits.append(g)
    ctr = H.complete_traj(m, gaits, 150)
    assert np.allclose(sw, ctr.reshape(300, 66), rtol=1e-5, atol=1e-6)
    pr = H.read_pgs_config(PGS_CONFIG, 8)
    pr.set_rec_rotation((0, 0, -1.571))
    assert rows["cot_rotated"][0][0] == pytest.approx(H.ModelPlayer(m).measure_cot(pr, 20), rel=1e-14)
