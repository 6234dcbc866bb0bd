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
