"""hs_math.h's sincos_k -- the sines and cosines of the joint values in the rollout kernels' kinematics
(a Cody-Waite reduction by pi/2 and fdlibm's kernel polynomials in place of the library sincos) -- run on
the host (the function is __host__ __device__; tests/cpp/sincos_k_check.hip) against the C library's sin
and cos, which the oracle uses: within 1 ulp (sin) and 2 ulp (cos) over 2e6 seeded arguments, a third of
them within 1e-9 of a multiple of pi/2, and over the doubles nearest to every multiple of pi/2 below 2^20
(with their neighbours: the reduction's worst cases), the same signs at the special points except sin(-0) (+0 here: the
reduction's x - 0 * pi/2 rounds to +0; the values compare equal), NaN for non-finite input."""
import os
import subprocess

import pytest

from conftest import ROOT

HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_sincos_k_against_libm(tmp_path):
    exe = tmp_path / "sincos_k_check"
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O2", "-std=c++17", "-ffp-contract=fast",
                    "-I", os.path.join(ROOT, "hslabs_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "cpp", "sincos_k_check.hip"), "-o", str(exe)],
                   check=True, capture_output=True, timeout=600)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=300).stdout
    vals = {}
    specials = []
    for line in out.splitlines():
        f = line.split()
        if f[0] == "special":
            specials.append((float(f[1]), int(f[2]), int(f[3]), int(f[4])))
        else:
            vals[f[0]] = float(f[1])
    assert vals["max_ulp_sin"] <= 1, out
    assert vals["max_ulp_cos"] <= 2, out
    assert vals["max_abs"] <= 2.3e-16, out
    for x, us, uc, sign_ok in specials:
        assert us <= 1 and uc <= 2, (x, us, uc)
        assert sign_ok or (x == 0 and str(x) == "-0.0"), (x, sign_ok)
    assert vals["nonfinite_nan"] == 1
