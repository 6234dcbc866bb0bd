"""Diagnostic (tuning aid): where do the limb-lane kernel's values first differ from hs_rollout_kernel's?
Runs the HS_DBG=n variant builds (hslabs_amd.build.build_variant('dbg<n>', ['HS_DBG=<n>'])): each writes
intermediate value n of every part / contact of every step into a device buffer in both kernels; the two
runs' buffers are compared per value.   python tools/limb_dbg.py 1 2 3 ...   (on the GPU box)"""
import ctypes
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NAMES = {1: "P0[0] link pos", 2: "f[0] link force", 3: "g torque[0]", 4: "x torque[0] (subtree)", 5: "U0[0] link ust",
         6: "D_c[0]", 7: "g_c[0]", 8: "y[0]", 9: "Um[0] link ust t-2dt", 10: "amr[0] link", 11: "Up[0] link ust t+2dt",
         12: "Pm[0] link pos t-2dt", 13: "f[1]", 14: "f[2] (gravity added)", 15: "o[0], o[1] (slots 31, 30)", 16: "amr[1]", 17: "d[0] = Jp - o (subtree stage)", 18: "F[0] subtree force",
         19: "nc=1 M[4]", 20: "nc=1 b[1] before solve", 21: "nc=1 y[0]", 22: "nc=2 y[0]", 23: "nc=2 b[0] (after solve)",
         24: "nc=2 t", 25: "foot fp[2]", 26: "nc=2 nv[2]", 27: "nc=2 M[5]",
         30: "forces ts[3]", 31: "forces S_l[0]", 32: "forces K_f[0]", 33: "forces K[0]", 34: "forces lam[0]",
         35: "forces y_f[0]", 36: "forces Ct[0]", 37: "forces r_f[0]", 38: "forces e_l[0]",
         40: "forces t0 = jz.x (motor 0)", 41: "forces z (motor 0)", 42: "forces X[0][0]", 43: "forces Z[0][0]"}


def child(n):
    sys.path.insert(0, ROOT)
    import torch

    import hslabs_amd as H
    from hslabs_amd import capi, synth
    L = capi.load()
    L.hs_debug_read_dbg.argtypes = [ctypes.c_void_p, ctypes.c_int]
    model = os.environ.get("MODEL", "hexapod")
    m = H.KinematicModel(os.path.join(ROOT, "models", f"{model}.xml"))
    B, K = 256, 20
    p = synth.gen_params(B, model, id0=4321, curved=os.environ.get("CURVED") == "1")
    out = []
    forces = os.environ.get("FORCES") == "1"  # solve_forces (hs_run_forces_calls) instead of the control step
    if forces:
        ctl = H.DeviceBatch(m, p, n_t=20, k0=0, horizon=K, outputs=("tau",))
        ctl.run_calls(K, call_horizon=1)
        tau_in = ctl.tau + 0.1
    for limb in ("1", "0"):
        os.environ["HS_LIMB"] = limb
        if forces:
            b = H.DeviceBatch(m, p, n_t=20, k0=0, horizon=K, outputs=("cf", "flags"))
            b.forces_launcher(tau_in, K)()
            b.tau = b.cf
        else:
            b = H.DeviceBatch(m, p, n_t=20, k0=0, horizon=K, outputs=("tau", "cf", "flags", "work_cot"))
            b.work_cot.zero_()
            b.run_calls(K, call_horizon=1, best=False, accumulate=True)
        torch.cuda.synchronize()
        buf = np.zeros(B * K * 32)
        capi.check(L.hs_debug_read_dbg(buf.ctypes.data, buf.size), "read")
        out.append((buf.reshape(B * K, 32), b.tau.cpu().numpy()))
    (a, ta), (o, to) = out
    both = (a != 0) & (o != 0)
    d = (a != o) & both
    print(f"dbg{n} {NAMES.get(n)}: {int(d.sum())} of {d.size} entries differ, max |diff| {np.abs(a - o)[both].max() if both.any() else 0:.3e}, "
          f"slots differing {sorted(set(np.nonzero(d)[1].tolist()))[:32]}; tau differ {int((ta != to).sum())}", flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(int(sys.argv[2]))
    else:
        for n in sys.argv[1:]:
            env = dict(os.environ, HSLABS_VARIANT=f"dbg{n}")
            subprocess.run([sys.executable, __file__, "--child", n], env=env, check=True, timeout=300)
