"""Per-phase shader-clock breakdown of the solve_forces step (diagnostic HS_STAMPS build, like
tools/stamps.py): one hs_run_forces launch of hexapod B rollouts. Never used by the product path.
  python tools/forces_stamps.py [--build]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hslabs_amd import build as B  # noqa: E402

LIB = os.path.join(B.OUT_DIR, "libhslabs_stamps.so")
# forces_solve's stamps: 10 after the particular solution, 4 after the limb blocks, 5 after the sums over
# limbs, 9 after the 6 x 6 system and the feet's solves (or the dense route), 11 after the outputs
PHASES = [("kinematics", 1, 2), ("dynamics+particular", 2, 10), ("limb blocks", 10, 4), ("sums over limbs", 4, 5),
          ("6x6 + feet", 5, 9), ("outputs", 9, 11), ("TOTAL", 1, 11)]


def main():
    if "--build" in sys.argv or not os.path.exists(LIB):
        B._compile(LIB, ["HS_STAMPS"])
    if "--build-only" in sys.argv:
        return
    import torch  # first: one HIP runtime per process (torch's), which the library then binds

    from hslabs_amd import capi
    L = ctypes.CDLL(LIB)
    capi._lib = None
    capi._build.LIB = LIB
    capi.load(build_if_missing=False)
    import hslabs_amd as H
    from hslabs_amd import synth

    n = int(os.environ.get("N", "4096"))
    m = H.KinematicModel(os.path.join(ROOT, "models", "hexapod.xml"))
    params = synth.gen_params(n, "hexapod")
    full = H.DeviceBatch(m, params, n_t=20, horizon=1, outputs=("tau",))
    full.run(best=False)
    fb = H.DeviceBatch(m, params, n_t=20, horizon=1, outputs=("cf", "flags"))
    fb.run_forces(full.tau)
    torch.cuda.synchronize()
    L.hs_debug_clear_stamps()
    fb.run_forces(full.tau)
    torch.cuda.synchronize()
    st = np.zeros((4096, 24), dtype=np.uint64)
    L.hs_debug_read_stamps(st.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), 4096)
    st = st[:min((n + 1) // 2, 4096)].astype(np.int64)
    for name, a, b in PHASES:
        d = st[:, b] - st[:, a]
        print(f"{name:22s} mean {d.mean():10.0f}  p50 {np.median(d):10.0f}  p90 {np.percentile(d, 90):10.0f}")


if __name__ == "__main__":
    main()
