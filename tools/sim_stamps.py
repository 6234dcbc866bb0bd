"""Per-phase shader-clock breakdown of hs_sim_kernel (diagnostic build, -DHS_SIM_STAMPS).

Builds hslabs_amd/_build/libhslabs_simstamps.so, runs N_STEPS closed-loop steps of a
B-rollout batch and prints the mean cycles per step and wavefront of each phase.
Never used by the product path.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hslabs_amd import build as Bd  # noqa: E402

LIB = os.path.join(Bd.OUT_DIR, "libhslabs_simstamps.so")
PHASES = ["load", "P control", "B bodies+collide", "offsets", "R rows", "A rhs/Ad", "shuffle+runs", "SOR runs",
          "U update+out"]


def main():
    if "--build" in sys.argv or not os.path.exists(LIB):
        Bd._compile(LIB, ["HS_SIM_STAMPS"])
    if "--build-only" in sys.argv:
        return
    import torch
    from hslabs_amd import capi
    L = ctypes.CDLL(LIB)
    capi._lib = None
    Bd.LIB = LIB
    capi.load(build_if_missing=False)
    import hslabs_amd as H
    from hslabs_amd import synth
    n = int(os.environ.get("N", "1024"))
    steps = int(os.environ.get("N_STEPS", "20"))
    m = H.KinematicModel(os.path.join(ROOT, "models", os.environ.get("MODEL", "hexapod") + ".xml"))
    sb = H.SimBatch(m, synth.gen_sim_params(n, os.environ.get("MODEL", "hexapod")))
    sb.step(2, outputs=())
    torch.cuda.synchronize()
    L.hs_debug_clear_sim_stamps()
    sb.step(steps, outputs=())
    torch.cuda.synchronize()
    st = np.zeros((4096, 16), dtype=np.uint64)
    L.hs_debug_read_sim_stamps(st.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), 4096)
    st = st[:min(n, 4096)].astype(np.float64)
    tot = st[:, :9].sum(axis=1) / steps
    for i, name in enumerate(PHASES):
        d = st[:, i] / steps
        print(f"{name:20s} mean {d.mean():10.0f}  p50 {np.median(d):10.0f}  p90 {np.percentile(d, 90):10.0f}"
              f"  ({100 * d.mean() / tot.mean():5.1f} %)")
    tot = tot + st[:, 11:14].sum(axis=1) / steps
    for i, name in ((11, "  reshuffle: trace"), (12, "  reshuffle: prev"), (13, "  reshuffle: relax")):
        d = st[:, i] / steps
        print(f"{name:20s} mean {d.mean():10.0f}  ({100 * d.mean() / tot.mean():5.1f} %)")
    print(f"{'TOTAL / step':20s} mean {tot.mean():10.0f}")
    print(f"rows per step {st[:, 10].mean() / steps:.1f}, SOR runs per reshuffle {st[:, 9].mean() / steps:.1f}")


if __name__ == "__main__":
    main()
