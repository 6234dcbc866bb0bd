"""Per-phase shader-clock breakdown of the limb-lane step kernel (hs_limb.h; diagnostic -DHS_STAMPS build
libhslabs_stamps.so, tools/stamps.py's). Runs the bench's fused path (hexapod B = 4096, 20 calls) and prints
mean / p50 / p90 cycles per phase over the wavefronts of one window of the launch (STEP=s: blocks from
s * 512). Tuning aid only.   python tools/limb_stamps.py [--build]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from hslabs_amd import build as B  # noqa: E402

LIB = os.path.join(B.OUT_DIR, "libhslabs_stamps.so")
PHASES = [("prelims (tv, o)", 15, 0), ("outer t-2dt FK", 0, 1), ("outer t+2dt FK", 1, 2), ("centre FK + D", 2, 3),
          ("torso + sync", 3, 4), ("subtree sums + root", 4, 5), ("contact list + zeroth", 5, 6),
          ("contact blocks + Schur sums", 6, 7), ("6x6 + y", 7, 8), ("outputs", 8, 9), ("TOTAL", 15, 9)]


def main():
    if "--build" in sys.argv or not os.path.exists(LIB):
        B._compile(LIB, ["HS_STAMPS"])
    if "--build-only" in sys.argv:
        return
    import torch
    from hslabs_amd import capi
    L = ctypes.CDLL(LIB)
    capi._lib = None
    capi._build.LIB = LIB
    capi.load(build_if_missing=False)
    import hslabs_amd as H
    from hslabs_amd import synth

    n = 4096
    m = H.KinematicModel(os.path.join(ROOT, "models", "hexapod.xml"))
    params = synth.gen_params(n, "hexapod")
    b = H.DeviceBatch(m, params, n_t=20, k0=0, horizon=20, outputs=("tau", "cf", "work_cot", "flags"))
    b.run_calls(20, best=True)
    torch.cuda.synchronize()
    L.hs_debug_set_stamp_base(ctypes.c_uint(int(os.environ.get("STEP", "4")) * (n // 8)))
    L.hs_debug_clear_stamps()
    b.run_calls(20, best=True)
    torch.cuda.synchronize()
    st = np.zeros((4096, 32), dtype=np.uint64)
    L.hs_debug_read_stamps(st.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), 4096)
    st = st.astype(np.int64)
    st = st[(st[:, 9] != 0) & (st[:, 15] != 0)]
    for name, a, c in PHASES:
        d = st[:, c] - st[:, a]
        print(f"{name:28s} mean {d.mean():9.0f}  p50 {np.median(d):9.0f}  p90 {np.percentile(d, 90):9.0f}  (n={len(d)})")
    t0 = st[:, 16].min()
    d = (st[:, 17] - st[:, 16]) / 100.0
    print(f"{'wave life (us)':28s} mean {d.mean():9.2f}  p50 {np.median(d):9.2f}  p90 {np.percentile(d, 90):9.2f}")
    s0 = (st[:, 16] - t0) / 100.0
    print(f"{'wave start (us)':28s} mean {s0.mean():9.2f}  max {s0.max():9.2f}")


if __name__ == "__main__":
    main()
