"""Per-phase shader-clock breakdown of hs_rollout_kernel (diagnostic build, -DHS_STAMPS).

Builds hslabs_amd/_build/libhslabs_stamps.so, runs one batch and prints mean /
p50 / p90 cycles per phase over the wavefronts (two rollouts each). Never used by the product path.
"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from hslabs_amd import build as B  # noqa: E402

LIB = os.path.join(B.OUT_DIR, os.environ.get("STAMPS_LIB", "libhslabs_stamps.so"))
PHASES = [("setup", 0, 1), ("kin(5 samples)", 1, 2), ("k:frames", 1, 20), ("k:table+sincos", 20, 21),
          ("k:(inline IK)", 21, 22), ("k:limb FK+features", 22, 2), ("dynamics", 3, 4), ("particular", 4, 5),
          ("contact list", 5, 6), ("contact solve", 6, 7), ("outputs", 7, 8), ("TOTAL", 0, 8)]
# general path (waves where it ran): grams, LU, LU solve + kernel, m, QR, QR solve
GENERAL = [("g:grams", 6, 9), ("g:LU", 9, 10), ("g:solve+kernel", 10, 11), ("g:m", 11, 12), ("g:QR", 12, 13),
           ("g:QR solve", 13, 14), ("g:rest", 14, 7)]


def build():
    extra = [d for d in os.environ.get("HS_DEFINES", "").split() if d]
    B._compile(LIB, ["HS_STAMPS", *extra])


def main():
    if "--build" in sys.argv or not os.path.exists(LIB):
        build()
    if "--build-only" in sys.argv:
        return
    if os.environ.get("FUSED"):
        import torch  # noqa: F401  (the HIP runtime torch loads, before the diagnostic library)
    from hslabs_amd import capi
    L = ctypes.CDLL(LIB)
    capi._lib = None
    capi._build.LIB = LIB  # load the diagnostic build through the normal binding
    capi.load(build_if_missing=False)
    import hslabs_amd as H
    from hslabs_amd import synth

    n = int(os.environ.get("N", "4096"))
    model = os.environ.get("MODEL", "hexapod")
    m = H.KinematicModel(os.path.join(ROOT, "models", f"{model}.xml"))
    params = synth.gen_params(n, model, curved=bool(os.environ.get("CURVED")))
    k0 = int(os.environ.get("K0", "0"))
    # horizon 2 (default): the stamps kept are the second launch's, which loads the gait setup
    # stored by the first (the steady state of hs_run_steps); HZ=1 stamps a computing launch
    hz = int(os.environ.get("HZ", "2"))
    fused = os.environ.get("FUSED")  # the bench's path: hs_run_calls of 20 steps (rows: steps 0, 1)
    if fused:
        import torch
        b = H.DeviceBatch(m, params, n_t=20, k0=k0, horizon=20, outputs=("tau", "cf", "work_cot", "flags"))
        b.run_calls(20, best=True)
        torch.cuda.synchronize()
        # STEP=s: blocks s * n_waves ... of the fused launch (with the grouped block order, fused_coords,
        # a window in the middle of the launch: group s * n_waves / (256 * 20)'s steps); the preparation
        # pass's rows are then not recorded
        L.hs_debug_set_stamp_base(ctypes.c_uint(int(os.environ.get("STEP", "0")) * ((n + 1) // 2)))
        L.hs_debug_clear_stamps()
        b.run_calls(20, best=True)
        if os.environ.get("B2B"):  # a second call queued behind the first: its stamps overwrite the first's
            b.run_calls(20, best=True)
        torch.cuda.synchronize()
    else:
        H.run_host(m, params, n_t=20, k0=k0, horizon=hz, want=("tau",))  # warm
        L.hs_debug_clear_stamps()
        H.run_host(m, params, n_t=20, k0=k0, horizon=hz, want=("tau",))
    st = np.zeros((4096, 32), dtype=np.uint64)
    L.hs_debug_read_stamps(st.ctypes.data_as(ctypes.POINTER(ctypes.c_ulonglong)), 4096)
    st = st.astype(np.int64)
    pr = st[st[:, 28] != 0]  # hs_prep_kernel's waves (fused: the call's preparation pass), slots 24..30
    if fused and len(pr):
        for name, x, y in (("p:setup", 24, 25), ("p:max radius", 25, 26), ("p:first row", 26, 27),
                           ("p:other rows", 27, 28), ("p:TOTAL", 24, 28)):
            d = pr[:, y] - pr[:, x]
            print(f"{name:22s} mean {d.mean():10.0f}  p50 {np.median(d):10.0f}  p90 {np.percentile(d, 90):10.0f}  max {d.max():10.0f}  (n={len(pr)})")
        t0 = pr[:, 29].min()
        for name, col in (("p:wave start (us)", 29), ("p:wave end (us)", 30)):
            d = (pr[:, col] - t0) / 100.0
            print(f"{name:22s} mean {d.mean():10.2f}  p50 {np.median(d):10.2f}  p90 {np.percentile(d, 90):10.2f}  max {d.max():10.2f}")
    st = st[:min((n + 1) // 2, 4096)]  # one row per wavefront (two rollouts)
    if fused and not int(os.environ.get("STEP", "0")):
        st = st[64:]  # the fixup + reduce launch's 64 workgroups restamp rows 0..63's entry slots
    if os.environ.get("STAMPS_RAW"):
        np.save(os.environ["STAMPS_RAW"], st)
    gen = st[:, 9] != 0
    sch = (st[:, 18] != 0) & (st[:, 19] != 0) & ~gen  # Schur tier: contact blocks | 6x6 solve | back-sub
    if sch.any():
        for name, x, y in (("s:blocks", 6, 18), ("s:schur 6x6", 18, 19), ("s:backsub", 19, 7)):
            d = st[sch, y] - st[sch, x]
            print(f"{name:22s} mean {d.mean():10.0f}  p50 {np.median(d):10.0f}  p90 {np.percentile(d, 90):10.0f}  max {d.max():10.0f}  (n={sch.sum()})")
    for name, a, b in PHASES + (GENERAL if gen.any() else []):
        d = (st[gen] if name.startswith("g:") else st)[:, b] - (st[gen] if name.startswith("g:") else st)[:, a]
        print(f"{name:22s} mean {d.mean():10.0f}  p50 {np.median(d):10.0f}  p90 {np.percentile(d, 90):10.0f}  max {d.max():10.0f}")
    # launch shape on the 100 MHz clock (slots 16, 17), relative to the first wave's entry, in us
    t0 = st[:, 16].min()
    d = st[:, 0] - st[:, 15]
    print(f"{'entry->setup (cyc)':22s} mean {d.mean():10.0f}  p50 {np.median(d):10.0f}  p90 {np.percentile(d, 90):10.0f}  max {d.max():10.0f}")
    for name, col in (("wave start (us)", 16), ("wave end (us)", 17)):
        d = (st[:, col] - t0) / 100.0
        print(f"{name:22s} mean {d.mean():10.2f}  p50 {np.median(d):10.2f}  p90 {np.percentile(d, 90):10.2f}  max {d.max():10.2f}")
    d = (st[:, 17] - st[:, 16]) / 100.0
    print(f"{'wave life (us)':22s} mean {d.mean():10.2f}  p50 {np.median(d):10.2f}  p90 {np.percentile(d, 90):10.2f}  max {d.max():10.2f}")
    hist = np.histogram((st[:, 16] - t0) / 100.0, bins=10)
    print("start histogram:", list(hist[0]), "edges(us):", [round(e, 1) for e in hist[1]])

if __name__ == "__main__":
    main()
