"""Steps where the kernel and the oracle's tree mode disagree without a near-rank flag on either
side (diagnostic for HS_FLAG_NEAR_RANK's bands; tests/test_gpu_rec_transform.py's batches).
    python tools/near_diag.py [name] [curved] [tilt]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch  # noqa: F401

    import hslabs_amd as H
    from conftest import record_to_oracle_gait, transformed
    from hslabs_amd import synth
    from oracle import oracle as O
    from test_gpu_parity import fused_cycle, near

    name = sys.argv[1] if len(sys.argv) > 1 else "hexapod"
    curved = (sys.argv[2] == "1") if len(sys.argv) > 2 else True
    tilt = float(sys.argv[3]) if len(sys.argv) > 3 else 0.05
    m = H.KinematicModel(os.path.join(ROOT, "models", f"{name}.xml"))
    om = O.Model(os.path.join(ROOT, "models", f"{name}.xml"))
    rng = np.random.default_rng(7 + curved)
    base = synth.gen_params(256, name, id0=900, curved=curved)
    params, on = transformed(base, rng, tilt=tilt)
    g = fused_cycle(H, m, params)
    gaits = [record_to_oracle_gait(O, r) for r in params]
    t = O.batch(om, gaits, 20, 0, 20, basis=O.BASIS_TREE, n_threads=16)
    f = O.batch(om, gaits, 20, 0, 20, basis=O.BASIS_FAST, n_threads=16)
    skip = near(g["flags"], t["flags"])
    scale = np.maximum(1, np.abs(t["tau"]).max(-1))
    err = np.abs(g["tau"] - t["tau"]).max(-1)
    bad = ((err >= 1e-6) | (err / scale >= 1e-9)) & ~skip
    print(f"{name} curved={curved} tilt={tilt}: {bad.sum()} unflagged steps over the bounds, {skip.sum()} flagged")
    for b, h in np.argwhere(bad)[:12]:
        ef = np.abs(g["tau"][b, h] - f["tau"][b, h]).max()
        print(f"  rollout {b} step {h}: |dtau| {err[b, h]:.3e} (scale {scale[b, h]:.1f}) vs fast {ef:.3e}; "
              f"flags gpu {int(g['flags'][b, h])} tree {int(t['flags'][b, h])} fast {int(f['flags'][b, h])}; "
              f"tree margin {t['near_margin'][b, h]:.2f} {O.NEAR_KINDS[int(t['near_kind'][b, h])]}, "
              f"fast margin {f['near_margin'][b, h]:.2f} {O.NEAR_KINDS[int(f['near_kind'][b, h])]}, "
              f"lu_kept {t['lu_kept'][b, h]:.2e} qr_kept {t['qr_kept'][b, h]:.2e}")


if __name__ == "__main__":
    main()
