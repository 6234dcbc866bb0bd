"""Dump the outputs of a fixed set of hs_run_host batches (all pgs setups, synthetic straight and
curved batches of the three models, fp64) to an .npz, for bitwise comparison of two library builds
(tuning aid). The library is the product's, or a build_variant named by HSLABS_VARIANT.

  HSLABS_VARIANT=s1 python tools/variant_dump.py out_s1.npz
  python tools/variant_dump.py out_new.npz
  python tools/variant_dump.py --compare out_s1.npz out_new.npz
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def dump(path):
    import hslabs_amd as H
    from hslabs_amd import synth

    out = {}
    models = {n: H.KinematicModel(os.path.join(ROOT, "models", f"{n}.xml")) for n in ("hexapod", "spider", "myant")}
    cfg = os.path.join(ROOT, "models", "pgs_config.txt")
    for i in range(28):
        p = H.read_pgs_config(cfg, i)
        r = H.run_host(models[p.fname.split(".")[0]], [p], n_t=20, horizon=20)
        for k, v in r.items():
            out[f"pgs{i}_{k}"] = v
    for name, m in models.items():
        for curved in (False, True):
            params = synth.gen_params(512, name, curved=curved)
            r = H.run_host(m, params, n_t=20, horizon=20)
            for k, v in r.items():
                out[f"{name}_{int(curved)}_{k}"] = v
    np.savez(path, **out)
    print("dumped", len(out), "arrays, library", H.capi.LOADED)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    worst = {}
    for k in A.files:
        x, y = A[k], B[k]
        if np.array_equal(x, y, equal_nan=True):
            continue
        d = np.nanmax(np.abs(x.astype(np.float64) - y.astype(np.float64)))
        worst[k] = d
    if not worst:
        print("bitwise equal:", len(A.files), "arrays")
    for k, d in sorted(worst.items(), key=lambda kv: -kv[1])[:30]:
        print(f"{k}: max |diff| {d:.3e}")
    return worst


if __name__ == "__main__":
    if sys.argv[1] == "--compare":
        compare(sys.argv[2], sys.argv[3])
    else:
        dump(sys.argv[1])
