"""Dump the fused path's outputs (tau, cf, flags, work_cot) for a transformed synthetic batch to an
npz (diagnostics of tests/test_gpu_rec_transform.py on the GPU box):
  python tools/diag_fused.py <model> <curved 0|1> <out.npz> [B] [id0] [seed]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import hslabs_amd as H
    from hslabs_amd import synth
    from conftest import MODELS, transformed
    from test_gpu_parity import fused_cycle

    name, curved, out = sys.argv[1], bool(int(sys.argv[2])), sys.argv[3]
    B = int(sys.argv[4]) if len(sys.argv) > 4 else 256
    id0 = int(sys.argv[5]) if len(sys.argv) > 5 else 900
    seed = int(sys.argv[6]) if len(sys.argv) > 6 else 7 + curved
    params, on = transformed(synth.gen_params(B, name, id0=id0, curved=curved), np.random.default_rng(seed))
    model = H.KinematicModel(os.path.join(MODELS, f"{name}.xml"))
    g = fused_cycle(H, model, params)
    solo = H.run_host(model, params, n_t=20, k0=0, horizon=20)
    np.savez(out, params=params, on=on, solo_tau=solo["tau"], solo_flags=solo["flags"], **g)
    print("saved", out, {k: v.shape for k, v in g.items()})


if __name__ == "__main__":
    main()
