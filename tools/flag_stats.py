"""Diagnostic: share of steps that take the general (Eigen-style) contact solve and the
histogram of contacts per step, for 4096 synthetic rollouts x one cycle of each model.

    python tools/flag_stats.py          (GPU)
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import hslabs_amd as H
    from hslabs_amd import synth

    for name in ("myant", "hexapod", "spider"):
        m = H.KinematicModel(os.path.join(ROOT, "models", f"{name}.xml"))
        p = synth.gen_params(4096, name)
        b = H.DeviceBatch(m, p, n_t=20, horizon=20, outputs=("flags", "cf"))
        b.run(best=False)
        torch.cuda.synchronize()
        f = b.flags.cpu().numpy()
        nc = (np.abs(b.cf.cpu().numpy().reshape(4096, 20, -1, 3)).max(axis=3) > 0).sum(axis=2)
        print(name, "general %.4f" % ((f & 64) != 0).mean(), "nc hist", np.bincount(nc.ravel(), minlength=7) / nc.size)


if __name__ == "__main__":
    main()
