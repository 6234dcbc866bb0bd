"""Kernel time of each step k0 of the cycle (HIP events around each launch) next to the
number of rollouts whose step took the general path (HS_FLAG_GENERAL). Tuning aid."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import hslabs_amd as H
    from hslabs_amd import synth

    name, B = os.environ.get("MODEL", "myant"), int(os.environ.get("B", "4096"))
    m = H.KinematicModel(os.path.join(ROOT, "models", f"{name}.xml"))
    b = H.DeviceBatch(m, synth.gen_params(B, name), n_t=20, horizon=1)
    full = H.DeviceBatch(m, synth.gen_params(B, name), n_t=20, horizon=20, outputs=("flags",))
    full.run(best=False)
    b.run_steps(40)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(40)]
    b.k0 = 0
    b.run_steps(20, events=ev)
    torch.cuda.synchronize()
    gen = ((full.flags.cpu().numpy() & 64) != 0).sum(axis=0)
    for k in range(20):
        print(f"k0 {k:2d}  {1e3 * ev[2 * k].elapsed_time(ev[2 * k + 1]):8.1f} us  general-path rollouts {gen[k]}")


if __name__ == "__main__":
    main()
