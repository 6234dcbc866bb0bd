"""Deferral counts of the limb-lane kernel (hs_limb_stats) on configs[4]'s mixed plan and on its two
models run alone with the same gait parameters (diagnostic)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hslabs_amd as H  # noqa: E402
from hslabs_amd import synth  # noqa: E402


def main():
    B, K = 4096, 20
    params, idx = synth.gen_mixed(B)
    ms = [H.KinematicModel(os.path.join(ROOT, "models", f"{n}.xml")) for n in synth.MIXED_MODELS]
    d0 = H.api.limb_deferred()
    mb = H.MixedBatch(ms, idx, params, n_t=20, k0=0, horizon=K, outputs=("tau", "cf", "flags", "work_cot"))
    mb.work_cot.zero_()
    mb.run_calls(K, call_horizon=1, best=False, accumulate=True)
    torch.cuda.synchronize()
    print(f"mixed B={B}: {H.api.limb_deferred() - d0} of {B * K} steps deferred")
    for k, n in enumerate(synth.MIXED_MODELS):
        sel = np.nonzero(idx == k)[0]
        d0 = H.api.limb_deferred()
        b = H.DeviceBatch(ms[k], params[sel], n_t=20, k0=0, horizon=K, outputs=("tau", "cf", "flags", "work_cot"))
        b.work_cot.zero_()
        b.run_calls(K, call_horizon=1, best=False, accumulate=True)
        torch.cuda.synchronize()
        print(f"{n} alone ({len(sel)} rollouts): {H.api.limb_deferred() - d0} of {len(sel) * K} steps deferred")


if __name__ == "__main__":
    main()
