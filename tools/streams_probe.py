"""Tuning probe: the B = 4096, H = 1 batch as S independent shards on S HIP streams (each shard
its own hs_run_steps loop), vs one stream. Prints steps/s per S.

    python tools/streams_probe.py [K]          (GPU)
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import hslabs_amd as H
    from hslabs_amd import synth

    K = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    B = 4096
    m = H.KinematicModel(os.path.join(ROOT, "models", "hexapod.xml"))
    for S in (1, 2, 4):
        n = B // S
        streams = [torch.cuda.Stream() for _ in range(S)]
        batches = [H.DeviceBatch(m, synth.gen_params(n, "hexapod", id0=s * n), n_t=20, k0=0, horizon=1,
                                 outputs=("tau", "cf", "work_cot", "flags"), rollout_id_base=s * n) for s in range(S)]
        for s in range(S):
            batches[s].run_steps(20, stream=streams[s], best=False, accumulate=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(S):
            batches[s].run_steps(K, stream=streams[s], best=False, accumulate=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        print(f"S={S}: {B * K / el / 1e6:.1f} M steps/s ({1e6 * el / K:.2f} us per step of the whole batch)", flush=True)


if __name__ == "__main__":
    main()
