"""solve_forces throughput (hs_run_forces_calls, fused, vs hs_run_forces, one launch per step of its
horizon): hexapod B rollouts, S steps of given motor torques. Tuning aid.
  python tools/forces_probe.py [B] [S]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import hslabs_amd as H
    from hslabs_amd import synth

    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    m = H.KinematicModel(os.path.join(ROOT, "models", "hexapod.xml"))
    params = synth.gen_params(B, "hexapod")
    full = H.DeviceBatch(m, params, n_t=20, horizon=S, outputs=("tau",))
    full.run_calls(S)
    tau = full.tau.clone()
    fb = H.DeviceBatch(m, params, n_t=20, horizon=S, outputs=("cf", "flags"))
    st = torch.cuda.current_stream()
    res = {}
    for name, fn in (("per-step launches", lambda: fb.run_forces(tau)),
                     ("fused", lambda: fb.run_forces_calls(tau, S))):
        for _ in range(3):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / 10
        res[name] = us
        print(f"{name}: {us:.1f} us per {S}-step job, {B * S / us:.1f} M steps/s")


if __name__ == "__main__":
    main()
