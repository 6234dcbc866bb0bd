"""Host-side overhead of one timed bench job (driver config: hexapod B=4096, 20 fused steps):
wall time vs the HIP events around the launches, for two ways of waiting for the stream
(torch.cuda.synchronize alone; polling the end event, then torch.cuda.synchronize). Tuning aid."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import hslabs_amd as H
    from hslabs_amd import synth

    dev = torch.device("cuda", 0)
    m = H.KinematicModel(os.path.join(ROOT, "models", "hexapod.xml"))
    K = 20
    b = H.DeviceBatch(m, synth.gen_params(4096, "hexapod"), n_t=20, k0=0, horizon=K,
                      outputs=("tau", "cf", "work_cot", "flags"), device=dev)
    st = torch.cuda.current_stream(dev)
    b.key_steps = K
    job = b.calls_launcher(K, stream=st, best=True)
    for _ in range(5):
        job()
    torch.cuda.synchronize()
    for mode, idle in (("sync", 0), ("poll", 0), ("sync", 1e-4), ("sync", 1e-3), ("sync", 1e-2), ("sync", 0.1)):
        walls, evs = [], []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            if idle:
                time.sleep(idle)
            t0 = time.perf_counter()
            e0.record(st)
            job()
            e1.record(st)
            if mode == "poll":
                while not e1.query():
                    pass
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) * 1e6)
            evs.append(e0.elapsed_time(e1) * 1e3)
        w, e = np.median(walls), np.median(evs)
        print(f"{mode} after {idle * 1e3:g} ms idle: wall {w:.1f} us, events {e:.1f} us, host overhead {w - e:.1f} us per job")


if __name__ == "__main__":
    main()
