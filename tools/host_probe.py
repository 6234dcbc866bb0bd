"""Host-side time of one driver-config job (hexapod B=4096, 20 fused steps): the enqueue time, the
wall time to a finished synchronize, and the HIP events around the kernels, for a few ways of issuing
and waiting. Tuning aid; one mode per process (device flags must precede the runtime's init).
  python tools/host_probe.py [plain|noevents|poll|graph|spin|idle|idle5]
(idle: 1 s of GPU idle, then the job as warmup and the timed job; idle5: the same with bench.py's
5-step warmup job; idle5spin: idle5 with the warmup's end polled on an event (the host thread kept
awake) before the synchronize; idle5spin2: also the timed job's end polled; idle5spin_noev: idle5spin without the events)"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "plain"
    label = mode
    if mode == "spin" or mode.startswith("spinflag"):  # hipDeviceScheduleSpin before the runtime initializes
        import importlib.util  # torch's own HIP runtime (same SONAME: the one every later library binds)
        tlib = os.path.join(os.path.dirname(importlib.util.find_spec("torch").origin), "lib", "libamdhip64.so")
        hip = ctypes.CDLL(tlib if os.path.exists(tlib) else "libamdhip64.so")
        print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(ctypes.c_uint(1)))
        label, mode = mode, mode[len("spinflag_"):] if mode.startswith("spinflag_") else mode
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
    warm = job
    if mode.startswith("idle5"):
        b.key_steps = 5
        warm = b.calls_launcher(5, stream=st, best=True)
        b.key_steps = K
        warm()
        torch.cuda.synchronize()
    if mode == "graph":
        gs = torch.cuda.Stream(dev)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(gs):
            j2 = b.calls_launcher(K, stream=gs, best=True)
            j2()
            torch.cuda.synchronize()
            with torch.cuda.graph(g, stream=gs):
                j2()
        torch.cuda.synchronize()
        job = g.replay
        for _ in range(3):
            job()
        torch.cuda.synchronize()
    enq, walls, evs = [], [], []
    for _ in range(10 if mode.startswith("idle") else 30):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if mode.startswith("idle"):
            time.sleep(1.0)
        warm()  # the warmup right before, as in bench.py
        if mode.startswith("idle5spin"):
            ew = torch.cuda.Event()
            ew.record(st)
            while not ew.query():
                pass
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        if mode not in ("noevents", "idle5spin_noev"):
            e0.record(st)
        job()
        if mode not in ("noevents", "idle5spin_noev"):
            e1.record(st)
        t1 = time.perf_counter()
        if mode in ("poll", "idle5spin2"):
            while not e1.query():
                pass
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        enq.append((t1 - t0) * 1e6)
        walls.append((t2 - t0) * 1e6)
        evs.append(e0.elapsed_time(e1) * 1e3 if mode not in ("noevents", "idle5spin_noev") else float("nan"))
    print(f"{label}: enqueue {np.median(enq):.1f} us, wall {np.median(walls):.1f} us (min {np.min(walls):.1f}), "
          f"events {np.median(evs):.1f} us -> {4096 * 20 / np.median(walls):.1f} M steps/s")


if __name__ == "__main__":
    main()
