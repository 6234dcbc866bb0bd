"""Wall time per launch of the H=1 batch under different launch schemes (tuning aid):
native loop with / without per-launch events, Python loop, HIP graph replay."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import hslabs_amd as H
    from hslabs_amd import synth

    B, K = int(os.environ.get("B", "4096")), int(os.environ.get("K", "200"))
    m = H.KinematicModel(os.path.join(ROOT, "models", "hexapod.xml"))
    b = H.DeviceBatch(m, synth.gen_params(B, "hexapod"), n_t=20, horizon=1)
    st = torch.cuda.current_stream()
    b.run_steps(20, stream=st)
    torch.cuda.synchronize()

    def wall(fn):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / K * 1e6

    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * K)]
    b.run_steps(K, stream=st, events=ev)
    torch.cuda.synchronize()
    kern = sum(ev[2 * i].elapsed_time(ev[2 * i + 1]) for i in range(K)) / K * 1e3
    print(f"native loop, no events     {wall(lambda: b.run_steps(K, stream=st)):8.1f} us/launch")
    print(f"native loop, events        {wall(lambda: b.run_steps(K, stream=st, events=ev)):8.1f} us/launch (event kernel avg {kern:.1f} us)")

    def pyloop():
        for s in range(K):
            b.k0 = s % 20
            b.run(stream=st, best=False, accumulate=True)
    print(f"python loop, no events     {wall(pyloop):8.1f} us/launch")
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        b.k0 = 0
        with torch.cuda.graph(g, stream=side):
            b.run_steps(K, stream=side)
    torch.cuda.synchronize()
    print(f"graph replay ({K} launches) {wall(g.replay):8.1f} us/launch")


if __name__ == "__main__":
    main()
