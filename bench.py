#!/usr/bin/env python3
"""Benchmark: batched control-loop steps/s on MI355X (BASELINE.json metric).

A bench "step" is one pass of the hot path over one batch: every rollout of
the batch advances one control-loop time step (pergen -> lik -> FK -> dynrec
-> ftsolver -> motor torques), i.e. `rollouts x horizon` control-loop steps.
Default workload = BASELINE.json configs[1]: hexapod.xml, 4096 rollouts per
GPU, horizon 1, fp64. Bench step s solves time step k = s mod n_t of every
rollout and accumulates positive work on the device, so 20 timed steps cover
exactly one reference cycle (n_t = 20, main.cpp:69) and the per-rollout COT
is the reference's measure_cot (player.cpp:269-285). After the timed steps
every rank min-reduces its best (COT, rollout id) key with ONE RCCL
all_reduce(MIN) of 8 bytes; that collective is inside the timed region.

Launch: python bench.py [--gpus N --steps K --warmup W]; N > 1 via
torch.distributed.run (one process per GPU, RCCL).

--sim benchmarks the closed-loop simulation instead (modelplayer::simulate_ode
with position control on ODE's QuickStep, hs_sim_step): a step is one
simulation step (play_dt) of every rollout; K steps run in one launch.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "batched control-loop steps/sec (hexapod.xml, 18-DoF) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6    # MI355X vector FP64 (spec), see DESIGN.md
# algorithmic HBM bytes per control-loop step = outputs
# tau 18*8 + contact forces 18*8 (+ 96 B of gait parameters amortized over H)
OUT_BYTES_PER_STEP = {"hexapod": 288, "spider": 288, "myant": 192}
PARAM_BYTES = 96


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rollouts", type=int, default=4096, help="rollouts per GPU")
    ap.add_argument("--horizon", type=int, default=1)
    ap.add_argument("--model", default="hexapod", choices=["hexapod", "spider", "myant"])
    ap.add_argument("--n_t", type=int, default=20)
    ap.add_argument("--curved", action="store_true")
    ap.add_argument("--fp32", action="store_true",
                    help="single-precision kernels (HS_PREC_F32), e.g. BASELINE configs[2]: --model spider "
                         "--rollouts 16384 --horizon 32 --fp32")
    ap.add_argument("--mixed", action="store_true",
                    help="BASELINE configs[4]: myant.xml + hexapod.xml 50/50, interleaved, one launch")
    ap.add_argument("--launch", choices=["fused", "steps"], default="fused",
                    help="fused: the K control steps in launches of up to 512k wavefronts over (step, rollout) "
                         "(hs_run_calls, every step its own output rows); steps: one launch per step "
                         "(hs_run_steps, the online loop)")
    ap.add_argument("--sim", action="store_true",
                    help="closed-loop simulation (PD control + ODE QuickStep, 20 SOR iterations) steps/s")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    return ap.parse_args()


def cpu_baseline(model_names, n_t, horizon, seconds, threads):
    """Oracle (CPU restatement, tree basis = same algorithm as the kernel) on a bounded sample
    (model_names: one model, or the models of a mixed batch in equal shares)."""
    from oracle import oracle as O
    from hslabs_amd import synth

    threads = max(1, min(threads, os.cpu_count() or 1))
    chunk = 256 * threads // len(model_names)
    work = []
    for name in model_names:
        om = O.Model(os.path.join(ROOT, "models", f"{name}.xml"))
        arr = synth.gen_params(chunk, name)
        work.append((om, [O.GaitParams(torso_pos=tuple(r["torso_pos"]), torso_angles=tuple(r["torso_angles"]),
                                       step_duration=float(r["step_duration"]), period=float(r["period"]),
                                       step_length=float(r["step_length"]), step_height=float(r["step_height"]),
                                       curvature=float(r["curvature"]), foot_shift_type=int(r["foot_shift_type"]),
                                       foot_shift=float(r["foot_shift"])) for r in arr]))
    model_name = "+".join(model_names)

    def timed(nthr, budget):
        done, t0 = 0, time.perf_counter()
        while True:
            for om, gaits in work:
                O.batch(om, gaits, n_t, 0, horizon, basis=O.BASIS_TREE, n_threads=nthr)
                done += len(gaits) * horizon
            el = time.perf_counter() - t0
            if el >= budget:
                return done / el, done, el

    single, _, _ = timed(1, min(2.0, seconds / 4))
    rate, done, el = timed(threads, seconds)
    return {"value": round(rate, 1), "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"{done} control-loop steps ({model_name}, H={horizon}, synthetic gaits) in {el:.1f}s, "
                      f"oracle tree-basis restatement, g++ -O2, std::thread x{threads}; "
                      f"single-thread {single:.1f} steps/s",
            "single_thread": round(single, 1)}


SIM_METRIC = "closed-loop simulation steps/sec (position control + ODE QuickStep SOR-LCP, 20 iterations)"


def sim_cpu_baseline(model, name, sb, seconds, threads):
    """Oracle QuickStep restatement on a bounded sample of the same batch (same tables/states)."""
    from oracle import oracle as O

    threads = max(1, min(threads, os.cpu_count() or 1))
    om = O.Model(os.path.join(ROOT, "models", f"{name}.xml"))
    nb = min(sb.B, 4 * threads)
    qt = sb.tables.q[:nb].cpu().numpy().astype(np.float64)
    dqt = sb.tables.dq[:nb].cpu().numpy().astype(np.float64)
    tt = sb.tables.tau[:nb].cpu().numpy().astype(np.float64)
    body0 = sb.body[:nb].cpu().numpy().astype(np.float64)
    P = O.SimParams()

    def timed(nthr, budget):
        body = body0.copy()
        seed = np.zeros(nb, np.uint32)
        tsi = np.full(nb, 2, np.int32)
        done, t0 = 0, time.perf_counter()
        while True:
            O.sim_batch(om, P, sb.n_t, qt, dqt, tt, body, seed, tsi, 10, nthr)
            done += nb * 10
            el = time.perf_counter() - t0
            if el >= budget:
                return done / el, done, el

    single, _, _ = timed(1, min(2.0, seconds / 4))
    rate, done, el = timed(threads, seconds)
    return {"value": round(rate, 1), "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"{done} simulation steps ({name}, {nb} rollouts of the batch, 10-step calls) in {el:.1f}s, "
                      f"oracle ODE-QuickStep restatement (double, as ODE computes), g++ -O2, std::thread x{threads}; "
                      f"single-thread {single:.1f} steps/s",
            "single_thread": round(single, 1)}


def main_sim(args, torch, dist, world, rank, dev):
    import hslabs_amd as H
    from hslabs_amd import synth

    B = args.rollouts
    model = H.KinematicModel(os.path.join(ROOT, "models", f"{args.model}.xml"))
    dtype = torch.float32 if args.fp32 else torch.float64
    sb = H.SimBatch(model, synth.gen_sim_params(B, args.model, id0=rank * B), device=dev, dtype=dtype)
    stream = torch.cuda.current_stream(dev)
    sb.step(args.warmup, stream=stream, outputs=())
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    sb.step(args.steps, stream=stream, outputs=())  # one launch, K steps (state stays in LDS)
    ev1.record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed, ev0.elapsed_time(ev1)], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])
    finite = bool(torch.isfinite(sb.body).all().item())
    if rank == 0:
        nmj = model.nmj
        # per rollout-step the kernel must read the controller row (q0, dq0, tau_ff: 3 nmj reals);
        # the body state (n x 13 reals) crosses HBM once per launch in each direction
        w = 4 if args.fp32 else 8
        alg_bytes = B * (args.steps * 3 * nmj * w + 2 * model.n_parts * 13 * w)
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        out = {
            "metric": SIM_METRIC, "value": round(B * args.steps * world / elapsed, 1), "unit": "steps/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 4), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "f32" if args.fp32 else "f64",
            "data": "synthetic (splitmix64 gait parameters around pgs id 8, period 3 -> n_t 300; SURVEY.md 8d)",
            "config": {"workload": f"{args.model}.xml B={B}/GPU closed-loop simulation, play_dt .01, QuickStep 20 "
                                   f"iterations, {args.steps} steps per launch, "
                                   f"{'fp32' if args.fp32 else 'fp64'} (SURVEY.md 8f row 4)",
                       "rollouts_per_gpu": B, "parallelism": f"rollout-sharded x{world}, no collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "hs_sim_kernel",
                         "kernel_ms": round(kern_ms, 5), "alg_bytes_per_launch": alg_bytes},
            "finite_state": finite,
        }
        out["cpu_baseline"] = None if (args.no_cpu or world > 1) else sim_cpu_baseline(
            model, args.model, sb, args.cpu_seconds, args.cpu_threads)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.sim:
        return main_sim(args, torch, dist, world, rank, dev)

    import hslabs_amd as H
    from hslabs_amd import synth

    B, Hh, n_t = args.rollouts, args.horizon, args.n_t
    id0 = rank * B
    outs = ("tau", "cf", "work_cot", "flags")
    dtype = torch.float32 if args.fp32 else torch.float64
    prec = "fp32" if args.fp32 else "fp64"
    width = 0.5 if args.fp32 else 1.0  # fp32 halves the output and parameter bytes
    if args.mixed:
        model_names = list(synth.MIXED_MODELS)
        models = [H.KinematicModel(os.path.join(ROOT, "models", f"{n}.xml")) for n in model_names]
        params, midx = synth.gen_mixed(B, id0=id0, curved=args.curved)
        fused = args.launch == "fused"
        rows = Hh * max(args.steps, args.warmup) if fused else Hh  # fused: one output row per step
        batch = H.MixedBatch(models, midx, params, n_t=n_t, k0=0, horizon=rows, outputs=outs, device=dev,
                             rollout_id_base=id0, dtype=dtype)
        out_bytes = float(np.mean([OUT_BYTES_PER_STEP[model_names[k]] for k in midx]))
        workload = (f"myant.xml+hexapod.xml 50/50 interleaved B={B}/GPU H={Hh} n_t={n_t} {prec} "
                    f"(BASELINE configs[4])")
        traffic_key = f"mixed B={B} H={Hh} {prec}"
    else:
        model_names = [args.model]
        model = H.KinematicModel(os.path.join(ROOT, "models", f"{args.model}.xml"))
        params = synth.gen_params(B, args.model, id0=id0, curved=args.curved)
        fused = args.launch == "fused"
        rows = Hh * max(args.steps, args.warmup) if fused else Hh  # fused: one output row per step
        batch = H.DeviceBatch(model, params, n_t=n_t, k0=0, horizon=rows, outputs=outs, device=dev,
                              rollout_id_base=id0, dtype=dtype)
        out_bytes = OUT_BYTES_PER_STEP[args.model]
        if args.model == "hexapod" and Hh == 1 and not args.fp32 and B == 4096:
            cfg = "configs[1]"
        elif args.model == "hexapod" and Hh == 1 and not args.fp32 and B * world == 262144:
            cfg = "configs[3]"  # 262144 rollouts sharded over the ranks
        elif args.model == "spider" and Hh == 32 and args.fp32 and B == 16384:
            cfg = "configs[2]"
        else:
            cfg = "custom"
        workload = f"{args.model}.xml B={B}/GPU H={Hh} n_t={n_t} {prec} (BASELINE {cfg})"
        traffic_key = f"{args.model} B={B} H={Hh}" + (" fp32" if args.fp32 else "")
    out_bytes *= width
    stream = torch.cuda.current_stream(dev)

    # warmup (untimed): the same native launch loop as the timed region
    batch.work_cot.zero_()
    batch.k0 = 0

    def run_k(k, best=False):
        if fused:
            batch.run_calls(k, call_horizon=Hh, stream=stream, best=best, accumulate=True)
        else:
            batch.run_steps(k, stream=stream, best=False, accumulate=True)

    run_k(args.warmup)
    torch.cuda.synchronize()
    batch.work_cot.zero_()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    from hslabs_amd import dist as hdist

    def best_key_local():
        return hdist.best_key(batch.work_cot[:, 1], id0)

    def job_key():
        # fused: the work reduce already took the shard's min key (atomicMin, hs_best_key_encode's
        # encoding); per-step launches: the key of the accumulated COTs, taken after the last step
        if fused:
            return batch.best_key ^ hdist._FLIP
        return best_key_local()

    # warm the key computation and the collective too (first use loads code objects)
    warm = job_key()
    hdist.reduce_best(warm)
    batch.reset_best()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # K steps, k0 = (s * H) mod n_t: fused (a setup pass, launches of up to 512k wavefronts, the in-order work
    # sum) or the native loop of K launches. Two HIP events on the launch stream bracket them
    # (per-launch events would drain the queue between kernels and add ~8 us each): GPU time per
    # step of the batch = GPU time / K.
    batch.k0 = 0
    ev0.record(stream)
    run_k(args.steps, best=True)
    ev1.record(stream)
    key = hdist.reduce_best(job_key())  # the single RCCL collective (8 B)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])
    best_cot, best_id = hdist.decode(key)
    check = hdist.reduce_best(best_key_local())  # untimed: the device key equals the host-side encoding
    if int(check.item()) != int(key.item()):
        raise RuntimeError(f"best key mismatch: kernel {int(key.item())} vs torch {int(check.item())}")
    nan_steps = int(((batch.flags & 8) != 0).sum().item())

    if rank == 0:
        steps_total = B * Hh * args.steps * world
        value = steps_total / elapsed
        ms_per_step = 1e3 * elapsed / args.steps
        alg_bytes = B * Hh * (out_bytes + width * PARAM_BYTES / Hh)
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        traffic = fp64_flops = None
        tf = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(tf):
            try:
                j = json.load(open(tf))
                if j.get("workload") == traffic_key:
                    traffic = j.get("hbm_bytes_per_launch")
                    fp64_flops = j.get("fp64_lane_flops_per_launch")
            except Exception:
                traffic = fp64_flops = None
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32" if args.fp32 else "f64",
            "data": "synthetic (splitmix64 gait parameters around pgs id 8; SURVEY.md 8d)",
            "config": {"workload": workload,
                       "rollouts_per_gpu": B, "horizon": Hh, "n_t": n_t,
                       "launch": ("fused: K calls in launches of up to 512k wavefronts over (step, rollout), every step "
                                  "its own output rows (hs_run_calls)") if fused else
                                 "one launch per step (hs_run_steps)",
                       "parallelism": f"rollout-sharded x{world}, 1 RCCL all_reduce(MIN, 8 B) per job"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "hs_rollout_kernel", "kernel_ms": round(kern_ms, 5),
                         "alg_bytes_per_launch": alg_bytes},
            # the bound that binds: FP64 VALU issue, from the committed PMC instruction counts of this
            # workload (profiles/pmc_traffic.json) over the live kernel time (inactive lanes included)
            "fp64_valu": None if fp64_flops is None else {
                "issued_tflops": round(fp64_flops / (kern_ms * 1e-3) / 1e12, 3), "peak_tflops": FP64_PEAK_TFLOPS,
                "frac": fp64_flops / (kern_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS},
            "best_rollout": {"id": best_id, "cot": best_cot},
            "nan_steps": nan_steps,
        }
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(model_names, n_t, Hh, args.cpu_seconds, args.cpu_threads)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
