#!/usr/bin/env python3
"""Benchmark: batched control-loop steps/s on MI355X (BASELINE.json metric).

A bench "step" is one pass of the hot path over one batch: every rollout of
the batch advances one control-loop time step (pergen -> lik -> FK -> dynrec
-> ftsolver -> motor torques), i.e. `rollouts x horizon` control-loop steps.
Bench step s solves time step k = s mod n_t of every rollout and accumulates
positive work on the device (n_t = 20, main.cpp:69).

Workloads (BASELINE.json configs):
  N = 1, no --rollouts      configs[1]: hexapod.xml, 4096 rollouts, horizon 1, fp64
  N > 1, no --rollouts      configs[3]: 262144 hexapod rollouts sharded over the N ranks in
                            contiguous id ranges (262144 / N per GPU), "scaling": "strong"
  --rollouts B              B rollouts per GPU ("weak"); --total-rollouts T: T sharded ("strong")
  --model spider --rollouts 16384 --horizon 32 --fp32   configs[2];  --mixed   configs[4]

After the timed steps each rank's best-rollout key (the work reduce's atomicMin; the selection
COT of hs_best_key_cot, normalized to one cycle) is all-reduced with ONE RCCL all-reduce(MIN) of
8 bytes issued by libhslabs itself (hs_comm_reduce_best); that collective is inside the timed
region.

Launch: `python bench.py --gpus N --steps K --warmup W`. With N > 1 and no torch.distributed
environment this process starts `torch.distributed.run` with N ranks (one per GPU) as a child
before touching the GPU and exits with its status; under torchrun every rank checks
WORLD_SIZE == N.

--sim benchmarks the closed-loop simulation instead (modelplayer::simulate_ode
with position control on ODE's QuickStep, hs_sim_step): a step is one
simulation step (play_dt) of every rollout; K steps run in one launch.

--stub-cpu (tests/test_bench_launcher.py): the same launcher, sharding, key encoding and
max-over-ranks timing on CPU ranks over gloo, with a stub in place of the GPU kernel.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "batched control-loop steps/sec (hexapod.xml, 18-DoF) at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6    # MI355X vector FP64 (AMD spec; the guide lists FP32 157.3 = 2x)
# algorithmic HBM bytes per control-loop step = outputs
# tau 18*8 + contact forces 18*8 (+ 96 B of gait parameters amortized over H)
OUT_BYTES_PER_STEP = {"hexapod": 288, "spider": 288, "myant": 192}
PARAM_BYTES = 96
CONFIG3_TOTAL = 262144     # BASELINE configs[3]


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--rollouts", type=int, default=None,
                    help="rollouts per GPU (default: 4096 = configs[1] at N = 1; configs[3]'s 262144 / N at N > 1)")
    ap.add_argument("--total-rollouts", type=int, default=None, help="rollouts of the whole job, sharded over the ranks")
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
    ap.add_argument("--forces", action="store_true",
                    help="solve_forces (contact forces given motor torques, ftsolver.cpp:331-378) steps/s: "
                         "the K steps' torques from an untimed control-loop run, then K fused steps "
                         "(hs_run_forces_calls)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=None, help="default: the host cores this process may use")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--stub-cpu", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ---------------------------------------------------------------------------------------------
# launcher and job layout
# ---------------------------------------------------------------------------------------------
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(args) -> int:
    """N ranks via torch.distributed.run, started as a child process before this process has made
    any GPU call (never exec: the parent only parsed arguments). Returns the job's exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def job_layout(args, world: int, rank: int) -> dict:
    """This rank's contiguous rollout range and the workload's BASELINE label."""
    from hslabs_amd.dist import shard

    if args.rollouts is not None and args.total_rollouts is not None:
        raise SystemExit("give --rollouts (per GPU) or --total-rollouts (sharded), not both")
    if args.total_rollouts is not None:
        total, scaling = args.total_rollouts, "strong"
    elif args.rollouts is not None:
        total, scaling = args.rollouts * world, "weak"
    elif world == 1:
        total, scaling = 4096, "weak"           # configs[1]
    else:
        total, scaling = CONFIG3_TOTAL, "strong"  # configs[3]
    if total < world:
        raise SystemExit(f"{total} rollouts cannot be sharded over {world} ranks")
    id0, count = shard(total, world, rank)
    std = args.model == "hexapod" and args.horizon == 1 and not args.fp32 and not args.mixed and not args.curved
    if std and world == 1 and total == 4096:
        cfg = "configs[1]"
    elif std and total == CONFIG3_TOTAL and scaling == "strong":
        cfg = "configs[3]"
    elif args.model == "spider" and args.horizon == 32 and args.fp32 and total == 16384 * world and not args.mixed:
        cfg = "configs[2]"
    elif args.mixed:
        cfg = "configs[4]"
    else:
        cfg = "custom"
    return dict(total=total, id0=id0, B=count, scaling=scaling, cfg=cfg)


def host_cpus() -> dict:
    """What this process may run on: nproc, the affinity mask, a cgroup CPU quota (GPU boxes give
    each lease a share of a large host), and the CPU model."""
    info = {"nproc": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except Exception:
        info["affinity"] = info["nproc"]
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) / int(p)))
    except Exception:
        pass
    info["cgroup_quota"] = quota
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    info["model"] = model
    usable = min(info["affinity"], quota or info["affinity"])
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 1:  # the GPU box exports its CPU share here (16)
        usable = min(usable, int(omp))
    info["usable"] = max(1, usable)
    return info


# ---------------------------------------------------------------------------------------------
# CPU baseline (rank 0, N = 1): the oracle's tree-basis restatement, -O3 -march=native
# ---------------------------------------------------------------------------------------------
def _oracle_gaits(O, arr):
    return [O.GaitParams(torso_pos=tuple(r["torso_pos"]), torso_angles=tuple(r["torso_angles"]),
                         step_duration=float(r["step_duration"]), period=float(r["period"]),
                         step_length=float(r["step_length"]), step_height=float(r["step_height"]),
                         curvature=float(r["curvature"]), foot_shift_type=int(r["foot_shift_type"]),
                         foot_shift=float(r["foot_shift"])) for r in arr]


def step_kernel(models, fused=True, fp32=False, forces=False):
    """the step launch's kernel for this workload, as the native library routes it (hs_capi.cpp
    limb_eligible, hs_run_steps, hs_run_forces_calls): the limb-lane kernel for the models of its class"""
    env = os.environ
    limb = env.get("HS_LIMB", "1") != "0" and all(m.limb_lane_ok for m in models)
    if fp32:
        limb = limb and env.get("HS_LIMB_F32", "1") != "0" and not forces
    if not fused:
        limb = limb and env.get("HS_LIMB_ONLINE") == "1"
    if forces:
        return "hs_limb_kernel<NM, true>" if limb else "hs_rollout_kernel<NM, true, 0>"
    if limb:
        return "hs_limb_kernel<NM, false>"
    return "hs_rollout_kernel<NM, false, 1>" if fused else "hs_rollout_kernel<NM, false, 0>"


def cpu_baseline(model_names, n_t, horizon, seconds, threads=None):
    """Oracle (CPU restatement, tree basis: the reference's FullPivLU / ColPivQR rank loop on the
    tree-built null basis) on a bounded sample, model_names = one model or a mixed batch's models in
    equal shares. Built -O3 -march=native for this host's CPU; the contract-off -O2
    build (the parity checker) if that compile fails."""
    from oracle import oracle as O
    from hslabs_amd import synth

    cpus = host_cpus()
    threads = max(1, threads or cpus["usable"])
    build = "g++ -O3 -march=native"
    try:
        L, _ = O.perf_lib(cpus["model"])
    except Exception as e:  # no compiler / compile failed: say so and time the parity build
        L, build = O.lib(), f"g++ -O2 -ffp-contract=off (native build failed: {type(e).__name__})"
    chunk = max(64, 256 * threads // len(model_names))
    work = []
    for name in model_names:
        om = O.Model(os.path.join(ROOT, "models", f"{name}.xml"), L=L)
        work.append((om, _oracle_gaits(O, synth.gen_params(chunk, name))))
    model_name = "+".join(model_names)

    def timed(nthr, budget):
        done, t0 = 0, time.perf_counter()
        while True:
            for om, gaits in work:
                O.batch(om, gaits, n_t, 0, horizon, basis=O.BASIS_TREE, n_threads=nthr, L=L)
                done += len(gaits) * horizon
            el = time.perf_counter() - t0
            if el >= budget:
                return done / el, done, el

    single, _, _ = timed(1, min(2.0, seconds / 4))
    rate, done, el = timed(threads, seconds)
    return {"value": round(rate, 1), "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"{done} control-loop steps ({model_name}, H={horizon}, synthetic gaits of the bench's "
                      f"distribution) in {el:.1f}s: oracle tree-basis restatement (Eigen-style rank loop), {build}, "
                      f"std::thread x{threads}; single-thread {single:.1f} steps/s",
            "single_thread": round(single, 1),
            "host": {"cpu_model": cpus["model"], "nproc": cpus["nproc"], "affinity": cpus["affinity"],
                     "cgroup_quota": cpus["cgroup_quota"], "threads_used": threads,
                     "why": "threads = the CPUs this process may use (affinity, cgroup quota, OMP_NUM_THREADS "
                            "share of the box), not nproc, which counts the whole host"}}


SIM_METRIC = "closed-loop simulation steps/sec (position control + ODE QuickStep SOR-LCP, 20 iterations)"


def sim_cpu_baseline(model, name, sb, seconds, threads=None):
    """Oracle QuickStep restatement on a bounded sample of the same batch (same tables/states)."""
    from oracle import oracle as O

    threads = max(1, threads or host_cpus()["usable"])
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

    B = args.rollouts or 4096
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

    def timed():
        ev0.record(stream)
        sb.step(args.steps, stream=stream, outputs=())  # one launch, K steps (state stays in LDS)
        ev1.record(stream)

    elapsed = timed_window(timed, torch.cuda.synchronize)
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


FORCES_METRIC = "solve_forces steps/sec: contact forces given motor torques (ftsolver.cpp:331-378)"


def forces_cpu_baseline(name, params, tau, n_t, seconds, threads=None):
    """Oracle solve_forces (the reference's B with the torque rows, torso columns out, a column-by-
    column Householder QR with the kernel's rank rule; oracle/hs_oracle.cpp) on a bounded sample of
    the same batch and torques, built and threaded like the control loop's baseline (cpu_baseline):
    g++ -O3 -march=native for this host's CPU, std::thread over the rollouts."""
    from oracle import oracle as O

    cpus = host_cpus()
    threads = max(1, threads or cpus["usable"])
    build = "g++ -O3 -march=native"
    try:
        L, _ = O.perf_lib(cpus["model"])
    except Exception as e:
        L, build = O.lib(), f"g++ -O2 -ffp-contract=off (native build failed: {type(e).__name__})"
    om = O.Model(os.path.join(ROOT, "models", f"{name}.xml"), L=L)
    gaits = _oracle_gaits(O, params)
    tau = np.ascontiguousarray(tau, dtype=np.float64)

    def timed(nthr, budget):
        done, t0 = 0, time.perf_counter()
        while True:
            O.forces_batch(om, gaits, tau, n_t=n_t, n_threads=nthr, L=L)
            done += tau.shape[0] * tau.shape[1]
            el = time.perf_counter() - t0
            if el >= budget:
                return done / el, done, el

    single, _, _ = timed(1, min(2.0, seconds / 4))
    rate, done, el = timed(threads, seconds)
    return {"value": round(rate, 1), "unit": "steps/s", "cores": threads, "kind": "port",
            "sample": f"{done} solve_forces steps ({name}, {tau.shape[0]} rollouts of the batch x {tau.shape[1]} steps, "
                      f"the batch's own torques) in {el:.1f}s: oracle least squares (Householder QR of the reference's "
                      f"B with the torque rows), {build}, std::thread x{threads}; single-thread {single:.1f} steps/s",
            "single_thread": round(single, 1),
            "host": {"cpu_model": cpus["model"], "threads_used": threads}}


def main_forces(args, torch, dist, world, rank, dev):
    """solve_forces on the control loop's workload: B rollouts, K steps of the
    motor torques the control loop computed for them (untimed), then the K steps of
    forcetorquesolver::solve_forces fused (hs_run_forces_calls) in the timed region."""
    import hslabs_amd as H
    from hslabs_amd import capi, synth

    lay = job_layout(args, world, rank)
    B, K, n_t = lay["B"], args.steps, args.n_t
    model = H.KinematicModel(os.path.join(ROOT, "models", f"{args.model}.xml"))
    params = synth.gen_params(B, args.model, id0=lay["id0"], curved=args.curved)
    rows = max(args.steps, args.warmup)
    ctl = H.DeviceBatch(model, params, n_t=n_t, k0=0, horizon=rows, outputs=("tau", "cf"), device=dev,
                        rollout_id_base=lay["id0"])
    ctl.run_calls(rows, call_horizon=1)  # the torques (and, for the check, the contact forces)
    stream = torch.cuda.current_stream(dev)
    fb = H.DeviceBatch(model, params, n_t=n_t, k0=0, horizon=K, outputs=("cf", "flags"), device=dev,
                       rollout_id_base=lay["id0"])
    job = fb.forces_launcher(ctl.tau[:, :K], K, stream=stream)
    warm_job = None
    if args.warmup:
        wb = H.DeviceBatch(model, params, n_t=n_t, k0=0, horizon=args.warmup, outputs=("cf",), device=dev)
        warm_job = wb.forces_launcher(ctl.tau[:, :args.warmup], args.warmup, stream=stream)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if warm_job:
        warm_job()
    done_ev = torch.cuda.Event()
    done_ev.record(stream)
    while not done_ev.query():
        pass
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    def timed():
        ev0.record(stream)
        job()
        ev1.record(stream)

    elapsed = timed_window(timed, torch.cuda.synchronize)
    kern_ms = ev0.elapsed_time(ev1) / K
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])
    # untimed check (playerexperim.cpp:95-121): the forces that realise the computed torques are the
    # computed contact forces
    cf, ref = fb.cf[:, :K].double(), ctl.cf[:, :K].double()
    err = float(((cf - ref).abs().amax(dim=2) / ref.abs().amax(dim=2).clamp(min=1)).max().item())
    general = int(((fb.flags[:, :K] & capi.HS_FLAG_GENERAL) != 0).sum().item())
    if rank == 0:
        nmj, nf = model.nmj, model.nfeet
        step_bytes = 8 * (nmj + 3 * nf) + PARAM_BYTES  # torques in, forces of all feet out, the gait record
        alg_bytes = B * step_bytes
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        lib = dict(capi.LOADED)
        pmc, pmc_note = pmc_for(f"forces {args.model} B={B}", lib["sha256"], "pmc_traffic_forces.json")
        traffic = None if pmc is None else int(round(pmc["hbm_bytes_per_step"] * B / pmc["rollouts"]))
        out = {
            "metric": FORCES_METRIC, "value": round(lay["total"] * K / elapsed, 1), "unit": "steps/s",
            "n_gpus": world, "steps": K, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / K, 4),
            "higher_is_better": True, "scaling": lay["scaling"], "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (splitmix64 gait parameters around pgs id 8; the torques the control loop computed)",
            "config": {"workload": f"{args.model}.xml B={B}/GPU, {K} fused solve_forces steps (hs_run_forces_calls), "
                                   f"n_t={n_t} fp64 (SURVEY.md 8f row 1)", "rollouts_per_gpu": B,
                       "parallelism": f"rollout-sharded x{world}, no collective"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_over_algorithmic": None if traffic is None else round(traffic / alg_bytes, 3),
                         "traffic_note": pmc_note, "kernel": step_kernel([model], forces=True),
                         "kernel_ms": round(kern_ms, 5), "alg_bytes_per_launch": alg_bytes,
                         "alg_bytes_per_step": step_bytes},
            "check": {"max_rel_cf_vs_control_loop": err, "general_steps": general},
            "lib": lib,
        }
        nb = min(B, 256)
        out["cpu_baseline"] = None if (args.no_cpu or world > 1) else forces_cpu_baseline(
            args.model, params[:nb], ctl.tau[:nb, :K].cpu().numpy(), n_t, args.cpu_seconds, args.cpu_threads)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------------------------
# measurement files committed under profiles/ (never read from /root/reference)
# ---------------------------------------------------------------------------------------------
def _profile_json(name):
    path = os.path.join(ROOT, "profiles", name)
    if not os.path.exists(path):
        return None
    try:
        return json.load(open(path))
    except Exception:
        return None


def pmc_for(traffic_key, lib_sha, name="pmc_traffic.json"):
    """HBM bytes and issued FP64 lane ops per step of the batch from the committed PMC summary
    (tools/gpu_pmc.sh + tools/pmc_summary.py), only when it was taken on the library this process
    loaded (same sha256 prefix); else None and the reason."""
    j = _profile_json(name)
    if j and "workloads" in j:  # one summary per workload (configs[1], [2], [4]), each keyed to its library
        j = j["workloads"].get(traffic_key)
    if not j or j.get("workload") != traffic_key:
        return None, "no PMC summary for this workload"
    if j.get("lib_sha256") != lib_sha:
        return None, f"PMC summary taken on library {j.get('lib_sha256')}, this run loaded {lib_sha}: stale, refused"
    return j, None


def flops_for(workload_key):
    """Algorithmic FP64 FLOPs per control-loop step of this workload: the oracle's counting build
    on the kernel's own path (tools/flop_count.py -> profiles/flops.json)."""
    j = _profile_json("flops.json")
    if not j:
        return None
    return (j.get("workloads") or {}).get(workload_key)


# ---------------------------------------------------------------------------------------------
# the timed window (every mode)
# ---------------------------------------------------------------------------------------------
def timed_window(run, sync, clock=time.perf_counter):
    """The timed region of every bench mode: a clock read, the job (its kernels and, with N > 1 ranks,
    the one best-key all-reduce the control-loop job issues), the device synchronize, a clock read.
    No other collective runs between the two reads: the ranks line up on a
    barrier BEFORE the first read, and the slowest rank is taken AFTER the second by a MAX all-reduce
    of the per-rank elapsed times."""
    t0 = clock()
    run()
    sync()
    return clock() - t0


class CollectiveCounter:
    """--stub-cpu instrumentation: counts the torch.distributed collectives issued and snapshots the
    count at each clock read, so tests/test_bench_launcher.py can assert exactly one collective
    inside the timed window."""
    NAMES = ("barrier", "all_reduce", "broadcast", "all_gather", "all_gather_object", "broadcast_object_list",
             "reduce", "reduce_scatter", "all_to_all", "gather", "scatter")

    def __init__(self, dist):
        self.n, self.reads = 0, []
        for name in self.NAMES:
            f = getattr(dist, name, None)
            if f is not None:
                setattr(dist, name, self._wrap(f))

    def _wrap(self, f):
        def g(*a, **k):
            self.n += 1
            return f(*a, **k)
        return g

    def clock(self):
        self.reads.append(self.n)
        return time.perf_counter()

    def in_window(self):
        return self.reads[1] - self.reads[0]


# ---------------------------------------------------------------------------------------------
# the control-loop bench
# ---------------------------------------------------------------------------------------------
def main_stub(args, world, rank):
    """--stub-cpu: launcher/sharding/key/timing skeleton on CPU ranks (gloo). The stub 'kernel'
    gives each rollout the work of a cycle = period * step_height (a deterministic, positive number)
    so the test can recompute the global winner; nothing here is the product's arithmetic."""
    import torch
    import torch.distributed as dist

    from hslabs_amd import dist as hdist
    from hslabs_amd import synth

    lay = job_layout(args, world, rank)
    params = synth.gen_params(lay["B"], args.model, id0=lay["id0"])
    counter = CollectiveCounter(dist)
    if world > 1:
        dist.barrier()
    res = {}

    def job():
        work = torch.from_numpy(params["period"] * params["step_height"] * (args.steps / args.n_t))
        cot = hdist.select_cot(work, torch.from_numpy(params["step_length"]), 22.0, args.n_t, args.steps)
        res["key"] = hdist.reduce_best(hdist.best_key(cot, lay["id0"]))

    elapsed = timed_window(job, lambda: None, counter.clock)
    key = res["key"]
    t = torch.tensor([elapsed], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    shards = [None] * world
    if world > 1:
        dist.all_gather_object(shards, (rank, lay["id0"], lay["B"], os.getpid()))
    else:
        shards = [(rank, lay["id0"], lay["B"], os.getpid())]
    c, rid = hdist.decode(key)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": lay["total"] * args.steps / float(t[0]), "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "scaling": lay["scaling"],
                          "config": {"workload": f"stub {lay['cfg']}", "total_rollouts": lay["total"]},
                          "stub_shards": shards, "best_rollout": {"id": rid, "cot": c},
                          "collectives_in_timed_window": counter.in_window()}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(args))  # N ranks, one per GPU; nothing here has touched the GPU

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU expected")
    if args.stub_cpu:
        if world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            dist.init_process_group("gloo")
        return main_stub(args, world, rank)
    if world > 1:
        torch.cuda.set_device(local)
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    if args.sim:
        return main_sim(args, torch, dist, world, rank, dev)
    if args.forces:
        return main_forces(args, torch, dist, world, rank, dev)

    import hslabs_amd as H
    from hslabs_amd import capi, synth
    from hslabs_amd import dist as hdist

    lay = job_layout(args, world, rank)
    B, Hh, n_t, id0 = lay["B"], args.horizon, args.n_t, lay["id0"]
    outs = ("tau", "cf", "work_cot", "flags")
    dtype = torch.float32 if args.fp32 else torch.float64
    prec = "fp32" if args.fp32 else "fp64"
    width = 0.5 if args.fp32 else 1.0  # fp32 halves the output and parameter bytes
    fused = args.launch == "fused"
    rows = Hh * max(args.steps, args.warmup) if fused else Hh  # fused: one output row per step
    if args.mixed:
        model_names = list(synth.MIXED_MODELS)
        models = [H.KinematicModel(os.path.join(ROOT, "models", f"{n}.xml")) for n in model_names]
        params, midx = synth.gen_mixed(B, id0=id0, curved=args.curved)
        batch = H.MixedBatch(models, midx, params, n_t=n_t, k0=0, horizon=rows, outputs=outs, device=dev,
                             rollout_id_base=id0, dtype=dtype)
        out_bytes = float(np.mean([OUT_BYTES_PER_STEP[model_names[k]] for k in midx]))
        mass = torch.tensor([models[k].total_mass for k in midx], dtype=torch.float64, device=dev)
        wl_name = "myant.xml+hexapod.xml 50/50 interleaved"
        traffic_key = f"mixed B={B} H={Hh} {prec}"
    else:
        model_names = [args.model]
        model = H.KinematicModel(os.path.join(ROOT, "models", f"{args.model}.xml"))
        models = [model]
        params = synth.gen_params(B, args.model, id0=id0, curved=args.curved)
        batch = H.DeviceBatch(model, params, n_t=n_t, k0=0, horizon=rows, outputs=outs, device=dev,
                              rollout_id_base=id0, dtype=dtype)
        out_bytes = OUT_BYTES_PER_STEP[args.model]
        mass = model.total_mass
        wl_name = f"{args.model}.xml" + (" curved" if args.curved else "")
        traffic_key = f"{args.model} B={B} H={Hh}" + (" fp32" if args.fp32 else "")
    shard_txt = f"B={B}/GPU" if lay["scaling"] == "weak" else f"{lay['total']} rollouts / {world} GPU (this rank {B})"
    workload = f"{wl_name} {shard_txt} H={Hh} n_t={n_t} {prec} (BASELINE {lay['cfg']})"
    out_bytes *= width
    stream = torch.cuda.current_stream(dev)
    L = capi.load()
    lib = dict(capi.LOADED)

    comm = None
    if world > 1:  # the job's RCCL communicator for the best-key all-reduce (hs_comm_*, untimed setup)
        uid = [H.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = H.Comm(world, rank, uid[0])

    def launcher_k(k, best):
        """a job of k steps (the native launches), its arguments resolved before the clock starts"""
        batch.key_steps = k * Hh
        if fused:
            return batch.calls_launcher(k, call_horizon=Hh, stream=stream, best=best, accumulate=True)

        def steps():
            batch.key_steps = k * Hh
            batch.run_steps(k, stream=stream, best=best, accumulate=True)
        return steps

    # warmup (untimed): the same native launches as the timed region, and the collective once. Every
    # host-side preparation of the timed job happens before it, so the timed job follows the warmup
    # with no more idle GPU time than the barrier and the synchronize (idle time lowers the clocks the
    # next job starts at: tools/sync_probe.py)
    batch.k0 = 0
    warm = launcher_k(args.warmup, best=True)
    job = launcher_k(args.steps, best=True)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    batch.work_cot.zero_()
    batch.reset_best()
    warm()
    if comm is not None:
        comm.reduce_best(batch.best_key, stream)
    batch.work_cot.zero_()  # queued behind the warmup on the same stream
    batch.reset_best()
    # wait for the warmup by polling an event instead of a blocking synchronize: a host thread that
    # slept through the wait enqueues the timed job at ~half speed (tools/host_probe.py idle5 vs
    # idle5spin: 30-35 -> 17-18 us before the first launch; profiles/r02_v9_host_probe.txt)
    warm_done = torch.cuda.Event()
    warm_done.record(stream)
    while not warm_done.query():
        pass
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()

    # K steps, k0 = (s * H) mod n_t: fused (a setup pass, launches of up to 512k wavefronts, the in-order work
    # sum whose atomicMin leaves the shard's best key) or the native loop of K launches (key after the last).
    # Two HIP events on the launch stream bracket the kernels (per-launch events would drain the queue
    # between kernels): GPU time per step of the batch = GPU time / K.
    def timed():
        ev0.record(stream)
        job()
        ev1.record(stream)
        if comm is not None:
            comm.reduce_best(batch.best_key, stream)  # the single collective: RCCL all-reduce(MIN) of 8 B

    elapsed = timed_window(timed, torch.cuda.synchronize)
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed, kern_ms = float(t[0]), float(t[1])
    key = batch.best_key.clone()

    # untimed checks: the device key equals the host-side encoding of the accumulated work, reduced
    # over the ranks by torch.distributed; NaN outputs are counted
    p_dev = torch.from_numpy(np.ascontiguousarray(params["step_length"])).to(dev)
    sel = hdist.select_cot(batch.work_cot[:, 0], p_dev, mass, n_t, args.steps * Hh)
    check = hdist.reduce_best(hdist.best_key(sel, id0))
    if int(check.item()) != int(key.item()) ^ hdist._FLIP:
        raise RuntimeError(f"best key mismatch: device {int(key.item())} vs host {int(check.item()) ^ hdist._FLIP}")
    best_cot, best_id = hdist.decode(check)
    nan_steps = torch.tensor([int(((batch.flags & 8) != 0).sum().item())], device=dev)
    if world > 1:
        dist.all_reduce(nan_steps)
    if comm is not None:
        comm.free()

    if rank == 0:
        steps_total = lay["total"] * Hh * args.steps
        value = steps_total / elapsed
        ms_per_step = 1e3 * elapsed / args.steps
        # the roofline's unit is one step of rank 0's batch: B x H control-loop steps
        alg_bytes = B * Hh * (out_bytes + width * PARAM_BYTES / Hh)
        achieved = alg_bytes / (kern_ms * 1e-3) / 1e9
        pmc, pmc_note = pmc_for(traffic_key, lib["sha256"])
        traffic = None if pmc is None else int(round(pmc["hbm_bytes_per_step"] * B / pmc["rollouts"]))
        flop = flops_for(f"{'mixed' if args.mixed else args.model}{' curved' if args.curved else ''} H={Hh}")
        fp64 = None
        if flop is not None and not args.fp32:
            alg_flops = flop["flops_per_step"] * B * Hh
            tf = alg_flops / (kern_ms * 1e-3) / 1e12
            fp64 = {"bound": "fp64 valu", "algorithmic_flops_per_step": flop["flops_per_step"],
                    "achieved_tflops": round(tf, 3), "peak_tflops": FP64_PEAK_TFLOPS, "frac": tf / FP64_PEAK_TFLOPS,
                    "source": "profiles/flops.json: " + str(flop.get("source"))}
            if pmc is not None and pmc.get("fp64_lane_flops_per_step"):
                issued = pmc["fp64_lane_flops_per_step"] * B / pmc["rollouts"]
                fp64["issued_lane_flops_per_step_of_batch"] = int(issued)
                fp64["issued_over_algorithmic"] = round(issued / alg_flops, 3)
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True, "scaling": lay["scaling"], "vs_baseline": None,
            "dtype": "f32" if args.fp32 else "f64",
            "data": "synthetic (splitmix64 gait parameters around pgs id 8; SURVEY.md 8d)",
            "config": {"workload": workload, "total_rollouts": lay["total"], "rollouts_per_gpu": B,
                       "horizon": Hh, "n_t": n_t,
                       "launch": ("fused: K calls in launches of up to 512k wavefronts over (step, rollout), every step "
                                  "its own output rows (hs_run_calls)") if fused else
                                 "one launch per step (hs_run_steps)",
                       "parallelism": f"rollout-sharded x{world}" + (
                           ", 1 RCCL all-reduce(MIN, 8 B) per job (hs_comm_reduce_best)" if world > 1 else "")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "traffic_over_algorithmic": None if traffic is None else round(traffic / alg_bytes, 3),
                         "traffic_note": pmc_note,
                         "kernel": step_kernel(models, fused, args.fp32) + " (+ the preparation pass (setup and IK table) "
                                   "and the fixup + work reduce; kernel_ms: the call's event-timed GPU time per step of the batch)",
                         "kernel_ms": round(kern_ms, 5), "alg_bytes_per_launch": alg_bytes},
            # the bound that binds: FP64 VALU issue/latency
            "fp64_valu": fp64,
            "best_rollout": {"id": best_id, "cot_per_cycle": best_cot},
            "nan_steps": int(nan_steps.item()),
            "lib": lib,
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
