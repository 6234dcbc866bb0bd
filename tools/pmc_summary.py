"""Summarise tools/gpu_pmc.sh output (gpurun_out/<dir>/p*/run_counter_collection.csv) for
hs_rollout_kernel's fused step launch: per-step medians of every counter over the timed job's dispatches
(a dispatch's counts / the steps it ran = its wavefronts / the batch's wavefronts; the warm-up job's
shorter launches and its preparation pass are left out), per-wave figures, and the HBM traffic per step of the batch
(MI355X_MICROARCH.md HBM/rocprofv3 section: FETCH_SIZE x2 on gfx950, sizes in KiB). The library
hash the bench printed in the same passes goes into the JSON, and bench.py refuses the figures for
any other library.

  python tools/pmc_summary.py gpurun_out/pmc "hexapod B=4096 H=1" profiles/r02_pmc_summary.txt \
      --rollouts 4096 [--traffic-json profiles/pmc_traffic.json]
"""
import argparse
import csv
import re
import glob
import json
import os
import statistics
from collections import defaultdict

KERNEL = "the fused step launch"
# the fused step launch: the limb-lane kernel (round 6: 8 rollouts per wavefront) or hs_rollout_kernel's
# FIX_DEFER instantiation (2 per wavefront)
STEP_LAUNCH = re.compile(r"hs_limb_kernel<\d+, false>|hs_rollout_kernel<\d+, false, 1>")
FORCES_LAUNCH = re.compile(r"hs_limb_kernel<\d+, true>|hs_rollout_kernel<\d+, true, 0>")  # solve_forces' step launches (--forces)


def collect(root, n_rollouts, step_launch=STEP_LAUNCH):
    """counter -> per-step values of the step launches of the timed job: in each pass, the dispatches with
    the most steps (the bench's warm-up job runs fewer steps per launch and is left out)"""
    vals = defaultdict(dict)  # counter -> dispatch -> per-step value
    for path in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        with open(path) as f:
            rows = [r for r in csv.DictReader(f) if step_launch.search(r["Kernel_Name"])]
        def waves_per_step(name):
            return (n_rollouts + 7) // 8 if "hs_limb_kernel" in name else (n_rollouts + 1) // 2
        steps_of = {r["Dispatch_Id"]: int(r.get("Grid_Size") or r.get("Grid_Size_X")) // 64 // waves_per_step(r["Kernel_Name"])
                    for r in rows}
        most = max(steps_of.values(), default=0)
        for row in rows:
            steps = steps_of[row["Dispatch_Id"]]
            if steps < 1 or steps != most:
                continue
            key = (path, row["Dispatch_Id"])
            d = vals[row["Counter_Name"]]
            d[key] = d.get(key, 0.0) + float(row["Counter_Value"]) / steps
    return {c: sorted(d.values()) for c, d in vals.items()}


def collect_job_kernels(root):
    """The call's other kernels (setup pass, IK table pass, fixup + work reduce): counter -> kernel ->
    the timed job's value in each pass (its last dispatch of the kernel: the warm-up job's preparation
    pass tabulates fewer rows)."""
    vals = defaultdict(lambda: defaultdict(list))
    for path in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        per = defaultdict(float)
        for row in csv.DictReader(open(path)):
            name = row["Kernel_Name"]
            for k in ("hs_setup_kernel", "hs_ktab_kernel", "hs_prep_kernel", "hs_rollout_kernel<22, false, 2>"):
                if k in name:
                    per[(row["Counter_Name"], k, int(row["Dispatch_Id"]))] += float(row["Counter_Value"])
        last = {}
        for (c, k, d) in per:
            last[(c, k)] = max(last.get((c, k), d), d)
        for (c, k), d in last.items():
            vals[c][k].append(per[(c, k, d)])
    return vals


def lib_of(root):
    for log in sorted(glob.glob(os.path.join(root, "p*.log"))):
        for ln in open(log):
            if ln.startswith("{") and '"lib"' in ln:
                return json.loads(ln)["lib"]["sha256"]
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("workload")
    ap.add_argument("out")
    ap.add_argument("--rollouts", type=int, required=True)
    ap.add_argument("--traffic-json")
    ap.add_argument("--cmd", default="bench.py --steps 20 --warmup 5 --no-cpu")
    ap.add_argument("--forces", action="store_true", help="solve_forces' step launches (bench.py --forces)")
    ap.add_argument("--job-steps", type=int, default=20, help="steps per job: the per-job kernels' share")
    ap.add_argument("--rows-per-step", type=int, default=1,
                    help="output rows (fused steps) per bench step: the call horizon H (configs[2]: 32)")
    a = ap.parse_args()
    v = collect(a.root, a.rollouts, FORCES_LAUNCH if a.forces else STEP_LAUNCH)
    v = {c: [x * a.rows_per_step for x in xs] for c, xs in v.items()}  # per bench step (H rows)
    med = {c: statistics.median(x) for c, x in v.items()}
    sha = lib_of(a.root)
    lines = [f"{KERNEL}, {a.workload} ({a.cmd}), rocprofv3 --pmc, one group per pass, library {sha}",
             "per STEP of the batch (fused dispatch counts / its steps), median over the timed job's fused "
             "dispatches (FETCH_SIZE/WRITE_SIZE in KiB)"]
    for c in sorted(med, key=lambda c: (not c.endswith("_SIZE"), c)):
        lines.append(f"{c:28s} n={len(v[c]):3d} median={med[c]:.6g}")
    waves = med.get("SQ_WAVES")
    if waves:
        lines.append(f"per wave ({waves:.0f} waves per step):")
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                  "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                  "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64", "SQ_WAVE_CYCLES"):
            if c in med:
                lines.append(f"  {c:26s} {med[c] / waves:10.1f}")
        if "SQ_WAVE_CYCLES" in med and "SQ_WAIT_ANY" in med:
            lines.append(f"  wait fraction (SQ_WAIT_ANY / SQ_WAVE_CYCLES) {med['SQ_WAIT_ANY'] / med['SQ_WAVE_CYCLES']:.3f}")
    traffic = fp64 = None
    job_steps = a.job_steps
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
        traffic = int(round((2 * med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024))
        lines.append(f"HBM traffic per step of the batch, step launch (FETCH_SIZE x2 + WRITE_SIZE): {traffic} bytes "
                     f"(FETCH_SIZE alone x1: {int(med['FETCH_SIZE'] * 1024)} B; x2 as calibrated on known byte counts at "
                     f"8 and 16 B per lane and 24-byte records, profiles/r04_fetch_calibration.txt)")
        if not a.forces:
            jk = collect_job_kernels(a.root)
            extra = 0.0
            for k in sorted(set(jk.get("FETCH_SIZE", {})) | set(jk.get("WRITE_SIZE", {}))):
                f_ = statistics.median(jk["FETCH_SIZE"].get(k, [0.0]))
                w_ = statistics.median(jk["WRITE_SIZE"].get(k, [0.0]))
                b_ = (2 * f_ + w_) * 1024
                extra += b_
                lines.append(f"  once per job: {k:32s} FETCH_SIZE {f_:.1f} KiB, WRITE_SIZE {w_:.1f} KiB -> {int(b_)} B")
            if extra:
                traffic += int(round(extra / job_steps))
                lines.append(f"HBM traffic per step of the batch at {job_steps} steps per job, those kernels included: "
                             f"{traffic} bytes")
    if all(c in med for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64")):
        fp64 = int(64 * (med["SQ_INSTS_VALU_ADD_F64"] + med["SQ_INSTS_VALU_MUL_F64"] +
                         2 * med["SQ_INSTS_VALU_FMA_F64"]))
        lines.append(f"issued FP64 lane flops per step of the batch (64 x (ADD + MUL + 2 FMA), inactive lanes "
                     f"included): {fp64}")
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    if a.traffic_json and traffic is not None:
        # one entry per workload (bench.py pmc_for looks its own up), merged into the file's others
        try:
            j = json.load(open(a.traffic_json))
        except (OSError, ValueError):
            j = {}
        if "workloads" not in j:
            j = {"workloads": {j["workload"]: j} if j.get("workload") else {}}
        j["workloads"][a.workload] = {
            "workload": a.workload, "rollouts": a.rollouts, "lib_sha256": sha,
            "hbm_bytes_per_step": traffic, "fp64_lane_flops_per_step": fp64,
            "source": f"{a.out} (FETCH_SIZE x2 + WRITE_SIZE per step of the batch; FP64 instruction counts; {a.cmd})"}
        with open(a.traffic_json, "w") as f:
            json.dump(j, f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
