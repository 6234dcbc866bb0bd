"""Summarise tools/gpu_pmc.sh output (gpurun_out/pmc/p*/run_counter_collection.csv) for
hs_rollout_kernel: per-dispatch medians of every counter, derived per-wave figures, and the
HBM traffic per launch (gfx950: FETCH_SIZE is reported in 64 B units of 32 B -> x2, sizes in
KiB; MI355X_MICROARCH.md HBM/rocprofv3 section).

  python tools/pmc_summary.py gpurun_out/pmc "hexapod B=4096 H=1" profiles/r01_v2_pmc_summary.txt \
      [--traffic-json profiles/pmc_traffic.json]
"""
import argparse
import csv
import glob
import json
import os
import statistics
from collections import defaultdict

KERNEL = "hs_rollout_kernel"


def collect(root):
    vals = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    for path in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
        with open(path) as f:
            for row in csv.DictReader(f):
                if KERNEL not in row["Kernel_Name"]:
                    continue
                key = (path, row["Dispatch_Id"])
                vals[row["Counter_Name"]][key] += float(row["Counter_Value"])
    return {c: sorted(d.values()) for c, d in vals.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("workload")
    ap.add_argument("out")
    ap.add_argument("--traffic-json")
    ap.add_argument("--cmd", default="bench.py --steps 10 --warmup 2 --no-cpu")
    a = ap.parse_args()
    v = collect(a.root)
    med = {c: statistics.median(x) for c, x in v.items()}
    lines = [f"{KERNEL}, {a.workload} ({a.cmd}), rocprofv3 --pmc, one group per pass",
             "per-dispatch medians over the kernel's dispatches (FETCH_SIZE/WRITE_SIZE in KiB)"]
    for c in sorted(med, key=lambda c: (not c.endswith("_SIZE"), c)):
        lines.append(f"{c:28s} n={len(v[c]):3d} median={med[c]:.6g}")
    waves = med.get("SQ_WAVES")
    if waves:
        lines.append("per wave:")
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD", "SQ_INSTS_BRANCH",
                  "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                  "SQ_INSTS_VALU_TRANS_F64"):
            if c in med:
                lines.append(f"  {c:26s} {med[c] / waves:10.1f}")
        if "SQ_WAVE_CYCLES" in med and "SQ_WAIT_ANY" in med:
            lines.append(f"  wait fraction (SQ_WAIT_ANY / SQ_WAVE_CYCLES) {med['SQ_WAIT_ANY'] / med['SQ_WAVE_CYCLES']:.3f}")
    traffic = None
    if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
        traffic = int(round((2 * med["FETCH_SIZE"] + med["WRITE_SIZE"]) * 1024))
        lines.append(f"HBM traffic per launch (gfx950 correction: FETCH_SIZE x2): {traffic} bytes")
    fp64 = None
    if all(c in med for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64")):
        # issued FP64 lane operations (64 lanes per wave instruction, FMA = 2): an upper bound on the
        # useful FP64 work, inactive lanes included
        fp64 = int(64 * (med["SQ_INSTS_VALU_ADD_F64"] + med["SQ_INSTS_VALU_MUL_F64"] +
                         2 * med["SQ_INSTS_VALU_FMA_F64"]))
        lines.append(f"issued FP64 lane flops per launch (64 x (ADD + MUL + 2 FMA)): {fp64}")
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))
    if a.traffic_json and traffic is not None:
        with open(a.traffic_json, "w") as f:
            json.dump({"workload": a.workload, "hbm_bytes_per_launch": traffic,
                       "fp64_lane_flops_per_launch": fp64,
                       "source": f"{a.out} (FETCH_SIZE x2 + WRITE_SIZE, KiB -> B; FP64 instruction counts)"},
                      f, indent=1)
            f.write("\n")


if __name__ == "__main__":
    main()
