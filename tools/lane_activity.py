"""Lane activity per phase of hs_rollout_kernel (diagnostic; tuning aid only).

tools/gpu_lanes.sh runs one rocprofv3 --pmc pass (SQ_THREAD_CYCLES_VALU, SQ_ACTIVE_INST_VALU,
SQ_INSTS_VALU, SQ_WAVES) on the product library and on timing-only builds that leave one phase out
(HS_EXP_KIN_FIRST=5: no kinematics samples; HS_EXP_NO_SOLVE: no contact solve; HS_EXP_NO_SCHUR: no
6x6 factorization). A phase's figures are the differences to the full build, so its mean active
lanes per VALU instruction cycle is dTHREAD_CYCLES / dACTIVE_INST (of 64; two rollouts per wave).
Only the kinematics difference is clean: leaving the contact solve (or its 6x6 factorization) out
RAISES the other phases' thread-cycles (SQ_THREAD_CYCLES_VALU counts the VALU's busy cycles, so
it moves with how the remaining fp64 work issues), so those rows are printed as measured but not
read as lane counts; DESIGN.md gives the solve's lane maps instead.

  python tools/lane_activity.py gpurun_out/lanes profiles/r02_lane_activity.txt --rollouts 4096
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import collect  # noqa: E402

VARIANTS = [("full", "base"), ("no kinematics", "xnokin"), ("no contact solve", "xnosolve"),
            ("no 6x6 Schur", "xnoschur")]
C = ("SQ_THREAD_CYCLES_VALU", "SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_WAVES")


def per_wave(root, name, n_waves):
    v = collect(os.path.join(root, name), n_waves)
    med = {c: statistics.median(v[c]) for c in C if c in v}
    w = med["SQ_WAVES"]
    return {c: med[c] / w for c in C[:3]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("out")
    ap.add_argument("--rollouts", type=int, required=True)
    a = ap.parse_args()
    n_waves = (a.rollouts + 1) // 2
    m = {label: per_wave(a.root, name, n_waves) for label, name in VARIANTS}
    full = m["full"]
    lines = ["hs_rollout_kernel lane activity (rocprofv3 --pmc, bench.py --steps 20 --warmup 5, per wavefront-step;",
             "two rollouts per wavefront, so 64 = every lane of both rollouts busy)",
             f"{'build / phase':32s} {'VALU insts':>11s} {'VALU cycles':>12s} {'lanes active':>13s}"]
    f_l = full["SQ_THREAD_CYCLES_VALU"] / full["SQ_ACTIVE_INST_VALU"]
    lines.append(f"{'whole step (full build)':32s} {full['SQ_INSTS_VALU']:11.0f} {full['SQ_ACTIVE_INST_VALU']:12.0f} "
                 f"{f_l:13.1f}")
    parts = [("kinematics (5 samples)", "no kinematics"), ("contact solve", "no contact solve"),
             ("  of which 6x6 Schur", "no 6x6 Schur")]
    rest = dict(full)
    for label, var in parts:
        d = {c: full[c] - m[var][c] for c in C[:3]}
        if not label.startswith("  "):
            for c in C[:3]:
                rest[c] -= d[c]
        lanes = d["SQ_THREAD_CYCLES_VALU"] / d["SQ_ACTIVE_INST_VALU"] if d["SQ_ACTIVE_INST_VALU"] > 0 else float("nan")
        lines.append(f"{label:32s} {d['SQ_INSTS_VALU']:11.0f} {d['SQ_ACTIVE_INST_VALU']:12.0f} {lanes:13.1f}")
    lanes = rest["SQ_THREAD_CYCLES_VALU"] / rest["SQ_ACTIVE_INST_VALU"]
    lines.append(f"{'rest (setup load, D, S1, outputs)':32s} {rest['SQ_INSTS_VALU']:11.0f} "
                 f"{rest['SQ_ACTIVE_INST_VALU']:12.0f} {lanes:13.1f}")
    with open(a.out, "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
