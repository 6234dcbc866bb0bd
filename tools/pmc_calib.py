"""FETCH_SIZE / WRITE_SIZE per byte moved, per access pattern (tools/fetch_calib.hip under
rocprofv3 --pmc, one counter per pass): the calibration factors DESIGN.md §5 applies to the step
kernel's counters.   python tools/pmc_calib.py gpurun_out/<dir> > profiles/r04_fetch_calibration.txt"""
import csv
import glob
import os
import sys

GiB = 1 << 30
BYTES = {"read_stream<double>": GiB, "read_stream<double2>": GiB, "read_records3": GiB // 24 * 24,
         "write_stream<double>": GiB, "write_stream<double2>": GiB, "write_rows18": GiB // 144 * 144}
root = sys.argv[1]
vals = {}


def pattern(name):
    for base in ("read_stream", "write_stream"):
        if base in name:
            return f"{base}<double2>" if ("vector" in name or "double2" in name) else f"{base}<double>"
    for k in ("read_records3", "write_rows18"):
        if k in name:
            return k
    return None


for path in sorted(glob.glob(os.path.join(root, "*", "run_counter_collection.csv"))):
    for row in csv.DictReader(open(path)):
        k = pattern(row["Kernel_Name"])
        if k:
            vals[(k, row["Counter_Name"])] = vals.get((k, row["Counter_Name"]), 0.0) + float(row["Counter_Value"])
print("pattern                  counter      counter KiB    bytes moved KiB   bytes per counted byte")
for (k, c), v in sorted(vals.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    if ("read" in k) != (c == "FETCH_SIZE"):
        continue  # a read kernel's WRITE_SIZE (0) and a write kernel's FETCH_SIZE (a few KiB)
    print(f"{k:24s} {c:11s} {v:14.0f} {BYTES[k] / 1024:17.0f}   {BYTES[k] / 1024 / v:8.3f}")
