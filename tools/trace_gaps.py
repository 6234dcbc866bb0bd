"""Per-kernel durations and the idle gaps between consecutive kernels of a rocprofv3 kernel trace
(csv), for the last N dispatches (the timed job of a bench run). Tuning aid.
  python tools/trace_gaps.py <run_kernel_trace.csv> [N]"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    rows = rows[-n:]
    prev = None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev is not None else float("nan")
        print(f"{r['Kernel_Name'][:60]:60s} dur {(e - s) / 1e3:9.2f} us  gap {gap:8.2f} us")
        prev = e


if __name__ == "__main__":
    main()
