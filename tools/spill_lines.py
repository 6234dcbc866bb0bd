"""Source lines of the scratch (spill) accesses of one kernel of hs_kernels.hip (tuning aid): compiles
the device code with line tables (-gline-tables-only) and attributes each scratch_* instruction of the
kernel to the .loc line before it.

  python tools/spill_lines.py [-D NAME=VAL ...] [--kernel substr]   (default: the fused hexapod step launch)
"""
import argparse
import collections
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "hslabs_amd", "csrc")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--kernel", default="hs_rollout_kernelILi22ELb0ELi1E")
    ap.add_argument("--src", default=SRC, help="the csrc directory (e.g. an older commit's, tools/build_prev.py)")
    ap.add_argument("--file", default="hs_kernels.hip", help="hs_kernels_f32.hip: the fp32 build")
    args = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast-honor-pragmas",
                        "--cuda-device-only", "-S", "-gline-tables-only", f"-I{args.src}",
                        f"-I{os.path.join(args.src, '..', '..', 'include')}", *[f"-D{d}" for d in args.D],
                        os.path.join(args.src, args.file), "-o", out], check=True, capture_output=True)
        s = open(out).read()
    files = {m.group(1): (m.group(3) or m.group(2)).split("/")[-1]
             for m in re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', s)}
    m = re.search(r"^(_Z\w*" + re.escape(args.kernel) + r"\w*):", s, re.M)
    if not m:
        raise SystemExit(f"kernel {args.kernel} not found")
    body = s[m.start():s.index(".Lfunc_end", m.start())].splitlines()
    loc, cnt = None, collections.Counter()
    for line in body:
        t = line.strip()
        lm = re.match(r"\.loc\s+(\d+)\s+(\d+)", t)
        if lm:
            loc = f"{files.get(lm.group(1), lm.group(1))}:{lm.group(2)}"
        elif t.startswith("scratch_"):
            cnt[(loc, t.split()[0])] += 1
    print(m.group(1)[:90])
    for (where, op), n in sorted(cnt.items(), key=lambda x: str(x[0])):
        print(f"  {where:28s} {op:24s} {n}")


if __name__ == "__main__":
    main()
