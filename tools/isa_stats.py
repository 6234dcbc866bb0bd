"""Per-function register / scratch / LDS / code-size summary of the device code of
hs_kernels.hip (hipcc -S for gfx950). Tuning aid only.

  python tools/isa_stats.py [-D NAME=VAL ...] [--src file.hip] [--filter substr]
"""
import argparse
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "hslabs_amd", "csrc")


def stats(src, defines=()):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast",
                        f"-I{SRC}", f"-I{os.path.join(ROOT, 'include')}", *[f"-D{d}" for d in defines],
                        "--cuda-device-only", "-S", src, "-o", out], check=True, stderr=subprocess.DEVNULL)
        text = open(out).read()
    rows, cur = [], None
    for line in text.splitlines():
        m = re.match(r"^(_Z\S+):\s*(;.*)?$", line)
        if m:
            cur = {"name": m.group(1)}
            rows.append(cur)
            continue
        if cur is None:
            continue
        for key in ("codeLenInByte", "TotalNumVgprs", "ScratchSize", "Occupancy", "LDSByteSize"):
            m = re.match(rf"^\s*; {key}[:=]\s*(\d+)", line)
            if m:
                cur[key] = int(m.group(1))
    return [r for r in rows if "TotalNumVgprs" in r]


def demangle(n):
    try:
        return subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-cxxfilt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        return n


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--src", default=os.path.join(SRC, "hs_kernels.hip"))
    ap.add_argument("--filter", default="")
    a = ap.parse_args()
    for r in stats(a.src, a.D):
        name = demangle(r["name"])
        name = re.sub(r"\(anonymous namespace\)::", "", name)
        name = name.split("(")[0]
        if a.filter and a.filter not in name:
            continue
        print(f"{name[:58]:58s} vgpr {r.get('TotalNumVgprs', 0):4d} scratch {r.get('ScratchSize', 0):5d} "
              f"lds {r.get('LDSByteSize', 0):6d} occ {r.get('Occupancy', '-')} code {r.get('codeLenInByte', 0)}")
