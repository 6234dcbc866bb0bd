"""Static instruction mix per stamped phase of hs_rollout_kernel (diagnostic; tuning aid only).

Compiles the HS_STAMPS build to assembly, slices the chosen kernel at its
s_memtime stamps (slot = the store offset / 8) and counts instruction classes
between consecutive stamps in code order.

  python tools/phase_isa.py [--nm 22] [--forces] [--mode 0|1|2] [-D NAME=VAL ...]
"""
import argparse
import collections
import os
import re
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "hslabs_amd", "csrc")

CLASSES = [
    ("vmem_load", r"^(global_load|buffer_load|flat_load)"),
    ("vmem_store", r"^(global_store|buffer_store|flat_store)"),
    ("smem", r"^s_(load|buffer_load)"),
    ("lds", r"^ds_"),
    ("wait_vm", r"^s_waitcnt.*vmcnt"),
    ("wait_lgkm", r"^s_waitcnt.*lgkmcnt"),
    ("f64", r"^v_\w+_f64"),
    ("valu", r"^v_"),
    ("salu", r"^s_"),
    ("branch", r"^s_(cbranch|branch)"),
    ("sgpr_spill", r"^v_(readlane|writelane)_b32"),
    ("vgpr_spill", r"^scratch_"),
    ("cndmask", r"^v_cndmask"),
    ("mov", r"^v_mov_b(32|64)"),
    ("div_f64", r"^v_div_fixup_f64"),
    ("sqrt_f64", r"^v_rsq_f64"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nm", type=int, default=22)
    ap.add_argument("--forces", action="store_true")
    ap.add_argument("--mode", type=int, default=1, help="hs::FIX_* instantiation (1: the fused step launch)")
    ap.add_argument("-D", action="append", default=[])
    ap.add_argument("--dump", help="write the kernel body here")
    a = ap.parse_args()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "k.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast-honor-pragmas",
                        "-DHS_STAMPS", f"-I{SRC}", f"-I{os.path.join(ROOT, 'include')}", *[f"-D{d}" for d in a.D],
                        "--cuda-device-only", "-S", os.path.join(SRC, "hs_kernels.hip"), "-o", out],
                       check=True, stderr=subprocess.DEVNULL)
        text = open(out).read()
    key = f"hs_rollout_kernelILi{a.nm}ELb{int(a.forces)}ELi{0 if a.forces else a.mode}E"
    m = re.search(rf"^(_Z\S*{key}\S*):", text, re.M)
    body = text[m.end():text.index(".Lfunc_end", m.end())].splitlines()
    if a.dump:
        open(a.dump, "w").write("\n".join(body))
    ins = [l.strip() for l in body if l.strip() and not l.strip().startswith((";", ".")) and not l.endswith(":")]
    segs, cur, slot = [], collections.Counter(), "entry"
    pending = False
    for l in ins:
        op = l.split()[0]
        if op == "s_memtime" or op == "s_memrealtime":
            pending = True
            continue
        if pending and op.startswith("global_store"):
            mo = re.search(r"offset:(\d+)", l)
            new = str(int(mo.group(1)) // 8) if mo else "0"
            segs.append((slot, cur))
            cur, slot, pending = collections.Counter(), new, False
            continue
        for name, rx in CLASSES:
            if re.match(rx, l if name.startswith("wait") else op):
                cur[name] += 1
        cur["total"] += 1
    segs.append((slot, cur))
    hdr = ["from"] + [c for c, _ in CLASSES] + ["total"]
    print(" ".join(f"{h:>9s}" for h in hdr))
    for s, c in segs:
        print(" ".join([f"{s:>9s}"] + [f"{c[h]:9d}" for h in hdr[1:]]))


if __name__ == "__main__":
    main()
