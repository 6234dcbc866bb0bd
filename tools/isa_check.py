"""Build-time check of the gfx950 device code for one miscompile pattern (hipcc of ROCm 7.2).

The pattern ("General path"): a vector instruction placed in the block
that a divergent loop falls through to when its last lanes leave, before that block restores
EXEC. The loop's back edge is

    s_andn2_b64 exec, exec, s[a:b]     ; drop the lanes that left
    s_cbranch_execnz <loop head>       ; backwards

so the fall-through runs with EXEC == 0 until the next instruction that writes EXEC. There a
VGPR spill store (scratch_store ... "Folded Spill") writes nothing and its later reload returns
whatever the scratch slot held: the Eigen-style contact solve inlined into the 3-waves/SIMD step
kernel (HS_GENERAL_INLINE, removed) got 7 such spill stores right after fullpiv_lu's lane-0
permutation loop and returned wrong forces on every step. v_writelane / v_readlane (SGPR spills
to VGPR lanes) ignore EXEC and are not affected; v_cmp results are masked by EXEC and harmless
here. Every other vector ALU, memory or LDS instruction in such a block is reported.

  python tools/isa_check.py [lib.so ...]   (default: the product library)
Exit status 1 when any function shows the pattern. hslabs_amd/build.py runs it on every build.

`work_add_check` is the second build-time check: work_over_period's accumulation `work_dt *= dt;
work += work_dt` (periodic.cpp:301-302) rounds twice in the reference's x86-64 build, and the fp64
work reduce (hs_fused_reduce_kernel, 32 steps unrolled) must issue it as a v_mul_f64 whose result a
v_add_f64 consumes, not as one v_fma*_f64 (plain -ffp-contract=fast ignored the `fp contract(off)`
pragma and fused all 32).
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"

_EXEC_WRITE = re.compile(r"^s_\w+\s+exec\b|_saveexec|^s_(setpc|swappc|endpgm|branch|cbranch)")
_VECTOR = re.compile(r"^(scratch_|buffer_|global_|flat_|ds_|v_(?!writelane|readlane|readfirstlane|cmp))")
_BACKEDGE_MASK = re.compile(r"^s_andn2_b64\s+exec,\s*exec,")


def _disasm_functions(text: str):
    """llvm-objdump -d output -> {symbol: [instruction text, ...]} (comments stripped)"""
    funcs, cur = {}, None
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(\S+)>:$", line)
        if m:
            cur = funcs.setdefault(m.group(1), [])
            continue
        if cur is None:
            continue
        s = line.split("//")[0].strip()
        if s:
            cur.append(s)
    return funcs


def scan(instructions):
    """Indices of vector instructions executed with EXEC == 0 after a divergent loop's exit."""
    hits = []
    n = len(instructions)
    for j, ins in enumerate(instructions):
        m = re.match(r"^s_cbranch_execnz\s+(-?\d+)", ins)
        if not m or j == 0:
            continue
        imm = int(m.group(1))
        if imm < 32768 and imm >= 0:  # forward branch (16-bit signed word offset): not a back edge
            continue
        if not _BACKEDGE_MASK.match(instructions[j - 1]):
            continue
        for k in range(j + 1, n):
            nxt = instructions[k]
            if _EXEC_WRITE.search(nxt):
                break
            if _VECTOR.match(nxt):
                hits.append(k)
    return hits


def code_objects(lib: str, workdir: str):
    """The gfx950 code objects bundled into a host shared library (extracted in workdir)."""
    copy = os.path.join(workdir, os.path.basename(lib))
    shutil.copy(lib, copy)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", copy], check=True, capture_output=True,
                   cwd=workdir)
    return sorted(os.path.join(workdir, f) for f in os.listdir(workdir) if "amdgcn" in f and "gfx950" in f)


def check(lib: str, verbose: bool = True) -> int:
    """Number of functions of lib's device code that show the pattern (printed when verbose)."""
    bad = 0
    with tempfile.TemporaryDirectory() as td:
        for co in code_objects(lib, td):
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co], check=True,
                                 capture_output=True, text=True).stdout
            for name, ins in _disasm_functions(dis).items():
                hits = scan(ins)
                if hits:
                    bad += 1
                    if verbose:
                        print(f"isa_check: {os.path.basename(lib)}: {name}: {len(hits)} vector instruction(s) at "
                              f"EXEC == 0 after a divergent loop exit, e.g. {ins[hits[0]]}", file=sys.stderr)
    return bad


_MUL_F64 = re.compile(r"^v_mul_f64(?:_e(?:32|64))?\s+(v\[\d+:\d+\])")
_ADD_F64 = re.compile(r"^v_add_f64(?:_e(?:32|64))?\s+v\[\d+:\d+\],\s*(\S+),\s*(\S+)")
WORK_ADD_UNROLL = 32  # reduce_rollouts' unrolled step loop (hs_kernels.hip)


def mul_add_pairs(instructions) -> int:
    """v_add_f64 instructions that read the destination of the latest v_mul_f64 writing that register
    pair: a product rounded before the sum (two roundings)"""
    last_mul, pairs = {}, 0
    for ins in instructions:
        m = _MUL_F64.match(ins)
        if m:
            last_mul[m.group(1)] = True
            continue
        a = _ADD_F64.match(ins)
        if a and any(last_mul.pop(r, False) for r in (a.group(1), a.group(2))):
            pairs += 1
    return pairs


def work_add_check(lib: str, verbose: bool = True) -> bool:
    """True when the fp64 work reduce of lib rounds work_dt * dt before the sum on all its unrolled
    steps (at least WORK_ADD_UNROLL mul -> add pairs)"""
    found = []
    with tempfile.TemporaryDirectory() as td:
        for co in code_objects(lib, td):
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co], check=True,
                                 capture_output=True, text=True).stdout
            for name, ins in _disasm_functions(dis).items():
                if "hs_fused_reduce_kernel" in name and "hs_run_argsd" in name:  # the fp64 instantiation
                    found.append(mul_add_pairs(ins))
    ok = bool(found) and min(found) >= WORK_ADD_UNROLL
    if verbose:
        print(f"work_add_check: {os.path.basename(lib)}: fp64 reduce mul->add pairs {found} "
              f"(need >= {WORK_ADD_UNROLL}): {'ok' if ok else 'FAIL'}", file=sys.stderr)
    return ok


if __name__ == "__main__":
    libs = sys.argv[1:] or [os.path.join(ROOT, "hslabs_amd", "_build", "libhslabs.so")]
    bad_work = [lib for lib in libs if not work_add_check(lib)]
    total = sum(check(lib) for lib in libs) + len(bad_work)
    print(f"isa_check: {total} function(s) with the EXEC == 0 spill pattern in {len(libs)} librar"
          f"{'y' if len(libs) == 1 else 'ies'}")
    sys.exit(1 if total else 0)
