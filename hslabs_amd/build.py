"""Build the gfx950 shared library libhslabs.so in-tree (hslabs_amd/_build/).

Only hipcc is needed (no cmake/ninja). Device code is compiled with
-ffp-contract=fast-honor-pragmas: a*b+c becomes one FMA (one rounding instead of the two of
the reference's x86-64 ``g++ -O2`` build, which has no FMA). That is 12 % fewer
cycles per step on gfx950 (the kernel is VALU-issue bound) and moves per-joint
torques by <= 2.3e-12 against the unfused CPU restatement on every pgs setup
(profiles/r01_parity_report.txt); host code (x86-64 baseline) is unaffected.
"honor-pragmas" keeps the one place that must round twice, work_over_period's
work_dt *= dt; work += work_dt (periodic.cpp:301-302, `work_add` under
`#pragma clang fp contract(off)`): plain -ffp-contract=fast ignores that pragma
and emitted one v_fmac_f64 there; tools/isa_check.py's
`work_add_check` verifies the reduce kernel's ISA.
The closed-loop simulation (hs_sim.hip) is the exception, built with
-ffp-contract=off: its contact test (depth >= 0) is decided within rounding for
stance feet, so it keeps the oracle's unfused rounding (a per-file flag).
So is hs_config.hip (the per-configuration FK / IK of the model.h API), which is
not on the hot path and keeps the reference's rounding.
Sources compile to objects in parallel, then link.
"""
from __future__ import annotations

import os
import shutil
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc")
OUT_DIR = os.path.join(HERE, "_build")
LIB = os.path.join(OUT_DIR, "libhslabs.so")
SOURCES = ["hs_kernels.hip", "hs_kernels_f32.hip", "hs_sim.hip", "hs_config.hip", "hs_capi.cpp", "hs_model.cpp",
           "hs_comm.cpp"]
# the best-rollout all-reduce (hs_comm.cpp) links RCCL; under torch the process's librccl.so.1
# (same SONAME) is the one bound
LIBS = ["-L/opt/rocm/lib", "-lrccl"]
VARIANT_DIR = os.path.join(OUT_DIR, "variants")
HEADERS = ["hs_topo.h", "hs_simtopo.h", "hs_ode.h", "hs_math.h", "hs_internal.h", "hs_limb.h", os.path.join("..", "..", "include", "hslabs.h")]
ARCH = os.environ.get("HSLABS_ARCH", "gfx950")
# per-source FMA contraction (default: fast, except where a `#pragma clang fp contract(off)` says not)
CONTRACT = {"hs_sim.hip": "off", "hs_config.hip": "off"}
# per-source compiler flags. Round 1 built the fp32 rollout kernels with the iterative ILP scheduler
# (+1.4 % for hs_rollout_kernel at 4 waves/SIMD); its register allocator crashes on the limb-lane kernel
# (hipcc, ROCm 7.2: RAGreedy segfault on hs_limb_kernel<18> in hs_kernels_f32.hip), so every source takes
# the default scheduler since round 6
SRC_FLAGS = {}


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm 7.x required)")


def _stale() -> bool:
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = [os.path.join(SRC, f) for f in SOURCES + HEADERS]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def _compile(out: str, defines=(), verbose: bool = False, flags=()) -> str:
    os.makedirs(os.path.dirname(out), exist_ok=True)
    tag = os.path.splitext(os.path.basename(out))[0]

    def obj(src):
        o = os.path.join(os.path.dirname(out), f"{tag}.{src}.o")
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-c",
               f"-ffp-contract={CONTRACT.get(src, 'fast-honor-pragmas')}", "-Wall", "-Wno-unused-function",
               *SRC_FLAGS.get(src, []), *flags,
               *[f"-D{d}" for d in defines], os.path.join(SRC, src), "-o", o]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        subprocess.run(cmd, check=True)
        return o

    jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 1))))
    with ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(obj, SOURCES))
    cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", *objs, *LIBS, "-o", out + ".tmp"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    for o in objs:
        os.remove(o)
    os.replace(out + ".tmp", out)
    return out


def _isa_check(lib: str, fatal: bool) -> None:
    """tools/isa_check.py on the built library: no vector instruction (a VGPR spill store, above all)
    may sit where a divergent loop exits with EXEC == 0, the miscompile that broke the inlined
    Eigen-style solve."""
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))
    try:
        import isa_check
    finally:
        sys.path.pop(0)
    if not os.path.exists(os.path.join(isa_check.LLVM, "llvm-objdump")):
        print("isa_check skipped: llvm-objdump not found", file=sys.stderr)
        return
    bad = isa_check.check(lib)
    if bad and fatal:
        os.remove(lib)
        raise RuntimeError(f"{lib}: {bad} device function(s) with vector instructions at EXEC == 0 after a "
                           "divergent loop exit (tools/isa_check.py); the library was removed")
    if not isa_check.work_add_check(lib, verbose=not fatal) and fatal:
        os.remove(lib)
        raise RuntimeError(f"{lib}: the fp64 work reduce contracts work_dt * dt + work into one FMA "
                           "(tools/isa_check.py work_add_check); the library was removed")


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and not _stale():
        return LIB
    _compile(LIB, verbose=verbose)
    _isa_check(LIB, fatal=True)
    return LIB


def build_variant(name: str, defines, verbose: bool = False, flags=()) -> str:
    """Tuning builds (e.g. HS_MIN_WAVES=N) in _build/variants/, never the product library; an A/B
    sweep selects one by name with HSLABS_VARIANT=<name> (capi.load reports the library it loaded,
    and bench.py prints its path and hash). Delete them after the sweep."""
    os.makedirs(VARIANT_DIR, exist_ok=True)
    out = _compile(os.path.join(VARIANT_DIR, f"libhslabs_{name}.so"), defines, verbose, flags)
    _isa_check(out, fatal=False)  # reported, not fatal: tuning builds may be inspected
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
