"""tools/isa_check.py: the build-time guard against the EXEC == 0 spill miscompile (DESIGN.md section 4,
"General path"). The known-bad sequence below is from the HS_GENERAL_INLINE build of
hs_rollout_kernel<22, false, FIX_NONE> (hipcc, ROCm 7.2, gfx950): fullpiv_lu's lane-0 permutation
loop, whose fall-through block stores seven VGPR spills before it restores EXEC."""
import os

import pytest

from conftest import ROOT

BAD = """\
s_mov_b64 s[12:13], 0
v_mov_b64_e32 v[2:3], v[0:1]
v_mov_b32_e32 v4, v166
global_load_sbyte v5, v[2:3], off offset:-18
v_add_u32_e32 v4, -1, v4
v_cmp_eq_u32_e32 vcc, 0, v4
s_or_b64 s[12:13], vcc, s[12:13]
s_waitcnt vmcnt(0)
global_load_ubyte v5, v[6:7], off
global_load_ubyte v8, v[2:3], off
global_store_byte v[2:3], v5, off
global_store_byte v[6:7], v8, off
v_lshl_add_u64 v[2:3], v[2:3], 0, 1
s_andn2_b64 exec, exec, s[12:13]
s_cbranch_execnz 65521
v_writelane_b32 v167, s38, 42
scratch_store_dword off, v82, off offset:120
scratch_store_dword off, v128, off offset:116
scratch_store_dwordx2 off, v[126:127], off offset:108
scratch_store_dwordx4 off, v[136:139], off offset:92
scratch_store_dwordx4 off, v[152:155], off offset:76
scratch_store_dword off, v146, off offset:72
scratch_store_dwordx2 off, v[150:151], off offset:64
v_writelane_b32 v167, s39, 43
s_or_b64 exec, exec, s[0:1]
scratch_store_dword off, v1, off offset:4
"""

GOOD = """\
s_andn2_b64 exec, exec, s[12:13]
s_cbranch_execnz 65521
s_or_b64 exec, exec, s[12:13]
scratch_store_dword off, v82, off offset:120
v_writelane_b32 v167, s38, 42
"""


# the fp64 work reduce's first steps (hs_fused_reduce_kernel, gfx950): built -ffp-contract=fast, the
# `fp contract(off)` pragma in work_add was ignored and each step was one FMA; built
# -ffp-contract=fast-honor-pragmas, a product rounded by v_mul_f64 and then summed
FUSED_WORK = """\
v_fma_f64 v[18:19], -v[18:19], v[24:25], v[22:23]
v_fmac_f64_e32 v[2:3], v[16:17], v[18:19]
v_fma_f64 v[18:19], v[16:17], v[22:23], v[2:3]
v_fmac_f64_e32 v[18:19], v[16:17], v[20:21]
"""
TWO_ROUNDINGS = """\
v_mul_f64 v[24:25], v[22:23], v[20:21]
v_fma_f64 v[18:19], -v[18:19], v[24:25], v[22:23]
v_mul_f64 v[20:21], v[16:17], v[20:21]
v_add_f64 v[2:3], v[2:3], v[20:21]
v_mul_f64 v[20:21], v[16:17], v[22:23]
v_add_f64 v[20:21], v[2:3], v[20:21]
"""


def _isa():
    import sys

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_check

    return isa_check


def test_scan_flags_the_known_bad_sequence():
    ic = _isa()
    ins = BAD.splitlines()
    hits = ic.scan(ins)
    assert [ins[h].split()[0] for h in hits] == ["scratch_store_dword", "scratch_store_dword", "scratch_store_dwordx2",
                                                 "scratch_store_dwordx4", "scratch_store_dwordx4",
                                                 "scratch_store_dword", "scratch_store_dwordx2"]
    assert ic.scan(GOOD.splitlines()) == []  # EXEC restored first: the spill is fine
    fwd = BAD.replace("s_cbranch_execnz 65521", "s_cbranch_execnz 12")  # a forward branch is no loop exit
    assert ic.scan(fwd.splitlines()) == []


def test_product_library_is_clean(product):
    lib = product.capi.lib_path()
    if not os.path.exists(os.path.join("/opt/rocm/lib/llvm/bin", "llvm-objdump")):
        pytest.skip("llvm-objdump not available")
    assert _isa().check(lib) == 0


def test_work_add_pairs_count_two_roundings():
    ic = _isa()
    assert ic.mul_add_pairs(FUSED_WORK.splitlines()) == 0
    # the first v_mul_f64 feeds an FMA (a division's Newton step), not an add: only two pairs
    assert ic.mul_add_pairs(TWO_ROUNDINGS.splitlines()) == 2


def test_product_work_reduce_rounds_twice(product):
    """work_over_period's work_dt *= dt; work += work_dt (periodic.cpp:301-302) in the shipped binary"""
    if not os.path.exists(os.path.join("/opt/rocm/lib/llvm/bin", "llvm-objdump")):
        pytest.skip("llvm-objdump not available")
    assert _isa().work_add_check(product.capi.lib_path())
