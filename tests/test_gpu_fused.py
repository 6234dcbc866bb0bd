"""Fused control steps (hs_run_calls): the steps of hs_run_steps in few launches over
(step, rollout), every step with its own output rows. Bitwise equality with the launch-per-step
path is expected: the same kernel code per step, the gait setup stored by a setup-only pass
(the same values the first launch of hs_run_steps stores), the work summed in step order, and
the steps the closed form declines (every step in HS_SOLVE_REFERENCE) recomputed by the fixup
launch after each step launch with the general path the per-step kernel calls inline.
"""
import os

import numpy as np
import pytest

from conftest import MODELS

pytestmark = pytest.mark.gpu

OUTS = ("q", "dq", "tau", "cf", "x", "flags", "work_cot")


@pytest.fixture(scope="module")
def gpu(product):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return product


@pytest.fixture(scope="module")
def hmodels(gpu):
    return {n: gpu.KinematicModel(os.path.join(MODELS, f"{n}.xml")) for n in ("hexapod", "spider", "myant")}


def npy(t):
    return None if t is None else t.cpu().numpy()


@pytest.mark.parametrize("name,B", [("hexapod", 1000), ("spider", 3), ("myant", 257)])
def test_fused_cycle_equals_horizon_run(gpu, hmodels, name, B):
    """n_t calls of H = 1 from k0 = 0 are the rows of one hs_run with H = n_t."""
    import torch
    from hslabs_amd import synth

    m = hmodels[name]
    p = synth.gen_params(B, name)
    ref = gpu.DeviceBatch(m, p, n_t=20, horizon=20, outputs=OUTS)
    ref.run(best=True)
    fz = gpu.DeviceBatch(m, p, n_t=20, horizon=20, outputs=OUTS)
    fz.work_cot.zero_()
    fz.run_calls(20, call_horizon=1, best=True, accumulate=False)
    torch.cuda.synchronize()
    for k in ("q", "dq", "tau", "cf", "x", "flags", "work_cot", "best_key"):
        assert np.array_equal(npy(getattr(ref, k)), npy(getattr(fz, k)), equal_nan=True), k


def test_fused_wraps_like_run_steps(gpu, hmodels):
    """45 calls (more than a cycle, k0 wrapping mod n_t) of H = 3 with accumulated work equal the
    launch-per-call loop, call by call."""
    import torch
    from hslabs_amd import synth

    m = hmodels["hexapod"]
    p = synth.gen_params(129, "hexapod", curved=True)
    n_calls, Hc = 45, 3
    seq = gpu.DeviceBatch(m, p, n_t=20, k0=5, horizon=Hc, outputs=OUTS)
    seq.work_cot.zero_()
    rows = {k: [] for k in ("q", "tau", "cf", "x", "flags")}
    for c in range(n_calls):
        seq.k0 = (5 + c * Hc) % 20
        seq.run(best=False, accumulate=True)
        for k in rows:
            rows[k].append(npy(getattr(seq, k)))
    fz = gpu.DeviceBatch(m, p, n_t=20, k0=5, horizon=n_calls * Hc, outputs=OUTS)
    fz.work_cot.zero_()
    fz.run_calls(n_calls, call_horizon=Hc, accumulate=True)
    torch.cuda.synchronize()
    for k in rows:
        want = np.concatenate(rows[k], axis=1)
        assert np.array_equal(want, npy(getattr(fz, k)), equal_nan=True), k
    assert np.array_equal(npy(seq.work_cot), npy(fz.work_cot))


def test_fused_fp32_equals_fp32_steps(gpu, hmodels):
    import torch
    from hslabs_amd import synth

    m = hmodels["spider"]
    p = synth.gen_params(512, "spider")
    ref = gpu.DeviceBatch(m, p, n_t=20, horizon=32, outputs=OUTS, dtype=torch.float32)
    ref.run(best=True)
    fz = gpu.DeviceBatch(m, p, n_t=20, horizon=32, outputs=OUTS, dtype=torch.float32)
    fz.work_cot.zero_()
    fz.run_calls(1, call_horizon=32, best=True, accumulate=False)
    torch.cuda.synchronize()
    for k in ("tau", "cf", "x", "flags", "work_cot", "best_key"):
        assert np.array_equal(npy(getattr(ref, k)), npy(getattr(fz, k)), equal_nan=True), k


def test_fused_argument_errors(gpu, hmodels):
    import ctypes

    from hslabs_amd import capi, synth

    b = gpu.DeviceBatch(hmodels["hexapod"], synth.gen_params(4, "hexapod"), horizon=2)
    a = b._args(None, False, True)
    L = capi.load()
    assert L.hs_run_calls(hmodels["hexapod"].handle, ctypes.byref(a), -1) != 0
    assert L.hs_run_calls(hmodels["hexapod"].handle, ctypes.byref(a), 0) == 0
    a.horizon = 0
    assert L.hs_run_calls(hmodels["hexapod"].handle, ctypes.byref(a), 2) != 0


def test_fused_mixed_plan_equals_steps(gpu, hmodels):
    """configs[4]'s plan (myant + hexapod interleaved): fused calls = one launch per call."""
    import torch
    from hslabs_amd import synth

    models = [hmodels[n] for n in synth.MIXED_MODELS]
    params, midx = synth.gen_mixed(301)
    n_calls = 25
    seq = gpu.MixedBatch(models, midx, params, n_t=20, k0=0, horizon=1, outputs=("tau", "cf", "flags", "work_cot"))
    seq.work_cot.zero_()
    rows = {k: [] for k in ("tau", "cf", "flags")}
    for c in range(n_calls):
        seq.k0 = c % 20
        seq.run(best=False, accumulate=True)
        for k in rows:
            rows[k].append(npy(getattr(seq, k)))
    fz = gpu.MixedBatch(models, midx, params, n_t=20, k0=0, horizon=n_calls,
                        outputs=("tau", "cf", "flags", "work_cot"))
    fz.work_cot.zero_()
    fz.run_calls(n_calls, call_horizon=1, accumulate=True, best=True)
    torch.cuda.synchronize()
    for k in rows:
        assert np.array_equal(np.concatenate(rows[k], axis=1), npy(getattr(fz, k)), equal_nan=True), k
    assert np.array_equal(npy(seq.work_cot), npy(fz.work_cot))
    key = npy(fz.best_key).view(np.uint64)[0]
    from hslabs_amd import capi

    L = capi.load()
    wc = npy(fz.work_cot)
    want = min(L.hs_best_key_encode(L.hs_best_key_cot(float(wc[i, 0]), models[midx[i]].total_mass,
                                                      float(params["step_length"][i]), 20, n_calls), i)
               for i in range(len(midx)))
    assert int(key) == want


def host_key(L, work, step_length, mass, n_t, steps, id0=0):
    return min(L.hs_best_key_encode(L.hs_best_key_cot(float(w), mass, float(l), n_t, steps), id0 + i)
               for i, (w, l) in enumerate(zip(work, step_length)))


def test_best_key_after_the_last_call(gpu, hmodels):
    """hs_run_steps(n, best) takes the key once, after the last call, over the accumulated work
    (ADVICE r1): equal to hs_run_calls(n, best)'s key and to the host encoding of the final work."""
    import torch

    from hslabs_amd import capi, synth

    m = hmodels["hexapod"]
    p = synth.gen_params(300, "hexapod", id0=50)
    keys = []
    for fused in (False, True):
        b = gpu.DeviceBatch(m, p, n_t=20, horizon=30 if fused else 1, outputs=("tau", "work_cot"),
                            rollout_id_base=50)
        b.work_cot.zero_()
        b.reset_best()
        if fused:
            b.run_calls(30, best=True, accumulate=True)
        else:
            b.run_steps(30, best=True, accumulate=True)
        torch.cuda.synchronize()
        keys.append(int(npy(b.best_key).view(np.uint64)[0]))
        want = host_key(capi.load(), npy(b.work_cot)[:, 0], p["step_length"], m.total_mass, 20, 30, 50)
        assert keys[-1] == want
    assert keys[0] == keys[1]


def test_forward_gait_beats_near_zero_backward_gaits(gpu, hmodels, oracle_mod, omodels):
    """The selection key ranks per-cycle COT with |L| (include/hslabs.h hs_best_key_cot): gaits that
    barely travel (|L| < 1e-3) are never selected and a slow backward gait no longer wins by a huge
    negative COT, which the signed COT of player.cpp:269-285 would give it."""
    import dataclasses

    import torch

    from conftest import PGS_CONFIG, to_oracle_gait

    base = gpu.read_pgs_config(PGS_CONFIG, 8)  # hexapod walking forward, L = 0.5
    lengths = [-0.0005, 0.0008, -0.01, -0.05, 0.5, 0.3, -0.5]
    gaits = [dataclasses.replace(base, step_length=L) for L in lengths]
    m = hmodels["hexapod"]
    b = gpu.DeviceBatch(m, gaits, n_t=20, horizon=20, outputs=("work_cot",))
    b.reset_best()
    b.run(best=True)
    torch.cuda.synchronize()
    _, rid = gpu.decode_best_key(int(npy(b.best_key).view(np.uint64)[0]))
    om = omodels["hexapod"]
    ref = [oracle_mod.rollout(om, to_oracle_gait(oracle_mod, g), 20, basis=oracle_mod.BASIS_FAST) for g in gaits]
    per_cycle = [r["work"] / (m.total_mass * abs(L)) if abs(L) >= 1e-3 else np.inf for r, L in zip(ref, lengths)]
    # the key holds float32 COTs, ties to the lowest id (L = +-0.5 mirror each other's work)
    assert rid == int(np.argmin(np.array(per_cycle, dtype=np.float32)))
    assert abs(lengths[rid]) >= 0.05
    signed = [r["cot"] for r in ref]
    assert lengths[int(np.argmin(signed))] < 0  # what a signed-COT minimum would have picked


def test_fused_more_steps_than_a_launch(gpu, hmodels):
    """S > CHUNK: 300 steps of 200 rollouts run as two fused launches (256 + 44 steps);
    every row, the work and the key equal the launch-per-step loop bitwise."""
    import torch

    from hslabs_amd import synth

    m = hmodels["hexapod"]
    p = synth.gen_params(200, "hexapod", curved=True)
    S = 300
    seq = gpu.DeviceBatch(m, p, n_t=20, horizon=1, outputs=("tau", "cf", "flags", "work_cot"))
    seq.work_cot.zero_()
    seq.reset_best()
    rows = {k: [] for k in ("tau", "cf", "flags")}
    for c in range(S):
        seq.k0 = c % 20
        seq.key_steps = S
        seq.run(best=c == S - 1, accumulate=True)
        for k in rows:
            rows[k].append(npy(getattr(seq, k)))
    fz = gpu.DeviceBatch(m, p, n_t=20, horizon=S, outputs=("tau", "cf", "flags", "work_cot"))
    fz.work_cot.zero_()
    fz.reset_best()
    fz.run_calls(S, best=True, accumulate=True)
    torch.cuda.synchronize()
    for k in rows:
        assert np.array_equal(np.concatenate(rows[k], axis=1), npy(getattr(fz, k))), k
    assert np.array_equal(npy(seq.work_cot), npy(fz.work_cot))
    assert np.array_equal(npy(seq.best_key), npy(fz.best_key))


def test_best_key_needs_work(gpu, hmodels):
    """A best key without work_cot is an argument error on every entry point."""
    import ctypes

    from hslabs_amd import capi, synth

    b = gpu.DeviceBatch(hmodels["hexapod"], synth.gen_params(4, "hexapod"), horizon=2, outputs=("tau",))
    a = b._args(None, True, True)
    L = capi.load()
    assert L.hs_run_calls(hmodels["hexapod"].handle, ctypes.byref(a), 2) != 0
    assert b"work_cot" in L.hs_last_error()
    assert L.hs_run_steps(hmodels["hexapod"].handle, ctypes.byref(a), 2, None) != 0


def test_fused_reference_mode_fixups_over_two_launches(gpu, hmodels):
    """HS_SOLVE_REFERENCE through hs_run_calls: every step is deferred by the step launch and solved
    by the fixup launch that follows it (its items counted per launch), over S > CHUNK (two step
    launches, each with its fixup) and an odd batch (an idle half-wave): rows, work and key equal
    the launch-per-step loop, where the general path runs inline, bitwise."""
    import torch

    from hslabs_amd import synth

    m = hmodels["myant"]
    p = synth.gen_params(61, "myant", curved=True)
    S = 270
    outs = ("tau", "cf", "flags", "work_cot")
    seq = gpu.DeviceBatch(m, p, n_t=20, horizon=1, outputs=outs)
    seq.solve_mode = gpu.capi.HS_SOLVE_REFERENCE
    seq.work_cot.zero_()
    seq.reset_best()
    rows = {k: [] for k in ("tau", "cf", "flags")}
    for c in range(S):
        seq.k0 = c % 20
        seq.key_steps = S
        seq.run(best=c == S - 1, accumulate=True)
        for k in rows:
            rows[k].append(npy(getattr(seq, k)))
    fz = gpu.DeviceBatch(m, p, n_t=20, horizon=S, outputs=outs)
    fz.solve_mode = gpu.capi.HS_SOLVE_REFERENCE
    fz.work_cot.zero_()
    fz.reset_best()
    fz.run_calls(S, best=True, accumulate=True)
    torch.cuda.synchronize()
    for k in rows:
        assert np.array_equal(np.concatenate(rows[k], axis=1), npy(getattr(fz, k)), equal_nan=True), k
    assert (npy(fz.flags).astype(np.uint32) & 64).all()  # HS_FLAG_GENERAL: every step took the general path
    assert np.array_equal(npy(seq.work_cot), npy(fz.work_cot))
    assert np.array_equal(npy(seq.best_key), npy(fz.best_key))
    # the fixup counters are left at zero: an AUTO call right after defers nothing stale
    fz.solve_mode = gpu.capi.HS_SOLVE_AUTO
    fz.work_cot.zero_()
    fz.run_calls(20, accumulate=True)
    torch.cuda.synchronize()
    flat = npy(fz.flags).reshape(-1)[:61 * 20]  # rows packed with stride n_calls * call_horizon = 20
    assert not (flat.astype(np.uint32) & 64).any()


@pytest.mark.parametrize("n_t,pattern", [(20, "alternate"), (20, "pairs"), (70, "alternate")])
def test_fused_straight_and_curved_rollouts(gpu, hmodels, n_t, pattern):
    """Straight gaits take the frame / IK-table kinematics (kin_sample_straight), curved ones the torso
    record and the same table (kin_sample_tab). Waves holding one of each ("alternate") run both;
    "pairs" keeps each wave uniform. Both sides build the call's tables (24 rows, hs::ktab_range, for the
    fused call and for the launch-per-step horizon run alike), so the fused call equals the horizon run
    bitwise; the table against the inline record, FK and IK is test_table_rows_match_inline_kinematics."""
    import torch
    from hslabs_amd import synth

    m = hmodels["hexapod"]
    B = 130
    p = synth.gen_params(B, "hexapod")
    pc = synth.gen_params(B, "hexapod", curved=True)
    sel = (np.arange(B) % 2 == 1) if pattern == "alternate" else ((np.arange(B) // 2) % 2 == 1)
    p[sel] = pc[sel]
    assert (p["curvature"] != 0).sum() == sel.sum()
    H = 20  # <= n_t: hs_run's horizon rows do not wrap k0, the fused calls' do
    ref = gpu.DeviceBatch(m, p, n_t=n_t, horizon=H, outputs=OUTS)
    ref.run(best=True)
    fz = gpu.DeviceBatch(m, p, n_t=n_t, horizon=H, outputs=OUTS)
    fz.work_cot.zero_()
    fz.run_calls(H, call_horizon=1, best=True, accumulate=False)
    torch.cuda.synchronize()
    for k in ("q", "dq", "tau", "cf", "x", "flags", "work_cot", "best_key"):
        assert np.array_equal(npy(getattr(ref, k)), npy(getattr(fz, k)), equal_nan=True), k
    assert np.isfinite(npy(fz.tau)).all()


@pytest.mark.parametrize("name,k0,H,n_calls", [("hexapod", 7, 5, 3), ("myant", 13, 2, 9), ("hexapod", 18, 1, 6)])
def test_ik_table_rows_match_single_steps(gpu, hmodels, name, k0, H, n_calls):
    """The IK table covers the samples [lo, lo + n) a call reads (hs::ktab_range; here lo > 0 and,
    for k0 = 18, calls that wrap mod n_t). Every step of the fused call equals the same step run on
    its own (one launch, one step: no table, the IK solved inline by the step kernel) to rounding:
    a table row off by one sample would move the torques by O(1)."""
    import torch
    from hslabs_amd import synth

    m = hmodels[name]
    B, n_t = 64, 20
    p = synth.gen_params(B, name, id0=555)
    fz = gpu.DeviceBatch(m, p, n_t=n_t, k0=k0, horizon=n_calls * H, outputs=("tau", "cf", "q"))
    fz.run_calls(n_calls, call_horizon=H)
    torch.cuda.synchronize()
    tau = npy(fz.tau)
    q = npy(fz.q)
    for c in range(n_calls):
        for h in range(H):
            kk = (k0 + c * H) % n_t + h
            if kk >= n_t:  # a single call from kk would start at kk mod n_t
                continue
            one = gpu.DeviceBatch(m, p, n_t=n_t, k0=kk, horizon=1, outputs=("tau", "cf", "q"))
            one.run(best=False)
            torch.cuda.synchronize()
            row = c * H + h
            ref_tau, ref_q = npy(one.tau)[:, 0], npy(one.q)[:, 0]
            assert np.allclose(q[:, row], ref_q, rtol=0, atol=1e-12), (c, h)
            assert np.allclose(tau[:, row], ref_tau, rtol=1e-9, atol=1e-9), (c, h)


@pytest.mark.parametrize("name,k0,H,n_calls,kind", [("hexapod", 7, 5, 3, "curved"), ("spider", 18, 1, 6, "curved"),
                                                    ("hexapod", 13, 2, 9, "transformed"),
                                                    ("myant", 3, 4, 4, "mixed"), ("hexapod", 0, 20, 1, "mixed")])
def test_table_rows_match_inline_kinematics(gpu, hmodels, name, k0, H, n_calls, kind):
    """The preparation pass tabulates every gait: straight ones (joint values), turning and record-
    transformed ones (joint values and the torso record, kin_sample_tab). Every step of the fused call
    equals the same step of a horizon run whose window is too long for a table (64 steps: 68 samples
    > HS_KTAB, hs::ktab_range), where the step kernel forms the gait record, torso FK, chain and limb
    IK inline (kin_sample, kin_sample_straight's straight_ik). The pass performs the inline sequence's
    operations in the same order, so the steps are bitwise equal (round 4: max |dtau| 0 on every case);
    a table row off by one sample, or a torso record of the wrong rollout, would move the torques by
    O(1). "mixed" waves hold straight, turning and transformed rollouts together."""
    import torch
    from conftest import transformed
    from hslabs_amd import synth

    m = hmodels[name]
    B, n_t = 64, 20
    rng = np.random.default_rng(41)
    p = synth.gen_params(B, name, id0=777, curved=kind != "transformed")
    if kind == "transformed":
        p, _ = transformed(p, rng, frac=0.7)
    elif kind == "mixed":
        plain = synth.gen_params(B, name, id0=777)
        sel = np.arange(B) % 3 == 0
        p[sel] = plain[sel]
        p, _ = transformed(p, rng, frac=0.3)
    outs = ("tau", "cf", "q", "flags")
    fz = gpu.DeviceBatch(m, p, n_t=n_t, k0=k0, horizon=n_calls * H, outputs=outs)
    fz.run_calls(n_calls, call_horizon=H)
    ref = gpu.DeviceBatch(m, p, n_t=n_t, k0=0, horizon=64, outputs=outs)
    ref.run(best=False)
    torch.cuda.synchronize()
    tau, q, fl = npy(fz.tau), npy(fz.q), npy(fz.flags).astype(np.uint32)
    rtau, rq, rfl = npy(ref.tau), npy(ref.q), npy(ref.flags).astype(np.uint32)
    cf, rcf = npy(fz.cf), npy(ref.cf)
    near = 0
    for c in range(n_calls):
        for h in range(H):
            kk = (k0 + c * H) % n_t + h
            row = c * H + h
            assert np.array_equal(q[:, row], rq[:, kk]), (c, h)
            assert np.array_equal(tau[:, row], rtau[:, kk], equal_nan=True), (c, h)
            assert np.array_equal(cf[:, row], rcf[:, kk], equal_nan=True), (c, h)
            assert np.array_equal(fl[:, row], rfl[:, kk]), (c, h)
            near += int(((fl[:, row] & gpu.capi.HS_FLAG_NEAR_RANK) != 0).sum())
    print(f"{name} {kind}: {n_calls * H * B} steps bitwise equal ({near} near-rank flagged)")


def _work_two_roundings(tau, dq, period, n_t, w0):
    """work_over_period (periodic.cpp:285-307) restated from the step outputs: per step the motors'
    positive work tau_j * jvel_j (jvel = the dq output of hinge j, compute_vel_traj's rate) summed in
    joint order, then work_dt *= dt; work += work_dt with TWO roundings (numpy never contracts)"""
    B, H, nmj = tau.shape
    dt = period / float(n_t)
    w = w0.copy()
    for s in range(H):
        dw = tau[:, s, :] * dq[:, s, 6:6 + nmj]
        dw = np.where(dw > 0, dw, 0.0)
        work_dt = np.zeros(B)
        for j in range(nmj):
            work_dt = work_dt + dw[:, j]
        w = w + work_dt * dt
    return w


def _work_one_rounding(tau, dq, period, n_t, w0):
    """the same with work + work_dt * dt as one correctly rounded FMA (exact rational arithmetic)"""
    from fractions import Fraction

    B, H, nmj = tau.shape
    out = np.empty(B)
    for b in range(B):
        dt = period[b] / float(n_t)
        w = float(w0[b])
        for s in range(H):
            dw = tau[b, s] * dq[b, s, 6:6 + nmj]
            work_dt = 0.0
            for v in np.where(dw > 0, dw, 0.0):
                work_dt = work_dt + float(v)
            w = float(Fraction(work_dt) * Fraction(dt) + Fraction(w))
        out[b] = w
    return out


@pytest.mark.parametrize("path", ["fused", "fused_reference", "steps"])
def test_work_rounds_twice_bitwise(gpu, hmodels, path):
    """work_over_period's work_dt *= dt_traj; work_period += work_dt (periodic.cpp:
    301-302) rounds twice in the reference's x86-64 build. The fused reduce (and the fixup + reduce
    launch that ends an HS_SOLVE_AUTO call), the HS_SOLVE_REFERENCE fixups and the launch-per-step
    path must give work_cot bitwise equal to that accumulation recomputed in numpy from the steps'
    torques and joint rates, starting from a nonzero accumulated work; the one-FMA accumulation the
    library shipped in round 5 differs on some rollouts (so the test can tell them apart).
    tools/isa_check.py's work_add_check pins the same in the ISA."""
    import torch
    from hslabs_amd import synth

    m = hmodels["hexapod"]
    B, K = 4096 if path != "fused_reference" else 256, 20
    p = synth.gen_params(B, "hexapod", id0=31337)
    w0 = np.random.default_rng(5).uniform(0.0, 3.0, B)
    b = gpu.DeviceBatch(m, p, n_t=20, k0=3, horizon=K if path != "steps" else 1,
                        outputs=("tau", "dq", "flags", "work_cot"))
    if path == "fused_reference":
        b.solve_mode = gpu.capi.HS_SOLVE_REFERENCE
    b.work_cot.zero_()
    b.work_cot[:, 0] = torch.from_numpy(w0).to(b.work_cot.device)
    if path == "steps":
        tau, dq = [], []
        for c in range(K):
            b.k0 = (3 + c) % 20
            b.run(best=False, accumulate=True)
            tau.append(npy(b.tau))
            dq.append(npy(b.dq))
        tau, dq = np.concatenate(tau, axis=1), np.concatenate(dq, axis=1)
    else:
        b.run_calls(K, call_horizon=1, best=False, accumulate=True)
        torch.cuda.synchronize()
        tau, dq = npy(b.tau), npy(b.dq)
    wc = npy(b.work_cot)
    period = np.ascontiguousarray(p["period"], dtype=np.float64)
    want = _work_two_roundings(tau, dq, period, 20, w0)
    assert np.array_equal(wc[:, 0], want), f"{int((wc[:, 0] != want).sum())} of {B} rollouts' work differ"
    cot = want / (m.total_mass * np.ascontiguousarray(p["step_length"], dtype=np.float64))
    assert np.array_equal(wc[:, 1], cot)
    if path == "fused":
        fma = _work_one_rounding(tau[:512], dq[:512], period[:512], 20, w0[:512])
        assert (fma != want[:512]).any(), "the one-rounding accumulation should differ somewhere"
