"""GPU parity at BASELINE sizes and on the solve paths round 1 left untested.

The oracle is the CPU restatement (oracle/, parity with the reference binary unpinned: SURVEY.md
8c); its three modes agree with each other to ~1e-12 on every step of these
batches, full-rank steps included (measured on CPU: fast vs tree <= 3e-12, ortho vs tree <= 5e-13).

Tolerances (written here, per the north_star): fp64 per-joint motor torque |GPU - oracle| <
1e-6 N*m (the north_star bound) and < 1e-9 * max(1, |tau|) (what the kernel achieves: ULPs of the
device transcendentals amplified by the 1 / (4 dt^2) stencil); contact forces < 1e-8 * max(1, |f|);
flags identical (HS_FLAG_GENERAL and HS_FLAG_NEAR_RANK aside). fp32 (configs[2]): 1e-3 * max(1, |tau|)
wherever the fp32 run chose the same contact set as the fp64 oracle.

HS_FLAG_NEAR_RANK (include/hslabs.h; the oracle's HSO_FLAG_NEAR_RANK, hs_oracle.cpp NearTrack) marks a
rank or routing decision within rounding of its threshold (FullPivLU pivots within 4x of the rank
threshold, a doubled threshold, rel_error in [1e-7, 1e-5], ColPivQR pivots, the closed form's guards;
ftsolver.cpp:205-232), where another rounding may take the decision the other way (hard
part 2). A flag does not excuse a step by itself (`compare`): where either side flags one, the oracle is
run again in the other reference-faithful null basis (tree <-> ortho: the tree-built basis and the
orthonormal one SparseQR(B^T).matrixQ() spans, ftsolver.cpp:187-202), and wherever the two agree to the
parity bounds the reference's answer does not hinge on the decision -- those steps are held to every
bound like the rest. Only steps whose two reference answers disagree are excluded; they are counted,
bounded per test and must be finite, and on at least 95 % of them the kernel must be, step by step,
within max(1e-6 N*m, 10x the two answers' spread) of the nearer answer (the per-step maximum of that
distance is printed). Where the
kernel's own path is the closed form, the batch is also compared step for step with the oracle's fast
mode (the same closed form) with no exclusion at all.
"""
import os

import numpy as np
import pytest

from conftest import MODELS, PGS_CONFIG, PGS_IDS, record_to_oracle_gait, to_oracle_gait

pytestmark = pytest.mark.gpu

TAU_REL = 1e-9
TAU_ABS = 1e-6  # north_star
CF_REL = 1e-8
FP32_TOL = 1e-3
GEN = np.uint32(64)  # HS_FLAG_GENERAL: which solve path ran, not a property of the step
NEAR = np.uint32(256)  # HS_FLAG_NEAR_RANK = HSO_FLAG_NEAR_RANK: a decision within rounding of its threshold
IGN = GEN | NEAR  # flag bits that describe the arithmetic, not the step


def near(*flags):
    """steps that any of the given flag arrays marks HS_FLAG_NEAR_RANK"""
    m = np.zeros(np.shape(flags[0]), dtype=bool)
    for f in flags:
        m |= (np.asarray(f).astype(np.uint32) & NEAR) != 0
    return m


def check_flags(g, r, what, skip=None):
    """flags identical on the steps not skipped, HS_FLAG_GENERAL / HS_FLAG_NEAR_RANK aside"""
    g, r = np.asarray(g).astype(np.uint32) & ~IGN, np.asarray(r).astype(np.uint32) & ~IGN
    keep = np.ones(g.shape, bool) if skip is None else ~skip
    bad = (g != r) & keep
    assert not bad.any(), f"{what}: flags differ on {bad.sum()} unflagged steps"


@pytest.fixture(scope="module")
def gpu(product):
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    return product


@pytest.fixture(scope="module")
def hmodels(gpu):
    return {n: gpu.KinematicModel(os.path.join(MODELS, f"{n}.xml")) for n in ("hexapod", "spider", "myant")}


def threads():
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(16, int(omp) if omp.isdigit() else (os.cpu_count() or 1)))


def npy(t):
    return t.cpu().numpy()


def check_tau(tau, ref, what, skip=None):
    """both bounds on every step (rows [..., nmj]) outside `skip` (the excluded steps); skipped steps
    must be finite"""
    if skip is not None:
        assert np.isfinite(tau[skip]).all(), f"{what}: non-finite torques on excluded steps"
        tau, ref = tau[~skip], ref[~skip]
    if tau.size == 0:
        return
    scale = np.maximum(1, np.abs(ref).max(axis=-1, keepdims=True))
    err = np.abs(tau - ref)
    assert err.max() < TAU_ABS, f"{what}: max |dtau| {err.max():.3e} over the north_star bound"
    rel = (err / scale).max(axis=-1)
    assert (rel < TAU_REL).all(), f"{what}: {(rel >= TAU_REL).sum()} steps over {TAU_REL} (max {rel.max():.3e})"


def check_cf(cf, ref, what, skip=None):
    if skip is not None:
        cf, ref = cf[~skip], ref[~skip]
    if cf.size == 0:
        return
    scale = np.maximum(1, np.abs(ref).max(axis=-1, keepdims=True))
    rel = (np.abs(cf - ref) / scale).max()
    assert rel < CF_REL, f"{what}: contact forces off by {rel:.3e}"


def as_batch(r):
    """an oracle.rollout() result as a one-rollout batch() result"""
    out = dict(r)
    for k in ("tau", "cf", "flags"):
        out[k] = np.asarray(r[k])[None]
    out["work"], out["cot"] = np.array([r["work"]]), np.array([r["cot"]])
    return out


def reference_agreement(oracle_mod, omodel, gaits, r, steps, basis, n_t=20, k0=0):
    """For the [B][H] mask `steps`: (agree, other) -- agree marks the steps where the oracle result r
    (null basis `basis`) and the same restatement in the other reference-faithful basis agree within
    the parity bounds (torques 1e-6 N*m and 1e-9 relative, contact forces 1e-8 relative), so the
    reference's answer does not depend on the near-threshold decision; other: that basis's torques
    ([B][H][nmj], only the rows of rollouts with a step in the mask filled)."""
    agree = np.zeros(steps.shape, bool)
    other = np.full(r["tau"].shape, np.nan)
    rows = np.nonzero(steps.any(axis=1))[0]
    if rows.size == 0:
        return agree, other
    alt = oracle_mod.BASIS_ORTHO if basis == oracle_mod.BASIS_TREE else oracle_mod.BASIS_TREE
    H = steps.shape[1]
    o = oracle_mod.batch(omodel, [gaits[i] for i in rows], n_t, k0, H, basis=alt, n_threads=threads())
    t, c = r["tau"][rows], r["cf"][rows]
    et = np.abs(t - o["tau"]).max(axis=-1)
    ec = np.abs(c - o["cf"]).max(axis=-1) / np.maximum(1, np.abs(c).max(axis=-1))
    ok = (et < TAU_ABS) & (et / np.maximum(1, np.abs(t).max(axis=-1)) < TAU_REL) & (ec < CF_REL)
    agree[rows] = ok & steps[rows]
    other[rows] = o["tau"]
    return agree, other


def compare(what, g, r, oracle_mod, omodel, gaits, basis, n_t=20, k0=0, max_excluded=0.0, cf=True, flags=True,
            work=True, min_work=0.9):
    """The kernel's batch g (tau, cf, flags [, work_cot]; [B][H][...]) against the oracle's r in null
    basis `basis`: every bound on every step except those flagged HS_FLAG_NEAR_RANK (either side) whose
    two reference-faithful answers disagree (reference_agreement). Asserts that excluded share <=
    max_excluded, prints the counts, and compares the work of every rollout without an excluded step
    (at least a fraction min_work of the rollouts). Returns the excluded mask."""
    flagged = near(g["flags"], r["flags"])
    agree, other = reference_agreement(oracle_mod, omodel, gaits, r, flagged, basis, n_t, k0)
    excl = flagged & ~agree
    if flagged.any():
        e = np.abs(g["tau"] - r["tau"]).max(axis=-1)
        eo = np.abs(g["tau"] - other).max(axis=-1)
        msg = (f"{what}: {int(flagged.sum())} of {flagged.size} steps flagged HS_FLAG_NEAR_RANK; "
               f"{int(agree.sum())} compared (tree and ortho agree; max |dtau| there {e[agree].max() if agree.any() else 0:.2e})")
        if excl.any():
            # per excluded step: the kernel's distance to the NEARER of the two reference answers, against
            # their spread (round 3's rule): the kernel must land on one of them
            d = np.minimum(e, eo)
            spread = np.abs(r["tau"] - other).max(axis=-1)
            on_one = d <= np.maximum(TAU_ABS, 10 * spread)
            msg += (f"; {int(excl.sum())} excluded ({100 * excl.mean():.3f} %: the two reference answers disagree, "
                    f"spread up to {np.nanmax(spread[excl]):.2e}); per step the kernel is within 10x the spread of "
                    f"one answer on {int(on_one[excl].sum())} of them, max distance to the nearer answer "
                    f"{np.nanmax(d[excl]):.2e} (on {int((excl & (eo < e)).sum())} the nearer is the other basis)")
            if "near_kind" in r:
                kinds = {}
                for kk in r["near_kind"][excl]:
                    name = oracle_mod.NEAR_KINDS.get(int(kk), str(kk))
                    kinds[name] = kinds.get(name, 0) + 1
                flips = {}
                for kk in r["near_kind"][excl & (eo < e)]:
                    name = oracle_mod.NEAR_KINDS.get(int(kk), str(kk))
                    flips[name] = flips.get(name, 0) + 1
                msg += f"; the oracle's nearest decision on them {kinds}, where the kernel took the other answer {flips}"
        print(msg)
    assert excl.mean() <= max_excluded, f"{what}: {100 * excl.mean():.3f} % of the steps excluded (limit {100 * max_excluded} %)"
    if excl.any():
        assert on_one[excl].mean() >= 0.95, \
            f"{what}: the kernel is within 10x the tree/ortho spread of either answer on only {int(on_one[excl].sum())} of {int(excl.sum())} excluded steps"
    check_tau(g["tau"], r["tau"], what, excl if excl.any() else None)
    if cf:
        check_cf(g["cf"], r["cf"], what, excl)
    if flags:
        check_flags(g["flags"], r["flags"], what, excl)
    if work and "work_cot" in g:
        whole = ~excl.any(axis=1) & np.isfinite(r["cot"])
        assert whole.sum() >= max(1, int(np.ceil(min_work * whole.size))), \
            f"{what}: work compared on only {int(whole.sum())} of {whole.size} rollouts"
        np.testing.assert_allclose(g["work_cot"][whole, 0], r["work"][whole], rtol=1e-9, atol=1e-12)
        np.testing.assert_allclose(g["work_cot"][whole, 1], r["cot"][whole], rtol=1e-9, atol=1e-12)
    return excl


def check_fast_every_step(what, g, f):
    """the kernel's closed form against the oracle's fast mode (the same closed form, same operation
    order) on EVERY step, no exclusion: neither side may flag a step here"""
    assert not near(f["flags"]).any(), f"{what}: the oracle's fast mode flagged {int(near(f['flags']).sum())} steps"
    assert not near(g["flags"]).any(), f"{what}: the kernel flagged {int(near(g['flags']).sum())} steps"
    check_tau(g["tau"], f["tau"], what + " vs fast")
    check_cf(g["cf"], f["cf"], what + " vs fast")
    check_flags(g["flags"], f["flags"], what + " vs fast")
    if "work_cot" in g:
        np.testing.assert_allclose(g["work_cot"][:, 0], f["work"], rtol=1e-9, atol=1e-12)


def fused_cycle(gpu, model, params, solve_mode=0, dtype=None, H=20):
    """H control steps of every rollout from k0 = 0 (H calls of horizon 1 through hs_run_calls, the
    bench's path): tau/cf/flags [B][H][...] on the host."""
    import torch

    b = gpu.DeviceBatch(model, params, n_t=20, k0=0, horizon=H, outputs=("tau", "cf", "flags", "work_cot"),
                        dtype=dtype)
    b.solve_mode = solve_mode
    b.work_cot.zero_()
    b.run_calls(H, call_horizon=1, best=False, accumulate=True)
    torch.cuda.synchronize()
    return {k: npy(getattr(b, k)) for k in ("tau", "cf", "flags", "work_cot")}


def test_configs1_full_size_matches_oracle_tree(gpu, hmodels, oracle_mod, omodels):
    """BASELINE configs[1] at full size: 4096 hexapod rollouts x the 20 steps of a cycle, the bench's
    fused path, every step against the oracle's tree mode (the same null basis)."""
    from hslabs_amd import synth

    params = synth.gen_params(4096, "hexapod")
    g = fused_cycle(gpu, hmodels["hexapod"], params)
    gaits = [record_to_oracle_gait(oracle_mod, r) for r in params]
    f = oracle_mod.batch(omodels["hexapod"], gaits, 20, 0, 20, basis=oracle_mod.BASIS_FAST, n_threads=threads())
    check_fast_every_step("configs[1]", g, f)  # all 81,920 steps, no exclusion
    r = oracle_mod.batch(omodels["hexapod"], gaits, 20, 0, 20, basis=oracle_mod.BASIS_TREE, n_threads=threads())
    compare("configs[1] vs tree", g, r, oracle_mod, omodels["hexapod"], gaits, oracle_mod.BASIS_TREE,
            max_excluded=0.001, min_work=0.99)


def test_configs3_last_rank_shard_matches_oracle(gpu, hmodels, oracle_mod, omodels):
    """BASELINE configs[3]'s per-rank workload at full size, through the bench's exact path: the LAST
    of 8 ranks' shard of the 262,144 rollouts (32,768 hexapod rollouts, global ids 229,376 ..
    262,143, rollout_id_base 229,376), K = 20 fused control steps with the best key (the launcher
    bench.py builds per rank: hs_run_calls, ~16k wavefronts per step, the fixup + reduce launch).
    Every step against the oracle's tree mode (ftsolver.cpp:78-102); the accumulated work bitwise
    equal to the per-step launches' (hs_run_steps, accumulate); the device best key equal to the
    host encoding of the accumulated selection COTs with the global ids (hdist.best_key, the minimum
    a caller of player.cpp:311-321 would take). The N > 1 RCCL reduce itself needs 8 GPUs: the
    launcher's sharding and reduce are covered by tests/test_bench_launcher.py."""
    import torch

    from hslabs_amd import dist as hdist
    from hslabs_amd import synth

    world, total, K = 8, 262144, 20
    id0, B = hdist.shard(total, world, world - 1)
    assert (id0, B) == (229376, 32768)
    model = hmodels["hexapod"]
    params = synth.gen_params(B, "hexapod", id0=id0)
    b = gpu.DeviceBatch(model, params, n_t=20, k0=0, horizon=K, outputs=("tau", "cf", "flags", "work_cot"),
                        rollout_id_base=id0)
    b.key_steps = K  # bench.py launcher_k
    b.work_cot.zero_()
    b.reset_best()
    launch = b.calls_launcher(K, call_horizon=1, best=True, accumulate=True)
    launch()
    torch.cuda.synchronize()
    g = {k: npy(getattr(b, k)) for k in ("tau", "cf", "flags", "work_cot")}
    gaits = [record_to_oracle_gait(oracle_mod, r) for r in params]
    f = oracle_mod.batch(omodels["hexapod"], gaits, 20, 0, K, basis=oracle_mod.BASIS_FAST, n_threads=threads())
    check_fast_every_step("configs[3] last rank", g, f)  # all 655,360 steps, no exclusion
    r = oracle_mod.batch(omodels["hexapod"], gaits, 20, 0, K, basis=oracle_mod.BASIS_TREE, n_threads=threads())
    compare("configs[3] last rank vs tree", g, r, oracle_mod, omodels["hexapod"], gaits, oracle_mod.BASIS_TREE,
            max_excluded=0.001, min_work=0.99)
    # the per-step launches accumulate the same work in the same order
    seq = gpu.DeviceBatch(model, params, n_t=20, k0=0, horizon=1, outputs=("work_cot",), rollout_id_base=id0)
    seq.work_cot.zero_()
    seq.run_steps(K, best=False, accumulate=True)
    torch.cuda.synchronize()
    assert np.array_equal(npy(seq.work_cot), g["work_cot"])
    # the shard's best key: the global id of the minimum selection COT
    sel = hdist.select_cot(b.work_cot[:, 0], torch.from_numpy(np.ascontiguousarray(params["step_length"])).cuda(),
                           model.total_mass, 20, K)
    host_key = int(hdist.best_key(sel, id0).item()) ^ hdist._FLIP
    assert int(b.best_key.item()) == host_key
    cot, rid = hdist.decode(torch.tensor([host_key ^ hdist._FLIP]))
    assert id0 <= rid < id0 + B and np.isfinite(cot)


def test_configs1_sample_matches_oracle_ortho(gpu, hmodels, oracle_mod, omodels):
    """256 rollouts of the same batch against the reference-faithful orthonormal null basis (the
    Q of a QR of B^T that SparseQR spans, ftsolver.cpp:185-202): basis invariance on the GPU."""
    from hslabs_amd import synth

    params = synth.gen_params(4096, "hexapod")[:256]
    g = fused_cycle(gpu, hmodels["hexapod"], params)
    gaits = [record_to_oracle_gait(oracle_mod, r) for r in params]
    r = oracle_mod.batch(omodels["hexapod"], gaits, 20, 0, 20, basis=oracle_mod.BASIS_ORTHO, n_threads=threads())
    compare("configs[1] sample vs ortho", g, r, oracle_mod, omodels["hexapod"], gaits, oracle_mod.BASIS_ORTHO,
            min_work=1.0)


@pytest.mark.parametrize("sid", PGS_IDS)
def test_reference_solve_mode_pgs_setups(gpu, hmodels, oracle_mod, omodels, sid):
    """HS_SOLVE_REFERENCE sends every step through the kernel's Eigen-style FullPivLU threshold
    loop + ColPivHouseholderQR (ftsolver.cpp:208-232): the same as the oracle's tree mode."""
    import torch

    p = gpu.read_pgs_config(PGS_CONFIG, sid)
    name = p.fname.replace(".xml", "")
    b = gpu.DeviceBatch(hmodels[name], [p], n_t=20, k0=0, horizon=20, outputs=("tau", "cf", "flags", "work_cot"))
    b.solve_mode = gpu.capi.HS_SOLVE_REFERENCE
    b.run(best=False)
    torch.cuda.synchronize()
    og = to_oracle_gait(oracle_mod, p)
    r = as_batch(oracle_mod.rollout(omodels[name], og, 20, basis=oracle_mod.BASIS_TREE))
    g = {k: npy(getattr(b, k)) for k in ("tau", "cf", "flags", "work_cot")}
    g["flags"] = g["flags"].astype(np.uint32)
    assert ((g["flags"] & GEN) != 0).all(), "every step must take the Eigen-style path"
    compare(f"pgs {sid} reference mode", g, r, oracle_mod, omodels[name], [og], oracle_mod.BASIS_TREE, min_work=1.0)


@pytest.mark.parametrize("name,curved", [("hexapod", False), ("hexapod", True), ("spider", True), ("myant", False)])
def test_reference_solve_mode_synthetic(gpu, hmodels, oracle_mod, omodels, name, curved):
    """The Eigen-style path on synthetic batches: 4-6 contacts of a hexapod (k = 12..18), 1-4 of
    myant, rank retries where they occur (the rollout's global-memory workspace, an out-of-line
    call from the 3-waves/SIMD kernel); the fused path (every step deferred by the step launch
    and solved by its fixup launch) equals the launch-per-call one bitwise."""
    import torch

    from hslabs_amd import synth

    params = synth.gen_params(256, name, id0=777, curved=curved)
    g = fused_cycle(gpu, hmodels[name], params, solve_mode=1)
    gaits = [record_to_oracle_gait(oracle_mod, r) for r in params]
    r = oracle_mod.batch(omodels[name], gaits, 20, 0, 20, basis=oracle_mod.BASIS_TREE, n_threads=threads())
    assert ((g["flags"] & GEN) != 0).all()
    compare(f"{name} reference mode", g, r, oracle_mod, omodels[name], gaits, oracle_mod.BASIS_TREE, min_work=1.0)
    seq = gpu.DeviceBatch(hmodels[name], params, n_t=20, k0=0, horizon=20, outputs=("tau", "cf", "flags"))
    seq.solve_mode = 1
    seq.run(best=False)
    torch.cuda.synchronize()
    assert np.array_equal(npy(seq.tau), g["tau"]) and np.array_equal(npy(seq.cf), g["cf"])


def test_full_rank_steps_match_oracle(gpu, hmodels, oracle_mod, omodels):
    """Steps with one foot down (k = 3): the zeroth-order Gram is full rank, and the reference's
    comma initializer `m << ntn1*Ny, ntn0*Ry` (ftsolver.cpp:223-224) gets a one-column empty kernel
    plus a k x k image, k + 1 columns for a k x k matrix: the reference, built without -DNDEBUG
    (makefile:1), aborts on Eigen's assertion there. The kernel returns the unique least-squares
    answer and flags the step HS_FLAG_FULL_RANK; the oracle's modes agree on it. Compared here on
    their own (round 1 excluded them)."""
    from hslabs_amd import synth

    params = synth.gen_params(1024, "myant")
    g = fused_cycle(gpu, hmodels["myant"], params)
    gaits = [record_to_oracle_gait(oracle_mod, r) for r in params]
    fr = (g["flags"] & 2) != 0
    assert fr.sum() >= 100, "the batch must contain single-contact steps"
    f = oracle_mod.batch(omodels["myant"], gaits, 20, 0, 20, basis=oracle_mod.BASIS_FAST, n_threads=threads())
    check_fast_every_step("myant batch", g, f)
    assert np.array_equal(fr, (f["flags"] & 2) != 0)
    r = oracle_mod.batch(omodels["myant"], gaits, 20, 0, 20, basis=oracle_mod.BASIS_TREE, n_threads=threads())
    excl = compare("myant batch vs tree", g, r, oracle_mod, omodels["myant"], gaits, oracle_mod.BASIS_TREE,
                   max_excluded=0.01, min_work=0.98)
    assert np.array_equal(fr[~excl], ((r["flags"] & 2) != 0)[~excl])


def test_fp32_configs2_matches_fp64_oracle(gpu, hmodels, oracle_mod, omodels):
    """BASELINE configs[2] (spider, 16384 rollouts x horizon 32, fp32) against the fp64 oracle
    directly (round 1 compared fp32 only with the fp64 kernel). A foot whose height is within
    rounding of the contact threshold (rcap + 1e-4) may switch contact sets between precisions; such
    steps are counted, and must be rare."""
    import torch

    from hslabs_amd import synth

    B, H = 16384, 32
    params = synth.gen_params(B, "spider")
    b = gpu.DeviceBatch(hmodels["spider"], params, n_t=20, k0=0, horizon=H, outputs=("tau", "cf", "flags"),
                        dtype=torch.float32)
    b.run(best=False)
    torch.cuda.synchronize()
    tau, cf, flags = npy(b.tau).astype(np.float64), npy(b.cf).astype(np.float64), npy(b.flags).astype(np.uint32)
    gaits = [record_to_oracle_gait(oracle_mod, r) for r in params]
    r = oracle_mod.batch(omodels["spider"], gaits, 20, 0, H, basis=oracle_mod.BASIS_TREE, n_threads=threads())
    down32 = (np.abs(cf.reshape(B, H, -1, 3)).max(axis=3) > 0)
    down64 = (np.abs(r["cf"].reshape(B, H, -1, 3)).max(axis=3) > 0)
    same = (down32 == down64).all(axis=2)
    assert same.mean() > 0.995, f"contact sets differ on {(~same).sum()} of {same.size} steps"
    flagged = near(flags, r["flags"])
    agree, _ = reference_agreement(oracle_mod, omodels["spider"], gaits, r, flagged & same, oracle_mod.BASIS_TREE)
    cmp = same & (~flagged | agree)
    print(f"configs[2] fp32: {int((same & flagged).sum())} of {int(same.sum())} same-contact steps flagged "
          f"HS_FLAG_NEAR_RANK, {int((same & flagged & ~agree).sum())} of them excluded (tree and ortho disagree)")
    assert cmp.sum() >= 0.99 * same.sum()
    check_flags(flags, r["flags"], "configs[2] fp32 vs fp64 oracle", ~cmp)
    scale = np.maximum(1, np.abs(r["tau"]).max(axis=2))
    err = np.abs(tau - r["tau"]).max(axis=2) / scale
    assert err[cmp].max() < FP32_TOL, f"fp32 vs fp64 oracle: {err[cmp].max():.3e}"
    assert np.median(err[cmp]) < 1e-5


@pytest.mark.parametrize("name", ["spider", "hexapod"])
def test_fp32_reference_solve_mode_matches_fp64_oracle(gpu, hmodels, oracle_mod, omodels, name):
    """The single-precision build's Eigen-style path (every step HS_SOLVE_REFERENCE) against the fp64
    oracle's tree mode, wherever both chose the same contact set. The path forms its Grams and runs
    FullPivLU / ColPivQR in double (round 5): in float the first stage's negligible pivots sat ~1e-6
    relative to the largest, within 4x of FullPivLU's eps * k on about a third of the hexapod's steps,
    so those steps were flagged rather than compared (round 4 required only 40 % unflagged). With the
    decisions taken on the Gram's exact rank structure the fp32 build flags what fp64 flags, the steps
    flagged on either side are compared wherever the oracle's tree and ortho answers agree, and at
    least 95 % of the same-contact steps must be compared. (In the product the fp32 build takes the
    closed form and falls back to this path only where the minimizer is not unique.)"""
    import torch

    from hslabs_amd import synth

    B, H = 256, 20
    params = synth.gen_params(B, name, id0=4242)
    b = gpu.DeviceBatch(hmodels[name], params, n_t=20, k0=0, horizon=H, outputs=("tau", "cf", "flags"),
                        dtype=torch.float32)
    b.solve_mode = gpu.capi.HS_SOLVE_REFERENCE
    b.run(best=False)
    torch.cuda.synchronize()
    tau, cf, flags = npy(b.tau).astype(np.float64), npy(b.cf).astype(np.float64), npy(b.flags).astype(np.uint32)
    assert ((flags & GEN) != 0).all()
    gaits = [record_to_oracle_gait(oracle_mod, r) for r in params]
    r = oracle_mod.batch(omodels[name], gaits, 20, 0, H, basis=oracle_mod.BASIS_TREE, n_threads=threads())
    down32 = (np.abs(cf.reshape(B, H, -1, 3)).max(axis=3) > 0)
    down64 = (np.abs(r["cf"].reshape(B, H, -1, 3)).max(axis=3) > 0)
    same = (down32 == down64).all(axis=2)
    assert same.mean() > 0.99, f"contact sets differ on {(~same).sum()} of {same.size} steps"
    assert np.isfinite(tau[same]).all()
    flagged = near(flags, r["flags"])
    agree, _ = reference_agreement(oracle_mod, omodels[name], gaits, r, flagged & same, oracle_mod.BASIS_TREE)
    cmp = same & (~flagged | agree)
    print(f"{name} fp32 reference mode: {int((same & flagged).sum())} of {int(same.sum())} same-contact steps "
          f"flagged HS_FLAG_NEAR_RANK (fp32 {int(near(flags).sum())}, fp64 oracle {int(near(r['flags']).sum())}), "
          f"{int((same & flagged & ~agree).sum())} of them excluded (tree and ortho disagree)")
    assert cmp.mean() >= 0.95
    scale = np.maximum(1, np.abs(r["tau"]).max(axis=2))
    err = np.abs(tau - r["tau"]).max(axis=2) / scale
    bad = err[cmp] >= FP32_TOL
    assert not bad.any(), f"fp32 reference mode vs fp64 oracle: {bad.sum()} of {bad.size} unflagged steps over the bound"
    assert np.median(err[cmp]) < 1e-5


def test_configs4_mixed_bench_size_matches_oracle(gpu, hmodels, oracle_mod, omodels):
    """BASELINE configs[4] at the bench's size: 4096 rollouts, myant and hexapod interleaved in one
    launch (bench.py --mixed: hs_run_mixed_calls, K = 20 fused control steps of horizon 1), every step
    of each model's rollouts against the oracle's fast mode with no exclusion and against its tree mode
    at the standard bounds (1e-6 N*m, 1e-9 relative; contact forces, flags, work)."""
    import torch

    from hslabs_amd import synth

    B, K = 4096, 20
    params, idx = synth.gen_mixed(B)
    ms = [hmodels[n] for n in synth.MIXED_MODELS]
    mb = gpu.MixedBatch(ms, idx, params, n_t=20, k0=0, horizon=K, outputs=("tau", "cf", "flags", "work_cot"))
    mb.work_cot.zero_()
    mb.run_calls(K, call_horizon=1, best=False, accumulate=True)
    torch.cuda.synchronize()
    out = {k: npy(getattr(mb, k)) for k in ("tau", "cf", "flags", "work_cot")}
    for k, name in enumerate(synth.MIXED_MODELS):
        sel = np.nonzero(idx == k)[0]
        m = hmodels[name]
        g = {"tau": out["tau"][sel][:, :, :m.nmj], "cf": out["cf"][sel][:, :, :3 * m.nfeet],
             "flags": out["flags"][sel], "work_cot": out["work_cot"][sel]}
        assert (out["tau"][sel][:, :, m.nmj:] == 0).all()
        gaits = [record_to_oracle_gait(oracle_mod, params[i]) for i in sel]
        f = oracle_mod.batch(omodels[name], gaits, 20, 0, K, basis=oracle_mod.BASIS_FAST, n_threads=threads())
        check_fast_every_step(f"configs[4] {name}", g, f)
        r = oracle_mod.batch(omodels[name], gaits, 20, 0, K, basis=oracle_mod.BASIS_TREE, n_threads=threads())
        compare(f"configs[4] {name} vs tree", g, r, oracle_mod, omodels[name], gaits, oracle_mod.BASIS_TREE,
                max_excluded=0.01, min_work=0.98)
