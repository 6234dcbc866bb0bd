"""GPU parity at BASELINE sizes and on the solve paths round 1 left untested.

The oracle is the CPU restatement (oracle/, parity with the reference binary unpinned: SURVEY.md
8c); its three modes agree with each other to ~1e-12 on every step of these
batches, full-rank steps included (measured on CPU: fast vs tree <= 3e-12, ortho vs tree <= 5e-13).

Tolerances (written here, per the north_star): fp64 per-joint motor torque |GPU - oracle| <
1e-6 N*m (the north_star bound) and < 1e-9 * max(1, |tau|) (what the kernel achieves: ULPs of the
device transcendentals amplified by the 1 / (4 dt^2) stencil); contact forces < 1e-8 * max(1, |f|);
flags identical (HS_FLAG_GENERAL and HS_FLAG_NEAR_RANK aside). fp32 (configs[2]): 1e-3 * max(1, |tau|)
wherever the fp32 run chose the same contact set as the fp64 oracle.

Every bound holds on EVERY step that neither side flags HS_FLAG_NEAR_RANK (include/hslabs.h; the
oracle's HSO_FLAG_NEAR_RANK, hs_oracle.cpp NearTrack): a rank or routing decision within rounding of
its threshold (FullPivLU pivots within 4x of the rank threshold, a doubled threshold, rel_error in
[1e-7, 1e-5], ColPivQR pivots, the closed form's guards; ftsolver.cpp:205-232), where another rounding
may take the decision the other way (hard part 2: flagged, not silently compared). The
flagged steps are counted and printed; they must be finite.
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
    """both bounds on every step (rows [..., nmj]) outside `skip` (steps flagged near a decision on
    either side); skipped steps must be finite, and are counted"""
    if skip is not None:
        assert np.isfinite(tau[skip]).all(), f"{what}: non-finite torques on flagged steps"
        if skip.any():
            print(f"{what}: {int(skip.sum())} of {skip.size} steps flagged HS_FLAG_NEAR_RANK, not compared")
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
    r = oracle_mod.batch(omodels["hexapod"], gaits, 20, 0, 20, basis=oracle_mod.BASIS_TREE, n_threads=threads())
    skip = near(g["flags"], r["flags"])
    assert not near(g["flags"]).any()  # the closed form's guards sit far from their thresholds on these gaits
    check_tau(g["tau"], r["tau"], "configs[1] vs tree", skip)
    check_cf(g["cf"], r["cf"], "configs[1] vs tree", skip)
    check_flags(g["flags"], r["flags"], "configs[1] vs tree", skip)
    whole = ~skip.any(axis=1)  # the work sums every step of the rollout
    np.testing.assert_allclose(g["work_cot"][whole, 0], r["work"][whole], rtol=1e-9, atol=1e-12)


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
    r = oracle_mod.batch(omodels["hexapod"], gaits, 20, 0, K, basis=oracle_mod.BASIS_TREE, n_threads=threads())
    skip = near(g["flags"], r["flags"])
    check_tau(g["tau"], r["tau"], "configs[3] last rank vs tree", skip)
    check_cf(g["cf"], r["cf"], "configs[3] last rank vs tree", skip)
    check_flags(g["flags"], r["flags"], "configs[3] last rank vs tree", skip)
    whole = ~skip.any(axis=1)
    np.testing.assert_allclose(g["work_cot"][whole, 0], r["work"][whole], rtol=1e-9, atol=1e-12)
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
    skip = near(g["flags"], r["flags"])
    check_tau(g["tau"], r["tau"], "configs[1] sample vs ortho", skip)
    check_cf(g["cf"], r["cf"], "configs[1] sample vs ortho", skip)
    check_flags(g["flags"], r["flags"], "configs[1] sample vs ortho", skip)


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
    r = oracle_mod.rollout(omodels[name], to_oracle_gait(oracle_mod, p), 20, basis=oracle_mod.BASIS_TREE)
    flags = npy(b.flags)[0].astype(np.uint32)
    assert ((flags & GEN) != 0).all(), "every step must take the Eigen-style path"
    skip = near(flags, r["flags"])
    check_flags(flags, r["flags"], f"pgs {sid} reference mode", skip)
    check_tau(npy(b.tau)[0], r["tau"], f"pgs {sid} reference mode", skip)
    check_cf(npy(b.cf)[0], r["cf"], f"pgs {sid} reference mode", skip)
    if not skip.any():
        assert float(npy(b.work_cot)[0, 1]) == pytest.approx(r["cot"], rel=1e-9, abs=1e-12)


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
    skip = near(g["flags"], r["flags"])
    check_flags(g["flags"], r["flags"], f"{name} reference mode", skip)
    check_tau(g["tau"], r["tau"], f"{name} reference mode", skip)
    check_cf(g["cf"], r["cf"], f"{name} reference mode", skip)
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
    for basis in (oracle_mod.BASIS_TREE, oracle_mod.BASIS_FAST):
        r = oracle_mod.batch(omodels["myant"], gaits, 20, 0, 20, basis=basis, n_threads=threads())
        skip = near(g["flags"], r["flags"])
        assert np.array_equal(fr[~skip], ((r["flags"] & 2) != 0)[~skip])
        check_tau(g["tau"][fr], r["tau"][fr], "full-rank steps", skip[fr])
        check_cf(g["cf"][fr], r["cf"][fr], "full-rank steps", skip[fr])
        check_tau(g["tau"], r["tau"], "myant batch", skip)


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
    skip = near(flags, r["flags"])
    cmp = same & ~skip
    print(f"configs[2] fp32: {int((same & skip).sum())} of {int(same.sum())} same-contact steps flagged HS_FLAG_NEAR_RANK")
    check_flags(flags, r["flags"], "configs[2] fp32 vs fp64 oracle", ~cmp)
    scale = np.maximum(1, np.abs(r["tau"]).max(axis=2))
    err = np.abs(tau - r["tau"]).max(axis=2) / scale
    assert err[cmp].max() < FP32_TOL, f"fp32 vs fp64 oracle: {err[cmp].max():.3e}"
    assert np.median(err[cmp]) < 1e-5


@pytest.mark.parametrize("name", ["spider", "hexapod"])
def test_fp32_reference_solve_mode_matches_fp64_oracle(gpu, hmodels, oracle_mod, omodels, name):
    """The single-precision build's Eigen-style path (every step HS_SOLVE_REFERENCE, thresholds
    scaled to float) against the fp64 oracle's tree mode, wherever both chose the same contact set.
    The first stage's Gram is rank deficient by construction (>= 3 contacts), and in float its
    negligible pivots sit ~1e-6 relative to the largest, near FullPivLU's threshold (eps * k): a
    few steps in 10^3 resolve the rank differently from fp64 and land on another point of the
    first stage's solution set. The fp32 kernel flags those decisions (HS_FLAG_NEAR_RANK, its own
    pivots against its own threshold: on the hexapod's 4-6 contacts about a third of the steps, whose
    float rounding-level pivots land within 4x of eps * k), and the bound holds on every unflagged
    step; at least 40 % of the steps must be unflagged (in the product the fp32 build takes the closed
    form, which has no rank decisions, and falls back to this path only where the minimizer is not
    unique)."""
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
    skip = near(flags, r["flags"])
    cmp = same & ~skip
    print(f"{name} fp32 reference mode: {int((same & skip).sum())} of {int(same.sum())} same-contact steps "
          f"flagged HS_FLAG_NEAR_RANK (fp32 {int(near(flags).sum())}, fp64 oracle {int(near(r['flags']).sum())})")
    assert cmp.mean() > 0.4
    scale = np.maximum(1, np.abs(r["tau"]).max(axis=2))
    err = np.abs(tau - r["tau"]).max(axis=2) / scale
    bad = err[cmp] >= FP32_TOL
    assert not bad.any(), f"fp32 reference mode vs fp64 oracle: {bad.sum()} of {bad.size} unflagged steps over the bound"
    assert np.median(err[cmp]) < 1e-5
