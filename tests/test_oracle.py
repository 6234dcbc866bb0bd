"""Oracle pinning (CPU): the reference's own self-checks restated as known-answer
tests, analytic properties of the force/torque system, and an independent
numpy/scipy formulation of the ftsolver problem. The reference binary cannot be
built here, so these are what pins the oracle.
"""
import os

import numpy as np
import pytest
import scipy.linalg as sla

from conftest import MODELS, PGS_CONFIG, PGS_IDS


def pgs(O, sid):
    return O.load_pgs_config(PGS_CONFIG, sid)


def model_for(O, omodels, g):
    return omodels[g.xml_file.replace(".xml", "")]


# --- visualization.cpp:24 rot_ztov built-in check: R z = v/|v| ------------------------------
@pytest.mark.parametrize("v", [(0, 1, 0), (1, 0, 0), (0, 0, 1), (0, 0, -1), (0, 0, -0.1), (0.4, 0.2, 0),
                               (-0.4, -0.2, 0), (0.3, -0.5, 0.7), (1e-12, 0, -1)])
def test_rot_ztov_maps_z_to_v(oracle_mod, v):
    R = oracle_mod.rot_ztov(v)
    v = np.asarray(v, float)
    # |v x z| < 1e-10 takes the (0,1,0) fallback axis: exact only to the reference's own 1e-3 check
    tiny = np.linalg.norm(np.cross(v, [0, 0, 1])) < 1e-10
    assert np.allclose(R @ [0, 0, 1], v / np.linalg.norm(v), atol=1e-3 if tiny else 1e-12)
    assert np.allclose(R @ R.T, np.eye(3), atol=1e-12)
    assert np.linalg.det(R) == pytest.approx(1.0, abs=1e-12)


# --- pergen.cpp:377-383 Euler round trip -------------------------------------------------------
def test_euler_roundtrip(oracle_mod):
    rng = np.random.default_rng(0)
    for _ in range(500):
        a = np.array([rng.uniform(-np.pi, np.pi), rng.uniform(-1.5, 1.5), rng.uniform(-np.pi, np.pi)])
        assert np.allclose(oracle_mod.euler_roundtrip(a), a, atol=1e-12)


# --- lik.cpp:371-404 solver_test_yxx (tolerance of the reference: 1e-3) -----------------------
@pytest.mark.parametrize("name", ["hexapod", "myant"])
def test_lik_roundtrip(oracle_mod, omodels, name):
    err = oracle_mod.lik_roundtrip(omodels[name], 2000, seed=7)
    assert err < 1e-9


# --- FK after IK reproduces the pergen foot targets -------------------------------------------
@pytest.mark.parametrize("sid", [0, 8, 10, 20, 23, 24, 25, 26, 27])
def test_fk_ik_feet_on_targets(oracle_mod, omodels, sid):
    g = pgs(oracle_mod, sid)
    m = model_for(oracle_mod, omodels, g)
    for t in np.linspace(0, 2 * g.period, 13):
        assert oracle_mod.fk_ik_check(m, g, t) < 1e-12


# --- B0 x0 = f and [B0 Bc] N = 0 (SURVEY.md 8c KAT 2) ---------------------------------------------
@pytest.mark.parametrize("sid", [0, 3, 8, 9, 20, 23, 24])
@pytest.mark.parametrize("basis", [0, 1])
def test_system_residuals(oracle_mod, omodels, sid, basis):
    g = pgs(oracle_mod, sid)
    m = model_for(oracle_mod, omodels, g)
    for step in (0, 5, 11):
        k, r0, r1 = oracle_mod.residuals(m, g, 20, step, basis)
        assert k % 3 == 0 and k > 0
        assert r0 < 1e-12 and r1 < 1e-12


# --- basis invariance: tree-built basis == orthonormal QR basis (SURVEY.md 8c KAT 5) -------------
@pytest.mark.parametrize("sid", PGS_IDS)
def test_basis_invariance(oracle_mod, omodels, sid):
    g = pgs(oracle_mod, sid)
    m = model_for(oracle_mod, omodels, g)
    ro = oracle_mod.rollout(m, g, 20, basis=oracle_mod.BASIS_ORTHO)
    rt = oracle_mod.rollout(m, g, 20, basis=oracle_mod.BASIS_TREE)
    assert np.abs(ro["tau"] - rt["tau"]).max() < 1e-9
    assert np.abs(ro["cf"] - rt["cf"]).max() < 1e-9
    assert abs(ro["cot"] - rt["cot"]) <= 1e-9 * abs(ro["cot"])
    # the adaptive-rank loop converges first time on every shipped setup (ftsolver.cpp:228-232)
    assert (ro["diag"][:, 2] == 1).all() and (ro["diag"][:, 3] < 1e-6).all()
    assert ((ro["flags"] & ~np.uint32(oracle_mod.FLAG_NEAR_RANK)) == 0).all()  # rank decisions near a threshold aside


# --- static stance (pgs ids 4, 5, 11): sum of contact forces = total weight (g = 1, m = 1) -------
@pytest.mark.parametrize("sid,weight", [(4, 22.0), (11, 22.0), (5, 17.0)])
def test_static_stance_force_balance(oracle_mod, omodels, sid, weight):
    g = pgs(oracle_mod, sid)
    m = model_for(oracle_mod, omodels, g)
    r = oracle_mod.rollout(m, g, 20)
    total = r["cf"].reshape(20, -1, 3).sum(axis=1)
    assert np.allclose(total[:, 2], weight, rtol=1e-4)
    assert np.abs(total[:, :2]).max() < 1e-3
    n = m.n
    # all feet down: torso actuation is eliminated exactly (zeroth-order solve)
    assert np.abs(r["x"][:, :3]).max() < 1e-12 and np.abs(r["x"][:, 3 * n:3 * n + 3]).max() < 1e-12


# --- >= 3 non-collinear feet: zero torso actuation; 2 feet (myant): rank-5 remainder ----------------
@pytest.mark.parametrize("sid", [8, 23, 24])
def test_torso_actuation_eliminated(oracle_mod, omodels, sid):
    g = pgs(oracle_mod, sid)
    m = model_for(oracle_mod, omodels, g)
    r = oracle_mod.rollout(m, g, 20)
    assert (r["diag"][:, 0] >= 9).all() and (r["diag"][:, 1] == 6).all()
    n = m.n
    assert np.abs(r["x"][:, :3]).max() < 1e-12 and np.abs(r["x"][:, 3 * n:3 * n + 3]).max() < 1e-12


def test_two_feet_rank_five(oracle_mod, omodels):
    g = pgs(oracle_mod, 9)  # myant, two feet down in most phases
    r = oracle_mod.rollout(omodels["myant"], g, 20)
    two = r["diag"][:, 0] == 6
    assert two.any() and (r["diag"][two, 1] == 5).all()


# --- independent numpy/scipy formulation of ftsolver (lexicographic least squares via SVD) --------
def build_system(d, n):
    """B0, f, Bc from a dynamics record, written from dynrec.cpp:227-344 independently of the oracle."""
    def cross(r):
        return np.array([[0, -r[2], r[1]], [r[2], 0, -r[0]], [-r[1], r[0], 0]])

    B0 = np.zeros((6 * n, 6 * n))
    f = np.zeros(6 * n)
    for i in range(n):
        p = d["parents"][i]
        B0[3 * i:3 * i + 3, 3 * i:3 * i + 3] = np.eye(3)
        B0[3 * (n + i):3 * (n + i) + 3, 3 * (n + i):3 * (n + i) + 3] = np.eye(3)
        if p >= 0:
            B0[3 * p:3 * p + 3, 3 * i:3 * i + 3] = -np.eye(3)
            B0[3 * (n + p):3 * (n + p) + 3, 3 * (n + i):3 * (n + i) + 3] = -np.eye(3)
            B0[3 * (n + i):3 * (n + i) + 3, 3 * i:3 * i + 3] = cross(d["jpos"][i] - d["pos"][i])
            B0[3 * (n + p):3 * (n + p) + 3, 3 * i:3 * i + 3] = cross(d["pos"][p] - d["jpos"][i])
        f[3 * i:3 * i + 3] = d["mom_rate"][i] + np.array([0, 0, 1.0])
        f[3 * (n + i):3 * (n + i) + 3] = d["amr"][i]
    cols = []
    for fi in range(len(d["footis"])):
        if not d["contacts"][fi]:
            continue
        p = d["footis"][fi]
        c = np.zeros((6 * n, 3))
        c[3 * p:3 * p + 3] = np.eye(3)
        c[3 * (n + p):3 * (n + p) + 3] = cross(d["fpos"][fi] - d["pos"][p])
        cols.append(c)
    Bc = np.hstack(cols)
    return B0, f, Bc


def scipy_solve(d, n, force=True, torque=True):
    """force / torque: switch_torso_penalty's zeroth-order torso rows (ftsolver.cpp:262-273)"""
    B0, f, Bc = build_system(d, n)
    k = Bc.shape[1]
    xp = np.linalg.solve(B0, f)
    N = sla.null_space(np.hstack([B0, Bc]))  # (6n+k) x k, orthonormal
    assert N.shape[1] == k
    Nu = N[:6 * n]
    c = np.ones(6 * n)
    c[3:3 * n] = 0
    c[3 * n + 3:] = d["jz"].reshape(-1)[3:]
    m0 = np.zeros(6 * n, bool)
    m0[[0, 1, 2]] = force
    m0[[3 * n, 3 * n + 1, 3 * n + 2]] = torque
    A0, b0 = (c[:, None] * Nu)[m0], (c * xp)[m0]
    A1, b1 = (c[:, None] * Nu)[~m0], (c * xp)[~m0]
    y0 = -np.linalg.lstsq(A0, b0, rcond=1e-10)[0]
    Z = sla.null_space(A0, rcond=1e-10)
    w = -np.linalg.lstsq(A1 @ Z, b1 + A1 @ y0, rcond=None)[0]
    y = y0 + Z @ w
    x = xp + Nu @ y
    tau = np.array([d["jz"][h] @ x[3 * n + 3 * h:3 * n + 3 * h + 3] for h in d["hinge_ids"]])
    wforce = N[6 * n:] @ y
    cf = np.zeros(3 * len(d["footis"]))
    ci = 0
    for fi in range(len(d["footis"])):
        if d["contacts"][fi]:
            cf[3 * fi:3 * fi + 3] = wforce[3 * ci:3 * ci + 3]
            ci += 1
    return tau, cf


@pytest.mark.parametrize("sid", [0, 3, 8, 9, 10, 12, 20, 23, 24, 25, 26])
def test_independent_scipy_formulation(oracle_mod, omodels, sid):
    g = pgs(oracle_mod, sid)
    m = model_for(oracle_mod, omodels, g)
    r = oracle_mod.rollout(m, g, 20)
    for step in range(0, 20, 3):
        d = oracle_mod.dynrec_dump(m, g, 20, step)
        tau, cf = scipy_solve(d, m.n)
        scale = max(1.0, np.abs(r["tau"][step]).max())
        assert np.abs(tau - r["tau"][step]).max() < 1e-8 * scale
        assert np.abs(cf - r["cf"][step]).max() < 1e-8 * max(1.0, np.abs(cf).max())


# --- switch_torso_penalty(force, torque) other than (1,1) (ftsolver.cpp:262-273) ----------------
@pytest.mark.parametrize("force,torque", [(1, 0), (0, 1)])
@pytest.mark.parametrize("sid", [0, 8, 12, 24])
def test_torso_penalty_masks(oracle_mod, sid, force, torque):
    """mask0 = the chosen torso rows, mask1 = the rest (set_penal_mask1): both bases and the closed-form
    mode (which declines to the Eigen-style path) agree, the independent scipy formulation with the same
    masks agrees, and the zeroth-order rows come out exactly actuation-free"""
    g = pgs(oracle_mod, sid)
    m = oracle_mod.Model(os.path.join(MODELS, g.xml_file))  # not the shared fixture: the setting persists
    m.switch_torso_penalty(force, torque)
    ro = oracle_mod.rollout(m, g, 20, basis=oracle_mod.BASIS_ORTHO)
    rt = oracle_mod.rollout(m, g, 20, basis=oracle_mod.BASIS_TREE)
    rf = oracle_mod.rollout(m, g, 20, basis=oracle_mod.BASIS_FAST)
    scale = max(1.0, np.abs(ro["tau"]).max())
    assert np.abs(ro["tau"] - rt["tau"]).max() < 1e-9 * scale
    assert np.array_equal(rt["tau"], rf["tau"])
    contact = (rf["flags"] & oracle_mod.FLAG_NO_CONTACT) == 0
    assert ((rf["flags"][contact] & oracle_mod.FLAG_GENERAL) != 0).all()
    n = m.n
    rows = [0, 1, 2] if force else [3 * n, 3 * n + 1, 3 * n + 2]
    xs = ro["x"][contact][:, rows]
    assert np.abs(xs).max() < 1e-9 * max(1.0, np.abs(ro["x"]).max())
    for step in range(0, 20, 4):
        d = oracle_mod.dynrec_dump(m, g, 20, step)
        tau, cf = scipy_solve(d, n, bool(force), bool(torque))
        assert np.abs(tau - ro["tau"][step]).max() < 1e-8 * scale
        assert np.abs(cf - ro["cf"][step]).max() < 1e-8 * max(1.0, np.abs(cf).max())
    # the setting matters: (1,1) gives other torques
    m11 = oracle_mod.Model(os.path.join(MODELS, g.xml_file))
    r11 = oracle_mod.rollout(m11, g, 20, basis=oracle_mod.BASIS_ORTHO)
    assert np.abs(r11["tau"] - ro["tau"]).max() > 1e-6 * scale
    with pytest.raises(ValueError):
        m.switch_torso_penalty(False, False)  # the reference exits (ftsolver.cpp:245)


# --- COT sweep shape (player.cpp:311-321, main.cpp:69) ------------------------------------------
def test_cot_sweep_period(oracle_mod, omodels):
    g = pgs(oracle_mod, 8)
    cots = []
    for vali in range(16):  # sweep period 3 -> 18 in 15 steps (n_val + 1 values)
        g.period = 3 + vali * (18 - 3) / 15
        cots.append(oracle_mod.rollout(omodels["hexapod"], g, 20, basis=1)["cot"])
    cots = np.array(cots)
    assert np.isfinite(cots).all() and (cots > 0).all()
    # slower gaits need less positive work per distance
    assert cots[-1] < cots[0]


# --- the kernel's closed-form solve (oracle FAST mode) == Eigen-style two-stage LS ----------------
@pytest.mark.parametrize("sid", PGS_IDS)
def test_closed_form_matches_two_stage_ls(oracle_mod, omodels, sid):
    g = pgs(oracle_mod, sid)
    m = model_for(oracle_mod, omodels, g)
    ro = oracle_mod.rollout(m, g, 20, basis=oracle_mod.BASIS_ORTHO)
    rf = oracle_mod.rollout(m, g, 20, basis=oracle_mod.BASIS_FAST)
    scale = max(1.0, np.abs(ro["tau"]).max())
    assert np.abs(ro["tau"] - rf["tau"]).max() < 1e-12 * scale
    assert np.abs(ro["cf"] - rf["cf"]).max() < 1e-12 * max(1.0, np.abs(ro["cf"]).max())
    assert not (rf["flags"] & oracle_mod.FLAG_GENERAL).any()


@pytest.mark.parametrize("name,curved", [("hexapod", False), ("hexapod", True), ("spider", True), ("myant", False)])
def test_closed_form_synthetic(oracle_mod, omodels, name, curved):
    from hslabs_amd import synth
    from conftest import record_to_oracle_gait

    arr = synth.gen_params(200, name, curved=curved, id0=777)
    gs = [record_to_oracle_gait(oracle_mod, r) for r in arr]
    rt = oracle_mod.batch(omodels[name], gs, 20, 0, 20, basis=oracle_mod.BASIS_TREE, n_threads=8)
    rf = oracle_mod.batch(omodels[name], gs, 20, 0, 20, basis=oracle_mod.BASIS_FAST, n_threads=8)
    err = np.abs(rt["tau"] - rf["tau"]).max(axis=2) / np.maximum(1, np.abs(rt["tau"]).max(axis=2))
    assert err.max() < 1e-10
    assert ((rf["flags"] & oracle_mod.FLAG_GENERAL) != 0).mean() < 0.01


# myant rollouts of gen_params(4096, "myant") whose IK-clamped (straight) legs make a
# first-order Gram block D_c singular: the per-contact Schur solve declines them
DEGENERATE_MYANT = (497, 737, 844, 1084)


def test_position_control_law(oracle_mod, omodels):
    """player.cpp:388-432: on the target state the command is the feedforward torque; the
    feedback is linear with gains (-k, -2 sqrt k); angle errors wrap into (-pi, pi]."""
    g = pgs(oracle_mod, 8)
    m = omodels["hexapod"]
    r = oracle_mod.rollout(m, g, 20, basis=oracle_mod.BASIS_FAST)
    for tsi in (2, 9, 21, 0, 1, 40):
        q0, dq0, ff = oracle_mod.motor_adas(m, g, tsi, 20)
        lifted = tsi % 20 + (20 if tsi % 20 < 2 else 0)
        assert np.array_equal(ff, r["tau"][lifted - 2])  # get_computed_torques(tsi)
        assert np.array_equal(q0, r["q"][lifted, 6:])
        tau, _, _ = oracle_mod.pd_torques(m, g, tsi, q0, dq0)
        assert np.array_equal(tau, ff)
        dq = np.linspace(-1, 1, m.nmj)
        tau, _, _ = oracle_mod.pd_torques(m, g, tsi, q0 + 0.01, dq0 + dq, k=49.0)
        assert np.allclose(tau - ff, -49.0 * 0.01 - 14.0 * dq, rtol=1e-12, atol=1e-12)
        tau2, _, _ = oracle_mod.pd_torques(m, g, tsi, q0 + 0.01 + 2 * np.pi, dq0 + dq, k=49.0)
        assert np.allclose(tau2, tau, rtol=1e-12, atol=1e-9)


def test_augmented_closed_form_on_straight_legs(oracle_mod, omodels):
    """Steps with a singular D_c: the augmented-system tier (K = D + rho A^T A) reproduces the
    Eigen-style two-stage LS (tree and orthonormal bases) -- the minimizer is unique there."""
    from hslabs_amd import synth
    from conftest import record_to_oracle_gait

    arr = synth.gen_params(4096, "myant")[list(DEGENERATE_MYANT)]
    m = omodels["myant"]
    n_aug = 0
    for r in arr:
        g = record_to_oracle_gait(oracle_mod, r)
        rf = oracle_mod.rollout(m, g, 20, basis=oracle_mod.BASIS_FAST)
        assert not (rf["flags"] & oracle_mod.FLAG_GENERAL).any()
        n_aug += int(((rf["flags"] & 16) != 0).sum())
        for basis in (oracle_mod.BASIS_TREE, oracle_mod.BASIS_ORTHO):
            rt = oracle_mod.rollout(m, g, 20, basis=basis)
            assert np.abs(rt["tau"] - rf["tau"]).max() < 1e-10 * max(1.0, np.abs(rt["tau"]).max())
            assert np.abs(rt["cf"] - rf["cf"]).max() < 1e-10 * max(1.0, np.abs(rt["cf"]).max())
    assert n_aug >= 10  # the clamped steps are really exercised


# --- solve_forces (ftsolver.cpp:331-378): contact forces given motor torques --------------------
def dense_forces(d, n, z):
    """Independent numpy statement of solve_forces: B0 + all-feet contact columns + jz torque rows,
    torso columns dropped, np.linalg.lstsq."""
    nf = len(d["footis"])
    d2 = dict(d)
    d2["contacts"] = np.ones(nf, np.int32)  # contact_feet_flag = false: all feet
    B0, f, Bc = build_system(d2, n)
    nmj = len(d["hinge_ids"])
    Tr = np.zeros((nmj, 6 * n))
    for jj, h in enumerate(d["hinge_ids"]):
        Tr[jj, 3 * n + 3 * h:3 * n + 3 * h + 3] = d["jz"][h]
    Bf = np.block([[B0, Bc], [Tr, np.zeros((nmj, 3 * nf))]])
    keep = [c for c in range(Bf.shape[1]) if not (c < 3 or 3 * n <= c < 3 * n + 3)]
    sol = np.linalg.lstsq(Bf[:, keep], np.concatenate([f, z]), rcond=None)[0]
    return sol[-3 * nf:]


@pytest.mark.parametrize("sid", PGS_IDS)
def test_solve_forces_round_trip(oracle_mod, omodels, sid):
    """modelplayer::test_dynamics (playerexperim.cpp:95-121): the contact forces solve_forces
    recovers from solve_forcetorques' motor torques equal its contact forces wherever the
    torso actuation vanished (>= 3 feet down)."""
    g = pgs(oracle_mod, sid)
    m = model_for(oracle_mod, omodels, g)
    r = oracle_mod.rollout(m, g, 20, basis=oracle_mod.BASIS_FAST)
    fo = oracle_mod.forces(m, g, r["tau"], 20)
    nc = (np.abs(r["cf"].reshape(20, -1, 3)).max(axis=2) > 0).sum(axis=1)
    sel = nc >= 3
    assert sel.any()
    scale = max(1.0, np.abs(r["cf"]).max())
    assert np.abs(fo["cf"][sel] - r["cf"][sel]).max() < 1e-10 * scale
    assert not (fo["flags"] & oracle_mod.FLAG_GENERAL).any()


@pytest.mark.parametrize("name", ["hexapod", "spider", "myant"])
def test_solve_forces_matches_independent_lstsq(oracle_mod, omodels, name):
    """Arbitrary torques (inconsistent with the trajectory): the oracle's Householder LS equals
    numpy's lstsq of the same system."""
    from hslabs_amd import synth
    from conftest import record_to_oracle_gait

    m = omodels[name]
    for r in synth.gen_params(3, name, id0=321):
        g = record_to_oracle_gait(oracle_mod, r)
        ro = oracle_mod.rollout(m, g, 20, basis=oracle_mod.BASIS_FAST)
        z = ro["tau"] + 0.25 * np.cos(np.arange(20)[:, None] + np.arange(m.nmj)[None, :])
        fo = oracle_mod.forces(m, g, z, 20)
        for step in (0, 6, 15):
            ref = dense_forces(oracle_mod.dynrec_dump(m, g, 20, step), m.n, z[step])
            assert np.abs(fo["cf"][step] - ref).max() < 1e-10 * max(1.0, np.abs(ref).max())


def test_oracle_per_configuration_kinematics(oracle_mod, omodels):
    """The oracle's set_rec / set_jvalues_with_lik / recompute_modelnodes exports (checkers of
    hs_pergen_rec / hs_model_lik / hs_model_fk): FK after IK puts the feet (the nodes whose joint
    A_ground the oracle reports last in each limb chain) where fk_ik_check says, and the joint
    frames are rigid."""
    O = oracle_mod
    for name, gid in (("hexapod", 8), ("myant", 0), ("spider", 24)):
        m = omodels[name]
        p = O.load_pgs_config(os.path.join(MODELS, "pgs_config.txt"), gid)
        for t in (0.0, 0.7, 2.3):
            rec = O.pergen_rec(m, p, t)
            assert rec.shape == (6 + 3 * m.n_limbs,)
            q, ok, _ = O.set_jvalues_with_lik(m, rec, ignore_reach=True)
            assert ok and np.all(q[:6] == rec[:6])
            ag, aj = O.recompute_modelnodes(m, q)
            for A in list(ag) + [a for a in aj if np.any(a)]:
                R = A[:, :3]
                assert np.abs(R @ R.T - np.eye(3)).max() < 1e-14
            assert O.fk_ik_check(m, p, t) < 1e-12
            # the configuration is a fixed point: IK of the FK'd feet returns it
            q2, ok2, _ = O.set_jvalues_with_lik(m, rec, ignore_reach=True, config=q)
            assert ok2 and np.array_equal(q, q2)


# --- pergensetup::transform_rec (pergen.cpp:238, 309-342): the record transform ------------------
def _euler_R(a):
    """dRFromEulerAngles in the affine's layout (model.cpp:45): Rz(psi) Ry(theta) Rx(phi)"""
    phi, th, psi = a
    cx, sx, cy, sy, cz, sz = np.cos(phi), np.sin(phi), np.cos(th), np.sin(th), np.cos(psi), np.sin(psi)
    Rz = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]])
    Ry = np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]])
    Rx = np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    return Rz @ Ry @ Rx


def _angles_from(R):
    """euler_angles_from_affine (visualization.cpp:81-101)"""
    th = -np.arcsin(R[2, 0])
    c = np.cos(th)
    return np.array([np.arctan2(R[2, 1] / c, R[2, 2] / c), th, np.arctan2(R[1, 0] / c, R[0, 0] / c)])


def test_rec_transform_matches_rigid_motion(oracle_mod, omodels):
    """Records of a gait with a record transform (translation t, Euler angles e) equal the
    untransformed records moved rigidly: torso frame R(e) R0 with position R(e) p0 + t, every foot
    target R(e) f + t (an independent numpy formulation); the identity transform changes nothing."""
    from dataclasses import replace

    O = oracle_mod
    rng = np.random.default_rng(11)
    for sid in (8, 10, 24, 0):
        g = pgs(O, sid)
        m = model_for(O, omodels, g)
        n = m.n_limbs
        ident = replace(g, rec_transform=((0.0, 0.0, 0.0), (0.0, 0.0, 0.0)))
        for t in (0.0, 0.9, 2.7):
            assert np.abs(O.pergen_rec(m, ident, t) - O.pergen_rec(m, g, t)).max() < 1e-15
        for trial in range(6):
            tr = rng.uniform(-1, 1, 3) if trial else np.zeros(3)
            ea = np.array([0, 0, -1.571]) if trial == 0 else rng.uniform([-0.5, -0.5, -np.pi], [0.5, 0.5, np.pi])
            gx = replace(g, rec_transform=(tuple(tr), tuple(ea)))
            R = _euler_R(ea)
            for t in (0.0, 1.3, 4.1):
                r0 = O.pergen_rec(m, g, t)
                r1 = O.pergen_rec(m, gx, t)
                R1 = R @ _euler_R(r0[3:6])
                assert np.abs(r1[0:3] - (R @ r0[0:3] + tr)).max() < 1e-12
                assert np.abs(_euler_R(r1[3:6]) - R1).max() < 1e-12
                assert np.abs(r1[3:6] - _angles_from(R1)).max() < 1e-12
                feet0 = r0[6:].reshape(n, 3)
                assert np.abs(r1[6:].reshape(n, 3) - (feet0 @ R.T + tr)).max() < 1e-12


@pytest.mark.parametrize("sid", [8, 20, 23, 0])
def test_rec_transform_translation_keeps_the_dynamics(oracle_mod, omodels, sid):
    """A horizontal translation of the records is a symmetry of the path (gravity along z, the ground
    plane z = 0, contacts by foot height, every force/torque row built from position differences):
    joint values, motor torques, contact forces, work and COT equal the untransformed gait's. (A yaw
    is not one: the angular velocity is the rate of the skew part of R, dynrec.cpp:142-145, 179,
    which does not rotate with the frame.)"""
    from dataclasses import replace

    O = oracle_mod
    g = pgs(O, sid)
    m = model_for(O, omodels, g)
    base = O.rollout(m, g, 20, basis=O.BASIS_TREE)
    for tr in ((0.7, -0.4, 0.0), (-3.0, 5.0, 0.0)):
        r = O.rollout(m, replace(g, rec_transform=(tr, (0.0, 0.0, 0.0))), 20, basis=O.BASIS_TREE)
        scale = max(1.0, np.abs(base["tau"]).max())
        assert np.abs(r["tau"] - base["tau"]).max() < 1e-9 * scale
        nr = ~np.uint32(O.FLAG_NEAR_RANK)  # which decisions sit near a threshold moves with the rounding
        assert np.array_equal(r["flags"] & nr, base["flags"] & nr)
        assert r["cot"] == pytest.approx(base["cot"], rel=1e-9)
        assert np.abs(r["cf"] - base["cf"]).max() < 1e-8 * max(1.0, np.abs(base["cf"]).max())
        assert np.abs(r["q"][:, :2] - base["q"][:, :2] - np.array(tr[:2])).max() < 1e-12
        assert np.abs(r["q"][:, 2:] - base["q"][:, 2:]).max() < 1e-12


def test_zeroth_guard_routes_collinear_contacts(oracle_mod, omodels):
    """Tilted / lifted records can leave three same-side hexapod feet in contact, nearly on one line.
    The reference's loop (ftsolver.cpp:205-232) then finds its first pass inconsistent and retries at
    lower ranks (tree mode's RANK_RETRY), and its answer is not the closed form's exact minimizer (which
    runs to kN forces there). Fast mode's zeroth_well_posed guard hands those steps to the Eigen-style
    path (GENERAL), so fast mode equals tree mode on every step of the batch."""
    from conftest import record_to_oracle_gait, transformed
    from hslabs_amd import synth

    O = oracle_mod
    params, on = transformed(synth.gen_params(256, "hexapod", id0=900), np.random.default_rng(7))
    gaits = [record_to_oracle_gait(O, r) for r in params]
    rt = O.batch(omodels["hexapod"], gaits, 20, 0, 20, basis=O.BASIS_TREE, n_threads=8)
    rf = O.batch(omodels["hexapod"], gaits, 20, 0, 20, basis=O.BASIS_FAST, n_threads=8)
    retry = (rt["flags"] & O.FLAG_RANK_RETRY) != 0
    assert retry.sum() >= 3 and on[np.nonzero(retry)[0]].all()
    assert ((rf["flags"][retry] & O.FLAG_GENERAL) != 0).all()
    scale = np.maximum(1, np.abs(rt["tau"]).max(axis=-1, keepdims=True))
    assert (np.abs(rf["tau"] - rt["tau"]) / scale).max() < 1e-9
    nr = ~np.uint32(O.FLAG_GENERAL | O.FLAG_NEAR_RANK)  # which path ran, and its own near decisions
    assert np.array_equal(rf["flags"] & nr, rt["flags"] & nr)
    # every retry decided at a doubled threshold or a rel_error near the loop's 1e-6 is flagged
    assert ((rt["flags"][retry] & O.FLAG_NEAR_RANK) != 0).mean() >= 0.5


@pytest.mark.parametrize("name,curved", [("hexapod", False), ("hexapod", True), ("spider", True), ("myant", False)])
def test_near_rank_flag_rare_on_plain_gaits(oracle_mod, omodels, name, curved):
    """HSO_FLAG_NEAR_RANK (a rank or routing decision within rounding of its threshold, hs_oracle.cpp
    NearTrack; the kernel's HS_FLAG_NEAR_RANK) is rare on the plain synthetic gaits the bench runs: the
    closed form's guards sit far from their thresholds there (< 1 % of the steps in fast mode, the
    kernel's path). The Eigen-style path on every step (tree mode) meets FullPivLU's threshold more
    often: the zeroth-order Gram of >= 3 contacts has rank 6, and its rounding-level pivots sometimes
    land within 4x of eps * k; those steps are the ones a parity comparison leaves out."""
    from conftest import record_to_oracle_gait
    from hslabs_amd import synth

    O = oracle_mod
    params = synth.gen_params(512, name, id0=31337, curved=curved)
    gaits = [record_to_oracle_gait(O, r) for r in params]
    rf = O.batch(omodels[name], gaits, 20, 0, 20, basis=O.BASIS_FAST, n_threads=8)
    near = (rf["flags"] & O.FLAG_NEAR_RANK) != 0
    kinds = {O.NEAR_KINDS[k]: int((rf["near_kind"][near] == k).sum()) for k in np.unique(rf["near_kind"][near])}
    print(f"{name} curved={curved}: fast-mode near-rank steps {near.sum()} of {near.size} {kinds}")
    assert near.mean() < 0.01
    assert (rf["near_margin"][near] <= 1).all() and (rf["near_margin"][~near] > 1).all()
    rt = O.batch(omodels[name], gaits, 20, 0, 20, basis=O.BASIS_TREE, n_threads=8)
    print(f"  tree mode: {((rt['flags'] & O.FLAG_NEAR_RANK) != 0).mean():.2%} of the steps flagged")
    assert ((rt["flags"] & O.FLAG_NEAR_RANK) != 0).mean() < 0.1


def LIFTED_CASES(O):
    """torso lifted beyond reach (every leg clamped straight down): solve_forces' rank-deficient cases"""
    return [(name, O.GaitParams(xml_file=f"{name}.xml", torso_pos=(0.0, 0.0, lift), step_duration=1.0, period=3.0,
                                step_length=0.2, step_height=0.05))
            for name, lift in (("hexapod", 1.5), ("hexapod", 1.0), ("myant", 1.2))]


def forces_system(O, m, g, step, z):
    """the literal least-squares system of solve_forces at `step` (ftsolver.cpp:331-378), torso force /
    torque columns removed (they are zeroed): A [rows][cols], b, and the index of the first force column"""
    d = O.dynrec_dump(m, g, 20, int(step))
    nf, n = len(d["footis"]), m.n
    d2 = dict(d)
    d2["contacts"] = np.ones(nf, np.int32)
    B0, f, Bc = build_system(d2, n)
    Tr = np.zeros((m.nmj, 6 * n))
    for jj, h in enumerate(d["hinge_ids"]):
        Tr[jj, 3 * n + 3 * h:3 * n + 3 * h + 3] = d["jz"][h]
    A = np.block([[B0, Bc], [Tr, np.zeros((m.nmj, 3 * nf))]])
    keep = [c for c in range(A.shape[1]) if not (c < 3 or 3 * n <= c < 3 * n + 3)]
    return A[:, keep], np.concatenate([f, z]), A[:, keep].shape[1] - 3 * nf


def test_solve_forces_kernel_rule_vs_sparseqr_rule(oracle_mod, omodels):
    """solve_forces' rank rule (VERDICT r04 missing 3): the reference factorizes the literal
    system with SparseQR (ftsolver.cpp:349-353), whose default threshold drops a column when its
    Householder |r_kk| falls under 20 (rows + cols) eps max_j |A_j| (~1e-12 relative here; Eigen 3.3
    SparseQR::factorize); the kernel (and the oracle's default rule) drops a force column whose squared
    pivot in the reduced normal equations falls under 1e-10 of the largest diagonal (|r_kk| ~1e-5
    relative) -- the normal equations square the conditioning, so the kernel cannot resolve SparseQR's
    threshold. hso_forces_rule restates SparseQR's rule (natural column order: COLAMD is not restated)
    and this test quantifies the difference on the lifted-torso cases: where neither rule drops a column
    the forces are bitwise equal; where the kernel rule drops more, both answers are least-squares
    solutions over their kept columns, SparseQR's residual is never larger (it keeps a superset), and the
    kernel rule's extra residual is printed with the force difference (SparseQR's answer there is the
    ill-conditioned one: kN forces). Such steps carry HS_FLAG_DEPENDENT, and parity with the reference
    is not claimed on them (include/hslabs.h)."""
    O = oracle_mod
    both_full = differ = 0
    worst = (0.0, 0.0, 0.0)
    for name, g in LIFTED_CASES(O):
        m = omodels[name]
        ro = O.rollout(m, g, 20, basis=O.BASIS_FAST)
        z = ro["tau"] + 0.25 * np.cos(np.arange(20)[:, None] + np.arange(m.nmj)[None, :])
        fk = O.forces(m, g, z, 20, rule=O.FORCES_KERNEL)
        fs = O.forces(m, g, z, 20, rule=O.FORCES_SPARSEQR)
        dk, ds = (fk["flags"] & O.FLAG_DEPENDENT) != 0, (fs["flags"] & O.FLAG_DEPENDENT) != 0
        assert not (ds & ~dk).any()  # SparseQR's threshold is the lower one
        full = ~dk & ~ds
        both_full += int(full.sum())
        assert np.array_equal(fk["cf"][full], fs["cf"][full])
        for step in np.nonzero(dk & ~ds)[0]:
            A, b, y0 = forces_system(O, m, g, step, z[step])
            res = []
            for y in (fk["cf"][step], fs["cf"][step]):  # the wrenches' least squares given the forces
                r = b - A[:, y0:] @ y
                xw = np.linalg.lstsq(A[:, :y0], r, rcond=None)[0]
                res.append(np.linalg.norm(A[:, :y0] @ xw - r))
            rk, rs = res
            assert rs <= rk * (1 + 1e-9) + 1e-12, f"{name} step {step}: SparseQR residual {rs} > kernel rule {rk}"
            dy = np.abs(fk["cf"][step] - fs["cf"][step]).max()
            worst = max(worst, (dy, rk - rs, np.linalg.norm(b)))
            differ += 1
    print(f"solve_forces rank rules on the lifted-torso cases: {both_full} steps full rank under both (forces "
          f"bitwise equal), {differ} where only the kernel rule drops a column: forces differ by up to "
          f"{worst[0]:.3g} N, the kernel rule's residual exceeds SparseQR's by {worst[1]:.3g} (|b| = {worst[2]:.3g})")
    assert both_full >= 10 and differ >= 5


def test_solve_forces_rank_deficient_basic_solution(oracle_mod, omodels):
    """solve_forces where the least squares is (nearly) rank deficient (ftsolver.cpp:349-353: the
    reference solves with SparseQR and returns its basic solution). With the torso lifted beyond
    reach every leg is clamped straight down, and the feet's forces along the legs meet only the
    torso's force / torque rows: the reduced normal matrix has a direction 1e-11 below its largest
    eigenvalue. The oracle (and the kernel's chol_packed, on the same squared pivot) drop a force
    column whose pivot falls to 1e-10 of the largest reduced diagonal, in the natural column order,
    and return the basic solution, flagged HSO_FLAG_GENERAL. Checked against numpy: the dropped
    components are exactly 0 and the answer is the least-squares solution over the kept columns
    (residual orthogonal to them). Printed: how far it lies from the full least-squares solution
    numpy's lstsq gives (the reference's SparseQR, whose threshold is ~20 (m + n) eps on |r_kk|,
    keeps such a column and returns that ill-conditioned solution: parity there is not claimed)."""
    O = oracle_mod
    n_def = 0
    for name, g in LIFTED_CASES(O):
        m = omodels[name]
        ro = O.rollout(m, g, 20, basis=O.BASIS_FAST)
        z = ro["tau"] + 0.25 * np.cos(np.arange(20)[:, None] + np.arange(m.nmj)[None, :])
        fo = O.forces(m, g, z, 20)
        assert np.array_equal((fo["flags"] & O.FLAG_GENERAL) != 0, (fo["flags"] & O.FLAG_DEPENDENT) != 0)
        for step in np.nonzero((fo["flags"] & O.FLAG_GENERAL) != 0)[0]:
            nf = m.nf
            A, b, _ = forces_system(O, m, g, step, z[step])
            assert np.isfinite(A).all() and np.isfinite(b).all(), f"{name} step {step}"
            y = fo["cf"][step]
            dropped = np.nonzero(y == 0)[0]
            assert len(dropped) >= 1
            kept = [c for c in range(A.shape[1]) if c - (A.shape[1] - 3 * nf) not in set(dropped)]
            Ak = A[:, kept]
            xk = np.linalg.lstsq(Ak, b, rcond=None)[0]  # the least squares over the kept columns
            yk = np.zeros(3 * nf)
            yk[[c - (A.shape[1] - 3 * nf) for c in kept if c >= A.shape[1] - 3 * nf]] = xk[-(3 * nf - len(dropped)):]
            scale = max(1.0, np.abs(yk).max())
            assert np.abs(y - yk).max() < 1e-7 * scale, f"{name} step {step}: {np.abs(y - yk).max():.3e}"
            full = np.linalg.lstsq(A, b, rcond=None)[0][-3 * nf:]
            res_b = np.linalg.norm(Ak @ xk - b)
            res_f = np.linalg.norm(A @ np.linalg.lstsq(A, b, rcond=None)[0] - b)
            n_def += 1
            if n_def <= 4:
                print(f"{name} step {step}: basic solution drops {len(dropped)} component(s); vs the full least squares "
                      f"the forces differ by up to {np.abs(y - full).max():.3g} N (largest {np.abs(full).max():.3g} N), "
                      f"residual {res_b:.6g} vs {res_f:.6g}")
    assert n_def >= 5
