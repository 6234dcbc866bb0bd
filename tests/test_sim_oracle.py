"""Known-answer tests of the closed-loop simulation restatement (oracle/hs_oracle_sim.cpp).

ODE is not in this image, so the restated QuickStep cannot be compared with ODE
itself ("parity unpinned" against the reference binary). It is pinned here by
physics the reference's own setup implies:
  * dJointGetHingeAngle of bodies oriented at a configuration returns that
    configuration's joint values (the position controller of player.cpp:388-432
    compares exactly these);
  * free fall (no contact, no control) integrates v = -g t semi-implicitly with
    the joints exactly satisfied;
  * without gravity and contacts, the joint and motor forces are internal:
    total linear momentum stays zero;
  * a static stance (pgs ids 4/5/11: step length ~0) stands: the contact normal
    forces carry the weight n * g (all masses 1, g = 1, visualization.cpp:144);
  * the gait of pgs id 8 walks: the torso advances one step length per period,
    the joints track the planned angles.
"""
import numpy as np
import pytest

from conftest import MODELS, PGS_CONFIG

N_T = 300  # setup_per_controller: int(T / play_dt + .5), T = 3, play_dt = .01


@pytest.fixture(scope="module")
def hexapod(oracle_mod):
    return oracle_mod.Model(f"{MODELS}/hexapod.xml")


def tables(O, model, pgs_id, n_t=N_T):
    g = O.load_pgs_config(PGS_CONFIG, pgs_id)
    return (g,) + O.controller_tables(model, g, n_t)


def test_hinge_angle_of_oriented_configuration(oracle_mod, hexapod):
    O = oracle_mod
    g, qt, dqt, tt = tables(O, hexapod, 8)
    for h in (0, 77, 150, 299):
        body = O.sim_reset(hexapod, qt[h])
        q, dq = O.sim_hinges(hexapod, body)
        assert np.abs(q - qt[h, 6:]).max() < 1e-12
        assert np.abs(dq).max() == 0.0


@pytest.mark.parametrize("xml", ["myant.xml", "spider.xml"])
def test_hinge_angle_other_models(oracle_mod, xml):
    O = oracle_mod
    m = O.Model(f"{MODELS}/{xml}")
    pid = 9 if xml == "myant.xml" else 24
    g = O.load_pgs_config(PGS_CONFIG, pid)
    qt, _, _ = O.controller_tables(m, g, 100)
    body = O.sim_reset(m, qt[10])
    q, _ = O.sim_hinges(m, body)
    d = (q - qt[10, 6:] + np.pi) % (2 * np.pi) - np.pi  # ODE angles are in (-pi, pi]; spider IK exceeds pi
    assert np.abs(d).max() < 1e-12


def test_free_fall(oracle_mod, hexapod):
    O = oracle_mod
    g, qt, dqt, tt = tables(O, hexapod, 8)
    c = qt[0].copy()
    c[2] += 10.0  # high above the plane
    body = O.sim_reset(hexapod, c)
    n = 50
    P = O.SimParams(k=0.0)
    r = O.sim_run(hexapod, P, N_T, qt, dqt, tt, body, 0, 2, n)
    b = r["body"]
    # semi-implicit Euler: v_n = -n h g, z_n = z_0 - h^2 g n (n + 1) / 2
    assert np.abs(b[:, 9] + n * P.dt * P.gravity).max() < 1e-12
    assert np.abs(b[:, 7:9]).max() < 1e-12 and np.abs(b[:, 10:13]).max() < 1e-12
    dz = b[:, 2] - body[:, 2]
    assert np.abs(dz + P.dt ** 2 * P.gravity * n * (n + 1) / 2).max() < 1e-10
    q, _ = O.sim_hinges(hexapod, b)
    assert np.abs(q - qt[0, 6:]).max() < 1e-12
    assert (r["n_contacts"] == 0).all()


def test_linear_momentum_without_gravity_and_contacts(oracle_mod, hexapod):
    O = oracle_mod
    g, qt, dqt, tt = tables(O, hexapod, 8)
    c = qt[0].copy()
    c[2] += 10.0
    body = O.sim_reset(hexapod, c)
    P = O.SimParams(gravity=0.0)  # position control on: motors exert internal torques
    r = O.sim_run(hexapod, P, N_T, qt, dqt, tt, body, 0, 2, 200)
    b = r["body"]
    assert np.abs(r["tau_cmd"]).max() > 1.0  # the motors did work
    assert np.abs(b[:, 7:10].sum(axis=0)).max() < 1e-10  # all masses 1
    assert np.abs(b[:, 10:13]).max() > 1e-3


@pytest.mark.parametrize("pgs_id", [4, 5])
def test_static_stance_carries_the_weight(oracle_mod, hexapod, pgs_id):
    O = oracle_mod
    g, qt, dqt, tt = tables(O, hexapod, pgs_id)
    body = O.sim_reset(hexapod, qt[0])
    r = O.sim_run(hexapod, O.SimParams(), N_T, qt, dqt, tt, body, 0, 2, 300)
    late = slice(200, 300)
    weight = hexapod.n * 1.0  # 22 parts of mass 1, g = 1
    assert (r["n_contacts"][late] >= 6).all()
    assert abs(r["normal_force"][late].mean() - weight) < 0.02 * weight
    z = r["torso"][:, 2]
    assert np.abs(z - body[0, 2]).max() < 0.02
    assert np.abs(r["torso"][-1, :2] - body[0, :2]).max() < 0.02


def test_walking_gait_advances_and_tracks(oracle_mod, hexapod):
    O = oracle_mod
    g, qt, dqt, tt = tables(O, hexapod, 8)
    body = O.sim_reset(hexapod, qt[0])
    n = 2 * N_T  # two periods
    r = O.sim_run(hexapod, O.SimParams(), N_T, qt, dqt, tt, body, 0, 2, n)
    adv = r["torso"][-1, 0] - body[0, 0]
    assert abs(adv - 2 * g.step_length) < 0.2 * 2 * g.step_length
    rows = (np.arange(2, 2 + n) % N_T + N_T - 2) % N_T
    err = r["q_meas"] - qt[rows, 6:]
    err = (err + np.pi) % (2 * np.pi) - np.pi
    assert np.abs(err).max() < 0.1
    z = r["torso"][:, 2]
    assert z.min() > body[0, 2] - 0.05 and z.max() < body[0, 2] + 0.05
    assert 0.5 * hexapod.n < r["normal_force"][N_T:].mean() < 1.5 * hexapod.n


def test_determinism_and_seed_advance(oracle_mod, hexapod):
    O = oracle_mod
    g, qt, dqt, tt = tables(O, hexapod, 8)
    body = O.sim_reset(hexapod, qt[0])
    a = O.sim_run(hexapod, O.SimParams(), N_T, qt, dqt, tt, body, 0, 2, 30)
    b1 = O.sim_run(hexapod, O.SimParams(), N_T, qt, dqt, tt, body, 0, 2, 10)
    b2 = O.sim_run(hexapod, O.SimParams(), N_T, qt, dqt, tt, b1["body"], b1["seed"], b1["tsi"], 20)
    assert np.array_equal(a["body"], b2["body"])  # state + seed + tsi fully describe a rollout
    assert a["tsi"] == 32 and a["seed"] != 0


def test_dRandInt_sequence():
    """ODE's dRand LCG (misc.cpp) restated: seed' = 1664525 seed + 1013904223 mod 2^32."""
    seed = 0
    seq = []
    for _ in range(3):
        seed = (1664525 * seed + 1013904223) & 0xFFFFFFFF
        seq.append(seed)
    assert seq == [1013904223, 1196435762, 3519870697]
