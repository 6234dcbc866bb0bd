import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

MODELS = os.path.join(ROOT, "models")
PGS_CONFIG = os.path.join(MODELS, "pgs_config.txt")
GOLDEN = os.path.join(ROOT, "tests", "golden")
# pgs ids whose model XML ships with the reference (ids 28-32 name missing weaver*.xml)
PGS_IDS = list(range(28))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle as O

    O.build()
    return O


@pytest.fixture(scope="session")
def product():
    """The product package with its in-tree gfx950 library (built if stale)."""
    from hslabs_amd import build as b

    b.build()
    import hslabs_amd as H

    H.capi.load(build_if_missing=False)
    return H


@pytest.fixture(scope="session")
def omodels(oracle_mod):
    return {name: oracle_mod.Model(os.path.join(MODELS, f"{name}.xml")) for name in ("hexapod", "spider", "myant")}


def to_oracle_gait(O, p):
    """hslabs_amd.PgsConfigParams -> oracle GaitParams"""
    return O.GaitParams(torso_pos=tuple(p.torso_pos), torso_angles=tuple(p.torso_angles),
                        step_duration=p.step_duration, period=p.period, step_length=p.step_length,
                        step_height=p.step_height, curvature=p.curvature, foot_shift_type=p.foot_shift[0],
                        foot_shift=p.foot_shift[1], rec_transform=p.rec_transform)


def record_to_oracle_gait(O, r):
    """GAIT_DTYPE record -> oracle GaitParams"""
    return O.GaitParams(torso_pos=tuple(float(v) for v in r["torso_pos"]),
                        torso_angles=tuple(float(v) for v in r["torso_angles"]),
                        step_duration=float(r["step_duration"]), period=float(r["period"]),
                        step_length=float(r["step_length"]), step_height=float(r["step_height"]),
                        curvature=float(r["curvature"]), foot_shift_type=int(r["foot_shift_type"]),
                        foot_shift=float(r["foot_shift"]),
                        rec_transform=((tuple(float(v) for v in r["rec_transl"]), tuple(float(v) for v in r["rec_eas"]))
                                       if int(r["rec_transform_flag"]) else None))


def golden_params(raw):
    """GAIT_DTYPE records from a fixture's raw bytes [B][record]: fixtures of ABI <= 11 hold 128-byte
    records, whose first 104 bytes are the current record's (the record transform was added after)."""
    import numpy as np

    from hslabs_amd import GAIT_DTYPE

    raw = np.asarray(raw, dtype=np.uint8).reshape(len(raw), -1)
    out = np.zeros(raw.shape[0], GAIT_DTYPE)
    out.view(np.uint8).reshape(raw.shape[0], -1)[:, :104] = raw[:, :104]
    return out


def transformed(params, rng, frac=0.5, tilt=0.05):
    """a copy of the GAIT_DTYPE batch with a random record transform on about `frac` of its rollouts
    (yaw anywhere, roll / pitch within +-tilt, translation within +-1 horizontally and +-0.02 up)"""
    import numpy as np

    out = params.copy()
    on = rng.random(len(out)) < frac
    n = int(on.sum())
    out["rec_transform_flag"][on] = 1
    out["rec_transl"][on] = np.stack([rng.uniform(-1, 1, n), rng.uniform(-1, 1, n), rng.uniform(-0.02, 0.02, n)], 1)
    out["rec_eas"][on] = np.stack([rng.uniform(-tilt, tilt, n), rng.uniform(-tilt, tilt, n),
                                   rng.uniform(-np.pi, np.pi, n)], 1)
    return out, on
