"""Synthetic gait batches.

Base setup: pgs id 8 (pgs_config.txt:9, main.cpp:35) for hexapod, 24 for
spider, 9 for myant. Per-rollout parameters are drawn i.i.d. uniform from a
counter-based splitmix64 stream (seed 0x48534C616273 = "HSLabs"), counter =
global rollout id, so any shard of any batch is reproducible on its own:
period in [3,18] (main.cpp:69), step_length in [-0.5,0.5] (main.cpp:56),
step_height in [0.02,0.2], step_duration in [0,1] (main.cpp:70), torso
z-offset in [-0.47,-0.05] (pgs ids 3-20), curvature 0 or, in the curved
pass, in [-0.15,0.5] (pgs ids 23-27).
"""
from __future__ import annotations

import numpy as np

from .api import GAIT_DTYPE

SEED = 0x48534C616273
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)

BASE = {  # pgs_config.txt lines 9 / 25 / 10
    "hexapod": dict(torso_pos=(0.0, 0.0, -0.1), step_duration=1.0, period=3.0, step_length=0.5, step_height=0.1,
                    curvature=0.0, foot_shift=(-1, 0.0)),
    "spider": dict(torso_pos=(0.0, 0.0, 0.1), step_duration=1.0, period=3.0, step_length=0.5, step_height=0.1,
                   curvature=-0.15, foot_shift=(0, 0.4)),
    "myant": dict(torso_pos=(0.0, 0.0, -0.07), step_duration=1.0, period=3.0, step_length=0.5, step_height=0.1,
                  curvature=0.0, foot_shift=(-1, 0.0)),
}


def _splitmix(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(ids: np.ndarray, stream: int, lo: float, hi: float, seed: int = SEED) -> np.ndarray:
    """U[lo,hi) for (rollout id, stream) pairs, 53-bit resolution."""
    with np.errstate(over="ignore"):
        x = np.uint64(seed) + ids.astype(np.uint64) * np.uint64(16) + np.uint64(stream)
    u = (_splitmix(x) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return lo + (hi - lo) * u


def gen_params(n: int, model: str = "hexapod", id0: int = 0, curved: bool = False, seed: int = SEED) -> np.ndarray:
    base = BASE[model]
    ids = np.arange(id0, id0 + n, dtype=np.int64)
    arr = np.zeros(n, GAIT_DTYPE)
    arr["torso_pos"][:, 0] = base["torso_pos"][0]
    arr["torso_pos"][:, 1] = base["torso_pos"][1]
    if model == "hexapod":
        arr["torso_pos"][:, 2] = uniform(ids, 4, -0.47, -0.05, seed)
    elif model == "myant":
        arr["torso_pos"][:, 2] = uniform(ids, 4, -0.10, -0.02, seed)
    else:
        arr["torso_pos"][:, 2] = uniform(ids, 4, 0.0, 0.1, seed)
    arr["period"] = uniform(ids, 0, 3.0, 18.0, seed)
    arr["step_length"] = uniform(ids, 1, -0.5, 0.5, seed)
    arr["step_height"] = uniform(ids, 2, 0.02, 0.2, seed)
    arr["step_duration"] = uniform(ids, 3, 0.0, 1.0, seed)
    if curved:
        arr["curvature"] = uniform(ids, 5, -0.15, 0.5, seed)
    else:
        arr["curvature"] = base["curvature"]
    arr["foot_shift_type"] = base["foot_shift"][0]
    arr["foot_shift"] = base["foot_shift"][1]
    return arr


MIXED_MODELS = ("myant", "hexapod")


def gen_mixed(n: int, id0: int = 0, curved: bool = False, seed: int = SEED):
    """BASELINE configs[4]: a 50/50 myant / hexapod batch, interleaved by rollout id
    (even id -> myant, odd -> hexapod). Returns (params, model_index into MIXED_MODELS);
    each rollout's parameters are those gen_params draws for its id and model."""
    ids = np.arange(id0, id0 + n, dtype=np.int64)
    idx = (ids % 2).astype(np.int32)
    out = gen_params(n, MIXED_MODELS[0], id0, curved, seed)
    other = gen_params(n, MIXED_MODELS[1], id0, curved, seed)
    out[idx == 1] = other[idx == 1]
    return out, idx


def gen_sim_params(n: int, model: str = "hexapod", id0: int = 0, period: float = 3.0, seed: int = SEED) -> np.ndarray:
    """Closed-loop simulation batches: gen_params with one period for the whole batch, so every
    rollout's controller table has the same length n_t = int(T / play_dt + .5)
    (setup_per_controller, player.cpp:370-382; pgs id 8 has T = 3 -> n_t = 300 at play_dt = .01)."""
    arr = gen_params(n, model, id0, False, seed)
    arr["period"] = period
    return arr
