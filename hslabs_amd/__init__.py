"""hslabs_amd -- MI355X-native batched legged-locomotion control-loop path.

pergen -> lik -> FK -> dynrec -> ftsolver -> motor torques, one wavefront per
gait rollout on gfx950, behind the C ABI in include/hslabs.h.
"""
from .api import (Comm, DeviceBatch, KinematicModel, MixedBatch, ModelPlayer, Periodic, PgsConfigParams, ShardedBatch, SimBatch,
                  complete_traj,
                  decode_best_key, save_2d_array,
                  params_array, read_pgs_config, run_host, GAIT_DTYPE)
from .capi import HSError

__all__ = ["Comm", "DeviceBatch", "KinematicModel", "MixedBatch", "ModelPlayer", "Periodic", "PgsConfigParams", "ShardedBatch",
           "SimBatch", "complete_traj",
           "save_2d_array", "decode_best_key",
           "params_array", "read_pgs_config", "run_host", "GAIT_DTYPE", "HSError"]
