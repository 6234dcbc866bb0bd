"""Generate the golden vectors in tests/golden/ from the oracle (reference-faithful
orthonormal-basis mode). Inputs are pgs_config.txt setups and a small synthetic
batch; outputs are the per-step motor torques, contact forces, trajectory
records, flags and the cycle work / COT. Run: python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402

PGS_IDS = [0, 3, 4, 8, 9, 10, 20, 23, 24, 25, 26]
N_T = 20


def main():
    cfg = os.path.join(ROOT, "models", "pgs_config.txt")
    models = {}
    for sid in PGS_IDS:
        g = O.load_pgs_config(cfg, sid)
        m = models.setdefault(g.xml_file, O.Model(os.path.join(ROOT, "models", g.xml_file)))
        r = O.rollout(m, g, N_T, basis=O.BASIS_ORTHO)
        np.savez_compressed(os.path.join(HERE, f"pgs_{sid:02d}.npz"), q=r["q"], tau=r["tau"], cf=r["cf"],
                            x=r["x"], flags=r["flags"], work=r["work"], cot=r["cot"], n_t=N_T, sid=sid,
                            xml=g.xml_file)
    # synthetic batch (hslabs_amd.synth stream, ids 0..15)
    from hslabs_amd import synth

    arr = synth.gen_params(16, "hexapod")
    m = models.setdefault("hexapod.xml", O.Model(os.path.join(ROOT, "models", "hexapod.xml")))
    taus, cfs, cots, works = [], [], [], []
    for rec in arr:
        g = O.GaitParams(torso_pos=tuple(rec["torso_pos"]), torso_angles=tuple(rec["torso_angles"]),
                         step_duration=float(rec["step_duration"]), period=float(rec["period"]),
                         step_length=float(rec["step_length"]), step_height=float(rec["step_height"]),
                         curvature=float(rec["curvature"]), foot_shift_type=int(rec["foot_shift_type"]),
                         foot_shift=float(rec["foot_shift"]))
        r = O.rollout(m, g, N_T, basis=O.BASIS_ORTHO)
        taus.append(r["tau"]); cfs.append(r["cf"]); cots.append(r["cot"]); works.append(r["work"])
    np.savez_compressed(os.path.join(HERE, "synth_hexapod16.npz"), params=arr.view(np.uint8).reshape(16, -1),
                        tau=np.array(taus), cf=np.array(cfs), cot=np.array(cots), work=np.array(works), n_t=N_T)
    print("golden written:", sorted(os.listdir(HERE)))


if __name__ == "__main__":
    main()
