"""GPU vs oracle parity report over every pgs_config.txt setup (diagnostic tool).

Usage: python tools/parity_report.py [--n_t 20] [--random 64]
Prints, per setup, max |GPU - oracle| for q (mod 2pi), tau, cf, x, COT, against
the oracle's closed-form mode (same operation sequence as the kernel's fast
path), its tree-basis two-stage LS mode and its reference-faithful
orthonormal-basis mode.
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import hslabs_amd as H  # noqa: E402
from oracle import oracle as O  # noqa: E402


def wrapdiff(a, b):
    d = a - b
    return np.abs((d + np.pi) % (2 * np.pi) - np.pi)


def gait_to_oracle(p: H.PgsConfigParams) -> O.GaitParams:
    return O.GaitParams(torso_pos=p.torso_pos, torso_angles=p.torso_angles, step_duration=p.step_duration,
                        period=p.period, step_length=p.step_length, step_height=p.step_height,
                        curvature=p.curvature, foot_shift_type=p.foot_shift[0], foot_shift=p.foot_shift[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n_t", type=int, default=20)
    ap.add_argument("--ids", type=str, default="0-27")
    args = ap.parse_args()
    a, b = args.ids.split("-")
    cfgp = os.path.join(ROOT, "models", "pgs_config.txt")
    worst = {}
    for sid in range(int(a), int(b) + 1):
        p = H.read_pgs_config(cfgp, sid)
        xml = os.path.join(ROOT, "models", p.fname)
        m = H.KinematicModel(xml)
        om = O.Model(xml)
        t0 = time.time()
        g = H.run_host(m, [p], n_t=args.n_t, k0=0, horizon=args.n_t)
        t1 = time.time()
        og = gait_to_oracle(p)
        rf = O.rollout(om, og, args.n_t, basis=O.BASIS_FAST)
        rt = O.rollout(om, og, args.n_t, basis=O.BASIS_TREE)
        ro = O.rollout(om, og, args.n_t, basis=O.BASIS_ORTHO)
        qg = g["q"][0]
        qo = rt["q"][2:2 + args.n_t]
        line = [f"{sid:2d} {p.fname:11s}"]
        for name, ref in (("fast", rf), ("tree", rt), ("ortho", ro)):
            dt = np.abs(g["tau"][0] - ref["tau"]).max()
            dc = np.abs(g["cf"][0] - ref["cf"]).max()
            dx = np.abs(g["x"][0] - ref["x"]).max()
            dcot = abs(g["work_cot"][0, 1] - ref["cot"]) / max(1e-300, abs(ref["cot"]))
            worst[name] = max(worst.get(name, 0), dt)
            line.append(f"{name}: tau {dt:.1e} cf {dc:.1e} x {dx:.1e} relcot {dcot:.1e}")
        line.append(f"q {wrapdiff(qg, qo).max():.1e} flags {int(np.bitwise_or.reduce(g['flags'][0]))}"
                    f"/{int(np.bitwise_or.reduce(rf['flags']))} {1e3 * (t1 - t0):.0f}ms")
        print(" | ".join(line), flush=True)
    print("worst tau diff:", worst)


if __name__ == "__main__":
    main()
