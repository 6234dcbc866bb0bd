import os, sys, torch, numpy as np
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import hslabs_amd as H
from hslabs_amd import synth
for name in ("myant", "hexapod", "spider"):
    m = H.KinematicModel(f"models/{name}.xml")
    p = synth.gen_params(4096, name)
    b = H.DeviceBatch(m, p, n_t=20, horizon=20, outputs=("flags", "cf"))
    b.run(best=False); torch.cuda.synchronize()
    f = b.flags.cpu().numpy()
    nc = (np.abs(b.cf.cpu().numpy().reshape(4096, 20, -1, 3)).max(axis=3) > 0).sum(axis=2)
    print(name, "general %.4f" % ((f & 64) != 0).mean(), "nc hist", np.bincount(nc.ravel(), minlength=7) / nc.size)
