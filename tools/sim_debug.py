"""Debug aid: per-part plane depths of the first simulation step, GPU vs oracle."""
import sys
import numpy as np
import torch
sys.path.insert(0, '/root/repo')
import hslabs_amd as H
from hslabs_amd import synth
from oracle import oracle as O

m = H.KinematicModel('/root/repo/models/hexapod.xml')
om = O.Model('/root/repo/models/hexapod.xml')
params = synth.gen_sim_params(16, 'hexapod')
sb = H.SimBatch(m, params)
body0 = sb.body.cpu().numpy()
qt = sb.tables.q.cpu().numpy(); dqt = sb.tables.dq.cpu().numpy(); tt = sb.tables.tau.cpu().numpy()
out = sb.step(1)
torch.cuda.synchronize()
gl = {3: 1.6, 4: .4, 5: .05}


def q2R(q):
    w, x, y, z = q
    qq1, qq2, qq3 = 2 * x * x, 2 * y * y, 2 * z * z
    return np.array([[1 - qq2 - qq3, 2 * (x * y - w * z), 2 * (x * z + w * y)],
                     [2 * (x * y + w * z), 1 - qq1 - qq3, 2 * (y * z - w * x)],
                     [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - qq1 - qq2]])


for b in (3, 6, 13):
    r = O.sim_run(om, O.SimParams(), sb.n_t, qt[b], dqt[b], tt[b], body0[b], 0, 2, 1)
    print("rollout", b, "gpu nc", int(out['n_contacts'][b, 0]), "oracle nc", r['n_contacts'][0])
    d = []
    for i in range(22):
        R = q2R(body0[b, i, 3:7])
        z = body0[b, i, 2] - abs(R[2, 2]) * 0.2
        d.append(0.08 - z)
    print("  approx depths (len .4 parts)", np.array(d)[[4, 7, 11, 14, 18, 21]])
