import sys, time, numpy as np, torch
sys.path.insert(0, '/root/repo')
import hslabs_amd as H
from hslabs_amd import synth
from oracle import oracle as O
m = H.KinematicModel('/root/repo/models/hexapod.xml')
om = O.Model('/root/repo/models/hexapod.xml')
B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
params = synth.gen_sim_params(B, 'hexapod')
sb = H.SimBatch(m, params)
torch.cuda.synchronize()
body0 = sb.body.cpu().numpy()
qt = sb.tables.q.cpu().numpy(); dqt = sb.tables.dq.cpu().numpy(); tt = sb.tables.tau.cpu().numpy()
# reset parity
for b in range(min(B, 8)):
    ob = O.sim_reset(om, qt[b, sb.table_row(2)])
    assert np.abs(ob - body0[b]).max() < 1e-12, np.abs(ob - body0[b]).max()
print("reset ok")
for nst in (1, 10, 100):
    sb.reset(2)
    out = sb.step(nst)
    torch.cuda.synchronize()
    bd = sb.body.cpu().numpy()
    errs = []
    nc_bad = 0
    for b in range(min(B, 16)):
        r = O.sim_run(om, O.SimParams(), sb.n_t, qt[b], dqt[b], tt[b], body0[b], 0, 2, nst)
        errs.append(np.abs(r['body'] - bd[b]).max())
        g = out['n_contacts'][b].cpu().numpy()
        if not (r['n_contacts'] == g).all():
            nc_bad += 1
            k = int(np.argmax(r['n_contacts'] != g))
            print("  rollout", b, "contact count differs first at step", k, r['n_contacts'][k], g[k])
    print(nst, "max body err", max(errs), "median", np.median(errs), "contact mismatches", nc_bad)
for BT in (B, 1024, 4096):
    sbt = H.SimBatch(m, synth.gen_sim_params(BT, 'hexapod'))
    sbt.step(5, outputs=())
    torch.cuda.synchronize()
    for ns in (10, 50):
        t0 = time.time()
        sbt.step(ns, outputs=())
        torch.cuda.synchronize()
        dt = time.time() - t0
        print(f"B={BT} {ns} steps {dt*1e3:.1f} ms -> {BT*ns/dt/1e6:.3f} M steps/s")
