import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from sds_amd.engine import JpegEngine
from tests.golden.synth import synth_jpegs
from tests.gpu_debug import snapshot
n = 2048
jpgs = synth_jpegs(n, seed=99)
eng = JpegEngine(max_batch=n)
out, st = eng.decode_resize(jpgs, (256, 256))
out, st = eng.decode_resize(jpgs, (256, 256))
descs, _ = snapshot(eng, n)
disc = np.array([d.it_sync for d in descs]); load = np.array([d.pad0 for d in descs]); tot = np.array([d.t_sync for d in descs])
it = np.array([d.sym_sync for d in descs]); r = np.array([d.sync_rounds for d in descs])
print("disc", disc.mean(), "load", load.mean(), "total", tot.mean(), "rest", (tot - disc - load).mean())
for k in range(4):
    m = r == k
    if m.any(): print("rounds", k, "n", m.sum(), "sync ticks", tot[m].mean(), "sym", it[m].mean())
nt = np.array([d.pad0 for d in descs])
print("tasks/image", nt.mean(), "hist", np.bincount(nt)[:12].tolist(), "sym/task", it.sum() / max(nt.sum(), 1))
print("bits/sub", descs[0].sub_bits)
m = nt > 0
for nm, f in (("disc", "it_sync"), ("stage", "t_spec"), ("refills", "it_spec")):
    v = np.array([getattr(d, f) for d in descs])
    print(nm, v[m].mean())
