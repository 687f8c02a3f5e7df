"""Prints entropy-kernel statistics (sync rounds, symbols per phase) for a batch of synthetic VGA JPEGs."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sds_amd.engine import JpegEngine  # noqa: E402
from tests.golden.synth import synth_jpegs  # noqa: E402
from tests.gpu_debug import snapshot  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 64
jpgs = synth_jpegs(n, seed=99)
eng = JpegEngine(max_batch=n)
out, st = eng.decode_resize(jpgs, (256, 256))
descs, _ = snapshot(eng, n)
r = np.array([d.sync_rounds for d in descs])
sp = np.array([d.sym_spec for d in descs])
sy = np.array([d.sym_sync for d in descs])
wr = np.array([d.sym_write for d in descs])
ns = np.array([d.nsub for d in descs])
print(f"images={n} status_ok={(st == 0).all()} nsub mean={ns.mean():.1f} bits/sub={descs[0].sub_bits}")
st = np.array([d.pad0 for d in descs])
print(f"sync rounds: mean={r.mean():.2f} max={r.max()} hist={np.bincount(r).tolist()}; tasks mean={st.mean():.2f}")
print(f"symbols/image: spec={sp.mean():.0f} sync={sy.mean():.0f} write={wr.mean():.0f} "
      f"-> {(sp + sy + wr).mean() / wr.mean():.2f}x the write pass")
ts = np.array([d.t_spec for d in descs]); ty = np.array([d.t_sync for d in descs]); tc = np.array([d.t_scan for d in descs])
tw = np.array([d.t_write for d in descs])
print(f"ticks/image (s_memtime, batch of {n}): spec={ts.mean():.0f} sync={ty.mean():.0f} scan={tc.mean():.0f} write={tw.mean():.0f}")
isp = np.array([d.it_spec for d in descs]); isy = np.array([d.it_sync for d in descs]); iw = np.array([d.it_write for d in descs])
print(f"lane utilisation: spec={sp.sum() / isp.sum():.2f} sync={sy.sum() / max(isy.sum(), 1):.2f} write={wr.sum() / iw.sum():.2f}")
