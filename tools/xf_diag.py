"""Ring statistics of the write pass (build: tools/build_variant.py xfdiag -DSDSJ_XF_DIAG=1; run with
SDSJ_LIBRARY=sds_amd/lib/exp/libsdsj_xfdiag.so): per image, the workgroup's write-pass ticks, the
transform waves' busy and waiting ticks, decode-lane spins on occupied ring slots, transform batches."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sds_amd.engine import JpegEngine  # noqa: E402
from tests.golden.synth import synth_jpegs  # noqa: E402
from tests.gpu_debug import snapshot  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
jpgs = synth_jpegs(64, seed=99)
jpgs = [jpgs[i % 64] for i in range(n)]
eng = JpegEngine(max_batch=n)
eng.set_lanes(1)
for _ in range(2):
    out, st = eng.decode_resize(jpgs, (256, 256))
descs, _ = snapshot(eng, n)
tw = np.array([d.t_write for d in descs], float)
busy = np.array([d.t_sync for d in descs], float)
wait = np.array([d.t_scan for d in descs], float)
spin = np.array([d.it_sync for d in descs], float)
nb = np.array([d.it_spec for d in descs], float)
print(f"images={n} ok={(st == 0).all()} write ticks/image={tw.mean():.0f}  transform busy={busy.mean():.0f} "
      f"wait={wait.mean():.0f} (summed over transform waves)  batches={nb.mean():.1f} "
      f"busy/batch={busy.sum() / max(nb.sum(), 1):.0f}  decode spins={spin.mean():.1f}")
