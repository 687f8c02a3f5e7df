"""Entropy phase ticks per image size for the configs[2] mixed pool (spec / sync / scan / write)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import _make_mixed_image  # noqa: E402
from sds_amd.engine import JpegEngine  # noqa: E402
from tests.gpu_debug import snapshot  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 96
jpgs = [_make_mixed_image(i) for i in range(n)]
os.environ["SDSJ_LANES"] = "1"
eng = JpegEngine(max_batch=n, scratch_bytes=int(n * 22e6) + (1 << 30))
out, st = eng.decode_resize(jpgs, (512, 512))
out, st = eng.decode_resize(jpgs, (512, 512))
descs, _ = snapshot(eng, n)
rows = {}
for d in descs:
    rows.setdefault((d.width, d.height), []).append(d)
for k, ds in sorted(rows.items(), key=lambda x: x[0][0] * x[0][1]):
    f = lambda a: np.mean([getattr(d, a) for d in ds])
    print(k, len(ds), f"nsub={f('nsub'):.0f} sub_bits={f('sub_bits'):.0f} warm={f('warm_bits'):.0f} rounds={f('sync_rounds'):.2f} "
          f"tasks={f('pad0'):.1f} spec={f('t_spec'):.0f} sync={f('t_sync'):.0f} scan={f('t_scan'):.0f} write={f('t_write'):.0f} "
          f"sym_spec={f('sym_spec'):.0f} sym_sync={f('sym_sync'):.0f} sym_write={f('sym_write'):.0f}")
