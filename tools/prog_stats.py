"""Where k_prog's time goes per scan kind (a -DSDSJ_PROG_STATS build: python tools/build_variant.py
pstats -DSDSJ_PROG_STATS=1, then SDSJ_LIBRARY=sds_amd/lib/exp/libsdsj_pstats.so python tools/prog_stats.py).
Per image: shader cycles and bytes of entropy data of the DC-first, AC-first, DC-refine and
AC-refine scans of synthetic 640x480 q90 progressive JPEGs (the prog_bench images)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sds_amd.engine import JpegEngine  # noqa: E402
from tests.golden.synth import encode_jpeg, synth_rgb  # noqa: E402
from tests.gpu_debug import snapshot  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
pool = [encode_jpeg(synth_rgb(np.random.default_rng(1234 + i), 640, 480), 90, progressive=True) for i in range(64)]
jpgs = [pool[i % len(pool)] for i in range(n)]
eng = JpegEngine(max_batch=n)
out, st = eng.decode_resize(jpgs, (256, 256))
assert (np.asarray(st) == 0).all()
descs, _ = snapshot(eng, n)
kinds = {"dc_first": ("t_spec", "sym_spec"), "ac_first": ("t_sync", "sym_sync"), "dc_refine": ("t_scan", "sym_write"),
         "ac_refine": ("t_write", "it_write")}
res = {}
for k, (tf, bf) in kinds.items():
    t = np.array([getattr(d, tf) for d in descs], dtype=np.float64)
    b = np.array([getattr(d, bf) for d in descs], dtype=np.float64)
    res[k] = {"mcycles_per_image": round(t.mean() / 1e6, 3), "bytes_per_image": round(b.mean(), 1),
              "cycles_per_byte": round(t.sum() / max(b.sum(), 1), 1)}
print(json.dumps({"images": n, "mean_jpeg_bytes": round(float(np.mean([len(j) for j in jpgs])), 1), "kinds": res}))
