import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from sds_amd.engine import JpegEngine
from tests.golden.synth import encode_jpeg, synth_rgb
from tests.gpu_debug import snapshot
os.environ["SDSJ_LANES"] = "1"
n = 256
jpgs = [encode_jpeg(synth_rgb(np.random.default_rng(1234 + i), 640, 480), 90, progressive=True) for i in range(n)]
eng = JpegEngine(max_batch=n)
eng.decode_resize(jpgs, (256, 256))
out, st = eng.decode_resize(jpgs, (256, 256))
descs, _ = snapshot(eng, n)
for nm in ("t_spec", "t_sync", "t_scan", "t_write"):
    print(nm, np.mean([getattr(d, nm) for d in descs]))
