"""Per-call latency of the host-bytes entry point with one image (the per-sample drop-in's call):
wall time per JpegEngine.decode_resize([jpg]) call and per transform call, single process.
    python tools/latency_probe.py [calls]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sds_amd.engine import get_engine  # noqa: E402
from sds_amd.presets import GpuDecodeResizeImageTransform  # noqa: E402
from tests.golden.synth import synth_jpegs  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 300
jpgs = synth_jpegs(16, seed=2024)
eng = get_engine("cuda")
for j in jpgs:  # warm-up (scratch growth, code objects)
    eng.decode_resize([j], (256, 256))
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(calls):
    eng.decode_resize([jpgs[i % 16]], (256, 256))
dt_engine = (time.perf_counter() - t0) / calls
tr = GpuDecodeResizeImageTransform("jpg", resolution=(256, 256), device="cuda")
for j in jpgs:
    tr({"jpg": j})
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(calls):
    tr({"jpg": jpgs[i % 16]})
torch.cuda.synchronize()
dt_tr = (time.perf_counter() - t0) / calls
print(json.dumps({"engine_call_us": round(dt_engine * 1e6, 1), "transform_call_us": round(dt_tr * 1e6, 1),
                  "transform_images_per_s": round(1 / dt_tr, 1), "calls": calls}))
