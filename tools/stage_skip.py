"""Timing experiments (outputs are NOT valid): configs[1] batches with engine stages skipped
(SDSJ_SKIP_STAGES bit k = the stage ending at run_lane's mark k+1: 6 entwrite, 7 idct, 12 resample;
never skip entspec/entsync: the write pass would then address coefficients from uninitialised state), or other env overrides (SDSJ_WARM_BITS, SDSJ_LANES).  Each configuration runs in
a fresh process.  usage: python tools/stage_skip.py  -> one JSON line per configuration."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CONFIGS = [
    {}, {"SDSJ_LANE_MID": "5"}, {"SDSJ_LANE_MID": "6"}, {"SDSJ_LANE_MID": "7"}, {"SDSJ_LANE_MID": "8"},
    {"SDSJ_LANES": "2", "SDSJ_LANE_MID": "6"}, {"SDSJ_LANES": "2", "SDSJ_LANE_MID": "8"},
    {"SDSJ_SKIP_STAGES": str(1 << 6)}, {"SDSJ_SKIP_STAGES": str(1 << 7)}, {"SDSJ_SKIP_STAGES": str(1 << 12)},
]

CHILD = r'''
import sys, time, json, numpy as np, torch
sys.path.insert(0, %r)
import bench
from sds_amd.engine import JpegEngine
pool = bench.make_pool(256, 16)
lens = np.array([len(p) for p in pool]); al = (lens + 15) // 16 * 16
offs = np.zeros(len(pool), np.int64); offs[1:] = np.cumsum(al)[:-1]
blob = np.zeros(int(offs[-1] + al[-1]), np.uint8)
for k, p in enumerate(pool): blob[offs[k]:offs[k] + lens[k]] = np.frombuffer(p, np.uint8)
B = 4096
idx = np.arange(B) %% len(pool)
d_blob = torch.from_numpy(blob).cuda(); d_off = torch.from_numpy(offs[idx]).cuda(); d_len = torch.from_numpy(lens[idx].astype(np.int32)).cuda()
eng = JpegEngine("cuda:0", max_batch=B, scratch_bytes=int(B * 7e6) + (256 << 20))
out = torch.empty((B, 3, 256, 256), dtype=torch.uint8, device="cuda"); st = torch.empty(B, dtype=torch.int32, device="cuda")
for _ in range(3): eng.decode_resize_device(d_blob, d_off, d_len, (256, 256), out=out, status=st)
torch.cuda.synchronize(); t0 = time.perf_counter()
for _ in range(20): eng.decode_resize_device(d_blob, d_off, d_len, (256, 256), out=out, status=st)
torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 20
print(json.dumps({"ms_per_step": round(dt * 1e3, 3), "images_per_s": round(B / dt, 1)}))
''' % REPO

for cfg in CONFIGS:
    env = dict(os.environ, **cfg)
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, env=env, timeout=300)
    line = [l for l in r.stdout.splitlines() if l.startswith("{")]
    rec = json.loads(line[-1]) if line else {"error": r.stderr[-500:]}
    print(json.dumps({"env": cfg, **rec}), flush=True)
