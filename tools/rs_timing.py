#!/usr/bin/env python3
"""k_resample phase timing (experiment): needs a library built with -DSDSJ_RS_TIMING=1, e.g.
    hipcc ... -DSDSJ_RS_TIMING=1 -o tools/_exp/libsdsj_t.so ;  SDSJ_LIBRARY=tools/_exp/libsdsj_t.so python tools/rs_timing.py
Prints mean s_memtime ticks per workgroup-wave for phases: stage+barrier, convert+barrier, H+V."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch

    from bench import make_pool
    from sds_amd.engine import JpegEngine
    from tests.gpu_debug import snapshot

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    pool = make_pool(256, 16)
    jpgs = [pool[i % 256] for i in range(n)]
    eng = JpegEngine("cuda:0", max_batch=n, scratch_bytes=int(n * 3.2e6) + (256 << 20))
    out, st = eng.decode_resize(jpgs, (256, 256))
    eng.set_timing(True)
    out, st = eng.decode_resize(jpgs, (256, 256))
    torch.cuda.synchronize()
    rs_ms = eng.stage_times().get("resample")
    eng.set_timing(False)
    descs, _ = snapshot(eng, n)
    waves = n * 4 * 4  # strips x waves per workgroup (256x256 output, 64-row strips)
    tot = [sum(d.t_rs[k] for d in descs) for k in range(3)]
    print({"images": n, "resample_ms": rs_ms, "ticks_per_wg_wave": [round(t / waves) for t in tot],
           "names": ["stage+barrier", "convert+barrier", "H+V"]})


if __name__ == "__main__":
    main()
