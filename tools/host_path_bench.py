#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-bytes path (BASELINE.json north_star: "the rate including H2D of
the compressed stream and D2H of the decoded tensor").

Encoded bytes start in host memory (as sds/downloader.py + the local cache leave them).
``JpegEngine.decode_resize`` stages them through pinned memory, copies them H2D, decodes and
resizes on the GPU, and the output batch is copied D2H into a pinned host tensor.  The timed
region covers all of it.  Prints one JSON line.  Never the bench ``value``: DESIGN.md §5/§8 quote it.

    python tools/host_path_bench.py [--batch 1024] [--steps 10] [--res 256]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--pool", type=int, default=256)
    args = ap.parse_args()

    import torch

    from bench import make_pool
    from sds_amd.engine import JpegEngine

    pool = make_pool(args.pool, min(16, os.cpu_count() or 1))
    jpgs = [pool[i % len(pool)] for i in range(args.batch)]
    dev = torch.device("cuda", 0)
    eng = JpegEngine(dev, max_batch=args.batch, scratch_bytes=int(args.batch * 3.2e6) + (256 << 20))
    out = torch.empty((args.batch, 3, args.res, args.res), dtype=torch.uint8, device=dev)
    host = torch.empty(out.shape, dtype=torch.uint8, pin_memory=True)

    def step():
        _, st = eng.decode_resize(jpgs, (args.res, args.res), out=out)
        host.copy_(out, non_blocking=True)
        return st

    st = step()
    torch.cuda.synchronize()
    assert (st == 0).all(), st
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = args.batch * args.steps
    mean_in = sum(len(b) for b in jpgs) / len(jpgs)
    print(json.dumps({"metric": "images/s host bytes -> H2D -> decode+resize -> D2H (PCIe-inclusive)",
                      "value": round(n / dt, 1), "unit": "images/s", "batch": args.batch, "steps": args.steps,
                      "res": args.res, "mean_jpeg_bytes": round(mean_in, 1),
                      "h2d_GBps": round(n * mean_in / dt / 1e9, 3),
                      "d2h_GBps": round(n * 3 * args.res * args.res / dt / 1e9, 3)}))


if __name__ == "__main__":
    main()
