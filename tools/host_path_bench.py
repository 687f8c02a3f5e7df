#!/usr/bin/env python3
"""PCIe-inclusive rate of the host-bytes path (BASELINE.json north_star: "the rate including H2D of
the compressed stream and D2H of the decoded tensor").

Encoded bytes start in host memory (as sds/downloader.py + the local cache leave them).
``JpegEngine.decode_resize`` stages them through pinned memory, copies them H2D, decodes and
resizes on the GPU, and the output batch is copied D2H into a pinned host tensor.  The timed
region covers all of it.  Prints one JSON line.  Never the bench ``value``: DESIGN.md §5/§8 quote it.

    python tools/host_path_bench.py [--batch 1024] [--steps 10] [--res 256] [--mode sync|stream] [--files]

--mode stream runs the asynchronous path: JpegEngine.decode_stream keeps
one batch in flight, so batch k + 1's host staging and H2D copy overlap batch k's decode; --files
reads the JPEGs from files (a local-cache directory, as sds's downloader leaves them) straight into
the pinned slots instead of from Python bytes.
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
    ap.add_argument("--mode", choices=["sync", "stream"], default="sync")
    ap.add_argument("--files", action="store_true", help="read the JPEGs from a local directory (stream mode)")
    args = ap.parse_args()

    import torch

    from bench import make_pool
    from sds_amd.engine import JpegEngine

    pool = make_pool(args.pool, min(16, os.cpu_count() or 1))
    jpgs = [pool[i % len(pool)] for i in range(args.batch)]
    dev = torch.device("cuda", 0)
    eng = JpegEngine(dev, max_batch=args.batch, scratch_bytes=int(args.batch * 7e6) + (256 << 20))
    out = torch.empty((args.batch, 3, args.res, args.res), dtype=torch.uint8, device=dev)
    host = torch.empty(out.shape, dtype=torch.uint8, pin_memory=True)

    if args.mode == "sync":
        def run(steps):
            for _ in range(steps):
                _, st = eng.decode_resize(jpgs, (args.res, args.res), out=out)
                host.copy_(out, non_blocking=True)
            return st
    else:
        import tempfile
        samples = jpgs
        if args.files:
            d = tempfile.mkdtemp(prefix="sdsj_cache_")
            paths = []
            for i, j in enumerate(pool):
                paths.append(os.path.join(d, f"{i}.jpg"))
                with open(paths[-1], "wb") as f:
                    f.write(j)
            samples = [paths[i % len(paths)] for i in range(args.batch)]
        hosts = [host, torch.empty_like(host).pin_memory()]

        d2h = torch.cuda.Stream(dev)  # D2H of batch k overlaps the decode of batch k + 1

        def run(steps):
            st = None
            for k, (o, st) in enumerate(eng.decode_stream((samples for _ in range(steps)), (args.res, args.res),
                                                          files=args.files, out=None)):
                with torch.cuda.stream(d2h):  # batch k is complete (wait() synchronised its event)
                    hosts[k % 2].copy_(o, non_blocking=True)
                    o.record_stream(d2h)
            d2h.synchronize()
            return st

    st = run(1)
    torch.cuda.synchronize()
    assert (st == 0).all(), st
    run(args.warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    n = args.batch * args.steps
    mean_in = sum(len(b) for b in jpgs) / len(jpgs)
    src = "files" if args.files and args.mode == "stream" else "host bytes"
    print(json.dumps({"metric": f"images/s {src} -> H2D -> decode+resize -> D2H (PCIe-inclusive)",
                      "value": round(n / dt, 1), "unit": "images/s", "mode": args.mode, "batch": args.batch,
                      "steps": args.steps,
                      "res": args.res, "mean_jpeg_bytes": round(mean_in, 1),
                      "h2d_GBps": round(n * mean_in / dt / 1e9, 3),
                      "d2h_GBps": round(n * 3 * args.res * args.res / dt / 1e9, 3)}))


if __name__ == "__main__":
    main()
