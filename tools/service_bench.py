"""Raw rate and latency of the node-local decode service (sds_amd/service.py, sdsj_service_serve): C client
processes (forked, no DataLoader, no GPU in the parent) each send one JPEG at a time -- the per-sample
transform's pattern -- for a few seconds; prints one JSON line per client count with images/s and the
per-request latency percentiles.  Inputs: synthetic 640x480 q90 JPEGs -> 256x256 uint8 (HWC, as the
transform asks).

    python tools/service_bench.py [seconds] [clients ...]
"""
import json
import multiprocessing as mp
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _client(args):
    address, jpgs, seconds, start_at = args
    from sds_amd import _lib
    from sds_amd import service as S
    op = _lib.SdsjOp(256, 256, 1, 1, _lib.DTYPE_U8, _lib.LAYOUT_HWC)
    c = S.client(address)
    st, _ = c.decode(jpgs[0], op)  # connect + map + first decode (not timed)
    assert st == 0, st
    while time.time() < start_at:
        time.sleep(0.001)
    lat, n, t0 = [], 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        a = time.perf_counter()
        st, arr = c.decode(jpgs[n % len(jpgs)], op)
        lat.append(time.perf_counter() - a)
        assert st == 0 and arr.shape == (256, 256, 3), st
        n += 1
    return n, time.perf_counter() - t0, lat


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    counts = [int(v) for v in sys.argv[2:]] or [1, 2, 4, 8, 16]
    from tests.golden.synth import synth_jpegs
    jpgs = synth_jpegs(32, seed=2024)
    from sds_amd import service as S
    address = S.ensure_service(0)
    ctx = mp.get_context("fork")  # (this process never touches the GPU)
    for k in counts:
        start_at = time.time() + 2.0 + 0.1 * k
        with ctx.Pool(k) as pool:
            res = pool.map(_client, [(address, jpgs, seconds, start_at)] * k)
        n = sum(r[0] for r in res)
        dt = max(r[1] for r in res)
        lat = sorted(x for r in res for x in r[2])
        q = lambda f: round(1e3 * lat[min(len(lat) - 1, int(f * len(lat)))], 3)  # noqa: E731
        print(json.dumps({"clients": k, "images_per_s": round(n / dt, 1), "images": n, "seconds": round(dt, 2),
                          "latency_ms": {"p50": q(0.5), "p90": q(0.9), "p99": q(0.99)}}), flush=True)


if __name__ == "__main__":
    main()
