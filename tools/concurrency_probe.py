"""Do small host-bytes batches on separate engines overlap on the GPU?  N Python threads, each with its own
JpegEngine (own scratch and stream), each calling decode_resize on `batch` images in a loop (the ctypes
call releases the GIL); prints images/s and the mean call time per thread count.  One engine per
thread is what the decode service runs (one batch in flight per engine).

    python tools/concurrency_probe.py [seconds] [batch] [threads ...]
"""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sds_amd.engine import JpegEngine  # noqa: E402
from tests.golden.synth import synth_jpegs  # noqa: E402


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 3.0
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    counts = [int(v) for v in sys.argv[3:]] or [1, 2, 4]
    jpgs = synth_jpegs(16, seed=2024)
    engines = [JpegEngine("cuda:0", max_batch=64) for _ in range(max(counts))]
    streams = [torch.cuda.Stream() for _ in engines]
    for e, s in zip(engines, streams):  # warm-up: scratch, code objects
        with torch.cuda.stream(s):
            for k in range(4):
                e.decode_resize([jpgs[(k + i) % 16] for i in range(batch)], (256, 256), layout="hwc")
    torch.cuda.synchronize()
    for k in counts:
        done = [0] * k
        calls = [0.0] * k
        stop = time.perf_counter() + seconds

        def run(i):
            e, s = engines[i], streams[i]
            with torch.cuda.stream(s):
                n = 0
                while time.perf_counter() < stop:
                    a = time.perf_counter()
                    _, st = e.decode_resize([jpgs[(n + j) % 16] for j in range(batch)], (256, 256), layout="hwc")
                    calls[i] += time.perf_counter() - a
                    assert (st == 0).all()
                    n += 1
                done[i] = n

        t0 = time.perf_counter()
        th = [threading.Thread(target=run, args=(i,)) for i in range(k)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        print(json.dumps({"threads": k, "batch": batch, "images_per_s": round(sum(done) * batch / dt, 1),
                          "mean_call_ms": round(1e3 * sum(calls) / max(1, sum(done)), 3)}), flush=True)


if __name__ == "__main__":
    main()
