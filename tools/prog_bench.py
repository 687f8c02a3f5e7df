"""Throughput of the progressive path (k_prog): synthetic 640x480 q90 progressive
JPEGs, device-resident, decode + resize 256x256; one lane walks each image's scans.  Prints JSON."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch

    from sds_amd.engine import JpegEngine
    from tests.golden.synth import encode_jpeg, synth_rgb
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    pool = [encode_jpeg(synth_rgb(np.random.default_rng(1234 + i), 640, 480), 90, progressive=True) for i in range(64)]
    jpgs = [pool[i % len(pool)] for i in range(n)]
    lens = [len(j) for j in jpgs]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    blob = torch.from_numpy(np.frombuffer(b"".join(jpgs), np.uint8).copy()).cuda()
    d_offs, d_lens = torch.from_numpy(offs).cuda(), torch.tensor(lens, dtype=torch.int32).cuda()
    eng = JpegEngine(max_batch=n, scratch_bytes=int(n * 7e6) + (256 << 20))
    out, st = eng.decode_resize_device(blob, d_offs, d_lens, (256, 256))
    torch.cuda.synchronize()
    assert (st == 0).all()
    t0 = time.perf_counter()
    for _ in range(3):
        eng.decode_resize_device(blob, d_offs, d_lens, (256, 256), out=out, status=st)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 3
    if len(sys.argv) > 2 and sys.argv[2] == "nocpu":  # (kernel A/B runs)
        print(json.dumps({"value": round(n / dt, 1), "batch": n, "library": os.environ.get("SDSJ_LIBRARY", "product")}))
        return
    import tempfile

    import bench
    folder = tempfile.mkdtemp()
    paths = []
    for i, j in enumerate(pool):  # the CPU baseline reads files (LoadFromDiskTransform)
        paths.append(os.path.join(folder, f"{i:03d}.jpg"))
        with open(paths[-1], "wb") as f:
            f.write(j)
    procs = min(16, bench.host_cores())
    cpu1 = bench.cpu_baseline(paths, 1, 2.0)
    cpup = bench.cpu_baseline(paths, procs, 4.0)
    print(json.dumps({"metric": "images/s progressive 640x480 q90 decode+resize@256 (device-resident)",
                      "value": round(n / dt, 1), "batch": n, "mean_jpeg_bytes": round(float(np.mean(lens)), 1),
                      "cpu_baseline": {"value": round(cpup, 1), "cores": procs, "single_core_value": round(cpu1, 1),
                                       "kind": "reference", "sample": "PIL open+convert, crop, BILINEAR 256x256, "
                                       "CHW tensor over the 64 progressive pool JPEGs read from files"}}))


if __name__ == "__main__":
    main()
