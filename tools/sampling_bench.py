"""Throughput per chroma sampling (4:2:0 / 4:2:2 / 4:4:4 / grayscale) of 640x480 q90 baseline JPEGs,
device-resident, decode + resize 256x256 uint8 CHW at batch 4096.  The 4:2:0 case is configs[1]'s
shape (fused k_rs420 route); the others take the generic k_resample route.  Prints one JSON line
per sampling."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import numpy as np
    import torch
    from PIL import Image

    from sds_amd.engine import JpegEngine
    from tests.golden.synth import encode_jpeg, synth_rgb
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    only = sys.argv[2] if len(sys.argv) > 2 else None  # one sampling (profiling runs)
    eng = JpegEngine(max_batch=n, scratch_bytes=int(n * 7e6) + (256 << 20))
    for name, kw in (("4:2:0", dict(subsampling=2)), ("4:2:2", dict(subsampling=1)), ("4:4:4", dict(subsampling=0)),
                     ("gray", None)):
        if only and name != only:
            continue
        pool = []
        for i in range(64):
            rgb = synth_rgb(np.random.default_rng(1234 + i), 640, 480)
            pool.append(encode_jpeg(np.array(Image.fromarray(rgb).convert("L")), 90) if kw is None
                        else encode_jpeg(rgb, 90, **kw))
        jpgs = [pool[i % len(pool)] for i in range(n)]
        eng.reserve(JpegEngine.scratch_need(jpgs, (256, 256)) + (64 << 20))
        lens = [len(j) for j in jpgs]
        offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        blob = torch.from_numpy(np.frombuffer(b"".join(jpgs), np.uint8).copy()).cuda()
        d_offs, d_lens = torch.from_numpy(offs).cuda(), torch.tensor(lens, dtype=torch.int32).cuda()
        out, st = eng.decode_resize_device(blob, d_offs, d_lens, (256, 256))
        torch.cuda.synchronize()
        assert (st == 0).all(), (name, torch.unique(st.cpu()))
        t0 = time.perf_counter()
        for _ in range(5):
            eng.decode_resize_device(blob, d_offs, d_lens, (256, 256), out=out, status=st)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / 5
        print(json.dumps({"sampling": name, "images_per_s": round(n / dt, 1), "batch": n,
                          "mean_jpeg_bytes": round(float(np.mean(lens)), 1)}), flush=True)
        del blob, out


if __name__ == "__main__":
    main()
