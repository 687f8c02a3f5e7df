"""Rate of the batched consumer-side decode (sds_amd/batched.py): CPU DataLoader
workers load the encoded bytes (create_deferred_image_pipeline), default_collate stacks them, and the
training process decodes each collated batch on the GPU -- synchronously (GpuDecodeBatch.__call__) or
with one batch in flight (GpuDecodeBatch.stream: pinned double buffering, H2D + host staging of batch
k + 1 overlapped with batch k's decode).  Inputs: a folder of synthetic 640x480 q90 JPEGs (configs[0]
shape) -> 256x256 uint8.  Prints one JSON line per mode.
    python tools/batched_bench.py [n_files] [seconds] [batch] [num_workers]"""
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import torch  # noqa: E402
from torch.utils.data import DataLoader  # noqa: E402


def main():
    n_files = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    bs = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    nw = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    from sds_amd.batched import GpuDecodeBatch, create_deferred_image_pipeline
    from tests.golden.synth import synth_jpegs
    from tests.loader_cases import FolderDataset
    jpgs = synth_jpegs(64, seed=2024)
    d = tempfile.mkdtemp()
    paths = []
    for i in range(n_files):
        p = os.path.join(d, f"{i:05d}.jpg")
        with open(p, "wb") as f:
            f.write(jpgs[i % len(jpgs)])
        paths.append(p)
    ds = FolderDataset(paths, create_deferred_image_pipeline("jpg"))
    # CPU-only workers (bytes), forked before the parent touches the GPU; persistent across epochs
    loader = DataLoader(ds, batch_size=bs, num_workers=nw, persistent_workers=True, prefetch_factor=4)
    dec = GpuDecodeBatch("jpg", (256, 256), device="cuda")

    def epochs():
        while True:
            yield from loader

    for mode in ("sync", "stream"):
        src = epochs()
        it = dec.stream(src) if mode == "stream" else (dec(b) for b in src)
        n, t0, first = 0, None, None
        for b in it:
            x = b["image"]
            if first is None:  # worker start-up and HIP initialisation excluded
                first = (str(x.device), list(x.shape))
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                continue
            n += x.shape[0]
            if time.perf_counter() - t0 >= seconds:
                break
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        it.close() if hasattr(it, "close") else None
        print(json.dumps({"mode": f"gpu_decode_batch_{mode}", "images_per_s": round(n / dt, 1), "images": n,
                          "seconds": round(dt, 2), "batch": bs, "num_workers": nw, "first_batch": first}), flush=True)


if __name__ == "__main__":
    main()
