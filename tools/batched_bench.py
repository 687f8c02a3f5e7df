"""Rate of the batched consumer-side decode (sds_amd/batched.py): CPU DataLoader
workers load the encoded bytes (create_deferred_image_pipeline), a collate function batches them, and the
training process decodes each collated batch on the GPU -- synchronously (GpuDecodeBatch.__call__) or
with one batch in flight (GpuDecodeBatch.stream).  Two transports: "list" = torch's default_collate (the
image field stays a list of B ``bytes``, pickled through the loader's result queue) and "packed" =
sds_amd.batched.collate_encoded (one shared-memory uint8 tensor + offsets, an EncodedBatch).

Per transport it prints the loader alone (no decode: the transport's ceiling), then sync and stream
decode rates, and a phase table of the stream loop: time waiting for the loader (next()), in
GpuDecodeBatch's host work + engine.submit (staging into the pinned slot, host planning, launches), and
in engine.wait.  Inputs: a folder of synthetic 640x480 q90 JPEGs (configs[0] shape) -> 256x256 uint8.
    python tools/batched_bench.py [n_files] [seconds] [batch] [num_workers] [transports]"""
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
    transports = (sys.argv[5] if len(sys.argv) > 5 else "list,packed").split(",")
    from sds_amd import batched as Bm
    from sds_amd.batched import GpuDecodeBatch, collate_encoded, create_deferred_image_pipeline
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
    loaders = {t: DataLoader(ds, batch_size=bs, num_workers=nw, persistent_workers=True, prefetch_factor=4,
                             collate_fn=collate_encoded("jpg") if t == "packed" else None) for t in transports}
    for ld in loaders.values():  # start every transport's workers before the GPU is touched
        iter(ld)
    dec = GpuDecodeBatch("jpg", (256, 256), device="cuda")

    def epochs(ld):
        while True:
            yield from ld

    def emit(rec):
        rec.update(batch=bs, num_workers=nw)
        print(json.dumps(rec), flush=True)

    for tr, ld in loaders.items():
        # the loader alone (no decode): what the transport delivers
        src, n, t0 = epochs(ld), 0, None
        for b in src:
            if t0 is None:
                t0 = time.perf_counter()
                continue
            n += len(b["jpg"])
            if time.perf_counter() - t0 >= seconds:
                break
        emit({"mode": f"loader_only_{tr}", "images_per_s": round(n / (time.perf_counter() - t0), 1)})
        for mode in ("sync", "stream"):
            src = epochs(ld)
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
            emit({"mode": f"gpu_decode_batch_{mode}_{tr}", "images_per_s": round(n / dt, 1), "images": n,
                  "seconds": round(dt, 2), "first_batch": first})
        # phase table of the stream loop: loader wait, submit (host staging, planning, launches), wait
        eng = Bm.get_engine("cuda")
        ph = {"loader_next": 0.0, "inputs": 0.0, "submit": 0.0, "wait": 0.0, "finish": 0.0, "release": 0.0}
        orig_submit, orig_wait = eng.submit, eng.wait
        orig_inputs, orig_finish = dec._inputs, dec._finish

        def inputs(*a, **k):
            t = time.perf_counter()
            r = orig_inputs(*a, **k)
            ph["inputs"] += time.perf_counter() - t
            return r

        def finish(*a, **k):
            t = time.perf_counter()
            r = orig_finish(*a, **k)
            ph["finish"] += time.perf_counter() - t
            return r

        def submit(*a, **k):
            t = time.perf_counter()
            r = orig_submit(*a, **k)
            ph["submit"] += time.perf_counter() - t
            return r

        def wait(*a, **k):
            t = time.perf_counter()
            r = orig_wait(*a, **k)
            ph["wait"] += time.perf_counter() - t
            return r

        def timed(src):
            while True:
                t = time.perf_counter()
                b = next(src)
                ph["loader_next"] += time.perf_counter() - t
                yield b

        eng.submit, eng.wait = submit, wait
        dec._inputs, dec._finish = inputs, finish
        try:
            it = dec.stream(timed(epochs(ld)))
            n, t0 = 0, None
            for b in it:
                if t0 is None:
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for k in ph:
                        ph[k] = 0.0
                    continue
                n += b["image"].shape[0]
                t = time.perf_counter()
                del b  # the consumer drops the batch: its shared-memory storage is unmapped here
                ph["release"] += time.perf_counter() - t
                if time.perf_counter() - t0 >= seconds:
                    break
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            it.close()
        finally:
            eng.submit, eng.wait = orig_submit, orig_wait
            dec._inputs, dec._finish = orig_inputs, orig_finish
        emit({"mode": f"phases_stream_{tr}", "images_per_s": round(n / dt, 1),
              "ms_per_batch": {k: round(v / max(1, n / bs) * 1e3, 3) for k, v in ph.items()},
              "ms_per_batch_total": round(dt / max(1, n / bs) * 1e3, 3)})


if __name__ == "__main__":
    main()
