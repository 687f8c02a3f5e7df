"""Rate of the per-sample drop-in (create_standard_image_pipeline(..., device="cuda")) in the reference's
loader shapes: the transform list applied sample by sample (sds/dataset.py:535-561) in the main
process, and inside DataLoader workers (examples/iter_image_dataset.py:72-80: batch 4 here,
num_workers 2 / 4 / 8, device outputs with pin_memory=False, host outputs with pin_memory=True).
Inputs: a folder of synthetic 640x480 q90 JPEGs (configs[0] shape) -> 256x256 uint8.

Run in a fresh process (the parent must not touch the GPU before the workers fork):
    python tools/persample_bench.py [n_files] [seconds]
Prints one JSON line per mode."""
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
    n_files = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    from sds_amd.presets import create_standard_image_pipeline
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

    def rate(loader_fn, label, **info):
        n, t0 = 0, time.perf_counter()
        first = None
        while time.perf_counter() - t0 < seconds:
            for b in loader_fn():
                x = b["image"]
                if first is None:
                    first = (str(x.device), list(x.shape))
                n += x.shape[0] if x.dim() == 4 else 1
                if time.perf_counter() - t0 >= seconds:
                    break
        if torch.cuda.is_initialized():
            torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        print(json.dumps({"mode": label, "images_per_s": round(n / dt, 1), "images": n, "seconds": round(dt, 2),
                          "first_batch": first, **info}), flush=True)

    # DataLoader workers first (the parent has not touched the GPU yet), then the main process
    for nw in (2, 4, 8):
        ts = create_standard_image_pipeline("jpg", (256, 256), device="cuda")
        rate(lambda: DataLoader(FolderDataset(paths, ts), batch_size=4, num_workers=nw, pin_memory=False),
             f"dataloader_workers{nw}_device_out", num_workers=nw, pin_memory=False)
    ts = create_standard_image_pipeline("jpg", (256, 256), device="cuda", output_device="cpu")
    rate(lambda: DataLoader(FolderDataset(paths, ts), batch_size=4, num_workers=2, pin_memory=True),
         "dataloader_workers2_pinned_cpu_out", num_workers=2, pin_memory=True)
    ts = create_standard_image_pipeline("jpg", (256, 256), device="cuda")
    rate(lambda: FolderDataset(paths, ts), "main_process_per_sample", num_workers=0)


if __name__ == "__main__":
    main()
