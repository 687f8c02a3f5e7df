"""Rate of the per-sample drop-in (create_standard_image_pipeline(..., device="cuda")) in the reference's
loader shapes: the transform list applied sample by sample (sds/dataset.py:535-561) in the main
process, and inside DataLoader workers (examples/iter_image_dataset.py:72-80: batch 4 here unless
PERSAMPLE_BATCH says otherwise, fork,
pin_memory=True) -- through the node-local decode service (the default, host outputs), or with an engine
per worker (service=None, device outputs with pin_memory=False).
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


MODES = {
    # name: (num_workers, pin_memory, multiprocessing_context, output_device, service)
    # the node-local decode service (the pipeline's default): the reference's loader shape unchanged
    "service_fork_workers2_pinned": (2, True, None, None, "auto"),
    "service_fork_workers4_pinned": (4, True, None, None, "auto"),
    "service_fork_workers8_pinned": (8, True, None, None, "auto"),
    "service_fork_workers16_pinned": (16, True, None, None, "auto"),
    # random_resize (RR below: three target sizes, np global RNG per sample) through the service: requests
    # of different sizes form separate engine batches; the loader collates each batch as a list
    "servicerr_fork_workers8_pinned": (8, True, None, None, "auto"),
    "servicerr_fork_workers16_pinned": (16, True, None, None, "auto"),
    # per-worker engines (service=None)
    "dataloader_fork_workers2_device_out": (2, False, None, None, None),
    "dataloader_fork_workers8_device_out": (8, False, None, None, None),
    "main_process_per_sample": (0, False, None, None, None),
    # the workers decode on the GPU but hand back only a tiny host tensor: the rate without the
    # device-tensor IPC (CUDA IPC handles opened by the parent per batch)
    "dataloader_fork_workers8_decode_only": (8, False, None, "discard", None),
    # comparators in the same loader shape (no sds_amd): a transform that only reads the file and returns
    # a constant 3x256x256 uint8 tensor (the loader's own ceiling), and plain Pillow decode + centre crop +
    # bilinear resize on the worker's CPU (the reference's per-sample library, not its exact transform)
    "null_fork_workers2_pinned": (2, True, None, None, "null"),
    "null_fork_workers4_pinned": (4, True, None, None, "null"),
    "null_fork_workers8_pinned": (8, True, None, None, "null"),
    "null_fork_workers16_pinned": (16, True, None, None, "null"),
    "pil_fork_workers2_pinned": (2, True, None, None, "pil"),
    "pil_fork_workers4_pinned": (4, True, None, None, "pil"),
    "pil_fork_workers8_pinned": (8, True, None, None, "pil"),
    "pil_fork_workers16_pinned": (16, True, None, None, "pil"),
}
BATCH = int(os.environ.get("PERSAMPLE_BATCH", "4"))
RR = {(256, 256): 0.5, (224, 224): 0.25, (192, 192): 0.25}


def _null_transform(s):
    with open(s["jpg"], "rb") as f:
        f.read()
    s["image"] = torch.zeros(3, 256, 256, dtype=torch.uint8)
    return s


def _pil_transform(s):
    import numpy as np
    from PIL import Image
    im = Image.open(s["jpg"]).convert("RGB")
    w, h = im.size
    c = min(w, h)
    im = im.crop(((w - c) // 2, (h - c) // 2, (w - c) // 2 + c, (h - c) // 2 + c)).resize((256, 256), Image.BILINEAR)
    s["image"] = torch.from_numpy(np.asarray(im).copy()).permute(2, 0, 1)
    return s


class _Discard(torch.utils.data.IterableDataset):
    def __init__(self, ds):
        self.ds = ds

    def __iter__(self):
        for s in self.ds:
            assert s["image"].is_cuda  # (the transform's status check has synchronised the decode)
            yield {"image": torch.zeros(3, 1, 1)}


def run_mode(mode, n_files, seconds):
    from sds_amd.presets import create_standard_image_pipeline
    from tests.golden.synth import synth_jpegs
    from tests.loader_cases import FolderDataset
    t_start = time.perf_counter()
    nw, pin, ctx, odev, service = MODES[mode]
    jpgs = synth_jpegs(64, seed=2024)
    d = tempfile.mkdtemp()
    paths = []
    for i in range(n_files):
        p = os.path.join(d, f"{i:05d}.jpg")
        with open(p, "wb") as f:
            f.write(jpgs[i % len(jpgs)])
        paths.append(p)
    discard = odev == "discard"
    if service == "null":
        ts = [_null_transform]
    elif service == "pil":
        ts = [_pil_transform]
    else:
        ts = create_standard_image_pipeline("jpg", (256, 256), device="cuda", output_device=None if discard else odev,
                                            service=service,
                                            resize_kwargs={"random_resize": RR} if mode.startswith("servicerr") else {})
    ds = FolderDataset(paths, ts)
    if discard:
        ds = _Discard(ds)
    if nw:
        # persistent workers: forked once, before the parent receives its first device tensor
        collate = (lambda b: {"image": [s["image"] for s in b]}) if mode.startswith("servicerr") else None
        src = DataLoader(ds, batch_size=BATCH, num_workers=nw, pin_memory=pin, multiprocessing_context=ctx,
                         persistent_workers=True, prefetch_factor=4, collate_fn=collate)
    else:
        src = ds
    n, t0, first = 0, time.perf_counter(), None
    while time.perf_counter() - t0 < seconds:
        for b in src:
            x = b["image"]
            if first is None:
                first = [(str(y.device), list(y.shape)) for y in x] if isinstance(x, list) else (str(x.device), list(x.shape))
                n, t0 = 0, time.perf_counter()  # worker start-up and HIP initialisation excluded
                continue
            n += len(x) if isinstance(x, list) else (x.shape[0] if x.dim() == 4 else 1)
            if time.perf_counter() - t0 >= seconds:
                break
    if torch.cuda.is_initialized():
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # CPU seconds of the decode service process over the whole run (start-up included), if one runs
    svc_cpu = None
    try:
        from sds_amd import service as _svc
        for h in _svc._handles.values():
            with open(f"/proc/{h.proc.pid}/stat") as f:
                fields = f.read().rsplit(")", 1)[1].split()
            svc_cpu = round((int(fields[11]) + int(fields[12])) / os.sysconf("SC_CLK_TCK"), 2)
    except Exception:  # noqa: BLE001  (no service, or not Linux)
        pass
    print(json.dumps({"mode": mode, "images_per_s": round(n / dt, 1), "images": n, "seconds": round(dt, 2),
                      "num_workers": nw, "pin_memory": pin, "context": ctx or "fork",
                      "output_device": "cpu" if service else (odev or "cuda"), "service": service,
                      "batch_size": BATCH if nw else None, "first_batch": first,
                      "service_cpu_s": svc_cpu, "wall_s_incl_startup": round(time.perf_counter() - t_start, 2)}), flush=True)


def main():
    n_files = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    seconds = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    if len(sys.argv) > 3 and sys.argv[3] in MODES:
        run_mode(sys.argv[3], n_files, seconds)
        return
    import subprocess
    # optional: a comma-separated list of modes (or prefixes) to run
    sel = sys.argv[3].split(",") if len(sys.argv) > 3 else None
    for mode in MODES:
        if sel and not any(mode.startswith(p) for p in sel):
            continue  # each mode in a fresh process (a forked worker needs a parent that never touched HIP)
        subprocess.run([sys.executable, os.path.abspath(__file__), str(n_files), str(seconds), mode], check=True,
                       timeout=300)


if __name__ == "__main__":
    main()
