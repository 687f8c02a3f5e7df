"""DataLoader cases of the per-sample drop-in, each run in a FRESH process by tests/test_gpu_dropin.py
(``python -m tests.loader_cases <case>``): the reference's loader shape is a torch DataLoader over the
StreamingDataset with ``num_workers=2, pin_memory=True`` (examples/iter_image_dataset.py:72-80,
sds/dataloader.py:191-192), whose workers are forked from a parent that must not have initialised
HIP.  The dataset here is a folder-backed IterableDataset stand-in that splits the files over the
workers (get_worker_info, as sds/distributed.py:442-453) and applies the transform list the way
sds/dataset.py:535-561 does.  Prints one JSON line."""
import json
import os
import sys
import tempfile

import torch
from torch.utils.data import DataLoader, IterableDataset, get_worker_info

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)


class FolderDataset(IterableDataset):
    def __init__(self, paths, transforms):
        self.paths, self.transforms = paths, transforms

    def __iter__(self):
        wi = get_worker_info()
        k, n = (wi.id, wi.num_workers) if wi else (0, 1)
        for i in range(k, len(self.paths), n):
            s = {"index": i, "jpg": self.paths[i], "__sample_key__": i, "__data_type__": "IMAGE"}
            for t in self.transforms:
                s = t(s)
            yield s


def run(case: str) -> dict:
    from sds_amd.presets import create_standard_image_pipeline
    from tests import goldens as G
    meta, jpgs = G.g2_jpegs()
    d = tempfile.mkdtemp()
    paths = []
    for i, j in enumerate(jpgs):
        p = os.path.join(d, f"{i}.jpg")
        with open(p, "wb") as f:
            f.write(j)
        paths.append(p)
    kw, dl_kw = {}, {"num_workers": 2, "pin_memory": False}
    epochs = 1
    if case == "workers_device":
        pass
    elif case == "workers_device_persistent_two_epochs":
        dl_kw["persistent_workers"] = True
        epochs = 2
    elif case == "workers_device_two_epochs":  # new workers each epoch, forked from a parent that now holds HIP
        epochs = 2
    elif case == "workers_pinned_fork":  # the reference example's exact shape
        dl_kw["pin_memory"] = True
    elif case == "workers_pinned_spawn_cpu_output":
        kw["output_device"] = "cpu"
        dl_kw.update(pin_memory=True, multiprocessing_context="spawn")
    elif case == "workers_pinned_spawn_device_output":
        dl_kw.update(pin_memory=True, multiprocessing_context="spawn")
    elif case in ("parent_touched_gpu_fork", "parent_touched_gpu_spawn"):
        torch.zeros(1, device="cuda")  # the parent initialises HIP before the workers start
        if case.endswith("spawn"):
            dl_kw["multiprocessing_context"] = "spawn"
    else:
        raise SystemExit(f"unknown case {case}")
    rec = {"case": case}
    try:
        dl = DataLoader(FolderDataset(paths, create_standard_image_pipeline("jpg", (256, 256), device="cuda", **kw)),
                        batch_size=4, **dl_kw)
        got = {}
        for b in (b for _ in range(epochs) for b in dl):
            rec["device"] = str(b["image"].device)
            rec["pinned"] = bool(b["image"].is_pinned()) if b["image"].device.type == "cpu" else None
            rec["stride"] = list(b["image"].stride())
            for i, im in zip(b["index"].tolist(), b["image"]):
                got[i] = G.sha(im.cpu().contiguous().numpy())
        rec["n"] = len(got)
        rec["epochs"] = epochs
        rec["equal_to_goldens"] = len(got) == len(jpgs) and all(
            got[i] == meta["images"][i]["u8_256_sha256"] for i in range(len(jpgs)))
    except Exception as e:  # noqa: BLE001  (the test inspects the error)
        rec["error_type"] = type(e).__name__
        rec["error"] = str(e)[-3000:]
    return rec


if __name__ == "__main__":
    print(json.dumps(run(sys.argv[1])), flush=True)
