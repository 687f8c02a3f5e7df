"""Probe: the per-sample drop-in inside torch DataLoader workers (examples/iter_image_dataset.py:72-80 shape).

Run in a fresh process (the parent must not touch the GPU before the workers fork).  Prints one JSON
line per case: whether device tensors come back from forked workers, with and without pin_memory.
"""
import json
import os
import sys
import tempfile
import traceback

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
from torch.utils.data import DataLoader, IterableDataset, get_worker_info  # noqa: E402


class Folder(IterableDataset):
    def __init__(self, paths, transforms):
        self.paths, self.transforms = paths, transforms

    def __iter__(self):
        wi = get_worker_info()
        k, n = (wi.id, wi.num_workers) if wi else (0, 1)
        for i in range(k, len(self.paths), n):
            s = {"index": i, "jpg": self.paths[i]}
            for t in self.transforms:
                s = t(s)
            yield s


def main():
    from tests import goldens as G
    from sds_amd.presets import create_standard_image_pipeline
    meta, jpgs = G.g2_jpegs()
    d = tempfile.mkdtemp()
    paths = []
    for i, j in enumerate(jpgs):
        p = os.path.join(d, f"{i}.jpg")
        with open(p, "wb") as f:
            f.write(j)
        paths.append(p)
    for pin in (False, True):
        rec = {"num_workers": 2, "pin_memory": pin}
        try:
            dl = DataLoader(Folder(paths, create_standard_image_pipeline("jpg", (256, 256), device="cuda")),
                            batch_size=4, num_workers=2, pin_memory=pin)
            got = {}
            for b in dl:
                rec["device"] = str(b["image"].device)
                for i, im in zip(b["index"].tolist(), b["image"]):
                    got[i] = G.sha(im.cpu().contiguous().numpy())
            rec["ok"] = all(got[i] == meta["images"][i]["u8_256_sha256"] for i in range(len(jpgs)))
            rec["n"] = len(got)
        except Exception as e:  # noqa: BLE001
            rec["error"] = f"{type(e).__name__}: {e}"[:600]
            rec["tb"] = traceback.format_exc()[-1500:]
        print(json.dumps(rec), flush=True)
    try:
        torch.empty(3, device="cuda").pin_memory()
        print(json.dumps({"cuda_tensor_pin_memory": "returned"}))
    except Exception as e:  # noqa: BLE001
        print(json.dumps({"cuda_tensor_pin_memory": f"{type(e).__name__}: {e}"[:400]}))


if __name__ == "__main__":
    main()
