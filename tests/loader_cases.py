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


def run_service_case(case: str) -> dict:
    """Cases of the node-local decode service (sds_amd/service.py): the pipeline's default service="auto"."""
    import numpy as np

    from sds_amd.presets import create_standard_image_pipeline
    from tests import goldens as G
    rec = {"case": case}
    d = tempfile.mkdtemp()
    try:
        if case in ("service_reference_shape", "service_parent_touched_gpu"):
            meta, jpgs = G.g2_jpegs()
            paths = []
            for i, j in enumerate(jpgs):
                p = os.path.join(d, f"{i}.jpg")
                with open(p, "wb") as f:
                    f.write(j)
                paths.append(p)
            ts = create_standard_image_pipeline("jpg", (256, 256), device="cuda")
            rec["service"] = ts[1].service_address is not None
            if case == "service_parent_touched_gpu":
                torch.zeros(1, device="cuda")  # HIP initialised in the parent before the workers fork
            # examples/iter_image_dataset.py:72-80's DataLoader arguments: fork, 2 workers, pin_memory=True
            dl = DataLoader(FolderDataset(paths, ts), batch_size=4, num_workers=2, pin_memory=True, drop_last=True)
            got = {}
            for b in dl:
                rec["device"] = str(b["image"].device)
                rec["pinned"] = bool(b["image"].is_pinned())
                rec["stride"] = list(b["image"].stride())
                for i, im in zip(b["index"].tolist(), b["image"]):
                    got[i] = G.sha(im.contiguous().numpy())
            rec["n"] = len(got)
            rec["equal_to_goldens"] = len(got) == len(jpgs) and all(
                got[i] == meta["images"][i]["u8_256_sha256"] for i in range(len(jpgs)))
        elif case == "service_g3_flip_normalize":
            meta, jpgs = G.g3_jpegs()
            paths = []
            for i, j in enumerate(jpgs):
                p = os.path.join(d, f"{i}.jpg")
                with open(p, "wb") as f:
                    f.write(j)
                paths.append(p)
            ok = True
            for flip in (False, True):
                for norm in (False, True):
                    ts = create_standard_image_pipeline("jpg", (512, 512), normalize=norm, device="cuda",
                                                        hflip_prob=1.0 if flip else 0.0)
                    sel = [i for i, im in enumerate(meta["images"]) if im["flip"] == flip]
                    dl = DataLoader(FolderDataset([paths[i] for i in sel], ts), batch_size=None, num_workers=3)
                    for k, s in enumerate(dl):
                        im = meta["images"][sel[s["index"]]]
                        key = "f32_512_sha256" if norm else "u8_512_sha256"
                        ok &= s["image"].device.type == "cpu" and G.sha(s["image"].contiguous().numpy()) == im[key]
            rec["equal_to_goldens"] = bool(ok)
        elif case == "service_random_resize":
            # random_resize (np global RNG, one draw per sample): requests of different target sizes in
            # flight together; every output equals the oracle at the size the sample drew
            from oracle import oracle as O  # checker only
            _, jpgs = G.g2_jpegs()
            paths = []
            for i in range(24):
                p = os.path.join(d, f"{i}.jpg")
                with open(p, "wb") as f:
                    f.write(jpgs[i % len(jpgs)])
                paths.append(p)
            rr = {(256, 256): 0.5, (192, 160): 0.25, (96, 128): 0.25}
            ts = create_standard_image_pipeline("jpg", (256, 256), device="cuda", resize_kwargs={"random_resize": rr})
            ok, shapes = True, set()
            dl = DataLoader(FolderDataset(paths, ts), batch_size=4, num_workers=4, pin_memory=True,
                            collate_fn=lambda b: b)
            for b in dl:
                for s in b:
                    im = s["image"]
                    ok &= im.device.type == "cpu"
                    shapes.add(tuple(im.shape))
                    ref = O.pipeline(jpgs[s["index"] % len(jpgs)], tuple(im.shape[1:]))
                    ok &= bool(np.array_equal(im.contiguous().numpy(), ref))
            rec["shapes"] = sorted(shapes)
            rec["equal_to_oracle"] = bool(ok)
        elif case == "service_fallback_g6":
            meta = G.load_json("g6_fallback.json")
            z = np.load(os.path.join(G.GOLDEN, "g6_fallback.npz"))
            ok, n = True, 0
            for vname, res, kw in meta["variants"]:
                paths, refs = [], []
                for c in meta["cases"]:
                    p = os.path.join(d, c["name"])
                    with open(p, "wb") as f:
                        f.write(z[f"{c['name']}__bytes"].tobytes())
                    paths.append(p)
                    refs.append(c["variants"][vname])
                ts = create_standard_image_pipeline("img", tuple(res), device="cuda", **kw)

                class _One(IterableDataset):
                    def __iter__(self):
                        wi = get_worker_info()
                        for i in range(wi.id, len(paths), wi.num_workers):
                            s = {"img": paths[i]}
                            try:
                                for t in ts:
                                    s = t(s)
                                yield {"i": i, "ok": True, "img": s["image"]}
                            except OSError:
                                yield {"i": i, "ok": False, "img": torch.zeros(1)}
                for s in DataLoader(_One(), batch_size=None, num_workers=2):
                    ref = refs[s["i"]]
                    ok &= bool(s["ok"]) == ref["ok"]
                    if ref["ok"]:
                        ok &= list(s["img"].shape) == ref["shape"] and G.sha(s["img"].contiguous().numpy()) == ref["sha256"]
                    n += 1
            rec["n"] = n
            rec["equal_to_goldens"] = bool(ok)
        else:
            raise SystemExit(f"unknown case {case}")
    except Exception as e:  # noqa: BLE001  (the test inspects the error)
        rec["error_type"] = type(e).__name__
        rec["error"] = str(e)[-3000:]
    return rec


def run(case: str) -> dict:
    if case.startswith("service_"):
        return run_service_case(case)
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
    # per-worker engines (service=None): each worker initialises HIP itself
    kw, dl_kw = {"service": None}, {"num_workers": 2, "pin_memory": False}
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
