#!/usr/bin/env python3
"""Generates G7 (tests/golden/g7_nearest.npz + .json): the reference pipeline with
``resize_kwargs={'interpolation_mode': 'nearest' | 'nearest-exact'}``.

Run in the build container only (it needs /root/reference), like make_golden.py whose stubbed import
of the reference's unmodified ``sds/transforms/presets.py`` / ``functional.py`` it reuses:

    python3 -B tests/golden/make_nearest.py

functional.py:84 calls ``TVF.resize(x, size, interpolation=TVF.InterpolationMode(interpolation_mode))``;
for PIL images torchvision maps NEAREST and NEAREST_EXACT to PIL NEAREST (pil_modes_mapping), which the
stub restates.  Cases: G2's synthetic 640x480 images at 256x256, G3's mixed sizes up to 1920x1080 at
512x512 (portrait ones with allow_vertical too), small JPEGs of G1 (4:2:0 / 4:2:2 / 4:4:4 / gray, odd
sizes, upscaling, no crop, normalize) and one PNG (a sample the GPU JPEG kernels hand to PIL).  Data only:
uint8 outputs of the small cases, SHA-256 digests of every output.
"""
from __future__ import annotations

import io
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

# (variant name, resolution, create_standard_image_pipeline kwargs) for the small cases
SMALL_VARIANTS = [
    ("n32", (32, 32), {"resize_kwargs": {"interpolation_mode": "nearest"}}),
    ("ne48x64", (48, 64), {"resize_kwargs": {"interpolation_mode": "nearest-exact"}}),
    ("n131x97_up", (131, 97), {"resize_kwargs": {"interpolation_mode": "nearest"}}),
    ("n20x50_nocrop", (20, 50), {"resize_kwargs": {"interpolation_mode": "nearest", "crop_before_resize": False}}),
    ("ne32_norm", (32, 32), {"normalize": True, "resize_kwargs": {"interpolation_mode": "nearest-exact"}}),
]
SMALL_CASES = ["s420_97x65_q90", "s420_1x1_q90", "s420_3x17_q50", "s420_121x91_rstrow", "s422_97x65_q90",
               "s444_40x31_q100", "gray_97x65_q90", "s420_200x120_q95", "progressive_64x48"]


def main():
    import numpy as np
    import PIL
    import torch
    from PIL import Image

    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    from make_golden import import_reference, sha  # noqa: E402
    from tests import goldens as G
    from tests.golden.synth import synth_rgb

    P = import_reference()

    def run(data: bytes, res, **kw):
        sample = {"img": data, "index": 0}
        try:
            for t in P.create_standard_image_pipeline("img", res, **kw)[1:]:  # skip LoadFromDisk
                sample = t(sample)
        except Exception as e:  # noqa: BLE001 -- the reference's outcome is the fixture
            return None, {"ok": False, "exception": type(e).__name__}
        out = sample["image"]
        return out, {"ok": True, "shape": list(out.shape), "dtype": str(out.dtype).replace("torch.", ""),
                     "sha256": sha(out.contiguous().numpy())}

    arrays, cases = {}, []
    g1 = {c["name"]: jpg for c, jpg, _ in G.g1()}
    for name in SMALL_CASES:
        data = g1[name]
        entry = {"name": name, "source": "g1", "variants": {}}
        for vname, res, kw in SMALL_VARIANTS:
            out, v = run(data, res, **kw)
            if out is not None and out.dtype == torch.uint8:
                arrays[f"{name}__{vname}"] = out.contiguous().numpy()
            v.update(resolution=list(res), kwargs=kw)
            entry["variants"][vname] = v
        cases.append(entry)

    rng = np.random.default_rng(7070)
    buf = io.BytesIO()
    Image.fromarray(synth_rgb(rng, 70, 45)).save(buf, format="PNG")
    png = buf.getvalue()
    arrays["png_70x45__bytes"] = np.frombuffer(png, np.uint8)
    entry = {"name": "png_70x45", "source": "npz bytes", "variants": {}}
    for vname, res, kw in SMALL_VARIANTS:
        out, v = run(png, res, **kw)
        if out is not None and out.dtype == torch.uint8:
            arrays[f"png_70x45__{vname}"] = out.contiguous().numpy()
        v.update(resolution=list(res), kwargs=kw)
        entry["variants"][vname] = v
    cases.append(entry)

    _, g2 = G.g2_jpegs()
    for k, jpg in enumerate(g2[:4]):
        entry = {"name": f"g2_{k}", "source": "g2", "index": k, "variants": {}}
        for vname, res, kw in [("n256", (256, 256), {"resize_kwargs": {"interpolation_mode": "nearest"}}),
                               ("ne256_norm", (256, 256), {"normalize": True,
                                                           "resize_kwargs": {"interpolation_mode": "nearest-exact"}})]:
            _, v = run(jpg, res, **kw)
            v.update(resolution=list(res), kwargs=kw)
            entry["variants"][vname] = v
        cases.append(entry)

    _, g3 = G.g3_jpegs()
    for k, jpg in enumerate(g3):
        entry = {"name": f"g3_{k}", "source": "g3", "index": k, "variants": {}}
        for vname, res, kw in [("n512", (512, 512), {"resize_kwargs": {"interpolation_mode": "nearest"}}),
                               ("ne384x512_vert", (384, 512), {"resize_kwargs": {"interpolation_mode": "nearest-exact",
                                                                                 "allow_vertical": True}})]:
            _, v = run(jpg, res, **kw)
            v.update(resolution=list(res), kwargs=kw)
            entry["variants"][vname] = v
        cases.append(entry)

    np.savez_compressed(os.path.join(HERE, "g7_nearest.npz"), **arrays)
    with open(os.path.join(HERE, "g7_nearest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_nearest.py (reference presets.py/functional.py, unmodified, "
                                "with make_golden.py's stubs; torchvision NEAREST / NEAREST_EXACT -> PIL NEAREST)",
                   "pillow": PIL.__version__, "cases": cases}, f, indent=1)
    print("G7:", len(cases), "cases,", len(arrays), "arrays")


if __name__ == "__main__":
    main()
