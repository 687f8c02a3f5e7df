#!/usr/bin/env python3
"""Generates G6 (tests/golden/g6_fallback.npz + .json): samples the MI355X JPEG kernels do not decode,
run through the REFERENCE pipeline.

Run in the build container only (it needs /root/reference), like make_golden.py whose stubbed import
of the reference's unmodified ``sds/transforms/presets.py`` / ``functional.py`` it reuses:

    python3 -B tests/golden/make_fallback.py

Cases: PNG (RGB, RGBA, L, P), WebP, GIF, BMP, TIFF, a CMYK JPEG, a JPEG whose EOI is missing but
followed by zero bytes (Pillow decodes it; the GPU parser reports the stream truncated), and inputs the
reference itself fails on (a truncated PNG, a JPEG cut inside its scan).  For each: the encoded
bytes, and per pipeline variant the reference outcome -- the uint8 [3, H, W] image, or the exception
type the reference raised.  Data only (no reference source).
"""
from __future__ import annotations

import io
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

# (name of the variant, resolution, create_standard_image_pipeline kwargs)
VARIANTS = [
    ("r32", (32, 32), {}),
    ("r24x40", (24, 40), {}),
    ("r32_norm", (32, 32), {"normalize": True}),
    ("r20_nocrop", (20, 20), {"resize_kwargs": {"crop_before_resize": False}}),
]


def main():
    import numpy as np
    import PIL
    import torch
    from PIL import Image

    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    from make_golden import import_reference, sha  # noqa: E402
    from tests.golden.synth import encode_jpeg, synth_rgb

    P = import_reference()
    rng = np.random.default_rng(6060)

    def enc(im: Image.Image, fmt: str, **kw) -> bytes:
        buf = io.BytesIO()
        im.save(buf, format=fmt, **kw)
        return buf.getvalue()

    rgb = lambda w, h: Image.fromarray(synth_rgb(rng, w, h))  # noqa: E731
    cases = []
    cases.append(("png_rgb_64x48", enc(rgb(64, 48), "PNG")))
    rgba = np.concatenate([synth_rgb(rng, 50, 40), rng.integers(0, 256, (40, 50, 1), dtype=np.uint8)], axis=2)
    cases.append(("png_rgba_50x40", enc(Image.fromarray(rgba, "RGBA"), "PNG")))
    cases.append(("png_l_40x30", enc(rgb(40, 30).convert("L"), "PNG")))
    cases.append(("png_p_33x27", enc(rgb(33, 27).convert("P", palette=Image.Palette.ADAPTIVE), "PNG")))
    cases.append(("webp_64x48", enc(rgb(64, 48), "WEBP", quality=80)))
    cases.append(("gif_32x32", enc(rgb(32, 32).convert("P", palette=Image.Palette.ADAPTIVE), "GIF")))
    cases.append(("bmp_20x30", enc(rgb(20, 30), "BMP")))
    cases.append(("tiff_36x20", enc(rgb(36, 20), "TIFF")))
    cases.append(("jpeg_cmyk_48x32", enc(rgb(48, 32).convert("CMYK"), "JPEG", quality=90)))
    jpg = encode_jpeg(synth_rgb(rng, 64, 48), 90)
    assert jpg[-2:] == b"\xff\xd9"
    cases.append(("jpeg_no_eoi_64x48", jpg[:-2] + bytes(16)))
    png = enc(rgb(64, 48), "PNG")
    cases.append(("png_truncated", png[: len(png) // 2]))
    jpg2 = encode_jpeg(synth_rgb(rng, 64, 48), 90)
    cases.append(("jpeg_truncated", jpg2[: len(jpg2) * 2 // 3]))

    arrays, meta = {}, []
    for name, data in cases:
        arrays[f"{name}__bytes"] = np.frombuffer(data, np.uint8)
        entry = {"name": name, "nbytes": len(data), "variants": {}}
        for vname, res, kw in VARIANTS:
            sample = {"img": data, "index": 0}
            try:
                for t in P.create_standard_image_pipeline("img", res, **kw)[1:]:  # skip LoadFromDisk
                    sample = t(sample)
                out = sample["image"]
                assert isinstance(out, torch.Tensor)
                v = {"ok": True, "shape": list(out.shape), "dtype": str(out.dtype).replace("torch.", ""),
                     "sha256": sha(out.contiguous().numpy())}
                if out.dtype == torch.uint8:
                    arrays[f"{name}__{vname}"] = out.contiguous().numpy()
            except Exception as e:  # noqa: BLE001 -- the reference's outcome is the fixture
                v = {"ok": False, "exception": type(e).__name__, "is_oserror": isinstance(e, OSError)}
            entry["variants"][vname] = v
        meta.append(entry)
        print(name, {k: (v["ok"], v.get("exception")) for k, v in entry["variants"].items()})
    np.savez_compressed(os.path.join(HERE, "g6_fallback.npz"), **arrays)
    with open(os.path.join(HERE, "g6_fallback.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_fallback.py (reference presets.py/functional.py, unmodified, "
                                "with make_golden.py's stubs)", "pillow": PIL.__version__,
                   "variants": [[v, list(r), kw] for v, r, kw in VARIANTS], "cases": meta}, f, indent=1)


if __name__ == "__main__":
    main()
