#!/usr/bin/env python3
"""Generates the golden parity vectors in tests/golden/ by running the REFERENCE pipeline.

Run in the build container only (it needs /root/reference):

    python3 -B tests/golden/make_golden.py

The reference's own ``sds/transforms/presets.py`` and ``functional.py`` are imported
unmodified from /root/reference.  Four of its imports are absent from this image and are
stubbed in a temporary directory (never inside /root/reference): ``loguru`` (no-op logger),
``beartype`` (identity decorator), ``boto3`` and ``av`` (empty modules, unused on the image
path), plus ``torchvision.transforms.functional.resize`` restated as torchvision's PIL branch
(``img.resize((w, h), PIL_MODE[interpolation])`` with its same-size shortcut; PIL_MODE is torchvision's
``pil_modes_mapping``, which sends both NEAREST and NEAREST_EXACT to PIL NEAREST).  The
arithmetic therefore comes from Pillow 12.2.0 + libjpeg-turbo 3.1.4 exactly as in the
reference's deployment.  Bytecode writing is disabled so nothing lands in /root/reference.

Outputs (all data, no reference source):
  g1_small.npz      G1: small JPEG bytes, decoded RGB, pipeline outputs at 3 resolutions
  g1_cases.json     G1: per-case parameters + reference outcome (ok / exception type)
  g2_synth.json     G2: 8 synthetic 640x480 q90 (bench generator) digests at 256x256
  g2_full0.npy      G2: one full 256x256 uint8 CHW output
  g3_mixed.json     G3: mixed sizes up to 1920x1080 at 512x512 (+hflip, +normalize) digests
  g4_routing.json   G4: field routing (key order / types / shapes / strides) per pipeline branch
  MANIFEST.json     library versions and generator settings
"""
from __future__ import annotations

import hashlib
import io
import json
import os
import sys
import tempfile

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFERENCE = os.environ.get("SDS_REFERENCE", "/root/reference")

STUBS = {
    "loguru/__init__.py": (
        "class _L:\n"
        "    def __getattr__(self, n):\n"
        "        return lambda *a, **k: None\n"
        "logger = _L()\n"),
    "beartype/__init__.py": "def beartype(x=None, **k):\n    return x\n",
    "boto3/__init__.py": "",
    "av/__init__.py": "",
    "torchvision/__init__.py": "",
    "torchvision/transforms/__init__.py": "",
    "torchvision/transforms/functional.py": (
        "import enum\n"
        "from PIL import Image\n"
        "class InterpolationMode(enum.Enum):\n"
        "    NEAREST = 'nearest'; NEAREST_EXACT = 'nearest-exact'; BILINEAR = 'bilinear'\n"
        "    BICUBIC = 'bicubic'; BOX = 'box'; HAMMING = 'hamming'; LANCZOS = 'lanczos'\n"
        "_PIL = {InterpolationMode.NEAREST: Image.NEAREST, InterpolationMode.NEAREST_EXACT: Image.NEAREST,\n"
        "        InterpolationMode.BILINEAR: Image.BILINEAR,\n"
        "        InterpolationMode.BICUBIC: Image.BICUBIC, InterpolationMode.BOX: Image.BOX,\n"
        "        InterpolationMode.HAMMING: Image.HAMMING, InterpolationMode.LANCZOS: Image.LANCZOS}\n"
        "def resize(img, size, interpolation=InterpolationMode.BILINEAR, max_size=None, antialias=True):\n"
        "    h, w = size\n"
        "    if (w, h) == img.size:\n"
        "        return img\n"
        "    return img.resize((w, h), _PIL[interpolation])\n"),
}


def import_reference():
    stubdir = tempfile.mkdtemp(prefix="sds_ref_stubs_")
    for rel, text in STUBS.items():
        p = os.path.join(stubdir, rel)
        os.makedirs(os.path.dirname(p), exist_ok=True)
        with open(p, "w") as f:
            f.write(text)
    sys.path.insert(0, stubdir)
    sys.path.insert(1, REFERENCE)
    import sds.transforms.presets as presets  # noqa: E402
    return presets


def sha(a) -> str:
    if isinstance(a, (bytes, bytearray)):
        return hashlib.sha256(a).hexdigest()
    import numpy as np
    a = np.ascontiguousarray(a)
    return hashlib.sha256(a.tobytes()).hexdigest()


def patch_422_to_440(d: bytes) -> bytes:
    """Re-labels a 4:2:2 stream (Y h2v1) as 4:4:0 (Y h1v2); the MCU count is unchanged when
    W is a multiple of 16 and H of 8, so the result is a valid stream that exercises h1v2."""
    d = bytearray(d)
    i = 2
    while True:
        m, length = d[i + 1], (d[i + 2] << 8) | d[i + 3]
        if m == 0xC0:
            s = i + 4
            h, w = (d[s + 1] << 8) | d[s + 2], (d[s + 3] << 8) | d[s + 4]
            assert d[s + 7] == 0x21
            d[s + 7] = 0x12
            d[s + 1:s + 3] = (h * 2).to_bytes(2, "big")
            d[s + 3:s + 5] = (w // 2).to_bytes(2, "big")
            return bytes(d)
        i += 2 + length


def main():
    import numpy as np
    import PIL
    import torch
    from PIL import Image, features

    sys.path.insert(0, REPO)
    from tests.golden.synth import encode_jpeg, synth_jpegs, synth_rgb

    P = import_reference()

    def run_pipeline(jpg: bytes, resolution, **kw):
        sample = {"jpg": jpg, "index": 0}
        for t in P.create_standard_image_pipeline("jpg", resolution, **kw)[1:]:  # skip LoadFromDisk
            sample = t(sample)
        return sample

    rng = np.random.default_rng(20251015)

    def content(kind, w, h):
        if kind == "noise":
            return rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        return synth_rgb(rng, w, h)

    # ---------------- G1: small JPEGs ----------------
    specs = [
        # (name, w, h, mode, save kwargs, content)
        ("s420_97x65_q90", 97, 65, "RGB", dict(quality=90), "smooth"),
        ("s420_64x64_q75", 64, 64, "RGB", dict(quality=75), "noise"),
        ("s420_1x1_q90", 1, 1, "RGB", dict(quality=90), "noise"),
        ("s420_2x3_q90", 2, 3, "RGB", dict(quality=90), "noise"),
        ("s420_3x17_q50", 3, 17, "RGB", dict(quality=50), "noise"),
        ("s420_5x5_q100", 5, 5, "RGB", dict(quality=100), "noise"),
        ("s420_33x8_q90", 33, 8, "RGB", dict(quality=90), "smooth"),
        ("s420_130x47_opt", 130, 47, "RGB", dict(quality=85, optimize=True), "smooth"),
        ("s420_120x90_rst1", 120, 90, "RGB", dict(quality=90, restart_marker_blocks=1), "smooth"),
        ("s420_121x91_rstrow", 121, 91, "RGB", dict(quality=70, restart_marker_rows=1), "noise"),
        ("s420_150x100_q10", 150, 100, "RGB", dict(quality=10), "noise"),
        ("s422_97x65_q90", 97, 65, "RGB", dict(quality=90, subsampling=1), "smooth"),
        ("s422_4x9_q90", 4, 9, "RGB", dict(quality=90, subsampling=1), "noise"),
        ("s422_66x40_opt_rst", 66, 40, "RGB", dict(quality=80, subsampling=1, optimize=True,
                                                   restart_marker_blocks=2), "noise"),
        ("s444_97x65_q90", 97, 65, "RGB", dict(quality=90, subsampling=0), "smooth"),
        ("s444_40x31_q100", 40, 31, "RGB", dict(quality=100, subsampling=0), "noise"),
        ("s444_71x71_rst", 71, 71, "RGB", dict(quality=60, subsampling=0, restart_marker_blocks=3), "noise"),
        ("gray_97x65_q90", 97, 65, "L", dict(quality=90), "smooth"),
        ("gray_1x7_q90", 1, 7, "L", dict(quality=90), "noise"),
        ("gray_80x50_opt_rst", 80, 50, "L", dict(quality=75, optimize=True, restart_marker_blocks=2), "noise"),
        ("s440_48x32", 96, 16, "RGB440", dict(quality=90, subsampling=1), "noise"),
        ("s420_200x120_q95", 200, 120, "RGB", dict(quality=95), "smooth"),
        ("s420_256x256_same", 256, 256, "RGB", dict(quality=90), "smooth"),
        ("s420_48x64_same", 64, 48, "RGB", dict(quality=90), "smooth"),
        # not decodable by the MI355X path (reference decodes them through PIL): status tests
        ("progressive_64x48", 64, 48, "RGB", dict(quality=90, progressive=True), "smooth"),
        ("truncated_64x48", 64, 48, "RGB", dict(quality=90), "noise"),
    ]
    resolutions = [(32, 32), (48, 64), (64, 48)]
    arrays = {}
    cases = []
    for name, w, h, mode, kw, kind in specs:
        rgb = content(kind, w, h)
        im = Image.fromarray(rgb)
        if mode == "L":
            im = im.convert("L")
        jpg = encode_jpeg(np.array(im), **kw) if mode != "RGB440" else patch_422_to_440(encode_jpeg(rgb, **kw))
        if name.startswith("truncated"):
            jpg = jpg[: len(jpg) * 2 // 3]
        arrays[f"{name}__jpg"] = np.frombuffer(jpg, np.uint8)
        case = {"name": name, "mode": mode, "save": kw, "nbytes": len(jpg)}
        try:
            dec = np.array(Image.open(io.BytesIO(jpg)).convert("RGB"))
            arrays[f"{name}__rgb"] = dec
            case["decode"] = "ok"
            case["size"] = [int(dec.shape[1]), int(dec.shape[0])]
        except Exception as e:  # reference raises -> recorded
            case["decode"] = type(e).__name__
        outs = {}
        for res in resolutions + ([tuple(case["size"][::-1])] if "size" in case else []):
            key = f"{res[0]}x{res[1]}"
            try:
                s = run_pipeline(jpg, res)
                img = s["image"]
                arrays[f"{name}__out_{key}"] = img.contiguous().numpy()
                sn = run_pipeline(jpg, res, normalize=True)
                outs[key] = {"status": "ok", "stride": list(img.stride()),
                             "norm_sha256": sha(sn["image"].contiguous().numpy()),
                             "norm_stride": list(sn["image"].stride())}
            except Exception as e:
                outs[key] = {"status": type(e).__name__}
        case["outputs"] = outs
        cases.append(case)
    np.savez_compressed(os.path.join(HERE, "g1_small.npz"), **arrays)
    with open(os.path.join(HERE, "g1_cases.json"), "w") as f:
        json.dump(cases, f, indent=1)

    # ---------------- G2: synthetic 640x480 q90 (bench generator) ----------------
    g2 = []
    jpgs = synth_jpegs(8, seed=1234)
    for k, jpg in enumerate(jpgs):
        dec = np.array(Image.open(io.BytesIO(jpg)).convert("RGB"))
        s = run_pipeline(jpg, (256, 256))
        out = s["image"].contiguous().numpy()
        sn = run_pipeline(jpg, (256, 256), normalize=True)
        if k == 0:
            np.save(os.path.join(HERE, "g2_full0.npy"), out)
        g2.append({"index": k, "jpg_sha256": sha(jpg), "nbytes": len(jpg), "rgb_sha256": sha(dec),
                   "u8_256_sha256": sha(out), "f32_256_sha256": sha(sn["image"].contiguous().numpy())})
    with open(os.path.join(HERE, "g2_synth.json"), "w") as f:
        json.dump({"seed": 1234, "w": 640, "h": 480, "quality": 90, "images": g2}, f, indent=1)

    # ---------------- G3: mixed sizes at 512x512 + hflip + normalize ----------------
    g3 = []
    g3rng = np.random.default_rng(777)
    sizes = [(640, 480), (1280, 720), (1366, 768), (1920, 1080), (480, 640), (720, 1280), (768, 1366), (853, 480),
             (1000, 1000), (333, 999)]
    for k, (w, h) in enumerate(sizes):
        jpg = encode_jpeg(synth_rgb(g3rng, w, h), 90)
        flip = bool(k % 2)
        s = run_pipeline(jpg, (512, 512))
        img = s["image"]
        sn = run_pipeline(jpg, (512, 512), normalize=True)
        nimg = sn["image"]
        if flip:  # README.md:99-108 HorizontalFlipTransform with the coin fixed
            img = torch.flip(img, dims=[2])
            nimg = torch.flip(nimg, dims=[2])
        g3.append({"index": k, "w": w, "h": h, "seed": 777, "jpg_sha256": sha(jpg), "nbytes": len(jpg),
                   "flip": flip, "u8_512_sha256": sha(img.contiguous().numpy()),
                   "f32_512_sha256": sha(nimg.contiguous().numpy())})
    with open(os.path.join(HERE, "g3_mixed.json"), "w") as f:
        json.dump({"generator": "synth_rgb(default_rng(777), w, h) in list order, q90", "images": g3}, f, indent=1)

    # ---------------- G4: field routing through the full pipeline ----------------
    tmpdir = tempfile.mkdtemp(prefix="sds_golden_")
    jpg = jpgs[0]
    path = os.path.join(tmpdir, "0.jpg")
    with open(path, "wb") as f:
        f.write(jpg)

    def describe(sample):
        out = []
        for k, v in sample.items():
            if isinstance(v, torch.Tensor):
                out.append([k, "tensor", str(v.dtype).replace("torch.", ""), list(v.shape), list(v.stride())])
            elif isinstance(v, bytes):
                out.append([k, "bytes", sha(v)])
            else:
                out.append([k, type(v).__name__, v])
        return out

    branches = {
        "default": dict(image_field="jpg", resolution=(256, 256)),
        "normalize": dict(image_field="jpg", resolution=(256, 256), normalize=True),
        "video": dict(image_field="jpg", resolution=(256, 256), return_image_as_single_frame_video=True),
        "video_normalize_custom_fields": dict(image_field="jpg", resolution=(128, 96), normalize=True,
                                              return_image_as_single_frame_video=True, output_field="img",
                                              video_output_field="clip"),
        "rect_no_crop": dict(image_field="jpg", resolution=(100, 200), resize_kwargs={"crop_before_resize": False}),
    }
    g4 = {}
    for bname, kw in branches.items():
        sample = {"index": 7, "jpg": path, "caption": "a cat", "__sample_key__": 7, "__data_type__": "IMAGE"}
        for t in P.create_standard_image_pipeline(**kw):
            sample = t(sample)
        entry = {"kwargs": {k: (list(v) if isinstance(v, tuple) else v) for k, v in kw.items()},
                 "keys": describe(sample)}
        tensor_key = [k for k, v in sample.items() if isinstance(v, torch.Tensor)][0]
        entry["tensor_sha256"] = sha(sample[tensor_key].contiguous().numpy())
        ens = P.EnsureFieldsTransform(fields_whitelist=["index", tensor_key], drop_others=True)
        entry["after_ensure_drop_others"] = describe(ens(dict(sample)))
        g4[bname] = entry
    with open(os.path.join(HERE, "g4_routing.json"), "w") as f:
        json.dump({"jpg_sha256": sha(jpg), "jpg_source": "g2 image 0", "branches": g4}, f, indent=1)

    manifest = {
        "generator": "tests/golden/make_golden.py (reference presets.py/functional.py, unmodified, with stubs)",
        "reference": REFERENCE,
        "pillow": PIL.__version__,
        "libjpeg_turbo": features.version("jpg"),
        "numpy": np.__version__,
        "torch": torch.__version__,
        "files": sorted(os.listdir(HERE)),
    }
    with open(os.path.join(HERE, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
