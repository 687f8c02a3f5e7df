#!/usr/bin/env python3
"""Generates G8 (tests/golden/g8_undistort.npz + .json): the reference's UndistortFramesTransform
(sds/transforms/presets.py:164-188), alone and followed by ResizeVideoTransform +
ConvertVideoToByteTensorTransform (presets.py:121-135), on PIL frames.

Run in the build container only (it needs /root/reference), like make_golden.py whose stubbed import
of the reference's unmodified ``sds/transforms/presets.py`` / ``functional.py`` it reuses:

    python3 -B tests/golden/make_undistort.py

Cases: no original resolution (skip), aspect ratios within the 0.02 tolerance (skip), frames made
wider or taller than the original (the resize branch: crop + Pillow bilinear, down- and upscaling),
float-valued original resolutions, a target equal to the frame height (lean_resize_frames's same-size
shortcut), a distinct output field, and non-numeric fields (the reference's AssertionError).  Data
only: the input frames, the undistorted frames and the [T, 3, h, w] uint8 chain outputs.
"""
from __future__ import annotations

import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))

# name, frame (w, h), frames T, original (height, width) field values, output_field, video resolution
CASES = [
    ("no_orig", (120, 90), 3, (None, None), None, (64, 64)),
    ("within_tol", (128, 96), 2, (480, 640), None, (48, 64)),
    ("squashed_wide", (160, 160), 3, (720, 1280), None, (64, 64)),
    ("stretched_tall", (120, 90), 3, (640, 480), None, (64, 64)),
    ("float_orig", (97, 61), 2, (479.0, 641.0), None, (40, 56)),
    ("portrait_orig", (200, 150), 2, (1920, 1080), None, (96, 64)),
    ("same_height", (2, 1), 2, (1.4, 2), None, (4, 4)),
    ("upscale_small", (33, 17), 2, (100, 100), None, (32, 32)),
    ("out_field", (150, 100), 2, (600, 400), "undist", (64, 64)),
    ("bad_type", (64, 48), 1, ("480", "640"), None, (32, 32)),
]


def main():
    import numpy as np
    import PIL
    from PIL import Image

    sys.path.insert(0, REPO)
    sys.path.insert(0, HERE)
    from make_golden import import_reference  # noqa: E402
    from tests.golden.synth import synth_rgb

    P = import_reference()
    rng = np.random.default_rng(8080)
    arrays, cases = {}, []
    for name, (w, h), t, (oh, ow), out_field, vres in CASES:
        frames = [synth_rgb(rng, w, h) for _ in range(t)]
        arrays[f"{name}__frames"] = np.stack(frames)
        entry = {"name": name, "w": w, "h": h, "t": t, "orig_height": oh, "orig_width": ow,
                 "output_field": out_field, "video_resolution": list(vres)}
        sample = {"video": [Image.fromarray(f) for f in frames], "index": 7}
        if oh is not None:
            sample["orig_h"], sample["orig_w"] = oh, ow
        und = P.UndistortFramesTransform("video", ("orig_h", "orig_w"), output_field=out_field)
        try:
            s1 = und(dict(sample))
        except Exception as e:  # noqa: BLE001 -- the reference's outcome is the fixture
            entry.update(ok=False, exception=type(e).__name__)
            cases.append(entry)
            continue
        dst = out_field or "video"
        entry["keys"] = list(s1.keys())
        entry["resized"] = s1.get(dst) is not sample["video"] if dst in s1 else False
        if dst in s1:
            und_frames = np.stack([np.asarray(f) for f in s1[dst]])
            arrays[f"{name}__undistorted"] = und_frames
            entry["undistorted_shape"] = list(und_frames.shape)
        chain = [P.ResizeVideoTransform(dst, resolution=tuple(vres)), P.ConvertVideoToByteTensorTransform(dst)]
        s2 = s1
        for tr in chain:
            s2 = tr(s2)
        v = s2[dst]
        arrays[f"{name}__video"] = v.contiguous().numpy()
        entry.update(ok=True, video_shape=list(v.shape), video_dtype=str(v.dtype).replace("torch.", ""))
        cases.append(entry)

    np.savez_compressed(os.path.join(HERE, "g8_undistort.npz"), **arrays)
    with open(os.path.join(HERE, "g8_undistort.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_undistort.py (reference presets.py UndistortFramesTransform, "
                                "ResizeVideoTransform, ConvertVideoToByteTensorTransform, unmodified, with "
                                "make_golden.py's stubs)",
                   "pillow": PIL.__version__, "cases": cases}, f, indent=1)
    print("G8:", len(cases), "cases,", len(arrays), "arrays")


if __name__ == "__main__":
    main()
