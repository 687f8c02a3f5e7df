"""UndistortFramesTransform (sds/transforms/presets.py:164-188), SURVEY.md §8(f) f2, on the CPU: the oracle's
restatement of its resize (lean_resize_frames: centre crop + Pillow bilinear, functional.py:42-86) and the
drop-in's host logic (the aspect check, the skip cases, the key routing, the reference's AssertionError)
against G8 -- fixtures made by running the reference (tests/golden/make_undistort.py).  The GPU values are
checked in tests/test_gpu_frames.py."""
import os

import numpy as np
import pytest

from oracle import oracle as O  # (checker only)
from tests import goldens as G

torch = pytest.importorskip("torch")


def _g8():
    meta = G.load_json("g8_undistort.json")
    z = np.load(os.path.join(G.GOLDEN, "g8_undistort.npz"))
    return meta["cases"], z


def _oracle_lean_resize(frames, res):
    """functional.py:42-86 with its defaults on HWC uint8 frames, restated with the oracle."""
    out_h, out_w = res
    t, h, w, _ = frames.shape
    if (w, h) == (out_w, out_h):
        return frames
    l, tp, r, b = O.crop_box(w, h, out_h, out_w)
    return np.stack([O.resize(np.ascontiguousarray(f[tp:b, l:r]), out_h, out_w, "bilinear") for f in frames])


def test_oracle_undistort_and_video_resize_match_the_reference():
    from sds_amd.presets import GpuUndistortFramesTransform as U
    cases, z = _g8()
    for c in cases:
        if not c["ok"]:
            continue
        fr = z[c["name"] + "__frames"]
        res = U.target(c["orig_height"], c["orig_width"], c["w"], c["h"])
        und = fr if res is None else _oracle_lean_resize(fr, res)
        np.testing.assert_array_equal(und, z[c["name"] + "__undistorted"], err_msg=c["name"])
        vid = _oracle_lean_resize(und, tuple(c["video_resolution"])).transpose(0, 3, 1, 2)
        np.testing.assert_array_equal(vid, z[c["name"] + "__video"], err_msg=c["name"])


def test_undistort_host_logic_skip_cases_and_errors():
    """The cases the reference leaves untouched need no GPU: the sample comes back as it went in (same
    list object, no output key); a non-numeric field raises the reference's AssertionError."""
    from PIL import Image

    from sds_amd.presets import GpuUndistortFramesTransform as U
    cases, z = _g8()
    for c in cases:
        fr = [Image.fromarray(f) for f in z[c["name"] + "__frames"]]
        sample = {"video": fr, "index": 7}
        if c["orig_height"] is not None:
            sample["orig_h"], sample["orig_w"] = c["orig_height"], c["orig_width"]
        t = U("video", ("orig_h", "orig_w"), output_field=c["output_field"])
        if not c["ok"]:
            with pytest.raises(AssertionError):
                t(sample)
            continue
        res = U.target(c["orig_height"], c["orig_width"], c["w"], c["h"])
        if c["resized"]:
            assert res is not None and res != (c["h"], c["w"]) and list(res) == c["undistorted_shape"][1:3]
            continue  # (values: the GPU test)
        if res is None:  # skipped: untouched, no GPU needed
            out = t(sample)
            assert out["video"] is fr and list(out.keys()) == c["keys"]
        else:  # the same-size shortcut: same values (the GPU copy of the frames)
            assert res == (c["h"], c["w"])
