"""GPU parity of the video-frame path: sdsj_resize_frames_device and the
GpuResizeVideoTransform drop-in vs the oracle's restatement of lean_resize_frames on PIL frames
(functional.py:42-86: centre crop, then Pillow's separable resample).  Bit-exact (integer path)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402  (checker only)


@pytest.fixture(scope="module")
def engine():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sds_amd.engine import JpegEngine
    return JpegEngine(max_batch=64)


def _frames(seed, t, w, h):
    from tests.golden.synth import synth_rgb
    rng = np.random.default_rng(seed)
    return np.stack([synth_rgb(rng, w, h) for _ in range(t)])


def _ref(frame, res, filt="bilinear", crop=True, flip=False, normalize=False):
    out_h, out_w = res
    h, w = frame.shape[:2]
    if (w, h) == (out_w, out_h):
        hwc = frame
    else:
        if crop:
            l, t, r, b = O.crop_box(w, h, out_h, out_w)
            frame = np.ascontiguousarray(frame[t:b, l:r])
        hwc = O.resize(frame, out_h, out_w, filt)
    chw = np.ascontiguousarray(hwc.transpose(2, 0, 1))
    if flip:
        chw = np.ascontiguousarray(chw[:, :, ::-1])
    if normalize:
        chw = O.normalize_lut()[chw]
    return chw


@pytest.mark.parametrize("size,res,filt", [((97, 61), (64, 80), "bilinear"), ((640, 360), (256, 256), "bilinear"),
                                           ((320, 240), (512, 512), "bilinear"), ((200, 150), (100, 60), "bicubic"),
                                           ((64, 48), (48, 64), "lanczos"), ((97, 61), (131, 40), "nearest"),
                                           ((640, 360), (256, 256), "nearest")])
def test_frames_match_oracle(engine, size, res, filt):
    w, h = size
    fr = _frames(7, 5, w, h)
    out, st = engine.resize_frames(torch.from_numpy(fr).cuda(), res, filter=filt)
    assert (st == 0).all()
    for k in range(fr.shape[0]):
        np.testing.assert_array_equal(out[k].cpu().numpy(), _ref(fr[k], res, filt), err_msg=f"frame {k}")


def test_frames_identity_flip_normalize_hwc_and_no_crop(engine):
    fr = _frames(8, 4, 96, 64)
    out, st = engine.resize_frames(torch.from_numpy(fr).cuda(), (64, 96))  # same size: copy
    assert (st == 0).all()
    np.testing.assert_array_equal(out.cpu().numpy(), fr.transpose(0, 3, 1, 2))
    flip = torch.tensor([1, 0, 1, 0], dtype=torch.uint8)
    out, st = engine.resize_frames(torch.from_numpy(fr).cuda(), (40, 40), flip=flip, normalize=True, layout="hwc")
    for k in range(4):
        ref = _ref(fr[k], (40, 40), flip=bool(flip[k]), normalize=True).transpose(1, 2, 0)
        np.testing.assert_array_equal(out[k].cpu().numpy(), ref)
    out, _ = engine.resize_frames(torch.from_numpy(fr).cuda(), (40, 40), crop_before_resize=False)
    for k in range(4):
        np.testing.assert_array_equal(out[k].cpu().numpy(), _ref(fr[k], (40, 40), crop=False))


def test_video_transform_on_pil_frames():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from PIL import Image

    from sds_amd.presets import GpuResizeVideoTransform
    fr = _frames(9, 6, 160, 90)
    sample = {"video": [Image.fromarray(f) for f in fr], "index": 3}
    t = GpuResizeVideoTransform("video", resolution=(64, 64))
    out = t(sample)
    assert list(out.keys()) == ["video", "index"]
    v = out["video"]
    assert v.is_cuda and v.dtype == torch.uint8 and v.shape == (6, 3, 64, 64)
    for k in range(6):
        np.testing.assert_array_equal(v[k].cpu().numpy(), _ref(fr[k], (64, 64)))


def test_undistort_then_video_resize_matches_the_reference_fixture():
    """f2's UndistortFramesTransform (presets.py:164-188) on the GPU: GpuUndistortFramesTransform (a
    uint8-rounded resize of its own) then GpuResizeVideoTransform, bit-exact against G8 -- the reference's
    UndistortFramesTransform -> ResizeVideoTransform -> ConvertVideoToByteTensorTransform on the same PIL
    frames (tests/golden/make_undistort.py) -- including the key routing and the skip / same-size cases."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import os

    from PIL import Image

    from sds_amd.presets import GpuResizeVideoTransform, GpuUndistortFramesTransform
    from tests import goldens as G
    meta = G.load_json("g8_undistort.json")
    z = np.load(os.path.join(G.GOLDEN, "g8_undistort.npz"))
    for c in meta["cases"]:
        name = c["name"]
        fr = z[name + "__frames"]
        sample = {"video": [Image.fromarray(f) for f in fr], "index": 7}
        if c["orig_height"] is not None:
            sample["orig_h"], sample["orig_w"] = c["orig_height"], c["orig_width"]
        und = GpuUndistortFramesTransform("video", ("orig_h", "orig_w"), output_field=c["output_field"])
        if not c["ok"]:
            with pytest.raises(AssertionError):
                und(sample)
            continue
        s1 = und(sample)
        assert list(s1.keys()) == c["keys"], name
        dst = c["output_field"] or "video"
        got = s1[dst]
        got = got.cpu().numpy() if isinstance(got, torch.Tensor) else np.stack([np.asarray(f) for f in got])
        np.testing.assert_array_equal(got, z[name + "__undistorted"], err_msg=f"{name}: undistorted frames")
        s2 = GpuResizeVideoTransform(dst, resolution=tuple(c["video_resolution"]))(s1)
        v = s2[dst]
        assert v.is_cuda and v.dtype == torch.uint8 and list(v.shape) == c["video_shape"], name
        np.testing.assert_array_equal(v.cpu().numpy(), z[name + "__video"], err_msg=f"{name}: video")


def test_undistort_random_frame_sizes_vs_oracle(engine):
    """Random frame sizes and original resolutions: both uint8 passes on the GPU vs the oracle's."""
    from sds_amd.presets import GpuUndistortFramesTransform as U
    rng = np.random.default_rng(31)
    done = 0
    while done < 12:
        w, h = int(rng.integers(8, 400)), int(rng.integers(8, 300))
        oh, ow = int(rng.integers(100, 2000)), int(rng.integers(100, 2000))
        res = U.target(oh, ow, w, h)
        if res is None or res == (h, w) or res[0] < 1:
            continue
        fr = _frames(100 + done, 2, w, h)
        und, st = engine.resize_frames(torch.from_numpy(fr).cuda(), res, layout="hwc")
        assert (st == 0).all()
        ref_und = np.stack([_ref(f, res).transpose(1, 2, 0) for f in fr])
        np.testing.assert_array_equal(und.cpu().numpy(), ref_und, err_msg=f"{w}x{h} orig {ow}x{oh}")
        vid, st = engine.resize_frames(und, (64, 48))
        assert (st == 0).all()
        for k in range(2):
            np.testing.assert_array_equal(vid[k].cpu().numpy(), _ref(ref_und[k], (64, 48)))
        done += 1
