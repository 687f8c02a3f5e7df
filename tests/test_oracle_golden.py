"""Pins the CPU oracle (oracle/) against the reference's golden vectors (CPU only)."""
import numpy as np
import pytest

from oracle import oracle as O
from tests import goldens as G

G1 = list(G.g1())


@pytest.mark.parametrize("case,jpg,arrs", G1, ids=[c["name"] for c, _, _ in G1])
def test_g1_decode_and_pipeline(case, jpg, arrs):
    name = case["name"]
    if case["decode"] != "ok":
        with pytest.raises(O.OracleError):
            O.decode(jpg)
        return
    np.testing.assert_array_equal(O.decode(jpg), arrs["rgb"])
    for key, out in case["outputs"].items():
        res = tuple(int(v) for v in key.split("x"))
        if out["status"] != "ok":
            with pytest.raises(O.OracleError):
                O.pipeline(jpg, res)
            continue
        np.testing.assert_array_equal(O.pipeline(jpg, res), arrs[f"out_{key}"])
        assert G.sha(O.pipeline(jpg, res, normalize=True)) == out["norm_sha256"]


def test_g2_synthetic_vga():
    meta, jpgs = G.g2_jpegs()
    full0 = np.load(f"{G.GOLDEN}/g2_full0.npy")
    for im, jpg in zip(meta["images"], jpgs):
        assert G.sha(jpg) == im["jpg_sha256"], "PIL encoder output changed; regenerate goldens"
        assert G.sha(O.decode(jpg)) == im["rgb_sha256"]
        out = O.pipeline(jpg, (256, 256))
        assert G.sha(out) == im["u8_256_sha256"]
        assert G.sha(O.pipeline(jpg, (256, 256), normalize=True)) == im["f32_256_sha256"]
        if im["index"] == 0:
            np.testing.assert_array_equal(out, full0)


def test_g3_mixed_sizes_flip_normalize():
    meta, jpgs = G.g3_jpegs()
    for im, jpg in zip(meta["images"], jpgs):
        assert G.sha(jpg) == im["jpg_sha256"]
        assert G.sha(O.pipeline(jpg, (512, 512), flip=im["flip"])) == im["u8_512_sha256"]
        assert G.sha(O.pipeline(jpg, (512, 512), flip=im["flip"], normalize=True)) == im["f32_512_sha256"]


def test_g5_edge_cases():
    """Table validation, scan termination and post-scan markers as the reference loader behaves."""
    import base64
    for c in G.load_json("g5_edge.json")["cases"]:
        jpg = base64.b64decode(c["jpg_b64"])
        if c["outcome"] == "ok":
            assert G.sha(O.decode(jpg)) == c["rgb_sha256"], c["name"]
        else:
            with pytest.raises(O.OracleError):
                O.decode(jpg)


@pytest.mark.parametrize("seed", [11, 12, 13])
def test_oracle_status_matches_pil_on_mutated_streams(seed):
    """Truncations, byte flips, fill bytes, premature EOI / RSTn: decodable exactly when PIL decodes them
    (libjpeg-turbo's warning-and-continue recovery).  Pixels are compared where no garbage coefficients
    are involved (premature markers); garbage blocks follow libjpeg's C IDCT, not the x86 SIMD one."""
    import io
    Image = pytest.importorskip("PIL.Image")
    from tests.golden.synth import mutated_jpegs
    for i, jpg in enumerate(mutated_jpegs(seed, 40)):
        try:
            ref = np.asarray(Image.open(io.BytesIO(jpg)).convert("RGB"))
        except OSError:
            ref = None
        try:
            got = O.decode(jpg)
        except O.OracleError:
            got = None
        assert (ref is None) == (got is None), f"sample {i}"
        if ref is not None and i % 5 in (3, 4):
            np.testing.assert_array_equal(got, ref, err_msg=f"sample {i}")


@pytest.mark.parametrize("size,res,filt", [((97, 61), (64, 80), "bilinear"), ((640, 360), (256, 256), "bilinear"),
                                           ((320, 240), (512, 512), "bilinear"), ((200, 150), (100, 60), "bicubic"),
                                           ((64, 48), (48, 64), "lanczos"), ((50, 40), (17, 9), "box")])
def test_oracle_resize_matches_pil_on_raw_frames(size, res, filt):
    """The frame path's arithmetic (lean_resize_frames on PIL frames, functional.py:42-86) pinned directly
    against Pillow, independent of JPEG decoding: crop_to_aspect_ratio then Image.resize."""
    Image = pytest.importorskip("PIL.Image")
    from tests.golden.synth import synth_rgb
    w, h = size
    out_h, out_w = res
    rgb = synth_rgb(np.random.default_rng(w * h), w, h)
    l, t, r, b = O.crop_box(w, h, out_h, out_w)
    img = Image.fromarray(rgb).crop((l, t, r, b)).resize((out_w, out_h), getattr(Image, filt.upper()))
    np.testing.assert_array_equal(O.resize(np.ascontiguousarray(rgb[t:b, l:r]), out_h, out_w, filt), np.asarray(img))


def test_oracle_progressive_matches_pil():
    """Progressive JPEGs: the oracle's restatement of jdphuff.c decodes what PIL
    decodes, bit for bit (random sizes, samplings, qualities, optimized tables, restart intervals, gray)."""
    import io

    from PIL import Image

    from tests.golden.synth import progressive_jpegs
    for k, j in enumerate(progressive_jpegs(5, 60)):
        ref = np.array(Image.open(io.BytesIO(j)).convert("RGB"))
        np.testing.assert_array_equal(O.decode(j), ref, err_msg=f"image {k}")


def test_oracle_progressive_damaged_status_matches_pil():
    """Damaged progressive streams (truncations, bit flips, a stray EOI): the oracle raises exactly when
    PIL raises.  Pixels are not compared: a scan cut short leaves coefficients incomplete and libjpeg
    then smooths blocks across (jdcoefct.c decompress_smooth_data), which is not restated."""
    import io

    from PIL import Image

    from tests.golden.synth import progressive_jpegs
    for seed in (7, 8, 9):
        rng = np.random.default_rng(seed)
        for j in progressive_jpegs(seed, 12):
            for _ in range(10):
                kind, jb = int(rng.integers(0, 3)), bytearray(j)
                if kind == 0:
                    jb = jb[:int(rng.integers(len(j) // 3, len(j)))]
                elif kind == 1:
                    jb[int(rng.integers(len(j) // 4, len(j) - 4))] ^= 1 << int(rng.integers(0, 8))
                else:
                    p = int(rng.integers(len(j) // 4, len(j) - 4))
                    jb[p:p] = b"\xff\xd9"
                jb = bytes(jb)
                try:
                    Image.open(io.BytesIO(jb)).convert("RGB")
                    pil_ok = True
                except Exception:
                    pil_ok = False
                try:
                    O.decode(jb)
                    oracle_ok = True
                except O.OracleError:
                    oracle_ok = False
                assert pil_ok == oracle_ok, (seed, kind)


def test_oracle_frame_resize_matches_g6_fallback_goldens():
    """G6 (tests/golden/make_fallback.py, made by the reference pipeline itself): for the samples the
    GPU JPEG kernels hand to PIL (PNG / WebP / GIF / BMP / TIFF / CMYK JPEG / JPEG without EOI), PIL's
    decode followed by the oracle's crop (functional.py:118-147) + resize (Pillow Resample.c) -- the
    checker of the GPU frame path that resizes them -- equals the reference's uint8 outputs."""
    import io
    import os

    from PIL import Image
    meta = G.load_json("g6_fallback.json")
    z = np.load(os.path.join(G.GOLDEN, "g6_fallback.npz"))
    checked = 0
    for case in meta["cases"]:
        data = z[f"{case['name']}__bytes"].tobytes()
        for vname, res, kw in meta["variants"]:
            key = f"{case['name']}__{vname}"
            if not case["variants"][vname]["ok"]:
                with pytest.raises(OSError):
                    Image.open(io.BytesIO(data)).convert("RGB")
                continue
            if key not in z.files:  # (float outputs are pinned by digest on the GPU side)
                continue
            rgb = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))
            h, w = rgb.shape[:2]
            out_h, out_w = res
            if (w, h) != (out_w, out_h):
                if kw.get("resize_kwargs", {}).get("crop_before_resize", True):
                    x0, y0, x1, y1 = O.crop_box(w, h, out_h, out_w)
                    rgb = rgb[y0:y1, x0:x1]
                rgb = O.resize(rgb, out_h, out_w)
            np.testing.assert_array_equal(rgb.transpose(2, 0, 1), z[key], err_msg=key)
            checked += 1
    assert checked >= 30
