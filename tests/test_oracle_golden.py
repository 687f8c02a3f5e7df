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
    (libjpeg-turbo's warning-and-continue recovery), with equal pixels -- garbage blocks included, through
    the 16-bit lanes of the SIMD IDCT Pillow runs.  Streams with fill bytes before a stuffed zero (FF FF
    .. 00) are compared by status only: the oracle restates jdhuff.c's slow path (one FF data byte), while
    PIL's decode_mcu_fast leaves its own coefficients under the slow path's in that MCU; the GPU reports
    them CORRUPT and the transforms rerun them on PIL (synth.has_fill_stuffing)."""
    import io
    Image = pytest.importorskip("PIL.Image")
    from tests.golden.synth import has_fill_stuffing, mutated_jpegs
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
        if ref is not None and not has_fill_stuffing(jpg):
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


def _scan_cuts(j: bytes) -> list:
    """Byte offsets of every SOS marker after the first: j[:cut] + EOI keeps the scans before it."""
    return [i for i in range(2, len(j) - 1) if j[i] == 0xFF and j[i + 1] == 0xDA][1:]


def test_oracle_progressive_smoothing_matches_pil():
    """Progressive images that end (EOI) before their last scans: libjpeg-turbo smooths the blocks whose
    coefficients 1..9 are still inexact (jdcoefct.c smoothing_ok / decompress_smooth_data: 5x5 DC
    neighbourhood, DC interpolation when a component has no AC data).  The oracle's restatement equals
    PIL bit for bit after every scan of every image: random sizes down to 1 pixel, gray, 4:2:0 / 4:2:2 /
    4:4:4, optimized tables, restart intervals."""
    import io

    from PIL import Image

    from tests.golden.synth import progressive_jpegs
    n = 0
    for seed, count, mw, mh in ((5, 24, 400, 300), (7, 24, 40, 40)):
        for k, j in enumerate(progressive_jpegs(seed, count, mw, mh)):
            for c in _scan_cuts(j):
                t = j[:c] + b"\xff\xd9"
                ref = np.array(Image.open(io.BytesIO(t)).convert("RGB"))
                np.testing.assert_array_equal(O.decode(t), ref, err_msg=f"seed {seed} image {k} cut {c}")
                n += 1
    assert n > 300


def test_oracle_progressive_damaged_status_matches_pil():
    """Damaged progressive streams (truncations, bit flips, a stray EOI): the oracle raises exactly when
    PIL raises, and the pixels are equal on all 210 decodable streams -- a scan cut short by a stray EOI
    switches its later iMCU rows to the previous scan's smoothing parameters (jdcoefct.c
    last_good_iMCU_row), and garbage coefficients whose dequantised values leave 16 bits go through the
    16-bit lanes of libjpeg-turbo's SIMD IDCT (13 of these streams; the C jpeg_idct_islow differs there)."""
    import io

    from PIL import Image

    from tests.golden.synth import progressive_jpegs
    decoded = 0
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
                    ref = np.array(Image.open(io.BytesIO(jb)).convert("RGB"))
                    pil_ok = True
                except Exception:
                    pil_ok = False
                try:
                    got = O.decode(jb)
                    oracle_ok = True
                except O.OracleError:
                    oracle_ok = False
                assert pil_ok == oracle_ok, (seed, kind)
                if pil_ok:
                    decoded += 1
                    np.testing.assert_array_equal(got, ref, err_msg=f"seed {seed} kind {kind}")
    assert decoded == 210, decoded


def test_oracle_progressive_dri_between_scans_matches_pil():
    """A DRI segment between the scans of a progressive image (jdmarker.c get_dri: restart intervals that
    change per scan; the scans after a non-zero DRI lack their RSTn markers, so they decode garbage): the
    oracle raises exactly when PIL raises and equals PIL's pixels (the GPU test of the same construction,
    test_progressive_dri_between_scans_vs_oracle, checks the kernels against this oracle)."""
    import io

    from PIL import Image

    from tests.golden.synth import progressive_jpegs
    n = 0
    for j in progressive_jpegs(11, 8):
        sos = [i for i in range(len(j) - 1) if j[i] == 0xFF and j[i + 1] == 0xDA]
        if len(sos) < 3:
            continue
        for at, interval in ((sos[2], 2), (sos[-1], 1), (sos[1], 0)):
            jb = j[:at] + b"\xff\xdd\x00\x04" + interval.to_bytes(2, "big") + j[at:]
            try:
                ref = np.array(Image.open(io.BytesIO(jb)).convert("RGB"))
            except OSError:
                ref = None
            try:
                got = O.decode(jb)
            except O.OracleError:
                got = None
            assert (ref is None) == (got is None), (n, at, interval)
            if ref is not None:
                np.testing.assert_array_equal(got, ref, err_msg=f"case {n}")
            n += 1
    assert n == 24


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


def test_oracle_nearest_matches_pil_on_random_shapes():
    """interpolation_mode 'nearest' / 'nearest-exact' (torchvision -> PIL NEAREST): the oracle's restatement
    of ImagingScaleAffine (running double sum of the scale, COORD truncation) equals Image.resize(NEAREST)
    on random up- and down-scales."""
    from PIL import Image
    rng = np.random.default_rng(44)
    for _ in range(300):
        w, h = (int(v) for v in rng.integers(1, 300, 2))
        ow, oh = (int(v) for v in rng.integers(1, 300, 2))
        a = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        ref = np.asarray(Image.fromarray(a).resize((ow, oh), Image.NEAREST))
        np.testing.assert_array_equal(O.resize(a, oh, ow, "nearest"), ref, err_msg=f"{w}x{h} -> {ow}x{oh}")


def test_oracle_matches_g7_nearest_goldens():
    """G7 (tests/golden/make_nearest.py, the reference pipeline with interpolation_mode nearest /
    nearest-exact): the oracle pipeline (decode, crop, NEAREST resize, flip-free, LUT normalise) equals the
    reference's outputs for every JPEG case; the PNG case through PIL's decode + the oracle's resize."""
    import io

    from PIL import Image
    meta = G.load_json("g7_nearest.json")
    z = np.load(f"{G.GOLDEN}/g7_nearest.npz")
    g1 = {c["name"]: jpg for c, jpg, _ in G.g1()}
    g2, g3 = G.g2_jpegs()[1], G.g3_jpegs()[1]
    checked = 0
    for case in meta["cases"]:
        src = case["source"]
        data = g1[case["name"]] if src == "g1" else g2[case["index"]] if src == "g2" else \
            g3[case["index"]] if src == "g3" else z[f"{case['name']}__bytes"].tobytes()
        for vname, ref in case["variants"].items():
            kw = ref["kwargs"]
            rk = kw.get("resize_kwargs", {})
            res = tuple(ref["resolution"])
            rgb = np.asarray(Image.open(io.BytesIO(data)).convert("RGB")) if src == "npz bytes" else O.decode(data)
            h, w = rgb.shape[:2]
            out_h, out_w = res
            if rk.get("allow_vertical") and h > w:
                out_h, out_w = max(res), min(res)
            if (w, h) != (out_w, out_h):
                if rk.get("crop_before_resize", True):
                    x0, y0, x1, y1 = O.crop_box(w, h, out_h, out_w)
                    rgb = rgb[y0:y1, x0:x1]
                # an empty crop (1x1 -> 48x64) resizes to zeros: every source index is outside the image
                rgb = O.resize(np.ascontiguousarray(rgb), out_h, out_w, "nearest") if rgb.size else \
                    np.zeros((out_h, out_w, 3), np.uint8)
            chw = np.ascontiguousarray(rgb.transpose(2, 0, 1))
            if kw.get("normalize"):
                chw = O.normalize_lut()[chw]
            assert G.sha(chw) == ref["sha256"], (case["name"], vname)
            checked += 1
    assert checked >= 70


def test_oracle_simd_idct_matches_pil_on_extreme_coefficients():
    """Baseline JPEGs written from chosen coefficients (tests/golden/coefjpeg.py) whose dequantised values
    leave 16 bits -- DC-only blocks (the SIMD pass-1 shortcut), row-0-only blocks, sparse and dense large AC
    terms, DC sums at the int16 limits, 8-bit and 16-bit quantisation tables, gray / 4:4:4 / 4:2:2 / 4:2:0:
    the oracle's restatement of libjpeg-turbo's x86 SIMD ISLOW IDCT equals PIL bit for bit (the C
    jpeg_idct_islow differs on every one of them)."""
    import io

    from PIL import Image

    from tests.golden.coefjpeg import extreme_jpegs
    for k, j in enumerate(extreme_jpegs(101, 120)):
        ref = np.asarray(Image.open(io.BytesIO(j)).convert("RGB"))
        np.testing.assert_array_equal(O.decode(j), ref, err_msg=f"image {k}")


def test_oracle_matches_pil_on_six_table_slot_jpegs():
    """Cb and Cr coded with their own DC/AC Huffman tables (6 distinct table slots; the kernels' 10-bit
    entropy route): the oracle equals PIL bit for bit (pins the GPU test of the same files)."""
    import io

    from PIL import Image

    from tests.golden.coefjpeg import six_slot_jpegs
    for k, j in enumerate(six_slot_jpegs(31, 6)):
        ref = np.asarray(Image.open(io.BytesIO(j)).convert("RGB"))
        np.testing.assert_array_equal(O.decode(j), ref, err_msg=f"image {k}")


def test_scan_components_out_of_frame_order_are_rejected_like_pil():
    """A baseline scan listing its components in another order than the frame (its MCUs then follow the
    scan's order) is rejected by PIL (libjpeg-turbo) and by the oracle alike."""
    import io

    import pytest
    from PIL import Image

    from tests.golden.coefjpeg import six_slot_jpegs
    for order in ([2, 1, 0], [1, 2, 0], [0, 2, 1]):
        for j in six_slot_jpegs(5, 2, 96, 64, order=order):
            with pytest.raises(OSError):
                Image.open(io.BytesIO(j)).convert("RGB")
            with pytest.raises(O.OracleError, match="status -2"):  # UNSUPPORTED
                O.decode(j)


def test_fill_stuffing_predicate():
    from tests.golden.synth import encode_jpeg, has_fill_stuffing, synth_rgb
    j = encode_jpeg(synth_rgb(np.random.default_rng(3), 64, 48), 90)
    assert not has_fill_stuffing(j)
    sos = j.index(b"\xff\xda")
    p = sos + 2 + ((j[sos + 2] << 8) | j[sos + 3]) + 40
    assert has_fill_stuffing(j[:p] + b"\xff\xff\xff\x00" + j[p:])
    assert not has_fill_stuffing(j[:p] + b"\xff\xff\xd9" + j[p:])  # fill bytes before a marker: valid
    jr = encode_jpeg(synth_rgb(np.random.default_rng(3), 64, 48), 90, restart_marker_blocks=2)
    sos = jr.index(b"\xff\xda")
    p = sos + 2 + ((jr[sos + 2] << 8) | jr[sos + 3]) + 40
    assert not has_fill_stuffing(jr[:p] + b"\xff\xff\x00" + jr[p:])  # restart intervals: slow path only
