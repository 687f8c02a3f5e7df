"""GPU parity of the MI355X path against the reference's golden vectors and the C oracle.

Every comparison is bit-exact (the decode, resize and routing steps are integer; the normalise
step is a 256-entry float32 table equal to the reference's ``x.float()/127.5 - 1``, so it is
bit-exact too: tolerance 0).  All calls go through the C-ABI (libsdsj.so via sds_amd).
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402  (checker only)
from tests import goldens as G  # noqa: E402


@pytest.fixture(scope="module")
def engine():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sds_amd.engine import JpegEngine
    return JpegEngine(max_batch=512)


def _status(engine, jpg):
    _, st = engine.decode_resize([jpg], (8, 8))
    return int(st[0])


G1 = list(G.g1())


@pytest.mark.parametrize("case,jpg,arrs", G1, ids=[c["name"] for c, _, _ in G1])
def test_g1_golden(engine, case, jpg, arrs):
    from sds_amd import _lib
    name = case["name"]
    if case["decode"] != "ok":
        assert _status(engine, jpg) == _lib.CORRUPT
        return
    w, h = case["size"]
    # full-resolution decode = same-size shortcut (functional.py:78-80)
    full, st = engine.decode_resize([jpg], (h, w), layout="hwc")
    assert st[0] == 0
    np.testing.assert_array_equal(full[0].cpu().numpy(), arrs["rgb"])
    for key, out in case["outputs"].items():
        res = tuple(int(v) for v in key.split("x"))
        got, st = engine.decode_resize([jpg], res)
        assert st[0] == 0
        np.testing.assert_array_equal(got[0].cpu().numpy(), arrs[f"out_{key}"])
        gn, st = engine.decode_resize([jpg], res, normalize=True)
        assert G.sha(gn[0].cpu().numpy()) == out["norm_sha256"]


def test_g1_as_one_batch(engine):
    """All decodable G1 cases in one launch at 48x64 (mixed sizes/samplings/restarts in a batch)."""
    cases = [(c, j, a) for c, j, a in G1 if c["decode"] == "ok"]
    got, st = engine.decode_resize([j for _, j, _ in cases], (48, 64))
    assert (st == 0).all()
    for k, (c, j, a) in enumerate(cases):
        np.testing.assert_array_equal(got[k].cpu().numpy(), a["out_48x64"], err_msg=c["name"])


def test_g2_synthetic_vga_batch(engine):
    meta, jpgs = G.g2_jpegs()
    got, st = engine.decode_resize(jpgs, (256, 256))
    assert (st == 0).all()
    gf, st = engine.decode_resize(jpgs, (256, 256), normalize=True)
    full0 = np.load(os.path.join(G.GOLDEN, "g2_full0.npy"))
    np.testing.assert_array_equal(got[0].cpu().numpy(), full0)
    for k, im in enumerate(meta["images"]):
        assert G.sha(got[k].cpu().numpy()) == im["u8_256_sha256"]
        assert G.sha(gf[k].cpu().numpy()) == im["f32_256_sha256"]


def test_g3_mixed_flip_normalize(engine):
    meta, jpgs = G.g3_jpegs()
    flips = [im["flip"] for im in meta["images"]]
    got, st = engine.decode_resize(jpgs, (512, 512), flip=flips)
    assert (st == 0).all()
    gf, _ = engine.decode_resize(jpgs, (512, 512), flip=flips, normalize=True)
    for k, im in enumerate(meta["images"]):
        assert G.sha(got[k].cpu().numpy()) == im["u8_512_sha256"], k
        assert G.sha(gf[k].cpu().numpy()) == im["f32_512_sha256"], k


def test_device_resident_api_matches_host_api(engine):
    _, jpgs = G.g2_jpegs()
    host, _ = engine.decode_resize(jpgs, (256, 256))
    lens = [len(j) for j in jpgs]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    blob = torch.from_numpy(np.frombuffer(b"".join(jpgs), np.uint8).copy()).cuda()
    out, st = engine.decode_resize_device(blob, torch.from_numpy(offs).cuda(),
                                          torch.tensor(lens, dtype=torch.int32).cuda(), (256, 256))
    assert (st.cpu() == 0).all()
    assert torch.equal(out, host)


def test_hwc_layout_and_flip(engine):
    _, jpgs = G.g2_jpegs()
    chw, _ = engine.decode_resize(jpgs[:2], (96, 128))
    hwc, _ = engine.decode_resize(jpgs[:2], (96, 128), layout="hwc", flip=[True, False])
    assert torch.equal(hwc[0].permute(2, 0, 1), torch.flip(chw[0], dims=[2]))
    assert torch.equal(hwc[1].permute(2, 0, 1), chw[1])


def test_pinned_host_output(engine):
    """out= pinned host memory: the kernels store the pixels over PCIe (bench.py --e2e-out pinned); same
    bytes as the device output, the failed sample zero-filled, and the host output of both lanes' slots"""
    _, jpgs = G.g2_jpegs()
    batch = list(jpgs) + [b"not a jpeg"]
    dev, st_d = engine.decode_resize(batch, (96, 128))
    host = torch.full((len(batch), 3, 96, 128), 7, dtype=torch.uint8).pin_memory()
    got, st_h = engine.decode_resize(batch, (96, 128), out=host)
    torch.cuda.synchronize()
    assert got.data_ptr() == host.data_ptr() and got.device.type == "cpu"
    assert (st_h == st_d).all() and st_h[-1] != 0 and (st_h[:-1] == 0).all()
    assert torch.equal(host, dev.cpu())
    assert int(host[-1].max()) == 0
    with pytest.raises(ValueError):
        engine.decode_resize(batch, (96, 128), out=torch.empty((len(batch), 3, 96, 128), dtype=torch.uint8))


def _random_jpegs(seed: int, n: int):
    from tests.golden.synth import encode_jpeg, synth_rgb
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        w, h = int(rng.integers(1, 300)), int(rng.integers(1, 300))
        rgb = rng.integers(0, 256, (h, w, 3), dtype=np.uint8) if i % 2 else synth_rgb(rng, w, h)
        kw = dict(quality=int(rng.integers(5, 101)))
        if i % 5 == 0:
            from PIL import Image
            rgb = np.array(Image.fromarray(rgb).convert("L"))
        else:
            kw["subsampling"] = int(rng.integers(0, 3))
        r = rng.random()
        if r < 0.2:
            kw["restart_marker_blocks"] = int(rng.integers(1, 6))
        elif r < 0.35:
            kw["restart_marker_rows"] = int(rng.integers(1, 3))
        if rng.random() < 0.25:
            kw["optimize"] = True
        out.append(encode_jpeg(rgb, **kw))
    return out


@pytest.mark.parametrize("seed", [0, 1])
def test_random_batch_vs_oracle(engine, seed):
    jpgs = _random_jpegs(seed, 64)
    rng = np.random.default_rng(seed + 100)
    res = (int(rng.integers(1, 200)), int(rng.integers(1, 200)))
    got, st = engine.decode_resize(jpgs, res)
    assert (st == 0).all()
    for k, j in enumerate(jpgs):
        np.testing.assert_array_equal(got[k].cpu().numpy(), O.pipeline(j, res), err_msg=f"image {k}")


@pytest.mark.parametrize("filt", ["box", "bicubic", "hamming", "lanczos", "nearest"])
def test_other_pillow_filters(engine, filt):
    _, jpgs = G.g2_jpegs()
    got, st = engine.decode_resize(jpgs[:2], (200, 150), filter=filt)
    for k in range(2):
        np.testing.assert_array_equal(got[k].cpu().numpy(), O.pipeline(jpgs[k], (200, 150), filter=filt))


@pytest.mark.parametrize("seed", [31, 32])
def test_nearest_random_batches_vs_oracle(engine, seed):
    """NEAREST (Pillow ImagingScaleAffine as one-tap resamples) on random JPEGs (samplings, restarts,
    optimized tables) at random up- and down-scaled resolutions, crop and no crop, flips and HWC."""
    jpgs = _random_jpegs(seed, 48)
    rng = np.random.default_rng(seed + 7)
    for crop in (True, False):
        res = (int(rng.integers(1, 300)), int(rng.integers(1, 300)))
        flip = [bool(v) for v in rng.integers(0, 2, len(jpgs))]
        got, st = engine.decode_resize(jpgs, res, filter="nearest", crop_before_resize=crop, flip=flip)
        assert (st == 0).all()
        for k, j in enumerate(jpgs):
            np.testing.assert_array_equal(got[k].cpu().numpy(),
                                          O.pipeline(j, res, crop_before_resize=crop, filter="nearest", flip=flip[k]),
                                          err_msg=f"image {k} res {res} crop {crop}")


def test_4k_vs_oracle(engine):
    from tests.golden.synth import encode_jpeg, synth_rgb
    rng = np.random.default_rng(5)
    jpg = encode_jpeg(synth_rgb(rng, 3840, 2160), 90)
    got, st = engine.decode_resize([jpg], (512, 512), flip=[True])
    assert st[0] == 0
    np.testing.assert_array_equal(got[0].cpu().numpy(), O.pipeline(jpg, (512, 512), flip=True))


def test_fused_tile_span_edges_vs_oracle(engine):
    """Bilinear scales at the 7-tap fused kernels' row bound (sds_amd/csrc/sdsj_common.h rs_span: 768
    source columns; a 256-column tile at scale s spans 256 s + 2 s + 4): square crops of 755..768 rows
    to 256 x 256 (tiles of 256 below 2.97, halved above), the 9-tap neighbour just past scale 3, and
    every chroma layout."""
    from PIL import Image
    from tests.golden.synth import encode_jpeg, synth_rgb
    rng = np.random.default_rng(77)
    jpgs = []
    for side, extra in ((755, 40), (760, 0), (765, 120), (768, 32), (771, 8)):
        rgb = synth_rgb(rng, side + extra, side)
        for sub in (2, 1, 0):
            jpgs.append(encode_jpeg(rgb, 90, subsampling=sub))
        jpgs.append(encode_jpeg(np.array(Image.fromarray(rgb).convert("L")), 90))
    for res in ((256, 256), (256, 200)):
        flip = [bool(v) for v in rng.integers(0, 2, len(jpgs))]
        got, st = engine.decode_resize(jpgs, res, flip=flip)
        assert (st == 0).all()
        for k, j in enumerate(jpgs):
            np.testing.assert_array_equal(got[k].cpu().numpy(), O.pipeline(j, res, flip=flip[k]),
                                          err_msg=f"image {k} res {res}")


@pytest.mark.parametrize("rst", [0, 3])
def test_tile_parallel_unstuff_vs_oracle(engine, rst):
    """Images of more than kUsSerialTiles (64) 8 KiB tiles take the tile-parallel unstuff passes: noise
    content (dense FF00 stuffing across tile boundaries), restart markers split across tiles, and a copy
    truncated mid-scan."""
    from tests.golden.synth import encode_jpeg
    rng = np.random.default_rng(40 + rst)
    rgb = rng.integers(0, 256, (1024, 1536, 3), dtype=np.uint8)
    kw = {"restart_marker_blocks": rst} if rst else {}
    jpg = encode_jpeg(rgb, 95, **kw)
    assert len(jpg) > 64 * 8192 + 4096
    cut = jpg[: len(jpg) * 2 // 3]
    res = (200, 300)
    got, st = engine.decode_resize([jpg, cut, jpg], res)
    for k, j in enumerate([jpg, cut, jpg]):
        ost, ref = _oracle_result(j, res)
        assert int(st[k]) == ost, f"sample {k}: gpu {int(st[k])} vs oracle {ost}"
        if ost == O.OK:
            np.testing.assert_array_equal(got[k].cpu().numpy(), ref, err_msg=f"sample {k}")


def _oracle_result(jpg, res):
    try:
        return O.OK, O.pipeline(jpg, res)
    except O.OracleError as e:
        return e.status, None


@pytest.mark.parametrize("seed", [11, 12])
def test_mutated_streams_match_oracle_status_and_pixels(engine, seed):
    """Status per sample equals the oracle's (OK / CORRUPT); OK samples are bit-exact.  Streams with fill
    bytes before a stuffed zero (FF FF .. 00, no restart intervals) report CORRUPT (libjpeg-turbo's fast
    path decodes them differently from the slow path the oracle restates; the transforms rerun them on PIL)."""
    from tests.golden.synth import has_fill_stuffing, mutated_jpegs
    jpgs = mutated_jpegs(seed, 40)
    res = (48, 64)
    got, st = engine.decode_resize(jpgs, res)
    for k, j in enumerate(jpgs):
        ost, ref = _oracle_result(j, res)
        if ost == O.OK and has_fill_stuffing(j):
            ost = O.CORRUPT
        assert int(st[k]) == ost, f"sample {k}: gpu {int(st[k])} vs oracle {ost}"
        if ost == O.OK:
            np.testing.assert_array_equal(got[k].cpu().numpy(), ref, err_msg=f"sample {k}")


def test_simd_idct_semantics_on_extreme_coefficients_vs_oracle(engine):
    """k_idct's 16-bit lane semantics (libjpeg-turbo's x86 SIMD ISLOW, which Pillow runs): JPEGs whose
    dequantised coefficients leave 16 bits (tests/golden/coefjpeg.py; the oracle equals PIL on them,
    test_oracle_simd_idct_matches_pil_on_extreme_coefficients) -- full-resolution HWC decodes, and
    crop + resize with flips -- bit-exact against the oracle."""
    from tests.golden.coefjpeg import extreme_jpegs
    jpgs = extreme_jpegs(202, 96)
    for j in jpgs[:24]:
        ref = O.decode(j)
        got, st = engine.decode_resize([j], ref.shape[:2], layout="hwc")
        assert st[0] == 0
        np.testing.assert_array_equal(got[0].cpu().numpy(), ref)
    res = (24, 20)
    flips = [k % 2 == 1 for k in range(len(jpgs))]
    got, st = engine.decode_resize(jpgs, res, flip=flips)
    assert (st == 0).all(), st
    for k, j in enumerate(jpgs):
        np.testing.assert_array_equal(got[k].cpu().numpy(), O.pipeline(j, res, flip=flips[k]), err_msg=f"image {k}")


@pytest.mark.parametrize("n", [1, 3, 40])
def test_six_table_slot_images_vs_oracle(engine, n):
    """Baseline images whose Cb and Cr use their own DC/AC Huffman tables (6 slots, the 10-bit entropy
    route), alone and mixed with PIL-encoded 4-slot images: batches of <= 32 host images run in latency
    mode, whose multi-hypothesis pass only the 11-bit routes launch (such an image must keep
    the ordinary speculative pass); 40 runs the throughput plan.  Bit-exact against the oracle."""
    from tests.golden.coefjpeg import six_slot_jpegs
    from tests.golden.synth import encode_jpeg, synth_rgb
    six = six_slot_jpegs(41, 4, 320, 240)
    rng = np.random.default_rng(5)
    jpgs = []
    for k in range(n):
        jpgs.append(six[k % 4] if k % 2 == 0 else encode_jpeg(synth_rgb(rng, 320, 240), 90))
    res = (96, 80)
    got, st = engine.decode_resize(jpgs, res)
    assert (st == 0).all(), st
    for k, j in enumerate(jpgs):
        np.testing.assert_array_equal(got[k].cpu().numpy(), O.pipeline(j, res), err_msg=f"image {k}")
    full, st = engine.decode_resize(six[:1], (240, 320), layout="hwc")
    assert st[0] == 0
    np.testing.assert_array_equal(full[0].cpu().numpy(), O.decode(six[0]))


def test_scan_components_out_of_frame_order_are_unsupported(engine):
    """Scan component order differing from the frame's: UNSUPPORTED on the GPU, as in the oracle (PIL rejects it
    too: test_scan_components_out_of_frame_order_are_rejected_like_pil); the write pass's predictor rotation
    follows the MCU's component cycle, which is then always the frame order."""
    from sds_amd import _lib
    from tests.golden.coefjpeg import six_slot_jpegs
    jpgs = [j for order in ([2, 1, 0], [1, 2, 0]) for j in six_slot_jpegs(5, 2, 96, 64, order=order)]
    _, st = engine.decode_resize(jpgs, (32, 32))
    assert all(int(v) == _lib.UNSUPPORTED for v in st), st


def test_fill_stuffed_streams_rerun_on_pil_through_the_transform(engine):
    """FF FF .. 00 inside a baseline scan: the GPU reports CORRUPT, the per-sample transform reruns the
    sample on PIL, so the output equals the reference's PIL decode + resize."""
    import io
    import tempfile

    from PIL import Image

    from sds_amd.presets import create_standard_image_pipeline
    from tests.golden.synth import encode_jpeg, has_fill_stuffing, synth_rgb
    tmp = tempfile.mkdtemp()
    n = 0
    for seed in range(6):
        j = encode_jpeg(synth_rgb(np.random.default_rng(seed), 160, 120), 90)
        sos = j.index(b"\xff\xda")
        p = sos + 2 + ((j[sos + 2] << 8) | j[sos + 3]) + 200 + 37 * seed
        jb = j[:p] + b"\xff\xff\xff\x00" + j[p:]
        assert has_fill_stuffing(jb)
        _, st = engine.decode_resize([jb], (32, 32))
        assert st[0] == O.CORRUPT
        path = f"{tmp}/{seed}.jpg"
        with open(path, "wb") as f:
            f.write(jb)
        img = {"jpg": path}
        for t in create_standard_image_pipeline("jpg", (32, 32), device="cuda"):
            img = t(img)
        pil = Image.open(io.BytesIO(jb)).convert("RGB")
        x0, y0, x1, y1 = O.crop_box(160, 120, 32, 32)
        ref = np.asarray(pil.crop((x0, y0, x1, y1)).resize((32, 32), Image.BILINEAR)).transpose(2, 0, 1)
        np.testing.assert_array_equal(img["image"].cpu().contiguous().numpy(), ref)
        n += 1
    assert n == 6


def test_empty_batch_and_single_pixel(engine):
    got, st = engine.decode_resize([], (32, 32))
    assert got.shape[0] == 0 and len(st) == 0
    from tests.golden.synth import encode_jpeg
    jpg = encode_jpeg(np.full((1, 1, 3), 200, np.uint8), 90)
    got, st = engine.decode_resize([jpg] * 3, (5, 7))
    assert (st == 0).all()
    for k in range(3):
        np.testing.assert_array_equal(got[k].cpu().numpy(), O.pipeline(jpg, (5, 7)))


def test_g5_edge_cases(engine):
    """Huffman-table validation, scan termination, premature markers and post-scan markers as the reference
    loader behaves (tests/golden/make_edge.py): decodable cases bit-exact at full resolution."""
    import base64
    from sds_amd import _lib
    for c in G.load_json("g5_edge.json")["cases"]:
        jpg = base64.b64decode(c["jpg_b64"])
        if c["outcome"] != "ok":
            assert _status(engine, jpg) == _lib.CORRUPT, c["name"]
            continue
        w, h = c["size"]
        full, st = engine.decode_resize([jpg], (h, w), layout="hwc")
        assert st[0] == 0, c["name"]
        assert G.sha(full[0].cpu().numpy()) == c["rgb_sha256"], c["name"]


def test_progressive_batch_vs_oracle(engine):
    """Progressive JPEGs (k_prog) mixed with baseline ones in one batch."""
    from tests.golden.synth import progressive_jpegs
    jpgs = progressive_jpegs(5, 40) + _random_jpegs(3, 24)
    res = (56, 72)
    got, st = engine.decode_resize(jpgs, res, flip=[k % 2 == 0 for k in range(len(jpgs))])
    assert (st == 0).all()
    for k, j in enumerate(jpgs):
        np.testing.assert_array_equal(got[k].cpu().numpy(), O.pipeline(j, res, flip=k % 2 == 0), err_msg=f"image {k}")


def test_progressive_full_resolution_and_damaged_streams(engine):
    from tests.golden.synth import progressive_jpegs
    jpgs = progressive_jpegs(6, 6)
    for j in jpgs:  # full-resolution decode = the same-size shortcut
        ref = O.decode(j)
        got, st = engine.decode_resize([j], ref.shape[:2], layout="hwc")
        assert st[0] == 0
        np.testing.assert_array_equal(got[0].cpu().numpy(), ref)
    rng = np.random.default_rng(17)
    bad = []
    for j in progressive_jpegs(7, 8):
        for _ in range(6):
            jb = bytearray(j)
            kind = int(rng.integers(0, 3))
            if kind == 0:
                jb = jb[:int(rng.integers(len(j) // 3, len(j)))]
            elif kind == 1:
                jb[int(rng.integers(len(j) // 4, len(j) - 4))] ^= 1 << int(rng.integers(0, 8))
            else:
                p = int(rng.integers(len(j) // 4, len(j) - 4))
                jb[p:p] = b"\xff\xd9"
            bad.append(bytes(jb))
    res = (40, 40)
    got, st = engine.decode_resize(bad, res)
    for k, j in enumerate(bad):
        ost, ref = _oracle_result(j, res)
        assert int(st[k]) == ost, f"sample {k}: gpu {int(st[k])} vs oracle {ost}"
        if ost == O.OK:
            np.testing.assert_array_equal(got[k].cpu().numpy(), ref, err_msg=f"sample {k}")


def test_progressive_bench_sized_images_vs_oracle(engine):
    """The progressive bench's own inputs (640x480 q90, PIL's scan script) and a 1920x1080 4:4:4
    one, decoded + resized on the GPU, bit-exact against the oracle (tools/prog_bench.py measures
    these shapes)."""
    from tests.golden.synth import encode_jpeg, synth_rgb
    jpgs = [encode_jpeg(synth_rgb(np.random.default_rng(1234 + i), 640, 480), 90, progressive=True) for i in range(3)]
    jpgs.append(encode_jpeg(synth_rgb(np.random.default_rng(99), 1920, 1080), 95, progressive=True, subsampling=0))
    for res in ((256, 256), (480, 640)):
        got, st = engine.decode_resize(jpgs, res)
        assert (st == 0).all(), st
        for k, j in enumerate(jpgs):
            np.testing.assert_array_equal(got[k].cpu().numpy(), O.pipeline(j, res), err_msg=f"image {k} at {res}")


def test_progressive_incomplete_scans_smoothing_vs_oracle(engine):
    """Progressive images that end (EOI) after each of their scans: k_prog records the coefficient bits
    and k_prog_smooth applies libjpeg-turbo's block smoothing (jdcoefct.c decompress_smooth_data, 5x5
    DC neighbourhood, DC interpolation) before k_idct -- bit-exact against the oracle, which is pinned
    to PIL on the same construction (test_oracle_progressive_smoothing_matches_pil).  Full-resolution
    HWC decodes and a crop + resize with flips, mixed in one batch with complete images."""
    from tests.golden.synth import progressive_jpegs
    cases = []
    for seed, mw, mh in ((5, 400, 300), (7, 40, 40)):
        for j in progressive_jpegs(seed, 10, mw, mh):
            sos = [i for i in range(2, len(j) - 1) if j[i] == 0xFF and j[i + 1] == 0xDA][1:]
            cases += [j[:c] + b"\xff\xd9" for c in sos] + [j]
    for j in cases[::7]:  # full resolution (the same-size shortcut: no resample)
        ref = O.decode(j)
        got, st = engine.decode_resize([j], ref.shape[:2], layout="hwc")
        assert st[0] == 0
        np.testing.assert_array_equal(got[0].cpu().numpy(), ref)
    res = (48, 40)
    flips = [k % 3 == 0 for k in range(len(cases))]
    got, st = engine.decode_resize(cases, res, flip=flips)
    assert (st == 0).all(), st
    for k, j in enumerate(cases):
        np.testing.assert_array_equal(got[k].cpu().numpy(), O.pipeline(j, res, flip=flips[k]), err_msg=f"case {k}")


def test_progressive_truncated_inside_scans_vs_oracle(engine):
    """Progressive images cut inside each scan's entropy-coded data (then EOI): the scan runs out of
    data mid-way (jdhuff.c insufficient_data -- the rest reads as zeros, later MCUs are skipped), which
    every scan kind meets here -- the lane-parallel AC refinement and the 32-blocks-per-read DC
    refinement included -- and the smoothing takes the row where the data ended.  Against the oracle
    (statuses and pixels, crop + resize)."""
    from tests.golden.synth import progressive_jpegs
    cases = []
    for seed, mw, mh in ((11, 400, 300), (13, 64, 48)):
        for j in progressive_jpegs(seed, 4, mw, mh):
            sos = [i for i in range(2, len(j) - 1) if j[i] == 0xFF and j[i + 1] == 0xDA]
            ends = sos[1:] + [len(j) - 2]
            for a, e in zip(sos, ends):
                for f in (0.2, 0.55, 0.9):
                    cases.append(j[:a + 14 + int((e - a - 14) * f)] + b"\xff\xd9")
    res = (40, 48)
    got, st = engine.decode_resize(cases, res)
    host = got.cpu().numpy()
    for k, j in enumerate(cases):
        try:
            ref, rst = O.pipeline(j, res), 0
        except O.OracleError as e:
            ref, rst = None, e.status
        assert st[k] == rst, (k, st[k], rst)
        if ref is not None:
            np.testing.assert_array_equal(host[k], ref, err_msg=f"case {k}")


def test_progressive_dri_between_scans_vs_oracle(engine):
    """A DRI segment between the scans of a progressive image (restart intervals that change per
    scan, jdmarker.c get_dri), with non-zero and zero intervals, against the oracle: status, and
    pixels where the oracle decodes.  (The scans after a non-zero DRI lack their RSTn markers, so
    they are damaged streams: on 6 of these 24 images PIL differs from the oracle in a few pixels
    swapped between 0 and 255 -- garbage coefficients past 16 bits, which Pillow's SIMD IDCT wraps
    and the C jpeg_idct_islow restated here does not: DESIGN.md §2, divergence 2.)"""
    from tests.golden.synth import progressive_jpegs
    cases = []
    for j in progressive_jpegs(11, 8):
        sos = [i for i in range(len(j) - 1) if j[i] == 0xFF and j[i + 1] == 0xDA]
        if len(sos) < 3:
            continue
        for at, interval in ((sos[2], 2), (sos[-1], 1), (sos[1], 0)):
            cases.append(j[:at] + b"\xff\xdd\x00\x04" + interval.to_bytes(2, "big") + j[at:])
    assert cases
    res = (40, 40)
    got, st = engine.decode_resize(cases, res)
    for k, j in enumerate(cases):
        ost, ref = _oracle_result(j, res)
        assert int(st[k]) == ost, f"case {k}: gpu {int(st[k])} vs oracle {ost}"
        if ost == O.OK:
            np.testing.assert_array_equal(got[k].cpu().numpy(), ref, err_msg=f"case {k}")


@pytest.mark.gpu
def test_device_entry_rejects_ranges_outside_the_blob():
    """ABI v2: sdsj_decode_resize_batch_device takes the blob's size; a sample whose [offset, offset +
    length) is negative or leaves the blob reports SDSJ_EINVAL (checked on the device before any read),
    and the valid samples of the same batch decode normally."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sds_amd import _lib
    from sds_amd.engine import JpegEngine
    _, jpgs = G.g2_jpegs()
    j = jpgs[0]
    blob = torch.from_numpy(np.frombuffer(j + bytes(64), np.uint8).copy()).cuda()
    n = blob.numel()
    offs = torch.tensor([0, n - 10, -16, 0, 32], dtype=torch.int64).cuda()
    lens = torch.tensor([len(j), 100, len(j), -1, n], dtype=torch.int32).cuda()
    eng = JpegEngine("cuda:0", max_batch=16)
    eng.reserve(JpegEngine.scratch_need([j], (64, 64)) * 2 + (16 << 20))
    out, st = eng.decode_resize_device(blob, offs, lens, (64, 64))
    torch.cuda.synchronize()
    assert st.cpu().tolist() == [_lib.OK, _lib.EINVAL, _lib.EINVAL, _lib.EINVAL, _lib.EINVAL]
    np.testing.assert_array_equal(out[0].cpu().numpy(), O.pipeline(j, (64, 64)))
    assert int(out[1:].abs().sum()) == 0  # failed samples are zero-filled
