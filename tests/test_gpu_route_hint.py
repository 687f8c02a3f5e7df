"""The device path's route hint (sdsj_kernels.h route_grid, sdsj_engine.hip run_chunk): after batches of
one kind (VGA 4:2:0 baseline: one unstuff, entropy and resample route), a batch that takes many other
routes -- small images of every G1 sampling / restart layout, 4:2:2 / 4:4:4 / gray, progressive,
6-slot Huffman tables, a large multi-group image -- runs those routes on small strided grids.  Its
outputs must still equal the oracle's bit for bit, and so must the next batch (full grids again)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402  (checker only)
from tests import goldens as G  # noqa: E402


def _device_batch(jpgs):
    lens = [len(j) for j in jpgs]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    blob = torch.from_numpy(np.frombuffer(b"".join(jpgs), np.uint8).copy()).cuda()
    return blob, torch.from_numpy(offs).cuda(), torch.tensor(lens, dtype=torch.int32).cuda()


def test_cold_routes_after_a_homogeneous_stream_match_the_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sds_amd.engine import JpegEngine
    from tests.golden.coefjpeg import six_slot_jpegs
    from tests.golden.synth import encode_jpeg, synth_rgb
    res = (48, 64)
    _, g2 = G.g2_jpegs()
    homog = [g2[k % len(g2)] for k in range(640)]  # 4 lanes of 160 images
    rng = np.random.default_rng(17)
    mixed = [j for c, j, _ in G.g1() if c["decode"] == "ok"]
    for kw in ({}, {"subsampling": "4:2:2"}, {"subsampling": "4:4:4"}, {"restart_marker_blocks": 3}):
        mixed.append(encode_jpeg(synth_rgb(rng, 200, 150), 85, **kw))
    import io

    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(synth_rgb(rng, 160, 120)).convert("L").save(buf, format="JPEG", quality=90)
    mixed.append(buf.getvalue())
    mixed.append(encode_jpeg(synth_rgb(rng, 180, 120), 90, progressive=True))
    mixed += six_slot_jpegs(43, 2, 160, 120)
    mixed.append(encode_jpeg(synth_rgb(rng, 1920, 1080), 95))  # > 256 x 8,192 entropy bits: multi-group
    batch = [mixed[k % len(mixed)] for k in range(640)]
    ref = {j: O.pipeline(j, res) for j in mixed}
    eng = JpegEngine("cuda:0", max_batch=640)
    eng.reserve(JpegEngine.scratch_need(batch, res) + JpegEngine.scratch_need(homog, res) + (64 << 20))
    hb = _device_batch(homog)
    for _ in range(3):  # the hint learns the homogeneous batch's routes (readbacks fold one call later)
        out, st = eng.decode_resize_device(*hb, res)
        torch.cuda.synchronize()
        assert (st.cpu() == 0).all()
    mb = _device_batch(batch)
    for rep in range(2):  # rep 0: the other routes are cold (small grids); rep 1: hinted again
        out, st = eng.decode_resize_device(*mb, res)
        torch.cuda.synchronize()
        assert (st.cpu() == 0).all(), st
        got = out.cpu().numpy()
        for k, j in enumerate(batch):
            np.testing.assert_array_equal(got[k], ref[j], err_msg=f"rep {rep} image {k}")
