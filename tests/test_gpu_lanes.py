"""Lanes (sdsj_engine.hip run_chunk): a chunk of >= 2 x 256 images runs as up to 4 image ranges on
separate streams.  Results must be those of one lane: per-image pixels and statuses, and -- with a
scratch capacity too small for the batch -- the same images failing with ECAPACITY (scratch is
taken in image order across lanes).  Checked against a one-lane engine and, on a sample, the oracle.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402  (checker only)


def _engine(monkeypatch, lanes, **kw):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sds_amd.engine import JpegEngine
    monkeypatch.setenv("SDSJ_LANES", str(lanes))
    return JpegEngine(**kw)


def _batch():
    from tests.golden.synth import mutated_jpegs
    from tests.test_gpu_parity import _random_jpegs
    return _random_jpegs(21, 400) + mutated_jpegs(21, 120) + _random_jpegs(22, 400)


def test_lanes_equal_one_lane_and_oracle(monkeypatch):
    from tests.golden.synth import has_fill_stuffing
    jpgs = _batch()
    res = (40, 56)
    got4, st4 = _engine(monkeypatch, 4, max_batch=1024).decode_resize(jpgs, res)
    got1, st1 = _engine(monkeypatch, 1, max_batch=1024).decode_resize(jpgs, res)
    np.testing.assert_array_equal(np.asarray(st4), np.asarray(st1))
    assert torch.equal(got4, got1)
    for k in range(0, len(jpgs), 9):
        try:
            ref, ost = O.pipeline(jpgs[k], res), O.OK
        except O.OracleError as e:
            ref, ost = None, e.status
        if ost == O.OK and has_fill_stuffing(jpgs[k]):  # (FF FF .. 00: reported CORRUPT, rerun on PIL)
            ref, ost = None, O.CORRUPT
        assert int(st4[k]) == ost, k
        if ref is not None:
            np.testing.assert_array_equal(got4[k].cpu().numpy(), ref, err_msg=f"image {k}")


def test_lanes_capacity_failures_in_image_order(monkeypatch):
    from tests.golden.synth import synth_jpegs
    jpgs = synth_jpegs(48, seed=5) * 12  # 576 VGA images: about a dozen fit in 64 MiB of scratch
    lens = [len(j) for j in jpgs]
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    blob = torch.from_numpy(np.frombuffer(b"".join(jpgs), np.uint8).copy()).cuda()
    d_offs, d_lens = torch.from_numpy(offs).cuda(), torch.tensor(lens, dtype=torch.int32).cuda()
    outs = []
    for lanes in (2, 1):
        eng = _engine(monkeypatch, lanes, max_batch=1024, scratch_bytes=64 << 20)
        out, st = eng.decode_resize_device(blob, d_offs, d_lens, (64, 64))
        outs.append((out, st.cpu().numpy()))
    (o2, s2), (o1, s1) = outs
    from sds_amd import _lib
    assert (s1 == _lib.ECAPACITY).any() and (s1 == 0).any()
    np.testing.assert_array_equal(s2, s1)
    ok = torch.from_numpy(s1 == 0).cuda()
    assert torch.equal(o2[ok], o1[ok])
