"""The headline configuration's batch-scale shortcuts, checked row by row at the bench's batch.

configs[1] runs 65,536 images per engine call in 4 lanes.  Several shortcuts exist only at that scale
and are invisible to small-batch tests: the decode tables shared within a lane from its image 0
(k_enttab, `ImgDesc::etab`), the resampling tables shared per crop geometry (k_coeffs), and the route
hint learnt from earlier batches (sdsj_engine.hip run_chunk).  Here 65,536 rows cycling G2's 8
synthetic 640x480 JPEGs (each row its own copy in HBM, as in bench.py) decode in one call, twice (the
second call runs on the hint of the first), and every row must equal its G2 golden -- the digests of
the reference pipeline (tests/golden/make_golden.py, functional.py:94-110).

Also: one engine alternating two output sizes (multi-scale training) keeps every call exact -- the
route hint is kept per op, so a call never runs on the routes of another size.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from oracle import oracle as O  # noqa: E402  (checker only)
from tests import goldens as G  # noqa: E402


def _rows(jpgs, nrows):
    """Device blob where row i holds its own 16-byte-aligned copy of jpgs[i % len(jpgs)]."""
    lens = np.array([len(j) for j in jpgs], np.int64)
    al = (lens + 15) // 16 * 16
    toffs = np.concatenate([[0], np.cumsum(al)[:-1]])
    T = int(al.sum())
    tmpl = np.zeros(T, np.uint8)
    for k, j in enumerate(jpgs):
        tmpl[toffs[k]:toffs[k] + lens[k]] = np.frombuffer(j, np.uint8)
    reps = (nrows + len(jpgs) - 1) // len(jpgs)
    blob = torch.from_numpy(tmpl).cuda().repeat(reps)
    i = np.arange(nrows)
    offs = (i // len(jpgs)) * T + toffs[i % len(jpgs)]
    return blob, torch.from_numpy(offs.astype(np.int64)).cuda(), torch.from_numpy(lens[i % len(jpgs)].astype(np.int32)).cuda()


def test_65536_rows_every_row_equals_its_golden():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sds_amd.engine import JpegEngine
    meta, jpgs = G.g2_jpegs()
    n, res = 65536, (256, 256)
    blob, offs, lens = _rows(jpgs, n)
    need = JpegEngine.scratch_need(jpgs, res)
    eng = JpegEngine("cuda:0", max_batch=n, scratch_bytes=need * (n // len(jpgs) + 1) + (64 << 20))
    eng.set_lanes(4)
    out = torch.empty((n, 3, 256, 256), dtype=torch.uint8, device="cuda:0")
    status = torch.empty(n, dtype=torch.int32, device="cuda:0")
    golden = [im["u8_256_sha256"] for im in meta["images"]]
    for call in range(2):  # call 1 runs on the route hint learnt from call 0
        out.fill_(0x5A)
        eng.decode_resize_device(blob, offs, lens, res, out=out, status=status)
        torch.cuda.synchronize()
        assert int((status != 0).sum()) == 0, f"call {call}: {int((status != 0).sum())} rows failed"
        for k in range(len(jpgs)):
            first = out[k].cpu().numpy()
            assert G.sha(first) == golden[k], f"call {call}: row {k} differs from its golden"
            rows = out[k::len(jpgs)]
            same = (rows == out[k]).flatten(1).all(1)
            bad = torch.nonzero(~same).flatten()
            assert bad.numel() == 0, f"call {call}: rows {(bad[:8] * len(jpgs) + k).tolist()} differ from row {k}"


def test_alternating_output_sizes_on_one_engine():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sds_amd.engine import JpegEngine
    _, jpgs = G.g2_jpegs()
    n = 1024
    blob, offs, lens = _rows(jpgs, n)
    sizes = [(256, 256), (224, 224), (160, 288)]
    ref = {r: [O.pipeline(j, r) for j in jpgs] for r in sizes}
    eng = JpegEngine("cuda:0", max_batch=n, scratch_bytes=JpegEngine.scratch_need(jpgs, (256, 256)) * (n // 8 + 1) +
                     (64 << 20))
    for call in range(9):
        r = sizes[call % len(sizes)]
        out, st = eng.decode_resize_device(blob, offs, lens, r)
        torch.cuda.synchronize()
        assert (st.cpu() == 0).all(), (call, r)
        got = out.cpu().numpy()
        for k in range(0, n, 61):
            np.testing.assert_array_equal(got[k], ref[r][k % len(jpgs)], err_msg=f"call {call} size {r} row {k}")
