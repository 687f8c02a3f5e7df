"""Asynchronous host path: double-buffered pinned slots, bytes or files read
straight into pinned memory (sdsj_submit_batch / sdsj_submit_files / sdsj_wait_batch).  Results must
equal the synchronous host path bit for bit; an unreadable file is a per-sample SDSJ_EINVAL."""
import os
import tempfile

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sds_amd.engine import JpegEngine
    return JpegEngine(max_batch=256)


def _batches():
    from tests.golden.synth import mutated_jpegs
    from tests.test_gpu_parity import _random_jpegs
    a = _random_jpegs(31, 40)
    return [a[:20], a[20:] + mutated_jpegs(31, 10), _random_jpegs(32, 33)]


def test_submit_wait_equals_sync_path(engine):
    res = (48, 40)
    for slot, batch in enumerate(_batches()[:2]):
        flip = [i % 3 == 0 for i in range(len(batch))]
        engine.submit(slot, batch, res, flip=flip, normalize=True)
    for slot, batch in enumerate(_batches()[:2]):
        out, st = engine.wait(slot)
        flip = [i % 3 == 0 for i in range(len(batch))]
        ref, rst = engine.decode_resize(batch, res, flip=flip, normalize=True)
        np.testing.assert_array_equal(st, rst)
        assert torch.equal(out, ref)


def test_decode_stream_of_files_with_a_missing_file(engine):
    d = tempfile.mkdtemp()
    batches, paths = _batches(), []
    for b, batch in enumerate(batches):
        ps = []
        for i, j in enumerate(batch):
            p = os.path.join(d, f"{b}_{i}.jpg")
            with open(p, "wb") as f:
                f.write(j)
            ps.append(p)
        paths.append(ps)
    paths[1][3] = os.path.join(d, "missing.jpg")
    from sds_amd import _lib
    got = list(engine.decode_stream(paths, (64, 64), files=True))
    assert len(got) == 3
    for b, (out, st) in enumerate(got):
        ref, rst = engine.decode_resize(batches[b], (64, 64))
        if b == 1:
            assert st[3] == _lib.EINVAL
            keep = [i for i in range(len(st)) if i != 3]
            np.testing.assert_array_equal(st[keep], rst[keep])
            assert torch.equal(out[keep], ref[keep])
        else:
            np.testing.assert_array_equal(st, rst)
            assert torch.equal(out, ref)


def test_resubmitting_a_busy_slot_waits_for_it(engine):
    a, b = _batches()[0], _batches()[2]
    out_a = engine.submit(0, a, (32, 32))
    out_b = engine.submit(0, b, (32, 32))  # the native side waits for batch a before restaging
    got_b, st_b = engine.wait(0)
    assert got_b is out_b
    ref_a, _ = engine.decode_resize(a, (32, 32))
    ref_b, rst_b = engine.decode_resize(b, (32, 32))
    assert torch.equal(out_a, ref_a) and torch.equal(got_b, ref_b)
    np.testing.assert_array_equal(st_b, rst_b)
    with pytest.raises(RuntimeError):
        engine.wait(0)
