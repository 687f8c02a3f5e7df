"""Asynchronous host path: double-buffered pinned slots, bytes or files read
straight into pinned memory (sdsj_submit_batch / sdsj_submit_files / sdsj_wait_batch).  Results are
checked against the oracle (the CPU restatement pinned to the reference's goldens), status and
pixels; an unreadable file is a per-sample SDSJ_EINVAL.  Includes configs[4]'s shape on one GPU:
640x480 JPEG files -> pinned slot -> H2D -> decode + resize 512x512 -> D2H."""
import os
import tempfile

import numpy as np
import pytest

from oracle import oracle as O

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


def _check_vs_oracle(jpgs, out, st, res, flip=None, normalize=False, skip=()):
    from sds_amd import _lib
    from tests.golden.synth import has_fill_stuffing
    host = out.cpu().numpy()
    for i, j in enumerate(jpgs):
        if i in skip:
            continue
        try:
            ref = O.pipeline(j, res, flip=bool(flip[i]) if flip else False, normalize=normalize)
            rst = _lib.OK
        except O.OracleError as e:
            ref, rst = None, e.status
        if rst == _lib.OK and has_fill_stuffing(j):  # (FF FF .. 00: reported CORRUPT, rerun on PIL)
            ref, rst = None, _lib.CORRUPT
        assert st[i] == rst, (i, st[i], rst)
        if ref is not None:
            np.testing.assert_array_equal(host[i], ref, err_msg=f"sample {i}")


def test_submit_wait_matches_oracle(engine):
    res = (48, 40)
    batches = _batches()[:2]
    flips = [[i % 3 == 0 for i in range(len(b))] for b in batches]
    for slot, batch in enumerate(batches):
        engine.submit(slot, batch, res, flip=flips[slot], normalize=True)
    for slot, batch in enumerate(batches):
        out, st = engine.wait(slot)
        _check_vs_oracle(batch, out, st, res, flip=flips[slot], normalize=True)


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
    before = engine.counters()
    got = list(engine.decode_stream(paths, (64, 64), files=True))
    after = engine.counters()
    assert len(got) == 3
    assert after["other"] == before["other"] + 1  # the unreadable file, counted as such
    # the missing file moves no other count: corrupt / unsupported grow by the returned statuses alone
    sts = np.concatenate([np.asarray(st) for _, st in got])
    assert after["corrupt"] - before["corrupt"] == int((sts == _lib.CORRUPT).sum())
    assert after["unsupported"] - before["unsupported"] == int((sts == _lib.UNSUPPORTED).sum())
    for b, (out, st) in enumerate(got):
        if b == 1:
            assert st[3] == _lib.EINVAL
        _check_vs_oracle(batches[b], out, st, (64, 64), skip=(3,) if b == 1 else ())


def test_resubmitting_a_busy_slot_waits_for_it(engine):
    a, b = _batches()[0], _batches()[2]
    out_a = engine.submit(0, a, (32, 32))
    out_b = engine.submit(0, b, (32, 32))  # the native side waits for batch a before restaging
    got_b, st_b = engine.wait(0)
    assert got_b is out_b
    _check_vs_oracle(a, out_a, np.zeros(len(a), np.int32), (32, 32))
    _check_vs_oracle(b, got_b, st_b, (32, 32))
    with pytest.raises(RuntimeError):
        engine.wait(0)


def test_config4_files_to_512_and_back_to_host_vs_oracle(engine):
    """configs[4] on one GPU: synthetic 640x480 q90 JPEG files (the downloader's local cache) -> pinned
    slot -> H2D -> decode + centre crop + resize 512x512 -> D2H into pinned host memory."""
    from tests.golden.synth import synth_jpegs
    jpgs = synth_jpegs(24, seed=4040)
    d = tempfile.mkdtemp()
    paths = []
    for i, j in enumerate(jpgs):
        p = os.path.join(d, f"{i}.jpg")
        with open(p, "wb") as f:
            f.write(j)
        paths.append(p)
    batches = [paths[:8], paths[8:16], paths[16:]]
    host = torch.empty((24, 3, 512, 512), dtype=torch.uint8).pin_memory()
    k = 0
    for out, st in engine.decode_stream(batches, (512, 512), files=True):
        assert (st == 0).all(), st
        host[k:k + len(st)].copy_(out, non_blocking=True)
        k += len(st)
    torch.cuda.synchronize()
    for i, j in enumerate(jpgs):
        np.testing.assert_array_equal(host[i].numpy(), O.pipeline(j, (512, 512)), err_msg=f"image {i}")
