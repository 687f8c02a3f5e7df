"""The restated local downloader (sds_amd/downloader.py) against the reference's semantics:
run_downloading_task (/root/reference/sds/downloader.py:117-131), LocalDownloader
(utils/download.py:830-861: copy to <dst>.tmp, rename), ParallelDownloader's completion stream and
failure cleanup (downloader.py:88-108), and the bounded completed queue (lazy_thread_pool.py:85-100)."""
import os
from itertools import islice

import pytest

from sds_amd.downloader import DownloadingTask, LocalDownloader, ParallelDownloader, run_downloading_task


def _src(tmp_path, n):
    d = tmp_path / "src"
    d.mkdir()
    out = []
    for i in range(n):
        p = d / f"{i:03d}.jpg"
        p.write_bytes(bytes([i % 256]) * (100 + i))
        out.append(str(p))
    return out


def test_cold_then_warm_task(tmp_path):
    src = _src(tmp_path, 2)
    cache = tmp_path / "cache"
    cache.mkdir()
    dst = [str(cache / "a.jpg"), str(cache / "b.jpg")]
    t = DownloadingTask("k", src, dst, 10, LocalDownloader(), True)
    assert run_downloading_task(t) == (100 + 101, 100 + 101)  # cold: everything copied
    for s, d in zip(src, dst):
        assert open(s, "rb").read() == open(d, "rb").read()
        assert not os.path.exists(d + ".tmp")
    assert run_downloading_task(t) == (201, 0)  # warm: skip_if_exists, nothing copied
    t.skip_if_exists = False
    assert run_downloading_task(t) == (201, 201)


def test_stale_tmp_is_replaced_and_file_url(tmp_path):
    src = _src(tmp_path, 1)
    dst = str(tmp_path / "x.jpg")
    with open(dst + ".tmp", "wb") as f:
        f.write(b"partial")
    LocalDownloader().download("file://" + src[0], dst)
    assert open(dst, "rb").read() == open(src[0], "rb").read()
    assert not os.path.exists(dst + ".tmp")
    with pytest.raises(ValueError):
        LocalDownloader().download("s3://bucket/key.jpg", dst)


def test_parallel_downloader_yields_every_row_once(tmp_path):
    src = _src(tmp_path, 40)
    cache = tmp_path / "cache"
    cache.mkdir()
    dl = ParallelDownloader(num_workers=4, prefetch=5, num_retries=1)
    try:
        for i, s in enumerate(src):
            dl.schedule_task(i, [s], [str(cache / f"{i}.jpg")])
        got = dict(islice(dl.yield_completed(), 15))  # a consumer taking a batch at a time
        got.update(dl.yield_completed())
        assert sorted(got) == list(range(40))
        assert all(got[i] == (100 + i, 100 + i) for i in range(40))
        assert dl.get_num_pending_tasks() == 0
    finally:
        dl.shutdown()


def test_failed_task_is_cleaned_and_not_yielded(tmp_path):
    src = _src(tmp_path, 2)
    cache = tmp_path / "cache"
    cache.mkdir()
    dl = ParallelDownloader(num_workers=2, prefetch=4, num_retries=2)
    try:
        dl.schedule_task("ok", [src[0]], [str(cache / "ok.jpg")])
        # the second file of the sample is missing: the first one was copied, then removed on failure
        dl.schedule_task("bad", [src[1], str(tmp_path / "missing.jpg")], [str(cache / "b1.jpg"), str(cache / "b2.jpg")])
        got = dict(dl.yield_completed())
        assert list(got) == ["ok"]
        assert not os.path.exists(cache / "b1.jpg") and not os.path.exists(cache / "b2.jpg")
    finally:
        dl.shutdown()
