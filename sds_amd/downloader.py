"""The local leg of sds's downloader, restated for configs[4] (files -> host cache -> H2D -> decode).

BASELINE configs[4] is "sds/downloader.py -> host cache -> H2D -> decode+resize@512 -> D2H".  For a
local source (`file://` or a plain path) sds copies each sample's file into its cache directory
through this chain, which this module restates with the same names and semantics so the bench can
time it ahead of the decode:

* ``ParallelDownloader`` -- /root/reference/sds/downloader.py:25-115: a lazy thread pool of
  ``num_workers`` threads, at most ``prefetch`` completed tasks waiting to be consumed
  (lazy_thread_pool.py:85-100: the completed queue is bounded), ``num_retries`` retries per task,
  ``skip_if_exists``; ``yield_completed`` yields ``(key, (total bytes, downloaded bytes))`` in completion
  order (downloader.py:101-108, lazy_thread_pool.py:155-170) and removes the destinations of a task that
  failed all its retries (downloader.py:88-99).
* ``run_downloading_task`` -- downloader.py:117-131: per (url, destination) pair, a destination that
  exists with a non-zero size is skipped when ``skip_if_exists`` (the warm cache), otherwise the file is
  downloaded; returns (total size, downloaded size).
* ``LocalDownloader.download`` -- utils/download.py:830-861 ``_download_file_impl``: remove a stale
  ``<dst>.tmp``, copy the source to ``<dst>.tmp``, rename it to ``<dst>`` (readers never see a partial file).

Only the local scheme is restated: S3 / GCS / HTTP clients are out of scope, and a url of
another scheme raises ``ValueError``.
"""
from __future__ import annotations

import os
import queue
import shutil
import threading
import urllib.parse
from dataclasses import dataclass
from typing import Iterator


class LocalDownloader:
    """utils/download.py:830-861: local filesystem -> local filesystem, through a ``.tmp`` file."""

    @staticmethod
    def _path(url: str) -> str:
        if "://" not in url and not url.startswith("file:"):  # a plain local path (no scheme to resolve)
            return url
        u = urllib.parse.urlparse(url)
        if u.scheme not in ("", "file"):
            raise ValueError(f"only local sources are restated here, got scheme {u.scheme!r} ({url})")
        return u.path if u.scheme == "file" else url

    def download(self, url: str, local: str, timeout: float = 10.0) -> None:
        local_tmp = local + ".tmp"
        if os.path.exists(local_tmp):
            os.remove(local_tmp)
        shutil.copy(self._path(url), local_tmp)
        os.rename(local_tmp, local)


@dataclass
class DownloadingTask:
    """downloader.py:13-21."""
    key: object
    source_urls: list
    destinations: list
    timeout: int
    downloader: LocalDownloader
    skip_if_exists: bool


def run_downloading_task(task: DownloadingTask) -> tuple[int, int]:
    """downloader.py:117-131: (total size of the sample's files, bytes actually copied)."""
    existing, downloaded = 0, 0
    for url, dst in zip(task.source_urls, task.destinations):
        try:  # (os.path.exists + getsize as one stat)
            cur = os.stat(dst).st_size
        except FileNotFoundError:
            cur = 0
        if task.skip_if_exists and cur > 0:
            existing += cur
            continue
        task.downloader.download(url, dst, timeout=task.timeout)
        downloaded += os.path.getsize(dst)
    return existing + downloaded, downloaded


class ParallelDownloader:
    """downloader.py:25-115 over a restated LazyThreadPool (lazy_thread_pool.py:10-170)."""

    def __init__(self, num_workers: int = 4, prefetch: int = 10, num_retries: int = 3, skip_if_exists: bool = True):
        self.num_workers = num_workers
        self.prefetch = prefetch
        self.num_retries = num_retries
        self.skip_if_exists = skip_if_exists
        self.downloader = LocalDownloader()
        self._tasks: queue.Queue = queue.Queue()
        self._done: queue.Queue = queue.Queue(maxsize=prefetch)
        self._stop = threading.Event()
        self._threads: list[threading.Thread] = []
        self.num_scheduled = 0
        self.num_yielded = 0

    def _worker(self) -> None:
        # lazy_thread_pool.py:31-66: take a task, run it with retries, put the result (blocks while
        # `prefetch` results wait to be consumed)
        while not self._stop.is_set():
            try:
                task, retries = self._tasks.get(timeout=0.1)
            except queue.Empty:
                continue
            result = {"task_input": task, "task_output": None, "success": True, "error": None}
            while True:
                try:
                    result["task_output"] = run_downloading_task(task)
                    break
                except Exception as e:  # noqa: BLE001  (the reference retries on any error)
                    if retries > 0:
                        retries -= 1
                        continue
                    result["success"], result["error"] = False, repr(e)
                    break
            while not self._stop.is_set():
                try:
                    self._done.put(result, timeout=0.1)
                    break
                except queue.Full:
                    continue
            self._tasks.task_done()

    def _start(self) -> None:
        if not self._threads:
            self._threads = [threading.Thread(target=self._worker, daemon=True) for _ in range(self.num_workers)]
            for t in self._threads:
                t.start()

    def schedule_task(self, key, source_urls: list, destinations: list, blocking: bool = False):
        """downloader.py:52-75."""
        task = DownloadingTask(key, list(source_urls), list(destinations), 10, self.downloader, self.skip_if_exists)
        for url in task.source_urls:
            LocalDownloader._path(url)  # (the reference resolves the scheme's downloader at scheduling time)
        if blocking:
            return run_downloading_task(task)
        self._start()
        self._tasks.put((task, self.num_retries))
        self.num_scheduled += 1
        return None

    def _clean_failed_download(self, task: DownloadingTask) -> None:
        for dst in task.destinations:
            if os.path.exists(dst):
                try:
                    os.remove(dst)
                except OSError:
                    pass

    def yield_completed(self) -> Iterator[tuple[object, tuple[int, int]]]:
        """downloader.py:101-108: completed tasks in completion order until every scheduled one is seen;
        failed ones are cleaned up and not yielded."""
        while self.num_yielded < self.num_scheduled:
            r = self._done.get()
            self.num_yielded += 1
            if r["success"]:
                yield r["task_input"].key, r["task_output"]
            else:
                self._clean_failed_download(r["task_input"])

    def get_num_pending_tasks(self) -> int:
        return self._tasks.qsize()

    def shutdown(self, timeout: float = 1.0) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(timeout=timeout)
        self._threads = []
