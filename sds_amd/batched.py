"""Batched GPU decode on the consumer side of the DataLoader.

The per-sample drop-in (``presets.create_standard_image_pipeline``) decodes inside whichever
process iterates the dataset -- for sds that is a DataLoader worker (sds/dataset.py:352-381
``_iter_chunks_``), so every worker holds its own HIP context and each call decodes one image.
The batched path keeps the workers CPU-only and decodes a whole collated batch in one engine call
on the training process's GPU:

    ds = StreamingDataset(..., transforms=create_deferred_image_pipeline("jpg"))   # bytes only
    loader = torch.utils.data.DataLoader(ds, batch_size=B, num_workers=W)            # default collate
    decode = GpuDecodeBatch("jpg", (256, 256), device="cuda")
    for batch in loader:              # or MultiStreamDataLoader's Batch (sds/dataloader.py:49-58)
        batch = decode(batch)         # batch["image"]: [B', 3, 256, 256] on the GPU
    for batch in decode.stream(loader):   # the same, batch k + 1 staged and copied while k decodes
        ...

torch's default collate leaves ``bytes`` fields as a list of B ``bytes``, which a DataLoader pickles
through its result queue (a pipe), and the consumer copies each again.  ``collate_encoded``
packs the image field into an ``EncodedBatch`` instead (one shared-memory uint8 tensor of the samples'
bytes back to back + offsets / lengths), which crosses to the training process as a file descriptor,
and the engine stages it from there:

    loader = DataLoader(ds, batch_size=B, num_workers=W, collate_fn=collate_encoded("jpg"))

torch's default collate leaves ``bytes`` fields as a list, so ``batch[image_field]`` arrives as the
B encoded images.  Values equal the per-sample pipeline's (presets.py:716-744) stacked the way
default_collate stacks them.  Samples the JPEG kernels do not decode (other formats, CMYK / arithmetic
/ 12-bit JPEG, streams reported damaged) rerun on PIL on the host (functional.py:94-100) and are
resized on the GPU into their row of the batch.  A sample the reference would have failed on (PIL's
OSError makes ``_iter_chunks_`` skip it, dataset.py:366-371) is dropped from every field of the batch
(``on_error="drop"``), or its exception is raised (``"raise"``).
"""
from __future__ import annotations

import os
import time
import weakref
from typing import Any, Iterable, Iterator, Optional, Sequence

import numpy as np
import torch

from . import _lib
from . import functional as F
from .engine import EncodedBatch, ImageDecodeError, UnsupportedImageError, get_engine, raise_for_status
from .presets import LoadFromDiskTransform, SampleTransform, _frames_to_device, pil_decode


def create_deferred_image_pipeline(image_field: str) -> Sequence[SampleTransform]:
    """The CPU half of create_standard_image_pipeline (presets.py:716-744) for batched GPU decode:
    ``LoadFromDiskTransform`` only (presets.py:613-626), so ``sample[image_field]`` holds the encoded
    bytes when the sample reaches the collate function."""
    return [LoadFromDiskTransform([image_field])]


# -- the workers' slot rings (collate_encoded) ---------------------------------------------------------
# A fresh shared-memory tensor per batch costs both processes a page fault per 4 KiB of it and the
# training process an unmap per batch -- on one MI355X box that was about half of the consumer's time per
# 256-image batch (tools/batched_bench.py phases, profiles/r06_f1_*).  So each worker keeps a ring of
# `slots` shared-memory slots, sent to the training process once with its first batch; a batch then
# travels as (worker, slot, offsets, lengths), and its EncodedBatch views the slot.  A slot is busy from
# the worker's write until the training process drops the EncodedBatch (and every selection of it):
# a weakref finalizer clears its flag in the ring's header, which the worker polls.  When no slot is
# free within `wait_s` (a consumer holding many batches), or the batch outgrows a slot, the worker falls
# back to a one-off shared-memory tensor, so nothing can deadlock.
_RING_HDR = 64  # bytes per slot flag (one cache line each)
_rings: dict = {}  # training process: ring serial (worker pid, n) -> ring tensor
_ring_serial = [0]


class _WorkerRing:
    def __init__(self, slots: int, slot_bytes: int):
        self.slots, self.slot_bytes = slots, slot_bytes
        self.tensor = torch.empty(_RING_HDR * slots + slots * slot_bytes, dtype=torch.uint8).share_memory_()
        self.flags = self.tensor[:_RING_HDR * slots].numpy().view(np.int32)[::_RING_HDR // 4]
        self.flags[:] = 0
        _ring_serial[0] += 1
        self.serial = (os.getpid(), _ring_serial[0])
        self.sent = False
        self.next = 0
        self.starved = False  # the last claim found every slot held: do not wait again until one frees

    def claim(self, wait_s: float):
        t0 = None
        if self.starved:
            wait_s = 0.0
        while True:
            for i in range(self.slots):
                s = (self.next + i) % self.slots
                if self.flags[s] == 0:
                    self.flags[s] = 1
                    self.next = s + 1
                    self.starved = False
                    return s
            t0 = t0 if t0 is not None else time.perf_counter()
            if time.perf_counter() - t0 >= wait_s:
                self.starved = True  # (a consumer holding its batches: fall back without waiting each time)
                return None
            time.sleep(0.0002)

    def data_off(self, slot: int) -> int:
        return _RING_HDR * self.slots + slot * self.slot_bytes


def _release_slot(ring: torch.Tensor, slots: int, slot: int) -> None:
    ring[:_RING_HDR * slots].numpy().view(np.int32)[slot * (_RING_HDR // 4)] = 0


def _pid_alive(pid: int) -> bool:
    try:
        os.kill(pid, 0)
        return True
    except ProcessLookupError:
        return False
    except PermissionError:
        return True


def _rebuild_ring_batch(serial, ring, slots, slot, off, total, offs, lens) -> EncodedBatch:
    """Training process side of a ring batch: the ring arrives with the worker's first batch (torch shares
    its storage), later batches look it up.  Rings of workers that have exited are dropped from the
    registry (their live batches keep their own reference)."""
    if ring is not None:
        for k in [k for k in _rings if not _pid_alive(k[0])]:
            del _rings[k]
        _rings[serial] = ring
    ring = _rings.get(serial)
    if ring is None:  # (cannot happen: a worker's batches arrive in order, its ring first)
        raise RuntimeError("encoded batch from an unknown slot ring")
    eb = EncodedBatch(ring[off:off + total], torch.from_numpy(np.frombuffer(offs, np.int64).copy()),
                      torch.from_numpy(np.frombuffer(lens, np.int64).copy()))
    weakref.finalize(eb, _release_slot, ring, slots, slot)
    return eb


class _RingBatch(EncodedBatch):
    """Worker side: an EncodedBatch in a ring slot, pickled as its ring coordinates."""

    __slots__ = ("_ring", "_slot")

    def __reduce__(self):
        r = self._ring
        ring = None if r.sent else r.tensor
        r.sent = True
        off = r.data_off(self._slot)
        return (_rebuild_ring_batch, (r.serial, ring, r.slots, self._slot, off, int(self.data.numel()),
                                      self.offsets.numpy().tobytes(), self.lengths.numpy().tobytes()))


class collate_encoded:
    """A DataLoader ``collate_fn`` for the batched consumer: ``image_field`` (the encoded bytes that
    create_deferred_image_pipeline leaves) becomes an ``EncodedBatch``; every other field goes through
    ``collate_fn`` (default_collate).  In a worker the bytes go into the worker's ring of shared-memory
    slots (above; ``slots`` per worker, each sized for 1.5x the worker's first batch); in the main process
    into a private tensor.  Picklable, so spawn-started workers can run it."""

    def __init__(self, image_field: str, collate_fn=None, slots: int = 8, wait_s: float = 0.05):
        self.image_field = image_field
        self.collate_fn = collate_fn
        self.slots = int(slots)
        self.wait_s = float(wait_s)
        self._ring = None  # (per worker process, created on its first batch)

    def __getstate__(self):
        d = dict(self.__dict__)
        d["_ring"] = None
        return d

    def _pack(self, items: list) -> EncodedBatch:
        from torch.utils.data import get_worker_info
        wi = get_worker_info()
        if wi is None or self.slots <= 0:
            return EncodedBatch.pack(items, shared=wi is not None)
        total = sum(len(b) for b in items)
        if self._ring is None:
            self._ring = _WorkerRing(self.slots, max(1 << 20, (total * 3 // 2 + 4095) // 4096 * 4096))
        r = self._ring
        slot = r.claim(self.wait_s) if total <= r.slot_bytes else None
        if slot is None:
            return EncodedBatch.pack(items, shared=True)
        off = r.data_off(slot)
        data = r.tensor[off:off + total]
        lens = np.fromiter((len(b) for b in items), dtype=np.int64, count=len(items))
        offs = np.zeros(len(items), np.int64)
        if len(items) > 1:
            np.cumsum(lens[:-1], out=offs[1:])
        buf = data.numpy()
        for b, o, n in zip(items, offs, lens):
            buf[o:o + n] = np.frombuffer(b, dtype=np.uint8)
        eb = _RingBatch(data, torch.from_numpy(offs), torch.from_numpy(lens))
        eb._ring, eb._slot = r, slot
        return eb

    def __call__(self, samples: Sequence[dict]) -> dict:
        from torch.utils.data import default_collate
        rest = [{k: v for k, v in s.items() if k != self.image_field} for s in samples]
        out = (self.collate_fn or default_collate)(rest)
        enc = self._pack([s[self.image_field] for s in samples])
        # (the image field keeps its place among the sample's keys)
        keys = list(samples[0].keys()) if samples else []
        return {k: (enc if k == self.image_field else out[k]) for k in keys}


def _select(value: Any, keep: list[int], n: int) -> Any:
    """The kept rows of one collated field (tensors along dim 0, lists/tuples by index)."""
    if isinstance(value, EncodedBatch) and len(value) == n:
        return value.select(keep)
    if isinstance(value, torch.Tensor) and value.ndim > 0 and value.shape[0] == n:
        return value[torch.as_tensor(keep, dtype=torch.long, device=value.device)]
    if isinstance(value, list) and len(value) == n:
        return [value[i] for i in keep]
    if isinstance(value, tuple) and len(value) == n:
        return tuple(value[i] for i in keep)
    if isinstance(value, dict):
        return {k: _select(v, keep, n) for k, v in value.items()}
    return value


class GpuDecodeBatch:
    """Decodes ``batch[image_field]`` (a list of encoded images) into ``batch[output_field]`` =
    ``[B, 3, H, W]`` on the GPU: uint8, or float32 ``x/127.5-1`` with ``normalize`` (presets.py:154-162).

    ``resize_kwargs`` follow lean_resize_frames (functional.py:42-50) for a fixed target:
    ``crop_before_resize`` and ``interpolation_mode``.  Per-sample target sizes (``random_resize``,
    ``allow_vertical``) cannot be stacked into one tensor and are rejected, as default_collate
    rejects the reference's differently sized tensors.  ``hflip_prob`` draws one
    ``torch.rand(1) < p`` coin per sample in batch order (README.md:99-108 HorizontalFlipTransform).
    ``return_image_as_single_frame_video`` mirrors presets.py:737-742 on the batch: ``video`` =
    ``[B, 1, 3, H, W]``, ``image`` removed, ``framerate`` = 960.0 per sample (float64, as
    default_collate stacks Python floats).
    """

    def __init__(self, image_field: str, resolution, output_field: str = "image", normalize: bool = False,
                 resize_kwargs: Optional[dict] = None, device=None, hflip_prob: float = 0.0,
                 on_error: str = "drop", return_image_as_single_frame_video: bool = False,
                 video_output_field: str = "video"):
        self.image_field = image_field
        self.output_field = output_field
        self.resolution = tuple(int(v) for v in resolution)
        assert len(self.resolution) == 2, f"Wrong resolution: {resolution}"
        self.normalize = bool(normalize)
        self.resize_kwargs = dict(resize_kwargs or {})
        F.check_resize_kwargs(self.resize_kwargs)
        if self.resize_kwargs.get("allow_vertical") or self.resize_kwargs.get("random_resize") is not None:
            raise ValueError("per-sample target sizes cannot be stacked into one batch; use the per-sample pipeline")
        if on_error not in ("drop", "raise"):
            raise ValueError(f"on_error must be 'drop' or 'raise', got {on_error!r}")
        self.on_error = on_error
        self.device = device
        self.hflip_prob = float(hflip_prob)
        self.as_video = bool(return_image_as_single_frame_video)
        self.video_output_field = video_output_field

    def _inputs(self, batch: dict):
        """The batch's encoded images and their hflip coins (one torch.rand(1) per sample, batch order)."""
        assert self.image_field in batch, f"Field '{self.image_field}' not found in batch with keys {list(batch.keys())}."
        encoded = batch[self.image_field]
        if isinstance(encoded, (bytes, bytearray, memoryview)):
            encoded = [encoded]
        if not isinstance(encoded, EncodedBatch):  # (an EncodedBatch goes to the engine as it is)
            encoded = [bytes(e) for e in encoded]
        flip = [bool(torch.rand(1) < self.hflip_prob) for _ in encoded] if self.hflip_prob > 0.0 else None
        return encoded, flip

    def _opts(self) -> dict:
        kw = self.resize_kwargs
        return dict(crop_before_resize=kw.get("crop_before_resize", True),
                    filter=F.filter_name(kw.get("interpolation_mode", "bilinear")), normalize=self.normalize)

    def __call__(self, batch: dict) -> dict:
        encoded, flip = self._inputs(batch)
        eng = get_engine(self.device)
        images, status = eng.decode_resize(encoded, self.resolution, flip=flip, **self._opts())
        return self._finish(eng, batch, encoded, flip, images, status)

    def stream(self, batches: Iterable[dict]) -> Iterator[dict]:
        """Yields ``self(batch)`` for each collated batch, with one batch in flight: batch k + 1's host
        staging, H2D copy and decode are queued (engine.submit, double-buffered pinned slots) before
        batch k is collected (engine.wait), so the copy and the host work of one batch overlap the
        other's decode.  Values and RNG draws equal the synchronous calls'; a batch larger than the
        engine's max_batch is decoded synchronously in its turn.

            for batch in GpuDecodeBatch("jpg", (256, 256), device="cuda").stream(loader): ...
        """
        eng = get_engine(self.device)
        cap = getattr(eng, "max_batch", None)
        pending = None  # (slot, batch, encoded, flip) of the batch in flight
        k = 0
        try:
            for batch in batches:
                encoded, flip = self._inputs(batch)
                if cap is not None and len(encoded) > cap:
                    if pending is not None:
                        prev, pending = pending, None
                        yield self._collect(eng, prev)
                    images, status = eng.decode_resize(encoded, self.resolution, flip=flip, **self._opts())
                    yield self._finish(eng, batch, encoded, flip, images, status)
                    continue
                slot = k % _lib.SLOTS
                k += 1
                eng.submit(slot, encoded, self.resolution, flip=flip, **self._opts())
                prev, pending = pending, (slot, batch, encoded, flip)
                batch = encoded = None  # (the consumer's reference is then the batch's last one)
                if prev is not None:
                    out, prev = self._collect(eng, prev), None
                    yield out
                    out = None
            if pending is not None:
                prev, pending = pending, None
                yield self._collect(eng, prev)
        finally:
            if pending is not None:  # (the consumer stopped early, or a batch raised): drain the slot
                eng.wait(pending[0])

    def _collect(self, eng, inflight) -> dict:
        slot, batch, encoded, flip = inflight
        images, status = eng.wait(slot)
        return self._finish(eng, batch, encoded, flip, images, status)

    def _finish(self, eng, batch: dict, encoded: list, flip, images: torch.Tensor, status) -> dict:
        """Host decode of the samples the kernels do not take, then the drop / raise rule and the
        output fields."""
        n = len(encoded)
        opts = self._opts()
        errors: dict[int, BaseException] = {}
        for i in range(n):
            st = int(status[i])
            if st in (_lib.UNSUPPORTED, _lib.CORRUPT):  # rerun on the reference's PIL decode
                try:
                    pil = pil_decode(encoded[i])
                except Exception as e:  # noqa: BLE001 -- what PIL raises is what the reference raises
                    errors[i] = e
                    continue
                frames = _frames_to_device([pil], images.device)
                img, fst = eng.resize_frames(frames, self.resolution, flip=None if flip is None else [flip[i]], **opts)
                raise_for_status(int(fst[0].item()), i)
                images[i].copy_(img[0])
                eng.note_fallback()
                status[i] = _lib.OK
            elif st != _lib.OK:
                errors[i] = ImageDecodeError(st, i)
        keep = [i for i in range(n) if i not in errors]
        if len(keep) < n:
            if self.on_error == "raise":
                raise errors[min(errors)]
            batch = {k: _select(v, keep, n) for k, v in batch.items()}
            images = images[torch.as_tensor(keep, dtype=torch.long, device=images.device)]
        if self.as_video:
            batch.pop(self.output_field, None)
            batch[self.video_output_field] = images.unsqueeze(1)
            batch["framerate"] = torch.full((images.shape[0],), 960.0, dtype=torch.float64)
        else:
            batch[self.output_field] = images
        return batch


__all__ = ["GpuDecodeBatch", "create_deferred_image_pipeline", "collate_encoded", "EncodedBatch", "ImageDecodeError",
           "UnsupportedImageError"]
