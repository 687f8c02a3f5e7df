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

from typing import Any, Iterable, Iterator, Optional, Sequence

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


class collate_encoded:
    """A DataLoader ``collate_fn`` for the batched consumer: ``image_field`` (the encoded bytes that
    create_deferred_image_pipeline leaves) becomes an ``EncodedBatch`` -- in shared memory when collated in
    a worker, as default_collate allocates its tensors there --, every other field goes through
    ``collate_fn`` (default_collate).  Picklable, so spawn-started workers can run it."""

    def __init__(self, image_field: str, collate_fn=None):
        self.image_field = image_field
        self.collate_fn = collate_fn

    def __call__(self, samples: Sequence[dict]) -> dict:
        from torch.utils.data import default_collate, get_worker_info
        rest = [{k: v for k, v in s.items() if k != self.image_field} for s in samples]
        out = (self.collate_fn or default_collate)(rest)
        enc = EncodedBatch.pack([s[self.image_field] for s in samples], shared=get_worker_info() is not None)
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
