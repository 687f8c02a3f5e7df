"""Python handle over the native engine (include/sdsj.h): batched JPEG decode + crop/resize on MI355X.

One engine per (process, device), created lazily on first use -- never in a parent process
before a DataLoader fork (the reference runs transforms inside forked workers,
sds/dataset.py:422-428 / README.md:283).  Outputs are torch tensors allocated by torch's caching
allocator on the current HIP stream; the engine only owns its scratch.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import SdsjCfg, SdsjOp


class ImageDecodeError(OSError):
    """A sample the MI355X path could not decode (PIL raises OSError for such inputs)."""

    def __init__(self, status: int, index: int = 0, msg: str = ""):
        name = _lib.STATUS_NAMES.get(status, str(status))
        super().__init__(msg or f"sample {index}: JPEG decode failed with status {name}")
        self.status = status
        self.index = index


class UnsupportedImageError(ImageDecodeError):
    """A valid image the MI355X JPEG kernels do not decode: a format other than JPEG (PNG, WebP, GIF,
    ... -- everything else in sds/structs.py:42 IMAGE_EXT), or an arithmetic-coded / 12-bit / lossless
    / CMYK JPEG (status UNSUPPORTED).  The transforms (presets.py, batched.py) rerun such samples on
    PIL (functional.py:94-100) instead of raising; the raw engine API reports the status."""


def raise_for_status(status: int, index: int = 0) -> None:
    if status == _lib.OK:
        return
    if status == _lib.UNSUPPORTED:
        raise UnsupportedImageError(status, index)
    raise ImageDecodeError(status, index)


class EncodedBatch:
    """A batch of encoded samples packed back to back in one host uint8 tensor (``data``), with int64
    ``offsets`` / ``lengths`` per sample -- the transport of the batched consumer (sds_amd/batched.py
    ``collate_encoded``).  Built in a DataLoader worker, ``data`` lives in shared memory, so the batch
    crosses to the training process as a file descriptor instead of B pickled ``bytes`` objects, and the
    engine stages it straight from there (no per-sample copies in Python).  Indexing gives one sample's
    bytes (the PIL fallback's input); ``len`` is the sample count."""

    __slots__ = ("data", "offsets", "lengths", "_keep", "__weakref__")

    def __init__(self, data: torch.Tensor, offsets: torch.Tensor, lengths: torch.Tensor, keep=None):
        if data.dtype != torch.uint8 or data.device.type != "cpu" or not data.is_contiguous() or data.dim() != 1:
            raise ValueError("data must be a contiguous 1-D uint8 CPU tensor")
        if offsets.shape != lengths.shape or offsets.dim() != 1:
            raise ValueError("offsets and lengths must be 1-D tensors of one entry per sample")
        off, ln = offsets.numpy(), lengths.numpy()
        if len(off) and (off.min() < 0 or ln.min() < 0 or (off + ln).max() > data.numel()):
            raise ValueError("a sample lies outside data")
        self.data, self.offsets, self.lengths = data, offsets, lengths
        self._keep = keep  # (an object whose lifetime guards ``data``: the batch a selection came from)

    @staticmethod
    def pack(samples: Sequence, shared: bool = False) -> "EncodedBatch":
        """Packs encoded samples (bytes-like); ``shared``: allocate ``data`` in shared memory (what a
        DataLoader worker sends without a copy, as default_collate does for tensors)."""
        lens = np.fromiter((len(s) for s in samples), dtype=np.int64, count=len(samples))
        offs = np.zeros(len(samples), np.int64)
        if len(samples) > 1:
            np.cumsum(lens[:-1], out=offs[1:])
        total = int(lens.sum())
        if shared:
            storage = torch.empty(0, dtype=torch.uint8)._typed_storage()._new_shared(max(total, 1), device="cpu")
            data = torch.empty(0, dtype=torch.uint8).new(storage)[:total]
        else:
            data = torch.empty(total, dtype=torch.uint8)
        buf = data.numpy()
        for s, o, n in zip(samples, offs, lens):
            buf[o:o + n] = np.frombuffer(s, dtype=np.uint8)
        return EncodedBatch(data, torch.from_numpy(offs), torch.from_numpy(lens))

    def __len__(self) -> int:
        return int(self.offsets.numel())

    def __getitem__(self, i: int) -> bytes:
        o, n = int(self.offsets[i]), int(self.lengths[i])
        return self.data.numpy()[o:o + n].tobytes()

    def __iter__(self):
        return (self[i] for i in range(len(self)))

    def select(self, keep: Sequence[int]) -> "EncodedBatch":
        """The kept samples (views into the same ``data``)."""
        k = torch.as_tensor(list(keep), dtype=torch.long)
        return EncodedBatch(self.data, self.offsets[k], self.lengths[k], keep=self)

    def pointers(self):
        """(uint64 sample addresses, uint64 lengths) for the C-ABI's pointer / length arrays; valid while
        ``data`` lives."""
        return (np.uint64(self.data.data_ptr()) + self.offsets.numpy().astype(np.uint64),
                self.lengths.numpy().astype(np.uint64))


def _c_samples(samples):
    """The C-ABI's (const uint8_t* const* jpg, const size_t* len) for a list of bytes or an EncodedBatch;
    the third value keeps the arrays alive."""
    n = len(samples)
    if isinstance(samples, EncodedBatch):
        ptr, ln = samples.pointers()
        ptr, ln = np.ascontiguousarray(ptr), np.ascontiguousarray(ln)
        return (ctypes.cast(ptr.ctypes.data, ctypes.POINTER(ctypes.c_char_p)),
                ctypes.cast(ln.ctypes.data, ctypes.POINTER(ctypes.c_size_t)), (ptr, ln, samples))
    ptrs = (ctypes.c_char_p * max(n, 1))(*samples)
    lens = (ctypes.c_size_t * max(n, 1))(*[len(b) for b in samples])
    return ptrs, lens, None


def _device_index(device) -> int:
    if device is None:
        return torch.cuda.current_device()
    d = torch.device(device)
    if d.type != "cuda":
        raise ValueError(f"the MI355X path needs a cuda (HIP) device, got {d}")
    return d.index if d.index is not None else torch.cuda.current_device()


class JpegEngine:
    """Owns one native ``sdsj_engine`` bound to one HIP device."""

    def __init__(self, device=None, max_batch: int = 4096, scratch_bytes: int = 0):
        if not torch.cuda.is_available():
            raise RuntimeError("sds_amd needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _lib.load()
        self.device = _device_index(device)
        self.max_batch = int(max_batch)
        cfg = SdsjCfg(_lib.SDSJ_ABI_VERSION, self.max_batch, int(scratch_bytes))
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            st = self.lib.sdsj_engine_create(self.device, ctypes.byref(cfg), ctypes.byref(h))
        if st != _lib.OK:
            raise RuntimeError(f"sdsj_engine_create failed: {_lib.STATUS_NAMES.get(st, st)}")
        self._h = h
        self._pid = os.getpid()
        self._inflight: dict[int, tuple[torch.Tensor, int]] = {}
        self._fallback = 0  # samples the transforms decoded with PIL on the host (counters()["fallback"])

    # -- lifetime --------------------------------------------------------------------------
    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value and self._pid == os.getpid():
            self.lib.sdsj_engine_destroy(self._h)
        self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc: int, what: str) -> None:
        if rc != _lib.OK:
            err = self.lib.sdsj_last_error(self._h)
            raise RuntimeError(f"{what} failed ({_lib.STATUS_NAMES.get(rc, rc)}): {err.decode() if err else ''}")

    # -- helpers ---------------------------------------------------------------------------
    @staticmethod
    def make_op(resolution, crop_before_resize=True, filter="bilinear", normalize=False, layout="chw") -> SdsjOp:
        out_h, out_w = (int(v) for v in resolution)
        if filter not in _lib.FILTERS:
            raise NotImplementedError(f"interpolation mode {filter!r} is not implemented on the MI355X path")
        lay = {"chw": _lib.LAYOUT_CHW, "hwc": _lib.LAYOUT_HWC}[layout.lower()]
        return SdsjOp(out_h, out_w, int(bool(crop_before_resize)), _lib.FILTERS[filter],
                      _lib.DTYPE_F32 if normalize else _lib.DTYPE_U8, lay)

    def _out_spec(self, n: int, op: SdsjOp):
        shape = (n, 3, op.out_h, op.out_w) if op.layout == _lib.LAYOUT_CHW else (n, op.out_h, op.out_w, 3)
        return shape, (torch.float32 if op.out_dtype == _lib.DTYPE_F32 else torch.uint8)

    def _alloc_out(self, n: int, op: SdsjOp) -> torch.Tensor:
        shape, dtype = self._out_spec(n, op)
        return torch.empty(shape, dtype=dtype, device=f"cuda:{self.device}")

    def _on_engine(self, t: torch.Tensor) -> bool:
        return t.device.type == "cuda" and (t.device.index if t.device.index is not None else
                                             torch.cuda.current_device()) == self.device

    def _check_out(self, out: torch.Tensor, n: int, op: SdsjOp) -> None:
        """The native side writes n * out_h * out_w * 3 elements of the op's dtype through a raw pointer:
        ``out`` must be exactly what _alloc_out would give (shape, dtype, contiguous, this engine's device),
        or a pinned host tensor of that shape and dtype: pinned host memory is mapped into the device's
        address space, so the kernels store the pixels straight over PCIe (no separate D2H copy)."""
        shape, dtype = self._out_spec(n, op)
        where = isinstance(out, torch.Tensor) and (self._on_engine(out) or (out.device.type == "cpu" and out.is_pinned()))
        if not isinstance(out, torch.Tensor) or tuple(out.shape) != shape or out.dtype != dtype or \
                not out.is_contiguous() or not where:
            raise ValueError(f"out must be a contiguous {dtype} tensor of shape {shape} on cuda:{self.device} (or pinned host memory), got "
                             f"{getattr(out, 'dtype', type(out))} {tuple(getattr(out, 'shape', ()))} on "
                             f"{getattr(out, 'device', '?')}")

    def _check_dev(self, t: torch.Tensor, name: str, dtype, n: Optional[int] = None) -> None:
        if not isinstance(t, torch.Tensor) or t.dtype != dtype or not t.is_contiguous() or not self._on_engine(t):
            raise ValueError(f"{name} must be a contiguous {dtype} tensor on cuda:{self.device}")
        if n is not None and t.numel() < n:
            raise ValueError(f"{name} holds {t.numel()} elements, the batch has {n} samples")

    # -- host-bytes batch ------------------------------------------------------------------
    def decode_resize(self, jpgs: Sequence[bytes], resolution, *, crop_before_resize: bool = True,
                      filter: str = "bilinear", normalize: bool = False, flip: Optional[Sequence[bool]] = None,
                      layout: str = "chw", out: Optional[torch.Tensor] = None) -> tuple[torch.Tensor, np.ndarray]:
        """Decodes host JPEG bytes (a list of bytes, or an EncodedBatch) into a [n, 3, H, W] (or
        [n, H, W, 3]) device tensor.

        Returns (tensor, per-sample status array).  Failed samples are zero-filled; use
        ``raise_for_status`` to turn a status into the reference's OSError semantics.
        """
        op = self.make_op(resolution, crop_before_resize, filter, normalize, layout)
        n = len(jpgs)
        if out is None:
            out = self._alloc_out(n, op)
        else:
            self._check_out(out, n, op)
        if flip is not None and len(flip) != n:
            raise ValueError(f"flip has {len(flip)} entries, the batch has {n} samples")
        status = (ctypes.c_int32 * max(n, 1))()
        if n == 0:
            return out, np.zeros(0, np.int32)
        ptrs, lens, _keep = _c_samples(jpgs)
        flip_arr = None
        if flip is not None:
            flip_arr = (ctypes.c_uint8 * n)(*[1 if f else 0 for f in flip])
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
            rc = self.lib.sdsj_decode_resize_batch(self._h, n, ptrs, lens, ctypes.byref(op),
                                                   ctypes.cast(flip_arr, ctypes.c_void_p) if flip_arr else None,
                                                   ctypes.c_void_p(out.data_ptr()), status, ctypes.c_void_p(stream))
        self._check(rc, "sdsj_decode_resize_batch")
        return out, np.frombuffer(status, dtype=np.int32, count=n).copy()

    # -- asynchronous host path ----------------------------------------
    def submit(self, slot: int, samples: Sequence, resolution, *, files: bool = False, crop_before_resize: bool = True,
               filter: str = "bilinear", normalize: bool = False, flip: Optional[Sequence[bool]] = None,
               layout: str = "chw", out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Stages a batch into pinned slot ``slot`` (0 or 1) and enqueues H2D + decode without waiting.

        ``samples``: encoded bytes (a list, or an EncodedBatch), or file paths with ``files=True`` (read straight into the pinned
        slot, as LoadFromDiskTransform presets.py:613-626 reads the downloader's local cache).  Returns
        the output tensor, valid after ``wait(slot)``; submitting batch k + 1 to the other slot before
        waiting for batch k overlaps its host staging and H2D copy with batch k's decode."""
        op = self.make_op(resolution, crop_before_resize, filter, normalize, layout)
        n = len(samples)
        if n > self.max_batch:
            raise ValueError(f"a slot holds at most max_batch={self.max_batch} samples, got {n}")
        if out is None:
            out = self._alloc_out(n, op)
        else:
            self._check_out(out, n, op)
        if flip is not None and len(flip) != n:
            raise ValueError(f"flip has {len(flip)} entries, the batch has {n} samples")
        if slot not in range(_lib.SLOTS):
            raise ValueError(f"slot must be in [0, {_lib.SLOTS})")
        flip_arr = (ctypes.c_uint8 * max(n, 1))(*[1 if f else 0 for f in flip]) if flip is not None else None
        with torch.cuda.device(self.device):
            stream = ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
            fl = ctypes.cast(flip_arr, ctypes.c_void_p) if flip_arr else None
            if files:
                paths = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(p) for p in samples])
                rc = self.lib.sdsj_submit_files(self._h, slot, n, paths, ctypes.byref(op), fl,
                                                ctypes.c_void_p(out.data_ptr()), stream)
            else:
                ptrs, lens, _keep = _c_samples(samples)  # (staged into the pinned slot before the call returns)
                rc = self.lib.sdsj_submit_batch(self._h, slot, n, ptrs, lens, ctypes.byref(op), fl,
                                                ctypes.c_void_p(out.data_ptr()), stream)
        self._check(rc, "sdsj_submit_files" if files else "sdsj_submit_batch")
        self._inflight[slot] = (out, n)
        return out

    def wait(self, slot: int) -> tuple[torch.Tensor, np.ndarray]:
        """Blocks until the batch in ``slot`` is decoded; returns (output tensor, per-sample status)."""
        if slot not in self._inflight:
            raise RuntimeError(f"no batch in flight on slot {slot}")
        out, n = self._inflight.pop(slot)
        status = (ctypes.c_int32 * max(n, 1))()
        self._check(self.lib.sdsj_wait_batch(self._h, slot, status), "sdsj_wait_batch")
        return out, np.frombuffer(status, dtype=np.int32, count=n).copy()

    def decode_stream(self, batches, resolution, *, files: bool = False, **kw):
        """Yields (out, status) per batch of ``batches`` (each a list of bytes, or of paths with
        ``files=True``), keeping one batch in flight: batch k + 1 is staged and copied while batch k
        decodes (double-buffered pinned slots)."""
        k, prev = 0, None
        for batch in batches:
            slot = k % _lib.SLOTS
            self.submit(slot, batch, resolution, files=files, **kw)
            if prev is not None:
                yield self.wait(prev)
            prev, k = slot, k + 1
        if prev is not None:
            yield self.wait(prev)

    # -- device-resident batch -------------------------------------------------------------
    def decode_resize_device(self, blob: torch.Tensor, offsets: torch.Tensor, lengths: torch.Tensor, resolution, *,
                             crop_before_resize: bool = True, filter: str = "bilinear", normalize: bool = False,
                             flip: Optional[torch.Tensor] = None, layout: str = "chw",
                             out: Optional[torch.Tensor] = None,
                             status: Optional[torch.Tensor] = None) -> tuple[torch.Tensor, torch.Tensor]:
        """Decodes JPEGs already resident in device memory (uint8 ``blob``; int64 ``offsets`` and
        int32 ``lengths`` per sample, both on the device).  Fully asynchronous on the current stream."""
        op = self.make_op(resolution, crop_before_resize, filter, normalize, layout)
        n = int(offsets.numel())
        self._check_dev(blob, "blob", torch.uint8)
        self._check_dev(offsets, "offsets", torch.int64)
        self._check_dev(lengths, "lengths", torch.int32)
        if lengths.numel() != n:
            raise ValueError(f"offsets ({n}) and lengths ({lengths.numel()}) must have one entry per sample")
        if out is None:
            out = self._alloc_out(n, op)
        else:
            self._check_out(out, n, op)
        if status is None:
            status = torch.empty(n, dtype=torch.int32, device=f"cuda:{self.device}")
        else:
            self._check_dev(status, "status", torch.int32, n)
        if flip is not None:
            self._check_dev(flip, "flip", torch.uint8, n)
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
            rc = self.lib.sdsj_decode_resize_batch_device(
                self._h, n, ctypes.c_void_p(blob.data_ptr()), blob.numel(), ctypes.c_void_p(offsets.data_ptr()),
                ctypes.c_void_p(lengths.data_ptr()), ctypes.byref(op),
                ctypes.c_void_p(flip.data_ptr()) if flip is not None else None, ctypes.c_void_p(out.data_ptr()),
                ctypes.c_void_p(status.data_ptr()), ctypes.c_void_p(stream))
        self._check(rc, "sdsj_decode_resize_batch_device")
        return out, status

    # -- raw RGB frames (video) --------------------------------------------------------------
    def resize_frames(self, frames: torch.Tensor, resolution, *, crop_before_resize: bool = True,
                      filter: str = "bilinear", normalize: bool = False, flip: Optional[torch.Tensor] = None,
                      layout: str = "chw", out: Optional[torch.Tensor] = None) -> tuple[torch.Tensor, torch.Tensor]:
        """Crop + resize of uint8 RGB frames [T, H, W, 3] in device memory (lean_resize_frames on PIL
        frames, functional.py:42-86, then the byte-tensor conversion, presets.py:129-135).
        Returns ([T, 3, h, w] (or [T, h, w, 3]) device tensor, device int32 status per frame)."""
        if frames.dim() != 4 or frames.shape[-1] != 3 or frames.dtype != torch.uint8 or frames.device.type != "cuda":
            raise ValueError("frames must be a cuda uint8 tensor [T, H, W, 3]")
        frames = frames.contiguous()
        op = self.make_op(resolution, crop_before_resize, filter, normalize, layout)
        if not self._on_engine(frames):
            raise ValueError(f"frames must live on cuda:{self.device}")
        t, h, w = int(frames.shape[0]), int(frames.shape[1]), int(frames.shape[2])
        if out is None:
            out = self._alloc_out(t, op)
        else:
            self._check_out(out, t, op)
        status = torch.empty(t, dtype=torch.int32, device=f"cuda:{self.device}")
        if flip is not None:
            flip = torch.as_tensor(flip, dtype=torch.uint8, device=f"cuda:{self.device}").contiguous()
            if flip.numel() != t:
                raise ValueError(f"flip has {flip.numel()} entries, there are {t} frames")
        if t == 0:
            return out, status
        with torch.cuda.device(self.device):
            stream = torch.cuda.current_stream(self.device).cuda_stream
            rc = self.lib.sdsj_resize_frames_device(
                self._h, t, ctypes.c_void_p(frames.data_ptr()), w, h, h * w * 3, ctypes.byref(op),
                ctypes.c_void_p(flip.data_ptr()) if flip is not None else None, ctypes.c_void_p(out.data_ptr()),
                ctypes.c_void_p(status.data_ptr()), ctypes.c_void_p(stream))
        self._check(rc, "sdsj_resize_frames_device")
        return out, status

    # -- metrics / control -------------------------------------------------------------------
    def counters(self, reset: bool = False) -> dict[str, int]:
        """Per-process counters of everything this engine decoded: samples by status,
        encoded bytes in, output bytes out.  Waits for the device."""
        buf = (ctypes.c_uint64 * _lib.NUM_COUNTERS)()
        self._check(self.lib.sdsj_engine_counters(self._h, buf, _lib.NUM_COUNTERS, int(bool(reset))),
                    "sdsj_engine_counters")
        out = {self.lib.sdsj_counter_name(k).decode(): int(buf[k]) for k in range(_lib.NUM_COUNTERS)}
        out["fallback"] = self._fallback
        if reset:
            self._fallback = 0
        return out

    def note_fallback(self, n: int = 1) -> None:
        """Counts samples decoded by PIL on the host and resized by this engine (the transforms' rerun of
        UNSUPPORTED / CORRUPT samples)."""
        self._fallback += int(n)

    def set_lanes(self, lanes: int) -> None:
        """Kernel lanes per batch (1..4; see include/sdsj.h)."""
        self._check(self.lib.sdsj_engine_set_lanes(self._h, int(lanes)), "sdsj_engine_set_lanes")

    @staticmethod
    def scratch_need(jpgs: Sequence[bytes], resolution, *, crop_before_resize: bool = True, filter: str = "bilinear",
                     normalize: bool = False, layout: str = "chw") -> int:
        """Device scratch bytes a batch of these JPEGs needs (host planning, sdsj_plan_need): what
        ``reserve`` must provide before ``decode_resize_device`` decodes them in one call."""
        op = JpegEngine.make_op(resolution, crop_before_resize, filter, normalize, layout)
        lib, tot, need = _lib.load(), 0, ctypes.c_int64()
        for j in jpgs:
            lib.sdsj_plan_need(j, len(j), ctypes.byref(op), ctypes.byref(need))
            tot += need.value
        return tot

    def reserve(self, nbytes: int) -> None:
        """Grows the device scratch (the device-resident entry point never grows it by itself)."""
        self._check(self.lib.sdsj_engine_reserve(self._h, int(nbytes)), "sdsj_engine_reserve")

    # -- diagnostics -----------------------------------------------------------------------
    def set_timing(self, enable: bool) -> None:
        self.lib.sdsj_engine_set_timing(self._h, int(bool(enable)))

    def stage_times(self) -> dict[str, float]:
        ms = (ctypes.c_float * 16)()
        n = ctypes.c_int()
        self._check(self.lib.sdsj_engine_stage_times(self._h, ms, 16, ctypes.byref(n)), "sdsj_engine_stage_times")
        return {self.lib.sdsj_stage_name(k).decode(): float(ms[k]) for k in range(n.value)}


_engines: dict[tuple[int, int], JpegEngine] = {}
_engines_lock = threading.Lock()


def get_engine(device=None) -> JpegEngine:
    """The per-(process, device) engine, created on first use (fork-safe: keyed by pid)."""
    idx = _device_index(device)
    key = (os.getpid(), idx)
    eng = _engines.get(key)
    if eng is None:
        with _engines_lock:
            eng = _engines.get(key)
            if eng is None:
                eng = JpegEngine(idx)
                _engines[key] = eng
    return eng
