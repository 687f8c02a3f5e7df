"""Drop-in image transform pipeline for sds.dataset.StreamingDataset, decoding on MI355X.

Mirrors the reference's transform-callable API (sds/structs.py:68-69: ``Callable[[dict], dict]``)
and its pipeline factory ``create_standard_image_pipeline`` (sds/transforms/presets.py:716-744):
same signature (plus a keyword-only ``device``), same sample-dict routing (key set, order and
values), but the decode/crop/resize/to-tensor/normalise steps run as one fused GPU transform that
leaves a device tensor in ``sample[output_field]``.

Transforms are plain picklable classes (presets.py:1-5): the native engine is created lazily in
the process that first calls them (a DataLoader worker after fork), never pickled.

Samples the MI355X JPEG path does not decode (other IMAGE_EXT formats, sds/structs.py:42; arithmetic /
12-bit / lossless / CMYK JPEG; streams it reports damaged) rerun on the reference's own PIL decode on the
host and are then cropped / resized on the GPU; PIL's exceptions propagate unchanged,
so sds's skip / retry handling (dataset.py:212-226, :366-371) sees what the reference raises.
"""
from __future__ import annotations

import io
import logging
import os
from typing import Any, Callable, Optional, Sequence

import numpy as np
import torch

from . import _lib
from . import functional as F
from . import service as _service
from .engine import ImageDecodeError, JpegEngine, get_engine, raise_for_status

log = logging.getLogger("sds_amd")
_fallback_seen = {"pid": None, "n": 0}


def _note_fallback(data: bytes, field: str) -> None:
    """Logs (first time per process, then every 1,000th) a sample decoded on the host."""
    if _fallback_seen["pid"] != os.getpid():
        _fallback_seen.update(pid=os.getpid(), n=0)
    _fallback_seen["n"] += 1
    n = _fallback_seen["n"]
    if n == 1 or n % 1000 == 0:
        log.info("sds_amd: field %r holds a %s image, decoded by PIL on the host and resized on the GPU "
                 "(%d such samples in this process so far)", field, F.sniff_format(data), n)


def pil_decode(data: bytes):
    """functional.py:94-100 load_image_from_bytes: ``Image.open(...).convert('RGB')`` -- the reference's
    own decode, run on the host for the samples the MI355X JPEG path does not decode (other formats,
    arithmetic / 12-bit / lossless / CMYK JPEG, streams it reports damaged).  Raises what PIL raises."""
    from PIL import Image
    return Image.open(io.BytesIO(data)).convert("RGB")


class _RngSnapshot:
    """The global RNG states a transform may draw from (np for random_resize, torch for the hflip
    coin), so that a sample whose GPU decode must be redone on the host draws in the reference's order:
    the reference draws only after its decode succeeded (functional.py:69-74, README.md:99-108)."""

    def __init__(self, np_rng: bool, torch_rng: bool):
        self.np_state = np.random.get_state() if np_rng else None
        self.torch_state = torch.get_rng_state() if torch_rng else None

    def restore(self) -> None:
        if self.np_state is not None:
            np.random.set_state(self.np_state)
        if self.torch_state is not None:
            torch.set_rng_state(self.torch_state)


def _engine_in_worker(device):
    """get_engine with a clear error for the one DataLoader set-up that cannot work: a worker forked
    after the parent process initialised HIP (the child cannot re-initialise it)."""
    try:
        return get_engine(device)
    except RuntimeError as e:
        if "forked subprocess" not in str(e):
            raise
        raise RuntimeError(
            "GpuDecodeResizeImageTransform runs in a DataLoader worker that was forked after the parent "
            "process initialised the GPU (any GPU call, and DataLoader(pin_memory=True) itself, which queries "
            "the GPU before forking its workers), and HIP cannot be re-initialised in a forked child. Pass "
            "multiprocessing_context='spawn' to the DataLoader (with pin_memory=True also output_device='cpu'), "
            "use pin_memory=False, persistent_workers=True and no GPU call in the parent before the workers "
            "start (device tensors received from the workers initialise HIP in the parent), or keep the workers on "
            "bytes and decode each collated batch in the main process with sds_amd.batched.GpuDecodeBatch "
            "(INTEGRATION.md §1).") from e

def _service_address(service, device) -> Optional[str]:
    """The decode-service address a transform's worker processes use (GpuDecodeResizeImageTransform's
    ``service``).  "auto" starts the service only where a GPU exists; counting devices does not
    initialise HIP in this process."""
    if service is None or service is False:
        return None
    if isinstance(service, str) and service != "auto":
        return service
    if torch.cuda.device_count() == 0:
        return None
    d = torch.device(device) if device is not None else None
    if d is not None and d.type != "cuda":
        return None
    idx = d.index if d is not None and d.index is not None else int(os.environ.get("LOCAL_RANK", 0))
    return _service.ensure_service(idx)


SampleData = dict  # sds/structs.py:68
SampleTransform = Callable[[SampleData], Any]  # sds/structs.py:69


# ------------------------------------------------------------------------------------------
# Field validation / routing helpers (presets.py:393-415, :906-917), restated.
# ------------------------------------------------------------------------------------------
def is_dummy_field(d: dict, field: str, return_reason: bool = False):
    """presets.py:393-415: absent, None, empty str/list/dict, float NaN or a tensor with NaN."""
    is_dummy, reason = False, ""
    if field not in d:
        is_dummy, reason = True, f"Field '{field}' is absent."
    elif d[field] is None:
        is_dummy, reason = True, f"Field '{field}' is None."
    elif isinstance(d[field], str) and d[field] == "":
        is_dummy, reason = True, f"Field '{field}' is an empty string."
    elif isinstance(d[field], (list, dict)) and len(d[field]) == 0:
        is_dummy, reason = True, f"Field '{field}' is an empty {type(d[field]).__name__}."
    elif isinstance(d[field], float) and np.isnan(d[field]):
        is_dummy, reason = True, f"Field '{field}' is float and NaN."
    elif isinstance(d[field], torch.Tensor) and torch.isnan(d[field]).any():
        is_dummy, reason = True, f"Field '{field}' is a torch.Tensor and contains NaN values."
    return (is_dummy, reason) if return_reason else is_dummy


def _validate_fields(sample: SampleData, present, absent: Sequence[str], check_dummy_values: bool = False) -> None:
    """presets.py:906-917."""
    for field in present:
        assert field in sample, f"Field '{field}' not found in sample with keys {list(sample.keys())}."
        if check_dummy_values:
            is_dummy, reason = is_dummy_field(sample, field, return_reason=True)
            assert not is_dummy, f"Field '{field}' is dummy: {reason} Sample keys: {list(sample.keys())}."
        if isinstance(present, dict) and present[field] is not None:
            assert isinstance(sample[field], present[field]), \
                f"Field '{field}' should be of type {present[field]}, but got {type(sample[field])}."
    for field in absent:
        assert field not in sample, f"Field '{field}' should not be present in sample with keys {list(sample.keys())}."


class BaseTransform:
    """presets.py:26-34."""

    def __init__(self, input_field: str, output_field: Optional[str] = None, **transform_kwargs):
        self.input_field = input_field
        self.output_field = output_field if output_field is not None else input_field
        self.transform_kwargs = transform_kwargs

    def __call__(self, sample: SampleData) -> SampleData:
        raise NotImplementedError


class LoadFromDiskTransform:
    """presets.py:613-626: replaces each path field by the file's bytes, in place."""

    def __init__(self, fields_to_load: Sequence[str], mode: str = "rb"):
        assert len(fields_to_load) > 0, "At least one field must be specified to load from disk."
        self.fields_to_load = fields_to_load
        self.mode = mode

    def __call__(self, sample: SampleData) -> SampleData:
        for field in self.fields_to_load:
            assert field in sample, f"Column {field} not found in sample with keys {list(sample.keys())}."
            with open(sample[field], self.mode) as f:
                sample[field] = f.read()
        return sample


class GpuDecodeResizeImageTransform(BaseTransform):
    """Fused replacement of DecodeImage -> ResizeImage -> ConvertImageToByteTensor [-> NormalizeFrames]
    (presets.py:39-58, :68-74, :154-162) running on the GPU.

    ``sample[output_field]`` becomes a device tensor [3, H, W] with the reference's exact values and
    strides (HWC storage viewed as CHW, functional.py:104-108): uint8, or float32 ``x/127.5-1`` when
    ``normalize``.  ``resize_kwargs`` are those of lean_resize_frames (functional.py:42-50):
    crop_before_resize, allow_vertical, random_resize (np global RNG, same calls), interpolation_mode.
    ``hflip_prob`` (extension, default 0) fuses README.md:99-108's HorizontalFlipTransform: the coin is
    ``torch.rand(1) < hflip_prob`` from the global torch RNG, as that transform draws it.

    ``output_device`` (extension): None = the tensor stays on the decoding GPU; ``"cpu"`` = it is
    copied back to host memory -- the reference's own output type -- for DataLoaders with
    ``pin_memory=True`` (examples/iter_image_dataset.py:72-80), whose pin step rejects device
    tensors.

    ``service`` (extension): ``"auto"`` (default) starts the node-local decode service
    (sds_amd/service.py) when the transform is built on a machine with a GPU; the transform then
    decodes in-process in the process that built it, and through the service in every other process --
    the DataLoader workers -- which get host tensors (the reference's type; pin_memory pins them) and
    never initialise HIP themselves.  ``None`` = every process creates its own engine (device outputs,
    reaching the parent through HIP IPC); a string = the address of a running service.
    """

    def __init__(self, input_field: str, output_field: Optional[str] = None, resolution=(256, 256),
                 normalize: bool = False, device=None, hflip_prob: float = 0.0, output_device=None,
                 service="auto", **resize_kwargs):
        super().__init__(input_field, output_field)
        self.output_device = None if output_device is None else torch.device(output_device)
        self.resolution = tuple(int(v) for v in resolution)
        assert len(self.resolution) == 2, f"Wrong resolution: {resolution}"
        self.normalize = bool(normalize)
        self.device = device
        self.hflip_prob = float(hflip_prob)
        self.resize_kwargs = dict(resize_kwargs)
        F.check_resize_kwargs(self.resize_kwargs)
        self._owner_pid = os.getpid()
        self.service_address = _service_address(service, device)

    def __getstate__(self):
        return dict(self.__dict__)  # no native handle is ever stored on the transform

    def _served(self) -> bool:
        return self.service_address is not None and os.getpid() != self._owner_pid

    def __call__(self, sample: SampleData) -> SampleData:
        _validate_fields(sample, present=[self.input_field], absent=[])
        data = sample[self.input_field]
        if not isinstance(data, (bytes, bytearray, memoryview)):
            raise TypeError(f"Field '{self.input_field}' must hold encoded image bytes, got {type(data)}")
        data = bytes(data)
        kw = self.resize_kwargs
        eng = None if self._served() else _engine_in_worker(self.device)
        need_size = bool(kw.get("allow_vertical")) or kw.get("random_resize") is not None
        resolution = self.resolution
        # taken before target_resolution's np.random.choice, so that a rerun on the host (which draws
        # again, after PIL's decode, as the reference does) leaves the RNGs one draw ahead, not two
        rng = _RngSnapshot(kw.get("random_resize") is not None, self.hflip_prob > 0.0)
        if need_size:
            st, info = _lib.probe(data)
            if st != _lib.OK or info.width <= 0 or info.height <= 0:  # not a JPEG this path decodes
                img = self._host(eng, data)
                sample[self.output_field] = img.permute(2, 0, 1)
                return sample
            resolution = F.target_resolution(int(info.width), int(info.height), self.resolution,
                                             kw.get("allow_vertical", False), kw.get("random_resize"))
        flip = [bool(torch.rand(1) < self.hflip_prob)] if self.hflip_prob > 0.0 else None
        if eng is None:  # a worker process: through the node-local decode service
            op = JpegEngine.make_op(resolution, kw.get("crop_before_resize", True),
                                    F.filter_name(kw.get("interpolation_mode", "bilinear")), self.normalize, "hwc")
            st, arr = _service.client(self.service_address).decode(data, op, bool(flip and flip[0]))
            img = torch.from_numpy(arr) if st == _lib.OK else None
        else:
            out, status = eng.decode_resize([data], resolution, crop_before_resize=kw.get("crop_before_resize", True),
                                            filter=F.filter_name(kw.get("interpolation_mode", "bilinear")),
                                            normalize=self.normalize, flip=flip, layout="hwc")
            st = int(status[0])
            img = out[0]
        if st in (_lib.UNSUPPORTED, _lib.CORRUPT):
            # the sample reruns on the reference's own PIL decode (bit-exact by
            # definition); PIL raises for what it cannot decode, as functional.py:100 would
            rng.restore()
            img = self._host(eng, data)
        elif st != _lib.OK:
            raise_for_status(st)
        if self.output_device is not None and self.output_device != img.device:
            img = img.to(self.output_device)
        sample[self.output_field] = img.permute(2, 0, 1)  # [3, h, w] view of HWC storage
        return sample

    def _host(self, eng, data: bytes) -> torch.Tensor:
        """PIL decode on the host (functional.py:94-100), then the same crop / resize / flip / layout /
        normalise on the GPU through the frame path (pinned bit-exact to PIL.Image.resize); returns the
        [h, w, 3] HWC tensor.  The RNG draws follow the decode, as in the reference."""
        kw = self.resize_kwargs
        pil = pil_decode(data)
        w, h = pil.size
        resolution = F.target_resolution(w, h, self.resolution, kw.get("allow_vertical", False),
                                         kw.get("random_resize"))
        flip = [bool(torch.rand(1) < self.hflip_prob)] if self.hflip_prob > 0.0 else None
        if eng is None:  # through the service's frame path
            op = JpegEngine.make_op(resolution, kw.get("crop_before_resize", True),
                                    F.filter_name(kw.get("interpolation_mode", "bilinear")), self.normalize, "hwc")
            st, arr = _service.client(self.service_address).resize_frame(np.asarray(pil), op, bool(flip and flip[0]))
            raise_for_status(st)
            _note_fallback(data, self.input_field)
            img = torch.from_numpy(arr)
            if self.output_device is not None and self.output_device != img.device:
                img = img.to(self.output_device)
            return img
        frames = _frames_to_device([pil], torch.device("cuda", eng.device))
        out, status = eng.resize_frames(frames, resolution, crop_before_resize=kw.get("crop_before_resize", True),
                                        filter=F.filter_name(kw.get("interpolation_mode", "bilinear")),
                                        normalize=self.normalize, flip=flip, layout="hwc")
        raise_for_status(int(status[0].item()))
        eng.note_fallback()
        _note_fallback(data, self.input_field)
        img = out[0]
        if self.output_device is not None and self.output_device != img.device:
            img = img.to(self.output_device)
        return img


def _frames_to_device(frames, device) -> torch.Tensor:
    """PIL frames / HWC uint8 arrays / a uint8 [T, H, W, 3] tensor -> contiguous uint8 [T, H, W, 3] on the GPU."""
    if isinstance(frames, torch.Tensor):
        if frames.dim() != 4 or frames.shape[-1] != 3 or frames.dtype != torch.uint8:
            raise NotImplementedError("tensor frames must be uint8 [T, H, W, 3]; the reference resizes CHW tensors "
                                      "with torchvision's tensor kernels, which this path does not restate")
        return frames.to(device, non_blocking=True).contiguous()
    arrs = []
    for f in frames:
        if isinstance(f, torch.Tensor):
            raise NotImplementedError("per-frame tensors take torchvision's tensor resize in the reference; "
                                      "pass PIL frames or HWC uint8 arrays")
        a = np.asarray(f.convert("RGB") if hasattr(f, "convert") else f)
        if a.dtype != np.uint8 or a.ndim != 3 or a.shape[2] != 3:
            raise ValueError(f"frames must be RGB uint8 HWC, got {a.dtype} {a.shape}")
        arrs.append(a)
    host = torch.from_numpy(np.stack(arrs)).pin_memory() if torch.cuda.is_available() else torch.from_numpy(np.stack(arrs))
    return host.to(device, non_blocking=True)


class GpuResizeVideoTransform(BaseTransform):
    """Fused ResizeVideoTransform + ConvertVideoToByteTensorTransform (+ NormalizeFramesTransform)
    (presets.py:121-135, :154-162) on the GPU: ``sample[input_field]`` = the decoded frames (PIL images,
    as PyAV's ``to_image`` gives them, or HWC uint8 arrays, or a uint8 [T, H, W, 3] tensor) ->
    ``sample[output_field]`` = device tensor [T, 3, h, w], uint8 (or float32 ``x/127.5-1``).
    ``transform_kwargs`` are lean_resize_frames's (functional.py:42-50): ``resolution``,
    ``crop_before_resize``, ``allow_vertical``, ``random_resize`` (one draw per video, np global RNG),
    ``interpolation_mode``; the same-size shortcut (functional.py:78-80) holds."""

    def __init__(self, input_field: str, output_field: Optional[str] = None, normalize: bool = False, device=None,
                 **transform_kwargs):
        super().__init__(input_field, output_field, **transform_kwargs)
        assert "resolution" in transform_kwargs, "lean_resize_frames needs a resolution"
        self.normalize = bool(normalize)
        self.device = device
        kw = dict(transform_kwargs)
        kw.pop("resolution")
        F.check_resize_kwargs(kw)

    def __call__(self, sample: SampleData) -> SampleData:
        _validate_fields(sample, present=[self.input_field], absent=[])
        kw = dict(self.transform_kwargs)
        eng = get_engine(self.device)
        frames = _frames_to_device(sample[self.input_field], torch.device("cuda", eng.device))
        t, h, w = int(frames.shape[0]), int(frames.shape[1]), int(frames.shape[2])
        resolution = F.target_resolution(w, h, kw["resolution"], kw.get("allow_vertical", False),
                                         kw.get("random_resize"))
        out, status = eng.resize_frames(frames, resolution, crop_before_resize=kw.get("crop_before_resize", True),
                                        filter=F.filter_name(kw.get("interpolation_mode", "bilinear")),
                                        normalize=self.normalize)
        bad = torch.nonzero(status != 0)
        if bad.numel():
            raise_for_status(int(status[int(bad[0])]), int(bad[0]))
        sample[self.output_field] = out
        return sample


class GpuUndistortFramesTransform(BaseTransform):
    """UndistortFramesTransform (presets.py:164-188) on the GPU frame path.

    When the sample's original resolution (``original_resolution_fields`` = (height field, width field))
    and the frames' aspect ratios differ by more than 0.02, the frames are resized to
    ``(round(cur_w / orig_ar), cur_w)`` by lean_resize_frames with its defaults (centre crop, Pillow
    bilinear, functional.py:42-86) -- a uint8-rounded resize of its own, ahead of the video resize (the
    reference rounds between the two, so the two passes are not fused).  ``sample[output_field]`` then
    holds the undistorted frames as a device uint8 [T, H', W, 3] tensor, which GpuResizeVideoTransform
    takes as its input.  Otherwise (no original resolution, or aspect ratios within the tolerance) the
    sample is returned untouched, as in the reference -- ``output_field`` is then not written either.

    Frames are what the reference reads ``.size`` from: PIL images (PyAV's ``to_image``); HWC uint8
    arrays and a uint8 [T, H, W, 3] tensor are accepted as well."""

    def __init__(self, input_field: str, original_resolution_fields: tuple, output_field: Optional[str] = None,
                 device=None):
        super().__init__(input_field, output_field)
        self.original_resolution_fields = tuple(original_resolution_fields)
        self.device = device

    @staticmethod
    def _frame_size(frames) -> tuple[int, int]:
        """(width, height) of the first frame, as the reference's ``frames[0].size``."""
        if isinstance(frames, torch.Tensor):
            return int(frames.shape[2]), int(frames.shape[1])
        f = frames[0]
        if hasattr(f, "size") and isinstance(f.size, tuple):
            return f.size
        a = np.asarray(f)
        return int(a.shape[1]), int(a.shape[0])

    @staticmethod
    def target(orig_height, orig_width, cur_width: int, cur_height: int) -> Optional[tuple[int, int]]:
        """presets.py:178-186: the (height, width) the frames are resized to, or None to leave them."""
        if orig_height is None or orig_width is None:
            return None  # no original resolution: skip undistortion
        assert isinstance(orig_height, (int, float)) and isinstance(orig_width, (int, float)), \
            f"Original resolution fields must be numeric, got {type(orig_height)} and {type(orig_width)}."
        orig_aspect_ratio = orig_width / orig_height
        cur_aspect_ratio = cur_width / cur_height
        if abs(orig_aspect_ratio - cur_aspect_ratio) > 0.02:  # the reference's tolerance
            return round(cur_width / orig_aspect_ratio), cur_width
        return None

    def __call__(self, sample: SampleData) -> SampleData:
        orig_h = sample.get(self.original_resolution_fields[0])
        orig_w = sample.get(self.original_resolution_fields[1])
        if orig_h is None or orig_w is None:
            return sample
        w, h = self._frame_size(sample[self.input_field])
        res = self.target(orig_h, orig_w, w, h)
        if res is None:
            return sample
        eng = get_engine(self.device)
        frames = _frames_to_device(sample[self.input_field], torch.device("cuda", eng.device))
        if res == (h, w):  # lean_resize_frames's same-size shortcut (functional.py:78-80): the frames as they are
            sample[self.output_field] = frames
            return sample
        out, status = eng.resize_frames(frames, res, crop_before_resize=True, filter="bilinear", layout="hwc")
        bad = torch.nonzero(status != 0)
        if bad.numel():
            raise_for_status(int(status[int(bad[0])]), int(bad[0]))
        sample[self.output_field] = out
        return sample


class ReshapeImageAsVideoTransform(BaseTransform):
    """presets.py:60-66 -> functional.py:88-92."""

    def __call__(self, sample: SampleData) -> SampleData:
        _validate_fields(sample, present=[self.input_field], absent=[self.output_field])
        image = sample[self.input_field]
        assert len(image.shape) == 3, f"Wrong shape: {image.shape}."
        sample[self.output_field] = image.unsqueeze(0)
        return sample


class NormalizeFramesTransform(BaseTransform):
    """presets.py:154-162 (device-agnostic; runs on the GPU tensor)."""

    def __call__(self, sample: SampleData) -> SampleData:
        _validate_fields(sample, present={self.input_field: torch.Tensor}, absent=[])
        assert sample[self.input_field].dtype == torch.uint8, \
            f"Expected input field '{self.input_field}' to be of type torch.uint8, but got {sample[self.input_field].dtype}."
        sample[self.output_field] = sample[self.input_field].float() / 127.5 - 1.0
        return sample


class FieldsFilteringTransform:
    """presets.py:628-644."""

    def __init__(self, fields_to_keep: Optional[Sequence[str]] = None, fields_to_remove: Optional[Sequence[str]] = None):
        assert fields_to_keep is not None or fields_to_remove is not None, \
            "At least one of fields_to_keep or fields_to_remove must be provided."
        self.fields_to_keep = fields_to_keep
        self.fields_to_remove = fields_to_remove

    def __call__(self, sample: SampleData) -> SampleData:
        if self.fields_to_remove is not None:
            for field in self.fields_to_remove:
                sample.pop(field, None)
        if self.fields_to_keep is not None:
            for field in list(sample.keys()):
                if field not in self.fields_to_keep:
                    sample.pop(field, None)
        return sample


class AugmentNewFieldsTransform:
    """presets.py:646-656."""

    def __init__(self, new_fields: dict):
        self.new_fields = new_fields

    def __call__(self, sample: SampleData) -> SampleData:
        for field, value in self.new_fields.items():
            assert field not in sample, f"Field '{field}' already exists in sample with keys {list(sample.keys())}."
            sample[field] = value
        return sample


class EnsureFieldsTransform:
    """presets.py:670-686: presence/type/dummy checks; ``drop_others`` keeps whitelisted keys in order."""

    def __init__(self, fields_whitelist, check_dummy_values: bool = False, drop_others: bool = False):
        self.fields_whitelist = fields_whitelist
        self.check_dummy_values = check_dummy_values
        self.drop_others = drop_others

    def __call__(self, sample: SampleData) -> SampleData:
        _validate_fields(sample, present=self.fields_whitelist, absent=[], check_dummy_values=self.check_dummy_values)
        if self.drop_others:
            for field in list(sample.keys()):
                if field not in self.fields_whitelist:
                    del sample[field]
        return sample


class HorizontalFlipTransform:
    """README.md:99-108 / examples/iter_img2img.py:29-41 (user code there), device-agnostic."""

    def __init__(self, image_field: str = "image"):
        self.image_field = image_field

    def __call__(self, sample: dict) -> dict:
        assert self.image_field in sample, f"Image field is missing in the sample: {sample.keys()}"
        img = sample[self.image_field]
        assert isinstance(img, torch.Tensor) and img.ndim == 3 and img.shape[0] in (1, 3)
        sample[self.image_field] = torch.flip(img, dims=[2]) if torch.rand(1) < 0.5 else img
        return sample


def create_standard_image_pipeline(
    image_field: str,
    resolution: tuple[int, int],
    return_image_as_single_frame_video: bool = False,
    normalize: bool = False,
    resize_kwargs: dict = {},  # noqa: B006  (same default as the reference signature)
    output_field: str = "image",
    video_output_field: str = "video",
    *,
    device=None,
    hflip_prob: float = 0.0,
    output_device=None,
    service="auto",
) -> Sequence[SampleTransform]:
    """presets.py:716-744 with the decode/resize/to-tensor/normalise chain fused on the GPU.  ``service``:
    see GpuDecodeResizeImageTransform (the decode service for DataLoader workers).

    Output device: with the default ``service="auto"`` and ``output_device=None`` the process that built
    the pipeline gets device tensors (it decodes in-process), while its forked DataLoader workers get
    host tensors (they decode through the service: the reference's type, which ``pin_memory=True``
    pins).  Pass ``output_device="cpu"`` for host tensors everywhere, or ``service=None`` for device
    tensors everywhere (workers then create their own engines: spawn / forkserver workers, INTEGRATION.md
    §1).  On a machine with a GPU, ``service="auto"`` starts the service process at construction -- it
    sleeps without a GPU context until a worker connects, and exits with this process."""
    transforms: list = [
        LoadFromDiskTransform([image_field]),
        GpuDecodeResizeImageTransform(input_field=image_field, output_field=output_field, resolution=resolution,
                                      normalize=normalize, device=device, hflip_prob=hflip_prob,
                                      output_device=output_device, service=service, **resize_kwargs),
    ]
    if return_image_as_single_frame_video:
        transforms.extend([
            ReshapeImageAsVideoTransform(input_field=output_field, output_field=video_output_field),
            FieldsFilteringTransform(fields_to_remove=[output_field]),
            AugmentNewFieldsTransform(new_fields=dict(framerate=960.0)),
        ])
    return transforms
