"""Host-side helpers of the image path (the parts of sds/transforms/functional.py that decide
*what* to compute; the arithmetic itself runs in the HIP kernels)."""
from __future__ import annotations

from typing import Optional

import numpy as np

from . import _lib

_RESIZE_KWARGS = {"crop_before_resize", "allow_vertical", "random_resize", "interpolation_mode"}


# torchvision's pil_modes_mapping: NEAREST_EXACT resizes a PIL image with PIL NEAREST, as NEAREST does
_TV_TO_PIL = {"nearest-exact": "nearest"}


def filter_name(mode) -> str:
    """torchvision InterpolationMode (enum or its string value) -> engine filter name.

    The reference resizes PIL images (functional.py:84), so TVF.resize delegates to PIL.Image.resize
    with the mapped Pillow filter: every Pillow separable filter (Resample.c) and NEAREST
    (Geometry.c ImagingScaleAffine, for both 'nearest' and 'nearest-exact') are implemented.  A name
    InterpolationMode does not define raises ValueError, as ``TVF.InterpolationMode(name)`` does."""
    name = getattr(mode, "value", mode)
    name = str(name).lower()
    name = _TV_TO_PIL.get(name, name)
    if name not in _lib.FILTERS:
        raise ValueError(f"{mode!r} is not a valid InterpolationMode")
    return name


def check_resize_kwargs(kw: dict) -> None:
    unknown = set(kw) - _RESIZE_KWARGS
    if unknown:
        raise TypeError(f"unexpected resize kwargs {sorted(unknown)} (lean_resize_frames, functional.py:42-50)")
    filter_name(kw.get("interpolation_mode", "bilinear"))


def image_size(data: bytes) -> tuple[int, int]:
    """(width, height) from the JPEG header (host parse, sdsj_probe)."""
    st, info = _lib.probe(data)
    if info.width <= 0 or info.height <= 0:
        from .engine import raise_for_status
        raise_for_status(st if st != _lib.OK else _lib.CORRUPT)
    return int(info.width), int(info.height)


def target_resolution(w: int, h: int, resolution, allow_vertical: bool = False,
                      random_resize: Optional[dict] = None) -> tuple[int, int]:
    """functional.py:62-76: random downsampling choice (np global RNG) and vertical flip of the
    target; returns (h_trg, w_trg)."""
    is_originally_vertical = h > w
    if random_resize is not None:
        assert sum(random_resize.values()) == 1.0, f"Probabilities should sum to 1.0: {random_resize}"
        random_resize = {k: v for k, v in random_resize.items() if k[0] <= w and k[1] <= h}
        if len(random_resize) > 0:
            resolutions, probs = zip(*random_resize.items())
            resolution = resolutions[np.random.choice(len(resolutions), p=np.array(probs) / sum(probs))]
    h_trg, w_trg = (max(resolution), min(resolution)) if is_originally_vertical and allow_vertical else resolution
    return int(h_trg), int(w_trg)


def crop_box(w: int, h: int, out_h: int, out_w: int) -> tuple[int, int, int, int]:
    """functional.py:118-140 crop_to_aspect_ratio box (left, top, right, bottom)."""
    cur = w / h
    tgt = out_w / out_h
    if cur > tgt:
        nw = int(h * tgt)
        left = (w - nw) // 2
        return left, 0, left + nw, h
    nh = int(w / tgt)
    top = (h - nh) // 2
    return 0, top, w, top + nh


_SIGNATURES = ((b"\x89PNG\r\n\x1a\n", "PNG"), (b"GIF87a", "GIF"), (b"GIF89a", "GIF"), (b"BM", "BMP"),
               (b"II*\x00", "TIFF"), (b"MM\x00*", "TIFF"), (b"\x00\x00\x01\x00", "ICO"), (b"8BPS", "PSD"),
               (b"\x00\x00\x00\x0cjP  ", "JPEG 2000"), (b"\xff\x4f\xff\x51", "JPEG 2000"))


def sniff_format(data: bytes) -> str:
    """Names the container of an encoded image for messages and logs (no decoding)."""
    head = bytes(data[:16])
    if head[:2] == b"\xff\xd8":
        return "JPEG (a mode this path does not decode: arithmetic, 12-bit, lossless, CMYK or multi-scan)"
    if head[:4] == b"RIFF" and head[8:12] == b"WEBP":
        return "WebP"
    for sig, name in _SIGNATURES:
        if head.startswith(sig):
            return name
    return "non-JPEG"
