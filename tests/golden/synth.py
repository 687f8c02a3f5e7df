"""Seeded synthetic JPEG generator, shared by tests, smoke and bench.

Each image: x,y grids; R = 127+100 sin(x/(20+40u)+6u), G = 127+100 cos(y/(20+40u)+6u),
B = 127+60 sin((x+y)/(30+30u)), plus N(0, 8) noise, clipped to uint8, with the three u ~ U[0,1)
drawn in that order from ``numpy.random.default_rng(seed)``.  Encoded by
``PIL.Image.save(format='JPEG', quality=q)`` defaults: baseline, 4:2:0, Annex-K tables, no DRI.
"""
from __future__ import annotations

import io

import numpy as np


def synth_rgb(rng: np.random.Generator, w: int = 640, h: int = 480) -> np.ndarray:
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    u = rng.random()
    r = 127 + 100 * np.sin(x / (20 + 40 * u) + 6 * u)
    u = rng.random()
    g = 127 + 100 * np.cos(y / (20 + 40 * u) + 6 * u)
    u = rng.random()
    b = 127 + 60 * np.sin((x + y) / (30 + 30 * u))
    img = np.stack([r, g, b], -1) + rng.normal(0, 8, (h, w, 3))
    return np.clip(img, 0, 255).astype(np.uint8)


def encode_jpeg(rgb: np.ndarray, quality: int = 90, **kw) -> bytes:
    from PIL import Image, ImageFile

    ImageFile.MAXBLOCK = max(ImageFile.MAXBLOCK, 1 << 24)
    buf = io.BytesIO()
    Image.fromarray(rgb).save(buf, format="JPEG", quality=quality, **kw)
    return buf.getvalue()


def synth_jpegs(n: int, seed: int = 1234, w: int = 640, h: int = 480, quality: int = 90, **kw) -> list[bytes]:
    rng = np.random.default_rng(seed)
    return [encode_jpeg(synth_rgb(rng, w, h), quality, **kw) for _ in range(n)]


# Config 3 size pool: landscape sizes and their portrait transposes.
MIXED_SIZES = [(640, 480), (1280, 720), (1366, 768), (1920, 1080), (2560, 1440), (3840, 2160)]
MIXED_SIZES = MIXED_SIZES + [(h, w) for (w, h) in MIXED_SIZES]


def synth_mixed(n: int, seed: int = 4321, quality: int = 90, max_side: int = 3840) -> list[bytes]:
    rng = np.random.default_rng(seed)
    pool = [s for s in MIXED_SIZES if max(s) <= max_side]
    out = []
    for _ in range(n):
        w, h = pool[int(rng.integers(0, len(pool)))]
        out.append(encode_jpeg(synth_rgb(rng, w, h), quality))
    return out


def mutated_jpegs(seed: int, n: int) -> list[bytes]:
    """Truncations, byte flips and marker-like insertions inside the entropy segment of synthetic JPEGs
    (the FF00 / fill-byte / RSTn / foreign-marker paths of jdhuff.c jpeg_fill_bit_buffer)."""
    from oracle import oracle as O  # only to locate the entropy segment (test infrastructure)
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        kw = {"restart_marker_blocks": 2} if i % 3 == 0 else {}
        jpg = bytearray(encode_jpeg(synth_rgb(rng, int(rng.integers(40, 200)), int(rng.integers(40, 200))), 90, **kw))
        _, info = O.probe(bytes(jpg))
        lo, hi = int(info.entropy_offset), len(jpg) - 2
        kind = i % 5
        p = int(rng.integers(lo, hi))
        if kind == 0:
            jpg = jpg[:p]                                   # truncated
        elif kind == 1:
            jpg[p] ^= int(rng.integers(1, 256))             # flipped byte (may break or keep the stream)
        elif kind == 2:
            jpg[p:p] = b"\xff\xff\xff\x00"                  # fill bytes before a stuffed zero
        elif kind == 3:
            jpg[p:p] = b"\xff\xd9"                          # a foreign marker mid-scan (EOI)
        else:
            jpg[p:p] = b"\xff\xd3"                          # an unexpected RSTn
        out.append(bytes(jpg))
    return out


def has_fill_stuffing(jpg: bytes) -> bool:
    """True if a baseline JPEG without restart intervals holds FF FF .. 00 (fill bytes before a stuffed
    zero) inside its scan -- before the first marker that ends it (RSTn and codes below SOF0 do not).
    jdhuff.c's slow path reads it as one FF data byte; libjpeg-turbo's decode_mcu_fast takes it for a
    marker and leaves that MCU's fast-path coefficients under the slow path's, so the MI355X kernels
    report such streams SDSJ_CORRUPT and the transforms rerun them on PIL (sdsj_kernels.hip us_classify)."""
    d, i, ri = jpg, 2, 0
    while i + 4 <= len(d) and d[i] == 0xFF:
        m, ln = d[i + 1], (d[i + 2] << 8) | d[i + 3]
        if m == 0xDD and ln == 4:
            ri = (d[i + 4] << 8) | d[i + 5]
        if m == 0xC2 or ri:
            return False
        if m == 0xDA:
            i += 2 + ln
            break
        i += 2 + ln
    else:
        return False
    n = len(d)
    while i < n:
        if d[i] != 0xFF:
            i += 1
            continue
        j = i + 1
        while j < n and d[j] == 0xFF:
            j += 1
        if j >= n:
            return False
        if d[j] == 0:
            if j - i >= 2:
                return True
        elif not (0xD0 <= d[j] <= 0xD7 or d[j] < 0xC0):
            return False
        i = j + 1
    return False


def progressive_jpegs(seed: int, n: int, max_w: int = 400, max_h: int = 300) -> list[bytes]:
    """Progressive JPEGs (PIL/libjpeg-turbo's default scan script) of random sizes, sampling,
    quality, optimized tables and restart intervals, grayscale every fifth."""
    from PIL import Image
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        w, h = int(rng.integers(1, max_w)), int(rng.integers(1, max_h))
        rgb = rng.integers(0, 256, (h, w, 3), dtype=np.uint8) if i % 3 == 0 else synth_rgb(rng, w, h)
        kw = dict(progressive=True)
        if i % 5 == 0:
            rgb = np.array(Image.fromarray(rgb).convert("L"))
        else:
            kw["subsampling"] = int(rng.integers(0, 3))
        if i % 4 == 1:
            kw["optimize"] = True
        if i % 7 == 2:
            kw["restart_marker_blocks"] = int(rng.integers(1, 5))
        out.append(encode_jpeg(rgb, int(rng.integers(5, 101)), **kw))
    return out
