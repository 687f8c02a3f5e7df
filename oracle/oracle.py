"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper around the C oracle (oracle/sdsj_oracle.c).

The oracle is the parity checker for the MI355X path.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this
module; the product package ``sds_amd`` never does (tests/test_no_oracle_in_product.py
checks that).

Reference behaviour restated (see the C file header for the full list):
  * ``sds/transforms/functional.py:94-100``  decode (PIL -> libjpeg-turbo 3.1.4, ISLOW, fancy)
  * ``sds/transforms/functional.py:118-147`` crop_to_aspect_ratio
  * ``sds/transforms/functional.py:42-86``   lean_resize_frames -> Pillow Resample.c
  * ``sds/transforms/functional.py:102-110`` HWC uint8 -> CHW view
  * ``sds/transforms/presets.py:154-162``    x.float() / 127.5 - 1.0
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libsdsj_oracle.so")

OK, EINVAL, UNSUPPORTED, CORRUPT, ENOMEM = 0, -1, -2, -3, -4
FILTERS = {"box": 0, "bilinear": 1, "hamming": 2, "bicubic": 3, "lanczos": 4, "nearest": 5}


class OracleInfo(ctypes.Structure):
    _fields_ = [
        ("width", ctypes.c_int32), ("height", ctypes.c_int32), ("ncomp", ctypes.c_int32),
        ("h", ctypes.c_int32 * 3), ("v", ctypes.c_int32 * 3),
        ("restart_interval", ctypes.c_int32), ("entropy_offset", ctypes.c_int64),
    ]


def build() -> str:
    """Compiles the oracle with its Makefile (gcc) if the shared library is missing or stale."""
    src = os.path.join(_HERE, "sdsj_oracle.c")
    if (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        u8p = ctypes.POINTER(ctypes.c_uint8)
        _lib.sdsj_oracle_probe.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(OracleInfo)]
        _lib.sdsj_oracle_decode.argtypes = [ctypes.c_char_p, ctypes.c_size_t, u8p, ctypes.c_int, ctypes.c_int]
        _lib.sdsj_oracle_coefficients.argtypes = [
            ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.POINTER(ctypes.c_int16), ctypes.c_int64,
            ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
        _lib.sdsj_oracle_crop_box.argtypes = [ctypes.c_int] * 4 + [ctypes.POINTER(ctypes.c_int)]
        _lib.sdsj_oracle_resize.argtypes = [u8p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, u8p]
        _lib.sdsj_oracle_pipeline.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_int,
                                              ctypes.c_int, ctypes.c_int, u8p]
    return _lib


def _u8p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


class OracleError(Exception):
    def __init__(self, status: int):
        super().__init__(f"oracle status {status}")
        self.status = status


def probe(jpg: bytes) -> tuple[int, OracleInfo]:
    info = OracleInfo()
    st = lib().sdsj_oracle_probe(jpg, len(jpg), ctypes.byref(info))
    return st, info


def decode(jpg: bytes) -> np.ndarray:
    """Full-resolution RGB decode, HWC uint8 (== np.array(PIL.Image.open(...).convert('RGB')))."""
    st, info = probe(jpg)
    if st != OK:
        raise OracleError(st)
    out = np.empty((info.height, info.width, 3), np.uint8)
    st = lib().sdsj_oracle_decode(jpg, len(jpg), _u8p(out), info.width, info.height)
    if st != OK:
        raise OracleError(st)
    return out


def coefficients(jpg: bytes, comp: int) -> np.ndarray:
    st, info = probe(jpg)
    if st != OK:
        raise OracleError(st)
    cap = (info.width // 8 + 8) * (info.height // 8 + 8) * 64 * 4
    buf = np.zeros(cap, np.int16)
    bw, bh = ctypes.c_int(), ctypes.c_int()
    st = lib().sdsj_oracle_coefficients(jpg, len(jpg), comp, buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)),
                                        cap, ctypes.byref(bw), ctypes.byref(bh))
    if st != OK:
        raise OracleError(st)
    return buf[: bw.value * bh.value * 64].reshape(bh.value, bw.value, 64)


def crop_box(w: int, h: int, out_h: int, out_w: int) -> tuple[int, int, int, int]:
    box = (ctypes.c_int * 4)()
    lib().sdsj_oracle_crop_box(w, h, out_h, out_w, box)
    return tuple(box)


def resize(rgb: np.ndarray, out_h: int, out_w: int, filter: str = "bilinear") -> np.ndarray:
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    h, w = rgb.shape[:2]
    out = np.empty((out_h, out_w, 3), np.uint8)
    st = lib().sdsj_oracle_resize(_u8p(rgb), w, h, out_w, out_h, FILTERS[filter], _u8p(out))
    if st != OK:
        raise OracleError(st)
    return out


def normalize_lut() -> np.ndarray:
    """presets.py:161 ``x.float() / 127.5 - 1.0`` in float32, as a 256-entry table."""
    v = np.arange(256, dtype=np.float32)
    return (v / np.float32(127.5) - np.float32(1.0)).astype(np.float32)


def pipeline(jpg: bytes, resolution: tuple[int, int], crop_before_resize: bool = True,
             filter: str = "bilinear", flip: bool = False, normalize: bool = False) -> np.ndarray:
    """Reference image pipeline for one JPEG; returns CHW (uint8, or float32 if normalize)."""
    out_h, out_w = resolution
    st, info = probe(jpg)
    if st != OK:
        raise OracleError(st)
    if (info.width, info.height) == (out_w, out_h):
        hwc = decode(jpg)
    else:
        hwc = np.empty((out_h, out_w, 3), np.uint8)
        st = lib().sdsj_oracle_pipeline(jpg, len(jpg), out_h, out_w, int(crop_before_resize),
                                        FILTERS[filter], _u8p(hwc))
        if st != OK:
            raise OracleError(st)
    chw = np.ascontiguousarray(hwc.transpose(2, 0, 1))
    if flip:
        chw = np.ascontiguousarray(chw[:, :, ::-1])
    if normalize:
        chw = normalize_lut()[chw]
    return chw
