"""ctypes binding of the C-ABI in include/sdsj.h (the in-tree ``sds_amd/lib/libsdsj.so``).

This is the binding a maintainer would add to sds.  ``torch`` is imported
first so that the process holds exactly one HIP runtime: the library's ``libamdhip64.so.7``
dependency then resolves to the copy torch already loaded (same SONAME as /opt/rocm's).

There is no CPU fallback: if the library is missing or cannot be loaded, every entry point
raises ``NativeLibraryError``.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
# SDSJ_LIBRARY: an alternative in-tree build (kernel experiments under tools/); default = the product
LIB_PATH = os.environ.get("SDSJ_LIBRARY") or os.path.join(_HERE, "lib", "libsdsj.so")

SDSJ_ABI_VERSION = 2
OK, EINVAL, UNSUPPORTED, CORRUPT, ENOMEM, EHIP, ECAPACITY = 0, -1, -2, -3, -4, -5, -6
STATUS_NAMES = {OK: "OK", EINVAL: "EINVAL", UNSUPPORTED: "UNSUPPORTED", CORRUPT: "CORRUPT", ENOMEM: "ENOMEM",
                EHIP: "EHIP", ECAPACITY: "ECAPACITY"}
FILTERS = {"box": 0, "bilinear": 1, "hamming": 2, "bicubic": 3, "lanczos": 4, "nearest": 5}
DTYPE_U8, DTYPE_F32 = 0, 1
LAYOUT_CHW, LAYOUT_HWC = 0, 1

# Every symbol include/sdsj.h declares (checked by tests/test_abi.py).
EXPORTS = [
    "sdsj_abi_version", "sdsj_probe", "sdsj_engine_create", "sdsj_engine_destroy", "sdsj_decode_resize_batch",
    "sdsj_decode_resize_batch_device", "sdsj_engine_set_timing", "sdsj_engine_stage_times", "sdsj_last_error",
    "sdsj_stage_name", "sdsj_engine_debug_buffers", "sdsj_resize_frames_device", "sdsj_submit_batch",
    "sdsj_submit_files", "sdsj_wait_batch", "sdsj_engine_counters", "sdsj_counter_name", "sdsj_engine_set_lanes",
    "sdsj_engine_reserve", "sdsj_plan_need", "sdsj_service_serve",
]
NUM_COUNTERS = 10  # SDSJ_NUM_COUNTERS
SLOTS = 2  # SDSJ_SLOTS: batches in flight on the asynchronous host path


class NativeLibraryError(RuntimeError):
    pass


class SdsjInfo(ctypes.Structure):
    _fields_ = [("width", ctypes.c_int32), ("height", ctypes.c_int32), ("ncomp", ctypes.c_int32),
                ("h_samp", ctypes.c_int32 * 3), ("v_samp", ctypes.c_int32 * 3),
                ("restart_interval", ctypes.c_int32), ("supported", ctypes.c_int32),
                ("entropy_offset", ctypes.c_int64)]


class SdsjCfg(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("max_batch", ctypes.c_int32), ("scratch_bytes", ctypes.c_int64)]


class SdsjOp(ctypes.Structure):
    _fields_ = [("out_h", ctypes.c_int32), ("out_w", ctypes.c_int32), ("crop_before_resize", ctypes.c_int32),
                ("filter", ctypes.c_int32), ("out_dtype", ctypes.c_int32), ("layout", ctypes.c_int32)]


class SdsjServiceCfg(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("device", ctypes.c_int32), ("engines", ctypes.c_int32),
                ("max_batch", ctypes.c_int32), ("listen_fd", ctypes.c_int32), ("parent_pid", ctypes.c_int32)]


_lib = None
_lock = threading.Lock()


def load() -> ctypes.CDLL:
    """Loads libsdsj.so (raises NativeLibraryError if it is absent or broken)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryError(
                f"{LIB_PATH} is missing: build the MI355X extension first "
                "(python -m sds_amd.build, or __graft_entry__.build()). There is no CPU fallback.")
        try:
            lib = ctypes.CDLL(LIB_PATH)
        except OSError as e:
            raise NativeLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        vp, i32, i64, sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_size_t
        lib.sdsj_abi_version.restype = ctypes.c_int
        lib.sdsj_probe.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(SdsjInfo)]
        lib.sdsj_engine_create.argtypes = [ctypes.c_int, ctypes.POINTER(SdsjCfg), ctypes.POINTER(vp)]
        lib.sdsj_engine_destroy.argtypes = [vp]
        lib.sdsj_decode_resize_batch.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                                 ctypes.POINTER(sz), ctypes.POINTER(SdsjOp), vp, vp,
                                                 ctypes.POINTER(i32), vp]
        lib.sdsj_decode_resize_batch_device.argtypes = [vp, ctypes.c_int, vp, sz, vp, vp, ctypes.POINTER(SdsjOp), vp, vp,
                                                        vp, vp]
        lib.sdsj_resize_frames_device.argtypes = [vp, ctypes.c_int, vp, i32, i32, i64, ctypes.POINTER(SdsjOp), vp, vp,
                                                  vp, vp]
        lib.sdsj_submit_batch.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                          ctypes.POINTER(sz), ctypes.POINTER(SdsjOp), vp, vp, vp]
        lib.sdsj_submit_files.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                          ctypes.POINTER(SdsjOp), vp, vp, vp]
        lib.sdsj_wait_batch.argtypes = [vp, ctypes.c_int, ctypes.POINTER(i32)]
        lib.sdsj_engine_set_timing.argtypes = [vp, ctypes.c_int]
        lib.sdsj_engine_stage_times.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.c_int,
                                                ctypes.POINTER(ctypes.c_int)]
        lib.sdsj_last_error.argtypes = [vp]
        lib.sdsj_last_error.restype = ctypes.c_char_p
        lib.sdsj_stage_name.argtypes = [ctypes.c_int]
        lib.sdsj_stage_name.restype = ctypes.c_char_p
        lib.sdsj_engine_debug_buffers.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp),
                                                  ctypes.POINTER(i64), ctypes.POINTER(i64)]
        lib.sdsj_engine_counters.argtypes = [vp, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int, ctypes.c_int]
        lib.sdsj_counter_name.argtypes = [ctypes.c_int]
        lib.sdsj_counter_name.restype = ctypes.c_char_p
        lib.sdsj_engine_set_lanes.argtypes = [vp, ctypes.c_int]
        lib.sdsj_engine_reserve.argtypes = [vp, i64]
        lib.sdsj_plan_need.argtypes = [ctypes.c_char_p, sz, ctypes.POINTER(SdsjOp), ctypes.POINTER(i64)]
        lib.sdsj_service_serve.argtypes = [ctypes.POINTER(SdsjServiceCfg)]
        for name in EXPORTS:
            getattr(lib, name)  # AttributeError if the library lacks a declared symbol
        if lib.sdsj_abi_version() != SDSJ_ABI_VERSION:
            raise NativeLibraryError(f"ABI version mismatch: {lib.sdsj_abi_version()} != {SDSJ_ABI_VERSION}")
        _lib = lib
        return lib


def probe(jpg: bytes) -> tuple[int, SdsjInfo]:
    info = SdsjInfo()
    st = load().sdsj_probe(jpg, len(jpg), ctypes.byref(info))
    return st, info
