"""Stage-level diagnostics for the GPU path (test infrastructure).

Mirrors ``sdsj::ImgDesc`` (sds_amd/csrc/sdsj_common.h) with ctypes so tests can pull the
intermediate buffers (unstuffed stream, coefficients, planes, RGB rows) of the most recent chunk
off the device and compare them with the oracle stage by stage.

    python tests/gpu_debug.py          # on the GPU box: one image through every stage
"""
from __future__ import annotations

import ctypes
import os
import sys

import numpy as np

i32, i64 = ctypes.c_int32, ctypes.c_int64


class CompDescC(ctypes.Structure):
    _fields_ = [(n, i32) for n in ("h", "v", "tq", "td", "ta", "rh", "rv", "dw", "dh", "bw", "bh", "pitch")] + \
               [("plane_off", i64)]


class ImgDescC(ctypes.Structure):
    _fields_ = [(n, i32) for n in ("status", "width", "height", "ncomp", "hmax", "vmax", "mcux", "mcuy", "bpm",
                                   "restart_interval", "nseg", "saw_jfif", "saw_adobe", "adobe_transform")] + \
               [("comp_id", i32 * 3), ("entropy_off", i64), ("entropy_len", i64), ("total_blocks", i64),
                ("blk_comp", i32 * 10), ("blk_dx", i32 * 10), ("blk_dy", i32 * 10), ("comp", CompDescC * 3)] + \
               [(n, i32) for n in ("geo", "cx0", "cy0", "cw", "ch", "need_h", "need_v", "ksh", "ksv", "yf", "yl",
                                   "src_y0", "src_y1", "src_x0", "src_w", "sub_bits", "nsub_cap")] + \
               [(n, i64) for n in ("off_ustream", "ustream_cap", "off_seg", "off_sub", "off_rec", "off_coef", "off_planes",
                                   "off_rgb", "off_tmp", "off_kh", "off_kv", "need")] + \
               [("nsub", i32), ("useg_found", i32), ("ulen", i64), ("sync_rounds", i32), ("pad0", i32),
                ("sym_spec", i64), ("sym_sync", i64), ("sym_write", i64),
                ("t_spec", i64), ("t_sync", i64), ("t_scan", i64), ("t_write", i64), ("it_spec", i64), ("it_sync", i64),
                ("it_write", i64), ("fused", i32), ("tile_w", i32), ("ring_rows", i32), ("rs_fast", i32), ("t_rs", i64 * 4),
                ("warm_bits", i32), ("scan_end_code", i32), ("scan_end_raw", i64),
                ("rgb_pitch", i32), ("ent_groups", i32),
                ("progressive", i32), ("lat", i32), ("sos_pos", i64), ("off_ptab", i64),
                ("off_tiles", i64), ("ntiles", i32), ("rs_lay", i32), ("plan_base", i64),
                ("smooth", i32), ("sm_good", i32), ("sm_bits", ctypes.c_int8 * 60), ("mh", ctypes.c_int8),
                ("sm_pad", ctypes.c_int8 * 3), ("etab", i32), ("etab_pad", i32)]


def _memcpy_d2h(ptr: int, nbytes: int) -> np.ndarray:
    import torch
    out = torch.empty(nbytes, dtype=torch.uint8)
    # wrap the raw device pointer as a tensor through the CUDA array interface
    class _Arr:
        __cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3}
    dev = torch.as_tensor(_Arr(), device="cuda")
    out.copy_(dev)
    return out.numpy()


def snapshot(engine, n: int):
    """(list of ImgDescC, function fetch(offset, nbytes) -> np.uint8 array) for the last chunk."""
    import torch
    torch.cuda.synchronize()
    lib = engine.lib
    sp, dp = ctypes.c_void_p(), ctypes.c_void_p()
    db, sb = ctypes.c_int64(), ctypes.c_int64()
    assert lib.sdsj_engine_debug_buffers(engine._h, ctypes.byref(sp), ctypes.byref(dp), ctypes.byref(db),
                                         ctypes.byref(sb)) == 0
    assert db.value == ctypes.sizeof(ImgDescC), (db.value, ctypes.sizeof(ImgDescC))
    raw = _memcpy_d2h(dp.value, db.value * n)
    descs = [ImgDescC.from_buffer_copy(raw[i * db.value:(i + 1) * db.value].tobytes()) for i in range(n)]

    def fetch(off: int, nbytes: int) -> np.ndarray:
        return _memcpy_d2h(sp.value + off, nbytes)

    return descs, fetch


def stage_report(engine, jpg: bytes, resolution=(256, 256)) -> list[str]:
    """Runs one image and compares each stage with the oracle; returns report lines."""
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from oracle import oracle as O
    out, st = engine.decode_resize([jpg], resolution)
    lines = [f"status {st.tolist()}"]
    d, fetch = snapshot(engine, 1)
    d = d[0]
    lines.append(f"desc: {d.width}x{d.height} ncomp={d.ncomp} bpm={d.bpm} mcu={d.mcux}x{d.mcuy} nseg={d.nseg} "
                 f"ulen={d.ulen} nsub={d.nsub} sub_bits={d.sub_bits} geo={d.geo} crop=({d.cx0},{d.cy0},{d.cw},{d.ch}) "
                 f"need_h={d.need_h} need_v={d.need_v} yf={d.yf} yl={d.yl} status={d.status}")
    # coefficients: device layout is decode order [g][64] in zigzag order; natural order for the comparison
    zz = fetch(d.off_coef, d.total_blocks * 128).view(np.int16).reshape(-1, 64)
    nat = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14,
           21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60,
           61, 54, 47, 55, 62, 63]
    coef = np.zeros_like(zz)
    coef[:, nat] = zz
    for c in range(d.ncomp):
        ref = O.coefficients(jpg, c)  # [bh][bw][64]
        cd = d.comp[c]
        got = np.zeros_like(ref)
        g = 0
        for m in range(d.mcux * d.mcuy):
            mx, my = m % d.mcux, m // d.mcux
            for b in range(d.bpm):
                cc = d.blk_comp[b]
                if d.ncomp == 1:
                    bx, by = mx, my
                else:
                    bx, by = mx * d.comp[cc].h + d.blk_dx[b], my * d.comp[cc].v + d.blk_dy[b]
                if cc == c:
                    got[by, bx] = coef[g]
                g += 1
        bad = np.argwhere((got != ref).any(-1))
        lines.append(f"coef comp{c}: {len(bad)} / {ref.shape[0] * ref.shape[1]} blocks differ "
                     f"{bad[:4].tolist()}")
    if not d.fused:  # the unfused path materialises the RGB rows
        rgb_ref = O.decode(jpg)
        h = d.src_y1 - d.src_y0
        rgb = fetch(d.off_rgb, d.src_w * h * 3).reshape(h, d.src_w, 3)
        ref_rows = rgb_ref[d.src_y0:d.src_y1, d.src_x0:d.src_x0 + d.src_w]
        lines.append(f"rgb rows: {int((rgb != ref_rows).any(-1).sum())} px differ of {rgb.shape[0] * rgb.shape[1]}")
    else:
        lines.append(f"fused resample, tile_w={d.tile_w}")
    ref_out = O.pipeline(jpg, resolution)
    got_out = out[0].cpu().numpy()
    lines.append(f"final: {int((got_out != ref_out).sum())} values differ")
    return lines


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from sds_amd.engine import JpegEngine
    from tests.golden.synth import synth_jpegs
    eng = JpegEngine()
    for line in stage_report(eng, synth_jpegs(1)[0]):
        print(line)
