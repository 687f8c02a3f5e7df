"""Baseline JPEGs written from chosen quantised coefficients (test input generator).

PIL's encoder only emits coefficients a forward DCT of 8-bit pixels can produce; the SIMD IDCT's 16-bit
semantics (libjpeg-turbo jidctint-avx2.asm: dequantisation wrapped to 16 bits, 16-bit sums, saturation
after each pass) only show on coefficients past that range, which damaged streams decode from garbage.
This writer produces such streams on purpose -- large DC sums, AC magnitudes up to 1023, quantisation
values up to 255 (8-bit DQT) or 65535 (16-bit DQT) -- as valid baseline files: SOF0, the Annex K
Huffman tables (taken from a PIL-encoded file's DHT segments, so no table is typed in here), one scan,
FF00 stuffing, EOI.  Used by the oracle-vs-PIL and GPU-vs-oracle tests of the IDCT.
"""
from __future__ import annotations

import io

import numpy as np

ZIGZAG_TO_NATURAL = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14,
    21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53,
    60, 61, 54, 47, 55, 62, 63])

_TABLES = None


def _annex_k_tables():
    """{(class, id): (bits[16], values)} from the DHT segments of a PIL baseline JPEG (standard tables)."""
    global _TABLES
    if _TABLES is None:
        from PIL import Image
        buf = io.BytesIO()
        Image.fromarray(np.zeros((16, 16, 3), np.uint8)).save(buf, format="JPEG", quality=90)
        d = buf.getvalue()
        tabs, i = {}, 2
        while i < len(d):
            m, ln = d[i + 1], (d[i + 2] << 8) | d[i + 3]
            if m == 0xC4:
                k = i + 4
                while k < i + 2 + ln:
                    tc, th = d[k] >> 4, d[k] & 15
                    bits = list(d[k + 1:k + 17])
                    vals = list(d[k + 17:k + 17 + sum(bits)])
                    tabs[(tc, th)] = (bits, vals)
                    k += 17 + sum(bits)
            if m == 0xDA:
                break
            i += 2 + ln
        _TABLES = tabs
    return _TABLES


def _codes(bits, vals):
    """Canonical Huffman codes (JPEG Annex C): symbol -> (code, length)."""
    out, code, k = {}, 0, 0
    for length in range(1, 17):
        for _ in range(bits[length - 1]):
            out[vals[k]] = (code, length)
            code += 1
            k += 1
        code <<= 1
    return out


class _BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, value: int, nbits: int):
        for b in range(nbits - 1, -1, -1):
            self.acc = (self.acc << 1) | ((value >> b) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0)
                self.acc = self.n = 0

    def flush(self):
        if self.n:
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)  # pad with ones


def _category(v: int) -> int:
    return int(abs(v)).bit_length()


def write_jpeg(w: int, h: int, comps, blocks, qtables, huff=None, order=None) -> bytes:
    """comps: [(h_samp, v_samp, tq)], 1 or 3 components; blocks: per component an int array
    [bh, bw, 64] of quantised coefficients in ZIGZAG order (DC as absolute values: the DPCM is done
    here); qtables: {tq: 64 values (zigzag order)}, a table with a value > 255 is written with 16-bit
    precision.  huff: per component its (DC, AC) table ids, default 0 for the first component and 1
    for the others; id 2 is a copy of the luma tables (Annex K ids 0) under its own id, so
    huff=[(0, 0), (1, 1), (2, 2)] makes a scan of 6 distinct table slots.  order: the components' order
    in the scan header (and so in each MCU), default the frame's."""
    tabs = dict(_annex_k_tables())
    tabs[(0, 2)], tabs[(1, 2)] = tabs[(0, 0)], tabs[(1, 0)]
    if huff is None:
        huff = [(0, 0) if ci == 0 else (1, 1) for ci in range(len(comps))]
    dc = [_codes(*tabs[(0, t)]) for t in range(3)]
    ac = [_codes(*tabs[(1, t)]) for t in range(3)]
    used = {(0, d) for d, _ in huff} | {(1, a) for _, a in huff}
    hmax = max(c[0] for c in comps)
    vmax = max(c[1] for c in comps)
    mcux = -(-w // (8 * hmax))
    mcuy = -(-h // (8 * vmax))
    seg = bytearray(b"\xff\xd8")

    def marker(m, payload):
        seg.extend(bytes([0xFF, m]) + (len(payload) + 2).to_bytes(2, "big") + payload)

    for tq, q in qtables.items():
        q = [int(v) for v in q]
        if max(q) > 255:
            marker(0xDB, bytes([0x10 | tq]) + b"".join(v.to_bytes(2, "big") for v in q))
        else:
            marker(0xDB, bytes([tq]) + bytes(q))
    sof = bytes([8]) + h.to_bytes(2, "big") + w.to_bytes(2, "big") + bytes([len(comps)])
    for ci, (hs, vs, tq) in enumerate(comps):
        sof += bytes([ci + 1, (hs << 4) | vs, tq])
    marker(0xC0, sof)
    for (tc, th), (bits, vals) in sorted(tabs.items()):
        if (tc, th) in used:
            marker(0xC4, bytes([(tc << 4) | th] + bits + vals))
    if order is None:
        order = list(range(len(comps)))
    sos = bytes([len(comps)])
    for ci in order:
        sos += bytes([ci + 1, (huff[ci][0] << 4) | huff[ci][1]])
    marker(0xDA, sos + bytes([0, 63, 0]))
    bw = _BitWriter()
    pred = [0] * len(comps)
    for my in range(mcuy):
        for mx in range(mcux):
            for ci in order:
                hs, vs, _ = comps[ci]
                td, ta = huff[ci]
                hh, vv = (hs, vs) if len(comps) > 1 else (1, 1)
                for dy in range(vv):
                    for dx in range(hh):
                        blk = blocks[ci][my * vv + dy, mx * hh + dx]
                        diff = int(blk[0]) - pred[ci]
                        pred[ci] = int(blk[0])
                        s = _category(diff)
                        code, ln = dc[td][s]
                        bw.put(code, ln)
                        if s:
                            bw.put(diff if diff > 0 else diff - 1 + (1 << s), s)
                        run = 0
                        last = max([k for k in range(1, 64) if blk[k] != 0], default=0)
                        for k in range(1, last + 1):
                            v = int(blk[k])
                            if v == 0:
                                run += 1
                                continue
                            while run > 15:
                                code, ln = ac[ta][0xF0]
                                bw.put(code, ln)
                                run -= 16
                            s = _category(v)
                            code, ln = ac[ta][(run << 4) | s]
                            bw.put(code, ln)
                            bw.put(v if v > 0 else v - 1 + (1 << s), s)
                            run = 0
                        if last < 63:
                            code, ln = ac[ta][0x00]
                            bw.put(code, ln)
    bw.flush()
    seg.extend(bw.out)
    seg.extend(b"\xff\xd9")
    return bytes(seg)


def extreme_jpegs(seed: int, n: int) -> list[bytes]:
    """Random small baseline JPEGs whose dequantised coefficients leave 16 bits: per block, one of
    DC-only (rows 1..7 zero: the SIMD pass-1 shortcut), sparse large AC terms, dense AC terms, or a
    block with only row 0 non-zero; DC values drifting to the int16 limits; quantisation tables of
    random 8-bit values, all-255, or 16-bit values.  Gray, 4:4:4, 4:2:2 and 4:2:0."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        kind = i % 4
        comps = [[(1, 1, 0)], [(1, 1, 0), (1, 1, 1), (1, 1, 1)], [(2, 1, 0), (1, 1, 1), (1, 1, 1)],
                 [(2, 2, 0), (1, 1, 1), (1, 1, 1)]][kind]
        w, h = int(rng.integers(1, 48)), int(rng.integers(1, 48))
        hmax, vmax = max(c[0] for c in comps), max(c[1] for c in comps)
        mcux, mcuy = -(-w // (8 * hmax)), -(-h // (8 * vmax))
        blocks = []
        for hs, vs, _ in comps:
            hh, vv = (hs, vs) if len(comps) > 1 else (1, 1)
            bh, bwid = mcuy * vv, mcux * hh
            b = np.zeros((bh, bwid, 64), np.int64)
            for y in range(bh):
                for x in range(bwid):
                    t = int(rng.integers(0, 4))
                    if t == 1:
                        for k in rng.choice(np.arange(1, 64), int(rng.integers(1, 6)), replace=False):
                            b[y, x, k] = int(rng.integers(-1023, 1024))
                    elif t == 2:
                        b[y, x, 1:] = rng.integers(-1023, 1024, 63)
                    elif t == 3:  # only natural row 0 (zigzag 1, 5, 6, 14, 15, 27, 28)
                        for k in (1, 5, 6, 14, 15, 27, 28):
                            b[y, x, k] = int(rng.integers(-1023, 1024))
            blocks.append(b)
        # DC values: a random walk in coding (MCU) order, steps within the DC table's 11-bit range
        for ci, (hs, vs, _) in enumerate(comps):
            hh, vv = (hs, vs) if len(comps) > 1 else (1, 1)
            dcv = 0
            for my in range(mcuy):
                for mx in range(mcux):
                    for dy in range(vv):
                        for dx in range(hh):
                            dcv = int(np.clip(dcv + rng.integers(-2047, 2048), -32767, 32767))
                            blocks[ci][my * vv + dy, mx * hh + dx, 0] = dcv
        qk = i % 3
        qtabs = {}
        for tq in range(2 if len(comps) > 1 else 1):
            if qk == 0:
                qtabs[tq] = rng.integers(1, 256, 64)
            elif qk == 1:
                qtabs[tq] = np.full(64, 255)
            else:
                qtabs[tq] = rng.integers(1, 65536, 64)
        out.append(write_jpeg(w, h, comps, blocks, qtabs))
    return out


def six_slot_jpegs(seed: int, n: int, w: int = 160, h: int = 120, order=None) -> list[bytes]:
    """Baseline 4:2:0 / 4:4:4 JPEGs whose Cb and Cr components use their own DC/AC Huffman tables
    (ids 1 and 2: 6 distinct table slots, the kernels' 10-bit entropy route), with natural-looking
    coefficients: a DC random walk and a few small low-frequency AC terms per block."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        comps = [(2, 2, 0), (1, 1, 1), (1, 1, 1)] if i % 2 == 0 else [(1, 1, 0), (1, 1, 1), (1, 1, 1)]
        hmax, vmax = max(c[0] for c in comps), max(c[1] for c in comps)
        mcux, mcuy = -(-w // (8 * hmax)), -(-h // (8 * vmax))
        blocks = []
        for hs, vs, _ in comps:
            bh, bwid = mcuy * vs, mcux * hs
            b = np.zeros((bh, bwid, 64), np.int64)
            nz = rng.integers(0, 12, (bh, bwid))
            for y in range(bh):
                for x in range(bwid):
                    k = rng.choice(np.arange(1, 40), int(nz[y, x]), replace=False)
                    b[y, x, k] = rng.integers(-40, 41, len(k))
            blocks.append(b)
        for ci, (hs, vs, _) in enumerate(comps):
            dcv = 0
            for my in range(mcuy):
                for mx in range(mcux):
                    for dy in range(vs):
                        for dx in range(hs):
                            dcv = int(np.clip(dcv + rng.integers(-60, 61), -1000, 1000))
                            blocks[ci][my * vs + dy, mx * hs + dx, 0] = dcv
        q = {0: rng.integers(2, 40, 64), 1: rng.integers(2, 60, 64)}
        out.append(write_jpeg(w, h, comps, blocks, q, huff=[(0, 0), (1, 1), (2, 2)], order=order))
    return out
