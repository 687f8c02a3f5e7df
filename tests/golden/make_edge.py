#!/usr/bin/env python3
"""Generates tests/golden/g5_edge.json: header/table/termination edge cases decoded by the REFERENCE.

Run in the build container only (it needs /root/reference):  python3 -B tests/golden/make_edge.py

Each case is a small JPEG built here from a Pillow-encoded base by editing markers (no reference
source involved).  The outcome is what the reference's own ``load_image_from_bytes``
(sds/transforms/functional.py:94-100, imported unmodified through make_golden.import_reference)
does with it: "ok" plus the SHA-256 of the decoded RGB, or the exception type.  What the cases pin
(libjpeg-turbo 3.1.4 behaviour behind Pillow 12.2.0):
  * only the Huffman tables the scan uses are derived/validated (jdhuff.c start_pass_huff_decoder);
  * DC tables with a symbol > 15 are rejected (jpeg_make_d_derived_tbl, JERR_BAD_HUFF_TABLE);
  * a missing EOI / a cut stream raises (Pillow: "image file is truncated");
  * fill bytes (FF FF ...) before a marker are skipped (jdmarker.c next_marker);
  * markers after the scan are read up to EOI (jdmarker.c read_markers): segments are skipped or
    checked, a second SOI/SOF/SOS or an unknown marker raises;
  * a marker inside the scan ends its data: zero fill, then uniform gray (jdhuff.c insufficient_data).
"""
from __future__ import annotations

import base64
import hashlib
import io
import json
import os
import struct
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def _dht_tables(j: bytes):
    """Yields (value offset, count, tc, th) of every Huffman table in every DHT segment."""
    i = 0
    while True:
        i = j.find(b"\xff\xc4", i)
        if i < 0:
            return
        n = struct.unpack(">H", j[i + 2:i + 4])[0]
        s, e = i + 4, i + 2 + n
        while s < e:
            t = j[s]
            cnt = sum(j[s + 1:s + 17])
            yield s + 17, cnt, t >> 4, t & 15
            s += 17 + cnt
        i = e


def cases():
    import numpy as np
    from PIL import Image
    sys.path.insert(0, REPO)
    from tests.golden.synth import synth_rgb
    rng = np.random.default_rng(5150)
    b = io.BytesIO()
    Image.fromarray(synth_rgb(rng, 40, 24)).save(b, "JPEG", quality=90)
    base = b.getvalue()
    sos = base.index(b"\xff\xda")
    out = {"base": base}
    # an extra, unused, over-subscribed DC table (id 3): three 1-bit codes
    bad = bytes([0x03]) + bytes([3] + [0] * 15) + bytes([0, 1, 2])
    out["unused_oversubscribed_dht"] = base[:sos] + b"\xff\xc4" + struct.pack(">H", 2 + len(bad)) + bad + base[sos:]
    # an unused DC table (id 2) holding symbol 16
    dc16 = bytes([0x02]) + bytes([0, 2] + [0] * 14) + bytes([0, 16])
    out["unused_dc_symbol_16"] = base[:sos] + b"\xff\xc4" + struct.pack(">H", 2 + len(dc16)) + dc16 + base[sos:]
    # the luma DC table (used) with its last symbol replaced by 16
    vo, cnt, _, _ = next(t for t in _dht_tables(base) if t[2] == 0 and t[3] == 0)
    j = bytearray(base)
    j[vo + cnt - 1] = 16
    out["used_dc_symbol_16"] = bytes(j)
    # fill bytes before the SOS marker and before EOI
    out["fill_bytes_before_markers"] = base[:sos] + b"\xff\xff\xff" + base[sos:-2] + b"\xff\xff" + base[-2:]
    out["missing_eoi"] = base[:-2]
    out["cut_in_scan"] = base[:sos + (len(base) - sos) * 2 // 3]
    # what follows the scan (jdmarker.c read_markers up to EOI)
    sos_seg = base[sos:sos + 2 + struct.unpack(">H", base[sos + 2:sos + 4])[0]]
    body = base[:-2]
    out["after_scan_tem_rst_dnl_dqt"] = (body + b"\xff\x01\xff\xd0\xff\xdc\x00\x04\x00\x18" +
                                         b"\xff\xdb\x00\x43\x00" + bytes(range(1, 65)) + b"\xff\xd9")
    out["after_scan_app_com"] = body + b"\xff\xe5\x00\x04ab\xff\xfe\x00\x05abc\xff\xd9"
    out["after_scan_second_sos"] = body + sos_seg + b"\x00\x00\xff\xd9"
    out["after_scan_soi"] = body + b"\xff\xd8\xff\xd9"
    out["after_scan_unknown_marker"] = body + b"\xff\x85\xff\xd9"
    out["after_scan_bad_dht"] = body + b"\xff\xc4\x00\x05\x00\x01\x02\xff\xd9"
    out["after_scan_jpg0"] = body + b"\xff\xf0\x00\x04ab\xff\xd9"
    out["garbage_after_eoi"] = base + b"\xff\x85garbage"
    # premature markers inside the scan: libjpeg zero-fills (JWRN_HIT_MARKER) and leaves the rest gray
    mid = sos + len(sos_seg) + (len(base) - sos - len(sos_seg)) // 2
    if base[mid - 1] == 0xFF:
        mid += 1
    out["eoi_mid_scan"] = base[:mid] + b"\xff\xd9"
    out["rst_mid_scan_no_dri"] = base[:mid] + b"\xff\xd3" + base[mid:]
    return out


def main():
    from make_golden import import_reference
    P = import_reference()
    import numpy as np
    F = sys.modules["sds.transforms.functional"]
    res = []
    for name, jpg in cases().items():
        try:
            rgb = np.asarray(F.load_image_from_bytes(jpg))
            r = {"name": name, "outcome": "ok", "rgb_sha256": hashlib.sha256(np.ascontiguousarray(rgb).tobytes()).hexdigest(),
                 "size": [int(rgb.shape[1]), int(rgb.shape[0])]}
        except Exception as e:  # noqa: BLE001 -- the exception type is the recorded outcome
            r = {"name": name, "outcome": type(e).__name__}
        r["jpg_b64"] = base64.b64encode(jpg).decode()
        res.append(r)
        print(name, r["outcome"])
    del P
    with open(os.path.join(HERE, "g5_edge.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_edge.py (reference functional.load_image_from_bytes)",
                   "cases": res}, f, indent=1)


if __name__ == "__main__":
    sys.path.insert(0, HERE)
    main()
