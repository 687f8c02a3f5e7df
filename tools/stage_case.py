#!/usr/bin/env python3
"""Stage-by-stage report (unstuffed stream, coefficients, output) of one G1 golden case or of a synthetic
VGA image against the oracle (debugging aid, test infrastructure).  usage: stage_case.py <g1 name | synth>"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def unstuff_ref(jpg: bytes, off: int) -> bytes:
    out = bytearray()
    i = off
    while i < len(jpg):
        c = jpg[i]
        if c == 0xFF:
            j = i + 1
            while j < len(jpg) and jpg[j] == 0xFF:
                j += 1
            if j < len(jpg) and jpg[j] == 0:
                out.append(0xFF)
                i = j + 1
                continue
            if j < len(jpg) and 0xD0 <= jpg[j] <= 0xD7:
                i = j + 1
                continue
            break
        out.append(c)
        i += 1
    return bytes(out)


def main():
    from oracle import oracle as O
    from sds_amd.engine import JpegEngine
    from tests import goldens as G
    from tests.gpu_debug import snapshot, stage_report
    name = sys.argv[1]
    if name == "synth":
        from tests.golden.synth import synth_jpegs
        jpg = synth_jpegs(1)[0]
    else:
        jpg = next(j for c, j, _ in G.g1() if c["name"] == name)
    eng = JpegEngine("cuda:0", max_batch=8)
    for line in stage_report(eng, jpg):
        print(line)
    d, fetch = snapshot(eng, 1)
    d = d[0]
    ref = unstuff_ref(jpg, d.entropy_off)
    got = fetch(d.off_ustream, d.ulen).tobytes()
    print(f"ustream: gpu {d.ulen} B, ref {len(ref)} B, nseg {d.nseg} found {d.useg_found}")
    n = min(len(ref), len(got))
    diff = [i for i in range(n) if ref[i] != got[i]]
    print(f"first differing bytes: {diff[:10]}")
    if diff:
        i = diff[0]
        print("gpu", got[max(0, i - 8):i + 8].hex(), "ref", ref[max(0, i - 8):i + 8].hex())
    pad = fetch(d.off_ustream + d.ulen, 128).tobytes()
    print("pad zero:", pad == bytes(128))


if __name__ == "__main__":
    main()
