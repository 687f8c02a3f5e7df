#!/usr/bin/env python3
"""Runs one G1 golden case through the GPU engine (SDSJ_LIBRARY selects the build) and prints the
per-channel mismatch against the golden outputs (debugging aid)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import numpy as np

    from sds_amd.engine import JpegEngine
    from tests import goldens as G
    name = sys.argv[1]
    eng = JpegEngine("cuda:0", max_batch=8)
    for case, jpg, arrs in G.g1():
        if case["name"] != name:
            continue
        for key in case["outputs"]:
            res = tuple(int(v) for v in key.split("x"))
            got, st = eng.decode_resize([jpg], res)
            g = got[0].cpu().numpy().astype(int)
            ref = arrs[f"out_{key}"].astype(int)
            bad = [(c, int((g[c] != ref[c]).sum()), np.argwhere(g[c] != ref[c])[:3].tolist()) for c in range(3)]
            print(name, key, "status", int(st[0]), bad)


if __name__ == "__main__":
    main()
