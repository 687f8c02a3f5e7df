"""Debug aid for the unstuff passes: decodes the random-batch test images repeatedly and, for any image
whose status is not OK, compares the device's unstuffed stream and scan bookkeeping with a plain
Python unstuff.  usage (GPU box): python tools/us_debug.py [repeats]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def py_unstuff(ent: bytes):
    """jdhuff.c fill semantics: FF00 -> FF, fill FFs skipped, RSTn / codes < SOF0 split, others end."""
    out, marks, i = bytearray(), [], 0
    while i < len(ent):
        b = ent[i]
        if b != 0xFF:
            out.append(b)
            i += 1
            continue
        j = i + 1
        while j < len(ent) and ent[j] == 0xFF:
            j += 1
        if j >= len(ent):
            return bytes(out), marks, None
        c = ent[j]
        if c == 0:
            out.append(0xFF)
        elif 0xD0 <= c <= 0xD7 or c < 0xC0:
            marks.append((len(out), c))
        else:
            return bytes(out), marks, (j - 1, c)
        i = j + 1
    return bytes(out), marks, None


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    from sds_amd.engine import JpegEngine
    from tests.gpu_debug import snapshot
    from tests.test_gpu_parity import _random_jpegs
    eng = JpegEngine()
    for seed in (0, 1):
        jpgs = _random_jpegs(seed, 64)
        for rep in range(reps):
            _, st = eng.decode_resize(jpgs, (64, 64))
            bad = np.nonzero(st.cpu().numpy() if hasattr(st, "cpu") else st)[0].tolist()
            print(f"seed {seed} rep {rep}: bad {bad}", flush=True)
            if not bad:
                continue
            descs, fetch = snapshot(eng, len(jpgs))
            for k in bad:
                d = descs[k]
                ent = jpgs[k][d.entropy_off:d.entropy_off + d.entropy_len]
                ref, marks, end = py_unstuff(ent)
                got = fetch(d.off_ustream, max(d.ulen, 0) + 128).tobytes()
                tiles = fetch(d.off_tiles, d.ntiles * 16).view(np.int32).reshape(-1, 4).tolist()
                diff = [i for i in range(min(len(ref), d.ulen)) if got[i] != ref[i]]
                print(f"  img {k}: status {d.status} ulen {d.ulen} ref {len(ref)} useg {d.useg_found} ref {1 + len(marks)} "
                      f"end {d.scan_end_code}/{d.scan_end_raw} ref {end} ntiles {d.ntiles} tiles {tiles[:4]} "
                      f"nseg {d.nseg} first diffs {diff[:8]} pad_nonzero {sum(1 for x in got[d.ulen:d.ulen + 128] if x)}",
                      flush=True)


if __name__ == "__main__":
    main()
