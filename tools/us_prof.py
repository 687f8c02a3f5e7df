"""Per-phase cycle counts of k_us_serial (build with SDSJ_CFLAGS=-DSDSJ_US_PROF; GPU box):
classify (loads + masks), tile end (atomicMin + 3 barriers), place (scan, LDS assembly, stores)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402


def main():
    from sds_amd.engine import JpegEngine
    from tests.gpu_debug import snapshot
    from tests.golden.synth import synth_jpegs
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    base = synth_jpegs(64, seed=2024)
    jpgs = [base[i % 64] for i in range(n)]
    eng = JpegEngine(max_batch=n, scratch_bytes=int(7e6 * n))
    eng.set_lanes(1)
    for _ in range(3):
        eng.decode_resize(jpgs, (256, 256))
    descs, _ = snapshot(eng, n)
    ph = np.array([[d.t_rs[k] for k in range(4)] for d in descs], dtype=np.float64)
    tiles = ph[:, 3].sum()
    print(f"images {n} tiles/image {tiles / n:.1f} cycles per tile: classify {ph[:, 0].sum() / tiles:.0f} "
          f"tile_end {ph[:, 1].sum() / tiles:.0f} place {ph[:, 2].sum() / tiles:.0f}")


if __name__ == "__main__":
    main()
