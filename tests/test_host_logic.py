"""Host-side logic of the drop-in (no GPU): crop boxes, target resolution, filters, sharding."""
import numpy as np
import pytest

from oracle import oracle as O
from sds_amd import functional as F
from sds_amd.distributed import compute_index_slice


def test_crop_box_matches_oracle_and_reference_formula():
    rng = np.random.default_rng(0)
    for _ in range(2000):
        w, h = int(rng.integers(1, 5000)), int(rng.integers(1, 5000))
        oh, ow = int(rng.integers(1, 2000)), int(rng.integers(1, 2000))
        assert F.crop_box(w, h, oh, ow) == O.crop_box(w, h, oh, ow)


def test_target_resolution_allow_vertical():
    # functional.py:76: vertical images swap to (max, min) when allow_vertical
    assert F.target_resolution(480, 640, (256, 512), allow_vertical=True) == (512, 256)
    assert F.target_resolution(640, 480, (256, 512), allow_vertical=True) == (256, 512)
    assert F.target_resolution(480, 640, (256, 512), allow_vertical=False) == (256, 512)


def test_target_resolution_random_resize_uses_numpy_global_rng():
    rr = {(128, 128): 0.5, (64, 64): 0.5, (4096, 4096): 0.0}
    np.random.seed(3)
    got = [F.target_resolution(640, 480, (256, 256), random_resize=rr) for _ in range(20)]
    np.random.seed(3)
    exp = []
    for _ in range(20):
        kept = {k: v for k, v in rr.items() if k[0] <= 640 and k[1] <= 480}
        res, probs = zip(*kept.items())
        exp.append(res[np.random.choice(len(res), p=np.array(probs) / sum(probs))])
    assert got == [tuple(int(v) for v in e) for e in exp]


def test_filter_names():
    assert F.filter_name("bilinear") == "bilinear"

    class Mode:  # torchvision InterpolationMode stand-in
        value = "bicubic"
    assert F.filter_name(Mode()) == "bicubic"
    # torchvision pil_modes_mapping: NEAREST and NEAREST_EXACT both resize PIL images with PIL NEAREST
    assert F.filter_name("nearest") == "nearest"
    assert F.filter_name("nearest-exact") == "nearest"

    class Exact:
        value = "nearest-exact"
    assert F.filter_name(Exact()) == "nearest"
    with pytest.raises(ValueError):  # TVF.InterpolationMode('cubic') raises ValueError
        F.filter_name("cubic")
    with pytest.raises(TypeError):
        F.check_resize_kwargs({"antialias": True})


def test_compute_index_slice_matches_reference_inter_node():
    # sds/index.py:235-246 (INTER_NODE): per_rank = N // R; start = r*per_rank (or r); step 1 (or R)
    for n in (0, 1, 7, 100, 1_000_000):
        for R in (1, 2, 3, 8):
            seen = []
            for r in range(R):
                s, e, st = compute_index_slice(n, r, R)
                assert (s, e, st) == (r * (n // R), min(r * (n // R) + n // R, n), 1)
                seen.extend(range(s, e, st))
                si, ei, sti = compute_index_slice(n, r, R, interleaved=True)
                assert (si, sti) == (r, R) and ei == min(r + (n // R) * R, n)
            assert seen == list(range(R * (n // R)))


def test_engine_needs_a_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from sds_amd.engine import JpegEngine
    with pytest.raises(RuntimeError):
        JpegEngine()
