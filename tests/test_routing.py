"""Field routing of the drop-in pipeline vs the reference (G4 goldens), on CPU.

The GPU decoder is replaced by a stand-in that returns the oracle's pixels in the engine's output
format (HWC storage), so this test checks the host-side routing bit-exactly: key set and order,
the encoded bytes left in ``image_field``, dtypes, shapes, strides, and the tensor bytes.
"""
import os
import tempfile

import numpy as np
import pytest
import torch

from oracle import oracle as O
from tests import goldens as G


class _StandInEngine:
    def decode_resize(self, jpgs, resolution, crop_before_resize=True, filter="bilinear", normalize=False,
                      flip=None, layout="chw", out=None):
        outs = []
        for k, j in enumerate(jpgs):
            chw = O.pipeline(j, resolution, crop_before_resize=crop_before_resize, filter=filter,
                             flip=bool(flip[k]) if flip else False, normalize=normalize)
            outs.append(torch.from_numpy(np.ascontiguousarray(chw.transpose(1, 2, 0) if layout == "hwc" else chw)))
        return torch.stack(outs), np.zeros(len(jpgs), np.int32)


def _describe(sample):
    out = []
    for k, v in sample.items():
        if isinstance(v, torch.Tensor):
            out.append([k, "tensor", str(v.dtype).replace("torch.", ""), list(v.shape), list(v.stride())])
        elif isinstance(v, bytes):
            out.append([k, "bytes", G.sha(v)])
        else:
            out.append([k, type(v).__name__, v])
    return out


@pytest.fixture()
def jpg_path():
    meta, jpgs = G.g2_jpegs()
    d = tempfile.mkdtemp()
    p = os.path.join(d, "0.jpg")
    with open(p, "wb") as f:
        f.write(jpgs[0])
    return p


@pytest.mark.parametrize("branch", list(G.load_json("g4_routing.json")["branches"]))
def test_routing_matches_reference(monkeypatch, jpg_path, branch):
    import sds_amd.presets as P
    monkeypatch.setattr(P, "get_engine", lambda device=None: _StandInEngine())
    g4 = G.load_json("g4_routing.json")
    entry = g4["branches"][branch]
    kw = dict(entry["kwargs"])
    kw["resolution"] = tuple(kw["resolution"])
    sample = {"index": 7, "jpg": jpg_path, "caption": "a cat", "__sample_key__": 7, "__data_type__": "IMAGE"}
    for t in P.create_standard_image_pipeline(**kw):
        sample = t(sample)
    assert _describe(sample) == entry["keys"]
    tkey = [k for k, v in sample.items() if isinstance(v, torch.Tensor)][0]
    assert G.sha(sample[tkey].contiguous().numpy()) == entry["tensor_sha256"]
    ens = P.EnsureFieldsTransform(fields_whitelist=["index", tkey], drop_others=True)
    assert _describe(ens(dict(sample))) == entry["after_ensure_drop_others"]


def test_transforms_are_picklable_without_native_state():
    import pickle

    import sds_amd.presets as P
    ts = P.create_standard_image_pipeline("jpg", (256, 256), normalize=True, return_image_as_single_frame_video=True)
    ts2 = pickle.loads(pickle.dumps(ts))
    assert [type(t).__name__ for t in ts2] == ["LoadFromDiskTransform", "GpuDecodeResizeImageTransform",
                                               "ReshapeImageAsVideoTransform", "FieldsFilteringTransform",
                                               "AugmentNewFieldsTransform"]


def test_ensure_fields_dummy_checks():
    import sds_amd.presets as P
    t = P.EnsureFieldsTransform(["a"], check_dummy_values=True)
    for bad in ({}, {"a": None}, {"a": ""}, {"a": []}, {"a": float("nan")}, {"a": torch.tensor([float("nan")])}):
        with pytest.raises(AssertionError):
            t(dict(bad))
    assert t({"a": 1}) == {"a": 1}


def test_hflip_prob_draws_the_global_torch_rng(monkeypatch, jpg_path):
    import sds_amd.presets as P
    monkeypatch.setattr(P, "get_engine", lambda device=None: _StandInEngine())
    ts = P.create_standard_image_pipeline("jpg", (64, 64), hflip_prob=0.5)
    torch.manual_seed(0)
    flips = []
    outs = []
    for _ in range(6):
        s = {"jpg": jpg_path}
        for t in ts:
            s = t(s)
        outs.append(s["image"])
    torch.manual_seed(0)
    for _ in range(6):
        flips.append(bool(torch.rand(1) < 0.5))
    base = torch.from_numpy(O.pipeline(open(jpg_path, "rb").read(), (64, 64)))
    for f, o in zip(flips, outs):
        assert torch.equal(o, torch.flip(base, dims=[2]) if f else base)
