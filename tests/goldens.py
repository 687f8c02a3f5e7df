"""Helpers to load the committed golden vectors (tests/golden/, made by make_golden.py)."""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(a) -> str:
    if isinstance(a, (bytes, bytearray)):
        return hashlib.sha256(a).hexdigest()
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def g1():
    """Yields (case dict, jpg bytes, arrays dict) for each G1 case."""
    with open(os.path.join(GOLDEN, "g1_cases.json")) as f:
        cases = json.load(f)
    z = np.load(os.path.join(GOLDEN, "g1_small.npz"))
    for c in cases:
        name = c["name"]
        jpg = z[f"{name}__jpg"].tobytes()
        arrs = {k[len(name) + 2:]: z[k] for k in z.files if k.startswith(name + "__")}
        yield c, jpg, arrs


def load_json(name: str):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def g2_jpegs():
    from tests.golden.synth import synth_jpegs
    meta = load_json("g2_synth.json")
    jpgs = synth_jpegs(len(meta["images"]), seed=meta["seed"], w=meta["w"], h=meta["h"], quality=meta["quality"])
    return meta, jpgs


def g3_jpegs():
    from tests.golden.synth import encode_jpeg, synth_rgb
    meta = load_json("g3_mixed.json")
    rng = np.random.default_rng(777)
    jpgs = [encode_jpeg(synth_rgb(rng, im["w"], im["h"]), 90) for im in meta["images"]]
    return meta, jpgs
