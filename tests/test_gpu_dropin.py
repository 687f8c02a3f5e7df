"""The per-sample drop-in (sds_amd.presets.create_standard_image_pipeline(..., device="cuda")) on the GPU:
the transform list the reference's factory returns (presets.py:716-744), run sample by sample as
sds/dataset.py:535-561 runs it, against the reference-generated goldens (G2, G3, G4) -- including
crop_before_resize=False and normalize with the single-frame-video branch -- and inside torch
DataLoader workers (examples/iter_image_dataset.py:72-80 shape, each case in a fresh process)."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from tests import goldens as G  # noqa: E402
from tests.test_routing import _describe  # noqa: E402

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _write(tmp, name, data):
    p = os.path.join(tmp, name)
    with open(p, "wb") as f:
        f.write(data)
    return p


def _run(transforms, sample):
    for t in transforms:
        sample = t(sample)
    return sample


def test_pipeline_on_g2_matches_reference_goldens():
    from sds_amd.presets import create_standard_image_pipeline
    meta, jpgs = G.g2_jpegs()
    tmp = tempfile.mkdtemp()
    ts = create_standard_image_pipeline("jpg", (256, 256), device="cuda")
    tn = create_standard_image_pipeline("jpg", (256, 256), normalize=True, device="cuda")
    for i, j in enumerate(jpgs):
        p = _write(tmp, f"{i}.jpg", j)
        s = _run(ts, {"index": i, "jpg": p})
        img = s["image"]
        assert img.device.type == "cuda" and img.dtype == torch.uint8 and tuple(img.shape) == (3, 256, 256)
        assert img.stride() == (1, 768, 3)  # the reference's HWC storage viewed as CHW (functional.py:104-108)
        assert s["jpg"] == j  # LoadFromDiskTransform leaves the encoded bytes in the image field
        assert G.sha(img.cpu().contiguous().numpy()) == meta["images"][i]["u8_256_sha256"]
        f = _run(tn, {"index": i, "jpg": p})["image"]
        assert f.dtype == torch.float32
        assert G.sha(f.cpu().contiguous().numpy()) == meta["images"][i]["f32_256_sha256"]


def test_pipeline_on_g3_mixed_sizes_with_flip_and_normalize():
    from sds_amd.presets import create_standard_image_pipeline
    meta, jpgs = G.g3_jpegs()
    tmp = tempfile.mkdtemp()
    for i, (im, j) in enumerate(zip(meta["images"], jpgs)):
        p = _write(tmp, f"{i}.jpg", j)
        hp = 1.0 if im["flip"] else 0.0  # torch.rand(1) < 1.0 always flips, < 0.0 never
        u8 = _run(create_standard_image_pipeline("jpg", (512, 512), device="cuda", hflip_prob=hp), {"jpg": p})
        f32 = _run(create_standard_image_pipeline("jpg", (512, 512), normalize=True, device="cuda", hflip_prob=hp),
                   {"jpg": p})
        assert G.sha(u8["image"].cpu().contiguous().numpy()) == im["u8_512_sha256"], im
        assert G.sha(f32["image"].cpu().contiguous().numpy()) == im["f32_512_sha256"], im


@pytest.mark.parametrize("branch", list(G.load_json("g4_routing.json")["branches"]))
def test_routing_branches_on_gpu(branch):
    """G4 with the real GPU engine: key order/values, the tensor's bytes (rect_no_crop is
    crop_before_resize=False; video_normalize_custom_fields is normalize + single-frame video)."""
    from sds_amd.presets import EnsureFieldsTransform, create_standard_image_pipeline
    meta, jpgs = G.g2_jpegs()
    p = _write(tempfile.mkdtemp(), "0.jpg", jpgs[0])
    entry = G.load_json("g4_routing.json")["branches"][branch]
    kw = dict(entry["kwargs"])
    kw["resolution"] = tuple(kw["resolution"])
    sample = {"index": 7, "jpg": p, "caption": "a cat", "__sample_key__": 7, "__data_type__": "IMAGE"}
    sample = _run(create_standard_image_pipeline(device="cuda", **kw), sample)
    tkey = [k for k, v in sample.items() if isinstance(v, torch.Tensor)][0]
    assert sample[tkey].device.type == "cuda"
    cpu = {k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in sample.items()}
    assert _describe(cpu) == entry["keys"]
    assert G.sha(cpu[tkey].contiguous().numpy()) == entry["tensor_sha256"]
    ens = EnsureFieldsTransform(fields_whitelist=["index", tkey], drop_others=True, check_dummy_values=True)
    out = ens(dict(sample))  # the dummy check runs torch.isnan on the device tensor
    assert _describe({k: (v.cpu() if isinstance(v, torch.Tensor) else v) for k, v in out.items()}) == \
        entry["after_ensure_drop_others"]


def test_output_device_cpu_returns_the_reference_type():
    from sds_amd.presets import create_standard_image_pipeline
    meta, jpgs = G.g2_jpegs()
    p = _write(tempfile.mkdtemp(), "0.jpg", jpgs[0])
    s = _run(create_standard_image_pipeline("jpg", (256, 256), device="cuda", output_device="cpu"), {"jpg": p})
    assert s["image"].device.type == "cpu" and s["image"].stride() == (1, 768, 3)
    assert G.sha(s["image"].contiguous().numpy()) == meta["images"][0]["u8_256_sha256"]


def _g6():
    meta = G.load_json("g6_fallback.json")
    z = np.load(os.path.join(G.GOLDEN, "g6_fallback.npz"))
    return meta, z


def test_fallback_samples_match_reference_g6():
    """SURVEY.md §8(b) UNSUPPORTED / CORRUPT contract: PNG (RGB, RGBA, L, P), WebP, GIF, BMP, TIFF, a
    CMYK JPEG and a JPEG without EOI (which the GPU parser reports truncated, and Pillow decodes) rerun on
    PIL on the host and are resized on the GPU: equal to the reference pipeline's outputs (G6, made by
    tests/golden/make_fallback.py from the reference itself) in every variant (two resolutions,
    normalize, crop_before_resize=False); samples the reference fails on raise its OSError."""
    from sds_amd.engine import get_engine
    from sds_amd.presets import create_standard_image_pipeline
    meta, z = _g6()
    eng = get_engine("cuda")
    before = eng.counters()
    tmp = tempfile.mkdtemp()
    n_ok = 0
    for case in meta["cases"]:
        data = z[f"{case['name']}__bytes"].tobytes()
        p = _write(tmp, case["name"], data)
        for vname, res, kw in meta["variants"]:
            ref = case["variants"][vname]
            ts = create_standard_image_pipeline("img", tuple(res), device="cuda", **kw)
            if not ref["ok"]:
                with pytest.raises(OSError):
                    _run(ts, {"img": p})
                continue
            img = _run(ts, {"img": p})["image"]
            assert img.device.type == "cuda" and list(img.shape) == ref["shape"], (case["name"], vname)
            assert str(img.dtype).replace("torch.", "") == ref["dtype"]
            h, w = ref["shape"][1:]
            assert img.stride() == (1, w * 3, 3)  # HWC storage viewed as CHW, as the reference's tensor
            got = img.cpu().contiguous().numpy()
            if f"{case['name']}__{vname}" in z.files:
                np.testing.assert_array_equal(got, z[f"{case['name']}__{vname}"], err_msg=f"{case['name']} {vname}")
            assert G.sha(got) == ref["sha256"], (case["name"], vname)
            n_ok += 1
    after = eng.counters()
    assert n_ok >= 40
    assert after["fallback"] - before["fallback"] == n_ok


def test_fallback_in_gpu_decode_batch():
    """f1 (sds_amd.batched.GpuDecodeBatch): a collated batch mixing JPEGs with G6 samples -- the fallback
    rows equal the reference's images, the sample the reference fails on is dropped from every field."""
    from sds_amd.batched import GpuDecodeBatch
    meta, z = _g6()
    _, jpgs = G.g2_jpegs()
    names = ["png_rgb_64x48", "png_truncated", "jpeg_cmyk_48x32", "webp_64x48", "jpeg_no_eoi_64x48"]
    enc = [jpgs[0]] + [z[f"{n}__bytes"].tobytes() for n in names] + [jpgs[1]]
    batch = {"img": enc, "index": torch.arange(len(enc))}
    out = GpuDecodeBatch("img", (32, 32), device="cuda")(batch)
    assert out["index"].tolist() == [0, 1, 3, 4, 5, 6]
    imgs = out["image"].cpu().numpy()
    for row, n in zip(imgs[1:5], [names[0], names[2], names[3], names[4]]):
        np.testing.assert_array_equal(row, z[f"{n}__r32"], err_msg=n)
    with pytest.raises(OSError):
        GpuDecodeBatch("img", (32, 32), device="cuda", on_error="raise")({"img": enc})


def _g7_data(case, g1, g2, g3, z):
    if case["source"] == "g1":
        return g1[case["name"]]
    if case["source"] == "g2":
        return g2[case["index"]]
    if case["source"] == "g3":
        return g3[case["index"]]
    return z[f"{case['name']}__bytes"].tobytes()


def test_nearest_interpolation_matches_reference_g7():
    """resize_kwargs interpolation_mode 'nearest' / 'nearest-exact' (functional.py:84: torchvision maps both
    to PIL NEAREST for PIL images): Pillow's ImagingScaleAffine source indices as one-tap GPU resamples,
    equal to G7 (tests/golden/make_nearest.py, made by the reference pipeline) -- G2 at 256, G3's mixed
    sizes at 512 (allow_vertical on the portrait ones), small 4:2:0 / 4:2:2 / 4:4:4 / gray / progressive
    JPEGs with upscaling, no crop and normalize, and a PNG through the host-decode route."""
    from sds_amd.presets import create_standard_image_pipeline
    meta = G.load_json("g7_nearest.json")
    z = np.load(os.path.join(G.GOLDEN, "g7_nearest.npz"))
    g1 = {c["name"]: jpg for c, jpg, _ in G.g1()}
    g2, g3 = G.g2_jpegs()[1], G.g3_jpegs()[1]
    tmp = tempfile.mkdtemp()
    n = 0
    for case in meta["cases"]:
        p = _write(tmp, case["name"], _g7_data(case, g1, g2, g3, z))
        for vname, ref in case["variants"].items():
            ts = create_standard_image_pipeline("img", tuple(ref["resolution"]), device="cuda", **ref["kwargs"])
            if not ref["ok"]:
                with pytest.raises(OSError):
                    _run(ts, {"img": p})
                continue
            img = _run(ts, {"img": p})["image"]
            assert img.device.type == "cuda" and list(img.shape) == ref["shape"], (case["name"], vname)
            got = img.cpu().contiguous().numpy()
            key = f"{case['name']}__{vname}"
            if key in z.files:
                np.testing.assert_array_equal(got, z[key], err_msg=key)
            assert G.sha(got) == ref["sha256"], key
            n += 1
    assert n >= 70


def test_corrupt_jpeg_with_random_resize_draws_the_np_rng_once():
    """A JPEG the GPU reports CORRUPT while its header probes fine (no EOI, which Pillow decodes) reruns
    on PIL: with random_resize the reference draws np.random.choice once, after its decode
    (functional.py:69-74), so the global numpy state afterwards equals one draw from the state before."""
    from sds_amd.presets import create_standard_image_pipeline
    meta, z = _g6()
    data = z["jpeg_no_eoi_64x48__bytes"].tobytes()
    p = _write(tempfile.mkdtemp(), "no_eoi.jpg", data)
    rr = {(16, 16): 0.25, (24, 32): 0.25, (32, 32): 0.5}
    ts = create_standard_image_pipeline("img", (32, 32), device="cuda", resize_kwargs={"random_resize": rr})
    for seed in range(6):
        np.random.seed(seed)
        img = _run(ts, {"img": p})["image"]
        got_state = np.random.get_state()[1].copy()
        np.random.seed(seed)
        res, probs = zip(*rr.items())
        choice = res[np.random.choice(len(res), p=np.array(probs) / sum(probs))]
        assert np.array_equal(got_state, np.random.get_state()[1]), seed
        assert tuple(img.shape[1:]) == tuple(choice), (seed, choice)


def _case(name):
    env = dict(os.environ)
    r = subprocess.run([sys.executable, "-m", "tests.loader_cases", name], capture_output=True, text=True,
                       timeout=240, cwd=REPO, env=env)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert r.returncode == 0 and lines, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])
    return json.loads(lines[-1])


def test_dataloader_workers_yield_device_tensors_equal_to_goldens():
    rec = _case("workers_device")
    assert "error" not in rec, rec
    assert rec["device"].startswith("cuda") and rec["n"] == 8 and rec["equal_to_goldens"], rec


def test_dataloader_persistent_workers_serve_every_epoch():
    rec = _case("workers_device_persistent_two_epochs")
    assert "error" not in rec, rec
    assert rec["epochs"] == 2 and rec["equal_to_goldens"], rec


def test_dataloader_refork_after_device_tensors_fails_with_a_clear_error():
    """Non-persistent workers are forked again for epoch 2, from a parent that has received device
    tensors (HIP initialised): the transform's error names the working set-ups."""
    rec = _case("workers_device_two_epochs")
    assert "persistent" in rec.get("error", "") or "GpuDecodeBatch" in rec.get("error", ""), rec


def test_dataloader_reference_shape_through_the_decode_service():
    """examples/iter_image_dataset.py:72-80's DataLoader arguments unchanged (fork, num_workers=2,
    pin_memory=True) over the default pipeline: the workers decode through the node-local service
    (sds_amd/service.py) and yield pinned host tensors -- the reference's type -- equal to G2."""
    rec = _case("service_reference_shape")
    assert "error" not in rec, rec
    assert rec["service"] and rec["device"] == "cpu" and rec["pinned"] and rec["n"] == 8, rec
    assert rec["stride"] == [3 * 256 * 256, 256 * 256, 256, 1] and rec["equal_to_goldens"], rec  # (collated)


def test_decode_service_after_parent_gpu_init():
    """The parent initialises HIP after building the pipeline and before its workers fork: the workers
    never touch HIP (the service decodes), so the fork is harmless."""
    rec = _case("service_parent_touched_gpu")
    assert "error" not in rec, rec
    assert rec["pinned"] and rec["equal_to_goldens"], rec


def test_decode_service_g3_mixed_sizes_flip_normalize():
    rec = _case("service_g3_flip_normalize")
    assert "error" not in rec and rec["equal_to_goldens"], rec


def test_decode_service_random_resize_matches_the_oracle():
    """random_resize through the service (fork, 4 workers, pin_memory=True): samples draw three target
    sizes, so requests of different ops are in flight together; each output equals the oracle at its size."""
    rec = _case("service_random_resize")
    assert "error" not in rec, rec
    assert len(rec["shapes"]) >= 2 and rec["equal_to_oracle"], rec


def test_decode_service_fallback_formats_match_g6():
    """PNG / WebP / GIF / BMP / TIFF / CMYK / no-EOI samples in service workers: PIL decodes them in the
    worker, the service resizes the frame (SDSJ_SVC_FRAME); outputs and OSErrors equal G6."""
    rec = _case("service_fallback_g6")
    assert "error" not in rec and rec["equal_to_goldens"] and rec["n"] >= 40, rec


def test_dataloader_reference_shape_without_service_fails_with_a_clear_error():
    """service=None (every worker its own engine) in the reference's shape (fork, pin_memory=True): the
    DataLoader queries the GPU in the parent before forking, so a worker cannot initialise HIP; the
    transform says so and names the working set-ups."""
    rec = _case("workers_pinned_fork")
    assert "GpuDecodeBatch" in rec.get("error", "") and "pin_memory=True" in rec["error"], rec


def test_dataloader_spawn_pin_memory_with_cpu_output_matches_goldens():
    rec = _case("workers_pinned_spawn_cpu_output")
    assert "error" not in rec, rec
    assert rec["device"] == "cpu" and rec["pinned"] and rec["equal_to_goldens"], rec


def test_dataloader_pin_memory_rejects_device_tensors():
    """pin_memory=True with device outputs (spawned workers): torch's pin step refuses device
    tensors (output_device='cpu', or pin_memory=False)."""
    rec = _case("workers_pinned_spawn_device_output")
    assert "cannot pin" in rec.get("error", ""), rec


def test_fork_after_parent_gpu_init_fails_with_a_clear_error():
    rec = _case("parent_touched_gpu_fork")
    assert "GpuDecodeBatch" in rec.get("error", "") and "forked" in rec["error"], rec


def test_spawned_workers_work_after_parent_gpu_init():
    rec = _case("parent_touched_gpu_spawn")
    assert "error" not in rec, rec
    assert rec["device"].startswith("cuda") and rec["equal_to_goldens"], rec
