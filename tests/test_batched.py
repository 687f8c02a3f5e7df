"""Batched consumer-side decode (sds_amd/batched.py).

CPU tests swap the GPU engine for a stand-in that returns the oracle's pixels, so the batch
semantics are checked bit-exactly here: default_collate of deferred samples -> one decode call ->
values equal to the per-sample pipeline stacked by default_collate; failed samples dropped from every
field; the hflip coin drawn per sample in batch order; the single-frame-video branch.  The GPU test
runs the real engine through the same path.
"""
import os
import tempfile

import numpy as np
import pytest
import torch
from torch.utils.data import default_collate

from oracle import oracle as O
from tests import goldens as G


class _StandInEngine:
    max_batch = 4

    def __init__(self):
        self.slots = {}

    def submit(self, slot, jpgs, resolution, **kw):
        assert slot not in self.slots and len(jpgs) <= self.max_batch
        self.slots[slot] = self.decode_resize(jpgs, resolution, **kw)
        return self.slots[slot][0]

    def wait(self, slot):
        return self.slots.pop(slot)

    def decode_resize(self, jpgs, resolution, crop_before_resize=True, filter="bilinear", normalize=False,
                      flip=None, layout="chw", out=None):
        outs, status = [], []
        h, w = resolution
        for k, j in enumerate(jpgs):
            try:
                outs.append(torch.from_numpy(O.pipeline(j, resolution, crop_before_resize=crop_before_resize,
                                                        filter=filter, flip=bool(flip[k]) if flip else False,
                                                        normalize=normalize)))
                status.append(0)
            except O.OracleError as e:
                outs.append(torch.zeros((3, h, w), dtype=torch.float32 if normalize else torch.uint8))
                status.append(e.status)
        return torch.stack(outs), np.array(status, np.int32)


def _samples(with_corrupt: bool):
    meta, jpgs = G.g2_jpegs()
    d = tempfile.mkdtemp()
    paths = []
    for i, j in enumerate(jpgs[:5]):
        if with_corrupt and i == 2:
            j = j[:len(j) // 2]  # truncated: PIL raises, the sample is skipped by sds
        p = os.path.join(d, f"{i}.jpg")
        with open(p, "wb") as f:
            f.write(j)
        paths.append(p)
    return [{"index": i, "jpg": p, "caption": f"c{i}"} for i, p in enumerate(paths)]


def _deferred_batch(samples):
    from sds_amd.batched import create_deferred_image_pipeline
    out = []
    for s in samples:
        for t in create_deferred_image_pipeline("jpg"):
            s = t(dict(s))
        out.append(s)
    return default_collate(out)


@pytest.fixture()
def standin(monkeypatch):
    import sds_amd.batched as B
    eng = _StandInEngine()
    monkeypatch.setattr(B, "get_engine", lambda device=None: eng)
    return eng


def test_batch_equals_per_sample_pipeline_stacked(standin):
    from sds_amd.batched import GpuDecodeBatch
    samples = _samples(False)
    batch = GpuDecodeBatch("jpg", (64, 96), normalize=True)(_deferred_batch(samples))
    ref = default_collate([{"image": torch.from_numpy(O.pipeline(open(s["jpg"], "rb").read(), (64, 96),
                                                                   normalize=True))} for s in samples])["image"]
    assert list(batch.keys()) == ["index", "jpg", "caption", "image"]
    assert batch["image"].dtype == torch.float32 and torch.equal(batch["image"], ref)
    assert batch["index"].tolist() == [0, 1, 2, 3, 4]


def test_failed_samples_are_dropped_from_every_field(standin):
    from sds_amd.batched import GpuDecodeBatch
    batch = _deferred_batch(_samples(True))
    out = GpuDecodeBatch("jpg", (32, 32))(dict(batch))
    assert out["index"].tolist() == [0, 1, 3, 4]
    assert out["caption"] == ["c0", "c1", "c3", "c4"] and len(out["jpg"]) == 4
    assert out["image"].shape == (4, 3, 32, 32)
    with pytest.raises(OSError):  # PIL's own error for the truncated sample (the reference's exception)
        GpuDecodeBatch("jpg", (32, 32), on_error="raise")(dict(batch))


def test_hflip_coins_in_batch_order_and_video_branch(standin):
    from sds_amd.batched import GpuDecodeBatch
    samples = _samples(False)
    torch.manual_seed(3)
    out = GpuDecodeBatch("jpg", (48, 48), hflip_prob=0.5, return_image_as_single_frame_video=True)(
        _deferred_batch(samples))
    torch.manual_seed(3)
    flips = [bool(torch.rand(1) < 0.5) for _ in samples]
    assert list(out.keys()) == ["index", "jpg", "caption", "video", "framerate"]
    assert out["video"].shape == (5, 1, 3, 48, 48) and out["framerate"].tolist() == [960.0] * 5
    for k, s in enumerate(samples):
        base = torch.from_numpy(O.pipeline(open(s["jpg"], "rb").read(), (48, 48)))
        assert torch.equal(out["video"][k, 0], torch.flip(base, dims=[2]) if flips[k] else base)


def _equal_batches(a: dict, b: dict) -> bool:
    return list(a) == list(b) and all(torch.equal(a[k], b[k]) if isinstance(a[k], torch.Tensor) else a[k] == b[k]
                                      for k in a)


def test_stream_equals_synchronous_calls(standin):
    """GpuDecodeBatch.stream (one batch in flight through engine.submit / wait) yields what the
    synchronous calls give -- values, dropped samples, hflip coins in batch order -- including a batch
    larger than the engine's max_batch (decoded synchronously in its turn), and leaves no slot in flight."""
    from sds_amd.batched import GpuDecodeBatch
    samples = _samples(True)
    batches = [_deferred_batch(samples[:3]), _deferred_batch(samples), _deferred_batch(samples[3:]),
               _deferred_batch(samples[1:4])]
    dec = GpuDecodeBatch("jpg", (40, 40), hflip_prob=0.5)
    torch.manual_seed(11)
    ref = [dec(dict(b)) for b in batches]
    torch.manual_seed(11)
    got = list(dec.stream(dict(b) for b in batches))
    assert len(got) == len(ref) and all(_equal_batches(a, b) for a, b in zip(got, ref))
    assert [b["index"].tolist() for b in got] == [[0, 1], [0, 1, 3, 4], [3, 4], [1, 3]]
    assert standin.slots == {}
    with pytest.raises(OSError):  # on_error="raise": the exception reaches the consumer, the other slot drains
        list(GpuDecodeBatch("jpg", (40, 40), on_error="raise").stream(dict(b) for b in batches))
    assert standin.slots == {}


def test_per_sample_target_sizes_are_rejected():
    from sds_amd.batched import GpuDecodeBatch
    with pytest.raises(ValueError):
        GpuDecodeBatch("jpg", (64, 64), resize_kwargs={"allow_vertical": True})


@pytest.mark.gpu
def test_gpu_batch_matches_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sds_amd.batched import GpuDecodeBatch
    samples = _samples(True)
    out = GpuDecodeBatch("jpg", (256, 256), device="cuda:0")(_deferred_batch(samples))
    assert out["index"].tolist() == [0, 1, 3, 4]
    assert out["image"].is_cuda and out["image"].shape == (4, 3, 256, 256)
    for k, i in enumerate([0, 1, 3, 4]):
        ref = O.pipeline(open(samples[i]["jpg"], "rb").read(), (256, 256))
        np.testing.assert_array_equal(out["image"][k].cpu().numpy(), ref)


@pytest.mark.gpu
def test_gpu_stream_matches_oracle():
    """f1 pipelined: GpuDecodeBatch.stream over several collated batches on the MI355X, bit-exact against
    the oracle, the damaged sample dropped from its batch."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sds_amd.batched import GpuDecodeBatch
    samples = _samples(True)
    batches = [_deferred_batch(samples[:3]), _deferred_batch(samples), _deferred_batch(samples[2:])]
    got = list(GpuDecodeBatch("jpg", (128, 96), device="cuda:0").stream(batches))
    assert [b["index"].tolist() for b in got] == [[0, 1], [0, 1, 3, 4], [3, 4]]
    for b in got:
        for k, i in enumerate(b["index"].tolist()):
            ref = O.pipeline(open(samples[i]["jpg"], "rb").read(), (128, 96))
            np.testing.assert_array_equal(b["image"][k].cpu().numpy(), ref)


def _loader_batches(samples, collate, workers: int, bs: int):
    from torch.utils.data import DataLoader

    from sds_amd.batched import create_deferred_image_pipeline
    from tests.loader_cases import FolderDataset
    ds = FolderDataset([s["jpg"] for s in samples], create_deferred_image_pipeline("jpg"))
    return list(DataLoader(ds, batch_size=bs, num_workers=workers, collate_fn=collate,
                           multiprocessing_context="fork" if workers else None))


def test_collate_encoded_packs_the_image_field_in_shared_memory():
    """collate_encoded in DataLoader workers: the image field arrives as one EncodedBatch whose bytes are the
    samples' (in order, shared memory), the other fields exactly as default_collate gives them."""
    from sds_amd.batched import EncodedBatch, collate_encoded
    samples = _samples(False)
    got = _loader_batches(samples, collate_encoded("jpg"), 1, 3)
    ref = _loader_batches(samples, None, 0, 3)
    assert len(got) == len(ref) == 2
    for g, r in zip(got, ref):
        assert list(g.keys()) == list(r.keys())
        assert isinstance(g["jpg"], EncodedBatch) and g["jpg"].data.is_shared()
        assert [g["jpg"][k] for k in range(len(g["jpg"]))] == list(r["jpg"])
        assert all(torch.equal(g[k], r[k]) if isinstance(r[k], torch.Tensor) else g[k] == r[k]
                   for k in r if k != "jpg")


def test_encoded_batch_transport_equals_the_list_transport(standin):
    """GpuDecodeBatch on EncodedBatch inputs (synchronous and stream) yields what the list-of-bytes batches
    give -- values, the damaged sample dropped from every field (the EncodedBatch too), hflip coins."""
    from sds_amd.batched import EncodedBatch, GpuDecodeBatch, collate_encoded
    samples = _samples(True)
    packed = _loader_batches(samples, collate_encoded("jpg"), 0, 2)
    plain = _loader_batches(samples, None, 0, 2)
    dec = GpuDecodeBatch("jpg", (40, 40), hflip_prob=0.5)
    for mode in ("sync", "stream"):
        torch.manual_seed(5)
        a = [dec(dict(b)) for b in plain] if mode == "sync" else list(dec.stream(dict(b) for b in plain))
        torch.manual_seed(5)
        b = [dec(dict(x)) for x in packed] if mode == "sync" else list(dec.stream(dict(x) for x in packed))
        assert [x["index"].tolist() for x in b] == [[0, 1], [3], [4]]
        for x, y in zip(a, b):
            assert torch.equal(x["image"], y["image"]) and torch.equal(x["index"], y["index"])
            assert isinstance(y["jpg"], EncodedBatch) and list(y["jpg"]) == list(x["jpg"])
    assert standin.slots == {}


def test_collate_encoded_slot_ring_reuses_and_releases_slots():
    """collate_encoded's worker rings: a worker's batches travel as slot coordinates after the first (which
    carries the ring); a slot returns to its worker once the training process drops the EncodedBatch and
    every selection of it; bytes stay those of each batch's samples across slot reuse; a worker whose
    slots are all held falls back to one-off shared memory instead of waiting forever."""
    import gc

    from torch.utils.data import DataLoader

    from sds_amd import batched as Bm
    from sds_amd.batched import EncodedBatch, collate_encoded, create_deferred_image_pipeline
    from tests.loader_cases import FolderDataset
    samples = _samples(False)
    paths = [s["jpg"] for s in samples] * 6  # 30 samples
    want = [open(p, "rb").read() for p in paths]
    ds = FolderDataset(paths, create_deferred_image_pipeline("jpg"))
    ld = DataLoader(ds, batch_size=2, num_workers=1, multiprocessing_context="fork",
                    collate_fn=collate_encoded("jpg", slots=2, wait_s=0.01), prefetch_factor=2)
    held, k = [], 0
    for b in ld:  # drop every batch at once: slots are reused
        e = b["jpg"]
        assert isinstance(e, EncodedBatch) and list(e) == want[k:k + len(e)]
        k += len(e)
        del b, e
        gc.collect()
    assert k == len(want)
    assert len(Bm._rings) >= 1
    k = 0
    for b in ld:  # hold every batch (and a selection of each): the worker falls back once its slots are held
        e = b["jpg"]
        held.append((b, e.select([0])))
        k += len(e)
    assert [list(x["jpg"]) for x, _ in held] == [want[i:i + 2] for i in range(0, len(want), 2)]
    assert [list(s) for _, s in held] == [[want[i]] for i in range(0, len(want), 2)]


def test_collate_encoded_with_spawned_persistent_workers():
    """The slot rings under spawn-started, persistent workers (the collate function is pickled to them
    without its ring; each creates its own): two epochs, every batch's bytes those of its samples."""
    from torch.utils.data import DataLoader

    from sds_amd.batched import EncodedBatch, collate_encoded, create_deferred_image_pipeline
    from tests.loader_cases import FolderDataset
    samples = _samples(False)
    paths = [s["jpg"] for s in samples] * 4  # 20 samples
    want = sorted(open(p, "rb").read() for p in paths)
    ds = FolderDataset(paths, create_deferred_image_pipeline("jpg"))
    ld = DataLoader(ds, batch_size=3, num_workers=2, multiprocessing_context="spawn", persistent_workers=True,
                    collate_fn=collate_encoded("jpg", slots=3))
    for _ in range(2):
        got = []
        for b in ld:
            assert isinstance(b["jpg"], EncodedBatch)
            got += list(b["jpg"])
        assert sorted(got) == want
