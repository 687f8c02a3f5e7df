"""configs[3] under -m gpu: bench.py's multi-rank path on the HIP engine.

``bench.py --gpus 2`` starts two rank processes (before anything touches the GPU in the parent), each
owning its slice of the index exactly as sds/index.py:235-246 compute_index_slice slices it, each
decoding its rows with the HIP engine and checking its pixels against PIL (a rank exits non-zero on a
mismatch).  On a one-GPU box both ranks share the card (ranks map round-robin onto the visible GPUs)
and the process group is gloo (RCCL needs one device per rank); the driver's 8-GPU run uses nccl.
"""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_index_sharded_on_hip():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--backend", "gloo", "--rows", "4096",
           "--batch", "1024", "--steps", "2", "--warmup", "1", "--pool", "64", "--roofline-steps", "1",
           "--no-cpu-baseline"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one line
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["process_group"]["world_size"] == 2
    assert d["process_group"]["backend"] == "gloo"
    assert d["config"]["workload"].startswith("configs[3]")
    assert d["config"]["global_batch"] == 2048 and d["config"]["rows_per_gpu"] == 4096
    # each rank read its compute_index_slice rows (sds/index.py:235-246) from the parquet index
    assert d["config"]["index"]["rows"] == 8192 and "parquet" in d["config"]["index"]["source"]
    assert d["config"]["index"]["slices"] == [[0, 4096], [4096, 8192]]
    assert len(d["per_rank_images_per_s"]) == 2 and all(v > 0 for v in d["per_rank_images_per_s"])
    assert d["pixel_check"]["equal_to_pil"] and d["pixel_check"]["golden_sha256_match"]
    assert d["value"] > 0


def test_bench_rccl_process_group_at_world_size_1():
    """The RCCL branch of the multi-GPU bench on one GPU: ``--force-pg --backend nccl`` creates the process
    group with ``device_id`` at world size 1 and runs the device-tensor all_reduce (max over ranks) and
    all_gather of the timed region (sds/utils/distributed.py:22-40 uses the 'nccl' backend)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--force-pg", "--backend", "nccl",
           "--rows", "4096", "--batch", "1024", "--steps", "2", "--warmup", "1", "--pool", "64",
           "--roofline-steps", "1", "--no-cpu-baseline"]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][0])
    pg = d["process_group"]
    assert pg["backend"] == "nccl" and pg["world_size"] == 1 and pg["forced_at_world_size_1"]
    assert pg["all_gather_device"].startswith("cuda"), pg
    assert d["pixel_check"]["equal_to_pil"] and d["pixel_check"]["walk"]["covers_every_resident_row"]
    assert d["pixel_check"]["rows_checked"] == 1024 and d["pixel_check"]["rows_equal"] == 1024
