"""bench.py's multi-rank launcher (configs[3] shape) on CPU: ``--gpus 2`` outside torchrun starts two
fresh rank processes that join a gloo process group, each owning its compute_index_slice rows, and
rank 0 prints one line with the aggregate rate and both per-rank rates.  The engine is the CPU
stand-in (``--engine stub``); the HIP path of the same script runs on the GPU box."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(gpus, *extra):
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(gpus), "--engine", "stub", "--backend",
           "gloo", "--rows", "64", "--pool", "4", "--batch", "16", "--steps", "3", "--warmup", "1",
           "--no-cpu-baseline", "--roofline-steps", "1", *extra]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    return json.loads(lines[0])


def test_two_rank_launch_reports_the_whole_job():
    line = _run(2)
    assert line["n_gpus"] == 2
    pg = line["process_group"]
    assert (pg["backend"], pg["world_size"], pg["gpus_visible"], pg["all_gather_device"]) == ("gloo", 2, 0, "cpu")
    assert len(line["per_rank_images_per_s"]) == 2
    assert line["config"]["global_batch"] == 32 and line["config"]["rows_per_gpu"] == 64
    # the parquet index the ranks sliced (sds/index.py:208-246): 2 x 64 rows, one contiguous slice each
    assert line["config"]["index"]["rows"] == 128 and "parquet" in line["config"]["index"]["source"]
    assert line["config"]["index"]["slices"] == [[0, 64], [64, 128]]
    # value = all ranks' images over the slowest rank's time
    slowest = min(line["per_rank_images_per_s"])
    assert abs(line["value"] - 2 * slowest) <= 0.01 * line["value"] + 1


def test_one_gpu_run_is_unchanged():
    line = _run(1)
    assert line["n_gpus"] == 1 and line["process_group"]["world_size"] == 1
    assert len(line["per_rank_images_per_s"]) == 1
    assert line["config"]["index"]["slices"] == [[0, 64]]


def test_forced_process_group_at_world_size_1():
    """--force-pg: one rank still creates the process group and runs the collectives of the multi-GPU path
    (the GPU test runs it with nccl = RCCL)."""
    line = _run(1, "--force-pg")
    pg = line["process_group"]
    assert pg["backend"] == "gloo" and pg["world_size"] == 1 and pg["forced_at_world_size_1"]
    assert pg["all_gather_device"] == "cpu"
    assert line["n_gpus"] == 1 and len(line["per_rank_images_per_s"]) == 1


def test_default_index_is_a_million_rows_on_several_gpus():
    """configs[3]: without --rows, --gpus N slices a 1,000,000-row parquet index (125,000 rows per rank at 8)."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--engine", "stub", "--backend",
           "gloo", "--pool", "4", "--batch", "16", "--steps", "1", "--warmup", "0", "--no-cpu-baseline",
           "--roofline-steps", "1"]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][0])
    assert line["config"]["index"]["rows"] == 1_000_000 and line["config"]["rows_per_gpu"] == 500_000
    assert line["config"]["index"]["slices"] == [[0, 500_000], [500_000, 1_000_000]]
    assert line["config"]["workload"].startswith("configs[3]: 1,000,000-row parquet index")
