#!/usr/bin/env python3
"""Device-resident JPEG decode + resize@256 throughput on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[1]): synthetic 640x480 q90 baseline JPEGs
(4:2:0, Annex-K tables, no DRI) resident in HBM -- 100,000 rows per GPU, row i holding the
encoded bytes of pool image i % POOL (each row is its own copy in HBM, so every launch reads its
compressed bytes from HBM) -- decoded, centre-cropped and bilinear-resized to 256x256 uint8 CHW
by the C-ABI engine.  One step = one batch of ``--batch`` rows.

Multi-GPU (configs[3]): one process per GPU.  ``--gpus N`` outside torchrun starts N fresh child
processes (before anything touches the GPU here), each with RANK / WORLD_SIZE / LOCAL_RANK set;
under torchrun the ranks come from its environment.  The index is a 1,000,000-row synthetic parquet
file (100,000 rows on one GPU, configs[1]); rank r reads and owns rows [r*N/R, (r+1)*N/R)
(sds/index.py:208-246 load_index_partition / compute_index_slice, INTER_NODE), no collective on the
data path ("scaling": "weak": the batch per GPU is fixed); the process group (RCCL) only carries the
barriers, the index slices and the max-over-ranks of the timed region.

``--workload mixed512`` is configs[2] (mixed VGA..4K -> 512 + hflip + float32 normalise, device-
resident); ``--workload e2e512`` is configs[4]: each rank's rows as JPEG files in a local cache
directory -> pinned slots -> H2D -> decode + resize 512 -> D2H into pinned host memory, two batches
in flight, reported next to the device-resident rate of the same rows (``device_resident_value``).

Prints ONE JSON line (rank 0).  ``roofline`` prices the dominant kernel: algorithmic bytes per
launch (compressed bytes in + output bytes out) / that kernel's mean duration,
measured with HIP events on its launch stream in a single-lane pass after the timed region (one
dispatch per kernel per batch, nothing overlapping it; rocprofv3 summaries under profiles/).
``cpu_baseline`` times the reference's PIL/libjpeg-turbo pipeline (functional.py:94-110 op order,
files read as LoadFromDiskTransform does) over a folder of the same JPEGs on this host's cores
(rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import shutil
import socket
import subprocess
import sys
import tempfile
import time
from typing import Optional

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md chip table)
# tools/pmc.sh + tools/pmc_summary.py output per workload (the counters of the batch that workload runs)
PMC_JSONS = {"vga256": os.path.join(REPO, "profiles", "pmc_latest.json"),
             "mixed512": os.path.join(REPO, "profiles", "pmc_latest_mixed512.json")}
PMC_JSON = PMC_JSONS["vga256"]
# engine stage -> kernels launched in it (rocprofv3 kernel names contain these)
STAGE_KERNELS = {"parse": ["k_parse"], "plan": ["k_plan"], "unstuff": ["k_us_", "k_scanmap"],
                 "prog": ["k_prog"], "entspec": ["k_enttab", "k_entspec"], "entsync": ["k_entsync"],
                 "entwrite": ["k_entwrite"], "idct": ["k_idct"],
                 "color": ["k_color"], "coeffs": ["k_coeffs"], "hpass": ["k_hpass"], "vpass": ["k_vpass"],
                 "resample": ["k_resample", "k_rs420", "k_finish"]}


def pmc_traffic(stage: str, batch: int, lanes: int, path: str = PMC_JSON):
    """HBM bytes per launch of `stage` from the committed PMC summary (FETCH_SIZE + WRITE_SIZE, KB as
    rocprofv3 reports them, summed over the stage's kernels), if collected at this batch and lane count."""
    try:
        with open(path) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None
    if pmc.get("batch") != batch or pmc.get("lanes", 1) != lanes:
        return None
    tot, hit = 0.0, False
    for name, ctr in pmc.get("kernels", {}).items():
        if any(k in name for k in STAGE_KERNELS.get(stage, [])) and "FETCH_SIZE" in ctr and "WRITE_SIZE" in ctr:
            tot += (ctr["FETCH_SIZE"] + ctr["WRITE_SIZE"]) * 1024.0
            hit = True
    return {"bytes_per_launch": round(tot), "source": os.path.relpath(path, REPO), "head": pmc.get("head"),
            "note": "FETCH_SIZE + WRITE_SIZE as reported, separate --pmc passes (MI355X_MICROARCH.md: FETCH_SIZE "
                    "counts 1/2 of 16-B/lane streaming reads; these kernels read <= 4 B/lane, uncalibrated)"} \
        if hit else None


def pmc_counters(stage: str, batch: int, lanes: int, path: str = PMC_JSON) -> Optional[dict]:
    """Per-launch PMC counters of `stage` (summed over its kernels) from the committed summary, if it
    was collected at this batch and lane count."""
    try:
        with open(path) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return None
    if pmc.get("batch") != batch or pmc.get("lanes", 1) != lanes:
        return None
    tot: dict = {}
    for name, ctr in pmc.get("kernels", {}).items():
        if any(k in name for k in STAGE_KERNELS.get(stage, [])):
            for k, v in ctr.items():
                tot[k] = tot.get(k, 0.0) + v
    return tot or None


def measured_limiter(stage: str, batch: int, launch_ms: float, traffic: Optional[dict], path: str = PMC_JSON) -> dict:
    """Which roof the dominant kernel is nearest, from its measured counters: HBM (implementation bytes
    per launch / launch time / peak) or VALU issue (wave-level VALU instructions x 2 cycles -- a wave64
    VALU op holds its SIMD 2 cycles when two or more waves share it -- / (1,024 SIMDs x 2.4 GHz x launch
    time)).  Neither near 1 = latency-bound (dependent LDS lookups / VALU chains)."""
    ctr = pmc_counters(stage, batch, 1, path)
    out = {"source": os.path.relpath(path, REPO) if ctr else None}
    if not ctr or launch_ms <= 0:
        out["verdict"] = "unmeasured (no PMC summary at this batch)"
        return out
    sec = launch_ms * 1e-3
    hbm = (traffic or {}).get("bytes_per_launch", 0) / sec / (HBM_PEAK_GBS * 1e9) if traffic else None
    valu = ctr.get("SQ_INSTS_VALU", 0.0) * 2 / (1024 * 2.4e9 * sec)
    out.update({"hbm_traffic_frac": round(hbm, 4) if hbm is not None else None, "valu_issue_frac": round(valu, 4)})
    best = max([("hbm", hbm or 0.0), ("valu_issue", valu)], key=lambda kv: kv[1])
    out["verdict"] = best[0] if best[1] >= 0.7 else f"latency (nearest roof: {best[0]} at {best[1]:.2f})"
    return out


def _make_pool_image(i: int) -> bytes:
    from tests.golden.synth import encode_jpeg, synth_rgb
    return encode_jpeg(synth_rgb(np.random.default_rng(1234 + i), 640, 480), 90)


def _make_mixed_image(i: int) -> bytes:
    # configs[2]: size drawn uniformly from the VGA..4K landscape sizes and their
    # portrait transposes, content from the same seeded generator
    from tests.golden.synth import MIXED_SIZES, encode_jpeg, synth_rgb
    rng = np.random.default_rng(4321 + i)
    w, h = MIXED_SIZES[int(rng.integers(0, len(MIXED_SIZES)))]
    return encode_jpeg(synth_rgb(rng, w, h), 90)


def _pool_map(fn, items, workers: int, chunksize: int = 1) -> list:
    """map over spawn-started worker processes that are closed and joined (they exit normally; the
    Pool context manager would terminate them, and SIGTERM handlers fire inside profiled runs)."""
    p = mp.get_context("spawn").Pool(workers)
    try:
        return p.map(fn, items, chunksize=chunksize)
    finally:
        p.close()
        p.join()


def make_pool(n: int, workers: int, maker=_make_pool_image) -> list[bytes]:
    if workers <= 1:
        return [maker(i) for i in range(n)]
    return _pool_map(maker, range(n), workers, chunksize=4)


# ---------------------------------------------------------------- CPU baseline (reference ops)
def _pil_pipeline(jpg: bytes, res: int = 256, flip: bool = False, normalize: bool = False):
    """functional.py:94-110 + presets.py:716-733 op order: open/convert, crop, resize, to tensor
    (+ the user hflip of README.md:99-108, + NormalizeFramesTransform presets.py:154-162)."""
    import io

    import torch
    from PIL import Image
    img = Image.open(io.BytesIO(jpg)).convert("RGB")
    w, h = img.size
    ar = res / res
    if w / h > ar:
        nw = int(h * ar)
        left = (w - nw) // 2
        img = img.crop((left, 0, left + nw, h))
    else:
        nh = int(w / ar)
        top = (h - nh) // 2
        img = img.crop((0, top, w, top + nh))
    if img.size != (res, res):
        img = img.resize((res, res), Image.BILINEAR)
    x = torch.from_numpy(np.array(img)).permute(2, 0, 1)
    if flip:
        x = torch.flip(x, dims=[2])
    if normalize:
        x = x.float() / 127.5 - 1.0
    return x


def _cpu_worker(args):
    paths, seconds, res, mixed = args
    import torch
    torch.set_num_threads(1)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        with open(paths[n % len(paths)], "rb") as f:  # LoadFromDiskTransform, presets.py:613-626
            jpg = f.read()
        _pil_pipeline(jpg, res, flip=mixed and n % 2 == 1, normalize=mixed)
        n += 1
    return n, time.perf_counter() - t0


def cpu_baseline(paths: list[str], procs: int, seconds: float, res: int = 256, mixed: bool = False) -> float:
    if procs <= 1:
        n, dt = _cpu_worker((paths, seconds, res, mixed))
        return n / dt
    res_ = _pool_map(_cpu_worker, [(paths[k::procs] or paths, seconds, res, mixed) for k in range(procs)], procs)
    return sum(n for n, _ in res_) / max(dt for _, dt in res_)


def host_cores() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_share() -> tuple[int, str]:
    """CPUs this process may use, and where that number comes from: the cgroup CPU quota (v2
    cpu.max, v1 cfs_quota_us), else the thread share the box declares (OMP_NUM_THREADS: a GPU box
    exports its per-GPU CPU share there, while nproc shows the whole machine), else nproc."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max" and int(per) > 0:
            return max(1, int(q) // int(per)), "cgroup v2 cpu.max quota"
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        if q > 0 and per > 0:
            return max(1, q // per), "cgroup v1 cfs quota"
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        return min(int(omp), host_cores()), "OMP_NUM_THREADS (the box's declared CPU share)"
    return host_cores(), "nproc (sched_getaffinity)"


# ---------------------------------------------------------------- output verification
def _pil_u8_sha(args) -> str:
    """SHA-256 of the reference pipeline's uint8 CHW output for one JPEG (functional.py:94-110 op order,
    no flip / normalise): the check of the engine's per-pool-image reference outputs."""
    import hashlib
    import io

    from PIL import Image
    jpg, res = args
    img = Image.open(io.BytesIO(jpg)).convert("RGB")
    w, h = img.size
    if w > h:
        left = (w - h) // 2
        img = img.crop((left, 0, left + h, h))
    else:
        top = (h - w) // 2
        img = img.crop((0, top, w, top + w))
    if img.size != (res, res):
        img = img.resize((res, res), Image.BILINEAR)
    return hashlib.sha256(np.ascontiguousarray(np.asarray(img).transpose(2, 0, 1)).tobytes()).hexdigest()


def verify_rows(eng, blob, d_offs, d_lens, out, status, flips, rows_ext, period, pool, nrows, B, res, mixed,
                last_start, dev_step, cursor, workers, e2e_last=None) -> dict:
    """Checks decoded rows on the device against per-pool-image references.

    The references: each distinct pool image of the rank's period, decoded once by the engine (uint8 CHW,
    no flip) and checked against PIL on the host by SHA-256 (_pil_u8_sha).  A row's expected output is
    its pool image's reference, flipped where the row's flag says so and mapped through the normalise LUT
    (``x.float() / 127.5 - 1`` per byte value, evaluated on the host) for configs[2].  Checked: every row of
    the batch ``out`` holds (rows [last_start, last_start + B), the last timed batch) and then every resident
    row of the rank -- ceil(nrows / B) batches from row 0 through ``dev_step``.  ``e2e_last`` (configs[4]):
    (host tensor, row indices) of the last batch the end-to-end pipeline delivered to host memory, checked
    the same way before the walk."""
    import hashlib

    import torch
    P = len(period)
    dev = out.device
    ref = torch.empty((P, 3, res, res), dtype=torch.uint8, device=dev)
    for a in range(0, P, B):  # (rows 0 .. P-1 hold the period's images in order)
        b = min(P, a + B)
        _, st = eng.decode_resize_device(blob, d_offs[a:b], d_lens[a:b], (res, res), out=ref[a:b])
        if int((st != 0).sum().item()):
            raise SystemExit("a pool image failed to decode in the reference pass")
    torch.cuda.synchronize(dev)
    ref_h = ref.cpu().numpy()
    ref_sha = [hashlib.sha256(ref_h[k].tobytes()).hexdigest() for k in range(P)]
    items = [(pool[p], res) for p in period]
    pil_sha = [_pil_u8_sha(it) for it in items] if workers <= 1 or P < 32 else \
        _pool_map(_pil_u8_sha, items, min(workers, 32), chunksize=8)
    refs_ok = sum(int(a == b) for a, b in zip(ref_sha, pil_sha))
    lut = (torch.arange(256, dtype=torch.float32) / 127.5 - 1.0).to(dev) if mixed else None
    pidx = torch.from_numpy((rows_ext % P).astype(np.int64)).to(dev)

    def check(start: int) -> int:
        """rows of `out` (batch starting at row `start`) equal to their expected output"""
        good = 0
        ch = 512 if mixed else 8192
        for a in range(0, B, ch):
            b = min(B, a + ch)
            exp = ref[pidx[start + a:start + b]]
            if mixed:
                f = flips[start + a:start + b].bool().view(-1, 1, 1, 1)
                exp = lut[torch.where(f, exp.flip(-1), exp).long()]
            eq = (out[a:b] == exp).flatten(1).all(1) & (status[a:b] == 0)
            good += int(eq.sum().item())
        return good

    res_d = {"method": "per-row device compare with the row's pool-image reference (engine output, uint8, "
                       "SHA-256-equal to PIL's on the host); configs[2] rows flipped per flag and mapped through "
                       "the fp32 normalise LUT",
             "pool_refs": P, "pool_refs_equal_to_pil": refs_ok}
    ok = refs_ok == P
    if last_start is not None:
        g = check(last_start)
        res_d.update(rows_checked=B, rows_equal=g, last_batch_first_row=int(last_start))
        ok = ok and g == B
    if e2e_last is not None:
        host, rows = e2e_last
        idx = torch.from_numpy(np.asarray(rows, dtype=np.int64) % P).to(dev)
        eq = (host.to(dev) == ref[idx]).flatten(1).all(1)
        g = int(eq.sum().item())
        res_d.update(e2e_rows_checked=len(rows), e2e_rows_equal=g)
        ok = ok and g == len(rows)
    walk_batches = (nrows + B - 1) // B
    cursor[0] = 0
    wg = 0
    for k in range(walk_batches):
        s0 = cursor[0]
        dev_step()
        wg += check(s0)
    res_d["walk"] = {"batches": walk_batches, "rows_checked": walk_batches * B, "rows_equal": wg,
                     "covers_every_resident_row": walk_batches * B >= nrows}
    ok = ok and wg == walk_batches * B
    res_d["equal_to_pil"] = bool(ok)
    res_d["_ref_sha"] = ref_sha
    return res_d


# ---------------------------------------------------------------- multi-rank launcher
def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int, argv: list[str], timeout: float = 3000.0) -> int:
    """Starts n fresh rank processes of this script (nothing here has touched the GPU) and waits for
    them; if one fails, the others are stopped (by PID) so no rank waits at a barrier forever."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    t0, rc = time.time(), 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is not None:
                live.remove(p)
                rc = rc or c
        if rc or time.time() - t0 > timeout:
            for p in live:
                p.kill()
            for p in live:
                p.wait()
            return rc or 124
        time.sleep(0.05)
    return rc


class StubEngine:
    """CPU stand-in of JpegEngine for the launcher test (--engine stub): touches its inputs, writes
    zeros and OK statuses; no decoding."""

    def __init__(self, *a, **k):
        self.lanes = 4

    def decode_resize_device(self, blob, offsets, lengths, resolution, *, out, status, normalize=False, flip=None,
                             **kw):
        out.zero_()
        status.zero_()
        return out, status

    def set_timing(self, enable):
        pass

    def set_lanes(self, lanes):
        self.lanes = lanes

    def stage_times(self):
        return {"entwrite": 1.0}

    def counters(self, reset=False):
        return {}


# ---------------------------------------------------------------- main
def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=["vga256", "mixed512", "e2e512"], default="vga256",
                    help="vga256 = configs[1] (the headline metric); mixed512 = configs[2]: VGA..4K -> centre crop + "
                         "resize 512 + hflip(p=0.5) + CHW float normalise")
    ap.add_argument("--batch", type=int, default=None)
    ap.add_argument("--rows", type=int, default=None, help="rows resident per GPU (sets --index-rows to rows x GPUs)")
    ap.add_argument("--index-rows", type=int, default=None,
                    help="rows of the synthetic parquet index the ranks slice (default: 100,000 on one GPU -- "
                         "configs[1] -- and 1,000,000 on several -- configs[3])")
    ap.add_argument("--pool", type=int, default=None, help="distinct encoded images")
    ap.add_argument("--res", type=int, default=None)
    ap.add_argument("--e2e-out", choices=["device", "pinned"], default="device",
                    help="configs[4]: decode into HBM and copy back on a D2H stream (device), or let the kernels "
                         "store the pixels straight into pinned host memory over PCIe (pinned)")
    ap.add_argument("--dl-workers", type=int, default=4,
                    help="configs[4]: threads of the restated ParallelDownloader (the reference's num_downloading_workers "
                         "default, dataset.py:61; 4 / 8 / 16 threads: 53-56k / 49-57k / 44-50k images/s warm and "
                         "10.0-10.3k / 5.8-8.3k / 5.5-6.7k cold, profiles/r06_e2e_dl_workers.txt)")
    ap.add_argument("--cpu-seconds", type=float, default=4.0)
    ap.add_argument("--cpu-files", type=int, default=1000, help="files in the CPU-baseline folder (configs[0])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--roofline-steps", type=int, default=5, help="single-lane steps timed for the roofline")
    ap.add_argument("--profile-steps", action="store_true", help="print per-stage times to stderr")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl", help="process group (nccl = RCCL)")
    ap.add_argument("--force-pg", action="store_true",
                    help="create the process group at world size 1 too, so that one GPU runs the collectives of the "
                         "multi-GPU path (init with device_id, device all_reduce / all_gather over --backend)")
    ap.add_argument("--engine", choices=["hip", "stub"], default="hip", help="stub: CPU stand-in (launcher tests)")
    ap.add_argument("--no-pixel-check", action="store_true",
                    help="experiments only (timing of deliberately wrong kernel variants): skip the pixel check; the "
                         "line then carries pixel_check null")
    args = ap.parse_args()
    mixed = args.workload == "mixed512"
    e2e = args.workload == "e2e512"
    # batches: one engine call per step, whose lanes drain at its end (the caller's stream orders the
    # next call after it), so larger batches amortise that (configs[1]: 455k images/s at 4096, 476k
    # at 16384; configs[2]: 45.0k at 512, 59.8k at 2048 -- DESIGN.md §5; round 5: 16,384 -> 32,768 +1.2 %,
    # 32,768 -> 65,536 +2.3 %; configs[2] 2,048 -> 4,096 -> 8,192: 80.5k -> 85.0k -> 87.8k; profiles/r05_batch.txt)
    defaults = {"batch": 8192, "rows": 16384, "pool": 1024, "res": 512} if mixed else \
        {"batch": 1024, "rows": 16384, "pool": 256, "res": 512} if e2e else \
        {"batch": 65536, "rows": None, "pool": 1024, "res": 256}
    for k, v in defaults.items():
        if getattr(args, k) is None:
            setattr(args, k, v)

    if args.gpus > 1 and "RANK" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))

    # stdout carries exactly one line, the JSON result: everything else written to file descriptor 1 --
    # RCCL's version banner, gloo's connection messages, library warnings -- goes to stderr
    result_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)

    import torch
    import torch.distributed as dist

    stub = args.engine == "stub"
    rank, world, local_rank = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)), \
        int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus and "RANK" in os.environ and args.gpus > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # one GPU per rank; more ranks than GPUs (a rehearsal on a smaller box, --backend gloo) share them
    # round-robin (torch.cuda.device_count() does not initialise the GPU)
    ndev = 0 if stub else torch.cuda.device_count()
    dev = torch.device("cpu") if stub else torch.device("cuda", local_rank % max(1, ndev))
    use_pg = world > 1 or args.force_pg
    if use_pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1:
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
        if stub:
            dist.init_process_group(args.backend, rank=rank, world_size=world)
        else:
            torch.cuda.set_device(dev)
            dist.init_process_group(args.backend, rank=rank, world_size=world, device_id=dev)
    elif not stub:
        torch.cuda.set_device(dev)

    def sync():
        if not stub:
            torch.cuda.synchronize()

    from sds_amd.distributed import compute_index_slice, max_over_ranks

    def barrier():
        if use_pg:
            dist.barrier()

    coll_dev = None if stub or args.backend == "gloo" else dev  # where the collectives' tensors live

    def max_ranks(v: float) -> float:
        return max_over_ranks(v, device=coll_dev, always=use_pg)

    workers = max(1, cpu_share()[0] // max(1, world))
    pool = make_pool(args.pool, workers, _make_mixed_image if mixed else _make_pool_image)

    # The sample index: a synthetic parquet file (sds's index layout, sds_amd/index.py) of
    # total_rows rows, row i referring to pool image i % POOL, written once by rank 0; each rank reads
    # its compute_index_slice rows from it (sds/index.py:208-246 load_index_partition) and checks them.
    # The rank's rows are laid out as a repeated template of one pool period (16-byte aligned rows),
    # tiled on the device, so every row is its own copy in HBM.
    if args.index_rows is None:
        args.index_rows = args.rows * world if args.rows else (1_000_000 if world > 1 else 100_000)
    total_rows = args.index_rows
    index_path = None
    try:
        import pyarrow  # noqa: F401
        index_path = os.path.join(tempfile.gettempdir(), f"sdsj_index_{os.environ.get('MASTER_PORT', os.getpid())}_"
                                                         f"{total_rows}_{args.pool}.parquet")
    except ImportError:
        pass
    if index_path:
        from sds_amd.index import load_index_partition, write_synthetic_index
        if rank == 0:
            write_synthetic_index(index_path + ".tmp", total_rows, args.pool)
            os.replace(index_path + ".tmp", index_path)
        barrier()
        r0, r1, rows_tab = load_index_partition(index_path, total_rows, rank, world, columns=["index", "pool_image"])
        ids = rows_tab.column("index").to_numpy()
        if not (np.array_equal(ids, np.arange(r0, r1)) and
                np.array_equal(rows_tab.column("pool_image").to_numpy(), ids % args.pool)):
            raise SystemExit(f"rank {rank}: the parquet index slice [{r0}, {r1}) does not hold the expected rows")
        del rows_tab, ids
    else:
        r0, r1, _ = compute_index_slice(total_rows, rank, world)
    nrows = r1 - r0
    B = args.batch
    slices = [[r0, r1]]
    if use_pg:
        slices = [None] * world
        dist.all_gather_object(slices, [r0, r1])
    period = [(r0 + k) % args.pool for k in range(min(args.pool, nrows))]
    t_lens = np.array([len(pool[p]) for p in period], np.int64)
    t_aligned = (t_lens + 15) // 16 * 16
    t_offs = np.zeros(len(period), np.int64)
    t_offs[1:] = np.cumsum(t_aligned)[:-1]
    T = int(t_offs[-1] + t_aligned[-1])
    template = np.zeros(T, np.uint8)
    for k, p in enumerate(period):
        template[t_offs[k]:t_offs[k] + t_lens[k]] = np.frombuffer(pool[p], np.uint8)
    # (the CPU stand-in engine reads nothing: its rows share one copy of the template)
    reps = 1 if stub else (nrows + len(period) - 1) // len(period)
    d_tmpl = torch.from_numpy(template).to(dev)
    blob = d_tmpl.repeat(reps)
    # every batch is a window of B consecutive rows, wrapping past the rank's last row to its first one (the
    # timed steps walk all resident rows): the row arrays are extended by B rows taken from the start
    j = np.arange(nrows + B) % nrows
    offs = (j // len(period)) % reps * T + t_offs[j % len(period)]
    lens = t_lens[j % len(period)]
    d_offs = torch.from_numpy(offs.astype(np.int64)).to(dev)
    d_lens = torch.from_numpy(lens.astype(np.int32)).to(dev)
    del d_tmpl
    sync()

    if stub:
        eng = StubEngine()
    else:
        from sds_amd.engine import JpegEngine
        # device scratch from host planning (sdsj_plan_need): the largest sum over any window of B
        # consecutive rows, wrap-around included (every batch is such a window)
        need_of = {p: JpegEngine.scratch_need([pool[p]], (args.res, args.res), normalize=mixed) for p in set(period)}
        cyc = np.array([need_of[p] for p in period], np.int64)
        row_need = cyc[j % len(period)]
        cum = np.concatenate([[0], np.cumsum(row_need)])
        win = int((cum[B:B + nrows] - cum[:nrows]).max())
        eng = JpegEngine(dev, max_batch=B, scratch_bytes=win + (64 << 20))
    out = torch.empty((B, 3, args.res, args.res), dtype=torch.float32 if mixed else torch.uint8, device=dev)
    status = torch.empty(B, dtype=torch.int32, device=dev)
    # hflip flags for every row, seeded (the user HorizontalFlipTransform, p = 0.5), extended like the rows
    h_flips = (np.random.default_rng(99 + rank).random(nrows) < 0.5).astype(np.uint8)[j]
    flips = torch.from_numpy(h_flips).to(dev)
    cursor = [0]
    walked = {"rows": 0}  # rows decoded by dev_step since the last reset (the timed region's count)

    def dev_step():
        # the batch = rows [s, s + B) of the rank, modulo nrows: consecutive steps walk every resident row
        s = cursor[0]
        eng.decode_resize_device(blob, d_offs[s:s + B], d_lens[s:s + B], (args.res, args.res), out=out,
                                 status=status, normalize=mixed, flip=flips[s:s + B] if mixed else None)
        cursor[0] = (s + B) % nrows
        walked["rows"] += B

    step = dev_step
    cache_dir = src_dir = None
    dl_rates = None
    if e2e:
        # configs[4]: sds/downloader.py -> host cache -> H2D -> decode + resize -> D2H.  The rank's rows
        # come from a source folder (one file per pool image, the "remote" of a local-scheme index)
        # through the restated ParallelDownloader (sds_amd/downloader.py: a thread pool copying each row's
        # file into the cache directory via <dst>.tmp + rename, skip_if_exists), whose completed rows --
        # in completion order, as StreamingDataset consumes them (dataset.py:361-384) -- form the batches
        # -> pinned slot -> H2D -> decode + resize -> D2H into pinned host memory.  One step submits
        # batch k and completes batch k - 1 (its D2H on a second stream), so batch k's downloads, file
        # reads and H2D overlap batch k - 1's decode; downloads run up to two batches ahead.
        from itertools import islice

        from sds_amd.downloader import ParallelDownloader
        src_dir = tempfile.mkdtemp(prefix=f"sdsj_src_r{rank}_")
        cache_dir = tempfile.mkdtemp(prefix=f"sdsj_cache_r{rank}_")
        src_paths = {}
        for p in set(period):
            src_paths[p] = os.path.join(src_dir, f"{p:06d}.jpg")
            with open(src_paths[p], "wb") as f:
                f.write(pool[p])
        dl_workers = args.dl_workers
        dl = ParallelDownloader(num_workers=dl_workers, prefetch=2 * B, num_retries=3, skip_if_exists=True)
        dst_of = lambda key: os.path.join(cache_dir, f"{key:08d}-jpg.jpg")  # noqa: E731  (dataset.py:250)
        sched = [0]

        def schedule_ahead(upto):
            while sched[0] < upto:
                j = sched[0] % nrows
                dl.schedule_task(r0 + j, [src_paths[period[j % len(period)]]], [dst_of(r0 + j)])
                sched[0] += 1

        hosts = [torch.empty(out.shape, dtype=out.dtype, pin_memory=True) for _ in range(2)]
        zero_copy = args.e2e_out == "pinned"
        outs = hosts if zero_copy else [out, torch.empty_like(out)]
        d2h = torch.cuda.Stream(dev)
        # the decode runs on a stream of its own, not the legacy default stream (which synchronises with
        # every blocking stream).  The device still serialises each D2H (a 15.0 ms blit kernel per
        # 1,024 rows) with the next batch's 3.1 ms decode: profiles/r06_e2e_trace.txt
        work = torch.cuda.Stream(dev)
        pipe = {"k": 0, "prev": None, "bad": 0, "done": 0, "taken": 0, "keys": [None, None], "last": None}

        def complete_prev():
            prev = pipe["prev"]
            o, st = eng.wait(prev)
            pipe["bad"] += int((st != 0).sum())
            pipe["done"] += len(st)
            if not zero_copy:
                with torch.cuda.stream(d2h):
                    hosts[prev].copy_(o, non_blocking=True)
            pipe["prev"], pipe["last"] = None, prev

        # host wall time per phase of the step (seconds, summed; reset with the timed region): scheduling the
        # downloads ahead, taking the batch's completed rows from the downloader, engine.submit (file reads
        # into the pinned slot, host planning, H2D + decode launches), completing the previous batch (its
        # wait, the D2H issue)
        ph = {"schedule": 0.0, "handoff": 0.0, "submit": 0.0, "complete": 0.0}

        def e2e_step():
            t0 = time.perf_counter()
            schedule_ahead(pipe["taken"] + 2 * B)
            t1 = time.perf_counter()
            keys = [key for key, _ in islice(dl.yield_completed(), B)]
            paths = [dst_of(key) for key in keys]
            if len(paths) != B:  # a row whose copy failed every retry: fail the run, never count it
                raise SystemExit(f"rank {rank}: the downloader delivered {len(paths)} of {B} rows")
            t2 = time.perf_counter()
            pipe["taken"] += B
            slot = pipe["k"] % 2
            with torch.cuda.stream(work):
                work.wait_stream(d2h)  # slot's previous output has left for the host
                eng.submit(slot, paths, (args.res, args.res), files=True, out=outs[slot])
            pipe["keys"][slot] = keys
            t3 = time.perf_counter()
            if pipe["prev"] is not None:
                complete_prev()
            t4 = time.perf_counter()
            pipe["prev"], pipe["k"] = slot, pipe["k"] + 1
            for k, a, b in (("schedule", t0, t1), ("handoff", t1, t2), ("submit", t2, t3), ("complete", t3, t4)):
                ph[k] += b - a

        def e2e_epoch_rate(nsteps):
            barrier()
            sync()
            t = time.perf_counter()
            for _ in range(nsteps):
                e2e_step()
            complete_prev()
            sync()
            return B * nsteps * world / max_ranks(time.perf_counter() - t)

        # correctness gate on the device-resident rows first (the engine's first call)
        dev_step()
        sync()
        if int((status != 0).sum().item()):
            raise SystemExit(f"rank {rank}: samples failed to decode")
        # cold epoch: every row of the rank copied into the empty cache (nrows / B whole batches)
        epoch_steps = max(1, nrows // B)
        cold = e2e_epoch_rate(epoch_steps)
        # the downloader's queue now holds the next two batches (already in the cache): the warm passes
        # below find every destination present (skip_if_exists: one stat per row)
        dl_rates = {"cold": round(cold, 1), "cold_rows_per_rank": epoch_steps * B, "workers": dl_workers,
                    "prefetch": 2 * B, "restated": "sds_amd/downloader.py (downloader.py:25-131, "
                                                   "utils/download.py:830-861)"}
        step = e2e_step

    # correctness gate before timing: the first batch's statuses are all OK
    step()
    if e2e:
        complete_prev()
    sync()
    n_bad = pipe["bad"] if e2e else int((status != 0).sum().item())
    if n_bad:
        raise SystemExit(f"rank {rank}: {n_bad} samples failed to decode")
    for _ in range(args.warmup):
        step()

    barrier()
    sync()
    walked["rows"] = 0
    if e2e:
        for k in ph:
            ph[k] = 0.0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    t1 = time.perf_counter()
    rows_timed = walked["rows"]
    last_start = (cursor[0] - B) % nrows  # the rows `out` holds: the last timed batch (device-resident path)
    barrier()
    if e2e:  # every batch completed in the pipeline decoded completely; the last one is drained here
        complete_prev()
        sync()
        n_bad = pipe["bad"]
        dl_rates["warm"] = round(B * args.steps * world / max_ranks(t1 - t0), 1)
        dl.shutdown()
        shutil.rmtree(cache_dir, ignore_errors=True)
        shutil.rmtree(src_dir, ignore_errors=True)
    else:
        n_bad = int((status != 0).sum().item())  # the last timed batch decoded completely as well
    if n_bad:
        raise SystemExit(f"rank {rank}: {n_bad} samples of the last timed batch failed to decode")
    my_elapsed = t1 - t0
    elapsed = max_ranks(my_elapsed)
    per_rank = [my_elapsed]
    gather_dev = None
    if use_pg:
        tl = [torch.zeros(1, dtype=torch.float64, device=coll_dev or "cpu") for _ in range(world)]
        dist.all_gather(tl, torch.tensor([my_elapsed], dtype=torch.float64, device=tl[0].device))
        per_rank = [float(x.item()) for x in tl]
        world_seen = dist.get_world_size()
        gather_dev = str(tl[0].device)
    else:
        world_seen = 1
    imgs = B * args.steps * world
    value = imgs / elapsed
    step = dev_step  # the pixel check and the roofline run the device-resident path on the same rows
    dev_value = None
    if e2e:  # configs[4] asks for the rate next to the device-resident one: same rows, batch, output
        for _ in range(args.warmup):
            step()
        barrier()
        sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        sync()
        dev_value = B * args.steps * world / max_ranks(time.perf_counter() - t0)

    # pixel check after timing (device-resident path): every row of the last timed batch, then every resident
    # row of the rank (ceil(nrows / B) more batches from row 0), each compared on the device with the output
    # of its pool image -- decoded once by the engine and checked against PIL (the reference's arithmetic)
    # on the host -- plus, for configs[1], pool image 0 against the reference-generated golden digest
    pixel_check = None
    if not stub and not args.no_pixel_check:
        pixel_check = verify_rows(eng, blob, d_offs, d_lens, out, status, flips, j, period, pool, nrows, B,
                                  args.res, mixed, None if e2e else last_start, dev_step, cursor, cpu_share()[0],
                                  e2e_last=(hosts[pipe["last"]], np.asarray(pipe["keys"][pipe["last"]]) - r0)
                                  if e2e else None)
        pixel_check.update(rows_decoded_in_timed_region=rows_timed if not e2e else None,
                           distinct_rows_in_timed_region=min(nrows, rows_timed) if not e2e else None,
                           resident_rows=nrows)
        k0 = next((k for k, p in enumerate(period) if p == 0), None)
        if not mixed and args.res == 256 and k0 is not None:  # (the golden digests are of the 256x256 output)
            from tests import goldens as G
            meta = G.load_json("g2_synth.json")
            if meta.get("seed") == 1234 and (meta.get("w"), meta.get("h"), meta.get("quality")) == (640, 480, 90):
                pixel_check["golden_sha256_match"] = pixel_check.pop("_ref_sha")[k0] == meta["images"][0]["u8_256_sha256"]
        pixel_check.pop("_ref_sha", None)
        if not pixel_check["equal_to_pil"] or not pixel_check.get("golden_sha256_match", True):
            raise SystemExit(f"rank {rank}: pixel check failed: {pixel_check}")

    # roofline: every kernel timed alone in a single-lane pass (one dispatch per kernel per batch)
    eng.set_lanes(1)
    eng.set_timing(True)
    for _ in range(args.roofline_steps):
        step()
    stages = eng.stage_times()  # summed device ms per stage over the roofline steps
    eng.set_timing(False)
    eng.set_lanes(4)
    sync()

    mean_in = float(np.mean(t_lens))
    out_bytes = 3 * args.res * args.res * (4 if mixed else 1)
    alg_bytes_per_img = mean_in + out_bytes
    dom = max(stages, key=stages.get)
    launch_ms = stages[dom] / args.roofline_steps
    launch_bytes = B * alg_bytes_per_img
    achieved = launch_bytes / (launch_ms * 1e-3) / 1e9 if launch_ms > 0 else 0.0
    pmc_path = PMC_JSONS["mixed512" if mixed else "vga256"]
    traffic = pmc_traffic(dom, B, 1, pmc_path)
    if args.profile_steps and rank == 0:
        print(json.dumps({"stage_ms_per_step_single_lane": {k: v / args.roofline_steps for k, v in stages.items()}}),
              file=sys.stderr)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not stub:
        procs, procs_src = cpu_share()
        folder = tempfile.mkdtemp(prefix="sdsj_cpu_")
        try:
            paths = []
            for i in range(args.cpu_files):  # configs[0]: a local folder of JPEG files
                p = os.path.join(folder, f"{i:05d}.jpg")
                with open(p, "wb") as f:
                    f.write(pool[i % len(pool)])
                paths.append(p)
            v1 = cpu_baseline(paths, 1, args.cpu_seconds / 2, args.res, mixed)
            vp = cpu_baseline(paths, procs, args.cpu_seconds, args.res, mixed)
        finally:
            shutil.rmtree(folder, ignore_errors=True)
        import platform
        what = (f"centre crop, BILINEAR resize {args.res}x{args.res}, to CHW tensor, hflip every other image, "
                f"x/127.5-1) over a folder of {args.cpu_files} files of the {len(pool)} mixed VGA..4K pool JPEGs"
                if mixed else
                f"centre crop, BILINEAR resize {args.res}x{args.res}, to CHW tensor) over a folder of "
                f"{args.cpu_files} 640x480 q90 JPEG files (configs[0] shape)")
        cpu = {"value": round(vp, 1), "unit": "images/s", "cores": procs, "kind": "reference",
               "sample": f"PIL {__import__('PIL').__version__}/libjpeg-turbo pipeline (functional.py:94-110 op order: "
                         f"file read, open+convert RGB, {what}, {procs} processes x {args.cpu_seconds:.0f} s "
                         f"(single process: {v1:.1f} images/s; {procs} processes from {procs_src}, "
                         f"{host_cores()} CPUs visible)",
               "single_core_value": round(v1, 1), "host": platform.processor() or platform.machine()}

    if rank == 0:
        workload = (f"configs[2]: synthetic mixed VGA..4K q90 4:2:0 baseline JPEGs resident in HBM -> centre crop + "
                    f"bilinear resize {args.res}x{args.res} + hflip (p=0.5, seeded) + float32 CHW x/127.5-1"
                    if mixed else
                    f"configs[4]: synthetic 640x480 q90 JPEG files -> restated sds ParallelDownloader (local "
                    f"scheme: copy to the rank's cache directory via .tmp + rename, skip_if_exists) -> pinned slot "
                    f"-> H2D -> centre crop + bilinear resize {args.res}x{args.res} uint8 CHW -> D2H into pinned "
                    f"host memory (two slots in flight); value = warm cache (every row present: one stat per "
                    f"row), downloader.cold = the first epoch into an empty cache"
                    if e2e else
                    ("configs[3]: " if world > 1 else "configs[1]: ") +
                    f"{total_rows:,}-row {'parquet' if index_path else 'in-memory'} index, one compute_index_slice "
                    f"slice per GPU; synthetic 640x480 q90 4:2:0 baseline JPEGs resident in HBM -> "
                    f"centre crop + bilinear resize {args.res}x{args.res} uint8 CHW")
        line = {
            "metric": ("images/s device-resident JPEG decode+crop+resize@512+hflip+normalise (mixed VGA..4K)" if mixed
                       else "images/s end-to-end JPEG files -> H2D -> decode+resize@512 -> D2H (PCIe-inclusive)" if e2e
                       else "images/s device-resident JPEG decode+resize@256, 1/2/4/8 MI355X; %HBM roofline"),
            "value": round(value, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32" if mixed else "u8", "data": "synthetic",
            "config": {"workload": workload,
                       "rows_per_gpu": nrows, "distinct_images": args.pool, "global_batch": B * world,
                       "batch_per_gpu": B, "mean_jpeg_bytes": round(mean_in, 1),
                       "parallelism": f"index-sharded x{world}, no collective on the data path",
                       "index": {"rows": total_rows,
                                 "source": "synthetic parquet read with pyarrow (sds_amd/index.py)" if index_path else
                                           "in-memory index (pyarrow not importable)",
                                 "slices": slices}},
            "per_rank_images_per_s": [round(B * args.steps / t, 1) for t in per_rank],
            "process_group": {"backend": dist.get_backend() if use_pg else None, "world_size": world_seen,
                              "gpus_visible": ndev if not stub else 0, "forced_at_world_size_1": bool(args.force_pg),
                              "all_gather_device": gather_dev},
            # bound: of the schema's roofs (HBM, MFMA) the path can only be priced against HBM -- it issues
            # no MFMA; `limiter` says from the counters which roof (HBM bytes or VALU issue) it is nearest
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": (traffic or {}).get("bytes_per_launch"),
                         "traffic_detail": traffic,
                         "algorithmic_bytes_per_launch": round(launch_bytes),
                         "algorithmic_bytes_per_image": round(alg_bytes_per_img, 1),
                         "launch_ms": round(launch_ms, 4), "images_per_launch": B, "lanes": 1,
                         "timing": "HIP events on the launch stream, single-lane pass after the timed region",
                         "limiter": measured_limiter(dom, B, launch_ms, traffic, pmc_path),
                         "pipeline_achieved": round(value / world * alg_bytes_per_img / 1e9, 2)},
            "stage_ms_per_step_single_lane": {k: round(v / args.roofline_steps, 4) for k, v in stages.items()},
            "pixel_check": pixel_check,
            "cpu_baseline": cpu,
        }
        if e2e:
            line["device_resident_value"] = round(dev_value, 1)
            line["e2e_over_device_resident"] = round(value / dev_value, 4)
            line["downloader"] = dl_rates
            line["e2e_out"] = args.e2e_out
            line["e2e_host_ms_per_step"] = {k: round(v / args.steps * 1e3, 3) for k, v in ph.items()}
            line["e2e_host_ms_per_step"]["step"] = round(elapsed / args.steps * 1e3, 3)
            line["roofline"]["note"] = "device-resident kernels of the same rows (the PCIe legs are not kernels)"
        print(json.dumps(line), file=result_out, flush=True)
    if use_pg:
        dist.barrier()
        dist.destroy_process_group()
    if index_path and rank == 0:
        try:
            os.remove(index_path)
        except OSError:
            pass


if __name__ == "__main__":
    main()
