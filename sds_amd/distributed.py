"""Per-GPU sharding of a sample index (no collective on the data path).

Mirrors ``sds.index.compute_index_slice`` (sds/index.py:227-246) for the INTER_NODE index type:
rank r of R owns rows [r * (N // R), (r + 1) * (N // R)) (contiguous) or r, r + R, ...
(interleaved), the last ``N % R`` rows being dropped exactly as in the reference.
"""
from __future__ import annotations

import os


def compute_index_slice(num_samples: int, rank: int, num_ranks: int, interleaved: bool = False) -> tuple[int, int, int]:
    per_rank = num_samples // num_ranks
    start = rank if interleaved else rank * per_rank
    step = num_ranks if interleaved else 1
    end = min(start + per_rank * step, num_samples)
    return start, end, step


def env_rank() -> tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1)),
            int(os.environ.get("LOCAL_RANK", 0)))


def max_over_ranks(value: float, device=None, always: bool = False) -> float:
    """Maximum of a per-rank scalar (the bench's timed region), via all_reduce(MAX).  ``always``: run the
    collective at world size 1 too (a process group created only to exercise its backend)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or (dist.get_world_size() == 1 and not always):
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
