"""World-size-2 gloo test of the multi-GPU data path: index slices per rank (no collective on the
data) and the max-over-ranks timing reduction that bench.py reports."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_rows, q):
    import torch
    import torch.distributed as dist

    from sds_amd.distributed import compute_index_slice, max_over_ranks
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s, e, st = compute_index_slice(n_rows, rank, world)
    rows = torch.arange(s, e, st, dtype=torch.int64)
    lens = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(lens, torch.tensor([rows.numel()]))
    gathered = [torch.zeros(int(l.item()), dtype=torch.int64) for l in lens]
    dist.all_gather(gathered, rows)
    elapsed = max_over_ranks(1.0 + rank)
    if rank == 0:
        q.put((torch.cat(gathered).tolist(), elapsed))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("n_rows", [10, 1001])
def test_two_rank_slices_partition_the_index(n_rows):
    ctx = mp.get_context("spawn")
    q = ctx.SimpleQueue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, n_rows, q)) for r in range(2)]
    for p in procs:
        p.start()
    rows, elapsed = q.get()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert rows == list(range(2 * (n_rows // 2)))  # disjoint, ordered, reference drops the remainder
    assert elapsed == 2.0
