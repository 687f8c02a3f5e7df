"""Parquet sample index for the multi-GPU workload (BASELINE.json configs[3]: a 1M-row synthetic parquet
index sharded one slice per GPU).

Restates the two reference pieces the sharding needs, for a local parquet file:
  * sds/index.py:208-215 load_index_partition -> compute_index_slice (sds/index.py:227-246, INTER_NODE,
    contiguous; sds_amd/distributed.py) -> data_utils.read_parquet_slice;
  * sds/utils/data_utils.py:19-93 read_parquet_slice, step 1: row groups wholly before the slice are
    skipped by their metadata, the ones it touches are read and cut, nothing after its end is read.
The index rows follow sds's index layout (sds/index.py:176-203 build_index_from_files_list: an
``index`` column plus one column per file extension holding the sample's path), with the synthetic
pool image each row refers to.  pyarrow is the only dependency (imported lazily).
"""
from __future__ import annotations

import numpy as np

from .distributed import compute_index_slice


def write_synthetic_index(path: str, num_samples: int, pool: int, row_group_size: int = 65536) -> None:
    """``num_samples`` rows: index i, jpg = the path key of pool image i % pool, pool_image = i % pool."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    idx = np.arange(num_samples, dtype=np.int64)
    img = (idx % pool).astype(np.int32)
    names = np.array([f"pool/{k:05d}.jpg" for k in range(pool)], dtype=object)
    table = pa.table({"index": idx, "jpg": pa.array(names[img], type=pa.string()), "pool_image": img})
    pq.write_table(table, path, row_group_size=row_group_size)


def read_parquet_slice(path: str, start: int, end: int, columns=None):
    """sds/utils/data_utils.py:19-93 (step 1) for a local file: the rows [start, end) as a pyarrow Table."""
    import pyarrow as pa
    import pyarrow.parquet as pq
    pf = pq.ParquetFile(path)
    seen, parts = 0, []
    for i in range(pf.num_row_groups):
        n = pf.metadata.row_group(i).num_rows
        if seen + n < start:  # (the reference's test: a group ending exactly at start is still read)
            seen += n
            continue
        if seen >= end:
            break
        t = pf.read_row_group(i, columns=columns)
        lo, hi = max(0, start - seen), min(n, end - seen)
        if hi > lo:
            parts.append(t.slice(lo, hi - lo))
        seen += n
    if not parts:
        schema = pf.schema_arrow
        if columns:
            schema = pa.schema([f for f in schema if f.name in columns])
        return schema.empty_table()
    return pa.concat_tables(parts)


def load_index_partition(path: str, num_samples: int, rank: int, num_ranks: int, columns=None):
    """sds/index.py:208-215: (start, end, rows of this rank's slice)."""
    start, end, _ = compute_index_slice(num_samples, rank, num_ranks)
    return start, end, read_parquet_slice(path, start, end, columns)
