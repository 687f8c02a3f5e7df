"""The parquet sample index of the multi-GPU workload (sds_amd/index.py): sds/index.py:208-246
load_index_partition / compute_index_slice and sds/utils/data_utils.py:19-93 read_parquet_slice (step 1)
restated for a local file -- every rank's rows, row-group boundaries, empty slices."""
import os
import tempfile

import numpy as np
import pytest

pa = pytest.importorskip("pyarrow")

from sds_amd.distributed import compute_index_slice  # noqa: E402
from sds_amd.index import load_index_partition, read_parquet_slice, write_synthetic_index  # noqa: E402


@pytest.fixture(scope="module")
def index_file():
    d = tempfile.mkdtemp()
    p = os.path.join(d, "index.parquet")
    write_synthetic_index(p, 10_007, 37, row_group_size=1000)
    return p


def test_synthetic_index_layout(index_file):
    import pyarrow.parquet as pq
    t = pq.read_table(index_file)
    assert t.column_names == ["index", "jpg", "pool_image"] and t.num_rows == 10_007
    assert pq.ParquetFile(index_file).num_row_groups == 11
    idx = t.column("index").to_numpy()
    assert np.array_equal(idx, np.arange(10_007))
    assert np.array_equal(t.column("pool_image").to_numpy(), idx % 37)
    assert t.column("jpg")[40].as_py() == "pool/00003.jpg"


@pytest.mark.parametrize("lo,hi", [(0, 0), (0, 1), (999, 1001), (1000, 2000), (1000, 1000), (3, 10_007),
                                   (9_999, 10_007), (10_007, 10_007), (5_500, 5_501)])
def test_read_parquet_slice_matches_the_full_table(index_file, lo, hi):
    import pyarrow.parquet as pq
    full = pq.read_table(index_file)
    got = read_parquet_slice(index_file, lo, hi)
    assert got.num_rows == hi - lo and got.schema == full.schema
    assert got.equals(full.slice(lo, hi - lo))


@pytest.mark.parametrize("ranks", [1, 2, 3, 8])
def test_partitions_cover_compute_index_slice(index_file, ranks):
    seen = []
    for r in range(ranks):
        s, e, t = load_index_partition(index_file, 10_007, r, ranks, columns=["index"])
        assert (s, e, 1) == compute_index_slice(10_007, r, ranks)
        ids = t.column("index").to_numpy()
        assert np.array_equal(ids, np.arange(s, e))
        seen.extend(ids.tolist())
    # the last N % R rows are dropped, as sds/index.py:235-246 does
    assert seen == list(range(ranks * (10_007 // ranks)))
