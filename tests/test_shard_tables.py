"""CPU: the canonical order the sharded-aggregation parity compares tables in (host logic only)."""
import numpy as np

from siddhi_amd.shard import canonical_table, merge_tables


def table(rows):
    """rows: (bucket, key, v0, v1) -> out_arrays-like dict"""
    a = np.array(rows, dtype=np.int64).reshape(-1, 4).T
    return {"keys": a[:2].copy(), "vals": a[2:].astype(np.uint64), "nulls": np.zeros((2, a.shape[1]), np.uint8)}


def test_union_of_owner_tables_is_sorted_by_bucket_then_key():
    a = table([(2000, 5, 1, 1), (1000, 7, 2, 2), (1000, 3, 3, 3)])
    b = table([(1000, 4, 4, 4), (2000, 2, 5, 5)])
    m = merge_tables([a, b])
    assert m["keys"].T.tolist() == [[1000, 3], [1000, 4], [1000, 7], [2000, 2], [2000, 5]]
    assert m["vals"][0].tolist() == [3, 4, 2, 5, 1]
    # the single table holding the same rows in another order compares equal
    s = canonical_table(table([(1000, 4, 4, 4), (2000, 5, 1, 1), (1000, 3, 3, 3), (2000, 2, 5, 5), (1000, 7, 2, 2)]))
    assert all(np.array_equal(m[k], s[k]) for k in ("keys", "vals", "nulls"))


def test_empty_tables_merge():
    e = table([])
    m = merge_tables([e, e])
    assert m["keys"].shape == (2, 0)
