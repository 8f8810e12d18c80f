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


def owner_out(order, clocks_per_flush, flush_offsets, vals):
    order = np.asarray(order, np.int64)
    n = order.size
    return {"order": order, "flush_offsets": np.asarray(flush_offsets, np.int64),
            "flush_clock": np.asarray(clocks_per_flush, np.int64), "ts": order * 10, "expired": np.zeros(n, np.uint8), "rep": order + 3,
            "keys": order[None, :] % 5, "vals": np.asarray(vals, np.uint64)[None, :], "nulls": np.zeros((1, n), np.uint8),
            "val_types": np.zeros(1, np.int32)}


def test_sliding_owner_outputs_merge_per_send():
    """Sliding windows: one flush per send (consecutive sends may share a clock); rows of a send in the
    order of their first events across owners (siddhi_amd.shard._merge_by_send)."""
    from siddhi_amd.shard import merge_owner_outputs
    # push starts at global index 100, send_size 4: sends 0 = [100,104), 1 = [104,108), 2 = [108,112)
    a = owner_out([101, 103, 109], [7, 8], [0, 2, 3], [1, 2, 3])        # sends 0 and 2
    b = owner_out([100, 105, 106, 111], [7, 7, 8], [0, 1, 3, 4], [4, 5, 6, 7])  # sends 0, 1, 2
    m = merge_owner_outputs([a, b], sends=(100, 4))
    assert m["order"].tolist() == [100, 101, 103, 105, 106, 109, 111]
    assert m["flush_offsets"].tolist() == [0, 3, 5, 7]
    assert m["flush_clock"].tolist() == [7, 7, 8]   # sends 0 and 1 share clock 7 but stay separate flushes
    assert m["vals"][0].tolist() == [4, 1, 2, 5, 6, 3, 7]
    e = merge_owner_outputs([owner_out([], [], [0], []), owner_out([], [], [0], [])], sends=(0, 1))
    assert e["flush_offsets"].tolist() == [0] and e["keys"].shape == (1, 0)


def test_merge_sends_per_query_kind():
    """how owners' flushes merge: by window for batch windows; by send for sliding windows and
    timeBatch(T, true); by passing event for lengthBatch(L, true)"""
    from siddhi_amd import abi
    from siddhi_amd.shard import merge_sends
    sch = abi.Schema.parse("k int, v double, ts long")
    q = lambda w, sc=False: abi.QuerySpec(sch, w, 100, group_by=["k"], aggs=[("count", None)], stream_current=sc)
    assert merge_sends(q("timeBatch"), (7, 4)) is None
    assert merge_sends(q("lengthBatch"), (7, 4)) is None
    assert merge_sends(q("time"), (7, 4)) == (7, 4)
    assert merge_sends(q("timeBatch", True), (7, 4)) == (7, 4)
    assert merge_sends(q("lengthBatch", True), (7, 4)) == (7, 1)
