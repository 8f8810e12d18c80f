"""GPU parity of the key-sharded incremental aggregation (C4 across G GPUs): G
owners, each fed a send-aligned slice of every global push and re-keyed through the sh_shard_*
protocol, must together hold exactly the single-stream oracle's roll-up tables at every duration —
the same (bucket, key) rows with bit-identical base values. Tables are keyed by
(AGG_TIMESTAMP, group key) (AggregationParser.initDefaultTables, @PrimaryKey), so rows are compared
in canonical (bucket, key) order.

The owners run in one process on one device and exchange through device copies (LocalShards); the
multi-process transport (torch.distributed all-to-all) carries the same bytes."""
import numpy as np
import pytest

from oracle.oracle import OracleAggregation
from siddhi_amd import abi, synth
from tests.parity import split_batches

pytestmark = pytest.mark.gpu


def cut_slices(ts, cols, world, fracs, send_size, dev):
    import torch
    n = len(ts)
    units = (n + send_size - 1) // send_size
    edges = [0] + sorted(min(n, int(units * f) * send_size) for f in fracs) + [n]
    out = []
    for g in range(world):
        a, b = edges[g], edges[g + 1]
        out.append((torch.from_numpy(np.ascontiguousarray(ts[a:b])).to(dev),
                    [torch.from_numpy(np.ascontiguousarray(c[a:b])).to(dev) for c in cols]))
    return out


def run_both(spec, world, pushes, send_size, fracs, advance):
    """pushes: list of (ts, cols) global pushes. Returns {duration: (sharded table, oracle table)}."""
    import torch
    from siddhi_amd.shard import LocalShards, canonical_table
    dev = torch.device("cuda", 0)
    ls = LocalShards(spec, world)
    o = OracleAggregation(spec)
    for i, (ts, cols) in enumerate(pushes):
        ls.push(cut_slices(ts, cols, world, fracs[i % len(fracs)], send_size, dev), send_size, dev)
        o.push(abi.HostBatch(spec.schema, ts, cols, send_size))
    for now in advance:
        ls.advance_time(now)
        o.advance_time(now)
    lo, hi = abi.DUR_NAMES[spec.durations[0]], abi.DUR_NAMES[spec.durations[1]]
    res = {}
    for d in range(lo, hi + 1):
        res[d] = (ls.tables(d), canonical_table(abi.out_arrays(o.table_raw(d))))
    ls.close()
    o.close()
    return res


def assert_tables(res, label):
    total = 0
    for d, (g, o) in res.items():
        assert g["keys"].shape == o["keys"].shape, f"{label} dur {d}: {g['keys'].shape} vs {o['keys'].shape} rows"
        assert np.array_equal(g["keys"], o["keys"]), f"{label} dur {d}: (bucket, key) rows differ"
        for b in range(o["vals"].shape[0]):
            bad = np.nonzero((g["vals"][b] != o["vals"][b]) | (g["nulls"][b] != o["nulls"][b]))[0]
            assert bad.size == 0, f"{label} dur {d} base {b}: differs at rows {bad[:8]}"
        total += o["keys"].shape[1]
    assert total > 0
    return total


def split(ts, cols, sizes):
    out, a = [], 0
    for s in sizes:
        out.append((ts[a:a + s], [c[a:a + s] for c in cols]))
        a += s
    return out


@pytest.mark.parametrize("world,key_type", [(2, "int"), (3, "string"), (8, "string")])
def test_sharded_c4_event_time_rollups(world, key_type):
    schema = abi.Schema.parse(f"k {key_type}, v double, ts long")
    ts, cols = synth.keyed_stream(1_700_000_000_000 - 15_000, 240_000, 0xC4, 3_000, 5)
    spec = abi.AggregationSpec(schema, [("sum", "v"), ("avg", "v"), ("count", None), ("min", "v"), ("max", "v")],
                               group_by=["k"], ts="ts", durations=("sec", "day"), key_capacity=3_000)
    fr = [[(g + 1) / world for g in range(world - 1)], [0.02 * (g + 1) for g in range(world - 1)]]
    res = run_both(spec, world, split(ts, cols, [100_000, 1, 139_999]), 1, fr,
                   [int(ts[-1]) + 3_600_000 * 30])
    assert_tables(res, f"C4 x{world}")


def test_sharded_late_events_chunked_sends_and_gaps():
    rng = np.random.default_rng(23)
    n = 80_000
    clock = 1_706_745_000_000 + np.cumsum(rng.integers(0, 20, n)).astype(np.int64)
    ext = clock - rng.integers(0, 60_000, n).astype(np.int64)
    k = rng.integers(0, 97, n).astype(np.int32)
    v = np.round(rng.normal(100, 30, n), 2)
    schema = abi.Schema.parse("k int, v double, ts long")
    spec = abi.AggregationSpec(schema, [("sum", "v"), ("count", None), ("max", "v"), ("min", "v")], group_by=["k"],
                               ts="ts", durations=("sec", "year"), key_capacity=128, filter=(">", "v", 80.0))
    pushes = [(clock[: n // 2], [k[: n // 2], v[: n // 2], ext[: n // 2]]),
              (clock[n // 2:], [k[n // 2:], v[n // 2:], ext[n // 2:]])]
    res = run_both(spec, 4, pushes, 250, [[0.1, 0.5, 0.7]],
                   [int(clock[-1]) + 40 * 86_400_000, int(clock[-1]) + 400 * 86_400_000])
    assert_tables(res, "late x4")


def test_sharded_processing_time_rollups():
    schema = abi.Schema.parse("k int, v double, ts long")
    ts, cols = synth.keyed_stream(1_600_000_000_000, 100_000, 7, 300, 2)
    spec = abi.AggregationSpec(schema, [("sum", "v"), ("count", None)], group_by=["k"], ts=None,
                               durations=("sec", "hour"), key_capacity=300)
    res = run_both(spec, 2, split(ts, cols, [30_000, 70_000]), 100, [[0.6]], [int(ts[-1]) + 90_000_000])
    assert_tables(res, "proc-time x2")


@pytest.mark.parametrize("key_type", ["int", "string"])
def test_sharded_aggregation_checkpoint(key_type):
    """sh_shard_snapshot of a key-sharded aggregation carries each owner's root window, roll-up
    executors and tables: G owners snapshotted between two global pushes and restored into fresh
    owners (a truncated blob refused first, leaving the owner as it was) end with the oracle's tables."""
    import torch
    from siddhi_amd.shard import LocalShards, canonical_table
    dev = torch.device("cuda", 0)
    world = 3
    schema = abi.Schema.parse(f"k {key_type}, v double, ts long")
    ts, cols = synth.keyed_stream(1_700_000_000_000 - 15_000, 180_000, 0xC4, 2_000, 5)
    spec = abi.AggregationSpec(schema, [("sum", "v"), ("avg", "v"), ("count", None), ("min", "v"), ("max", "v")],
                               group_by=["k"], ts="ts", durations=("sec", "hour"), key_capacity=2_000)
    pushes = split(ts, cols, [70_000, 50_000, 60_000])
    fr = [(g + 1) / world for g in range(world - 1)]
    ls = LocalShards(spec, world)
    o = OracleAggregation(spec)
    for i, (t, c) in enumerate(pushes):
        if i == 2:
            blobs, seq = ls.snapshot(), ls.seq
            with pytest.raises(Exception, match="truncated|does not match|restore"):
                ls.shards[0].restore(blobs[0][:len(blobs[0]) - 7])
            ls.close()
            ls = LocalShards(spec, world)
            ls.restore(blobs, seq)
        ls.push(cut_slices(t, c, world, fr, 1, dev), 1, dev)
        o.push(abi.HostBatch(spec.schema, t, c, 1))
    end = int(ts[-1]) + 3 * 3_600_000
    ls.advance_time(end)
    o.advance_time(end)
    res = {d: (ls.tables(d), canonical_table(abi.out_arrays(o.table_raw(d))))
           for d in range(abi.DUR_SECONDS, abi.DUR_HOURS + 1)}
    ls.close()
    o.close()
    assert assert_tables(res, f"checkpointed C4 x{world} {key_type}") > 2_000
