"""GPU checkpoint parity (f3; State.snapshot/restore, SnapshotService): a query snapshotted after some
pushes and restored into a fresh query built from the same descriptor must continue exactly as the
uninterrupted run — compared, bit for bit, with the oracle run over the whole stream."""
import numpy as np
import pytest

from oracle.oracle import OracleQuery
from siddhi_amd import abi, synth
from tests.parity import assert_same, run_pushes, split_batches

pytestmark = pytest.mark.gpu


def checkpointed(spec, pushes, cut):
    from siddhi_amd import runtime
    g = runtime.GpuQuery(spec)
    a = run_pushes(g, pushes[:cut])
    blob = g.snapshot()
    g.close()
    g2 = runtime.GpuQuery(spec)
    g2.restore(blob)
    b = run_pushes(g2, pushes[cut:])
    g2.close()
    o = OracleQuery(spec)
    ref = run_pushes(o, pushes)
    o.close()
    return abi.concat_arrays([a, b]), ref, len(blob)


C1 = abi.Schema.parse("symbol string, price double, volume long, ts long")
C2 = abi.Schema.parse("k int, v double, ts long")


@pytest.mark.parametrize("cut", [1, 2])
def test_lengthbatch_checkpoint(cut):
    ts, cols = synth.c1_stock(0, 120_000)
    spec = abi.QuerySpec(C1, "lengthBatch", 7000, group_by=["symbol"], aggs=[("sum", "volume"), ("avg", "price")],
                         filter=(">", "price", 100), key_capacity=1000)
    pushes = split_batches(C1, ts, cols, [33_333, 50_001, 90_000], 100)
    got, ref, nbytes = checkpointed(spec, pushes, cut)
    assert nbytes > 1000  # the open batch's queued events travel in the blob
    assert_same(got, ref, label="lengthBatch ckpt")


def test_timebatch_hashed_keys_checkpoint_mid_window():
    ts, cols = synth.keyed_stream(0, 400_000, 0xC2, 50_000, 100)
    spec = abi.QuerySpec(C2, "timeBatch", 1000, group_by=["k"], start_time=250,
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=50_000)
    pushes = split_batches(C2, ts, cols, [123_457, 250_000], 1)
    pushes.append(("advance", int(ts[-1]) + 5000))
    got, ref, _ = checkpointed(spec, pushes, 1)
    assert_same(got, ref, label="timeBatch ckpt")


def test_sliding_checkpoint_keeps_rings_and_deques():
    ts, cols = synth.keyed_stream(0, 150_000, 0xC3, 2_000, 20, quantized=True)
    spec = abi.QuerySpec(C2, "time", 3_000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v"), ("sum", "v")],
                         key_capacity=2_000)
    pushes = split_batches(C2, ts, cols, [60_000, 61_000], 1)
    got, ref, _ = checkpointed(spec, pushes, 2)
    assert_same(got, ref, label="sliding ckpt")


def test_sliding_rollback_into_a_running_query_whose_rings_grew():
    """Restore an earlier revision into the SAME running query after its per-key rings grew past the
    snapshot's capacity (SnapshotService.restoreRevision into a live runtime): the rings are rebuilt at
    the snapshot's capacity, never copied over, and the query continues like the uninterrupted run."""
    from siddhi_amd import runtime
    ts, cols = synth.keyed_stream(0, 200_000, 0xC3, 64, 20)
    spec = abi.QuerySpec(C2, "time", 5_000, group_by=["k"], aggs=[("count", None), ("min", "v"), ("avg", "v")],
                         key_capacity=64)
    pushes = split_batches(C2, ts, cols, [2_000, 150_000], 1)
    g = runtime.GpuQuery(spec)
    a = run_pushes(g, pushes[:1])        # ~30 events per key: small rings
    blob = g.snapshot()
    run_pushes(g, pushes[1:2])           # ~1500 events per key: the rings grow
    g.restore(blob)                      # roll back into the grown query
    b = run_pushes(g, pushes[1:])
    g.close()
    o = OracleQuery(spec)
    ref = run_pushes(o, pushes)
    o.close()
    assert_same(abi.concat_arrays([a, b]), ref, label="sliding rollback")


def test_partitioned_timebatch_checkpoint():
    rng = np.random.default_rng(5)
    n = 30_000
    ts = 1_000 + np.arange(n, dtype=np.int64) // 3
    sym = rng.integers(0, 4, n).astype(np.int32)
    v = rng.integers(0, 100, n).astype(np.int64)
    sch = abi.Schema.parse("symbol string, v long, ts long")
    spec = abi.QuerySpec(sch, "timeBatch", 500, group_by=["symbol"], aggs=[("sum", "v"), ("count", None)],
                         partition="symbol", key_capacity=8)
    pushes = split_batches(sch, ts, [sym, v, ts.copy()], [10_000, 20_000], 1)
    got, ref, _ = checkpointed(spec, pushes, 1)
    assert_same(got, ref, label="partition ckpt")


def test_restore_into_a_different_query_fails_loudly():
    from siddhi_amd import runtime
    ts, cols = synth.keyed_stream(0, 5_000, 0xC2, 100, 10)
    a = abi.QuerySpec(C2, "timeBatch", 1000, group_by=["k"], aggs=[("count", None)], key_capacity=128)
    b = abi.QuerySpec(C2, "timeBatch", 2000, group_by=["k"], aggs=[("count", None)], key_capacity=128)
    g = runtime.GpuQuery(a)
    g.push(abi.HostBatch(C2, ts, cols, 1))
    blob = g.snapshot()
    h = runtime.GpuQuery(b)
    with pytest.raises(runtime.SiddhiError, match="different query"):
        h.restore(blob)
    with pytest.raises(runtime.SiddhiError):
        runtime.GpuQuery(a).restore(blob[:40])


@pytest.mark.parametrize("window", ["timeBatch", "time"])
def test_truncated_blob_leaves_query_unchanged(window):
    """A restore from a truncated blob fails and leaves the query exactly as it was (sh_query_restore
    snapshots the current state first and rolls back): the query, restored from a blob cut at several
    points after it moved on, continues identically to the uninterrupted oracle."""
    from siddhi_amd import runtime
    ts, cols = synth.keyed_stream(0, 200_000, 0xC2, 5_000, 50, quantized=True)
    spec = abi.QuerySpec(C2, window, 700, group_by=["k"], aggs=[("count", None), ("min", "v"), ("sum", "v")],
                         key_capacity=5_000)
    pushes = split_batches(C2, ts, cols, [60_000, 120_000], 1)
    g = runtime.GpuQuery(spec)
    a = run_pushes(g, pushes[:1])
    blob = g.snapshot()
    b = run_pushes(g, pushes[1:2])  # moves on past the snapshot
    for cut in (24, len(blob) // 3, len(blob) - 9):
        with pytest.raises(Exception, match="truncated|does not match|restore"):
            g.restore(blob[:cut])
    c = run_pushes(g, pushes[2:])
    g.close()
    o = OracleQuery(spec)
    ref = run_pushes(o, pushes)
    o.close()
    assert_same(abi.concat_arrays([a, b, c]), ref, label=f"{window} after failed restores")


# ---- checkpoints of the state that round 2 refused: expired / all-events output (the carried batch,
# the sliding expiry FIFO), pass-through sliding windows and every output rate limiter ------------------
def _xstream(n=120_000, keys=3_000, per_ms=40):
    ts, cols = synth.keyed_stream(0, n, 0xE5, keys, per_ms, quantized=True)
    return ts, cols


@pytest.mark.parametrize("window,param,output,group", [
    ("timeBatch", 500, "all", True), ("lengthBatch", 4_000, "expired", True), ("timeBatch", 700, "all", False),
    ("time", 400, "all", True), ("time", 300, "expired", False), ("time", 250, "current", None)])
def test_expired_output_checkpoint(window, param, output, group):
    """(group None: `select *` pass-through, whose sliding form keeps the expiry FIFO too)"""
    ts, cols = _xstream()
    aggs = [] if group is None else [("count", None), ("min", "v"), ("sum", "v")]
    spec = abi.QuerySpec(C2, window, param, group_by=["k"] if group else [], aggs=aggs, output=output,
                         key_capacity=3_000)
    pushes = split_batches(C2, ts, cols, [40_000, 41_000, 90_000], 1)
    pushes.append(("advance", int(ts[-1]) + 5_000))
    for cut in (1, 3):
        got, ref, _ = checkpointed(spec, pushes, cut)
        assert_same(got, ref, label=f"{window} {output} ckpt at {cut}")


@pytest.mark.parametrize("rate", [("all", 7), ("first", 5), ("last", 6), ("first_time", 300)])
@pytest.mark.parametrize("group", [True, False])
def test_rate_limited_checkpoint(rate, group):
    """the limiter's counters, carried rows and key tables travel in the blob (restored into a query
    with the same `output ... every`)"""
    ts, cols = _xstream(80_000, 500, 20)
    spec = abi.QuerySpec(C2, "lengthBatch", 900, group_by=["k"] if group else [],
                         aggs=[("count", None), ("max", "v")], rate=rate, key_capacity=500)
    pushes = split_batches(C2, ts, cols, [20_011, 50_000], 3)
    got, ref, _ = checkpointed(spec, pushes, 1)
    assert_same(got, ref, label=f"rate {rate} group {group} ckpt")


@pytest.mark.parametrize("window,param,output,sc", [("lengthBatch", 5, "all", False), ("lengthBatch", 3, "current", True),
                                                    ("time", 120, "all", False), ("time", 300, "expired", False)])
@pytest.mark.parametrize("cut", [1, 2])
def test_partition_lanes_checkpoint(window, param, output, sc, cut):
    """The partition lanes (sh_plane.cpp): per-partition window / aggregator state, and for time windows the
    host-side Scheduler — pending notify times per partition and PartitionStateHolder.states' HashMap
    structure (string partition keys, many of one hash: tree bins) — restored into a fresh query."""
    from tests.test_gpu_partition import _same_hash_strings
    schema = abi.Schema.parse("p string, v double, ts long")
    names = _same_hash_strings(4) + [f"sym{i}" for i in range(200)]
    rng = np.random.default_rng(17 + cut)
    n = 60_000
    ts = (np.cumsum(rng.integers(0, 2, n)) + 10_000).astype(np.int64)
    p = np.where(rng.random(n) < 0.4, rng.integers(0, 16, n), rng.integers(16, len(names), n)).astype(np.int32)
    v = rng.integers(-400, 400, n).astype(np.float64) / 8.0
    spec = abi.QuerySpec(schema, window, param, aggs=[("count", None), ("sum", "v"), ("max", "v")], partition="p",
                         output=output, stream_current=sc, key_capacity=256, strings={"p": names})
    pushes = split_batches(schema, ts, [p, v, ts.copy()], [20_000, 41_000], 1)
    pushes.append(("advance", int(ts[-1]) + 1_000))
    got, ref, _ = checkpointed(spec, pushes, cut)
    assert_same(got, ref, label=f"lanes ckpt {window} {output}")


@pytest.mark.parametrize("output", ["current", "all"])
@pytest.mark.parametrize("cut", [1, 2])
def test_partition_group_lanes_checkpoint(output, cut):
    """lane 3 (partitioned lengthBatch grouped by another column): the carried open and last completed
    batches and the group key table, restored into a fresh query"""
    from tests.test_gpu_partition import GSCHEMA, gstream
    ts, cols = gstream(60_000, 40, 9, 19 + cut)
    spec = abi.QuerySpec(GSCHEMA, "lengthBatch", 50, group_by=["g"], aggs=[("count", None), ("sum", "v"), ("min", "x")],
                         partition="p", output=output, key_capacity=128)
    pushes = split_batches(GSCHEMA, ts, cols, [20_000, 41_000], 1)
    got, ref, _ = checkpointed(spec, pushes, cut)
    assert_same(got, ref, label=f"group lanes ckpt {output}")


@pytest.mark.parametrize("rate,group_by", [(("all", 3), []), (("first", 2), []), (("first_time", 50), []),
                                           (("last", 4), ["g"]), (("first", 3), ["g"])])
def test_partition_lanes_rate_checkpoint(rate, group_by):
    """per-partition limiters: counters, output times and carried rows with their partitions"""
    from tests.test_gpu_rate import PSCHEMA, pstream
    ts, cols = pstream(30_000, 23, 13)
    spec = abi.QuerySpec(PSCHEMA, "lengthBatch", 3, group_by=group_by, aggs=[("count", None), ("sum", "v")], partition="p",
                         output="all", key_capacity=64, rate=rate)
    pushes = split_batches(PSCHEMA, ts, cols, [10_000, 20_001], 1)
    got, ref, _ = checkpointed(spec, pushes, 1)
    assert_same(got, ref, label=f"lanes rate ckpt {rate}")


@pytest.mark.parametrize("cut", [1, 2])
def test_partition_time_group_lanes_checkpoint(cut):
    """time lanes grouped by other columns: the rings (with each entry's group), the (partition, group)
    states and both key tables, and the Scheduler, restored into a fresh query"""
    from tests.test_gpu_partition import GSCHEMA, gstream
    ts, cols = gstream(50_000, 30, 5, 29 + cut)
    spec = abi.QuerySpec(GSCHEMA, "time", 200, group_by=["g"], aggs=[("count", None), ("sum", "v"), ("min", "v"),
                                                                     ("max", "x")], partition="p",
                         output="all", key_capacity=128)
    pushes = split_batches(GSCHEMA, ts, cols, [15_000, 33_000], 1) + [("advance", int(ts[-1]) + 1_000)]
    got, ref, _ = checkpointed(spec, pushes, cut)
    assert_same(got, ref, label=f"time group lanes ckpt {cut}")


@pytest.mark.parametrize("window,group_by", [("time", []), ("lengthBatch", []), ("time", ["g"]), ("lengthBatch", ["g"])])
def test_truncated_partition_lane_blob_leaves_query_unchanged(window, group_by):
    """Partition lanes (one lane per partition, lane 3, the grouped time lanes): a truncated blob cut in the
    device section, in the host Scheduler section and in the pair / group tables fails and the query — it
    has moved on past the snapshot — continues identically to the uninterrupted oracle (the restore rolls
    back to the state it snapshotted first)."""
    from siddhi_amd import runtime
    from tests.test_gpu_partition import GSCHEMA, gstream
    ts, cols = gstream(45_000, 60, 9, 23)
    spec = abi.QuerySpec(GSCHEMA, window, 120 if window == "time" else 7, group_by=group_by,
                         aggs=[("count", None), ("sum", "v"), ("max", "v")], partition="p", output="all",
                         key_capacity=128)
    pushes = split_batches(GSCHEMA, ts, cols, [15_000, 30_000], 1) + [("advance", int(ts[-1]) + 1_000)]
    g = runtime.GpuQuery(spec)
    a = run_pushes(g, pushes[:1])
    blob = g.snapshot()
    b = run_pushes(g, pushes[1:2])
    for cut in (24, len(blob) // 4, len(blob) // 2, len(blob) - 40, len(blob) - 3):
        with pytest.raises(Exception, match="truncated|does not match|restore|unreadable"):
            g.restore(blob[:cut])
    c = run_pushes(g, pushes[2:])
    g.close()
    o = OracleQuery(spec)
    ref = run_pushes(o, pushes)
    o.close()
    assert_same(abi.concat_arrays([a, b, c]), ref, label=f"lanes {window} {group_by} after failed restores")
