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
