"""Double-buffered host ingest (sh_stage / sh_push_staged): pinned SoA micro-batches copied on the
copy stream while the previous batch is processed give exactly the output of sh_push and of the
oracle (InputHandler.send(Event[]) per micro-batch, InputHandler.java:85-96). Small batches of batch
windows are read in place by the small-push kernel (zero-copy), and copied on the compute stream when
they close a window."""
import numpy as np
import pytest

from oracle.oracle import OracleQuery
from siddhi_amd import abi, synth
from tests.parity import assert_same, run_pushes

pytestmark = pytest.mark.gpu

SCHEMA = abi.Schema.parse("k string, v double, ts long")


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def staged_run(rt, g, schema, ts, cols, chunk, send_size):
    """Stage batch i+1 before pushing batch i (two pinned buffers in rotation)."""
    bufs = [rt.PinnedBatch(schema, chunk), rt.PinnedBatch(schema, chunk)]
    edges = list(range(0, len(ts), chunk)) + [len(ts)]
    parts, tickets = [], []
    for i, (a, b) in enumerate(zip(edges[:-1], edges[1:])):
        pb = bufs[i % 2].fill(ts[a:b], [c[a:b] for c in cols], send_size)
        tickets.append(g.stage(pb))
        if len(tickets) == 2:
            parts.append(abi.out_arrays(g.push_staged_raw(tickets.pop(0))))
    while tickets:
        parts.append(abi.out_arrays(g.push_staged_raw(tickets.pop(0))))
    ms, nb = g.ingest_stats()
    if chunk > 8192:  # copied; smaller pinned batches of small-push queries are read in place (zero-copy)
        assert nb > 0 and ms > 0
    for b in bufs:
        b.close()
    return abi.concat_arrays(parts), edges


@pytest.mark.parametrize("window,param,chunk", [("timeBatch", 1000, 50_000), ("time", 500, 20_000),
                                                ("lengthBatch", 3000, 1000), ("timeBatch", 300, 1000),
                                                ("timeBatch", 50, 777), ("time", 500, 1000)])
def test_staged_ingest_matches_oracle(rt, window, param, chunk):
    ts, cols = synth.keyed_stream(0, 200_000, 0xC2, 5_000, 100)
    spec = abi.QuerySpec(SCHEMA, window, param, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=5_000)
    g = rt.GpuQuery(spec)
    gout, edges = staged_run(rt, g, SCHEMA, ts, cols, chunk, 1)
    o = OracleQuery(spec)
    pushes = [abi.HostBatch(SCHEMA, ts[a:b], [c[a:b] for c in cols], 1) for a, b in zip(edges[:-1], edges[1:])]
    assert_same(gout, run_pushes(o, pushes), label=f"staged {window}")
    g.close()
    o.close()


def test_staged_tickets_are_checked(rt):
    from siddhi_amd.runtime import SiddhiError
    ts, cols = synth.keyed_stream(0, 3_000, 0xC2, 100, 10)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 100, group_by=["k"], aggs=[("count", None)], key_capacity=128)
    g = rt.GpuQuery(spec)
    bs = [abi.HostBatch(SCHEMA, ts[i * 1000:(i + 1) * 1000], [c[i * 1000:(i + 1) * 1000] for c in cols], 1)
          for i in range(3)]
    t0 = g.stage(bs[0])
    t1 = g.stage(bs[1])
    with pytest.raises(SiddhiError, match="two staged"):
        g.stage(bs[2])
    with pytest.raises(SiddhiError, match="order they were staged"):
        g.push_staged(t1)
    g.push_staged(t0)
    g.push_staged(t1)
    with pytest.raises(SiddhiError, match="order they were staged"):
        g.push_staged(t1)
    g.close()


def test_async_small_push_reports_errors_on_the_next_call(rt):
    """A staged small push that closes no window returns before its kernel ran (the batch was copied
    into the library's pinned ring); a dictionary id beyond the key capacity in it is reported by the
    next call that synchronises — loudly, one call late."""
    from siddhi_amd.runtime import SiddhiError
    ts, cols = synth.keyed_stream(0, 3_000, 0xC2, 100, 10)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 100_000, group_by=["k"], aggs=[("count", None)], key_capacity=128)
    g = rt.GpuQuery(spec)
    pb = [rt.PinnedBatch(SCHEMA, 1000), rt.PinnedBatch(SCHEMA, 1000)]
    g.push_staged(g.stage(pb[0].fill(ts[:1000], [c[:1000] for c in cols], 1)))  # opens the window
    bad = cols[0][1000:2000].copy()
    bad[500] = 5_000  # outside [0, key_capacity)
    g.push_staged(g.stage(pb[1].fill(ts[1000:2000], [bad, cols[1][1000:2000], cols[2][1000:2000]], 1)))
    with pytest.raises(SiddhiError, match="dictionary id"):
        g.advance_time(int(ts[-1]) + 1_000_000)
    for b in pb:
        b.close()
    g.close()


def test_async_small_pushes_then_unstaged_pushes_and_advance(rt):
    """Asynchronous small pushes interleaved with ordinary pushes and a TIMER: the same rows as the
    oracle (the queued appends land before the next call's work on the stream)."""
    ts, cols = synth.keyed_stream(0, 60_000, 0xC2, 2_000, 20)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 700, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=2_000)
    g, o = rt.GpuQuery(spec), OracleQuery(spec)
    bufs = [rt.PinnedBatch(SCHEMA, 1000) for _ in range(2)]
    parts, want = [], []
    for i, a in enumerate(range(0, 60_000, 1000)):
        sl = slice(a, a + 1000)
        hb = abi.HostBatch(SCHEMA, ts[sl], [c[sl] for c in cols], 1)
        if i % 7 == 3:
            parts.append(abi.out_arrays(g.push_raw(hb)))
        else:
            parts.append(abi.out_arrays(g.push_staged_raw(g.stage(bufs[i % 2].fill(ts[sl], [c[sl] for c in cols], 1)))))
        want.append(abi.out_arrays(o.push_raw(hb)))
        if i == 30:
            parts.append(abi.out_arrays(g.advance_time_raw(int(ts[a + 999]) + 3)))
            want.append(abi.out_arrays(o.advance_time_raw(int(ts[a + 999]) + 3)))
    assert_same(abi.concat_arrays(parts), abi.concat_arrays(want), label="async small pushes")
    for b in bufs:
        b.close()
    g.close()
    o.close()


def test_async_small_pushes_hashed_keys_grow_the_table(rt):
    """int group keys (a hashed, growable key table): asynchronous small pushes that bring ever new keys.
    A push is queued unverified only while the verified key count plus one key per queued event stays
    within half the table; past that the reports are waited for and the table grows first. Also a
    snapshot and restore right after queued pushes (the reports are drained first)."""
    schema = abi.Schema.parse("k int, v double, ts long")
    n = 120_000
    rng = np.random.default_rng(5)
    ts = (np.arange(n) // 2 + 1_000).astype(np.int64)  # 4,000 events per window
    k = (np.arange(n) * 7 + rng.integers(0, 3, n)).astype(np.int32)  # mostly new keys: dead keys pile up
    v = rng.integers(-100, 100, n).astype(np.float64)
    cols = [k, v, ts.copy()]
    spec = abi.QuerySpec(schema, "timeBatch", 2_000, group_by=["k"], aggs=[("count", None), ("sum", "v")],
                         key_capacity=5_000)
    g, o = rt.GpuQuery(spec), OracleQuery(spec)
    bufs = [rt.PinnedBatch(schema, 1000) for _ in range(2)]
    parts, want = [], []
    for i, a in enumerate(range(0, n, 1000)):
        sl = slice(a, a + 1000)
        parts.append(abi.out_arrays(g.push_staged_raw(g.stage(bufs[i % 2].fill(ts[sl], [c[sl] for c in cols], 1)))))
        want.append(abi.out_arrays(o.push_raw(abi.HostBatch(schema, ts[sl], [c[sl] for c in cols], 1))))
        if i == 40:
            g.restore(g.snapshot())
    assert_same(abi.concat_arrays(parts), abi.concat_arrays(want), label="async hashed keys")
    for b in bufs:
        b.close()
    g.close()
    o.close()


@pytest.mark.parametrize("chunk", [1000, 60_000])
def test_unread_columns_may_be_null(rt, chunk):
    """The shim packs only the columns the query reads (20 B/event for C2: the `ts` attribute column is not
    read by `select k, count(), min(v), max(v), avg(v)`): a NULL pointer for it gives the oracle's output,
    staged (zero-copy small batches and copied ones) and through sh_push; a NULL column the query reads is
    refused before anything runs."""
    from siddhi_amd.runtime import SiddhiError
    ts, cols = synth.keyed_stream(0, 240_000, 0xC2, 5_000, 100)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=5_000)
    g, o = rt.GpuQuery(spec), OracleQuery(spec)
    bufs = [rt.PinnedBatch(SCHEMA, chunk), rt.PinnedBatch(SCHEMA, chunk)]
    parts, want, tickets = [], [], []
    edges = list(range(0, len(ts), chunk)) + [len(ts)]
    for i, (a, b) in enumerate(zip(edges[:-1], edges[1:])):
        want.append(abi.out_arrays(o.push_raw(abi.HostBatch(SCHEMA, ts[a:b], [c[a:b] for c in cols], 1))))
        if i % 5 == 4:
            while tickets:
                parts.append(abi.out_arrays(g.push_staged_raw(tickets.pop(0))))
            hb = abi.HostBatch(SCHEMA, ts[a:b], [c[a:b] for c in cols], 1)
            hb.b.cols[2] = None
            parts.append(abi.out_arrays(g.push_raw(hb)))
            continue
        pb = bufs[i % 2].fill(ts[a:b], [c[a:b] for c in cols], 1)
        pb.b.cols[2] = None
        tickets.append(g.stage(pb))
        if len(tickets) == 2:
            parts.append(abi.out_arrays(g.push_staged_raw(tickets.pop(0))))
    while tickets:
        parts.append(abi.out_arrays(g.push_staged_raw(tickets.pop(0))))
    assert_same(abi.concat_arrays(parts), abi.concat_arrays(want), label=f"null unread column {chunk}")
    hb = abi.HostBatch(SCHEMA, ts[:100] + 10**9, [c[:100] for c in cols], 1)
    hb.b.cols[1] = None  # v is read by min / max / avg
    with pytest.raises(SiddhiError, match="column 1 is NULL"):
        g.push_raw(hb)
    for b in bufs:
        b.close()
    g.close()
    o.close()
