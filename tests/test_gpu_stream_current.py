"""GPU parity of `#window.lengthBatch(L, true)` / `#window.timeBatch(T, true)` (stream.current.event, current
events output): every arriving event is emitted at once with its key's running aggregates since the last
batch reset (LengthBatchWindowProcessor.processStreamCurrentEvents :245-274, TimeBatchWindowProcessor RESET
mode :262-340, QuerySelector :315-374 grouping each chunk). The reference KAT lengthBatch11 runs in
test_gpu_parity.py."""
import numpy as np
import pytest

from siddhi_amd import abi
from tests.parity import split_batches
from tests.test_gpu_parity import both

pytestmark = pytest.mark.gpu

SCHEMA = abi.Schema.parse("k int, v double, x long, ts long")
AGGS = [("count", None), ("sum", "v"), ("min", "v"), ("max", "x"), ("avg", "x"), ("sum", "x")]


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def stream(n, keys, seed, step=40, gap_at=None):
    rng = np.random.default_rng(seed)
    ts = np.cumsum(rng.integers(0, step, n)).astype(np.int64) + 5_000
    if gap_at is not None:
        ts[gap_at:] += 20_000
    k = rng.integers(0, keys, n).astype(np.int32)
    v = rng.integers(-4000, 4000, n).astype(np.float64) / 16.0
    x = rng.integers(-10**6, 10**6, n).astype(np.int64)
    return ts, [k, v, x, ts.copy()]


@pytest.mark.parametrize("L,cuts,send_size", [(100, [1, 777, 5_000], 3), (7, [3, 4_000], 1), (1, [10], 5),
                                              (5_000, [2_500, 12_000], 0)])
@pytest.mark.parametrize("group_by", [True, False])
def test_lengthbatch_stream_current(rt, L, cuts, send_size, group_by):
    ts, cols = stream(15_000, 60, 3)
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", L, group_by=["k"] if group_by else (), aggs=AGGS,
                         filter=(">", "v", -180.0), stream_current=True, key_capacity=64)
    out = both(rt, spec, split_batches(SCHEMA, ts, cols, cuts, send_size), label=f"lengthBatch({L}, true)")
    assert out["ts"].size > 0


@pytest.mark.parametrize("send_size", [1, 13, 0])
@pytest.mark.parametrize("group_by", [True, False])
def test_timebatch_stream_current(rt, send_size, group_by):
    ts, cols = stream(30_000, 300, 7, gap_at=17_000)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 700, group_by=["k"] if group_by else (), aggs=AGGS,
                         filter=(">", "v", -150.0), stream_current=True, key_capacity=512)
    pushes = split_batches(SCHEMA, ts, cols, [1, 2_000, 16_999, 17_000, 25_000], send_size)
    pushes.insert(3, ("advance", int(ts[16_999]) + 1_500))
    pushes.append(("advance", int(ts[-1]) + 5_000))
    out = both(rt, spec, pushes, label=f"timeBatch stream current send {send_size}")
    assert out["flush_offsets"].size > (10 if send_size else 4)


def test_timebatch_stream_current_start_time(rt):
    ts, cols = stream(8_000, 20, 9)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 333, group_by=["k"], aggs=[("sum", "v"), ("count", None)],
                         start_time=100, stream_current=True, key_capacity=32)
    both(rt, spec, split_batches(SCHEMA, ts, cols, [4_000], 2), label="timeBatch start")


@pytest.mark.parametrize("output", ["all", "expired"])
@pytest.mark.parametrize("L,cuts,send_size", [(50, [1, 777, 5_000], 3), (4, [3, 4_000, 4_001], 1), (1, [10], 2),
                                              (2_000, [2_000, 6_000], 0)])
@pytest.mark.parametrize("group_by", [True, False])
def test_lengthbatch_stream_current_expired(rt, output, L, cuts, send_size, group_by):
    """Batch w + 1's first event carries batch w's keys as EXPIRED rows (empty state) in its chunk."""
    ts, cols = stream(12_000, 40, 13)
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", L, group_by=["k"] if group_by else (), aggs=AGGS,
                         filter=(">", "v", -180.0), stream_current=True, output=output, key_capacity=64)
    out = both(rt, spec, split_batches(SCHEMA, ts, cols, cuts, send_size), label=f"lengthBatch({L}, true) {output}")
    if output == "expired" or group_by:  # (without group-by, `all` shows the new event's row in the key's place)
        assert out["expired"].sum() > 0


@pytest.mark.parametrize("output", ["all", "expired"])
@pytest.mark.parametrize("send_size", [1, 13, 0])
@pytest.mark.parametrize("group_by", [True, False])
def test_timebatch_stream_current_expired(rt, output, send_size, group_by):
    """A window closes in the scheduler's TIMER chunk before the crossing send's own chunk: a flush of
    its keys' EXPIRED rows (also when no event of the push passes, and at advance_time)."""
    ts, cols = stream(30_000, 300, 19, gap_at=17_000)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 700, group_by=["k"] if group_by else (), aggs=AGGS,
                         filter=(">", "v", -150.0), stream_current=True, output=output, key_capacity=512)
    pushes = split_batches(SCHEMA, ts, cols, [1, 2_000, 16_999, 17_000, 25_000], send_size)
    none_pass = abi.HostBatch(SCHEMA, ts[25_000:25_100] + 900, [cols[0][:100], np.full(100, -500.0), cols[2][:100],
                                                                 ts[25_000:25_100] + 900], send_size)
    pushes.insert(3, ("advance", int(ts[16_999]) + 1_500))
    pushes.insert(6, none_pass)
    pushes.append(("advance", int(ts[-1]) + 5_000))
    out = both(rt, spec, pushes, label=f"timeBatch stream current {output} send {send_size}")
    assert out["expired"].sum() > 0


@pytest.mark.parametrize("window,param", [("timeBatch", 700), ("lengthBatch", 50)])
def test_compact_flushes(rt, window, param):
    """sh_query_set_compact_flushes: per-event sends give one row per flush at its row's timestamp, so the
    flush arrays come back NULL (n_flushes = n_rows) and are rebuilt from the rows; sends of several events
    keep the full arrays. Host and device outputs equal the oracle's either way."""
    import torch
    from oracle.oracle import OracleQuery
    from tests.parity import assert_same
    ts, cols = stream(20_000, 300, 17)
    spec = abi.QuerySpec(SCHEMA, window, param, group_by=["k"], aggs=AGGS, filter=(">", "v", -150.0),
                         stream_current=True, key_capacity=512)
    g, o = rt.GpuQuery(spec), OracleQuery(spec)
    g.set_compact_flushes()
    compact = []
    for a, b, send in ((0, 6_000, 1), (6_000, 9_000, 13), (9_000, 14_000, 1)):
        hb = abi.HostBatch(SCHEMA, ts[a:b], [c[a:b] for c in cols], send)
        raw = g.push_raw(hb)
        compact.append(not raw.contents.flush_offsets)
        assert_same(abi.out_arrays(raw), abi.out_arrays(o.push_raw(hb)), label=f"compact host {a}")
    assert compact == [True, False, True]
    dev = torch.device("cuda", 0)
    t = torch.from_numpy(ts[14_000:]).to(dev)
    dc = [torch.from_numpy(np.ascontiguousarray(c[14_000:])).to(dev) for c in cols]
    torch.cuda.synchronize()
    raw = g.push_device(len(t), t.data_ptr(), [c.data_ptr() for c in dc], 1)
    assert not raw.contents.flush_offsets and raw.contents.n_flushes == raw.contents.n_rows > 0
    got = rt.device_out_arrays(raw)
    ref = abi.out_arrays(o.push_raw(abi.HostBatch(SCHEMA, ts[14_000:], [c[14_000:] for c in cols], 1)))
    assert_same(got, ref, label="compact device")
    g.close()
    o.close()


@pytest.mark.parametrize("window", ["time", "externalTime"])
def test_sliding_device_output_flush_layout(rt, window):
    """sh_push_device of a sliding window: the flush layout is host memory (the ABI contract) — read here
    as host arrays — or, with compact flushes and one row per event at its clock, NULL."""
    import torch
    from oracle.oracle import OracleQuery
    from tests.parity import assert_same
    ts, cols = stream(12_000, 200, 23)
    spec = abi.QuerySpec(SCHEMA, window, 2_000, group_by=["k"], aggs=AGGS, key_capacity=256,
                         ts_attr="ts" if window == "externalTime" else None)
    dev = torch.device("cuda", 0)
    for compact, send, devf in ((False, 1, False), (True, 1, False), (True, 7, False), (False, 3, True),
                                (True, 5, True)):
        g, o = rt.GpuQuery(spec), OracleQuery(spec)
        if compact:
            g.set_compact_flushes()
        if devf:
            g.set_device_flushes()
        t = torch.from_numpy(ts).to(dev)
        dc = [torch.from_numpy(np.ascontiguousarray(c)).to(dev) for c in cols]
        torch.cuda.synchronize()
        raw = g.push_device(len(ts), t.data_ptr(), [c.data_ptr() for c in dc], send)
        assert bool(raw.contents.flush_offsets) == (not compact or send > 1)
        got = rt.device_out_arrays(raw, device_flushes=devf)
        ref = abi.out_arrays(o.push_raw(abi.HostBatch(SCHEMA, ts, cols, send)))
        assert_same(got, ref, label=f"{window} device compact={compact} send={send} device flushes={devf}")
        g.close()
        o.close()



@pytest.mark.parametrize("output", ["current", "all"])
def test_batch_window_device_flush_layout(rt, output):
    """sh_query_set_device_flushes on a timeBatch query: the flush layout of sh_push_device comes back in
    device memory (current output: the windows' flushes; all events: the expired rows' path)."""
    import torch
    from oracle.oracle import OracleQuery
    from tests.parity import assert_same
    ts, cols = stream(15_000, 100, 29)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 700, group_by=["k"], aggs=AGGS, output=output, key_capacity=128)
    g, o = rt.GpuQuery(spec), OracleQuery(spec)
    g.set_device_flushes()
    dev = torch.device("cuda", 0)
    t = torch.from_numpy(ts).to(dev)
    dc = [torch.from_numpy(np.ascontiguousarray(c)).to(dev) for c in cols]
    torch.cuda.synchronize()
    got = rt.device_out_arrays(g.push_device(len(ts), t.data_ptr(), [c.data_ptr() for c in dc], 2), device_flushes=True)
    ref = abi.out_arrays(o.push_raw(abi.HostBatch(SCHEMA, ts, cols, 2)))
    assert ref["flush_clock"].size > 5
    assert_same(got, ref, label=f"timeBatch device flushes {output}")
    g.close()
    o.close()
