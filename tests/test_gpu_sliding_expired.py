"""GPU parity of `insert expired events` / `insert all events` on the sliding time(T) and
externalTime(ts, T) windows, and of their pass-through (`select *`) form, against the oracle's
restatement of TimeWindowProcessor.process (:132-169: one expiry queue, heads re-stamped with the
clock and inserted before the current event), the Scheduler's TIMER chunks (Scheduler.java:71-104,
171-209: notifyAt(ts + T) at every new maximum, fired before the send whose clock reaches it),
ExternalTimeWindowProcessor.process (:126-161) and QuerySelector.processInBatchGroupBy (:315-374),
including the min/max deque's removeFirstOccurrence quirk and nulls at count 0.
The reference KATs of these modes (playback7, max_sliding_time, externalTime_test1) run in
test_gpu_parity.py."""
import numpy as np
import pytest

from oracle.oracle import OracleQuery
from siddhi_amd import abi, synth
from tests.parity import assert_same, run_pushes, split_batches

pytestmark = pytest.mark.gpu

SCHEMA = abi.Schema.parse("k int, v double, x long, et long, ts long")
AGGS = [("count", None), ("sum", "v"), ("min", "v"), ("max", "x"), ("avg", "x"), ("sum", "x")]


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def both(rt, spec, pushes, label):
    g, o = rt.GpuQuery(spec), OracleQuery(spec)
    got, ref = run_pushes(g, pushes), run_pushes(o, pushes)
    g.close()
    o.close()
    assert_same(got, ref, label=label)
    return ref


def stream(n, keys, seed, step=6, back=0, gap_at=None):
    """ts advance by 0..step-1 ms per event; with back > 0 a tenth of the events lag behind by up to
    `back` ms (the queue head blocks); gap_at: the stream jumps 30 s there (the window drains)."""
    rng = np.random.default_rng(seed)
    ts = np.cumsum(rng.integers(0, step, n)).astype(np.int64) + 10_000
    if back:
        late = rng.random(n) < 0.1
        ts = ts - late * rng.integers(0, back, n)
    if gap_at is not None:
        ts[gap_at:] += 30_000
    k = rng.integers(0, keys, n).astype(np.int32)
    v = rng.integers(-400, 400, n).astype(np.float64) / 8.0  # repeats: the deque quirk happens
    x = rng.integers(-50, 50, n).astype(np.int64)
    et = ts - rng.integers(0, 5, n)
    return ts.astype(np.int64), [k, v, x, et.astype(np.int64), ts.copy()]


@pytest.mark.parametrize("output", ["all", "expired"])
@pytest.mark.parametrize("send_size", [1, 7])
def test_time_group_by_expired_output(rt, output, send_size):
    ts, cols = stream(40_000, 200, 3, gap_at=25_000)
    spec = abi.QuerySpec(SCHEMA, "time", 500, group_by=["k"], aggs=AGGS, filter=(">", "v", -40.0),
                         output=output, key_capacity=256)
    pushes = split_batches(SCHEMA, ts, cols, [1, 2_000, 24_999, 25_000, 31_000], send_size)
    pushes.insert(4, ("advance", int(ts[24_999]) + 250))   # a TIMER call between pushes
    pushes.append(("advance", int(ts[-1]) + 300))
    pushes.append(("advance", int(ts[-1]) + 10_000))       # the window drains: counts reach 0, nulls
    ref = both(rt, spec, pushes, f"time {output} send {send_size}")
    assert ref["expired"].sum() > 0
    assert ref["nulls"].any()


@pytest.mark.parametrize("output", ["all", "expired"])
def test_time_out_of_order_timestamps(rt, output):
    """late events: the head blocks expiry of newer events behind it; sends whose last ts is below
    the clock fire no timer"""
    ts, cols = stream(30_000, 50, 11, step=4, back=900)
    spec = abi.QuerySpec(SCHEMA, "time", 700, group_by=["k"], aggs=[("count", None), ("min", "v"), ("max", "v")],
                         output=output, key_capacity=64)
    pushes = split_batches(SCHEMA, ts, cols, [5_000, 17_777], 5) + [("advance", int(ts.max()) + 2_000)]
    both(rt, spec, pushes, f"time late {output}")


def test_time_no_group_by_and_hashed_long_keys(rt):
    ts, cols = stream(20_000, 30, 17)
    spec = abi.QuerySpec(SCHEMA, "time", 300, aggs=[("sum", "x"), ("count", None), ("max", "v")], output="all")
    both(rt, spec, split_batches(SCHEMA, ts, cols, [999], 3) + [("advance", int(ts[-1]) + 400)], "time no group-by")
    spec = abi.QuerySpec(SCHEMA, "time", 300, group_by=["x"], aggs=[("avg", "v"), ("min", "x")], output="all",
                         key_capacity=128)
    both(rt, spec, split_batches(SCHEMA, ts, cols, [7_000], 1), "time long key")


def test_time_key_churn_rebuilds_table(rt):
    """hashed keys that come and go: the table is rebuilt from the live keys (window not empty or a
    double-sum residue) while expired rows of the dropped keys were already emitted"""
    n = 60_000
    ts, cols = stream(n, 10, 23, step=3)
    cols[2] = (np.arange(n, dtype=np.int64) // 40) * 7 + cols[0]  # keys drift: 15k distinct over the run,
    # ~500 per push, ~40 alive at a time: the 1024-slot table is rebuilt every other push
    spec = abi.QuerySpec(SCHEMA, "time", 200, group_by=["x"], aggs=[("sum", "v"), ("count", None)], output="all",
                         key_capacity=400)
    both(rt, spec, split_batches(SCHEMA, ts, cols, list(range(2_000, n, 2_000)), 1), "time churn all")


@pytest.mark.parametrize("output", ["all", "expired"])
@pytest.mark.parametrize("send_size", [1, 16])
def test_external_time_expired_output(rt, output, send_size):
    """externalTime(et, T): expiry by the attribute (no timers), rows re-stamped with the attribute of
    the event that expired them, flushes at the send's playback clock"""
    ts, cols = stream(40_000, 100, 29, step=5)
    rng = np.random.default_rng(5)
    cols[3] = cols[3] - (rng.random(40_000) < 0.1) * rng.integers(0, 600, 40_000)  # late attribute values
    spec = abi.QuerySpec(SCHEMA, "externalTime", 400, group_by=["k"], ts_attr="et", output=output,
                         aggs=[("count", None), ("sum", "v"), ("min", "x"), ("avg", "v")], key_capacity=128)
    both(rt, spec, split_batches(SCHEMA, ts, cols, [10_000, 10_001, 33_333], send_size), f"externalTime {output}")


@pytest.mark.parametrize("window", ["time", "externalTime"])
@pytest.mark.parametrize("output", ["current", "all", "expired"])
def test_pass_through(rt, window, output):
    ts, cols = stream(15_000, 10, 31, gap_at=9_000)
    kw = {"ts_attr": "et"} if window == "externalTime" else {}
    spec = abi.QuerySpec(SCHEMA, window, 250, filter=("<", "x", 30), output=output, **kw)
    pushes = split_batches(SCHEMA, ts, cols, [1, 4_000, 9_000], 4) + [("advance", int(ts[-1]) + 2_000)]
    ref = both(rt, spec, pushes, f"pass-through {window} {output}")
    assert ref["ts"].size > 0


def test_c3_size_all_events(rt):
    """C3's shape at size: time(10 sec), count/min/max/avg by 10k keys, 1M events per event-time
    second, per-event sends, `insert all events`: 12M events, the window fills past 1k events per
    key and expires ~1 per current event from the 10 s mark on (TIMER chunks carry them)."""
    ks = abi.Schema.parse("k string, v double, ts long")
    spec = abi.QuerySpec(ks, "time", 10_000, group_by=["k"], output="all", key_capacity=10_000,
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")])
    g, o = rt.GpuQuery(spec), OracleQuery(spec)
    step, total, n_exp = 1_000_000, 12_000_000, 0
    for a in range(0, total, step):
        ts, cols = synth.keyed_stream(a, step, 0xC3, 10_000, 1000)
        b = abi.HostBatch(ks, ts, cols, 1)
        go, oo = abi.out_arrays(g.push_raw(b)), abi.out_arrays(o.push_raw(b))
        assert_same(go, oo, label=f"C3 all events {a}..{a + step}")
        n_exp += int(oo["expired"].sum())
    assert n_exp > 1_000_000
    g.close()
    o.close()


# ---- the wave-per-key replay (k_slx_wkey, round 5) against the oracle, and the lane walk it replaced
# (SH_SLX_WAVE=0) on the same streams: count / sum / avg / min / max of one double column

DAGGS = [("count", None), ("sum", "v"), ("min", "v"), ("max", "v"), ("avg", "v")]


def dstream(n, keys, seed, step=6, distinct=True, nan_at=None, gap_at=None):
    ts, cols = stream(n, keys, seed, step=step, gap_at=gap_at)
    rng = np.random.default_rng(seed + 1)
    if distinct:  # no repeated values: the parallel min / max path
        cols[1] = rng.standard_normal(n) * 100.0
    if nan_at is not None:
        cols[1][nan_at] = np.nan
    return ts, cols


@pytest.mark.parametrize("wave", ["1", "0"])
@pytest.mark.parametrize("output", ["all", "expired"])
@pytest.mark.parametrize("distinct", [True, False])
def test_wave_replay(rt, monkeypatch, wave, output, distinct):
    """repeated values (the deque quirk: chunks fall back to the sequential deque) or distinct ones
    (parallel range bests), TIMER calls, a gap that drains the window (counts 0, nulls), a filter"""
    monkeypatch.setenv("SH_SLX_WAVE", wave)
    ts, cols = dstream(40_000, 150, 41, distinct=distinct, gap_at=25_000)
    spec = abi.QuerySpec(SCHEMA, "time", 500, group_by=["k"], aggs=DAGGS, filter=(">", "x", -45), output=output,
                         key_capacity=256)
    pushes = split_batches(SCHEMA, ts, cols, [1, 3_000, 24_999, 25_000, 31_000], 1)
    pushes.insert(4, ("advance", int(ts[24_999]) + 250))
    pushes.append(("advance", int(ts[-1]) + 300))
    pushes.append(("advance", int(ts[-1]) + 10_000))
    ref = both(rt, spec, pushes, f"wave={wave} {output} distinct={distinct}")
    assert ref["expired"].sum() > 0 and ref["nulls"].any()


@pytest.mark.parametrize("wave", ["1", "0"])
@pytest.mark.parametrize("T,keys", [(30, 3), (5_000, 20), (200, 1)])
def test_wave_replay_window_sizes(rt, monkeypatch, wave, T, keys):
    """short windows (a chunk's own adds expire within it), long ones (deques past the LDS ring), one
    key (every operation of the stream in one wave); send sizes 3"""
    monkeypatch.setenv("SH_SLX_WAVE", wave)
    ts, cols = dstream(30_000, keys, 43, step=3)
    spec = abi.QuerySpec(SCHEMA, "time", T, group_by=["k"], aggs=[("max", "v"), ("avg", "v"), ("min", "v")],
                         output="all", key_capacity=64)
    pushes = split_batches(SCHEMA, ts, cols, [7_000, 7_001, 19_000], 3) + [("advance", int(ts[-1]) + T + 1)]
    both(rt, spec, pushes, f"wave={wave} T={T} keys={keys}")


@pytest.mark.parametrize("wave", ["1", "0"])
def test_wave_replay_nan_sorted_values_and_sum_only(rt, monkeypatch, wave):
    """a NaN breaks the deque's order (sequential from there); ascending / descending value runs (the
    deque holds the whole window, spilling past the LDS ring); sum / count only (no deque)"""
    monkeypatch.setenv("SH_SLX_WAVE", wave)
    n = 24_000
    ts, cols = dstream(n, 4, 47, step=2, nan_at=[9_000, 9_001])
    cols[1][12_000:16_000] = np.arange(4_000, dtype=np.float64)          # ascending: max deque length 1,
    cols[1][16_000:20_000] = -np.arange(4_000, dtype=np.float64) * 0.5    # min deque grows
    spec = abi.QuerySpec(SCHEMA, "time", 2_000, group_by=["k"], aggs=DAGGS, output="all", key_capacity=16)
    pushes = split_batches(SCHEMA, ts, cols, [5_000, 11_000, 17_000], 1) + [("advance", int(ts[-1]) + 5_000)]
    both(rt, spec, pushes, f"wave={wave} nan / runs")
    spec = abi.QuerySpec(SCHEMA, "time", 700, group_by=["k"], aggs=[("sum", "v"), ("count", None)],
                         output="expired", key_capacity=16)
    ts, cols = stream(n, 6, 53, step=2)  # eighths: exact cancellations reach 0.0 (canDestroy restarts)
    both(rt, spec, split_batches(SCHEMA, ts, cols, [8_000], 1) + [("advance", int(ts[-1]) + 800)],
         f"wave={wave} sum only")


@pytest.mark.parametrize("wave", ["1", "0"])
def test_wave_replay_external_time(rt, monkeypatch, wave):
    monkeypatch.setenv("SH_SLX_WAVE", wave)
    ts, cols = dstream(30_000, 40, 59, step=5)
    rng = np.random.default_rng(6)
    cols[3] = cols[3] - (rng.random(30_000) < 0.1) * rng.integers(0, 600, 30_000)
    spec = abi.QuerySpec(SCHEMA, "externalTime", 400, group_by=["k"], ts_attr="et", output="all", aggs=DAGGS,
                         key_capacity=64)
    both(rt, spec, split_batches(SCHEMA, ts, cols, [10_000, 10_001], 16), f"wave={wave} externalTime")
