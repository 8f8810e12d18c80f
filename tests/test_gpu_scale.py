"""GPU parity at the BASELINE.json configurations' own sizes (VERDICT r01 `configs_untested`):

* C3 — sliding `time(10 sec)` count/min/max/avg by 10k keys at 1M events per event-time second:
  12M events, so the window fills to ~10M resident events (~1k per key) and the last 2M events
  each expire one; per-event sends.
* C4 — `define aggregation ... every sec...day` with 1M keys at 1M events per event-time second, run
  by 8 key-sharded owners (LocalShards, the sh_shard_* protocol), and one owner's share (125k keys,
  1.25M events per second) on a single GPU.
* C5 — `partition with (k of S)` timeBatch(1 sec) over 10M Zipf(1.1) keys, single GPU and 8 owners.

Every comparison is bit-exact against the oracle (tests/parity.py) on the same seeded streams."""
import numpy as np
import pytest

from oracle.oracle import OracleAggregation, OracleQuery
from siddhi_amd import abi, synth
from tests.parity import assert_same
from tests.test_gpu_shard import run_oracle, run_sharded
from tests.test_gpu_shard_agg import assert_tables, run_both

pytestmark = pytest.mark.gpu

KSCHEMA = abi.Schema.parse("k string, v double, ts long")
AGGS4 = [("count", None), ("min", "v"), ("max", "v"), ("avg", "v")]


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def test_c3_time_10s_10k_keys_1k_resident_per_key(rt):
    """C3 at size: every key's window holds ~1000 events when expiry starts (TimeWindowProcessor
    :132-169 with the SLIDE-mode deque of MinAttributeAggregatorExecutor :86-236)."""
    spec = abi.QuerySpec(KSCHEMA, "time", 10_000, group_by=["k"], aggs=AGGS4, key_capacity=10_000)
    g, o = rt.GpuQuery(spec), OracleQuery(spec)
    step, total = 2_000_000, 12_000_000
    rows = 0
    for a in range(0, total, step):
        ts, cols = synth.keyed_stream(a, step, 0xC3, 10_000, 1000)
        b = abi.HostBatch(KSCHEMA, ts, cols, 1)
        go, oo = abi.out_arrays(g.push_raw(b)), abi.out_arrays(o.push_raw(b))
        assert_same(go, oo, label=f"C3 events {a}..{a + step}")
        rows += len(oo["ts"])
    assert rows == total  # one row per per-event send
    g.close()
    o.close()


def test_c4_one_owner_share_125k_keys_sec_to_day(rt):
    """One GPU's share of C4 on 8 GPUs: 125k keys at 1.25M events per event-time second."""
    spec = abi.AggregationSpec(KSCHEMA, [("sum", "v"), ("avg", "v"), ("count", None), ("min", "v"), ("max", "v")],
                               group_by=["k"], ts="ts", durations=("sec", "day"), key_capacity=125_000)
    g, o = rt.GpuAggregation(spec), OracleAggregation(spec)
    for a in range(0, 3_000_000, 1_000_000):
        ts, cols = synth.keyed_stream(a, 1_000_000, 0xC4, 125_000, 1250)
        b = abi.HostBatch(KSCHEMA, ts, cols, 1)
        g.push(b)
        o.push(b)
    end = int(ts[-1]) + 2 * 86_400_000
    g.advance_time(end)
    o.advance_time(end)
    from siddhi_amd.shard import canonical_table
    res = {d: (canonical_table(abi.out_arrays(g.table_raw(d))), canonical_table(abi.out_arrays(o.table_raw(d))))
           for d in range(abi.DUR_SECONDS, abi.DUR_DAYS + 1)}
    assert assert_tables(res, "C4 125k") > 125_000
    g.close()
    o.close()


def test_c4_1m_keys_eight_owners_sec_to_day():
    """C4 at size: 1M keys, 1M events per event-time second, key-sharded over 8 owners."""
    spec = abi.AggregationSpec(KSCHEMA, [("sum", "v"), ("avg", "v"), ("count", None), ("min", "v"), ("max", "v")],
                               group_by=["k"], ts="ts", durations=("sec", "day"), key_capacity=1_000_000)
    pushes = []
    for a in range(0, 2_000_000, 1_000_000):
        pushes.append(synth.keyed_stream(a, 1_000_000, 0xC4, 1_000_000, 1000))
    fr = [[(g + 1) / 8 for g in range(7)], [0.01 * (g + 1) for g in range(7)]]
    res = run_both(spec, 8, pushes, 1, fr, [int(pushes[-1][0][-1]) + 2 * 86_400_000])
    assert assert_tables(res, "C4 1M x8") > 1_000_000


def c5_stream(n):
    ts = synth.T0 + np.arange(n, dtype=np.int64) // 1000
    k = synth.zipf_keys(0, n, 0xC5, 10_000_000)
    v = synth.uniform_price(synth.draws(0xC5 ^ 1, 0, n, 1)[:, 0])
    return ts, [k, v, ts.copy()]


C5_SPEC = dict(group_by=["k"], aggs=[("sum", "v"), ("count", None)], partition="k", key_capacity=10_000_000)


def test_c5_partitioned_zipf_10m_keys(rt):
    """C5 at size: R12 leaves the partition of the first passing event as the only one that ever
    flushes (PartitionStreamReceiver :176-272 + the shared nextEmitTime of TimeBatchWindowProcessor)."""
    spec = abi.QuerySpec(KSCHEMA, "timeBatch", 1000, **C5_SPEC)
    ts, cols = c5_stream(3_000_000)
    assert len(np.unique(cols[0])) > 300_000
    g, o = rt.GpuQuery(spec), OracleQuery(spec)
    for a in range(0, len(ts), 1_000_000):
        b = abi.HostBatch(KSCHEMA, ts[a:a + 1_000_000], [c[a:a + 1_000_000] for c in cols], 1)
        assert_same(abi.out_arrays(g.push_raw(b)), abi.out_arrays(o.push_raw(b)), label=f"C5 {a}")
    end = int(ts[-1]) + 3000
    assert_same(abi.out_arrays(g.advance_time_raw(end)), abi.out_arrays(o.advance_time_raw(end)), label="C5 end")
    g.close()
    o.close()


def test_c5_partitioned_zipf_10m_keys_eight_owners():
    spec = abi.QuerySpec(KSCHEMA, "timeBatch", 1000, **C5_SPEC)
    ts, cols = c5_stream(2_000_000)
    pushes = [(ts[:1_000_000], [c[:1_000_000] for c in cols]), (ts[1_000_000:], [c[1_000_000:] for c in cols])]
    adv = int(ts[-1]) + 3000
    got = run_sharded(spec, 8, pushes, 1, [[(g + 1) / 8 for g in range(7)]], advance=adv)
    ref = run_oracle(spec, pushes, 1, advance=adv)
    assert ref["flush_offsets"].size >= 2
    assert_same(got, ref, label="C5 x8")
