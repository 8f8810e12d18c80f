"""GPU parity: the HIP path (through the C-ABI) against the CPU restatement on identical pushes.
Marked `gpu`: needs an MI355X; the library refuses to run without one (no CPU fallback)."""
import numpy as np
import pytest

from oracle.oracle import OracleQuery
from siddhi_amd import abi, synth
from tests import kat_runner
from tests.parity import assert_same, run_pushes, split_batches

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def both(rt, spec, pushes, rtol=None, label=""):
    g = rt.GpuQuery(spec)
    o = OracleQuery(spec)
    gout = run_pushes(g, pushes)
    oout = run_pushes(o, pushes)
    assert_same(gout, oout, rtol=rtol, label=label)
    g.close()
    o.close()
    return gout


# ---- reference KATs that the GPU path runs: aggregating or pass-through lengthBatch / timeBatch /
# time / externalTime windows with current, expired or all-events output ----
def _gpu_runs(c):
    q = c.get("query", {})
    if c.get("kind") == "aggregation":
        return False
    if q.get("stream_current"):
        if q.get("partition"):  # the lengthBatch lanes: no group-by or grouped by the partition key
            return (q.get("window") == "lengthBatch" and bool(q.get("aggs"))
                    and q.get("group_by", []) in ([], [q["partition"]]))
        return bool(q.get("aggs")) and (q.get("output", "current") == "current" or q.get("window") == "lengthBatch")
    if q.get("window") in ("lengthBatch", "timeBatch"):
        return bool(q.get("aggs")) or not q.get("group_by")
    if q.get("window") in ("time", "externalTime"):
        if q.get("partition"):  # the partition lanes: no group-by or grouped by the partition key
            return bool(q.get("aggs")) and q.get("group_by", []) in ([], [q["partition"]])
        return bool(q.get("aggs")) or not q.get("group_by")
    return False


GPU_KATS = [c for c in kat_runner.load_cases() if _gpu_runs(c)]


@pytest.mark.parametrize("case", GPU_KATS, ids=[c["name"] for c in GPU_KATS])
def test_reference_kat_on_gpu(rt, case):
    schema, spec, dic, flushes = kat_runner.run_query(case, rt.GpuQuery)
    kat_runner.check_query(case, flushes, schema, dic)
    # and identical to the oracle
    _, _, _, oflushes = kat_runner.run_query(case, OracleQuery)
    assert [(f.clock, f.rows) for f in flushes] == [(f.clock, f.rows) for f in oflushes]


# ---- the FilterTestCase1 promotion KATs through the GPU filter program (sh_device.h java_cmp) ----
# The GPU runs aggregating windows only, so each case is wrapped as `from S[cond]#window.lengthBatch(1)
# select count() insert into O`: every passing event completes a batch of one and emits one row, so
# the row count is the number of events the reference's FilterProcessor let through.
FILTER_KATS = [c for c in kat_runner.load_cases() if c.get("kind") != "aggregation" and c["query"].get("window") is None
               and c["query"].get("filter") is not None]


@pytest.mark.parametrize("case", FILTER_KATS, ids=[c["name"] for c in FILTER_KATS])
def test_reference_filter_kat_on_gpu(rt, case):
    wrapped = dict(case, query=dict(case["query"], window="lengthBatch", param=1, aggs=[["count", None]]))
    _, _, _, flushes = kat_runner.run_query(wrapped, rt.GpuQuery)
    rows = [r for f in flushes for r in f.rows]
    assert len(rows) == case["expect"]["in_count"], (len(rows), case["expect"])
    assert all(r[3] == (1,) for r in rows)


# ---- C1: filtered lengthBatch group-by, 1k symbols --------------------------------------------------
C1_SCHEMA = abi.Schema.parse("symbol string, price double, volume long, ts long")


def c1_spec(L=10000):
    return abi.QuerySpec(C1_SCHEMA, "lengthBatch", L, group_by=["symbol"], aggs=[("sum", "volume"), ("avg", "price")],
                         filter=(">", "price", 100), key_capacity=1000)


@pytest.mark.parametrize("send_size,cuts", [(1000, [250_000]), (1, [7, 123_457]), (0, [99_999, 100_000, 100_001])])
def test_c1_lengthbatch_matches_oracle(rt, send_size, cuts):
    ts, cols = synth.c1_stock(0, 300_000)
    pushes = split_batches(C1_SCHEMA, ts, cols, cuts, send_size)
    out = both(rt, c1_spec(), pushes, label="C1")
    assert out["flush_offsets"].size >= 15


@pytest.mark.parametrize("send_size,cuts", [(1000, [4_000_000]), (1, [3_333_331, 6_666_667]), (0, [5_000_000])])
def test_c1_full_size_matches_oracle(rt, send_size, cuts):
    """C1 at its configuration size (BASELINE.json configs[0]: 10M events, 1k symbols) through sh_push in
    the three send modes: send(Event[1000]), per-event sends, one send per push."""
    ts, cols = synth.c1_stock(0, 10_000_000)
    pushes = split_batches(C1_SCHEMA, ts, cols, cuts, send_size)
    out = both(rt, c1_spec(), pushes, label=f"C1-10M-{send_size}")
    assert out["flush_offsets"].size > 400


def test_c1_quantized_prices(rt):
    ts, cols = synth.c1_stock(0, 120_000, quantized=True)
    both(rt, c1_spec(L=777), split_batches(C1_SCHEMA, ts, cols, [50_000], 1000), label="C1q")


# ---- C2: timeBatch(1 sec) count/min/max/avg by 100k keys (partitioned LDS path) ----------------------
C2_SCHEMA = abi.Schema.parse("k int, v double, ts long")


def c2_spec(keys=100_000, start=None):
    return abi.QuerySpec(C2_SCHEMA, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], start_time=start,
                         key_capacity=keys)


@pytest.mark.parametrize("send_size", [1, 1000])
def test_c2_timebatch_matches_oracle(rt, send_size):
    ts, cols = synth.keyed_stream(0, 600_000, 0xC2, 100_000, 100)  # 100 events/ms -> 100k per window
    pushes = split_batches(C2_SCHEMA, ts, cols, [123_456, 400_000], send_size)
    pushes.append(("advance", int(ts[-1]) + 5000))
    out = both(rt, c2_spec(), pushes, label="C2")
    assert out["flush_offsets"].size >= 6


C2S_SCHEMA = abi.Schema.parse("k string, v double, ts long")


@pytest.mark.parametrize("send_size,direct", [(1, False), (1000, False), (1, True)])
def test_c2_dictionary_keys_dense_slots(rt, send_size, direct, monkeypatch):
    """k as a dictionary-encoded string: ids are the key slots (no hashing); same output as the oracle.
    direct: the opt-in path that reads the slots from the key column (SH_DIRECT_POS, no slot column)."""
    if direct:
        monkeypatch.setenv("SH_DIRECT_POS", "1")
    ts, cols = synth.keyed_stream(0, 600_000, 0xC2, 100_000, 100)
    spec = abi.QuerySpec(C2S_SCHEMA, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=100_000)
    pushes = split_batches(C2S_SCHEMA, ts, cols, [123_456, 400_000], send_size)
    pushes.append(("advance", int(ts[-1]) + 5000))
    out = both(rt, spec, pushes, label="C2 dict")
    assert out["flush_offsets"].size >= 6


def test_c3_sliding_dictionary_keys(rt):
    ts, cols = synth.keyed_stream(0, 200_000, 0xC3, 3_000, 50)
    spec = abi.QuerySpec(C2S_SCHEMA, "time", 2_000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=3_000)
    both(rt, spec, split_batches(C2S_SCHEMA, ts, cols, [77_777], 1), label="C3 dict")


def test_dictionary_id_beyond_capacity_fails_loudly(rt):
    from siddhi_amd.runtime import SiddhiError
    ts, cols = synth.keyed_stream(0, 10_000, 0xC2, 5000, 10)
    spec = abi.QuerySpec(C2S_SCHEMA, "timeBatch", 100, group_by=["k"], aggs=[("count", None)], key_capacity=1000)
    g = rt.GpuQuery(spec)
    with pytest.raises(SiddhiError, match="dictionary id"):
        g.push(abi.HostBatch(C2S_SCHEMA, ts, cols, 1))


def test_timebatch_small_keys_start_time_and_gaps(rt):
    # clock jumps (empty windows), start.time alignment, filter that drops whole sends
    rng = np.random.default_rng(7)
    n = 40_000
    ts = np.cumsum(rng.integers(0, 40, n)).astype(np.int64) + 5_000
    ts[20_000:] += 100_000  # a long idle gap
    k = rng.integers(0, 50, n).astype(np.int32)
    v = rng.integers(-1000, 1000, n).astype(np.float64) / 8.0
    schema = abi.Schema.parse("k int, v double, ts long")
    spec = abi.QuerySpec(schema, "timeBatch", 2500, group_by=["k"], start_time=1000,
                         aggs=[("sum", "v"), ("min", "v"), ("max", "v"), ("count", None), ("avg", "v")],
                         filter=(">", "v", -50.0), key_capacity=64)
    pushes = split_batches(schema, ts, [k, v, ts.copy()], [1, 17_000, 20_000, 20_001, 33_333], 10)
    pushes.append(("advance", int(ts[-1]) + 10_000))
    both(rt, spec, pushes, label="gaps")


@pytest.mark.parametrize("send_size", [1, 7])
def test_timebatch_out_of_order_timestamps(rt, send_size):
    """Later pushes (nextEmitTime known) take the single-pass window assignment, which holds only for
    non-decreasing timestamps: jittered and stepped-back timestamps must fall back to the prefix passes
    and still match the oracle (TimeBatchWindowProcessor :262-340 with the send clock of
    InputHandler :85-96). Sorted pushes in between take the single pass."""
    rng = np.random.default_rng(23)
    n = 300_000
    ts = (np.arange(n, dtype=np.int64) // 40) + 10_000          # 40 events / ms, sorted
    ts[100_000:160_000] += rng.integers(-60, 60, 60_000)        # jitter inside one push
    ts[230_000:] -= 900                                         # a step back below the clock
    k = rng.integers(0, 5_000, n).astype(np.int32)
    v = rng.standard_normal(n)
    schema = abi.Schema.parse("k int, v double, ts long")
    spec = abi.QuerySpec(schema, "timeBatch", 500, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=5_000)
    pushes = split_batches(schema, ts, [k, v, ts.copy()], [50_000, 100_000, 160_000, 230_000, 260_000], send_size)
    pushes.append(("advance", int(ts.max()) + 2_000))
    out = both(rt, spec, pushes, label="out-of-order ts")
    assert out["flush_offsets"].size >= 10


def test_lengthbatch_types_and_two_keys(rt):
    rng = np.random.default_rng(11)
    n = 50_000
    schema = abi.Schema.parse("a int, b string, x int, y long, f float, d double")
    cols = [rng.integers(-3, 3, n).astype(np.int32), rng.integers(0, 7, n).astype(np.int32),
            rng.integers(-10**6, 10**6, n).astype(np.int32), rng.integers(-10**12, 10**12, n).astype(np.int64),
            (rng.standard_normal(n) * 100).astype(np.float32), rng.standard_normal(n) * 1e6]
    ts = np.arange(n, dtype=np.int64)
    spec = abi.QuerySpec(schema, "lengthBatch", 333, group_by=["a", "b"],
                         aggs=[("sum", "x"), ("sum", "y"), ("sum", "f"), ("avg", "x"), ("avg", "f"), ("min", "f"),
                               ("max", "y"), ("min", "d")], key_capacity=64)
    both(rt, spec, split_batches(schema, ts, cols, [1000, 1001, 30_000], 7), label="types")


def test_no_group_by_single_key(rt):
    ts, cols = synth.c1_stock(0, 20_000)
    spec = abi.QuerySpec(C1_SCHEMA, "lengthBatch", 1500, aggs=[("sum", "price"), ("count", None), ("max", "volume")])
    both(rt, spec, split_batches(C1_SCHEMA, ts, cols, [5000], 100), label="nogroup")


def test_empty_and_all_filtered_pushes(rt):
    ts, cols = synth.c1_stock(0, 30_000)
    spec = abi.QuerySpec(C1_SCHEMA, "lengthBatch", 1000, group_by=["symbol"], aggs=[("sum", "volume")],
                         filter=(">", "price", 150.0), key_capacity=1000)
    pushes = split_batches(C1_SCHEMA, ts, cols, [10, 10, 2000], 50)
    empty = abi.HostBatch(C1_SCHEMA, ts[:0], [c[:0] for c in cols], 0)
    none_pass = abi.HostBatch(C1_SCHEMA, ts[:100], [cols[0][:100], np.zeros(100), cols[2][:100], cols[3][:100]], 0)
    both(rt, spec, [empty] + pushes[:2] + [none_pass] + pushes[2:] + [empty], label="empty")


def test_key_capacity_overflow_fails_loudly(rt):
    from siddhi_amd.runtime import SiddhiError
    ts, cols = synth.keyed_stream(0, 10_000, 0xC2, 5000, 10)
    spec = abi.QuerySpec(C2_SCHEMA, "timeBatch", 100, group_by=["k"], aggs=[("count", None)], key_capacity=8)
    g = rt.GpuQuery(spec)
    with pytest.raises(SiddhiError):
        g.push(abi.HostBatch(C2_SCHEMA, ts, cols, 1))


# ---- C3: sliding time window (per-key sequential state, SLIDE-mode aggregators) -----------------------
def c3_spec(keys=10_000, T=10_000):
    return abi.QuerySpec(C2_SCHEMA, "time", T, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=keys)


def test_sliding_key_churn_bound(rt):
    """A time() window with hashed keys rebuilds its table from the live keys (every key whose window
    events can no longer be in any later window is dropped, as the reference destroys its state), so a
    stream bringing far more distinct keys over time than key_capacity matches the oracle; more keys
    alive at once than the table holds fails loudly instead of mixing keys."""
    from siddhi_amd.runtime import SiddhiError
    sch = abi.Schema.parse("k long, v double, ts long")  # hashed keys (no dictionary ids)
    n = 6_000
    ts = (np.arange(n, dtype=np.int64) * 3 + 1_000)
    v = (np.arange(n) % 97).astype(np.float64) / 8
    k = (np.arange(n, dtype=np.int64) // 4) * 1_000_003  # a new key every 4 events: 1500 keys over time
    cuts = [500, 1_000, 2_000, 3_000, 4_000, 5_000]
    # cap 64 (a 128-slot table): pushes of 100 events bring 25 new keys each, the table is rebuilt
    # every few pushes (a push's own new keys must fit: the rebuild runs between pushes)
    for cap, cc in ((4_096, cuts), (64, list(range(100, n, 100)))):
        spec = abi.QuerySpec(sch, "time", 50, group_by=["k"], aggs=[("sum", "v"), ("count", None), ("max", "v")],
                             key_capacity=cap)
        both(rt, spec, split_batches(sch, ts, [k, v, ts.copy()], cc, 1), label=f"churn cap {cap}")
    alive = abi.QuerySpec(sch, "time", 1_000_000, group_by=["k"], aggs=[("sum", "v")], key_capacity=64)
    g = rt.GpuQuery(alive)
    with pytest.raises(SiddhiError, match="key table full"):
        for b in split_batches(sch, ts, [k, v, ts.copy()], cuts, 1):
            g.push(b)
    g.close()


@pytest.mark.parametrize("output", ["current", "all"])
def test_sliding_many_live_keys_rebuild_hysteresis(rt, output):
    """More than half of a time() window's hashed key table stays live across many pushes: the rebuild
    keeps every key (none can be dropped), and the hysteresis (next rebuild only after size/8 more
    keys) must not change the output — 40 pushes, ~80 of 128 slots live, a few new keys per push."""
    sch = abi.Schema.parse("k long, v double, ts long")
    n = 12_000
    rng = np.random.default_rng(11)
    ts = (np.arange(n, dtype=np.int64) * 2 + 5_000)
    # 70 long-lived keys plus a slowly moving band of short-lived ones
    hot = rng.integers(0, 70, n)
    band = 1_000 + np.arange(n) // 150
    k = np.where(rng.random(n) < 0.8, hot, band).astype(np.int64) * 7_919
    v = rng.integers(-200, 200, n).astype(np.float64) / 4
    spec = abi.QuerySpec(sch, "time", 400, group_by=["k"], aggs=[("sum", "v"), ("count", None), ("min", "v")],
                         key_capacity=64, output=output)
    both(rt, spec, split_batches(sch, ts, [k, v, ts.copy()], list(range(300, n, 300)), 1),
         label=f"live keys {output}")


@pytest.mark.parametrize("send_size", [1, 250])
def test_c3_sliding_matches_oracle(rt, send_size):
    ts, cols = synth.keyed_stream(0, 200_000, 0xC3, 2000, 20)   # 20 events/ms, 10 s window ~ 100 per key
    pushes = split_batches(C2_SCHEMA, ts, cols, [77_777, 150_000], send_size)
    both(rt, c3_spec(keys=2000, T=1000), pushes, label="C3")


def test_sliding_quantized_deque_quirk(rt):
    # few distinct values -> duplicates -> removeFirstOccurrence hits other equal elements (R9 quirk)
    rng = np.random.default_rng(3)
    n = 60_000
    ts = np.cumsum(rng.integers(0, 3, n)).astype(np.int64)
    k = rng.integers(0, 40, n).astype(np.int32)
    v = rng.integers(0, 6, n).astype(np.float64)
    schema = abi.Schema.parse("k int, v double, ts long")
    spec = abi.QuerySpec(schema, "time", 300, group_by=["k"],
                         aggs=[("min", "v"), ("max", "v"), ("sum", "v"), ("count", None), ("avg", "v")], key_capacity=64)
    both(rt, spec, split_batches(schema, ts, [k, v, ts.copy()], [1, 20_000, 40_001], 1), label="quirk")


def test_sliding_nonmonotone_ts_filter_and_longs(rt):
    rng = np.random.default_rng(5)
    n = 80_000
    ts = (np.arange(n) // 4 + rng.integers(-50, 50, n)).astype(np.int64) + 10_000
    k = rng.integers(0, 300, n).astype(np.int32)
    x = rng.integers(-10**9, 10**9, n).astype(np.int64)
    f = (rng.standard_normal(n) * 10).astype(np.float32)
    schema = abi.Schema.parse("k int, x long, f float, ts long")
    spec = abi.QuerySpec(schema, "time", 500, group_by=["k"], filter=(">", "f", ("float", -5.0)),
                         aggs=[("sum", "x"), ("min", "f"), ("max", "x"), ("avg", "f"), ("sum", "f")], key_capacity=512)
    both(rt, spec, split_batches(schema, ts, [k, x, f, ts.copy()], [33_333], 7), label="nonmono")


def test_sliding_no_group_by(rt):
    ts, cols = synth.keyed_stream(0, 30_000, 0xC3, 100, 5)
    spec = abi.QuerySpec(C2_SCHEMA, "time", 700, aggs=[("sum", "v"), ("max", "v"), ("count", None)])
    both(rt, spec, split_batches(C2_SCHEMA, ts, cols, [10_000], 3), label="slide-nogroup")


def test_sliding_monotone_values_long_deques(rt):
    """Per-key rising then falling values: the min (then max) deque grows to the whole window, past the
    LDS deque capacity of k_sl_own, so those keys run on the spilled global deques; NaN/-0.0 mixed in
    break the deque's order (Java comparisons with NaN are false) and Double.equals."""
    rng = np.random.default_rng(17)
    n = 50_000
    ts = (np.arange(n, dtype=np.int64) // 5) + 1_000
    k = rng.integers(0, 20, n).astype(np.int32)
    v = np.where(np.arange(n) < n // 2, np.arange(n, dtype=np.float64), (n - np.arange(n)).astype(np.float64))
    v[rng.integers(0, n, 40)] = np.nan
    v[rng.integers(0, n, 40)] = -0.0
    v[rng.integers(0, n, 40)] = 0.0
    schema = abi.Schema.parse("k int, v double, ts long")
    spec = abi.QuerySpec(schema, "time", 400, group_by=["k"],
                         aggs=[("min", "v"), ("max", "v"), ("count", None), ("sum", "v")], key_capacity=32)
    both(rt, spec, split_batches(schema, ts, [k, v, ts.copy()], [20_000, 20_001], 1), label="monotone")


def test_lengthbatch_batch_completing_on_the_push_end_flushes_in_that_push(rt):
    """LengthBatchWindowProcessor flushes a batch in the send of its L-th event (:206-243): a push
    whose last event completes a batch must emit it in that push's output, not the next one's."""
    ts, cols = synth.c1_stock(0, 40_000)
    spec = abi.QuerySpec(C1_SCHEMA, "lengthBatch", 1000, group_by=["symbol"], aggs=[("sum", "volume"), ("count", None)],
                         key_capacity=1000)
    g, o = rt.GpuQuery(spec), OracleQuery(spec)
    for p in split_batches(C1_SCHEMA, ts, cols, [3_000, 3_500, 10_000, 10_001, 25_000], 500):
        assert_same(abi.out_arrays(g.push_raw(p)), abi.out_arrays(o.push_raw(p)), label="per push")
    g.close()
    o.close()


@pytest.mark.parametrize("key_type,keys,filt", [("string", 100_000, None), ("int", 30_000, None),
                                                ("string", 5_000, (">", "v", 50.0))])
def test_c2_counting_split(rt, key_type, keys, filt):
    """timeBatch at C2 shape (per-event sends, pushes of >= 2^18 events): the early key-partition split
    behind the window assignment gives the oracle's rows; the third push carries a decreasing timestamp
    (the single-pass sortedness check hands over to the prefix passes)."""
    schema = abi.Schema.parse(f"k {key_type}, v double, ts long")
    ts, cols = synth.keyed_stream(0, 1_400_000, 0xC2, keys, 1000)
    ts = ts.copy()
    ts[1_000_500] -= 3  # late
    cols[2] = ts.copy()
    spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"], filter=filt,
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=keys)
    both(rt, spec, split_batches(schema, ts, cols, [300_000, 700_000, 1_100_000], 1), label=f"split {key_type} {keys}")


def test_c2_hot_key_split(rt):
    """A hot key (a quarter of the events) makes one key partition far larger than the others; output =
    oracle."""
    schema = abi.Schema.parse("k string, v double, ts long")
    ts, cols = synth.keyed_stream(0, 1_200_000, 0xC2, 50_000, 1000)
    k = cols[0].copy()
    k[::4] = 7
    cols[0] = k
    spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("sum", "v"), ("max", "v")], key_capacity=50_000)
    both(rt, spec, split_batches(schema, ts, cols, [300_000, 700_000], 1), label="hot key split")
