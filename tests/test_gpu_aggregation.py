"""GPU parity of `define aggregation ... every sec...year` (incremental roll-ups) against the CPU
restatement: every duration's table, row for row (insertion order, bit-exact base values)."""
import numpy as np
import pytest

from oracle.oracle import OracleAggregation
from siddhi_amd import abi, synth
from tests import kat_runner
from tests.parity import split_batches

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def tables(a, spec):
    lo, hi = abi.DUR_NAMES[spec.durations[0]], abi.DUR_NAMES[spec.durations[1]]
    return {d: abi.out_arrays(a.table_raw(d)) for d in range(lo, hi + 1)}


def assert_tables_equal(gt, ot, label):
    assert gt.keys() == ot.keys()
    for d in gt:
        g, o = gt[d], ot[d]
        assert np.array_equal(g["keys"], o["keys"]), f"{label} dur {d}: rows differ ({g['keys'].shape} vs {o['keys'].shape})"
        assert np.array_equal(g["ts"], o["ts"]), f"{label} dur {d}: timestamps differ"
        assert np.array_equal(g["val_types"], o["val_types"]), f"{label} dur {d}: value types differ"
        for b in range(len(o["val_types"])):
            bad = np.nonzero(g["vals"][b] != o["vals"][b])[0]
            assert bad.size == 0, f"{label} dur {d} base {b}: differs at rows {bad[:8]}"


def drive(a, pushes):
    for p in pushes:
        if isinstance(p, tuple):
            a.advance_time(p[1])
        else:
            a.push(p)


def both(rt, spec, pushes, label, checkpoints=()):
    """Run GPU and oracle; compare the tables after every push index in `checkpoints` and at the end."""
    g = rt.GpuAggregation(spec)
    o = OracleAggregation(spec)
    n_rows = 0
    for i, p in enumerate(pushes):
        drive(g, [p])
        drive(o, [p])
        if i in checkpoints or i == len(pushes) - 1:
            gt, ot = tables(g, spec), tables(o, spec)
            assert_tables_equal(gt, ot, f"{label}@{i}")
            n_rows += sum(len(t["ts"]) for t in ot.values())
    g.close()
    o.close()
    return n_rows


# (month / year roots included: the root runs as a timeBatch of calendar months / years)
AGG_KATS = [c for c in kat_runner.load_cases() if c.get("kind") == "aggregation"]


@pytest.mark.parametrize("case", AGG_KATS, ids=[c["name"] for c in AGG_KATS])
def test_reference_aggregation_kat_on_gpu(rt, case):
    schema, spec, dic, a = kat_runner.run_aggregation(case, rt.GpuAggregation)
    kat_runner.check_aggregation_table(case, spec, dic, kat_runner.aggregation_rows(case, a))
    if "find" in case["expect"]:
        # the retrieval identical to the oracle's, and to itself after the tables were drained
        _, _, _, o = kat_runner.run_aggregation(case, OracleAggregation)
        f = case["expect"]["find"]
        args = (abi.DUR_NAMES[f["per"]], f["start"], f["end"])
        assert a.find(*args) == o.find(*args)
        tables(a, spec)
        assert a.find(*args) == o.find(*args)
    # every duration identical to the oracle (tables drain on read, so run both afresh)
    _, _, _, a = kat_runner.run_aggregation(case, rt.GpuAggregation)
    _, _, _, o = kat_runner.run_aggregation(case, OracleAggregation)
    assert_tables_equal(tables(a, spec), tables(o, spec), case["name"])


C4_SCHEMA = abi.Schema.parse("k int, v double, ts long")


def c4_spec(durations=("sec", "day"), ts="ts", keys=10_000, aggs=None):
    aggs = aggs or [("sum", "v"), ("avg", "v"), ("count", None), ("min", "v"), ("max", "v")]
    return abi.AggregationSpec(C4_SCHEMA, aggs, group_by=["k"], ts=ts, durations=durations, key_capacity=keys)


@pytest.mark.parametrize("send_size", [1, 500])
def test_c4_event_time_rollups(rt, send_size):
    # 200k events, 2k keys, 5 events/ms -> 40 s of event time across minute boundaries
    ts, cols = synth.keyed_stream(1_700_000_000_000 - 15_000, 200_000, 0xC4, 2_000, 5)
    pushes = split_batches(C4_SCHEMA, ts, cols, [33_333, 100_000, 150_001], send_size)
    pushes.append(("advance", int(ts[-1]) + 3_600_000 * 30))  # close sec ... day
    n = both(rt, c4_spec(keys=2_000), pushes, "C4", checkpoints=(1, 2))
    assert n > 0


STR_SCHEMA = abi.Schema.parse("k string, v double, ts long")


@pytest.mark.parametrize("send_size", [1, 500])
def test_c4_string_keys_band_rollups(rt, send_size):
    """Dictionary keys under `aggregate by`: the root keys (bucket, id) by arithmetic in a band of
    consecutive buckets, re-based as the stream moves on (sh_aggregation.cpp band_reserve)."""
    ts, cols = synth.keyed_stream(1_700_000_000_000 - 15_000, 200_000, 0xC4, 2_000, 5)
    pushes = split_batches(STR_SCHEMA, ts, cols, [33_333, 100_000, 150_001], send_size)
    pushes.append(("advance", int(ts[-1]) + 3_600_000 * 30))
    spec = abi.AggregationSpec(STR_SCHEMA, [("sum", "v"), ("avg", "v"), ("count", None), ("min", "v"), ("max", "v")],
                               group_by=["k"], ts="ts", durations=("sec", "day"), key_capacity=2_000)
    assert both(rt, spec, pushes, "C4 band", checkpoints=(0, 1, 2)) > 0


def test_band_keys_fall_back_and_return(rt):
    """A push whose event times spread over 30 s of sec buckets leaves the band for the open-addressing
    table; once the queued events' buckets fit again the root returns to band keys. Tables equal the
    oracle's after every push."""
    rng = np.random.default_rng(21)
    n = 90_000
    clock = 1_700_000_000_000 + np.arange(n, dtype=np.int64) // 10  # 10 events per ms: pushes span 1-2 s
    lag = np.zeros(n, np.int64)
    lag[30_000:50_000] = rng.integers(0, 30_000, 20_000)
    ext = clock - lag
    k = rng.integers(0, 3_000, n).astype(np.int32)
    v = np.round(rng.normal(50, 20, n), 2)
    spec = abi.AggregationSpec(STR_SCHEMA, [("sum", "v"), ("count", None), ("min", "v"), ("max", "v")],
                               group_by=["k"], ts="ts", durations=("sec", "hour"), key_capacity=3_000)
    cuts = [0, 10_000, 30_000, 50_000, 70_000, n]
    pushes = [abi.HostBatch(STR_SCHEMA, clock[a:b], [k[a:b], v[a:b], ext[a:b]], 1) for a, b in zip(cuts, cuts[1:])]
    pushes.append(("advance", int(clock[-1]) + 2 * 3_600_000))
    both(rt, spec, pushes, "band fallback", checkpoints=(0, 1, 2, 3, 4))


def test_processing_time_rollups_without_aggregate_by(rt):
    ts, cols = synth.keyed_stream(1_600_000_000_000, 100_000, 7, 300, 2)
    pushes = split_batches(C4_SCHEMA, ts, cols, [10_000, 60_000], 100)
    pushes.append(("advance", int(ts[-1]) + 90_000_000))
    both(rt, c4_spec(ts=None, durations=("sec", "hour"), keys=300), pushes, "proc-time")


def test_late_events_and_long_gaps_to_month_and_year(rt):
    # event time lags the clock by up to a minute (late rows land in older buckets), then idle gaps
    rng = np.random.default_rng(11)
    n = 60_000
    clock = 1_706_745_000_000 + np.cumsum(rng.integers(0, 20, n)).astype(np.int64)  # late Jan 2024
    ext = clock - rng.integers(0, 60_000, n).astype(np.int64)
    k = rng.integers(0, 50, n).astype(np.int32)
    v = np.round(rng.normal(100, 30, n), 2)
    schema = abi.Schema.parse("k int, v double, ts long")
    spec = abi.AggregationSpec(schema, [("sum", "v"), ("count", None), ("max", "v")], group_by=["k"], ts="ts",
                               durations=("min", "year"), key_capacity=64)
    b1 = abi.HostBatch(schema, clock[: n // 2], [k[: n // 2], v[: n // 2], ext[: n // 2]], 250)
    b2 = abi.HostBatch(schema, clock[n // 2:], [k[n // 2:], v[n // 2:], ext[n // 2:]], 1)
    pushes = [b1, ("advance", int(clock[n // 2 - 1]) + 40 * 86_400_000), b2,
              ("advance", int(clock[-1]) + 400 * 86_400_000)]
    both(rt, spec, pushes, "late+gaps", checkpoints=(0, 1, 2))


def test_no_group_by_and_filter(rt):
    ts, cols = synth.keyed_stream(1_650_000_000_000, 50_000, 3, 100, 3)
    spec = abi.AggregationSpec(C4_SCHEMA, [("sum", "v"), ("min", "k"), ("count", None)], ts="ts",
                               durations=("sec", "min"), filter=(">", "v", 0.5))
    pushes = split_batches(C4_SCHEMA, ts, cols, [25_000], 7) + [("advance", int(ts[-1]) + 120_000)]
    both(rt, spec, pushes, "nogroup")


def test_long_sums_and_int_min_max(rt):
    schema = abi.Schema.parse("k int, q long, p int, ts long")
    rng = np.random.default_rng(5)
    n = 80_000
    ts = 1_690_000_000_000 + np.arange(n, dtype=np.int64) * 3
    cols = [rng.integers(0, 700, n).astype(np.int32), rng.integers(-10**12, 10**12, n).astype(np.int64),
            rng.integers(-1000, 1000, n).astype(np.int32), ts]
    spec = abi.AggregationSpec(schema, [("sum", "q"), ("avg", "p"), ("min", "p"), ("max", "q")], group_by=["k"],
                               ts="ts", durations=("sec", "hour"), key_capacity=700)
    pushes = split_batches(schema, ts, cols, [40_000], 1000) + [("advance", int(ts[-1]) + 7_200_000)]
    both(rt, spec, pushes, "longs")


# ---- retrieval `from A within start, end per "<per>"` (sh_aggregation_find) against the oracle ------
def _finds(a, spans):
    return [a.find(per, lo, hi) for per, lo, hi in spans]


@pytest.mark.parametrize("proc_time", [False, True])
def test_retrieval_mid_stream_matches_oracle(rt, proc_time):
    """Retrievals between pushes: the `per` table plus the in-memory stores of every executor below it
    (root window pending events, roll-up levels mid-bucket) with late events (IncrementalDataAggregator /
    OutOfOrderEventsDataAggregator) — GPU = oracle at every per duration and several ranges."""
    rng = np.random.default_rng(31)
    n = 40_000
    clock = 1_706_745_000_000 + np.cumsum(rng.integers(0, 40, n)).astype(np.int64)
    ext = clock - rng.integers(0, 90_000, n).astype(np.int64)
    k = rng.integers(0, 40, n).astype(np.int32)
    v = np.round(rng.normal(100, 30, n), 3)
    schema = abi.Schema.parse("k int, v double, ts long")
    spec = abi.AggregationSpec(schema, [("sum", "v"), ("count", None), ("min", "v"), ("max", "v")], group_by=["k"],
                               ts=None if proc_time else "ts", durations=("sec", "day"), key_capacity=64)
    g = rt.GpuAggregation(spec)
    o = OracleAggregation(spec)
    lo, hi = int(ext.min()) - 86_400_000, int(clock.max()) + 86_400_000
    mid = int(clock[n // 2])
    spans = [(abi.DUR_NAMES[d], lo, hi) for d in ("sec", "min", "hour", "day")] + \
            [(abi.DUR_NAMES["min"], mid - 600_000, mid), (abi.DUR_NAMES["sec"], mid, hi)]
    cuts = [0, 7_000, 7_001, 19_000, 33_333, n]
    for a_, b_ in zip(cuts[:-1], cuts[1:]):
        for q in (g, o):
            q.push(abi.HostBatch(schema, clock[a_:b_], [k[a_:b_], v[a_:b_], ext[a_:b_]], 25))
        gf, of = _finds(g, spans), _finds(o, spans)
        assert gf == of, f"retrieval differs after {b_} events"
        assert sum(len(x) for x in gf) > 0
    for q in (g, o):
        q.advance_time(int(clock[-1]) + 3 * 86_400_000)
    assert _finds(g, spans) == _finds(o, spans)
    g.close()
    o.close()


# ---- checkpoint of an aggregation (sh_aggregation_snapshot / restore) --------------------------------
@pytest.mark.parametrize("ktype,lag", [("int", 70_000), ("string", 70_000), ("string", 1_000)])
def test_aggregation_checkpoint_restores_executors_and_tables(rt, ktype, lag):
    """Snapshot mid-stream (root window pending, roll-up stores mid-bucket, late events); the rest of the
    stream pushed into (a) a fresh aggregation restored from the blob and (b) the original rolled back
    after it had moved on must give the uninterrupted oracle's tables and retrievals. String keys with
    short lags snapshot the root in band mode, with 70 s lags in its open-addressing mode."""
    rng = np.random.default_rng(47)
    n = 30_000
    clock = 1_706_745_000_000 + np.cumsum(rng.integers(0, 50, n)).astype(np.int64)
    if lag < 10_000:
        clock = 1_706_745_000_000 + np.arange(n, dtype=np.int64) // 4  # pushes span a few sec buckets
    ext = clock - rng.integers(0, lag, n).astype(np.int64)
    k = rng.integers(0, 30, n).astype(np.int32)
    v = np.round(rng.normal(50, 20, n), 3)
    schema = abi.Schema.parse(f"k {ktype}, v double, ts long")
    spec = abi.AggregationSpec(schema, [("sum", "v"), ("avg", "v"), ("min", "v"), ("max", "v")], group_by=["k"],
                               ts="ts", durations=("sec", "day"), key_capacity=64)
    bat = lambda a_, b_: abi.HostBatch(schema, clock[a_:b_], [k[a_:b_], v[a_:b_], ext[a_:b_]], 9)
    cut = 13_001
    g = rt.GpuAggregation(spec)
    g.push(bat(0, cut))
    blob = g.snapshot()
    g.push(bat(cut, 20_000))  # moves on past the snapshot
    fresh = rt.GpuAggregation(spec)
    fresh.restore(blob)
    g.restore(blob)  # roll back the running aggregation
    o = OracleAggregation(spec)
    o.push(bat(0, cut))
    rest = [bat(cut, n), ("advance", int(clock[-1]) + 2 * 86_400_000)]
    spans = [(abi.DUR_NAMES[d], 0, 1 << 62) for d in ("sec", "hour", "day")]
    assert _finds(fresh, spans) == _finds(o, spans) == _finds(g, spans)
    for x in (g, fresh, o):
        drive(x, rest[:1])
    assert _finds(fresh, spans) == _finds(o, spans) == _finds(g, spans)
    for x in (g, fresh, o):
        drive(x, rest[1:])
    ot = tables(o, spec)
    assert_tables_equal(tables(fresh, spec), ot, "restored")
    assert_tables_equal(tables(g, spec), ot, "rolled back")
    with pytest.raises(Exception, match="different aggregation|does not match"):
        other = rt.GpuAggregation(abi.AggregationSpec(schema, [("sum", "v")], group_by=["k"], ts="ts",
                                                      durations=("sec", "day"), key_capacity=64))
        other.restore(blob)
    for x in (g, fresh, o):
        x.close()


@pytest.mark.parametrize("ktype", ["int", "string"])
def test_aggregation_truncated_blob_rolls_back(rt, ktype):
    """sh_aggregation_restore from a truncated blob fails part-way (after the root window or inside an
    executor / table section) and rolls the aggregation back to its state before the call."""
    rng = np.random.default_rng(5)
    n = 20_000
    clock = 1_706_745_000_000 + np.cumsum(rng.integers(0, 40, n)).astype(np.int64)
    k = rng.integers(0, 20, n).astype(np.int32)
    v = np.round(rng.normal(10, 3, n), 2)
    schema = abi.Schema.parse(f"k {ktype}, v double, ts long")
    spec = abi.AggregationSpec(schema, [("sum", "v"), ("max", "v")], group_by=["k"], ts="ts",
                               durations=("sec", "hour"), key_capacity=32)
    bat = lambda a_, b_: abi.HostBatch(schema, clock[a_:b_], [k[a_:b_], v[a_:b_], clock[a_:b_]], 1)
    g, o = rt.GpuAggregation(spec), OracleAggregation(spec)
    for x in (g, o):
        x.push(bat(0, 8_000))
    blob = g.snapshot()
    for x in (g, o):
        x.push(bat(8_000, 12_000))
    for cut in (30, len(blob) // 2, len(blob) - 3):
        with pytest.raises(Exception, match="truncated|does not match|restore"):
            g.restore(blob[:cut])
    for x in (g, o):
        drive(x, [bat(12_000, n), ("advance", int(clock[-1]) + 7_200_000)])
    assert_tables_equal(tables(g, spec), tables(o, spec), "after failed restores")
    for x in (g, o):
        x.close()


def test_device_pushes_speculative_band(rt):
    """Device pushes of a band-keyed root place the band from the queued events' bucket range measured
    behind the previous push (no probe round trip); k_boundaries validates it and a push with a bucket
    outside the band is probed and pushed again before anything was committed. Pushes of in-order events
    (the speculation holds), pushes with events up to 40 s late (retried), a push after a TIMER and a push
    after a checkpoint restore: every table equal to the oracle's (host pushes of the same events)."""
    import torch
    rng = np.random.default_rng(33)
    n = 1_200_000
    clock = 1_700_000_000_000 + np.arange(n, dtype=np.int64) // 200  # 200 events per ms: 100k events span 0.5 s
    lag = np.zeros(n, np.int64)
    lag[500_000:520_000] = rng.integers(0, 40_000, 20_000)
    lag[900_000:900_050] = 3_000
    ext = clock - lag
    k = rng.integers(0, 4_000, n).astype(np.int32)
    v = np.round(rng.normal(50, 20, n), 2)
    spec = abi.AggregationSpec(STR_SCHEMA, [("sum", "v"), ("avg", "v"), ("count", None), ("min", "v"), ("max", "v")],
                               group_by=["k"], ts="ts", durations=("sec", "hour"), key_capacity=4_000)
    cuts = [0, 100_000, 200_000, 330_000, 480_000, 600_000, 700_000, 800_000, 1_000_000, n]
    dev = torch.device("cuda", 0)
    g, o = rt.GpuAggregation(spec), OracleAggregation(spec)
    for i, (a, b) in enumerate(zip(cuts, cuts[1:])):
        cols = [torch.from_numpy(np.ascontiguousarray(x[a:b])).to(dev) for x in (k, v, ext)]
        t = torch.from_numpy(np.ascontiguousarray(clock[a:b])).to(dev)
        torch.cuda.synchronize()
        g.push_device(b - a, t.data_ptr(), [c.data_ptr() for c in cols], 1)
        o.push(abi.HostBatch(STR_SCHEMA, clock[a:b], [k[a:b], v[a:b], ext[a:b]], 1))
        if i == 3:
            now = int(clock[b - 1]) + 1_500
            g.advance_time(now)
            o.advance_time(now)
        if i == 5:
            blob = g.snapshot()
            g.close()
            g = rt.GpuAggregation(spec)
            g.restore(blob)
        if i in (2, 6):
            assert_tables_equal(tables(g, spec), tables(o, spec), f"spec band@{i}")
        del cols, t
    now = int(clock[-1]) + 2 * 3_600_000
    g.advance_time(now)
    o.advance_time(now)
    assert_tables_equal(tables(g, spec), tables(o, spec), "spec band end")
    g.close()
    o.close()


# ---- group keys the root cannot key directly: two group-by columns, 64-bit keys (interned) ------------
@pytest.mark.parametrize("schema_text,group_by", [
    ("k int, s string, v double, ts long", ["k", "s"]),
    ("k long, s string, v double, ts long", ["k"]),
    ("k int, s string, v double, ts long", ["s", "k"]),
    ("k long, s string, v double, ts long", ["s", "k"]),
])
def test_interned_group_keys_rollups_retrieval_checkpoint(rt, schema_text, group_by):
    """`group by a, b` and `group by <long>` under `aggregate by`: the group key is interned to a dense
    id on the device (sh_aggregation.cpp intern) and decoded back on every table row and retrieval.
    Late events, a mid-stream checkpoint restored into a fresh aggregation, retrievals and every
    duration's table equal the oracle's."""
    rng = np.random.default_rng(71)
    n = 40_000
    clock = 1_706_745_000_000 + np.cumsum(rng.integers(0, 30, n)).astype(np.int64)
    ext = clock - rng.integers(0, 50_000, n).astype(np.int64)
    schema = abi.Schema.parse(schema_text)
    k = rng.integers(0, 40, n)
    k = (k * 3_000_000_007 - 60_000_000_000).astype(np.int64) if schema_text.startswith("k long") else k.astype(np.int32)
    s = rng.integers(0, 7, n).astype(np.int32)
    v = np.round(rng.normal(50, 20, n), 3)
    spec = abi.AggregationSpec(schema, [("sum", "v"), ("count", None), ("min", "v"), ("max", "v")],
                               group_by=group_by, ts="ts", durations=("sec", "day"), key_capacity=512)
    bat = lambda a_, b_: abi.HostBatch(schema, clock[a_:b_], [k[a_:b_], s[a_:b_], v[a_:b_], ext[a_:b_]], 7)
    g, o = rt.GpuAggregation(spec), OracleAggregation(spec)
    cut = 17_001
    for x in (g, o):
        x.push(bat(0, cut))
    spans = [(abi.DUR_NAMES[d], 0, 1 << 62) for d in ("sec", "min", "day")]
    assert _finds(g, spans) == _finds(o, spans)
    blob = g.snapshot()
    fresh = rt.GpuAggregation(spec)
    fresh.restore(blob)
    rest = [bat(cut, 30_000), bat(30_000, n), ("advance", int(clock[-1]) + 2 * 86_400_000)]
    for x in (g, fresh, o):
        drive(x, rest[:2])
    assert _finds(fresh, spans) == _finds(o, spans) == _finds(g, spans)
    for x in (g, fresh, o):
        drive(x, rest[2:])
    ot = tables(o, spec)
    assert sum(len(t["ts"]) for t in ot.values()) > 0
    assert_tables_equal(tables(g, spec), ot, "interned")
    # tables drain on read: the restored copy is compared against a re-run oracle
    o2 = OracleAggregation(spec)
    for p in [bat(0, cut)] + rest:
        drive(o2, [p])
    assert_tables_equal(tables(fresh, spec), tables(o2, spec), "interned restored")
    for x in (g, fresh, o, o2):
        x.close()


@pytest.mark.parametrize("tz_hours", [8, -5])
def test_agg_time_zone_offset_buckets(rt, tz_hours):
    """`@store(aggTimeZone)` as a fixed offset: hour and day buckets start at local boundaries
    (IncrementalTimeConverterUtil with a zone); sec/min are offset-invariant."""
    ts, cols = synth.keyed_stream(1_700_000_000_000 - 15_000, 120_000, 0xA7, 300, 1)
    cols[2] = ts - (np.arange(len(ts)) % 97) * 1_000  # late events crossing hour boundaries
    pushes = split_batches(C4_SCHEMA, ts, cols, [40_000, 80_000], 300)
    pushes.append(("advance", int(ts[-1]) + 3 * 86_400_000))
    spec = abi.AggregationSpec(C4_SCHEMA, [("sum", "v"), ("count", None), ("max", "v")], group_by=["k"], ts="ts",
                               durations=("min", "day"), key_capacity=300, tz_offset_ms=tz_hours * 3_600_000)
    assert both(rt, spec, pushes, f"tz{tz_hours}", checkpoints=(0, 1)) > 0


@pytest.mark.parametrize("root,tz_hours,proc_time", [("month", 0, False), ("month", 8, False), ("year", -5, False),
                                                     ("month", 0, True)])
def test_calendar_roots(rt, root, tz_hours, proc_time):
    """`every month ...` / `every year` roots: the root window closes at calendar boundaries of the clock
    (getNextEmitTime MONTHS / YEARS) and its buckets are the events' calendar months / years in the zone
    offset; late events, idle gaps of several months, retrievals and a checkpoint = oracle."""
    rng = np.random.default_rng(91)
    n = 30_000
    day = 86_400_000
    step = 40 * day // n if root == "month" else 900 * day // n  # ~40 days or ~2.5 years of clock
    clock = 1_700_000_000_000 + np.cumsum(rng.integers(0, 2 * step, n)).astype(np.int64)
    clock[n // 2:] += (95 if root == "month" else 800) * day  # an idle gap
    ext = clock - rng.integers(0, 20 * day, n).astype(np.int64)
    k = rng.integers(0, 25, n).astype(np.int32)
    v = np.round(rng.normal(50, 20, n), 3)
    schema = abi.Schema.parse("k int, v double, ts long")
    durs = (root, "year")
    spec = abi.AggregationSpec(schema, [("sum", "v"), ("count", None), ("min", "v"), ("max", "v")], group_by=["k"],
                               ts=None if proc_time else "ts", durations=durs, key_capacity=32,
                               tz_offset_ms=tz_hours * 3_600_000)
    bat = lambda a_, b_: abi.HostBatch(schema, clock[a_:b_], [k[a_:b_], v[a_:b_], ext[a_:b_]], 11)
    cuts = [0, 5_000, 14_999, 15_000, 22_000, n]
    g, o = rt.GpuAggregation(spec), OracleAggregation(spec)
    spans = [(abi.DUR_NAMES[d], 0, 1 << 62) for d in dict.fromkeys(durs)]
    blob = None
    for a_, b_ in zip(cuts[:-1], cuts[1:]):
        for x in (g, o):
            x.push(bat(a_, b_))
        assert _finds(g, spans) == _finds(o, spans), f"retrieval after {b_}"
        if b_ == 14_999:
            blob = g.snapshot()
    for x in (g, o):
        x.advance_time(int(clock[-1]) + 800 * day)
    ot = tables(o, spec)
    assert sum(len(t["ts"]) for t in ot.values()) > 0
    assert_tables_equal(tables(g, spec), ot, f"{root} root")
    fresh, o2 = rt.GpuAggregation(spec), OracleAggregation(spec)
    fresh.restore(blob)
    o2.push(bat(0, 5_000))
    o2.push(bat(5_000, 14_999))
    for a_, b_ in zip(cuts[2:-1], cuts[3:]):
        for x in (fresh, o2):
            x.push(bat(a_, b_))
    for x in (fresh, o2):
        x.advance_time(int(clock[-1]) + 800 * day)
    assert_tables_equal(tables(fresh, spec), tables(o2, spec), f"{root} root restored")
    for x in (g, o, fresh, o2):
        x.close()


def test_three_group_by_columns_rollups_and_retrieval(rt):
    """`group by k, s, l` (int, string, long) under `aggregate by`: interned by the chain of sh_wide.h;
    tables, retrievals and a checkpoint = oracle."""
    rng = np.random.default_rng(73)
    n = 30_000
    clock = 1_706_745_000_000 + np.cumsum(rng.integers(0, 30, n)).astype(np.int64)
    ext = clock - rng.integers(0, 40_000, n).astype(np.int64)
    schema = abi.Schema.parse("k int, s string, l long, v double, ts long")
    k = rng.integers(-4, 5, n).astype(np.int32)
    s = rng.integers(0, 4, n).astype(np.int32)
    l = (rng.integers(0, 5, n) * 7_000_000_001).astype(np.int64)
    v = np.round(rng.normal(50, 20, n), 3)
    spec = abi.AggregationSpec(schema, [("sum", "v"), ("count", None), ("max", "v")], group_by=["s", "k", "l"],
                               ts="ts", durations=("sec", "hour"), key_capacity=512)
    bat = lambda a_, b_: abi.HostBatch(schema, clock[a_:b_], [k[a_:b_], s[a_:b_], l[a_:b_], v[a_:b_], ext[a_:b_]], 5)
    g, o = rt.GpuAggregation(spec), OracleAggregation(spec)
    spans = [(abi.DUR_NAMES[d], 0, 1 << 62) for d in ("sec", "min", "hour")]
    for a_, b_ in ((0, 9_000), (9_000, 21_000)):
        for x in (g, o):
            x.push(bat(a_, b_))
        assert _finds(g, spans) == _finds(o, spans)
    blob = g.snapshot()
    fresh = rt.GpuAggregation(spec)
    fresh.restore(blob)
    for x in (g, fresh, o):
        x.push(bat(21_000, n))
    assert _finds(fresh, spans) == _finds(o, spans) == _finds(g, spans)
    for x in (g, o):
        x.advance_time(int(clock[-1]) + 7_200_000)
    ot = tables(o, spec)
    assert all(t["keys"].shape[0] == 4 for t in ot.values())
    assert_tables_equal(tables(g, spec), ot, "three group-by columns")
    for x in (g, fresh, o):
        x.close()


def test_negative_aggregate_by_timestamps_refused(rt):
    """Events before 1970 (negative `aggregate by` values) fail loudly instead of landing in wrong buckets."""
    schema = abi.Schema.parse("k int, v double, ts long")
    spec = abi.AggregationSpec(schema, [("sum", "v")], group_by=["k"], ts="ts", durations=("sec", "hour"), key_capacity=16)
    g = rt.GpuAggregation(spec)
    n = 70_000
    clock = 1_700_000_000_000 + np.arange(n, dtype=np.int64)
    k = (np.arange(n) % 7).astype(np.int32)
    v = np.ones(n)
    g.push(abi.HostBatch(schema, clock, [k, v, clock.copy()], 1))
    bad = clock.copy()
    bad[n // 2] = -5_000
    with pytest.raises(rt.SiddhiError, match="before 1970"):
        g.push(abi.HostBatch(schema, clock + n, [k, v, bad], 1))
    g.close()
