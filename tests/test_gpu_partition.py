"""GPU parity of `partition with (p of S)` around lengthBatch(L) and time(T) windows grouped by the
partition key or without group-by (sh_plane.cpp: one lane per partition), against the oracle's
restatement of PartitionStreamReceiver.receive (:176-272: runs of equal partition keys per send, one
window / aggregator state per partition), LengthBatchWindowProcessor (:153-243), TimeWindowProcessor
(:132-169) and the Scheduler's TIMER calls per partition (Scheduler.java:71-104, 171-209, including
its TreeMultimap tie rule: of several partitions due at the same time only the first met while walking
PartitionStateHolder.states fires — java.util.HashMap<String, …> order of String.valueOf(partition key),
restated twice and independently: oracle/jhashmap.h and siddhi_amd/csrc/sh_jmap.h).
The reference KATs (WindowPartitionTestCase partition2 lengthBatch, partition3 time) run in
test_gpu_parity.py."""
import numpy as np
import pytest

from siddhi_amd import abi, synth
from tests.parity import split_batches
from tests.test_gpu_sliding_expired import both

pytestmark = pytest.mark.gpu

SCHEMA = abi.Schema.parse("p int, v double, x long, ts long")
AGGS = [("count", None), ("sum", "v"), ("min", "v"), ("max", "x"), ("avg", "x"), ("sum", "x")]


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def stream(n, parts, seed, step=3, runs=False, zipf=False):
    rng = np.random.default_rng(seed)
    ts = (np.cumsum(rng.integers(0, step, n)) + 10_000).astype(np.int64)
    if zipf:
        p = (synth.zipf_keys(0, n, seed, parts) % parts).astype(np.int32)
    else:
        p = rng.integers(0, parts, n).astype(np.int32)
    if runs:  # runs of equal partition keys (the receiver's chunks hold several events)
        p = np.repeat(p[: (n + 3) // 4], 4)[:n]
    v = rng.integers(-400, 400, n).astype(np.float64) / 8.0
    x = rng.integers(-50, 50, n).astype(np.int64)
    return ts, [p, v, x, ts.copy()]


@pytest.mark.parametrize("output", ["current", "all", "expired"])
@pytest.mark.parametrize("L,group,parts", [(1, True, 200), (3, False, 200), (100, True, 40)])
def test_partitioned_lengthbatch(rt, output, L, group, parts):
    """(L = 100 over 40 partitions: several batches per partition, so expired rows exist)"""
    ts, cols = stream(30_000, parts, 41, runs=True)
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", L, group_by=["p"] if group else [], aggs=AGGS, partition="p",
                         filter=(">", "v", -30.0), output=output, key_capacity=256)
    ref = both(rt, spec, split_batches(SCHEMA, ts, cols, [1, 7_777, 20_000], 5), f"plb {L} {output}")
    assert ref["ts"].size > 0


def test_partitioned_lengthbatch_zipf_100k_partitions(rt):
    ts, cols = stream(2_000_000, 1_000_000, 43, zipf=True)  # ~231k distinct partitions
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", 3, group_by=["p"], aggs=[("count", None), ("sum", "v"), ("max", "x")],
                         partition="p", output="all", key_capacity=1_000_000)
    ref = both(rt, spec, split_batches(SCHEMA, ts, cols, [700_000], 1), "plb zipf")
    assert len(np.unique(cols[0])) > 100_000 and ref["ts"].size > 10_000


@pytest.mark.parametrize("output", ["current", "all", "expired"])
@pytest.mark.parametrize("send_size", [1, 6])
def test_partitioned_time(rt, output, send_size):
    """ms timestamps shared by many partitions: several partitions are due at the same TIMER call"""
    ts, cols = stream(30_000, 60, 47, step=2, runs=send_size > 1)
    spec = abi.QuerySpec(SCHEMA, "time", 150, group_by=["p"], aggs=AGGS, partition="p", filter=(">", "v", -40.0),
                         output=output, key_capacity=64)
    pushes = split_batches(SCHEMA, ts, cols, [1, 5_000, 18_000], send_size)
    pushes.insert(3, ("advance", int(ts[17_999]) + 100))
    pushes.append(("advance", int(ts[-1]) + 120))
    pushes.append(("advance", int(ts[-1]) + 5_000))
    ref = both(rt, spec, pushes, f"ptime {output} {send_size}")
    assert ref["ts"].size > 0


@pytest.mark.parametrize("output", ["current", "all"])
def test_partitioned_time_min_max_with_nan(rt, output):
    """NaN values: no comparison pops them from the deque, so minValue is no longer the deque's front
    (MinAttributeAggregatorExecutor.processAdd :178-190 keeps `minValue > value`)"""
    ts, cols = stream(20_000, 8, 61, step=2)
    rng = np.random.default_rng(62)
    cols[1][rng.random(20_000) < 0.01] = np.nan
    spec = abi.QuerySpec(SCHEMA, "time", 120, group_by=["p"], aggs=[("min", "v"), ("max", "v"), ("count", None)],
                         partition="p", output=output, key_capacity=16)
    both(rt, spec, split_batches(SCHEMA, ts, cols, [6_000], 1) + [("advance", int(ts[-1]) + 200)], f"ptime nan {output}")


def test_partitioned_time_no_group_by_zipf(rt):
    ts, cols = stream(300_000, 100_000, 53, step=2, zipf=True)
    spec = abi.QuerySpec(SCHEMA, "time", 500, aggs=[("sum", "v"), ("count", None)], partition="p", output="all",
                         key_capacity=100_000)
    pushes = split_batches(SCHEMA, ts, cols, [100_000, 200_000], 1) + [("advance", int(ts[-1]) + 1_000)]
    ref = both(rt, spec, pushes, "ptime zipf")
    assert ref["expired"].sum() > 0


def _same_hash_strings(k):
    """2^k distinct strings of one String.hashCode ("Aa" and "BB" both hash to 2112): one HashMap bin at
    every capacity, so ties among them are ordered inside a red-black tree bin once 8 share it."""
    out = [""]
    for _ in range(k):
        out = [x + y for x in out for y in ("Aa", "BB")]
    return out


def test_partitioned_time_string_keys_tree_bins(rt):
    """String partition keys: 32 of equal hashCode (a tree bin as soon as 8 are armed on a table of >= 64
    bins) among 300 others; ties at every ms; partitions drained, removed and re-inserted all the time"""
    names = _same_hash_strings(5) + [f"sym{i}" for i in range(300)]
    rng = np.random.default_rng(71)
    n = 40_000
    ts = (np.cumsum(rng.integers(0, 2, n)) + 50_000).astype(np.int64)
    hot = rng.random(n) < 0.5
    pid = np.where(hot, rng.integers(0, 32, n), rng.integers(32, len(names), n)).astype(np.int32)
    v = rng.integers(-400, 400, n).astype(np.float64) / 8.0
    x = rng.integers(-50, 50, n).astype(np.int64)
    schema = abi.Schema.parse("p string, v double, x long, ts long")
    cols = [pid, v, x, ts.copy()]
    spec = abi.QuerySpec(schema, "time", 120, aggs=[("count", None), ("sum", "v"), ("max", "x")], partition="p",
                         output="all", key_capacity=512, strings={"p": names})
    pushes = split_batches(schema, ts, cols, [3_000, 20_000], 1) + [("advance", int(ts[-1]) + 60),
                                                                     ("advance", int(ts[-1]) + 1_000)]
    ref = both(rt, spec, pushes, "ptime tree bins")
    assert ref["expired"].sum() > 1000


def test_partition_key_without_text_fails_loudly(rt):
    schema = abi.Schema.parse("p string, v double, ts long")
    spec = abi.QuerySpec(schema, "time", 100, aggs=[("sum", "v")], partition="p", output="all", key_capacity=16)
    g = rt.GpuQuery(spec)
    g.set_strings("p", ["a", "b"])
    b = abi.HostBatch.from_rows(schema, [(1000, 0, 1.0, 1000), (1000, 2, 2.0, 1000)], 1)
    with pytest.raises(rt.SiddhiError, match="no text"):
        g.push(b)
    g.close()


@pytest.mark.parametrize("output", ["current", "all", "expired"])
@pytest.mark.parametrize("L,group,parts,zipf", [(1, False, 50, False), (2, True, 300, False), (7, False, 40, False),
                                               (3, True, 200_000, True)])
def test_partitioned_lengthbatch_stream_current(rt, output, L, group, parts, zipf):
    """lengthBatch(L, true) under `partition with`: a row per event (the partition's running aggregates),
    the (L + 1)-th event of a batch resetting it (PartitionTestCase2.java:681-736's shape at scale)"""
    ts, cols = stream(60_000 if not zipf else 400_000, parts, 61, runs=not zipf, zipf=zipf)
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", L, group_by=["p"] if group else [], aggs=AGGS, partition="p",
                         filter=(">", "v", -30.0), output=output, stream_current=True,
                         key_capacity=max(256, parts))
    ref = both(rt, spec, split_batches(SCHEMA, ts, cols, [1, 17_777, 40_000], 3), f"plb sc {L} {output}")
    assert ref["ts"].size > 0


# ---- lane 3: partitioned lengthBatch grouped by columns other than the partition key --------------------
GSCHEMA = abi.Schema.parse("p int, g int, v double, x long, h int, ts long")


def gstream(n, parts, groups, seed, runs=False, zipf=False):
    ts, (p, v, x, ts2) = stream(n, parts, seed, runs=runs, zipf=zipf)
    rng = np.random.default_rng(seed + 1)
    g = rng.integers(0, groups, n).astype(np.int32)
    h = rng.integers(0, 3, n).astype(np.int32)
    return ts, [p, g, v, x, h, ts2]


@pytest.mark.parametrize("L,group_by,parts,runs,zipf", [(1, ["g"], 50, False, False), (4, ["g"], 30, True, False),
                                                        (37, ["g", "h"], 12, False, False),
                                                        (5, ["h", "p"], 80, True, False),
                                                        (3, ["g"], 100_000, False, True)])
def test_partitioned_lengthbatch_stream_current_group_by_other(rt, L, group_by, parts, runs, zipf):
    """lengthBatch(L, true) grouped by other columns: every event its own chunk, its row the group's fold
    over the partition's batch so far (the partition's (L + 1)-th event of a batch resets every group);
    open batches carried across pushes fold without emitting again"""
    ts, cols = gstream(200_000 if zipf else 30_000, parts, 7, 67, runs=runs, zipf=zipf)
    spec = abi.QuerySpec(GSCHEMA, "lengthBatch", L, group_by=group_by, aggs=AGGS, partition="p",
                         filter=(">", "v", -30.0), stream_current=True, key_capacity=max(256, parts))
    ref = both(rt, spec, split_batches(GSCHEMA, ts, cols, [1, 9_999, 17_000], 3), f"plg sc {L} {group_by}")
    assert ref["ts"].size > 0


def test_partitioned_stream_current_group_by_other_expired_refused(rt):
    spec = abi.QuerySpec(GSCHEMA, "lengthBatch", 3, group_by=["g"], aggs=AGGS, partition="p", output="all",
                         stream_current=True, key_capacity=64)
    with pytest.raises(rt.SiddhiError, match="not on the GPU|stream.current|partitioned"):
        rt.GpuQuery(spec)


@pytest.mark.parametrize("output", ["current", "all", "expired"])
@pytest.mark.parametrize("L,group_by,parts,runs", [(1, ["g"], 50, False), (4, ["g"], 30, True),
                                                   (37, ["g", "h"], 12, False), (5, ["h", "p"], 80, True),
                                                   (9, ["x"], 20, False)])
def test_partitioned_lengthbatch_group_by_other(rt, output, L, group_by, parts, runs):
    """Every completed batch of a partition is one chunk [previous batch EXPIRED, RESET, batch] whose
    rows are one per group key in first-insertion order (QuerySelector.processInBatchGroupBy :315-374);
    pushes cut batches open and send sizes put several partitions' batches into one send."""
    ts, cols = gstream(30_000, parts, 7, 61, runs=runs)
    spec = abi.QuerySpec(GSCHEMA, "lengthBatch", L, group_by=group_by, aggs=AGGS, partition="p",
                         filter=(">", "v", -30.0), output=output, key_capacity=1024)
    ref = both(rt, spec, split_batches(GSCHEMA, ts, cols, [1, 9_001, 9_002, 21_000], 3), f"plg {L} {group_by} {output}")
    assert ref["ts"].size > 0
    if output != "current" and L > 1:
        assert ref["expired"].sum() > 0


def test_partitioned_lengthbatch_group_by_other_long_batches(rt):
    """L larger than a push: batches stay open across pushes (carried records) before completing"""
    ts, cols = gstream(40_000, 6, 20, 67)
    spec = abi.QuerySpec(GSCHEMA, "lengthBatch", 2_500, group_by=["g"], aggs=AGGS, partition="p", output="all",
                         key_capacity=64)
    pushes = split_batches(GSCHEMA, ts, cols, [700, 1_500, 8_000, 8_100, 30_000], 1)
    ref = both(rt, spec, pushes, "plg long")
    assert ref["ts"].size > 0


def test_partitioned_lengthbatch_zipf_100k_partitions_second_group_column(rt):
    """>= 100k Zipf partitions, grouped by (partition, a second column)"""
    ts, cols = gstream(2_000_000, 1_000_000, 5, 73, zipf=True)
    spec = abi.QuerySpec(GSCHEMA, "lengthBatch", 3, group_by=["p", "g"],
                         aggs=[("count", None), ("sum", "v"), ("max", "x")], partition="p", output="all",
                         key_capacity=1 << 21)
    ref = both(rt, spec, split_batches(GSCHEMA, ts, cols, [700_000], 1), "plg zipf")
    assert len(np.unique(cols[0])) > 100_000 and ref["ts"].size > 10_000


@pytest.mark.parametrize("output", ["current", "all", "expired"])
@pytest.mark.parametrize("L,group", [(1, True), (3, False), (100, True)])
def test_partitioned_lengthbatch_walk_lanes(rt, monkeypatch, output, L, group):
    """SH_PL_SORT=0: lengthBatch keyed by the partition (or without group-by) on one sequential lane per
    partition instead of the sorted chunks (the default) — the same rows"""
    monkeypatch.setenv("SH_PL_SORT", "0")
    ts, cols = stream(30_000, 40 if L == 100 else 200, 41, runs=True)
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", L, group_by=["p"] if group else [], aggs=AGGS, partition="p",
                         filter=(">", "v", -30.0), output=output, key_capacity=256)
    ref = both(rt, spec, split_batches(SCHEMA, ts, cols, [1, 7_777, 20_000], 5), f"plb walk {L} {output}")
    assert ref["ts"].size > 0


def test_partitioned_lengthbatch_walk_lanes_zipf(rt, monkeypatch):
    monkeypatch.setenv("SH_PL_SORT", "0")
    ts, cols = stream(2_000_000, 1_000_000, 43, zipf=True)
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", 3, group_by=["p"], aggs=[("count", None), ("sum", "v"), ("max", "x")],
                         partition="p", output="all", key_capacity=1_000_000)
    ref = both(rt, spec, split_batches(SCHEMA, ts, cols, [700_000], 1), "plb walk zipf")
    assert ref["ts"].size > 10_000


# ---- time / externalTime lanes grouped by other columns (operations per partition, replayed per
# (partition, group) state) -----------------------------------------------------------------------------
GAGGS = [("count", None), ("sum", "v"), ("avg", "x"), ("sum", "x")]


@pytest.mark.parametrize("output", ["current", "all", "expired"])
@pytest.mark.parametrize("send_size,group_by", [(1, ["g"]), (6, ["g", "h"]), (1, ["h", "p"])])
def test_partitioned_time_group_by_other(rt, output, send_size, group_by):
    ts, cols = gstream(30_000, 40, 6, 79, runs=send_size > 1)
    spec = abi.QuerySpec(GSCHEMA, "time", 150, group_by=group_by, aggs=GAGGS, partition="p", filter=(">", "v", -40.0),
                         output=output, key_capacity=512)
    pushes = split_batches(GSCHEMA, ts, cols, [1, 5_000, 18_000], send_size)
    pushes.insert(3, ("advance", int(ts[17_999]) + 100))
    pushes.append(("advance", int(ts[-1]) + 120))
    pushes.append(("advance", int(ts[-1]) + 5_000))
    ref = both(rt, spec, pushes, f"ptime group {group_by} {output} {send_size}")
    assert ref["ts"].size > 0


def test_partitioned_time_group_by_other_zipf(rt):
    ts, cols = gstream(300_000, 100_000, 4, 83, zipf=True)
    spec = abi.QuerySpec(GSCHEMA, "time", 400, group_by=["g"], aggs=[("sum", "v"), ("count", None)], partition="p",
                         output="all", key_capacity=100_000)
    pushes = split_batches(GSCHEMA, ts, cols, [100_000, 200_000], 1) + [("advance", int(ts[-1]) + 1_000)]
    ref = both(rt, spec, pushes, "ptime group zipf")
    assert ref["expired"].sum() > 0


@pytest.mark.parametrize("output", ["current", "all", "expired"])
@pytest.mark.parametrize("send_size", [1, 5])
def test_partitioned_time_group_by_other_min_max(rt, output, send_size):
    """min / max per (partition, group) state: MinAttributeAggregatorExecutor's deque with
    removeFirstOccurrence (values repeat: the quirk fires), carried between pushes in a pool"""
    ts, cols = gstream(40_000, 25, 4, 89, runs=send_size > 1)
    spec = abi.QuerySpec(GSCHEMA, "time", 120, group_by=["g"],
                         aggs=[("min", "v"), ("max", "v"), ("max", "x"), ("count", None), ("min", "h")], partition="p",
                         filter=(">", "v", -45.0), output=output, key_capacity=256)
    pushes = split_batches(GSCHEMA, ts, cols, [1, 9_000, 9_001, 25_000], send_size)
    pushes.insert(3, ("advance", int(ts[8_999]) + 60))
    pushes.append(("advance", int(ts[-1]) + 5_000))
    ref = both(rt, spec, pushes, f"ptime group minmax {output} {send_size}")
    assert ref["ts"].size > 0


def test_partitioned_time_group_by_other_pair_churn(rt):
    """Many more (partition, group) pairs over the stream than the pair table holds at creation (400 x 400
    pairs, key_capacity 400: 64k pairs fit at half load), few alive at once: emptied states are dropped
    (PartitionStateHolder.returnState) when the table is rebuilt before a push could overfill it. Min / max
    deques ride along. A snapshot taken after the rebuilds restores into a fresh query (the pair table at
    the blob's size) and continues like the oracle."""
    from oracle.oracle import OracleQuery
    from tests.parity import assert_same, run_pushes
    from siddhi_amd import abi as _abi
    ts, cols = gstream(400_000, 400, 400, 97)
    spec = abi.QuerySpec(GSCHEMA, "time", 100, group_by=["g"], aggs=[("count", None), ("sum", "v"), ("max", "v")],
                         partition="p", output="all", key_capacity=400)
    pushes = split_batches(GSCHEMA, ts, cols, [50_000, 120_000, 200_000, 290_000, 330_000], 1)
    g = rt.GpuQuery(spec)
    part1 = run_pushes(g, pushes[:4])
    blob = g.snapshot()
    g.close()
    g2 = rt.GpuQuery(spec)
    g2.restore(blob)
    part2 = run_pushes(g2, pushes[4:] + [("advance", int(ts[-1]) + 1_000)])
    g2.close()
    o = OracleQuery(spec)
    want = run_pushes(o, pushes + [("advance", int(ts[-1]) + 1_000)])
    o.close()
    assert_same(_abi.concat_arrays([part1, part2]), want, label="pair churn")
    assert want["expired"].sum() > 0


# ---- float / double partition keys (round 5): String.valueOf(value) names the partitions — the bits,
# every NaN one partition, 0.0 and -0.0 two; where the Scheduler's tie order decides the output (time windows
# with expired output) it hashes that text, Double.toString / Float.toString
FSCHEMA = abi.Schema.parse("p double, g int, v double, x long, f float, ts long")


def fstream(n, parts, seed, runs=False):
    ts, (p, g, v, x, h, ts2) = gstream(n, parts, 7, seed, runs=runs)
    vals = np.array([0.0, -0.0, np.nan, 1.5, -2.25, 1e300, 3.0, -7.0] + [0.5 * i for i in range(8, parts)], np.float64)
    pd = vals[p % len(vals)]
    pd[(np.arange(n) % 97) == 5] = np.frombuffer(np.uint64(0x7FF0000000000123).tobytes(), np.float64)[0]  # a NaN payload
    with np.errstate(over="ignore", invalid="ignore"):  # (1e300 -> inf, the NaN payload -> a float NaN)
        f32 = pd.astype(np.float32)
    return ts, [pd, g, v, x, f32, ts2]


@pytest.mark.parametrize("window,L,group_by,output,stream_current",
                         [("lengthBatch", 3, ["p"], "all", False), ("lengthBatch", 4, ["g"], "current", False),
                          ("lengthBatch", 2, [], "current", True), ("lengthBatch", 5, ["g"], "current", True),
                          ("time", 40, ["p"], "current", False), ("timeBatch", 30, ["g"], "all", False),
                          ("externalTimeBatch", 25, ["g"], "current", False)])
@pytest.mark.parametrize("pcol", ["p", "f"])
def test_float_partition_keys(rt, window, L, group_by, output, stream_current, pcol):
    ts, cols = fstream(20_000, 12, 71, runs=True)
    if pcol == "f":
        group_by = ["f" if c == "p" else c for c in group_by]
    kw = {"ts_attr": "ts"} if window == "externalTimeBatch" else {}
    spec = abi.QuerySpec(FSCHEMA, window, L, group_by=group_by, aggs=[("count", None), ("sum", "v"), ("max", "x")],
                         partition=pcol, output=output, stream_current=stream_current, key_capacity=64, **kw)
    pushes = split_batches(FSCHEMA, ts, cols, [1, 7_000], 3)
    if window in ("time", "timeBatch"):
        pushes.append(("advance", int(ts[-1]) + 10 * L))
    ref = both(rt, spec, pushes, f"fp partition {window} {group_by} {pcol}")
    assert ref["ts"].size > 0


@pytest.mark.parametrize("pcol,group_by,output", [("p", ["p"], "all"), ("p", [], "expired"), ("f", ["f"], "all"),
                                                  ("f", [], "all")])
def test_float_partition_keys_time_expired(rt, pcol, group_by, output):
    """time windows with expired output: partitions due at one clock fire in the HashMap order of their
    String.valueOf texts — Double.toString / Float.toString ("-0.0", "NaN", "1.0E300", "Infinity", "4.9E-324")
    (sh_jmap.h java_fp_text; oracle jhashmap.h fp_decimal)"""
    ts, cols = fstream(20_000, 40, 73)
    rng = np.random.default_rng(74)
    ts = (10_000 + np.cumsum(rng.random(ts.size) < 0.15)).astype(np.int64)  # ~7 events per ms: ties
    cols[5] = ts.copy()
    cols[0][::53] = 5e-324
    cols[0][7::61] = 1e-5
    cols[0][9::67] = 12345678.9
    if pcol == "f":
        with np.errstate(over="ignore", invalid="ignore"):
            cols[4] = cols[0].astype(np.float32)
    spec = abi.QuerySpec(FSCHEMA, "time", 40, group_by=group_by, aggs=[("count", None), ("sum", "v")], partition=pcol,
                         output=output, key_capacity=128)
    pushes = split_batches(FSCHEMA, ts, cols, [3_000, 11_000], 2)
    pushes.append(("advance", int(ts[-1]) + 400))
    ref = both(rt, spec, pushes, f"fp partition time expired {pcol} {group_by} {output}")
    assert ref["expired"].sum() > 0


# ---- partitioned timeBatch(T, true) — stream.current.event, current output (lane 4): every partition
# chunk goes out with its groups' running values; TimeBatchWindowProcessor's nextEmitTime is one field
# for all partitions (:128), so a partition's state is RESET only when its own chunk or TIMER finds the
# playback clock at or past it — the first partition's TIMERs while events keep coming, whichever
# partition meets a lagging nextEmitTime after an idle stretch (it then schedules the next TIMER) ---------
def gap_stream(n, parts, seed, zipf=False, gaps=True, runs=False):
    ts, cols = stream(n, parts, seed, step=3, runs=runs, zipf=zipf)
    if gaps:  # idle stretches of several periods: nextEmitTime lags and other partitions reset
        rng = np.random.default_rng(seed + 1)
        jump = (rng.random(n) < 1 / 3000) * rng.integers(2_000, 9_000, n)
        ts = ts + np.cumsum(jump).astype(np.int64)
        cols[3] = ts.copy()
    return ts, cols


TB_SCHEMA = abi.Schema.parse("p int, g int, v double, x long, ts long")


@pytest.mark.parametrize("group_by,send_size,runs", [(["p"], 1, False), ([], 5, True), (["g"], 1, False),
                                                      (["g", "p"], 3, True)])
def test_partitioned_timebatch_stream_current(rt, group_by, send_size, runs):
    ts, cols = gap_stream(40_000, 97, 61, runs=runs)
    g = ((cols[0].astype(np.int64) * 7 + np.arange(len(ts))) % 5).astype(np.int32)
    tcols = [cols[0], g, cols[1], cols[2], cols[3]]
    spec = abi.QuerySpec(TB_SCHEMA, "timeBatch", 700, group_by=group_by, aggs=AGGS, partition="p",
                         stream_current=True, filter=(">", "v", -40.0), key_capacity=256)
    pushes = split_batches(TB_SCHEMA, ts, tcols, [1, 9_000, 9_001, 25_000], send_size)
    out = []
    for i, p in enumerate(pushes):  # advance_time between some pushes (TIMER calls without events)
        out.append(p)
        if i % 2 == 1:
            out.append(("advance", int(p.ts[-1]) + (3_000 if i % 4 == 1 else 1)))
    ref = both(rt, spec, out, f"ptbsc {group_by} {send_size}")
    assert ref["ts"].size > 1000


def test_partitioned_timebatch_stream_current_zipf_100k_partitions(rt):
    ts, cols = gap_stream(2_000_000, 1_000_000, 62, zipf=True)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 1000, group_by=["p"], aggs=[("count", None), ("sum", "v"), ("max", "x")],
                         partition="p", stream_current=True, key_capacity=1_000_000)
    ref = both(rt, spec, split_batches(SCHEMA, ts, cols, [700_000, 1_400_000], 1), "ptbsc zipf")
    assert len(np.unique(cols[0])) > 100_000 and ref["ts"].size > 100_000


def test_partitioned_timebatch_stream_current_checkpoint_and_rate(rt):
    from tests.parity import assert_same
    from tests.test_gpu_snapshot import checkpointed
    ts, cols = gap_stream(30_000, 41, 63)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 500, group_by=["p"], aggs=[("count", None), ("sum", "v"), ("min", "v")],
                         partition="p", stream_current=True, key_capacity=64)
    pushes = split_batches(SCHEMA, ts, cols, [8_000, 19_000], 1)
    got, ref, _ = checkpointed(spec, pushes, 1)
    assert_same(got, ref, label="ptbsc ckpt")
    spec.rate = ("first", 4)
    both(rt, spec, pushes, "ptbsc rate")
