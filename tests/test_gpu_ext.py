"""GPU parity of externalTimeBatch (f4; ExternalTimeBatchWindowProcessor): event-time batches keyed on
an attribute, flushed by the first event at or past the batch end — per event, clock-free. The HIP
path (window = bucket of the running maximum of the attribute over the events that reach the
window) must emit exactly what the oracle's line-by-line restatement of the Java state machine
emits: late events, filters, constant and attribute start times, chunked sends, many pushes."""
import numpy as np
import pytest

from oracle.oracle import OracleQuery
from siddhi_amd import abi, synth
from tests import kat_runner
from tests.parity import assert_same, run_pushes, split_batches

pytestmark = pytest.mark.gpu

SCH = abi.Schema.parse("k string, v double, et long, st long, ts long")


def both(spec, pushes, label):
    from siddhi_amd import runtime
    g = runtime.GpuQuery(spec)
    o = OracleQuery(spec)
    got, ref = run_pushes(g, pushes), run_pushes(o, pushes)
    g.close()
    o.close()
    assert_same(got, ref, label=label)
    assert ref["flush_offsets"].size > 3
    return got


def stream(n, keys, seed, late_ms=0, per_ms=20, start_ms=5_000):
    """event time `et` advances 1 ms per `per_ms` events; with late_ms > 0 10% of events lag behind."""
    ts, cols = synth.keyed_stream(0, n, seed, keys, per_ms)
    rng = np.random.default_rng(seed)
    et = start_ms + np.arange(n, dtype=np.int64) // per_ms
    if late_ms:
        late = rng.random(n) < 0.1
        et = et - late * rng.integers(0, late_ms, n)
    st = np.full(n, 4_321, dtype=np.int64)
    return ts, [cols[0], cols[1], et.astype(np.int64), st, ts.copy()]


def spec(T=1000, start=None, start_attr=None, filt=None, keys=1000, aggs=None, output="current", group=True):
    return abi.QuerySpec(SCH, "externalTimeBatch", T, group_by=["k"] if group else [], ts_attr="et", start_time=start,
                         start_attr=start_attr, filter=filt, key_capacity=keys, output=output,
                         aggs=[("count", None), ("sum", "v"), ("min", "v"), ("max", "et")] if aggs is None else aggs)


@pytest.mark.parametrize("send_size", [1, 64])
def test_ext_batches_in_order(send_size):
    ts, cols = stream(120_000, 700, 0xE1)
    both(spec(), split_batches(SCH, ts, cols, [30_000, 30_001, 77_777], send_size), "ext in-order")


def test_ext_late_events_filter_and_constant_start():
    ts, cols = stream(150_000, 2_000, 0xE2, late_ms=3_000)
    both(spec(T=2500, start=1_000, filt=(">", "v", 40.0), keys=2_000),
         split_batches(SCH, ts, cols, [50_000, 100_000], 10), "ext late/start")


def test_ext_start_from_attribute_and_many_keys():
    ts, cols = stream(200_000, 60_000, 0xE3, late_ms=500, per_ms=50)
    both(spec(T=700, start_attr="st", keys=60_000), split_batches(SCH, ts, cols, [1, 99_999], 1), "ext attr start")


def test_ext_first_event_before_start_fails_loudly():
    from siddhi_amd import runtime
    ts, cols = stream(1000, 10, 0xE4)
    g = runtime.GpuQuery(spec(start=10_000_000))
    with pytest.raises(runtime.SiddhiError, match="before its start"):
        g.push(abi.HostBatch(SCH, ts, cols, 1))


EXT_KATS = [c for c in kat_runner.load_cases()
            if c.get("query", {}).get("window") == "externalTimeBatch" and c["query"].get("aggs")]


@pytest.mark.parametrize("case", EXT_KATS, ids=[c["name"] for c in EXT_KATS])
def test_ext_reference_kat_on_gpu(case):
    from siddhi_amd import runtime
    schema, sp, dic, flushes = kat_runner.run_query(case, runtime.GpuQuery)
    kat_runner.check_query(case, flushes, schema, dic)


# ---- externalTime(et, T): sliding over the attribute (ExternalTimeWindowProcessor :126-161) ----
def ext_time_spec(T, keys, filt=None, aggs=None):
    return abi.QuerySpec(SCH, "externalTime", T, group_by=["k"], ts_attr="et", filter=filt,
                         aggs=aggs or [("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=keys)


@pytest.mark.parametrize("send_size", [1, 64])
def test_external_time_sliding_matches_oracle(send_size):
    """late events (the attribute goes backwards: the head blocks, nothing newer expires past it) and
    chunked sends; one output chunk per send."""
    ts, cols = stream(120_000, 500, 0xE8, late_ms=700)
    both(ext_time_spec(1500, 512), split_batches(SCH, ts, cols, [40_000, 40_001], send_size), "externalTime")


def test_external_time_filter_sum_and_dictionary_keys():
    ts, cols = stream(90_000, 40, 0xE9, late_ms=3000, per_ms=5)
    sp = ext_time_spec(800, 64, filt=(">", "v", 60.0), aggs=[("sum", "v"), ("max", "v"), ("count", None)])
    both(sp, split_batches(SCH, ts, cols, [1, 30_000, 59_998], 3), "externalTime filter")


@pytest.mark.parametrize("output,group", [("all", True), ("expired", True), ("all", False), ("expired", None)])
def test_ext_expired_and_all_events(output, group):
    """ExternalTimeBatchWindowProcessor.flushToOutputChunk (:336-383): the flush closing batch X carries
    batch X-1's events as EXPIRED (stamped with the attribute time that closed X: the running max of
    `et`), then RESET, then X's events; batches are never empty, so X-1 is the previous flush. Late
    events, bucket gaps (an idle stretch of event time) and batches carried across pushes.
    group None: `select *` pass-through."""
    ts, cols = stream(90_000, 20_000, 0xE7, late_ms=1_500)
    cols[2] = cols[2] + (np.arange(len(ts)) >= 50_000) * 7_000  # a gap of several empty buckets
    aggs = [] if group is None else None
    got = both(spec(T=700, output=output, group=bool(group), aggs=aggs, keys=20_000),
               split_batches(SCH, ts, cols, [20_000, 20_001, 64_000], 5), f"ext {output} {group}")
    if group is not False:  # (without group-by a chunk is one row: the current one replaces the expired)
        assert got["expired"].sum() > 1000


# ---- `partition with (p of S)` around externalTimeBatch: every partition's own event-time batches
# (the sorted partition lanes, sh_plane_group_kernels.hip) ----------------------------------------------
PSCH = abi.Schema.parse("p int, k string, v double, et long, st long, ts long")


def pstream(n, parts, seed, late_ms=0):
    ts, cols = stream(n, 50, seed, late_ms=late_ms, per_ms=5)
    rng = np.random.default_rng(seed + 7)
    p = rng.integers(0, parts, n).astype(np.int32)
    # each partition's event time starts at its own offset (its first event sets its start)
    et = cols[2] + (p.astype(np.int64) % 7) * 333
    st = cols[3] + (p.astype(np.int64) % 5) * 101
    return ts, [p, cols[0], cols[1], et, st, cols[4]]


@pytest.mark.parametrize("output", ["current", "all", "expired"])
@pytest.mark.parametrize("group_by,start,start_attr,late", [(["p"], None, None, 0), (["k"], 1_000, None, 800),
                                                            ([], None, "st", 0), (["k", "p"], None, None, 400)])
def test_partitioned_ext(output, group_by, start, start_attr, late):
    ts, cols = pstream(60_000, 37, 0xE5, late_ms=late)
    sp = abi.QuerySpec(PSCH, "externalTimeBatch", 700, group_by=group_by, ts_attr="et", start_time=start,
                       start_attr=start_attr, partition="p", key_capacity=4096, output=output,
                       aggs=[("count", None), ("sum", "v"), ("min", "v"), ("max", "et")])
    both(sp, split_batches(PSCH, ts, cols, [1, 20_000, 20_001, 41_000], 3), f"pext {group_by} {output}")


def test_partitioned_ext_checkpoint():
    from tests.test_gpu_snapshot import checkpointed
    ts, cols = pstream(40_000, 23, 0xE6, late_ms=300)
    sp = abi.QuerySpec(PSCH, "externalTimeBatch", 500, group_by=["k"], ts_attr="et", partition="p", key_capacity=4096,
                       output="all", aggs=[("count", None), ("sum", "v"), ("max", "v")])
    got, ref, _ = checkpointed(sp, split_batches(PSCH, ts, cols, [15_000, 30_000], 1), 1)
    assert_same(got, ref, label="pext ckpt")


@pytest.mark.parametrize("output", ["current", "all", "expired"])
@pytest.mark.parametrize("group,late,send_size", [(True, 0, 1), (False, 600, 4), (True, 900, 1)])
def test_partitioned_external_time(output, group, late, send_size):
    """`partition with` around externalTime(et, T): one lane per partition whose queue expires by the
    event's attribute (ExternalTimeWindowProcessor :126-161 per partition state)"""
    ts, cols = pstream(40_000, 29, 0xE8, late_ms=late)
    sp = abi.QuerySpec(PSCH, "externalTime", 400, group_by=["p"] if group else [], ts_attr="et", partition="p",
                       key_capacity=64, output=output, aggs=[("count", None), ("sum", "v"), ("min", "v"), ("max", "et")])
    pushes = split_batches(PSCH, ts, cols, [1, 12_000, 30_000], send_size) + [("advance", int(ts[-1]) + 5_000)]
    both(sp, pushes, f"pxt {group} {output}")


def test_partitioned_external_time_checkpoint():
    from tests.test_gpu_snapshot import checkpointed
    ts, cols = pstream(30_000, 17, 0xE9, late_ms=300)
    sp = abi.QuerySpec(PSCH, "externalTime", 300, group_by=["p"], ts_attr="et", partition="p", key_capacity=64,
                       output="all", aggs=[("count", None), ("sum", "v"), ("max", "v")])
    got, ref, _ = checkpointed(sp, split_batches(PSCH, ts, cols, [10_000, 20_000], 1), 1)
    assert_same(got, ref, label="pxt ckpt")


@pytest.mark.parametrize("output", ["current", "all"])
def test_partitioned_external_time_group_by_other(output):
    ts, cols = pstream(40_000, 29, 0xEA, late_ms=500)
    sp = abi.QuerySpec(PSCH, "externalTime", 400, group_by=["k"], ts_attr="et", partition="p", key_capacity=128,
                       output=output, aggs=[("count", None), ("sum", "v"), ("avg", "et"), ("min", "v"), ("max", "et")])
    both(sp, split_batches(PSCH, ts, cols, [1, 12_000, 30_000], 3), f"pxt group {output}")


# ---- externalTimeBatch(et, T, start, timeout): the scheduler timeout sends the open batch so far
# (ExternalTimeBatchWindowProcessor.process :256-305, appendToOutputChunk :385-438) --------------------
def tstream(n, seed, pause_p=1 / 3000, per_ms=20, keys=50, late_ms=0):
    """arrival clock `ts` mostly 0-2 ms apart with rare pauses of 2-9 s (each fires a 1.5 s timeout:
    several per batch, some just before a crossing); event time `et` 1 ms per `per_ms` events."""
    ts0, cols = stream(n, keys, seed, late_ms=late_ms, per_ms=per_ms)
    rng = np.random.default_rng(seed + 11)
    gaps = rng.integers(0, 3, n) + (rng.random(n) < pause_p) * rng.integers(2_000, 9_000, n)
    ts = 1_000_000 + np.cumsum(gaps).astype(np.int64)
    cols[4] = ts.copy()
    return ts, cols


def tspec(output="current", group=True, aggs=None, filt=None, timeout=1500, T=1000, start=0):
    sp = spec(T=T, start=start, filt=filt, keys=64, output=output, group=group,
              aggs=[("count", None), ("sum", "v"), ("min", "v"), ("max", "et"), ("avg", "v")] if aggs is None else aggs)
    sp.timeout = timeout
    return sp


def with_advances(pushes, ts, every=2):
    """advance_time between some pushes: past the next timeout (+4 s) or barely (+1 ms)"""
    out, clock = [], None
    for i, p in enumerate(pushes):
        out.append(p)
        clock = int(p.ts[-1]) if clock is None else max(clock, int(p.ts[-1]))
        if i % every == 0:
            clock += 4_000 if i % 4 == 0 else 1
            out.append(("advance", clock))
    return out


@pytest.mark.parametrize("send_size", [1, 7, 0])
def test_ext_timeout_group_by(send_size):
    ts, cols = tstream(80_000, 0xF1)
    pushes = split_batches(SCH, ts, cols, [1, 9_000, 9_001, 30_000, 52_345, 60_000], send_size)
    got = both(tspec(), with_advances(pushes, ts), f"ext timeout {send_size}")
    assert got["flush_offsets"].size > (5 if send_size == 0 else 20)


@pytest.mark.parametrize("output,group,aggs", [("all", False, None), ("current", False, [("count", None), ("avg", "v")]),
                                               ("current", None, [])])
def test_ext_timeout_no_group_by(output, group, aggs):
    """all events without group-by: every emission ends in the batch's current events, so each flush is
    one CURRENT row; `select *` (group None) re-sends a timed-out batch's events at its next emission"""
    ts, cols = tstream(40_000, 0xF2, late_ms=300)
    got = both(tspec(output=output, group=bool(group), aggs=aggs),
               with_advances(split_batches(SCH, ts, cols, [10_000, 20_000, 30_000], 3), ts), f"ext timeout {output}")
    assert got["expired"].sum() == 0


def test_ext_timeout_filter_late_and_attribute_start():
    ts, cols = tstream(60_000, 0xF3, late_ms=2_000, pause_p=1 / 1500)
    sp = tspec(filt=(">", "v", 30.0), timeout=800, T=2500, start=None)
    sp.start_attr = "st"
    both(sp, with_advances(split_batches(SCH, ts, cols, [20_000, 40_000], 5), ts, every=1), "ext timeout filter")


def test_ext_timeout_fires_then_crossing_sends_nothing():
    """a timeout sends the whole batch; the event that then crosses into the next batch finds nothing
    new (appendToOutputChunk with an empty current chunk emits nothing) — across an advance_time"""
    n = 40
    ts = 1_000_000 + np.arange(n, dtype=np.int64)
    et = 5_000 + np.arange(n, dtype=np.int64) * 10  # 100 events per 1 s batch: batch 0 = events 0..39
    et[20:] += 1_000                                  # event 20 crosses into the next batch
    cols = [np.zeros(n, np.int32), np.arange(n, dtype=np.float64), et, np.full(n, 4_321, np.int64), ts.copy()]
    pushes = [abi.HostBatch(SCH, ts[:20], [c[:20] for c in cols], 1), ("advance", int(ts[19]) + 2_000),
              abi.HostBatch(SCH, ts[20:] + 2_000, [c[20:] for c in cols], 1), ("advance", int(ts[-1]) + 9_000)]
    pushes[2].cols[4][:] = pushes[2].ts
    from siddhi_amd import runtime
    sp = tspec(group=False, aggs=[("count", None)])
    g, o = runtime.GpuQuery(sp), OracleQuery(sp)
    got, ref = run_pushes(g, pushes), run_pushes(o, pushes)
    g.close()
    o.close()
    assert_same(got, ref, label="ext timeout then crossing")
    assert got["vals"][0].tolist() == [20, 20]
    assert got["flush_clock"].tolist() == [int(ts[19]) + 2_000, int(ts[-1]) + 9_000]


def test_ext_timeout_checkpoint():
    from tests.test_gpu_snapshot import checkpointed
    ts, cols = tstream(50_000, 0xF4)
    pushes = with_advances(split_batches(SCH, ts, cols, [12_000, 25_000, 37_000], 1), ts)
    for cut in (2, 5):
        got, ref, _ = checkpointed(tspec(), pushes, cut)
        assert_same(got, ref, label=f"ext timeout ckpt {cut}")


@pytest.mark.parametrize("output,group,send_size", [("all", True, 1), ("expired", True, 7), ("all", None, 3),
                                                     ("expired", None, 1), ("expired", False, 1)])
def test_ext_timeout_expired_rows(output, group, send_size):
    """timeouts with expired output (flushToOutputChunk / appendToOutputChunk :336-438): every emission
    carries the previous emission's events as EXPIRED (stamped with lastCurrentEventTime), then RESET and
    the open batch from its first event — group-by rows merged by key, `select *` (group None) rows one
    per event; across advance_time calls and pushes"""
    ts, cols = tstream(60_000, 0xF5, late_ms=300)
    aggs = [] if group is None else None
    pushes = with_advances(split_batches(SCH, ts, cols, [1, 15_000, 15_001, 41_000], send_size), ts)
    got = both(tspec(output=output, group=bool(group), aggs=aggs), pushes, f"ext timeout {output} {group}")
    # (all events: a key in both parts shows its current row at its expired position)
    assert got["expired"].sum() > 10 or output == "all"


def test_ext_timeout_expired_rows_checkpoint():
    from tests.test_gpu_snapshot import checkpointed
    ts, cols = tstream(50_000, 0xF8)
    pushes = with_advances(split_batches(SCH, ts, cols, [12_000, 25_000, 37_000], 1), ts)
    for cut in (2, 5):
        got, ref, _ = checkpointed(tspec(output="all"), pushes, cut)
        assert_same(got, ref, label=f"ext timeout all ckpt {cut}")


# ---- the timeout under `partition with`: every partition's own lastScheduledTime; partitions due at
# the same time fire in PartitionStateHolder's HashMap order, one per due time per call (Scheduler
# .onTimeChange :71-104), the others at later calls ------------------------------------------------------
def ptstream(n, parts, seed, late_ms=0, pause_p=1 / 2000, zero_gaps=False):
    """arrival clock with pauses (timeouts fire) — with zero_gaps most sends share their clock, so many
    partitions schedule the same due time (ties); event time 1 ms per 20 events, per-partition offsets"""
    ts, cols = tstream(n, seed, pause_p=pause_p, late_ms=late_ms)
    if zero_gaps:
        rng = np.random.default_rng(seed + 3)
        gaps = (rng.random(n) < 0.02) * rng.integers(1, 4, n) + (rng.random(n) < pause_p) * rng.integers(2_000, 9_000, n)
        ts = 1_000_000 + np.cumsum(gaps).astype(np.int64)
        cols[4] = ts.copy()
    rng = np.random.default_rng(seed + 5)
    p = rng.integers(0, parts, n).astype(np.int32)
    et = cols[2] + (p.astype(np.int64) % 7) * 333
    return ts, [p, cols[0], cols[1], et, cols[3], cols[4]]


def ptspec(output="current", group_by=("p",), timeout=1500, T=1000, start=0, start_attr=None, aggs=None):
    sp = abi.QuerySpec(PSCH, "externalTimeBatch", T, group_by=list(group_by), ts_attr="et", start_time=start,
                       start_attr=start_attr, partition="p", key_capacity=4096, output=output,
                       aggs=[("count", None), ("sum", "v"), ("min", "v"), ("max", "et")] if aggs is None else aggs)
    sp.timeout = timeout
    return sp


@pytest.mark.parametrize("output", ["current", "all", "expired"])
@pytest.mark.parametrize("group_by,send_size,zero_gaps", [(("p",), 1, False), (("k",), 5, True), ((), 1, True),
                                                          (("k", "p"), 3, False)])
def test_partitioned_ext_timeout(output, group_by, send_size, zero_gaps):
    """ExternalTimeBatchWindowProcessor.process (:238-311) per partition with its timeout: a partition's
    TIMER re-sends its open batch (flushToOutputChunk, then appendToOutputChunk), crossings send the batch
    whole, expired rows are the previous emission's — ties between partitions at one due time resolved in
    HashMap order; across pushes and advance_time calls"""
    ts, cols = ptstream(60_000, 23, 0xD1, late_ms=300, zero_gaps=zero_gaps)
    pushes = split_batches(PSCH, ts, cols, [1, 14_000, 14_001, 37_000], send_size)
    got = both(ptspec(output=output, group_by=group_by), with_advances(pushes, ts), f"pext timeout {group_by} {output}")
    assert len(got["ts"]) > 100


def test_partitioned_ext_timeout_attribute_start_filter_replace():
    """start from an attribute (a first event may already be past its first batch: a reschedule with
    nothing to send), a filter, many partitions, and the replaced timestamp attribute"""
    ts, cols = ptstream(50_000, 400, 0xD2, late_ms=500, zero_gaps=True)
    cols[4] = cols[4] - 1_000 * (cols[0] % 3)  # (the start attribute: some partitions start 1-2 s early)
    sp = ptspec(output="all", group_by=("k",), timeout=700, T=900, start=None, start_attr="st",
                aggs=[("count", None), ("sum", "v"), ("max", "v")])
    sp.filter = (">", "v", 25.0)
    sp.replace_ts = True
    got = both(sp, with_advances(split_batches(PSCH, ts, cols, [20_000, 35_000], 2), ts, every=1), "pext timeout attr")
    assert len(got["rep_attr"]) == len(got["ts"])


def test_partitioned_ext_timeout_checkpoint_and_rate():
    from tests.test_gpu_snapshot import checkpointed
    ts, cols = ptstream(40_000, 31, 0xD3, zero_gaps=True)
    pushes = with_advances(split_batches(PSCH, ts, cols, [9_000, 21_000, 30_000], 1), ts)
    for cut in (2, 5):
        got, ref, _ = checkpointed(ptspec(output="all", group_by=("k",)), pushes, cut)
        assert_same(got, ref, label=f"pext timeout ckpt {cut}")
    sp = ptspec(output="current")
    sp.rate = ("last", 3)
    both(sp, pushes, "pext timeout rate")


@pytest.mark.parametrize("ptype", ["double", "float"])
def test_partitioned_ext_timeout_float_keys(ptype):
    """float / double partition keys: the timeout ties between partitions go in the HashMap order of
    Double.toString / Float.toString of the keys"""
    sch = abi.Schema.parse(f"p {ptype}, k string, v double, et long, st long, ts long")
    ts, cols = ptstream(40_000, 19, 0xD4, zero_gaps=True)
    vals = np.array([0.0, -0.0, np.nan, 1.5, -2.25, 1e300, 5e-324, 1e-5, 12345678.9, 0.1, 1 / 3, 100.0, 1e7, -7.0,
                     2.5e-3, 6.02e23, 9999999.0, 0.3, 42.0], np.float64)
    with np.errstate(over="ignore"):
        p = vals[cols[0]].astype(np.float32 if ptype == "float" else np.float64)
    cols[0] = p
    sp = abi.QuerySpec(sch, "externalTimeBatch", 1000, group_by=["p"], ts_attr="et", start_time=0, partition="p",
                       key_capacity=256, output="all", aggs=[("count", None), ("sum", "v"), ("max", "et")])
    sp.timeout = 1500
    got = both(sp, with_advances(split_batches(sch, ts, cols, [9_000, 21_000], 1), ts), f"pext timeout {ptype} keys")
    assert len(got["ts"]) > 100


@pytest.mark.parametrize("rate", [("all", 3), ("last", 2)])
def test_ext_timeout_through_rate_limiter(rate):
    """the timeouts' emissions reach the output rate limiter like any flush (device rows of several
    runs uploaded as one push's output)"""
    ts, cols = tstream(40_000, 0xF6)
    sp = tspec()
    sp.rate = rate
    both(sp, with_advances(split_batches(SCH, ts, cols, [10_000, 25_000], 1), ts), f"ext timeout rate {rate}")


# ---- replaceTimestampWithBatchEndTime (the 5th parameter; ExternalTimeBatchWindowProcessor :210-220,
# cloneAppend :446-456): every row's representative event carries its batch's end time ------------------
RAGGS = [("count", None), ("sum", "v"), ("min", "v")]


@pytest.mark.parametrize("output,group,timeout", [("current", True, 0), ("all", True, 0), ("expired", True, 0),
                                                  ("all", False, 0), ("current", True, 1500), ("all", False, 1500)])
def test_ext_replace_timestamp_with_batch_end(output, group, timeout):
    """the rows' replaced timestamp attribute (sh_query_rep_ts_attr) equals the oracle's — batch ends of
    current rows, of expired rows (the previous batch) and of timeout emissions — with late events, gaps
    of several empty buckets and pushes cut inside batches; rows otherwise unchanged"""
    if timeout:
        ts, cols = tstream(60_000, 0xF7, late_ms=500)
    else:
        ts, cols = stream(60_000, 3_000, 0xF8, late_ms=1_200)
        cols[2] = cols[2] + (np.arange(len(ts)) >= 30_000) * 5_000
    sp = spec(T=800 if timeout else 300, start=0 if timeout else None, keys=3_000, output=output, group=group, aggs=RAGGS)
    sp.replace_ts = True
    if timeout:
        sp.timeout = timeout
    pushes = split_batches(SCH, ts, cols, [1, 15_000, 15_001, 41_000], 1 if timeout else 3)
    if timeout:
        pushes = with_advances(pushes, ts)
    got = both(sp, pushes, f"ext replace {output} {group} {timeout}")
    assert np.all(got["rep_attr"] % 800 == 0) or not timeout  # (start 0: every batch end is a multiple of T)


def test_ext_replace_timestamp_device_output_and_checkpoint():
    """device output (sh_push_device: the representative events are read back for the attribute) and a
    checkpoint taken between batches that restores into a fresh query"""
    import torch
    from siddhi_amd import runtime
    from tests.test_gpu_snapshot import checkpointed
    ts, cols = stream(40_000, 500, 0xF9, late_ms=300)
    sp = spec(T=600, keys=500, output="all", aggs=RAGGS)
    sp.replace_ts = True
    got, ref, _ = checkpointed(sp, split_batches(SCH, ts, cols, [9_000, 22_000], 1), 1)
    assert_same(got, ref, label="ext replace ckpt")
    g, o = runtime.GpuQuery(sp), OracleQuery(sp)
    dev = torch.device("cuda", 0)
    t = torch.from_numpy(ts).to(dev)
    dc = [torch.from_numpy(np.ascontiguousarray(c)).to(dev) for c in cols]
    torch.cuda.synchronize()
    out = g.push_device(len(ts), t.data_ptr(), [c.data_ptr() for c in dc], 1)
    a = runtime.device_out_arrays(out)
    b = abi.out_arrays(o.push_raw(abi.HostBatch(SCH, ts, cols, 1)))
    assert np.array_equal(a["rep"], b["rep"]) and np.array_equal(g.rep_ts_attr(), o.rep_ts_attr())
    g.close()
    o.close()


def test_ext_replace_timestamp_refusals():
    from siddhi_amd import runtime
    sp = spec(T=600, keys=64, aggs=[("count", None), ("max", "et")])
    sp.replace_ts = True
    with pytest.raises(runtime.SiddhiError, match="aggregator over the timestamp"):
        runtime.GpuQuery(sp)
    sp = abi.QuerySpec(PSCH, "externalTimeBatch", 700, ts_attr="et", partition="p", key_capacity=64,
                       aggs=[("count", None)])
    sp.replace_ts = True
    sp.rate = ("all", 5)
    with pytest.raises(runtime.SiddhiError, match="rate limiter"):
        runtime.GpuQuery(sp)


@pytest.mark.parametrize("output", ["current", "all", "expired"])
@pytest.mark.parametrize("group_by,start,start_attr,late", [(["p"], None, None, 0), (["k"], 1_000, None, 800),
                                                            ([], None, "st", 300)])
def test_partitioned_ext_replace_timestamp(output, group_by, start, start_attr, late):
    """`partition with` around externalTimeBatch(et, T, start, 0, true): every partition's cloneAppend
    writes its own batch's endTime into the event (:446-456), so each row's replaced attribute is the
    end of the batch holding its representative event — current rows their batch, expired rows the
    previous one — carried across pushes with the partitions' open batches"""
    ts, cols = pstream(50_000, 31, 0xEB, late_ms=late)
    sp = abi.QuerySpec(PSCH, "externalTimeBatch", 600, group_by=group_by, ts_attr="et", start_time=start,
                       start_attr=start_attr, partition="p", key_capacity=4096, output=output,
                       aggs=[("count", None), ("sum", "v"), ("min", "v")])
    sp.replace_ts = True
    got = both(sp, split_batches(PSCH, ts, cols, [1, 17_000, 17_001, 36_000], 3), f"pext replace {group_by} {output}")
    assert len(got["rep_attr"]) == len(got["ts"]) > 0


def test_partitioned_ext_replace_timestamp_checkpoint():
    from tests.test_gpu_snapshot import checkpointed
    ts, cols = pstream(40_000, 19, 0xEC, late_ms=200)
    sp = abi.QuerySpec(PSCH, "externalTimeBatch", 500, group_by=["k"], ts_attr="et", partition="p", key_capacity=4096,
                       output="all", aggs=[("count", None), ("sum", "v")])
    sp.replace_ts = True
    got, ref, _ = checkpointed(sp, split_batches(PSCH, ts, cols, [15_000, 30_000], 1), 1)
    assert_same(got, ref, label="pext replace ckpt")


@pytest.mark.parametrize("rate", [("all", 7919), ("last", 4001), ("first", 3001)])
def test_ext_replace_timestamp_through_rate_limiter(rate):
    """rows an output rate limiter holds across many later batches still show their own batch's end time
    (the recorded batch starts are kept back to the oldest row the limiter carries)"""
    ts, cols = stream(60_000, 3_000, 0xFA, late_ms=200)
    sp = spec(T=40, keys=3_000, output="all", aggs=RAGGS)
    sp.replace_ts = True
    sp.rate = rate
    got = both(sp, split_batches(SCH, ts, cols, [1, 7_000, 7_001, 30_000, 45_000], 1), f"ext replace rate {rate}")
    assert len(got["rep_attr"]) > 0
