"""GPU parity of the sharded ingest: G shards of a timeBatch group-by query — each
holding a slice of every global push, re-keying its events to the owner GPU — must together emit
exactly what the single-stream oracle emits for the whole stream: same flushes, flush clocks, rows,
row order (merged by the global first-occurrence index), timestamps and bit-identical values.

The G shards run in one process on one device and exchange through device copies (LocalShards);
the multi-process transport (torch.distributed all-to-all) carries the same bytes."""
import numpy as np
import pytest

from oracle.oracle import OracleQuery
from siddhi_amd import abi, synth
from tests.parity import assert_same, run_pushes

pytestmark = pytest.mark.gpu

SCHEMA = abi.Schema.parse("k int, v double, ts long")


def spec(keys, filt=None, start=None, aggs=None, group_by=("k",), schema=SCHEMA):
    return abi.QuerySpec(schema, "timeBatch", 1000, group_by=list(group_by),
                         aggs=aggs or [("count", None), ("min", "v"), ("max", "v"), ("avg", "v")],
                         filter=filt, start_time=start, key_capacity=keys)


def run_sharded(sp, world, pushes, send_size, cut_fracs, advance=None):
    """pushes: list of (ts, cols) numpy global pushes; each is cut into `world` send-aligned slices. A spec
    with an output rate runs its limiter over the merged output (MergedRateLimiter)."""
    import torch
    from siddhi_amd.shard import LocalShards, MergedRateLimiter, merge_owner_outputs, merge_sends
    dev = torch.device("cuda", 0)
    ls = LocalShards(sp, world)
    rl = MergedRateLimiter(sp) if sp.rate else None
    parts = []
    for pi, (ts, cols) in enumerate(pushes):
        n = len(ts)
        units = (n + send_size - 1) // send_size
        cuts = sorted(min(n, int(units * f) * send_size) for f in cut_fracs[pi % len(cut_fracs)])
        edges = [0] + cuts + [n]
        slices = []
        for g in range(world):
            a, b = edges[g], edges[g + 1]
            slices.append((torch.from_numpy(np.ascontiguousarray(ts[a:b])).to(dev),
                           [torch.from_numpy(np.ascontiguousarray(c[a:b])).to(dev) for c in cols]))
        outs = ls.push(slices, send_size, dev)
        parts.append(merge_owner_outputs(outs, ls.last_bounds, merge_sends(sp, ls.last_sends)))
    if advance is not None:
        parts.append(merge_owner_outputs(ls.advance_time(advance)))
    ls.close()
    if rl is not None:
        parts = [rl.apply(p) for p in parts]
        rl.close()
    return abi.concat_arrays(parts)


def run_oracle(sp, pushes, send_size, advance=None):
    o = OracleQuery(sp)
    bl = [abi.HostBatch(sp.schema, ts, cols, send_size) for ts, cols in pushes]
    if advance is not None:
        bl.append(("advance", advance))
    out = run_pushes(o, bl)
    o.close()
    return out


def stream_pushes(n, sizes, seed, keys, per_ms, quantized=False):
    ts, cols = synth.keyed_stream(0, n, seed, keys, per_ms, quantized)
    out, a = [], 0
    for s in sizes:
        out.append((ts[a:a + s], [c[a:a + s] for c in cols]))
        a += s
    return out


@pytest.mark.parametrize("world", [2, 3, 8])
def test_sharded_c2_matches_single_stream(world):
    sp = spec(20_000)
    pushes = stream_pushes(600_000, [150_000, 1, 249_999, 200_000], 0xC2, 20_000, 100)
    fr = [[(g + 1) / world for g in range(world - 1)], [0.0] * (world - 1), [0.1 * (g + 1) for g in range(world - 1)]]
    adv = int(pushes[-1][0][-1]) + 5000
    got = run_sharded(sp, world, pushes, 1, fr, advance=adv)
    ref = run_oracle(sp, pushes, 1, advance=adv)
    assert ref["flush_offsets"].size > 5
    assert_same(got, ref, label=f"sharded x{world}")


def test_compact_records_and_wide_fallback():
    """C2's records carry ts as a 32-bit offset from the push's minimum timestamp: 20 bytes per event
    (key, slice position, ts offset, value) instead of 24; a push spanning 2^32 ms or more falls back
    to the 64-bit ts. Both forms consume to the single-stream output."""
    import torch
    from siddhi_amd.shard import LocalShards
    sp = spec(2_000)
    ts, cols = synth.keyed_stream(0, 200_000, 0xB1, 2_000, 100)
    ts = ts.copy()
    ts[150_000:] += 5_000_000_000  # the second push spans more than 2^32 ms
    pushes = [(ts[:100_000], [c[:100_000] for c in cols]), (ts[100_000:], [c[100_000:] for c in cols])]
    adv = int(ts[-1]) + 5_000
    got = run_sharded(sp, 3, pushes, 1, [[0.3, 0.6]], advance=adv)
    ref = run_oracle(sp, pushes, 1, advance=adv)
    assert_same(got, ref, label="compact / wide records")
    dev = torch.device("cuda", 0)
    ls = LocalShards(sp, 2)
    per = []
    for pts, pcols in pushes:
        sl = [(torch.from_numpy(np.ascontiguousarray(x[a:b])).to(dev),
               [torch.from_numpy(np.ascontiguousarray(c[a:b])).to(dev) for c in pcols])
              for a, b in ((0, 50_000), (50_000, len(pts))) for x in [pts]]
        ls.push(sl, 1, dev)
        per.append(ls.last_send_bytes / len(pts))
    ls.close()
    assert per == [20.0, 24.0], per


def test_sharded_filter_send_chunks_start_time():
    sp = spec(5_000, filt=(">", "v", 150.0), start=137)
    pushes = stream_pushes(300_000, [100_000, 200_000], 0xC5, 5_000, 50)
    fr = [[0.25, 0.5, 0.75], [0.05, 0.06, 0.9]]
    got = run_sharded(sp, 4, pushes, 100, fr, advance=int(pushes[-1][0][-1]) + 10_000)
    ref = run_oracle(sp, pushes, 100, advance=int(pushes[-1][0][-1]) + 10_000)
    assert_same(got, ref, label="sharded filter/start")


def test_sharded_two_keys_long_sums_and_quiet_owner():
    sch = abi.Schema.parse("a int, b int, x long, v double, ts long")
    ts, cols = synth.keyed_stream(0, 120_000, 0xA7, 3, 20)
    rng = np.random.default_rng(7)
    a = cols[0]
    b = rng.integers(0, 2, size=len(ts)).astype(np.int32)
    x = rng.integers(-1000, 1000, size=len(ts)).astype(np.int64)
    full = [a, b, x, cols[1], cols[2]]
    sp = spec(64, aggs=[("sum", "x"), ("max", "x"), ("sum", "v"), ("count", None)], group_by=("a", "b"), schema=sch)
    pushes = [(ts[:60_000], [c[:60_000] for c in full]), (ts[60_000:], [c[60_000:] for c in full])]
    # 6 keys over 5 owners: some owners receive nothing and only close windows on the global clock
    got = run_sharded(sp, 5, pushes, 1, [[0.2, 0.4, 0.6, 0.8]], advance=int(ts[-1]) + 3000)
    ref = run_oracle(sp, pushes, 1, advance=int(ts[-1]) + 3000)
    assert_same(got, ref, label="sharded two keys")


def test_sharded_dictionary_keys_round_robin_owners():
    """string (dictionary id) keys: owner = id % G and each owner keeps its ids dense as id / G."""
    sch = abi.Schema.parse("k string, v double, ts long")
    sp = spec(30_000, schema=sch)
    pushes = stream_pushes(400_000, [180_000, 220_000], 0xD1, 30_000, 80)
    adv = int(pushes[-1][0][-1]) + 4000
    got = run_sharded(sp, 4, pushes, 1, [[0.3, 0.5, 0.9]], advance=adv)
    ref = run_oracle(sp, pushes, 1, advance=adv)
    assert_same(got, ref, label="sharded dict x4")


@pytest.mark.parametrize("world", [3, 8])
def test_sharded_partition_with_zipf_keys(world):
    """C5: `partition with (k of S) begin from S#window.timeBatch(1 sec) select k, sum(v), count()
    group by k` — R12: only the partition of the globally first passing event ever flushes; here the
    first slices hold no passing event, so a later rank's slice decides it."""
    sch = abi.Schema.parse("k int, v long, ts long")
    n = 60_000  # the oracle's scheduler scans every partition per send (Scheduler.java:75-98)
    ts = synth.T0 + np.arange(n, dtype=np.int64) // 10
    ts[30_000:] += 7_500  # an idle gap of several windows
    k = synth.zipf_keys(0, n, 0xC5, 1_000)
    v = (np.arange(n, dtype=np.int64) * 7919) % 1000
    sp = abi.QuerySpec(sch, "timeBatch", 1000, group_by=["k"], aggs=[("sum", "v"), ("count", None)],
                       filter=(">", "ts", int(ts[int(0.5 * n / world)])), partition="k", key_capacity=1_000)
    pushes = [(ts[:20_000], [k[:20_000], v[:20_000], ts[:20_000]]),
              (ts[20_000:], [k[20_000:], v[20_000:], ts[20_000:]])]
    adv = int(ts[-1]) + 5000
    got = run_sharded(sp, world, pushes, 1, [[(g + 1) / world for g in range(world - 1)]], advance=adv)
    ref = run_oracle(sp, pushes, 1, advance=adv)
    assert ref["flush_offsets"].size > 5
    assert_same(got, ref, label=f"sharded partition x{world}")


# ---- C1 over G GPUs: lengthBatch (the batch index is global: passing events of the slices before) ----
C1_SCHEMA = abi.Schema.parse("symbol string, price double, volume long, ts long")


def c1_pushes(n, sizes, quantized=False):
    ts, cols = synth.c1_stock(0, n, quantized=quantized)
    out, a = [], 0
    for s in sizes:
        out.append((ts[a:a + s], [c[a:a + s] for c in cols]))
        a += s
    return out


@pytest.mark.parametrize("world,send_size", [(2, 1), (3, 1000), (8, 1)])
def test_sharded_c1_lengthbatch_matches_single_stream(world, send_size):
    """`from StockStream[price>100]#window.lengthBatch(L) select symbol, sum(volume), avg(price) group
    by symbol`: batch b = events whose global filtered index is in [bL, (b+1)L), flushed in the send
    of its L-th event; owners flush batch b at that send's clock."""
    sp = abi.QuerySpec(C1_SCHEMA, "lengthBatch", 3000, group_by=["symbol"], aggs=[("sum", "volume"), ("avg", "price")],
                       filter=(">", "price", 100), key_capacity=1000)
    pushes = c1_pushes(200_000, [70_000, 1000, 129_000])
    fr = [[(g + 1) / world for g in range(world - 1)], [0.0] * (world - 1), [0.05 * (g + 1) for g in range(world - 1)]]
    got = run_sharded(sp, world, pushes, send_size, fr)
    ref = run_oracle(sp, pushes, send_size)
    assert ref["flush_offsets"].size > 20
    assert_same(got, ref, label=f"sharded C1 x{world}")


def test_sharded_lengthbatch_batches_ending_at_push_and_slice_ends():
    """Batches that complete on the last event of a slice or of a push, several batches in one send
    (send_size > L), and a quiet owner: flush clocks and row order still match the single stream."""
    sp = abi.QuerySpec(C1_SCHEMA, "lengthBatch", 500, group_by=["symbol"],
                       aggs=[("sum", "volume"), ("count", None), ("max", "price")], key_capacity=1000)
    # no filter: push sizes that are multiples of L end exactly on a batch
    pushes = c1_pushes(30_000, [5_000, 7_250, 17_750])
    fr = [[0.5, 0.5, 0.75]]
    got = run_sharded(sp, 4, pushes, 2_000, fr)
    ref = run_oracle(sp, pushes, 2_000)
    assert_same(got, ref, label="sharded lengthBatch edges")
    got1 = run_sharded(sp, 4, pushes, 1, [[0.1, 0.2, 0.3]])
    ref1 = run_oracle(sp, pushes, 1)
    assert_same(got1, ref1, label="sharded lengthBatch edges per-event")


# ---- C3 over G GPUs: sliding time(T) (the clock and PM of every event are global: the source slice
# computes them from the all-gathered summaries; the owner replays its keys' windows with them) ----
def c3_spec(keys, T, filt=None, aggs=None, schema=SCHEMA, group_by=("k",)):
    return abi.QuerySpec(schema, "time", T, group_by=list(group_by),
                         aggs=aggs or [("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], filter=filt,
                         key_capacity=keys)


@pytest.mark.parametrize("world,send_size", [(2, 1), (3, 250), (8, 1)])
def test_sharded_c3_sliding_matches_single_stream(world, send_size):
    sp = c3_spec(2000, 1000)
    pushes = stream_pushes(200_000, [77_777, 1, 122_222], 0xC3, 2000, 20)
    fr = [[(g + 1) / world for g in range(world - 1)], [0.0] * (world - 1), [0.1 * (g + 1) for g in range(world - 1)]]
    got = run_sharded(sp, world, pushes, send_size, fr, advance=int(pushes[-1][0][-1]) + 5000)
    ref = run_oracle(sp, pushes, send_size, advance=int(pushes[-1][0][-1]) + 5000)
    assert ref["flush_offsets"].size > 500
    assert_same(got, ref, label=f"sharded C3 x{world}")


def test_sharded_sliding_filter_nonmonotone_ts_dictionary_keys():
    """Out-of-order timestamps (PM, not ts, decides expiry), a filter, dictionary-id keys (owner =
    id % G) and the deque quirk on few distinct values, with a quiet owner."""
    rng = np.random.default_rng(11)
    n = 60_000
    ts = (np.arange(n) // 4 + rng.integers(-50, 50, n)).astype(np.int64) + 10_000
    k = rng.integers(0, 7, n).astype(np.int32)
    v = rng.integers(0, 6, n).astype(np.float64)
    x = rng.integers(-10**9, 10**9, n).astype(np.int64)
    sch = abi.Schema.parse("k string, v double, x long, ts long")
    sp = c3_spec(16, 300, filt=(">", "x", -5 * 10**8), schema=sch,
                 aggs=[("min", "v"), ("max", "v"), ("sum", "x"), ("count", None), ("avg", "v")])
    full = [k, v, x, ts.copy()]
    pushes = [(ts[:25_000], [c[:25_000] for c in full]), (ts[25_000:], [c[25_000:] for c in full])]
    got = run_sharded(sp, 5, pushes, 7, [[0.2, 0.4, 0.6, 0.8], [0.0, 0.5, 0.5, 0.99]])
    ref = run_oracle(sp, pushes, 7)
    assert_same(got, ref, label="sharded sliding nonmono")


# ---- `insert expired events` / `insert all events` over G GPUs: an owner's flush closing global window
# W carries its keys' expired rows of W-1 (order: their first occurrence in W-1) and its current rows
# of W; the merge matches owner flushes by (clock, window) (sh_shard_flush_windows) ----------------------
@pytest.mark.parametrize("output,world", [("all", 2), ("expired", 3), ("all", 8)])
def test_sharded_timebatch_expired_and_all_events(output, world):
    sp = abi.QuerySpec(SCHEMA, "timeBatch", 1000, group_by=["k"],
                       aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=3_000,
                       output=output)
    pushes = stream_pushes(240_000, [90_000, 1, 149_999], 0xE1, 3_000, 40)
    # an idle stretch: windows that close empty (their close carries only the expired rows)
    pushes[2] = (pushes[2][0] + (np.arange(len(pushes[2][0])) >= 70_000) * 4_500, pushes[2][1])
    pushes[2][1][2] = pushes[2][0].copy()
    fr = [[(g + 1) / world for g in range(world - 1)], [0.0] * (world - 1), [0.07 * (g + 1) for g in range(world - 1)]]
    adv = int(pushes[-1][0][-1]) + 5_000
    got = run_sharded(sp, world, pushes, 1, fr, advance=adv)
    ref = run_oracle(sp, pushes, 1, advance=adv)
    assert ref["expired"].sum() > 1_000
    assert_same(got, ref, label=f"sharded {output} x{world}")


@pytest.mark.parametrize("output", ["all", "expired"])
def test_sharded_lengthbatch_expired_and_all_events(output):
    sp = abi.QuerySpec(C1_SCHEMA, "lengthBatch", 2_000, group_by=["symbol"], aggs=[("sum", "volume"), ("avg", "price")],
                       filter=(">", "price", 100), key_capacity=1000, output=output)
    pushes = c1_pushes(120_000, [50_000, 1000, 69_000])
    got = run_sharded(sp, 4, pushes, 10, [[0.25, 0.5, 0.75], [0.0, 0.0, 0.5], [0.1, 0.2, 0.3]])
    ref = run_oracle(sp, pushes, 10)
    assert ref["expired"].sum() > 100
    assert_same(got, ref, label=f"sharded lengthBatch {output}")


# ---- stream.current.event over G GPUs: a row per passing event with its key's running values since the
# batch reset (TimeBatchWindowProcessor :262-340 RESET mode, LengthBatchWindowProcessor
# .processStreamCurrentEvents :245-274); the owner folds its keys' records in global order and stamps each
# row with its send's global clock (carried in the record), rows merge by global stream index ----------
@pytest.mark.parametrize("window,param,world,send_size", [("timeBatch", 1000, 2, 1), ("timeBatch", 700, 3, 50),
                                                          ("lengthBatch", 97, 4, 1), ("lengthBatch", 500, 3, 20),
                                                          ("timeBatch", 300, 8, 1)])
def test_sharded_stream_current(window, param, world, send_size):
    sp = abi.QuerySpec(SCHEMA, window, param, group_by=["k"], stream_current=True, key_capacity=3_000,
                       aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], filter=(">", "v", 20.0))
    pushes = stream_pushes(150_000, [60_000, 1, 89_999], 0xC7, 3_000, 40)
    # an idle stretch of several periods: batches reset with no event
    pushes[2] = (pushes[2][0] + (np.arange(len(pushes[2][0])) >= 40_000) * 3_500, pushes[2][1])
    pushes[2][1][2] = pushes[2][0].copy()
    fr = [[(g + 1) / world for g in range(world - 1)], [0.0] * (world - 1), [0.07 * (g + 1) for g in range(world - 1)]]
    adv = int(pushes[-1][0][-1]) + 5_000
    got = run_sharded(sp, world, pushes, send_size, fr, advance=adv)
    ref = run_oracle(sp, pushes, send_size, advance=adv)
    assert ref["ts"].size > 100_000
    assert_same(got, ref, label=f"sharded stream.current {window} x{world} send {send_size}")


def test_sharded_stream_current_two_keys():
    sch = abi.Schema.parse("a int, b int, x long, v double, ts long")
    ts, cols = synth.keyed_stream(0, 80_000, 0xA9, 5, 20)
    rng = np.random.default_rng(9)
    full = [cols[0], rng.integers(0, 3, len(ts)).astype(np.int32), rng.integers(-1000, 1000, len(ts)).astype(np.int64),
            cols[1], cols[2]]
    sp = abi.QuerySpec(sch, "timeBatch", 500, group_by=["a", "b"], stream_current=True, key_capacity=64,
                       aggs=[("sum", "x"), ("max", "x"), ("sum", "v"), ("count", None)])
    pushes = [(ts[:30_000], [c[:30_000] for c in full]), (ts[30_000:], [c[30_000:] for c in full])]
    got = run_sharded(sp, 5, pushes, 3, [[0.2, 0.4, 0.6, 0.8]], advance=int(ts[-1]) + 3000)
    ref = run_oracle(sp, pushes, 3, advance=int(ts[-1]) + 3000)
    assert_same(got, ref, label="sharded stream.current two keys")


# ---- output rate limiting of a sharded query: the limiter sits after the selector
# (OutputRateLimiter.process), so it runs over the merged single-stream output, call by call ----------
@pytest.mark.parametrize("rate,window,param,send_size,grouped", [
    (("first", 7), "timeBatch", 25, 1, False), (("last", 5), "timeBatch", 35, 3, False),
    (("all", 4), "lengthBatch", 40, 1, False), (("first", 3), "timeBatch", 600, 1, True),
    (("last", 4), "lengthBatch", 300, 2, True), (("first_time", 70), "timeBatch", 20, 1, False),
    (("first_time", 900), "timeBatch", 500, 1, True), (("last", 6), "time", 400, 1, True)])
def test_sharded_output_rate(rate, window, param, send_size, grouped):
    sp = abi.QuerySpec(SCHEMA, window, param, group_by=["k"] if grouped else [], key_capacity=2_000, rate=rate,
                       aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")])
    pushes = stream_pushes(90_000, [30_000, 1, 59_999], 0xB7, 2_000, 30)
    fr = [[0.3, 0.6], [0.0, 0.0], [0.2, 0.9]]
    adv = int(pushes[-1][0][-1]) + 4_000
    got = run_sharded(sp, 3, pushes, send_size, fr, advance=adv)
    ref = run_oracle(sp, pushes, send_size, advance=adv)
    assert ref["ts"].size > 10
    assert_same(got, ref, label=f"sharded rate {rate} {window} grouped={grouped}")


# ---- group keys the owners intern (three columns, a long beside another): owners by a prefix of the key
# (all of a key's events share it), the other group-by columns travel raw, each owner interns its keys
WSCH = abi.Schema.parse("a int, s string, l long, v double, ts long")


def wide_pushes(n, sizes, seed):
    rng = np.random.default_rng(seed)
    ts = (synth.T0 + np.arange(n, dtype=np.int64) // 30).astype(np.int64)
    a = rng.integers(-4, 5, n).astype(np.int32)
    s = rng.integers(0, 40, n).astype(np.int32)
    l = (rng.integers(0, 7, n) * 10_000_000_019 - 30_000_000_000).astype(np.int64)
    v = rng.integers(-500, 500, n).astype(np.float64) / 4
    cols = [a, s, l, v, ts.copy()]
    out, o = [], 0
    for z in sizes:
        out.append((ts[o:o + z], [c[o:o + z] for c in cols]))
        o += z
    return out


@pytest.mark.parametrize("window,param,group,world,send_size,sc", [
    ("timeBatch", 700, ["a", "s", "l"], 3, 1, False), ("timeBatch", 400, ["l", "a"], 2, 5, False),
    ("lengthBatch", 900, ["s", "l", "a"], 4, 1, False), ("lengthBatch", 333, ["a", "l"], 3, 2, False),
    ("timeBatch", 500, ["s", "a", "l"], 3, 1, True)])
def test_sharded_wide_group_keys(window, param, group, world, send_size, sc):
    sp = abi.QuerySpec(WSCH, window, param, group_by=group, stream_current=sc, key_capacity=4_096,
                       aggs=[("count", None), ("sum", "v"), ("min", "v"), ("max", "l")], filter=(">", "v", -100.0))
    pushes = wide_pushes(60_000, [20_000, 1, 39_999], 0xA1)
    fr = [[(g + 1) / world for g in range(world - 1)], [0.0] * (world - 1), [0.1 * (g + 1) for g in range(world - 1)]]
    adv = int(pushes[-1][0][-1]) + 3_000
    got = run_sharded(sp, world, pushes, send_size, fr, advance=adv)
    ref = run_oracle(sp, pushes, send_size, advance=adv)
    assert ref["keys"].shape[0] == len(group) and ref["ts"].size > 100
    assert_same(got, ref, label=f"sharded wide {window} {group} x{world} sc={sc}")


def test_sharded_wide_group_keys_refusals():
    from siddhi_amd.runtime import SiddhiError
    from siddhi_amd.shard import ShardedQuery
    for sp in (abi.QuerySpec(WSCH, "time", 100, group_by=["a", "s", "l"], aggs=[("count", None)]),
               abi.QuerySpec(WSCH, "timeBatch", 100, group_by=["a", "s", "l"], aggs=[("count", None)], output="all")):
        with pytest.raises(SiddhiError, match="wide group keys"):
            ShardedQuery(sp, 0, 2)


def test_sharded_wide_group_keys_float_and_checkpoint():
    """a float key column in the owner prefix (its 64-bit wire form) and a 2-part level over a float, then a
    checkpoint of the owners' interned keys between pushes"""
    from tests.test_gpu_shard_snapshot import run_sharded_restored
    sch = abi.Schema.parse("f float, a int, l long, v double, ts long")
    rng = np.random.default_rng(5)
    n = 40_000
    ts = (synth.T0 + np.arange(n, dtype=np.int64) // 20).astype(np.int64)
    f = np.array([0.5, -1.25, np.nan, 3.0, -0.0, 0.0], np.float32)[rng.integers(0, 6, n)]
    cols = [f, rng.integers(-3, 4, n).astype(np.int32), (rng.integers(0, 5, n) * 7_000_000_001).astype(np.int64),
            rng.integers(-99, 99, n).astype(np.float64) / 8, ts.copy()]
    pushes = [(ts[a:b], [c[a:b] for c in cols]) for a, b in ((0, 15_000), (15_000, 27_000), (27_000, n))]
    for group in (["f", "a", "l"], ["a", "f", "l"]):
        sp = abi.QuerySpec(sch, "timeBatch", 300, group_by=group, key_capacity=1_024,
                           aggs=[("count", None), ("sum", "v"), ("max", "l")])
        adv = int(ts[-1]) + 2_000
        ref = run_oracle(sp, pushes, 1, advance=adv)
        assert_same(run_sharded(sp, 3, pushes, 1, [[0.4, 0.7]], advance=adv), ref, label=f"sharded wide float {group}")
        assert_same(run_sharded_restored(sp, 2, pushes, 1, 2, advance=adv), ref, label=f"sharded wide ckpt {group}")
