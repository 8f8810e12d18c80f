"""GPU parity of `output [all|first|last] every N events` (sh_rate.cpp / sh_rate_kernels.hip) against
the oracle's restatement of the reference's event rate limiters (core/query/output/ratelimit/event/
AllPerEvent, FirstPerEvent, LastPerEvent, FirstGroupByPerEvent, LastGroupByPerEventOutputRateLimiter).
The oracle's limiters are pinned by EventOutputRateLimitTestCase (tests/golden, rate1..rate18); the
windowed ones (rate12..16) also run on the GPU through test_gpu_parity.py, and the no-window ones run
here as `#window.lengthBatch(1)` (one event per send: every send is one chunk either way)."""

import numpy as np
import pytest

from oracle.oracle import OracleQuery
from siddhi_amd import abi
from tests import kat_runner
from tests.parity import assert_same, run_pushes, split_batches
from tests.test_gpu_parity import both

pytestmark = pytest.mark.gpu

SCHEMA = abi.Schema.parse("k int, v double, x long, ts long")


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def stream(n, keys, seed, step=40):
    rng = np.random.default_rng(seed)
    ts = np.cumsum(rng.integers(0, step, n)).astype(np.int64) + 5_000
    k = rng.integers(0, keys, n).astype(np.int32)
    v = rng.integers(-4000, 4000, n).astype(np.float64) / 16.0
    x = rng.integers(-10**6, 10**6, n).astype(np.int64)
    return ts, [k, v, x, ts.copy()]


NOWIN_RATE_KATS = [c for c in kat_runner.load_cases()
                   if c.get("kind") != "aggregation" and c["query"].get("rate") and c["query"].get("window") is None]


@pytest.mark.parametrize("case", NOWIN_RATE_KATS, ids=[c["name"] for c in NOWIN_RATE_KATS])
def test_reference_rate_kat_on_gpu(rt, case):
    q = case["query"]
    aggs = [["count", None]] if q.get("group_by") else []
    wrapped = dict(case, query=dict(q, window="lengthBatch", param=1, aggs=aggs))
    schema, _, dic, flushes = kat_runner.run_query(wrapped, rt.GpuQuery)
    kat_runner.check_query(case, flushes, schema, dic)
    _, _, _, oflushes = kat_runner.run_query(wrapped, OracleQuery)
    assert [(f.clock, f.rows) for f in flushes] == [(f.clock, f.rows) for f in oflushes]


AGGS = [("count", None), ("sum", "v"), ("max", "x")]
KINDS = [("all", 1), ("all", 7), ("first", 1), ("first", 3), ("last", 1), ("last", 4), ("first", 50), ("last", 33),
         ("first_time", 0), ("first_time", 700)]


@pytest.mark.parametrize("kind,n", KINDS)
@pytest.mark.parametrize("group_by", [True, False])
def test_lengthbatch_rate(rt, kind, n, group_by):
    ts, cols = stream(30_000, 40, 3)
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", 97, group_by=["k"] if group_by else (), aggs=AGGS,
                         key_capacity=64, rate=(kind, n))
    out = both(rt, spec, split_batches(SCHEMA, ts, cols, [1, 500, 12_345, 12_346], 3),
               label=f"lengthBatch {kind} {n} gb={group_by}")
    assert out["ts"].size > 0


@pytest.mark.parametrize("kind,n", [("all", 5), ("first", 4), ("last", 6)])
@pytest.mark.parametrize("output", ["all", "expired"])
def test_timebatch_expired_rate(rt, kind, n, output):
    ts, cols = stream(40_000, 200, 5)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 600, group_by=["k"], aggs=AGGS, filter=(">", "v", -100.0),
                         output=output, key_capacity=256, rate=(kind, n))
    pushes = split_batches(SCHEMA, ts, cols, [2_000, 20_000, 20_001], 7)
    pushes += [("advance", int(ts[-1]) + 300), ("advance", int(ts[-1]) + 5_000)]
    out = both(rt, spec, pushes, label=f"timeBatch {output} {kind} {n}")
    assert out["expired"].sum() > 0


@pytest.mark.parametrize("kind,n", [("all", 3), ("first", 5), ("last", 2), ("first", 1)])
@pytest.mark.parametrize("group_by", [True, False])
def test_sliding_time_rate(rt, kind, n, group_by):
    ts, cols = stream(20_000, 30, 11)
    spec = abi.QuerySpec(SCHEMA, "time", 500, group_by=["k"] if group_by else (), aggs=[("sum", "v"), ("min", "x")],
                         key_capacity=64, rate=(kind, n))
    both(rt, spec, split_batches(SCHEMA, ts, cols, [1, 9_999], 4), label=f"time {kind} {n} gb={group_by}")


@pytest.mark.parametrize("kind,n", [("all", 4), ("last", 3)])
def test_pass_through_rate(rt, kind, n):
    ts, cols = stream(10_000, 10, 21)
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", 13, filter=("<", "x", 500_000), rate=(kind, n))
    both(rt, spec, split_batches(SCHEMA, ts, cols, [5, 4_000], 2), label=f"pass-through {kind} {n}")


def test_first_group_by_table_growth(rt):
    """FirstGroupBy's key -> count table grows (rehash) while counts carry across pushes."""
    ts, cols = stream(120_000, 50_000, 23, step=3)
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", 1000, group_by=["k"], aggs=[("count", None)],
                         key_capacity=65_536, rate=("first", 3))
    both(rt, spec, split_batches(SCHEMA, ts, cols, [100, 1_000, 30_000, 60_000], 0), label="first gb growth")


def _dev_arrays(out_ptr):
    from siddhi_amd import runtime
    return runtime.device_out_arrays(out_ptr)


@pytest.mark.parametrize("window,param", [("lengthBatch", 50), ("timeBatch", 300)])
def test_device_output_rate(rt, window, param):
    """sh_push_device: the limiter's rows stay in HBM, flush metadata on the host."""
    import torch
    ts, cols = stream(20_000, 25, 31)
    spec = abi.QuerySpec(SCHEMA, window, param, group_by=["k"], aggs=AGGS, key_capacity=32, rate=("last", 5))
    g = rt.GpuQuery(spec)
    parts = []
    for b in split_batches(SCHEMA, ts, cols, [7_000, 7_001], 0):
        keep = [torch.from_numpy(np.ascontiguousarray(a)).cuda() for a in [b.ts] + b.cols]
        torch.cuda.synchronize()
        parts.append(_dev_arrays(g.push_device(len(b.ts), keep[0].data_ptr(), [t.data_ptr() for t in keep[1:]])))
    g.close()
    o = OracleQuery(spec)
    ora = run_pushes(o, split_batches(SCHEMA, ts, cols, [7_000, 7_001], 0))
    o.close()
    assert_same(abi.concat_arrays(parts), ora, label=f"device {window}")


@pytest.mark.parametrize("kind,n", [("all", 3), ("first", 2), ("last", 4)])
def test_partitioned_timebatch_rate(rt, kind, n):
    """One limiter per partition instance; only p0 ever flushes (R12), so the GPU's one limiter is p0's."""
    sch = abi.Schema.parse("k int, p int, v double, ts long")
    rng = np.random.default_rng(41)
    m = 30_000
    ts = (np.arange(m) // 20 + 10_000).astype(np.int64)
    cols = [rng.integers(0, 50, m).astype(np.int32), rng.integers(0, 3, m).astype(np.int32),
            rng.integers(-99, 99, m).astype(np.float64) / 4, ts.copy()]
    spec = abi.QuerySpec(sch, "timeBatch", 400, group_by=["k"], aggs=[("count", None), ("sum", "v")], partition="p",
                         key_capacity=64, rate=(kind, n))
    pushes = split_batches(sch, ts, cols, [7_000, 20_000], 1) + [("advance", int(ts[-1]) + 1_000)]
    out = both(rt, spec, pushes, label=f"partitioned {kind} {n}")
    assert out["ts"].size > 0


def test_rate_rejects(rt):
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", 10, aggs=AGGS, rate=("first", 0))
    with pytest.raises(rt.SiddhiError, match="every >= 1"):
        rt.GpuQuery(spec)


# `output first every <t>` (FirstPerTime / FirstGroupByPerTimeOutputRateLimiter): the chunk's playback
# clock decides, also for the sliding windows' per-send chunks and TIMER chunks (expired output)
@pytest.mark.parametrize("window,param,output", [("time", 300, "current"), ("time", 300, "all"),
                                                 ("timeBatch", 500, "all"), ("externalTime", 250, "expired")])
@pytest.mark.parametrize("group_by", [True, False])
@pytest.mark.parametrize("t", [1, 900])
def test_first_every_time(rt, window, param, output, group_by, t):
    ts, cols = stream(20_000, 30, 9, step=8)
    kw = {"ts_attr": "x"} if window == "externalTime" else {}
    if window == "externalTime":
        cols[2] = cols[3].copy()  # the attribute clock
    spec = abi.QuerySpec(SCHEMA, window, param, group_by=["k"] if group_by else (), aggs=AGGS, output=output,
                         key_capacity=64, rate=("first_time", t), **kw)
    pushes = split_batches(SCHEMA, ts, cols, [3_000, 11_111], 2) + [("advance", int(ts[-1]) + 2_000)]
    out = both(rt, spec, pushes, label=f"{window} {output} first every {t} gb={group_by}")
    assert out["ts"].size > 0


# ---- one limiter per partition instance on the partition lanes (sh_rate.cpp rate_part) ----------------
PSCHEMA = abi.Schema.parse("p int, g int, v double, x long, ts long")
PKINDS = [("all", 1), ("all", 3), ("first", 1), ("first", 2), ("last", 1), ("last", 3), ("first_time", 0),
          ("first_time", 90)]


def pstream(n, parts, seed):
    rng = np.random.default_rng(seed)
    ts = np.cumsum(rng.integers(0, 4, n)).astype(np.int64) + 5_000
    p = rng.integers(0, parts, n).astype(np.int32)
    g = rng.integers(0, 5, n).astype(np.int32)
    v = rng.integers(-4000, 4000, n).astype(np.float64) / 16.0
    x = rng.integers(-10**6, 10**6, n).astype(np.int64)
    return ts, [p, g, v, x, ts.copy()]


@pytest.mark.parametrize("kind,n", PKINDS)
@pytest.mark.parametrize("window,param,group_by,output", [("lengthBatch", 3, [], "all"), ("lengthBatch", 4, ["p"], "current"),
                                                         ("time", 60, ["p"], "all"), ("lengthBatch", 5, ["g"], "all"),
                                                         ("time", 80, ["g"], "all")])
def test_partition_lanes_rate(rt, kind, n, window, param, group_by, output):
    """`partition with (p of S)` clones the query with its OutputRateLimiter per partition: each
    partition's rows are counted (and, for `first every <t>`, timed) on their own"""
    ts, cols = pstream(20_000, 37, 7)
    spec = abi.QuerySpec(PSCHEMA, window, param, group_by=group_by, aggs=[("count", None), ("sum", "v")],
                         partition="p", output=output, key_capacity=64, rate=(kind, n))
    pushes = split_batches(PSCHEMA, ts, cols, [1, 3_000, 11_111], 1)
    if window == "time":
        pushes.append(("advance", int(ts[-1]) + 1_000))
    out = both(rt, spec, pushes, label=f"lanes {window} {group_by} {kind} {n}")
    assert out["ts"].size > 0


@pytest.mark.parametrize("kind,n", [("first", 2), ("last", 3), ("first_time", 90)])
@pytest.mark.parametrize("group_by", [["x"], ["g", "x"], ["p", "g"]])
def test_partition_lanes_keyed_rate_interned_group_keys(rt, kind, n, group_by):
    """keyed limiters of lanes grouped by a long or two-column key: the key is interned to one 32-bit id
    (sh_wide.h), which the lanes and the limiter key on"""
    ts, cols = pstream(12_000, 23, 11)
    cols[3] = (cols[3] % 7) * 1_000_000_007  # (few distinct long values: keys repeat within a partition)
    spec = abi.QuerySpec(PSCHEMA, "lengthBatch", 5, group_by=group_by, aggs=[("count", None), ("sum", "v")],
                         partition="p", output="all", key_capacity=256, rate=(kind, n))
    out = both(rt, spec, split_batches(PSCHEMA, ts, cols, [1, 4_000], 1), label=f"lanes interned {group_by} {kind} {n}")
    assert out["ts"].size > 0
