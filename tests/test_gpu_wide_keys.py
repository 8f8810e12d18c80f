"""Group keys of any number of columns (GroupByKeyGenerator.constructEventKey,
core/query/selector/GroupByKeyGenerator.java:63-73 joins every group-by attribute into the key): three or
more columns, or a long / double beside another column. The GPU interns such keys into one 32-bit id per
distinct key (sh_wide.h: a chain of two-component levels) and keys the window by it; rows get the
group-by values back. GPU = oracle for batch and sliding windows, every output mode, stream.current,
a rate limiter, partition lanes, checkpoints and device output. No reference KAT groups by more than two attributes:
these cases are GPU = oracle only (the oracle keys by the attributes' values, as the reference does)."""
import numpy as np
import pytest

from siddhi_amd import abi
from tests.parity import assert_same, split_batches
from tests.test_gpu_parity import both

pytestmark = pytest.mark.gpu

SCH = abi.Schema.parse("a int, s string, l long, d double, v double, ts long")
AGGS = [("count", None), ("sum", "v"), ("min", "v"), ("max", "l"), ("avg", "v")]


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def stream(n, seed, step=3):
    rng = np.random.default_rng(seed)
    ts = (np.cumsum(rng.integers(0, step, n)) + 10_000).astype(np.int64)
    a = rng.integers(-3, 4, n).astype(np.int32)
    s = rng.integers(0, 5, n).astype(np.int32)
    l = (rng.integers(0, 6, n) * 10_000_000_019 - 30_000_000_000).astype(np.int64)
    d = np.array([0.0, -0.0, 1.5, np.nan, -2.75])[rng.integers(0, 5, n)]
    v = rng.integers(-500, 500, n).astype(np.float64) / 4
    return ts, [a, s, l, d, v, ts.copy()]


@pytest.mark.parametrize("group", [["a", "s", "l"], ["l", "a"], ["d", "s"], ["s", "d", "a", "l"], ["a", "s", "a"]])
@pytest.mark.parametrize("window,param,output", [("timeBatch", 400, "current"), ("lengthBatch", 997, "all"),
                                                 ("time", 300, "all"), ("timeBatch", 250, "expired")])
def test_wide_group_keys(rt, group, window, param, output):
    ts, cols = stream(30_000, 3)
    spec = abi.QuerySpec(SCH, window, param, group_by=group, aggs=AGGS, filter=(">", "v", -100.0), output=output,
                         key_capacity=2048)
    pushes = split_batches(SCH, ts, cols, [1, 7_777, 20_000], 3)
    pushes.append(("advance", int(ts[-1]) + 5_000))
    out = both(rt, spec, pushes, label=f"wide {group} {window} {output}")
    assert out["keys"].shape[0] == len(group) and out["ts"].size > 0


def test_wide_keys_external_windows_and_stream_current(rt):
    ts, cols = stream(20_000, 5)
    for spec in (abi.QuerySpec(SCH, "externalTimeBatch", 500, group_by=["a", "l"], ts_attr="ts", aggs=AGGS,
                               output="all", key_capacity=512),
                 abi.QuerySpec(SCH, "externalTime", 400, group_by=["s", "a", "d"], ts_attr="ts", aggs=AGGS,
                               key_capacity=512),
                 abi.QuerySpec(SCH, "timeBatch", 300, group_by=["a", "s", "l"], aggs=AGGS, stream_current=True,
                               key_capacity=512),
                 abi.QuerySpec(SCH, "lengthBatch", 50, group_by=["l", "d"], aggs=AGGS, stream_current=True,
                               output="all", key_capacity=512)):
        both(rt, spec, split_batches(SCH, ts, cols, [5_000, 12_000], 4), label=f"wide {spec.window}")


@pytest.mark.parametrize("kind", ["first", "last", "all"])
def test_wide_keys_rate_limiter(rt, kind):
    ts, cols = stream(20_000, 7)
    spec = abi.QuerySpec(SCH, "timeBatch", 200, group_by=["a", "s", "l"], aggs=AGGS, key_capacity=512, rate=(kind, 7))
    both(rt, spec, split_batches(SCH, ts, cols, [3_000, 11_000], 2), label=f"wide rate {kind}")


@pytest.mark.parametrize("window", ["timeBatch", "time"])
def test_wide_keys_checkpoint(window):
    from tests.test_gpu_snapshot import checkpointed
    ts, cols = stream(24_000, 9)
    spec = abi.QuerySpec(SCH, window, 350, group_by=["s", "l", "a"], aggs=AGGS, output="all", key_capacity=1024)
    pushes = split_batches(SCH, ts, cols, [6_000, 13_000, 19_000], 5)
    got, ref, _ = checkpointed(spec, pushes, 2)
    assert_same(got, ref, label=f"wide ckpt {window}")


def test_wide_keys_device_output(rt):
    import torch
    from oracle.oracle import OracleQuery
    ts, cols = stream(16_000, 11)
    spec = abi.QuerySpec(SCH, "timeBatch", 300, group_by=["a", "l", "s"], aggs=AGGS, key_capacity=512)
    g, o = rt.GpuQuery(spec), OracleQuery(spec)
    dev = torch.device("cuda", 0)
    t = torch.from_numpy(ts).to(dev)
    dc = [torch.from_numpy(np.ascontiguousarray(c)).to(dev) for c in cols]
    torch.cuda.synchronize()
    got = rt.device_out_arrays(g.push_device(len(ts), t.data_ptr(), [c.data_ptr() for c in dc], 1))
    ref = abi.out_arrays(o.push_raw(abi.HostBatch(SCH, ts, cols, 1)))
    assert got["keys"].shape == (3, ref["ts"].size)
    assert_same(got, ref, label="wide device")
    g.close()
    o.close()


@pytest.mark.parametrize("window,param,output,group", [
    ("lengthBatch", 20, "current", ["a", "s", "l"]), ("lengthBatch", 7, "all", ["s", "d", "a"]),
    ("time", 300, "all", ["a", "s", "l"]), ("timeBatch", 250, "all", ["s", "l", "d"]),
    ("externalTimeBatch", 400, "current", ["a", "l", "s"])])
def test_wide_keys_partitioned(rt, window, param, output, group):
    """`partition with (a of S)` around a query grouped by a wide key: the key is interned before the
    partition lanes (which then group by its id) and decoded after them."""
    ts, cols = stream(20_000, 13)
    spec = abi.QuerySpec(SCH, window, param, group_by=group, aggs=AGGS, output=output, partition="a", key_capacity=2048,
                         ts_attr="ts" if window.startswith("external") else None)
    out = both(rt, spec, split_batches(SCH, ts, cols, [5_000, 12_000], 3), label=f"wide partitioned {window} {output}")
    assert out["ts"].size > 0


@pytest.mark.parametrize("kind", ["first", "last"])
def test_wide_keys_partitioned_keyed_rate(rt, kind):
    ts, cols = stream(12_000, 17)
    spec = abi.QuerySpec(SCH, "lengthBatch", 9, group_by=["s", "l", "d"], aggs=AGGS, partition="a", key_capacity=1024,
                         rate=(kind, 4))
    both(rt, spec, split_batches(SCH, ts, cols, [4_000], 2), label=f"wide partitioned rate {kind}")


def test_wide_keys_refusals(rt):
    full = abi.Schema.parse("a int, b int, c int, d int, e int, f int, v double, ts long")
    with pytest.raises(rt.SiddhiError, match="spare column"):
        rt.GpuQuery(abi.QuerySpec(full, "lengthBatch", 10, group_by=["a", "b", "c"], aggs=[("sum", "v")]))
    q = rt.GpuQuery(abi.QuerySpec(SCH, "lengthBatch", 10, group_by=["a", "s", "l"], aggs=AGGS, key_capacity=64))
    ts, cols = stream(100, 1)
    with pytest.raises(rt.SiddhiError, match="sh_push"):
        q.stage(abi.HostBatch(SCH, ts, cols, 1))
    q.close()
