"""GPU parity of `insert expired events` / `insert all events` on lengthBatch and timeBatch windows and
of pass-through (`select *`) batch queries, against the oracle's restatement of
LengthBatchWindowProcessor.processFullBatchEvents (:206-243), TimeBatchWindowProcessor.process
(:297-333) and QuerySelector.processInBatchGroupBy (:315-374) / processNoGroupBy (:161-205).
The reference KATs of these modes (lengthBatch3/5/6, playback1) run in test_gpu_parity.py."""
import numpy as np
import pytest

from siddhi_amd import abi
from tests.parity import split_batches
from tests.test_gpu_parity import both

pytestmark = pytest.mark.gpu

SCHEMA = abi.Schema.parse("k int, v double, x long, ts long")


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def stream(n, keys, seed, step=40, gap_at=None):
    rng = np.random.default_rng(seed)
    ts = np.cumsum(rng.integers(0, step, n)).astype(np.int64) + 5_000
    if gap_at is not None:
        ts[gap_at:] += 20_000  # several empty windows
    k = rng.integers(0, keys, n).astype(np.int32)
    v = rng.integers(-4000, 4000, n).astype(np.float64) / 16.0
    x = rng.integers(-10**6, 10**6, n).astype(np.int64)
    return ts, [k, v, x, ts.copy()]


AGGS = [("count", None), ("sum", "v"), ("min", "v"), ("max", "x"), ("avg", "x"), ("sum", "x")]


@pytest.mark.parametrize("output", ["all", "expired"])
@pytest.mark.parametrize("send_size", [1, 9])
def test_timebatch_group_by_expired_output(rt, output, send_size):
    ts, cols = stream(60_000, 300, 5, gap_at=31_000)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 700, group_by=["k"], aggs=AGGS, filter=(">", "v", -150.0),
                         output=output, key_capacity=512)
    pushes = split_batches(SCHEMA, ts, cols, [1, 2_000, 30_999, 31_000, 45_000], send_size)
    pushes.append(("advance", int(ts[-1]) + 350))   # closes the open window
    pushes.append(("advance", int(ts[-1]) + 5_000))  # and the empty one after it: expired-only flush
    out = both(rt, spec, pushes, label=f"timeBatch {output}")
    assert out["expired"].sum() > 0
    if output == "all":
        assert (out["expired"] == 0).sum() > 0


@pytest.mark.parametrize("output", ["all", "expired"])
@pytest.mark.parametrize("L,cuts", [(1000, [777, 5_000, 5_001]), (7, [3, 40_000]), (1, [10, 11])])
def test_lengthbatch_group_by_expired_output(rt, output, L, cuts):
    ts, cols = stream(50_000 if L > 1 else 3_000, 50, 9)
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", L, group_by=["k"], aggs=AGGS, output=output, key_capacity=64)
    both(rt, spec, split_batches(SCHEMA, ts, cols, cuts, 5), label=f"lengthBatch({L}) {output}")


def test_timebatch_many_keys_all_events(rt):
    """100k keys: the partitioned aggregation path underneath, tables per merged flush."""
    ts, cols = stream(400_000, 100_000, 13, step=2)
    spec = abi.QuerySpec(SCHEMA, "timeBatch", 100, group_by=["k"], aggs=[("count", None), ("avg", "v")],
                         output="all", key_capacity=100_000)
    pushes = split_batches(SCHEMA, ts, cols, [150_000], 1) + [("advance", int(ts[-1]) + 1000)]
    out = both(rt, spec, pushes, label="timeBatch 100k keys all")
    assert out["flush_offsets"].size > 4


@pytest.mark.parametrize("output", ["all", "expired"])
def test_no_group_by_aggregates(rt, output):
    ts, cols = stream(20_000, 10, 17)
    spec = abi.QuerySpec(SCHEMA, "lengthBatch", 100, aggs=[("sum", "v"), ("count", None)], output=output)
    both(rt, spec, split_batches(SCHEMA, ts, cols, [999], 3), label=f"no group-by {output}")


@pytest.mark.parametrize("window,param", [("lengthBatch", 5), ("lengthBatch", 333), ("timeBatch", 250)])
@pytest.mark.parametrize("output", ["current", "all", "expired"])
def test_pass_through(rt, window, param, output):
    ts, cols = stream(20_000, 10, 21, gap_at=12_000)
    spec = abi.QuerySpec(SCHEMA, window, param, filter=("<", "x", 500_000), output=output)
    pushes = split_batches(SCHEMA, ts, cols, [1, 7_000, 12_000], 4) + [("advance", int(ts[-1]) + 2_000)]
    out = both(rt, spec, pushes, label=f"pass-through {window} {output}")
    assert out["ts"].size > 0


PSCHEMA = abi.Schema.parse("k int, p int, v double, x long, ts long")


@pytest.mark.parametrize("output", ["all", "expired"])
@pytest.mark.parametrize("group_by,send_size", [(["k"], 1), (["p"], 7), ([], 1), (["k", "p"], 3)])
def test_partitioned_timebatch_expired_output(rt, output, group_by, send_size):
    """`partition with (p of S)` around timeBatch with expired / all-events output: nextEmitTime is shared
    by the partitions and only the partition that armed it flushes (R12, TimeBatchWindowProcessor.process
    :262-340), emitting its previous batch as EXPIRED then its current batch — also across empty windows
    and with the first passing event of a later push"""
    rng = np.random.default_rng(77)
    n = 40_000
    ts = np.cumsum(rng.integers(0, 30, n)).astype(np.int64) + 5_000
    ts[22_000:] += 9_000  # empty windows
    cols = [rng.integers(0, 60, n).astype(np.int32), rng.integers(0, 4, n).astype(np.int32),
            rng.integers(-4000, 4000, n).astype(np.float64) / 16.0, rng.integers(-10**6, 10**6, n).astype(np.int64),
            ts.copy()]
    spec = abi.QuerySpec(PSCHEMA, "timeBatch", 700, group_by=group_by, aggs=AGGS, partition="p", output=output,
                         filter=(">", "v", -120.0), key_capacity=256)
    pushes = split_batches(PSCHEMA, ts, cols, [1, 9_000, 30_000], send_size) + [("advance", int(ts[-1]) + 3_000)]
    ref = both(rt, spec, pushes, label=f"p timeBatch {output} {group_by}")
    assert ref["expired"].sum() > 0
