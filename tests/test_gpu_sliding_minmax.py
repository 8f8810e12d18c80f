"""The keyed sliding replay's parallel min / max (k_sl_wkey, round 4) against the oracle's sequential
restatement of MinAttributeAggregatorExecutor / MaxAttributeAggregatorExecutor (:187-236, the LinkedList
deque with removeFirstOccurrence) inside TimeWindowProcessor (:132-169). The parallel form holds while no
expiring event meets a bit-equal value and no NaN is in sight; every other chunk falls back to the
sequential deque. These streams drive each branch: distinct values (parallel throughout), few distinct
values (the quirk: fallback), NaN and signed zeros, windows shorter than a 64-record chunk, and
monotone runs whose deque outgrows the LDS ring (and spills to global memory)."""
import numpy as np
import pytest

from siddhi_amd import abi
from tests.parity import split_batches
from tests.test_gpu_sliding_expired import both

pytestmark = pytest.mark.gpu

SCHEMA = abi.Schema.parse("k int, v double, ts long")
AGGS = [("count", None), ("min", "v"), ("max", "v"), ("avg", "v")]


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def stream(n, keys, seed, kind, per_ms=20):
    rng = np.random.default_rng(seed)
    ts = (np.arange(n) // per_ms + 5_000).astype(np.int64)
    k = rng.integers(0, keys, n).astype(np.int32)
    if kind == "distinct":
        v = rng.random(n) * 1000.0
    elif kind == "few":
        v = rng.integers(0, 6, n).astype(np.float64)
    elif kind == "specials":
        v = rng.random(n) * 10.0
        pick = rng.random(n)
        v[pick < 0.002] = np.nan
        v[(pick >= 0.002) & (pick < 0.01)] = 0.0
        v[(pick >= 0.01) & (pick < 0.018)] = -0.0
        v[(pick >= 0.018) & (pick < 0.03)] = 3.5  # an occasional repeat
    elif kind == "monotone":
        # per key long increasing then decreasing runs: deques far longer than the LDS ring
        v = np.sin(np.arange(n) / 20_000.0) * 100.0 + np.arange(n) * 1e-9
    return ts, [k, v, ts.copy()]


@pytest.mark.parametrize("kind", ["distinct", "few", "specials", "monotone"])
@pytest.mark.parametrize("T,keys", [(2_000, 40), (30, 40), (500, 3)])
def test_keyed_sliding_min_max_parallel_and_sequential(rt, kind, T, keys):
    ts, cols = stream(120_000, keys, 91, kind)
    spec = abi.QuerySpec(SCHEMA, "time", T, group_by=["k"], aggs=AGGS, key_capacity=64)
    pushes = split_batches(SCHEMA, ts, cols, [1_000, 50_000, 90_000], 1)
    ref = both(rt, spec, pushes, f"minmax {kind} T={T} keys={keys}")
    assert ref["ts"].size == 120_000


def test_keyed_sliding_min_only_and_max_only(rt):
    ts, cols = stream(60_000, 16, 93, "specials")
    for aggs in ([("min", "v")], [("max", "v"), ("sum", "v")]):
        spec = abi.QuerySpec(SCHEMA, "time", 700, group_by=["k"], aggs=aggs, key_capacity=16)
        both(rt, spec, split_batches(SCHEMA, ts, cols, [30_000], 1), f"minmax {aggs}")


@pytest.mark.parametrize("seq", ["0", "1"])
def test_sliding_records_forms(rt, seq, monkeypatch):
    """Both forms of the sliding records pass (k_sl_records and the lane-strided k_sl_records_seq, chosen
    per query by SH_SL_RECORDS_SEQ at creation) give the oracle's rows on a C3-shaped stream."""
    from siddhi_amd import synth
    monkeypatch.setenv("SH_SL_RECORDS_SEQ", seq)
    schema = abi.Schema.parse("k string, v double, ts long")
    ts, cols = synth.keyed_stream(0, 300_000, 0xC3, 2_000, 100)
    spec = abi.QuerySpec(schema, "time", 1_000, group_by=["k"], aggs=AGGS, key_capacity=2_000)
    both(rt, spec, split_batches(schema, ts, cols, [100_000, 250_000], 1), f"records seq={seq}")
