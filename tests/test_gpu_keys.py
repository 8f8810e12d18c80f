"""Group keys beyond integral columns (GroupByKeyGenerator.constructEventKey,
core/query/selector/GroupByKeyGenerator.java:63-73: the key is the values' String.valueOf form): a
double or float column names every value apart — 0.0 and -0.0 too — except NaN, whose payloads all
print "NaN". The GPU keys by the value's bits with NaN made canonical (one float column, alone or
beside a 32-bit one); the oracle restates the same rule. sh_out reports a floating-point key as the
bits of its value widened to double. No reference KAT groups by a floating-point column: these cases
are GPU = oracle only (parity unpinned by reference fixtures)."""
import numpy as np
import pytest

from siddhi_amd import abi
from tests.parity import split_batches
from tests.test_gpu_parity import both

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    from siddhi_amd import runtime
    return runtime


def _fp_keys(n, rng, dtype):
    base = np.array([0.0, -0.0, 1.5, -2.25, np.nan, np.inf, -np.inf, 3e-300, 1e300, 7.0], dtype=np.float64)
    k = base[rng.integers(0, base.size, n)]
    # NaNs with other payloads: one key with the canonical NaN
    nan2 = np.frombuffer(np.uint64(0x7FF0000000000123).tobytes(), dtype=np.float64)[0]
    k = np.where(rng.random(n) < 0.05, nan2, k)
    if dtype == np.float32:
        with np.errstate(over="ignore", invalid="ignore"):
            k = k.astype(np.float32)
        nanf = np.frombuffer(np.uint32(0x7F800123).tobytes(), dtype=np.float32)[0]
        k = np.where(rng.random(n) < 0.05, nanf, k).astype(np.float32)
    return k


@pytest.mark.parametrize("ktype", ["double", "float"])
@pytest.mark.parametrize("window,param", [("timeBatch", 500), ("lengthBatch", 777), ("time", 300)])
def test_floating_point_group_key(rt, ktype, window, param):
    rng = np.random.default_rng(5)
    n = 40_000
    sch = abi.Schema.parse(f"k {ktype}, v double, ts long")
    ts = (np.cumsum(rng.integers(0, 3, n)) + 10_000).astype(np.int64)
    k = _fp_keys(n, rng, np.float32 if ktype == "float" else np.float64)
    v = rng.integers(-500, 500, n).astype(np.float64) / 4
    spec = abi.QuerySpec(sch, window, param, group_by=["k"],
                         aggs=[("count", None), ("sum", "v"), ("min", "v"), ("max", "v")], key_capacity=64)
    pushes = split_batches(sch, ts, [k, v, ts.copy()], [1, 9_999, 25_000], 3)
    pushes.append(("advance", int(ts[-1]) + 5_000))
    out = both(rt, spec, pushes, label=f"{ktype} key {window}")
    keys = out["keys"][0].view(np.float64)
    assert np.isnan(keys).any() and (np.signbit(keys) & (keys == 0)).any() and ((keys == 0) & ~np.signbit(keys)).any()
    # NaN payloads collapse to one key: at most one NaN row per flush
    fo = out["flush_offsets"]
    assert max(int(np.isnan(keys[a:b]).sum()) for a, b in zip(fo[:-1], fo[1:])) <= 1


def test_float_and_int_group_key(rt):
    """two 32-bit components: an int and a float (the float by its own canonical bits)"""
    rng = np.random.default_rng(9)
    n = 30_000
    sch = abi.Schema.parse("a int, f float, v double, ts long")
    ts = (np.cumsum(rng.integers(0, 3, n)) + 10_000).astype(np.int64)
    a = rng.integers(-3, 4, n).astype(np.int32)
    f = _fp_keys(n, rng, np.float32)
    v = rng.integers(-500, 500, n).astype(np.float64) / 4
    spec = abi.QuerySpec(sch, "timeBatch", 400, group_by=["a", "f"], aggs=[("count", None), ("avg", "v")],
                         key_capacity=256)
    both(rt, spec, split_batches(sch, ts, [a, f, v, ts.copy()], [7_000, 20_000], 1) +
         [("advance", int(ts[-1]) + 5_000)], label="int+float key")
