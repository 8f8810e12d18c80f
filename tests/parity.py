"""Parity helpers: drive the HIP library (through the C-ABI) and the oracle with identical pushes and
compare the emitted flushes. Integer outputs, window boundaries, row order and timestamps must be
bit-exact; double outputs are compared bit-exact too unless `rtol` is given (the north_star bar is
1e-9 relative for double sum/avg; the ordered per-key kernels reproduce Java's summation order, so
the tests demand identity)."""
import numpy as np

from siddhi_amd import abi


def run_pushes(q, pushes):
    """pushes: list of HostBatch or ('advance', now). Returns concatenated out_arrays."""
    parts = []
    replace = getattr(getattr(q, "spec", None), "replace_ts", False)
    for p in pushes:
        if isinstance(p, tuple) and p[0] == "advance":
            parts.append(abi.out_arrays(q.advance_time_raw(p[1])))
        else:
            parts.append(abi.out_arrays(q.push_raw(p)))
        if replace:  # the batch end time in every row's representative event (replaceTimestampWithBatchEndTime)
            parts[-1]["rep_attr"] = q.rep_ts_attr()
    return abi.concat_arrays(parts)


def assert_same(gpu, ora, rtol=None, label=""):
    assert np.array_equal(gpu["flush_offsets"], ora["flush_offsets"]), \
        f"{label}: flush offsets differ\n gpu={gpu['flush_offsets'][:20]}\n ora={ora['flush_offsets'][:20]}"
    assert np.array_equal(gpu["flush_clock"], ora["flush_clock"]), f"{label}: flush clocks differ"
    assert np.array_equal(gpu["ts"], ora["ts"]), f"{label}: row timestamps differ"
    assert np.array_equal(gpu["keys"], ora["keys"]), f"{label}: group keys / row order differ"
    assert np.array_equal(gpu["nulls"], ora["nulls"]), f"{label}: null flags differ"
    assert np.array_equal(gpu["expired"], ora["expired"]), f"{label}: expired flags differ"
    assert np.array_equal(gpu["rep"], ora["rep"]), f"{label}: representative events differ"
    if "rep_attr" in ora:
        assert np.array_equal(gpu["rep_attr"], ora["rep_attr"]), f"{label}: replaced timestamp attributes differ"
    vt = ora["val_types"]
    assert np.array_equal(gpu["val_types"], vt)
    for a in range(len(vt)):
        g, o = gpu["vals"][a], ora["vals"][a]
        if vt[a] in (abi.DOUBLE, abi.FLOAT) and rtol is not None:
            gd, od = g.view(np.float64), o.view(np.float64)
            np.testing.assert_allclose(gd, od, rtol=rtol, atol=0, err_msg=f"{label}: agg {a}")
        else:
            bad = np.nonzero(g != o)[0]
            assert bad.size == 0, f"{label}: agg {a} differs at rows {bad[:10]} gpu={g[bad[:5]]} ora={o[bad[:5]]}"


def split_batches(schema, ts, cols, cuts, send_size=0):
    """Cut one stream into pushes at the given event indices."""
    out = []
    edges = [0] + list(cuts) + [len(ts)]
    for a, b in zip(edges[:-1], edges[1:]):
        if b > a:
            out.append(abi.HostBatch(schema, ts[a:b], [c[a:b] for c in cols], send_size))
    return out
