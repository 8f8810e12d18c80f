"""One-off diagnostic: first mismatching rows of the sliding expired-output path vs the oracle."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle.oracle import OracleQuery
from siddhi_amd import abi, runtime
from tests.parity import run_pushes, split_batches
import tests.test_gpu_sliding_expired as t

ts, cols = t.stream(3_000, 20, 3)
for aggs in ([("min", "v")], [("max", "x")], [("count", None), ("min", "v")], [("sum", "v"), ("min", "v")], t.AGGS):
    for out in ("all", "current"):
        spec = abi.QuerySpec(t.SCHEMA, "time", 500, group_by=["k"], aggs=aggs, output=out, key_capacity=32)
        pushes = split_batches(t.SCHEMA, ts, cols, [1000], 1)
        g, o = runtime.GpuQuery(spec), OracleQuery(spec)
        a, b = run_pushes(g, pushes), run_pushes(o, pushes)
        for i in range(len(aggs)):
            bad = np.nonzero(a["vals"][i] != b["vals"][i])[0]
            print(aggs, out, "agg", i, "rows", len(a["ts"]), len(b["ts"]), "bad", bad.size, bad[:5])
            if bad.size:
                r = bad[0]
                print("  row", r, "key", a["keys"][0][r], "gpu", a["vals"][i][r:r+3].view(np.float64),
                      "ora", b["vals"][i][r:r+3].view(np.float64), "exp", a["expired"][r])
                k = a["keys"][0][r]
                idx = [j for j in range(r + 1) if b["keys"][0][j] == k]
                print("  key history ora", [(int(b["expired"][j]), b["vals"][i][j:j+1].view(np.float64)[0]) for j in idx][-8:])
                print("  key history gpu", [(int(a["expired"][j]), a["vals"][i][j:j+1].view(np.float64)[0]) for j in idx][-8:])
        g.close(); o.close()
