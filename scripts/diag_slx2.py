"""One-off diagnostic of the sliding expired-output replay (debug build)."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle.oracle import OracleQuery
from siddhi_amd import abi, runtime
from tests.parity import run_pushes, split_batches
import tests.test_gpu_sliding_expired as t

ts, cols = t.stream(60, 20, 3)
spec = abi.QuerySpec(t.SCHEMA, "time", 500, group_by=["k"], aggs=[("min", "v")], output="all", key_capacity=32)
g = runtime.GpuQuery(spec)
a = run_pushes(g, split_batches(t.SCHEMA, ts, cols, [], 1))
print("keys", a["keys"][0][:10], "vals", a["vals"][0][:10].view(np.float64))
print("k", cols[0][:10], "v", cols[1][:10])
