"""debug: first row where the GPU and the oracle differ for an ext-timeout pass-through case"""
import numpy as np
from oracle.oracle import OracleQuery
from siddhi_amd import abi, runtime
from tests.parity import run_pushes, split_batches
from tests.test_gpu_ext import SCH, tstream, tspec, with_advances

ts, cols = tstream(40_000, 0xF2, late_ms=300)
pushes = with_advances(split_batches(SCH, ts, cols, [10_000, 20_000, 30_000], 3), ts)
sp = tspec(output="current", group=False, aggs=[])
g, o = runtime.GpuQuery(sp), OracleQuery(sp)
a, b = run_pushes(g, pushes), run_pushes(o, pushes)
print("rows", a["ts"].size, b["ts"].size)
bad = np.nonzero(a["ts"] != b["ts"])[0]
print("n bad", bad.size, "first", bad[:10])
fo = b["flush_offsets"]
if bad.size:
    i = bad[0]
    f = np.searchsorted(fo, i, side="right") - 1
    print("flush", f, "range", fo[f], fo[f + 1], "clock", b["flush_clock"][f])
    print("gpu ts", a["ts"][fo[f]:fo[f + 1]][:12], "rep", a["rep"][fo[f]:fo[f + 1]][:12])
    print("ora ts", b["ts"][fo[f]:fo[f + 1]][:12], "rep", b["rep"][fo[f]:fo[f + 1]][:12])
    print("gpu rep == ora rep", np.array_equal(a["rep"], b["rep"]))
