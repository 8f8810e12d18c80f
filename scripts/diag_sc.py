"""Diagnostic: first flush where the GPU and the oracle differ for timeBatch(T, true) all-events."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from oracle.oracle import OracleQuery
from siddhi_amd import abi, runtime as rt
from tests.parity import run_pushes, split_batches
from tests.test_gpu_stream_current import SCHEMA, AGGS, stream

ts, cols = stream(30_000, 300, 19, gap_at=17_000)
spec = abi.QuerySpec(SCHEMA, "timeBatch", 700, group_by=["k"], aggs=AGGS, filter=(">", "v", -150.0),
                     stream_current=True, output="all", key_capacity=512)
pushes = split_batches(SCHEMA, ts, cols, [1, 2_000, 16_999, 17_000, 25_000], 1)
none_pass = abi.HostBatch(SCHEMA, ts[25_000:25_100] + 900, [cols[0][:100], np.full(100, -500.0), cols[2][:100],
                                                             ts[25_000:25_100] + 900], 1)
pushes.insert(3, ("advance", int(ts[16_999]) + 1_500))
pushes.insert(6, none_pass)
pushes.append(("advance", int(ts[-1]) + 5_000))
for i, p in enumerate(pushes):
    g = rt.GpuQuery(spec) if i == 0 else g
    o = OracleQuery(spec) if i == 0 else o
for pi in range(len(pushes)):
    pass
g = rt.GpuQuery(spec); o = OracleQuery(spec)
for pi, p in enumerate(pushes):
    ga = abi.out_arrays(g.advance_time_raw(p[1]) if isinstance(p, tuple) else g.push_raw(p))
    oa = abi.out_arrays(o.advance_time_raw(p[1]) if isinstance(p, tuple) else o.push_raw(p))
    same = all(np.array_equal(ga[k], oa[k]) for k in ("flush_offsets", "flush_clock", "ts", "keys", "expired", "rep"))
    print("push", pi, "advance" if isinstance(p, tuple) else len(p.ts), "flushes", len(ga["flush_clock"]),
          len(oa["flush_clock"]), "rows", ga["ts"].size, oa["ts"].size, "same" if same else "DIFF")
    if not same:
        fg, fo = ga["flush_offsets"], oa["flush_offsets"]
        n = min(len(fg), len(fo))
        d = next((i for i in range(n) if fg[i] != fo[i] or (i < n - 1 and ga["flush_clock"][i] != oa["flush_clock"][i])), n)
        print(" first diff flush", d, "gpu off", fg[max(0, d - 2):d + 3], "ora off", fo[max(0, d - 2):d + 3])
        print(" gpu clk", ga["flush_clock"][max(0, d - 2):d + 3], "ora clk", oa["flush_clock"][max(0, d - 2):d + 3])
        a = fo[max(0, d - 1)]
        print(" gpu exp", ga["expired"][a:a + 12], "keys", ga["keys"][0, a:a + 12])
        print(" ora exp", oa["expired"][a:a + 12], "keys", oa["keys"][0, a:a + 12])
        break
