"""One-off diagnostic: first divergence of the C3 all-events stream, GPU vs oracle."""
import sys
import numpy as np
sys.path.insert(0, ".")
from oracle.oracle import OracleQuery
from siddhi_amd import abi, runtime, synth

import tests.test_gpu_sliding_expired as t
for out in ("all", "expired"):
    for ss in (1, 7):
        t.test_time_group_by_expired_output(runtime, out, ss)
for out in ("all", "expired"):
    t.test_time_out_of_order_timestamps(runtime, out)
t.test_time_no_group_by_and_hashed_long_keys(runtime)
t.test_time_key_churn_rebuilds_table(runtime)
for out in ("all", "expired"):
    for ss in (1, 16):
        t.test_external_time_expired_output(runtime, out, ss)
for w in ("time", "externalTime"):
    for out in ("current", "all", "expired"):
        t.test_pass_through(runtime, w, out)
print("warm-up tests done", flush=True)
ks = abi.Schema.parse("k string, v double, ts long")
spec = abi.QuerySpec(ks, "time", 10_000, group_by=["k"], output="all", key_capacity=10_000,
                     aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")])
g, o = runtime.GpuQuery(spec), OracleQuery(spec)
step, total = 1_000_000, 12_000_000
for a in range(0, total, step):
    ts, cols = synth.keyed_stream(a, step, 0xC3, 10_000, 1000)
    b = abi.HostBatch(ks, ts, cols, 1)
    go, oo = abi.out_arrays(g.push_raw(b)), abi.out_arrays(o.push_raw(b))
    if not np.array_equal(go["flush_offsets"], oo["flush_offsets"]):
        fg, fo = go["flush_offsets"], oo["flush_offsets"]
        print("push", a, "flushes", len(fg), len(fo), "rows", len(go["ts"]), len(oo["ts"]))
        n = min(len(fg), len(fo))
        d = int(np.nonzero(fg[:n] != fo[:n])[0][0]) if np.any(fg[:n] != fo[:n]) else n
        print("first flush diff at", d, "gpu", fg[d - 2:d + 3], "ora", fo[d - 2:d + 3])
        print("clocks gpu", go["flush_clock"][d - 3:d + 3], "ora", oo["flush_clock"][d - 3:d + 3])
        r0 = int(min(fg[d - 1], fo[d - 1]))
        for name, x in (("gpu", go), ("ora", oo)):
            sl = slice(r0, r0 + 8)
            print(name, "keys", x["keys"][0][sl], "exp", x["expired"][sl], "ts", x["ts"][sl], "rep", x["rep"][sl])
        ne = np.nonzero(go["expired"][:min(len(go['ts']), len(oo['ts']))] != oo["expired"][:min(len(go['ts']), len(oo['ts']))])[0]
        print("first expired-flag diff row", ne[:5])
        print("event ts around", ts[:3], "clock at start", ts[0])
        sz = len(fo) - 1
        for name, x in (("gpu", go), ("ora", oo)):
            f = x["flush_offsets"]
            sizes = np.diff(f)
            print(name, "flush sizes hist", np.bincount(np.minimum(sizes, 20)), "n expired", int(x["expired"].sum()))
        break
    print("push", a, "ok", len(oo["ts"]), int(oo["expired"].sum()))
