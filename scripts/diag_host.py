"""Diagnostics only: per-call time split of the send(Event[n]) host path (sh_stage vs
sh_push_staged) at a given batch size; run with SH_TIMING=1 for the library's internal points."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from siddhi_amd import abi, runtime, synth

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1000
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3000
schema = abi.Schema.parse("k string, v double, ts long")
spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"],
                     aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=100_000)
q = runtime.GpuQuery(spec)
bufs = []
for i in range(n):
    ts, cols = synth.keyed_stream(i * B, B, 0xC2, 100_000, 1000)
    bufs.append(runtime.PinnedBatch(schema, B, 1).fill(ts, cols, 1))
st, pu = [], []
t = q.stage(bufs[0])
for i in range(n):
    a = time.perf_counter()
    nt = q.stage(bufs[i + 1]) if i + 1 < n else None
    b = time.perf_counter()
    q.push_staged_raw(t)
    c = time.perf_counter()
    t = nt
    st.append(b - a)
    pu.append(c - b)
st, pu = np.array(st[100:]) * 1e6, np.array(pu[100:]) * 1e6
print(f"batch {B}: stage p50 {np.median(st):.1f} us, push p50 {np.median(pu):.1f} us p99 {np.percentile(pu, 99):.1f}; "
      f"{B / (np.median(st) + np.median(pu)) * 1e6:.3e} events/s at p50")
q.close()
