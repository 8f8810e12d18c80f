"""Sliding-window replay timing probe (diagnostics): C3-shaped pushes with several aggregator sets.
usage: python scripts/sl_probe.py [pushes]"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from siddhi_amd import abi, runtime, synth  # noqa: E402

n_push = int(sys.argv[1]) if len(sys.argv) > 1 else 4
B = 1 << 24
schema = abi.Schema.parse("k string, v double, ts long")
T = int(os.environ.get("SH_PROBE_T", "10000"))
sets = ([("count", None)], [("count", None), ("avg", "v")], [("count", None), ("min", "v")],
        [("count", None), ("min", "v"), ("max", "v"), ("avg", "v")])
if os.environ.get("SH_PROBE_ONE"):
    sets = sets[1:2]
for aggs in sets:
    spec = abi.QuerySpec(schema, "time", T, group_by=["k"], aggs=aggs, key_capacity=10_000)
    q = runtime.GpuQuery(spec)
    dev = torch.device("cuda", 0)
    ms = []
    for i in range(n_push):
        ts, cols = synth.torch_keyed_stream(i * B, B, 0xC3, 10_000, 1000, dev)
        torch.cuda.synchronize()
        q.push_device(B, ts.data_ptr(), [c.data_ptr() for c in cols], 1)
        st = q.stats()
        ms.append((st.main_kernel_ms, st.push_ms))
    print([a for a, _ in aggs], "main ms per push:", " ".join(f"{a:.2f}" for a, _ in ms),
          "| push ms:", " ".join(f"{b:.2f}" for _, b in ms), flush=True)
    q.close()
