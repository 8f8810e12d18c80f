"""The headline configuration itself, on the GPU, exactly as bench.py runs it (BASELINE.json configs[1]):
two sh_push_device calls of 2^25 events generated in HBM by synth.torch_keyed_stream (seed 0xC2, 100k
dictionary-encoded string keys, 1,000 events per event-time ms, one send per event) through
`timeBatch(1 sec) select k, count(), min(v), max(v), avg(v) group by k` — 33.5 windows per push, ~10
events per key per window, the packed multisplit records' wide re-split past 2^22 events per segment.
The canonical SHA-256 of the output (siddhi_amd.digest) must equal the CPU restatement's on the same
stream, committed as tests/golden/c2_bench_digest.json by tests/golden/make_c2_digest.py: bit-exact
doubles, row order, flush clocks and representative events."""
import json
import os

import pytest

from siddhi_amd import abi, digest, synth

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_headline_c2_bench_path_matches_golden_digest():
    import torch
    from siddhi_amd import runtime
    gold = json.load(open(os.path.join(HERE, "golden", "c2_bench_digest.json")))
    cfg = gold["config"]
    B = cfg["events_per_push"]
    schema = abi.Schema.parse("k string, v double, ts long")
    spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=cfg["keys"])
    dev = torch.device("cuda", 0)
    q = runtime.GpuQuery(spec)
    parts = []
    for i, name in enumerate(("push0", "push01")):
        ts, cols = synth.torch_keyed_stream(i * B, B, cfg["seed"], cfg["keys"], cfg["events_per_ms"], dev)
        torch.cuda.synchronize()
        d = q.device_batch(B, ts.data_ptr(), [c.data_ptr() for c in cols], cfg["send_size"])
        out = q.push_device_batch(d)
        torch.cuda.synchronize()
        parts.append(runtime.device_out_arrays(out))
        a = abi.concat_arrays(parts)
        assert a["ts"].size == gold[name]["rows"] and a["flush_clock"].size == gold[name]["flushes"]
        assert digest.output_digest(a) == gold[name]["sha256"], name
        del ts, cols
    q.close()


def test_c1_bench_path_matches_golden_digest():
    """C1 (BASELINE.json configs[0]) exactly as `bench.py --workload c1` runs it: two sh_push_device calls of
    33,554,000 events (send(Event[1000])) through the filtered lengthBatch(10000) group-by; the second push
    starts with the batch carried across the push boundary. Golden: tests/golden/make_c1_digest.py."""
    import numpy as np
    import torch
    from siddhi_amd import runtime
    gold = json.load(open(os.path.join(HERE, "golden", "c1_bench_digest.json")))
    cfg = gold["config"]
    B = cfg["events_per_push"]
    schema = abi.Schema.parse("symbol string, price double, volume long, ts long")
    spec = abi.QuerySpec(schema, "lengthBatch", 10000, group_by=["symbol"], aggs=[("sum", "volume"), ("avg", "price")],
                         filter=(">", "price", 100), key_capacity=1000)
    dev = torch.device("cuda", 0)
    q = runtime.GpuQuery(spec)
    parts = []
    for i, name in enumerate(("push0", "push01")):
        cols = [torch.from_numpy(np.ascontiguousarray(c)).to(dev) for c in synth.c1_stock(i * B, B)[1]]
        torch.cuda.synchronize()
        out = q.push_device(B, cols[3].data_ptr(), [c.data_ptr() for c in cols], cfg["send_size"])
        torch.cuda.synchronize()
        parts.append(runtime.device_out_arrays(out))
        a = abi.concat_arrays(parts)
        assert a["ts"].size == gold[name]["rows"] and a["flush_clock"].size == gold[name]["flushes"]
        assert digest.output_digest(a) == gold[name]["sha256"], name
        del cols
    q.close()
