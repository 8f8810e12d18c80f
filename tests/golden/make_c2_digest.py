"""Golden digest of the headline configuration's output (BASELINE.json configs[1] as bench.py runs it).

Runs the CPU restatement (oracle/, the checker pinned by the reference's KATs) over bench.py's exact C2
stream — `timeBatch(1 sec) select k, count(), min(v), max(v), avg(v) group by k`, k a dictionary-encoded
string over 100k uniform keys, 1,000 events per event-time ms, one send per event, SplitMix64 seed 0xC2
(siddhi_amd.synth.keyed_stream, identical to the torch generator bench.py uses in HBM) — as two pushes of
2^25 events, and writes the SHA-256 of the canonical output (siddhi_amd.digest) of push 0 (bench.py's
first warm-up push) and of pushes 0 + 1 to tests/golden/c2_bench_digest.json. The GPU test
tests/test_gpu_headline.py and bench.py compare against it.

Run: python tests/golden/make_c2_digest.py   (about a minute, single thread)
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.oracle import OracleQuery  # noqa: E402
from siddhi_amd import abi, digest, synth  # noqa: E402

B, KEYS, EPM, SEND, SEED = 1 << 25, 100_000, 1000, 1, 0xC2


def spec():
    schema = abi.Schema.parse("k string, v double, ts long")
    return schema, abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"],
                                 aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=KEYS)


def main():
    schema, sp = spec()
    q = OracleQuery(sp)
    parts, res = [], {}
    t0 = time.time()
    for i in range(2):
        ts, cols = synth.keyed_stream(i * B, B, SEED, KEYS, EPM)
        parts.append(abi.out_arrays(q.push_raw(abi.HostBatch(schema, ts, cols, SEND))))
        a = abi.concat_arrays(parts)
        res[f"push0{'1' if i else ''}"] = {"sha256": digest.output_digest(a), "rows": int(a["ts"].size),
                                            "flushes": int(a["flush_clock"].size)}
        print(i, res, f"{time.time() - t0:.1f} s", flush=True)
    res["config"] = {"events_per_push": B, "keys": KEYS, "events_per_ms": EPM, "send_size": SEND, "seed": SEED,
                     "query": "timeBatch(1 sec) select k, count(), min(v), max(v), avg(v) group by k; k string",
                     "generator": "siddhi_amd.synth.keyed_stream", "made_by": "tests/golden/make_c2_digest.py"}
    with open(os.path.join(HERE, "c2_bench_digest.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
