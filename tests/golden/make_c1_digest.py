"""Golden digest of the C1 configuration's output as `bench.py --workload c1` runs it (BASELINE.json configs[0]).

Runs the CPU restatement (oracle/, the checker pinned by the reference's KATs) over the bench's exact C1
stream — `from StockStream[price > 100]#window.lengthBatch(10000) select symbol, sum(volume), avg(price)
group by symbol`, 1k dictionary-encoded symbols, `send(Event[1000])` (siddhi_amd.synth.c1_stock, seed 0xC1)
— as two pushes of 33,554,000 events (2^25 cut at a send boundary), and writes the SHA-256 of the canonical
output (siddhi_amd.digest) of push 0 (the bench's first warm-up push) and of pushes 0 + 1 to
tests/golden/c1_bench_digest.json. Push 1 starts with the batch carried across the push boundary and both
pushes re-split segments longer than 2^22 events. tests/test_gpu_headline.py and bench.py compare against it.

Run: python tests/golden/make_c1_digest.py   (about a minute, single thread)
"""
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle.oracle import OracleQuery  # noqa: E402
from siddhi_amd import abi, digest, synth  # noqa: E402

SEND = 1000
B = (1 << 25) - (1 << 25) % SEND


def spec():
    schema = abi.Schema.parse("symbol string, price double, volume long, ts long")
    return schema, abi.QuerySpec(schema, "lengthBatch", 10000, group_by=["symbol"],
                                 aggs=[("sum", "volume"), ("avg", "price")], filter=(">", "price", 100),
                                 key_capacity=1000)


def main():
    schema, sp = spec()
    q = OracleQuery(sp)
    parts, res = [], {}
    t0 = time.time()
    for i in range(2):
        ts, cols = synth.c1_stock(i * B, B)
        parts.append(abi.out_arrays(q.push_raw(abi.HostBatch(schema, ts, cols, SEND))))
        a = abi.concat_arrays(parts)
        res[f"push0{'1' if i else ''}"] = {"sha256": digest.output_digest(a), "rows": int(a["ts"].size),
                                            "flushes": int(a["flush_clock"].size)}
        print(i, res, f"{time.time() - t0:.1f} s", flush=True)
    res["config"] = {"events_per_push": B, "send_size": SEND, "seed": 0xC1, "symbols": 1000,
                     "query": "StockStream[price > 100]#window.lengthBatch(10000) select symbol, sum(volume), "
                              "avg(price) group by symbol; symbol string",
                     "generator": "siddhi_amd.synth.c1_stock", "made_by": "tests/golden/make_c1_digest.py"}
    with open(os.path.join(HERE, "c1_bench_digest.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
