"""Two processes on the one GPU, world 2 over gloo, for the sharded shapes test_gpu_dist.py does not
cover: lengthBatch (C1: the batch index is global), partitioned timeBatch (C5: R12's first partition
is agreed from the slice summaries) and the incremental aggregation (C4: each owner's roll-up tables
hold its keys' rows). Each rank runs the library's real phases through siddhi_amd.shard.distributed_push
(the driver bench.py runs over RCCL), pipelined where the shape allows; the merged output (or the union
of the owners' tables) must equal the single-stream oracle's, bit for bit."""
import os
import pickle
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle.oracle import OracleAggregation, OracleQuery
from siddhi_amd import abi, synth
from tests.parity import assert_same, run_pushes

pytestmark = pytest.mark.gpu

C1 = abi.Schema.parse("symbol string, price double, volume long, ts long")
C2 = abi.Schema.parse("k int, v double, ts long")
C4 = abi.Schema.parse("k int, v double, et long")
N_PUSH, B = 3, 60_000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _case(shape):
    """(spec, per-push stream (ts, cols), send size)"""
    if shape == "lengthBatch":
        spec = abi.QuerySpec(C1, "lengthBatch", 997, group_by=["symbol"], aggs=[("sum", "volume"), ("avg", "price")],
                             filter=(">", "price", 100), key_capacity=1000)
        return spec, (lambda i: synth.c1_stock(i * B, B)), 100
    if shape == "partition":
        spec = abi.QuerySpec(C2, "timeBatch", 1000, group_by=["k"], aggs=[("sum", "v"), ("count", None)],
                             partition="k", key_capacity=4_000)
        def stream(i):
            ts, cols = synth.keyed_stream(i * B, B, 0xC5, 4_000, 30)
            cols[0] = (cols[0] * 7919 % 4_000).astype(cols[0].dtype)
            return ts, cols
        return spec, stream, 1
    spec = abi.AggregationSpec(C4, [("sum", "v"), ("avg", "v"), ("min", "v"), ("max", "v"), ("count", None)],
                               group_by=["k"], ts="et", durations=("sec", "hour"), key_capacity=2_000)
    def stream(i):
        ts, cols = synth.keyed_stream(i * B, B, 0xC4, 2_000, 40)
        cols[2] = ts - (np.arange(B) % 1500)  # event time lags the clock: late events hit old buckets
        return ts, cols
    return spec, stream, 9


def _worker(rank, world, port, shape, outdir):
    import torch
    import torch.distributed as dist
    from siddhi_amd.shard import (PipelinedPush, ShardedAggregation, ShardedQuery, TorchExchange,
                                  distributed_push, host_rows)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    spec, stream, send = _case(shape)
    agg = shape == "aggregation"
    q = ShardedAggregation(spec, rank, world) if agg else ShardedQuery(spec, rank, world)
    ex = TorchExchange(torch.device("cpu"))
    send_buf = torch.empty(B * q.record_bytes, dtype=torch.uint8, device=dev)
    pp = None if agg else PipelinedPush(q, ex, [send_buf, torch.empty_like(send_buf)], host_out=True)
    outs = []
    for i in range(N_PUSH):
        ts, cols = stream(i)
        cut = (int(B * (0.3 + 0.2 * i)) // send) * send  # uneven send-aligned slices
        lo, hi = (0, cut) if rank == 0 else (cut, B)
        t = torch.from_numpy(np.ascontiguousarray(ts[lo:hi])).to(dev)
        cs = [torch.from_numpy(np.ascontiguousarray(c[lo:hi])).to(dev) for c in cols]
        torch.cuda.synchronize()
        if agg:
            distributed_push(q, ex, hi - lo, t.data_ptr(), [c.data_ptr() for c in cs], send, send_buf, host_out=False)
            continue
        res = pp.push(hi - lo, t.data_ptr(), [c.data_ptr() for c in cs], send)
        if res is not None:
            outs.append((host_rows(*res), q.last_bounds))
    if agg:
        q.advance_time(int(ts[-1]) + 2 * 3_600_000, False)
        lo_d, hi_d = abi.DUR_NAMES[spec.durations[0]], abi.DUR_NAMES[spec.durations[1]]
        outs = {d: q.table_arrays(d) for d in range(lo_d, hi_d + 1)}
    else:
        res = pp.finish()
        outs.append((host_rows(*res), q.last_bounds))
    with open(os.path.join(outdir, f"rank{rank}.pkl"), "wb") as f:
        pickle.dump(outs, f)
    q.close()
    dist.barrier()
    dist.destroy_process_group()


def _run(shape):
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), shape, d), nprocs=world, join=True)
        per_rank = []
        for r in range(world):
            with open(os.path.join(d, f"rank{r}.pkl"), "rb") as f:
                per_rank.append(pickle.load(f))
    return per_rank


@pytest.mark.parametrize("shape", ["lengthBatch", "partition"])
def test_two_process_sharded_batch_shapes_match_oracle(shape):
    from siddhi_amd.shard import merge_owner_outputs
    per_rank = _run(shape)
    spec, stream, send = _case(shape)
    parts = [merge_owner_outputs([per_rank[r][i][0] for r in range(2)], per_rank[0][i][1]) for i in range(N_PUSH)]
    got = abi.concat_arrays(parts)
    o = OracleQuery(spec)
    want = run_pushes(o, [abi.HostBatch(spec.schema, *stream(i), send) for i in range(N_PUSH)])
    o.close()
    assert_same(got, want, label=f"2-process {shape}")
    assert got["flush_offsets"].size > 3


def test_two_process_sharded_aggregation_matches_oracle():
    from siddhi_amd.shard import canonical_table, merge_tables
    per_rank = _run("aggregation")
    spec, stream, send = _case("aggregation")
    o = OracleAggregation(spec)
    last = None
    for i in range(N_PUSH):
        ts, cols = stream(i)
        o.push(abi.HostBatch(spec.schema, ts, cols, send))
        last = int(ts[-1])
    o.advance_time(last + 2 * 3_600_000)
    rows = 0
    for d in per_rank[0]:
        got = merge_tables([per_rank[0][d], per_rank[1][d]])
        want = canonical_table(abi.out_arrays(o.table_raw(d)))
        assert np.array_equal(got["keys"], want["keys"]), f"duration {d}: (bucket, key) rows differ"
        assert np.array_equal(got["vals"], want["vals"]), f"duration {d}: base values differ"
        rows += want["keys"].shape[-1]
    o.close()
    assert rows > 1000
