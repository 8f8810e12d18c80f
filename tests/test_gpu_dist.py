"""Two processes on the one GPU, world 2 over gloo: the sharded query's real library phases
(sh_shard_summarize -> all-gather -> sh_shard_pack -> all-to-all -> sh_shard_consume) driven by
siddhi_amd.shard.distributed_push, exactly as bench.py runs them over RCCL on N GPUs. Rank r ingests
slice r of every global push; the owners' merged output must equal the single-stream oracle's
(timeBatch group-by: flushes, clocks, row order by global first occurrence, bit-identical values)."""
import os
import pickle
import socket
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle.oracle import OracleQuery
from siddhi_amd import abi, synth
from tests.parity import assert_same, run_pushes

pytestmark = pytest.mark.gpu

SCHEMA = abi.Schema.parse("k int, v double, ts long")
N_PUSH, B, KEYS, SEND = 3, 90_000, 3_000, 7


def _spec(window):
    if window == "time":
        return abi.QuerySpec(SCHEMA, "time", 700, group_by=["k"],
                             aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=KEYS)
    return abi.QuerySpec(SCHEMA, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=KEYS)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, window, outdir, pipelined=False):
    import torch
    import torch.distributed as dist
    from siddhi_amd.shard import PipelinedPush, ShardedQuery, TorchExchange, distributed_push, host_rows
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    q = ShardedQuery(_spec(window), rank, world)
    ex = TorchExchange(torch.device("cpu"))
    send_buf = torch.empty(B * q.record_bytes, dtype=torch.uint8, device=dev)
    pp = PipelinedPush(q, ex, [send_buf, torch.empty_like(send_buf)], host_out=True) if pipelined else None
    outs = []
    for i in range(N_PUSH):
        ts, cols = synth.keyed_stream(i * B, B, 0xD2, KEYS, 20)
        # send-aligned uneven slices: rank 0 the first 40 %, rank 1 the rest
        cut = (int(B * 0.4) // SEND) * SEND
        lo, hi = (0, cut) if rank == 0 else (cut, B)
        t = torch.from_numpy(np.ascontiguousarray(ts[lo:hi])).to(dev)
        cs = [torch.from_numpy(np.ascontiguousarray(c[lo:hi])).to(dev) for c in cols]
        torch.cuda.synchronize()
        if pp is not None:  # the output of push i - 1 comes back while push i is exchanged
            res = pp.push(hi - lo, t.data_ptr(), [c.data_ptr() for c in cs], SEND)
            if res is not None:
                outs.append((host_rows(*res), q.last_bounds, ((i - 1) * B, SEND)))
            continue
        res = distributed_push(q, ex, hi - lo, t.data_ptr(), [c.data_ptr() for c in cs], SEND, send_buf,
                               host_out=True)
        outs.append((host_rows(*res), q.last_bounds, (i * B, SEND)))
    if pp is not None:
        res = pp.finish()
        outs.append((host_rows(*res), q.last_bounds, ((N_PUSH - 1) * B, SEND)))
    with open(os.path.join(outdir, f"rank{rank}.pkl"), "wb") as f:
        pickle.dump(outs, f)
    q.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("pipelined", [False, True])
@pytest.mark.parametrize("window", ["timeBatch", "time"])
def test_two_process_sharded_push_matches_oracle(window, pipelined):
    """pipelined: PipelinedPush, the exchange of push i overlapping the consume of push i - 1."""
    from siddhi_amd.shard import merge_owner_outputs
    world = 2
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), window, d, pipelined), nprocs=world, join=True)
        per_rank = []
        for r in range(world):
            with open(os.path.join(d, f"rank{r}.pkl"), "rb") as f:
                per_rank.append(pickle.load(f))
    parts = []
    for i in range(N_PUSH):
        owner_outs = [per_rank[r][i] for r in range(world)]
        parts.append(merge_owner_outputs([o[0] for o in owner_outs], owner_outs[0][1],
                                         owner_outs[0][2] if window == "time" else None))
    got = abi.concat_arrays(parts)
    o = OracleQuery(_spec(window))
    pushes = []
    for i in range(N_PUSH):
        ts, cols = synth.keyed_stream(i * B, B, 0xD2, KEYS, 20)
        pushes.append(abi.HostBatch(SCHEMA, ts, cols, SEND))
    want = run_pushes(o, pushes)
    o.close()
    assert_same(got, want, label=f"2-process {window} pipelined={pipelined}")
    assert got["flush_offsets"].size > 5
