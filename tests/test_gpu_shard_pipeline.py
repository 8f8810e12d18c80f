"""Two packed pushes in flight per shard (sh_shard_pack / sh_shard_consume FIFO, PipelinedPush): every
shard packs push i before the owners consume push i - 1, as when the record exchange of push i
overlaps the consume of push i - 1. The merged output must still equal the single-stream oracle."""
import numpy as np
import pytest

from siddhi_amd import abi
from tests.parity import assert_same
from tests.test_gpu_shard import SCHEMA, run_oracle, spec, stream_pushes

pytestmark = pytest.mark.gpu


def run_pipelined(sp, world, pushes, send_size, advance=None):
    import torch
    from siddhi_amd.shard import ShardedQuery, host_rows, merge_owner_outputs
    dev = torch.device("cuda", 0)
    shards = [ShardedQuery(sp, r, world) for r in range(world)]
    parts, pending, seq = [], None, 0

    def consume(p):
        sends, counts, all_bounds, sends_meta = p
        outs = []
        for o, s in enumerate(shards):
            blocks, rbytes = [], []
            for g in range(world):
                start = int(counts[g][:o].sum())
                n = int(counts[g][o])
                blocks.append(sends[g][start:start + n])
                rbytes.append(n)
            recv = torch.cat(blocks) if sum(rbytes) else torch.empty(1, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            outs.append(host_rows(*s.consume(recv.data_ptr(), rbytes, all_bounds, True)))
        return merge_owner_outputs(outs, all_bounds, sends_meta if sp.window == "time" else None)

    for ts, cols in pushes:
        n = len(ts)
        units = (n + send_size - 1) // send_size
        edges = [0] + sorted(min(n, int(units * (g + 1) / world) * send_size) for g in range(world - 1)) + [n]
        slices = [(torch.from_numpy(np.ascontiguousarray(ts[edges[g]:edges[g + 1]])).to(dev),
                   [torch.from_numpy(np.ascontiguousarray(c[edges[g]:edges[g + 1]])).to(dev) for c in cols])
                  for g in range(world)]
        summ = np.stack([s.summarize(int(t.numel()), t.data_ptr(), [c.data_ptr() for c in cs], send_size)
                         for s, (t, cs) in zip(shards, slices)])
        sends, counts, bounds = [], [], []
        for s, (t, cs) in zip(shards, slices):
            cap = max(1, int(t.numel()) * s.record_bytes)
            buf = torch.empty(cap, dtype=torch.uint8, device=dev)
            sb, bd = s.pack(summ, buf.data_ptr(), cap)
            sends.append(buf)
            counts.append(sb)
            bounds.append(bd)
        cur = (sends, counts, np.concatenate(bounds), (seq, send_size))
        seq += n
        if pending is not None:  # push i - 1 is consumed after push i was packed
            parts.append(consume(pending))
        pending = cur
    parts.append(consume(pending))
    if advance is not None:
        parts.append(merge_owner_outputs([host_rows(*s.advance_time(advance, True)) for s in shards]))
    for s in shards:
        s.close()
    return abi.concat_arrays(parts)


@pytest.mark.parametrize("world", [2, 3])
def test_two_in_flight_timebatch(world):
    sp = spec(4_000)
    pushes = stream_pushes(250_000, [80_000, 1, 90_000, 79_999], 0xC2, 4_000, 100)
    adv = int(pushes[-1][0][-1]) + 5000
    assert_same(run_pipelined(sp, world, pushes, 1, advance=adv), run_oracle(sp, pushes, 1, advance=adv),
                label=f"pipelined timeBatch x{world}")


def test_two_in_flight_lengthbatch_and_sliding():
    sp = abi.QuerySpec(SCHEMA, "lengthBatch", 501, group_by=["k"], aggs=[("sum", "v"), ("count", None)],
                       key_capacity=2_000)
    pushes = stream_pushes(100_000, [40_000, 3_333, 56_667], 7, 2_000, 50)
    assert_same(run_pipelined(sp, 2, pushes, 3), run_oracle(sp, pushes, 3), label="pipelined lengthBatch")
    sp = abi.QuerySpec(SCHEMA, "time", 300, group_by=["k"], aggs=[("sum", "v"), ("max", "v")], key_capacity=1_000)
    pushes = stream_pushes(60_000, [20_000, 20_000, 20_000], 11, 1_000, 20)
    assert_same(run_pipelined(sp, 2, pushes, 1), run_oracle(sp, pushes, 1), label="pipelined time")


def test_third_pack_refused():
    import torch
    from siddhi_amd.runtime import SiddhiError
    from siddhi_amd.shard import ShardedQuery
    dev = torch.device("cuda", 0)
    q = ShardedQuery(spec(100), 0, 1)
    ts, cols = stream_pushes(3_000, [1_000, 1_000, 1_000], 3, 100, 10)[0]
    t = torch.from_numpy(ts).to(dev)
    cs = [torch.from_numpy(np.ascontiguousarray(c)).to(dev) for c in cols]
    buf = torch.empty(len(ts) * q.record_bytes, dtype=torch.uint8, device=dev)
    for i in range(3):
        summ = q.summarize(len(ts), t.data_ptr(), [c.data_ptr() for c in cs], 1)[None, :]
        if i < 2:
            q.pack(summ, buf.data_ptr(), int(buf.numel()))
        else:
            with pytest.raises(SiddhiError, match="two packed pushes"):
                q.pack(summ, buf.data_ptr(), int(buf.numel()))
    q.close()
