"""Checkpoint of a sharded query (sh_shard_snapshot / sh_shard_restore, SnapshotService.persist/restore):
G shards snapshotted between two global pushes and restored into fresh shards (new device state) must
continue exactly like the single-stream oracle does over the whole stream."""
import numpy as np
import pytest

from siddhi_amd import abi
from tests.parity import assert_same
from tests.test_gpu_shard import SCHEMA, run_oracle, spec, stream_pushes

pytestmark = pytest.mark.gpu


def run_sharded_restored(sp, world, pushes, send_size, cut_at, advance=None):
    import torch
    from siddhi_amd.shard import LocalShards, merge_owner_outputs, merge_sends
    dev = torch.device("cuda", 0)
    ls = LocalShards(sp, world)
    parts = []
    for pi, (ts, cols) in enumerate(pushes):
        if pi == cut_at:  # checkpoint, drop every shard, continue on restored ones
            blobs, seq = ls.snapshot(), ls.seq
            ls.close()
            ls = LocalShards(sp, world)
            ls.restore(blobs, seq)
        n = len(ts)
        units = (n + send_size - 1) // send_size
        edges = [0] + sorted(min(n, int(units * (g + 1) / world) * send_size) for g in range(world - 1)) + [n]
        slices = [(torch.from_numpy(np.ascontiguousarray(ts[edges[g]:edges[g + 1]])).to(dev),
                   [torch.from_numpy(np.ascontiguousarray(c[edges[g]:edges[g + 1]])).to(dev) for c in cols])
                  for g in range(world)]
        outs = ls.push(slices, send_size, dev)
        parts.append(merge_owner_outputs(outs, ls.last_bounds, merge_sends(sp, ls.last_sends)))
    if advance is not None:
        parts.append(merge_owner_outputs(ls.advance_time(advance)))
    ls.close()
    return abi.concat_arrays(parts)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("cut_at", [1, 2])
def test_sharded_timebatch_checkpoint(world, cut_at):
    sp = spec(5_000)
    pushes = stream_pushes(300_000, [90_000, 60_001, 149_999], 0xC2, 5_000, 100)
    adv = int(pushes[-1][0][-1]) + 5000
    got = run_sharded_restored(sp, world, pushes, 1, cut_at, advance=adv)
    assert_same(got, run_oracle(sp, pushes, 1, advance=adv), label=f"timeBatch x{world} cut {cut_at}")


def test_sharded_lengthbatch_checkpoint():
    sp = abi.QuerySpec(SCHEMA, "lengthBatch", 777, group_by=["k"], aggs=[("sum", "v"), ("count", None)],
                       key_capacity=2_000)
    pushes = stream_pushes(120_000, [50_000, 3_333, 66_667], 7, 2_000, 50)
    got = run_sharded_restored(sp, 2, pushes, 3, 1)
    assert_same(got, run_oracle(sp, pushes, 3), label="lengthBatch x2")


@pytest.mark.parametrize("window,param,send_size", [("timeBatch", 600, 4), ("lengthBatch", 333, 1)])
def test_sharded_stream_current_checkpoint(window, param, send_size):
    """stream.current.event owners keep their open batch's entries (the running values) across the cut"""
    sp = abi.QuerySpec(SCHEMA, window, param, group_by=["k"], aggs=[("sum", "v"), ("count", None), ("min", "v")],
                       stream_current=True, key_capacity=2_000)
    pushes = stream_pushes(90_000, [30_001, 29_999, 30_000], 13, 2_000, 40)
    adv = int(pushes[-1][0][-1]) + 3_000
    got = run_sharded_restored(sp, 3, pushes, send_size, 1, advance=adv)
    assert_same(got, run_oracle(sp, pushes, send_size, advance=adv), label=f"stream.current {window} x3")


def test_sharded_sliding_checkpoint():
    sp = abi.QuerySpec(SCHEMA, "time", 400, group_by=["k"], aggs=[("sum", "v"), ("max", "v")], key_capacity=1_000)
    pushes = stream_pushes(60_000, [20_000, 20_000, 20_000], 11, 1_000, 20)
    got = run_sharded_restored(sp, 2, pushes, 1, 2)
    assert_same(got, run_oracle(sp, pushes, 1), label="time x2")


def test_sharded_partitioned_checkpoint():
    sch = abi.Schema.parse("k int, p int, v double, ts long")
    sp = abi.QuerySpec(sch, "timeBatch", 500, group_by=["k"], aggs=[("count", None), ("avg", "v")], partition="p",
                       key_capacity=1_000)
    rng = np.random.default_rng(5)
    n = 80_000
    ts = (np.arange(n) // 30 + 10_000).astype(np.int64)
    cols = [rng.integers(0, 500, n).astype(np.int32), rng.integers(0, 4, n).astype(np.int32),
            rng.integers(-999, 999, n).astype(np.float64) / 8, ts.copy()]
    pushes = [(ts[a:b], [c[a:b] for c in cols]) for a, b in ((0, 30_000), (30_000, 50_000), (50_000, n))]
    adv = int(ts[-1]) + 2_000
    got = run_sharded_restored(sp, 2, pushes, 1, 1, advance=adv)
    assert_same(got, run_oracle(sp, pushes, 1, advance=adv), label="partitioned x2")


def test_sharded_snapshot_rejects_other_rank():
    from siddhi_amd.runtime import SiddhiError
    from siddhi_amd.shard import ShardedQuery
    sp = spec(100)
    a, b = ShardedQuery(sp, 0, 2), ShardedQuery(sp, 1, 2)
    with pytest.raises(SiddhiError, match="different shard"):
        b.restore(a.snapshot())
    a.close()
    b.close()


def test_truncated_shard_blob_leaves_shard_unchanged():
    """sh_shard_restore from a truncated blob fails without touching the shard: the rank's global
    stream state is applied only after its owner restored, and a failure rolls both back."""
    import torch
    from siddhi_amd.shard import LocalShards, merge_owner_outputs
    sp = spec(4_000)
    pushes = stream_pushes(90_000, [30_000, 30_000, 30_000], 0xC2, 4_000, 100)
    dev = torch.device("cuda", 0)
    ls = LocalShards(sp, 2)
    parts = []
    for pi, (ts, cols) in enumerate(pushes):
        if pi == 1:
            blobs = ls.snapshot()
            for g, sh in enumerate(ls.shards):
                for cut in (40, len(blobs[g]) // 2, len(blobs[g]) - 5):
                    with pytest.raises(Exception, match="truncated|does not match|restore"):
                        sh.restore(blobs[g][:cut])
        n = len(ts)
        half = (n // 2)
        slices = [(torch.from_numpy(np.ascontiguousarray(ts[a:b])).to(dev),
                   [torch.from_numpy(np.ascontiguousarray(c[a:b])).to(dev) for c in cols])
                  for a, b in ((0, half), (half, n))]
        outs = ls.push(slices, 1, dev)
        parts.append(merge_owner_outputs(outs, ls.last_bounds, None))
    ls.close()
    assert_same(abi.concat_arrays(parts), run_oracle(sp, pushes, 1), label="shard after failed restores")


@pytest.mark.parametrize("window,output", [("timeBatch", "all"), ("lengthBatch", "expired")])
def test_sharded_expired_output_checkpoint(window, output):
    """the carried batch (its keys, representative events and global order) survives the checkpoint"""
    sp = abi.QuerySpec(SCHEMA, window, 1000 if window == "timeBatch" else 1_500, group_by=["k"],
                       aggs=[("count", None), ("sum", "v")], key_capacity=2_000, output=output)
    pushes = stream_pushes(120_000, [50_000, 3_333, 66_667], 0xE5, 2_000, 40)
    adv = int(pushes[-1][0][-1]) + 5000 if window == "timeBatch" else None
    got = run_sharded_restored(sp, 3, pushes, 1, 1, advance=adv)
    assert_same(got, run_oracle(sp, pushes, 1, advance=adv), label=f"{window} {output} ckpt")
