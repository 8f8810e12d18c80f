"""CPU, world_size 2 over gloo: the transport of the sharded ingest (siddhi_amd.shard.TorchExchange)
— summaries all-gather, variable-size record all-to-all, bound all-gather — and the merge of the
owners' outputs. The records are packed here the way k_shard_pack packs them (per-owner runs in
stream order); on the GPU the same calls run over RCCL (backend nccl)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_total, q):
    import torch.distributed as dist
    from siddhi_amd.shard import TorchExchange
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ex = TorchExchange(torch.device("cpu"))
        rng = np.random.default_rng(11)
        keys = rng.integers(0, 97, size=n_total)
        cut = [0, n_total // 3, n_total]  # uneven slices
        lo, hi = cut[rank], cut[rank + 1]
        summ = np.array([hi - lo, rank, 100 + rank, -rank, 7, 5 - rank, 9 + rank], np.int64)
        allsumm = ex.all_gather_summaries(summ)
        assert allsumm.shape == (world, 7) and list(allsumm[:, 2]) == [100, 101] and list(allsumm[:, 6]) == [9, 10]
        # records: (gidx, key) int64 pairs, grouped by owner = key % world in stream order
        gidx = np.arange(lo, hi)
        k = keys[lo:hi]
        runs = [np.stack([gidx[k % world == o], k[k % world == o]], 1) for o in range(world)]
        send = torch.from_numpy(np.concatenate(runs).astype(np.int64).view(np.uint8).reshape(-1).copy())
        send_bytes = np.array([r.nbytes for r in runs], np.int64)
        recv, recv_bytes = ex.all_to_all(send, send_bytes)
        got = recv[:int(recv_bytes.sum())].numpy().view(np.int64).reshape(-1, 2)
        mine = np.nonzero(keys % world == rank)[0]
        assert np.array_equal(got[:, 0], mine), "owner must receive its keys' events in global order"
        assert np.array_equal(got[:, 1], keys[mine])
        bounds = np.array([[rank * 10 + i, 5, lo + i, 0] for i in range(rank + 1)], np.int64)
        allb = ex.all_gather_bounds(bounds)
        assert allb.shape == (3, 4) and sorted(allb[:, 0].tolist()) == [0, 10, 11]
        empty = ex.all_gather_bounds(np.zeros((0, 4), np.int64))
        assert empty.shape == (0, 4)
        q.put((rank, "ok"))
    except Exception as e:  # report to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def test_torch_exchange_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, 5000, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert res == {0: "ok", 1: "ok"}, res


def test_merge_owner_outputs_orders_rows_by_first_occurrence():
    from siddhi_amd.shard import merge_owner_outputs

    def part(fo, fc, order, keys):
        n = len(order)
        return {"flush_offsets": np.array(fo, np.int64), "flush_clock": np.array(fc, np.int64),
                "val_types": np.array([2], np.int32), "ts": np.array(order, np.int64) * 10,
                "expired": np.zeros(n, np.uint8), "order": np.array(order, np.int64),
                "rep": np.array(order, np.int64) + 1,
                "keys": np.array([keys], np.int64), "vals": np.array([keys], np.uint64),
                "nulls": np.zeros((1, n), np.uint8)}

    a = part([0, 2, 3], [1000, 2000], [0, 5, 7], [1, 3, 1])
    b = part([0, 1], [2000], [6], [2])
    m = merge_owner_outputs([a, b])
    assert m["flush_offsets"].tolist() == [0, 2, 4]
    assert m["flush_clock"].tolist() == [1000, 2000]
    assert m["keys"][0].tolist() == [1, 3, 2, 1]
    assert m["order"].tolist() == [0, 5, 6, 7]
    assert m["rep"].tolist() == [1, 6, 7, 8]


def test_merge_owner_outputs_separates_batches_of_one_send():
    """lengthBatch: two batches completing in one send share its flush clock; the window starts
    (bounds) keep them apart."""
    from siddhi_amd.shard import BOUND_WORDS, merge_owner_outputs

    def part(fo, fc, order, keys):
        n = len(order)
        return {"flush_offsets": np.array(fo, np.int64), "flush_clock": np.array(fc, np.int64),
                "val_types": np.array([2], np.int32), "ts": np.array(order, np.int64),
                "expired": np.zeros(n, np.uint8), "order": np.array(order, np.int64),
                "rep": np.array(order, np.int64) + 1,
                "keys": np.array([keys], np.int64), "vals": np.array([keys], np.uint64),
                "nulls": np.zeros((1, n), np.uint8)}

    # batch 0 = events [0, 4), batch 1 = [4, 8): both closed by the same send (clock 500)
    a = part([0, 1, 2], [500, 500], [1, 5], [10, 10])
    b = part([0, 2, 3], [500, 500], [0, 2, 4], [11, 12, 11])
    bounds = np.array([[1, 500, 4, 0], [2, 500, 8, 0]], np.int64).reshape(-1, BOUND_WORDS)
    m = merge_owner_outputs([a, b], bounds)
    assert m["flush_offsets"].tolist() == [0, 3, 5]
    assert m["order"].tolist() == [0, 1, 2, 4, 5]
    assert m["keys"][0].tolist() == [11, 10, 12, 11, 10]
