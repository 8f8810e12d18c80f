"""Sharded ingest of a timeBatch group-by query across G GPUs (one process per GPU).

Rank g holds slice g of every global micro-batch (a contiguous, send-aligned run of the stream).
The library (`sh_shard_*`, include/siddhi_hip.h) computes the global clock, nextEmitTime and the
window of every event from the all-gathered slice summaries, packs every passing event into the
run of the GPU that owns its key (owner = mix64(key) % G), and aggregates what an owner receives.
The exchange itself is done here, over `torch.distributed` — RCCL over xGMI with the `nccl`
backend on MI355X, or gloo on CPU tensors in the CPU tests:

    summaries  all_gather_into_tensor   7 x int64 per rank
    records    all_to_all_single        variable bytes per (source, owner), counts exchanged first
    bounds     all_gather               the window starts of every slice (few per push)

`LocalShards` runs G shards inside one process on one device, exchanging through device copies:
the same protocol without a transport (used by the single-GPU parity tests).
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import abi
from .runtime import Context, _check, default_context, lib

SUMMARY_WORDS = 7
BOUND_WORDS = 4


def _batch(n: int, ts_ptr: int, col_ptrs: Sequence[int], send_size: int) -> abi.Batch:
    b = abi.Batch()
    b.n = n
    b.send_size = send_size
    b.ts = ts_ptr
    for i, p in enumerate(col_ptrs):
        b.cols[i] = p
    return b


class ShardedQuery:
    """Rank `rank` of `world` of a sharded `from S[cond]#window.timeBatch(T) select k, aggs group by k`."""

    def __init__(self, spec: abi.QuerySpec, rank: int, world: int, ctx: Optional[Context] = None):
        self.spec, self.rank, self.world = spec, rank, world
        self.ctx = ctx or default_context()
        self._desc = spec.desc()
        self.h = C.c_void_p()
        _check(lib().sh_shard_create(self.ctx.h, C.byref(self._desc), rank, world, C.byref(self.h)))
        rb = C.c_int64()
        _check(lib().sh_shard_record_bytes(self.h, C.byref(rb)))
        self.record_bytes = rb.value

    def summarize(self, n: int, ts_ptr: int, col_ptrs: Sequence[int], send_size: int) -> np.ndarray:
        self._b = _batch(n, ts_ptr, col_ptrs, send_size)
        s = abi.SliceSummary()
        _check(lib().sh_shard_summarize(self.h, C.byref(self._b), C.byref(s)))
        return np.array([s.n, s.n_pass, s.max_tl, s.first_clock, s.first_key, s.ts_min, s.ts_max], dtype=np.int64)

    def pack(self, summaries: np.ndarray, send_ptr: int, send_cap: int) -> Tuple[np.ndarray, np.ndarray]:
        """summaries: [world, SUMMARY_WORDS] int64. Returns (send_bytes[world], bounds[k, 4] int64)."""
        summ = np.ascontiguousarray(summaries, dtype=np.int64).reshape(self.world, SUMMARY_WORDS)
        arr = (abi.SliceSummary * self.world)()
        for r in range(self.world):
            (arr[r].n, arr[r].n_pass, arr[r].max_tl, arr[r].first_clock, arr[r].first_key, arr[r].ts_min,
             arr[r].ts_max) = (int(x) for x in summ[r])
        sb = (C.c_int64 * self.world)()
        bp = C.POINTER(abi.Bound)()
        nb = C.c_int64()
        _check(lib().sh_shard_pack(self.h, arr, C.byref(self._b), send_ptr, send_cap, sb, C.byref(bp), C.byref(nb)))
        bounds = np.zeros((nb.value, BOUND_WORDS), dtype=np.int64)
        for i in range(nb.value):
            bounds[i] = (bp[i].W, bp[i].clock, bp[i].gidx, 0)
        return np.frombuffer(sb, dtype=np.int64).copy(), bounds

    def consume(self, recv_ptr: int, recv_bytes: Sequence[int], bounds: np.ndarray, host_out: bool = True):
        """Returns (sh_out pointer, order pointer): rows of this owner's keys."""
        rb = (C.c_int64 * self.world)(*[int(x) for x in recv_bytes])
        bd = np.ascontiguousarray(bounds, dtype=np.int64).reshape(-1, BOUND_WORDS)
        barr = (abi.Bound * max(1, len(bd)))()
        for i, row in enumerate(bd):
            barr[i].W, barr[i].clock, barr[i].gidx = int(row[0]), int(row[1]), int(row[2])
        out = C.POINTER(abi.Out)()
        order = C.POINTER(C.c_int64)()
        _check(lib().sh_shard_consume(self.h, recv_ptr, rb, barr, len(bd), int(host_out), C.byref(out),
                                      C.byref(order)))
        return out, order, self.flush_windows()

    def advance_time(self, now: int, host_out: bool = True):
        out = C.POINTER(abi.Out)()
        order = C.POINTER(C.c_int64)()
        _check(lib().sh_shard_advance_time(self.h, now, int(host_out), C.byref(out), C.byref(order)))
        return out, order, self.flush_windows()

    def flush_windows(self) -> np.ndarray:
        """The window each flush of the last consume / advance closes (sh_shard_flush_windows)."""
        w = C.POINTER(C.c_int64)()
        n = C.c_int64()
        _check(lib().sh_shard_flush_windows(self.h, C.byref(w), C.byref(n)))
        return np.ctypeslib.as_array(w, shape=(n.value,)).copy() if n.value else np.zeros(0, np.int64)

    def stats(self) -> abi.Stats:
        st = abi.Stats()
        _check(lib().sh_shard_stats(self.h, C.byref(st)))
        return st

    def snapshot(self) -> bytes:
        """This rank's checkpoint (sh_shard_snapshot), taken between pushes."""
        n = C.c_int64()
        _check(lib().sh_shard_snapshot(self.h, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        _check(lib().sh_shard_snapshot(self.h, buf, n.value, C.byref(n)))
        return buf.raw[:n.value]

    def restore(self, blob: bytes):
        _check(lib().sh_shard_restore(self.h, blob, len(blob)))

    def close(self):
        if self.h:
            lib().sh_shard_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ShardedAggregation(ShardedQuery):
    """Rank `rank` of `world` of a key-sharded `define aggregation ... every sec...year` (C4): the
    same three-phase ingest as ShardedQuery; this rank's roll-up tables hold the rows of its keys."""

    def __init__(self, spec: abi.AggregationSpec, rank: int, world: int, ctx: Optional[Context] = None):
        self.spec, self.rank, self.world = spec, rank, world
        self.ctx = ctx or default_context()
        self._desc = spec.desc()
        self.h = C.c_void_p()
        self.agg = C.c_void_p()
        _check(lib().sh_aggregation_shard_create(self.ctx.h, C.byref(self._desc), rank, world, C.byref(self.h),
                                                 C.byref(self.agg)))
        rb = C.c_int64()
        _check(lib().sh_shard_record_bytes(self.h, C.byref(rb)))
        self.record_bytes = rb.value

    def table_arrays(self, duration: int) -> dict:
        out = C.POINTER(abi.Out)()
        _check(lib().sh_aggregation_table(self.agg, duration, C.byref(out)))
        return abi.out_arrays(out)

    def close(self):
        if self.h:
            lib().sh_shard_destroy(self.h)  # releases the aggregation handle too
            self.h = None
            self.agg = None


def merge_tables(parts: List[dict]) -> dict:
    """Union of the owners' rows of one duration's table, in (bucket, key, values) order. An
    aggregation table is keyed by (AGG_TIMESTAMP, group key) (AggregationParser.initDefaultTables,
    @PrimaryKey), so its row order carries no meaning; compare tables in this canonical order."""
    keys = np.concatenate([p["keys"] for p in parts], axis=1)
    vals = np.concatenate([p["vals"] for p in parts], axis=1)
    nulls = np.concatenate([p["nulls"] for p in parts], axis=1)
    return canonical_table({"keys": keys, "vals": vals, "nulls": nulls})


def canonical_table(t: dict) -> dict:
    keys, vals, nulls = t["keys"], t["vals"], t["nulls"]
    cols = [vals.view(np.int64)[i] for i in range(vals.shape[0] - 1, -1, -1)]
    cols += [keys[i] for i in range(keys.shape[0] - 1, -1, -1)]
    perm = np.lexsort(cols) if keys.shape[1] else np.zeros(0, np.int64)
    return {"keys": keys[:, perm], "vals": vals[:, perm], "nulls": nulls[:, perm]}


def host_rows(out, order, windows=None) -> dict:
    """Host sh_out + order (+ the flushes' windows) -> out_arrays dict with an 'order' column."""
    d = abi.out_arrays(out)
    n = int(out.contents.n_rows)
    d["order"] = np.ctypeslib.as_array(order, shape=(n,)).copy() if n else np.zeros(0, np.int64)
    if windows is not None and len(windows) == len(d["flush_clock"]) and len(windows):
        d["window"] = np.asarray(windows, np.int64)
    return d


def merge_owner_outputs(parts: List[dict], bounds: Optional[np.ndarray] = None,
                        sends: Optional[Tuple[int, int]] = None) -> dict:
    """Merge the G owners' outputs of one global push into the single-stream output: flushes are
    matched by flush clock (every owner flushes window w at the same global clock) and, when `bounds`
    (the push's all-gathered window starts) is given, by the window their rows' first events fall in
    — several lengthBatch batches can complete in one send and share its clock. Sliding windows emit
    one flush per send (QuerySelector output per chunk, R8) and consecutive sends can share a clock:
    `sends` = (global index of the push's first event, send_size) keys their flushes by send number.
    Rows inside a flush are ordered by the global first-occurrence index."""
    if sends is not None:
        return _merge_by_send(parts, sends)
    starts = np.sort(np.asarray(bounds, np.int64).reshape(-1, BOUND_WORDS)[:, 2]) if bounds is not None \
        else np.zeros(0, np.int64)

    def fkey(p, f):
        a = int(p["flush_offsets"][f])
        if sends is not None:
            return (int(p["flush_clock"][f]), (int(p["order"][a]) - sends[0]) // max(1, sends[1]))
        if "window" in p:  # the window the owner's flush closes (sh_shard_flush_windows)
            return (int(p["flush_clock"][f]), int(p["window"][f]))
        w = int(np.searchsorted(starts, int(p["order"][a]), side="right")) if starts.size else 0
        return (int(p["flush_clock"][f]), w)

    keys = sorted(set(fkey(p, f) for p in parts for f in range(len(p["flush_clock"]))
                      if p["flush_offsets"][f + 1] > p["flush_offsets"][f]))
    fo, fc, rows = [0], [], []
    for ky in keys:
        ck = ky[0]
        sel = []
        for p in parts:
            for f in range(len(p["flush_clock"])):
                a, b = int(p["flush_offsets"][f]), int(p["flush_offsets"][f + 1])
                if b > a and fkey(p, f) == ky:
                    sel.append((p, a, b))
        order = np.concatenate([p["order"][a:b] for p, a, b in sel])
        perm = np.argsort(order, kind="stable")
        rows.append((sel, perm))
        fo.append(fo[-1] + len(perm))
        fc.append(ck)

    def gather(key, axis_rows=True):
        out = []
        for sel, perm in rows:
            if key in ("keys", "vals", "nulls"):
                cat = np.concatenate([p[key][:, a:b] for p, a, b in sel], axis=1)
                out.append(cat[:, perm])
            else:
                cat = np.concatenate([p[key][a:b] for p, a, b in sel])
                out.append(cat[perm])
        return out

    ref = parts[0]
    res = {"flush_offsets": np.array(fo, np.int64), "flush_clock": np.array(fc, np.int64),
           "val_types": ref["val_types"]}
    for key in ("ts", "expired", "order", "rep"):
        g = gather(key)
        res[key] = np.concatenate(g) if g else np.zeros(0, ref[key].dtype)
    for key in ("keys", "vals", "nulls"):
        g = gather(key)
        res[key] = np.concatenate(g, axis=1) if g else np.zeros((ref[key].shape[0], 0), ref[key].dtype)
    return res


class MergedRateLimiter:
    """`output … every …` of a sharded query: OutputRateLimiter.process sits after the selector, so it sees
    the merged single-stream output. The merging rank holds one never-pushed query of the same spec (its
    rate set) and passes every merged call output through it on its GPU (sh_rate_apply_merged)."""

    def __init__(self, spec, ctx: Optional[Context] = None):
        from siddhi_amd import runtime
        self.q = runtime.GpuQuery(spec, ctx)

    def apply(self, merged: dict) -> dict:
        return self.q.rate_apply_merged(merged)

    def close(self):
        self.q.close()


def merge_sends(spec, last_sends: Tuple[int, int]) -> Optional[Tuple[int, int]]:
    """The `sends` argument of merge_owner_outputs for a query: sliding windows and timeBatch(T, true) flush
    once per send (the send's chunk), lengthBatch(L, true) once per passing event (LengthBatchWindowProcessor
    sends each event's chunk on its own, :160-182); other batch windows merge by window (None)."""
    if spec.window == "time" or (spec.stream_current and spec.window == "timeBatch"):
        return last_sends
    if spec.stream_current and spec.window == "lengthBatch":
        return (last_sends[0], 1)
    return None


def _merge_by_send(parts: List[dict], sends: Tuple[int, int]) -> dict:
    """One flush per send: the global row order is the order of the rows' first events (rows of an
    earlier send come first), and a flush ends where the send number changes."""
    seq0, ss = int(sends[0]), max(1, int(sends[1]))
    ref = parts[0]
    order = np.concatenate([p["order"] for p in parts])
    clock = np.concatenate([np.repeat(p["flush_clock"], np.diff(p["flush_offsets"])) for p in parts])
    perm = np.argsort(order, kind="stable")
    order = order[perm]
    send = (order - seq0) // ss
    starts = np.flatnonzero(np.r_[True, send[1:] != send[:-1]]) if order.size else np.zeros(0, np.int64)
    res = {"flush_offsets": np.r_[starts, order.size].astype(np.int64),
           "flush_clock": clock[perm][starts].astype(np.int64), "val_types": ref["val_types"], "order": order}
    for key in ("ts", "expired", "rep"):
        res[key] = np.concatenate([p[key] for p in parts])[perm]
    for key in ("keys", "vals", "nulls"):
        res[key] = np.concatenate([p[key] for p in parts], axis=1)[:, perm]
    return res


class LocalShards:
    """G shards of one query in one process on one device; the exchange is a device copy.
    Drives exactly the protocol a multi-process run drives over torch.distributed."""

    def __init__(self, spec, world: int, ctx: Optional[Context] = None):
        cls = ShardedAggregation if isinstance(spec, abi.AggregationSpec) else ShardedQuery
        self.shards = [cls(spec, r, world, ctx) for r in range(world)]
        self.world = world
        self.seq = 0  # global stream index of the next push's first event

    def push(self, slices, send_size: int, device) -> List[dict]:
        """slices: per rank (ts tensor, [col tensors]) on `device`. Returns per-owner host outputs."""
        import torch
        G = self.world
        summ = np.stack([s.summarize(int(ts.numel()), ts.data_ptr(), [c.data_ptr() for c in cols], send_size)
                         for s, (ts, cols) in zip(self.shards, slices)])
        sends, counts, bounds = [], [], []
        for s, (ts, cols) in zip(self.shards, slices):
            cap = max(1, int(ts.numel()) * s.record_bytes)
            buf = torch.empty(cap, dtype=torch.uint8, device=device)
            sb, bd = s.pack(summ, buf.data_ptr(), cap)
            sends.append(buf)
            counts.append(sb)
            bounds.append(bd)
        all_bounds = np.concatenate(bounds) if bounds else np.zeros((0, BOUND_WORDS), np.int64)
        self.last_bounds = all_bounds
        self.last_send_bytes = int(sum(int(np.sum(c)) for c in counts))  # bytes the push exchanged
        self.last_sends = (self.seq, send_size)
        self.seq += sum(int(ts.numel()) for ts, _ in slices)
        outs = []
        for o, s in enumerate(self.shards):
            blocks, rbytes = [], []
            for g in range(G):
                start = int(counts[g][:o].sum())
                n = int(counts[g][o])
                blocks.append(sends[g][start:start + n])
                rbytes.append(n)
            recv = torch.cat(blocks) if sum(rbytes) else torch.empty(1, dtype=torch.uint8, device=device)
            torch.cuda.current_stream(device).synchronize()  # the library runs on its own HIP stream
            if isinstance(s, ShardedAggregation):  # rows go to the roll-up tables
                s.consume(recv.data_ptr(), rbytes, all_bounds, host_out=False)
                outs.append(None)
                continue
            out, order, windows = s.consume(recv.data_ptr(), rbytes, all_bounds, host_out=True)
            outs.append(host_rows(out, order, windows))
        return outs

    def advance_time(self, now: int) -> List[dict]:
        if isinstance(self.shards[0], ShardedAggregation):
            for s in self.shards:
                s.advance_time(now, False)
            return [None] * self.world
        return [host_rows(*s.advance_time(now, True)) for s in self.shards]

    def snapshot(self) -> List[bytes]:
        return [s.snapshot() for s in self.shards]

    def restore(self, blobs: List[bytes], seq: int):
        """Continue from snapshot() blobs; seq = global stream index of the next event."""
        for s, b in zip(self.shards, blobs):
            s.restore(b)
        self.seq = seq

    def tables(self, duration: int) -> dict:
        """The merged (canonical-order) table of one duration over all owners."""
        return merge_tables([s.table_arrays(duration) for s in self.shards])

    def close(self):
        for s in self.shards:
            s.close()


class TorchExchange:
    """The three collectives of a sharded push over torch.distributed (nccl = RCCL on ROCm, or gloo).
    Tensors live on `device` (a CUDA device for nccl, CPU for gloo)."""

    def __init__(self, device, group=None, separate_control: bool = True):
        """separate_control: the small collectives (slice summaries, window starts, record counts) run
        on a communicator of their own (dist.new_group, collective over `group`'s ranks), so the next
        push's summary all-gather does not queue behind the previous push's record all-to-all still
        in flight on the data communicator (PipelinedPush)."""
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.device = device
        self.world = dist.get_world_size(group)
        ranks = None if group is None else dist.get_process_group_ranks(group)
        self.ctrl = dist.new_group(ranks=ranks) if separate_control else group

    def all_gather_summaries(self, summary: np.ndarray) -> np.ndarray:
        import torch
        t = torch.as_tensor(summary, dtype=torch.int64).to(self.device)
        out = torch.empty(self.world * SUMMARY_WORDS, dtype=torch.int64, device=self.device)
        self.dist.all_gather_into_tensor(out, t, group=self.ctrl)
        return out.cpu().numpy().reshape(self.world, SUMMARY_WORDS)

    def all_to_all(self, send, send_bytes: np.ndarray):
        """send: uint8 tensor holding the per-owner runs back to back. Returns (recv tensor, recv_bytes)."""
        import torch
        sc = torch.as_tensor(np.asarray(send_bytes, dtype=np.int64)).to(self.device)
        rc = torch.empty_like(sc)
        self.dist.all_to_all_single(rc, sc, group=self.ctrl)
        recv_bytes = rc.cpu().numpy()
        total = int(recv_bytes.sum())
        recv = torch.empty(max(1, total), dtype=torch.uint8, device=self.device)
        used = int(np.asarray(send_bytes).sum())
        send = send[:used].to(self.device)
        self.dist.all_to_all_single(recv[:total], send, [int(x) for x in recv_bytes],
                                    [int(x) for x in send_bytes], group=self.group)
        return recv, recv_bytes

    def all_to_all_start(self, send, send_bytes: np.ndarray):
        """all_to_all with the record payload left in flight: (recv, recv_bytes, work); work.wait()
        before reading recv (the counts exchange is synchronous, it is 8 bytes per rank)."""
        import torch
        sc = torch.as_tensor(np.asarray(send_bytes, dtype=np.int64)).to(self.device)
        rc = torch.empty_like(sc)
        self.dist.all_to_all_single(rc, sc, group=self.ctrl)
        recv_bytes = rc.cpu().numpy()
        total = int(recv_bytes.sum())
        recv = torch.empty(max(1, total), dtype=torch.uint8, device=self.device)
        used = int(np.asarray(send_bytes).sum())
        send = send[:used].to(self.device)
        work = self.dist.all_to_all_single(recv[:total], send, [int(x) for x in recv_bytes],
                                           [int(x) for x in send_bytes], group=self.group, async_op=True)
        return recv, recv_bytes, (work, send)

    def all_gather_bounds(self, bounds: np.ndarray) -> np.ndarray:
        import torch
        n = torch.tensor([len(bounds)], dtype=torch.int64, device=self.device)
        ns = torch.empty(self.world, dtype=torch.int64, device=self.device)
        self.dist.all_gather_into_tensor(ns, n, group=self.ctrl)
        counts = ns.cpu().numpy()
        mx = int(counts.max())
        if mx == 0:
            return np.zeros((0, BOUND_WORDS), np.int64)
        pad = np.zeros((mx, BOUND_WORDS), np.int64)
        pad[:len(bounds)] = bounds
        t = torch.as_tensor(pad).to(self.device)
        out = torch.empty(self.world * mx * BOUND_WORDS, dtype=torch.int64, device=self.device)
        self.dist.all_gather_into_tensor(out, t.reshape(-1), group=self.ctrl)
        allb = out.cpu().numpy().reshape(self.world, mx, BOUND_WORDS)
        return np.concatenate([allb[r, :counts[r]] for r in range(self.world)])


def distributed_push(q: ShardedQuery, ex: TorchExchange, n: int, ts_ptr: int, col_ptrs: Sequence[int],
                     send_size: int, send_buf, host_out: bool = False, timings: Optional[dict] = None):
    """One global push on this rank: summarize -> all-gather -> pack -> all-to-all + all-gather ->
    consume. send_buf: uint8 device tensor of >= n * record_bytes bytes. `timings` (optional)
    accumulates wall milliseconds per phase (each phase ends in a host synchronisation anyway)."""
    import time
    import torch
    t0 = time.perf_counter()
    summ = q.summarize(n, ts_ptr, col_ptrs, send_size)
    all_summ = ex.all_gather_summaries(summ)
    t1 = time.perf_counter()
    send_bytes, bounds = q.pack(all_summ, send_buf.data_ptr(), int(send_buf.numel()))
    t2 = time.perf_counter()
    recv, recv_bytes = ex.all_to_all(send_buf, send_bytes)
    if recv.device != send_buf.device:  # host transport (gloo): the owner consumes device memory
        recv = recv.to(send_buf.device)
    all_bounds = ex.all_gather_bounds(bounds)
    torch.cuda.current_stream(send_buf.device).synchronize()  # recv was written on torch's stream
    t3 = time.perf_counter()
    res = q.consume(recv.data_ptr(), recv_bytes, all_bounds, host_out)
    q.last_bounds = all_bounds  # (the merge of the owners' outputs matches flushes by these)
    if timings is not None:
        t4 = time.perf_counter()
        for k, v in (("summarize", t1 - t0), ("pack", t2 - t1), ("exchange", t3 - t2), ("consume", t4 - t3)):
            timings[k] = timings.get(k, 0.0) + v * 1e3
        timings["bytes_sent"] = timings.get("bytes_sent", 0) + int(np.asarray(send_bytes).sum())
    return res


class PipelinedPush:
    """distributed_push with the record exchange of push i in flight while push i - 1 is consumed
    (the library keeps up to two packed pushes per shard, sh_shard_pack / sh_shard_consume FIFO).
    push() returns the output of the previous push (None for the first); finish() the last one.
    Two send buffers alternate: pack(i + 1) writes one while the exchange of i still reads the other."""

    def __init__(self, q: ShardedQuery, ex: TorchExchange, send_bufs, host_out: bool = False):
        self.q, self.ex, self.bufs, self.host_out = q, ex, list(send_bufs), host_out
        self.k = 0
        self.pending = None

    def push(self, n: int, ts_ptr: int, col_ptrs: Sequence[int], send_size: int, timings: Optional[dict] = None):
        import time
        t0 = time.perf_counter()
        summ = self.q.summarize(n, ts_ptr, col_ptrs, send_size)
        all_summ = self.ex.all_gather_summaries(summ)  # control communicator: not behind push i - 1's payload
        buf = self.bufs[self.k % len(self.bufs)]
        self.k += 1
        t1 = time.perf_counter()
        send_bytes, bounds = self.q.pack(all_summ, buf.data_ptr(), int(buf.numel()))
        t2 = time.perf_counter()
        all_bounds = self.ex.all_gather_bounds(bounds)
        recv, recv_bytes, work = self.ex.all_to_all_start(buf, send_bytes)
        t3 = time.perf_counter()
        res = self._consume_pending()  # push i - 1 aggregates while push i's records move
        self.pending = (recv, recv_bytes, all_bounds, work, buf.device)
        if timings is not None:
            t4 = time.perf_counter()
            for key, v in (("summarize", t1 - t0), ("pack", t2 - t1), ("exchange_start", t3 - t2),
                           ("consume_prev", t4 - t3)):
                timings[key] = timings.get(key, 0.0) + v * 1e3
            timings["bytes_sent"] = timings.get("bytes_sent", 0) + int(np.asarray(send_bytes).sum())
        return res

    def finish(self):
        return self._consume_pending()

    def _consume_pending(self):
        import torch
        if self.pending is None:
            return None
        recv, recv_bytes, all_bounds, (work, _send), dev = self.pending
        self.pending = None
        work.wait()
        if recv.device != dev:  # host transport (gloo)
            recv = recv.to(dev)
        torch.cuda.current_stream(dev).synchronize()
        res = self.q.consume(recv.data_ptr(), recv_bytes, all_bounds, self.host_out)
        self.q.last_bounds = all_bounds
        return res
