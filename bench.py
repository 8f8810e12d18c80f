#!/usr/bin/env python3
"""bench.py — events/sec of the MI355X windowed group-by path (BASELINE.json metric).

Workload (BASELINE.json configs[1], the configuration the metric is quoted on for one GPU):
  C2: `@app:playback from S#window.timeBatch(1 sec) select k, count(), min(v), max(v), avg(v)
       group by k insert into O` over (k int, v double, ts long), 100k uniform keys,
       1,000,000 events per event-time second, one InputHandler.send per event (PER_EVENT clock).
A step = one sh_push_device of `--batch` events (inputs already resident in HBM; the window state,
key table and outputs stay on the device).

N > 1 (`--ingest slice`, the default; north_star / SURVEY.md §8e): ONE global stream with N x the
keys and N x the event rate; every step each rank ingests a contiguous slice of `--batch` events,
the global clock / windows are agreed from all-gathered slice summaries, and every event is
re-keyed to the GPU owning its key over an RCCL all-to-all (xGMI), then aggregated by its owner
(sh_shard_*). Per-GPU work equals the N = 1 configuration (weak scaling). `--ingest keyed` instead
gives each rank its own pre-partitioned stream (no data-path collective).

Launch: python bench.py [--gpus 1 --steps K --warmup W]
   or:  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "events/sec (node) windowed group-by agg at 1/2/4/8 GPUs; % HBM roofline"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)
C2_BYTES_PER_EVENT = 24.4  # 20 B/event in + 100k rows x 44 B per 1M-event window


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--batch", type=int, default=1 << 25, help="events per step (per GPU)")
    ap.add_argument("--keys", type=int, default=100_000)
    ap.add_argument("--keys-total", type=int, default=0,
                    help="N > 1 slice ingest (and --shard-loopback): the global key count (default N x --keys; "
                         "north_star's 8-GPU target is the 1M-key timeBatch: --keys-total 1000000)")
    ap.add_argument("--shard-loopback", type=int, default=0, metavar="G",
                    help="one GPU: the sharded C2 pipeline of G owners (summarize, pack, exchange = device copy, "
                         "consume), each owner ingesting --batch events per step; per-phase ms per owner-step")
    ap.add_argument("--events-per-ms", type=int, default=1000)
    ap.add_argument("--send-size", type=int, default=1, help="events per InputHandler.send (1 = PER_EVENT)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="budget of the oracle CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-fed (PCIe) leg of the default line")
    ap.add_argument("--no-pipeline", action="store_true",
                    help="N > 1 slice ingest: exchange and consume each push in turn (no overlap)")
    ap.add_argument("--ingest", choices=["slice", "keyed"], default="slice",
                    help="N>1: slice = one global stream re-keyed over RCCL all-to-all; keyed = per-rank streams")
    ap.add_argument("--key-type", choices=["string", "int"], default="string",
                    help="k as a dictionary-encoded string (ids are dense key slots) or as an int (hashed)")
    ap.add_argument("--workload", choices=["c2", "c1", "c3", "c4", "c5", "ext", "c2all", "c2cur", "c3all", "plb", "plg"],
                    default="c2",
                    help="c2 = the headline (BASELINE configs[1]); c1/c3/c4/ext = secondary single-GPU lines; "
                         "c2all / c3all = C2 / C3 with `insert all events` (expired rows too), c2cur = C2 with "
                         "timeBatch(1 sec, true) (stream.current.event)")
    ap.add_argument("--host", action="store_true",
                    help="C2 from pinned host batches: double-buffered sh_stage / sh_push_staged, rows copied back "
                         "(PCIe-inclusive rate, H2D GB/s, per-call latency); never the headline value")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="torch.distributed backend (nccl = RCCL over xGMI; gloo only to rehearse N>1 on one GPU)")
    return ap.parse_args()


def cpu_baseline(args):
    """Time the C++ restatement (oracle/, single thread) on a bounded sample of the same workload."""
    import numpy as np
    from oracle.oracle import OracleQuery
    from siddhi_amd import abi, synth
    schema = abi.Schema.parse(f"k {args.key_type}, v double, ts long")
    spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=args.keys)
    q = OracleQuery(spec)
    n_done, t_used, chunk = 0, 0.0, 500_000
    while t_used < args.cpu_seconds and n_done < 60_000_000:
        ts, cols = synth.keyed_stream(n_done, chunk, 0xC2, args.keys, args.events_per_ms)
        b = abi.HostBatch(schema, ts, cols, args.send_size)
        t0 = time.perf_counter()
        q.push_raw(b)
        t_used += time.perf_counter() - t0
        n_done += chunk
    q.close()
    return {"value": n_done / t_used, "unit": "events/s", "cores": 1, "kind": "port",
            "sample": f"{n_done} events of the same C2 stream (seed 0xC2, {args.keys} keys, per-event sends), "
                      f"{t_used:.1f} s single-thread in the C++ restatement (oracle/), not stock Siddhi (no JVM)"}


def _cpu_shard_worker(job):
    """All-cores baseline, one worker: its key-hash shard (id % P == i) of the C2 sample stream through
    its own oracle runtime (P runtimes on disjoint key-hash shards). Only push_raw is timed."""
    key_type, keys, epm, send_size, seconds, P, i = job
    from oracle.oracle import OracleQuery
    from siddhi_amd import abi, synth
    schema = abi.Schema.parse(f"k {key_type}, v double, ts long")
    spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=keys)
    q = OracleQuery(spec)
    n_done, t_used, pos, chunk = 0, 0.0, 0, 1_000_000
    while t_used < seconds and pos < 400_000_000:
        ts, cols = synth.keyed_stream(pos, chunk, 0xC2, keys, epm)
        m = (cols[0] % P) == i
        b = abi.HostBatch(schema, ts[m], [c[m] for c in cols], send_size)
        t0 = time.perf_counter()
        q.push_raw(b)
        t_used += time.perf_counter() - t0
        n_done += int(m.sum())
        pos += chunk
    q.close()
    return n_done, t_used, pos


def cpu_baseline_all_cores(args, pool, P):
    """P oracle runtimes in parallel worker processes (started before the GPU was touched), each on
    its key-hash shard; rate = the shards' events / the slowest shard's push time."""
    t0 = time.perf_counter()
    res = pool.map(_cpu_shard_worker, [(args.key_type, args.keys, args.events_per_ms, args.send_size,
                                        max(1.0, args.cpu_seconds / 4), P, i) for i in range(P)])
    wall = time.perf_counter() - t0
    n = sum(r[0] for r in res)
    t = max(r[1] for r in res)
    return {"value": n / t, "unit": "events/s", "cores": P, "kind": "port",
            "sample": f"{n} events: the first {max(r[2] for r in res)} events (at most) of the same C2 stream split into {P} "
                      f"key-hash shards (id % {P}), each through its own oracle runtime in its own process; "
                      f"slowest shard {t:.1f} s of push time ({wall:.1f} s wall with stream generation)"}


# The PMC summary the roofline's `traffic` is read from: collected on exactly the default C2
# configuration with the current kernels (scripts/gpu_run.sh r6final pmc=c2 + scripts/pmc_summary.py).
TRAFFIC_SUMMARY = "profiles/r06_final_c2_pmc.json"
TRAFFIC_KERNEL = "shd::k_aggregate_own"


def measured_traffic(args, sliced):
    """HBM bytes per launch of the dominant kernel and of the whole push from TRAFFIC_SUMMARY
    (FETCH_SIZE x 2 + WRITE_SIZE per launch, gfx950-corrected), valid only for the default
    single-GPU configuration it was collected on."""
    if sliced or args.batch != 1 << 25 or args.keys != 100_000 or args.key_type != "string" or args.send_size != 1:
        return None, None
    try:
        ks = json.load(open(os.path.join(ROOT, TRAFFIC_SUMMARY)))["kernels"]
    except (OSError, ValueError, KeyError):
        return None, None
    main = next((v["hbm_bytes"] for n, v in ks.items() if n.startswith(TRAFFIC_KERNEL)), None)
    # every kernel of the push (one launch each per push; k_scan_sum runs twice)
    push = sum(v["hbm_bytes"] * v.get("launches", 1) for v in ks.values()) / max(
        1, next((v.get("launches", 1) for n, v in ks.items() if n.startswith(TRAFFIC_KERNEL)), 1))
    return main, push


GOLDEN_DIGEST = "tests/golden/c2_bench_digest.json"
C1_GOLDEN_DIGEST = "tests/golden/c1_bench_digest.json"


def output_digest_check(args, arrays, golden=GOLDEN_DIGEST, c1_batch=None):
    """SHA-256 of the first warm-up push's canonical output (siddhi_amd.digest; computed outside the timed
    region) against the CPU restatement's digest of the same stream (tests/golden/make_c2_digest.py,
    make_c1_digest.py). Only the default configurations have a golden digest."""
    from siddhi_amd import digest
    gold = json.load(open(os.path.join(ROOT, golden)))
    cfg = gold["config"]
    if c1_batch is not None:
        if c1_batch != cfg["events_per_push"]:
            return None
    elif (args.batch, args.keys, args.events_per_ms, args.send_size, args.key_type) != (
            cfg["events_per_push"], cfg["keys"], cfg["events_per_ms"], cfg["send_size"], "string"):
        return None
    got = digest.output_digest(arrays)
    return {"match": got == gold["push0"]["sha256"], "sha256": got, "rows": int(arrays["ts"].size),
            "expected": gold["push0"]["sha256"], "source": golden + " (oracle/ on the same stream)"}


# ---- secondary single-GPU workloads (BASELINE.json configs[0], [2], [3]; externalTimeBatch) ---------
SECONDARY = {
    # name: (description, algorithmic bytes per event from SURVEY.md §8d)
    "c1": ("C1 lengthBatch(10000) [price>100] sum(volume), avg(price) group by symbol, 1k symbols, send(Event[1000])",
           29.4),
    "c3": ("C3 sliding time(10 sec) count/min/max/avg group by k, 10k keys, per-event sends", 84.0),
    "c4": ("C4 define aggregation sum/avg/count/min/max group by k aggregate by ts every sec...day; one GPU's share "
           "of C4 on 8 GPUs: 125k of the 1M keys, 1.25M of the 10M events per event-time second", 25.2),
    "ext": ("externalTimeBatch(et, 1 sec) count/min/max/avg group by k, 100k keys, per-event sends", 32.4),
    # output modes on the C2 / C3 streams (algorithmic bytes: the input plus the extra rows written)
    "c2all": ("C2 with `insert all events`: every flush also re-emits the previous batch's keys as EXPIRED rows "
              "(count 0, other aggregators null)", 28.8),
    "c2cur": ("C2 on timeBatch(1 sec, true) (stream.current.event): a row per passing event with its key's running "
              "aggregates since the batch reset", 64.0),
    "c3all": ("C3 with `insert all events`: every expired event re-stamped and emitted before the current one", 168.0),
    # every event is read (20 B); only the partition that armed the shared timer is aggregated (R12)
    "c5": ("C5 partition with (k of S) begin from S#window.timeBatch(1 sec) select k, sum(v), count() group by k; "
           "10M Zipf(1.1) keys, 1M events per event-time second per GPU, per-event sends", 20.0),
    # partition lanes (sh_plane*): input 20 B (+ 4 B group column) and the rows of the completed batches
    "plb": ("partition with (k of S) begin from S#window.lengthBatch(16) select k, sum(v), count(), max(v) group by k; "
            "C5's 10M Zipf(1.1) keys, per-event sends (one lane per partition)", 22.8),
    "plg": ("partition with (k of S) begin from S#window.lengthBatch(16) select g, sum(v), count(), max(v) group by g; "
            "C5's 10M Zipf(1.1) partition keys, 8 groups, per-event sends (sorted chunks, lane 3)", 43.0),
}


def run_secondary(args, dev, rank=0, world=1, dist=None):
    """Inputs resident in HBM, `--steps` pushes of `--batch` events (per GPU) of the workload. C1, C4
    and C5 also run at N > 1: one global stream (C4, C5: N x the per-GPU key count and event rate) is
    sliced across the ranks and key-sharded; C3 likewise with N x the keys and the event rate (ShardedQuery / ShardedAggregation over RCCL all-to-all)."""
    import numpy as np
    import torch
    from siddhi_amd import abi, runtime, synth
    ctx = runtime.Context(dev.index)
    if args.workload == "c4" and args.batch == 1 << 25:
        args.batch = 1 << 22  # 3.4 s of event time per push: ~4 open second-buckets x 125k keys per GPU
    B, nb = args.batch, args.warmup + args.steps
    agg = None
    sliced = world > 1
    if args.workload == "c1":
        schema = abi.Schema.parse("symbol string, price double, volume long, ts long")
        spec = abi.QuerySpec(schema, "lengthBatch", 10000, group_by=["symbol"], aggs=[("sum", "volume"), ("avg", "price")],
                             filter=(">", "price", 100), key_capacity=1000)
        send = 1000
        B = args.batch = B - B % send  # slices are cut at send boundaries (sh_shard_pack checks it)
        # N > 1: one global stream, rank r holds slice r of every global push
        gen = lambda i: [torch.from_numpy(np.ascontiguousarray(c)).to(dev)
                         for c in synth.c1_stock((i * world + rank) * B, B)[1]]
        mk = lambda cols: (cols[3], cols)
    elif args.workload == "c4":
        schema = abi.Schema.parse("k string, v double, ts long")
        # C4 = 1M keys at 10M events per event-time second on 8 GPUs: 125k keys and 1.25M ev/s per GPU
        agg = abi.AggregationSpec(schema, [("sum", "v"), ("avg", "v"), ("count", None), ("min", "v"), ("max", "v")],
                                  group_by=["k"], ts="ts", durations=("sec", "day"), key_capacity=125_000 * world)
        send = 1
        gen = lambda i: synth.torch_keyed_stream((i * world + rank) * B, B, 0xC4, 125_000 * world, 1_250 * world,
                                                 dev)[1]
        mk = lambda cols: (cols[2], cols)
    elif args.workload == "c5":
        schema = abi.Schema.parse("k string, v double, ts long")
        spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"], aggs=[("sum", "v"), ("count", None)],
                             partition="k", key_capacity=10_000_000)
        send = 1
        gen = lambda i: synth.torch_zipf_stream((i * world + rank) * B, B, 0xC5, 10_000_000, 1000 * world, dev)[1]
        mk = lambda cols: (cols[2], cols)
    elif args.workload in ("plb", "plg"):
        g = args.workload == "plg"
        schema = abi.Schema.parse("k string, v double, ts long, g int" if g else "k string, v double, ts long")
        spec = abi.QuerySpec(schema, "lengthBatch", 16, group_by=["g"] if g else ["k"],
                             aggs=[("sum", "v"), ("count", None), ("max", "v")], partition="k", key_capacity=10_000_000)
        send = 1

        def gen(i):
            cols = synth.torch_zipf_stream(i * B, B, 0xC5, 10_000_000, 1000, dev)[1]
            if g:
                cols.append(((cols[2] * 7 + torch.arange(B, device=dev)) % 8).to(torch.int32).contiguous())
            return cols
        mk = lambda cols: (cols[2], cols)
    else:
        if args.workload == "c3":
            schema = abi.Schema.parse("k string, v double, ts long")
            # N > 1: one global stream with N x the keys and N x the event rate, sliced across the ranks
            spec = abi.QuerySpec(schema, "time", 10_000, group_by=["k"],
                                 aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")],
                                 key_capacity=10_000 * world)
            gen = lambda i: synth.torch_keyed_stream((i * world + rank) * B, B, 0xC3, 10_000 * world, 1000 * world,
                                                     dev)[1]
        elif args.workload == "c3all":
            schema = abi.Schema.parse("k string, v double, ts long")
            spec = abi.QuerySpec(schema, "time", 10_000, group_by=["k"],
                                 aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")],
                                 key_capacity=10_000, output="all")
            gen = lambda i: synth.torch_keyed_stream(i * B, B, 0xC3, 10_000, 1000, dev)[1]
        elif args.workload in ("c2all", "c2cur"):
            schema = abi.Schema.parse("k string, v double, ts long")
            spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"],
                                 aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=100_000,
                                 output="all" if args.workload == "c2all" else "current",
                                 stream_current=args.workload == "c2cur")
            gen = lambda i: synth.torch_keyed_stream(i * B, B, 0xC2, 100_000, 1000, dev)[1]
        else:
            schema = abi.Schema.parse("k string, v double, ts long")
            spec = abi.QuerySpec(schema, "externalTimeBatch", 1000, group_by=["k"], ts_attr="ts",
                                 aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=100_000)
            gen = lambda i: synth.torch_keyed_stream(i * B, B, 0xE7, 100_000, 1000, dev)[1]
        send = 1
        mk = lambda cols: (cols[2], cols)
    if sliced:
        if args.workload not in ("c1", "c3", "c4", "c5"):
            raise SystemExit("of the secondary workloads only c1, c3, c4 and c5 run on N > 1 GPUs")
        from siddhi_amd.shard import ShardedAggregation, ShardedQuery, TorchExchange, distributed_push
        q = ShardedAggregation(agg, rank, world, ctx) if agg else ShardedQuery(spec, rank, world, ctx)
        ex = TorchExchange(dev if args.backend == "nccl" else torch.device("cpu"))
        send_buf = torch.empty(B * q.record_bytes, dtype=torch.uint8, device=dev)
    else:
        q = runtime.GpuAggregation(agg, ctx) if agg else runtime.GpuQuery(spec, ctx)
        if args.workload in ("c2cur", "c3"):
            q.set_compact_flushes()  # a row per event: flush i = row i at its ts (no 16 B/row flush arrays)
        if args.workload in ("c3all", "plb", "plg"):
            q.set_device_flushes()  # the per-send flush layout stays in HBM with the rows (nothing crosses PCIe)
    batches = [mk(gen(i)) for i in range(nb)]
    torch.cuda.synchronize()
    phases, timing = {}, False

    def push(i):
        ts, cols = batches[i]
        if sliced:
            return distributed_push(q, ex, B, ts.data_ptr(), [c.data_ptr() for c in cols], send, send_buf,
                                    host_out=False, timings=phases if timing else None)
        return q.push_device(B, ts.data_ptr(), [c.data_ptr() for c in cols], send)

    digest_check = None
    for i in range(args.warmup):
        op = push(i)
        if i == 0 and args.workload == "c1" and not sliced:
            torch.cuda.synchronize()
            digest_check = output_digest_check(args, runtime.device_out_arrays(op), C1_GOLDEN_DIGEST, B)
    torch.cuda.synchronize()
    timing = True
    # an aggregation's device time is summed by the library from per-push HIP events, read after the
    # loop (its per-push stats would wait for every push)
    agg_timed = agg is not None and not sliced
    if agg_timed:
        q.timing(reset=True)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    kern_ms, t0 = 0.0, time.perf_counter()
    for i in range(args.warmup, nb):
        push(i)
        if not sliced and not agg_timed:
            st = q.stats()
            # the whole device pipeline of the push (HIP events around it on the library's stream): the
            # algorithmic bytes are the whole push's, so the fraction is the push's, not one kernel's
            # (profiles/r06_*_kernel_stats.txt name the kernels and their shares)
            kern_ms += st.push_ms
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if agg_timed:
        kern_ms, n_timed = q.timing()
        assert n_timed == args.steps, (n_timed, args.steps)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    if rank != 0:
        q.close()
        return
    desc, bpe = SECONDARY[args.workload]
    roof = None
    if kern_ms > 0:
        ach = bpe * B * args.steps / (kern_ms / 1e3) / 1e9
        kname = ("whole device pipeline of the push (root window + sec..day roll-up levels)" if args.workload == "c4"
                 else "whole device pipeline of the push")
        roof = {"bound": "hbm", "kernel": kname, "achieved": ach, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": None, "kernel_ms_per_step": kern_ms / args.steps,
                "bytes_per_event": bpe}
    config = {"workload": desc, "events_per_step_per_gpu": B, "send_size": send,
              # sh_out's flush layout for sh_push_device: host arrays (the ABI default), compact (NULL: a row per
              # flush at its timestamp) or left in device memory (sh_query_set_device_flushes)
              "flush_layout": ("compact" if args.workload in ("c2cur", "c3") else
                               "device" if args.workload in ("c3all", "plb", "plg") else "host") if not sliced else "host"}
    if sliced:
        config.update(parallelism=f"slice ingest x{world}, key re-shard over "
                                  f"{'RCCL' if args.backend == 'nccl' else 'gloo (host)'} all-to-all",
                      keys_total=125_000 * world if agg else 1000 if args.workload == "c1" else
                      10_000 * world if args.workload == "c3" else 10_000_000,
                      phases_ms_per_step_rank0={k: v / args.steps for k, v in phases.items()})
    print(json.dumps({"metric": METRIC, "value": B * args.steps * world / elapsed, "unit": "events/s",
                      "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                      "ms_per_step": elapsed * 1e3 / args.steps, "higher_is_better": True, "scaling": "weak",
                      "vs_baseline": None, "dtype": "f64",
                      "data": "synthetic SplitMix64 stream (SURVEY.md §8d seeds), resident in HBM",
                      "config": config, "roofline": roof,
                      **({"output_sha256_match": digest_check["match"], "output_check": digest_check}
                         if digest_check else {})}), flush=True)
    q.close()


PCIE_PEAK_GBS = 63.0  # PCIe Gen5 x16 host link (MI355X_MICROARCH.md)
H2D_BYTES_PER_EVENT = 20  # the columns the C2 query reads: ts 8 + k 4 + v 8 (the unread `ts` attribute is NULL)


def host_leg(args, dev, B, steps, warmup, ctx=None):
    """C2 from host memory, as the Java shim would drive it: every micro-batch packed into pinned SoA
    buffers (only the columns the query reads: the `ts` attribute column is passed as NULL), its H2D
    copy staged on the copy stream while the previous batch is processed (sh_stage / sh_push_staged),
    output rows copied back to the host. Returns the PCIe-inclusive event rate, the copy engine's H2D
    GB/s (HIP events on the copy stream) and the per-call latency."""
    import torch
    from siddhi_amd import abi, runtime, synth
    ctx = ctx or runtime.Context(dev.index)
    schema = abi.Schema.parse(f"k {args.key_type}, v double, ts long")
    spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=args.keys)
    nb = warmup + steps
    q = runtime.GpuQuery(spec, ctx)
    bufs = []  # one pinned batch per call: consecutive slices of one stream
    for i in range(nb):
        ts, cols = synth.torch_keyed_stream(i * B, B, 0xC2, args.keys, args.events_per_ms, dev)
        pb = runtime.PinnedBatch(schema, B, args.send_size)
        for a, t in zip(pb.arrays, [ts] + cols):
            torch.from_numpy(a).copy_(t)  # D2H into the pinned SoA buffers (outside the timed region)
        pb.set_n(B)
        pb.b.cols[2] = None  # the query does not read the `ts` attribute: 20 B/event cross PCIe
        bufs.append(pb)
    torch.cuda.synchronize()

    lat, h2d_ms, h2d_bytes, rows = [], 0.0, 0, 0

    def run(lo, hi, timed):
        nonlocal h2d_ms, h2d_bytes, rows
        tickets = [q.stage(bufs[lo])]
        for i in range(lo, hi):
            if i + 1 < hi:
                tickets.append(q.stage(bufs[i + 1]))
            ta = time.perf_counter()
            o = q.push_staged_raw(tickets.pop(0)).contents
            if timed:
                lat.append(time.perf_counter() - ta)
                ms, nbytes = q.ingest_stats()
                h2d_ms += ms
                h2d_bytes += nbytes
                rows += o.n_rows
    run(0, warmup, False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(warmup, nb, True)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    h2d = h2d_bytes / (h2d_ms / 1e3) / 1e9 if h2d_ms > 0 else None
    lat_ms = sorted(x * 1e3 for x in lat)
    rate = B * steps / elapsed
    for b in bufs:
        b.close()
    q.close()
    return {"events_per_s": rate, "events_per_call": B, "calls": steps, "ms_per_call": elapsed * 1e3 / steps,
            "h2d_bytes_per_event": H2D_BYTES_PER_EVENT, "h2d_bytes_per_call": h2d_bytes / steps,
            "h2d_copy_GBps": h2d, "peak_GBps": PCIE_PEAK_GBS,
            "frac": h2d / PCIE_PEAK_GBS if h2d else None,
            # the host-fed event rate's input bytes over the link peak (the copy overlaps the kernels)
            "end_to_end_frac": rate * H2D_BYTES_PER_EVENT / 1e9 / PCIE_PEAK_GBS, "rows_copied_back": rows,
            "call_latency_ms": {"p50": lat_ms[len(lat_ms) // 2], "p99": lat_ms[int(0.99 * (len(lat_ms) - 1))],
                                "max": lat_ms[-1]}}


def pcie_line(args, dev, ctx):
    """The driver line's `pcie` object (the H2D roofline fraction): the C2 stream fed from
    pinned host batches of 2^25 events (bandwidth) and of 1000 events (send(Event[1000]) latency)."""
    big = host_leg(args, dev, 1 << 25, 5, 1, ctx)
    small = host_leg(args, dev, 1000, 400, 40, ctx)
    return {"source": "C2 from pinned host SoA batches (sh_stage / sh_push_staged, double-buffered H2D on the "
                      "copy stream, output rows copied back); never the headline value",
            "bulk": big, "send_1000": small,
            "events_per_s": big["events_per_s"], "h2d_copy_GBps": big["h2d_copy_GBps"],
            "peak_GBps": PCIE_PEAK_GBS, "frac": big["frac"], "end_to_end_frac": big["end_to_end_frac"],
            "p50_ms_at_1000": small["call_latency_ms"]["p50"], "p99_ms_at_1000": small["call_latency_ms"]["p99"]}


def run_host(args, dev):
    """`--host`: the host-fed leg alone, as its own JSON line."""
    r = host_leg(args, dev, args.batch, args.steps, args.warmup)
    print(json.dumps({
        "metric": METRIC, "value": r["events_per_s"], "unit": "events/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": r["ms_per_call"], "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic SplitMix64 stream seed 0xC2 packed into pinned host SoA buffers before the timed region",
        "config": {"workload": "C2 timeBatch(1 sec) count/min/max/avg group by k from HOST batches "
                               "(PCIe-inclusive: H2D of every batch, D2H of every output row; not the HBM headline)",
                   "key_type": args.key_type, "keys": args.keys, "events_per_call": args.batch,
                   "send_size": args.send_size,
                   "ingest": "double-buffered sh_stage / sh_push_staged (copy stream + compute stream)"},
        "pcie": r}), flush=True)


def run_shard_loopback(args, dev):
    """What one GPU of an N-GPU sliced C2 run spends per step, measured on one GPU: G owners of the
    sharded query (ShardedQuery: sh_shard_summarize / pack / consume) in one process, each ingesting
    --batch events of one global stream per step (G x --events-per-ms, --keys-total or G x --keys keys),
    the all-to-all replaced by device copies of the owners' record runs. Every phase ends in a device
    synchronisation; the per-owner figures are the phase totals / G. Not a driver line (no `value` of
    the headline): it bounds the per-GPU rate of the multi-GPU path apart from the xGMI transfer."""
    import numpy as np
    import torch
    from siddhi_amd import abi, runtime, synth
    from siddhi_amd.shard import ShardedQuery
    G, B = args.shard_loopback, args.batch
    ctx = runtime.Context(dev.index)
    keys_total = args.keys_total or args.keys * G
    schema = abi.Schema.parse(f"k {args.key_type}, v double, ts long")
    spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=keys_total)
    shards = [ShardedQuery(spec, r, G, ctx) for r in range(G)]
    rb = shards[0].record_bytes
    send = [torch.empty(B * rb, dtype=torch.uint8, device=dev) for _ in range(G)]
    recv = [torch.empty(2 * B * rb, dtype=torch.uint8, device=dev) for _ in range(G)]
    nb = args.warmup + args.steps

    def slices(i):
        return [synth.torch_keyed_stream((i * G + r) * B, B, 0xC2, keys_total, args.events_per_ms * G, dev)
                for r in range(G)]

    ph = {"summarize": 0.0, "pack": 0.0, "exchange_device_copy": 0.0, "consume": 0.0}
    sent_bytes, rows = 0, 0

    def step(sl, timed):
        nonlocal sent_bytes, rows
        t0 = time.perf_counter()
        summ = np.stack([s.summarize(B, ts.data_ptr(), [c.data_ptr() for c in cols], 1)
                         for s, (ts, cols) in zip(shards, sl)])
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        counts, bounds = [], []
        for s, buf in zip(shards, send):
            sb, bd = s.pack(summ, buf.data_ptr(), int(buf.numel()))
            counts.append(np.asarray(sb))
            bounds.append(bd)
        all_bounds = np.concatenate(bounds)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        rbytes = []
        for o in range(G):
            off, rb_o = 0, []
            for g in range(G):
                start, n = int(counts[g][:o].sum()), int(counts[g][o])
                if off + n > recv[o].numel():
                    raise SystemExit("loopback receive buffer too small")
                recv[o][off:off + n].copy_(send[g][start:start + n])
                off += n
                rb_o.append(n)
            rbytes.append(rb_o)
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        for o, s in enumerate(shards):
            out = s.consume(recv[o].data_ptr(), rbytes[o], all_bounds, host_out=False)[0]
            if timed:
                rows += int(out.contents.n_rows)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        if timed:
            for k, v in zip(ph, (t1 - t0, t2 - t1, t3 - t2, t4 - t3)):
                ph[k] += v * 1e3
            sent_bytes += int(sum(c.sum() for c in counts))

    for i in range(nb):
        sl = slices(i)
        torch.cuda.synchronize()
        step(sl, i >= args.warmup)
        del sl
    per_owner = {k: v / args.steps / G for k, v in ph.items()}
    compute_ms = per_owner["summarize"] + per_owner["pack"] + per_owner["consume"]
    off_gpu = sent_bytes / args.steps / G * (G - 1) / G  # bytes one owner sends to other GPUs per step
    print(json.dumps({
        "metric": "sharded C2 pipeline, one GPU's share measured on one GPU (not the headline)",
        "shards": G, "events_per_owner_step": B, "keys_total": keys_total,
        "event_rate": f"{args.events_per_ms * 1000 * G} events per event-time second",
        "ms_per_owner_step": per_owner,
        "owner_events_per_s_without_xgmi": B / (compute_ms / 1e3),
        "exchange_bytes_per_owner_step": sent_bytes / args.steps / G,
        "off_gpu_bytes_per_owner_step": off_gpu,
        # all-to-all over the 7 xGMI links (≈153 GB/s each, MI355X_MICROARCH.md): one owner's share
        "xgmi_ms_per_owner_step_at_peak": off_gpu / (7 * 153e9) * 1e3,
        "rows_per_step": rows / args.steps,
        "record_bytes": rb,
    }), flush=True)
    for s in shards:
        s.close()


def main():
    args = parse()
    # all-cores CPU baseline workers: started before anything touches the GPU (rank 0, N = 1 only)
    pool, P = None, 0
    if (not args.no_cpu_baseline and int(os.environ.get("WORLD_SIZE", "1")) == 1 and args.workload == "c2"
            and not args.host):
        import multiprocessing as mp
        P = max(2, min(15, os.cpu_count() or 2))
        # the workers run the oracle only: they must not load a HIP runtime (siddhi_amd binds one at
        # import), or each would hold the GPU open next to this process
        os.environ["SIDDHI_AMD_BIND_HIP"] = "0"
        pool = mp.get_context("spawn").Pool(P)
        os.environ.pop("SIDDHI_AMD_BIND_HIP", None)
    import torch
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = max(1, torch.cuda.device_count())
    if args.backend == "nccl" and world > 1 and local >= ndev:
        raise SystemExit(f"rank {local} has no GPU of its own ({ndev} visible)")
    torch.cuda.set_device(local % ndev)
    dev = torch.device("cuda", local % ndev)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    if args.workload != "c2":
        return run_secondary(args, dev, rank, world, dist)
    if args.shard_loopback:
        if world > 1:
            raise SystemExit("--shard-loopback runs on one GPU")
        return run_shard_loopback(args, dev)
    if args.host:
        if world > 1:
            raise SystemExit("--host runs on one GPU")
        return run_host(args, dev)
    from siddhi_amd import abi, runtime, synth
    ctx = runtime.Context(local % ndev)
    schema = abi.Schema.parse(f"k {args.key_type}, v double, ts long")
    sliced = world > 1 and args.ingest == "slice"
    keys_total = (args.keys_total or args.keys * world) if sliced else args.keys
    cap = keys_total  # whole-stream key capacity (each owner sizes its table for its share)
    spec = abi.QuerySpec(schema, "timeBatch", 1000, group_by=["k"],
                         aggs=[("count", None), ("min", "v"), ("max", "v"), ("avg", "v")], key_capacity=cap)
    B = args.batch
    nb = args.warmup + args.steps
    batches = []
    if sliced:
        # rank r's slice of global push i: events [(i*N + r)*B, (i*N + r + 1)*B) of one stream
        from siddhi_amd.shard import PipelinedPush, ShardedQuery, TorchExchange, distributed_push
        q = ShardedQuery(spec, rank, world, ctx)
        ex = TorchExchange(dev if args.backend == "nccl" else torch.device("cpu"))
        send_buf = torch.empty(B * q.record_bytes, dtype=torch.uint8, device=dev)
        # the record exchange of push i overlaps the consume of push i - 1 (two send buffers)
        pp = None if args.no_pipeline else PipelinedPush(q, ex, [send_buf, torch.empty_like(send_buf)])
        for i in range(nb):
            batches.append(synth.torch_keyed_stream((i * world + rank) * B, B, 0xC2, keys_total,
                                                    args.events_per_ms * world, dev))
    else:
        # keyed: this rank's own stream; keys offset so ranks own disjoint keys
        q = runtime.GpuQuery(spec, ctx)
        for i in range(nb):
            ts, cols = synth.torch_keyed_stream(i * B, B, 0xC2 ^ (rank * 0x9E37), args.keys, args.events_per_ms, dev)
            if rank:
                cols[0] += rank * args.keys
            batches.append((ts, cols))
        # the batch descriptors, built once (a host shim keeps one per buffer)
        descs = [q.device_batch(B, ts.data_ptr(), [c.data_ptr() for c in cols], args.send_size)
                 for ts, cols in batches]
    torch.cuda.synchronize()

    def push(i):
        """The output of push i (pipelined sharded ingest: of push i - 1, None for the first)."""
        ts, cols = batches[i]
        if sliced:
            if pp is not None:
                r = pp.push(B, ts.data_ptr(), [c.data_ptr() for c in cols], args.send_size,
                            timings=phases if timing else None)
                return r[0] if r is not None else None
            return distributed_push(q, ex, B, ts.data_ptr(), [c.data_ptr() for c in cols], args.send_size,
                                    send_buf, host_out=False, timings=phases if timing else None)[0]
        return q.push_device_batch(descs[i])

    def drain():
        if sliced and pp is not None:
            r = pp.finish()
            return r[0] if r is not None else None
        return None

    phases, timing = {}, False
    digest_check = None
    for i in range(args.warmup):
        op = push(i)
        if i == 0 and not sliced and world == 1 and op is not None:
            torch.cuda.synchronize()
            digest_check = output_digest_check(args, runtime.device_out_arrays(op))
    drain()
    torch.cuda.synchronize()
    timing = True
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    kern_ms, kern_bytes, flushes, rows = 0.0, 0, 0, 0
    host_t = [] if os.environ.get("SH_TIMING") else None
    t0 = time.perf_counter()
    for i in range(args.warmup, nb + 1):
        ta = time.perf_counter()
        op = push(i) if i < nb else drain()  # (the pipelined ingest consumes its last push here)
        tb = time.perf_counter()
        if op is None:
            continue
        o = op.contents
        st = q.stats()
        kern_ms += st.main_kernel_ms
        flushes += o.n_flushes
        rows += o.n_rows
        if host_t is not None:
            host_t.append((tb - ta, time.perf_counter() - tb))
    t_sync = time.perf_counter()
    torch.cuda.synchronize()
    if host_t:
        import statistics
        print(f"[bench timing] loop {(t_sync - t0) * 1e3:.2f} ms, pushes {sum(a for a, _ in host_t) * 1e3:.2f} ms, "
              f"bookkeeping {sum(b for _, b in host_t) * 1e3:.2f} ms, final sync {(time.perf_counter() - t_sync) * 1e3:.2f} ms",
              file=sys.stderr)
        print(f"[bench timing] push call median {statistics.median(a for a, _ in host_t) * 1e6:.1f} us, "
              f"bookkeeping median {statistics.median(b for _, b in host_t) * 1e6:.1f} us; per push: "
              + " ".join(f"{a * 1e6:.0f}" for a, _ in host_t), file=sys.stderr)
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    total_events = B * args.steps * world
    # roofline of the dominant kernel (k_aggregate): algorithmic bytes per launch / its HIP-event time
    n_launch = args.steps
    ach = (C2_BYTES_PER_EVENT * B * n_launch) / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else 0.0
    traffic, push_traffic = measured_traffic(args, sliced)
    result = {
        "metric": METRIC,
        "value": total_events / elapsed,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed * 1e3 / args.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": ("synthetic: SplitMix64 stream seed 0xC2, one global stream sliced across ranks, generated in HBM"
                 if sliced else "synthetic: SplitMix64 stream seed 0xC2 (per rank seed ^ rank*0x9E37), generated in HBM"),
        "config": {"workload": "C2 timeBatch(1 sec) count/min/max/avg group by k, per-event sends",
                   "key_type": f"{args.key_type} ({'dictionary ids = dense slots' if args.key_type == 'string' else 'hashed'})",
                   "keys_per_gpu": args.keys, "keys_total": keys_total, "events_per_step_per_gpu": B,
                   "event_rate": f"{args.events_per_ms * 1000 * (world if sliced else 1)} events per event-time second",
                   "send_size": args.send_size,
                   "parallelism": (f"slice ingest x{world}, key re-shard over {'RCCL' if args.backend == 'nccl' else 'gloo (host)'} all-to-all"
                                   + ("" if args.no_pipeline else ", exchange of push i overlapped with consume of push i-1") if sliced
                                   else f"key-sharded x{world}"),
                   "flushes": flushes, "rows": rows},
        "roofline": {"bound": "hbm", "kernel": "k_aggregate_own", "achieved": ach, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": ach / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel_ms_per_step": kern_ms / args.steps,
                     "bytes_per_event": C2_BYTES_PER_EVENT,
                     # the same algorithmic bytes over the whole step's wall time (every kernel, launch
                     # gaps and host synchronisation included), and the PMC bytes of the whole push
                     "end_to_end": {"achieved": C2_BYTES_PER_EVENT * B * world / (elapsed / args.steps) / 1e9,
                                    "frac": C2_BYTES_PER_EVENT * B * world / (elapsed / args.steps) / 1e9 / HBM_PEAK_GBS,
                                    "traffic_per_step": push_traffic,
                                    "traffic_source": TRAFFIC_SUMMARY if traffic else None}},
    }
    if digest_check is not None:
        result["output_sha256_match"] = digest_check["match"]
        result["output_check"] = digest_check
    if sliced:
        # rank 0's wall time per step in each phase of the sharded push (summaries all-gather,
        # pack, record all-to-all over RCCL, owner pipeline) and its bytes sent per step
        result["config"]["phases_ms_per_step_rank0"] = {k: v / args.steps for k, v in phases.items()}
    if rank == 0 and world == 1 and not sliced and not args.no_pcie:
        result["pcie"] = pcie_line(args, dev, ctx)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args)
        if pool is not None:
            result["cpu_baseline_all_cores"] = cpu_baseline_all_cores(args, pool, P)
            pool.close()
            pool.join()
    if rank == 0:
        print(json.dumps(result), flush=True)
    q.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
