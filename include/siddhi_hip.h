/*
 * siddhi_hip.h — C ABI of libsiddhi_hip.so, the MI355X (gfx950) execution path for Siddhi's
 * filtered, windowed group-by aggregation and incremental `define aggregation` roll-ups.
 *
 * The reference (Arshardh/siddhi, Java) has no native code; this ABI is what the Java window /
 * aggregator extension shim binds through JNI or Panama FFM. Every entry
 * point names the reference interface whose behaviour it replaces. Citations use
 *   core/  = modules/siddhi-core/src/main/java/io/siddhi/core/
 *   qapi/  = modules/siddhi-query-api/src/main/java/io/siddhi/query/api/
 *
 * Rules of the ABI:
 *  - plain C types only; no C++ or torch types cross it;
 *  - every call returns an int: SH_OK (0) or a negative SH_ERR_* code; sh_last_error() gives a
 *    thread-local message (the Java shim turns it into SiddhiAppRuntimeException, which the
 *    StreamJunction publisher routes by @OnError, core/stream/StreamJunction.java:486-535);
 *  - a query handle is single-threaded, matching the per-query LockWrapper the reference takes in
 *    ProcessStreamReceiver.process (core/query/input/ProcessStreamReceiver.java:74-96) and in
 *    Scheduler.sendTimerEvents (core/util/Scheduler.java:171-209);
 *  - output buffers are owned by the library and stay valid until the next call on that handle.
 */
#ifndef SIDDHI_HIP_H
#define SIDDHI_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SH_ABI_VERSION 16

/* ---- return codes ---------------------------------------------------------------------- */
#define SH_OK 0
#define SH_ERR_INVALID (-1)     /* malformed descriptor or batch (SiddhiAppValidationException) */
#define SH_ERR_UNSUPPORTED (-2) /* a feature this build does not run on the GPU (fails loudly)   */
#define SH_ERR_DEVICE (-3)      /* HIP / RCCL failure                                           */
#define SH_ERR_OOM (-4)         /* device allocation failed                                     */
#define SH_ERR_STATE (-5)       /* call out of order (e.g. clock moved backwards in a batch)    */

/* ---- attribute types: qapi/definition/Attribute.java:105-113 ---------------------------- */
#define SH_T_INT 1    /* int32                                                              */
#define SH_T_LONG 2   /* int64                                                              */
#define SH_T_FLOAT 3  /* float                                                              */
#define SH_T_DOUBLE 4 /* double                                                             */
#define SH_T_STRID 5  /* string, dictionary-encoded by the host to int32 ids (equality only) */
#define SH_T_BOOL 6   /* uint8 0/1                                                          */

/* ---- filter program: postfix form of the `S[cond]` expression --------------------------
 * Replaces FilterProcessor.process (core/query/processor/filter/FilterProcessor.java:47-60)
 * and the Compare/And/Or/Not condition executors (core/executor/condition/ and compare/). Comparisons
 * follow the reference's per-type-pair executors: relational ops use Java binary numeric
 * promotion; ==/!= do too except Float<->Long which compare as double
 * (compare/equal/EqualCompareConditionExpressionExecutorFloatLong.java).                    */
#define SH_OP_COL 1   /* push column `col`                                                 */
#define SH_OP_CONST 2 /* push constant of `type` (ival for INT/LONG/STRID/BOOL, dval FLOAT/DOUBLE) */
#define SH_OP_GT 3
#define SH_OP_GE 4
#define SH_OP_LT 5
#define SH_OP_LE 6
#define SH_OP_EQ 7
#define SH_OP_NE 8
#define SH_OP_AND 9
#define SH_OP_OR 10
#define SH_OP_NOT 11

typedef struct {
    int32_t op;
    int32_t type; /* SH_T_* of the constant (SH_OP_CONST)                                  */
    int32_t col;  /* column index (SH_OP_COL)                                              */
    int32_t pad;
    int64_t ival;
    double dval;
} sh_filter_op;

/* ---- windows ---------------------------------------------------------------------------- */
#define SH_WIN_NONE 0         /* no window: filter -> selector (oracle/KAT use; not a GPU path) */
#define SH_WIN_LENGTH_BATCH 1 /* core/query/processor/stream/window/LengthBatchWindowProcessor.java */
#define SH_WIN_TIME_BATCH 2   /* core/query/processor/stream/window/TimeBatchWindowProcessor.java   */
#define SH_WIN_TIME 3         /* core/query/processor/stream/window/TimeWindowProcessor.java        */
#define SH_WIN_EXT_TIME_BATCH 4 /* core/query/processor/stream/window/ExternalTimeBatchWindowProcessor.java:
                                   externalTimeBatch(ts_col, T[, start[, timeout]]) — event-time batches;
                                   the timeout through sh_query_set_ext_timeout */
#define SH_WIN_EXT_TIME 5     /* core/query/processor/stream/window/ExternalTimeWindowProcessor.java:
                                 externalTime(ts_col, T) — sliding over the LONG attribute ts_col    */

/* ---- aggregators: core/query/selector/attribute/aggregator/ [Sum,Avg,Count,Min,Max]AttributeAggregatorExecutor ---- */
#define SH_AGG_SUM 1
#define SH_AGG_AVG 2
#define SH_AGG_COUNT 3
#define SH_AGG_MIN 4
#define SH_AGG_MAX 5

typedef struct {
    int32_t fn;  /* SH_AGG_*                                     */
    int32_t col; /* input column (ignored for SH_AGG_COUNT)      */
} sh_agg_spec;

#define SH_MAX_COLS 8
#define SH_MAX_AGGS 8
/* group-by columns: any number up to SH_MAX_GROUP; one column of any type or two 32-bit ones (int, string
 * id, bool, float) key the window directly, any other combination is interned on the device into one
 * 32-bit id per distinct key (needs a spare column slot: n_cols < SH_MAX_COLS; not sharded) */
#define SH_MAX_GROUP 8

/* Compiled form of
 *   [partition with (pcol of S) begin]
 *   from S[filter]#window.<kind>(param[, start][, streamCurrent])
 *   select g..., agg(col)... group by g... insert [current|all|expired] events into O;
 * built by the Java shim from the parsed Query (the reference parser stays in charge). */
typedef struct {
    int32_t n_cols;
    int32_t col_types[SH_MAX_COLS];
    int32_t n_filter_ops; /* 0 = no filter                                              */
    const sh_filter_op* filter;
    int32_t window;         /* SH_WIN_*                                                 */
    int32_t stream_current; /* lengthBatch/timeBatch `stream.current.event` flag        */
    int64_t window_param;   /* lengthBatch: length; timeBatch/time: milliseconds        */
    int32_t has_start_time; /* timeBatch(T, start) / externalTimeBatch(.., T, start): 1 = constant
                               start_time; 2 = externalTimeBatch start from attribute start_col */
    int32_t n_group_by;     /* 0..SH_MAX_GROUP                                           */
    int64_t start_time;
    int32_t group_by[SH_MAX_GROUP];
    int32_t n_aggs;
    int32_t current_on;     /* insert [current|all] events  (QueryParser.java:221-223)   */
    sh_agg_spec aggs[SH_MAX_AGGS];
    int32_t expired_on;     /* insert [expired|all] events                               */
    int32_t partition_col;  /* -1: not partitioned; else `partition with (col of S)`: int / long /
                               string id / float / double (not float / double for time windows
                               with expired output)                                        */
    int64_t key_capacity;   /* upper bound on distinct group keys (device table sizing). Batch and
                             * time() windows rebuild their hashed table from the live keys when it
                             * is half full (a time() key is live while an event of it can still be
                             * in a later window); externalTime windows keep a key's slot for the
                             * query's lifetime; dictionary-id keys: the id range. Exceeding it
                             * fails the push with "group key table full: raise key_capacity". */
    int32_t ts_col;         /* externalTimeBatch / externalTime: the LONG timestamp attribute  */
    int32_t start_col;      /* externalTimeBatch: LONG start-time attribute (has_start_time 2) */
} sh_query_desc;

/* ---- incremental aggregation: core/aggregation/ + util/parser/AggregationParser.java ---- */
#define SH_DUR_SECONDS 0
#define SH_DUR_MINUTES 1
#define SH_DUR_HOURS 2
#define SH_DUR_DAYS 3
#define SH_DUR_MONTHS 4
#define SH_DUR_YEARS 5

/* `define aggregation A from S[filter] select g..., agg(col)... group by g...
 *   aggregate [by ts_col] every min_dur ... max_dur;` in the aggTimeZone system configuration
 *   (IncrementalTimeConverterUtil.java:33-231: hour / day / month / year buckets start at the zone's
 *   local boundaries), given as a fixed offset from GMT (tz_offset_ms, whole minutes; 0 = GMT).
 * Per duration the library keeps the base values AggregationParser derives
 * (avg -> sum + count, count -> sum of 1L; AggregationParser.java:693-728). */
typedef struct {
    int32_t n_cols;
    int32_t col_types[SH_MAX_COLS];
    int32_t n_filter_ops;
    const sh_filter_op* filter;
    int32_t n_group_by;
    int32_t group_by[SH_MAX_GROUP];
    int32_t n_aggs;
    sh_agg_spec aggs[SH_MAX_AGGS];
    int32_t ts_col;       /* `aggregate by` attribute (LONG); -1 = processing time only */
    int32_t min_duration; /* SH_DUR_*                                                    */
    int32_t max_duration;
    int64_t key_capacity;
    int64_t tz_offset_ms; /* aggTimeZone as a fixed offset (e.g. Asia/Singapore: +8 h = 28800000) */
} sh_aggregation_desc;

/* ---- input batch: a run of InputHandler.send(Event[]) calls -----------------------------
 * One sh_batch stands for `n_sends` consecutive sends (core/stream/input/InputHandler.java:85-96),
 * processed with the per-send semantics of the reference (clock set from the send's last event
 * in playback mode, timers fired before the send is processed: Scheduler.java:71-104).
 *   send_size > 0 : consecutive sends of send_size events (the last may be shorter);
 *   send_size == 0: one send of all n events.
 * Columns are SoA, column c holds n values of col_types[c] (int32 for INT/STRID, uint8 BOOL).
 * For sh_push the pointers are host memory; for sh_push_device they are device memory. A column
 * the query does not read (not in the filter, group-by, partition key, aggregators or time
 * attributes) may be NULL: the shim packs only what the query reads; a NULL column the query reads
 * fails the call (SH_ERR_INVALID) before anything runs (sh_push, sh_push_device, sh_stage). */
typedef struct {
    int64_t n;
    int64_t send_size;
    const int64_t* ts; /* Event.getTimestamp() per event                                 */
    const void* cols[SH_MAX_COLS];
} sh_batch;

/* ---- output -------------------------------------------------------------------------------
 * One flush = one selector output chunk = one StreamCallback.receive(Event[]) call
 * (core/query/output/ratelimit/OutputRateLimiter.java:64-104). Rows are in the reference's
 * order (first-occurrence order of the group key inside the flush, QuerySelector.java:315-374);
 * a row carries the timestamp and aggregate values of the key's last qualifying event.
 * vals are raw 8-byte slots: int64 for LONG/INT outputs, IEEE double bits for DOUBLE/FLOAT.
 * rep is that last qualifying event itself — the event QuerySelector.processInBatchGroupBy keeps
 * per key in its LinkedHashMap (QuerySelector.java:315-374) and whose non-aggregated select
 * attributes (e.g. `volume` in `select symbol, sum(price), volume`) the output event carries — as
 * its stream index: events are numbered from 0 in arrival order over every event ever pushed into
 * the query (filtered-out ones included; for sh_shard_* the global stream index). The Java shim
 * keeps the events of the open window and reads the row's other attributes from rep. NULL for
 * aggregation tables. */
typedef struct {
    int64_t n_flushes;
    int64_t n_rows;
    int32_t n_keys;
    int32_t n_vals;
    int32_t val_types[SH_MAX_AGGS];
    const int64_t* flush_offsets; /* [n_flushes + 1]                                       */
    const int64_t* flush_clock;   /* [n_flushes] clock of the send / timer that emitted it */
    const int64_t* ts;            /* [n_rows]                                              */
    const uint8_t* expired;       /* [n_rows] 1 = EXPIRED before OutputRateLimiter's flip  */
    const int64_t* keys;          /* [n_keys][n_rows] group-by values widened to int64     */
    const uint64_t* vals;         /* [n_vals][n_rows]                                      */
    const uint8_t* nulls;         /* [n_vals][n_rows] 1 = Java null                         */
    const int64_t* rep;           /* [n_rows] stream index of the row's representative event */
} sh_out;

/* Rows written to one duration's aggregation table (core/aggregation/IncrementalExecutor.java:
 * 201-258). keys[0] is AGG_TIMESTAMP of the bucket (event-time bucket when `aggregate by` is
 * used), keys[1..] the group-by values; vals are the base values in the order
 * (per agg: SUM -> sum, AVG -> sum,count, COUNT -> count, MIN -> min, MAX -> max),
 * de-duplicated as AggregationParser.populateFinalBaseAggregators does.                  */

/* ---- lifecycle ---------------------------------------------------------------------------*/
typedef struct sh_ctx sh_ctx;
typedef struct sh_query sh_query;
typedef struct sh_aggregation sh_aggregation;

/* Device context on `device` (HIP ordinal). Multi-GPU: one process per GPU, each with its own
 * context; sharding is done by the caller.                       */
int sh_init(int32_t device, sh_ctx** out);
int sh_ctx_destroy(sh_ctx* ctx);

/* Replaces WindowProcessor.init + AttributeAggregatorExecutor.initAggregator + SelectorParser
 * (core/query/processor/stream/window/BatchingWindowProcessor.java:63-67,
 *  core/query/selector/attribute/aggregator/AttributeAggregatorExecutor.java:43-57).        */
int sh_query_create(sh_ctx* ctx, const sh_query_desc* desc, sh_query** out);
int sh_query_destroy(sh_query* q);

/* Replaces InputHandler.send(Event[]) -> filter -> window.process -> QuerySelector.process ->
 * OutputRateLimiter for every send in the batch. Host-memory batch (H2D included).          */
int sh_push(sh_query* q, const sh_batch* batch, const sh_out** out);
/* Same with device-resident columns (the HBM-resident hot path). flush_offsets/flush_clock of
 * *out are host memory (NULL in the compact form, sh_query_set_compact_flushes), for every window
 * kind; ts/expired/keys/vals/nulls/rep are device pointers (results stay in HBM). */
int sh_push_device(sh_query* q, const sh_batch* batch, const sh_out** out);
/* TIMER path: advance the playback clock to `now` without events (Scheduler.onTimeChange). */
int sh_advance_time(sh_query* q, int64_t now, const sh_out** out);

/* Output rate limiting `output [all|first|last] every <n> events` (core/query/output/ratelimit/event/:
 * AllPerEvent, FirstPerEvent, LastPerEvent and, for group-by queries, FirstGroupByPerEvent /
 * LastGroupByPerEventOutputRateLimiter.java) and `output first every <n> milliseconds`
 * (core/query/output/ratelimit/time/FirstPerTimeOutputRateLimiter.java:54-78, for group-by queries
 * FirstGroupByPerTimeOutputRateLimiter.java:54-80: they read the playback clock, so they are
 * deterministic; the all/last time limiters arm a wall-clock schedule and are not offered). Set once,
 * before the first push; every later output (push, advance_time) goes through the limiter: one flush
 * per input flush that emits rows. */
#define SH_RATE_NONE 0
#define SH_RATE_ALL 1
#define SH_RATE_FIRST 2
#define SH_RATE_LAST 3
#define SH_RATE_FIRST_TIME 4
int sh_query_set_output_rate(sh_query* q, int32_t kind, int64_t n);
/* The limiter of a sharded query (ABI 16; OutputRateLimiter.process sits after the selector, so it sees
 * the merged single-stream output): `q` is a query created from the same descriptor with its rate set
 * and never pushed; the merging rank passes every merged call output (host arrays, flush by flush, in
 * stream order — pushes and advance_time calls alike) and gets the limited output back (host arrays).
 * The limiter's kernels run on q's device. */
int sh_rate_apply_merged(sh_query* q, const sh_out* merged, const sh_out** out);

/* externalTimeBatch's fourth parameter, the scheduler timeout in milliseconds
 * (ExternalTimeBatchWindowProcessor.java:196-207, `externalTimeBatch(ts, 1 sec, 0, 6 sec)`): when the
 * playback clock passes the last scheduled time (clock of the window's first event, of every batch
 * crossing and of every timeout, + ms) the open batch goes out so far (:256-275) — again whole, with
 * its new events, at a later timeout or at its crossing (appendToOutputChunk, :385-438); with expired
 * output every emission carries the previous emission's events as EXPIRED. Under `partition with` every
 * partition keeps its own last scheduled time and partitions due at the same time fire in the
 * Scheduler's HashMap order (Scheduler.java:71-104; int / long / bool keys, or string keys with their
 * text set through sh_query_set_strings). Replaces the Java window's timeout argument. Set once, before
 * the first push; refused (SH_ERR_UNSUPPORTED) on sharded queries, with stream.current.event and with
 * float / double partition keys. ms == 0 is no timeout. */
int sh_query_set_ext_timeout(sh_query* q, int64_t ms);

/* externalTimeBatch's fifth parameter, replaceTimestampWithBatchEndTime (ExternalTimeBatchWindowProcessor.java:
 * 210-220, cloneAppend :446-456; `externalTimeBatch(ts, 1 sec, 0, 100, true)`): the window's copy of every event
 * carries its batch's end time in the timestamp attribute (ts_col), so the output events built from the rows'
 * representative events show the batch end, not the sent value. sh_query_rep_ts_attr returns that attribute for
 * every row of the last output (host array, valid until the next call on the query); the shim writes it into
 * the row's select attributes. Set once, before the first push, on an externalTimeBatch query (partitioned:
 * each partition's own batch ends); aggregators and group keys over the timestamp attribute (which would fold
 * the replaced values), sharded queries and partitioned queries with an output rate limiter are refused
 * (SH_ERR_UNSUPPORTED). Replaces the Java window's fifth argument. */
int sh_query_set_ext_replace_ts(sh_query* q, int32_t on);
int sh_query_rep_ts_attr(sh_query* q, const int64_t** values, int64_t* n);

/* Compact flushes: when on, an output in which every flush holds exactly one row and every flush's clock
 * equals that row's timestamp (stream.current.event output, `timeBatch(T, true)` / `lengthBatch(L, true)`,
 * sends of one event) comes back with flush_offsets = flush_clock = NULL and n_flushes = n_rows: flush i
 * is row i, emitted at clock ts[i]. Any other output keeps the full arrays, so a caller that sets this
 * checks flush_offsets for NULL. Saves the 16 B per row the flush arrays would cost (host memory even for
 * sh_push_device). Off by default; queries with an output rate limiter always get the full form. */
int sh_query_set_compact_flushes(sh_query* q, int32_t on);
/* Device flush layout: when on, sh_push_device leaves flush_offsets / flush_clock in device memory too
 * (a consumer on the GPU: nothing of the output crosses PCIe). The compact form, when it applies, still
 * comes first (NULL arrays). Queries with an output rate limiter keep the host layout. Off by default. */
int sh_query_set_device_flushes(sh_query* q, int32_t on);

/* The text of dictionary ids [first_id, first_id + n) of string column `col`, as UTF-16 code units (what a
 * java.lang.String holds): id first_id + i is units[offsets[i] .. offsets[i + 1]) (offsets has n + 1
 * entries). May be called again to extend the range as the shim's dictionary grows; an id keeps its text.
 * Needed where the reference's output depends on the string itself, not only on equality: the partition
 * key of `partition with (k of S)` around a `time` window with expired / all-events output, whose
 * Scheduler fires, of several partitions due at the same time, the first in java.util.HashMap<String, …>
 * iteration order (String.hashCode, String.compareTo; Scheduler.java:71-104,363-366,
 * PartitionStateHolder.java:36-83). A push that needs an id without text fails (SH_ERR_INVALID).
 * Replaces nothing in the reference: the Java shim calls it when it assigns dictionary ids. */
int sh_query_set_strings(sh_query* q, int32_t col, int64_t first_id, int64_t n, const uint16_t* units,
                         const int64_t* offsets);

/* Checkpoint of the query's state: State.snapshot()/restore() (core/util/snapshot/state/State.java:
 * 26-36) driven by SnapshotService.persist/restore (core/util/snapshot/SnapshotService.java:90-296)
 * — the open window's queued events (and lengthBatch count), the sliding window's queue with every
 * key's aggregator state and min/max deques, the partition key, the playback clock and
 * nextEmitTime. Two calls: buf = NULL returns the size in *len. A blob restores only into a query
 * created from the same descriptor (SH_ERR_INVALID otherwise); the restored query then continues
 * exactly as the snapshotted one would have. */
int sh_query_snapshot(sh_query* q, void* buf, int64_t cap, int64_t* len);
int sh_query_restore(sh_query* q, const void* buf, int64_t len);

int sh_aggregation_create(sh_ctx* ctx, const sh_aggregation_desc* desc, sh_aggregation** out);
int sh_aggregation_destroy(sh_aggregation* a);
/* AggregationRuntime.processEvents via IncrementalAggregationProcessor.process
 * (core/aggregation/IncrementalAggregationProcessor.java:66-101). */
int sh_aggregation_push(sh_aggregation* a, const sh_batch* batch);
int sh_aggregation_push_device(sh_aggregation* a, const sh_batch* batch);
int sh_aggregation_advance_time(sh_aggregation* a, int64_t now);
/* Rows added to the table of `duration` since the previous call for that duration. */
int sh_aggregation_table(sh_aggregation* a, int32_t duration, const sh_out** out);
/* Retrieval `from A within start, end per "<per>"` (AggregationRuntime.find ->
 * IncrementalAggregateCompileCondition.find, core/util/collection/operator/
 * IncrementalAggregateCompileCondition.java:180-290): the `per` table's rows plus the in-memory
 * stores of the executors `per` .. root re-bucketed to `per` (IncrementalDataAggregator.java:92-143),
 * merged by (AGG_TIMESTAMP, key) and restricted to start <= AGG_TIMESTAMP < end. Host rows as
 * sh_aggregation_table (keys[0] = AGG_TIMESTAMP, keys[1] = the group key, base values), ordered by
 * (AGG_TIMESTAMP, key). The caller evaluates the select expressions (avg = sum / count, ...) and
 * resolves `within` patterns / time strings to [start, end). */
int sh_aggregation_find(sh_aggregation* a, int32_t per, int64_t start, int64_t end, const sh_out** out);
/* Checkpoint of an aggregation (SnapshotService.persist/restore, SnapshotService.java:90-296): the root
 * window, every roll-up executor's state and store (IncrementalExecutor.java:283-317,
 * BaseIncrementalValueStore.java:231-262) and the duration tables. Two calls as sh_query_snapshot;
 * restores only into an aggregation created from the same descriptor. Not for sharded aggregations. */
int sh_aggregation_snapshot(sh_aggregation* a, void* buf, int64_t cap, int64_t* len);
int sh_aggregation_restore(sh_aggregation* a, const void* buf, int64_t len);

/* ---- sharded ingest across G GPUs (one process per GPU) ---------------------
 * Rank g of G holds slice g of every global micro-batch: a contiguous run of the global stream
 * (rank order = stream order), cut at send boundaries (send_size >= 1). Group keys are re-sharded
 * to owner = mix64(key) % G over an all-to-all that the CALLER performs (RCCL through
 * torch.distributed, or any transport): the library only packs and consumes device buffers.
 * The playback clock, nextEmitTime and the window of every event are global quantities
 * (TimeBatchWindowProcessor.java:262-347, Scheduler.java:71-127); they are computed from the G
 * slice summaries, which every rank all-gathers, so each owner reproduces the single-stream
 * windows exactly. One global push is:
 *   1. sh_shard_summarize(slice)                 -> sh_slice_summary      [caller: all-gather]
 *   2. sh_shard_pack(all summaries, slice, buf)  -> per-owner byte counts + this slice's window
 *                                                   starts                [caller: all-to-all the
 *                                                   bytes, all-gather the sh_bound lists]
 *   3. sh_shard_consume(received bytes, all bounds) -> this owner's flushes (its keys only) plus
 *                                                   `order`: the global stream index of each row's
 *                                                   first event, so merging the G outputs of a
 *                                                   flush by `order` yields the single-stream row
 *                                                   order of QuerySelector.processInBatchGroupBy.
 * Supported: timeBatch group-by, partitioned or not (`partition with (p of S)`: R12 — every rank
 * restricts the stream to the partition of the globally first passing event), lengthBatch
 * group-by (batch = global filtered index / L, LengthBatchWindowProcessor.java:206-243: the
 * summaries' pass counts give every slice its offset; a batch's sh_bound carries the clock of the
 * send of its L-th event, where it is flushed), and incremental aggregations through
 * sh_aggregation_shard_create (below). Several lengthBatch batches can close in one send (same
 * flush clock): merge owner flushes by (clock, window of their rows' `order`). Sliding time(T)
 * group-by (TimeWindowProcessor.java:132-169, not partitioned): the source slice gives every passing
 * event its send's global clock and PM (max ts over the stream's passing events up to it, the expiry
 * key) — both travel in the record — and the owner replays its keys' windows; it emits one flush per
 * global send, so merge owner flushes by send number ((order - push's first index) / send_size) and
 * rows by `order`. Sliding records carry 2 extra words: at most 6 stream columns.
 * `insert expired events` / `insert all events` of the batch windows: an owner's flush closing global
 * window W holds the expired rows of its keys of W-1 and the current rows of W; a row's `order` is
 * the first occurrence of its key in W-1 where it takes an expired row's place (LinkedHashMap.put,
 * QuerySelector.processInBatchGroupBy :315-374), else in W — so merge owner flushes by (clock,
 * sh_shard_flush_windows) and rows by `order`.                                                  */
typedef struct {
    int64_t n;           /* events in the slice                                              */
    int64_t n_pass;      /* events passing the filter                                        */
    int64_t max_tl;      /* max timestamp over the slice's send-last events (INT64_MIN: none) */
    int64_t first_clock; /* clock of the send of the slice's first passing event, without the
                            clock carried in (INT64_MIN: no passing event)                    */
    int64_t first_key;   /* partitioned queries: partition key of that event (R12: the globally
                            first one picks the only partition that ever flushes); sliding
                            time(T): max ts over the slice's passing events (INT64_MIN: none,
                            the slice's PM contribution); else 0                              */
    int64_t ts_min;      /* min / max timestamp over the slice's events (INT64_MAX / INT64_MIN:  */
    int64_t ts_max;      /* empty): when the whole push spans less than 2^32, every record carries
                            its timestamp as a 32-bit offset from the push's minimum (ABI 11:
                            20-byte C2 records instead of 24)                                 */
} sh_slice_summary;

typedef struct {
    int64_t W;     /* window number that starts here                                         */
    int64_t clock; /* flush clock of window W-1: timeBatch, the clock of the send that opened
                      W; lengthBatch, the clock of the send holding W-1's L-th event          */
    int64_t gidx;  /* global stream index of the first event of window W                    */
    int64_t pad;
} sh_bound;

typedef struct sh_shard sh_shard;
int sh_shard_create(sh_ctx* ctx, const sh_query_desc* desc, int32_t rank, int32_t world, sh_shard** out);
int sh_shard_destroy(sh_shard* s);
/* Bytes per packed event record at most (depends on the query's value columns; a push whose events
 * span less than 2^32 in time packs 4 bytes less per record when the wire key is 32-bit). */
int sh_shard_record_bytes(sh_shard* s, int64_t* out);
/* Phase 1 (device slice). */
int sh_shard_summarize(sh_shard* s, const sh_batch* slice, sh_slice_summary* out);
/* Phase 2: `all` = the G summaries in rank order; `send_buf` = caller-owned device buffer of at
 * least slice.n * record_bytes; on return send_bytes[o] bytes for owner o lie contiguously in
 * owner order; *bounds (host, valid until the next call) lists the windows starting in this slice. */
int sh_shard_pack(sh_shard* s, const sh_slice_summary* all, const sh_batch* slice, void* send_buf,
                  int64_t send_cap, int64_t* send_bytes, const sh_bound** bounds, int64_t* n_bounds);
/* Phase 3: recv_buf = the G received blocks concatenated in source-rank order (device),
 * recv_bytes[g] their sizes; all_bounds = every rank's bound list (any order). host_out selects
 * host (1) or device (0) row arrays, as sh_push / sh_push_device. *order has n_rows entries. */
int sh_shard_consume(sh_shard* s, const void* recv_buf, const int64_t* recv_bytes, const sh_bound* all_bounds,
                     int64_t n_all_bounds, int32_t host_out, const sh_out** out, const int64_t** order);
/* TIMER path of the sharded query: every rank calls it with the same `now`. */
int sh_shard_advance_time(sh_shard* s, int64_t now, int32_t host_out, const sh_out** out, const int64_t** order);
/* The window each flush of the last consume / advance closes (host array of *n entries, valid until the
 * next call; n = 0 for sliding windows): the G owners' flushes of one global flush share (clock, window). */
int sh_shard_flush_windows(sh_shard* s, const int64_t** windows, int64_t* n);
/* Checkpoint of one rank's shard (SnapshotService.persist/restore, SnapshotService.java:90-296): the
 * global stream state every rank keeps (clock, nextEmitTime, batch count, stream index, p0) and its
 * owner query's windows. Taken between pushes on every rank; restored into a shard created from the
 * same descriptor, rank and world. Two calls as sh_query_snapshot. A sharded aggregation's shard
 * (sh_aggregation_shard_create) also carries its roll-up executors and duration tables. */
int sh_shard_snapshot(sh_shard* s, void* buf, int64_t cap, int64_t* len);
int sh_shard_restore(sh_shard* s, const void* buf, int64_t len);
/* Key-sharded incremental aggregation (C4 across G GPUs): *shard ingests through the three phases
 * above (owner = the group key's owner; an event's time bucket travels as its raw `aggregate by`
 * column), and every owner runs the root and all roll-up levels of its keys, so the union of the G
 * owners' sh_aggregation_table rows is the single-stream table. Replaces the single-stream
 * AggregationRuntime.processEvents -> IncrementalExecutor.execute chain (IncrementalExecutor.java:
 * 110-258). consume/advance_time output the root's flushes (device); tables are read with
 * sh_aggregation_table(*agg, ...); sh_shard_destroy(*shard) releases both handles. */
int sh_aggregation_shard_create(sh_ctx* ctx, const sh_aggregation_desc* desc, int32_t rank, int32_t world,
                                sh_shard** shard, sh_aggregation** agg);

/* Pinned host buffers for zero-copy packing of Event[] chunks (hipHostMalloc). */
int sh_alloc_pinned(int64_t bytes, void** out);
int sh_free_pinned(void* p);

/* Double-buffered host ingest: the Java side packs each ComplexEventChunk micro-batch into pinned
 * SoA buffers (sh_alloc_pinned) and hands it over as InputHandler.send(Event[]) would
 * (InputHandler.java:85-96 -> StreamJunction.sendEvent, StreamJunction.java:104-131; the @async
 * junction's batching, :279-316). sh_stage queues the batch's H2D copy into one of the query's two
 * device staging slots on the context's copy stream and returns at once with a ticket;
 * sh_push_staged(ticket) runs the push once that copy has landed, with host output as sh_push.
 * Staging batch i+1 before pushing batch i overlaps its PCIe copy with batch i's kernels. At most
 * two tickets are outstanding; they are pushed in staging order; a staged batch's host buffers must
 * stay unchanged until its push returns. sh_ingest_stats: HIP-event time and bytes of the H2D copy
 * of the last pushed batch (copy stream). */
int sh_stage(sh_query* q, const sh_batch* batch, int32_t* ticket);
int sh_push_staged(sh_query* q, int32_t ticket, const sh_out** out);
int sh_ingest_stats(sh_query* q, double* h2d_ms, int64_t* h2d_bytes);

/* Device timing of the last push: kernel time of the dominant kernel and of the whole push. */
typedef struct {
    double push_ms;        /* HIP-event time of the whole device pipeline of the last push */
    double main_kernel_ms; /* HIP-event time of the aggregation kernel(s)                   */
    int64_t main_kernel_bytes; /* algorithmic bytes the aggregation kernel(s) moved          */
    int64_t events;        /* events consumed by the last push                              */
} sh_stats;
int sh_query_stats(sh_query* q, sh_stats* out);
/* The same for the owner pipeline of a sharded query (its last sh_shard_consume). */
int sh_shard_stats(sh_shard* s, sh_stats* out);
/* The same for an aggregation's last push: push_ms covers the root window and every roll-up level
 * (IncrementalExecutor chain, core/aggregation/IncrementalExecutor.java:110-258), main_kernel_ms the
 * root's base aggregation. */
int sh_aggregation_stats(sh_aggregation* a, sh_stats* out);
/* HIP-event device time of the whole pipeline summed over every push since the last reset, read
 * without a wait per push (sh_aggregation_stats waits for the last push): pushes still running are
 * waited for by this call. reset != 0 zeroes the sum after reading it. */
int sh_aggregation_timing(sh_aggregation* a, double* total_ms, int64_t* pushes, int32_t reset);

const char* sh_last_error(void);
int32_t sh_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* SIDDHI_HIP_H */
