// sh_window.cpp — batch-window group-by queries (lengthBatch / timeBatch) behind sh_query_*.
//
// Replaces, for the query shape `from S[cond]#window.lengthBatch|timeBatch(...) select k, aggs group by k
// insert into O`, the chain FilterProcessor -> {LengthBatch,TimeBatch}WindowProcessor -> QuerySelector
// (processInBatchGroupBy) -> OutputRateLimiter of the reference. The window's queued events are kept on
// the device (pending buffer); a push runs whole windows in parallel and emits every window that
// closed during the push as one flush, exactly as the reference emits one chunk per flush.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sh_agg.h"
#include "sh_internal.h"
#include "sh_runtime.h"
#include "sh_wide.h"

using namespace shd;

#define HIPCHK(x)                                                                                          \
    do {                                                                                                   \
        hipError_t _e = (x);                                                                               \
        if (_e != hipSuccess) return sh_fail(SH_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
    } while (0)
#define RCHK(x)            \
    do {                   \
        int _r = (x);      \
        if (_r) return _r; \
    } while (0)

size_t type_size(int t) {
    switch (t) {
        case SH_T_LONG: case SH_T_DOUBLE: return 8;
        case SH_T_BOOL: return 1;
        default: return 4;
    }
}

int StagedBatch::stage(hipStream_t s, const sh_batch* b, int n_cols, const int32_t* types, sh_batch* dev) {
    *dev = *b;
    size_t n = (size_t)b->n;
    if (n == 0) return SH_OK;
    // a host batch laid out as one region — ts[n], then each column's n values, every run 16-byte
    // aligned (the pinned layout the shim packs) — goes over in ONE copy
    {
        auto a16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
        const char* base = (const char*)b->ts;
        size_t off = a16(n * 8), offs[SH_MAX_COLS] = {}, end = n * 8;
        bool contig = true;
        for (int c = 0; c < n_cols && contig; c++) {
            if (!b->cols[c]) continue;
            contig = (const char*)b->cols[c] == base + off;
            offs[c] = off;
            end = off + n * type_size(types[c]);  // the copy stops at the last column's last value
            off = a16(end);
        }
        if (contig) {
            RCHK(blk.reserve(off, false));
            HIPCHK(hipMemcpyAsync(blk.p, base, end, hipMemcpyHostToDevice, s));
            dev->ts = blk.as<int64_t>();
            for (int c = 0; c < n_cols; c++) dev->cols[c] = b->cols[c] ? blk.as<char>() + offs[c] : nullptr;
            return SH_OK;
        }
    }
    RCHK(ts.reserve(n * 8, false));
    HIPCHK(hipMemcpyAsync(ts.p, b->ts, n * 8, hipMemcpyHostToDevice, s));
    dev->ts = ts.as<int64_t>();
    for (int c = 0; c < n_cols; c++) {
        if (!b->cols[c]) { dev->cols[c] = nullptr; continue; }
        size_t bytes = n * type_size(types[c]);
        RCHK(cols[c].reserve(bytes, false));
        HIPCHK(hipMemcpyAsync(cols[c].p, b->cols[c], bytes, hipMemcpyHostToDevice, s));
        dev->cols[c] = cols[c].p;
    }
    return SH_OK;
}

int64_t cal_idx_h(int64_t t, int cal, int64_t tz);
static int64_t wfun_host(const sh_query* q, int64_t clock) {
    if (!q->e0_valid) return q->W_open;
    if (q->cal) return clock < q->E0 ? 0 : cal_idx_h(clock, q->cal, q->cal_tz) - cal_idx_h(q->E0, q->cal, q->cal_tz) + 1;
    return clock < q->E0 ? 0 : (clock - q->E0) / q->d.window_param + 1;
}

static int grow_pending(sh_query* q, int64_t need, int64_t keep) {
    if (need <= q->pend_cap) return SH_OK;
    int64_t ncap = std::max<int64_t>(need, q->pend_cap + q->pend_cap / 2);
    ncap = std::max<int64_t>(ncap, 4096);
    DevBuf np, nt, nv, ng;
    RCHK(np.reserve(ncap * 4, false));
    RCHK(nt.reserve(ncap * 8, false));
    RCHK(nv.reserve(std::max(1, q->ap.n_vcols) * ncap * 8, false));
    RCHK(ng.reserve(ncap * 8, false));
    hipStream_t s = q->ctx->stream;
    if (keep > 0) {
        HIPCHK(hipMemcpyAsync(ng.p, q->pend_gidx.p, keep * 8, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(np.p, q->pend_pos.p, keep * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(nt.p, q->pend_ts.p, keep * 8, hipMemcpyDeviceToDevice, s));
        for (int j = 0; j < q->ap.n_vcols; j++)
            HIPCHK(hipMemcpyAsync((char*)nv.p + j * ncap * 8, (char*)q->pend_vals.p + j * q->pend_cap * 8, keep * 8,
                                  hipMemcpyDeviceToDevice, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    q->pend_pos = std::move(np); q->pend_ts = std::move(nt); q->pend_vals = std::move(nv); q->pend_gidx = std::move(ng);
    q->pend_cap = ncap;
    return SH_OK;
}

static int query_create(sh_ctx* ctx, const sh_query_desc* d, const KeyPlan* kp_override, sh_query** out);
int query_set_partition(sh_query* q, int64_t key);

// Key partitions: the smallest power of two P that leaves at most 512 local keys per partition (the
// aggregation kernel's threads own one local key each, state in registers), as long as the
// multisplit's per-tile LDS (staging + per-wave partition counters) fits a CU.
static bool scatter_fits(const sh_query* q, int p) {
    const int nv = q->ap.n_vcols;
    size_t v = nv <= 1 ? 1 : nv <= 2 ? 2 : nv <= 4 ? 4 : 8;
    return v * kTile * 8 + (size_t)kTile * 8 + (size_t)p * 20 + 64 <= 160 * 1024;
}

// the largest key table the partitioning supports (512 local keys per partition)
static size_t max_table_size(const sh_query* q) {
    int P = 1;
    while (P < 16384 && scatter_fits(q, P << 1)) P <<= 1;
    return (size_t)P * 512;
}

static int size_partitions(sh_query* q) {
    const size_t ts = q->kt.size_;
    auto scatter_fits = [&](int p) { return ::scatter_fits(q, p); };
    int P = 1;
    // local keys per partition: at most 512 (one per thread of k_aggregate_own) or, for experiments,
    // 1024 (two per thread) — SH_PART_KEYS
    const size_t nl_max = q->tune.part_keys_1024 ? 1024 : 512;
    while (ts / P > nl_max && P < 16384 && scatter_fits(P << 1)) P <<= 1;
    if (ts / P > nl_max) return sh_fail(SH_ERR_UNSUPPORTED, "key capacity too large for one GPU (shard the query over GPUs)");
    q->P = P;
    q->logP = 0;
    while ((1 << q->logP) < P) q->logP++;
    // local keys per partition: the hash table's sentinel slot (mask + 1) adds one to partition 0
    q->NL = (int)(ts / P) + (q->kt.dense ? 0 : 1);
    return SH_OK;
}

// Move the open window's keys into a fresh table of `size` slots: keys of closed windows are dead
// (their group states were destroyed on flush, R9), so the rebuild drops them; the pending events'
// slot positions are remapped.
// On return `nk` holds the old table (a caller may keep it as a spare: no allocation next time). A band
// target (arithmetic slots, the caller placed every queued bucket inside it) is not read back: no sync.
int query_swap_keys(sh_query* q, KeyTableHost& nk) {
    launch_rekey(q->ctx->stream, q->n_pend, q->pend_pos.as<u32>(), q->kt.dev(), nk.dev());
    HIPCHK(hipGetLastError());
    if (!nk.lk) RCHK(nk.check(q->ctx->stream));
    std::swap(q->kt, nk);
    return size_partitions(q);
}

static int rekey(sh_query* q, size_t size) {
    KeyTableHost nk;
    RCHK(nk.init_size(size));
    return query_swap_keys(q, nk);
}

int query_reserve_keys(sh_query* q, int64_t extra) {
    if (q->kt.dense) return SH_OK;  // slots are the dictionary ids themselves
    int64_t ts = (int64_t)q->kt.size_;
    if (q->kt.n_keys + extra <= ts / 2) return SH_OK;
    auto pow2_for = [](int64_t n) {
        size_t w = 16;
        while ((int64_t)w < 2 * n) w <<= 1;
        return w;
    };
    // the open window's keys survive the rebuild: at most min(keys so far, queued events)
    int64_t live = std::min<int64_t>(q->kt.n_keys, q->n_pend);
    bool compacted = false;
    if (std::max(pow2_for(live + extra), q->kt_min_size) > max_table_size(q)) {
        // that bound is too loose to fit: compact to the live keys first (the rebuild counts them)
        RCHK(rekey(q, std::max(pow2_for(live), q->kt_min_size)));
        live = q->kt.n_keys;
        compacted = true;
        SH_TRACE("reserve_keys: compacted to %lld live keys", (long long)live);
    }
    const size_t want = std::max(pow2_for(live + extra), q->kt_min_size);
    SH_TRACE("reserve_keys: n_keys=%lld n_pend=%lld extra=%lld size=%lld -> %lld", (long long)q->kt.n_keys,
             (long long)q->n_pend, (long long)extra, (long long)ts, (long long)want);
    return compacted && want == q->kt.size_ ? SH_OK : rekey(q, want);
}

// Group keys the window cannot key directly (three or more columns, a long / double beside another
// column; GroupByKeyGenerator.java:63-73): the query is built over the stream plus one synthetic
// dictionary column holding every event's interned key id (sh_wide.h), grouped by that column alone.
static int wide_create(sh_ctx* ctx, const sh_query_desc* d, sh_query** out) {
    if (d->n_cols <= 0 || d->n_cols >= SH_MAX_COLS)
        return sh_fail(SH_ERR_UNSUPPORTED, "wide group keys need a spare column slot (fewer than 8 columns)");
    for (int i = 0; i < d->n_group_by; i++)
        if (d->group_by[i] < 0 || d->group_by[i] >= d->n_cols) return sh_fail(SH_ERR_INVALID, "group-by column out of range");
    for (int c = 0; c < d->n_cols; c++)
        if (d->col_types[c] < SH_T_INT || d->col_types[c] > SH_T_BOOL) return sh_fail(SH_ERR_INVALID, "bad column type");
    WideKeys* w = new WideKeys();
    int rc = w->init(d->n_group_by, d->group_by, d->n_cols, d->col_types,
                     d->key_capacity > 0 ? d->key_capacity : (1 << 16));
    if (rc) { delete w; return rc; }
    sh_query_desc in = *d;
    in.n_cols = d->n_cols + 1;
    in.col_types[d->n_cols] = SH_T_STRID;
    in.n_group_by = 1;
    in.group_by[0] = d->n_cols;
    in.key_capacity = w->id_space();
    sh_query* q = nullptr;
    if ((rc = query_create(ctx, &in, nullptr, &q))) { delete w; return rc; }
    q->wide = w;
    q->wide_n_cols = d->n_cols;
    uint32_t m = q->cols_used & ~(1u << d->n_cols);
    for (int i = 0; i < d->n_group_by; i++) m |= 1u << d->group_by[i];
    q->wide_cols_used = m;
    *out = q;
    return SH_OK;
}

extern "C" int sh_query_create(sh_ctx* ctx, const sh_query_desc* d, sh_query** out) {
    StreamScope _ss(ctx ? ctx->stream : nullptr);
    if (d && out && d->n_group_by > 0 && d->n_group_by <= SH_MAX_GROUP && d->n_cols > 0 && d->n_cols <= SH_MAX_COLS) {
        bool in_range = true;
        for (int i = 0; i < d->n_group_by; i++) in_range &= d->group_by[i] >= 0 && d->group_by[i] < d->n_cols;
        // partitioned: the lanes key their (partition, group) pairs by one 32-bit group id, so a group key of
        // two columns or of one 64-bit / floating column other than the partition key is interned too (its
        // keyed output rate limiters then run on the id)
        bool lanes_wide = false;
        if (in_range && d->partition_col >= 0 && d->n_cols < SH_MAX_COLS) {
            const int t0 = d->col_types[d->group_by[0]];
            lanes_wide = d->n_group_by >= 2 ||
                         (d->group_by[0] != d->partition_col && (t0 == SH_T_LONG || t0 == SH_T_DOUBLE || t0 == SH_T_FLOAT));
        }
        if (in_range && (lanes_wide || WideKeys::needed(d->n_group_by, d->group_by, d->col_types)))
            return wide_create(ctx, d, out);
    }
    return query_create(ctx, d, nullptr, out);
}

int sh_query_create_internal(sh_ctx* ctx, const sh_query_desc* d, const KeyPlan& kp, sh_query** out) {
    return query_create(ctx, d, &kp, out);
}

static int query_create(sh_ctx* ctx, const sh_query_desc* d, const KeyPlan* kp_override, sh_query** out) {
    if (!ctx || !d || !out) return sh_fail(SH_ERR_INVALID, "sh_query_create: NULL argument");
    if (d->n_cols <= 0 || d->n_cols > SH_MAX_COLS) return sh_fail(SH_ERR_INVALID, "bad column count");
    for (int c = 0; c < d->n_cols; c++)
        if (d->col_types[c] < SH_T_INT || d->col_types[c] > SH_T_BOOL) return sh_fail(SH_ERR_INVALID, "bad column type");
    const bool batch_win = d->window == SH_WIN_LENGTH_BATCH || d->window == SH_WIN_TIME_BATCH;
    const bool pass_through = d->n_aggs == 0 && d->n_group_by == 0 && d->partition_col < 0 &&
                              (batch_win || d->window == SH_WIN_EXT_TIME_BATCH || d->window == SH_WIN_TIME ||
                               d->window == SH_WIN_EXT_TIME);
    if ((d->n_aggs < 1 && !pass_through) || d->n_aggs > SH_MAX_AGGS)
        return sh_fail(SH_ERR_UNSUPPORTED,
                       "GPU path runs aggregation queries (1..8 aggregators) or pass-through lengthBatch / timeBatch / "
                       "time / externalTime windows");
    if (d->window != SH_WIN_LENGTH_BATCH && d->window != SH_WIN_TIME_BATCH && d->window != SH_WIN_TIME &&
        d->window != SH_WIN_EXT_TIME_BATCH && d->window != SH_WIN_EXT_TIME)
        return sh_fail(SH_ERR_UNSUPPORTED,
                       "GPU path needs a lengthBatch, timeBatch, time, externalTimeBatch or externalTime window");
    if (d->window == SH_WIN_EXT_TIME &&
        (d->ts_col < 0 || d->ts_col >= d->n_cols || d->col_types[d->ts_col] != SH_T_LONG))
        return sh_fail(SH_ERR_INVALID, "externalTime timestamp must be a long attribute");
    if (d->window == SH_WIN_EXT_TIME_BATCH) {
        if (d->ts_col < 0 || d->ts_col >= d->n_cols || d->col_types[d->ts_col] != SH_T_LONG)
            return sh_fail(SH_ERR_INVALID, "externalTimeBatch timestamp must be a long attribute");
        if (d->has_start_time == 2 &&
            (d->start_col < 0 || d->start_col >= d->n_cols || d->col_types[d->start_col] != SH_T_LONG))
            return sh_fail(SH_ERR_INVALID, "externalTimeBatch start time attribute must be long");
    }
    if (d->window_param <= 0) return sh_fail(SH_ERR_INVALID, "window length/period must be > 0");
    if (!d->current_on && !d->expired_on) return sh_fail(SH_ERR_INVALID, "query emits neither current nor expired events");
    const bool sliding_win = d->window == SH_WIN_TIME || d->window == SH_WIN_EXT_TIME;
    // partitioned lengthBatch / time keyed by the partition (no group-by, or group by the partition
    // key): one lane per partition (sh_plane.cpp)
    const bool by_partition = d->n_group_by == 0 || (d->n_group_by == 1 && d->group_by[0] == d->partition_col);
    // ... and partitioned lengthBatch grouped by other columns: (partition, group) rows by sorting (lane 3)
    // (and partitioned externalTimeBatch, any group-by: the same sorted chunks with batches by attribute time)
    const bool plane_ext = d->partition_col >= 0 && d->window == SH_WIN_EXT_TIME_BATCH && d->n_aggs >= 1;
    // (lengthBatch(L, true) grouped by other columns: current output, a row per event — k_pg_sc_*)
    const bool plane_group = (d->partition_col >= 0 && d->window == SH_WIN_LENGTH_BATCH && !by_partition &&
                              (!d->stream_current || !d->expired_on) && d->n_aggs >= 1) || plane_ext;
    // ... and time / externalTime grouped by other columns: the time lanes' operations, replayed per
    // (partition, group) state (count / sum / avg)
    const bool plane_time_group = d->partition_col >= 0 && (d->window == SH_WIN_TIME || d->window == SH_WIN_EXT_TIME) &&
                                  !by_partition && d->n_aggs >= 1;
    // ... and timeBatch(T, true) (stream.current.event), current output: every partition's chunks go out
    // with its groups' running values, a partition RESET only where its own chunk or TIMER meets the shared
    // nextEmitTime (lane 4)
    const bool plane_tbsc = d->partition_col >= 0 && d->window == SH_WIN_TIME_BATCH && d->stream_current &&
                            d->n_aggs >= 1 && d->current_on && !d->expired_on;
    const bool plane = (d->partition_col >= 0 &&
                        (d->window == SH_WIN_LENGTH_BATCH || d->window == SH_WIN_TIME || d->window == SH_WIN_EXT_TIME) &&
                        by_partition) || plane_group || plane_time_group || plane_tbsc;
    // partitioned timeBatch (R12): only the partition that armed the shared nextEmitTime ever flushes, with
    // its own expired queue (TimeBatchWindowProcessor.process :262-340 per partition state), so its expired
    // / all-events output is the unpartitioned form over that partition's events
    const bool r12_batch = d->partition_col >= 0 && d->window == SH_WIN_TIME_BATCH && !d->stream_current && !plane;
    if ((!d->current_on || d->expired_on) &&
        !((batch_win || sliding_win || d->window == SH_WIN_EXT_TIME_BATCH) && d->partition_col < 0) && !plane &&
        !r12_batch)
        return sh_fail(SH_ERR_UNSUPPORTED,
                       "expired / all-events output runs on lengthBatch, timeBatch, externalTimeBatch, time and "
                       "externalTime windows (partitioned: timeBatch, lengthBatch, and time grouped by the partition key)");
    // (partitioned: lengthBatch lanes, every event its own chunk of one key)
    if (d->stream_current &&
        !(batch_win && d->n_aggs >= 1 && (d->partition_col < 0 || (plane && d->window == SH_WIN_LENGTH_BATCH) || plane_tbsc)))
        return sh_fail(SH_ERR_UNSUPPORTED,
                       "stream.current.event runs on aggregating lengthBatch / timeBatch windows (partitioned: "
                       "lengthBatch; grouped by other columns with current output; timeBatch with current output)");
    if (d->partition_col >= 0 && d->window != SH_WIN_TIME_BATCH && !plane)
        return sh_fail(SH_ERR_UNSUPPORTED,
                       "partitioned GPU queries support timeBatch, lengthBatch, externalTimeBatch, and time with no group-by or "
                       "grouped by the partition key (lengthBatch(L, true) likewise)");
    if (d->partition_col >= 0) {
        const int pt = d->partition_col < d->n_cols ? d->col_types[d->partition_col] : -1;
        const bool fp_key = pt == SH_T_FLOAT || pt == SH_T_DOUBLE;
        if (!(pt == SH_T_INT || pt == SH_T_LONG || pt == SH_T_STRID || fp_key))
            return sh_fail(SH_ERR_UNSUPPORTED, "partition key must be an int/long/float/double/string column");
        // float / double keys: partitions are String.valueOf(value) (bits, NaN canonical); the Scheduler's
        // tie order among partitions due together hashes that text (Double / Float.toString, sh_jmap.h)
    }

    sh_query* q = new sh_query();
    q->ctx = ctx;
    q->d = *d;
    q->d.filter = nullptr;
    int rc;
    const int32_t pkey[1] = {d->partition_col};
    if ((rc = compile_filter(d->n_filter_ops, d->filter, d->n_cols, d->col_types, q->fp)) ||
        (rc = compile_aggs(d->n_aggs, d->aggs, d->n_cols, d->col_types, q->ap, q->vtypes)) ||
        (!kp_override && plane && (rc = compile_keys(1, pkey, d->n_cols, d->col_types, q->kp))) ||
        (!kp_override && !plane && (rc = compile_keys(d->n_group_by, d->group_by, d->n_cols, d->col_types, q->kp)))) {
        delete q;
        return rc;
    }
    if (kp_override) { q->kp = *kp_override; q->internal_keys = true; }
    // lane 3: grouped by other columns, or (opt-in, SH_PL_SORT=1) lengthBatch keyed by the partition —
    // the sorted chunks have no per-partition sequential walk, so a hot partition does not serialise
    q->group_other = (plane_group && !by_partition) || plane_time_group;
    q->plane_tbsc = plane_tbsc;
    if (plane_time_group || plane_tbsc) {
        if ((rc = compile_keys(d->n_group_by, d->group_by, d->n_cols, d->col_types, q->gkp))) {
            delete q;
            return rc;
        }
    }
    q->plane_sorted = plane_group || (plane && !kp_override && d->window == SH_WIN_LENGTH_BATCH && !d->stream_current &&
                                      q->tune.pl_sort);
    if (q->plane_sorted && (rc = compile_keys(d->n_group_by, d->group_by, d->n_cols, d->col_types, q->gkp))) {
        delete q;
        return rc;
    }
    int64_t cap = d->key_capacity > 0 ? d->key_capacity : (d->n_group_by == 0 ? 1 : (1 << 16));
    if (d->partition_col >= 0 && !plane) {
        // R12: only partition p0 is ever aggregated. Its group keys are a sparse subset of the
        // dictionary, so they go to the hash table; grouped by the partition key alone it is one key.
        q->kp.dense = 0;
        if (d->n_group_by == 1 && d->group_by[0] == d->partition_col) cap = 1;
    }
    if ((rc = q->kp.dense ? q->kt.init_dense(cap, 1, 0) : q->kt.init(cap))) { delete q; return rc; }
    if ((q->plane_sorted || plane_time_group || plane_tbsc) &&
        (rc = q->gkp.dense ? q->gkt.init_dense(cap, 1, 0) : q->gkt.init(q->gkp.n ? cap : 1))) {
        delete q;
        return rc;
    }
    // (partition, group) pairs: room for four per group key, at least 64k
    if ((plane_time_group || plane_tbsc) && (rc = q->pgkt.init(std::max<int64_t>(4 * cap, 1 << 16)))) { delete q; return rc; }
    q->pg_min_size = q->pgkt.size_;
    q->fp_orig = q->fp;
    for (int c = 0; c < d->n_cols; c++) q->load_type[c] = d->col_types[c];
    {
        uint32_t m = 0;
        auto use = [&](int c) { if (c >= 0 && c < d->n_cols) m |= 1u << c; };
        for (int i = 0; i < d->n_filter_ops; i++) if (d->filter[i].op == SH_OP_COL) use(d->filter[i].col);
        for (int i = 0; i < d->n_group_by; i++) use(d->group_by[i]);
        for (int i = 0; i < d->n_aggs; i++) if (d->aggs[i].fn != SH_AGG_COUNT) use(d->aggs[i].col);
        use(d->partition_col);
        if (kp_override)  // (an aggregation root keys on the time bucket and its group-by column)
            for (int i = 0; i < q->kp.n; i++) use(q->kp.col[i]);
        if (d->window == SH_WIN_EXT_TIME_BATCH || d->window == SH_WIN_EXT_TIME) use(d->ts_col);
        if (d->window == SH_WIN_EXT_TIME_BATCH && d->has_start_time == 2) use(d->start_col);
        q->cols_used = m;
    }
    q->partitioned = d->partition_col >= 0 && !plane;
    q->xmode = d->expired_on != 0 && !d->stream_current;
    if (d->window == SH_WIN_TIME || d->window == SH_WIN_EXT_TIME || plane) {
        q->kind = 1;
        if ((rc = sliding_create(q))) { delete q; return rc; }
        *out = q;
        return SH_OK;
    }
    q->kt_min_size = q->kt.size_;
    if ((rc = size_partitions(q))) { delete q; return rc; }
    if (hipHostMalloc((void**)&q->h_info, sizeof(PushInfo), hipHostMallocDefault) != hipSuccess) {
        delete q;
        return sh_fail(SH_ERR_OOM, "pinned alloc failed");
    }
    if ((rc = q->info.reserve(sizeof(PushInfo), false)) || (rc = q->counters.reserve(64, false))) { delete q; return rc; }
    (void)hipEventCreate(&q->ev_push0); (void)hipEventCreate(&q->ev_push1);
    (void)hipEventCreate(&q->ev_agg0); (void)hipEventCreate(&q->ev_agg1);
    (void)hipEventCreateWithFlags(&q->ev_mid, hipEventDisableTiming);
    *out = q;
    return SH_OK;
}

// Aggregate the closed segments [segs[i].lo, segs[i].hi) of the combined (pending + new) sequence
// and append one flush per non-empty segment. Device output: everything is queued on the stream and
// the flush bookkeeping (rows per segment) completes in closed_finish after the push's final
// synchronisation. Host output synchronises here for the row copies.
// Where the push's key slots come from (PosSrc): dictionary ids that are their own slots, with no
// filter and no consumer of the slot column but the multisplit path, are read from the key column.
static bool direct_pos_ok(const sh_query* q) {
    const int kc = q->kp.n == 1 ? q->kp.col[0] : -1;
    return q->kt.dense && q->kt.dmul == 1 && q->kt.dadd == 0 && kc >= 0 && q->kp.div[0] == 0 &&
           (q->load_type[kc] == SH_T_STRID || q->load_type[kc] == SH_T_INT) && filter_kind(q->fp) == 0 &&
           !q->xmode && !q->d.stream_current && q->ap.n > 0 && q->P > 1 && !q->partitioned && !q->given;
}

static bool want_direct_pos(const sh_query* q) {
    // opt-in (SH_DIRECT_POS=1) for the two-pass split: measured slower on MI355X — k_ms_scatter 290 vs
    // 236 us per C2 push reading the key column instead of the slot column k_boundaries writes
    // (profiles/r03_c2_v3*)
    return q->tune.direct_pos && direct_pos_ok(q);
}

static PosSrc pos_src(const sh_query* q, const sh_batch* b) {
    PosSrc ps{};
    if (!b) return ps;
    if (q->direct_pos) {
        ps.key = (const int*)b->cols[q->kp.col[0]];
        ps.mask = q->kt.dev().mask;
    } else {
        ps.np = q->new_pos.as<u32>();
    }
    return ps;
}

static int closed_finish(sh_query* q, bool host_out);

static int run_closed(sh_query* q, const std::vector<Segment>& segs, const std::vector<int64_t>& clocks,
                      const std::vector<int64_t>& windows, const sh_batch* b, bool host_out) {
    hipStream_t s = q->ctx->stream;
    int nseg = (int)segs.size();
    int64_t closed_hi = segs.back().hi;
    ColSet cs{};
    cs.n = q->d.n_cols;
    for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->load_type[c]; cs.ptr[c] = b ? b->cols[c] : nullptr; }
    const int64_t* ts = b ? b->ts : nullptr;
    if (q->ap.n == 0) {
        // pass-through (`select *` without aggregators or group-by): every passing event of the
        // closed batches is a row, in stream order (QuerySelector.processNoGroupBy :161-205)
        RCHK(q->pass_pos.reserve((size_t)(closed_hi + 1) * 4, false));
        RCHK(q->x_tmp.reserve((size_t)((closed_hi + 1 + kTile - 1) / kTile + 16) * 8, false));
        RCHK(q->counters.reserve(64 + (size_t)nseg * 4, false));
        RCHK(q->h_up.reserve((size_t)nseg * sizeof(Segment)));
        RCHK(q->segs.reserve(nseg * sizeof(Segment), false));
        std::memcpy(q->h_up.p, segs.data(), (size_t)nseg * sizeof(Segment));
        HIPCHK(hipMemcpyAsync(q->segs.p, q->h_up.p, nseg * sizeof(Segment), hipMemcpyHostToDevice, s));
        const int64_t cap = std::max<int64_t>(closed_hi, 1);
        RCHK(q->out_ts.reserve(cap * 8, false));
        RCHK(q->out_rep.reserve(cap * 8, false));
        RCHK(q->out_keys.reserve(8, false));
        RCHK(q->out_vals.reserve(8, false));
        RCHK(q->out_nulls.reserve(8, false));
        RCHK(q->out_expired.reserve(cap, false));
        HIPCHK(hipMemsetAsync(q->out_expired.p, 0, cap, s));
        q->zeroed_expired = nullptr;
        uint32_t* unit_rows = (uint32_t*)(q->counters.as<char>() + 64);
        HIPCHK(hipEventRecord(q->ev_agg0, s));
        launch_pass_rows(s, closed_hi, q->n_pend, b ? q->new_pos.as<u32>() : nullptr, q->pass_pos.as<u32>(),
                         q->x_tmp.as<int64_t>(), q->pend_ts.as<int64_t>(), q->pend_gidx.as<u64>(), ts, q->seq,
                         q->segs.as<Segment>(), nseg, q->out_ts.as<int64_t>(), q->out_rep.as<int64_t>(), unit_rows,
                         q->counters.as<u32>());
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(q->ev_agg1, s));
        RCHK(q->h_tail.reserve(16 + (size_t)nseg * 4));
        HIPCHK(hipMemcpyAsync(q->h_tail.as<char>() + 16, unit_rows, nseg * 4, hipMemcpyDeviceToHost, s));
        auto& t = q->tail;
        t.active = true;
        t.host_done = false;
        t.nseg = nseg;
        t.units_per_seg = 1;
        t.closed_hi = closed_hi;
        t.clocks = clocks;
        t.windows = windows;
        if (host_out) {
            HIPCHK(hipStreamSynchronize(s));
            RCHK(closed_finish(q, true));
        }
        return SH_OK;
    }
    // row capacity: per segment at most min(len, distinct keys)
    int64_t row_cap = 0;
    for (auto& sg : segs) row_cap += std::min<int64_t>(sg.hi - sg.lo, (int64_t)q->kt.size_ + 1);
    row_cap = std::max<int64_t>(row_cap, 1);
    const int na = q->ap.n, nk = q->kp.n, RW = row_words(na);
    const int64_t n_words = (closed_hi >> 5) + 1;  // first-occurrence bitmap over the combined index space
    // One flat workgroup per segment walks every event of the segment, passing or not, and
    // serialises a key's events in conflict rounds: fine for short batches of few keys. Key
    // partitions, long windows and sparse partitions (R12 keeps one partition) take the compacting
    // multisplit (usually launched already by push_core) and the thread-ownership kernel.
    const bool own = q->P > 1 || q->partitioned || closed_hi / nseg >= 65536;
    const int64_t n_units = own ? (int64_t)nseg * q->P : nseg;
    const int unit_stride = agg_unit_rows(q->P, q->NL, own);
    RCHK(q->rows.reserve((size_t)n_units * unit_stride * RW * 8, false));
    RCHK(q->first_bits.reserve((size_t)n_words * 4, false));
    RCHK(q->counters.reserve(64 + (size_t)n_units * 4, false));
    uint32_t* unit_rows = (uint32_t*)(q->counters.as<char>() + 64);  // written by every unit's workgroup
    HIPCHK(hipMemsetAsync(q->first_bits.p, 0, (size_t)n_words * 4, s));
    // the segment list goes up from pinned memory (an async copy from pageable memory may read it
    // after this function returned)
    RCHK(q->h_up.reserve((size_t)nseg * sizeof(Segment)));
    RCHK(q->segs.reserve(nseg * sizeof(Segment), false));
    std::memcpy(q->h_up.p, segs.data(), (size_t)nseg * sizeof(Segment));
    HIPCHK(hipMemcpyAsync(q->segs.p, q->h_up.p, nseg * sizeof(Segment), hipMemcpyHostToDevice, s));
    const Segment* dsegs = q->segs.as<Segment>();
    // One flat workgroup per segment walks every event of the segment, passing or not, and
    // serialises a key's events in conflict rounds: fine for short batches of few keys. Key
    // partitions, long windows and sparse partitions (R12 keeps one partition) take the compacting
    // multisplit (usually launched already by push_core) and the thread-ownership kernel.
    SH_TRACE("run_closed nseg=%d closed_hi=%lld row_cap=%lld own=%d P=%d NL=%d ms_ready=%d", nseg, (long long)closed_hi,
             (long long)row_cap, (int)own, q->P, q->NL, (int)q->ms_ready);
    if (own) {
        // a packed split (kPackIdxBits of event index per record) serves segments up to 2^22 events
        bool long_seg = false;
        for (auto& sg : segs) long_seg |= sg.hi - sg.lo > (int64_t)kPackIdxMask + 1;
        if (q->ms_ready && q->rec_packed && long_seg) q->ms_ready = false;
        if (!q->ms_ready) RCHK(run_multisplit(q, closed_hi, b, false, long_seg));
        RCHK(q->seg_off.reserve((size_t)(nseg + 1) * q->P * 8, false));
        launch_seg_offsets(s, dsegs, nseg, q->n_pend, q->pend_pos.as<u32>(), pos_src(q, b), q->P,
                           q->ms_counts.as<u32>(), q->ms_map, q->seg_off.as<int64_t>());
    }
    // (the record buffers' addresses only after run_multisplit: it may have grown them)
    const u32* rec_pos = q->rec_pos.as<u32>();
    const u32* rec_idx = q->rec_idx.as<u32>();
    const u64* rec_vals = q->rec_vals.as<u64>();
    // multisplit units leave every row at its key's slot and one pass emits them (k_emit_gather; the
    // round-4 rank scatter + column split remain for the other units)
    const bool gather = own;
    HIPCHK(hipEventRecord(q->ev_agg0, s));
    launch_aggregate(s, dsegs, nseg, q->P, q->logP, q->NL, q->n_pend, q->pend_pos.as<u32>(), q->pend_vals.as<u64>(),
                     q->pend_cap, b ? q->new_pos.as<u32>() : nullptr, cs, q->ap, q->rows.as<u64>(), RW,
                     unit_rows, q->first_bits.as<u32>(),
                     rec_pos, own ? rec_idx : nullptr, rec_vals, (int64_t)q->rec_cap, q->seg_off.as<int64_t>(),
                     q->rec_packed,
                     EvSrc{q->n_pend, q->pend_ts.as<int64_t>(), ts, q->pend_gidx.as<u64>(),
                           q->given && b ? q->given_gidx : nullptr, q->seq},
                     gather);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(q->ev_agg1, s));
    // output columns sized for the row capacity; the emit kernels read the row count on the device
    const int64_t cap = row_cap;
    RCHK(q->out_ts.reserve(cap * 8, false));
    RCHK(q->out_keys.reserve(std::max(1, nk) * cap * 8, false));
    RCHK(q->out_vals.reserve(na * cap * 8, false));
    RCHK(q->out_nulls.reserve(na * cap, false));
    RCHK(q->out_expired.reserve(cap, false));
    RCHK(q->out_rep.reserve(cap * 8, false));
    if (q->given) RCHK(q->out_order.reserve(cap * 8, false));
    const int nbt = (int)((n_words + kTile - 1) / kTile);
    RCHK(q->blk_cnt.reserve((nbt + 16) * 8, false));
    RCHK(q->word_pre.reserve((size_t)n_words * 8, false));
    if (!gather) RCHK(q->emit_stage.reserve(emit_stage_bytes(nk, na, q->given ? 1 : 0, cap), false));
    launch_bits_prefix(s, q->first_bits.as<u32>(), n_words, q->blk_cnt.as<int64_t>(), q->word_pre.as<u64>(),
                       q->counters.as<u32>());
    if (gather)
        launch_emit_gather(s, q->word_pre.as<u64>(), n_words, dsegs, nseg, q->P, q->logP, unit_stride, q->rows.as<u64>(),
                           RW, pos_src(q, b), q->pend_pos.as<u32>(), q->n_pend, q->counters.as<u32>(), na, q->kt.dev(),
                           q->kp, q->out_ts.as<int64_t>(), q->out_keys.as<int64_t>(), q->out_vals.as<u64>(),
                           q->pend_gidx.as<u64>(), q->given && b ? q->given_gidx : nullptr,
                           q->given ? q->out_order.as<int64_t>() : nullptr, q->seq, q->out_rep.as<int64_t>());
    else
    launch_emit_rows(s, q->rows.as<u64>(), RW, unit_rows, n_units, unit_stride, cap, q->counters.as<u32>(),
                     q->word_pre.as<u64>(), na, q->kt.dev(), q->kp, q->n_pend,
                     q->pend_ts.as<int64_t>(), ts, cap,
                     q->out_ts.as<int64_t>(), q->out_keys.as<int64_t>(), q->out_vals.as<u64>(), q->pend_gidx.as<u64>(),
                     q->given && b ? q->given_gidx : nullptr, q->given ? q->out_order.as<int64_t>() : nullptr, q->seq,
                     q->out_rep.as<int64_t>(), q->emit_stage.as<u64>());
    // batch-window rows always have a value (count >= 1) and are CURRENT events: the null and
    // expired flags are zeroed once per buffer, nothing here ever sets them
    if (q->out_nulls.p != q->zeroed_nulls) {
        HIPCHK(hipMemsetAsync(q->out_nulls.p, 0, q->out_nulls.cap, s));
        q->zeroed_nulls = q->out_nulls.p;
    }
    if (q->out_expired.p != q->zeroed_expired) {
        HIPCHK(hipMemsetAsync(q->out_expired.p, 0, q->out_expired.cap, s));
        q->zeroed_expired = q->out_expired.p;
    }
    HIPCHK(hipGetLastError());
    // rows per unit land in pinned memory with the push's final copies
    RCHK(q->h_tail.reserve(16 + (size_t)n_units * 4));
    HIPCHK(hipMemcpyAsync(q->h_tail.as<char>() + 16, unit_rows, n_units * 4, hipMemcpyDeviceToHost, s));
    auto& t = q->tail;
    t.active = true;
    t.host_done = false;
    t.nseg = nseg;
    t.units_per_seg = own ? q->P : 1;
    t.closed_hi = closed_hi;
    t.clocks = clocks;
    t.windows = windows;
    SH_TRACE("run_closed queued");
    if (host_out) {
        HIPCHK(hipStreamSynchronize(s));
        RCHK(closed_finish(q, true));
    }
    return SH_OK;
}

// After the stream synchronised: rows per segment -> flush offsets / clocks; host output copies.
static int closed_finish(sh_query* q, bool host_out) {
    auto& t = q->tail;
    if (!t.active || t.host_done) return SH_OK;
    t.host_done = true;
    hipStream_t s = q->ctx->stream;
    const uint32_t* unit_rows = (const uint32_t*)(q->h_tail.as<char>() + 16);
    std::vector<int64_t> seg_rows(t.nseg, 0);
    for (int i = 0; i < t.nseg; i++)
        for (int u = 0; u < t.units_per_seg; u++) seg_rows[i] += unit_rows[(size_t)i * t.units_per_seg + u];
    const int na = q->ap.n, nk = q->kp.n;
    int64_t n_rows = 0;
    for (int i = 0; i < t.nseg; i++) n_rows += seg_rows[i];
    float agg_ms = 0;
    (void)hipEventElapsedTime(&agg_ms, q->ev_agg0, q->ev_agg1);
    q->stats.main_kernel_ms += agg_ms;
    // algorithmic bytes of the aggregation kernel: every closed event's referenced columns + rows out
    q->agg_bytes += t.closed_hi * (int64_t)(4 + 8 * q->ap.n_vcols) + n_rows * (int64_t)(8 * row_words(na));
    if (host_out && n_rows > 0) {
        size_t base = q->out.ts.size();
        size_t nb = base + n_rows;
        q->out.ts.resize(nb);
        q->out.expired.resize(nb, 0);
        q->out.rep.resize(nb);
        HIPCHK(hipMemcpyAsync(q->out.ts.data() + base, q->out_ts.p, n_rows * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(q->out.rep.data() + base, q->out_rep.p, n_rows * 8, hipMemcpyDeviceToHost, s));
        // keys / vals / nulls are [k][n_rows] blocks straight into the pinned output vectors (a push
        // closes windows through run_closed at most once, so they start empty)
        if (base != 0 && (q->xt_timeout == 0 || q->given))
            return sh_fail(SH_ERR_INVALID, "host output appended twice in one push");
        if (base != 0) {
            // (an externalTimeBatch timeout's later run: its [k][n_rows] blocks join the earlier rows)
            PinnedVec<int64_t> nkeys((size_t)nk * n_rows);
            PinnedVec<uint64_t> nvals((size_t)na * n_rows);
            if (nk) HIPCHK(hipMemcpyAsync(nkeys.data(), q->out_keys.p, nk * n_rows * 8, hipMemcpyDeviceToHost, s));
            if (na) HIPCHK(hipMemcpyAsync(nvals.data(), q->out_vals.p, na * n_rows * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            auto join = [&](auto& v, const auto& add, int nc) {
                std::remove_reference_t<decltype(v)> old(v);
                v.resize((size_t)nc * nb);
                for (int k = 0; k < nc; k++) {
                    std::copy(old.begin() + (size_t)k * base, old.begin() + (size_t)(k + 1) * base, v.begin() + (size_t)k * nb);
                    std::copy(add.begin() + (size_t)k * n_rows, add.begin() + (size_t)(k + 1) * n_rows,
                              v.begin() + (size_t)k * nb + base);
                }
            };
            join(q->out.keys, nkeys, nk);
            join(q->out.vals, nvals, na);
            q->out.nulls.assign((size_t)na * nb, 0);
        } else {
            q->out.keys.resize((size_t)nk * n_rows);
            q->out.vals.resize((size_t)na * n_rows);
            if (nk) HIPCHK(hipMemcpyAsync(q->out.keys.data(), q->out_keys.p, nk * n_rows * 8, hipMemcpyDeviceToHost, s));
            if (q->given) {
                size_t ob = q->order_host.size();
                q->order_host.resize(ob + n_rows);
                HIPCHK(hipMemcpyAsync(q->order_host.data() + ob, q->out_order.p, n_rows * 8, hipMemcpyDeviceToHost, s));
            }
            if (na) HIPCHK(hipMemcpyAsync(q->out.vals.data(), q->out_vals.p, na * n_rows * 8, hipMemcpyDeviceToHost, s));
            q->out.nulls.assign((size_t)na * n_rows, 0);
            HIPCHK(hipStreamSynchronize(s));
        }
    }
    // flush bookkeeping (one flush per non-empty closed segment)
    PinnedVec<int64_t>& fo = host_out ? q->out.flush_offsets : q->dev_flush_offsets;
    PinnedVec<int64_t>& fc = host_out ? q->out.flush_clock : q->dev_flush_clock;
    int64_t acc = fo.back();
    for (int i = 0; i < t.nseg; i++) {
        if (seg_rows[i] == 0) continue;
        acc += seg_rows[i];
        fo.push_back(acc);
        fc.push_back(t.clocks[i]);
        q->flush_window.push_back(t.windows[i]);
    }
    if (!host_out) q->dev_out.n_rows = n_rows;
    return SH_OK;
}

// sh_query_set_device_flushes: a batch window's flush layout (built on the host: a few entries per
// push) goes up to the device, so sh_push_device's whole output is in device memory
int flush_layout_to_device(sh_query* q, sh_out& o) {
    if (!q->device_flushes || q->rate.kind != SH_RATE_NONE || q->wide || !o.flush_offsets) return SH_OK;
    const size_t nf = (size_t)o.n_flushes;
    hipStream_t s = q->ctx->stream;
    RCHK(q->fl_dev.reserve((2 * nf + 1) * 8, false));
    HIPCHK(hipMemcpyAsync(q->fl_dev.p, o.flush_offsets, (nf + 1) * 8, hipMemcpyHostToDevice, s));
    if (nf) HIPCHK(hipMemcpyAsync(q->fl_dev.as<int64_t>() + nf + 1, o.flush_clock, nf * 8, hipMemcpyHostToDevice, s));
    HIPCHK(hipStreamSynchronize(s));
    o.flush_offsets = q->fl_dev.as<int64_t>();
    o.flush_clock = q->fl_dev.as<int64_t>() + nf + 1;
    return SH_OK;
}

static void finish_out(sh_query* q, bool host_out, const sh_out** out) {
    const bool compact = q->compact_now;
    q->compact_now = false;
    if (host_out) {
        q->out.view(q->kp.n, q->ap.n, q->vtypes);
        if (compact) {
            q->out.out.n_flushes = q->out.out.n_rows;
            q->out.out.flush_offsets = nullptr;
            q->out.out.flush_clock = nullptr;
        }
        *out = &q->out.out;
    } else {
        sh_out& o = q->dev_out;
        o.n_flushes = compact ? o.n_rows : (int64_t)q->dev_flush_clock.size();
        o.n_keys = q->kp.n;
        o.n_vals = q->ap.n;
        for (int i = 0; i < q->ap.n; i++) o.val_types[i] = q->vtypes[i];
        o.flush_offsets = compact ? nullptr : q->dev_flush_offsets.data();
        o.flush_clock = compact ? nullptr : q->dev_flush_clock.data();
        if (!compact) (void)flush_layout_to_device(q, o);
        o.ts = q->out_ts.as<int64_t>();
        o.expired = q->out_expired.as<uint8_t>();
        o.keys = q->out_keys.as<int64_t>();
        o.vals = q->out_vals.as<uint64_t>();
        o.nulls = q->out_nulls.as<uint8_t>();
        o.rep = q->out_rep.as<int64_t>();
        *out = &o;
    }
}

// Partitioned timeBatch (`partition with (pcol of S)`): TimeBatchWindowProcessor.nextEmitTime is a
// processor field shared by every partition (:128) and only the partition that first initialised it
// registered a scheduler timer (:266-276, Scheduler.notifyAt under that partition flow); timers re-arm
// under the same flow, so only that partition (p0) is ever flushed (the reference test
// WindowPartitionTestCase:291-348 tolerates exactly this). The GPU runs the query restricted to p0.
static int resolve_first_partition(sh_query* q, const sh_batch* b) {
    hipStream_t s = q->ctx->stream;
    int64_t N = b->n;
    ColSet cs{};
    cs.n = q->d.n_cols;
    for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->d.col_types[c]; cs.ptr[c] = b->cols[c]; }
    int nblk = (int)((N + kTile - 1) / kTile);
    RCHK(q->blk_pass.reserve(nblk * 8, false));
    RCHK(q->blk_tl.reserve(nblk * 8, false));
    RCHK(q->blk_first.reserve(scan_blocks_first_bytes(nblk), false));
    WinParams wp{};
    wp.kind = SH_WIN_LENGTH_BATCH;  // no nextEmitTime initialisation in this probe
    wp.N = N;
    wp.send_size = b->send_size;
    wp.pcol1 = q->d.partition_col + 1;
    launch_blockagg(s, b->ts, cs, q->fp_orig, N, b->send_size, q->blk_pass.as<int64_t>(), q->blk_tl.as<int64_t>(),
                    q->blk_first.as<int64_t>(), nblk);
    launch_scan_blocks(s, q->blk_pass.as<int64_t>(), q->blk_tl.as<int64_t>(), q->blk_first.as<int64_t>(), nblk, b->ts,
                       wp, q->info.as<PushInfo>(), nullptr, cs);
    HIPCHK(hipMemcpyAsync(q->h_info, q->info.p, sizeof(PushInfo), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    int64_t first = q->h_info->first_pass;
    if (first == INT64_MAX) {
        // nothing reached the window; the playback clock still advances (InputHandler.send)
        q->clock = q->clock_valid ? std::max(q->clock, q->h_info->max_tl) : q->h_info->max_tl;
        q->clock_valid = true;
        return SH_OK;
    }
    // the partition key of that event, read by k_scan_blocks (no extra round trip)
    const int64_t key = q->h_info->first_key;
    return query_set_partition(q, key);
}

// Restrict the query to partition key p0 (the partition that armed the shared timer, R12).
int partition_filter(const FilterProg& base, int pcol, int ptype, int64_t key, FilterProg* out) {
    FilterProg fp = base;
    if (fp.n + 4 > kMaxFilterOps) return sh_fail(SH_ERR_UNSUPPORTED, "filter too long for a partitioned query");
    fp.ops[fp.n++] = FilterOpD{SH_OP_COL, 0, pcol, 0, 0, 0.0};
    if (ptype == SH_T_FLOAT || ptype == SH_T_DOUBLE) {
        // String.valueOf equality (ValuePartitionExecutor :34-40): bits, every NaN one key, 0.0 != -0.0
        double dv;
        std::memcpy(&dv, &key, 8);
        fp.ops[fp.n++] = FilterOpD{SH_OP_CONST, SH_T_DOUBLE, 0, 0, 0, dv};
        fp.ops[fp.n++] = FilterOpD{kOpKeyEq, 0, 0, 0, 0, 0.0};
    } else {
        fp.ops[fp.n++] = FilterOpD{SH_OP_CONST, ptype, 0, 0, key, 0.0};
        fp.ops[fp.n++] = FilterOpD{SH_OP_EQ, 0, 0, 0, 0, 0.0};
    }
    if (base.n > 0) fp.ops[fp.n++] = FilterOpD{SH_OP_AND, 0, 0, 0, 0, 0.0};
    *out = fp;
    return SH_OK;
}

int query_set_partition(sh_query* q, int64_t key) {
    int pc = q->d.partition_col;
    q->p0 = key;
    q->p0_known = true;
    return partition_filter(q->fp_orig, pc, q->d.col_types[pc], key, &q->fp);
}

// sh_query_restore: a key table of the snapshot's size and room for its queued events.
int query_resize_for_restore(sh_query* q, size_t table_size, int64_t n_pend, const KeyBand* band) {
    if (band) {
        q->kt.release();
        RCHK(q->kt.init_band(band->lk, band->rows, band->base, q->band_mul, q->band_add));
        if (table_size != q->kt.size_) return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
    } else if (q->kt.dense && !q->kt.lk) {
        if (table_size != q->kt.size_) return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
    } else if (table_size != q->kt.size_ || q->kt.lk) {
        q->kt.release();
        RCHK(q->kt.init_size(table_size));
    }
    RCHK(size_partitions(q));
    q->n_pend = 0;
    return grow_pending(q, n_pend, 0);
}

// stream.current.event batch windows (LengthBatchWindowProcessor.processStreamCurrentEvents :245-274,
// TimeBatchWindowProcessor RESET mode :262-340): the pending entries [0, n_old) are the open window's
// earlier events, [n_old, M) this push's passing events (sh_kernels.hip k_sc_*). One flush per chunk:
// every passing event for lengthBatch (:160-182 sends each event's chunk on its own), every send with
// passing events for timeBatch; the flush clock is the send's playback clock.
static int sc_rows(sh_query* q, const sh_batch* b, const std::vector<Bound>& bounds, int64_t n_old, int64_t M,
                   bool cv0, int64_t clock0, int64_t seq0, bool host_out) {
    hipStream_t s = q->ctx->stream;
    const int nk = q->kp.n, na = q->ap.n;
    const int nb = (int)bounds.size();
    const bool per_event = q->d.window == SH_WIN_LENGTH_BATCH;
    const int64_t N = b->n, ss = b->send_size;
    const int64_t n_sends = ss > 0 ? (N + ss - 1) / ss : 1;
    RCHK(q->sc_hp.reserve((size_t)std::max(nb, 1) * 8 + 64));
    for (int i = 0; i < nb; i++) q->sc_hp.as<int64_t>()[i] = bounds[i].pcb;
    RCHK(q->sc_pcb.reserve((size_t)std::max(nb, 1) * 8, false));
    if (nb) HIPCHK(hipMemcpyAsync(q->sc_pcb.p, q->sc_hp.p, (size_t)nb * 8, hipMemcpyHostToDevice, s));
    RCHK(q->sc_skey.reserve((size_t)M * 8, false));
    RCHK(q->sc_skey2.reserve((size_t)M * 8, false));
    RCHK(q->sc_idx.reserve((size_t)M * 4, false));
    RCHK(q->sc_idx2.reserve((size_t)M * 4, false));
    RCHK(q->sc_chunk.reserve((size_t)M * 8, false));
    RCHK(q->sc_send.reserve((size_t)M * 8, false));
    RCHK(q->sc_hd.reserve((size_t)(M + 1) * 4, false));
    RCHK(q->sc_pos.reserve((size_t)(M + 1) * 4, false));
    RCHK(q->sc_starts.reserve((size_t)(M + 1) * 4, false));
    RCHK(q->sc_ghead.reserve((size_t)(M + 1) * 4, false));
    RCHK(q->sc_pre.reserve((size_t)(M + 1) * 4, false));
    RCHK(q->sc_slast.reserve((size_t)M * 4, false));
    RCHK(q->sc_sval.reserve((size_t)std::max(na, 1) * M * 8, false));
    RCHK(q->sc_tmp.reserve((size_t)((M + 1 + kTile - 1) / kTile + 16) * 8, false));
    RCHK(q->sc_sl.reserve((size_t)n_sends * 8, false));
    // (a sharded owner: records are one send each for their clocks, chunks are the global sends)
    const bool gv = q->given_clk != nullptr;
    const bool xs = q->d.expired_on && per_event;   // lengthBatch(L, true) with expired / all events
    const bool xt = q->d.expired_on && !per_event;  // timeBatch(T, true) with expired / all events
    // every new entry its own chunk (per-event sends, lengthBatch(L, true)): each is its own row, no head
    // flags, no scan of them, no chunk column and no read-back of the row count (current rows only)
    const bool all_heads = !(xs || xt) && (per_event || (gv ? q->given_ss : ss) == 1);
    launch_sc_keys(s, M, n_old, q->sc_pcb.as<int64_t>(), nb, q->pend_pos.as<u32>(), q->pend_gidx.as<u64>(),
                   per_event ? 1 : 0, gv ? q->given_ss : ss, gv ? q->given_seq0 : seq0, q->sc_skey.as<u64>(),
                   q->sc_idx.as<u32>(), all_heads ? nullptr : q->sc_chunk.as<int64_t>(), q->sc_send.as<int64_t>(),
                   gv ? 1 : 0);
    // current rows only: the sorted keys are compared for equality alone, so the window index goes right
    // above the slot bits and the radix sort reads those bits only (C2: 24 of 64)
    unsigned end_bit = 64;
    if (!(xs || xt)) {
        unsigned kb = 1, wb = 1;
        while (kb < 32 && ((uint64_t)1 << kb) < (uint64_t)q->kt.size_) kb++;
        while (wb < 31 && ((int64_t)1 << wb) <= (int64_t)nb) wb++;
        if (kb + wb <= 48) {
            launch_sc_pack_keys(s, M, kb, q->sc_skey.as<u64>());
            end_bit = kb + wb;
        }
    }
    size_t tb = 0;
    if (sort_u64_pairs_bits(nullptr, &tb, nullptr, nullptr, nullptr, nullptr, M, end_bit, s))
        return sh_fail(SH_ERR_DEVICE, "stream.current: sort sizing");
    RCHK(q->sc_sort.reserve(std::max<size_t>(tb, 16), false));
    if (sort_u64_pairs_bits(q->sc_sort.p, &tb, q->sc_skey.as<u64>(), q->sc_skey2.as<u64>(), q->sc_idx.as<u32>(),
                            q->sc_idx2.as<u32>(), M, end_bit, s))
        return sh_fail(SH_ERR_DEVICE, "stream.current: sort failed");
    launch_rate_segments(s, M, q->sc_skey2.as<u64>(), q->sc_idx2.as<u32>(), 1, 0, q->sc_hd.as<u32>(),
                         q->sc_pos.as<u32>(), q->sc_starts.as<u32>(), q->sc_tmp.as<int64_t>());
    if (!all_heads) HIPCHK(hipMemsetAsync(q->sc_ghead.p, 0, (size_t)(M + 1) * 4, s));
    HIPCHK(hipEventRecord(q->ev_agg0, s));
    launch_sc_walk(s, M, q->sc_hd.as<u32>(), q->sc_pos.as<u32>(), q->sc_starts.as<u32>(), q->sc_idx2.as<u32>(),
                   q->sc_chunk.as<int64_t>(), q->pend_vals.as<u64>(), q->pend_cap, q->ap, n_old,
                   all_heads ? nullptr : q->sc_ghead.as<u32>(),
                   q->sc_sval.as<u64>(), q->sc_slast.as<u32>());
    HIPCHK(hipEventRecord(q->ev_agg1, s));
    const int64_t nn = M - n_old;
    // the sends' playback clocks: TimestampGeneratorImpl only moves forward (prefix max of send-last ts);
    // a sharded owner's records (one send each) carry their global send's clock instead
    if (q->given_clk) {
        if (ss != 1) return sh_fail(SH_ERR_INVALID, "sharded stream.current: records are one send each");
        cv0 = false;  // (the records' clocks are whole; the owner's clock is already the push's end clock)
        HIPCHK(hipMemcpyAsync(q->sc_sl.p, q->given_clk, (size_t)N * 8, hipMemcpyDeviceToDevice, s));
    } else {
        launch_sc_send_last(s, b->ts, N, ss, n_sends, q->sc_sl.as<int64_t>());
    }
    HIPCHK(hipGetLastError());
    // (host scratch kept by the query: a fresh 8-byte-per-send vector per push faulted in its pages —
    // hundreds of MB per C2-sized push)
    std::vector<int64_t>& sl = q->sc_sl_host;
    if (xs || xt) {
        RCHK(q->sc_h.reserve((size_t)n_sends * 8 + 64));
        HIPCHK(hipMemcpyAsync(q->sc_h.p, q->sc_sl.p, (size_t)n_sends * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        sl.resize((size_t)n_sends);
        const int64_t* hs = q->sc_h.as<int64_t>();
        bool cv = cv0;
        int64_t c = clock0;
        for (int64_t i = 0; i < n_sends; i++) {
            c = cv ? std::max(c, hs[i]) : hs[i];
            cv = true;
            sl[i] = c;
        }
    } else {
        // current rows only: the sends' clocks stay on the device (the flushes are built there too)
        size_t stb = 0;
        RCHK(q->sc_slp.reserve((size_t)n_sends * 8, false));
        if (scan_max_i64(nullptr, &stb, q->sc_sl.as<int64_t>(), q->sc_slp.as<int64_t>(), n_sends, s))
            return sh_fail(SH_ERR_DEVICE, "stream.current: scan sizing");
        RCHK(q->sc_sort.reserve(std::max<size_t>(stb, 16), false));
        if (scan_max_i64(q->sc_sort.p, &stb, q->sc_sl.as<int64_t>(), q->sc_slp.as<int64_t>(), n_sends, s))
            return sh_fail(SH_ERR_DEVICE, "stream.current: scan failed");
    }
    const int cur_on = q->d.current_on ? 1 : 0;
    int64_t T = 0;
    if (xs || xt) {
        RCHK(q->scx_fe.reserve((size_t)(M + 1) * 4, false));
        RCHK(q->scx_fpre.reserve((size_t)(M + 1) * 4, false));
        RCHK(q->scx_last.reserve((size_t)M * 4, false));
        RCHK(q->scx_rows.reserve((size_t)(nn + 2) * 4, false));
        RCHK(q->scx_rank.reserve((size_t)std::max<int64_t>(nn, 1) * 8, false));
        RCHK(q->scx_clk.reserve((size_t)n_sends * 8, false));
        HIPCHK(hipMemsetAsync(q->scx_fe.p, 0, (size_t)(M + 1) * 4, s));
        launch_scx_first(s, M, q->sc_hd.as<u32>(), q->sc_pos.as<u32>(), q->sc_starts.as<u32>(), q->sc_idx2.as<u32>(),
                         q->scx_fe.as<u32>(), q->scx_fpre.as<u32>(), q->scx_last.as<u32>());
        HIPCHK(hipMemcpyAsync(q->scx_fpre.p, q->scx_fe.p, (size_t)(M + 1) * 4, hipMemcpyDeviceToDevice, s));
        launch_scan_sum_large_u32(s, q->scx_fpre.as<u32>(), M + 1, q->sc_tmp.as<int64_t>());
        if (xs)
            launch_scx_count(s, M, n_old, q->sc_pcb.as<int64_t>(), q->sc_skey.as<u64>(), q->sc_skey2.as<u64>(),
                             q->sc_idx2.as<u32>(), q->scx_fpre.as<u32>(), cur_on, 1, q->scx_rows.as<u32>(),
                             q->scx_rank.as<int64_t>());
        else
            launch_scxt_count(s, M, n_old, q->sc_pcb.as<int64_t>(), nb, q->sc_skey.as<u64>(), q->scx_fpre.as<u32>(),
                              q->sc_ghead.as<u32>(), cur_on, q->scx_rows.as<u32>());
        const int64_t nr = xs ? nn + 1 : nn + 2;  // (timeBatch: rows[nn] = windows closing after the last entry)
        launch_scan_sum_large_u32(s, q->scx_rows.as<u32>(), nr, q->sc_tmp.as<int64_t>());
        if (xs) {
            std::memcpy(q->sc_h.p, sl.data(), (size_t)n_sends * 8);
            HIPCHK(hipMemcpyAsync(q->scx_clk.p, q->sc_h.p, (size_t)n_sends * 8, hipMemcpyHostToDevice, s));
        } else {  // timeBatch: the clock of each window start (the TIMER chunk's clock)
            RCHK(q->scx_clk.reserve((size_t)std::max(nb, 1) * 8, false));
            RCHK(q->sc_h.reserve((size_t)std::max<int64_t>(nb, n_sends) * 8 + 64));
            for (int i = 0; i < nb; i++) q->sc_h.as<int64_t>()[i] = bounds[i].clock;
            if (nb) HIPCHK(hipMemcpyAsync(q->scx_clk.p, q->sc_h.p, (size_t)nb * 8, hipMemcpyHostToDevice, s));
        }
        HIPCHK(hipGetLastError());
        RCHK(q->h_small_sc.reserve(64));
        HIPCHK(hipMemcpyAsync(q->h_small_sc.p, q->scx_rows.as<uint32_t>() + nr - 1, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        T = *q->h_small_sc.as<uint32_t>();
    } else if (all_heads) {
        T = nn;
    } else {
        HIPCHK(hipMemcpyAsync(q->sc_pre.p, q->sc_ghead.as<uint32_t>() + n_old, (size_t)(nn + 1) * 4,
                              hipMemcpyDeviceToDevice, s));
        launch_scan_sum_large_u32(s, q->sc_pre.as<u32>(), nn + 1, q->sc_tmp.as<int64_t>());
        HIPCHK(hipGetLastError());
        RCHK(q->h_small_sc.reserve(64));
        HIPCHK(hipMemcpyAsync(q->h_small_sc.p, q->sc_pre.as<uint32_t>() + nn, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        T = *q->h_small_sc.as<uint32_t>();
    }
    const int64_t TC = std::max<int64_t>(T, 1);
    RCHK(q->out_ts.reserve(TC * 8, false));
    RCHK(q->out_keys.reserve((size_t)std::max(1, nk) * TC * 8, false));
    RCHK(q->out_vals.reserve((size_t)std::max(1, na) * TC * 8, false));
    RCHK(q->out_nulls.reserve((size_t)std::max(1, na) * TC, false));
    RCHK(q->out_expired.reserve(TC, false));
    RCHK(q->out_rep.reserve(TC * 8, false));
    RCHK(q->sc_ochunk.reserve(TC * 8, false));
    RCHK(q->sc_osend.reserve(TC * 8, false));
    if (q->given) RCHK(q->out_order.reserve(TC * 8, false));
    HIPCHK(hipMemsetAsync(q->out_nulls.p, 0, q->out_nulls.cap, s));
    HIPCHK(hipMemsetAsync(q->out_expired.p, 0, q->out_expired.cap, s));
    q->zeroed_nulls = q->out_nulls.p;
    q->zeroed_expired = q->out_expired.p;
    if (xs) {
        launch_scx_rows(s, M, n_old, q->sc_pcb.as<int64_t>(), nb, q->sc_skey.as<u64>(), q->scx_fe.as<u32>(),
                        q->scx_fpre.as<u32>(), q->scx_last.as<u32>(), q->scx_rows.as<u32>(), q->scx_rank.as<int64_t>(),
                        q->sc_sval.as<u64>(), q->sc_send.as<int64_t>(), q->scx_clk.as<int64_t>(),
                        q->pend_ts.as<int64_t>(), q->pend_gidx.as<u64>(), q->kt.dev(), q->kp, q->ap, cur_on, 1, T,
                        q->out_ts.as<int64_t>(), q->out_keys.as<int64_t>(), q->out_vals.as<u64>(),
                        q->out_nulls.as<unsigned char>(), q->out_expired.as<unsigned char>(), q->out_rep.as<int64_t>(),
                        q->sc_ochunk.as<int64_t>(), q->sc_osend.as<int64_t>());
    } else if (xt) {
        launch_scxt_rows(s, M, n_old, q->sc_pcb.as<int64_t>(), nb, q->sc_skey.as<u64>(), q->scx_fe.as<u32>(),
                         q->scx_fpre.as<u32>(), q->scx_last.as<u32>(), q->sc_ghead.as<u32>(), q->scx_rows.as<u32>(),
                         q->sc_slast.as<u32>(), q->sc_sval.as<u64>(), q->sc_chunk.as<int64_t>(),
                         q->sc_send.as<int64_t>(), q->scx_clk.as<int64_t>(), q->pend_ts.as<int64_t>(),
                         q->pend_gidx.as<u64>(), q->kt.dev(), q->kp, q->ap, cur_on, T, q->out_ts.as<int64_t>(),
                         q->out_keys.as<int64_t>(), q->out_vals.as<u64>(), q->out_nulls.as<unsigned char>(),
                         q->out_expired.as<unsigned char>(), q->out_rep.as<int64_t>(), q->sc_ochunk.as<int64_t>(),
                         q->sc_osend.as<int64_t>());
    } else {
        launch_sc_emit(s, M, n_old, all_heads ? nullptr : q->sc_ghead.as<u32>(), q->sc_pre.as<u32>(), q->sc_slast.as<u32>(),
                       q->sc_sval.as<u64>(), q->pend_pos.as<u32>(), q->pend_ts.as<int64_t>(), q->pend_gidx.as<u64>(),
                       q->sc_chunk.as<int64_t>(), q->sc_send.as<int64_t>(), q->kt.dev(), q->kp, na, T,
                       q->out_ts.as<int64_t>(), q->out_keys.as<int64_t>(), q->out_vals.as<u64>(),
                       q->out_rep.as<int64_t>(), all_heads ? nullptr : q->sc_ochunk.as<int64_t>(),
                       q->sc_osend.as<int64_t>(), q->given ? q->out_order.as<int64_t>() : nullptr);
    }
    HIPCHK(hipGetLastError());
    PinnedVec<int64_t>& fo = host_out ? q->out.flush_offsets : q->dev_flush_offsets;
    PinnedVec<int64_t>& fc = host_out ? q->out.flush_clock : q->dev_flush_clock;
    fo.assign(1, 0);
    fc.clear();
    if (!(xs || xt)) {
        // a flush ends where the row's chunk changes: flags, their scan, the offsets and clocks
        RCHK(q->sc_bclk.reserve((size_t)std::max(nb, 1) * 8, false));
        RCHK(q->sc_h.reserve((size_t)std::max(nb, 1) * 8 + 64));
        for (int i = 0; i < nb; i++) q->sc_h.as<int64_t>()[i] = bounds[i].clock;
        if (nb) HIPCHK(hipMemcpyAsync(q->sc_bclk.p, q->sc_h.p, (size_t)nb * 8, hipMemcpyHostToDevice, s));
        RCHK(q->h_small_sc.reserve(64));
        int64_t nf = T;  // (every row its own chunk: a flush per row, no flags to scan)
        if (!all_heads) {
            RCHK(q->sc_fflag.reserve((size_t)(T + 1) * 4, false));
            RCHK(q->sc_tmp.reserve((size_t)((T + 1 + kTile - 1) / kTile + 16) * 8, false));
            launch_sc_flush_flags(s, T, q->sc_ochunk.as<int64_t>(), q->sc_fflag.as<u32>());
            launch_scan_sum_large_u32(s, q->sc_fflag.as<u32>(), T + 1, q->sc_tmp.as<int64_t>());
            HIPCHK(hipMemcpyAsync(q->h_small_sc.p, q->sc_fflag.as<uint32_t>() + T, 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            nf = *q->h_small_sc.as<uint32_t>();
        }
        q->compact_now = false;
        const bool want_compact = q->compact_flushes && q->rate.kind == SH_RATE_NONE && !q->xmode && nf > 0 && nf == T;
        if (all_heads && want_compact) {
            // (a flush per row: check the rows' clocks against their timestamps before writing any flush)
            launch_sc_clock_is_ts(s, T, q->sc_osend.as<int64_t>(), q->sc_slp.as<int64_t>(), cv0 ? 1 : 0, clock0,
                                  q->out_ts.as<int64_t>(), q->h_small_sc.as<uint32_t>() + 1);
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamSynchronize(s));
            q->compact_now = q->h_small_sc.as<uint32_t>()[1] == 1u;
        }
        if (!q->compact_now) {
            RCHK(q->sc_fo.reserve((size_t)std::max<int64_t>(nf, 1) * 8, false));
            RCHK(q->sc_fc.reserve((size_t)std::max<int64_t>(nf, 1) * 8, false));
            launch_sc_flushes(s, T, q->sc_osend.as<int64_t>(), all_heads ? nullptr : q->sc_fflag.as<u32>(),
                              q->sc_slp.as<int64_t>(), cv0 ? 1 : 0, clock0, q->sc_bclk.as<int64_t>(),
                              q->sc_fo.as<int64_t>(), q->sc_fc.as<int64_t>());
            HIPCHK(hipGetLastError());
        }
        if (!all_heads && want_compact) {
            // one row per flush: offsets implicit; clocks implicit too when each equals its row's ts
            launch_flush_clock_is_ts(s, nf, q->sc_fc.as<int64_t>(), q->out_ts.as<int64_t>(), q->h_small_sc.as<uint32_t>() + 1);
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamSynchronize(s));
            q->compact_now = q->h_small_sc.as<uint32_t>()[1] == 1u;
        }
        if (!q->compact_now) {
            fo.resize((size_t)nf + 1);
            fc.resize((size_t)nf);
            if (nf) {
                HIPCHK(hipMemcpyAsync(fo.data() + 1, q->sc_fo.p, (size_t)nf * 8, hipMemcpyDeviceToHost, s));
                HIPCHK(hipMemcpyAsync(fc.data(), q->sc_fc.p, (size_t)nf * 8, hipMemcpyDeviceToHost, s));
            }
        }
        HIPCHK(hipStreamSynchronize(s));
    }
    // every row's chunk and send
    const int64_t* och = nullptr;
    const int64_t* osd = nullptr;
    if (T && (xs || xt)) {
        RCHK(q->sc_ho.reserve((size_t)2 * T * 8 + 64));
        int64_t* hs = q->sc_ho.as<int64_t>();
        HIPCHK(hipMemcpyAsync(hs, q->sc_ochunk.p, (size_t)T * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(hs + T, q->sc_osend.p, (size_t)T * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        och = hs;  // read in place from the pinned landing area
        osd = hs + T;
    }
    if (xs || xt) {
        fo.reserve((size_t)T + 1);  // (one pinned allocation, not a doubling series)
        fc.reserve((size_t)T);
        for (int64_t i = 0; i < T; i++) {
            if (i + 1 == T || och[i + 1] != och[i]) {
                fo.push_back(i + 1);
                fc.push_back(osd[i] >= 0 ? sl[osd[i]] : bounds[-osd[i] - 1].clock);
            }
        }
    }
    float ms = 0;
    (void)hipEventElapsedTime(&ms, q->ev_agg0, q->ev_agg1);
    q->stats.main_kernel_ms += ms;
    if (host_out) {
        OutHost& o = q->out;
        o.ts.resize(T);
        o.expired.resize(T);
        o.rep.resize(T);
        o.keys.resize((size_t)nk * T);
        o.vals.resize((size_t)na * T);
        o.nulls.resize((size_t)na * T);
        if (T) {
            HIPCHK(hipMemcpyAsync(o.expired.data(), q->out_expired.p, T, hipMemcpyDeviceToHost, s));
            if (na) HIPCHK(hipMemcpyAsync(o.nulls.data(), q->out_nulls.p, (size_t)na * T, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(o.ts.data(), q->out_ts.p, T * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(o.rep.data(), q->out_rep.p, T * 8, hipMemcpyDeviceToHost, s));
            if (nk) HIPCHK(hipMemcpyAsync(o.keys.data(), q->out_keys.p, (size_t)nk * T * 8, hipMemcpyDeviceToHost, s));
            if (na) HIPCHK(hipMemcpyAsync(o.vals.data(), q->out_vals.p, (size_t)na * T * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
        // sharded owner: a row's merge order is the global stream index of its group's first event in the chunk
        if (q->given) {
            q->order_host.resize(T);
            if (T) HIPCHK(hipMemcpyAsync(q->order_host.data(), q->out_order.p, T * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
    } else {
        q->dev_out.n_rows = T;
    }
    return SH_OK;
}

// timeBatch(T, true) with expired output: the open window closed by a TIMER without events
// (sh_advance_time): one flush of its keys' EXPIRED rows (empty state) at clock `now`
static int sc_expire_pending(sh_query* q, int64_t now, bool host_out) {
    hipStream_t s = q->ctx->stream;
    const int64_t M = q->n_pend;
    const int nk = q->kp.n, na = q->ap.n;
    RCHK(q->sc_skey.reserve((size_t)M * 8, false));
    RCHK(q->sc_skey2.reserve((size_t)M * 8, false));
    RCHK(q->sc_idx.reserve((size_t)M * 4, false));
    RCHK(q->sc_idx2.reserve((size_t)M * 4, false));
    RCHK(q->sc_chunk.reserve((size_t)M * 8, false));
    RCHK(q->sc_send.reserve((size_t)M * 8, false));
    RCHK(q->sc_hd.reserve((size_t)(M + 1) * 4, false));
    RCHK(q->sc_pos.reserve((size_t)(M + 1) * 4, false));
    RCHK(q->sc_starts.reserve((size_t)(M + 1) * 4, false));
    RCHK(q->sc_tmp.reserve((size_t)((M + 1 + kTile - 1) / kTile + 16) * 8, false));
    RCHK(q->scx_fe.reserve((size_t)(M + 1) * 4, false));
    RCHK(q->scx_fpre.reserve((size_t)(M + 1) * 4, false));
    RCHK(q->scx_last.reserve((size_t)M * 4, false));
    RCHK(q->sc_pcb.reserve(8, false));
    launch_sc_keys(s, M, M, q->sc_pcb.as<int64_t>(), 0, q->pend_pos.as<u32>(), q->pend_gidx.as<u64>(), 0, 0, 0,
                   q->sc_skey.as<u64>(), q->sc_idx.as<u32>(), q->sc_chunk.as<int64_t>(), q->sc_send.as<int64_t>());
    size_t tb = 0;
    if (sort_u64_pairs(nullptr, &tb, nullptr, nullptr, nullptr, nullptr, M, s))
        return sh_fail(SH_ERR_DEVICE, "stream.current: sort sizing");
    RCHK(q->sc_sort.reserve(std::max<size_t>(tb, 16), false));
    if (sort_u64_pairs(q->sc_sort.p, &tb, q->sc_skey.as<u64>(), q->sc_skey2.as<u64>(), q->sc_idx.as<u32>(),
                       q->sc_idx2.as<u32>(), M, s))
        return sh_fail(SH_ERR_DEVICE, "stream.current: sort failed");
    launch_rate_segments(s, M, q->sc_skey2.as<u64>(), q->sc_idx2.as<u32>(), 1, 0, q->sc_hd.as<u32>(),
                         q->sc_pos.as<u32>(), q->sc_starts.as<u32>(), q->sc_tmp.as<int64_t>());
    HIPCHK(hipMemsetAsync(q->scx_fe.p, 0, (size_t)(M + 1) * 4, s));
    launch_scx_first(s, M, q->sc_hd.as<u32>(), q->sc_pos.as<u32>(), q->sc_starts.as<u32>(), q->sc_idx2.as<u32>(),
                     q->scx_fe.as<u32>(), q->scx_fpre.as<u32>(), q->scx_last.as<u32>());
    HIPCHK(hipMemcpyAsync(q->scx_fpre.p, q->scx_fe.p, (size_t)(M + 1) * 4, hipMemcpyDeviceToDevice, s));
    launch_scan_sum_large_u32(s, q->scx_fpre.as<u32>(), M + 1, q->sc_tmp.as<int64_t>());
    RCHK(q->h_small_sc.reserve(64));
    HIPCHK(hipMemcpyAsync(q->h_small_sc.p, q->scx_fpre.as<uint32_t>() + M, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const int64_t T = *q->h_small_sc.as<uint32_t>();
    const int64_t TC = std::max<int64_t>(T, 1);
    RCHK(q->out_ts.reserve(TC * 8, false));
    RCHK(q->out_keys.reserve((size_t)std::max(1, nk) * TC * 8, false));
    RCHK(q->out_vals.reserve((size_t)std::max(1, na) * TC * 8, false));
    RCHK(q->out_nulls.reserve((size_t)std::max(1, na) * TC, false));
    RCHK(q->out_expired.reserve(TC, false));
    RCHK(q->out_rep.reserve(TC * 8, false));
    q->zeroed_nulls = nullptr;
    q->zeroed_expired = nullptr;
    launch_scx_pending_rows(s, M, q->scx_fe.as<u32>(), q->scx_fpre.as<u32>(), q->scx_last.as<u32>(),
                            q->pend_pos.as<u32>(), q->pend_gidx.as<u64>(), q->kt.dev(), q->kp, q->ap, now, T,
                            q->out_ts.as<int64_t>(), q->out_keys.as<int64_t>(), q->out_vals.as<u64>(),
                            q->out_nulls.as<unsigned char>(), q->out_expired.as<unsigned char>(),
                            q->out_rep.as<int64_t>());
    HIPCHK(hipGetLastError());
    PinnedVec<int64_t>& fo = host_out ? q->out.flush_offsets : q->dev_flush_offsets;
    PinnedVec<int64_t>& fc = host_out ? q->out.flush_clock : q->dev_flush_clock;
    fo.assign(1, 0);
    fc.clear();
    if (T) {
        fo.push_back(T);
        fc.push_back(now);
    }
    if (host_out) {
        OutHost& o = q->out;
        o.ts.resize(T);
        o.expired.resize(T);
        o.rep.resize(T);
        o.keys.resize((size_t)nk * T);
        o.vals.resize((size_t)na * T);
        o.nulls.resize((size_t)na * T);
        if (T) {
            HIPCHK(hipMemcpyAsync(o.expired.data(), q->out_expired.p, T, hipMemcpyDeviceToHost, s));
            if (na) HIPCHK(hipMemcpyAsync(o.nulls.data(), q->out_nulls.p, (size_t)na * T, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(o.ts.data(), q->out_ts.p, T * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(o.rep.data(), q->out_rep.p, T * 8, hipMemcpyDeviceToHost, s));
            if (nk) HIPCHK(hipMemcpyAsync(o.keys.data(), q->out_keys.p, (size_t)nk * T * 8, hipMemcpyDeviceToHost, s));
            if (na) HIPCHK(hipMemcpyAsync(o.vals.data(), q->out_vals.p, (size_t)na * T * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
        }
    } else {
        q->dev_out.n_rows = T;
    }
    return SH_OK;
}

// entries [lo, lo + n) of the pending buffer moved to its front: one copy per column when the ranges
// do not overlap, else through the query's staging buffer (r05: a buffer allocated per push cost a
// hipMalloc, a stream drain and a hipFree on every stream.current push)
static int pending_to_front(sh_query* q, int64_t lo, int64_t n) {
    if (lo == 0 || n == 0) return SH_OK;
    hipStream_t s = q->ctx->stream;
    const bool direct = lo >= n;
    if (!direct) RCHK(q->pend_tmp.reserve((size_t)n * 8, false));
    auto move = [&](void* base, size_t elem) -> int {
        if (direct) {
            HIPCHK(hipMemcpyAsync(base, (char*)base + (size_t)lo * elem, (size_t)n * elem, hipMemcpyDeviceToDevice, s));
            return SH_OK;
        }
        void* t = q->pend_tmp.p;
        HIPCHK(hipMemcpyAsync(t, (char*)base + (size_t)lo * elem, (size_t)n * elem, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(base, t, (size_t)n * elem, hipMemcpyDeviceToDevice, s));
        return SH_OK;
    };
    RCHK(move(q->pend_pos.p, 4));
    RCHK(move(q->pend_ts.p, 8));
    RCHK(move(q->pend_gidx.p, 8));
    for (int j = 0; j < q->ap.n_vcols; j++) RCHK(move(q->pend_vals.as<char>() + (size_t)j * q->pend_cap * 8, 8));
    return SH_OK;
}

// Small pushes that close no window — most calls of send(Event[n]) with small n: one kernel
// (k_small_push) appends the passing events to the open window and reports through coherent pinned
// memory, which the host polls instead of synchronising the stream. A push that would close a window
// (or whose timestamps decrease) is reported back untouched and runs through the full pipeline.
bool query_small_eligible(const sh_query* q, int64_t N) {
    if (N <= 0 || N > kSmallMax || q->kind != 0 || q->xmode || q->d.stream_current || q->partitioned || q->given ||
        q->rate.kind != SH_RATE_NONE || q->ap.n == 0)
        return false;
    const int w = q->d.window;
    return w == SH_WIN_LENGTH_BATCH || (w == SH_WIN_TIME_BATCH && q->e0_valid && q->clock_valid);
}

// The last asynchronous small push's report: verified once its token has arrived (wait: spin for
// it). Reports arrive in launch order and the key table's overflow flag is sticky, so any later
// report covers the earlier pushes too.
static int small_verify(sh_query* q, bool wait) {
    if (!q->async_tok) return SH_OK;
    volatile SmallRes* r = q->small_res;
    hipStream_t s = q->ctx->stream;
    for (int spin = 0; *(volatile uint64_t*)&r->token < q->async_tok; spin++) {
        if (!wait) return SH_OK;
        if ((spin & 1023) == 1023) {
            const hipError_t e = hipStreamQuery(s);
            if (e == hipSuccess) {
                if (*(volatile uint64_t*)&r->token < q->async_tok) return sh_fail(SH_ERR_DEVICE, "small push: no report");
                break;
            }
            if (e != hipErrorNotReady) return sh_fail(SH_ERR_DEVICE, std::string("small push: ") + hipGetErrorString(e));
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    uint32_t ctrl[4];
    for (int i = 0; i < 4; i++) ctrl[i] = r->ctrl[i];
    q->async_tok = 0;
    q->async_keys = 0;
    return q->kt.check_result(ctrl);
}

// every queued asynchronous small push verified (snapshot, restore and destroy read or replace the
// state its report describes)
int query_drain_async(sh_query* q) { return small_verify(q, true); }

// Asynchronous small push (InputHandler.send returning once the junction has the events,
// StreamJunction :104-131): a zero-copy batch of a query without a filter whose timestamps do not
// decrease and that closes no window — the host checks both on the pinned batch itself — is copied
// into a pinned ring slot (the caller may reuse its buffer as soon as the call returns), the append
// kernel is queued and the call returns at once. Its report is verified by a later call.
static int small_async(sh_query* q, bool* done) {
    const sh_batch* hb = q->zc_host;
    const int64_t N = hb->n;
    if (filter_kind(q->fp) != 0 || q->tune.no_async_small) return SH_OK;
    // a hashed key table may take at most one new key per event: only while that bound stays within
    // the table's half (the growth threshold, checked on verified counts) is the push queued unverified
    if (!q->kt.dense && q->kt.n_keys + q->async_keys + N > (int64_t)q->kt.size_ / 2) return SH_OK;
    const int64_t* hts = hb->ts;
    for (int64_t i = 1; i < N; i++)
        if (hts[i] < hts[i - 1]) return SH_OK;
    const int64_t clk = q->clock_valid ? std::max(q->clock, hts[N - 1]) : hts[N - 1];
    if (q->d.window == SH_WIN_LENGTH_BATCH ? q->n_pend + N >= q->d.window_param : wfun_host(q, clk) > q->W_open)
        return SH_OK;
    const int nc = q->d.n_cols;
    auto a16 = [](size_t x) { return (x + 15) & ~(size_t)15; };
    if (!q->zc_ring) {
        size_t sl = a16((size_t)kSmallMax * 8);
        for (int c = 0; c < nc; c++) sl += a16((size_t)kSmallMax * type_size(q->d.col_types[c]));
        if (hipHostMalloc((void**)&q->zc_ring, sl * sh_query::kZcRing, hipHostMallocMapped) != hipSuccess ||
            hipHostGetDevicePointer((void**)&q->zc_ring_dev, q->zc_ring, 0) != hipSuccess) {
            q->zc_ring = nullptr;
            return sh_fail(SH_ERR_OOM, "pinned allocation failed");
        }
        q->zc_slot = sl;
    }
    volatile SmallRes* r = q->small_res;
    hipStream_t s = q->ctx->stream;
    const int slot = q->zc_next;
    // the slot's previous reader has finished (reports arrive in launch order)
    for (int spin = 0; *(volatile uint64_t*)&r->token < q->zc_tok[slot]; spin++) {
        if ((spin & 1023) == 1023) {
            const hipError_t e = hipStreamQuery(s);
            if (e == hipSuccess) break;
            if (e != hipErrorNotReady) return sh_fail(SH_ERR_DEVICE, std::string("small push: ") + hipGetErrorString(e));
        }
    }
    char* hbase = q->zc_ring + (size_t)slot * q->zc_slot;
    char* dbase = q->zc_ring_dev + (size_t)slot * q->zc_slot;
    sh_batch dv = *hb;
    size_t off = 0;
    std::memcpy(hbase, hts, (size_t)N * 8);
    dv.ts = (const int64_t*)dbase;
    off = a16((size_t)kSmallMax * 8);
    ColSet cs{};
    cs.n = nc;
    for (int c = 0; c < nc; c++) {
        const size_t ts_ = type_size(q->d.col_types[c]);
        cs.type[c] = q->load_type[c];
        cs.ptr[c] = nullptr;
        if (hb->cols[c]) {
            std::memcpy(hbase + off, hb->cols[c], (size_t)N * ts_);
            cs.ptr[c] = dbase + off;
        }
        off += a16((size_t)kSmallMax * ts_);
    }
    WinParams wp{};
    wp.kind = q->d.window;
    wp.e0_valid = q->e0_valid;
    wp.clock_valid = q->clock_valid;
    wp.L = wp.T = q->d.window_param;
    wp.cal = q->cal;
    wp.cal_tz = q->cal_tz;
    wp.E0 = q->E0;
    wp.clock0 = q->clock;
    wp.W_open = q->W_open;
    wp.n_pend = q->n_pend;
    wp.send_size = hb->send_size;
    wp.N = N;
    const uint64_t token = ++q->small_token;
    launch_small_push(s, dv.ts, cs, q->fp, wp, q->kp, q->kt.dev(), q->ap, q->pend_pos.as<u32>(), q->pend_ts.as<int64_t>(),
                      q->pend_vals.as<u64>(), q->pend_cap, q->pend_gidx.as<u64>(), q->seq, q->small_res_dev, token,
                      true);
    HIPCHK(hipGetLastError());
    q->zc_tok[slot] = token;
    q->zc_next = (slot + 1) % sh_query::kZcRing;
    q->async_tok = token;
    q->async_keys += N;
    q->n_pend += N;  // no filter: every event joins the open window
    q->seq += N;
    q->clock = clk;
    q->clock_valid = true;
    q->stats.events = N;
    *done = true;
    return SH_OK;
}

// ---- externalTimeBatch timeout (ExternalTimeBatchWindowProcessor.process :256-305) -----------------
// lastScheduledTime L is the clock of the window's first event, of every batch crossing and of every
// timeout, + the timeout. A timeout fires where the clock reaches L: at the start of the first send
// whose last event reaches L (Scheduler timers run before the send's events). It sends the open batch
// so far, when it holds events not yet sent (flushToOutputChunk the first time, appendToOutputChunk —
// the batch again, whole — after that); a crossing sends the batch likewise, and nothing when a
// timeout already sent all of it. Every emission aggregates the open batch from its first event.
extern "C" int sh_query_set_ext_timeout(sh_query* q, int64_t ms) {
    if (!q) return sh_fail(SH_ERR_INVALID, "sh_query_set_ext_timeout: NULL query");
    if (q->d.window != SH_WIN_EXT_TIME_BATCH || ms < 0)
        return sh_fail(SH_ERR_INVALID, "a timeout needs an externalTimeBatch window and >= 0 ms");
    if (q->seq != 0 || q->n_pend != 0 || q->clock_valid)
        return sh_fail(SH_ERR_INVALID, "sh_query_set_ext_timeout: set it before the first push");
    if (ms == 0) { q->xt_timeout = 0; return SH_OK; }
    // partitioned: on the sorted partition lanes (lane 3), the Scheduler walked on the host (sh_plane.cpp
    // xt_walk) with its HashMap tie order, which hashes String.valueOf of the partition key
    const bool lanes = q->kind == 1 && q->d.partition_col >= 0 && q->sl && plane_is_sorted_lane(q);
    if ((q->kind != 0 && !lanes) || (q->d.partition_col >= 0 && !lanes) || q->given || q->internal_keys)
        return sh_fail(SH_ERR_UNSUPPORTED, "externalTimeBatch timeout of a sharded query");
    if (lanes) {
        if (q->d.stream_current) return sh_fail(SH_ERR_UNSUPPORTED, "externalTimeBatch timeout with stream.current.event");
        q->xt_timeout = ms;
        return SH_OK;
    }
    if (q->d.stream_current)
        return sh_fail(SH_ERR_UNSUPPORTED, "externalTimeBatch timeout with stream.current.event output");
    q->xt_timeout = ms;
    // Every emission — a timeout's flushToOutputChunk / appendToOutputChunk or a crossing's (:336-438) —
    // is [expired copies of the previous emission's events, RESET, the open batch from its first event]:
    // the expired chunk always holds exactly what the previous emission sent as CURRENT (a flush moves
    // its current events there, an append adds the new ones to the re-sent ones). So the expired rows
    // follow the batch windows' rule (sh_expired.cpp, flush j + 1 carries flush j's rows re-stamped with
    // lastCurrentEventTime). Aggregating without group-by, all events: the chunk's one row is its last
    // CURRENT event's (processInBatchNoGroupBy), so no expired rows are needed.
    q->xmode = q->d.expired_on && !(q->d.current_on && q->d.n_group_by == 0 && q->ap.n > 0);
    return SH_OK;
}

namespace {
struct XtEmit {
    Segment seg;
    int64_t clock, window;
    int64_t stamp;  // lastCurrentEventTime at the emission (the expired rows' timestamp)
};
}  // namespace

// The timeout due where the push's clock reaches L: its send's first event (push index), that send's
// clock, and the push's passing events before it.
static int xt_probe(sh_query* q, const sh_batch* b, int64_t L, int64_t* f, int64_t* clk, int64_t* pcb, int64_t* xmax) {
    hipStream_t s = q->ctx->stream;
    const int64_t N = b->n, ss = b->send_size;
    RCHK(q->xt_dev.reserve(24, false));
    RCHK(q->xt_host.reserve(24));
    auto* d = q->xt_dev.as<unsigned long long>();
    int64_t* h = q->xt_host.as<int64_t>();
    HIPCHK(hipMemsetAsync(d, 0xFF, 8, s));
    launch_xt_first_send(s, b->ts, N, ss, L, d);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h, d, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const uint64_t j = (uint64_t)h[0];
    if (j == ~0ull) return sh_fail(SH_ERR_INVALID, "externalTimeBatch timeout: no send reaches the scheduled time");
    *f = ss > 0 ? (int64_t)j * ss : 0;
    const int64_t last = ss > 0 ? std::min<int64_t>(((int64_t)j + 1) * ss, N) - 1 : N - 1;
    ColSet cs{};
    cs.n = q->d.n_cols;
    for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->load_type[c]; cs.ptr[c] = b->cols[c]; }
    const int64_t lo_m = INT64_MIN;
    HIPCHK(hipMemsetAsync(d + 1, 0, 8, s));
    HIPCHK(hipMemcpyAsync(d + 2, &lo_m, 8, hipMemcpyHostToDevice, s));
    launch_xt_count_pass(s, cs, q->fp, *f, d + 1, q->d.ts_col, (long long*)(d + 2));
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h + 1, d + 1, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(h, b->ts + last, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    *clk = h[0];
    *pcb = h[1];
    *xmax = h[2];
    return SH_OK;
}

// The push's emissions in stream order: timeouts and the crossings (bounds) that have events to send.
static int xt_plan(sh_query* q, const sh_batch* b, const PushInfo& info, const std::vector<Bound>& bounds,
                   int64_t clock0, bool cv0, int64_t xm0, std::vector<XtEmit>& em) {
    const int64_t T = q->xt_timeout;
    if (!q->xt_Lvalid && info.total_pass > 0) {
        // initTiming (:313-334): scheduled from the clock of the window's first event's send
        q->xt_L = (cv0 ? std::max(clock0, info.first_clk) : info.first_clk) + T;
        q->xt_Lvalid = true;
    }
    const int64_t nnew0 = q->xt_nnew;
    bool sent = false;
    int64_t last_pcb = 0, lo = 0, w = q->W_open;
    auto nnew_at = [&](int64_t pcb) { return (sent ? 0 : nnew0) + pcb - last_pcb; };
    auto timeouts = [&](int64_t clk) -> int {
        while (q->xt_Lvalid && clk >= q->xt_L) {
            int64_t f, cf, pf, xf;
            RCHK(xt_probe(q, b, q->xt_L, &f, &cf, &pf, &xf));
            if (nnew_at(pf) > 0) em.push_back(XtEmit{Segment{lo, q->n_pend + f}, cf, w, std::max(xm0, xf)});
            sent = true;
            last_pcb = pf;
            q->xt_L = cf + T;
        }
        return SH_OK;
    };
    for (const Bound& bd : bounds) {
        RCHK(timeouts(bd.clock));
        if (nnew_at(bd.pcb) > 0) em.push_back(XtEmit{Segment{lo, bd.idx}, bd.clock, w, bd.pad});
        sent = true;
        last_pcb = bd.pcb;
        lo = bd.idx;
        w = bd.W;
        q->xt_L = bd.clock + T;
    }
    RCHK(timeouts(cv0 ? std::max(clock0, info.max_tl) : info.max_tl));
    q->xt_nnew = nnew_at(info.total_pass);
    return SH_OK;
}

// Host rows of the push (q->out) as its device output.
static int xt_upload(sh_query* q) {
    hipStream_t s = q->ctx->stream;
    const int64_t n = (int64_t)q->out.ts.size();
    const int nk = q->kp.n, na = q->ap.n;
    const int64_t cap = std::max<int64_t>(n, 1);
    RCHK(q->out_ts.reserve(cap * 8, false));
    RCHK(q->out_rep.reserve(cap * 8, false));
    RCHK(q->out_keys.reserve(std::max(1, nk) * cap * 8, false));
    RCHK(q->out_vals.reserve(std::max(1, na) * cap * 8, false));
    RCHK(q->out_nulls.reserve(std::max(1, na) * cap, false));
    RCHK(q->out_expired.reserve(cap, false));
    if (n) {
        HIPCHK(hipMemcpyAsync(q->out_ts.p, q->out.ts.data(), n * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(q->out_rep.p, q->out.rep.data(), n * 8, hipMemcpyHostToDevice, s));
        if (nk) HIPCHK(hipMemcpyAsync(q->out_keys.p, q->out.keys.data(), (size_t)nk * n * 8, hipMemcpyHostToDevice, s));
        if (na) HIPCHK(hipMemcpyAsync(q->out_vals.p, q->out.vals.data(), (size_t)na * n * 8, hipMemcpyHostToDevice, s));
    }
    HIPCHK(hipMemsetAsync(q->out_nulls.p, 0, q->out_nulls.cap, s));
    HIPCHK(hipMemsetAsync(q->out_expired.p, 0, q->out_expired.cap, s));
    q->zeroed_nulls = q->out_nulls.p;
    q->zeroed_expired = q->out_expired.p;
    HIPCHK(hipStreamSynchronize(s));
    q->dev_flush_offsets.assign(1, 0);
    q->dev_flush_clock.clear();
    for (size_t i = 1; i < q->out.flush_offsets.size(); i++) q->dev_flush_offsets.push_back(q->out.flush_offsets[i]);
    for (size_t i = 0; i < q->out.flush_clock.size(); i++) q->dev_flush_clock.push_back(q->out.flush_clock[i]);
    q->dev_out.n_rows = n;
    q->out.reset();
    return SH_OK;
}

// The emissions, in runs of disjoint segments (a timeout's segment overlaps its batch's later ones):
// one run goes out like any push's closed batches; several collect host rows run by run.
static int xt_emit(sh_query* q, const std::vector<XtEmit>& em, const sh_batch* b, bool host_out) {
    if (em.empty()) return SH_OK;
    std::vector<std::vector<XtEmit>> runs;
    for (const XtEmit& e : em) {
        if (runs.empty() || e.seg.lo < runs.back().back().seg.hi) runs.emplace_back();
        runs.back().push_back(e);
    }
    for (size_t i = 0; i < runs.size(); i++) {
        std::vector<Segment> segs;
        std::vector<int64_t> clocks, windows;
        for (const XtEmit& e : runs[i]) {
            segs.push_back(e.seg);
            clocks.push_back(e.clock);
            windows.push_back(e.window);
        }
        if (i) q->ms_ready = false;  // (the split of the first run may not reach this run's events)
        RCHK(run_closed(q, segs, clocks, windows, b, runs.size() == 1 ? host_out : true));
    }
    if (runs.size() > 1 && !host_out) RCHK(xt_upload(q));
    return SH_OK;
}

static int try_small_push(sh_query* q, const sh_batch* b, bool* done) {
    *done = false;
    const int64_t N = b->n;
    if (!query_small_eligible(q, N)) return SH_OK;
    const int w = q->d.window;
    if (!q->small_res) {
        if (hipHostMalloc((void**)&q->small_res, sizeof(SmallRes), hipHostMallocCoherent | hipHostMallocMapped) !=
                hipSuccess ||
            hipHostGetDevicePointer((void**)&q->small_res_dev, q->small_res, 0) != hipSuccess)
            return sh_fail(SH_ERR_OOM, "pinned allocation failed");
        std::memset(q->small_res, 0, sizeof(SmallRes));
    }
    RCHK(grow_pending(q, q->n_pend + N, q->n_pend));
    if (q->zc_host) {
        RCHK(small_async(q, done));
        if (*done) return SH_OK;
    }
    SH_TMARK(1);
    hipStream_t s = q->ctx->stream;
    ColSet cs{};
    cs.n = q->d.n_cols;
    for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->load_type[c]; cs.ptr[c] = b->cols[c]; }
    WinParams wp{};
    wp.kind = w;
    wp.e0_valid = q->e0_valid;
    wp.clock_valid = q->clock_valid;
    wp.L = wp.T = q->d.window_param;
    wp.cal = q->cal;
    wp.cal_tz = q->cal_tz;
    wp.E0 = q->E0;
    wp.clock0 = q->clock;
    wp.W_open = q->W_open;
    wp.n_pend = q->n_pend;
    wp.send_size = b->send_size;
    wp.N = N;
    const uint64_t token = ++q->small_token;
    launch_small_push(s, b->ts, cs, q->fp, wp, q->kp, q->kt.dev(), q->ap, q->pend_pos.as<u32>(), q->pend_ts.as<int64_t>(),
                      q->pend_vals.as<u64>(), q->pend_cap, q->pend_gidx.as<u64>(), q->seq, q->small_res_dev, token);
    HIPCHK(hipGetLastError());
    SH_TMARK(2);
    volatile SmallRes* r = q->small_res;
    for (int spin = 0; *(volatile uint64_t*)&r->token != token; spin++) {
        if ((spin & 1023) == 1023) {  // every ~1000 polls: is the stream still running?
            const hipError_t e = hipStreamQuery(s);
            if (e == hipSuccess) {
                if (*(volatile uint64_t*)&r->token != token) return sh_fail(SH_ERR_DEVICE, "small push: no report");
                break;
            }
            if (e != hipErrorNotReady) return sh_fail(SH_ERR_DEVICE, std::string("small push: ") + hipGetErrorString(e));
        }
    }
    std::atomic_thread_fence(std::memory_order_acquire);
    SH_TMARK(3);
    uint32_t ctrl[4];
    for (int i = 0; i < 4; i++) ctrl[i] = r->ctrl[i];
    if (r->fallback) return SH_OK;  // nothing was appended (the key lookups it made are kept)
    RCHK(q->kt.check_result(ctrl));
    q->n_pend += r->total_pass;
    q->seq += N;
    q->clock = std::max(q->clock, (int64_t)r->max_tl);
    q->stats.events = N;
    *done = true;
    return SH_OK;
}

static void given_closes(sh_query* q);

static int xr_trim(sh_query* q);
static int push_core(sh_query* q, const sh_batch* b, bool host_out_req, const sh_out** out) {
    SH_TMARK(0);
    // expired / all-events output: the current rows stay on the device for xout_finish
    const bool host_out = host_out_req && !q->xmode;
    q->x_closes.clear();
    q->x_stamps.clear();
    hipStream_t s = q->ctx->stream;
    q->out.reset();
    q->dev_flush_offsets.assign(1, 0);
    q->dev_flush_clock.clear();
    q->flush_window.clear();
    q->dev_out = sh_out{};
    q->stats = sh_stats{};
    q->agg_bytes = 0;
    q->order_host.clear();
    q->ms_ready = false;
    q->tail.active = false;
    int64_t N = b->n;
    const bool cv0 = q->clock_valid;
    const int64_t clock0 = q->clock, seq0 = q->seq;
    if (N < 0) return sh_fail(SH_ERR_INVALID, "negative batch size");
    if (N > 0 && (!b->ts)) return sh_fail(SH_ERR_INVALID, "batch without timestamps");
    if (q->n_pend + N >= (int64_t)0xFFFFFFF0ll) return sh_fail(SH_ERR_INVALID, "push larger than 4G events");
    RCHK(small_verify(q, false));
    if (N > 0 && !q->internal_keys && q->kt.n_keys + q->async_keys > (int64_t)q->kt.size_ / 2) {
        // unverified asynchronous pushes may have added keys: their report first, then the growth check
        RCHK(small_verify(q, true));
        if (q->kt.n_keys > (int64_t)q->kt.size_ / 2) RCHK(query_reserve_keys(q, 0));
    }
    {
        bool done = false;
        RCHK(try_small_push(q, b, &done));
        if (done) {
            finish_out(q, host_out, out);
            return SH_OK;
        }
        RCHK(small_verify(q, true));  // the full pipeline reads the state the queued appends left
    }
    sh_batch zc_dev;
    if (q->zc_host) {
        // a zero-copy batch that needs the full pipeline: on the device first
        RCHK(q->staged.stage(s, q->zc_host, q->d.n_cols, q->d.col_types, &zc_dev));
        q->zc_host = nullptr;
        b = &zc_dev;
    }
    HIPCHK(hipEventRecord(q->ev_push0, s));
    if (N > 0 && q->partitioned && !q->p0_known) RCHK(resolve_first_partition(q, b));
    if (N > 0 && !(q->partitioned && !q->p0_known)) {
        ColSet cs{};
        cs.n = q->d.n_cols;
        for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->load_type[c]; cs.ptr[c] = b->cols[c]; }
        int nblk = (int)((N + kTile - 1) / kTile);
        RCHK(q->blk_pass.reserve(nblk * 8, false));
        RCHK(q->blk_tl.reserve(nblk * 8, false));
        RCHK(q->blk_first.reserve(scan_blocks_first_bytes(nblk), false));
        WinParams wp{};
        wp.kind = q->d.window;
        wp.e0_valid = q->e0_valid;
        wp.clock_valid = q->clock_valid;
        wp.has_start = q->d.has_start_time;
        wp.L = q->d.window_param;
        wp.T = q->d.window_param;
        wp.cal = q->cal;
        wp.cal_tz = q->cal_tz;
        wp.E0 = q->E0;
        wp.start_time = q->d.start_time;
        wp.clock0 = q->clock;
        wp.W_open = q->W_open;
        wp.n_pend = q->n_pend;
        wp.send_size = b->send_size;
        wp.N = N;
        wp.ts_col = q->d.ts_col;
        wp.start_col = q->d.start_col;
        wp.xm0 = q->xm;
        const bool ext = q->d.window == SH_WIN_EXT_TIME_BATCH;
        if (ext) RCHK(q->blk_xm.reserve(nblk * 8, false));
        if (q->given) {
            // sharded owner: windows were assigned from the global clock by the ingest ranks
            wp.kind = SH_WIN_TIME_BATCH;
            wp.e0_valid = 1;
            wp.wcol = q->given_wcol;
            wp.W_base = q->given_W_base;
        }
        // timeBatch once nextEmitTime is known: one pass assigns the windows if the timestamps do not
        // decrease (checked by the pass itself, redone below with the prefix passes if they do);
        // otherwise (first timeBatch push, lengthBatch, externalTimeBatch, the sharded owner's given
        // windows) the block-aggregate + scan passes run first
        const bool single_pass = !ext && !q->given && wp.pcol1 == 0 && wp.kind == SH_WIN_TIME_BATCH && wp.e0_valid;
        auto prefix_passes = [&] {
            launch_blockagg(s, b->ts, cs, q->fp, N, b->send_size, q->blk_pass.as<int64_t>(), q->blk_tl.as<int64_t>(),
                            q->blk_first.as<int64_t>(), nblk, ext ? q->blk_xm.as<int64_t>() : nullptr,
                            ext ? q->d.ts_col : -1);
            launch_scan_blocks(s, q->blk_pass.as<int64_t>(), q->blk_tl.as<int64_t>(), q->blk_first.as<int64_t>(), nblk,
                               b->ts, wp, q->info.as<PushInfo>(), ext ? q->blk_xm.as<int64_t>() : nullptr, cs);
        };
        if (single_pass) {
            RCHK(q->blk_pass.reserve((size_t)(nblk + 1) * 8, false));
            launch_zero2(s, q->info.p, (int)sizeof(PushInfo), q->blk_pass.as<int64_t>() + nblk, 8);
            HIPCHK(hipGetLastError());
        } else {
            prefix_passes();
        }
        int max_bounds = (int)std::min<int64_t>(N + 1, 1 << 22);
        RCHK(q->bounds.reserve((size_t)max_bounds * sizeof(Bound), false));
        q->direct_pos = want_direct_pos(q);
        if (!q->direct_pos) RCHK(q->new_pos.reserve((size_t)N * 4, false));
        u32* slot_col = q->direct_pos ? nullptr : q->new_pos.as<u32>();
        // large pushes split the whole push into key partitions right behind k_boundaries, which
        // counts the push's tiles for it (a small push usually closes no window: no split then)
        const bool early_split = (q->P > 1 || q->partitioned) && N >= (1 << 18) && !q->d.stream_current;
        const TileMap ms_map = make_tile_map(q->n_pend, q->n_pend + N);
        if (early_split) RCHK(reserve_ms_counts(q, ms_map));
        launch_boundaries(s, b->ts, cs, q->fp, wp, q->blk_pass.as<int64_t>(), q->blk_tl.as<int64_t>(),
                          q->info.as<PushInfo>(), q->bounds.as<Bound>(), max_bounds, nblk, q->kp, q->kt.dev(),
                          slot_col, ext ? q->blk_xm.as<int64_t>() : nullptr,
                          early_split ? q->ms_counts.as<u32>() : nullptr, q->P, ms_map.nblk, ms_map.np_t,
                          single_pass, q->blk_tl.as<int64_t>());
        HIPCHK(hipGetLastError());
        // the push info and the first boundaries come back in one copy; the key partitioning of the
        // push's events (independent of where the windows close) is queued behind it and runs while
        // the host reads them
        // (as many as the last push found, with room: a push closing thousands of windows — C1 — would
        // otherwise read the rest after the split queued behind this copy, the host waiting for it)
        constexpr int kFirstBounds = 256;
        const int nb0 = (int)std::min<int64_t>(max_bounds, std::max<int64_t>(kFirstBounds, q->last_nb + q->last_nb / 4 + 64));
        RCHK(q->h_bounds.reserve((size_t)nb0 * sizeof(Bound)));
        HIPCHK(hipMemcpyAsync(q->h_info, q->info.p, sizeof(PushInfo), hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(q->h_bounds.p, q->bounds.p, (size_t)nb0 * sizeof(Bound), hipMemcpyDeviceToHost, s));
        if (q->band_spec) {
            // (a speculatively placed band: its overflow word comes back with the push info)
            RCHK(q->h_spec.reserve(16));
            RCHK(q->kt.check_async(s, q->h_spec.as<uint32_t>()));
        }
        HIPCHK(hipEventRecord(q->ev_mid, s));
        SH_TMARK(1);
        if (early_split) RCHK(run_multisplit(q, q->n_pend + N, b, true));
        SH_TRACE("push N=%lld n_pend=%lld: boundaries queued", (long long)N, (long long)q->n_pend);
        SH_TMARK(2);
        if (q->mid_hook) {
            RCHK(q->mid_hook(q->mid_arg));
            SH_TMARK(12);
        }
        HIPCHK(sh_wait_event(q->ev_mid));
        SH_TMARK(3);
        PushInfo info = *q->h_info;
        SH_TRACE("push info: pass=%lld bounds=%d", (long long)info.total_pass, info.n_bounds);
        if (q->band_spec && q->h_spec.as<uint32_t>()[2] == 3) {
            SH_TRACE("push: a bucket outside the speculative key band, retried after a probe");
            return kRetryBand;
        }
        if (single_pass && info.unsorted) {
            // a timestamp decreased: the send clocks need the prefix passes after all (the key slots,
            // the multisplit counts and the split already queued do not depend on the windows)
            SH_TRACE("push: unsorted timestamps, window assignment redone with the prefix passes");
            prefix_passes();
            launch_boundaries(s, b->ts, cs, q->fp, wp, q->blk_pass.as<int64_t>(), q->blk_tl.as<int64_t>(),
                              q->info.as<PushInfo>(), q->bounds.as<Bound>(), max_bounds, nblk, q->kp, q->kt.dev(),
                              slot_col, nullptr);
            HIPCHK(hipGetLastError());
            HIPCHK(hipMemcpyAsync(q->h_info, q->info.p, sizeof(PushInfo), hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(q->h_bounds.p, q->bounds.p, (size_t)nb0 * sizeof(Bound), hipMemcpyDeviceToHost, s));
            HIPCHK(sh_wait_stream(s));
            info = *q->h_info;
        }
        if (info.n_bounds > max_bounds) return sh_fail(SH_ERR_INVALID, "more than 4M windows closed in one push");
        if (ext && info.err)
            return sh_fail(SH_ERR_UNSUPPORTED,
                           "externalTimeBatch: the first event's timestamp is before its start time (not on the GPU)");
        const int64_t xm0 = q->xm;  // (lastCurrentEventTime before the push: timeout stamps)
        if (ext) q->xm = std::max(q->xm, info.max_xm);
        std::vector<Bound> bounds(info.n_bounds);
        q->last_nb = std::min<int64_t>(info.n_bounds, 1 << 16);
        if (info.n_bounds) {
            if (info.n_bounds <= nb0) {
                std::memcpy(bounds.data(), q->h_bounds.p, info.n_bounds * sizeof(Bound));
            } else {
                HIPCHK(hipMemcpyAsync(bounds.data(), q->bounds.p, info.n_bounds * sizeof(Bound), hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
            }
            std::sort(bounds.begin(), bounds.end(), [](const Bound& a, const Bound& c) { return a.idx < c.idx; });
        }
        if (q->xt_replace) {  // (the windows start at new events: stream index = seq0 + combined index - queued)
            RCHK(xr_trim(q));  // (what earlier calls left, so a call failing after this point leaves few)
            for (auto& bd : bounds) q->xr_starts.emplace_back(seq0 + std::max<int64_t>(0, bd.idx - q->n_pend), bd.W);
        }
        if (q->xmode) {
            q->x_stamps.clear();
            if (q->given) {
                given_closes(q);
            } else {
                for (auto& bd : bounds) {
                    q->x_closes.emplace_back(bd.W, bd.clock);
                    q->x_stamps.push_back(bd.pad);  // (externalTimeBatch: the attribute max at the close)
                }
            }
        }
        if (!q->given) {
            q->e0_valid = info.e0_valid;
            q->E0 = info.E0;
            q->clock = q->clock_valid ? std::max(q->clock, info.max_tl) : info.max_tl;
            q->clock_valid = true;
        }
        int64_t e_lo, pcb_lo, dst_base, new_pend;
        // sharded owner: the global clock closed every window below given_W_end during this push,
        // including the one this owner's last events belong to (a timer flush, Scheduler.java:171-209)
        const int64_t W_last = bounds.empty() ? q->W_open : bounds.back().W;
        // lengthBatch whose L-th event is the push's last event: LengthBatchWindowProcessor flushes
        // the batch while processing that send (:206-243), not when the next event arrives
        const int64_t open_cnt = bounds.empty() ? q->n_pend + info.total_pass : info.total_pass - bounds.back().pcb;
        const bool lb_full = !q->given && !q->d.stream_current && q->d.window == SH_WIN_LENGTH_BATCH && info.total_pass > 0 &&
                             open_cnt == q->d.window_param;
        const bool close_all = (q->given && q->given_W_end > W_last) || lb_full;
        if (q->xt_timeout > 0) {
            std::vector<XtEmit> em;
            RCHK(xt_plan(q, b, info, bounds, clock0, cv0, xm0, em));
            if (q->xmode) {  // (the emissions, not the crossings, are the flushes carrying expired rows)
                q->x_stamps.clear();
                for (const XtEmit& e : em) q->x_stamps.push_back(e.stamp);
            }
            RCHK(xt_emit(q, em, b, host_out));
        }
        if (!bounds.empty() || close_all) {
            std::vector<Segment> segs;
            std::vector<int64_t> clocks, windows;
            int64_t lo = 0, wprev = q->W_open;
            for (auto& bd : bounds) {
                segs.push_back(Segment{lo, bd.idx});
                clocks.push_back(q->given ? given_flush_clock(q, wprev)
                                          : q->d.window == SH_WIN_LENGTH_BATCH ? bd.clock_prev : bd.clock);
                windows.push_back(wprev);
                lo = bd.idx;
                wprev = bd.W;
            }
            if (close_all) {
                segs.push_back(Segment{lo, q->n_pend + N});
                clocks.push_back(lb_full ? q->clock : given_flush_clock(q, wprev));
                windows.push_back(wprev);
            }
            if (!q->d.stream_current && q->xt_timeout == 0) RCHK(run_closed(q, segs, clocks, windows, b, host_out));
            if (close_all) {
                e_lo = N;
                pcb_lo = info.total_pass;
                dst_base = 0;
                new_pend = 0;
                q->W_open = lb_full ? 0 : q->given_W_end;
            } else {
                e_lo = bounds.back().idx - q->n_pend;
                pcb_lo = bounds.back().pcb;
                dst_base = 0;
                new_pend = info.total_pass - pcb_lo;
                // lengthBatch windows are numbered relative to the open batch (W = (n_pend + pcb) / L)
                q->W_open = (!q->given && q->d.window == SH_WIN_LENGTH_BATCH) ? 0 : bounds.back().W;
            }
        } else {
            e_lo = 0;
            pcb_lo = 0;
            dst_base = q->n_pend;
            new_pend = q->n_pend + info.total_pass;
        }
        if (q->d.stream_current) {
            // every passing event is emitted now: all of them join the pending entries, the rows come
            // from the open window's earlier events + these; the last window's entries stay queued
            const int64_t n_old = q->n_pend, M = n_old + info.total_pass;
            RCHK(grow_pending(q, M, n_old));
            launch_compact_pending(s, b->ts, cs, pos_src(q, b), q->ap, 0, N, 0, n_old,
                                   q->blk_pass.as<int64_t>(), q->pend_pos.as<u32>(), q->pend_ts.as<int64_t>(),
                                   q->pend_vals.as<u64>(), q->pend_cap, q->given ? q->given_gidx : nullptr,
                                   q->pend_gidx.as<u64>(), q->seq);
            HIPCHK(hipGetLastError());
            // (a window may close with no passing event in the push: its expired rows still go out)
            if (M > n_old || (q->d.expired_on && !bounds.empty() && n_old > 0))
                RCHK(sc_rows(q, b, bounds, n_old, M, cv0, clock0, seq0, host_out));
            RCHK(pending_to_front(q, M - new_pend, new_pend));
        } else {
            RCHK(grow_pending(q, new_pend, dst_base));
            launch_compact_pending(s, b->ts, cs, pos_src(q, b), q->ap, e_lo, N, pcb_lo, dst_base,
                                   q->blk_pass.as<int64_t>(), q->pend_pos.as<u32>(), q->pend_ts.as<int64_t>(),
                                   q->pend_vals.as<u64>(), q->pend_cap, q->given ? q->given_gidx : nullptr,
                                   q->pend_gidx.as<u64>(), q->seq);
            HIPCHK(hipGetLastError());
        }
        q->n_pend = new_pend;
    }
    q->seq += N;
    HIPCHK(hipEventRecord(q->ev_push1, s));
    // the push's one final synchronisation: key-table counters and rows per segment
    RCHK(q->h_tail.reserve(16));
    RCHK(q->kt.check_async(s, q->h_tail.as<uint32_t>()));
    SH_TRACE("push final sync");
    SH_TMARK(4);
    HIPCHK(sh_wait_stream(s));
    SH_TMARK(5);
    SH_TRACE("push done");
    RCHK(q->kt.check_result(q->h_tail.as<uint32_t>()));
    RCHK(closed_finish(q, host_out));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, q->ev_push0, q->ev_push1);
    q->stats.push_ms = ms;
    q->stats.events = N;
    q->stats.main_kernel_bytes = q->agg_bytes;
    if (q->xmode) return xout_finish(q, host_out_req, out);
    finish_out(q, host_out, out);
    SH_TMARK(6);
    return SH_OK;
}

// The host-output path stores keys/vals/nulls as [col][n] blocks per segment batch; when several
// run_closed calls append (only one per push today) the layout stays [col][n_rows] because a push
// calls run_closed at most once.
int check_batch_cols(const sh_query* q, const sh_batch* b) {
    if (b->n <= 0) return SH_OK;
    const int nc = q->wide ? q->wide_n_cols : q->d.n_cols;
    const uint64_t used = q->wide ? q->wide_cols_used : q->cols_used;
    for (int c = 0; c < nc; c++)
        if ((used >> c & 1) && !b->cols[c])
            return sh_fail(SH_ERR_INVALID, "batch column " + std::to_string(c) + " is NULL but the query reads it");
    return SH_OK;
}

extern "C" int sh_push(sh_query* q, const sh_batch* b, const sh_out** out) {
    SH_RANGE("sh_push");
    StreamScope _ss(q && q->ctx ? q->ctx->stream : nullptr);
    if (!q || !b || !out) return sh_fail(SH_ERR_INVALID, "sh_push: NULL argument");
    RCHK(check_batch_cols(q, b));
    sh_batch dev;
    RCHK(q->staged.stage(q->ctx->stream, b, q->wide ? q->wide_n_cols : q->d.n_cols, q->d.col_types, &dev));
    return query_push_staged(q, &dev, out);
}

// replaceTimestampWithBatchEndTime's recorded batch starts that later rows can still name: the open
// batch and the one before it (expired rows) — the last 4 entries — and, with an output rate limiter,
// every batch holding a row the limiter carries into a later call (its rep is the oldest it can show)
static int xr_trim(sh_query* q) {
    auto& st = q->xr_starts;
    size_t keep_from = st.size() > 4 ? st.size() - 4 : 0;
    if (keep_from > 0 && q->rate.kind != SH_RATE_NONE && q->rate.nc > 0) {
        std::vector<int64_t> reps((size_t)q->rate.nc);
        HIPCHK(hipMemcpyAsync(reps.data(), q->rate.c_rep.p, reps.size() * 8, hipMemcpyDeviceToHost, q->ctx->stream));
        HIPCHK(hipStreamSynchronize(q->ctx->stream));
        const int64_t lo = *std::min_element(reps.begin(), reps.end());
        auto it = std::upper_bound(st.begin(), st.end(), lo,
                                   [](int64_t v, const std::pair<int64_t, int64_t>& e) { return v < e.first; });
        const size_t cover = it == st.begin() ? 0 : (size_t)(std::prev(it) - st.begin());
        keep_from = std::min(keep_from, cover);
    }
    if (keep_from > 0) st.erase(st.begin(), st.begin() + (ptrdiff_t)keep_from);
    return SH_OK;
}

// replaceTimestampWithBatchEndTime: the timestamp attribute the window wrote into every row's
// representative event — the end time E0 + T (W + 1) of its batch W (ExternalTimeBatchWindowProcessor
// cloneAppend :446-456, findEndTime :440-444) — for sh_query_rep_ts_attr
static int rep_attr_finish(sh_query* q, const sh_out* o, bool host) {
    if (!q->xt_replace) return SH_OK;
    const int64_t n = o->n_rows;
    q->xr_rep.resize((size_t)n);
    q->xr_vals.resize((size_t)n);
    if (q->kind == 1) {
        // partition lanes: every row carries its representative event's batch end (sh_plane_group_kernels)
        if (n) {
            HIPCHK(hipMemcpyAsync(q->xr_vals.data(), plane_out_rep_attr(q), (size_t)n * 8, hipMemcpyDeviceToHost,
                                  q->ctx->stream));
            HIPCHK(hipStreamSynchronize(q->ctx->stream));
        }
        return SH_OK;
    }
    if (n) {
        if (host) {
            std::memcpy(q->xr_rep.data(), o->rep, (size_t)n * 8);
        } else {
            HIPCHK(hipMemcpyAsync(q->xr_rep.data(), o->rep, (size_t)n * 8, hipMemcpyDeviceToHost, q->ctx->stream));
            HIPCHK(hipStreamSynchronize(q->ctx->stream));
        }
    }
    const auto& st = q->xr_starts;
    const int64_t T = q->d.window_param;
    for (int64_t i = 0; i < n; i++) {
        auto it = std::upper_bound(st.begin(), st.end(), q->xr_rep[i],
                                   [](int64_t v, const std::pair<int64_t, int64_t>& e) { return v < e.first; });
        const int64_t W = it == st.begin() ? 0 : std::prev(it)->second;
        q->xr_vals[i] = q->E0 + T * (W + 1);
    }
    return xr_trim(q);
}

extern "C" int sh_query_set_device_flushes(sh_query* q, int32_t on) {
    if (!q) return sh_fail(SH_ERR_INVALID, "sh_query_set_device_flushes: NULL query");
    q->device_flushes = on != 0;
    return SH_OK;
}

extern "C" int sh_query_set_compact_flushes(sh_query* q, int32_t on) {
    if (!q) return sh_fail(SH_ERR_INVALID, "sh_query_set_compact_flushes: NULL query");
    q->compact_flushes = on != 0;
    return SH_OK;
}

extern "C" int sh_query_set_ext_replace_ts(sh_query* q, int32_t on) {
    if (!q) return sh_fail(SH_ERR_INVALID, "sh_query_set_ext_replace_ts: NULL query");
    if (q->d.window != SH_WIN_EXT_TIME_BATCH)
        return sh_fail(SH_ERR_INVALID, "replaceTimestampWithBatchEndTime needs an externalTimeBatch window");
    if (q->seq != 0 || q->n_pend != 0 || q->clock_valid)
        return sh_fail(SH_ERR_INVALID, "sh_query_set_ext_replace_ts: set it before the first push");
    if (!on) { q->xt_replace = false; return SH_OK; }
    // unpartitioned, or partitioned on the sorted partition lanes (lane 3), whose rows carry the batch end
    const bool lanes = q->kind == 1 && q->d.partition_col >= 0 && q->sl && plane_is_sorted_lane(q);
    if ((q->kind != 0 && !lanes) || (q->d.partition_col >= 0 && !lanes) || q->given || q->internal_keys)
        return sh_fail(SH_ERR_UNSUPPORTED,
                       "replaceTimestampWithBatchEndTime runs on externalTimeBatch queries (not sharded)");
    if (lanes && q->rate.kind != SH_RATE_NONE)
        return sh_fail(SH_ERR_UNSUPPORTED,
                       "replaceTimestampWithBatchEndTime of a partitioned query with an output rate limiter");
    for (int i = 0; i < q->d.n_group_by; i++)
        if (q->d.group_by[i] == q->d.ts_col)
            return sh_fail(SH_ERR_UNSUPPORTED, "replaceTimestampWithBatchEndTime with a group-by on the timestamp attribute");
    for (int i = 0; q->wide && i < q->wide->n; i++)
        if (q->wide->col[i] == q->d.ts_col)
            return sh_fail(SH_ERR_UNSUPPORTED, "replaceTimestampWithBatchEndTime with a group-by on the timestamp attribute");
    for (int i = 0; i < q->d.n_aggs; i++)
        if (q->d.aggs[i].fn != SH_AGG_COUNT && q->d.aggs[i].col == q->d.ts_col)
            return sh_fail(SH_ERR_UNSUPPORTED,
                           "replaceTimestampWithBatchEndTime with an aggregator over the timestamp attribute");
    q->xt_replace = true;
    return SH_OK;
}

extern "C" int sh_query_rep_ts_attr(sh_query* q, const int64_t** values, int64_t* n) {
    if (!q || !values || !n) return sh_fail(SH_ERR_INVALID, "sh_query_rep_ts_attr: NULL argument");
    if (!q->xt_replace) return sh_fail(SH_ERR_INVALID, "sh_query_rep_ts_attr: replaceTimestampWithBatchEndTime is not set");
    *values = q->xr_vals.data();
    *n = (int64_t)q->xr_vals.size();
    return SH_OK;
}

static int push_any_core(sh_query* q, const sh_batch* dev, bool host_out, const sh_out** out);
static int push_any(sh_query* q, const sh_batch* dev, bool host_out, const sh_out** out) {
    RCHK(push_any_core(q, dev, host_out, out));
    return rep_attr_finish(q, *out, host_out);
}

static int push_any_core(sh_query* q, const sh_batch* dev, bool host_out, const sh_out** out) {
    if (q->rate.kind != SH_RATE_NONE) {
        const bool sl = q->kind == 1;
        RCHK(sl ? sliding_push(q, dev, false, out) : push_core(q, dev, false, out));
        return rate_apply(q, *out, false, host_out, out);  // (flush layout in host memory, sliding_output)
    }
    if (q->kind == 1) return sliding_push(q, dev, host_out, out);
    return push_core(q, dev, host_out, out);
}

// The open window's pending events aggregated per key without closing it (the aggregation root's
// in-memory store for a retrieval, sh_aggregation_find): device rows in q->out_* ([col][n_rows],
// first-occurrence order); no flush is recorded and the window stays open.
int query_peek(sh_query* q, int64_t* n_rows) {
    *n_rows = 0;
    if (q->n_pend == 0) return SH_OK;
    hipStream_t s = q->ctx->stream;
    q->dev_flush_offsets.assign(1, 0);
    q->dev_flush_clock.clear();
    q->flush_window.clear();
    q->dev_out = sh_out{};
    q->ms_ready = false;
    q->tail.active = false;
    std::vector<Segment> segs{Segment{0, q->n_pend}};
    std::vector<int64_t> clocks{q->clock}, windows{q->W_open};
    RCHK(run_closed(q, segs, clocks, windows, nullptr, false));
    HIPCHK(hipStreamSynchronize(s));
    RCHK(closed_finish(q, false));
    *n_rows = q->dev_out.n_rows;
    q->dev_flush_offsets.assign(1, 0);
    q->dev_flush_clock.clear();
    q->flush_window.clear();
    q->tail.active = false;
    return SH_OK;
}

// a push whose batch is already on the device, with host output (sh_push_staged)
static int wide_push(sh_query* q, const sh_batch* dev, bool host_out, const sh_out** out);
int query_push_staged(sh_query* q, const sh_batch* dev, const sh_out** out) {
    if (q->wide) return wide_push(q, dev, true, out);
    return push_any(q, dev, true, out);
}

extern "C" int sh_push_device(sh_query* q, const sh_batch* b, const sh_out** out) {
    SH_RANGE("sh_push_device");
    StreamScope _ss(q && q->ctx ? q->ctx->stream : nullptr);
    if (!q || !b || !out) return sh_fail(SH_ERR_INVALID, "sh_push_device: NULL argument");
    RCHK(check_batch_cols(q, b));
    if (q->wide) return wide_push(q, b, false, out);
    return push_any(q, b, false, out);
}

// ---- wide group keys: intern before the window, decode after it -----------------------------------
// the call's device output with its rows' group-by values decoded; host output copies every column
static int wide_finish(sh_query* q, bool host_out, const sh_out** out) {
    hipStream_t s = q->ctx->stream;
    const sh_out& o = **out;
    const int64_t n = o.n_rows;
    const int N = q->wide->n;
    RCHK(q->wide_keys.reserve((size_t)std::max<int64_t>(n, 1) * N * 8, false));
    RCHK(q->wide->decode(s, o.keys, n, q->wide_keys.as<int64_t>()));
    sh_out v = o;
    v.n_keys = N;
    v.keys = q->wide_keys.as<int64_t>();
    if (!host_out) {
        q->wide_out = v;
        *out = &q->wide_out;
        return SH_OK;
    }
    OutHost& h = q->wide_host;
    h.reset();
    h.ts.resize(n);
    h.expired.resize(n);
    h.rep.resize(n);
    h.keys.resize((size_t)N * n);
    h.vals.resize((size_t)v.n_vals * n);
    h.nulls.resize((size_t)v.n_vals * n);
    if (n) {
        HIPCHK(hipMemcpyAsync(h.ts.data(), v.ts, n * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(h.expired.data(), v.expired, n, hipMemcpyDeviceToHost, s));
        if (v.rep) HIPCHK(hipMemcpyAsync(h.rep.data(), v.rep, n * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(h.keys.data(), v.keys, (size_t)N * n * 8, hipMemcpyDeviceToHost, s));
        if (v.n_vals) {
            HIPCHK(hipMemcpyAsync(h.vals.data(), v.vals, (size_t)v.n_vals * n * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(h.nulls.data(), v.nulls, (size_t)v.n_vals * n, hipMemcpyDeviceToHost, s));
        }
    }
    HIPCHK(hipStreamSynchronize(s));
    if (v.flush_offsets) {
        h.flush_offsets.assign(v.flush_offsets, v.flush_offsets + v.n_flushes + 1);
        h.flush_clock.assign(v.flush_clock, v.flush_clock + v.n_flushes);
    }
    if (!v.rep) h.rep.assign(n, -1);
    h.view(N, v.n_vals, v.val_types);
    if (!v.flush_offsets) {  // (compact flushes: one row each at its timestamp)
        h.out.n_flushes = v.n_flushes;
        h.out.flush_offsets = nullptr;
        h.out.flush_clock = nullptr;
    }
    *out = &h.out;
    return SH_OK;
}

static int wide_push(sh_query* q, const sh_batch* dev, bool host_out, const sh_out** out) {
    hipStream_t s = q->ctx->stream;
    sh_batch b = *dev;
    const uint32_t* ids = nullptr;
    if (b.n > 0) {
        ColSet full{};
        full.n = q->wide_n_cols;
        // (at the query's load widths: a sharded owner's columns are in their 8-byte raw form)
        for (int c = 0; c < q->wide_n_cols; c++) { full.type[c] = q->load_type[c]; full.ptr[c] = b.cols[c]; }
        RCHK(q->wide->intern(s, full, q->fp, b.n, &ids));
    }
    b.cols[q->wide_n_cols] = ids;
    RCHK(push_any(q, &b, false, out));
    return wide_finish(q, host_out, out);
}

static int advance_core(sh_query* q, int64_t now, bool host_out_req, const sh_out** out) {
    RCHK(small_verify(q, true));
    const bool host_out = host_out_req && !q->xmode;
    q->x_closes.clear();
    q->out.reset();
    q->order_host.clear();
    q->dev_flush_offsets.assign(1, 0);
    q->dev_flush_clock.clear();
    q->flush_window.clear();
    q->dev_out = sh_out{};
    q->ms_ready = false;
    q->tail.active = false;
    // TimestampGeneratorImpl.setCurrentTimestamp only moves the clock forward (:104-122)
    if (q->clock_valid && now < q->clock) {
        if (q->xmode) return xout_finish(q, host_out_req, out);
        finish_out(q, host_out, out);
        return SH_OK;
    }
    q->clock = now;
    q->clock_valid = true;
    if (q->xt_timeout > 0 && q->xt_Lvalid && now >= q->xt_L) {
        // an externalTimeBatch timeout: the open batch, if it holds events not yet sent (:256-275)
        if (q->xt_nnew > 0 && q->n_pend > 0) {
            if (q->xmode) q->x_stamps.assign(1, q->xm);  // (lastCurrentEventTime: the expired rows' stamp)
            std::vector<Segment> segs{Segment{0, q->n_pend}};
            std::vector<int64_t> clocks{now}, windows{q->W_open};
            RCHK(run_closed(q, segs, clocks, windows, nullptr, host_out));
            HIPCHK(hipStreamSynchronize(q->ctx->stream));
            RCHK(closed_finish(q, host_out));
        }
        q->xt_nnew = 0;
        q->xt_L = now + q->xt_timeout;
    }
    if (q->d.window == SH_WIN_TIME_BATCH && q->e0_valid) {
        int64_t W = wfun_host(q, now);
        if (q->xmode && W > q->W_open) q->x_closes.emplace_back(W, now);
        if (W > q->W_open && q->n_pend > 0 && q->d.stream_current) {
            // RESET: the events were emitted as they arrived; with expired output the TIMER chunk
            // carries the window's keys as EXPIRED rows
            if (q->d.expired_on) RCHK(sc_expire_pending(q, now, host_out));
            q->n_pend = 0;
        } else if (W > q->W_open && q->n_pend > 0) {
            std::vector<Segment> segs{Segment{0, q->n_pend}};
            std::vector<int64_t> clocks{now}, windows{q->W_open};
            RCHK(run_closed(q, segs, clocks, windows, nullptr, host_out));
            q->n_pend = 0;
            HIPCHK(hipStreamSynchronize(q->ctx->stream));
            RCHK(closed_finish(q, host_out));
        }
        q->W_open = std::max(q->W_open, W);
    }
    if (q->xmode) return xout_finish(q, host_out_req, out);
    finish_out(q, host_out, out);
    return SH_OK;
}

static int advance_any(sh_query* q, int64_t now, const sh_out** out);
extern "C" int sh_advance_time(sh_query* q, int64_t now, const sh_out** out) {
    SH_RANGE("sh_advance_time");
    StreamScope _ss(q && q->ctx ? q->ctx->stream : nullptr);
    if (!q || !out) return sh_fail(SH_ERR_INVALID, "sh_advance_time: NULL argument");
    RCHK(advance_any(q, now, out));
    return rep_attr_finish(q, *out, true);
}

static int advance_any(sh_query* q, int64_t now, const sh_out** out) {
    if (q->wide) {  // (device output, then the group-by values decoded and copied to the host)
        if (q->kind == 1) {
            RCHK(sliding_advance(q, now, out, false));
            if (q->rate.kind != SH_RATE_NONE) RCHK(rate_apply(q, *out, false, false, out));
        } else {
            RCHK(advance_core(q, now, false, out));
            if (q->rate.kind != SH_RATE_NONE) RCHK(rate_apply(q, *out, false, false, out));
        }
        return wide_finish(q, true, out);
    }
    if (q->kind == 1) {
        if (q->rate.kind == SH_RATE_NONE) return sliding_advance(q, now, out, true);
        RCHK(sliding_advance(q, now, out, false));  // the TIMER chunks' rows reach the limiter too
        return rate_apply(q, *out, false, true, out);
    }
    if (q->rate.kind != SH_RATE_NONE) {
        RCHK(advance_core(q, now, false, out));
        return rate_apply(q, *out, false, true, out);
    }
    return advance_core(q, now, true, out);
}

// device-output variant for the aggregation root (batch windows only)
int sh_advance_time_device(sh_query* q, int64_t now, const sh_out** out) {
    return advance_core(q, now, false, out);
}

extern "C" int sh_query_destroy(sh_query* q) {
    StreamScope _ss(q && q->ctx ? q->ctx->stream : nullptr);
    if (!q) return SH_OK;
    (void)small_verify(q, true);  // the queued appends read the ring and pending buffers freed below
    (void)hipStreamSynchronize(q->ctx->stream);
    (void)hipStreamSynchronize(q->ctx->copy_stream);
    {
        // staging slots were allocated outside stream order (sh_ingest.cpp)
        StreamScope none(nullptr);
        for (auto& sl : q->ing.slot) {
            sl.ts.release();
            for (auto& c : sl.cols) c.release();
        }
    }
    ingest_destroy(q);
    if (q->kind == 1) sliding_destroy(q);
    // device buffers are released by their destructors (stream-ordered on this context)
    q->kt.release();
    q->gkt.release();
    q->pgkt.release();
    delete q->wide;
    if (q->h_info) (void)hipHostFree(q->h_info);
    if (q->small_res) (void)hipHostFree(q->small_res);
    if (q->zc_ring) (void)hipHostFree(q->zc_ring);
    hipEvent_t evs[] = {q->ev_push0, q->ev_push1, q->ev_agg0, q->ev_agg1, q->ev_mid, q->ev_srt0, q->ev_srt1};
    for (auto e : evs) if (e) (void)hipEventDestroy(e);
    delete q;
    return SH_OK;
}

extern "C" int sh_query_stats(sh_query* q, sh_stats* out) {
    if (!q || !out) return sh_fail(SH_ERR_INVALID, "sh_query_stats: NULL argument");
    *out = q->stats;
    return SH_OK;
}

// ---- multisplit: the combined events into P key partitions (stable) -------------------------------
int reserve_ms_counts(sh_query* q, const TileMap& m) {
    const int64_t ncnt = (int64_t)q->P * (m.nblk + 1);  // [tile][partition] + the partition-end row
    RCHK(q->ms_counts.reserve((ncnt + 4) * 4, false));
    return q->ms_tmp.reserve(ms_offsets_tmp_bytes(m.nblk, q->P), false);
}

int run_multisplit(sh_query* q, int64_t hi, const sh_batch* b, bool counted, bool wide) {
    hipStream_t s = q->ctx->stream;
    int P = q->P;
    ColSet cs{};
    cs.n = q->d.n_cols;
    for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->load_type[c]; cs.ptr[c] = b ? b->cols[c] : nullptr; }
    const TileMap m = counted ? make_tile_map(q->n_pend, hi) : make_tile_map(0, hi);
    RCHK(reserve_ms_counts(q, m));  // (the size k_boundaries' counts were written into: no regrowth)
    RCHK(q->part_off.reserve((P + 1) * 8, false));
    int64_t cap = std::max<int64_t>(hi, 1);
    // packed records (local key | low index bits in one word) unless a segment may be too long
    const bool pack = !wide && q->NL <= 1024;
    if (!pack) RCHK(q->rec_pos.reserve(cap * 4, false));
    RCHK(q->rec_idx.reserve(cap * 4, false));
    RCHK(q->rec_vals.reserve(std::max(1, q->ap.n_vcols) * cap * 8, false));
    const PosSrc np = pos_src(q, b);
    // the queued events' tiles (every tile when k_boundaries did not count); also zeroes the total slot
    launch_ms_count(s, m, counted ? m.np_t : m.nblk, q->n_pend, q->pend_pos.as<u32>(), np, P, q->ms_counts.as<u32>());
    // counts (u32: a push holds fewer than 2^32 events) are laid out [p][blk]; one exclusive scan
    // gives every (partition, block) its offset, and partition p starts at offset[p * nblk]
    launch_ms_offsets(s, q->ms_counts.as<u32>(), m.nblk, P, q->ms_tmp.as<int64_t>());
    launch_ms_scatter(s, m, q->n_pend, q->pend_pos.as<u32>(), q->pend_vals.as<u64>(), q->pend_cap, np, cs, q->ap, P,
                      q->logP, q->ms_counts.as<u32>(), pack ? nullptr : q->rec_pos.as<u32>(), q->rec_idx.as<u32>(),
                      q->rec_vals.as<u64>(), cap, pack);
    HIPCHK(hipGetLastError());
    q->ms_ready = true;
    q->rec_packed = pack;
    q->ms_map = m;
    q->rec_cap = cap;
    return SH_OK;
}

// ---- sharded owner (given windows) ------------------------------------------------------------
// expired / all-events output: the global window starts of the push close the owner's batches (its
// own events may start none of them)
static void given_closes(sh_query* q) {
    q->x_closes.clear();
    for (const sh_bound& b : q->gbounds) q->x_closes.emplace_back(b.W, b.clock);
}

// Flush clock of window W: the clock of the first global window start above W in this push (the
// send whose clock fired the timer, Scheduler.sendTimerEvents :171-209).
int64_t given_flush_clock(const sh_query* q, int64_t W) {
    for (const sh_bound& b : q->gbounds)
        if (b.W > W) return b.clock;
    return q->clock;
}

// a sharded owner grouped by a wide key runs the window on the interned ids (device output); its rows get
// their group-by values back (wide_finish) and the merge order comes back from the device
static int given_order_host(sh_query* q, bool host_out, const sh_out* o) {
    if (!q->given || !host_out) return SH_OK;
    const int64_t n = o->n_rows;
    q->order_host.resize(n);
    if (n) {
        HIPCHK(hipMemcpyAsync(q->order_host.data(), q->out_order.p, n * 8, hipMemcpyDeviceToHost, q->ctx->stream));
        HIPCHK(hipStreamSynchronize(q->ctx->stream));
    }
    return SH_OK;
}

int query_push_given(sh_query* q, const sh_batch* b, bool host_out, const sh_out** out) {
    if (q->wide) {
        RCHK(wide_push(q, b, host_out, out));
        return given_order_host(q, host_out, *out);
    }
    return push_core(q, b, host_out, out);
}

// No events reached this owner in the push: close its open window if the global clock moved past it.
int query_close_given(sh_query* q, bool host_out_req, const sh_out** out) {
    const bool host_out = host_out_req && !q->xmode && !q->wide;
    if (q->xmode) given_closes(q);
    q->out.reset();
    q->order_host.clear();
    q->dev_flush_offsets.assign(1, 0);
    q->dev_flush_clock.clear();
    q->flush_window.clear();
    q->dev_out = sh_out{};
    q->stats = sh_stats{};
    q->ms_ready = false;
    q->tail.active = false;
    if (q->given_W_end > q->W_open) {
        if (q->n_pend > 0 && q->d.stream_current) {
            q->n_pend = 0;  // (RESET: the events went out as they arrived; current output only)
        } else if (q->n_pend > 0) {
            std::vector<Segment> segs{Segment{0, q->n_pend}};
            std::vector<int64_t> clocks{given_flush_clock(q, q->W_open)}, windows{q->W_open};
            RCHK(run_closed(q, segs, clocks, windows, nullptr, host_out));
            q->n_pend = 0;
            HIPCHK(hipStreamSynchronize(q->ctx->stream));
            RCHK(closed_finish(q, host_out));
        }
        q->W_open = q->given_W_end;
    }
    if (q->xmode) return xout_finish(q, host_out_req, out);
    finish_out(q, host_out, out);
    if (q->wide) {
        RCHK(wide_finish(q, host_out_req, out));
        return given_order_host(q, host_out_req, *out);
    }
    return SH_OK;
}

int query_advance(sh_query* q, int64_t now, bool host_out, const sh_out** out) {
    if (q->wide) {
        RCHK(advance_core(q, now, false, out));
        RCHK(wide_finish(q, host_out, out));
        return given_order_host(q, host_out, *out);
    }
    return advance_core(q, now, host_out, out);
}
