// sh_shard.cpp — sharded ingest of a timeBatch group-by query across G GPUs (one process per GPU),
// behind sh_shard_* (include/siddhi_hip.h). SURVEY.md §8e: the per-key aggregates are independent,
// so keys are owned by GPU mix64(key) % G; three quantities are global and are reproduced here from
// the all-gathered slice summaries:
//   - the playback clock (InputHandler.send sets it per send, TimestampGeneratorImpl :77-122): the
//     clock carried into slice g is the max over the clock before the push and slices < g;
//   - nextEmitTime, initialised by the first send that reaches the window anywhere in the stream
//     (TimeBatchWindowProcessor.process :266-276) — it is a processor field shared by all keys;
//   - the window of every event and therefore every flush boundary and flush clock
//     (TimeBatchWindowProcessor :278-340 with Scheduler.sendTimerEvents :171-209).
// Output order inside a flush (first occurrence, QuerySelector.processInBatchGroupBy :315-374) is
// global too: each owner reports the global stream index of every row's first event.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <deque>
#include <vector>

#include "sh_agg.h"
#include "sh_internal.h"
#include "sh_runtime.h"
#include "sh_sliding.h"
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

struct sh_shard {
    sh_ctx* ctx = nullptr;
    sh_query_desc d{};
    int rank = 0, world = 1;
    FilterProg fp{};     // the ingest filter (partitioned: AND partition == p0 once p0 is known)
    FilterProg fp_orig{};
    bool partitioned = false, p0_known = false;
    KeyPlan kp{};        // the owner query's group key
    KeyPlan wkp{};       // the key word a record carries (kp without time-bucket components)
    RawPlan rp{};        // the 8-byte raw columns a record carries
    AggPlan ap{};
    int rec_words = 6;   // 4-byte words per record
    int key32 = 0;       // the wire key fits 32 bits
    sh_query* owner = nullptr;
    sh_aggregation* agg = nullptr;  // incremental aggregation fed by the owner (its root), or null
    // global stream state (identical on every rank)
    bool clock_valid = false;
    int64_t clock = 0;
    bool e0_valid = false;
    int64_t E0 = 0;
    int64_t W = 0;        // window of the last event of the stream so far
    int64_t carry = 0;    // lengthBatch: passing events in the open batch (count, :206-243)
    uint64_t seq = 0;     // events of the stream so far (global index of the next event)
    // sliding time(T): PM (max ts over the stream's passing events so far) and sends so far
    bool sliding = false;
    bool sc = false;      // stream.current.event (batch windows): records carry their send's global clock
    int64_t sl_pm = INT64_MIN;
    int64_t send_base = 0, cur_send_base = 0, cur_send_size = 1, cur_n = 0;
    DevBuf sl_clk, sl_pmv;
    // the push in flight (pack -> consume)
    bool packed = false;
    int64_t cur_W_base = 0, cur_W_end = 0;
    int64_t cur_seq = 0;                  // global index of the push's first event
    std::vector<int64_t> cur_off;         // stream offset of every slice in the push
    // packed pushes waiting for their consume, oldest first (two at most: the exchange of push i may
    // run while push i - 1 is consumed)
    struct InFlight {
        int64_t W_base, W_end, seq, send_base, send_size, n;
        std::vector<int64_t> off;
        int64_t clock, E0;
        bool clock_valid, e0_valid;
        int narrow;      // the push's records carry ts as a 32-bit offset from tsbase
        int64_t tsbase;
    };
    // the stream state as of the push being consumed (the ingest may already be a push ahead)
    int64_t cur_clock = 0, cur_E0 = 0;
    bool cur_clock_valid = false, cur_e0_valid = false;
    int cur_narrow = 0;
    int64_t cur_tsbase = 0;
    std::deque<InFlight> fl;
    PinnedBuf h_bgw;                      // pinned copies of the window starts being uploaded
    // ingest scratch
    int64_t slice_n = -1;
    DevBuf blk_pass, blk_tl, blk_first, info, code, counts, tmp, part_off, bounds, tsmm;
    PushInfo* h_info = nullptr;
    int64_t* h_tsmm = nullptr;  // pinned: the slice's ts min / max
    std::vector<sh_bound> my_bounds;
    // owner scratch
    DevBuf u_ts, u_wcol, u_gidx, u_cols[SH_MAX_COLS], u_bg, u_bw;
    ColRoles roles{};
};

static int64_t wfun_g(const sh_shard* s, int64_t clock) {
    if (!s->e0_valid) return 0;
    return clock < s->E0 ? 0 : (clock - s->E0) / s->d.window_param + 1;
}

static int shard_create(sh_ctx* ctx, const sh_query_desc* d, const KeyPlan* kp_override, int32_t rank, int32_t world,
                        sh_shard** out) {
    if (!ctx || !d || !out) return sh_fail(SH_ERR_INVALID, "sh_shard_create: NULL argument");
    if (world < 1 || world > kMaxShards || rank < 0 || rank >= world)
        return sh_fail(SH_ERR_INVALID, "sh_shard_create: need 0 <= rank < world <= 16");
    if (d->window != SH_WIN_TIME_BATCH && d->window != SH_WIN_LENGTH_BATCH && d->window != SH_WIN_TIME)
        return sh_fail(SH_ERR_UNSUPPORTED, "sharded ingest runs timeBatch / lengthBatch / time group-by queries");
    if (d->window == SH_WIN_TIME && (d->partition_col >= 0 || kp_override))
        return sh_fail(SH_ERR_UNSUPPORTED, "partitioned sliding windows are not on the GPU");
    if (d->window == SH_WIN_TIME && d->n_cols + 2 > SH_MAX_COLS)
        return sh_fail(SH_ERR_UNSUPPORTED, "sharded sliding windows carry 2 extra columns: at most 6 stream columns");
    if (d->window == SH_WIN_LENGTH_BATCH && d->partition_col >= 0)
        return sh_fail(SH_ERR_UNSUPPORTED, "partitioned lengthBatch is not on the GPU");
    // stream.current.event: a row per passing event with its key's running values since the batch reset;
    // the owner needs each record's global send clock (its flush clock), carried as one extra raw column
    if (d->stream_current && (d->partition_col >= 0 || d->expired_on || d->window == SH_WIN_TIME))
        return sh_fail(SH_ERR_UNSUPPORTED, "sharded stream.current.event windows: unpartitioned batch windows "
                                           "with current output only");
    if (d->stream_current && d->n_cols + 1 > SH_MAX_COLS)
        return sh_fail(SH_ERR_UNSUPPORTED, "sharded stream.current.event carries 1 extra column: at most 7 stream columns");
    if (d->n_aggs < 1) return sh_fail(SH_ERR_UNSUPPORTED, "sharded queries run aggregations");
    if (d->window == SH_WIN_TIME && (d->expired_on || !d->current_on))
        return sh_fail(SH_ERR_UNSUPPORTED, "sharded sliding windows emit current events (`insert into`)");
    if (d->n_cols <= 0 || d->n_cols > SH_MAX_COLS) return sh_fail(SH_ERR_INVALID, "bad column count");
    // group keys the owner interns (more than two columns, or a 64-bit / floating one beside another): owners by
    // a prefix of the key (one 64-bit column or two 32-bit ones — all of a key's events share it), the other
    // group-by columns travel raw; batch windows with current output (or stream.current.event)
    const bool wide = !kp_override && d->n_group_by > 0 && d->n_group_by <= SH_MAX_GROUP &&
                      WideKeys::needed(d->n_group_by, d->group_by, d->col_types);
    if (wide && (d->window == SH_WIN_TIME || d->partition_col >= 0 || d->expired_on || d->n_cols + 1 >= SH_MAX_COLS))
        return sh_fail(SH_ERR_UNSUPPORTED, "sharded queries with wide group keys: unpartitioned batch windows, current "
                                           "output, at most 6 stream columns");
    sh_shard* s = new sh_shard();
    s->ctx = ctx;
    s->d = *d;
    s->d.filter = nullptr;
    s->rank = rank;
    s->world = world;
    int32_t vt[SH_MAX_AGGS];
    int rc;
    int32_t kg[2] = {d->n_group_by > 0 ? d->group_by[0] : 0, d->n_group_by > 1 ? d->group_by[1] : 0};
    int nkg = d->n_group_by;
    if (wide) {
        const auto w64 = [&](int c) { const int t = d->col_types[c]; return t == SH_T_LONG || t == SH_T_DOUBLE || t == SH_T_FLOAT; };
        nkg = (w64(kg[0]) || w64(kg[1])) ? 1 : 2;
    }
    if ((rc = compile_filter(d->n_filter_ops, d->filter, d->n_cols, d->col_types, s->fp)) ||
        (rc = compile_aggs(d->n_aggs, d->aggs, d->n_cols, d->col_types, s->ap, vt)) ||
        (!kp_override && (rc = compile_keys(nkg, wide ? kg : d->group_by, d->n_cols, d->col_types, s->kp)))) {
        delete s;
        return rc;
    }
    if (kp_override) s->kp = *kp_override;
    s->fp_orig = s->fp;
    s->partitioned = d->partition_col >= 0;
    // wire plan: the key word holds the components that are column values; a time-bucket component
    // (aggregation roots) travels as its raw column and the owner re-derives the bucket. Owners are
    // chosen from the key word alone, so a group key keeps its owner across buckets.
    s->wkp = KeyPlan{};
    s->rp.n = 0;
    for (int j = 0; j < s->ap.n_vcols; j++) s->rp.src[s->rp.n++] = s->ap.vcol_src[j];
    for (int g = 0; g < s->kp.n; g++) {
        if (s->kp.div[g] > 0) {
            bool have = false;
            for (int j = 0; j < s->rp.n; j++) have |= s->rp.src[j] == s->kp.col[g];
            if (!have) s->rp.src[s->rp.n++] = s->kp.col[g];
        } else {
            s->wkp.col[s->wkp.n] = s->kp.col[g];
            s->wkp.type[s->wkp.n] = s->kp.type[g];
            s->wkp.div[s->wkp.n] = 0;
            s->wkp.n++;
        }
    }
    if (wide) {  // (the group-by columns beyond the owner prefix travel raw)
        for (int g = 0; g < d->n_group_by; g++) {
            const int c = d->group_by[g];
            bool have = false;
            for (int j = 0; j < s->wkp.n; j++) have |= s->wkp.col[j] == c;
            for (int j = 0; j < s->rp.n; j++) have |= s->rp.src[j] == c;
            if (!have) s->rp.src[s->rp.n++] = c;
        }
    }
    // sliding: the send's global clock and the global PM travel as two extra raw columns
    // (stream.current.event batch windows: the send's global clock)
    s->sliding = d->window == SH_WIN_TIME;
    s->sc = d->stream_current != 0;
    if (s->sliding) {
        s->rp.src[s->rp.n++] = d->n_cols;
        s->rp.src[s->rp.n++] = d->n_cols + 1;
    } else if (s->sc) {
        s->rp.src[s->rp.n++] = d->n_cols;
    }
    // round-robin owners for one dictionary-id component (dense ids stay dense per owner)
    s->wkp.dense = (s->wkp.n == 1 && s->wkp.type[0] == SH_T_STRID) ? 1 : 0;
    // floating-point keys travel as the 64-bit pattern of the value widened to double
    const bool wide1 = s->wkp.n == 1 && (s->wkp.type[0] == SH_T_LONG || s->wkp.type[0] == SH_T_DOUBLE ||
                                         s->wkp.type[0] == SH_T_FLOAT);
    s->key32 = (s->wkp.n == 0 || (s->wkp.n == 1 && !wide1)) ? 1 : 0;
    if (s->wkp.n == 2 && (s->wkp.type[0] == SH_T_FLOAT || s->wkp.type[1] == SH_T_FLOAT)) {
        delete s;
        return sh_fail(SH_ERR_UNSUPPORTED, "sharded queries: a float group-by column must be the only one");
    }
    s->rec_words = (s->key32 ? 4 : 6) + 2 * s->rp.n;
    // the owner runs the same query over the records it receives: no filter (applied at ingest),
    // 8-byte raw columns, windows given per event
    // key_capacity is the whole stream's; an owner holds about 1/G of the keys (dictionary ids
    // exactly the ids = rank mod G, compacted to id / G)
    sh_query_desc od = *d;
    od.n_filter_ops = 0;
    od.filter = nullptr;
    int64_t cap = d->key_capacity > 0 ? d->key_capacity : (1 << 16);
    od.key_capacity = wide ? cap : s->kp.dense ? (cap + world - 1) / world : cap / world + cap / (4 * world) + 64;
    if ((rc = kp_override ? sh_query_create_internal(ctx, &od, *kp_override, &s->owner)
                          : sh_query_create(ctx, &od, &s->owner))) {
        delete s;
        return rc;
    }
    sh_query* q = s->owner;
    q->given = true;
    if (q->kp.dense && !q->wide) {  // (a wide owner's ids are its own interned ones)
        q->kt.dmul = (uint32_t)world;
        q->kt.dadd = (uint32_t)rank;
    }
    s->roles.n = d->n_cols + (s->sliding ? 2 : s->sc ? 1 : 0);
    for (int c = 0; c < s->roles.n; c++) {
        int t = c < d->n_cols ? d->col_types[c] : SH_T_LONG;
        if (c < d->n_cols) q->load_type[c] = (t == SH_T_FLOAT || t == SH_T_DOUBLE) ? SH_T_DOUBLE : SH_T_LONG;
        s->roles.role[c] = -1;
        for (int g = 0; g < s->wkp.n; g++) if (s->wkp.col[g] == c) s->roles.role[c] = 16 + g;
        for (int j = 0; j < s->rp.n; j++) if (s->rp.src[j] == c) s->roles.role[c] = j;
    }
    if (hipHostMalloc((void**)&s->h_info, sizeof(PushInfo), hipHostMallocDefault) != hipSuccess) {
        sh_query_destroy(s->owner);
        delete s;
        return sh_fail(SH_ERR_OOM, "pinned alloc failed");
    }
    if ((rc = s->info.reserve(sizeof(PushInfo), false))) { sh_shard_destroy(s); return rc; }
    *out = s;
    return SH_OK;
}

extern "C" int sh_shard_create(sh_ctx* ctx, const sh_query_desc* d, int32_t rank, int32_t world, sh_shard** out) {
    StreamScope _ss(ctx ? ctx->stream : nullptr);
    return shard_create(ctx, d, nullptr, rank, world, out);
}

// the root query of a sharded incremental aggregation (sh_aggregation.cpp)
int shard_create_root(sh_ctx* ctx, const sh_query_desc* d, const KeyPlan& kp, int32_t rank, int32_t world,
                      sh_shard** out, sh_query** owner) {
    int rc = shard_create(ctx, d, &kp, rank, world, out);
    if (rc) return rc;
    *owner = (*out)->owner;
    return SH_OK;
}

void shard_attach_aggregation(sh_shard* s, sh_aggregation* a) { s->agg = a; }

extern "C" int sh_shard_destroy(sh_shard* s) {
    StreamScope _ss(s && s->ctx ? s->ctx->stream : nullptr);
    if (!s) return SH_OK;
    (void)hipStreamSynchronize(s->ctx->stream);
    if (s->agg) agg_release_sharded(s->agg);
    if (s->owner) sh_query_destroy(s->owner);
    DevBuf* bufs[] = {&s->blk_pass, &s->blk_tl, &s->blk_first, &s->info, &s->code, &s->counts, &s->tmp,
                      &s->part_off, &s->bounds, &s->u_ts, &s->u_wcol, &s->u_gidx, &s->u_bg, &s->u_bw,
                      &s->sl_clk, &s->sl_pmv, &s->tsmm};
    for (DevBuf* b : bufs) b->release();
    for (auto& c : s->u_cols) c.release();
    if (s->h_info) (void)hipHostFree(s->h_info);
    if (s->h_tsmm) (void)hipHostFree(s->h_tsmm);
    delete s;
    return SH_OK;
}

extern "C" int sh_shard_record_bytes(sh_shard* s, int64_t* out) {
    if (!s || !out) return sh_fail(SH_ERR_INVALID, "sh_shard_record_bytes: NULL argument");
    *out = 4 * (int64_t)s->rec_words;
    return SH_OK;
}

static ColSet colset(const sh_shard* s, const sh_batch* b) {
    ColSet cs{};
    cs.n = s->d.n_cols;
    for (int c = 0; c < s->d.n_cols; c++) { cs.type[c] = s->d.col_types[c]; cs.ptr[c] = b->cols[c]; }
    return cs;
}

// the slice's timestamp range (every event: a superset of the passing ones), read with the summary
static int slice_ts_range(sh_shard* s, const sh_batch* b, sh_slice_summary* out) {
    (void)out;
    RCHK(s->tsmm.reserve(minmax_scratch_bytes(), false));
    if (!s->h_tsmm) {
        if (hipHostMalloc((void**)&s->h_tsmm, 16, hipHostMallocDefault) != hipSuccess)
            return sh_fail(SH_ERR_OOM, "pinned alloc failed");
    }
    launch_minmax_i64(s->ctx->stream, b->ts, b->n, s->tsmm.as<int64_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(s->h_tsmm, s->tsmm.p, 16, hipMemcpyDeviceToHost, s->ctx->stream));
    return SH_OK;
}

// Phase 1: pass count, send clocks and the first passing send of the slice (k_blockagg + k_scan_blocks).
extern "C" int sh_shard_summarize(sh_shard* s, const sh_batch* b, sh_slice_summary* out) {
    SH_RANGE("sh_shard_summarize");
    StreamScope _ss(s && s->ctx ? s->ctx->stream : nullptr);
    if (!s || !b || !out) return sh_fail(SH_ERR_INVALID, "sh_shard_summarize: NULL argument");
    if (b->n < 0) return sh_fail(SH_ERR_INVALID, "negative slice size");
    if (b->n > 0 && (b->send_size < 1 || !b->ts))
        return sh_fail(SH_ERR_UNSUPPORTED, "sharded slices need send_size >= 1 (slices cut at send boundaries)");
    *out = sh_slice_summary{b->n, 0, INT64_MIN, INT64_MIN, 0, INT64_MAX, INT64_MIN};
    s->slice_n = b->n;
    if (b->n == 0) return SH_OK;
    hipStream_t st = s->ctx->stream;
    int nblk = (int)((b->n + kTile - 1) / kTile);
    RCHK(s->blk_pass.reserve(nblk * 8, false));
    RCHK(s->blk_tl.reserve(nblk * 8, false));
    RCHK(s->blk_first.reserve(scan_blocks_first_bytes(nblk), false));
    if (s->sliding) {
        // pass count, max send-last ts, max passing ts (PM) of the slice; blk_first holds the PM prefix
        WinParams wp{};
        wp.kind = SH_WIN_TIME;
        wp.N = b->n;
        wp.send_size = b->send_size;
        launch_sl_prefix(st, b->ts, colset(s, b), s->fp, wp, s->blk_pass.as<int64_t>(), s->blk_tl.as<int64_t>(),
                         s->blk_first.as<int64_t>(), nblk, s->info.as<SlInfo>());
        RCHK(slice_ts_range(s, b, out));
        SlInfo si{};
        HIPCHK(hipMemcpyAsync(s->h_info, s->info.p, sizeof(SlInfo), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        out->ts_min = s->h_tsmm[0];
        out->ts_max = s->h_tsmm[1];
        si = *(const SlInfo*)s->h_info;
        out->n_pass = si.total_pass;
        out->max_tl = si.max_tl;
        out->first_key = si.max_pm;
        return SH_OK;
    }
    launch_blockagg(st, b->ts, colset(s, b), s->fp, b->n, b->send_size, s->blk_pass.as<int64_t>(),
                    s->blk_tl.as<int64_t>(), s->blk_first.as<int64_t>(), nblk);
    WinParams wp{};
    wp.kind = SH_WIN_LENGTH_BATCH;  // no nextEmitTime initialisation: that is a global decision
    wp.N = b->n;
    wp.send_size = b->send_size;
    wp.want_first_clk = 1;
    wp.pcol1 = (s->partitioned && !s->p0_known) ? s->d.partition_col + 1 : 0;
    launch_scan_blocks(st, s->blk_pass.as<int64_t>(), s->blk_tl.as<int64_t>(), s->blk_first.as<int64_t>(), nblk, b->ts,
                       wp, s->info.as<PushInfo>(), nullptr, colset(s, b));
    RCHK(slice_ts_range(s, b, out));
    HIPCHK(hipMemcpyAsync(s->h_info, s->info.p, sizeof(PushInfo), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    out->ts_min = s->h_tsmm[0];
    out->ts_max = s->h_tsmm[1];
    out->n_pass = s->h_info->total_pass;
    out->max_tl = s->h_info->max_tl;
    out->first_clock = s->h_info->first_pass == INT64_MAX ? INT64_MIN : s->h_info->first_clk;
    // partition key of the slice's first passing event (PartitionStreamReceiver :176-272), read by
    // k_scan_blocks in the same pass
    out->first_key = (wp.pcol1 > 0 && s->h_info->first_pass != INT64_MAX) ? s->h_info->first_key : 0;
    return SH_OK;
}

static sh_shard::InFlight Shard_InFlight(const sh_shard* s) {
    return sh_shard::InFlight{s->cur_W_base, s->cur_W_end, s->cur_seq, s->cur_send_base, s->cur_send_size, s->cur_n,
                              s->cur_off, s->clock, s->E0, s->clock_valid, s->e0_valid, s->cur_narrow, s->cur_tsbase};
}

// The record format of a push, from the G summaries (the same on every rank): with a 32-bit wire key
// and all of the push's timestamps within 2^32 of its minimum, ts travels as a 32-bit offset from that
// minimum (C2: 20 bytes per record instead of 24 — the xGMI bytes of the all-to-all).
static void push_format(sh_shard* s, const sh_slice_summary* all) {
    int64_t lo = INT64_MAX, hi = INT64_MIN;
    for (int r = 0; r < s->world; r++) {
        if (all[r].n <= 0) continue;
        lo = std::min(lo, all[r].ts_min);
        hi = std::max(hi, all[r].ts_max);
    }
    s->cur_narrow = s->key32 && lo <= hi && (uint64_t)hi - (uint64_t)lo <= 0xFFFFFFFFull;
    s->cur_tsbase = s->cur_narrow ? lo : 0;
}

// Phase 2 of a sliding time(T) query: every passing event gets its send's global clock and the global
// PM (max ts over the passing events of the stream up to it: the slices before contribute their
// summaries' PM, carried in sh_slice_summary.first_key) and goes to its key's owner.
static int pack_sliding(sh_shard* s, const sh_slice_summary* all, const sh_batch* b, void* send_buf,
                        int64_t* send_bytes, const sh_bound** bounds, int64_t* n_bounds,
                        const std::vector<int64_t>& cin, const std::vector<int64_t>& off, int64_t clock_end,
                        int64_t n_total) {
    const int G = s->world;
    push_format(s, all);
    const int RW = s->rec_words - s->cur_narrow;
    const int64_t RB = 4 * (int64_t)RW;
    int64_t pm_in = s->sl_pm, pm_end = s->sl_pm, sends = 0;
    const int64_t ss = std::max<int64_t>(1, b->send_size);
    for (int r = 0; r < G; r++) {
        if (r < s->rank) pm_in = std::max(pm_in, all[r].first_key);
        pm_end = std::max(pm_end, all[r].first_key);
        sends += (all[r].n + ss - 1) / ss;
    }
    s->my_bounds.clear();
    for (int r = 0; r < G; r++) send_bytes[r] = 0;
    const int64_t N = b->n;
    if (N > 0) {
        hipStream_t st = s->ctx->stream;
        int nblk = (int)((N + kTile - 1) / kTile);
        int64_t ncnt = (int64_t)G * nblk;
        RCHK(s->code.reserve(N * 4, false));
        RCHK(s->counts.reserve((ncnt + 1) * 8, false));
        RCHK(s->tmp.reserve(((ncnt + kTile) / kTile + 16) * 8, false));
        RCHK(s->part_off.reserve((G + 1) * 8, false));
        RCHK(s->sl_clk.reserve(N * 8, false));
        RCHK(s->sl_pmv.reserve(N * 8, false));
        WinParams wp{};
        wp.kind = SH_WIN_TIME;
        wp.clock_valid = cin[s->rank] != INT64_MIN;
        wp.clock0 = cin[s->rank];
        wp.N = N;
        wp.send_size = b->send_size;
        launch_shard_sl_assign(st, b->ts, colset(s, b), s->fp, wp, s->blk_tl.as<int64_t>(), s->blk_first.as<int64_t>(),
                               pm_in, s->wkp, G, nblk, s->code.as<u32>(), s->counts.as<int64_t>(),
                               s->sl_clk.as<int64_t>(), s->sl_pmv.as<int64_t>());
        HIPCHK(hipMemsetAsync(s->counts.as<int64_t>() + ncnt, 0, 8, st));
        launch_scan_sum_large(st, s->counts.as<int64_t>(), ncnt + 1, s->tmp.as<int64_t>());
        ColSet cs = colset(s, b);
        cs.ptr[cs.n] = s->sl_clk.p; cs.type[cs.n] = SH_T_LONG;
        cs.ptr[cs.n + 1] = s->sl_pmv.p; cs.type[cs.n + 1] = SH_T_LONG;
        cs.n += 2;
        launch_shard_pack(st, cs, b->ts, s->code.as<u32>(), s->wkp, s->rp, G, N, nblk, s->counts.as<int64_t>(),
                          (unsigned char*)send_buf, RW, s->key32, s->cur_narrow, s->cur_tsbase);
        launch_part_off(st, s->counts.as<int64_t>(), nblk, G, s->part_off.as<int64_t>());
        HIPCHK(hipGetLastError());
        std::vector<int64_t> po(G + 1);
        HIPCHK(hipMemcpyAsync(po.data(), s->part_off.p, (G + 1) * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (int r = 0; r < G; r++) send_bytes[r] = (po[r + 1] - po[r]) * RB;
    }
    s->cur_seq = (int64_t)s->seq;
    s->cur_off = off;
    s->cur_send_base = s->send_base;
    s->cur_send_size = ss;
    s->cur_n = n_total;
    if (clock_end != INT64_MIN) {
        s->clock = clock_end;
        s->clock_valid = true;
    }
    s->sl_pm = pm_end;
    s->send_base += sends;
    s->seq += (uint64_t)n_total;
    s->fl.push_back(Shard_InFlight(s));
    s->packed = true;
    s->slice_n = -1;
    *bounds = s->my_bounds.data();
    *n_bounds = 0;
    return SH_OK;
}

// Phase 2: global clock / nextEmitTime / windows from the G summaries, then the per-owner records.
extern "C" int sh_shard_pack(sh_shard* s, const sh_slice_summary* all, const sh_batch* b, void* send_buf,
                             int64_t send_cap, int64_t* send_bytes, const sh_bound** bounds, int64_t* n_bounds) {
    SH_RANGE("sh_shard_pack");
    StreamScope _ss(s && s->ctx ? s->ctx->stream : nullptr);
    if (!s || !all || !b || !send_bytes || !bounds || !n_bounds)
        return sh_fail(SH_ERR_INVALID, "sh_shard_pack: NULL argument");
    if (s->slice_n != b->n || all[s->rank].n != b->n)
        return sh_fail(SH_ERR_STATE, "sh_shard_pack: call sh_shard_summarize on the same slice first");
    if (s->fl.size() >= 2) return sh_fail(SH_ERR_STATE, "sh_shard_pack: two packed pushes already wait for consume");
    // slices are cut at send boundaries: every slice but the last holds whole sends, otherwise one
    // send's events would get different clocks / send numbers on two ranks (InputHandler.send :85-96)
    if (b->send_size > 0)
        for (int r = 0; r + 1 < s->world; r++)
            if (all[r].n % b->send_size != 0)
                return sh_fail(SH_ERR_INVALID, "sh_shard_pack: slice " + std::to_string(r) +
                                                   " is not a whole number of sends (cut slices at send boundaries)");
    const int G = s->world;
    const int64_t RB = 4 * (int64_t)s->rec_words;
    if (b->n > 0 && (!send_buf || send_cap < b->n * RB))
        return sh_fail(SH_ERR_INVALID, "sh_shard_pack: send buffer smaller than slice.n * record_bytes");
    // clock carried into every slice; stream offset of every slice
    std::vector<int64_t> cin(G), off(G);
    int64_t c = s->clock_valid ? s->clock : INT64_MIN, o = 0;
    for (int r = 0; r < G; r++) {
        cin[r] = c;
        off[r] = o;
        c = std::max(c, all[r].max_tl);
        o += all[r].n;
    }
    const int64_t clock_end = c, n_total = o;
    if (s->seq + (uint64_t)n_total >= (1ull << 40)) return sh_fail(SH_ERR_UNSUPPORTED, "stream longer than 2^40 events");
    push_format(s, all);
    const int RW = s->rec_words - s->cur_narrow;  // this push's record words
    if (s->sliding) return pack_sliding(s, all, b, send_buf, send_bytes, bounds, n_bounds, cin, off, clock_end, n_total);
    // R12: the partition of the stream's first passing event armed the shared timer and is the only
    // one that ever flushes; from here on the ingest keeps only its events (the owner needs no filter)
    if (s->partitioned && !s->p0_known) {
        for (int r = 0; r < G; r++) {
            if (all[r].n_pass == 0) continue;
            const int pc = s->d.partition_col;
            RCHK(partition_filter(s->fp_orig, pc, s->d.col_types[pc], all[r].first_key, &s->fp));
            s->p0_known = true;
            s->owner->p0 = all[r].first_key;
            s->owner->p0_known = true;
            break;
        }
    }
    const bool lb = s->d.window == SH_WIN_LENGTH_BATCH;
    // passing events of the slices before each slice (lengthBatch: the global batch index)
    std::vector<int64_t> poff(G);
    int64_t total_pass = 0;
    for (int r = 0; r < G; r++) { poff[r] = total_pass; total_pass += all[r].n_pass; }
    // nextEmitTime: initialised by the first send that reaches the window (TimeBatch :266-276, 342-347)
    if (!lb && !s->e0_valid) {
        for (int r = 0; r < G; r++) {
            if (all[r].n_pass == 0) continue;
            int64_t ck = std::max(cin[r], all[r].first_clock);
            const int64_t T = s->d.window_param;
            s->E0 = s->d.has_start_time ? ck + (T - (ck - s->d.start_time) % T) : ck + T;
            s->e0_valid = true;
            break;
        }
    }
    const int64_t W_start = s->W;
    // lengthBatch: a batch is complete (and flushed in the send of its L-th event) once L passing
    // events reached it, so every window below (carry + passes) / L closes in this push
    const int64_t W_end = lb ? W_start + (s->carry + total_pass) / s->d.window_param
                             : std::max(W_start, wfun_g(s, clock_end));
    if (W_end - W_start >= (1 << 23)) return sh_fail(SH_ERR_UNSUPPORTED, "more than 8M windows in one push");
    s->cur_W_base = W_start;
    s->cur_W_end = W_end;
    s->cur_seq = (int64_t)s->seq;
    s->cur_off = off;
    s->cur_send_size = std::max<int64_t>(1, b->send_size);  // (stream.current.event rows are per send)
    s->cur_n = n_total;
    s->my_bounds.clear();
    for (int r = 0; r < G; r++) send_bytes[r] = 0;
    const int64_t N = b->n;
    if (N > 0) {
        hipStream_t st = s->ctx->stream;
        int nblk = (int)((N + kTile - 1) / kTile);
        int64_t ncnt = (int64_t)G * nblk;
        RCHK(s->code.reserve(N * 4, false));
        RCHK(s->counts.reserve((ncnt + 1) * 8, false));
        RCHK(s->tmp.reserve(((ncnt + kTile) / kTile + 16) * 8, false));
        RCHK(s->part_off.reserve((G + 1) * 8, false));
        int max_bounds = (int)std::min<int64_t>(N + 1, 1 << 22);
        RCHK(s->bounds.reserve((size_t)max_bounds * sizeof(Bound), false));
        HIPCHK(hipMemsetAsync(s->info.p, 0, sizeof(PushInfo), st));
        WinParams wp{};
        wp.kind = lb ? SH_WIN_LENGTH_BATCH : SH_WIN_TIME_BATCH;
        wp.L = s->d.window_param;
        wp.n_pend = s->carry + poff[s->rank];
        wp.e0_valid = s->e0_valid;
        wp.E0 = s->E0;
        wp.T = s->d.window_param;
        wp.clock_valid = cin[s->rank] != INT64_MIN;
        wp.clock0 = cin[s->rank];
        // window of the event before this slice: the last event of the slices before it
        wp.W_open = (off[s->rank] > 0 && wp.clock_valid) ? std::max(W_start, wfun_g(s, cin[s->rank])) : W_start;
        wp.W_base = W_start;
        wp.N = N;
        wp.send_size = b->send_size;
        PushInfo* info = s->info.as<PushInfo>();
        if (s->sc) RCHK(s->sl_clk.reserve(N * 8, false));
        launch_shard_assign(st, b->ts, colset(s, b), s->fp, wp, s->blk_tl.as<int64_t>(), s->blk_pass.as<int64_t>(),
                            info, s->wkp, G, nblk,
                            s->code.as<u32>(), s->counts.as<int64_t>(), s->bounds.as<Bound>(), max_bounds,
                            &info->n_bounds, s->sc ? s->sl_clk.as<int64_t>() : nullptr);
        HIPCHK(hipMemsetAsync(s->counts.as<int64_t>() + ncnt, 0, 8, st));
        launch_scan_sum_large(st, s->counts.as<int64_t>(), ncnt + 1, s->tmp.as<int64_t>());
        ColSet pcs = colset(s, b);
        if (s->sc) {
            pcs.ptr[pcs.n] = s->sl_clk.p;
            pcs.type[pcs.n] = SH_T_LONG;
            pcs.n += 1;
        }
        launch_shard_pack(st, pcs, b->ts, s->code.as<u32>(), s->wkp, s->rp, G, N, nblk,
                          s->counts.as<int64_t>(), (unsigned char*)send_buf, RW, s->key32, s->cur_narrow,
                          s->cur_tsbase);
        launch_part_off(st, s->counts.as<int64_t>(), nblk, G, s->part_off.as<int64_t>());
        HIPCHK(hipGetLastError());
        std::vector<int64_t> po(G + 1);
        HIPCHK(hipMemcpyAsync(po.data(), s->part_off.p, (G + 1) * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipMemcpyAsync(s->h_info, s->info.p, sizeof(PushInfo), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        int nb = s->h_info->n_bounds;
        if (nb > max_bounds) return sh_fail(SH_ERR_UNSUPPORTED, "more than 4M windows started in one slice");
        std::vector<Bound> bd(nb);
        if (nb) {
            HIPCHK(hipMemcpyAsync(bd.data(), s->bounds.p, nb * sizeof(Bound), hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
        }
        for (const Bound& x : bd)
            s->my_bounds.push_back(sh_bound{x.W, x.clock, (int64_t)s->seq + off[s->rank] + x.idx, 0});
        std::sort(s->my_bounds.begin(), s->my_bounds.end(),
                  [](const sh_bound& a, const sh_bound& c2) { return a.gidx < c2.gidx; });
        for (int r = 0; r < G; r++) send_bytes[r] = (po[r + 1] - po[r]) * 4 * (int64_t)RW;
    }
    // commit the global stream state (every rank computes the same values)
    if (clock_end != INT64_MIN) {
        s->clock = clock_end;
        s->clock_valid = true;
    }
    s->W = W_end;
    if (lb) s->carry = (s->carry + total_pass) % s->d.window_param;
    s->seq += (uint64_t)n_total;
    s->fl.push_back(Shard_InFlight(s));
    s->packed = true;
    s->slice_n = -1;
    *bounds = s->my_bounds.data();
    *n_bounds = (int64_t)s->my_bounds.size();
    return SH_OK;
}

static void sync_owner(sh_shard* s) {
    sh_query* q = s->owner;
    q->clock = s->cur_clock;
    q->clock_valid = s->cur_clock_valid;
    q->E0 = s->cur_E0;
    q->e0_valid = s->cur_e0_valid;
}

static void set_order(sh_shard* s, bool host_out, const int64_t** order) {
    if (!order) return;
    sh_query* q = s->owner;
    *order = host_out ? q->order_host.data() : q->xmode ? q->x_order.as<int64_t>() : q->out_order.as<int64_t>();
}

// The window every flush of the last consume / advance closes (batch windows; none for sliding ones):
// the owners' flushes of one global flush carry the same (clock, window), whatever rows they hold.
extern "C" int sh_shard_flush_windows(sh_shard* s, const int64_t** windows, int64_t* n) {
    if (!s || !windows || !n) return sh_fail(SH_ERR_INVALID, "sh_shard_flush_windows: NULL argument");
    sh_query* q = s->owner;
    *n = s->sliding ? 0 : (int64_t)q->flush_window.size();
    *windows = q->flush_window.data();
    return SH_OK;
}

// Phase 3 of a sliding query: unpack, then the owner's per-key replay with the records' global clock,
// PM and stream index (one flush per global send that touched the owner's keys).
static int consume_sliding(sh_shard* s, const void* recv_buf, const int64_t* recv_bytes, int64_t M, bool host_out,
                           const sh_out** out, const int64_t** order) {
    sh_query* q = s->owner;
    hipStream_t st = s->ctx->stream;
    const int64_t cap = std::max<int64_t>(M, 1);
    RCHK(s->u_ts.reserve(cap * 8, false));
    RCHK(s->u_wcol.reserve(cap * 4, false));
    RCHK(s->u_gidx.reserve(cap * 8, false));
    ColPtrs cp{};
    const void* cols[SH_MAX_COLS] = {};
    for (int c = 0; c < s->roles.n; c++) {
        if (s->roles.role[c] < 0) continue;
        RCHK(s->u_cols[c].reserve(cap * 8, false));
        cp.p[c] = s->u_cols[c].as<u64>();
        cols[c] = cp.p[c];
    }
    ShardSrc src{};
    src.G = s->world;
    src.key32 = s->key32;
    src.narrow = s->cur_narrow;
    src.tsbase = s->cur_tsbase;
    int64_t acc = 0;
    const int RW = s->rec_words - s->cur_narrow;
    const int64_t RB = 4 * (int64_t)RW;
    for (int g = 0; g < s->world; g++) {
        src.start[g] = acc;
        acc += recv_bytes[g] / RB;
        src.gbase[g] = s->cur_seq + s->cur_off[g];
    }
    src.start[s->world] = acc;
    if (M > 0)
        launch_shard_unpack(st, (const unsigned char*)recv_buf, M, RW, s->wkp, s->roles, src, nullptr,
                            nullptr, 0, 0, s->u_ts.as<int64_t>(), cp, s->u_wcol.as<int>(), s->u_gidx.as<u64>());
    HIPCHK(hipGetLastError());
    const int nc = s->d.n_cols;
    RCHK(sliding_push_given(q, M, s->u_ts.as<int64_t>(), cols, s->u_cols[nc].as<int64_t>(),
                            s->u_cols[nc + 1].as<int64_t>(), (const uint64_t*)s->u_gidx.p, s->cur_seq,
                            s->cur_send_size, s->cur_send_base, host_out, out, s->cur_n));
    q->clock = s->cur_clock;
    q->clock_valid = s->cur_clock_valid;
    set_order(s, host_out, order);
    return SH_OK;
}

// Phase 3: the owner aggregates the records of its keys (event order preserved: sources are
// concatenated in rank order and every source run is in stream order).
extern "C" int sh_shard_consume(sh_shard* s, const void* recv_buf, const int64_t* recv_bytes, const sh_bound* all_bounds,
                                int64_t n_all_bounds, int32_t host_out, const sh_out** out, const int64_t** order) {
    SH_RANGE("sh_shard_consume");
    StreamScope _ss(s && s->ctx ? s->ctx->stream : nullptr);
    if (!s || !recv_bytes || !out || (n_all_bounds > 0 && !all_bounds))
        return sh_fail(SH_ERR_INVALID, "sh_shard_consume: NULL argument");
    if (s->fl.empty()) return sh_fail(SH_ERR_STATE, "sh_shard_consume: no packed push in flight");
    {
        const sh_shard::InFlight f = s->fl.front();
        s->fl.pop_front();
        s->cur_W_base = f.W_base;
        s->cur_W_end = f.W_end;
        s->cur_seq = f.seq;
        s->cur_send_base = f.send_base;
        s->cur_send_size = f.send_size;
        s->cur_n = f.n;
        s->cur_off = f.off;
        s->cur_clock = f.clock;
        s->cur_clock_valid = f.clock_valid;
        s->cur_E0 = f.E0;
        s->cur_e0_valid = f.e0_valid;
        s->cur_narrow = f.narrow;
        s->cur_tsbase = f.tsbase;
    }
    s->packed = !s->fl.empty();
    if (s->agg) host_out = 0;  // the root's flushes feed the roll-up levels on the device
    const int RW = s->rec_words - s->cur_narrow;  // the consumed push's record words
    const int64_t RB = 4 * (int64_t)RW;
    int64_t bytes = 0;
    for (int r = 0; r < s->world; r++) {
        if (recv_bytes[r] < 0 || recv_bytes[r] % RB) return sh_fail(SH_ERR_INVALID, "received block not a whole number of records");
        bytes += recv_bytes[r];
    }
    const int64_t M = bytes / RB;
    if (M > 0 && !recv_buf) return sh_fail(SH_ERR_INVALID, "sh_shard_consume: NULL receive buffer");
    sh_query* q = s->owner;
    if (s->sliding) return consume_sliding(s, recv_buf, recv_bytes, M, host_out != 0, out, order);
    q->gbounds.assign(all_bounds, all_bounds + n_all_bounds);
    std::sort(q->gbounds.begin(), q->gbounds.end(), [](const sh_bound& a, const sh_bound& c) { return a.gidx < c.gidx; });
    q->given_W_base = s->cur_W_base;
    q->given_W_end = s->cur_W_end;
    sync_owner(s);
    if (M == 0) {
        RCHK(query_close_given(q, host_out != 0, out));
        if (s->agg) RCHK(agg_after_root(s->agg, *out));
        set_order(s, host_out != 0, order);
        return SH_OK;
    }
    hipStream_t st = s->ctx->stream;
    RCHK(s->u_ts.reserve(M * 8, false));
    RCHK(s->u_wcol.reserve(M * 4, false));
    RCHK(s->u_gidx.reserve(M * 8, false));
    ColPtrs cp{};
    sh_batch b{};
    b.n = M;
    b.send_size = 1;
    for (int c = 0; c < s->roles.n; c++) {
        if (s->roles.role[c] < 0) continue;
        RCHK(s->u_cols[c].reserve(M * 8, false));
        cp.p[c] = s->u_cols[c].as<u64>();
        if (c < s->d.n_cols) b.cols[c] = cp.p[c];
    }
    // the global window starts, sorted by stream index, for the per-record window lookup
    const int nb = (int)q->gbounds.size();
    RCHK(s->h_bgw.reserve((size_t)std::max(1, nb) * 16));
    int64_t* bg = s->h_bgw.as<int64_t>();
    int64_t* bw = bg + std::max(1, nb);
    for (int i = 0; i < nb; i++) { bg[i] = q->gbounds[i].gidx; bw[i] = q->gbounds[i].W; }
    RCHK(s->u_bg.reserve(std::max(1, nb) * 8, false));
    RCHK(s->u_bw.reserve(std::max(1, nb) * 8, false));
    if (nb) {
        HIPCHK(hipMemcpyAsync(s->u_bg.p, bg, nb * 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(s->u_bw.p, bw, nb * 8, hipMemcpyHostToDevice, st));
    }
    ShardSrc src{};
    src.G = s->world;
    src.key32 = s->key32;
    src.narrow = s->cur_narrow;
    src.tsbase = s->cur_tsbase;
    int64_t acc = 0;
    for (int g = 0; g < s->world; g++) {
        src.start[g] = acc;
        acc += recv_bytes[g] / RB;
        src.gbase[g] = s->cur_seq + s->cur_off[g];
    }
    src.start[s->world] = acc;
    launch_shard_unpack(st, (const unsigned char*)recv_buf, M, RW, s->wkp, s->roles, src,
                        s->u_bg.as<int64_t>(), s->u_bw.as<int64_t>(), nb, s->cur_W_base, s->u_ts.as<int64_t>(), cp,
                        s->u_wcol.as<int>(), s->u_gidx.as<u64>());
    HIPCHK(hipGetLastError());
    b.ts = s->u_ts.as<int64_t>();
    q->given_wcol = s->u_wcol.as<int>();
    q->given_gidx = s->u_gidx.as<u64>();
    q->given_clk = s->sc ? s->u_cols[s->d.n_cols].as<int64_t>() : nullptr;
    q->given_seq0 = s->cur_seq;
    q->given_ss = s->cur_send_size;
    int rc = s->agg ? agg_reserve_root(s->agg, &b) : SH_OK;
    if (!rc) rc = query_push_given(q, &b, host_out != 0, out);
    q->given_wcol = nullptr;
    q->given_gidx = nullptr;
    q->given_clk = nullptr;
    if (rc) return rc;
    sync_owner(s);
    if (s->agg) RCHK(agg_after_root(s->agg, *out));
    set_order(s, host_out != 0, order);
    return SH_OK;
}

extern "C" int sh_shard_advance_time(sh_shard* s, int64_t now, int32_t host_out, const sh_out** out,
                                     const int64_t** order) {
    SH_RANGE("sh_shard_advance_time");
    StreamScope _ss(s && s->ctx ? s->ctx->stream : nullptr);
    if (!s || !out) return sh_fail(SH_ERR_INVALID, "sh_shard_advance_time: NULL argument");
    if (s->packed) return sh_fail(SH_ERR_STATE, "sh_shard_advance_time: a packed push is still in flight");
    // nothing in flight: the consumed stream state is the ingest's
    s->cur_clock = s->clock;
    s->cur_clock_valid = s->clock_valid;
    s->cur_E0 = s->E0;
    s->cur_e0_valid = s->e0_valid;
    sh_query* q = s->owner;
    if (s->sliding) {
        // expiry is lazy (applied at each key's next event): the TIMER only moves the clock
        RCHK(sliding_advance(q, now, out));
        if (!(s->clock_valid && now < s->clock)) {
            s->clock = now;
            s->clock_valid = true;
        }
        q->order_host.clear();
        set_order(s, true, order);
        return SH_OK;
    }
    sync_owner(s);
    if (s->agg) host_out = 0;
    RCHK(query_advance(q, now, host_out != 0, out));
    if (s->agg) RCHK(agg_after_root(s->agg, *out));
    if (!(s->clock_valid && now < s->clock)) {
        s->clock = now;
        s->clock_valid = true;
        if (s->d.window == SH_WIN_TIME_BATCH) s->W = std::max(s->W, wfun_g(s, now));
    }
    set_order(s, host_out != 0, order);
    return SH_OK;
}

extern "C" int sh_shard_stats(sh_shard* s, sh_stats* out) {
    if (!s || !out) return sh_fail(SH_ERR_INVALID, "sh_shard_stats: NULL argument");
    return sh_query_stats(s->owner, out);
}

// ---- checkpoint (sh_snapshot.cpp): the shard's global stream state; the owner query is snapshotted
// by the query sections. sc = {clock_valid, clock, e0_valid, E0, W, carry, seq, sl_pm, send_base,
// p0_known, p0, rank, world, sliding}.
sh_aggregation* shard_aggregation(sh_shard* s) { return s->agg; }

int shard_checkpoint_state(sh_shard* s, int64_t* sc, int n, bool set, sh_query** owner) {
    if (n != 14) return sh_fail(SH_ERR_INVALID, "shard snapshot layout");
    *owner = s->owner;
    if (s->packed) return sh_fail(SH_ERR_INVALID, "shard snapshot between pack and consume");
    if (!set) {
        const int64_t v[14] = {s->clock_valid, s->clock, s->e0_valid, s->E0, s->W, s->carry, (int64_t)s->seq,
                               s->sl_pm, s->send_base, s->p0_known, s->owner->p0, s->rank, s->world, s->sliding};
        for (int i = 0; i < 14; i++) sc[i] = v[i];
        return SH_OK;
    }
    if (sc[11] != s->rank || sc[12] != s->world || (sc[13] != 0) != s->sliding)
        return sh_fail(SH_ERR_INVALID, "snapshot was taken from a different shard (rank / world / window)");
    s->clock_valid = sc[0] != 0;
    s->clock = sc[1];
    s->e0_valid = sc[2] != 0;
    s->E0 = sc[3];
    s->W = sc[4];
    s->carry = sc[5];
    s->seq = (uint64_t)sc[6];
    s->sl_pm = sc[7];
    s->send_base = sc[8];
    s->p0_known = sc[9] != 0;
    s->cur_clock = s->clock;
    s->cur_clock_valid = s->clock_valid;
    s->cur_E0 = s->E0;
    s->cur_e0_valid = s->e0_valid;
    s->fp = s->fp_orig;
    if (s->p0_known) {
        const int pc = s->d.partition_col;
        RCHK(partition_filter(s->fp_orig, pc, s->d.col_types[pc], sc[10], &s->fp));
    }
    return SH_OK;
}
