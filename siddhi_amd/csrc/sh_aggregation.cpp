// sh_aggregation.cpp — `define aggregation A from S[cond] select k, aggs group by k aggregate [by ts]
// every <min> ... <max>` on the GPU (core/aggregation/*, util/parser/AggregationParser.java).
//
// Root duration: AGG_TIMESTAMP = currentTimeMillis() = the playback clock (AggregationParser.java:977-990),
// so the root executor's stores are processing-time buckets that close when the clock crosses the next
// bucket boundary (IncrementalExecutor.execute :110-139). That is exactly timeBatch(T_root, 0) with group
// key (event-time bucket of `ts` at the root duration, k) — the root runs on the batch-window pipeline.
// Upper durations fold the dispatched rows in device hash tables; their emission cascade (rows with the
// parent's store timestamp, then a TIMER with the parent's new bucket start, :141-150) is scalar control
// flow driven here on the host, restated from IncrementalExecutor.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sh_agg.h"
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

// ---- host restatement of IncrementalTimeConverterUtil (GMT) ----------------------------------------
static int64_t h_floor_div(int64_t a, int64_t b) {
    int64_t q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) q--;
    return q;
}
static int64_t h_days_from_civil(int64_t y, unsigned m, unsigned d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const unsigned yoe = (unsigned)(y - era * 400);
    const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + (int64_t)doe - 719468;
}
static void h_civil_from_days(int64_t z, int64_t& y, unsigned& m, unsigned& d) {
    z += 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const unsigned doe = (unsigned)(z - era * 146097);
    const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    y = (int64_t)yoe + era * 400;
    const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const unsigned mp = (5 * doy + 2) / 153;
    d = doy - (153 * mp + 2) / 5 + 1;
    m = mp + (mp < 10 ? 3 : -9);
    y += (m <= 2);
}
struct HCivil { int64_t y; unsigned m, d; int64_t h; };
static HCivil h_civil(int64_t ms) {
    int64_t days = h_floor_div(ms, 86400000);
    HCivil c;
    h_civil_from_days(days, c.y, c.m, c.d);
    c.h = (ms - days * 86400000) / 3600000;
    return c;
}
static int64_t h_epoch(int64_t y, int64_t m, int64_t d, int64_t h) {
    return (h_days_from_civil(y, (unsigned)m, (unsigned)d) * 86400 + h * 3600) * 1000;
}
static int h_month_len(unsigned m, bool leap) {
    static const int L[13] = {0, 31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    return (m == 2 && leap) ? 29 : L[m];
}
static int64_t h_start_of(int64_t t, int dur) {
    switch (dur) {
        case SH_DUR_SECONDS: return t - t % 1000;
        case SH_DUR_MINUTES: return t - t % 60000;
        case SH_DUR_HOURS: { HCivil c = h_civil(t); return h_epoch(c.y, c.m, c.d, c.h); }
        case SH_DUR_DAYS: { HCivil c = h_civil(t); return h_epoch(c.y, c.m, c.d, 0); }
        case SH_DUR_MONTHS: { HCivil c = h_civil(t); return h_epoch(c.y, c.m, 1, 0); }
        default: { HCivil c = h_civil(t); return h_epoch(c.y, 1, 1, 0); }
    }
}
// getNextEmitTime (IncrementalTimeConverterUtil.java:33-50, 89-160), month length via `year % 4 == 0`
static int64_t h_next_emit(int64_t t, int dur) {
    switch (dur) {
        case SH_DUR_SECONDS: return t - t % 1000 + 1000;
        case SH_DUR_MINUTES: return t - t % 60000 + 60000;
        case SH_DUR_HOURS: {
            HCivil c = h_civil(t);
            if (c.h == 23) {
                if ((int)c.d + 1 > h_month_len(c.m, c.y % 4 == 0)) {
                    if (c.m == 12) return h_epoch(c.y + 1, 1, 1, 0);
                    return h_epoch(c.y, c.m + 1, 1, 0);
                }
                return h_epoch(c.y, c.m, c.d + 1, 0);
            }
            return h_epoch(c.y, c.m, c.d, c.h + 1);
        }
        case SH_DUR_DAYS: {
            HCivil c = h_civil(t);
            if ((int)c.d + 1 > h_month_len(c.m, c.y % 4 == 0)) {
                if (c.m == 12) return h_epoch(c.y + 1, 1, 1, 0);
                return h_epoch(c.y, c.m + 1, 1, 0);
            }
            return h_epoch(c.y, c.m, c.d + 1, 0);
        }
        case SH_DUR_MONTHS: {
            HCivil c = h_civil(t);
            if (c.m == 12) return h_epoch(c.y + 1, 1, 1, 0);
            return h_epoch(c.y, c.m + 1, 1, 0);
        }
        default: { HCivil c = h_civil(t); return h_epoch(c.y + 1, 1, 1, 0); }
    }
}

// ... in the aggregation's time zone, a fixed offset tz from GMT: hours and longer at local boundaries
static int64_t h_start_of(int64_t t, int dur, int64_t tz) {
    return dur >= SH_DUR_HOURS ? h_start_of(t + tz, dur) - tz : h_start_of(t, dur);
}
static int64_t h_next_emit(int64_t t, int dur, int64_t tz) {
    return dur >= SH_DUR_HOURS ? h_next_emit(t + tz, dur) - tz : h_next_emit(t, dur);
}

// calendar buckets of a month (cal 1) / year (cal 2) root in the zone offset tz (sh_device.h cal_idx_d)
int64_t cal_idx_h(int64_t t, int cal, int64_t tz) {
    const HCivil c = h_civil(t + tz);
    return cal == 1 ? c.y * 12 + (int64_t)(c.m - 1) : c.y;
}
int64_t cal_start_h(int64_t i, int cal, int64_t tz) {
    if (cal == 1) {
        const int64_t y = h_floor_div(i, 12);
        return h_epoch(y, i - y * 12 + 1, 1, 0) - tz;
    }
    return h_epoch(i, 1, 1, 0) - tz;
}

// A batch of rows on the device: bucket / key / base values (stride = cap).
struct RowBatch {
    int64_t n = 0, cap = 0;
    const int64_t* bucket = nullptr;
    const int64_t* key = nullptr;
    const u64* vals = nullptr;
};

// Rows accumulated in a duration's table.
struct TableBuf {
    DevBuf bucket, key, vals;
    int64_t n = 0, cap = 0;
    int64_t drained = 0;  // rows [0, drained) were returned by sh_aggregation_table; all stay for retrieval
};

struct Level {
    int dur = 0;
    // IncrementalExecutor.ExecutorState (:283-317) + BaseIncrementalValueStore store state (:231-262)
    int64_t next_emit = -1, start = -1, store_ts = -1;
    bool processed = false;
    KeyTableHost kt;
    DevBuf vals, tag, first_seq, order, slots, dup, blk, out_bucket, out_key, out_vals;
    int64_t n_in = 0;  // rows merged since the last dispatch
    int64_t nslots = 0;
    uint32_t epoch = 0;
    int* dup_host = nullptr;
    uint32_t* chk = nullptr;  // pinned landing area of the key table's counters (checked after a sync)
    bool dirty = false;       // merged into since its counters were last fetched
};

struct sh_aggregation {
    sh_ctx* ctx = nullptr;
    sh_aggregation_desc d{};
    BasePlan bp{};
    int32_t btypes[SH_MAX_AGGS]{};
    int nb = 0;
    bool has_bucket = false;
    int64_t T_root = 0;
    int64_t tz = 0;       // aggTimeZone as a fixed offset (ms)
    int64_t tz_root = 0;  // the root's bucket offset: tz for hour / day roots (sec / min are zone-free)
    int cal = 0;          // a month (1) / year (2) root: calendar buckets and windows, T_root unused
    sh_query* root = nullptr;
    sh_shard* shard = nullptr;  // sharded: the root is this shard's owner query (owned by the shard)
    bool root_init = false;
    int64_t root_bucket = 0;
    std::vector<Level> levels;            // durations above the root
    TableBuf tables[SH_DUR_YEARS + 1];
    // a grown table's old blocks, freed at the next call that synchronises anyway (a hipFree drains the
    // device: in a push it would stall the queued root and level work)
    std::vector<DevBuf> retired;
    // the last push's root flushes, handed to the levels during the next call (agg_settle)
    bool dfr_on = false;
    sh_out dfr_out{};
    std::vector<int64_t> dfr_offs, dfr_windows;
    int64_t dfr_clock = 0;
    OutHost tout, fout;
    // retrieval scratch (sh_aggregation_find)
    DevBuf m_bucket, m_key, m_vals, f_bucket, f_key, f_vals, g_bucket, g_idx, g_k64, g_k64s, g_idx1, g_idx2, g_dk, g_flag,
        g_pre, g_tmp, g_sort, v_bucket, v_key, v_vals;
    DevBuf root_bucket_col, root_key_col, minmax;
    int64_t* h_minmax = nullptr;
    // device time of the last push: ev0 before the root's key reservation, ev1 after the roll-up
    // levels' kernels are queued (read lazily by sh_aggregation_stats)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int64_t last_events = 0;
    bool timed = false;
    // every push's device time, summed without a wait per push (sh_aggregation_timing): a ring of
    // event pairs, each read once its push has completed (at the latest when the ring wraps)
    static constexpr int kRing = 64;
    hipEvent_t r0[kRing] = {}, r1[kRing] = {};
    int64_t r_next = 0, r_done = 0, r_pushes = 0;
    double r_ms = 0;
    // band keys for the root (KeyTable::lk): (bucket, dictionary id) slots by arithmetic while the live
    // buckets fit `band_rows` consecutive buckets; the open-addressing table otherwise
    bool band_ok = false;
    uint32_t band_lk = 0, band_rows = 0, band_mul = 1, band_add = 0;
    bool chk_pending = false;  // level key-table counters queued to pinned memory, not yet verified
    // band re-bases swap the root's table with this spare (init_band reuses its buffers: no hipMalloc /
    // hipFree, whose implicit device synchronisation cost ~0.2 ms per push)
    KeyTableHost band_spare;
    // the roll-up levels (merges, dispatches, upper-duration tables) run on their own stream: a push's
    // level kernels overlap the next push's root window instead of delaying it. They read the root's
    // rows from the root duration's table (appended on the compute stream, ev_tab), never the root's
    // output buffers, which the next push overwrites.
    hipStream_t lstream = nullptr;
    hipEvent_t ev_tab = nullptr, ev_lchk = nullptr;
    // the queued events' bucket range after the last device push, measured behind it on the stream
    // (k_pend_bucket_range, read at the next push once ev_pr completed): the next push places its band
    // from it without a probe round trip
    bool pr_valid = false;
    int64_t pr_b0 = 0;
    hipEvent_t ev_pr = nullptr;
    DevBuf pr_dev;
    int64_t* h_pr = nullptr;
    // group keys wider than the root key's 32-bit half — two group-by columns, or one long / double column
    // beside the `aggregate by` bucket: every passing event's key is interned into a table (ikt) and its
    // slot travels as a synthetic dictionary column (index d.n_cols of the root's batch); tables and
    // retrievals map the slots back to the group-by values (k_agg_unintern)
    bool intern = false;
    WideKeys wk;  // (sh_wide.h: any number of group-by columns, 64-bit ones included)
    DevBuf dkeys;
};

// The levels' key-table overflow checks are queued with each merge and verified after the next
// synchronisation the aggregation makes anyway (a full table still fails the call loudly, one sync
// later, instead of stalling the stream after every merge).
static int agg_verify(sh_aggregation* a) {
    if (!a->chk_pending) return SH_OK;
    a->chk_pending = false;
    HIPCHK(sh_wait_event(a->ev_lchk));
    for (auto& L : a->levels) RCHK(L.kt.check_result(L.chk));
    return SH_OK;
}

static int agg_sync(sh_aggregation* a) {
    HIPCHK(sh_wait_stream(a->ctx->stream));
    if (a->lstream) HIPCHK(sh_wait_stream(a->lstream));
    a->retired.clear();  // (both streams are idle: nothing reads the grown tables' old blocks)
    return agg_verify(a);
}

// the stream of the roll-up levels' work
static hipStream_t lvl(const sh_aggregation* a) { return a->lstream ? a->lstream : a->ctx->stream; }

static LevelDev level_dev(Level& L, int nb) {
    LevelDev D;
    D.kt = L.kt.dev();
    D.nslots = L.nslots;
    D.vals = L.vals.as<u64>();
    D.vs = nb + 1;
    D.tag = L.tag.as<u32>();
    D.first_seq = L.first_seq.as<u32>();
    D.order = L.order.as<u32>();
    return D;
}

// append rows to the duration's table buffer
static int table_append(sh_aggregation* a, int dur, const RowBatch& rb) {
    if (rb.n == 0) return SH_OK;
    TableBuf& t = a->tables[dur];
    hipStream_t s = dur == a->d.min_duration ? a->ctx->stream : lvl(a);
    int64_t need = t.n + rb.n;
    if (need > t.cap) {
        // the rows so far copied on the stream that appends to this table (after its earlier appends);
        // the old block stays allocated until a synchronising call (level merges queued on the other
        // stream may still read the root table's old block) — no wait inside the push
        int64_t ncap = std::max<int64_t>(need, std::max<int64_t>(1024, t.cap * 2));
        DevBuf b2, k2, v2;
        RCHK(b2.reserve(ncap * 8, false));
        RCHK(k2.reserve(ncap * 8, false));
        RCHK(v2.reserve((size_t)a->nb * ncap * 8, false));
        if (t.n) {
            HIPCHK(hipMemcpyAsync(b2.p, t.bucket.p, t.n * 8, hipMemcpyDeviceToDevice, s));
            HIPCHK(hipMemcpyAsync(k2.p, t.key.p, t.n * 8, hipMemcpyDeviceToDevice, s));
            for (int b = 0; b < a->nb; b++)
                HIPCHK(hipMemcpyAsync((char*)v2.p + (size_t)b * ncap * 8, (char*)t.vals.p + (size_t)b * t.cap * 8,
                                      t.n * 8, hipMemcpyDeviceToDevice, s));
        }
        a->retired.push_back(std::move(t.bucket));
        a->retired.push_back(std::move(t.key));
        a->retired.push_back(std::move(t.vals));
        t.bucket = std::move(b2); t.key = std::move(k2); t.vals = std::move(v2);
        t.cap = ncap;
    }
    launch_table_append(s, rb.n, rb.bucket, rb.key, rb.vals, rb.cap, a->nb, t.bucket.as<int64_t>() + t.n,
                        t.key.as<int64_t>() + t.n, t.vals.as<u64>() + t.n, t.cap);
    HIPCHK(hipGetLastError());
    t.n = need;
    return SH_OK;
}

static int level_timer(sh_aggregation* a, size_t li, int64_t ts);
static int level_rows(sh_aggregation* a, size_t li, const RowBatch& rb, int64_t ts);

// dispatchEvent (:201-258) + cleanBaseIncrementalValueStore (:260-266)
static int level_dispatch(sh_aggregation* a, size_t li, int64_t start_of_new) {
    Level& L = a->levels[li];
    static const bool atrace = getenv("SH_ALLOC_TRACE") != nullptr;
    if (atrace && L.processed) fprintf(stderr, "[sh alloc] dispatch level %zu (%lld rows in)\n", li, (long long)L.n_in);
    hipStream_t s = lvl(a);
    StreamScope _sc(s);
    if (L.processed) {
        int64_t n_in = L.n_in;
        int nblk = (int)((n_in + kTile - 1) / kTile);
        RCHK(L.blk.reserve((nblk + 8) * 8, false));
        RCHK(L.order.reserve(std::max<int64_t>(n_in, 1) * 4, false));
        LevelDev D = level_dev(L, a->nb);
        launch_level_mark(s, D, n_in);
        launch_level_count(s, D, n_in, L.blk.as<int64_t>(), nblk);
        std::vector<int64_t> bc(nblk);
        HIPCHK(hipMemcpyAsync(bc.data(), L.blk.p, nblk * 8, hipMemcpyDeviceToHost, s));
        RCHK(agg_sync(a));
        int64_t n = 0;
        for (auto c : bc) n += c;
        int64_t cap = std::max<int64_t>(n, 1);
        RCHK(L.out_bucket.reserve(cap * 8, false));
        RCHK(L.out_key.reserve(cap * 8, false));
        RCHK(L.out_vals.reserve((size_t)a->nb * cap * 8, false));
        launch_scan_sum(s, L.blk.as<int64_t>(), nblk);
        launch_level_extract(s, D, a->bp, a->has_bucket, L.store_ts, n_in, L.blk.as<int64_t>(), nblk, cap,
                             L.out_bucket.as<int64_t>(), L.out_key.as<int64_t>(), L.out_vals.as<u64>());
        HIPCHK(hipGetLastError());
        L.n_in = 0;
        RowBatch rb;
        rb.n = n; rb.cap = cap;
        rb.bucket = L.out_bucket.as<int64_t>();
        rb.key = L.out_key.as<int64_t>();
        rb.vals = L.out_vals.as<u64>();
        RCHK(table_append(a, L.dur, rb));
        if (li + 1 < a->levels.size()) RCHK(level_rows(a, li + 1, rb, L.store_ts));
    }
    L.store_ts = start_of_new;
    L.processed = false;
    return SH_OK;
}

// IncrementalExecutor.execute for a chunk of rows that share AGG_TIMESTAMP `ts` (:110-139)
static int level_rows(sh_aggregation* a, size_t li, const RowBatch& rb, int64_t ts) {
    Level& L = a->levels[li];
    L.start = h_start_of(ts, L.dur, a->tz);
    if (ts >= L.next_emit) {
        L.next_emit = h_next_emit(ts, L.dur, a->tz);
        RCHK(level_dispatch(a, li, L.start));
        if (li + 1 < a->levels.size()) RCHK(level_timer(a, li + 1, L.start));
    }
    if (rb.n > 0) {
        hipStream_t s = lvl(a);
        StreamScope _sc(s);
        RCHK(L.slots.reserve(rb.n * 4, false));
        L.epoch++;
        if (L.n_in + rb.n >= (int64_t)0xFFFFFFF0ll) return sh_fail(SH_ERR_INVALID, "too many rows in one roll-up bucket");
        launch_level_merge(s, rb.n, rb.bucket, rb.key, a->has_bucket, L.dur, rb.vals, rb.cap, level_dev(L, a->nb),
                           a->bp, L.epoch, (u32)L.n_in, L.slots.as<u32>(), L.dup.as<int>(), a->tz);
        L.n_in += rb.n;
        HIPCHK(hipGetLastError());
        L.dirty = true;  // its key-table counters are fetched once per push (agg_after_root)
        L.processed = true;
    }
    return SH_OK;
}

// TIMER event at a child executor (getTimestamp for non-CURRENT events, :163-168)
static int level_timer(sh_aggregation* a, size_t li, int64_t ts) {
    RowBatch none;
    return level_rows(a, li, none, ts);
}

// a run of `count` TIMERs at first, first+step, ... (one per root bucket the clock passed)
static int level_timer_run(sh_aggregation* a, size_t li, int64_t first, int64_t step, int64_t count) {
    Level& L = a->levels[li];
    while (count > 0) {
        if (first >= L.next_emit) {
            RCHK(level_timer(a, li, first));
            first += step;
            count--;
        } else {
            // timers below nextEmitTime only refresh startTimeOfAggregates
            int64_t k = (L.next_emit - first + step - 1) / step;
            if (k >= count) {
                L.start = h_start_of(first + (count - 1) * step, L.dur, a->tz);
                return SH_OK;
            }
            first += k * step;
            count -= k;
        }
    }
    return SH_OK;
}

// the root's buckets: fixed periods T_root from the zone's offset, or calendar months / years
static int64_t root_floor(const sh_aggregation* a, int64_t t) {
    if (a->cal) return cal_start_h(cal_idx_h(t, a->cal, a->tz_root), a->cal, a->tz_root);
    return h_floor_div(t + a->tz_root, a->T_root) * a->T_root - a->tz_root;
}
static int64_t root_shift(const sh_aggregation* a, int64_t start, int64_t k) {  // the bucket k after start's
    if (a->cal) return cal_start_h(cal_idx_h(start, a->cal, a->tz_root) + k, a->cal, a->tz_root);
    return start + k * a->T_root;
}
static int64_t root_count(const sh_aggregation* a, int64_t from, int64_t to) {  // buckets from -> to
    if (a->cal) return cal_idx_h(to, a->cal, a->tz_root) - cal_idx_h(from, a->cal, a->tz_root);
    return (to - from) / a->T_root;
}
// start of the root's window W (window 1 starts at E0, the first nextEmitTime)
static int64_t root_window_start(const sh_aggregation* a, int64_t W) { return root_shift(a, a->root->E0, W - 1); }

// TIMERs of the root buckets after `last` up to `cb` (one per bucket the clock passed)
static int root_timers(sh_aggregation* a, int64_t last, int64_t cb) {
    if (cb <= last || a->levels.empty()) return SH_OK;
    if (!a->cal) return level_timer_run(a, 0, last + a->T_root, a->T_root, (cb - last) / a->T_root);
    const int64_t n = root_count(a, last, cb);
    for (int64_t k = 1; k <= n; k++) RCHK(level_timer(a, 0, root_shift(a, last, k)));
    return SH_OK;
}

static int pass_root_flushes(sh_aggregation* a, const sh_out* o, const int64_t* windows) {
    int nk = o->n_keys;
    for (int64_t f = 0; f < o->n_flushes; f++) {
        int64_t W = windows[f];
        int64_t s_f = root_window_start(a, W);  // processing bucket of the closed root store
        int64_t lo = o->flush_offsets[f], hi = o->flush_offsets[f + 1];
        RowBatch rb;
        rb.n = hi - lo;
        rb.cap = o->n_rows;
        const int64_t* keys = o->keys;
        if (a->has_bucket) {
            rb.bucket = keys + lo;
            rb.key = nk > 1 ? keys + (size_t)o->n_rows + lo : a->root_key_col.as<int64_t>();
        } else {
            rb.bucket = a->root_bucket_col.as<int64_t>();
            rb.key = nk > 0 ? keys + lo : a->root_key_col.as<int64_t>();
        }
        rb.vals = (const u64*)o->vals + lo;
        // timers of the empty root buckets before s_f
        RCHK(root_timers(a, a->root_bucket, s_f));
        a->root_bucket = std::max(a->root_bucket, s_f);
        // the root table gets the rows; without `aggregate by` AGG_TIMESTAMP is the store timestamp
        if (!a->has_bucket) {
            RCHK(a->root_bucket_col.reserve(std::max<int64_t>(rb.n, 1) * 8, false));
            launch_fill_i64(a->ctx->stream, a->root_bucket_col.as<int64_t>(), rb.n, s_f);
            rb.bucket = a->root_bucket_col.as<int64_t>();
        }
        const int64_t n0 = a->tables[a->d.min_duration].n;
        RCHK(table_append(a, a->d.min_duration, rb));
        if (!a->levels.empty()) {
            // the level stream reads the rows from the root table's copy, once it is written
            const TableBuf& t = a->tables[a->d.min_duration];
            RowBatch tb;
            tb.n = rb.n;
            tb.cap = t.cap;
            tb.bucket = t.bucket.as<int64_t>() + n0;
            tb.key = t.key.as<int64_t>() + n0;
            tb.vals = t.vals.as<u64>() + n0;
            if (a->lstream && rb.n > 0) {
                HIPCHK(hipEventRecord(a->ev_tab, a->ctx->stream));
                HIPCHK(hipStreamWaitEvent(a->lstream, a->ev_tab, 0));
            }
            RCHK(level_rows(a, 0, rb.n > 0 ? tb : rb, s_f));
            RCHK(level_timer(a, 0, root_shift(a, s_f, 1)));
        }
        a->root_bucket = root_shift(a, s_f, 1);
    }
    return SH_OK;
}

// after a push / advance: timers of the root buckets up to the clock
static int catch_up(sh_aggregation* a, int64_t clock) {
    sh_query* q = a->root;
    if (!q->e0_valid) return SH_OK;
    if (!a->root_init) {
        // first event: root store opens at the bucket of the first clock and TIMERs its child (:141-150)
        a->root_init = true;
        a->root_bucket = root_shift(a, q->E0, -1);
        if (!a->levels.empty()) RCHK(level_timer(a, 0, a->root_bucket));
    }
    int64_t cb = root_floor(a, clock);
    RCHK(root_timers(a, a->root_bucket, cb));
    a->root_bucket = std::max(a->root_bucket, cb);
    return SH_OK;
}

static int agg_mid_hook(void* p);
static int agg_create(sh_ctx* ctx, const sh_aggregation_desc* d, int32_t rank, int32_t world, sh_shard** shard,
                      sh_aggregation** out) {
    if (!ctx || !d || !out) return sh_fail(SH_ERR_INVALID, "sh_aggregation_create: NULL argument");
    if (d->n_cols <= 0 || d->n_cols > SH_MAX_COLS || d->n_aggs <= 0 || d->n_aggs > SH_MAX_AGGS ||
        d->min_duration < 0 || d->max_duration > SH_DUR_YEARS || d->min_duration > d->max_duration)
        return sh_fail(SH_ERR_INVALID, "invalid aggregation descriptor");
    if (d->n_group_by > SH_MAX_GROUP) return sh_fail(SH_ERR_INVALID, "invalid aggregation descriptor");
    if (d->ts_col >= 0 && (d->ts_col >= d->n_cols || d->col_types[d->ts_col] != SH_T_LONG))
        return sh_fail(SH_ERR_INVALID, "`aggregate by` attribute must be a long");
    sh_aggregation* a = new sh_aggregation();
    a->ctx = ctx;
    a->d = *d;
    a->d.filter = nullptr;
    a->has_bucket = d->ts_col >= 0;
    // (month / year roots: calendar windows and buckets; T_root is only a nominal positive period)
    static const int64_t unit[] = {1000, 60000, 3600000, 86400000, 31 * 86400000ll, 366 * 86400000ll};
    a->T_root = unit[d->min_duration];
    a->cal = d->min_duration == SH_DUR_MONTHS ? 1 : d->min_duration == SH_DUR_YEARS ? 2 : 0;
    if (d->tz_offset_ms % 60000 != 0 || d->tz_offset_ms <= -86400000 || d->tz_offset_ms >= 86400000) {
        delete a;
        return sh_fail(SH_ERR_INVALID, "aggTimeZone offset must be whole minutes within a day");
    }
    a->tz = d->tz_offset_ms;
    a->tz_root = d->min_duration >= SH_DUR_HOURS ? a->tz : 0;
    // base values, de-duplicated like AggregationParser.populateFinalBaseAggregators
    struct B { int kind; int col; };
    std::vector<B> bases;
    auto add = [&](int kind, int col) {
        for (auto& b : bases) if (b.kind == kind && (kind == 0 || b.col == col)) return;
        bases.push_back(B{kind, col});
    };
    for (int i = 0; i < d->n_aggs; i++) {
        int fn = d->aggs[i].fn, col = d->aggs[i].col;
        if (fn != SH_AGG_COUNT && (col < 0 || col >= d->n_cols)) { delete a; return sh_fail(SH_ERR_INVALID, "bad aggregator column"); }
        if (fn == SH_AGG_SUM) add(1, col);
        else if (fn == SH_AGG_AVG) { add(1, col); add(0, -1); }
        else if (fn == SH_AGG_COUNT) add(0, -1);
        else if (fn == SH_AGG_MIN) add(2, col);
        else add(3, col);
    }
    // the root query's aggregators restate those base executors over the raw events
    sh_query_desc rd{};
    rd.n_cols = d->n_cols;
    for (int c = 0; c < d->n_cols; c++) rd.col_types[c] = d->col_types[c];
    rd.n_filter_ops = d->n_filter_ops;
    rd.filter = d->filter;
    rd.window = SH_WIN_TIME_BATCH;
    rd.window_param = a->T_root;
    rd.has_start_time = 1;
    rd.start_time = -a->tz_root;  // (hour / day roots close at the zone's local boundaries)
    rd.current_on = 1;
    rd.partition_col = -1;
    rd.n_aggs = (int)bases.size();
    for (size_t i = 0; i < bases.size(); i++) {
        static const int fn[] = {SH_AGG_COUNT, SH_AGG_SUM, SH_AGG_MIN, SH_AGG_MAX};
        rd.aggs[i].fn = fn[bases[i].kind];
        rd.aggs[i].col = bases[i].col < 0 ? 0 : bases[i].col;
    }
    rd.key_capacity = d->key_capacity > 0 ? d->key_capacity : (1 << 16);
    KeyPlan kp{};
    int g = 0;
    if (a->has_bucket) {
        kp.col[g] = d->ts_col; kp.type[g] = SH_T_LONG; kp.div[g] = a->cal ? -a->cal : a->T_root; kp.add[g] = a->tz_root;
        g++;
    }
    int gtype = -1;  // the root key's group component type
    if (d->n_group_by >= 1) {
        const int t = d->col_types[d->group_by[0]];
        a->intern = d->n_group_by >= 2 ||
                    !(t == SH_T_INT || t == SH_T_STRID || t == SH_T_BOOL || (t == SH_T_LONG && !a->has_bucket));
        if (a->intern) {
            if (shard) { delete a; return sh_fail(SH_ERR_UNSUPPORTED, "a sharded aggregation groups by one 32-bit column"); }
            if (d->n_cols + 1 > SH_MAX_COLS) { delete a; return sh_fail(SH_ERR_UNSUPPORTED, "too many columns to intern group keys"); }
            int rc0 = a->wk.init(d->n_group_by, d->group_by, d->n_cols, d->col_types, rd.key_capacity);
            if (rc0) { delete a; return rc0; }
            // the interned id: a dictionary column past the stream's own (dense in [0, id space))
            rd.n_cols = d->n_cols + 1;
            rd.col_types[d->n_cols] = SH_T_STRID;
            rd.key_capacity = a->wk.id_space();
            kp.col[g] = d->n_cols; kp.type[g] = SH_T_STRID; kp.div[g] = 0; g++;
            gtype = SH_T_STRID;
        } else {
            kp.col[g] = d->group_by[0]; kp.type[g] = t; kp.div[g] = 0; g++;
            gtype = t;
        }
    }
    kp.n = g;
    rd.n_group_by = 0;
    int rc = shard ? shard_create_root(ctx, &rd, kp, rank, world, &a->shard, &a->root)
                   : sh_query_create_internal(ctx, &rd, kp, &a->root);
    if (rc) { delete a; return rc; }
    a->root->cal = a->cal;
    a->root->cal_tz = a->tz_root;
    if (!shard) {
        a->root->mid_hook = agg_mid_hook;
        a->root->mid_arg = a;
    }
    if (shard) {
        shard_attach_aggregation(a->shard, a);
        *shard = a->shard;
    }
    if (a->has_bucket && d->n_group_by >= 1 && gtype == SH_T_STRID && !a->cal) {
        // ids per bucket row: the GPU's share of the dictionary (sharded owners hold the ids = rank mod G)
        const int64_t cap = rd.key_capacity, per = shard ? (cap + world - 1) / world : cap;
        // (A/B switch SH_AGG_BAND_ROWS, 0 = hash keys only)
        uint32_t lk = 4, rows = (uint32_t)std::max(0, Tuning::from_env().agg_band_rows);
        while (((int64_t)1 << lk) < per) lk++;
        while (rows > 4 && ((int64_t)rows << lk) > (8 << 20)) rows >>= 1;
        if (rows >= 2 && ((int64_t)rows << lk) <= (8 << 20)) {
            a->band_ok = true;
            a->band_lk = lk;
            a->band_rows = rows;
            a->band_mul = shard ? (uint32_t)world : 1u;
            a->band_add = shard ? (uint32_t)rank : 0u;
            sh_query* q = a->root;
            q->band_keys = true;
            q->band_lk = lk;
            q->band_rows = rows;
            q->band_mul = a->band_mul;
            q->band_add = a->band_add;
        }
    }
    a->nb = a->root->ap.n;
    a->bp.n = a->nb;
    for (int i = 0; i < a->nb; i++) {
        a->bp.kind[i] = a->root->ap.kind[i];
        a->btypes[i] = a->root->vtypes[i];
    }
    HIPCHK(hipEventCreate(&a->ev0));
    HIPCHK(hipEventCreate(&a->ev1));
    HIPCHK(hipStreamCreateWithFlags(&a->lstream, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&a->ev_tab, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&a->ev_lchk, hipEventDisableTiming));
    // constant key / bucket columns for rows without them
    RCHK(a->minmax.reserve(minmax_scratch_bytes(), false));
    HIPCHK(hipHostMalloc((void**)&a->h_minmax, 16, hipHostMallocDefault));
    RCHK(a->root_key_col.reserve(8 << 20, false));
    HIPCHK(hipMemsetAsync(a->root_key_col.p, 0, 8 << 20, ctx->stream));
    // upper durations
    for (int dur = d->min_duration + 1; dur <= d->max_duration; dur++) {
        a->levels.emplace_back();
        Level& L = a->levels.back();
        L.dur = dur;
        RCHK(L.kt.init(std::max<int64_t>(2 * rd.key_capacity, 64)));
        L.nslots = (int64_t)L.kt.size_ + 1;
        RCHK(L.vals.reserve((size_t)(a->nb + 1) * L.nslots * 8, false));
        RCHK(L.tag.reserve(L.nslots * 4, false));
        RCHK(L.first_seq.reserve(L.nslots * 4, false));
        HIPCHK(hipMemsetAsync(L.first_seq.p, 0xFF, L.nslots * 4, ctx->stream));
        RCHK(L.dup.reserve(64, false));
        HIPCHK(hipMemsetAsync(L.dup.p, 0, 64, ctx->stream));
        HIPCHK(hipMemsetAsync(L.vals.p, 0, (size_t)(a->nb + 1) * L.nslots * 8, ctx->stream));
        HIPCHK(hipMemsetAsync(L.tag.p, 0, L.nslots * 4, ctx->stream));
        HIPCHK(hipHostMalloc((void**)&L.dup_host, 64, hipHostMallocDefault));
        HIPCHK(hipHostMalloc((void**)&L.chk, 16, hipHostMallocDefault));
        std::memset(L.chk, 0, 16);
    }
    *out = a;
    return SH_OK;
}

extern "C" int sh_aggregation_create(sh_ctx* ctx, const sh_aggregation_desc* d, sh_aggregation** out) {
    StreamScope _ss(ctx ? ctx->stream : nullptr);
    return agg_create(ctx, d, 0, 1, nullptr, out);
}

// Rank `rank` of `world` of a key-sharded aggregation: events reach the GPU that
// owns their group key through the sh_shard_* protocol; each owner runs the root and every roll-up
// level for its keys. The clock, the root buckets and every TIMER are global, so the owners' tables
// together hold exactly the single-stream tables' rows.
extern "C" int sh_aggregation_shard_create(sh_ctx* ctx, const sh_aggregation_desc* d, int32_t rank, int32_t world,
                                           sh_shard** shard, sh_aggregation** out) {
    StreamScope _ss(ctx ? ctx->stream : nullptr);
    if (!shard) return sh_fail(SH_ERR_INVALID, "sh_aggregation_shard_create: NULL argument");
    if (d && d->n_group_by != 1) return sh_fail(SH_ERR_UNSUPPORTED, "sharded aggregations need one group-by key");
    if (d && d->min_duration > SH_DUR_DAYS)
        return sh_fail(SH_ERR_UNSUPPORTED, "sharded aggregations have sec / min / hour / day roots");
    return agg_create(ctx, d, rank, world, shard, out);
}

static void agg_free(sh_aggregation* a) {
    if (a->lstream) (void)hipStreamSynchronize(a->lstream);
    for (auto& L : a->levels) {
        DevBuf* bufs[] = {&L.vals, &L.tag, &L.first_seq, &L.order, &L.slots, &L.dup, &L.blk, &L.out_bucket, &L.out_key, &L.out_vals};
        for (auto* b : bufs) b->release();
        L.kt.release();
        if (L.dup_host) (void)hipHostFree(L.dup_host);
        if (L.chk) (void)hipHostFree(L.chk);
    }
    for (auto& t : a->tables) { t.bucket.release(); t.key.release(); t.vals.release(); }
    a->root_bucket_col.release();
    a->root_key_col.release();
    a->minmax.release();
    if (a->h_minmax) (void)hipHostFree(a->h_minmax);
    a->band_spare.release();
    a->pr_dev.release();
    if (a->h_pr) (void)hipHostFree(a->h_pr);
    if (a->ev_pr) (void)hipEventDestroy(a->ev_pr);
    if (a->ev_tab) (void)hipEventDestroy(a->ev_tab);
    if (a->ev_lchk) (void)hipEventDestroy(a->ev_lchk);
    if (a->lstream) {
        (void)hipStreamSynchronize(a->lstream);
        (void)hipStreamDestroy(a->lstream);
    }
    if (a->ev0) (void)hipEventDestroy(a->ev0);
    if (a->ev1) (void)hipEventDestroy(a->ev1);
    for (int i = 0; i < sh_aggregation::kRing; i++) {
        if (a->r0[i]) (void)hipEventDestroy(a->r0[i]);
        if (a->r1[i]) (void)hipEventDestroy(a->r1[i]);
    }
    delete a;
}

extern "C" int sh_aggregation_destroy(sh_aggregation* a) {
    StreamScope _ss(a && a->ctx ? a->ctx->stream : nullptr);
    if (!a) return SH_OK;
    if (a->shard) return sh_fail(SH_ERR_STATE, "a sharded aggregation is released by sh_shard_destroy");
    (void)hipStreamSynchronize(a->ctx->stream);
    sh_query_destroy(a->root);
    a->root = nullptr;
    agg_free(a);
    return SH_OK;
}

void agg_release_sharded(sh_aggregation* a) { agg_free(a); }

// Room in the root's key table for this push: (event-time bucket, key) pairs are bounded by
// min(N, keys x buckets spanned); closed buckets' keys are dropped by the rebuild.
// Band keys (KeyTable::lk): the push's buckets [lo, hi] and the queued events' buckets must lie in
// band_rows consecutive buckets; the band is re-based (the queued events' slots re-derived) when the
// push runs past it, and the root falls back to the open-addressing table while they do not fit.
// The queued events' bucket range: from the measurement queued behind the last device push (pr_valid),
// else probed now (one round trip).
static int pend_range(sh_aggregation* a, int64_t* lo, int64_t* hi) {
    sh_query* q = a->root;
    if (a->pr_valid) {
        HIPCHK(sh_wait_event(a->ev_pr));
        *lo = a->pr_b0 + a->h_pr[0];
        *hi = a->pr_b0 + a->h_pr[1];
        return SH_OK;
    }
    hipStream_t s = a->ctx->stream;
    const u32 ref = q->kt.lk ? q->kt.b0 : 0u;
    const int64_t base = q->kt.lk ? q->kt.band_base : 0;
    launch_pend_bucket_range(s, q->pend_pos.as<u32>(), q->n_pend, q->kt.dev(), ref, a->minmax.as<int64_t>());
    HIPCHK(hipMemcpyAsync(a->h_minmax, a->minmax.p, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(sh_wait_stream(s));
    *lo = base + a->h_minmax[0];
    *hi = base + a->h_minmax[1];
    return SH_OK;
}

// After a device push of a band-keyed root: the queued events' bucket range, measured on the stream
// (no wait) and read by the next push.
static int pend_range_queue(sh_aggregation* a) {
    sh_query* q = a->root;
    a->pr_valid = false;
    if (!a->band_ok || !q->kt.lk || q->n_pend <= 0) return SH_OK;
    hipStream_t s = a->ctx->stream;
    if (!a->ev_pr) HIPCHK(hipEventCreateWithFlags(&a->ev_pr, hipEventDisableTiming));
    if (!a->h_pr) HIPCHK(hipHostMalloc((void**)&a->h_pr, 16, hipHostMallocDefault));
    RCHK(a->pr_dev.reserve(16, false));
    launch_pend_bucket_range(s, q->pend_pos.as<u32>(), q->n_pend, q->kt.dev(), q->kt.b0, a->pr_dev.as<int64_t>());
    HIPCHK(hipMemcpyAsync(a->h_pr, a->pr_dev.p, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipEventRecord(a->ev_pr, s));
    a->pr_b0 = q->kt.band_base;
    a->pr_valid = true;
    return SH_OK;
}

// A device push of a band-keyed root without the probe round trip: the band is placed from the queued
// events' range (or the clock's bucket) and the push validates it — k_boundaries flags any bucket
// outside the band and push_core returns kRetryBand at its first synchronisation, before anything was
// committed; the push is then probed and pushed again. Returns 1 when the speculative push was taken.
static int spec_push(sh_aggregation* a, const sh_batch* dev, const sh_out** o, int* taken) {
    sh_query* q = a->root;
    *taken = 0;
    const int64_t R = a->band_rows;
    if (!a->band_ok || !a->has_bucket || !q->kt.lk || dev->n < (1 << 16) || a->shard || !q->clock_valid) return SH_OK;
    int64_t b0;
    if (q->n_pend > 0) {
        if (!a->pr_valid) return SH_OK;
        int64_t plo, phi;
        RCHK(pend_range(a, &plo, &phi));
        if (phi - plo >= R || plo < 0) return SH_OK;
        b0 = plo;
    } else {
        if (q->clock < 0) return SH_OK;
        b0 = (q->clock + a->tz_root) / a->T_root;
    }
    if (b0 != q->kt.band_base) {
        RCHK(a->band_spare.init_band(a->band_lk, a->band_rows, b0, a->band_mul, a->band_add));
        RCHK(query_swap_keys(q, a->band_spare));
    }
    q->band_spec = true;
    SH_TMARK(10);
    const int rc = sh_push_device(q, dev, o);
    q->band_spec = false;
    if (rc == kRetryBand) {
        // the overflow word of the band the push left: cleared before the probed push
        HIPCHK(hipMemsetAsync((char*)q->kt.ctrl.p + 8, 0, 8, a->ctx->stream));
        a->pr_valid = false;
        return SH_OK;
    }
    RCHK(rc);
    *taken = 1;
    return SH_OK;
}

static int band_reserve(sh_aggregation* a, int64_t lo, int64_t hi, int64_t bound) {
    sh_query* q = a->root;
    const int64_t R = a->band_rows;
    if (q->kt.lk && lo >= q->kt.band_base && hi < q->kt.band_base + R) return SH_OK;
    int64_t ulo = lo, uhi = hi;
    if (hi - lo < R && q->n_pend > 0) {
        int64_t plo = 0, phi = 0;
        RCHK(pend_range(a, &plo, &phi));
        ulo = std::min(ulo, plo);
        uhi = std::max(uhi, phi);
    }
    if (uhi - ulo < R) {
        RCHK(a->band_spare.init_band(a->band_lk, a->band_rows, ulo, a->band_mul, a->band_add));
        SH_TRACE("aggregation root: key band [%lld, %lld)", (long long)ulo, (long long)(ulo + R));
        return query_swap_keys(q, a->band_spare);
    }
    if (q->kt.lk) {
        // buckets too far apart for the band: the open-addressing table, sized for the queued keys too
        KeyTableHost nk;
        RCHK(nk.init(std::min<int64_t>(q->n_pend, (int64_t)q->kt.size_) + bound));
        SH_TRACE("aggregation root: buckets [%lld, %lld] leave the band", (long long)ulo, (long long)uhi);
        RCHK(query_swap_keys(q, nk));
    }
    return query_reserve_keys(q, bound);
}

int agg_reserve_root(sh_aggregation* a, const sh_batch* dev, bool side) {
    int64_t N = dev->n;
    if (N <= 0) return SH_OK;
    int64_t keys = a->d.n_group_by ? std::max<int64_t>(1, a->d.key_capacity > 0 ? a->d.key_capacity : (1 << 16)) : 1;
    int64_t bound = std::min(N, keys);
    if (a->has_bucket) {
        // side: a caller's device batch (ready when the call is made) is probed on the side stream, so
        // the wait does not take in the previous push's roll-up kernels still running on the compute
        // stream, and this push's kernels queue behind them without a gap
        hipStream_t s = side ? a->ctx->copy_stream : a->ctx->stream;
        launch_minmax_i64(s, (const int64_t*)dev->cols[a->d.ts_col], N, a->minmax.as<int64_t>());
        HIPCHK(hipMemcpyAsync(a->h_minmax, a->minmax.p, 16, hipMemcpyDeviceToHost, s));
        if (side) HIPCHK(sh_wait_stream(s));
        else RCHK(agg_sync(a));
        // (bucket indices are unsigned and the reference floors hours / days but truncates seconds /
        // minutes: events before 1970 are not restated)
        if (a->h_minmax[0] < 0)
            return sh_fail(SH_ERR_UNSUPPORTED, "aggregate-by timestamps before 1970 (negative) are not on the GPU");
        // the key's bucket component: ts / T truncated (sh_device.h key_part)
        const int64_t lo = a->cal ? cal_idx_h(a->h_minmax[0], a->cal, a->tz_root) : (a->h_minmax[0] + a->tz_root) / a->T_root;
        const int64_t hi = a->cal ? cal_idx_h(a->h_minmax[1], a->cal, a->tz_root) : (a->h_minmax[1] + a->tz_root) / a->T_root;
        int64_t nb = hi - lo + 1;
        bound = (nb > 0 && keys <= N / nb) ? keys * nb : N;
        if (a->band_ok) return band_reserve(a, lo, hi, bound);
    }
    return query_reserve_keys(a->root, bound);
}

// the oldest timed pushes' device time into the sum, down to `keep` still outstanding
static int ring_collect(sh_aggregation* a, int64_t keep) {
    while (a->r_next - a->r_done > keep) {
        const int k = (int)(a->r_done % sh_aggregation::kRing);
        HIPCHK(hipEventSynchronize(a->r1[k]));
        float ms = 0;
        HIPCHK(hipEventElapsedTime(&ms, a->r0[k], a->r1[k]));
        a->r_ms += ms;
        a->r_pushes++;
        a->r_done++;
    }
    return SH_OK;
}

static int agg_settle(sh_aggregation* a);
static void agg_defer(sh_aggregation* a, const sh_out* o);
static int agg_mid_hook(void* p);

static int agg_push(sh_aggregation* a, const sh_batch* b, bool host) {
    SH_TMARK(11);  // (since the previous push's last point: the caller's time between pushes)
    SH_TMARK(0);
    static const bool atrace = getenv("SH_ALLOC_TRACE") != nullptr;
    if (atrace) {
        static auto prev = std::chrono::steady_clock::now();
        const auto now = std::chrono::steady_clock::now();
        fprintf(stderr, "[sh alloc] --- push %lld (%.1f us since the previous push began)\n", (long long)a->r_next,
                std::chrono::duration<double, std::micro>(now - prev).count());
        prev = now;
    }
    const sh_out* o = nullptr;
    sh_batch dev;
    if (a->intern) {  // (the stream's own columns: the interned slot column is the aggregation's)
        if (b->n > 0)
            for (int c = 0; c < a->d.n_cols; c++)
                if ((a->root->cols_used >> c & 1) && !b->cols[c])
                    return sh_fail(SH_ERR_INVALID, "batch column " + std::to_string(c) + " is NULL but the query reads it");
    } else {
        RCHK(check_batch_cols(a->root, b));
    }
    if (host) {
        RCHK(a->root->staged.stage(a->ctx->stream, b, a->d.n_cols, a->root->d.col_types, &dev));
    } else {
        dev = *b;
    }
    if (a->intern) {
        // every passing event's group key -> its interned id, the root's synthetic dictionary column
        ColSet cs{};
        cs.n = a->d.n_cols;
        for (int c = 0; c < a->d.n_cols; c++) { cs.type[c] = a->d.col_types[c]; cs.ptr[c] = dev.cols[c]; }
        const uint32_t* ids = nullptr;
        RCHK(a->wk.intern(a->ctx->stream, cs, a->root->fp, dev.n, &ids));
        dev.cols[a->d.n_cols] = ids;
    }
    RCHK(ring_collect(a, sh_aggregation::kRing - 1));
    const int rk = (int)(a->r_next % sh_aggregation::kRing);
    if (!a->r0[rk]) {
        HIPCHK(hipEventCreate(&a->r0[rk]));
        HIPCHK(hipEventCreate(&a->r1[rk]));
    }
    HIPCHK(hipEventRecord(a->ev0, a->ctx->stream));
    HIPCHK(hipEventRecord(a->r0[rk], a->ctx->stream));
    SH_TMARK(9);
    int taken = 0;
    if (!host) RCHK(spec_push(a, &dev, &o, &taken));
    if (!taken) {
        a->pr_valid = a->pr_valid && a->root->n_pend > 0;
        RCHK(agg_reserve_root(a, &dev, !host));
        SH_TMARK(7);  // (the root's push marks 0..6 follow)
        RCHK(sh_push_device(a->root, &dev, &o));
    }
    RCHK(agg_settle(a));  // (pushes that did not reach the root's mid point: no events, small pushes)
    RCHK(agg_verify(a));  // (the root's push synchronised the stream: the last push's level checks are in)
    RCHK(pend_range_queue(a));
    agg_defer(a, o);
    SH_TMARK(8);
    // the push's end: its root work (compute stream) and its level work (level stream)
    if (a->lstream) {
        HIPCHK(hipEventRecord(a->ev_tab, a->ctx->stream));
        HIPCHK(hipStreamWaitEvent(a->lstream, a->ev_tab, 0));
    }
    HIPCHK(hipEventRecord(a->ev1, lvl(a)));
    HIPCHK(hipEventRecord(a->r1[rk], lvl(a)));
    a->r_next++;
    a->last_events = dev.n;
    a->timed = true;
    return SH_OK;
}

// Device time summed over every push since the last reset, without a wait per push: the pushes still
// running are waited for here. reset != 0 zeroes the sum after reading it.
extern "C" int sh_aggregation_timing(sh_aggregation* a, double* total_ms, int64_t* pushes, int32_t reset) {
    StreamScope _ss(a && a->ctx ? a->ctx->stream : nullptr);
    if (!a || !total_ms || !pushes) return sh_fail(SH_ERR_INVALID, "sh_aggregation_timing: NULL argument");
    if (a->dfr_on) {
        // the last push's deferred level work belongs to it: timed as part of the sum
        RCHK(ring_collect(a, sh_aggregation::kRing - 1));
        const int rk = (int)(a->r_next % sh_aggregation::kRing);
        if (!a->r0[rk]) {
            HIPCHK(hipEventCreate(&a->r0[rk]));
            HIPCHK(hipEventCreate(&a->r1[rk]));
        }
        HIPCHK(hipEventRecord(a->r0[rk], a->ctx->stream));
        RCHK(agg_settle(a));
        if (a->lstream) {
            HIPCHK(hipEventRecord(a->ev_tab, a->ctx->stream));
            HIPCHK(hipStreamWaitEvent(a->lstream, a->ev_tab, 0));
        }
        HIPCHK(hipEventRecord(a->r1[rk], lvl(a)));
        a->r_next++;
        RCHK(ring_collect(a, 0));
        a->r_pushes--;  // (the same push: its time, not another push)
    }
    RCHK(ring_collect(a, 0));
    *total_ms = a->r_ms;
    *pushes = a->r_pushes;
    if (reset) {
        a->r_ms = 0;
        a->r_pushes = 0;
    }
    return SH_OK;
}

// Device time of the last push: the whole pipeline (root window + every roll-up level) and the
// root's aggregation kernel (IncrementalExecutor's base aggregation over the raw events).
extern "C" int sh_aggregation_stats(sh_aggregation* a, sh_stats* out) {
    StreamScope _ss(a && a->ctx ? a->ctx->stream : nullptr);
    if (!a || !out) return sh_fail(SH_ERR_INVALID, "sh_aggregation_stats: NULL argument");
    if (a->lstream) HIPCHK(hipStreamSynchronize(a->lstream));  // (the level stream's tables / states)
    *out = sh_stats{};
    if (!a->timed) return SH_OK;
    HIPCHK(hipEventSynchronize(a->ev1));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, a->ev0, a->ev1));
    sh_stats rs{};
    RCHK(sh_query_stats(a->root, &rs));
    out->push_ms = ms;
    out->main_kernel_ms = rs.main_kernel_ms;
    out->main_kernel_bytes = rs.main_kernel_bytes;
    out->events = a->last_events;
    return SH_OK;
}

static int after_root_core(sh_aggregation* a, const sh_out* o, const int64_t* windows, int64_t clock) {
    if (o->n_rows > (8 << 20) / 8 && a->d.n_group_by == 0)
        return sh_fail(SH_ERR_UNSUPPORTED, "too many rows in one flush for a constant key column");
    if (!a->root_init && a->root->e0_valid) {
        a->root_init = true;
        a->root_bucket = root_shift(a, a->root->E0, -1);
        if (!a->levels.empty()) RCHK(level_timer(a, 0, a->root_bucket));
    }
    RCHK(pass_root_flushes(a, o, windows));
    RCHK(catch_up(a, clock));
    // the merged levels' key-table counters, verified after the next synchronisation (agg_verify)
    for (auto& L : a->levels) {
        if (!L.dirty) continue;
        RCHK(L.kt.check_async(lvl(a), L.chk));
        L.dirty = false;
        a->chk_pending = true;
    }
    if (a->chk_pending) HIPCHK(hipEventRecord(a->ev_lchk, lvl(a)));
    return SH_OK;
}

int agg_after_root(sh_aggregation* a, const sh_out* o) {
    return after_root_core(a, o, a->root->flush_window.data(), a->root->clock);
}

// A push's root flushes are handed to the roll-up levels (host logic + the table / level launches, a few
// hundred microseconds of host time) while the NEXT push's first kernels run: the root query calls
// back here just before it waits for its boundaries (sh_query.mid_hook). The flushes' rows stay in the
// root's output buffers until then: the next push writes them only after this work is queued ahead on
// the same stream. Every other entry point runs the deferred work first (agg_settle).
static int agg_settle(sh_aggregation* a) {
    if (!a->dfr_on) return SH_OK;
    a->dfr_on = false;
    return after_root_core(a, &a->dfr_out, a->dfr_windows.data(), a->dfr_clock);
}
static int agg_mid_hook(void* p) { return agg_settle((sh_aggregation*)p); }
static void agg_defer(sh_aggregation* a, const sh_out* o) {
    a->dfr_out = *o;
    a->dfr_offs.assign(o->flush_offsets, o->flush_offsets + o->n_flushes + 1);
    a->dfr_out.flush_offsets = a->dfr_offs.data();
    a->dfr_out.flush_clock = nullptr;
    a->dfr_windows.assign(a->root->flush_window.begin(), a->root->flush_window.end());
    a->dfr_clock = a->root->clock;
    a->dfr_on = true;
}

extern "C" int sh_aggregation_push(sh_aggregation* a, const sh_batch* b) {
    SH_RANGE("sh_aggregation_push");
    StreamScope _ss(a && a->ctx ? a->ctx->stream : nullptr);
    if (!a || !b) return sh_fail(SH_ERR_INVALID, "sh_aggregation_push: NULL argument");
    if (a->shard) return sh_fail(SH_ERR_STATE, "a sharded aggregation ingests through sh_shard_*");
    return agg_push(a, b, true);
}

extern "C" int sh_aggregation_push_device(sh_aggregation* a, const sh_batch* b) {
    SH_RANGE("sh_aggregation_push_device");
    StreamScope _ss(a && a->ctx ? a->ctx->stream : nullptr);
    if (!a || !b) return sh_fail(SH_ERR_INVALID, "sh_aggregation_push_device: NULL argument");
    if (a->shard) return sh_fail(SH_ERR_STATE, "a sharded aggregation ingests through sh_shard_*");
    return agg_push(a, b, false);
}



extern "C" int sh_aggregation_advance_time(sh_aggregation* a, int64_t now) {
    SH_RANGE("sh_aggregation_advance_time");
    StreamScope _ss(a && a->ctx ? a->ctx->stream : nullptr);
    if (!a) return sh_fail(SH_ERR_INVALID, "sh_aggregation_advance_time: NULL argument");
    if (a->shard) return sh_fail(SH_ERR_STATE, "a sharded aggregation advances through sh_shard_advance_time");
    const sh_out* o = nullptr;
    RCHK(agg_settle(a));
    a->pr_valid = false;  // (the TIMER may flush the queued events)
    RCHK(sh_advance_time_device(a->root, now, &o));
    RCHK(pass_root_flushes(a, o, a->root->flush_window.data()));
    RCHK(catch_up(a, a->root->clock));
    // the merged levels' key-table counters, verified after the next synchronisation (agg_verify)
    for (auto& L : a->levels) {
        if (!L.dirty) continue;
        RCHK(L.kt.check_async(lvl(a), L.chk));
        L.dirty = false;
        a->chk_pending = true;
    }
    if (a->chk_pending) HIPCHK(hipEventRecord(a->ev_lchk, lvl(a)));
    return SH_OK;
}

// the group-by columns of n table / retrieval rows (device keys) into host memory ([column][n]); interned
// keys are mapped back to their values on the device first
static int agg_keys_out(sh_aggregation* a, const int64_t* keys, int64_t n, int64_t* host) {
    hipStream_t s = a->ctx->stream;
    if (!a->intern) {
        HIPCHK(hipMemcpyAsync(host, keys, n * 8, hipMemcpyDeviceToHost, s));
        return SH_OK;
    }
    const int ng = a->d.n_group_by;
    RCHK(a->dkeys.reserve((size_t)ng * n * 8, false));
    RCHK(a->wk.decode(s, keys, n, a->dkeys.as<int64_t>()));
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(host, a->dkeys.p, (size_t)ng * n * 8, hipMemcpyDeviceToHost, s));
    return SH_OK;
}

extern "C" int sh_aggregation_table(sh_aggregation* a, int32_t dur, const sh_out** out) {
    SH_RANGE("sh_aggregation_table");
    StreamScope _ss(a && a->ctx ? a->ctx->stream : nullptr);
    if (!a || !out) return sh_fail(SH_ERR_INVALID, "sh_aggregation_table: NULL argument");
    RCHK(agg_settle(a));
    if (a->lstream) HIPCHK(hipStreamSynchronize(a->lstream));  // (the level stream's tables / states)
    if (dur < a->d.min_duration || dur > a->d.max_duration) return sh_fail(SH_ERR_INVALID, "duration not aggregated");
    TableBuf& t = a->tables[dur];
    hipStream_t s = a->ctx->stream;
    OutHost& o = a->tout;
    o.reset();
    const int64_t r0 = t.drained;
    int64_t n = t.n - r0;
    int nk = 1 + a->d.n_group_by;
    o.ts.resize(n);
    o.expired.assign(n, 0);
    o.keys.resize((size_t)nk * n);
    o.vals.resize((size_t)a->nb * n);
    o.nulls.assign((size_t)a->nb * n, 0);
    if (n) {
        HIPCHK(hipMemcpyAsync(o.ts.data(), t.bucket.as<int64_t>() + r0, n * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(o.keys.data(), t.bucket.as<int64_t>() + r0, n * 8, hipMemcpyDeviceToHost, s));
        if (nk > 1) RCHK(agg_keys_out(a, t.key.as<int64_t>() + r0, n, o.keys.data() + n));
        for (int b = 0; b < a->nb; b++)
            HIPCHK(hipMemcpyAsync(o.vals.data() + (size_t)b * n, t.vals.as<u64>() + (size_t)b * t.cap + r0, n * 8,
                                  hipMemcpyDeviceToHost, s));
        RCHK(agg_sync(a));
        o.flush_offsets.push_back(n);
        o.flush_clock.push_back(a->root->clock);
    }
    t.drained = t.n;
    o.view(nk, a->nb, a->btypes);
    o.out.rep = nullptr;  // table rows have no representative event
    *out = &o.out;
    return SH_OK;
}

// ---- retrieval: `from A within start, end per "<per>"` (AggregationRuntime.find ->
// IncrementalAggregateCompileCondition.find :180-290) ---------------------------------------------
// The rows of the `per` table plus the in-memory stores of the executors `per` .. root
// (IncrementalDataAggregator.aggregateInMemoryData :92-143: re-bucketed to `per` and folded per
// (bucket, key) in executor order), merged with the table rows by (AGG_TIMESTAMP, key)
// (OutOfOrderEventsDataAggregator: table rows first), restricted to start <= AGG_TIMESTAMP < end.
// Rows come out in (AGG_TIMESTAMP, key) order (the reference's order is a HashMap's).

// rows (bucket at their own duration, key, vals [nb][vstride]) -> grouped by (`per` bucket, key) in
// (bucket, key) order, each group's rows folded in input order; rows outside [start, end) dropped
static int group_fold(sh_aggregation* a, const int64_t* bucket, const int64_t* key, const u64* vals, int64_t n,
                      int64_t vstride, int per, int64_t start, int64_t end, DevBuf& ob, DevBuf& ok, DevBuf& ov,
                      int64_t* n_out) {
    *n_out = 0;
    if (n <= 0) return SH_OK;
    hipStream_t s = a->ctx->stream;
    RCHK(a->g_bucket.reserve(n * 8, false));
    RCHK(a->g_idx.reserve(n * 4, false));
    RCHK(a->g_k64.reserve(n * 8, false));
    RCHK(a->g_k64s.reserve(n * 8, false));
    RCHK(a->g_idx1.reserve(n * 4, false));
    RCHK(a->g_idx2.reserve(n * 4, false));
    RCHK(a->g_flag.reserve((n + 1) * 4, false));
    RCHK(a->g_pre.reserve((n + 1) * 4, false));
    RCHK(a->g_tmp.reserve((size_t)((n + 1 + kTile - 1) / kTile + 16) * 8, false));
    launch_find_rebucket(s, n, bucket, per, start, end, a->g_bucket.as<int64_t>(), a->g_idx.as<u32>(), a->tz);
    // (bucket, key) order, input order within a group: stable LSD sorts by key, then by bucket. Interned
    // keys sort by their group-by values (signed, last column first), not by their slots
    size_t tb = 0;
    if (sort_u64_pairs(nullptr, &tb, nullptr, nullptr, nullptr, nullptr, n, s)) return sh_fail(SH_ERR_DEVICE, "sort sizing");
    RCHK(a->g_sort.reserve(std::max<size_t>(tb, 16), false));
    u32* idx[3] = {a->g_idx.as<u32>(), a->g_idx1.as<u32>(), a->g_idx2.as<u32>()};
    int c = 0;
    auto pass = [&](const int64_t* src, u64 flip) -> int {
        launch_find_gather_u64(s, n, idx[c], src, a->g_k64.as<u64>(), flip);
        if (sort_u64_pairs(a->g_sort.p, &tb, a->g_k64.as<u64>(), a->g_k64s.as<u64>(), idx[c], idx[(c + 1) % 3], n, s))
            return sh_fail(SH_ERR_DEVICE, "retrieval sort failed");
        c = (c + 1) % 3;
        return SH_OK;
    };
    if (a->intern) {
        const int ng = a->d.n_group_by;
        RCHK(a->g_dk.reserve((size_t)ng * n * 8, false));
        RCHK(a->wk.decode(s, key, n, a->g_dk.as<int64_t>()));
        for (int x = ng - 1; x >= 0; x--) RCHK(pass(a->g_dk.as<int64_t>() + (size_t)x * n, 1ull << 63));
    } else {
        RCHK(pass(key, 0));
    }
    RCHK(pass(a->g_bucket.as<int64_t>(), 0));
    if (c != 2) HIPCHK(hipMemcpyAsync(idx[2], idx[c], n * 4, hipMemcpyDeviceToDevice, s));
    launch_find_starts(s, n, a->g_idx2.as<u32>(), a->g_bucket.as<int64_t>(), key, a->g_flag.as<u32>());
    HIPCHK(hipMemcpyAsync(a->g_pre.p, a->g_flag.p, (n + 1) * 4, hipMemcpyDeviceToDevice, s));
    launch_scan_sum_large_u32(s, a->g_pre.as<u32>(), n + 1, a->g_tmp.as<int64_t>());
    uint32_t groups = 0;
    HIPCHK(hipMemcpyAsync(a->h_minmax, a->g_pre.as<u32>() + n, 4, hipMemcpyDeviceToHost, s));
    RCHK(agg_sync(a));
    std::memcpy(&groups, a->h_minmax, 4);
    const int64_t cap = std::max<int64_t>(groups, 1);
    RCHK(ob.reserve(cap * 8, false));
    RCHK(ok.reserve(cap * 8, false));
    RCHK(ov.reserve((size_t)a->nb * cap * 8, false));
    launch_find_fold(s, n, a->g_idx2.as<u32>(), a->g_flag.as<u32>(), a->g_pre.as<u32>(), a->g_bucket.as<int64_t>(), key,
                     vals, vstride, a->bp, cap, ob.as<int64_t>(), ok.as<int64_t>(), ov.as<u64>());
    HIPCHK(hipGetLastError());
    *n_out = groups;
    return SH_OK;
}

extern "C" int sh_aggregation_find(sh_aggregation* a, int32_t per, int64_t start, int64_t end, const sh_out** out) {
    SH_RANGE("sh_aggregation_find");
    StreamScope _ss(a && a->ctx ? a->ctx->stream : nullptr);
    if (!a || !out) return sh_fail(SH_ERR_INVALID, "sh_aggregation_find: NULL argument");
    RCHK(agg_settle(a));
    if (a->lstream) HIPCHK(hipStreamSynchronize(a->lstream));  // (the level stream's tables / states)
    if (per < a->d.min_duration || per > a->d.max_duration)
        return sh_fail(SH_ERR_INVALID, "the aggregation does not contain the `per` duration");
    hipStream_t s = a->ctx->stream;
    const int nb = a->nb;
    // in-memory rows, executors `per` down to the root: sizes first
    std::vector<int64_t> level_n;
    int64_t total = 0;
    for (int dur = per; dur > a->d.min_duration; dur--) {
        Level& L = a->levels[dur - a->d.min_duration - 1];
        level_n.push_back(L.processed ? L.n_in : 0);
        total += level_n.back();
    }
    int64_t root_rows = 0;
    RCHK(query_peek(a->root, &root_rows));
    total += root_rows;
    const int64_t mcap = std::max<int64_t>(total, 1);
    RCHK(a->m_bucket.reserve(mcap * 8, false));
    RCHK(a->m_key.reserve(mcap * 8, false));
    RCHK(a->m_vals.reserve((size_t)nb * mcap * 8, false));
    int64_t m = 0;
    for (size_t i = 0; i < level_n.size(); i++) {
        const int dur = per - (int)i;
        Level& L = a->levels[dur - a->d.min_duration - 1];
        const int64_t n_in = level_n[i];
        if (n_in == 0) continue;
        // the store's entries in first-arrival order (its insertion order), left in place
        const int nblk = (int)((n_in + kTile - 1) / kTile);
        RCHK(L.blk.reserve((nblk + 8) * 8, false));
        RCHK(L.order.reserve(n_in * 4, false));
        LevelDev D = level_dev(L, nb);
        launch_level_mark(s, D, n_in, false);
        launch_level_count(s, D, n_in, L.blk.as<int64_t>(), nblk);
        std::vector<int64_t> bc(nblk);
        HIPCHK(hipMemcpyAsync(bc.data(), L.blk.p, nblk * 8, hipMemcpyDeviceToHost, s));
        RCHK(agg_sync(a));
        int64_t entries = 0;  // distinct (bucket, key) slots; rows merged into one slot count once
        for (auto c : bc) entries += c;
        launch_scan_sum(s, L.blk.as<int64_t>(), nblk);
        launch_level_extract(s, D, a->bp, a->has_bucket, L.store_ts, n_in, L.blk.as<int64_t>(), nblk, mcap,
                             a->m_bucket.as<int64_t>() + m, a->m_key.as<int64_t>() + m, a->m_vals.as<u64>() + m, false);
        HIPCHK(hipGetLastError());
        m += entries;
    }
    if (root_rows > 0) {
        sh_query* q = a->root;
        const int64_t R = root_rows;
        const int nk = q->kp.n;
        const int64_t* keys = q->out_keys.as<int64_t>();
        if (a->has_bucket) {
            HIPCHK(hipMemcpyAsync(a->m_bucket.as<int64_t>() + m, keys, R * 8, hipMemcpyDeviceToDevice, s));
            if (nk > 1) HIPCHK(hipMemcpyAsync(a->m_key.as<int64_t>() + m, keys + R, R * 8, hipMemcpyDeviceToDevice, s));
            else HIPCHK(hipMemsetAsync(a->m_key.as<int64_t>() + m, 0, R * 8, s));
        } else {
            // processing time: AGG_TIMESTAMP of the root store = the open window's start
            launch_fill_i64(s, a->m_bucket.as<int64_t>() + m, R, root_window_start(a, q->W_open));
            if (nk > 0) HIPCHK(hipMemcpyAsync(a->m_key.as<int64_t>() + m, keys, R * 8, hipMemcpyDeviceToDevice, s));
            else HIPCHK(hipMemsetAsync(a->m_key.as<int64_t>() + m, 0, R * 8, s));
        }
        for (int b = 0; b < nb; b++)
            HIPCHK(hipMemcpyAsync(a->m_vals.as<u64>() + (size_t)b * mcap + m, q->out_vals.as<u64>() + (size_t)b * R, R * 8,
                                  hipMemcpyDeviceToDevice, s));
        m += R;
    }
    // in-memory values per (`per` bucket, key): IncrementalDataAggregator
    int64_t nv = 0;
    RCHK(group_fold(a, a->m_bucket.as<int64_t>(), a->m_key.as<int64_t>(), a->m_vals.as<u64>(), m, mcap, per, INT64_MIN,
                    INT64_MAX, a->v_bucket, a->v_key, a->v_vals, &nv));
    // the `per` table's rows first, then the in-memory values: OutOfOrderEventsDataAggregator
    TableBuf& t = a->tables[per];
    const int64_t n2 = t.n + nv, cap2 = std::max<int64_t>(n2, 1);
    RCHK(a->f_bucket.reserve(cap2 * 8, false));
    RCHK(a->f_key.reserve(cap2 * 8, false));
    RCHK(a->f_vals.reserve((size_t)nb * cap2 * 8, false));
    if (t.n) {
        HIPCHK(hipMemcpyAsync(a->f_bucket.p, t.bucket.p, t.n * 8, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(a->f_key.p, t.key.p, t.n * 8, hipMemcpyDeviceToDevice, s));
        for (int b = 0; b < nb; b++)
            HIPCHK(hipMemcpyAsync(a->f_vals.as<u64>() + (size_t)b * cap2, t.vals.as<u64>() + (size_t)b * t.cap, t.n * 8,
                                  hipMemcpyDeviceToDevice, s));
    }
    if (nv) {
        HIPCHK(hipMemcpyAsync(a->f_bucket.as<int64_t>() + t.n, a->v_bucket.p, nv * 8, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(a->f_key.as<int64_t>() + t.n, a->v_key.p, nv * 8, hipMemcpyDeviceToDevice, s));
        const int64_t vcap = std::max<int64_t>(nv, 1);
        for (int b = 0; b < nb; b++)
            HIPCHK(hipMemcpyAsync(a->f_vals.as<u64>() + (size_t)b * cap2 + t.n, a->v_vals.as<u64>() + (size_t)b * vcap,
                                  nv * 8, hipMemcpyDeviceToDevice, s));
    }
    int64_t nr = 0;
    RCHK(group_fold(a, a->f_bucket.as<int64_t>(), a->f_key.as<int64_t>(), a->f_vals.as<u64>(), n2, cap2, per, start, end,
                    a->v_bucket, a->v_key, a->v_vals, &nr));
    // host rows: AGG_TIMESTAMP, [key], base values (as sh_aggregation_table)
    OutHost& o = a->fout;
    o.reset();
    const int nk = 1 + a->d.n_group_by;
    o.ts.resize(nr);
    o.expired.assign(nr, 0);
    o.keys.resize((size_t)nk * nr);
    o.vals.resize((size_t)nb * nr);
    o.nulls.assign((size_t)nb * nr, 0);
    if (nr) {
        const int64_t vcap = std::max<int64_t>(nr, 1);
        HIPCHK(hipMemcpyAsync(o.ts.data(), a->v_bucket.p, nr * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipMemcpyAsync(o.keys.data(), a->v_bucket.p, nr * 8, hipMemcpyDeviceToHost, s));
        if (nk > 1) RCHK(agg_keys_out(a, a->v_key.as<int64_t>(), nr, o.keys.data() + nr));
        for (int b = 0; b < nb; b++)
            HIPCHK(hipMemcpyAsync(o.vals.data() + (size_t)b * nr, a->v_vals.as<u64>() + (size_t)b * vcap, nr * 8,
                                  hipMemcpyDeviceToHost, s));
        RCHK(agg_sync(a));
        o.flush_offsets.push_back(nr);
        o.flush_clock.push_back(a->root->clock);
    }
    o.view(nk, nb, a->btypes);
    o.out.rep = nullptr;
    *out = &o.out;
    return SH_OK;
}

// ---- checkpoint: State.snapshot()/restore() of an aggregation (SnapshotService.persist/restore,
// core/util/snapshot/SnapshotService.java:90-296) — the root window (its sh_query snapshot), every
// roll-up executor's ExecutorState (IncrementalExecutor.java:283-317: nextEmitTime,
// startTimeOfAggregates) and BaseIncrementalValueStore (:231-262: store timestamp, processed flag,
// the per-(bucket, key) base values), and the duration tables. A restored aggregation continues
// exactly as the snapshotted one (same tables, same retrievals). --------------------------------------
namespace {
struct ABlob {
    std::vector<uint8_t> b;
    template <typename T> void val(const T& x) { b.insert(b.end(), (const uint8_t*)&x, (const uint8_t*)&x + sizeof(T)); }
    int dev(const void* d, size_t n, hipStream_t s) {
        val<uint64_t>(n);
        size_t o = b.size();
        b.resize(o + n);
        if (n && (hipMemcpyAsync(b.data() + o, d, n, hipMemcpyDeviceToHost, s) != hipSuccess ||
                  hipStreamSynchronize(s) != hipSuccess))
            return sh_fail(SH_ERR_DEVICE, "aggregation snapshot: device read failed");
        return SH_OK;
    }
};
struct AReader {
    const uint8_t* p;
    size_t n, o = 0;
    bool ok = true;
    template <typename T> T val() {
        T x{};
        if (o + sizeof(T) > n) { ok = false; return x; }
        std::memcpy(&x, p + o, sizeof(T));
        o += sizeof(T);
        return x;
    }
    // a device section of exactly `want` bytes into d (-1: any length, returned in *got)
    int dev(void* d, int64_t want, hipStream_t s, uint64_t* got = nullptr) {
        const uint64_t len = val<uint64_t>();
        if (!ok || o + len > n || (want >= 0 && (uint64_t)want != len)) {
            ok = false;
            return sh_fail(SH_ERR_INVALID, "aggregation snapshot does not match this aggregation");
        }
        if (got) *got = len;
        if (len && (hipMemcpyAsync(d, p + o, len, hipMemcpyHostToDevice, s) != hipSuccess ||
                    hipStreamSynchronize(s) != hipSuccess))
            return sh_fail(SH_ERR_DEVICE, "aggregation restore: device write failed");
        o += len;
        return SH_OK;
    }
};
uint64_t agg_fingerprint(const sh_aggregation* a) {
    const sh_aggregation_desc& d = a->d;
    uint64_t h = 1469598103934665603ull;
    auto mix = [&](const void* p, size_t n) {
        for (size_t i = 0; i < n; i++) h = (h ^ ((const uint8_t*)p)[i]) * 1099511628211ull;
    };
    int32_t ints[] = {d.n_cols, d.n_group_by, d.n_aggs, d.ts_col, d.min_duration, d.max_duration, d.n_filter_ops};
    mix(ints, sizeof(ints));
    mix(d.col_types, sizeof(int32_t) * d.n_cols);
    mix(d.group_by, sizeof(int32_t) * d.n_group_by);
    mix(d.aggs, sizeof(sh_agg_spec) * d.n_aggs);
    mix(&d.key_capacity, 8);
    return h;
}
constexpr uint32_t kAggSnapVersion = 2;  // 2: level stores as [slot][base + has-mask] records
}  // namespace

static int agg_state_write(sh_aggregation* a, ABlob& w);
static int agg_state_read(sh_aggregation* a, AReader& r);

static int agg_snapshot_blob(sh_aggregation* a, ABlob& w) {
    w.b.insert(w.b.end(), {'S', 'H', 'A', '1'});
    w.val<uint32_t>(kAggSnapVersion);
    w.val<uint64_t>(agg_fingerprint(a));
    // the root window
    int64_t rl = 0;
    RCHK(sh_query_snapshot(a->root, nullptr, 0, &rl));
    std::vector<uint8_t> rb((size_t)rl);
    RCHK(sh_query_snapshot(a->root, rb.data(), rl, &rl));
    w.val<int64_t>(rl);
    w.b.insert(w.b.end(), rb.begin(), rb.end());
    return agg_state_write(a, w);
}

// Everything of an aggregation beyond its root window: the root bucket cursor, the roll-up executors
// and the duration tables (the sharded form appends this to the shard's blob).
static int agg_state_write(sh_aggregation* a, ABlob& w) {
    hipStream_t s = a->ctx->stream;
    w.val<uint8_t>(a->root_init);
    w.val<int64_t>(a->root_bucket);
    // roll-up executors
    w.val<uint32_t>((uint32_t)a->levels.size());
    for (Level& L : a->levels) {
        w.val<int64_t>(L.next_emit);
        w.val<int64_t>(L.start);
        w.val<int64_t>(L.store_ts);
        w.val<uint8_t>(L.processed);
        w.val<int64_t>(L.n_in);
        w.val<uint32_t>(L.epoch);
        w.val<uint64_t>(L.kt.size_);
        RCHK(L.kt.check(s));
        w.val<int64_t>(L.kt.n_keys);
        RCHK(w.dev(L.kt.keys.p, L.kt.size_ * 8, s));
        RCHK(w.dev(L.vals.p, (size_t)(a->nb + 1) * L.nslots * 8, s));
        RCHK(w.dev(L.tag.p, (size_t)L.nslots * 4, s));
        RCHK(w.dev(L.first_seq.p, (size_t)L.nslots * 4, s));
    }
    // duration tables (every row: retrievals read the whole table) and their drain cursors
    for (int dur = a->d.min_duration; dur <= a->d.max_duration; dur++) {
        TableBuf& t = a->tables[dur];
        w.val<int64_t>(t.n);
        w.val<int64_t>(t.drained);
        RCHK(w.dev(t.bucket.p, t.n * 8, s));
        RCHK(w.dev(t.key.p, t.n * 8, s));
        for (int b = 0; b < a->nb; b++) RCHK(w.dev(t.vals.as<u64>() + (size_t)b * t.cap, t.n * 8, s));
    }
    if (a->intern) {  // the interned group keys (their ids are the root's and the tables' keys)
        std::vector<uint8_t> kb;
        RCHK(a->wk.save(kb, s));
        w.val<uint64_t>(kb.size());
        w.b.insert(w.b.end(), kb.begin(), kb.end());
    }
    return SH_OK;
}

extern "C" int sh_aggregation_snapshot(sh_aggregation* a, void* buf, int64_t cap, int64_t* len) {
    SH_RANGE("sh_aggregation_snapshot");
    StreamScope _ss(a && a->ctx ? a->ctx->stream : nullptr);
    if (!a || !len) return sh_fail(SH_ERR_INVALID, "sh_aggregation_snapshot: NULL argument");
    RCHK(agg_settle(a));
    if (a->lstream) HIPCHK(hipStreamSynchronize(a->lstream));  // (the level stream's tables / states)
    if (a->shard) return sh_fail(SH_ERR_UNSUPPORTED, "a sharded aggregation is checkpointed by sh_shard_snapshot");
    ABlob w;
    RCHK(agg_snapshot_blob(a, w));
    *len = (int64_t)w.b.size();
    if (buf) {
        if (cap < *len) return sh_fail(SH_ERR_INVALID, "sh_aggregation_snapshot: buffer too small (call with buf=NULL for the size)");
        std::memcpy(buf, w.b.data(), w.b.size());
    }
    return SH_OK;
}

static int agg_restore_blob(sh_aggregation* a, const void* buf, int64_t len) {
    if (len < 20 || std::memcmp(buf, "SHA1", 4) != 0) return sh_fail(SH_ERR_INVALID, "not a siddhi_hip aggregation snapshot");
    hipStream_t s = a->ctx->stream;
    AReader r{(const uint8_t*)buf, (size_t)len};
    r.o = 4;
    if (r.val<uint32_t>() != kAggSnapVersion) return sh_fail(SH_ERR_INVALID, "snapshot version mismatch");
    if (r.val<uint64_t>() != agg_fingerprint(a)) return sh_fail(SH_ERR_INVALID, "snapshot was taken from a different aggregation");
    const int64_t rl = r.val<int64_t>();
    if (!r.ok || rl <= 0 || r.o + (size_t)rl > r.n) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    (void)hipStreamSynchronize(s);
    a->pr_valid = false;
    RCHK(sh_query_restore(a->root, r.p + r.o, rl));
    r.o += (size_t)rl;
    return agg_state_read(a, r);
}

static int agg_state_read(sh_aggregation* a, AReader& r) {
    hipStream_t s = a->ctx->stream;
    a->root_init = r.val<uint8_t>();
    a->root_bucket = r.val<int64_t>();
    if (r.val<uint32_t>() != (uint32_t)a->levels.size() || !r.ok)
        return sh_fail(SH_ERR_INVALID, "snapshot does not match this aggregation");
    for (Level& L : a->levels) {
        L.next_emit = r.val<int64_t>();
        L.start = r.val<int64_t>();
        L.store_ts = r.val<int64_t>();
        L.processed = r.val<uint8_t>();
        L.n_in = r.val<int64_t>();
        L.epoch = r.val<uint32_t>();
        const uint64_t ks = r.val<uint64_t>();
        const int64_t nk = r.val<int64_t>();
        if (!r.ok || ks != L.kt.size_) return sh_fail(SH_ERR_INVALID, "snapshot does not match this aggregation");
        RCHK(r.dev(L.kt.keys.p, (int64_t)ks * 8, s));
        // the key table's insert counter (stream-ordered, from pinned memory)
        RCHK(L.kt.h_ctrl.reserve(16));
        uint32_t* c = L.kt.h_ctrl.as<uint32_t>();
        c[0] = (uint32_t)nk; c[1] = c[2] = c[3] = 0;
        HIPCHK(hipMemcpyAsync(L.kt.ctrl.p, c, 16, hipMemcpyHostToDevice, s));
        HIPCHK(hipStreamSynchronize(s));
        L.kt.n_keys = nk;
        RCHK(r.dev(L.vals.p, (int64_t)(a->nb + 1) * L.nslots * 8, s));
        RCHK(r.dev(L.tag.p, L.nslots * 4, s));
        RCHK(r.dev(L.first_seq.p, L.nslots * 4, s));
    }
    for (int dur = a->d.min_duration; dur <= a->d.max_duration; dur++) {
        TableBuf& t = a->tables[dur];
        const int64_t n = r.val<int64_t>(), drained = r.val<int64_t>();
        if (!r.ok || n < 0 || drained < 0 || drained > n) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        const int64_t ncap = std::max<int64_t>(n, 1024);
        if (ncap > t.cap) {
            DevBuf b2, k2, v2;
            RCHK(b2.reserve(ncap * 8, false));
            RCHK(k2.reserve(ncap * 8, false));
            RCHK(v2.reserve((size_t)a->nb * ncap * 8, false));
            t.bucket = std::move(b2); t.key = std::move(k2); t.vals = std::move(v2);
            t.cap = ncap;
        }
        RCHK(r.dev(t.bucket.p, n * 8, s));
        RCHK(r.dev(t.key.p, n * 8, s));
        for (int b = 0; b < a->nb; b++) RCHK(r.dev(t.vals.as<u64>() + (size_t)b * t.cap, n * 8, s));
        t.n = n;
        t.drained = drained;
    }
    if (a->intern) {
        const uint64_t kn = r.val<uint64_t>();
        if (!r.ok || r.o + kn > r.n) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        size_t off = 0;
        RCHK(a->wk.load(r.p + r.o, (size_t)kn, off, s));
        r.o += kn;
    }
    if (!r.ok) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    return SH_OK;
}

// The sharded aggregation's sections after the shard's blob (sh_snapshot.cpp shard_snapshot_blob):
// the aggregation's fingerprint, then agg_state_write's sections.
int agg_shard_state_write(sh_aggregation* a, std::vector<uint8_t>& out) {
    if (a->lstream) HIPCHK(hipStreamSynchronize(a->lstream));  // (the level stream's tables / states)
    ABlob w;
    w.val<uint64_t>(agg_fingerprint(a));
    RCHK(agg_state_write(a, w));
    out = std::move(w.b);
    return SH_OK;
}

int agg_shard_state_read(sh_aggregation* a, const uint8_t* p, size_t n) {
    if (a->lstream) HIPCHK(hipStreamSynchronize(a->lstream));  // (the level stream's tables / states)
    AReader r{p, n};
    if (r.val<uint64_t>() != agg_fingerprint(a) || !r.ok)
        return sh_fail(SH_ERR_INVALID, "snapshot was taken from a different aggregation");
    a->chk_pending = false;
    return agg_state_read(a, r);
}

// All or nothing: the aggregation's current state is snapshotted first and put back when the blob
// fails part-way (the root window, an executor or a table section), keeping the first error.
extern "C" int sh_aggregation_restore(sh_aggregation* a, const void* buf, int64_t len) {
    SH_RANGE("sh_aggregation_restore");
    StreamScope _ss(a && a->ctx ? a->ctx->stream : nullptr);
    if (!a || !buf || len < 20) return sh_fail(SH_ERR_INVALID, "sh_aggregation_restore: bad arguments");
    RCHK(agg_settle(a));
    if (a->lstream) HIPCHK(hipStreamSynchronize(a->lstream));  // (the level stream's tables / states)
    if (a->shard) return sh_fail(SH_ERR_UNSUPPORTED, "a sharded aggregation is restored by sh_shard_restore");
    ABlob backup;
    const bool have = agg_snapshot_blob(a, backup) == SH_OK;
    const int rc = agg_restore_blob(a, buf, len);
    if (rc != SH_OK && have) {
        const std::string msg = sh_last_error();
        (void)agg_restore_blob(a, backup.b.data(), (int64_t)backup.b.size());
        return sh_fail(rc, msg);
    }
    return rc;
}
