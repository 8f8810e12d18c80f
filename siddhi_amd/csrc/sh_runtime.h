// sh_runtime.h — host-side objects behind the C ABI (not part of the public interface).
#pragma once

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cstdio>
#include <new>
#include <utility>
#include <string>
#include <unordered_map>
#include <vector>

#include "sh_internal.h"

struct sh_ctx {
    int device = 0;
    int num_cus = 0;
    int max_lds = 0;
    hipStream_t stream = nullptr;
    hipStream_t copy_stream = nullptr;  // H2D staging of host batches (sh_stage), beside the compute stream
};

int sh_fail(int code, const std::string& msg);

// SH_TRACE=1 in the environment: one stderr line per pipeline step (diagnostics only)
bool sh_trace_on();
#define SH_TRACE(...)                                    \
    do {                                                 \
        if (sh_trace_on()) {                             \
            fprintf(stderr, "[sh] " __VA_ARGS__);        \
            fputc('\n', stderr);                         \
            fflush(stderr);                              \
        }                                                \
    } while (0)

// SH_TIMING=1 in the environment: host-side time between numbered points of a push, accumulated and
// printed to stderr at exit (diagnostics only; one clock read per point otherwise skipped)
bool sh_timing_on();
void sh_timing_mark(int point);
#define SH_TMARK(p)                          \
    do {                                     \
        if (sh_timing_on()) sh_timing_mark(p); \
    } while (0)

// Waits that poll the stream / event instead of sleeping in the driver: a push waits for work that
// completes within a millisecond or two, and a blocking wait's wake-up adds tens of microseconds to
// every push. After ~20 ms of polling they fall back to the blocking call.
hipError_t sh_wait_stream(hipStream_t s);
hipError_t sh_wait_event(hipEvent_t e);

// A roctx range around every data-path C-ABI call (rocprofv3 --marker-trace shows the calls next to
// their kernels; without a profiler attached a push/pop is a table lookup in librocprofiler-sdk-roctx).
struct ShRange {
    explicit ShRange(const char* n) { roctxRangePush(n); }
    ~ShRange() { roctxRangePop(); }
    ShRange(const ShRange&) = delete;
    ShRange& operator=(const ShRange&) = delete;
};
#define SH_RANGE(name) ShRange _sh_range(name)

// The stream of the context whose API call is running on this thread. A device buffer's growth or
// release drains that stream before the old block is freed, so no queued kernel or copy still reads
// it (DevBuf::reserve). Every extern "C" entry point that touches a context opens a StreamScope.
extern thread_local hipStream_t g_stream;
struct StreamScope {
    hipStream_t prev;
    explicit StreamScope(hipStream_t s) : prev(g_stream) { g_stream = s; }
    ~StreamScope() { g_stream = prev; }
    StreamScope(const StreamScope&) = delete;
    StreamScope& operator=(const StreamScope&) = delete;
};

// Growable device allocation (move-only; released on destruction, so early error returns do not
// leak). `used` is the byte count that must survive a grow (keep=true).
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    size_t used = 0;
    DevBuf() = default;
    DevBuf(const DevBuf&) = delete;
    DevBuf& operator=(const DevBuf&) = delete;
    DevBuf(DevBuf&& o) noexcept : p(o.p), cap(o.cap), used(o.used) { o.p = nullptr; o.cap = o.used = 0; }
    DevBuf& operator=(DevBuf&& o) noexcept {
        if (this != &o) {
            release();
            p = o.p; cap = o.cap; used = o.used;
            o.p = nullptr; o.cap = o.used = 0;
        }
        return *this;
    }
    ~DevBuf() { release(); }
    int reserve(size_t n, bool keep);
    void release();
    template <typename T> T* as() const { return (T*)p; }
};

// Pinned host allocation (hipHostMalloc), move-only, freed on destruction.
struct PinnedBuf {
    void* p = nullptr;
    size_t cap = 0;
    PinnedBuf() = default;
    PinnedBuf(const PinnedBuf&) = delete;
    PinnedBuf& operator=(const PinnedBuf&) = delete;
    PinnedBuf(PinnedBuf&& o) noexcept : p(o.p), cap(o.cap) { o.p = nullptr; o.cap = 0; }
    PinnedBuf& operator=(PinnedBuf&& o) noexcept {
        if (this != &o) {
            release();
            p = o.p; cap = o.cap;
            o.p = nullptr; o.cap = 0;
        }
        return *this;
    }
    ~PinnedBuf() { release(); }
    int reserve(size_t n);
    void release();
    template <typename T> T* as() const { return (T*)p; }
};

// Open-addressing group-key table on the device (key -> position).
struct KeyTableHost {
    DevBuf keys, ctrl;
    PinnedBuf h_ctrl;  // landing area of check()
    size_t size_ = 0;
    int64_t n_keys = 0;  // keys inserted so far (read back by check)
    bool dense = false;  // dictionary ids: slot = (id - dadd) / dmul, no hashing
    uint32_t dmul = 1, dadd = 0;
    // band mode (KeyTable::lk): rows of 2^lk slots for the time buckets [b0, b0 + rows)
    uint32_t lk = 0, b0 = 0, rows = 0;
    int64_t band_base = 0;  // b0 before truncation to 32 bits
    int init(int64_t capacity);
    int init_dense(int64_t capacity, uint32_t mul, uint32_t add);
    int init_band(uint32_t lk, uint32_t rows, int64_t base, uint32_t mul, uint32_t add);
    int init_size(size_t ts);
    shd::KeyTable dev() const;
    int check(hipStream_t s);
    // check() in two halves: queue the counter copy into pinned memory, read it after a sync
    int check_async(hipStream_t s, uint32_t* pinned4);
    int check_result(const uint32_t* pinned4);
    void release() { keys.release(); ctrl.release(); }
};

// a band key table's shape (snapshot / restore)
struct KeyBand {
    uint32_t lk = 0, rows = 0;
    int64_t base = 0;
};

// Host vectors in pinned memory (hipHostMalloc) without value-initialisation on resize: the row
// arrays of a push are D2H copy targets, refilled every push, so they land at the copy engine's rate
// instead of through a pageable bounce buffer, and a resize does not first zero them.
template <typename T>
struct PinnedAlloc {
    typedef T value_type;
    PinnedAlloc() = default;
    template <typename U> PinnedAlloc(const PinnedAlloc<U>&) {}
    T* allocate(size_t n) {
        void* p = nullptr;
        if (hipHostMalloc(&p, std::max<size_t>(n, 1) * sizeof(T), hipHostMallocDefault) != hipSuccess)
            throw std::bad_alloc();
        return (T*)p;
    }
    void deallocate(T* p, size_t) { (void)hipHostFree(p); }
    template <typename U> void construct(U* p) { ::new ((void*)p) U; }  // default-init: no zeroing
    template <typename U, typename... A> void construct(U* p, A&&... a) { ::new ((void*)p) U(std::forward<A>(a)...); }
    template <typename U> bool operator==(const PinnedAlloc<U>&) const { return true; }
    template <typename U> bool operator!=(const PinnedAlloc<U>&) const { return false; }
};
template <typename T> using PinnedVec = std::vector<T, PinnedAlloc<T>>;

// Host copy of a push's output (sh_out points into these vectors).
struct OutHost {
    PinnedVec<int64_t> flush_offsets{0}, flush_clock, ts, keys, rep;
    PinnedVec<uint8_t> expired, nulls;
    PinnedVec<uint64_t> vals;
    sh_out out{};
    void reset() {
        flush_offsets.assign(1, 0);
        flush_clock.clear();
        ts.clear(); keys.clear(); expired.clear(); nulls.clear(); vals.clear(); rep.clear();
    }
    const sh_out* view(int n_keys, int n_vals, const int32_t* vtypes) {
        out = sh_out{};
        out.n_flushes = (int64_t)flush_clock.size();
        out.n_rows = (int64_t)ts.size();
        out.n_keys = n_keys;
        out.n_vals = n_vals;
        for (int i = 0; i < n_vals; i++) out.val_types[i] = vtypes[i];
        out.flush_offsets = flush_offsets.data();
        out.flush_clock = flush_clock.data();
        out.ts = ts.data();
        out.expired = expired.data();
        out.keys = keys.data();
        out.vals = vals.data();
        out.nulls = nulls.data();
        rep.resize(ts.size(), -1);
        out.rep = rep.data();
        return &out;
    }
};

int compile_filter(int n_ops, const sh_filter_op* ops, int n_cols, const int32_t* types, shd::FilterProg& fp);
int compile_aggs(int n_aggs, const sh_agg_spec* aggs, int n_cols, const int32_t* types, shd::AggPlan& ap,
                 int32_t* out_types);
int compile_keys(int n_group, const int32_t* group, int n_cols, const int32_t* types, shd::KeyPlan& kp);

// Host batch staged to the device (sh_push): one DevBuf per column + timestamps.
struct StagedBatch {
    DevBuf ts, cols[SH_MAX_COLS];
    DevBuf blk;  // one block when the host batch is one contiguous region (PinnedBatch layout)
    int stage(hipStream_t s, const sh_batch* b, int n_cols, const int32_t* types, sh_batch* dev);
};

size_t type_size(int t);

using shd::AggPlan;
using shd::FilterProg;
using shd::KeyPlan;
using shd::PushInfo;
using shd::TileMap;

struct SlidingImpl;

// A/B switches of the measured alternatives, read from the environment once per query,
// when it is created, so a process can run queries with different settings side by side:
// SH_DIRECT_POS=1, SH_PART_KEYS=1024, SH_NO_ASYNC_SMALL=1, SH_SL_RECORDS_SEQ=0/1, SH_AGG_BAND_ROWS=n,
struct Tuning {
    bool direct_pos = false, part_keys_1024 = false, no_async_small = false, sl_records_seq = false;
    bool pl_sort = true;   // partitioned lengthBatch keyed by the partition on the sorted lanes (lane 3)
    bool slx_wave = true;     // expired / all-events sliding replay with a wave per key (k_slx_wkey); SH_SLX_WAVE=0: a lane per key
    int agg_band_rows = 8;
    static Tuning from_env();
};

struct WideKeys;
struct sh_query {
    int kind = 0;
    Tuning tune = Tuning::from_env();            // 0 = batch window (lengthBatch/timeBatch), 1 = sliding time window
    SlidingImpl* sl = nullptr;
    // text of dictionary ids per string column (sh_query_set_strings), UTF-16 as Java holds it
    std::unordered_map<int, std::vector<std::u16string>> strings;
    std::unordered_map<int, std::vector<char>> strings_set;
    // partitioned timeBatch (R12): only the first partition key ever flushes
    bool partitioned = false, p0_known = false;
    int64_t p0 = 0;
    FilterProg fp_orig{};
    sh_ctx* ctx = nullptr;
    sh_query_desc d{};
    FilterProg fp{};
    AggPlan ap{};
    KeyPlan kp{};
    int32_t vtypes[SH_MAX_AGGS]{};
    KeyTableHost kt;
    // partitioned lengthBatch grouped by other columns (sh_plane.cpp, lane 3): kp / kt key the
    // partitions, gkp / gkt the output groups
    KeyPlan gkp{};
    KeyTableHost gkt;
    bool plane_sorted = false;  // lane 3 (also for lengthBatch keyed by the partition with Tuning::pl_sort)
    KeyTableHost pgkt;          // time lanes grouped by other columns: (partition slot, group slot) -> state
    size_t pg_min_size = 0;     // its size at creation (a rebuild never shrinks below it)
    bool group_other = false;   // ... grouped by columns other than the partition key
    bool plane_tbsc = false;    // lane 4: partitioned timeBatch(T, true), current output
    int P = 1, logP = 0, NL = 0;
    // playback clock + window state
    bool clock_valid = false;
    int64_t clock = 0;
    bool e0_valid = false;
    int64_t E0 = 0;
    // timeBatch windows of calendar months (1) / years (2) in the zone offset cal_tz: the root of an
    // aggregation `every month` / `every year` (set by the aggregation before its first push)
    int cal = 0;
    int64_t cal_tz = 0;
    // called by push_core while the push's first kernels run, before it waits for their results (an
    // aggregation hands its previous push's root flushes to the roll-up levels there)
    int (*mid_hook)(void*) = nullptr;
    void* mid_arg = nullptr;
    // wide group keys (sh_wide.h): the window is keyed by an interned id in a synthetic column past the
    // stream's own (d.n_cols = wide_n_cols + 1); rows get their group-by values back at the end of a call
    WideKeys* wide = nullptr;
    int wide_n_cols = 0;
    uint64_t wide_cols_used = 0;  // the stream columns a batch must carry
    DevBuf wide_keys;
    sh_out wide_out{};
    OutHost wide_host;
    int64_t W_open = 0;
    int64_t xm = 0;  // externalTimeBatch: lastCurrentEventTime (running max of the timestamp attribute)
    // externalTimeBatch timeout (sh_query_set_ext_timeout): lastScheduledTime, and the open batch's
    // passing events since its last emission (the window's currentEventChunk is empty when 0)
    int64_t xt_timeout = 0;
    // replaceTimestampWithBatchEndTime (sh_query_set_ext_replace_ts): the stream index of the first event
    // of the last windows, with their number (a row's representative event lies in the last window that
    // starts at or before it), and the batch end times of the last output's rows
    bool xt_replace = false;
    // sh_query_set_compact_flushes: an output of one row per flush whose clocks equal the rows' ts leaves
    // flush_offsets / flush_clock NULL (compact_now: this call's output is in that form)
    bool compact_flushes = false, compact_now = false;
    // sh_query_set_device_flushes: sh_push_device's flush layout stays in device memory (fl_dev)
    bool device_flushes = false;
    DevBuf fl_dev;
    std::vector<std::pair<int64_t, int64_t>> xr_starts;
    std::vector<int64_t> xr_rep, xr_vals;
    bool xt_Lvalid = false;
    int64_t xt_L = 0;
    int64_t xt_nnew = 0;
    // stream.current.event flushes built on the device (sc_rows): send clocks, flags, offsets, clocks
    DevBuf sc_slp, sc_fflag, sc_fo, sc_fc, sc_bclk;
    DevBuf xt_dev;
    PinnedBuf xt_host;
    int64_t n_pend = 0, pend_cap = 0;
    int64_t last_nb = 0;  // window starts the last push found (sizes the first read-back of the next)
    int64_t seq = 0;  // stream index of the next event pushed (sh_out.rep numbering)
    DevBuf pend_pos, pend_ts, pend_vals;
    DevBuf pend_tmp;  // staging of pending_to_front's overlapping moves (kept: no allocation per push)
    // scratch
    DevBuf blk_pass, blk_tl, blk_first, blk_xm, info, bounds, segs, seg_rows, rows, counters, out_ts, out_keys, out_vals,
        out_nulls, out_expired, out_rep, blk_cnt;
    DevBuf first_bits, word_pre;  // first-occurrence bitmap of the closed events and its word prefix
    DevBuf emit_stage;            // output rows staged at their output position (k_emit_rank)
    const void* zeroed_nulls = nullptr;    // out_nulls / out_expired buffers already zeroed
    const void* zeroed_expired = nullptr;
    DevBuf ms_counts, ms_tmp, rec_pos, rec_idx, rec_vals, part_off;
    DevBuf new_pos, seg_off;  // key slot per event of the push (kNoPos = filtered out); segment record offsets
    PushInfo* h_info = nullptr;
    PinnedBuf h_up;    // pinned segment list of the closed windows (read by the kernels in place)
    PinnedBuf h_tail;  // pinned landing area of the push's final copies: key-table counters, rows per segment
    PinnedBuf h_bounds;  // pinned landing area of the push's window boundaries
    // the multisplit of the push's events, launched before the host reads the window boundaries
    bool ms_ready = false;
    bool rec_packed = false;
    bool direct_pos = false;
    // set during a zero-copy staged push: the host batch, staged on the compute stream if the push
    // leaves the small-push path (sh_ingest.cpp)
    const sh_batch* zc_host = nullptr;
    std::vector<int64_t> sc_sl_host;  // stream.current: the sends' clocks (host scratch, kept)
    // an aggregation root whose key table may switch to band mode (sh_aggregation.cpp band_reserve)
    bool band_keys = false;
    // the band was placed without probing the push (sh_aggregation.cpp agg_push): a push one of whose
    // buckets falls outside it returns kRetryBand at its first synchronisation, before any state changed
    bool band_spec = false;
    PinnedBuf h_spec;
    uint32_t band_lk = 0, band_rows = 0, band_mul = 1, band_add = 0;
    // small-push fast path (try_small_push): the kernel's report in coherent pinned host memory
    shd::SmallRes* small_res = nullptr;
    shd::SmallRes* small_res_dev = nullptr;
    uint64_t small_token = 0;
    // asynchronous small pushes (sh_window.cpp small_async): the batch is copied into one of
    // kZcRing pinned slots the kernel reads in place, and the call returns without waiting; the
    // kernel's report (key-table counters) is verified by the next call that finds it, or waits for it
    static constexpr int kZcRing = 8;
    char* zc_ring = nullptr;      // pinned, mapped: kZcRing slots of zc_slot bytes
    char* zc_ring_dev = nullptr;
    size_t zc_slot = 0;
    uint64_t zc_tok[kZcRing]{};   // token of the kernel that reads each slot
    int zc_next = 0;
    uint64_t async_tok = 0;       // last asynchronous push not yet verified (0: none)
    int64_t async_keys = 0;       // events of the unverified asynchronous pushes (a bound on their new keys)
    TileMap ms_map{};  // tiling of the last multisplit
    int64_t rec_cap = 0;
    // flush bookkeeping of the closed windows, completed after the push's final synchronisation
    struct ClosedTail {
        bool active = false, host_done = false;
        int nseg = 0, units_per_seg = 1;
        int64_t closed_hi = 0;
        std::vector<int64_t> clocks, windows;
    } tail;
    StagedBatch staged;
    OutHost out;
    sh_out dev_out{};
    PinnedVec<int64_t> dev_flush_offsets{0}, dev_flush_clock;
    hipEvent_t ev_push0 = nullptr, ev_push1 = nullptr, ev_agg0 = nullptr, ev_agg1 = nullptr;
    // the presorted sliding replay's key sort, timed apart from the replay (the host sync lies between)
    hipEvent_t ev_srt0 = nullptr, ev_srt1 = nullptr;
    bool srt_timed = false;
    hipEvent_t ev_mid = nullptr;  // the push info and boundaries are on the host (work queued after it runs on)
    sh_stats stats{};
    int64_t agg_bytes = 0;
    // per flush of the last push: window number (internal use by the aggregation root)
    std::vector<int64_t> flush_window;
    bool internal_keys = false;  // key plan set by an internal owner (aggregation root)
    size_t kt_min_size = 0;      // table size at creation (rebuilds never shrink below it)
    // column widths as loaded by the kernels (the sharded owner reads 8-byte raw columns)
    int32_t load_type[SH_MAX_COLS]{};
    // columns the query reads (filter, group-by, partition key, aggregators, time attributes): a batch
    // may leave the others NULL — the shim packs only what the query reads (20 B/event for C2)
    uint32_t cols_used = 0;
    // sharded owner (sh_shard.cpp): windows given per event, flush clocks from the global
    // window starts, global stream index carried per pending event and reported per row
    bool given = false;
    const int* given_wcol = nullptr;
    const shd::u64* given_gidx = nullptr;
    const int64_t* given_clk = nullptr;  // stream.current.event owners: each record's global send clock,
    int64_t given_seq0 = 0, given_ss = 1;  // the push's first global index and send size (rows per send)
    int64_t given_W_base = 0, given_W_end = 0;
    std::vector<sh_bound> gbounds;  // this push's global window starts, sorted by gidx
    DevBuf pend_gidx, out_order;  // pend_gidx: stream index of every queued event (all modes)
    std::vector<int64_t> order_host;
    // `expired` / `all events` output (sh_expired.cpp): the current rows of a call are turned into
    // the output flushes; the last flushed batch is carried until its successor closes
    bool xmode = false;
    bool xc_valid = false;
    int64_t xc_n = 0, xc_W = 0;
    DevBuf xc_keys, xc_rep, xc_keys2, xc_rep2;                   // carried rows
    DevBuf xs_ts, xs_keys, xs_vals, xs_nulls, xs_rep;            // source rows of a call
    DevBuf x_ts, x_keys, x_vals, x_nulls, x_expired, x_rep;      // output rows
    // sharded owner (given): the rows' global order (a row at an expired row's place keeps its order:
    // the previous batch's first occurrence), carried with the last flushed batch
    DevBuf xc_order, xc_order2, xs_order, x_order;
    DevBuf x_items, x_keep, x_rank, x_match, x_tmp, x_matched, x_trow, x_tkey, pass_pos;
    PinnedBuf x_h;
    std::vector<std::pair<int64_t, int64_t>> x_closes;  // (window start W, clock) seen by the call
    std::vector<int64_t> x_stamps;  // externalTimeBatch: attribute time (running max) closing flush j
    // stream.current.event batch windows (sh_window.cpp sc_rows): scratch of a push
    DevBuf sc_pcb, sc_skey, sc_skey2, sc_idx, sc_idx2, sc_chunk, sc_send, sc_hd, sc_pos, sc_starts, sc_tmp, sc_ghead,
        sc_pre, sc_sval, sc_slast, sc_ochunk, sc_osend, sc_sl, sc_sort, scx_fe, scx_fpre, scx_last, scx_rows, scx_rank,
        scx_clk;
    PinnedBuf sc_h, sc_hp, sc_ho, h_small_sc;
    // `output [all|first|last] every N events` (sh_rate.cpp): the limiter's state across calls
    struct Rate {
        int kind = SH_RATE_NONE;
        int64_t N = 0;
        bool gb = false;          // group-by variants (FirstGroupBy / LastGroupBy)
        int64_t seq = 0;          // rows seen (First/LastPerEvent counters)
        int64_t nc = 0;           // carried rows (AllPerEvent chunk, LastGroupBy open window)
        DevBuf c_ts, c_exp, c_rep, c_keys, c_vals, c_nulls;          // carried rows (stride nc)
        DevBuf s_ts, s_exp, s_rep, s_keys, s_vals, s_nulls;          // source rows of a call
        DevBuf o_ts, o_exp, o_rep, o_keys, o_vals, o_nulls, o_flush;  // kept rows
        DevBuf m_ts, m_exp, m_rep, m_keys, m_vals, m_nulls;          // merged sharded rows (sh_rate_apply_merged)
        DevBuf foff, flag, pre, src, eflush, tmp, skey, skey2, idx, idx2, hd, pos, starts, seg_c0, seg_new, sort_tmp;
        DevBuf tk, tc, tk2, tc2, n_keys;  // FirstGroupBy key -> count table
        int64_t t_cap = 0, t_keys = 0;
        // `output first every <t>`: outputTime (no group-by) / the key -> last output time table
        bool ft_has = false;
        int64_t ft_last = 0;
        DevBuf ftk, ftt, ftk2, ftt2, fclk, chosen;
        int64_t ft_cap = 0, ft_keys = 0;
        // one limiter per partition instance (the partition lanes): per partition slot the running row
        // count (First/LastPerEvent) and `first every <t>`'s output time; the carried rows' partitions
        bool part = false;
        bool pkey = false;  // keyed First limiters of lanes grouped by other columns: key = (partition, group)
        bool lkey = false;  // keyed Last of lanes grouped by other columns (per-partition windows, keyed inside)
        DevBuf lk_ord, lk_cidx, lk_key, lk_key2, lk_idx, lk_idx2;
        int64_t nparts = 0;
        DevBuf c_part, s_part, t_part, pseq, pft_has, pft_last, keep, okey, okey2, olist, olist2;
        PinnedVec<int64_t> h_off, h_clk, flush_offsets, flush_clock;
        PinnedVec<int> h_flush;
        PinnedBuf h_small;
        sh_out dev_out{};
    } rate;
    // double-buffered host ingest (sh_ingest.cpp): two device staging slots filled on the copy stream
    struct Ingest {
        StagedBatch slot[2];
        sh_batch dev[2]{};
        hipEvent_t copied[2]{}, consumed[2]{}, c0[2]{}, c1[2]{};
        bool used[2]{};
        int next_stage = 0, next_push = 0, outstanding = 0;
        uint32_t gen = 0;
        uint32_t ticket_gen[2]{};
        int64_t bytes[2]{};
        // zero-copy slot: a small pinned batch the small-push kernel reads in place over PCIe (host[]
        // is copied on the compute stream only if the push needs the full pipeline)
        bool zc[2]{};
        sh_batch host[2]{};
        double last_h2d_ms = 0;
        int64_t last_h2d_bytes = 0;
    } ing;
};

// push_core's return when a speculatively placed key band missed one of the push's buckets (nothing of
// the push was committed; the aggregation probes the push and pushes again)
constexpr int kRetryBand = 17;
// every column the query reads has a pointer in `b` (SH_ERR_INVALID otherwise)
const int64_t* plane_out_rep_attr(sh_query* q);
bool plane_is_sorted_lane(const sh_query* q);
int check_batch_cols(const sh_query* q, const sh_batch* b);
// the open window aggregated per key without closing it (sh_window.cpp; aggregation retrieval)
int query_peek(sh_query* q, int64_t* n_rows);
// push of a batch staged on the device by sh_stage, host output (sh_window.cpp)
int query_push_staged(sh_query* q, const sh_batch* dev, const sh_out** out);
// a push the small-push kernel can take whole (no window state that forces the full pipeline)
bool query_small_eligible(const sh_query* q, int64_t n);
void ingest_destroy(sh_query* q);  // (sh_ingest.cpp)

// expired / all-events output of a batch query's call (sh_expired.cpp)
int xout_finish(sh_query* q, bool host_out, const sh_out** out);
// output rate limiting over a call's device output (sh_rate.cpp); flush_dev: the input's flush
// arrays are device memory (sliding windows)
int rate_apply(sh_query* q, const sh_out* in, bool flush_dev, bool host_out, const sh_out** out);

// the filter restricted to partition key `key` (R12): base AND (pcol == key)
int partition_filter(const FilterProg& base, int pcol, int ptype, int64_t key, FilterProg* out);

// sharded owner helpers (sh_window.cpp)
int64_t given_flush_clock(const sh_query* q, int64_t W);
int query_push_given(sh_query* q, const sh_batch* b, bool host_out, const sh_out** out);
int query_close_given(sh_query* q, bool host_out, const sh_out** out);
int query_advance(sh_query* q, int64_t now, bool host_out, const sh_out** out);

// make room for `extra` new keys in a batch query's table (rebuild / grow; batch windows only)
int query_reserve_keys(sh_query* q, int64_t extra);
int query_drain_async(sh_query* q);
// move the queued events' key slots into table `nk` (any mode to any mode) and make it the query's
int query_swap_keys(sh_query* q, KeyTableHost& nk);

// internal constructor for the aggregation root: a batch query with a prepared key plan
int sh_query_create_internal(sh_ctx* ctx, const sh_query_desc* d, const KeyPlan& kp, sh_query** out);
// device-output advance (aggregation root)
int sh_advance_time_device(sh_query* q, int64_t now, const sh_out** out);

// sharded incremental aggregation: the shard's owner query is the aggregation's root
// (sh_shard.cpp)
int shard_create_root(sh_ctx* ctx, const sh_query_desc* d, const KeyPlan& kp, int32_t rank, int32_t world,
                      sh_shard** out, sh_query** owner);
void shard_attach_aggregation(sh_shard* s, sh_aggregation* a);
// (sh_aggregation.cpp)
int flush_layout_to_device(sh_query* q, sh_out& o);  // (sh_query_set_device_flushes)
int agg_reserve_root(sh_aggregation* a, const sh_batch* dev, bool side = false);  // key room before the root's push
int agg_after_root(sh_aggregation* a, const sh_out* root_out);  // root flushes -> roll-up levels
void agg_release_sharded(sh_aggregation* a);                     // called by sh_shard_destroy


// sliding time window (sh_sliding.cpp)
int sliding_create(sh_query* q);
int sliding_push(sh_query* q, const sh_batch* b, bool host_out, const sh_out** out);
int sliding_advance(sh_query* q, int64_t now, const sh_out** out, bool host_out = true);
int sliding_push_given(sh_query* q, int64_t M, const int64_t* ts, const void* const* cols, const int64_t* gclk,
                       const int64_t* gpm, const uint64_t* gidx, int64_t raw_base, int64_t send_size,
                       int64_t send_base, bool host_out, const sh_out** out, int64_t n_global);
void sliding_destroy(sh_query* q);
// stable multisplit of the combined events [0, hi) into the query's P key partitions: records
// (q->rec_pos / rec_idx / rec_vals, capacity q->rec_cap), per-(partition, tile) offsets in q->ms_counts
// counted: k_boundaries already wrote the counts of the push's tiles (tiling make_tile_map(n_pend, hi),
// buffers sized by reserve_ms_counts before it ran)
int reserve_ms_counts(sh_query* q, const TileMap& m);
int run_multisplit(sh_query* q, int64_t hi, const sh_batch* b, bool counted = false, bool wide = false);

