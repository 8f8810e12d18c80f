// sh_internal.h — structures shared by the host runtime (sh_runtime.cpp) and the gfx950 kernels
// (sh_kernels.hip). Nothing here crosses the public C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/siddhi_hip.h"

namespace shd {

typedef unsigned long long u64;
typedef int64_t i64;
typedef unsigned int u32;

constexpr int kMaxFilterOps = 32;
constexpr int kBlock = 256;           // threads per workgroup (4 wave64)
constexpr int kItems = 8;             // events per thread in the scan-type passes
constexpr int kTile = kBlock * kItems;  // events per workgroup in the scan-type passes
constexpr u64 kEmptyKey = 0x8000000000000001ull;  // open-addressing EMPTY sentinel
constexpr u32 kNoPos = 0xFFFFFFFFu;              // event filtered out (no key slot)
// Packed multisplit record (one u32 per event): local key (< 1024) << 22 | the low 22 bits of the
// combined event index. The aggregation restores the index from its segment's start, so a packed
// split serves every closed segment shorter than 2^22 events (longer ones re-split wide).
constexpr int kPackIdxBits = 22;
constexpr u32 kPackIdxMask = (1u << kPackIdxBits) - 1u;

// Filter program (postfix), evaluated per event on device. Mirrors sh_filter_op.
struct FilterOpD {
    int op, type, col, pad;
    i64 ival;
    double dval;
};
struct FilterProg {
    int n;
    int pad;
    FilterOpD ops[kMaxFilterOps];
};

// Which kernel instance evaluates a filter program (eval_filter's FK): 0 none, 1 `col <cmp> const`
// or two of those joined by AND / OR (evaluated in registers), 2 anything else (the stack machine).
// internal filter op (never in a caller's program): the two operands' partition-key forms equal —
// String.valueOf equality, i.e. the bits with NaN canonical for float / double (partition_filter, R12)
constexpr int kOpKeyEq = 32;

inline int filter_kind(const FilterProg& f) {
    auto leaf = [&](int i) {
        return f.ops[i].op == SH_OP_COL && f.ops[i + 1].op == SH_OP_CONST && f.ops[i + 2].op >= SH_OP_GT &&
               f.ops[i + 2].op <= SH_OP_NE;
    };
    if (f.n == 0) return 0;
    if (f.n == 3 && leaf(0)) return 1;
    if (f.n == 7 && leaf(0) && leaf(3) && (f.ops[6].op == SH_OP_AND || f.ops[6].op == SH_OP_OR)) return 1;
    return 2;
}

// Stream columns of one batch (device pointers) with their SH_T_* types.
struct ColSet {
    const void* ptr[SH_MAX_COLS];
    int type[SH_MAX_COLS];
    int n;
    int pad;
};

// Aggregator execution plan. kinds restate the Java State classes for BATCH (add-only) use:
//   Sum{Long,Int} -> SUM_L, Sum{Double,Float} -> SUM_D, Avg* -> AVG (double value, long count),
//   Count -> COUNT, Min/Max typed compare on the input type.
enum AggKind {
    AK_COUNT = 0, AK_SUM_L, AK_SUM_D, AK_AVG, AK_MIN_L, AK_MIN_F, AK_MIN_D, AK_MAX_L, AK_MAX_F, AK_MAX_D
};
struct AggPlan {
    int n;         // aggregators
    int n_fields;  // 8-byte LDS fields per key
    int n_vcols;   // distinct value columns carried by records / pending
    int pad;
    int kind[SH_MAX_AGGS];
    int field[SH_MAX_AGGS];  // LDS field index (-1 for COUNT)
    int vcol[SH_MAX_AGGS];   // value-column slot (-1 for COUNT)
    int vcol_src[SH_MAX_AGGS];   // stream column index of value slot v
    int vcol_type[SH_MAX_AGGS];  // SH_T_* of value slot v
    // per LDS field f (batch folds): update op and the value slot it reads
    int fop[SH_MAX_AGGS];
    int fvcol[SH_MAX_AGGS];
};
// field update ops: sums (long, double, int->double for avg) and typed min/max
enum FieldOp { FOP_ADD_I = 0, FOP_ADD_D, FOP_ADD_DI, FOP_MIN_I, FOP_MAX_I, FOP_MIN_D, FOP_MAX_D, FOP_MIN_F, FOP_MAX_F };

// Group key plan: 0, 1 or 2 integral columns packed into a u64.
// a window's key: one column of any type or two 32-bit columns packed into one u64 (wider group keys are
// interned first, sh_wide.h, and key the window by their 32-bit id)
constexpr int kKeyParts = 2;
struct KeyPlan {
    int n;
    int col[kKeyParts];
    int type[kKeyParts];
    int dense;  // one STRID column: dictionary ids are dense in [0, key_capacity) -> slot = id
    i64 div[kKeyParts];  // > 0: the component is (u32)((value + add) / div) (aggregation time buckets)
    i64 add[kKeyParts];  // (the aggregation time zone's offset for hour / day buckets)
};

// Hash table (key -> position = group slot). positions [0, mask] plus the reserved mask+1
// for a key equal to the EMPTY sentinel.
struct KeyTable {
    u64* keys;
    u32 mask;
    u32 shift;        // 64 - log2(mask + 1): Fibonacci-hash shift
    u32* n_keys;      // distinct keys inserted
    int* overflow;    // set when probing exhausts the table
    // dense mode (dictionary ids): slot = (id - dadd) / dmul, no probing, no table
    int dense;
    u32 dmul, dadd;
    // band mode (dense, lk > 0): an aggregation root's (time bucket, dictionary id) keys; bucket b
    // owns slot row b - b0 of 2^lk slots, rows in [0, rows), so slot = (row << lk) | id slot
    u32 lk, b0, rows;
};

// Window assignment for one push (see DESIGN.md "Window assignment").
struct WinParams {
    int kind;          // SH_WIN_LENGTH_BATCH / SH_WIN_TIME_BATCH
    int e0_valid;      // timeBatch: nextEmitTime initialised
    int clock_valid;   // playback clock initialised before the push
    int has_start;
    i64 L;             // lengthBatch length
    i64 T;             // timeBatch period
    i64 E0;            // timeBatch: first nextEmitTime
    i64 start_time;
    i64 clock0;        // clock before the push
    i64 W_open;        // window number of the pending events
    i64 n_pend;        // pending (open-window) events carried in
    i64 send_size;     // events per send (0 = one send)
    i64 N;             // new events in this push
    const int* wcol;   // sharded owner: window of every event given (W_base + wcol[e]); else null
    i64 W_base;
    int want_first_clk;  // sharded summary: report PushInfo.first_clk
    int pcol1;           // partitioned queries: report PushInfo.first_key from column pcol1 - 1 (0: none)
    // externalTimeBatch: window of an event = bucket (from the start time E0) of the running max of
    // the ts_col attribute over the events reaching the window; xm0 = that max before the push
    int ts_col, start_col;
    i64 xm0;
    int rec_seq;  // sliding records: the lane-strided form (k_sl_records_seq) where it applies
    int cal;      // timeBatch of calendar months (1) / years (2) in the zone offset cal_tz (aggregation roots)
    i64 cal_tz;
};

// Result of the block-aggregate scan (written by k_scan_blocks, read back by the host).
struct PushInfo {
    i64 total_pass;
    i64 max_tl;        // max ts over send-last events (INT64_MIN if none)
    i64 first_pass;    // first passing new event (INT64_MAX if none)
    i64 E0;            // nextEmitTime after initialisation
    int e0_valid;
    int n_bounds;      // boundaries appended by k_boundaries
    i64 first_clk;     // clock of the first passing event's send, before the carried-in clock
    i64 max_xm;        // externalTimeBatch: max of the timestamp attribute over passing events
    int err;           // externalTimeBatch: first event before its start time
    int unsorted;      // single-pass form: a timestamp decreased (redo with the prefix passes)
    i64 first_key;     // column WinParams.pcol1 - 1 of the first passing event (partitioned queries, R12)
};

// A window boundary inside the push: first combined index of a new window.
struct Bound {
    i64 idx;         // combined index (pending first, then new events)
    i64 W;           // window number starting at idx
    i64 clock;       // clock of event idx
    i64 clock_prev;  // clock of event idx-1
    i64 pcb;         // passing new events before idx (new-event space)
    i64 pad;
};

// A closed segment handed to the aggregation kernel: combined index range of one window.
struct Segment {
    i64 lo, hi;
};

// Key slot of a push event: from the key-slot column k_boundaries wrote (np), or — dictionary keys
// that are their own slots, no filter (k_boundaries then writes no slot column) — the key column
// itself, clamped to the table (an id outside it has already failed the push).
struct PosSrc {
    const u32* np;
    const int* key;
    u32 mask;
    int pad;
};
__host__ __device__ inline u32 pos_at(const PosSrc& ps, i64 x) {
    if (ps.np) return ps.np[x];
    const u32 id = (u32)ps.key[x];
    return id > ps.mask ? ps.mask : id;
}
__host__ __device__ inline bool pos_any(const PosSrc& ps) { return ps.np || ps.key; }

// Row record of the aggregation kernels: row_words(n_aggs) u64 words — slot | count << 32,
// first | last << 32 (combined event indices), the last event's timestamp and stream index (read by
// the aggregation kernel itself, so the emission only permutes whole records), then the values.
__host__ __device__ constexpr int row_words(int n_aggs) { return (4 + n_aggs + 1) & ~1; }
// where a row's last-event timestamp and stream index come from (combined index space)
struct EvSrc {
    i64 n_pend;
    const i64* pend_ts;
    const i64* ts;
    const u64* pend_gidx;
    const u64* new_gidx;  // sharded owner: global stream index of every new event; else seq_base + e
    i64 seq_base;
};
__host__ __device__ inline i64 ev_ts(const EvSrc& es, u32 c) { return c < es.n_pend ? es.pend_ts[c] : es.ts[c - es.n_pend]; }
__host__ __device__ inline i64 ev_seq(const EvSrc& es, u32 c) {
    if (c < es.n_pend) return (i64)es.pend_gidx[c];
    return es.new_gidx ? (i64)es.new_gidx[c - es.n_pend] : es.seq_base + (i64)(c - es.n_pend);
}

// Launchers (sh_kernels.hip).
void launch_blockagg(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, i64 N, i64 send_size,
                     i64* blk_pass, i64* blk_tl, i64* blk_first, int nblk, i64* blk_xm = nullptr, int ts_col = -1);
// bytes of blk_first for launch_scan_blocks: the tiles' values, then the chunk totals
size_t scan_blocks_first_bytes(int nblk);
void launch_scan_blocks(hipStream_t s, i64* blk_pass, i64* blk_tl, i64* blk_first, int nblk, const i64* ts,
                        WinParams wp, PushInfo* info, i64* blk_xm = nullptr, ColSet cols = ColSet{});
// sorted: the single-pass form for non-decreasing timestamps (timeBatch with nextEmitTime known); it
// also scans blk_pass (nblk + 1 entries, the last zeroed) with scan_tmp and fixes the boundaries
void launch_boundaries(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp,
                       i64* blk_pass_pre, const i64* blk_tl_pre, PushInfo* info, Bound* bounds,
                       int max_bounds, int nblk, KeyPlan kp, KeyTable kt, u32* new_pos, const i64* blk_xm_pre = nullptr,
                       u32* ms_counts = nullptr, int P = 1, int ms_nblk = 0, int ms_col0 = 0, bool sorted = false,
                       i64* scan_tmp = nullptr);
// Rows of one aggregation unit — (segment, key partition) for the multisplit kernel, the segment for
// the flat one — fill the unit's own region of agg_unit_rows() row slots; unit_rows[u] = its count.
int agg_unit_rows(int P, int NL, bool own);
void launch_aggregate(hipStream_t s, const Segment* segs, int nseg, int P, int logP, int NL, i64 n_pend,
                      const u32* pend_pos, const u64* pend_vals, i64 pend_cap, const u32* new_pos, ColSet cols,
                      AggPlan ap, u64* rows, int RW, u32* unit_rows, u32* first_bits,
                      // multisplit source (P > 1 or long windows; null: the flat kernel reads the batch)
                      const u32* rec_pos, const u32* rec_idx, const u64* rec_vals, i64 rec_cap, const i64* seg_off,
                      bool pack, EvSrc es, bool dense_rows = false);
void launch_count_flags(hipStream_t s, const unsigned char* flags, i64 n, i64* blk_cnt, int nblk);
void launch_scan_sum(hipStream_t s, i64* a, int n);
// word_pre[w] = exclusive popcount prefix of the first-occurrence bitmap before word w (low 32 bits)
// with word w itself (high 32 bits); *total = the bitmap's popcount
void launch_bits_prefix(hipStream_t s, const u32* bits, i64 nw, i64* tile_sum, u64* word_pre, u32* total);
// rows: the aggregation units' regions; the row count (for the output columns' stride) is read on
// the device (launch_bits_prefix's total); row_cap bounds it
void launch_emit_rows(hipStream_t s, const u64* rows, int RW, const u32* unit_rows, i64 n_units, int unit_stride,
                      i64 row_cap, const u32* n_rows_dev, const u64* word_pre, int n_aggs, KeyTable kt,
                      KeyPlan kp, i64 n_pend, const i64* pend_ts, const i64* ts, i64 out_cap, i64* out_ts,
                      i64* out_keys, u64* out_vals, const u64* pend_gidx, const u64* new_gidx, i64* out_order,
                      i64 seq_base, i64* out_rep, u64* stage);
size_t emit_stage_bytes(int nk, int na, int order, i64 n_rows);
// dense rows (launch_aggregate dense_rows, multisplit units): one-pass emission from the bitmap words
void launch_emit_gather(hipStream_t s, const u64* word_pre, i64 nw, const Segment* segs, int nseg, int P, int logP,
                        int unit_stride, const u64* rows, int RW, PosSrc ps, const u32* pend_pos, i64 n_pend,
                        const u32* n_rows_dev, int n_aggs, KeyTable kt, KeyPlan kp, i64* out_ts, i64* out_keys,
                        u64* out_vals, const u64* pend_gidx, const u64* new_gidx, i64* out_order, i64 seq_base,
                        i64* out_rep);
void launch_compact_pending(hipStream_t s, const i64* ts, ColSet cols, PosSrc new_pos, AggPlan ap, i64 e_lo,
                            i64 N, i64 pcb_lo, i64 base, const i64* blk_pass_pre, u32* pend_pos, i64* pend_ts,
                            u64* pend_vals, i64 pend_cap, const u64* new_gidx, u64* pend_gidx, i64 seq_base);
// small pushes that close no window (sh_window.cpp try_small_push): one workgroup of kSmallT threads
constexpr int kSmallT = 1024;
constexpr int kSmallMax = kSmallT * kItems;
struct SmallRes {
    i64 total_pass;  // passing events appended to the open window
    i64 max_tl;      // the push's last timestamp (its clock; timestamps are non-decreasing here)
    int fallback;    // a window closes / timestamps decrease: nothing appended, run the full pipeline
    int pad;
    u32 ctrl[4];     // the key table's control words after the lookups (KeyTableHost::check_result)
    u64 token;       // written last: the host waits for it
};
// force: the host established that the push closes no window and its timestamps do not decrease
// (an asynchronous small push), so the kernel appends without re-checking
void launch_small_push(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp, KeyPlan kp, KeyTable kt,
                       AggPlan ap, u32* pend_pos, i64* pend_ts, u64* pend_vals, i64 pend_cap, u64* pend_gidx,
                       i64 seq_base, SmallRes* res, u64 token, bool force = false);
// multisplit (partitioned aggregation, P > 1)
// Multisplit tiles over the combined index space [0, hi) of queued + new events: tiles of kTile
// events over [0, split) (the queued events), then tiles of kTile over [split, hi) (the push's
// events, aligned with k_boundaries' tiles so that it can count them). split = 0: one uniform run.
struct TileMap {
    i64 split;
    i64 hi;
    int np_t;   // tiles over [0, split)
    int nblk;   // all tiles
};
inline TileMap make_tile_map(i64 split, i64 hi) {
    TileMap m;
    m.split = split < hi ? split : hi;
    m.hi = hi;
    m.np_t = (int)((m.split + kTile - 1) / kTile);
    m.nblk = m.np_t + (int)((hi - m.split + kTile - 1) / kTile);
    return m;
}
__host__ __device__ inline i64 tile_lo(const TileMap& m, int t) {
    return t < m.np_t ? (i64)t * kTile : m.split + (i64)(t - m.np_t) * kTile;
}
__host__ __device__ inline i64 tile_hi(const TileMap& m, int t) {
    const i64 lo = tile_lo(m, t), end = t < m.np_t ? m.split : m.hi;
    return lo + kTile < end ? lo + kTile : end;
}
// the tile holding index b (b == hi: one past the last tile, whose count column the scan's layout
// makes the next partition's start)
__host__ __device__ inline int tile_of(const TileMap& m, i64 b) {
    if (b < m.split) return (int)(b / kTile);
    return m.np_t + (int)((b - m.split) / kTile);
}

// counts the first n_count tiles of the map (k_boundaries counted the others) and zeroes the total slot
void launch_ms_count(hipStream_t s, TileMap m, int n_count, i64 n_pend, const u32* pend_pos, PosSrc new_pos, int P,
                     u32* counts);
void launch_fix_bounds(hipStream_t s, Bound* bounds, int max_bounds, const i64* blk_pass_pre, int nblk, const i64* ts,
                       WinParams wp, PushInfo* info);
void launch_ms_scatter(hipStream_t s, TileMap m, i64 n_pend, const u32* pend_pos, const u64* pend_vals,
                       i64 pend_cap, PosSrc new_pos, ColSet cols, AggPlan ap, int P, int logP, const u32* offsets,
                       u32* rec_pos, u32* rec_idx, u64* rec_vals, i64 rec_cap, bool pack);
void launch_scan_sum_large(hipStream_t s, i64* a, i64 n, i64* tmp);
// the multisplit's [tile][partition] count matrix -> record offsets in place (row nblk: partition ends)
size_t ms_offsets_tmp_bytes(int nblk, int P);
void launch_ms_offsets(hipStream_t s, u32* counts, int nblk, int P, i64* tmp);
void launch_scan_sum_large_u32(hipStream_t s, u32* a, i64 n, i64* tmp);
void launch_part_off(hipStream_t s, const i64* counts, int nblk, int P, i64* part_off);
void launch_seg_offsets(hipStream_t s, const Segment* segs, int nseg, i64 n_pend, const u32* pend_pos,
                        PosSrc new_pos, int P, const u32* counts, TileMap m, i64* seg_off);
void launch_zero2(hipStream_t s, void* a, int na, void* b, int nb);
void launch_rekey(hipStream_t s, i64 n, u32* pos, KeyTable old_kt, KeyTable new_kt);

// sharded ingest (sh_shard_kernels.hip)
constexpr int kMaxShards = 16;
void launch_shard_assign(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp, const i64* blk_tl_pre,
                         const i64* blk_pass_pre, const PushInfo* info, KeyPlan kp, int G, int nblk, u32* code,
                         i64* counts, Bound* bounds, int max_bounds, int* n_bounds, i64* clk_out = nullptr);
void launch_shard_sl_assign(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp,
                            const i64* blk_tl_pre, const i64* blk_pm_pre, i64 pm0, KeyPlan kp, int G, int nblk,
                            u32* code, i64* counts, i64* clk_out, i64* pm_out);
// Record of one re-keyed event (4-byte words): [key u32 | key u64][slice position u32 (+pad)][ts i64]
// [values u64...]; the owner derives the global index from the source and position, and the
// window from the global window starts.
struct ShardSrc {
    i64 start[kMaxShards + 1];  // first record of each source's block in the received buffer
    i64 gbase[kMaxShards];      // global stream index of each source slice's first event
    int G;
    int key32;
    int narrow;                 // ts as a 32-bit offset from tsbase (the push's minimum timestamp)
    i64 tsbase;
};
// 8-byte raw columns a shard record carries: the value columns, then the columns of time-bucket key
// components (their raw value is needed to re-derive the bucket; only the other components travel
// in the record's key word)
struct RawPlan {
    int n;
    int src[SH_MAX_COLS];
};
void launch_shard_pack(hipStream_t s, ColSet cols, const i64* ts, const u32* code, KeyPlan wkp, RawPlan rp, int G,
                       i64 N, int nblk, const i64* offsets, unsigned char* out, int rec_words, int key32,
                       int narrow = 0, i64 tsbase = 0);
struct ColRoles {
    int role[SH_MAX_COLS];  // -1 unused, 0..15 raw slot, 16 + g wire-key component g
    int n;
};
struct ColPtrs {
    u64* p[SH_MAX_COLS];
};
void launch_shard_unpack(hipStream_t s, const unsigned char* rec, i64 M, int rec_words, KeyPlan kp, ColRoles roles,
                         ShardSrc src, const i64* bound_gidx, const i64* bound_W, int n_bounds, i64 W_base, i64* ts,
                         ColPtrs cols, int* wcol, u64* gidx);

// ---- expired / all-events output of batch windows, pass-through batch queries (sh_expired*) ----
// One output flush: expired rows of the previous batch [p_lo, p_lo + p_n) and/or current rows
// [c_lo, c_lo + c_n) of the source array; tab_size > 0: merged by key through a table at tab_off.
struct XItem {
    i64 p_lo, p_n, c_lo, c_n, clock, tab_off, tab_size, out_base;
    i64 xts;  // timestamp of the expired rows (the flush clock; externalTimeBatch: the attribute time)
    i64 pad;
};
struct XOut {
    i64* ts;
    unsigned char* expired;
    i64* keys;
    u64* vals;
    unsigned char* nulls;
    i64* rep;
    i64* order;            // sharded owner: the rows' global order (else null)
    const i64* s_order;    // ... and the source rows' order
};
void launch_x_merge(hipStream_t s, const XItem* items, const i64* cum_c, const i64* cum_p, int n_items, i64 tot_c,
                    i64 tot_p, const i64* s_keys, i64 S, int nk, u32* trow, u64* tkey, int* match, u32* keep,
                    u32* item_matched);
void launch_x_scatter(hipStream_t s, const XItem* items, const i64* cum, int n_items, i64 total, const i64* s_ts,
                      const i64* s_keys, const u64* s_vals, const unsigned char* s_nulls, const i64* s_rep, i64 S,
                      int nk, int na, u32 count_mask, const int* match, const u32* keep, const u32* rank, i64 T,
                      XOut out);
// pass-through rows of the closed segments: pos = exclusive prefix of passing events over [0, hi]
void launch_pass_rows(hipStream_t s, i64 hi, i64 n_pend, const u32* new_pos, u32* pos, i64* tmp, const i64* pend_ts,
                      const u64* pend_gidx, const i64* ts, i64 seq_base, const Segment* segs, int nseg, i64* out_ts,
                      i64* out_rep, u32* seg_rows, u32* n_rows);

// ---- output rate limiting (sh_rate.cpp, sh_rate_kernels.hip) ----
struct RateRows {
    i64* ts;
    unsigned char* expired;
    i64* rep;
    i64* keys;
    u64* vals;
    unsigned char* nulls;
};
void launch_rate_pos(hipStream_t s, i64 n_src, i64 n_carry, int mode, i64 N, i64 seq0, const i64* flush_off, int nf,
                     u32* flag, int* eflush, u32* src);
void launch_rate_clear(hipStream_t s, i64 n, u32* src, u32* flag);
void launch_rate_pack(hipStream_t s, i64 n, const i64* keys, i64 stride, int nk, u64* skey, u32* idx);
void launch_rate_segments(hipStream_t s, i64 n, const u64* skey, const u32* idx, i64 N, int with_win, u32* hd, u32* pos,
                          u32* starts, i64* tmp);
void launch_rate_first(hipStream_t s, i64 n, const u32* hd, const u32* pos, const u32* starts, const u64* skey,
                       const u32* idx, i64 N, u64* tk, i64* tc, u32 tmask, i64* seg_c0, u32* seg_new, u32* n_keys,
                       const i64* flush_off, int nf, u32* flag, int* eflush);
void launch_rate_rehash(hipStream_t s, i64 old_cap, const u64* otk, const i64* otc, u64* tk, i64* tc, u32 tmask);
void launch_rate_last(hipStream_t s, i64 n, const u32* hd, const u32* pos, const u32* starts, const u32* idx, i64 N,
                      i64 n_carry, const i64* flush_off, int nf, u32* flag, u32* src, int* eflush);
void launch_rate_ftime_rows(hipStream_t s, i64 n, const i64* foff, int nf, const unsigned char* chosen, u32* flag,
                            int* eflush, u32* src);
void launch_rate_ftime_walk(hipStream_t s, i64 n, const u32* hd, const u32* pos, const u32* starts, const u64* skey,
                            const u32* idx, const i64* foff, const i64* fclk, int nf, i64 T, u64* tk, i64* tt, u32 tmask,
                            u32* flag, u32* n_new);
void launch_rate_ftime_rehash(hipStream_t s, i64 old_cap, const u64* otk, const i64* ott, u64* tk, i64* tt, u32 tmask);
void launch_rate_gather(hipStream_t s, i64 n, const u32* flag, const u32* pre, const u32* src, const int* eflush,
                        RateRows in, i64 in_stride, RateRows out, i64 T, int nk, int na, int* out_flush);

// one limiter per partition instance (the partition lanes' rows carry their partition slot)
void launch_ratep_pack(hipStream_t s, i64 S, i64 nc, const u32* c_part, const u32* in_part, u64* skey, u32* idx);
void launch_ratep_pkey(hipStream_t s, i64 n, const i64* keys, const u32* part, u64* skey, u32* idx);
void launch_ratep_last_keyed(hipStream_t s, i64 S, const u32* hd, const u32* pos, const u32* starts, const u32* idx, i64 N,
                             const i64* keys, i64 kstride, const u32* sp, i64* ord, u32* cidx, u32* keep, u64* skey,
                             u32* sidx);
void launch_ratep_last_keyed_rows(hipStream_t s, i64 S, const u64* skey, const u32* idx, const u32* cidx, const i64* ord,
                                  i64 N, i64 nc, const i64* flush_off, int nf, u32* hd, u32* pos, u32* flag, u32* src,
                                  int* eflush);
void launch_ratep_flags(hipStream_t s, i64 S, const u32* hd, const u32* pos, const u32* starts, const u64* skey,
                        const u32* idx, int mode, i64 N, i64 nc, i64* pseq, const i64* flush_off, int nf, u32* flag,
                        int* eflush, u32* src, u32* keep);
void launch_ratep_fparts(hipStream_t s, int nf, const i64* foff, const u32* in_part, u32 none, u64* fkey, u32* fidx);
void launch_ratep_ftime(hipStream_t s, int nf, const u32* hd, const u32* pos, const u32* starts, const u64* fkey,
                        const u32* fidx, const i64* fclk, u32 none, i64 T, unsigned char* has, i64* last,
                        unsigned char* chosen);
void launch_ratep_list(hipStream_t s, i64 S, const u32* flag, const u32* pre, const int* eflush, const u32* src, u64* okey,
                       u32* olist);
void launch_ratep_gather(hipStream_t s, i64 T, const u32* list, const u64* okey, RateRows in, i64 in_stride,
                         const u32* in_part, RateRows out, int nk, int na, int* out_flush, u32* out_part);

// ---- stream.current.event batch windows (sh_kernels.hip, driven by sh_window.cpp) ----
// (w << 32 | slot) -> (w << kb | slot): the sort then reads kb + the window bits only
void launch_sc_pack_keys(hipStream_t s, i64 M, unsigned kb, u64* skey);
void launch_sc_keys(hipStream_t s, i64 M, i64 n_old, const i64* pcb, int nb, const u32* pend_pos, const u64* pend_gidx,
                    int per_event, i64 send_size, i64 seq0, u64* skey, u32* idx, i64* chunk, i64* send,
                    int by_entry = 0);
void launch_sc_walk(hipStream_t s, i64 M, const u32* hd, const u32* pos, const u32* starts, const u32* idx,
                    const i64* chunk, const u64* pend_vals, i64 pend_cap, AggPlan ap, i64 n_old, u32* ghead, u64* sval,
                    u32* slast);
void launch_sc_emit(hipStream_t s, i64 M, i64 n_old, const u32* ghead, const u32* pre, const u32* slast, const u64* sval,
                    const u32* pend_pos, const i64* pend_ts, const u64* pend_gidx, const i64* chunk, const i64* send,
                    KeyTable kt, KeyPlan kp, int na, i64 T, i64* out_ts, i64* out_keys, u64* out_vals, i64* out_rep,
                    i64* out_chunk, i64* out_send, i64* out_order = nullptr);
void launch_sc_send_last(hipStream_t s, const i64* ts, i64 N, i64 send_size, i64 n_sends, i64* out);
int scan_max_i64(void* temp, size_t* bytes, const i64* in, i64* out, i64 n, hipStream_t s);
void launch_sc_flush_flags(hipStream_t s, i64 T, const i64* och, u32* flag);
void launch_sc_clock_is_ts(hipStream_t s, i64 n, const i64* osd, const i64* slp, int cv0, i64 clock0, const i64* ts,
                           u32* ok);
void launch_flush_clock_is_ts(hipStream_t s, i64 n, const i64* fc, const i64* ts, u32* ok);
void launch_sc_flushes(hipStream_t s, i64 T, const i64* osd, const u32* pre, const i64* slp, int cv0, i64 clock0,
                       const i64* bclk, i64* fo1, i64* fc);
void launch_xt_first_send(hipStream_t s, const i64* ts, i64 N, i64 send_size, i64 L, unsigned long long* out);
void launch_xt_count_pass(hipStream_t s, ColSet cols, FilterProg f, i64 hi, unsigned long long* out, int xcol = -1,
                          long long* xmax = nullptr);
void launch_scx_first(hipStream_t s, i64 M, const u32* hd, const u32* pos, const u32* starts, const u32* idx, u32* fe,
                      u32* fpre, u32* lastidx);
void launch_scx_count(hipStream_t s, i64 M, i64 n_old, const i64* pcb, const u64* skey, const u64* skey2,
                      const u32* idx2, const u32* fpre, int cur_on, int exp_on, u32* rows, i64* rank_e);
void launch_scx_rows(hipStream_t s, i64 M, i64 n_old, const i64* pcb, int nb, const u64* skey, const u32* fe,
                     const u32* fpre, const u32* lastidx, const u32* base, const i64* rank_e, const u64* sval,
                     const i64* send, const i64* send_clock, const i64* pend_ts, const u64* pend_gidx, KeyTable kt,
                     KeyPlan kp, AggPlan ap, int cur_on, int exp_on, i64 T, i64* out_ts, i64* out_keys, u64* out_vals,
                     unsigned char* out_nulls, unsigned char* out_exp, i64* out_rep, i64* out_chunk, i64* out_send);
void launch_scxt_count(hipStream_t s, i64 M, i64 n_old, const i64* pcb, int nb, const u64* skey, const u32* fpre,
                       const u32* ghead, int cur_on, u32* rows);
void launch_scxt_rows(hipStream_t s, i64 M, i64 n_old, const i64* pcb, int nb, const u64* skey, const u32* fe,
                      const u32* fpre, const u32* lastidx, const u32* ghead, const u32* base, const u32* slast,
                      const u64* sval, const i64* chunk, const i64* send, const i64* bclk, const i64* pend_ts,
                      const u64* pend_gidx, KeyTable kt, KeyPlan kp, AggPlan ap, int cur_on, i64 T, i64* out_ts,
                      i64* out_keys, u64* out_vals, unsigned char* out_nulls, unsigned char* out_exp, i64* out_rep,
                      i64* out_chunk, i64* out_send);
void launch_scx_pending_rows(hipStream_t s, i64 M, const u32* fe, const u32* fpre, const u32* lastidx,
                             const u32* pend_pos, const u64* pend_gidx, KeyTable kt, KeyPlan kp, AggPlan ap, i64 now,
                             i64 T, i64* out_ts, i64* out_keys, u64* out_vals, unsigned char* out_nulls,
                             unsigned char* out_exp, i64* out_rep);

}  // namespace shd
