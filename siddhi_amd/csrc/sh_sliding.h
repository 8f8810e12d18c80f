// sh_sliding.h — device structures of the sliding time-window path (sh_sliding_kernels.hip).
#pragma once
#include "sh_internal.h"

namespace shd {

struct SlInfo {
    i64 total_pass, max_tl, max_pm, need;
};

// rank-indexed records of the passing events of one push
struct SlRecords {
    u32* raw;     // event index in the push
    u32* slot;    // group key slot
    i64* clock;   // playback clock of the event's send
    i64* pm;      // max ts over passing events up to and including this one (all pushes)
    i64* ts;
    u64* vals;    // [n_vcols][cap]
    i64 cap;
    // keyed replay (k_sl_wkey): one 48-byte record per event instead of the clock / pm / ts / vals
    // columns — {clock, pm, ts, value, raw, 0} — so the key-order walk reads each record as one line
    u64* aos = nullptr;
};
constexpr int kSlAosWords = 6;

// persistent per-key state (indexed by key slot)
struct SlState {
    i64 nslots, rc;       // slots, ring capacity (power of two)
    i64* cnt;             // Count / Avg / Sum counts (equal for every aggregator)
    u64* f;               // [n_fields][nslots] sums (raw)
    u64* mm;              // [n_fields][nslots] minValue / maxValue
    unsigned char* mm_has;
    i64* dq_head;         // [n_fields][nslots]
    i64* dq_len;
    u64* dq;              // [n_fields][nslots][rc] monotone deque rings
    i64* rhead;           // [nslots] window ring of the key
    i64* rlen;
    i64* rpm;             // [nslots][rc] PM of each window event
    u64* rval;            // [n_vcols][nslots][rc] values of each window event
    i64* cur_send;        // last send that touched the key (global send number)
    i64* cur_first;       // rank of the key's first event in that send
};

// rows indexed by the rank of the (send, key) first occurrence
struct SlRows {
    i64* ts;
    u32* rep;             // push index of the row's representative event (the key's last in the send)
    u32* slot;
    i64* send;
    i64* clock;
    u64* vals;            // [n_aggs][cap]
    unsigned char* nulls; // [n_aggs][cap]
    i64 cap;
};

void launch_sl_prefix(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp, i64* blk_pass,
                      i64* blk_tl, i64* blk_pm, int nblk, SlInfo* info);
void launch_sl_records(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp, KeyPlan kp,
                       KeyTable kt, AggPlan ap, const i64* blk_pass_pre, const i64* blk_tl_pre, const i64* blk_pm_pre,
                       i64 pm0, SlRecords rec, u32* slot_cnt, int nblk, i64* send_clock = nullptr);
void launch_sl_need(hipStream_t s, const u32* slot_cnt, const i64* rlen, i64 n, i64* out);
// the lane-strided records kernel applies (no filter, per-event sends, time window): every event passes,
// M = N, and it may skip the per-slot counts (slot_cnt null) for launch_counts_sorted after the sort
bool sl_records_seq_applies(FilterProg f, WinParams wp, AggPlan ap);
// per-slot counts (slot_cnt zeroed by the caller) from the slot-sorted records
void launch_counts_sorted(hipStream_t s, const u32* ps, i64 M, u32* slot_cnt);
void launch_sl_multisplit(hipStream_t s, const u32* slot, i64 n, int P, i64* counts, i64* tmp, u32* out_rank,
                          i64* part_off);
int sliding_keys_per_partition(AggPlan ap);
// key-sorted replay (k_sl_key) for the count / sum / avg / min / max-of-one-double shape: ranks =
// the records' ranks sorted stably by slot (sort_slot_ranks, sh_sort.hip); key_off [nslots + 1]
bool sliding_keyed_ok(AggPlan ap);
int sort_slot_ranks(void* temp, size_t* bytes, const u32* slot, u32* slot_out, u32* rank_out, i64 M, i64 nslots,
                    hipStream_t s);
void launch_sliding_keyed(hipStream_t s, const u32* slot_cnt, u32* key_off, i64* tmp, const u32* sorted_rank,
                          SlRecords rec, i64* g_pm, u64* g_v, SlState S, AggPlan ap, i64 T,
                          i64 send_size, i64 send_base, u64* rowsK, unsigned char* flags);
// compact: per-event sends (no flags), the row holds its values only
int sliding_keyed_row_words(int n_aggs, bool compact = false);
// rowsK: the keyed replay's rows at the stream rank of their first record (flags NULL: per-event sends,
// every rank holds a row)
void launch_slk_emit(hipStream_t s, const unsigned char* flags, i64 n, const i64* blk_pre, int nblk,
                     const u64* rowsK, int RW, int n_aggs, KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts,
                     i64* out_keys, u64* out_vals, unsigned char* out_nulls, i64* out_send, i64* out_clock,
                     const u32* rank_raw, i64 raw_base, i64* out_order, i64* out_rep, const u64* aos = nullptr,
                     const u32* rank_slot = nullptr);
void launch_sl_gather(hipStream_t s, const u32* ranks, i64 M, SlRecords rec, SlRecords out, int nv);
// rec: the records gathered into partition order (k_sl_own); rec_by_rank: the same records in rank
// order, read through rank_list by k_sl_own_d (sliding_keys_per_partition(ap) == 8 shapes)
void launch_sliding_own(hipStream_t s, const u32* rank_list, const i64* part_off, int P, int logP, SlRecords rec,
                        SlState S, AggPlan ap, i64 T, i64 send_size, i64 send_base, SlRows rows,
                        unsigned char* flags, SlRecords rec_by_rank);
void launch_sl_emit(hipStream_t s, const unsigned char* flags, i64 n, const i64* blk_pre, int nblk, SlRows rows,
                    int n_aggs, KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals,
                    unsigned char* out_nulls, i64* out_send, i64* out_clock, const u32* rank_raw, i64 raw_base,
                    i64* out_order, const i64* clock_by_rank, i64* out_rep);
void launch_sl_records_given(hipStream_t s, i64 M, const i64* ts, ColSet cols, KeyPlan kp, KeyTable kt, AggPlan ap,
                             const i64* gclk, const i64* gpm, const u64* gidx, i64 raw_base, SlRecords rec,
                             u32* slot_cnt);
void launch_flush_starts(hipStream_t s, const i64* out_send, i64 n_rows, i64* blk_cnt, int nb);
void launch_iota_i64(hipStream_t s, i64* a, i64 n);
void launch_flush_write(hipStream_t s, const i64* out_send, const i64* out_clock, i64 n_rows, const i64* blk_pre,
                        int nb, i64* flush_off, i64* flush_clock);
void launch_sl_regrow(hipStream_t s, const u64* old_buf, u64* new_buf, const i64* head, const i64* len, i64 nslots,
                      int nsub, i64 old_rc, i64 new_rc, bool per_sub);
void launch_sl_rekey_map(hipStream_t s, i64 size, KeyTable old_kt, KeyTable new_kt, const i64* rhead, const i64* rlen,
                         const i64* rpm, i64 rc, i64 T, i64 bound, u32* map);
void launch_sl_rekey_copy(hipStream_t s, const void* src, void* dst, i64 outer, i64 n, i64 inner, const u32* map);

// ---- expired / all-events output of time / externalTime windows (sh_slx_kernels.hip) ----
// rows indexed by operation index (the position of the row's first qualifying operation)
struct SlxRows {
    i64* ts;
    i64* rep;
    u32* slot;
    i64* ch;   // chunk: 2 * send (timer chunk before the send) or 2 * send + 1 (the send's own chunk)
    i64* clk;  // flush clock of the chunk
    unsigned char* exp;
    u64* vals;
    unsigned char* nulls;
    i64 cap;
    // k_slx_wkey: one record of rw words per row instead of the columns above — {ts, rep, ch, clk,
    // slot | exp << 32 | nulls << 40, values...} — one contiguous store per row (r05: the eight column
    // stores per row were 23 of the replay's 34 ms in c3all)
    u64* aos = nullptr;
    int rw = 0;
    // partitioned externalTimeBatch with replaceTimestampWithBatchEndTime: the rows' representative
    // events' batch end (the timestamp attribute the window wrote into them)
    i64* xa = nullptr;
};
constexpr int slx_row_words(int n_aggs) { return (5 + n_aggs + 1) & ~1; }
void launch_slx_sends(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp, const i64* blk_pass_pre,
                      const i64* blk_tl_pre, int nblk, i64* sK, i64* scb, i64* slast);
// kind 0: the calls among n sends -> (oK, oC, oS); kind 1: indices of the set flags -> oS.
// blk: (n + kTile - 1) / kTile + 1 entries; blk[last] = the count
void launch_slx_compact(hipStream_t s, int kind, const unsigned char* flags, const i64* sK, const i64* scb,
                        const i64* slast, i64 n, i64* blk, i64* oK, i64* oC, i64* oS);
void launch_slx_notify(hipStream_t s, const i64* pend, i64 n_pend, const i64* pm, i64 M, i64 pm0, const i64* cK,
                       const i64* cC, i64 nC, i64 T, unsigned char* fire, unsigned char* keep);
void launch_slx_gather_calls(hipStream_t s, const i64* idx, i64 n, const i64* cK, const i64* cC, const i64* cS, i64* fK,
                             i64* fC, i64* fS);
void launch_slx_gather_pend(hipStream_t s, const i64* idx, i64 n, const i64* pend, i64 n_pend, const i64* pm,
                            i64* out);
void launch_slx_append(hipStream_t s, const i64* pm, const u32* raw, i64 M, i64 seq_base, i64* upm, i64* useq);
// xx (nullable): the record form for k_slx_wkey instead of the xop / xch / xts / xclk columns (useq and
// the records' first value column fill it)
void launch_slx_expiry(hipStream_t s, const i64* upm, i64 n_u, i64 W0, i64 M, const i64* rclk, const i64* rsclk,
                       const u32* raw, i64 send_size, const i64* fK, const i64* fC, const i64* fS, i64 nF, i64 T,
                       u64* xop, i64* xch, i64* xts, i64* xclk, unsigned long long* n_exp, u64* xx,
                       const i64* useq, const u64* rvals, i64* bnd);  // bnd: 3 * (n_u / kBlock + 2) words
// xa (nullable): the record form for k_slx_wkey, from rec and (externalTime) the sends' clocks
void launch_slx_aop(hipStream_t s, const i64* rclk, i64 M, const i64* upm, i64 n_u, i64 W0, i64 T, u64* aop,
                    u64* xa, SlRecords rec, const i64* rsclk, i64* bnd);  // bnd: M / kBlock + 2 words
void launch_slx_keyoff(hipStream_t s, const u32* slot_cnt, i64 nslots, u32* key_off, i64* tmp);
void launch_slx_walk(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, SlRecords rec,
                     const u64* aop, const u64* xop, const i64* xch, const i64* xts, const i64* xclk, const i64* useq,
                     i64 n_u, i64 X0, i64 G0, i64 seq_base, i64 send_size, SlState S, i64* rg, AggPlan ap, int cur_on,
                     int exp_on, SlxRows rows, unsigned char* flags, const i64* rsclk);
// the same replay with one wave per key (sh_sliding_kernels.hip) for the count / sum / avg / min / max of
// one double column shape (slx_keyed_ok)
bool slx_keyed_ok(AggPlan ap);
// xa: per record {aop, value, ts, clock, raw, pm}; xx: per window position {xop, value (this push's
// records), ts, clock, event, chunk} (k_slx_aop / k_slx_expiry with their record outputs)
constexpr int kXaWords = 6;
void launch_slx_wkey(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, const u64* xa,
                     const u64* xx, i64 n_u, i64 X0, i64 G0, i64 seq_base, i64 send_size, SlState S, i64* rg,
                     AggPlan ap, int cur_on, int exp_on, SlxRows rows, unsigned char* flags);
void launch_slx_pass(hipStream_t s, SlRecords rec, i64 M, const u64* aop, const u64* xop, const i64* xch, const i64* xts,
                     const i64* xclk, const i64* useq, i64 n_u, i64 seq_base, i64 send_size, int cur_on, int exp_on,
                     SlxRows rows, unsigned char* flags, const i64* rsclk);
// emission from the row records of k_slx_wkey (SlxRows.aos)
void launch_slx_emit_aos(hipStream_t s, const unsigned char* flags, i64 n, const i64* blk_pre, int nblk, SlxRows rows,
                         int n_aggs, KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals,
                         unsigned char* out_nulls, unsigned char* out_exp, i64* out_ch, i64* out_clock, i64* out_rep);
void launch_slx_emit(hipStream_t s, const unsigned char* flags, i64 n, const i64* blk_pre, int nblk, SlxRows rows,
                     int n_aggs, KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals,
                     unsigned char* out_nulls, unsigned char* out_exp, i64* out_ch, i64* out_clock, i64* out_rep);
void launch_slx_shift(hipStream_t s, const i64* upm, const i64* useq, i64 from, i64 n, i64* opm, i64* oseq);
void launch_slx_rekey_map(hipStream_t s, i64 size, KeyTable old_kt, KeyTable new_kt, const i64* rlen, const i64* cnt,
                          const u64* f, i64 nslots, AggPlan ap, u32* map);

// ---- partitioned lengthBatch / time windows keyed by the partition (sh_plane_kernels.hip) ----
void launch_pl_walk_lb(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, SlRecords rec, i64 L,
                       i64 seq_base, SlState S, i64* last_ts, i64* last_seq, i64* prev_seq, AggPlan ap, int cur_on,
                       int exp_on, int sc, SlxRows rows, unsigned char* flags);
void launch_pl_runs(hipStream_t s, ColSet cols, int pcol, i64 N, i64 send_size, unsigned char* start, i64* blk,
                    i64* run);
void launch_pl_slot_key(hipStream_t s, ColSet cols, KeyPlan kp, KeyTable kt, i64 N, i64* slot_key);
void launch_pl_notify(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, const i64* ts, i64* last_ts,
                      unsigned char* reg);
void launch_pl_walk_tm(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, SlRecords rec,
                       const i64* run, i64 T, i64 seq_base, i64 send_size, const i64* t_off, const i64* t_send,
                       const i64* t_clk, const i64* t_pos, const i64* f_send, i64 nF, SlState S, i64* rseq, AggPlan ap,
                       int cur_on, int exp_on, SlxRows rows, unsigned char* flags, const i64* xattr = nullptr);
void launch_pl_xattr(hipStream_t s, ColSet cols, int xcol, const u32* raw, i64 M, i64* x);
void launch_pl_emit(hipStream_t s, const unsigned char* flags, i64 n, const i64* blk_pre, int nblk, SlxRows rows,
                    int n_aggs, int nk, KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals,
                    unsigned char* out_nulls, unsigned char* out_exp, i64* out_ch, i64* out_clock, i64* out_rep,
                    u32* out_part);

}  // namespace shd
