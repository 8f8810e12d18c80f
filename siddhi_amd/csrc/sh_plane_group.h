// sh_plane_group.h — partitioned lengthBatch grouped by a key other than the partition key
// (sh_plane_group_kernels.hip, driven by sh_plane.cpp).
#pragma once
#include "sh_sliding.h"

namespace shd {

// records carried between pushes (the partitions' open batches and, with expired output, their last
// completed batch) followed by the push's own: the combined order is stream order
struct PgRecs {
    u32* ps;             // partition slot
    u32* gs;             // group slot
    i64* ts;
    i64* seq;            // stream index of the event
    i64* clk;            // playback clock of the event's send
    u64* vals;           // [n_vcols][cap]
    unsigned char* prev; // carried as the partition's last completed batch
    i64 cap;
    i64* x;              // externalTimeBatch: the timestamp attribute
    i64* xe;             // externalTimeBatch: the end time of the event's batch (cloneAppend :446-456)
    i64* xm;             // externalTimeBatch: lastCurrentEventTime once the event is in (its partition's max)
};


// externalTimeBatch under `partition with` (ExternalTimeBatchWindowProcessor.process :238-311 per
// partition): per partition slot the running max of the attribute (lastCurrentEventTime), the start,
// and the bucket (M - start) / T of its open batch
struct PgExt {
    i64* M;
    i64* start;
    unsigned char* has;
    i64* bopen;
    int has_start;       // 0: first event's attribute, 1: constant, 2: start attribute
    int xcol, scol;
    i64 start_time, T;
};

// externalTimeBatch's timeout under `partition with`: one emission (a selector chunk) of partition p —
// [its previous emission's events as EXPIRED, RESET, the open batch from its first event] — found by the
// host's Scheduler walk (sh_plane.cpp xt_walk); ranges are relative to the partition's sorted run
struct PgXtEmit {
    u32 p, pad;
    i64 lo, hi;    // CURRENT: the open batch so far [lo, hi)
    i64 xlo, xhi;  // EXPIRED: the previous emission's CURRENT range
    i64 off;       // first entry of the emission in the expanded entry list
    i64 sidx;      // the record whose running max stamps the expired rows (lastCurrentEventTime)
    i64 clock;     // flush clock
};
// per push position: running max, batch end, and flags for the host walk (bit 1 the partition's first
// event — initTiming; bit 0 a crossing into a higher bucket — a new batch)
void launch_pg_xt_flags(hipStream_t s, const u32* key_off, const u32* ranks, const u32* prev_cnt, const u32* pend_cnt,
                        PgRecs C, const i64* xs, const i64* ms, PgExt X, i64 n, unsigned char* flag, int* err);
// the emissions' entries (EXPIRED first, then CURRENT, each in stream order): key (emission, group slot),
// value = entry index | CURRENT << 31, epos = sorted position
void launch_pg_xt_expand(hipStream_t s, const PgXtEmit* em, i64 ne, i64 n_ent, const u32* key_off, const u32* ranks,
                         PgRecs C, int gbits, int cur_on, int exp_on, u64* ekey, u32* eval, u32* epos);
// keep[c] = 2 for the records at or past their partition's keep-from index kf[p] (run-relative)
void launch_pg_xt_keep(hipStream_t s, const u32* key_off, const u32* ranks, PgRecs C, i64 n, const u32* kf,
                       unsigned char* keep);
void launch_pg_xt_kf(hipStream_t s, const u32* slots, const u32* vals, i64 n, u32* kf);

void launch_pg_append(hipStream_t s, SlRecords rec, i64 M, i64 n_old, i64 seq_base, ColSet cols, KeyPlan gkp,
                      KeyTable gkt, int nv, PgRecs C, u32* slot_cnt, u32* prev_cnt, int xcol = -1, int scol = -1,
                      i64* xs = nullptr, u32* pend_cnt = nullptr);
// externalTimeBatch: the attribute in sorted order, its running max per partition run (rocPRIM
// scan-by-key), the entries, then the partitions' state
int launch_pg_ext_scan(hipStream_t s, const u32* ranks, const u32* p_sorted, PgRecs C, i64 n, i64* xv, i64* ms,
                       void* temp, size_t* temp_bytes);
void launch_pg_assign_ext(hipStream_t s, const u32* key_off, const u32* ranks, const u32* prev_cnt, const u32* pend_cnt,
                          PgRecs C, const i64* xs, const i64* ms, PgExt X, i64 n, int cur_on, int exp_on, int gbits,
                          u64 none, u64* ekey, u32* eval, unsigned char* keep, unsigned long long* n_entries, i64* chunk_ts,
                          int* err);
void launch_pg_ext_state(hipStream_t s, const u32* key_off, const u32* ranks, const u32* prev_cnt, const u32* pend_cnt,
                         PgRecs C, const i64* xs, const i64* ms, PgExt X, i64 nslots);
void launch_pg_assign(hipStream_t s, const u32* key_off, const u32* ranks, const u32* p_sorted, const u32* prev_cnt,
                      PgRecs C, i64 n, i64 L, int cur_on, int exp_on, int gbits, u64 none, u64* ekey, u32* eval,
                      unsigned char* keep, unsigned long long* n_entries);
void launch_pg_heads(hipStream_t s, const u64* key, i64 n, unsigned char* head);
// lengthBatch(L, true) grouped by other columns: entries by (batch, group), a row per event of the push
void launch_pg_sc_assign(hipStream_t s, const u32* key_off, const u32* ranks, const u32* p_sorted, PgRecs C, i64 n,
                         i64 L, int gbits, u64* ekey, u32* eval, unsigned char* keep);
void launch_pg_sc_fold(hipStream_t s, const i64* seg_start, i64 n_seg, i64 n_e, const u64* ekey, const u32* eval,
                       const u32* ranks, PgRecs C, AggPlan ap, int gbits, i64 n_old, SlxRows rows, u32* row_part);
void launch_pg_fold(hipStream_t s, const i64* seg_start, i64 n_seg, i64 n_e, const u64* ekey, const u32* eval,
                    const u32* ranks, PgRecs C, AggPlan ap, int gbits, SlxRows rows, u64* row_key, u32* row_part,
                    const i64* chunk_ts = nullptr, const PgXtEmit* xem = nullptr, const u32* epos = nullptr,
                    const u32* key_off = nullptr);
void launch_pg_emit(hipStream_t s, const u32* order, i64 n, SlxRows rows, int n_aggs, int nk, KeyTable kt, KeyPlan kp,
                    i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals, unsigned char* out_nulls,
                    unsigned char* out_exp, i64* out_ch, i64* out_clock, i64* out_rep, const u32* row_part,
                    u32* out_part, i64* out_xa = nullptr);
void launch_pg_gather(hipStream_t s, const i64* idx, i64 n, const unsigned char* keep, PgRecs C, PgRecs D, int nv);
// stable sort of (u64 key, u32 value) pairs over key bits [0, end_bit)
int sort_u64_pairs_bits(void* temp, size_t* bytes, const u64* keys, u64* keys_out, const u32* vals, u32* vals_out,
                        i64 n, unsigned end_bit, hipStream_t s);
int sort_u64_pairs_range(void* temp, size_t* bytes, const u64* keys, u64* keys_out, const u32* vals, u32* vals_out,
                         i64 n, unsigned begin_bit, unsigned end_bit, hipStream_t s);
// time / externalTime windows grouped by other columns: the partitions' operations in order
struct PgOps {
    i64* pos;            // chunk position (the lanes' output position of the point)
    u32* pg;             // (partition, group) state slot; 0xFFFFFFFF = no operation
    unsigned char* kind; // 1 add (CURRENT), 2 remove (EXPIRED)
    i64* seq;
    i64* ts;             // the row timestamp: the event's (add) or the point's clock / attribute (remove)
    i64* clk;
    u64* vals;           // [n_vcols][cap]
    i64 cap;
};
void launch_pg_ops_room(hipStream_t s, const u32* slot_cnt, const i64* rlen, i64 n, i64* room);
void launch_pg_rec_group(hipStream_t s, SlRecords rec, i64 M, ColSet cols, KeyPlan gkp, KeyTable gkt, int nv);
void launch_pg_walk_ops(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, SlRecords rec,
                        const i64* run, i64 T, i64 seq_base, i64 send_size, const i64* t_off, const i64* t_send,
                        const i64* t_clk, const i64* t_pos, const i64* f_send, i64 nF, SlState S, i64* rseq, int nv,
                        const i64* xattr, KeyTable pgkt, const i64* obase, PgOps O, u32* o_cnt);
// min / max deques of the (partition, group) states: pool[off[f * n + s], + len[f * n + s]) for the
// min / max fields field[0 .. nf)
struct PgDeques {
    int nf;
    int field[SH_MAX_AGGS];
    i64 n;               // states
    u64* pool;
    i64* off;
    i64* len;
    u64* scratch;        // the push's working areas
    i64* new_at;         // after the replay: scratch index / length of an active state's deque
    i64* new_len;
    unsigned char* active;
};
void launch_pg_dq_need(hipStream_t s, const i64* seg_start, i64 n_seg, i64 n_ops, const u32* skey, const u32* sidx,
                       PgOps O, PgDeques D, i64* need);
void launch_pg_replay(hipStream_t s, const i64* seg_start, i64 n_seg, i64 n_ops, const u32* skey, const u32* sidx,
                      PgOps O, KeyTable pgkt, i64* st_cnt, u64* st_f, i64 st_n, AggPlan ap, int cur_on, int exp_on,
                      SlxRows rows, u64* row_key, u32* row_part, unsigned int* n_rows, PgDeques D, const i64* scr_off);
void launch_pg_dq_len(hipStream_t s, PgDeques D, i64* out_len);
void launch_pg_dq_pool(hipStream_t s, PgDeques D, const i64* off_out, u64* pool_out, i64* new_off);
// rebuild of the pair table: live states counted, then moved into a fresh table (state arrays of n slots,
// the last the sentinel; F fields, field-major)
void launch_pg_count_live(hipStream_t s, KeyTable kt, i64 n, const i64* cnt, const u64* f, const i64* dql, int F,
                          unsigned long long* n_live);
void launch_pg_rehash(hipStream_t s, KeyTable okt, i64 on, const i64* cnt, const u64* f, const i64* dqo, const i64* dql,
                      int F, KeyTable nkt, i64 nn, i64* ncnt, u64* nf, i64* ndqo, i64* ndql);
void launch_pg_heads32(hipStream_t s, const u32* key, i64 n, unsigned char* head);
void launch_pg_sum_u32(hipStream_t s, const u32* a, i64 n, unsigned long long* out);
int sort_u64_iota_bits(void* temp, size_t* bytes, const u64* keys, u64* keys_out, u32* vals_out, i64 n,
                       unsigned end_bit, hipStream_t s);
// partitioned timeBatch(T, true) (lane 4): per (partition, group) state — batch number, count and per
// aggregator its running value and has-flag ([a][n] layouts)
struct TbState {
    i64* cnt;
    i64* bid;
    u64* f;
    unsigned char* has;
    i64 n;
};
void launch_tb_chunk_flags(hipStream_t s, SlRecords rec, i64 M, const i64* run, unsigned char* flag);
void launch_tb_chunk_info(hipStream_t s, SlRecords rec, const i64* first, i64 nch, i64 send_size, u32* slot, i64* send,
                          i64* clock);
void launch_tb_chunk_of(hipStream_t s, const i64* first, i64 nch, i64 M, i64* chunk_of);
void launch_tb_pairs(hipStream_t s, SlRecords rec, i64 M, ColSet cols, KeyPlan gkp, KeyTable gkt, KeyTable pgkt,
                     u32* pair, u32* gslot);
void launch_tb_fold(hipStream_t s, const i64* seg_start, i64 n_seg, i64 M, const u32* skey, const u32* sidx,
                    SlRecords rec, const i64* chunk_of, const i64* chunk_bid, const u32* gslot, AggPlan ap, TbState S,
                    i64 chunk_base, SlxRows rows, u64* row_key, u32* row_part, unsigned int* n_rows, i64 seq_base);

}  // namespace shd
