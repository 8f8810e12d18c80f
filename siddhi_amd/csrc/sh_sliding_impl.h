// sh_sliding_impl.h — host state of a query of kind 1 (sh_sliding.cpp: time / externalTime windows;
// sh_plane.cpp: partitioned lengthBatch / time windows keyed by the partition).
#pragma once
#include <cstdint>
#include <deque>
#include <set>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "sh_runtime.h"
#include "sh_jmap.h"
#include "sh_sliding.h"
#include "sh_plane_group.h"

using shd::SlInfo;

// lane 3 (partitioned lengthBatch grouped by other columns): a set of carried / combined records
struct PgBufs {
    DevBuf ps, gs, ts, seq, clk, vals, prev, x, xe, xm;
    int64_t cap = 0;
    shd::PgRecs view() const {
        return shd::PgRecs{ps.as<uint32_t>(), gs.as<uint32_t>(), ts.as<int64_t>(), seq.as<int64_t>(), clk.as<int64_t>(),
                           vals.as<shd::u64>(), prev.as<unsigned char>(), cap, x.as<int64_t>(),
                           xe.as<int64_t>(), xm.as<int64_t>()};
    }
};

struct SlidingImpl {
    int64_t nslots = 0, rc = 0;
    int P = 1, logP = 0;
    int64_t pm = INT64_MIN;   // PM carried across pushes
    int64_t send_base = 0;    // global send number of the push's first send
    int64_t rekey_floor = 0;  // key count above which the next key-table rebuild runs (hysteresis)
    DevBuf cnt, f, mm, mm_has, dq_head, dq_len, dq, rhead, rlen, rpm, rval, cur_send, cur_first;
    // per push scratch
    DevBuf blk_pass, blk_tl, blk_pm, info, rec_raw, rec_slot, rec_clock, rec_pm, rec_ts, rec_vals, slot_cnt, counts,
        tmp, ranks, part_off, flags, rec_sclk, p_raw, p_slot, p_clock, p_pm, p_ts, p_vals, rows_ts, rows_rep, rows_slot, rows_send, rows_clock, rows_vals, rows_nulls, blk_cnt, out_ts,
        out_keys, out_vals, out_nulls, out_send, out_clock, out_expired, out_rep, flush_off, flush_clock, sort_tmp,
        key_off, g_rank, inv, rows_k, rec_aos;
    SlInfo* h_info = nullptr;
    PinnedBuf h_up;  // pinned staging of small host->device uploads
    sh_out dev_out{};
    // the push's flush offsets / clocks: flush_off / flush_clock, or (a row per send) the persistent
    // identity `iota` and the rows' own clocks
    DevBuf iota;
    int64_t iota_n = 0;
    const int64_t* fo = nullptr;
    const int64_t* fc = nullptr;

    // `insert expired events` / `insert all events` (sh_slx_kernels.hip): the expiry queue as a FIFO
    // of the window's events (PM and stream index, global arrival order X0 .. G0), each ring entry's
    // arrival index, and the scheduler's pending notify times (ascending)
    bool xm = false;
    DevBuf rg, upm, useq, upm2, useq2, npend, npend2;
    int64_t x0 = 0, g0 = 0, w0 = 0, n_np = 0, np_front = 0;
    DevBuf x_sK, x_scb, x_slast, x_cK, x_cC, x_cS, x_fire, x_keep, x_idx, x_fK, x_fC, x_fS, x_blk, x_xop, x_xch,
        x_xts, x_xclk, x_aop, x_nexp, xr_ts, xr_rep, xr_slot, xr_ch, xr_clk, xr_exp, xr_vals, xr_nulls, xr_aos, x_xa, x_xx, x_bnd;
    PinnedBuf x_h;
    // partitioned windows keyed by the partition (sh_plane.cpp): lane = 1 lengthBatch, 2 time; per slot the
    // open batch's last event, the last flushed batch's last event (expired rows), lastTimestamp, the
    // partition key; host side the Scheduler: pending notify times per partition, the armed partitions by
    // front due time, and PartitionStateHolder.states in java.util.HashMap order (sh_jmap.h) over the
    // partitions' String.valueOf(key)
    int lane = 0;
    int nk_out = -1;  // output key columns (0: no group-by, the partition key is internal)
    DevBuf pl_last_ts, pl_last_seq, pl_prev_seq, pl_key, pl_start, pl_run, pl_reg, pl_toff, pl_tsend, pl_tclk,
        pl_tpos, pl_fsend, pl_x;
    std::unordered_map<uint32_t, std::deque<int64_t>> pl_pend;
    std::set<std::pair<int64_t, uint32_t>> pl_armed;  // (front notify time, slot)
    shj::JavaStringMap pl_states;
    std::unordered_map<uint32_t, std::u16string> pl_flow;  // slot -> String.valueOf(partition key)
    // lane 3: the carried records (pg[0], pg_n of them in stream order), the compaction target pg[1],
    // and the push's entry / segment / row scratch
    PgBufs pg[2];
    int64_t pg_n = 0;
    DevBuf out_part;  // the lanes' output rows: partition slot of each (per-partition rate limiters)
    // externalTimeBatch lanes: per partition slot the running max, start, started flag, open bucket
    DevBuf xr_xa, out_xa;
    // partitioned externalTimeBatch with a timeout: per partition slot the window state the Scheduler walk
    // needs (ExternalTimeBatchWindowProcessor.WindowState :495-517), indices relative to the partition's run
    // of carried + new records; the device's keep-from array and the push's emissions / entries
    struct XtPart {
        int64_t n = 0;                // records of the partition in the run so far
        int64_t bs = 0;               // first record of the open batch
        int64_t cur0 = 0;             // first record not yet sent (currentEventChunk)
        int64_t pe_lo = 0, pe_hi = 0; // the previous emission's CURRENT records (expiredEventChunk)
        int64_t L = 0;                // lastScheduledTime
        bool flushed = false;
    };
    std::unordered_map<uint32_t, XtPart> xt_parts;
    // partitioned timeBatch(T, true) (lane 4): the shared nextEmitTime, every partition's RESET count
    // (its batch number), the (partition, group) states and the push's scratch
    int64_t tb_next_emit = -1, tb_chunk_base = 0;
    std::unordered_map<uint32_t, int64_t> tb_bids;
    DevBuf tb_cnt, tb_bid, tb_f, tb_has, tb_run, tb_start, tb_blk, tb_flag, tb_first, tb_cslot, tb_csend, tb_cclk,
        tb_chunk_of, tb_chbid, tb_pair, tb_gslot, tb_skey, tb_sidx, tb_seg, tb_head, tb_rkey, tb_rkey2, tb_order, tb_nrows;
    DevBuf xt_kf, xt_em, xt_epos, xt_flag, xt_up;  // partitioned externalTimeBatch, replaceTimestampWithBatchEndTime: rows' batch ends
    DevBuf pg_M, pg_start, pg_has, pg_bopen, pg_pendcnt, pg_xs, pg_xv, pg_ms, pg_cts, pg_err;
    // time lanes grouped by other columns: operation lists, their sort, the (partition, group) states
    DevBuf pg_room, op_pos, op_pg, op_kind, op_seq, op_ts, op_clk, op_vals, pg_ocnt, pg_skey, pg_sidx, pg_st_cnt, pg_st_f;
    int64_t pg_st_n = 0;
    // their min / max deques: a pool with per (field, state) offsets / lengths, the push's scratch
    DevBuf pg_dq_pool, pg_dq_pool2, pg_dq_off, pg_dq_off2, pg_dq_len, pg_dq_scr, pg_dq_at, pg_dq_nlen, pg_dq_act,
        pg_dq_need, pg_dq_lens;
    int64_t pg_dq_words = 0;
    DevBuf pg_rpart, pg_prevcnt, pg_ekey, pg_ekey2, pg_eval, pg_eval2, pg_keep, pg_head, pg_seg, pg_rkey, pg_rkey2, pg_order,
        pg_cnt;
};


// shared by sh_sliding.cpp and sh_plane.cpp
shd::SlState state_of(SlidingImpl* s);
int size_rings(sh_query* q, int64_t new_rc, bool keep = true);
int empty_out(sh_query* q, const sh_out** out);
int sliding_flushes(sh_query* q, int64_t n_rows, int64_t* n_flushes_out, bool per_row = false);
int sliding_output(sh_query* q, int64_t n_rows, int64_t n_flushes, bool want_order, bool host_out, const sh_out** out);
int read_count(sh_query* q, const int64_t* dev, int64_t* out);
int plane_create(sh_query* q);
int plane_push(sh_query* q, const sh_batch* b, bool host_out, const sh_out** out);
int plane_advance(sh_query* q, int64_t now, const sh_out** out, bool host_out);
void plane_state_buffers(sh_query* q, std::vector<std::pair<DevBuf*, size_t>>& bufs);
int plane_host_save(sh_query* q, std::vector<uint8_t>& out);
int plane_host_load(sh_query* q, const uint8_t* p, size_t n, size_t* used);
