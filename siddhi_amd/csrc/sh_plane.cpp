// sh_plane.cpp — `partition with (p of S) begin from S[cond]#window.lengthBatch(L) | time(T) select
// [p,] aggs [group by p] insert [current|all|expired] events into O; end` on the GPU.
//
// PartitionStreamReceiver.receive (core/partition/PartitionStreamReceiver.java:176-272) gives every
// partition its own window and aggregator states (PartitionRuntimeImpl.initPartition :346-367). With
// the group key equal to the partition key (or no group-by) a selector chunk holds one key, so each
// partition is an independent sequential machine: one GPU lane per partition replays it
// (sh_plane_kernels.hip). Every chunk yields at most one row and is its own flush:
//  * lengthBatch: each batch a partition completes (LengthBatchWindowProcessor.processFullBatchEvents
//    :206-243), at its L-th event's position in the stream;
//  * time: each run of consecutive same-partition events of a send (the receiver's chunk), and each
//    TIMER call the Scheduler fires for the partition (Scheduler.onTimeChange :71-104). Which partition
//    fires at which call is the Scheduler's own logic — notify times per partition, a TreeMultimap keyed
//    by due time whose equal keys keep only the first state met while walking PartitionStateHolder.states,
//    a java.util.HashMap<String, …> (sh_jmap.h) — and runs here on the host over the device-computed
//    notify registrations; the windows and aggregators stay on the GPU.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <numeric>
#include <string>
#include <vector>

#include "sh_sliding_impl.h"

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

static int fill(DevBuf& b, size_t bytes, int v) {
    RCHK(b.reserve(std::max<size_t>(bytes, 8), false));
    HIPCHK(hipMemsetAsync(b.p, v, std::max<size_t>(bytes, 8), g_stream));
    return SH_OK;
}

int plane_create(sh_query* q) {
    SlidingImpl* s = q->sl;
    s->lane = q->plane_tbsc ? 4 : q->plane_sorted ? 3 : q->d.window == SH_WIN_LENGTH_BATCH ? 1 : 2;
    s->nk_out = q->d.n_group_by;
    const size_t n = (size_t)s->nslots;
    RCHK(fill(s->pl_last_ts, n * 8, 0x80));  // lastTimestamp = Long.MIN_VALUE (0x8080... < any real ts)
    RCHK(fill(s->pl_last_seq, n * 8, 0));
    RCHK(fill(s->pl_prev_seq, n * 8, 0xff));  // -1: no batch flushed yet
    RCHK(fill(s->pl_key, n * 8, 0));
    if (s->lane == 2 && !s->rg.p) RCHK(s->rg.reserve(n * s->rc * 8, false));
    if (q->group_other && s->lane == 2) {
        // (partition, group) states of the time lanes grouped by other columns: count and sums
        s->pg_st_n = (int64_t)q->pgkt.size_ + 1;
        const size_t F = (size_t)std::max(1, q->ap.n_fields);
        RCHK(fill(s->pg_st_cnt, (size_t)s->pg_st_n * 8, 0));
        RCHK(fill(s->pg_st_f, F * s->pg_st_n * 8, 0));
        RCHK(fill(s->pg_dq_off, F * s->pg_st_n * 8, 0));
        RCHK(fill(s->pg_dq_len, F * s->pg_st_n * 8, 0));
        RCHK(fill(s->pg_dq_pool, 64, 0));
        s->pg_dq_words = 0;
    }
    if (s->lane == 4) {
        // the (partition, group) states: batch number 0, count 0, no value
        const size_t ns = q->pgkt.size_ + 1, A = (size_t)std::max(1, q->ap.n);
        RCHK(fill(s->tb_cnt, ns * 8, 0));
        RCHK(fill(s->tb_bid, ns * 8, 0));
        RCHK(fill(s->tb_f, A * ns * 8, 0));
        RCHK(fill(s->tb_has, A * ns, 0));
    }
    if (q->d.window == SH_WIN_EXT_TIME_BATCH) {
        RCHK(fill(s->pg_M, n * 8, 0));
        RCHK(fill(s->pg_start, n * 8, 0));
        RCHK(fill(s->pg_has, n, 0));
        RCHK(fill(s->pg_bopen, n * 8, 0));
    }
    return SH_OK;
}

// host copy of n i64 from the device
static int d2h(sh_query* q, std::vector<int64_t>& v, const void* dev, int64_t n) {
    v.resize((size_t)std::max<int64_t>(n, 0));
    if (n > 0) {
        HIPCHK(hipMemcpyAsync(v.data(), dev, (size_t)n * 8, hipMemcpyDeviceToHost, q->ctx->stream));
        HIPCHK(hipStreamSynchronize(q->ctx->stream));
    }
    return SH_OK;
}

static int h2d(sh_query* q, DevBuf& b, const std::vector<int64_t>& v) {
    RCHK(b.reserve(std::max<size_t>(v.size(), 1) * 8, false));
    if (!v.empty()) HIPCHK(hipMemcpyAsync(b.p, v.data(), v.size() * 8, hipMemcpyHostToDevice, q->ctx->stream));
    HIPCHK(hipStreamSynchronize(q->ctx->stream));  // v is pageable and may be freed after the call
    return SH_OK;
}

struct Firing {
    int64_t send, clock, K;
    uint32_t slot;
};

// String.valueOf(partition key) (ValuePartitionExecutor.execute :34-40): Integer / Long / Float /
// Double.toString, Boolean.toString, or the string itself (its UTF-16 text from sh_query_set_strings)
static int flow_id(sh_query* q, int64_t key, std::u16string* out) {
    const int c = q->d.partition_col;
    switch (q->d.col_types[c]) {
        case SH_T_INT:
        case SH_T_LONG: {
            const std::string d = std::to_string(key);
            out->assign(d.begin(), d.end());
            return SH_OK;
        }
        case SH_T_BOOL: *out = key ? u"true" : u"false"; return SH_OK;
        case SH_T_STRID: {
            auto it = q->strings.find(c);
            if (it != q->strings.end() && key >= 0 && key < (int64_t)it->second.size() && q->strings_set[c][(size_t)key]) {
                *out = it->second[(size_t)key];
                return SH_OK;
            }
            return sh_fail(SH_ERR_INVALID, "partition key string id " + std::to_string(key) +
                                               " has no text: the Scheduler's tie rule orders partitions by "
                                               "String.hashCode (call sh_query_set_strings)");
        }
        case SH_T_FLOAT:
        case SH_T_DOUBLE: {  // Float / Double.toString of the value (the key is its bits widened to double)
            double v;
            std::memcpy(&v, &key, 8);
            *out = shj::java_fp_text(v, q->d.col_types[c] == SH_T_FLOAT);
            return SH_OK;
        }
        default: return sh_fail(SH_ERR_UNSUPPORTED, "partition key type without a String.valueOf restatement");
    }
}

// Scheduler.onTimeChange at one call (clock c). getAllStates() is walked in HashMap order and each due
// state is put into a TreeMultimap<Long, SchedulerState> whose values compare equal: per distinct due time
// the first state met fires, popping all of its due times (sendTimerEvents :171-209); returnAllStates then
// removes the emptied states (canDestroy :343-346) through the iterator, in iteration order.
static void sched_call(SlidingImpl* s, int64_t send, int64_t c, int64_t K, std::vector<Firing>& out) {
    std::vector<std::pair<int64_t, uint32_t>> win;  // (due time, slot) per distinct due time
    int64_t best = 0;
    for (auto it = s->pl_armed.begin(); it != s->pl_armed.end() && it->first <= c; ++it) {
        int64_t r = 0;
        s->pl_states.rank(s->pl_flow[it->second], &r);
        if (win.empty() || win.back().first != it->first) {
            win.push_back(*it);
            best = r;
        } else if (r < best) {
            win.back() = *it;
            best = r;
        }
    }
    std::vector<std::pair<int64_t, uint32_t>> gone;  // (HashMap rank, slot) of the emptied states
    for (auto& w : win) {
        s->pl_armed.erase(w);
        const uint32_t slot = w.second;
        auto& pend = s->pl_pend[slot];
        while (!pend.empty() && pend.front() <= c) pend.pop_front();
        out.push_back(Firing{send, c, K, slot});
        if (pend.empty()) {
            s->pl_pend.erase(slot);
            int64_t r = 0;
            s->pl_states.rank(s->pl_flow[slot], &r);
            gone.emplace_back(r, slot);
        } else {
            s->pl_armed.insert(std::make_pair(pend.front(), slot));
        }
    }
    std::sort(gone.begin(), gone.end());
    for (auto& g : gone) s->pl_states.erase(s->pl_flow[g.second]);
}

// Scheduler.notifyAt (:113-127): stateHolder.getState() = states.computeIfAbsent(flow id) (a resize
// check even for a present key), then the time joins the partition's queue
static int sched_register(sh_query* q, uint32_t slot, int64_t t, const std::vector<int64_t>& slot_key) {
    SlidingImpl* s = q->sl;
    auto fl = s->pl_flow.find(slot);
    if (fl == s->pl_flow.end()) {
        std::u16string name;
        RCHK(flow_id(q, slot_key[slot], &name));
        fl = s->pl_flow.emplace(slot, std::move(name)).first;
    }
    s->pl_states.touch(fl->second, slot);
    auto& pend = s->pl_pend[slot];
    if (pend.empty()) s->pl_armed.insert(std::make_pair(t, slot));
    pend.push_back(t);
    return SH_OK;
}

// Scheduler.onTimeChange at one call (clock c) whose TIMER events act on the window at once
// (sendTimerEvents :171-209 runs the window, which may notifyAt again, before returnAllStates): per
// distinct due time the first state met in HashMap order fires all its due times, each TIMER handed to
// on_timer(slot, due time) in queue order.
template <typename F>
static int sched_fire(SlidingImpl* s, int64_t c, F on_timer) {
    std::vector<std::pair<int64_t, uint32_t>> win;
    int64_t best = 0;
    for (auto it = s->pl_armed.begin(); it != s->pl_armed.end() && it->first <= c; ++it) {
        int64_t r = 0;
        s->pl_states.rank(s->pl_flow[it->second], &r);
        if (win.empty() || win.back().first != it->first) {
            win.push_back(*it);
            best = r;
        } else if (r < best) {
            win.back() = *it;
            best = r;
        }
    }
    std::vector<std::pair<int64_t, uint32_t>> gone;
    for (auto& w : win) {
        s->pl_armed.erase(w);
        const uint32_t slot = w.second;
        for (;;) {
            auto it = s->pl_pend.find(slot);
            if (it == s->pl_pend.end() || it->second.empty() || it->second.front() > c) break;
            const int64_t t = it->second.front();
            it->second.pop_front();
            RCHK(on_timer(slot, t));
        }
        auto it = s->pl_pend.find(slot);
        if (it == s->pl_pend.end() || it->second.empty()) {
            if (it != s->pl_pend.end()) s->pl_pend.erase(it);
            int64_t r = 0;
            s->pl_states.rank(s->pl_flow[slot], &r);
            gone.emplace_back(r, slot);
        } else {
            s->pl_armed.insert(std::make_pair(it->second.front(), slot));
        }
    }
    std::sort(gone.begin(), gone.end());
    for (auto& g : gone) s->pl_states.erase(s->pl_flow[g.second]);
    return SH_OK;
}

// externalTimeBatch(ts, T, start, timeout) under `partition with`: ExternalTimeBatchWindowProcessor.process
// (:238-311) per partition, walked in stream order over the push's calls (each a Scheduler.onTimeChange
// before its send's events) and passing events (flag bit 1: initTiming :313-334, bit 0: the event crosses
// into a new batch). Every emission — a TIMER's flushToOutputChunk / appendToOutputChunk (:256-275) or a
// crossing's (:292-305) — sends the open batch from its first record, behind the previous emission's
// records as EXPIRED (the expired chunk always holds what the previous emission sent as CURRENT).
static int xt_walk(sh_query* q, const std::vector<int64_t>& calls_s, const std::vector<int64_t>& calls_c,
                   const std::vector<uint32_t>& ev_slot, const std::vector<unsigned char>& ev_flag,
                   const std::vector<uint32_t>& ev_raw, int64_t ss, int64_t clock0,
                   const std::vector<int64_t>& slot_key, std::vector<PgXtEmit>& em, std::vector<uint32_t>& touched) {
    SlidingImpl* s = q->sl;
    const int64_t tau = q->xt_timeout;
    const bool exp_on = q->d.expired_on != 0;
    std::unordered_map<uint32_t, char> seen;
    auto touch = [&](uint32_t p) { if (seen.emplace(p, 1).second) touched.push_back(p); };
    auto emit = [&](uint32_t p, SlidingImpl::XtPart& P, int64_t hi, int64_t clock, int64_t sidx) {
        PgXtEmit e{};
        e.p = p;
        e.lo = P.bs;
        e.hi = hi;
        e.xlo = exp_on ? P.pe_lo : 0;
        e.xhi = exp_on ? P.pe_hi : 0;
        e.clock = clock;
        e.sidx = sidx;
        em.push_back(e);
        P.pe_lo = P.bs;
        P.pe_hi = hi;
    };
    int64_t clock = clock0;
    auto on_timer = [&](uint32_t p, int64_t t) -> int {
        auto it = s->xt_parts.find(p);
        if (it == s->xt_parts.end()) return sh_fail(SH_ERR_STATE, "externalTimeBatch timeout: a timer without window state");
        SlidingImpl::XtPart& P = it->second;
        if (P.L > t) return SH_OK;  // (rescheduled since: :258)
        touch(p);
        if (!P.flushed) {
            if (P.n > P.bs) emit(p, P, P.n, clock, P.n - 1);
            P.flushed = true;
        } else if (P.n > P.cur0) {
            emit(p, P, P.n, clock, P.n - 1);
        }
        P.cur0 = P.n;
        P.L = clock + tau;
        return sched_register(q, p, P.L, slot_key);
    };
    size_t e = 0;
    auto events_before = [&](int64_t send_end) -> int {  // the passing events of the sends before send_end
        for (; e < ev_slot.size(); e++) {
            const int64_t snd = ss > 0 ? (int64_t)ev_raw[e] / ss : 0;
            if (snd >= send_end) break;
            const uint32_t p = ev_slot[e];
            const unsigned char f = ev_flag[e];
            touch(p);
            SlidingImpl::XtPart& P = s->xt_parts[p];
            if (f & 2) {
                P = SlidingImpl::XtPart{};
                P.L = clock + tau;
                RCHK(sched_register(q, p, P.L, slot_key));
            }
            if (f & 1) {
                if (P.flushed) {
                    if (P.n > P.cur0) emit(p, P, P.n, clock, P.n);
                    P.flushed = false;
                } else if (P.n > P.bs) {
                    emit(p, P, P.n, clock, P.n);
                }
                P.bs = P.n;
                P.cur0 = P.n;
                P.L = clock + tau;
                RCHK(sched_register(q, p, P.L, slot_key));
            }
            P.n++;
        }
        return SH_OK;
    };
    for (size_t k = 0; k < calls_s.size(); k++) {
        RCHK(events_before(calls_s[k]));
        clock = calls_c[k];
        if (!s->pl_armed.empty() && s->pl_armed.begin()->first <= clock) RCHK(sched_fire(s, clock, on_timer));
    }
    return events_before(INT64_MAX);
}

// bits needed for values < n
static int bits_for(int64_t n) {
    int b = 1;
    while (b < 62 && ((int64_t)1 << b) < n) b++;
    return b;
}

// a record set with room for n records; `keep` records of `from` are copied over (column strides change)
static int pg_grow(sh_query* q, PgBufs& to, const PgBufs& from, int64_t n, int64_t keep, int V) {
    hipStream_t st = q->ctx->stream;
    if (to.cap < n) {
        const int64_t cap = std::max<int64_t>(n, to.cap + to.cap / 2);
        PgBufs nb;
        RCHK(nb.ps.reserve(cap * 4, false));
        RCHK(nb.gs.reserve(cap * 4, false));
        RCHK(nb.ts.reserve(cap * 8, false));
        RCHK(nb.seq.reserve(cap * 8, false));
        RCHK(nb.clk.reserve(cap * 8, false));
        RCHK(nb.vals.reserve((size_t)V * cap * 8, false));
        RCHK(nb.prev.reserve(cap, false));
        RCHK(nb.x.reserve(cap * 8, false));
        if (q->d.window == SH_WIN_EXT_TIME_BATCH) {  // (batch ends / attribute maxima: externalTimeBatch only)
            RCHK(nb.xe.reserve(cap * 8, false));
            RCHK(nb.xm.reserve(cap * 8, false));
        }
        nb.cap = cap;
        to = std::move(nb);
    }
    if (keep > 0 && &to != &from) {
        HIPCHK(hipMemcpyAsync(to.ps.p, from.ps.p, keep * 4, hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemcpyAsync(to.gs.p, from.gs.p, keep * 4, hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemcpyAsync(to.ts.p, from.ts.p, keep * 8, hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemcpyAsync(to.seq.p, from.seq.p, keep * 8, hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemcpyAsync(to.clk.p, from.clk.p, keep * 8, hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemcpyAsync(to.prev.p, from.prev.p, keep, hipMemcpyDeviceToDevice, st));
        HIPCHK(hipMemcpyAsync(to.x.p, from.x.p, keep * 8, hipMemcpyDeviceToDevice, st));
        if (to.xe.p && from.xe.p) {
            HIPCHK(hipMemcpyAsync(to.xe.p, from.xe.p, keep * 8, hipMemcpyDeviceToDevice, st));
            HIPCHK(hipMemcpyAsync(to.xm.p, from.xm.p, keep * 8, hipMemcpyDeviceToDevice, st));
        }
        HIPCHK(hipMemcpy2DAsync(to.vals.p, to.cap * 8, from.vals.p, from.cap * 8, keep * 8, V, hipMemcpyDeviceToDevice, st));
    }
    return SH_OK;
}

// Lane 3: partitioned lengthBatch(L) grouped by columns other than the partition key, and partitioned
// externalTimeBatch, by sorting (sh_plane_group_kernels.hip). The records carried from earlier pushes
// (every partition's open batch and, with expired output, its last completed batch) precede the push's
// own in one combined array.
// b == null: a TIMER call at `now` (sh_advance_time; only the externalTimeBatch timeout acts on it)
static int plane_run_group(sh_query* q, const sh_batch* b, int64_t now, bool host_out, const sh_out** out) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    q->stats = sh_stats{};
    const int64_t N = b ? b->n : 0, ss = b ? b->send_size : 0, L = q->d.window_param;
    const int V = std::max(1, q->ap.n_vcols), na = q->ap.n;
    const bool ext = q->d.window == SH_WIN_EXT_TIME_BATCH;
    const bool xt = ext && q->xt_timeout > 0;  // (the Scheduler decides when batches go out: xt_walk)
    const bool sc = q->d.stream_current != 0;  // lengthBatch(L, true), current output (k_pg_sc_*)
    if (N >= (int64_t)0x3FFFFFF0ll) return sh_fail(SH_ERR_INVALID, "push larger than 1G events");
    if (!b && !xt) {
        if (!q->clock_valid || now >= q->clock) {
            q->clock = now;
            q->clock_valid = true;
        }
        return empty_out(q, out);
    }
    HIPCHK(hipEventRecord(q->ev_push0, st));
    const int64_t cap = std::max<int64_t>(N, 1);
    RCHK(s->rec_raw.reserve(cap * 4, false));
    RCHK(s->rec_slot.reserve(cap * 4, false));
    RCHK(s->rec_clock.reserve(cap * 8, false));
    RCHK(s->rec_pm.reserve(cap * 8, false));
    RCHK(s->rec_ts.reserve(cap * 8, false));
    RCHK(s->rec_vals.reserve((size_t)V * cap * 8, false));
    RCHK(s->slot_cnt.reserve(s->nslots * 4, false));
    RCHK(s->pg_prevcnt.reserve(s->nslots * 4, false));
    RCHK(s->pg_pendcnt.reserve(s->nslots * 4, false));
    HIPCHK(hipMemsetAsync(s->slot_cnt.p, 0, s->nslots * 4, st));
    HIPCHK(hipMemsetAsync(s->pg_prevcnt.p, 0, s->nslots * 4, st));
    HIPCHK(hipMemsetAsync(s->pg_pendcnt.p, 0, s->nslots * 4, st));
    SlRecords rec{s->rec_raw.as<u32>(), s->rec_slot.as<u32>(), s->rec_clock.as<int64_t>(), s->rec_pm.as<int64_t>(),
                  s->rec_ts.as<int64_t>(), s->rec_vals.as<u64>(), cap};
    ColSet cs{};
    cs.n = q->d.n_cols;
    for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->d.col_types[c]; cs.ptr[c] = b ? b->cols[c] : nullptr; }
    const int nblk = (int)((N + kTile - 1) / kTile);
    RCHK(s->blk_pass.reserve(nblk * 8, false));
    RCHK(s->blk_tl.reserve(nblk * 8, false));
    RCHK(s->blk_pm.reserve(nblk * 8, false));
    WinParams wp{};
    wp.kind = SH_WIN_TIME;  // the clock / pass-count prefix of the sliding path
    wp.clock_valid = q->clock_valid;
    wp.clock0 = q->clock;
    wp.send_size = ss;
    wp.N = N;
    wp.rec_seq = q->tune.sl_records_seq;  // (the lane-strided records where they apply, as the sliding path)
    const bool sorted_off = b && sl_records_seq_applies(q->fp, wp, q->ap);
    SlInfo info{};
    if (b) {
        launch_sl_prefix(st, b->ts, cs, q->fp, wp, s->blk_pass.as<int64_t>(), s->blk_tl.as<int64_t>(),
                         s->blk_pm.as<int64_t>(), nblk, s->info.as<SlInfo>());
        // lane-strided records (every event passes): no per-slot counts; the partitions' offsets come from
        // the sorted slots below (k_counts_sorted; the LDS tables and atomics were 5.2 of plb's 20 ms)
        launch_sl_records(st, b->ts, cs, q->fp, wp, q->kp, q->kt.dev(), q->ap, s->blk_pass.as<int64_t>(),
                          s->blk_tl.as<int64_t>(), s->blk_pm.as<int64_t>(), s->pm, rec,
                          sorted_off ? nullptr : s->slot_cnt.as<u32>(), nblk);
        if (xt) launch_pl_slot_key(st, cs, q->kp, q->kt.dev(), N, s->pl_key.as<int64_t>());
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(s->h_info, s->info.p, sizeof(SlInfo), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        RCHK(q->kt.check(st));
        info = *s->h_info;
    }
    const int64_t M = info.total_pass, n_old = s->pg_n, n = n_old + M;
    int64_t n_rows = 0, n_flushes = 0;
    // the timeout: the push's calls (a send whose last event does not move the clock calls nobody,
    // TimestampGeneratorImpl :104-122), or the advance_time call
    std::vector<int64_t> calls_s, calls_c;
    bool xt_fire = false;
    if (xt) {
        if (b) {
            const int64_t NS = ss > 0 ? (N + ss - 1) / ss : 1;
            const int nbS = (int)((NS + kTile - 1) / kTile);
            RCHK(s->x_sK.reserve(NS * 8, false));
            RCHK(s->x_scb.reserve(NS * 8, false));
            RCHK(s->x_slast.reserve(NS * 8, false));
            RCHK(s->x_cK.reserve(NS * 8, false));
            RCHK(s->x_cC.reserve(NS * 8, false));
            RCHK(s->x_cS.reserve(NS * 8, false));
            RCHK(s->x_blk.reserve((size_t)((NS + kTile - 1) / kTile + 2) * 8, false));
            launch_slx_sends(st, b->ts, cs, q->fp, wp, s->blk_pass.as<int64_t>(), s->blk_tl.as<int64_t>(), nblk,
                             s->x_sK.as<int64_t>(), s->x_scb.as<int64_t>(), s->x_slast.as<int64_t>());
            launch_slx_compact(st, 0, nullptr, s->x_sK.as<int64_t>(), s->x_scb.as<int64_t>(), s->x_slast.as<int64_t>(),
                               NS, s->x_blk.as<int64_t>(), s->x_cK.as<int64_t>(), s->x_cC.as<int64_t>(),
                               s->x_cS.as<int64_t>());
            HIPCHK(hipGetLastError());
            int64_t nC = 0;
            RCHK(read_count(q, s->x_blk.as<int64_t>() + nbS, &nC));
            RCHK(d2h(q, calls_s, s->x_cS.p, nC));
            RCHK(d2h(q, calls_c, s->x_cC.p, nC));
        } else if (!q->clock_valid || now >= q->clock) {
            calls_s.push_back(0);
            calls_c.push_back(now);
        }
        xt_fire = !s->pl_armed.empty() && !calls_c.empty() && calls_c.back() >= s->pl_armed.begin()->first;
    }
    if (M > 0 || (xt_fire && n_old > 0)) {
        if (n >= (int64_t)0x7FFFFFF0ll) return sh_fail(SH_ERR_INVALID, "partition lanes: more than 2G carried + new events");
        // ---- combined records: carried, then the push's
        if (s->pg[0].cap < n) {
            RCHK(pg_grow(q, s->pg[1], s->pg[0], n, n_old, V));
            std::swap(s->pg[0], s->pg[1]);
        }
        const PgRecs C = s->pg[0].view();
        if (ext) {
            RCHK(s->pg_xs.reserve(n * 8, false));
            RCHK(s->pg_xv.reserve(n * 8, false));
            RCHK(s->pg_ms.reserve(n * 8, false));
            RCHK(s->pg_cts.reserve(n * 8, false));
            RCHK(s->pg_err.reserve(64, false));
            HIPCHK(hipMemsetAsync(s->pg_err.p, 0, 8, st));
        }
        launch_pg_append(st, rec, M, n_old, q->seq, cs, q->gkp, q->gkt.dev(), V, C,
                         sorted_off ? nullptr : s->slot_cnt.as<u32>(),
                         s->pg_prevcnt.as<u32>(), ext ? q->d.ts_col : -1,
                         ext && q->d.has_start_time == 2 ? q->d.start_col : -1, s->pg_xs.as<int64_t>(),
                         s->pg_pendcnt.as<u32>());
        HIPCHK(hipGetLastError());
        // ---- every partition's records in stream order
        RCHK(s->ranks.reserve(n * 4, false));
        RCHK(s->p_slot.reserve(n * 4, false));
        size_t tb = 0;
        if (sort_slot_ranks(nullptr, &tb, C.ps, nullptr, nullptr, n, s->nslots, st))
            return sh_fail(SH_ERR_DEVICE, "radix sort sizing failed");
        RCHK(s->sort_tmp.reserve(std::max<size_t>(tb, 16), false));
        if (sort_slot_ranks(s->sort_tmp.p, &tb, C.ps, s->p_slot.as<u32>(), s->ranks.as<u32>(), n, s->nslots, st))
            return sh_fail(SH_ERR_DEVICE, "radix sort failed");
        RCHK(s->key_off.reserve((size_t)(s->nslots + 1) * 4, false));
        RCHK(s->tmp.reserve((size_t)((s->nslots + 1 + kTile - 1) / kTile + 16) * 8, false));
        if (sorted_off) launch_counts_sorted(st, s->p_slot.as<u32>(), n, s->slot_cnt.as<u32>());
        launch_slx_keyoff(st, s->slot_cnt.as<u32>(), s->nslots, s->key_off.as<u32>(), s->tmp.as<int64_t>());
        // ---- entries keyed (chunk, group slot)
        const int gbits = bits_for((int64_t)q->gkt.size_ + 2), cbits = bits_for(n + 1);
        const unsigned ebits = (unsigned)(gbits + cbits);
        if (ebits > 64) return sh_fail(SH_ERR_UNSUPPORTED, "partition lanes: entry key wider than 64 bits");
        const u64 none = ebits == 64 ? ~0ull : ((1ull << ebits) - 1);
        const int64_t ne_cap = 2 * n;
        RCHK(s->pg_ekey.reserve(ne_cap * 8, false));
        RCHK(s->pg_ekey2.reserve(ne_cap * 8, false));
        RCHK(s->pg_eval.reserve(ne_cap * 4, false));
        RCHK(s->pg_eval2.reserve(ne_cap * 4, false));
        RCHK(s->pg_keep.reserve(n + 16, false));
        RCHK(s->pg_cnt.reserve(64, false));
        HIPCHK(hipMemsetAsync(s->pg_cnt.p, 0, 8, st));
        PgExt X{};
        if (ext) {
            // the attribute's running max along every partition's run (rocPRIM scan by key)
            X = PgExt{s->pg_M.as<int64_t>(), s->pg_start.as<int64_t>(), s->pg_has.as<unsigned char>(),
                      s->pg_bopen.as<int64_t>(), q->d.has_start_time, q->d.ts_col, q->d.start_col, q->d.start_time,
                      q->d.window_param};
            tb = 0;
            if (launch_pg_ext_scan(st, s->ranks.as<u32>(), s->p_slot.as<u32>(), C, n, s->pg_xv.as<int64_t>(),
                                   s->pg_ms.as<int64_t>(), nullptr, &tb))
                return sh_fail(SH_ERR_DEVICE, "scan sizing failed");
            RCHK(s->sort_tmp.reserve(std::max<size_t>(tb, 16), false));
            if (launch_pg_ext_scan(st, s->ranks.as<u32>(), s->p_slot.as<u32>(), C, n, s->pg_xv.as<int64_t>(),
                                   s->pg_ms.as<int64_t>(), s->sort_tmp.p, &tb))
                return sh_fail(SH_ERR_DEVICE, "scan failed");
            if (xt) {
                RCHK(s->xt_flag.reserve(n + 16, false));
                launch_pg_xt_flags(st, s->key_off.as<u32>(), s->ranks.as<u32>(), s->pg_prevcnt.as<u32>(),
                                   s->pg_pendcnt.as<u32>(), C, s->pg_xs.as<int64_t>(), s->pg_ms.as<int64_t>(), X, n,
                                   s->xt_flag.as<unsigned char>(), s->pg_err.as<int>());
            } else {
                launch_pg_assign_ext(st, s->key_off.as<u32>(), s->ranks.as<u32>(), s->pg_prevcnt.as<u32>(),
                                     s->pg_pendcnt.as<u32>(), C, s->pg_xs.as<int64_t>(), s->pg_ms.as<int64_t>(), X, n,
                                     q->d.current_on, q->d.expired_on, gbits, none, s->pg_ekey.as<u64>(),
                                     s->pg_eval.as<u32>(), s->pg_keep.as<unsigned char>(),
                                     s->pg_cnt.as<unsigned long long>(), s->pg_cts.as<int64_t>(), s->pg_err.as<int>());
            }
            launch_pg_ext_state(st, s->key_off.as<u32>(), s->ranks.as<u32>(), s->pg_prevcnt.as<u32>(),
                                s->pg_pendcnt.as<u32>(), C, s->pg_xs.as<int64_t>(), s->pg_ms.as<int64_t>(), X, s->nslots);
        } else if (sc) {
            launch_pg_sc_assign(st, s->key_off.as<u32>(), s->ranks.as<u32>(), s->p_slot.as<u32>(), C, n, L, gbits,
                                s->pg_ekey.as<u64>(), s->pg_eval.as<u32>(), s->pg_keep.as<unsigned char>());
        } else {
            launch_pg_assign(st, s->key_off.as<u32>(), s->ranks.as<u32>(), s->p_slot.as<u32>(), s->pg_prevcnt.as<u32>(), C, n, L,
                             q->d.current_on, q->d.expired_on, gbits, none, s->pg_ekey.as<u64>(), s->pg_eval.as<u32>(),
                             s->pg_keep.as<unsigned char>(), s->pg_cnt.as<unsigned long long>());
        }
        HIPCHK(hipGetLastError());
        RCHK(q->gkt.check(st));
        if (ext) {
            int64_t err = 0;
            RCHK(read_count(q, s->pg_err.as<int64_t>(), &err));
            if ((int32_t)err)
                return sh_fail(SH_ERR_UNSUPPORTED, "externalTimeBatch: a partition's first event is before its start time "
                                                   "(not on the GPU)");
        }
        int64_t n_e = n;  // (stream.current: one entry per event)
        std::vector<PgXtEmit> em;
        std::vector<uint32_t> touched;
        if (xt) {
            // ---- the Scheduler walk over the push's calls and passing events (host), then the
            // emissions' entries (device)
            std::vector<uint32_t> ev_slot((size_t)M), ev_raw((size_t)M);
            std::vector<unsigned char> ev_flag((size_t)M);
            if (M > 0) {
                HIPCHK(hipMemcpyAsync(ev_slot.data(), C.ps + n_old, M * 4, hipMemcpyDeviceToHost, st));
                HIPCHK(hipMemcpyAsync(ev_raw.data(), rec.raw, M * 4, hipMemcpyDeviceToHost, st));
                HIPCHK(hipMemcpyAsync(ev_flag.data(), s->xt_flag.as<unsigned char>() + n_old, M, hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
            }
            std::vector<int64_t> slot_key;
            bool fresh = false;
            for (unsigned char f : ev_flag) fresh |= (f & 2) != 0;
            if (fresh || xt_fire) RCHK(d2h(q, slot_key, s->pl_key.p, s->nslots));
            RCHK(xt_walk(q, calls_s, calls_c, ev_slot, ev_flag, ev_raw, ss, q->clock_valid ? q->clock : INT64_MIN,
                         slot_key, em, touched));
            int64_t tot = 0;
            for (auto& e : em) {
                e.off = tot;
                tot += (q->d.expired_on ? e.xhi - e.xlo : 0) + (q->d.current_on ? e.hi - e.lo : 0);
                if (!q->d.current_on) e.hi = e.lo;  // (expired rows only: no CURRENT entries)
            }
            n_e = tot;
            const int ebits_x = gbits + bits_for((int64_t)em.size() + 1);
            if (ebits_x > 64) return sh_fail(SH_ERR_UNSUPPORTED, "partition lanes: entry key wider than 64 bits");
            if (n_e > 0) {
                if (n_e >= (int64_t)0x7FFFFFF0ll) return sh_fail(SH_ERR_UNSUPPORTED, "partition lanes: more than 2G entries");
                RCHK(s->pg_ekey.reserve(n_e * 8, false));
                RCHK(s->pg_ekey2.reserve(n_e * 8, false));
                RCHK(s->pg_eval.reserve(n_e * 4, false));
                RCHK(s->pg_eval2.reserve(n_e * 4, false));
                RCHK(s->xt_epos.reserve(n_e * 4, false));
                RCHK(s->xt_up.reserve(em.size() * sizeof(PgXtEmit), false));
                RCHK(s->xt_em.reserve(em.size() * sizeof(PgXtEmit), false));
                HIPCHK(hipMemcpyAsync(s->xt_em.p, em.data(), em.size() * sizeof(PgXtEmit), hipMemcpyHostToDevice, st));
                launch_pg_xt_expand(st, s->xt_em.as<PgXtEmit>(), (int64_t)em.size(), n_e, s->key_off.as<u32>(),
                                    s->ranks.as<u32>(), C, gbits, q->d.current_on, q->d.expired_on, s->pg_ekey.as<u64>(),
                                    s->pg_eval.as<u32>(), s->xt_epos.as<u32>());
                HIPCHK(hipGetLastError());
                HIPCHK(hipStreamSynchronize(st));  // (em is pageable)
            }
        } else if (!sc) {
            RCHK(read_count(q, s->pg_cnt.as<int64_t>(), &n_e));
        }
        if (n_e > 0) {
            tb = 0;
            // (current only: one entry per event; the timeout's entries are exactly n_e)
            const int64_t ne_sort = xt ? n_e : q->d.expired_on ? ne_cap : n;
            const unsigned sbits = xt ? (unsigned)(gbits + bits_for((int64_t)em.size() + 1)) : ebits;
            // grouped by the partition key (or not at all) a chunk — one partition's batch — has one group, so
            // the (chunk, group) order is the chunk order: the radix sort skips the group bits (stable: a
            // chunk's entries keep their order either way; the `none` key's chunk bits are all ones)
            const unsigned sbeg = (!xt && !q->group_other) ? (unsigned)gbits : 0u;
            if (sort_u64_pairs_range(nullptr, &tb, s->pg_ekey.as<u64>(), nullptr, s->pg_eval.as<u32>(), nullptr, ne_sort,
                                     sbeg, sbits, st))
                return sh_fail(SH_ERR_DEVICE, "radix sort sizing failed");
            RCHK(s->sort_tmp.reserve(std::max<size_t>(tb, 16), false));
            if (sort_u64_pairs_range(s->sort_tmp.p, &tb, s->pg_ekey.as<u64>(), s->pg_ekey2.as<u64>(), s->pg_eval.as<u32>(),
                                     s->pg_eval2.as<u32>(), ne_sort, sbeg, sbits, st))
                return sh_fail(SH_ERR_DEVICE, "radix sort failed");
            // ---- segments = rows
            RCHK(s->pg_head.reserve(n_e + 16, false));
            RCHK(s->pg_seg.reserve(n_e * 8, false));
            RCHK(s->x_blk.reserve((size_t)((n_e + kTile - 1) / kTile + 2) * 8, false));
            launch_pg_heads(st, s->pg_ekey2.as<u64>(), n_e, s->pg_head.as<unsigned char>());
            launch_slx_compact(st, 1, s->pg_head.as<unsigned char>(), nullptr, nullptr, nullptr, n_e,
                               s->x_blk.as<int64_t>(), nullptr, nullptr, s->pg_seg.as<int64_t>());
            HIPCHK(hipGetLastError());
            int64_t n_seg = 0;
            RCHK(read_count(q, s->x_blk.as<int64_t>() + (n_e + kTile - 1) / kTile, &n_seg));
            n_rows = sc ? M : n_seg;  // (stream.current: a row per event of the push, else one per segment)
            const int64_t rc = std::max<int64_t>(n_rows, 1);
            RCHK(s->xr_ts.reserve(rc * 8, false));
            RCHK(s->xr_rep.reserve(rc * 8, false));
            RCHK(s->xr_slot.reserve(rc * 4, false));
            RCHK(s->xr_ch.reserve(rc * 8, false));
            RCHK(s->xr_clk.reserve(rc * 8, false));
            RCHK(s->xr_exp.reserve(rc, false));
            RCHK(s->xr_vals.reserve((size_t)std::max(na, 1) * rc * 8, false));
            RCHK(s->xr_nulls.reserve((size_t)std::max(na, 1) * rc, false));
            RCHK(s->pg_rkey.reserve(rc * 8, false));
            RCHK(s->pg_rkey2.reserve(rc * 8, false));
            RCHK(s->pg_order.reserve(rc * 4, false));
            RCHK(s->pg_rpart.reserve(rc * 4, false));
            RCHK(s->out_part.reserve(rc * 4, false));
            SlxRows rows{s->xr_ts.as<int64_t>(), s->xr_rep.as<int64_t>(), s->xr_slot.as<u32>(), s->xr_ch.as<int64_t>(),
                         s->xr_clk.as<int64_t>(), s->xr_exp.as<unsigned char>(), s->xr_vals.as<u64>(),
                         s->xr_nulls.as<unsigned char>(), rc};
            const bool xa = ext && q->xt_replace;  // (the rows' batch ends: sh_query_rep_ts_attr)
            if (xa) {
                RCHK(s->xr_xa.reserve(rc * 8, false));
                RCHK(s->out_xa.reserve(rc * 8, false));
                rows.xa = s->xr_xa.as<int64_t>();
            }
            HIPCHK(hipEventRecord(q->ev_agg0, st));
            if (sc) {
                launch_pg_sc_fold(st, s->pg_seg.as<int64_t>(), n_seg, n_e, s->pg_ekey2.as<u64>(), s->pg_eval2.as<u32>(),
                                  s->ranks.as<u32>(), C, q->ap, gbits, n_old, rows, s->pg_rpart.as<u32>());
                HIPCHK(hipEventRecord(q->ev_agg1, st));
            } else {
                launch_pg_fold(st, s->pg_seg.as<int64_t>(), n_rows, n_e, s->pg_ekey2.as<u64>(), s->pg_eval2.as<u32>(),
                               s->ranks.as<u32>(), C, q->ap, gbits, rows, s->pg_rkey.as<u64>(), s->pg_rpart.as<u32>(),
                               ext ? s->pg_cts.as<int64_t>() : nullptr, xt ? s->xt_em.as<PgXtEmit>() : nullptr,
                               xt ? s->xt_epos.as<u32>() : nullptr, s->key_off.as<u32>());
                HIPCHK(hipEventRecord(q->ev_agg1, st));
                // ---- rows in (chunk, first entry) order
                const unsigned rbits = (unsigned)(32 + (xt ? bits_for((int64_t)em.size() + 1) : cbits));
                tb = 0;
                if (sort_u64_iota_bits(nullptr, &tb, s->pg_rkey.as<u64>(), nullptr, nullptr, n_rows, rbits, st))
                    return sh_fail(SH_ERR_DEVICE, "radix sort sizing failed");
                RCHK(s->sort_tmp.reserve(std::max<size_t>(tb, 16), false));
                if (sort_u64_iota_bits(s->sort_tmp.p, &tb, s->pg_rkey.as<u64>(), s->pg_rkey2.as<u64>(),
                                       s->pg_order.as<u32>(), n_rows, rbits, st))
                    return sh_fail(SH_ERR_DEVICE, "radix sort failed");
            }
            RCHK(s->out_ts.reserve(rc * 8, false));
            RCHK(s->out_keys.reserve((size_t)std::max(1, q->gkp.n) * rc * 8, false));
            RCHK(s->out_vals.reserve((size_t)std::max(na, 1) * rc * 8, false));
            RCHK(s->out_nulls.reserve((size_t)std::max(na, 1) * rc, false));
            RCHK(s->out_send.reserve(rc * 8, false));
            RCHK(s->out_clock.reserve(rc * 8, false));
            RCHK(s->out_expired.reserve(rc, false));
            RCHK(s->out_rep.reserve(rc * 8, false));
            launch_pg_emit(st, sc ? nullptr : s->pg_order.as<u32>(), n_rows, rows, na, s->nk_out, q->gkt.dev(), q->gkp, rc,
                           s->out_ts.as<int64_t>(), s->out_keys.as<int64_t>(), s->out_vals.as<u64>(),
                           s->out_nulls.as<unsigned char>(), s->out_expired.as<unsigned char>(),
                           s->out_send.as<int64_t>(), s->out_clock.as<int64_t>(), s->out_rep.as<int64_t>(),
                           s->pg_rpart.as<u32>(), s->out_part.as<u32>(), xa ? s->out_xa.as<int64_t>() : nullptr);
            HIPCHK(hipGetLastError());
            float kms = 0;
            (void)hipEventSynchronize(q->ev_agg1);
            (void)hipEventElapsedTime(&kms, q->ev_agg0, q->ev_agg1);
            q->stats.main_kernel_ms = kms;
        }
        // one flush per chunk (out_send = the completing event's stream index)
        RCHK(sliding_flushes(q, n_rows, &n_flushes));
        if (xt) {
            // ---- what each partition keeps: its open batch, and with expired output the previous
            // emission's records (they go out again as EXPIRED); the walk's indices then start there
            const bool exp_on = q->d.expired_on != 0;
            std::vector<uint32_t> kslot, kval;
            for (uint32_t p : touched) {
                SlidingImpl::XtPart& P = s->xt_parts[p];
                const int64_t kf = exp_on && P.pe_hi > P.pe_lo ? std::min(P.pe_lo, P.bs) : P.bs;
                if (kf <= 0) continue;
                kslot.push_back(p);
                kval.push_back((uint32_t)kf);
                P.n -= kf;
                P.bs -= kf;
                P.cur0 -= kf;
                P.pe_lo = std::max<int64_t>(P.pe_lo - kf, 0);
                P.pe_hi = std::max<int64_t>(P.pe_hi - kf, 0);
            }
            if (s->xt_kf.cap < (size_t)s->nslots * 4) {
                RCHK(s->xt_kf.reserve((size_t)s->nslots * 4, false));
                HIPCHK(hipMemsetAsync(s->xt_kf.p, 0, (size_t)s->nslots * 4, st));
            }
            const int64_t nk = (int64_t)kslot.size();
            if (nk) {
                RCHK(s->xt_up.reserve((size_t)nk * 8, false));
                HIPCHK(hipMemcpyAsync(s->xt_up.p, kslot.data(), nk * 4, hipMemcpyHostToDevice, st));
                HIPCHK(hipMemcpyAsync(s->xt_up.as<uint32_t>() + nk, kval.data(), nk * 4, hipMemcpyHostToDevice, st));
                launch_pg_xt_kf(st, s->xt_up.as<uint32_t>(), s->xt_up.as<uint32_t>() + nk, nk, s->xt_kf.as<uint32_t>());
            }
            launch_pg_xt_keep(st, s->key_off.as<u32>(), s->ranks.as<u32>(), C, n, s->xt_kf.as<uint32_t>(),
                              s->pg_keep.as<unsigned char>());
            if (nk) launch_pg_xt_kf(st, s->xt_up.as<uint32_t>(), nullptr, nk, s->xt_kf.as<uint32_t>());
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamSynchronize(st));  // (kslot / kval are pageable)
        }
        // ---- carry the open batches (and the last completed ones) in stream order
        RCHK(s->x_idx.reserve(n * 8, false));
        RCHK(s->x_blk.reserve((size_t)((n + kTile - 1) / kTile + 2) * 8, false));
        launch_slx_compact(st, 1, s->pg_keep.as<unsigned char>(), nullptr, nullptr, nullptr, n, s->x_blk.as<int64_t>(),
                           nullptr, nullptr, s->x_idx.as<int64_t>());
        HIPCHK(hipGetLastError());
        int64_t n_keep = 0;
        RCHK(read_count(q, s->x_blk.as<int64_t>() + (n + kTile - 1) / kTile, &n_keep));
        RCHK(pg_grow(q, s->pg[1], s->pg[1], std::max<int64_t>(n_keep, 1), 0, V));
        launch_pg_gather(st, s->x_idx.as<int64_t>(), n_keep, s->pg_keep.as<unsigned char>(), C, s->pg[1].view(), V);
        HIPCHK(hipGetLastError());
        std::swap(s->pg[0], s->pg[1]);
        s->pg_n = n_keep;
    }
    q->seq += N;
    if (b) {
        q->clock = q->clock_valid ? std::max(q->clock, info.max_tl) : info.max_tl;
        q->clock_valid = true;
    } else if (!q->clock_valid || now >= q->clock) {
        q->clock = now;
        q->clock_valid = true;
    }
    q->stats.events = N;
    HIPCHK(hipEventRecord(q->ev_push1, st));
    HIPCHK(hipStreamSynchronize(st));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, q->ev_push0, q->ev_push1);
    q->stats.push_ms = ms;
    q->stats.main_kernel_bytes = M * (int64_t)(16 + 8 * V) + n_rows * (int64_t)(8 + 8 * na);
    return sliding_output(q, n_rows, n_flushes, false, host_out, out);
}

// ---- lane 4: `partition with (p of S) begin from S#window.timeBatch(T[, start], true) select g…, aggs
// group by g… insert [current] events into O; end` (TimeBatchWindowProcessor.process :262-340 per partition
// state, nextEmitTime a processor field shared by the partitions, :128). Every partition chunk goes out at
// once with its groups' running values; a partition's state is RESET by its own chunk or TIMER that finds
// the playback clock at or past nextEmitTime — that chunk advances nextEmitTime and schedules the next
// TIMER under its own partition (so the TIMERs stay with the first partition while events keep coming, and
// pass to whichever partition meets a lagging nextEmitTime after an idle stretch). The host walks those
// calls (the Scheduler as in the other lanes); the device folds every (partition, group) state.
static int tb_register(sh_query* q, uint32_t p, int64_t t, std::vector<int64_t>& slot_key) {
    SlidingImpl* s = q->sl;
    if (s->pl_flow.find(p) == s->pl_flow.end() && slot_key.empty()) {
        HIPCHK(hipStreamSynchronize(q->ctx->stream));
        RCHK(d2h(q, slot_key, s->pl_key.p, s->nslots));
    }
    return sched_register(q, p, t, slot_key);
}

// the window's send check at `clock` for partition p (:266-281): true when p's state is RESET
static int tb_check(sh_query* q, uint32_t p, int64_t clock, std::vector<int64_t>& slot_key, bool* reset) {
    SlidingImpl* s = q->sl;
    const int64_t T = q->d.window_param;
    *reset = false;
    if (s->tb_next_emit == -1) {
        s->tb_next_emit = q->d.has_start_time ? clock + (T - (clock - q->d.start_time) % T) : clock + T;
        RCHK(tb_register(q, p, s->tb_next_emit, slot_key));
    }
    if (clock >= s->tb_next_emit) {
        s->tb_next_emit += T;
        RCHK(tb_register(q, p, s->tb_next_emit, slot_key));
        *reset = true;
    }
    return SH_OK;
}

static int plane_run_tbsc(sh_query* q, const sh_batch* b, int64_t now, bool host_out, const sh_out** out) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    q->stats = sh_stats{};
    std::vector<int64_t> slot_key;
    if (!b) {
        // a TIMER call: the due partition's window RESETs (no row: its current events went out already)
        if (q->clock_valid && now < q->clock) return empty_out(q, out);
        q->clock = now;
        q->clock_valid = true;
        if (!s->pl_armed.empty() && s->pl_armed.begin()->first <= now)
            RCHK(sched_fire(s, now, [&](uint32_t p, int64_t) -> int {
                bool r;
                RCHK(tb_check(q, p, now, slot_key, &r));
                if (r) s->tb_bids[p]++;
                return SH_OK;
            }));
        return empty_out(q, out);
    }
    const int64_t N = b->n, ss = b->send_size;
    const int V = std::max(1, q->ap.n_vcols), na = q->ap.n;
    if (N >= (int64_t)0x3FFFFFF0ll) return sh_fail(SH_ERR_INVALID, "push larger than 1G events");
    HIPCHK(hipEventRecord(q->ev_push0, st));
    const int64_t cap = std::max<int64_t>(N, 1);
    RCHK(s->rec_raw.reserve(cap * 4, false));
    RCHK(s->rec_slot.reserve(cap * 4, false));
    RCHK(s->rec_clock.reserve(cap * 8, false));
    RCHK(s->rec_pm.reserve(cap * 8, false));
    RCHK(s->rec_ts.reserve(cap * 8, false));
    RCHK(s->rec_vals.reserve((size_t)V * cap * 8, false));
    RCHK(s->slot_cnt.reserve(s->nslots * 4, false));
    HIPCHK(hipMemsetAsync(s->slot_cnt.p, 0, s->nslots * 4, st));
    SlRecords rec{s->rec_raw.as<u32>(), s->rec_slot.as<u32>(), s->rec_clock.as<int64_t>(), s->rec_pm.as<int64_t>(),
                  s->rec_ts.as<int64_t>(), s->rec_vals.as<u64>(), cap};
    ColSet cs{};
    cs.n = q->d.n_cols;
    for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->d.col_types[c]; cs.ptr[c] = b->cols[c]; }
    const int nblk = (int)((N + kTile - 1) / kTile);
    RCHK(s->blk_pass.reserve(nblk * 8, false));
    RCHK(s->blk_tl.reserve(nblk * 8, false));
    RCHK(s->blk_pm.reserve(nblk * 8, false));
    WinParams wp{};
    wp.kind = SH_WIN_TIME;  // the clock / pass-count prefix of the sliding path
    wp.clock_valid = q->clock_valid;
    wp.clock0 = q->clock;
    wp.send_size = ss;
    wp.N = N;
    wp.rec_seq = q->tune.sl_records_seq;
    launch_sl_prefix(st, b->ts, cs, q->fp, wp, s->blk_pass.as<int64_t>(), s->blk_tl.as<int64_t>(),
                     s->blk_pm.as<int64_t>(), nblk, s->info.as<SlInfo>());
    launch_sl_records(st, b->ts, cs, q->fp, wp, q->kp, q->kt.dev(), q->ap, s->blk_pass.as<int64_t>(),
                      s->blk_tl.as<int64_t>(), s->blk_pm.as<int64_t>(), s->pm, rec, s->slot_cnt.as<u32>(), nblk);
    launch_pl_slot_key(st, cs, q->kp, q->kt.dev(), N, s->pl_key.as<int64_t>());
    // partition runs over every event (the receiver cuts a send at key changes, before the filter)
    RCHK(s->tb_start.reserve(cap + 16, false));
    RCHK(s->tb_run.reserve(cap * 8, false));
    RCHK(s->tb_blk.reserve((size_t)(nblk + 16) * 8, false));
    launch_pl_runs(st, cs, q->d.partition_col, N, ss, s->tb_start.as<unsigned char>(), s->tb_blk.as<int64_t>(),
                   s->tb_run.as<int64_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(s->h_info, s->info.p, sizeof(SlInfo), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    RCHK(q->kt.check(st));
    const SlInfo info = *s->h_info;
    const int64_t M = info.total_pass;
    // the push's calls (a send whose last event does not move the clock calls nobody)
    std::vector<int64_t> calls_s, calls_c;
    {
        const int64_t NS = ss > 0 ? (N + ss - 1) / ss : 1;
        const int nbS = (int)((NS + kTile - 1) / kTile);
        RCHK(s->x_sK.reserve(NS * 8, false));
        RCHK(s->x_scb.reserve(NS * 8, false));
        RCHK(s->x_slast.reserve(NS * 8, false));
        RCHK(s->x_cK.reserve(NS * 8, false));
        RCHK(s->x_cC.reserve(NS * 8, false));
        RCHK(s->x_cS.reserve(NS * 8, false));
        RCHK(s->x_blk.reserve((size_t)((std::max(NS, M) + kTile - 1) / kTile + 2) * 8, false));
        launch_slx_sends(st, b->ts, cs, q->fp, wp, s->blk_pass.as<int64_t>(), s->blk_tl.as<int64_t>(), nblk,
                         s->x_sK.as<int64_t>(), s->x_scb.as<int64_t>(), s->x_slast.as<int64_t>());
        launch_slx_compact(st, 0, nullptr, s->x_sK.as<int64_t>(), s->x_scb.as<int64_t>(), s->x_slast.as<int64_t>(), NS,
                           s->x_blk.as<int64_t>(), s->x_cK.as<int64_t>(), s->x_cC.as<int64_t>(), s->x_cS.as<int64_t>());
        HIPCHK(hipGetLastError());
        int64_t nC = 0;
        RCHK(read_count(q, s->x_blk.as<int64_t>() + nbS, &nC));
        RCHK(d2h(q, calls_s, s->x_cS.p, nC));
        RCHK(d2h(q, calls_c, s->x_cC.p, nC));
    }
    // the chunks (partition runs with passing events) and their partition, send and clock
    int64_t nch = 0;
    std::vector<int64_t> ch_send, ch_clk, ch_bid;
    std::vector<uint32_t> ch_slot;
    if (M > 0) {
        RCHK(s->tb_flag.reserve(M + 16, false));
        RCHK(s->tb_first.reserve(M * 8, false));
        launch_tb_chunk_flags(st, rec, M, s->tb_run.as<int64_t>(), s->tb_flag.as<unsigned char>());
        launch_slx_compact(st, 1, s->tb_flag.as<unsigned char>(), nullptr, nullptr, nullptr, M, s->x_blk.as<int64_t>(),
                           nullptr, nullptr, s->tb_first.as<int64_t>());
        HIPCHK(hipGetLastError());
        RCHK(read_count(q, s->x_blk.as<int64_t>() + (M + kTile - 1) / kTile, &nch));
        RCHK(s->tb_cslot.reserve(nch * 4 + 16, false));
        RCHK(s->tb_csend.reserve(nch * 8 + 16, false));
        RCHK(s->tb_cclk.reserve(nch * 8 + 16, false));
        launch_tb_chunk_info(st, rec, s->tb_first.as<int64_t>(), nch, ss, s->tb_cslot.as<u32>(), s->tb_csend.as<int64_t>(),
                             s->tb_cclk.as<int64_t>());
        HIPCHK(hipGetLastError());
        ch_slot.resize((size_t)nch);
        HIPCHK(hipMemcpyAsync(ch_slot.data(), s->tb_cslot.p, nch * 4, hipMemcpyDeviceToHost, st));
        RCHK(d2h(q, ch_send, s->tb_csend.p, nch));
    }
    // ---- the walk: each call's TIMERs, then the chunks of the sends before the next call
    ch_bid.resize((size_t)nch);
    int64_t clock = q->clock_valid ? q->clock : INT64_MIN;
    size_t k = 0;
    auto chunks_before = [&](int64_t send_end) -> int {
        for (; k < (size_t)nch && ch_send[k] < send_end; k++) {
            const uint32_t p = ch_slot[k];
            bool r;
            RCHK(tb_check(q, p, clock, slot_key, &r));
            int64_t& bid = s->tb_bids[p];
            ch_bid[k] = bid;
            if (r) bid++;  // (the RESET follows the chunk's events: they went out with the old state)
        }
        return SH_OK;
    };
    for (size_t c = 0; c < calls_s.size(); c++) {
        RCHK(chunks_before(calls_s[c]));
        clock = calls_c[c];
        if (!s->pl_armed.empty() && s->pl_armed.begin()->first <= clock)
            RCHK(sched_fire(s, clock, [&](uint32_t p, int64_t) -> int {
                bool r;
                RCHK(tb_check(q, p, clock, slot_key, &r));
                if (r) s->tb_bids[p]++;
                return SH_OK;
            }));
    }
    RCHK(chunks_before(INT64_MAX));
    int64_t n_rows = 0, n_flushes = 0;
    if (M > 0) {
        RCHK(s->tb_chbid.reserve(nch * 8 + 16, false));
        HIPCHK(hipMemcpyAsync(s->tb_chbid.p, ch_bid.data(), nch * 8, hipMemcpyHostToDevice, st));
        RCHK(s->tb_chunk_of.reserve(M * 8, false));
        launch_tb_chunk_of(st, s->tb_first.as<int64_t>(), nch, M, s->tb_chunk_of.as<int64_t>());
        RCHK(s->tb_pair.reserve(M * 4, false));
        RCHK(s->tb_gslot.reserve(M * 4, false));
        launch_tb_pairs(st, rec, M, cs, q->gkp, q->gkt.dev(), q->pgkt.dev(), s->tb_pair.as<u32>(), s->tb_gslot.as<u32>());
        HIPCHK(hipGetLastError());
        RCHK(q->gkt.check(st));
        RCHK(q->pgkt.check(st));
        // ---- the records by (partition, group) state, stably
        const int64_t nst = (int64_t)q->pgkt.size_ + 1;
        RCHK(s->tb_skey.reserve(M * 4, false));
        RCHK(s->tb_sidx.reserve(M * 4, false));
        size_t tb = 0;
        if (sort_slot_ranks(nullptr, &tb, s->tb_pair.as<u32>(), nullptr, nullptr, M, nst, st))
            return sh_fail(SH_ERR_DEVICE, "radix sort sizing failed");
        RCHK(s->sort_tmp.reserve(std::max<size_t>(tb, 16), false));
        if (sort_slot_ranks(s->sort_tmp.p, &tb, s->tb_pair.as<u32>(), s->tb_skey.as<u32>(), s->tb_sidx.as<u32>(), M, nst,
                            st))
            return sh_fail(SH_ERR_DEVICE, "radix sort failed");
        RCHK(s->tb_head.reserve(M + 16, false));
        RCHK(s->tb_seg.reserve(M * 8, false));
        launch_pg_heads32(st, s->tb_skey.as<u32>(), M, s->tb_head.as<unsigned char>());
        launch_slx_compact(st, 1, s->tb_head.as<unsigned char>(), nullptr, nullptr, nullptr, M, s->x_blk.as<int64_t>(),
                           nullptr, nullptr, s->tb_seg.as<int64_t>());
        HIPCHK(hipGetLastError());
        int64_t n_seg = 0;
        RCHK(read_count(q, s->x_blk.as<int64_t>() + (M + kTile - 1) / kTile, &n_seg));
        // ---- a row per (chunk, group): the states fold their records from the carried values
        const int64_t rc = M;
        RCHK(s->xr_ts.reserve(rc * 8, false));
        RCHK(s->xr_rep.reserve(rc * 8, false));
        RCHK(s->xr_slot.reserve(rc * 4, false));
        RCHK(s->xr_ch.reserve(rc * 8, false));
        RCHK(s->xr_clk.reserve(rc * 8, false));
        RCHK(s->xr_exp.reserve(rc, false));
        RCHK(s->xr_vals.reserve((size_t)std::max(na, 1) * rc * 8, false));
        RCHK(s->xr_nulls.reserve((size_t)std::max(na, 1) * rc, false));
        RCHK(s->tb_rkey.reserve(rc * 8, false));
        RCHK(s->tb_rkey2.reserve(rc * 8, false));
        RCHK(s->tb_order.reserve(rc * 4, false));
        RCHK(s->pg_rpart.reserve(rc * 4, false));
        RCHK(s->out_part.reserve(rc * 4, false));
        RCHK(s->tb_nrows.reserve(16, false));
        HIPCHK(hipMemsetAsync(s->tb_nrows.p, 0, 8, st));
        SlxRows rows{s->xr_ts.as<int64_t>(), s->xr_rep.as<int64_t>(), s->xr_slot.as<u32>(), s->xr_ch.as<int64_t>(),
                     s->xr_clk.as<int64_t>(), s->xr_exp.as<unsigned char>(), s->xr_vals.as<u64>(),
                     s->xr_nulls.as<unsigned char>(), rc};
        TbState S{s->tb_cnt.as<int64_t>(), s->tb_bid.as<int64_t>(), s->tb_f.as<u64>(), s->tb_has.as<unsigned char>(), nst};
        HIPCHK(hipEventRecord(q->ev_agg0, st));
        launch_tb_fold(st, s->tb_seg.as<int64_t>(), n_seg, M, s->tb_skey.as<u32>(), s->tb_sidx.as<u32>(), rec,
                       s->tb_chunk_of.as<int64_t>(), s->tb_chbid.as<int64_t>(), s->tb_gslot.as<u32>(), q->ap, S,
                       s->tb_chunk_base, rows, s->tb_rkey.as<u64>(), s->pg_rpart.as<u32>(),
                       s->tb_nrows.as<unsigned int>(), q->seq);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(q->ev_agg1, st));
        RCHK(read_count(q, s->tb_nrows.as<int64_t>(), &n_rows));
        n_rows &= 0xFFFFFFFFll;
        // ---- rows in (chunk, first record) order -> the output columns
        const unsigned rbits = (unsigned)(32 + bits_for(nch + 1));
        tb = 0;
        if (sort_u64_iota_bits(nullptr, &tb, s->tb_rkey.as<u64>(), nullptr, nullptr, n_rows, rbits, st))
            return sh_fail(SH_ERR_DEVICE, "radix sort sizing failed");
        RCHK(s->sort_tmp.reserve(std::max<size_t>(tb, 16), false));
        if (sort_u64_iota_bits(s->sort_tmp.p, &tb, s->tb_rkey.as<u64>(), s->tb_rkey2.as<u64>(), s->tb_order.as<u32>(),
                               n_rows, rbits, st))
            return sh_fail(SH_ERR_DEVICE, "radix sort failed");
        const int64_t oc = std::max<int64_t>(n_rows, 1);
        RCHK(s->out_ts.reserve(oc * 8, false));
        RCHK(s->out_keys.reserve((size_t)std::max(1, q->gkp.n) * oc * 8, false));
        RCHK(s->out_vals.reserve((size_t)std::max(na, 1) * oc * 8, false));
        RCHK(s->out_nulls.reserve((size_t)std::max(na, 1) * oc, false));
        RCHK(s->out_send.reserve(oc * 8, false));
        RCHK(s->out_clock.reserve(oc * 8, false));
        RCHK(s->out_expired.reserve(oc, false));
        RCHK(s->out_rep.reserve(oc * 8, false));
        launch_pg_emit(st, s->tb_order.as<u32>(), n_rows, rows, na, s->nk_out, q->gkt.dev(), q->gkp, n_rows,
                       s->out_ts.as<int64_t>(), s->out_keys.as<int64_t>(), s->out_vals.as<u64>(),
                       s->out_nulls.as<unsigned char>(), s->out_expired.as<unsigned char>(), s->out_send.as<int64_t>(),
                       s->out_clock.as<int64_t>(), s->out_rep.as<int64_t>(), s->pg_rpart.as<u32>(),
                       s->out_part.as<u32>());
        HIPCHK(hipGetLastError());
        float kms = 0;
        (void)hipEventSynchronize(q->ev_agg1);
        (void)hipEventElapsedTime(&kms, q->ev_agg0, q->ev_agg1);
        q->stats.main_kernel_ms = kms;
        RCHK(sliding_flushes(q, n_rows, &n_flushes));
        s->tb_chunk_base += nch;
    }
    q->seq += N;
    q->clock = q->clock_valid ? std::max(q->clock, info.max_tl) : info.max_tl;
    q->clock_valid = true;
    q->stats.events = N;
    HIPCHK(hipEventRecord(q->ev_push1, st));
    HIPCHK(hipStreamSynchronize(st));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, q->ev_push0, q->ev_push1);
    q->stats.push_ms = ms;
    q->stats.main_kernel_bytes = M * (int64_t)(16 + 8 * V) + n_rows * (int64_t)(8 + 8 * na);
    return sliding_output(q, n_rows, n_flushes, false, host_out, out);
}

// Time / externalTime lanes grouped by other columns (sh_plane_group_kernels.hip, k_pg_walk_ops /
// k_pg_replay): the partitions' walks write their add / remove operations, the operations sorted stably
// by (partition, group) state are replayed one thread per state, rows sorted by (chunk, first operation).
// the min / max fields of the grouped time lanes' states and their deque pool
static PgDeques pg_deques(sh_query* q) {
    SlidingImpl* s = q->sl;
    PgDeques D{};
    for (int a = 0; a < q->ap.n; a++) {
        if (q->ap.kind[a] < AK_MIN_L) continue;
        bool seen = false;
        for (int f = 0; f < D.nf; f++) seen |= D.field[f] == q->ap.field[a];
        if (!seen) D.field[D.nf++] = q->ap.field[a];
    }
    D.n = s->pg_st_n;
    D.pool = s->pg_dq_pool.as<u64>();
    D.off = s->pg_dq_off.as<int64_t>();
    D.len = s->pg_dq_len.as<int64_t>();
    D.scratch = s->pg_dq_scr.as<u64>();
    D.new_at = s->pg_dq_at.as<int64_t>();
    D.new_len = s->pg_dq_nlen.as<int64_t>();
    D.active = s->pg_dq_act.as<unsigned char>();
    return D;
}

// Room in the (partition, group) pair table for the push's new pairs (at most one per add, M) before
// the walk inserts them: the walk advances every partition's ring, so a table that overflowed there
// would fail the push after the query state changed. When the table could pass half full, the live
// states move to a fresh table sized for them plus M (dead pairs dropped, PartitionStateHolder's
// returnState), and the state arrays follow (sh_plane_group_kernels.hip k_pg_rehash).
static int pg_reserve_pairs(sh_query* q, int64_t M) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    if (q->pgkt.n_keys + M <= (int64_t)q->pgkt.size_ / 2) return SH_OK;
    const int F = std::max(1, q->ap.n_fields);
    const int64_t on = s->pg_st_n;
    RCHK(s->pg_cnt.reserve(64, false));
    HIPCHK(hipMemsetAsync(s->pg_cnt.p, 0, 8, st));
    launch_pg_count_live(st, q->pgkt.dev(), on, s->pg_st_cnt.as<int64_t>(), s->pg_st_f.as<u64>(),
                         s->pg_dq_len.as<int64_t>(), F, (unsigned long long*)s->pg_cnt.p);
    HIPCHK(hipGetLastError());
    int64_t live = 0;
    RCHK(read_count(q, s->pg_cnt.as<int64_t>(), &live));
    size_t ts = std::max<size_t>(q->pg_min_size, 16);
    while ((int64_t)ts < 2 * (live + M)) ts <<= 1;
    if (ts > ((size_t)1 << 31)) return sh_fail(SH_ERR_UNSUPPORTED, "partition lanes: more than 2^30 (partition, group) states");
    KeyTableHost nk;
    RCHK(nk.init_size(ts));
    const int64_t nn = (int64_t)ts + 1;
    DevBuf ncnt, nf, ndqo, ndql;
    RCHK(fill(ncnt, (size_t)nn * 8, 0));
    RCHK(fill(nf, (size_t)F * nn * 8, 0));
    RCHK(fill(ndqo, (size_t)F * nn * 8, 0));
    RCHK(fill(ndql, (size_t)F * nn * 8, 0));
    launch_pg_rehash(st, q->pgkt.dev(), on, s->pg_st_cnt.as<int64_t>(), s->pg_st_f.as<u64>(), s->pg_dq_off.as<int64_t>(),
                     s->pg_dq_len.as<int64_t>(), F, nk.dev(), nn, ncnt.as<int64_t>(), nf.as<u64>(), ndqo.as<int64_t>(),
                     ndql.as<int64_t>());
    HIPCHK(hipGetLastError());
    RCHK(nk.check(st));
    HIPCHK(hipStreamSynchronize(st));  // the old arrays are released below
    SH_TRACE("pg_reserve_pairs: %lld pairs (%lld live) in %zu slots -> %zu slots", (long long)q->pgkt.n_keys,
             (long long)live, q->pgkt.size_, ts);
    q->pgkt = std::move(nk);
    s->pg_st_n = nn;
    s->pg_st_cnt = std::move(ncnt);
    s->pg_st_f = std::move(nf);
    s->pg_dq_off = std::move(ndqo);
    s->pg_dq_len = std::move(ndql);
    return SH_OK;
}

static int group_time_rows(sh_query* q, const ColSet* cs, SlRecords rec, int64_t M, int64_t nF, int64_t T, int64_t ss,
                           bool xt, int64_t* n_rows_out) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    const int nv = std::max(1, q->ap.n_vcols), na = q->ap.n;
    const int64_t np = s->nslots;
    RCHK(pg_reserve_pairs(q, M));
    if (cs && M > 0) {
        launch_pg_rec_group(st, rec, M, *cs, q->gkp, q->gkt.dev(), nv);
        HIPCHK(hipGetLastError());
    }
    // every partition's operation region
    RCHK(s->pg_room.reserve((size_t)(np + 1) * 8, false));
    RCHK(s->tmp.reserve((size_t)((np + 1 + kTile - 1) / kTile + 16) * 8, false));
    HIPCHK(hipMemsetAsync(s->pg_room.as<int64_t>() + np, 0, 8, st));
    launch_pg_ops_room(st, s->slot_cnt.as<u32>(), s->rlen.as<int64_t>(), np, s->pg_room.as<int64_t>());
    launch_scan_sum_large(st, s->pg_room.as<int64_t>(), np + 1, s->tmp.as<int64_t>());
    HIPCHK(hipGetLastError());
    int64_t ocap = 0;
    RCHK(read_count(q, s->pg_room.as<int64_t>() + np, &ocap));
    RCHK(q->gkt.check(st));
    if (ocap >= (int64_t)0xFFFFFFF0ll) return sh_fail(SH_ERR_INVALID, "partition lanes: more than 4G window operations");
    const int64_t oc = std::max<int64_t>(ocap, 1);
    RCHK(s->op_pos.reserve(oc * 8, false));
    RCHK(s->op_pg.reserve(oc * 4, false));
    RCHK(s->op_kind.reserve(oc, false));
    RCHK(s->op_seq.reserve(oc * 8, false));
    RCHK(s->op_ts.reserve(oc * 8, false));
    RCHK(s->op_clk.reserve(oc * 8, false));
    RCHK(s->op_vals.reserve((size_t)nv * oc * 8, false));
    RCHK(s->pg_ocnt.reserve((size_t)np * 4, false));
    HIPCHK(hipMemsetAsync(s->op_pg.p, 0xff, oc * 4, st));
    HIPCHK(hipMemsetAsync(s->pg_ocnt.p, 0, (size_t)np * 4, st));
    PgOps O{s->op_pos.as<int64_t>(), s->op_pg.as<u32>(), s->op_kind.as<unsigned char>(), s->op_seq.as<int64_t>(),
            s->op_ts.as<int64_t>(), s->op_clk.as<int64_t>(), s->op_vals.as<u64>(), oc};
    HIPCHK(hipEventRecord(q->ev_agg0, st));
    launch_pg_walk_ops(st, s->key_off.as<u32>(), s->ranks.as<u32>(), np, rec, s->pl_run.as<int64_t>(), T, q->seq, ss,
                       nF ? s->pl_toff.as<int64_t>() : nullptr, s->pl_tsend.as<int64_t>(), s->pl_tclk.as<int64_t>(),
                       s->pl_tpos.as<int64_t>(), s->pl_fsend.as<int64_t>(), nF, state_of(s), s->rg.as<int64_t>(), nv,
                       xt ? s->pl_x.as<int64_t>() : nullptr, q->pgkt.dev(), s->pg_room.as<int64_t>(), O,
                       s->pg_ocnt.as<u32>());
    HIPCHK(hipGetLastError());
    RCHK(q->pgkt.check(st));
    RCHK(s->pg_cnt.reserve(64, false));
    HIPCHK(hipMemsetAsync(s->pg_cnt.p, 0, 16, st));
    launch_pg_sum_u32(st, s->pg_ocnt.as<u32>(), np, s->pg_cnt.as<unsigned long long>());
    int64_t n_ops = 0;
    RCHK(read_count(q, s->pg_cnt.as<int64_t>(), &n_ops));
    int64_t n_rows = 0;
    if (n_ops > 0) {
        // operations by state slot, each state's in its partition's order
        RCHK(s->pg_skey.reserve(oc * 4, false));
        RCHK(s->pg_sidx.reserve(oc * 4, false));
        size_t tb = 0;
        if (sort_slot_ranks(nullptr, &tb, O.pg, nullptr, nullptr, ocap, (int64_t)1 << 32, st))
            return sh_fail(SH_ERR_DEVICE, "radix sort sizing failed");
        RCHK(s->sort_tmp.reserve(std::max<size_t>(tb, 16), false));
        if (sort_slot_ranks(s->sort_tmp.p, &tb, O.pg, s->pg_skey.as<u32>(), s->pg_sidx.as<u32>(), ocap, (int64_t)1 << 32, st))
            return sh_fail(SH_ERR_DEVICE, "radix sort failed");
        RCHK(s->pg_head.reserve(n_ops + 16, false));
        RCHK(s->pg_seg.reserve(n_ops * 8, false));
        RCHK(s->x_blk.reserve((size_t)((n_ops + kTile - 1) / kTile + 2) * 8, false));
        launch_pg_heads32(st, s->pg_skey.as<u32>(), n_ops, s->pg_head.as<unsigned char>());
        launch_slx_compact(st, 1, s->pg_head.as<unsigned char>(), nullptr, nullptr, nullptr, n_ops, s->x_blk.as<int64_t>(),
                           nullptr, nullptr, s->pg_seg.as<int64_t>());
        HIPCHK(hipGetLastError());
        int64_t n_seg = 0;
        RCHK(read_count(q, s->x_blk.as<int64_t>() + (n_ops + kTile - 1) / kTile, &n_seg));
        // replay: at most one row per operation
        const int64_t rc = n_ops;
        RCHK(s->xr_ts.reserve(rc * 8, false));
        RCHK(s->xr_rep.reserve(rc * 8, false));
        RCHK(s->xr_slot.reserve(rc * 4, false));
        RCHK(s->xr_ch.reserve(rc * 8, false));
        RCHK(s->xr_clk.reserve(rc * 8, false));
        RCHK(s->xr_exp.reserve(rc, false));
        RCHK(s->xr_vals.reserve((size_t)std::max(na, 1) * rc * 8, false));
        RCHK(s->xr_nulls.reserve((size_t)std::max(na, 1) * rc, false));
        RCHK(s->pg_rkey.reserve(rc * 8, false));
        RCHK(s->pg_rkey2.reserve(rc * 8, false));
        RCHK(s->pg_order.reserve(rc * 4, false));
        RCHK(s->pg_rpart.reserve(rc * 4, false));
        SlxRows rows{s->xr_ts.as<int64_t>(), s->xr_rep.as<int64_t>(), s->xr_slot.as<u32>(), s->xr_ch.as<int64_t>(),
                     s->xr_clk.as<int64_t>(), s->xr_exp.as<unsigned char>(), s->xr_vals.as<u64>(),
                     s->xr_nulls.as<unsigned char>(), rc};
        HIPCHK(hipMemsetAsync(s->pg_cnt.p, 0, 16, st));
        PgDeques D = pg_deques(q);
        if (D.nf > 0) {
            // every segment's scratch: its carried deques plus one entry per add of the push
            const size_t FN = (size_t)std::max(1, q->ap.n_fields) * D.n;
            RCHK(s->pg_dq_need.reserve((size_t)(n_seg + 1) * 8, false));
            RCHK(s->tmp.reserve((size_t)((std::max<int64_t>(n_seg + 1, (int64_t)FN + 1) + kTile - 1) / kTile + 16) * 8, false));
            launch_pg_dq_need(st, s->pg_seg.as<int64_t>(), n_seg, n_ops, s->pg_skey.as<u32>(), s->pg_sidx.as<u32>(), O, D,
                              s->pg_dq_need.as<int64_t>());
            launch_scan_sum_large(st, s->pg_dq_need.as<int64_t>(), n_seg + 1, s->tmp.as<int64_t>());
            int64_t scr = 0;
            RCHK(read_count(q, s->pg_dq_need.as<int64_t>() + n_seg, &scr));
            RCHK(s->pg_dq_scr.reserve((size_t)std::max<int64_t>(scr, 1) * 8, false));
            RCHK(s->pg_dq_at.reserve(FN * 8, false));
            RCHK(s->pg_dq_nlen.reserve(FN * 8, false));
            RCHK(s->pg_dq_act.reserve((size_t)D.n, false));
            HIPCHK(hipMemsetAsync(s->pg_dq_act.p, 0, (size_t)D.n, st));
            D = pg_deques(q);
        }
        launch_pg_replay(st, s->pg_seg.as<int64_t>(), n_seg, n_ops, s->pg_skey.as<u32>(), s->pg_sidx.as<u32>(), O,
                         q->pgkt.dev(), s->pg_st_cnt.as<int64_t>(), s->pg_st_f.as<u64>(), s->pg_st_n, q->ap, q->d.current_on,
                         q->d.expired_on, rows, s->pg_rkey.as<u64>(), s->pg_rpart.as<u32>(),
                         (unsigned int*)s->pg_cnt.p, D, s->pg_dq_need.as<int64_t>());
        HIPCHK(hipGetLastError());
        if (D.nf > 0) {
            // the deques back into a fresh pool, (field, state)-major
            const int64_t tot = (int64_t)D.nf * D.n;
            RCHK(s->pg_dq_lens.reserve((size_t)(tot + 1) * 8, false));
            RCHK(s->tmp.reserve((size_t)((tot + 1 + kTile - 1) / kTile + 16) * 8, false));
            launch_pg_dq_len(st, D, s->pg_dq_lens.as<int64_t>());
            launch_scan_sum_large(st, s->pg_dq_lens.as<int64_t>(), tot + 1, s->tmp.as<int64_t>());
            int64_t words = 0;
            RCHK(read_count(q, s->pg_dq_lens.as<int64_t>() + tot, &words));
            RCHK(s->pg_dq_pool2.reserve((size_t)std::max<int64_t>(words, 8) * 8, false));
            RCHK(s->pg_dq_off2.reserve((size_t)std::max(1, q->ap.n_fields) * D.n * 8, false));
            launch_pg_dq_pool(st, D, s->pg_dq_lens.as<int64_t>(), s->pg_dq_pool2.as<u64>(), s->pg_dq_off2.as<int64_t>());
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamSynchronize(st));  // the old pool is released below
            std::swap(s->pg_dq_pool, s->pg_dq_pool2);
            std::swap(s->pg_dq_off, s->pg_dq_off2);
            s->pg_dq_words = words;
        }
        RCHK(read_count(q, s->pg_cnt.as<int64_t>(), &n_rows));
        n_rows &= 0xFFFFFFFFll;
        if (n_rows > 0) {
            // rows in (chunk, first operation) order
            int pbits = 1;
            while (pbits < 31 && ((int64_t)1 << pbits) <= M + nF) pbits++;
            size_t tb2 = 0;
            if (sort_u64_iota_bits(nullptr, &tb2, s->pg_rkey.as<u64>(), nullptr, nullptr, n_rows, 32 + pbits, st))
                return sh_fail(SH_ERR_DEVICE, "radix sort sizing failed");
            RCHK(s->sort_tmp.reserve(std::max<size_t>(tb2, 16), false));
            if (sort_u64_iota_bits(s->sort_tmp.p, &tb2, s->pg_rkey.as<u64>(), s->pg_rkey2.as<u64>(), s->pg_order.as<u32>(),
                                   n_rows, 32 + pbits, st))
                return sh_fail(SH_ERR_DEVICE, "radix sort failed");
        }
        const int64_t rcap = std::max<int64_t>(n_rows, 1);
        RCHK(s->out_ts.reserve(rcap * 8, false));
        RCHK(s->out_keys.reserve((size_t)std::max(1, q->gkp.n) * rcap * 8, false));
        RCHK(s->out_vals.reserve((size_t)std::max(na, 1) * rcap * 8, false));
        RCHK(s->out_nulls.reserve((size_t)std::max(na, 1) * rcap, false));
        RCHK(s->out_send.reserve(rcap * 8, false));
        RCHK(s->out_clock.reserve(rcap * 8, false));
        RCHK(s->out_expired.reserve(rcap, false));
        RCHK(s->out_rep.reserve(rcap * 8, false));
        RCHK(s->out_part.reserve(rcap * 4, false));
        launch_pg_emit(st, s->pg_order.as<u32>(), n_rows, rows, na, s->nk_out, q->gkt.dev(), q->gkp, rcap,
                       s->out_ts.as<int64_t>(), s->out_keys.as<int64_t>(), s->out_vals.as<u64>(),
                       s->out_nulls.as<unsigned char>(), s->out_expired.as<unsigned char>(), s->out_send.as<int64_t>(),
                       s->out_clock.as<int64_t>(), s->out_rep.as<int64_t>(), s->pg_rpart.as<u32>(), s->out_part.as<u32>());
        HIPCHK(hipGetLastError());
    }
    *n_rows_out = n_rows;
    return SH_OK;
}

int64_t plane_slots(sh_query* q) { return q->sl->nslots; }
// partitioned externalTimeBatch with replaceTimestampWithBatchEndTime: the output rows' batch ends
const int64_t* plane_out_rep_attr(sh_query* q) { return q->sl->out_xa.as<int64_t>(); }
bool plane_is_sorted_lane(const sh_query* q) { return q->sl && q->sl->lane == 3; }
// key columns of the query's output rows (the lanes without group-by keep the partition key internal)
int query_out_keys(sh_query* q) { return q->kind == 1 && q->sl && q->sl->nk_out >= 0 ? q->sl->nk_out : q->kp.n; }
const u32* plane_out_part(sh_query* q) { return q->sl->out_part.as<u32>(); }

// Lane pass of the push: records of M passing events sorted by slot (b == null: a TIMER call at `now`).
static int plane_run(sh_query* q, const sh_batch* b, int64_t now, bool host_out, const sh_out** out) {
    SlidingImpl* s = q->sl;
    if (s->lane == 3) return plane_run_group(q, b, now, host_out, out);
    if (s->lane == 4) return plane_run_tbsc(q, b, now, host_out, out);
    hipStream_t st = q->ctx->stream;
    q->stats = sh_stats{};
    // (externalTime lanes: the window runs on the timestamp attribute, no TIMER calls reach it)
    const bool xt = q->d.window == SH_WIN_EXT_TIME;
    const bool tm = s->lane == 2, sched = tm && q->d.expired_on && !xt;
    const bool grp = tm && q->group_other;  // time lanes grouped by other columns (operations, then states)
    const int64_t N = b ? b->n : 0, ss = b ? b->send_size : 0, T = q->d.window_param;
    const int V = std::max(1, q->ap.n_vcols) + (grp ? 1 : 0), na = q->ap.n;
    if (!b) {
        if (q->clock_valid && now < q->clock) return empty_out(q, out);
        q->clock = now;
        q->clock_valid = true;
        if (!sched || s->pl_armed.empty() || s->pl_armed.begin()->first > now) return empty_out(q, out);
    }
    if (N >= (int64_t)0x7FFFFFF0ll) return sh_fail(SH_ERR_INVALID, "push larger than 2G events");
    HIPCHK(hipEventRecord(q->ev_push0, st));
    const int64_t cap = std::max<int64_t>(N, 1);
    RCHK(s->rec_raw.reserve(cap * 4, false));
    RCHK(s->rec_slot.reserve(cap * 4, false));
    RCHK(s->rec_clock.reserve(cap * 8, false));
    RCHK(s->rec_pm.reserve(cap * 8, false));
    RCHK(s->rec_ts.reserve(cap * 8, false));
    RCHK(s->rec_vals.reserve((size_t)V * cap * 8, false));
    RCHK(s->slot_cnt.reserve(s->nslots * 4, false));
    HIPCHK(hipMemsetAsync(s->slot_cnt.p, 0, s->nslots * 4, st));
    SlRecords rec{s->rec_raw.as<u32>(), s->rec_slot.as<u32>(), s->rec_clock.as<int64_t>(), s->rec_pm.as<int64_t>(),
                  s->rec_ts.as<int64_t>(), s->rec_vals.as<u64>(), cap};
    ColSet cs{};
    cs.n = q->d.n_cols;
    WinParams wp{};
    int nblk = 0;
    int64_t M = 0;
    SlInfo info{};
    bool sorted_off = false;  // records sorted and partition offsets made before the push's sync
    if (b) {
        for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->d.col_types[c]; cs.ptr[c] = b->cols[c]; }
        nblk = (int)((N + kTile - 1) / kTile);
        RCHK(s->blk_pass.reserve(nblk * 8, false));
        RCHK(s->blk_tl.reserve(nblk * 8, false));
        RCHK(s->blk_pm.reserve(nblk * 8, false));
        wp.kind = SH_WIN_TIME;  // the clock / pass-count prefix of the sliding path
        wp.clock_valid = q->clock_valid;
        wp.clock0 = q->clock;
        wp.send_size = ss;
        wp.N = N;
        wp.rec_seq = q->tune.sl_records_seq;
        launch_sl_prefix(st, b->ts, cs, q->fp, wp, s->blk_pass.as<int64_t>(), s->blk_tl.as<int64_t>(),
                         s->blk_pm.as<int64_t>(), nblk, s->info.as<SlInfo>());
        // (lanes keyed by the partition, every event passing: the partition offsets and the ring need come
        // from the sorted slots instead of per-slot counts)
        sorted_off = !q->group_other && sl_records_seq_applies(q->fp, wp, q->ap);
        launch_sl_records(st, b->ts, cs, q->fp, wp, q->kp, q->kt.dev(), q->ap, s->blk_pass.as<int64_t>(),
                          s->blk_tl.as<int64_t>(), s->blk_pm.as<int64_t>(), s->pm, rec,
                          sorted_off ? nullptr : s->slot_cnt.as<u32>(), nblk);
        if (sched) launch_pl_slot_key(st, cs, q->kp, q->kt.dev(), N, s->pl_key.as<int64_t>());
        HIPCHK(hipMemsetAsync((char*)s->info.p + offsetof(SlInfo, need), 0, 8, st));
        int64_t* need_dev = (int64_t*)((char*)s->info.p + offsetof(SlInfo, need));
        if (sorted_off) {
            RCHK(s->ranks.reserve(cap * 4, false));
            RCHK(s->p_slot.reserve(cap * 4, false));
            RCHK(s->key_off.reserve((size_t)(s->nslots + 1) * 4, false));
            size_t tb = 0;
            if (sort_slot_ranks(nullptr, &tb, rec.slot, nullptr, nullptr, N, s->nslots, st))
                return sh_fail(SH_ERR_DEVICE, "radix sort sizing failed");
            RCHK(s->sort_tmp.reserve(std::max<size_t>(tb, 16), false));
            if (sort_slot_ranks(s->sort_tmp.p, &tb, rec.slot, s->p_slot.as<u32>(), s->ranks.as<u32>(), N, s->nslots, st))
                return sh_fail(SH_ERR_DEVICE, "radix sort failed");
            launch_counts_sorted(st, s->p_slot.as<u32>(), N, s->slot_cnt.as<u32>());
        }
        launch_sl_need(st, s->slot_cnt.as<u32>(), s->rlen.as<int64_t>(), s->nslots, need_dev);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(s->h_info, s->info.p, sizeof(SlInfo), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        RCHK(q->kt.check(st));
        info = *s->h_info;
        M = info.total_pass;
        if (tm && info.need > s->rc) {
            int64_t nrc = s->rc;
            while (nrc < info.need) nrc <<= 1;
            RCHK(size_rings(q, nrc));
        }
    }
    // each partition's records in stream order
    if (!sorted_off) {
        RCHK(s->ranks.reserve(cap * 4, false));
        RCHK(s->p_slot.reserve(cap * 4, false));
        if (M > 0) {
            size_t tb = 0;
            if (sort_slot_ranks(nullptr, &tb, rec.slot, nullptr, nullptr, M, s->nslots, st))
                return sh_fail(SH_ERR_DEVICE, "radix sort sizing failed");
            RCHK(s->sort_tmp.reserve(std::max<size_t>(tb, 16), false));
            if (sort_slot_ranks(s->sort_tmp.p, &tb, rec.slot, s->p_slot.as<u32>(), s->ranks.as<u32>(), M, s->nslots, st))
                return sh_fail(SH_ERR_DEVICE, "radix sort failed");
        }
    }
    RCHK(s->key_off.reserve((size_t)(s->nslots + 1) * 4, false));
    RCHK(s->tmp.reserve((size_t)((s->nslots + 1 + kTile - 1) / kTile + 16) * 8, false));
    launch_slx_keyoff(st, s->slot_cnt.as<u32>(), s->nslots, s->key_off.as<u32>(), s->tmp.as<int64_t>());
    HIPCHK(hipGetLastError());

    // ---- time windows with expired output: the Scheduler's TIMER calls per partition
    std::vector<Firing> fire;
    if (sched) {
        std::vector<int64_t> calls_s, calls_c, calls_k, reg_r;
        if (b) {
            const int64_t NS = ss > 0 ? (N + ss - 1) / ss : 1;
            const int nbS = (int)((NS + kTile - 1) / kTile);
            RCHK(s->x_sK.reserve(NS * 8, false));
            RCHK(s->x_scb.reserve(NS * 8, false));
            RCHK(s->x_slast.reserve(NS * 8, false));
            RCHK(s->x_cK.reserve(NS * 8, false));
            RCHK(s->x_cC.reserve(NS * 8, false));
            RCHK(s->x_cS.reserve(NS * 8, false));
            RCHK(s->x_blk.reserve((size_t)((std::max(NS, M) + kTile - 1) / kTile + 2) * 8, false));
            launch_slx_sends(st, b->ts, cs, q->fp, wp, s->blk_pass.as<int64_t>(), s->blk_tl.as<int64_t>(), nblk,
                             s->x_sK.as<int64_t>(), s->x_scb.as<int64_t>(), s->x_slast.as<int64_t>());
            launch_slx_compact(st, 0, nullptr, s->x_sK.as<int64_t>(), s->x_scb.as<int64_t>(), s->x_slast.as<int64_t>(),
                               NS, s->x_blk.as<int64_t>(), s->x_cK.as<int64_t>(), s->x_cC.as<int64_t>(),
                               s->x_cS.as<int64_t>());
            HIPCHK(hipGetLastError());
            int64_t nC = 0;
            RCHK(read_count(q, s->x_blk.as<int64_t>() + nbS, &nC));
            RCHK(d2h(q, calls_s, s->x_cS.p, nC));
            RCHK(d2h(q, calls_c, s->x_cC.p, nC));
            RCHK(d2h(q, calls_k, s->x_cK.p, nC));
            // notify registrations: the records that raise their partition's lastTimestamp
            RCHK(s->pl_reg.reserve(cap + 16, false));
            launch_pl_notify(st, s->key_off.as<u32>(), s->ranks.as<u32>(), s->nslots, rec.ts, s->pl_last_ts.as<int64_t>(),
                             s->pl_reg.as<unsigned char>());
            RCHK(s->x_idx.reserve(cap * 8, false));
            launch_slx_compact(st, 1, s->pl_reg.as<unsigned char>(), nullptr, nullptr, nullptr, M,
                               s->x_blk.as<int64_t>(), nullptr, nullptr, s->x_idx.as<int64_t>());
            HIPCHK(hipGetLastError());
            int64_t n_reg = 0;
            RCHK(read_count(q, s->x_blk.as<int64_t>() + (M + kTile - 1) / kTile, &n_reg));
            RCHK(d2h(q, reg_r, s->x_idx.p, n_reg));
        } else {
            calls_s.push_back(0);
            calls_c.push_back(now);
            calls_k.push_back(0);
        }
        std::vector<uint32_t> raw(M), slot(M);
        std::vector<int64_t> tsv(M), slot_key;
        if (!reg_r.empty()) {
            HIPCHK(hipMemcpyAsync(raw.data(), rec.raw, M * 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(slot.data(), rec.slot, M * 4, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(tsv.data(), rec.ts, M * 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
        }
        if (!reg_r.empty()) RCHK(d2h(q, slot_key, s->pl_key.p, s->nslots));
        // replay the Scheduler: registrations of a send happen after that send's call
        size_t j = 0;
        for (size_t c = 0; c < calls_s.size(); c++) {
            for (; j < reg_r.size(); j++) {
                const uint32_t r = (uint32_t)reg_r[j];
                const int64_t snd = ss > 0 ? (int64_t)raw[r] / ss : 0;
                if (snd >= calls_s[c]) break;
                RCHK(sched_register(q, slot[r], tsv[r] + T, slot_key));
            }
            if (!s->pl_armed.empty() && s->pl_armed.begin()->first <= calls_c[c])
                sched_call(s, calls_s[c], calls_c[c], calls_k[c], fire);
        }
        for (; j < reg_r.size(); j++) {
            const uint32_t r = (uint32_t)reg_r[j];
            RCHK(sched_register(q, slot[r], tsv[r] + T, slot_key));
        }
    }
    const int64_t nF = (int64_t)fire.size();
    if (nF > 0) {
        // per partition its firings in order; positions K + t in the push's output order
        std::vector<int64_t> fsend(nF), order(nF), toff(s->nslots + 1, 0), tsend(nF), tclk(nF), tpos(nF);
        for (int64_t t = 0; t < nF; t++) { fsend[t] = fire[t].send; toff[fire[t].slot + 1]++; }
        for (int64_t k = 0; k < s->nslots; k++) toff[k + 1] += toff[k];
        std::iota(order.begin(), order.end(), 0);
        std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t c) { return fire[a].slot < fire[c].slot; });
        for (int64_t i = 0; i < nF; i++) {
            const Firing& f = fire[order[i]];
            tsend[i] = f.send;
            tclk[i] = f.clock;
            tpos[i] = f.K + order[i];
        }
        RCHK(h2d(q, s->pl_toff, toff));
        RCHK(h2d(q, s->pl_tsend, tsend));
        RCHK(h2d(q, s->pl_tclk, tclk));
        RCHK(h2d(q, s->pl_tpos, tpos));
        RCHK(h2d(q, s->pl_fsend, fsend));
    }
    // ---- the lanes
    const int64_t n_pos = M + nF, pc = std::max<int64_t>(n_pos, 1);
    RCHK(s->flags.reserve(pc + 16, false));
    RCHK(s->xr_ts.reserve(pc * 8, false));
    RCHK(s->xr_rep.reserve(pc * 8, false));
    RCHK(s->xr_slot.reserve(pc * 4, false));
    RCHK(s->xr_ch.reserve(pc * 8, false));
    RCHK(s->xr_clk.reserve(pc * 8, false));
    RCHK(s->xr_exp.reserve(pc, false));
    RCHK(s->xr_vals.reserve((size_t)std::max(na, 1) * pc * 8, false));
    RCHK(s->xr_nulls.reserve((size_t)std::max(na, 1) * pc, false));
    HIPCHK(hipMemsetAsync(s->flags.p, 0, pc + 16, st));
    SlxRows rows{s->xr_ts.as<int64_t>(), s->xr_rep.as<int64_t>(), s->xr_slot.as<u32>(), s->xr_ch.as<int64_t>(),
                 s->xr_clk.as<int64_t>(), s->xr_exp.as<unsigned char>(), s->xr_vals.as<u64>(),
                 s->xr_nulls.as<unsigned char>(), pc};
    HIPCHK(hipEventRecord(q->ev_agg0, st));
    if (!tm) {
        launch_pl_walk_lb(st, s->key_off.as<u32>(), s->ranks.as<u32>(), s->nslots, rec, T, q->seq, state_of(s),
                          s->pl_last_ts.as<int64_t>(), s->pl_last_seq.as<int64_t>(), s->pl_prev_seq.as<int64_t>(), q->ap,
                          q->d.current_on, q->d.expired_on, q->d.stream_current, rows, s->flags.as<unsigned char>());
    } else {
        if (b) {
            RCHK(s->pl_start.reserve(cap + 16, false));
            RCHK(s->pl_run.reserve(cap * 8, false));
            RCHK(s->x_blk.reserve((size_t)((N + kTile - 1) / kTile + 2) * 8, false));
            launch_pl_runs(st, cs, q->d.partition_col, N, ss, s->pl_start.as<unsigned char>(), s->x_blk.as<int64_t>(),
                           s->pl_run.as<int64_t>());
            if (xt) {
                RCHK(s->pl_x.reserve(cap * 8, false));
                launch_pl_xattr(st, cs, q->d.ts_col, rec.raw, M, s->pl_x.as<int64_t>());
            }
        }
        if (!grp)
            launch_pl_walk_tm(st, s->key_off.as<u32>(), s->ranks.as<u32>(), s->nslots, rec, s->pl_run.as<int64_t>(), T,
                              q->seq, ss, nF ? s->pl_toff.as<int64_t>() : nullptr, s->pl_tsend.as<int64_t>(),
                              s->pl_tclk.as<int64_t>(), s->pl_tpos.as<int64_t>(), s->pl_fsend.as<int64_t>(), nF, state_of(s),
                              s->rg.as<int64_t>(), q->ap, q->d.current_on, q->d.expired_on, rows,
                              s->flags.as<unsigned char>(), xt && b ? s->pl_x.as<int64_t>() : nullptr);
    }
    int64_t n_rows = 0;
    if (grp) {
        RCHK(group_time_rows(q, b ? &cs : nullptr, rec, M, nF, T, ss, xt && b, &n_rows));
        HIPCHK(hipEventRecord(q->ev_agg1, st));
        int64_t n_flushes = 0;
        RCHK(sliding_flushes(q, n_rows, &n_flushes));
        if (b) {
            q->seq += N;
            q->clock = q->clock_valid ? std::max(q->clock, info.max_tl) : info.max_tl;
            q->clock_valid = true;
            q->stats.events = N;
        }
        HIPCHK(hipEventRecord(q->ev_push1, st));
        HIPCHK(hipStreamSynchronize(st));
        float ms = 0, kms = 0;
        (void)hipEventElapsedTime(&ms, q->ev_push0, q->ev_push1);
        (void)hipEventElapsedTime(&kms, q->ev_agg0, q->ev_agg1);
        q->stats.push_ms = ms;
        q->stats.main_kernel_ms = kms;
        q->stats.main_kernel_bytes = M * (int64_t)(16 + 8 * V) + n_rows * (int64_t)(8 + 8 * na);
        return sliding_output(q, n_rows, n_flushes, false, host_out, out);
    }
    HIPCHK(hipEventRecord(q->ev_agg1, st));
    HIPCHK(hipGetLastError());
    // ---- rows in position order, one flush each
    const int fblk = (int)((n_pos + kTile - 1) / kTile);
    if (n_pos > 0) {
        RCHK(s->blk_cnt.reserve((size_t)(fblk + 16) * 8, false));
        launch_count_flags(st, s->flags.as<unsigned char>(), n_pos, s->blk_cnt.as<int64_t>(), fblk);
        HIPCHK(hipMemsetAsync(s->blk_cnt.as<int64_t>() + fblk, 0, 8, st));
        launch_scan_sum(st, s->blk_cnt.as<int64_t>(), fblk + 1);
        RCHK(read_count(q, s->blk_cnt.as<int64_t>() + fblk, &n_rows));
    }
    float kms = 0;
    (void)hipEventElapsedTime(&kms, q->ev_agg0, q->ev_agg1);
    q->stats.main_kernel_ms = kms;
    {
        const int64_t rcap = std::max<int64_t>(n_rows, 1);
        RCHK(s->out_ts.reserve(rcap * 8, false));
        RCHK(s->out_keys.reserve((size_t)std::max(1, q->kp.n) * rcap * 8, false));
        RCHK(s->out_vals.reserve((size_t)std::max(na, 1) * rcap * 8, false));
        RCHK(s->out_nulls.reserve((size_t)std::max(na, 1) * rcap, false));
        RCHK(s->out_send.reserve(rcap * 8, false));
        RCHK(s->out_clock.reserve(rcap * 8, false));
        RCHK(s->out_expired.reserve(rcap, false));
        RCHK(s->out_rep.reserve(rcap * 8, false));
        RCHK(s->out_part.reserve(rcap * 4, false));
        if (n_rows > 0)
            launch_pl_emit(st, s->flags.as<unsigned char>(), n_pos, s->blk_cnt.as<int64_t>(), fblk, rows, na, s->nk_out,
                           q->kt.dev(), q->kp, rcap, s->out_ts.as<int64_t>(), s->out_keys.as<int64_t>(),
                           s->out_vals.as<u64>(), s->out_nulls.as<unsigned char>(), s->out_expired.as<unsigned char>(),
                           s->out_send.as<int64_t>(), s->out_clock.as<int64_t>(), s->out_rep.as<int64_t>(),
                           s->out_part.as<u32>());
        HIPCHK(hipGetLastError());
    }
    int64_t n_flushes = 0;
    RCHK(sliding_flushes(q, n_rows, &n_flushes));
    if (b) {
        q->seq += N;
        q->clock = q->clock_valid ? std::max(q->clock, info.max_tl) : info.max_tl;
        q->clock_valid = true;
        q->stats.events = N;
    }
    HIPCHK(hipEventRecord(q->ev_push1, st));
    HIPCHK(hipStreamSynchronize(st));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, q->ev_push0, q->ev_push1);
    q->stats.push_ms = ms;
    q->stats.main_kernel_bytes = M * (int64_t)(16 + 8 * V) + n_rows * (int64_t)(8 + 8 * na);
    return sliding_output(q, n_rows, n_flushes, false, host_out, out);
}

int plane_push(sh_query* q, const sh_batch* b, bool host_out, const sh_out** out) {
    if (b->n < 0) return sh_fail(SH_ERR_INVALID, "negative batch size");
    if (b->n == 0) return empty_out(q, out);
    return plane_run(q, b, 0, host_out, out);
}

int plane_advance(sh_query* q, int64_t now, const sh_out** out, bool host_out) {
    return plane_run(q, nullptr, now, host_out, out);  // (externalTime: only the clock moves)
}

// ---- checkpoint of the partition lanes (sh_snapshot.cpp): per slot the lanes' device state beside the
// sliding state buffers, and on the host the Scheduler — every partition's pending notify times and
// PartitionStateHolder.states as a java.util.HashMap structure (its iteration order is its history) ----
void plane_state_buffers(sh_query* q, std::vector<std::pair<DevBuf*, size_t>>& bufs) {
    SlidingImpl* s = q->sl;
    const size_t n = (size_t)s->nslots;
    bufs = {{&s->pl_last_ts, n * 8}, {&s->pl_last_seq, n * 8}, {&s->pl_prev_seq, n * 8}, {&s->pl_key, n * 8}};
    if (s->lane == 2) bufs.push_back({&s->rg, n * (size_t)s->rc * 8});
    if (q->d.window == SH_WIN_EXT_TIME_BATCH)
        for (auto b : {std::make_pair(&s->pg_M, n * 8), std::make_pair(&s->pg_start, n * 8), std::make_pair(&s->pg_has, n),
                       std::make_pair(&s->pg_bopen, n * 8)})
            bufs.push_back(b);
    if (q->group_other && s->lane == 2) {
        const size_t FN = (size_t)std::max(1, q->ap.n_fields) * s->pg_st_n;
        bufs.push_back({&s->pg_st_cnt, (size_t)s->pg_st_n * 8});
        bufs.push_back({&s->pg_st_f, FN * 8});
        bufs.push_back({&s->pg_dq_off, FN * 8});
        bufs.push_back({&s->pg_dq_len, FN * 8});
    }
}

// a key table's size, key count and keys (hashed tables; a dense table is its size alone)
static int table_save(sh_query* q, KeyTableHost& kt, std::vector<uint8_t>& out) {
    hipStream_t st = q->ctx->stream;
    RCHK(kt.check(st));
    const uint64_t size = kt.size_;
    const int64_t nk = kt.n_keys;
    const size_t kb = kt.dense ? 0 : size * 8;
    const size_t o = out.size();
    out.resize(o + 16 + kb);
    std::memcpy(out.data() + o, &size, 8);
    std::memcpy(out.data() + o + 8, &nk, 8);
    if (kb) {
        HIPCHK(hipMemcpyAsync(out.data() + o + 16, kt.keys.p, kb, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    return SH_OK;
}

static int table_load(sh_query* q, KeyTableHost& kt, const uint8_t* p, size_t len, size_t* used, bool resizable = false) {
    hipStream_t st = q->ctx->stream;
    uint64_t size = 0;
    int64_t nk = 0;
    if (len < 16) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    std::memcpy(&size, p, 8);
    std::memcpy(&nk, p + 8, 8);
    const size_t kb = kt.dense ? 0 : size * 8;
    if (resizable && !kt.dense && size != kt.size_ && size >= 16 && (size & (size - 1)) == 0 && size <= ((uint64_t)1 << 31) &&
        16 + kb <= len)
        RCHK(kt.init_size(size));  // a pair table that grew after the query was created
    if (size != kt.size_ || nk < 0 || nk > (int64_t)size + 1) return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
    if (16 + kb > len) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    if (kb) HIPCHK(hipMemcpyAsync(kt.keys.p, p + 16, kb, hipMemcpyHostToDevice, st));
    PinnedBuf h;
    RCHK(h.reserve(16));
    uint32_t* c = h.as<uint32_t>();
    c[0] = (uint32_t)nk; c[1] = c[2] = c[3] = 0;
    HIPCHK(hipMemcpyAsync(kt.ctrl.p, c, 16, hipMemcpyHostToDevice, st));
    HIPCHK(hipStreamSynchronize(st));
    kt.n_keys = nk;
    *used = 16 + kb;
    return SH_OK;
}

// lane 3: the group key table and the carried records (in stream order)
static int pg_save(sh_query* q, std::vector<uint8_t>& out) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    auto put = [&](const void* p, size_t k) { out.insert(out.end(), (const uint8_t*)p, (const uint8_t*)p + k); };
    auto dev = [&](const void* p, size_t k) -> int {
        const size_t o = out.size();
        out.resize(o + k);
        if (k) {
            HIPCHK(hipMemcpyAsync(out.data() + o, p, k, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
        }
        return SH_OK;
    };
    RCHK(q->gkt.check(st));
    const uint64_t gsize = q->gkt.size_;
    const int64_t gnk = q->gkt.n_keys, n = s->pg_n;
    const int V = std::max(1, q->ap.n_vcols);
    put(&gsize, 8);
    put(&gnk, 8);
    RCHK(dev(q->gkt.keys.p, q->gkt.dense ? 0 : gsize * 8));
    put(&n, 8);
    const PgBufs& B = s->pg[0];
    RCHK(dev(B.ps.p, n * 4));
    RCHK(dev(B.gs.p, n * 4));
    RCHK(dev(B.ts.p, n * 8));
    RCHK(dev(B.seq.p, n * 8));
    RCHK(dev(B.clk.p, n * 8));
    RCHK(dev(B.prev.p, n));
    for (int v = 0; v < V; v++) RCHK(dev(B.vals.as<u64>() + (size_t)v * B.cap, n * 8));
    RCHK(dev(B.x.p, n * 8));
    if (B.xe.p) {
        RCHK(dev(B.xe.p, n * 8));
        RCHK(dev(B.xm.p, n * 8));
    }
    // the timeout's per-partition window state (xt_walk), in slot order
    std::vector<uint32_t> xs;
    for (auto& kv : s->xt_parts) xs.push_back(kv.first);
    std::sort(xs.begin(), xs.end());
    const uint64_t nx = xs.size();
    put(&nx, 8);
    for (uint32_t sl : xs) {
        const SlidingImpl::XtPart& P = s->xt_parts[sl];
        const int64_t v[6] = {P.n, P.bs, P.cur0, P.pe_lo, P.pe_hi, P.L};
        const uint8_t fl = P.flushed;
        put(&sl, 4);
        put(v, sizeof v);
        put(&fl, 1);
    }
    return SH_OK;
}

static int pg_load(sh_query* q, const uint8_t* p, size_t len, size_t* used) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    size_t o = 0;
    auto get = [&](void* d, size_t k) {
        if (o + k > len) return false;
        std::memcpy(d, p + o, k);
        o += k;
        return true;
    };
    uint64_t gsize = 0;
    int64_t gnk = 0, n = 0;
    if (!get(&gsize, 8) || !get(&gnk, 8) || gsize != q->gkt.size_ || gnk < 0 || gnk > (int64_t)gsize + 1)
        return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
    const size_t kb = q->gkt.dense ? 0 : gsize * 8;
    if (o + kb + 8 > len) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    const uint8_t* keys = p + o;
    o += kb;
    get(&n, 8);
    const int V = std::max(1, q->ap.n_vcols);
    const size_t xb = q->d.window == SH_WIN_EXT_TIME_BATCH ? 16 : 0;  // (batch ends, attribute maxima)
    if (n < 0 || n > (int64_t)(len / 8) || o + (size_t)n * (4 + 4 + 8 + 8 + 8 + 1 + 8 * (size_t)V + 8 + xb) > len)
        return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    // validated: now replace the state
    if (kb) HIPCHK(hipMemcpyAsync(q->gkt.keys.p, keys, kb, hipMemcpyHostToDevice, st));
    {
        PinnedBuf h;
        RCHK(h.reserve(16));
        uint32_t* c = h.as<uint32_t>();
        c[0] = (uint32_t)gnk; c[1] = c[2] = c[3] = 0;
        HIPCHK(hipMemcpyAsync(q->gkt.ctrl.p, c, 16, hipMemcpyHostToDevice, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    q->gkt.n_keys = gnk;
    RCHK(pg_grow(q, s->pg[0], s->pg[0], std::max<int64_t>(n, 1), 0, V));
    const PgBufs& B = s->pg[0];
    auto up = [&](void* d, size_t k) -> int {
        if (k) HIPCHK(hipMemcpyAsync(d, p + o, k, hipMemcpyHostToDevice, st));
        o += k;
        return SH_OK;
    };
    RCHK(up(B.ps.p, n * 4));
    RCHK(up(B.gs.p, n * 4));
    RCHK(up(B.ts.p, n * 8));
    RCHK(up(B.seq.p, n * 8));
    RCHK(up(B.clk.p, n * 8));
    RCHK(up(B.prev.p, n));
    for (int v = 0; v < V; v++) RCHK(up(B.vals.as<u64>() + (size_t)v * B.cap, n * 8));
    RCHK(up(B.x.p, n * 8));
    if (B.xe.p) {
        RCHK(up(B.xe.p, n * 8));
        RCHK(up(B.xm.p, n * 8));
    }
    HIPCHK(hipStreamSynchronize(st));  // the blob may be freed after the call
    s->pg_n = n;
    uint64_t nx = 0;
    if (!get(&nx, 8) || nx > (len - o) / 53) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    std::unordered_map<uint32_t, SlidingImpl::XtPart> parts;
    for (uint64_t i = 0; i < nx; i++) {
        uint32_t sl = 0;
        int64_t v[6];
        uint8_t fl = 0;
        get(&sl, 4);
        get(v, sizeof v);
        get(&fl, 1);
        if (sl >= (uint64_t)s->nslots) return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
        SlidingImpl::XtPart P;
        P.n = v[0]; P.bs = v[1]; P.cur0 = v[2]; P.pe_lo = v[3]; P.pe_hi = v[4]; P.L = v[5];
        P.flushed = fl != 0;
        parts[sl] = P;
    }
    s->xt_parts = std::move(parts);
    *used = o;
    return SH_OK;
}

int plane_host_save(sh_query* q, std::vector<uint8_t>& out) {
    SlidingImpl* s = q->sl;
    auto put = [&](const void* p, size_t k) { out.insert(out.end(), (const uint8_t*)p, (const uint8_t*)p + k); };
    // pending notify times by slot, in slot order (the armed set is their fronts)
    std::vector<uint32_t> slots;
    for (auto& kv : s->pl_pend) slots.push_back(kv.first);
    std::sort(slots.begin(), slots.end());
    const uint64_t np = slots.size();
    put(&np, 8);
    for (uint32_t sl : slots) {
        const auto& d = s->pl_pend[sl];
        const uint64_t len = d.size();
        put(&sl, 4);
        put(&len, 8);
        for (int64_t t : d) put(&t, 8);
    }
    std::vector<uint8_t> m;
    s->pl_states.save(m);
    const uint64_t ml = m.size();
    put(&ml, 8);
    put(m.data(), m.size());
    if (s->lane == 2 && q->group_other) {
        RCHK(table_save(q, q->gkt, out));
        RCHK(table_save(q, q->pgkt, out));
        // the min / max deque pool
        const uint64_t w = (uint64_t)s->pg_dq_words;
        const size_t o = out.size();
        out.resize(o + 8 + w * 8);
        std::memcpy(out.data() + o, &w, 8);
        if (w) {
            HIPCHK(hipMemcpyAsync(out.data() + o + 8, s->pg_dq_pool.p, w * 8, hipMemcpyDeviceToHost, q->ctx->stream));
            HIPCHK(hipStreamSynchronize(q->ctx->stream));
        }
    }
    if (s->lane == 4) {
        // partitioned timeBatch(T, true): the group and (partition, group) tables, the shared nextEmitTime,
        // every partition's RESET count and the states
        RCHK(table_save(q, q->gkt, out));
        RCHK(table_save(q, q->pgkt, out));
        std::vector<uint32_t> sl;
        for (auto& kv : s->tb_bids) sl.push_back(kv.first);
        std::sort(sl.begin(), sl.end());
        const uint64_t nb = sl.size();
        put(&s->tb_next_emit, 8);
        put(&s->tb_chunk_base, 8);
        put(&nb, 8);
        for (uint32_t x : sl) {
            put(&x, 4);
            put(&s->tb_bids[x], 8);
        }
        const size_t ns = q->pgkt.size_ + 1, A = (size_t)std::max(1, q->ap.n);
        const std::pair<const DevBuf*, size_t> bufs[] = {{&s->tb_cnt, ns * 8}, {&s->tb_bid, ns * 8},
                                                         {&s->tb_f, A * ns * 8}, {&s->tb_has, A * ns}};
        for (auto& b : bufs) {
            const size_t o = out.size();
            out.resize(o + b.second);
            HIPCHK(hipMemcpyAsync(out.data() + o, b.first->p, b.second, hipMemcpyDeviceToHost, q->ctx->stream));
        }
        HIPCHK(hipStreamSynchronize(q->ctx->stream));
    }
    return s->lane == 3 ? pg_save(q, out) : SH_OK;
}

int plane_host_load(sh_query* q, const uint8_t* p, size_t n, size_t* used) {
    SlidingImpl* s = q->sl;
    size_t o = 0;
    auto get = [&](void* d, size_t k) {
        if (o + k > n) return false;
        std::memcpy(d, p + o, k);
        o += k;
        return true;
    };
    std::unordered_map<uint32_t, std::deque<int64_t>> pend;
    std::set<std::pair<int64_t, uint32_t>> armed;
    uint64_t np = 0;
    if (!get(&np, 8) || np > (uint64_t)s->nslots) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    for (uint64_t i = 0; i < np; i++) {
        uint32_t sl;
        uint64_t len;
        if (!get(&sl, 4) || !get(&len, 8) || sl >= (uint64_t)s->nslots || len == 0 || len > n)
            return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        auto& d = pend[sl];
        for (uint64_t j = 0; j < len; j++) {
            int64_t t;
            if (!get(&t, 8)) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
            d.push_back(t);
        }
        armed.insert(std::make_pair(d.front(), sl));
    }
    uint64_t ml = 0;
    if (!get(&ml, 8) || o + ml > n) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    shj::JavaStringMap m;
    if (!m.load(p + o, (size_t)ml)) return sh_fail(SH_ERR_INVALID, "snapshot: scheduler state unreadable");
    o += ml;
    if (s->lane == 2 && q->group_other) {
        size_t u = 0;
        RCHK(table_load(q, q->gkt, p + o, n - o, &u));
        o += u;
        RCHK(table_load(q, q->pgkt, p + o, n - o, &u, true));
        o += u;
        // the state arrays were restored at the blob's size (sh_snapshot.cpp): they must match the table's
        if (s->pg_st_n != (int64_t)q->pgkt.size_ + 1) {
            s->pg_st_n = (int64_t)q->pgkt.size_ + 1;
            const size_t FN = (size_t)std::max(1, q->ap.n_fields) * s->pg_st_n;
            if (s->pg_st_cnt.cap < (size_t)s->pg_st_n * 8 || s->pg_st_f.cap < FN * 8 || s->pg_dq_off.cap < FN * 8 ||
                s->pg_dq_len.cap < FN * 8)
                return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
        }
        uint64_t w = 0;
        if (!get(&w, 8) || w > (n - o) / 8) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        RCHK(s->pg_dq_pool.reserve((size_t)std::max<uint64_t>(w, 8) * 8, false));
        if (w) HIPCHK(hipMemcpyAsync(s->pg_dq_pool.p, p + o, w * 8, hipMemcpyHostToDevice, q->ctx->stream));
        HIPCHK(hipStreamSynchronize(q->ctx->stream));
        s->pg_dq_words = (int64_t)w;
        o += w * 8;
    }
    if (s->lane == 4) {
        size_t u = 0;
        RCHK(table_load(q, q->gkt, p + o, n - o, &u));
        o += u;
        RCHK(table_load(q, q->pgkt, p + o, n - o, &u));
        o += u;
        int64_t ne = 0, cb = 0;
        uint64_t nb = 0;
        if (!get(&ne, 8) || !get(&cb, 8) || !get(&nb, 8) || nb > (n - o) / 12)
            return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        std::unordered_map<uint32_t, int64_t> bids;
        for (uint64_t i = 0; i < nb; i++) {
            uint32_t x = 0;
            int64_t v = 0;
            get(&x, 4);
            get(&v, 8);
            bids[x] = v;
        }
        const size_t ns = q->pgkt.size_ + 1, A = (size_t)std::max(1, q->ap.n);
        const std::pair<DevBuf*, size_t> bufs[] = {{&s->tb_cnt, ns * 8}, {&s->tb_bid, ns * 8}, {&s->tb_f, A * ns * 8},
                                                   {&s->tb_has, A * ns}};
        for (auto& b : bufs) {
            if (o + b.second > n) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
            HIPCHK(hipMemcpyAsync(b.first->p, p + o, b.second, hipMemcpyHostToDevice, q->ctx->stream));
            o += b.second;
        }
        HIPCHK(hipStreamSynchronize(q->ctx->stream));
        s->tb_next_emit = ne;
        s->tb_chunk_base = cb;
        s->tb_bids = std::move(bids);
    }
    size_t pg_used = 0;
    if (s->lane == 3) {
        // (the lanes of lane 3 carry no Scheduler: its part above is empty)
        RCHK(pg_load(q, p + o, n - o, &pg_used));
        o += pg_used;
    }
    std::unordered_map<uint32_t, std::u16string> flow;
    m.visit_keys([&](uint32_t slot, const std::u16string& k) { flow[slot] = k; });
    s->pl_pend = std::move(pend);
    s->pl_armed = std::move(armed);
    s->pl_states = std::move(m);
    s->pl_flow = std::move(flow);
    *used = o;
    return SH_OK;
}
