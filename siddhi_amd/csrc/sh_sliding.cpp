// sh_sliding.cpp — sliding `from S[cond]#window.time(T) select k, aggs group by k insert into O`
// (TimeWindowProcessor + QuerySelector in SLIDE mode) behind sh_query_* (kind 1).
//
// The window contents of every key live on the device in per-key rings; aggregator state per key
// (counts, running sums with Java's residue, min/max deques) persists across pushes. A push emits,
// per send, one row per key that had a current event in that send (first-occurrence order), with
// the aggregate values after that key's last event in the send (QuerySelector.java:315-374).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "sh_runtime.h"
#include "sh_sliding.h"

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

#include "sh_sliding_impl.h"

SlState state_of(SlidingImpl* s) {
    SlState S;
    S.nslots = s->nslots;
    S.rc = s->rc;
    S.cnt = s->cnt.as<int64_t>();
    S.f = s->f.as<u64>();
    S.mm = s->mm.as<u64>();
    S.mm_has = s->mm_has.as<unsigned char>();
    S.dq_head = s->dq_head.as<int64_t>();
    S.dq_len = s->dq_len.as<int64_t>();
    S.dq = s->dq.as<u64>();
    S.rhead = s->rhead.as<int64_t>();
    S.rlen = s->rlen.as<int64_t>();
    S.rpm = s->rpm.as<int64_t>();
    S.rval = s->rval.as<u64>();
    S.cur_send = s->cur_send.as<int64_t>();
    S.cur_first = s->cur_first.as<int64_t>();
    return S;
}

static int alloc_zero(DevBuf& b, size_t bytes, int fill = 0) {
    RCHK(b.reserve(std::max<size_t>(bytes, 8), false));
    if (hipMemsetAsync(b.p, fill, std::max<size_t>(bytes, 8), g_stream) != hipSuccess) return sh_fail(SH_ERR_DEVICE, "memset failed");
    return SH_OK;
}

// (re)size the per-key rings and deques to capacity rc (power of two), keeping their contents
// (keep = false: fresh buffers, e.g. before a restore overwrites them — the live rings may hold more
// entries than the new capacity, so they must not be copied over)
// value columns of a ring entry: the aggregated ones, plus the group slot on time lanes grouped by
// other columns (sh_plane.cpp)
int ring_vcols(const sh_query* q) {
    return std::max(1, q->ap.n_vcols) +
           (q->group_other && (q->d.window == SH_WIN_TIME || q->d.window == SH_WIN_EXT_TIME) ? 1 : 0);
}

int size_rings(sh_query* q, int64_t new_rc, bool keep) {
    SlidingImpl* s = q->sl;
    int F = std::max(1, q->ap.n_fields), V = ring_vcols(q);
    int64_t n = s->nslots;
    DevBuf rpm2, rval2, dq2;
    RCHK(rpm2.reserve((size_t)n * new_rc * 8, false));
    RCHK(rval2.reserve((size_t)V * n * new_rc * 8, false));
    RCHK(dq2.reserve((size_t)F * n * new_rc * 8, false));
    DevBuf rg2;
    if (s->xm) RCHK(rg2.reserve((size_t)n * new_rc * 8, false));
    hipStream_t st = q->ctx->stream;
    if (s->rc > 0 && keep) {
        launch_sl_regrow(st, (const u64*)s->rpm.p, (u64*)rpm2.p, s->rhead.as<int64_t>(), s->rlen.as<int64_t>(), n, 1,
                         s->rc, new_rc, false);
        launch_sl_regrow(st, s->rval.as<u64>(), rval2.as<u64>(), s->rhead.as<int64_t>(), s->rlen.as<int64_t>(), n, V,
                         s->rc, new_rc, false);
        launch_sl_regrow(st, s->dq.as<u64>(), dq2.as<u64>(), s->dq_head.as<int64_t>(), s->dq_len.as<int64_t>(), n, F,
                         s->rc, new_rc, true);
        if (s->xm)
            launch_sl_regrow(st, (const u64*)s->rg.p, (u64*)rg2.p, s->rhead.as<int64_t>(), s->rlen.as<int64_t>(), n, 1,
                             s->rc, new_rc, false);
        HIPCHK(hipMemsetAsync(s->rhead.p, 0, n * 8, st));
        HIPCHK(hipMemsetAsync(s->dq_head.p, 0, (size_t)F * n * 8, st));
        HIPCHK(hipStreamSynchronize(st));
    }
    s->rpm = std::move(rpm2); s->rval = std::move(rval2); s->dq = std::move(dq2);
    if (s->xm) s->rg = std::move(rg2);
    s->rc = new_rc;
    return SH_OK;
}

int sliding_create(sh_query* q) {
    if (q->partitioned) return sh_fail(SH_ERR_UNSUPPORTED, "partitioned sliding windows are not on the GPU");
    SlidingImpl* s = new SlidingImpl();
    q->sl = s;
    const bool plane = q->d.partition_col >= 0;  // partitioned lengthBatch / time keyed by the partition
    // expired output, pass-through, and the partition lanes' time windows keep each ring entry's 2nd word
    s->xm = q->d.expired_on != 0 || q->ap.n == 0 || (plane && (q->d.window == SH_WIN_TIME || q->d.window == SH_WIN_EXT_TIME));
    s->nslots = (int64_t)q->kt.size_ + 1;
    int F = std::max(1, q->ap.n_fields);
    int64_t n = s->nslots;
    RCHK(alloc_zero(s->cnt, n * 8));
    RCHK(alloc_zero(s->f, (size_t)F * n * 8));
    RCHK(alloc_zero(s->mm, (size_t)F * n * 8));
    RCHK(alloc_zero(s->mm_has, (size_t)F * n));
    RCHK(alloc_zero(s->dq_head, (size_t)F * n * 8));
    RCHK(alloc_zero(s->dq_len, (size_t)F * n * 8));
    RCHK(alloc_zero(s->rhead, n * 8));
    RCHK(alloc_zero(s->rlen, n * 8));
    RCHK(alloc_zero(s->cur_send, n * 8, 0xff));
    RCHK(alloc_zero(s->cur_first, n * 8));
    RCHK(s->info.reserve(sizeof(SlInfo), false));
    if (hipHostMalloc((void**)&s->h_info, sizeof(SlInfo), hipHostMallocDefault) != hipSuccess)
        return sh_fail(SH_ERR_OOM, "pinned alloc failed");
    RCHK(size_rings(q, 64));
    int P = 1;
    // key partitions small enough for one replay lane per key (64 for k_sl_own, kSlKeyLanes for
    // k_sl_own_d); the multisplit's LDS histogram caps P at 4096, beyond that lanes own several keys
    const int per = sliding_keys_per_partition(q->ap);
    while (P < 4096 && (int64_t)P * per < n) P <<= 1;
    s->P = P;
    s->logP = 0;
    while ((1 << s->logP) < P) s->logP++;
    (void)hipEventCreate(&q->ev_push0); (void)hipEventCreate(&q->ev_push1);
    (void)hipEventCreate(&q->ev_agg0); (void)hipEventCreate(&q->ev_agg1);
    (void)hipEventCreate(&q->ev_srt0); (void)hipEventCreate(&q->ev_srt1);
    if (plane) RCHK(plane_create(q));
    return SH_OK;
}

void sliding_destroy(sh_query* q) {
    SlidingImpl* s = q->sl;
    if (!s) return;
    DevBuf* bufs[] = {&s->cnt, &s->f, &s->mm, &s->mm_has, &s->dq_head, &s->dq_len, &s->dq, &s->rhead, &s->rlen,
                      &s->rpm, &s->rval, &s->cur_send, &s->cur_first, &s->blk_pass, &s->blk_tl, &s->blk_pm,
                      &s->info, &s->rec_raw, &s->rec_slot, &s->rec_clock, &s->rec_pm, &s->rec_ts, &s->rec_vals, &s->rec_aos,
                      &s->slot_cnt, &s->counts, &s->tmp, &s->ranks, &s->part_off, &s->flags, &s->p_raw,
                      &s->p_slot, &s->p_clock, &s->p_pm, &s->p_ts, &s->p_vals, &s->rows_ts,
                      &s->rows_slot, &s->rows_send, &s->rows_clock, &s->rows_vals, &s->rows_nulls, &s->blk_cnt,
                      &s->out_ts, &s->out_keys, &s->out_vals, &s->out_nulls, &s->out_send, &s->out_clock,
                      &s->out_expired, &s->flush_off, &s->flush_clock, &s->iota, &s->rec_sclk, &s->sort_tmp, &s->key_off, &s->g_rank, &s->inv, &s->rows_k,
                      &s->rg, &s->upm, &s->useq, &s->upm2, &s->useq2, &s->npend, &s->npend2, &s->x_sK, &s->x_scb,
                      &s->x_slast, &s->x_cK, &s->x_cC, &s->x_cS, &s->x_fire, &s->x_keep, &s->x_idx, &s->x_fK,
                      &s->x_fC, &s->x_fS, &s->x_blk, &s->x_xop, &s->x_xch, &s->x_xts, &s->x_xclk, &s->x_aop,
                      &s->x_nexp, &s->xr_ts, &s->xr_rep, &s->xr_slot, &s->xr_ch, &s->xr_clk, &s->xr_exp,
                      &s->xr_vals, &s->xr_nulls, &s->xr_aos, &s->x_xa, &s->x_xx, &s->x_bnd, &s->pl_last_ts, &s->pl_last_seq, &s->pl_prev_seq, &s->pl_key,
                      &s->pl_start, &s->pl_run, &s->pl_reg, &s->pl_toff, &s->pl_tsend, &s->pl_tclk, &s->pl_tpos,
                      &s->pl_fsend};
    for (DevBuf* b : bufs) b->release();
    s->x_h.release();
    if (s->h_info) (void)hipHostFree(s->h_info);
    delete s;
    q->sl = nullptr;
}

int empty_out(sh_query* q, const sh_out** out) {
    q->out.reset();
    // (the partition lanes without group-by report no key column: the partition key is internal)
    const int nk = q->sl && q->sl->nk_out >= 0 ? q->sl->nk_out : q->kp.n;
    *out = q->out.view(nk, q->ap.n, q->vtypes);
    return SH_OK;
}

static int sliding_finish(sh_query* q, int64_t M, int64_t rec_cap, int64_t need, int64_t send_size,
                          int64_t send_base, int64_t raw_base, bool want_order, bool host_out, const sh_out** out,
                          bool presorted = false);

// the push's records sorted stably by key slot (p_slot, ranks) and room for the key offsets
static int sort_keyed(sh_query* q, const u32* slot, int64_t M) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    size_t tb = 0;
    if (sort_slot_ranks(nullptr, &tb, slot, nullptr, nullptr, M, s->nslots, st))
        return sh_fail(SH_ERR_DEVICE, "radix sort sizing failed");
    RCHK(s->sort_tmp.reserve(std::max<size_t>(tb, 16), false));
    RCHK(s->p_slot.reserve(M * 4, false));
    RCHK(s->ranks.reserve(M * 4, false));
    RCHK(s->key_off.reserve((size_t)(s->nslots + 1) * 4, false));
    if (sort_slot_ranks(s->sort_tmp.p, &tb, slot, s->p_slot.as<u32>(), s->ranks.as<u32>(), M, s->nslots, st))
        return sh_fail(SH_ERR_DEVICE, "radix sort failed");
    return SH_OK;
}
static int slx_run(sh_query* q, const sh_batch* b, int64_t now, bool host_out, const sh_out** out);

// Hashed keys of a time() window get a fresh table once more than half full: keys whose every window
// event has expired for any later event (last PM + T <= the playback clock) are dropped — the state the
// reference destroys (AttributeAggregatorExecutor canDestroy) — and the live keys' state moves to
// their new slots. Same table size, so the per-slot layouts keep their strides.
static int sliding_rekey(sh_query* q) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    const int64_t size = (int64_t)q->kt.size_, n = s->nslots;
    if (n != size + 1) return SH_OK;
    KeyTableHost nk;
    RCHK(nk.init_size((size_t)size));
    DevBuf map;
    RCHK(map.reserve((size_t)n * 4, false));
    if (s->xm)
        launch_slx_rekey_map(st, size, q->kt.dev(), nk.dev(), s->rlen.as<int64_t>(), s->cnt.as<int64_t>(),
                             s->f.as<u64>(), n, q->ap, map.as<u32>());
    else
        launch_sl_rekey_map(st, size, q->kt.dev(), nk.dev(), s->rhead.as<int64_t>(), s->rlen.as<int64_t>(),
                            s->rpm.as<int64_t>(), s->rc, q->d.window_param, q->clock, map.as<u32>());
    HIPCHK(hipGetLastError());
    RCHK(nk.check(st));
    const int64_t F = std::max(1, q->ap.n_fields), V = std::max(1, q->ap.n_vcols), rc = s->rc;
    struct L { DevBuf* b; int64_t outer, inner; int fill; };
    const L lay[] = {{&s->cnt, 1, 8, 0},        {&s->f, F, 8, 0},          {&s->mm, F, 8, 0},
                     {&s->mm_has, F, 1, 0},     {&s->dq_head, F, 8, 0},    {&s->dq_len, F, 8, 0},
                     {&s->dq, F, rc * 8, 0},    {&s->rhead, 1, 8, 0},      {&s->rlen, 1, 8, 0},
                     {&s->rpm, 1, rc * 8, 0},   {&s->rval, V, rc * 8, 0},  {&s->cur_send, 1, 8, 0xff},
                     {&s->cur_first, 1, 8, 0}, {&s->rg, 1, rc * 8, 0}};
    for (const L& l : lay) {
        if (l.b == &s->rg && !s->xm) continue;
        DevBuf nb;
        const size_t bytes = (size_t)l.outer * n * l.inner;
        RCHK(nb.reserve(std::max<size_t>(bytes, 8), false));
        HIPCHK(hipMemsetAsync(nb.p, l.fill, std::max<size_t>(bytes, 8), st));
        launch_sl_rekey_copy(st, l.b->p, nb.p, l.outer, n, l.inner, map.as<u32>());
        HIPCHK(hipGetLastError());
        *l.b = std::move(nb);  // (stream-ordered release of the old buffer)
    }
    HIPCHK(hipStreamSynchronize(st));
    q->kt = std::move(nk);
    return SH_OK;
}

// the key-sorted replay with 48-byte records (k_sl_wkey<AOS>): time windows of the count / sum / avg
// / min / max-of-one-double shape with a min or max (sliding_keyed_ok)
static bool keyed_aos(const sh_query* q) { return q->d.window == SH_WIN_TIME && sliding_keyed_ok(q->ap); }

int sliding_push(sh_query* q, const sh_batch* b, bool host_out, const sh_out** out) {
    SlidingImpl* s = q->sl;
    if (s->lane) return plane_push(q, b, host_out, out);
    hipStream_t st = q->ctx->stream;
    q->stats = sh_stats{};
    int64_t N = b->n;
    if (N < 0) return sh_fail(SH_ERR_INVALID, "negative batch size");
    if (N == 0) return empty_out(q, out);
    if (N >= (int64_t)0xFFFFFFF0ll) return sh_fail(SH_ERR_INVALID, "push larger than 4G events");
    // hysteresis: after a rebuild that kept many live keys, the next one waits until size/8 more keys
    // arrived (capped at 7/8 full), instead of copying every slot's state on every push
    const int64_t tsz = (int64_t)q->kt.size_;
    if (!q->kt.dense && q->kp.n > 0 && (q->d.window == SH_WIN_TIME || s->xm) && q->clock_valid &&
        q->kt.n_keys > std::max<int64_t>(tsz / 2, s->rekey_floor)) {
        RCHK(sliding_rekey(q));
        s->rekey_floor = std::min<int64_t>(q->kt.n_keys + tsz / 8, tsz * 7 / 8);
    }
    if (s->xm) return slx_run(q, b, 0, host_out, out);
    HIPCHK(hipEventRecord(q->ev_push0, st));
    ColSet cs{};
    cs.n = q->d.n_cols;
    for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->d.col_types[c]; cs.ptr[c] = b->cols[c]; }
    int nblk = (int)((N + kTile - 1) / kTile);
    RCHK(s->blk_pass.reserve(nblk * 8, false));
    RCHK(s->blk_tl.reserve(nblk * 8, false));
    RCHK(s->blk_pm.reserve(nblk * 8, false));
    WinParams wp{};
    wp.kind = q->d.window;  // SH_WIN_TIME or SH_WIN_EXT_TIME
    wp.ts_col = q->d.ts_col;
    wp.clock_valid = q->clock_valid;
    wp.clock0 = q->clock;
    wp.send_size = b->send_size;
    wp.N = N;
    wp.rec_seq = q->tune.sl_records_seq;
    launch_sl_prefix(st, b->ts, cs, q->fp, wp, s->blk_pass.as<int64_t>(), s->blk_tl.as<int64_t>(),
                     s->blk_pm.as<int64_t>(), nblk, s->info.as<SlInfo>());
    // records of all passing events (capacity N; the exact count is known after the prefix scan)
    int V = std::max(1, q->ap.n_vcols);
    RCHK(s->rec_raw.reserve(N * 4, false));
    RCHK(s->rec_slot.reserve(N * 4, false));
    RCHK(s->rec_clock.reserve(N * 8, false));
    RCHK(s->rec_pm.reserve(N * 8, false));
    RCHK(s->rec_ts.reserve(N * 8, false));
    RCHK(s->rec_vals.reserve((size_t)V * N * 8, false));
    RCHK(s->slot_cnt.reserve(s->nslots * 4, false));
    // keyed replay over lane-strided records (every event passes, M = N): the records are sorted by key
    // slot right away and the key offsets and ring need come from the sorted slots (no per-slot counts)
    const bool pre = keyed_aos(q) && sl_records_seq_applies(q->fp, wp, q->ap);
    HIPCHK(hipMemsetAsync(s->slot_cnt.p, 0, s->nslots * 4, st));
    SlRecords rec{s->rec_raw.as<u32>(), s->rec_slot.as<u32>(), s->rec_clock.as<int64_t>(), s->rec_pm.as<int64_t>(),
                  s->rec_ts.as<int64_t>(), s->rec_vals.as<u64>(), N};
    if (keyed_aos(q)) {
        RCHK(s->rec_aos.reserve((size_t)N * kSlAosWords * 8, false));
        rec.aos = s->rec_aos.as<u64>();
    }
    const bool ext = q->d.window == SH_WIN_EXT_TIME;
    if (ext) RCHK(s->rec_sclk.reserve(N * 8, false));
    launch_sl_records(st, b->ts, cs, q->fp, wp, q->kp, q->kt.dev(), q->ap, s->blk_pass.as<int64_t>(),
                      s->blk_tl.as<int64_t>(), s->blk_pm.as<int64_t>(), s->pm, rec,
                      pre ? nullptr : s->slot_cnt.as<u32>(), nblk, ext ? s->rec_sclk.as<int64_t>() : nullptr);
    HIPCHK(hipMemsetAsync((char*)s->info.p + offsetof(SlInfo, need), 0, 8, st));
    int64_t* need_dev = (int64_t*)((char*)s->info.p + offsetof(SlInfo, need));
    q->srt_timed = pre;
    if (pre) {
        HIPCHK(hipEventRecord(q->ev_srt0, st));  // (the sort is part of the replay's time)
        RCHK(sort_keyed(q, rec.slot, N));
        HIPCHK(hipEventRecord(q->ev_srt1, st));
        launch_counts_sorted(st, s->p_slot.as<u32>(), N, s->slot_cnt.as<u32>());
    }
    launch_sl_need(st, s->slot_cnt.as<u32>(), s->rlen.as<int64_t>(), s->nslots, need_dev);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(s->h_info, s->info.p, sizeof(SlInfo), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    RCHK(q->kt.check(st));
    SlInfo info = *s->h_info;
    RCHK(sliding_finish(q, info.total_pass, N, info.need, b->send_size, s->send_base, q->seq, false, host_out, out,
                        pre));
    q->seq += N;
    // window state moves on
    q->clock = q->clock_valid ? std::max(q->clock, info.max_tl) : info.max_tl;
    q->clock_valid = true;
    s->pm = std::max(s->pm, info.max_pm);
    s->send_base += b->send_size > 0 ? (N + b->send_size - 1) / b->send_size : 1;
    q->stats.events = N;
    return SH_OK;
}

// Sharded owner push (sh_shard.cpp): M records of this owner's keys, already filtered, in stream
// order, with their send's global clock, the global PM and their global stream index. The push's
// sends are numbered from send_base; raw = gidx - raw_base is the position in the global push.
int sliding_push_given(sh_query* q, int64_t M, const int64_t* ts, const void* const* cols, const int64_t* gclk,
                       const int64_t* gpm, const uint64_t* gidx, int64_t raw_base, int64_t send_size,
                       int64_t send_base, bool host_out, const sh_out** out, int64_t n_global) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    q->stats = sh_stats{};
    if (M < 0 || n_global >= (int64_t)0xFFFFFFF0ll) return sh_fail(SH_ERR_INVALID, "bad sharded sliding push");
    HIPCHK(hipEventRecord(q->ev_push0, st));
    int V = std::max(1, q->ap.n_vcols);
    int64_t cap = std::max<int64_t>(M, 1);
    RCHK(s->rec_raw.reserve(cap * 4, false));
    RCHK(s->rec_slot.reserve(cap * 4, false));
    RCHK(s->rec_clock.reserve(cap * 8, false));
    RCHK(s->rec_pm.reserve(cap * 8, false));
    RCHK(s->rec_ts.reserve(cap * 8, false));
    RCHK(s->rec_vals.reserve((size_t)V * cap * 8, false));
    RCHK(s->slot_cnt.reserve(s->nslots * 4, false));
    RCHK(s->info.reserve(sizeof(SlInfo), false));
    HIPCHK(hipMemsetAsync(s->slot_cnt.p, 0, s->nslots * 4, st));
    ColSet cs{};
    cs.n = q->d.n_cols;
    for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->load_type[c]; cs.ptr[c] = cols[c]; }
    SlRecords rec{s->rec_raw.as<u32>(), s->rec_slot.as<u32>(), s->rec_clock.as<int64_t>(), s->rec_pm.as<int64_t>(),
                  s->rec_ts.as<int64_t>(), s->rec_vals.as<u64>(), cap};
    if (keyed_aos(q)) {
        RCHK(s->rec_aos.reserve((size_t)cap * kSlAosWords * 8, false));
        rec.aos = s->rec_aos.as<u64>();
    }
    launch_sl_records_given(st, M, ts, cs, q->kp, q->kt.dev(), q->ap, gclk, gpm, (const u64*)gidx, raw_base, rec,
                            s->slot_cnt.as<u32>());
    HIPCHK(hipMemsetAsync((char*)s->info.p + offsetof(SlInfo, need), 0, 8, st));
    launch_sl_need(st, s->slot_cnt.as<u32>(), s->rlen.as<int64_t>(), s->nslots,
                   (int64_t*)((char*)s->info.p + offsetof(SlInfo, need)));
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(s->h_info, s->info.p, sizeof(SlInfo), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    RCHK(q->kt.check(st));
    RCHK(sliding_finish(q, M, cap, s->h_info->need, send_size, send_base, raw_base, true, host_out, out));
    q->stats.events = M;
    return SH_OK;
}

// The rest of a push once its M rank-ordered records are in place: ring growth, the per-key-partition
// replay (launch_sliding_own), rows in rank order, one flush per send. want_order: also the global
// stream index of every row's first event (raw_base + raw), into q->order_host / q->out_order.
static int sliding_finish(sh_query* q, int64_t M, int64_t rec_cap, int64_t need, int64_t send_size,
                          int64_t send_base, int64_t raw_base, bool want_order, bool host_out, const sh_out** out,
                          bool presorted) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    int V = std::max(1, q->ap.n_vcols);
    SlRecords rec{s->rec_raw.as<u32>(), s->rec_slot.as<u32>(), s->rec_clock.as<int64_t>(), s->rec_pm.as<int64_t>(),
                  s->rec_ts.as<int64_t>(), s->rec_vals.as<u64>(), rec_cap};
    if (keyed_aos(q)) rec.aos = s->rec_aos.as<u64>();
    if (need > s->rc) {
        int64_t nrc = s->rc;
        while (nrc < need) nrc <<= 1;
        RCHK(size_rings(q, nrc));
    }
    int64_t n_rows = 0;
    if (M > 0) {
        const int na = q->ap.n;
        const bool keyed = keyed_aos(q);
        // per-event sends through the keyed replay: every record opens its own row, so there are no
        // first-occurrence flags to write, count or scan (n_rows = M)
        const bool all_rows = keyed && send_size == 1;
        // rows indexed by first-occurrence rank
        RCHK(s->flags.reserve(M + 16, false));
        RCHK(s->rows_ts.reserve(M * 8, false));
        RCHK(s->rows_rep.reserve(M * 4, false));
        RCHK(s->rows_slot.reserve(M * 4, false));
        RCHK(s->rows_send.reserve(M * 8, false));
        RCHK(s->rows_clock.reserve(M * 8, false));
        RCHK(s->rows_vals.reserve((size_t)na * M * 8, false));
        RCHK(s->rows_nulls.reserve((size_t)na * M, false));
        if (!all_rows) HIPCHK(hipMemsetAsync(s->flags.p, 0, M, st));
        SlRows rows{s->rows_ts.as<int64_t>(), s->rows_rep.as<u32>(), s->rows_slot.as<u32>(), s->rows_send.as<int64_t>(),
                    s->rows_clock.as<int64_t>(), s->rows_vals.as<u64>(), s->rows_nulls.as<unsigned char>(), M};
        // the common shape (count / sum / avg / min / max of one double column, time window): records
        // sorted stably by key, one lane per key (k_sl_key); other shapes: key-partition replay
        if (keyed) {
            if (!presorted) {  // (presorted: sorted and key offsets made before the push's sync, sliding_push)
                HIPCHK(hipEventRecord(q->ev_agg0, st));  // the sort is part of the replay's time
                RCHK(sort_keyed(q, rec.slot, M));
            }
            RCHK(s->tmp.reserve((size_t)((s->nslots + 1 + kTile - 1) / kTile + 16) * 8, false));
            RCHK(s->p_pm.reserve(M * 8, false));
            RCHK(s->p_vals.reserve(M * 8, false));
            RCHK(s->rows_k.reserve((size_t)M * sliding_keyed_row_words(na, all_rows) * 8, false));
            RCHK(s->key_off.reserve((size_t)(s->nslots + 1) * 4, false));
            RCHK(s->tmp.reserve((size_t)((s->nslots + 1 + kTile - 1) / kTile + 16) * 8, false));
            if (presorted) HIPCHK(hipEventRecord(q->ev_agg0, st));  // (the sort's own time is added below)
            launch_sliding_keyed(st, s->slot_cnt.as<u32>(), s->key_off.as<u32>(), s->tmp.as<int64_t>(), s->ranks.as<u32>(),
                                 rec, s->p_pm.as<int64_t>(), s->p_vals.as<u64>(), state_of(s), q->ap,
                                 q->d.window_param, send_size, send_base, s->rows_k.as<u64>(),
                                 all_rows ? nullptr : s->flags.as<unsigned char>());
        } else {
            // stable split of the records by key partition
            int P = s->P;
            int mblk = (int)((M + kTile - 1) / kTile);
            int64_t ncnt = (int64_t)P * mblk;
            RCHK(s->counts.reserve((ncnt + 1) * 8, false));
            RCHK(s->tmp.reserve(((ncnt + kTile) / kTile + 16) * 8, false));
            RCHK(s->ranks.reserve(M * 4, false));
            RCHK(s->part_off.reserve((P + 1) * 8, false));
            launch_sl_multisplit(st, s->rec_slot.as<u32>(), M, P, s->counts.as<int64_t>(), s->tmp.as<int64_t>(),
                                 s->ranks.as<u32>(), s->part_off.as<int64_t>());
            // the records in partition order
            RCHK(s->p_raw.reserve(M * 4, false));
            RCHK(s->p_slot.reserve(M * 4, false));
            RCHK(s->p_clock.reserve(M * 8, false));
            RCHK(s->p_pm.reserve(M * 8, false));
            RCHK(s->p_ts.reserve(M * 8, false));
            RCHK(s->p_vals.reserve((size_t)V * M * 8, false));
            SlRecords prec{s->p_raw.as<u32>(), s->p_slot.as<u32>(), s->p_clock.as<int64_t>(), s->p_pm.as<int64_t>(),
                           s->p_ts.as<int64_t>(), s->p_vals.as<u64>(), M};
            // the double-column replay (k_sl_own_d) reads the records through the rank lists itself
            if (sliding_keys_per_partition(q->ap) == 64) launch_sl_gather(st, s->ranks.as<u32>(), M, rec, prec, q->ap.n_vcols);
            HIPCHK(hipEventRecord(q->ev_agg0, st));
            launch_sliding_own(st, s->ranks.as<u32>(), s->part_off.as<int64_t>(), P, s->logP, prec, state_of(s), q->ap,
                               q->d.window_param, send_size, send_base, rows, s->flags.as<unsigned char>(), rec);
        }
        HIPCHK(hipEventRecord(q->ev_agg1, st));
        HIPCHK(hipGetLastError());
        // emit in rank order
        int fblk = (int)((M + kTile - 1) / kTile);
        RCHK(s->blk_cnt.reserve((fblk + 16) * 8, false));
        if (all_rows) {
            n_rows = M;
        } else {
            launch_count_flags(st, s->flags.as<unsigned char>(), M, s->blk_cnt.as<int64_t>(), fblk);
            std::vector<int64_t> bc(fblk);
            HIPCHK(hipMemcpyAsync(bc.data(), s->blk_cnt.p, fblk * 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            for (auto c : bc) n_rows += c;
        }
        int nk = q->kp.n;
        int64_t cap = std::max<int64_t>(n_rows, 1);
        RCHK(s->out_ts.reserve(cap * 8, false));
        RCHK(s->out_keys.reserve(std::max(1, nk) * cap * 8, false));
        RCHK(s->out_vals.reserve((size_t)na * cap * 8, false));
        RCHK(s->out_nulls.reserve((size_t)na * cap, false));
        RCHK(s->out_send.reserve(cap * 8, false));
        RCHK(s->out_clock.reserve(cap * 8, false));
        RCHK(s->out_expired.reserve(cap, false));
        RCHK(s->out_rep.reserve(cap * 8, false));
        HIPCHK(hipMemsetAsync(s->out_expired.p, 0, cap, st));
        if (want_order) RCHK(q->out_order.reserve(cap * 8, false));
        if (!all_rows) launch_scan_sum(st, s->blk_cnt.as<int64_t>(), fblk);
        if (keyed)
            launch_slk_emit(st, all_rows ? nullptr : s->flags.as<unsigned char>(), M, s->blk_cnt.as<int64_t>(), fblk,
                            s->rows_k.as<u64>(), sliding_keyed_row_words(na, all_rows), na, q->kt.dev(), q->kp, cap,
                            s->out_ts.as<int64_t>(), s->out_keys.as<int64_t>(), s->out_vals.as<u64>(),
                            s->out_nulls.as<unsigned char>(), send_size == 1 ? nullptr : s->out_send.as<int64_t>(),
                            s->out_clock.as<int64_t>(),
                            s->rec_raw.as<u32>(), raw_base, want_order ? q->out_order.as<int64_t>() : nullptr,
                            s->out_rep.as<int64_t>(), rec.aos, rec.slot);
        else
        launch_sl_emit(st, s->flags.as<unsigned char>(), M, s->blk_cnt.as<int64_t>(), fblk, rows, na, q->kt.dev(),
                       q->kp, cap, s->out_ts.as<int64_t>(), s->out_keys.as<int64_t>(), s->out_vals.as<u64>(),
                       s->out_nulls.as<unsigned char>(), s->out_send.as<int64_t>(), s->out_clock.as<int64_t>(),
                       s->rec_raw.as<u32>(), raw_base, want_order ? q->out_order.as<int64_t>() : nullptr,
                       q->d.window == SH_WIN_EXT_TIME ? s->rec_sclk.as<int64_t>() : nullptr, s->out_rep.as<int64_t>());
        HIPCHK(hipGetLastError());
    }
    // flush structure: a flush per send that produced rows (one selector output chunk per send)
    int64_t n_flushes = 0;
    RCHK(sliding_flushes(q, n_rows, &n_flushes, send_size == 1));
    HIPCHK(hipEventRecord(q->ev_push1, st));
    HIPCHK(hipStreamSynchronize(st));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, q->ev_push0, q->ev_push1);
    q->stats.push_ms = ms;
    if (M > 0) {
        float ams = 0;
        (void)hipEventElapsedTime(&ams, q->ev_agg0, q->ev_agg1);
        if (presorted && q->srt_timed) {
            float sms = 0;
            (void)hipEventElapsedTime(&sms, q->ev_srt0, q->ev_srt1);
            ams += sms;
        }
        q->stats.main_kernel_ms = ams;
    }
    q->stats.main_kernel_bytes = M * (int64_t)(4 + 8 + 8 + 8 + 8 * q->ap.n_vcols) + n_rows * (int64_t)(8 + 8 * q->ap.n);
    return sliding_output(q, n_rows, n_flushes, want_order, host_out, out);
}

// flush offsets / clocks of n_rows output rows: a flush starts where out_send (the send, or the
// chunk in expired mode) changes; flush_off[n_flushes] = n_rows
int sliding_flushes(sh_query* q, int64_t n_rows, int64_t* n_flushes_out, bool per_row) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    s->fo = s->flush_off.as<int64_t>();
    s->fc = s->flush_clock.as<int64_t>();
    if (per_row) {
        // one row per send (per-event sends): every row is a flush of its own, so the offsets are the
        // identity (a persistent iota) and the clocks the rows' own
        if (s->iota_n < n_rows + 1) {
            const int64_t n = std::max<int64_t>(n_rows + 1, s->iota_n * 2);
            RCHK(s->iota.reserve((size_t)n * 8, false));
            launch_iota_i64(st, s->iota.as<int64_t>(), n);
            HIPCHK(hipGetLastError());
            s->iota_n = n;
        }
        s->fo = s->iota.as<int64_t>();
        s->fc = s->out_clock.as<int64_t>();
        *n_flushes_out = n_rows;
        return SH_OK;
    }
    int64_t n_flushes = 0;
    if (n_rows > 0) {
        int rb = (int)((n_rows + kTile - 1) / kTile);
        RCHK(s->blk_cnt.reserve((rb + 16) * 8, false));
        launch_flush_starts(st, s->out_send.as<int64_t>(), n_rows, s->blk_cnt.as<int64_t>(), rb);
        std::vector<int64_t> fc(rb);
        HIPCHK(hipMemcpyAsync(fc.data(), s->blk_cnt.p, rb * 8, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        for (auto c : fc) n_flushes += c;
        RCHK(s->flush_off.reserve((n_flushes + 1) * 8, false));
        RCHK(s->flush_clock.reserve((n_flushes + 1) * 8, false));
        launch_scan_sum(st, s->blk_cnt.as<int64_t>(), rb);
        launch_flush_write(st, s->out_send.as<int64_t>(), s->out_clock.as<int64_t>(), n_rows, s->blk_cnt.as<int64_t>(),
                           rb, s->flush_off.as<int64_t>(), s->flush_clock.as<int64_t>());
        RCHK(s->h_up.reserve(8));
        *s->h_up.as<int64_t>() = n_rows;
        HIPCHK(hipMemcpyAsync(s->flush_off.as<int64_t>() + n_flushes, s->h_up.p, 8, hipMemcpyHostToDevice, st));
        HIPCHK(hipGetLastError());
    }
    // (after the reserves above, which may have moved the buffers)
    s->fo = s->flush_off.as<int64_t>();
    s->fc = s->flush_clock.as<int64_t>();
    *n_flushes_out = n_flushes;
    return SH_OK;
}

// the push's rows (device arrays of stride n_rows) and flush arrays -> host vectors or the device view
int sliding_output(sh_query* q, int64_t n_rows, int64_t n_flushes, bool want_order, bool host_out,
                   const sh_out** out) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    int nk = s->nk_out >= 0 ? s->nk_out : q->kp.n, na = q->ap.n;
    if (host_out) {
        OutHost& o = q->out;
        o.reset();
        o.flush_offsets.resize(n_flushes + 1);
        o.flush_clock.resize(n_flushes);
        o.ts.resize(n_rows);
        o.expired.resize(n_rows);
        o.keys.resize((size_t)nk * n_rows);
        o.vals.resize((size_t)na * n_rows);
        o.nulls.resize((size_t)na * n_rows);
        o.rep.resize(n_rows);
        if (n_rows > 0) {
            HIPCHK(hipMemcpyAsync(o.flush_offsets.data(), s->fo, (n_flushes + 1) * 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(o.flush_clock.data(), s->fc, n_flushes * 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(o.ts.data(), s->out_ts.p, n_rows * 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(o.expired.data(), s->out_expired.p, n_rows, hipMemcpyDeviceToHost, st));
            // device arrays have stride cap == n_rows
            if (nk) HIPCHK(hipMemcpyAsync(o.keys.data(), s->out_keys.p, (size_t)nk * n_rows * 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(o.vals.data(), s->out_vals.p, (size_t)na * n_rows * 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(o.nulls.data(), s->out_nulls.p, (size_t)na * n_rows, hipMemcpyDeviceToHost, st));
            HIPCHK(hipMemcpyAsync(o.rep.data(), s->out_rep.p, n_rows * 8, hipMemcpyDeviceToHost, st));
            if (want_order) {
                q->order_host.resize(n_rows);
                HIPCHK(hipMemcpyAsync(q->order_host.data(), q->out_order.p, n_rows * 8, hipMemcpyDeviceToHost, st));
            }
            HIPCHK(hipStreamSynchronize(st));
        } else {
            q->order_host.clear();
            o.flush_offsets.assign(1, 0);
        }
        *out = o.view(nk, na, q->vtypes);
    } else {
        sh_out& o = s->dev_out;
        o = sh_out{};
        o.n_flushes = n_flushes;
        o.n_rows = n_rows;
        o.n_keys = nk;
        o.n_vals = na;
        for (int i = 0; i < na; i++) o.val_types[i] = q->vtypes[i];
        // the flush layout in host memory (the ABI's sh_push_device contract), or compact: one row per
        // flush at its row's timestamp (sh_query_set_compact_flushes) leaves both arrays NULL
        bool compact = false;
        if (q->compact_flushes && q->rate.kind == SH_RATE_NONE && n_flushes > 0 && n_flushes == n_rows) {
            RCHK(q->h_small_sc.reserve(64));
            launch_flush_clock_is_ts(st, n_flushes, s->fc, s->out_ts.as<int64_t>(), q->h_small_sc.as<uint32_t>() + 1);
            HIPCHK(hipGetLastError());
            HIPCHK(hipStreamSynchronize(st));
            compact = q->h_small_sc.as<uint32_t>()[1] == 1u;
        }
        if (compact) {
            o.flush_offsets = nullptr;
            o.flush_clock = nullptr;
        } else if (q->device_flushes && q->rate.kind == SH_RATE_NONE && !q->wide) {
            o.flush_offsets = const_cast<int64_t*>(s->fo);  // (sh_query_set_device_flushes)
            o.flush_clock = const_cast<int64_t*>(s->fc);
        } else {
            q->dev_flush_offsets.resize((size_t)n_flushes + 1);
            q->dev_flush_clock.resize((size_t)n_flushes);
            if (n_flushes > 0) {
                HIPCHK(hipMemcpyAsync(q->dev_flush_offsets.data(), s->fo, (n_flushes + 1) * 8, hipMemcpyDeviceToHost, st));
                HIPCHK(hipMemcpyAsync(q->dev_flush_clock.data(), s->fc, n_flushes * 8, hipMemcpyDeviceToHost, st));
                HIPCHK(hipStreamSynchronize(st));
            } else {
                q->dev_flush_offsets[0] = 0;
            }
            o.flush_offsets = q->dev_flush_offsets.data();
            o.flush_clock = q->dev_flush_clock.data();
        }
        o.ts = s->out_ts.as<int64_t>();
        o.expired = s->out_expired.as<uint8_t>();
        o.keys = s->out_keys.as<int64_t>();
        o.vals = s->out_vals.as<uint64_t>();
        o.nulls = s->out_nulls.as<uint8_t>();
        o.rep = s->out_rep.as<int64_t>();
        *out = &o;
    }
    return SH_OK;
}

// ---- `insert expired events` / `insert all events` (sh_slx_kernels.hip) -----------------------------
// One push (b) or one TIMER call (b == nullptr: the playback clock moves to `now`, sh_advance_time).
// The window's events form one expiry queue in arrival order (TimeWindowProcessor.java:132-169); every
// event's removal point and every operation's place in the push's operation sequence come from the
// monotone PM / clock sequences, then one lane per key replays its adds and removes in that order.
int read_count(sh_query* q, const int64_t* dev, int64_t* out) {
    SlidingImpl* s = q->sl;
    RCHK(s->x_h.reserve(64));
    HIPCHK(hipMemcpyAsync(s->x_h.p, dev, 8, hipMemcpyDeviceToHost, q->ctx->stream));
    HIPCHK(hipStreamSynchronize(q->ctx->stream));
    *out = *s->x_h.as<int64_t>();
    return SH_OK;
}

static int slx_run(sh_query* q, const sh_batch* b, int64_t now, bool host_out, const sh_out** out) {
    SlidingImpl* s = q->sl;
    hipStream_t st = q->ctx->stream;
    q->stats = sh_stats{};
    const bool ext = q->d.window == SH_WIN_EXT_TIME;
    const int64_t T = q->d.window_param;
    const int64_t N = b ? b->n : 0;
    const int64_t ss = b ? b->send_size : 0;
    const int V = std::max(1, q->ap.n_vcols);
    if (!b) {
        // TimestampGeneratorImpl.setCurrentTimestamp: the clock only moves forward, then onTimeChange
        if (q->clock_valid && now < q->clock) return empty_out(q, out);
        q->clock = now;
        q->clock_valid = true;
        if (s->n_np == 0) return empty_out(q, out);  // no notify time pending: no TIMER
    }
    if (N >= (int64_t)0x7FFFFFF0ll) return sh_fail(SH_ERR_INVALID, "push larger than 2G events");
    HIPCHK(hipEventRecord(q->ev_push0, st));
    ColSet cs{};
    cs.n = q->d.n_cols;
    WinParams wp{};
    int nblk = 0;
    int64_t M = 0;
    SlInfo info{};
    bool presorted = false;
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
    if (b) {
        for (int c = 0; c < q->d.n_cols; c++) { cs.type[c] = q->d.col_types[c]; cs.ptr[c] = b->cols[c]; }
        nblk = (int)((N + kTile - 1) / kTile);
        RCHK(s->blk_pass.reserve(nblk * 8, false));
        RCHK(s->blk_tl.reserve(nblk * 8, false));
        RCHK(s->blk_pm.reserve(nblk * 8, false));
        wp.kind = q->d.window;
        wp.ts_col = q->d.ts_col;
        wp.clock_valid = q->clock_valid;
        wp.clock0 = q->clock;
        wp.send_size = ss;
        wp.N = N;
        wp.rec_seq = q->tune.sl_records_seq;  // (lane-strided records where they apply)
        launch_sl_prefix(st, b->ts, cs, q->fp, wp, s->blk_pass.as<int64_t>(), s->blk_tl.as<int64_t>(),
                         s->blk_pm.as<int64_t>(), nblk, s->info.as<SlInfo>());
        if (ext) RCHK(s->rec_sclk.reserve(cap * 8, false));
        // (lane-strided records, every event passes: sorted by key slot right away, offsets and ring need
        // from the sorted slots instead of per-slot counts)
        presorted = q->ap.n > 0 && sl_records_seq_applies(q->fp, wp, q->ap);
        launch_sl_records(st, b->ts, cs, q->fp, wp, q->kp, q->kt.dev(), q->ap, s->blk_pass.as<int64_t>(),
                          s->blk_tl.as<int64_t>(), s->blk_pm.as<int64_t>(), s->pm, rec,
                          presorted ? nullptr : s->slot_cnt.as<u32>(), nblk, ext ? s->rec_sclk.as<int64_t>() : nullptr);
        HIPCHK(hipMemsetAsync((char*)s->info.p + offsetof(SlInfo, need), 0, 8, st));
        int64_t* need_dev = (int64_t*)((char*)s->info.p + offsetof(SlInfo, need));
        q->srt_timed = presorted;
        if (presorted) {
            HIPCHK(hipEventRecord(q->ev_srt0, st));
            RCHK(sort_keyed(q, rec.slot, N));
            HIPCHK(hipEventRecord(q->ev_srt1, st));
            launch_counts_sorted(st, s->p_slot.as<u32>(), N, s->slot_cnt.as<u32>());
        }
        launch_sl_need(st, s->slot_cnt.as<u32>(), s->rlen.as<int64_t>(), s->nslots, need_dev);
        HIPCHK(hipGetLastError());
        HIPCHK(hipMemcpyAsync(s->h_info, s->info.p, sizeof(SlInfo), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        RCHK(q->kt.check(st));
        info = *s->h_info;
        M = info.total_pass;
        if (info.need > s->rc) {
            int64_t nrc = s->rc;
            while (nrc < info.need) nrc <<= 1;
            RCHK(size_rings(q, nrc));
        }
    }
    // ---- the calls of the push (sends that set the clock) and which of them fire a TIMER chunk
    int64_t nC = 0, nF = 0, n_keep = 0;
    if (!ext) {
        if (b) {
            const int64_t NS = ss > 0 ? (N + ss - 1) / ss : 1;
            const int nbS = (int)((NS + kTile - 1) / kTile);
            RCHK(s->x_sK.reserve(NS * 8, false));
            RCHK(s->x_scb.reserve(NS * 8, false));
            RCHK(s->x_slast.reserve(NS * 8, false));
            RCHK(s->x_cK.reserve(NS * 8, false));
            RCHK(s->x_cC.reserve(NS * 8, false));
            RCHK(s->x_cS.reserve(NS * 8, false));
            RCHK(s->x_blk.reserve((size_t)(nbS + 2) * 8, false));
            launch_slx_sends(st, b->ts, cs, q->fp, wp, s->blk_pass.as<int64_t>(), s->blk_tl.as<int64_t>(), nblk,
                             s->x_sK.as<int64_t>(), s->x_scb.as<int64_t>(), s->x_slast.as<int64_t>());
            launch_slx_compact(st, 0, nullptr, s->x_sK.as<int64_t>(), s->x_scb.as<int64_t>(), s->x_slast.as<int64_t>(),
                               NS, s->x_blk.as<int64_t>(), s->x_cK.as<int64_t>(), s->x_cC.as<int64_t>(),
                               s->x_cS.as<int64_t>());
            HIPCHK(hipGetLastError());
            RCHK(read_count(q, s->x_blk.as<int64_t>() + nbS, &nC));
        } else {
            nC = 1;
            RCHK(s->x_cK.reserve(8, false));
            RCHK(s->x_cC.reserve(8, false));
            RCHK(s->x_cS.reserve(8, false));
            RCHK(s->x_h.reserve(64));
            int64_t* h = s->x_h.as<int64_t>();
            h[0] = 0; h[1] = now; h[2] = 0;
            HIPCHK(hipMemcpyAsync(s->x_cK.p, h, 8, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(s->x_cC.p, h + 1, 8, hipMemcpyHostToDevice, st));
            HIPCHK(hipMemcpyAsync(s->x_cS.p, h + 2, 8, hipMemcpyHostToDevice, st));
        }
        const int64_t n_cand = s->n_np + M;
        const int64_t n_big = std::max<int64_t>({nC, n_cand, 1});
        RCHK(s->x_fire.reserve(nC + 16, false));
        RCHK(s->x_keep.reserve(n_cand + 16, false));
        RCHK(s->x_idx.reserve(n_big * 8, false));
        RCHK(s->x_fK.reserve(std::max<int64_t>(nC, 1) * 8, false));
        RCHK(s->x_fC.reserve(std::max<int64_t>(nC, 1) * 8, false));
        RCHK(s->x_fS.reserve(std::max<int64_t>(nC, 1) * 8, false));
        RCHK(s->npend2.reserve(std::max<int64_t>(n_cand, 1) * 8, false));
        RCHK(s->x_blk.reserve((size_t)((n_big + kTile - 1) / kTile + 2) * 8, false));
        HIPCHK(hipMemsetAsync(s->x_fire.p, 0, nC + 16, st));
        launch_slx_notify(st, s->npend.as<int64_t>(), s->n_np, rec.pm, M, s->pm, s->x_cK.as<int64_t>(),
                          s->x_cC.as<int64_t>(), nC, T, s->x_fire.as<unsigned char>(), s->x_keep.as<unsigned char>());
        launch_slx_compact(st, 1, s->x_fire.as<unsigned char>(), nullptr, nullptr, nullptr, nC, s->x_blk.as<int64_t>(),
                           nullptr, nullptr, s->x_idx.as<int64_t>());
        HIPCHK(hipGetLastError());
        RCHK(read_count(q, s->x_blk.as<int64_t>() + (nC + kTile - 1) / kTile, &nF));
        launch_slx_gather_calls(st, s->x_idx.as<int64_t>(), nF, s->x_cK.as<int64_t>(), s->x_cC.as<int64_t>(),
                                s->x_cS.as<int64_t>(), s->x_fK.as<int64_t>(), s->x_fC.as<int64_t>(),
                                s->x_fS.as<int64_t>());
        launch_slx_compact(st, 1, s->x_keep.as<unsigned char>(), nullptr, nullptr, nullptr, n_cand,
                           s->x_blk.as<int64_t>(), nullptr, nullptr, s->x_idx.as<int64_t>());
        HIPCHK(hipGetLastError());
        RCHK(read_count(q, s->x_blk.as<int64_t>() + (n_cand + kTile - 1) / kTile, &n_keep));
        launch_slx_gather_pend(st, s->x_idx.as<int64_t>(), n_keep, s->npend.as<int64_t>(), s->n_np, rec.pm,
                               s->npend2.as<int64_t>());
        if (!b && nF == 0) {
            // no notify time due: the clock moved, nothing expired
            std::swap(s->npend, s->npend2);
            s->n_np = n_keep;
            return empty_out(q, out);
        }
    }
    // ---- the window FIFO gets the push's records; expiry points and operation indices
    const int64_t W0 = s->w0, n_u = W0 + M;
    s->upm.used = (size_t)W0 * 8;
    s->useq.used = (size_t)W0 * 8;
    RCHK(s->upm.reserve(std::max<int64_t>(n_u, 1) * 8, true));
    RCHK(s->useq.reserve(std::max<int64_t>(n_u, 1) * 8, true));
    launch_slx_append(st, rec.pm, rec.raw, M, q->seq, s->upm.as<int64_t>() + W0, s->useq.as<int64_t>() + W0);
    const int64_t nu1 = std::max<int64_t>(n_u, 1);
    const int na = q->ap.n;
    // the wave-per-key replay reads one record per add (xa) and per window position (xx) and writes one
    // record per row; the lane walk and pass-through use the columns
    const bool wave = na > 0 && q->tune.slx_wave && slx_keyed_ok(q->ap);
    if (wave) {
        RCHK(s->x_xa.reserve((size_t)cap * kXaWords * 8, false));
        RCHK(s->x_xx.reserve((size_t)nu1 * kXaWords * 8, false));
    } else {
        RCHK(s->x_xop.reserve(nu1 * 8, false));
        RCHK(s->x_xch.reserve(nu1 * 8, false));
        RCHK(s->x_xts.reserve(nu1 * 8, false));
        RCHK(s->x_xclk.reserve(nu1 * 8, false));
        RCHK(s->x_aop.reserve(cap * 8, false));
    }
    RCHK(s->x_nexp.reserve(8, false));
    RCHK(s->x_bnd.reserve((size_t)(3 * (nu1 / kBlock + 2) + cap / kBlock + 2) * 8, false));
    HIPCHK(hipMemsetAsync(s->x_nexp.p, 0, 8, st));
    const int64_t* rsclk = ext ? s->rec_sclk.as<int64_t>() : nullptr;
    launch_slx_expiry(st, s->upm.as<int64_t>(), n_u, W0, M, rec.clock, rsclk, rec.raw, ss, s->x_fK.as<int64_t>(),
                      s->x_fC.as<int64_t>(), s->x_fS.as<int64_t>(), nF, T, s->x_xop.as<u64>(), s->x_xch.as<int64_t>(),
                      s->x_xts.as<int64_t>(), s->x_xclk.as<int64_t>(), (unsigned long long*)s->x_nexp.p,
                      wave ? s->x_xx.as<u64>() : nullptr, s->useq.as<int64_t>(), rec.vals, s->x_bnd.as<int64_t>());
    launch_slx_aop(st, rec.clock, M, s->upm.as<int64_t>(), n_u, W0, T, s->x_aop.as<u64>(),
                   wave ? s->x_xa.as<u64>() : nullptr, rec, rsclk, s->x_bnd.as<int64_t>() + 3 * (nu1 / kBlock + 2));
    // the push's records sorted stably by key slot: each key's adds in arrival order
    if (!presorted) {
        RCHK(s->ranks.reserve(cap * 4, false));
        RCHK(s->p_slot.reserve(cap * 4, false));
        if (M > 0 && q->ap.n > 0) RCHK(sort_keyed(q, rec.slot, M));
    }
    RCHK(s->key_off.reserve((size_t)(s->nslots + 1) * 4, false));
    RCHK(s->tmp.reserve((size_t)((s->nslots + 1 + kTile - 1) / kTile + 16) * 8, false));
    launch_slx_keyoff(st, s->slot_cnt.as<u32>(), s->nslots, s->key_off.as<u32>(), s->tmp.as<int64_t>());
    HIPCHK(hipGetLastError());
    int64_t R = 0;
    RCHK(read_count(q, (const int64_t*)s->x_nexp.p, &R));
    // ---- the replay (one lane per key slot) writes one row per (chunk, key) at its operation index
    const int64_t n_ops = M + R;
    const int64_t oc = std::max<int64_t>(n_ops, 1);
    RCHK(s->flags.reserve(oc + 16, false));
    SlxRows rows{};
    rows.cap = oc;
    if (wave) {
        rows.rw = slx_row_words(na);
        RCHK(s->xr_aos.reserve((size_t)oc * rows.rw * 8, false));
        rows.aos = s->xr_aos.as<u64>();
    } else {
        RCHK(s->xr_ts.reserve(oc * 8, false));
        RCHK(s->xr_rep.reserve(oc * 8, false));
        RCHK(s->xr_slot.reserve(oc * 4, false));
        RCHK(s->xr_ch.reserve(oc * 8, false));
        RCHK(s->xr_clk.reserve(oc * 8, false));
        RCHK(s->xr_exp.reserve(oc, false));
        RCHK(s->xr_vals.reserve((size_t)std::max(na, 1) * oc * 8, false));
        RCHK(s->xr_nulls.reserve((size_t)std::max(na, 1) * oc, false));
        rows = SlxRows{s->xr_ts.as<int64_t>(), s->xr_rep.as<int64_t>(), s->xr_slot.as<u32>(), s->xr_ch.as<int64_t>(),
                       s->xr_clk.as<int64_t>(), s->xr_exp.as<unsigned char>(), s->xr_vals.as<u64>(),
                       s->xr_nulls.as<unsigned char>(), oc};
    }
    HIPCHK(hipMemsetAsync(s->flags.p, 0, oc + 16, st));
    HIPCHK(hipEventRecord(q->ev_agg0, st));
    if (q->ap.n == 0)
        launch_slx_pass(st, rec, M, s->x_aop.as<u64>(), s->x_xop.as<u64>(), s->x_xch.as<int64_t>(),
                        s->x_xts.as<int64_t>(), s->x_xclk.as<int64_t>(), s->useq.as<int64_t>(), n_u, q->seq, ss,
                        q->d.current_on, q->d.expired_on, rows, s->flags.as<unsigned char>(),
                        ext ? s->rec_sclk.as<int64_t>() : nullptr);
    else if (wave)
        launch_slx_wkey(st, s->key_off.as<u32>(), s->ranks.as<u32>(), s->nslots, s->x_xa.as<u64>(), s->x_xx.as<u64>(),
                        n_u, s->x0, s->g0, q->seq, ss, state_of(s), s->rg.as<int64_t>(), q->ap, q->d.current_on,
                        q->d.expired_on, rows, s->flags.as<unsigned char>());
    else
        launch_slx_walk(st, s->key_off.as<u32>(), s->ranks.as<u32>(), s->nslots, rec, s->x_aop.as<u64>(),
                        s->x_xop.as<u64>(), s->x_xch.as<int64_t>(), s->x_xts.as<int64_t>(), s->x_xclk.as<int64_t>(),
                        s->useq.as<int64_t>(), n_u, s->x0, s->g0, q->seq, ss, state_of(s), s->rg.as<int64_t>(), q->ap,
                        q->d.current_on, q->d.expired_on, rows, s->flags.as<unsigned char>(), rsclk);
    HIPCHK(hipEventRecord(q->ev_agg1, st));
    HIPCHK(hipGetLastError());
    // ---- rows in operation order, one flush per chunk
    int64_t n_rows = 0;
    const int fblk = (int)((n_ops + kTile - 1) / kTile);
    if (n_ops > 0) {
        RCHK(s->blk_cnt.reserve((size_t)(fblk + 16) * 8, false));
        launch_count_flags(st, s->flags.as<unsigned char>(), n_ops, s->blk_cnt.as<int64_t>(), fblk);
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
        if (n_rows > 0)
            (wave ? launch_slx_emit_aos : launch_slx_emit)(st, s->flags.as<unsigned char>(), n_ops, s->blk_cnt.as<int64_t>(), fblk, rows, na,
                            q->kt.dev(), q->kp, rcap, s->out_ts.as<int64_t>(), s->out_keys.as<int64_t>(),
                            s->out_vals.as<u64>(), s->out_nulls.as<unsigned char>(), s->out_expired.as<unsigned char>(),
                            s->out_send.as<int64_t>(), s->out_clock.as<int64_t>(), s->out_rep.as<int64_t>());
        HIPCHK(hipGetLastError());
    }
    int64_t n_flushes = 0;
    RCHK(sliding_flushes(q, n_rows, &n_flushes));
    // ---- the state moves on: unexpired FIFO tail, pending notify times, counters, clock
    const int64_t new_w = n_u - R;
    RCHK(s->upm2.reserve(std::max<int64_t>(new_w, 1) * 8, false));
    RCHK(s->useq2.reserve(std::max<int64_t>(new_w, 1) * 8, false));
    launch_slx_shift(st, s->upm.as<int64_t>(), s->useq.as<int64_t>(), R, new_w, s->upm2.as<int64_t>(),
                     s->useq2.as<int64_t>());
    HIPCHK(hipGetLastError());
    std::swap(s->upm, s->upm2);
    std::swap(s->useq, s->useq2);
    if (!ext) {
        std::swap(s->npend, s->npend2);
        s->n_np = n_keep;
    }
    s->x0 += R;
    s->g0 += M;
    s->w0 = new_w;
    if (b) {
        q->seq += N;
        q->clock = q->clock_valid ? std::max(q->clock, info.max_tl) : info.max_tl;
        q->clock_valid = true;
        s->pm = std::max(s->pm, info.max_pm);
        s->send_base += ss > 0 ? (N + ss - 1) / ss : 1;
        q->stats.events = N;
    }
    HIPCHK(hipEventRecord(q->ev_push1, st));
    HIPCHK(hipStreamSynchronize(st));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, q->ev_push0, q->ev_push1);
    q->stats.push_ms = ms;
    q->stats.main_kernel_bytes = n_ops * (int64_t)(16 + 8 * V) + n_rows * (int64_t)(8 + 8 * na);
    return sliding_output(q, n_rows, n_flushes, false, host_out, out);
}

int sliding_advance(sh_query* q, int64_t now, const sh_out** out, bool host_out) {
    if (q->sl->lane) return plane_advance(q, now, out, host_out);
    // expired output: the TIMER chunk's expired events (Scheduler.onTimeChange -> the window)
    if (q->sl->xm && q->d.window == SH_WIN_TIME) return slx_run(q, nullptr, now, host_out, out);
    // expiry is applied lazily at each key's next event; with current-events-only output the
    // timer path changes no visible result, only the clock (TimestampGeneratorImpl :104-122)
    if (!q->clock_valid || now >= q->clock) {
        q->clock = now;
        q->clock_valid = true;
    }
    return empty_out(q, out);
}

// Persistent buffers of the sliding state and their byte sizes, for sh_query_snapshot/restore
// (sh_snapshot.cpp). scalars = {nslots, rc, pm, send_base}; with set = true the ring capacity is
// first made `new_rc` and the scalars are taken from the snapshot.
int sliding_state_buffers(sh_query* q, std::vector<std::pair<DevBuf*, size_t>>& bufs, int64_t* sc, int n_sc, bool set,
                          int64_t new_rc) {
    SlidingImpl* s = q->sl;
    if (n_sc != 4) return sh_fail(SH_ERR_INVALID, "sliding snapshot layout");
    if (set) {
        if (sc[0] != s->nslots) return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
        if (new_rc <= 0 || (new_rc & (new_rc - 1))) return sh_fail(SH_ERR_INVALID, "snapshot ring capacity");
        if (new_rc != s->rc) RCHK(size_rings(q, new_rc, false));
        s->pm = sc[2];
        s->send_base = sc[3];
    } else {
        sc[0] = s->nslots; sc[1] = s->rc; sc[2] = s->pm; sc[3] = s->send_base;
    }
    const size_t n = (size_t)s->nslots, rc = (size_t)s->rc;
    const size_t F = (size_t)std::max(1, q->ap.n_fields), V = (size_t)ring_vcols(q);
    bufs = {{&s->cnt, n * 8},          {&s->f, F * n * 8},         {&s->mm, F * n * 8},      {&s->mm_has, F * n},
            {&s->dq_head, F * n * 8},  {&s->dq_len, F * n * 8},    {&s->dq, F * n * rc * 8}, {&s->rhead, n * 8},
            {&s->rlen, n * 8},         {&s->rpm, n * rc * 8},      {&s->rval, V * n * rc * 8},
            {&s->cur_send, n * 8},     {&s->cur_first, n * 8}};
    return SH_OK;
}

// Checkpoint of the expiry FIFO of `insert expired / all events` and pass-through sliding windows
// (sh_slx_kernels.hip): arrival indices X0 / G0, the unexpired FIFO (PM, stream index), the pending
// notify times and each ring entry's arrival index. sc = {x0, g0, w0, n_np, np_front}. The partition
// lanes (sh_plane.cpp) keep host-side scheduler state and are not checkpointed (lane != 0).
int sliding_fifo_state(sh_query* q, std::vector<std::pair<DevBuf*, size_t>>& bufs, int64_t* sc, bool set, int* kind) {
    SlidingImpl* s = q->sl;
    *kind = s->lane ? 2 : s->xm ? 1 : 0;
    bufs.clear();
    if (*kind != 1) return SH_OK;
    if (set) {
        if (sc[2] < 0 || sc[3] < 0) return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
        s->x0 = sc[0]; s->g0 = sc[1]; s->w0 = sc[2]; s->n_np = sc[3]; s->np_front = sc[4];
    } else {
        sc[0] = s->x0; sc[1] = s->g0; sc[2] = s->w0; sc[3] = s->n_np; sc[4] = s->np_front;
    }
    const size_t n = (size_t)s->nslots, rc = (size_t)s->rc;
    bufs = {{&s->rg, n * rc * 8}, {&s->upm, (size_t)s->w0 * 8}, {&s->useq, (size_t)s->w0 * 8},
            {&s->npend, (size_t)s->n_np * 8}};
    return SH_OK;
}
