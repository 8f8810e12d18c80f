// sh_snapshot.cpp — checkpoint of a query's device state behind sh_query_snapshot / sh_query_restore.
//
// Replaces State.snapshot()/restore() (core/util/snapshot/state/State.java:26-36) as driven by
// SnapshotService.persist/restore (core/util/snapshot/SnapshotService.java:90-296) for the states
// this path owns: the batch windows' queued events and count (LengthBatchWindowProcessor
// WindowState :302-350, TimeBatchWindowProcessor WindowState :376-418), the sliding window's
// queue and every key's aggregator state (TimeWindowProcessor :196-222, the Sum/Avg/Count/Min/Max
// State classes incl. the min/max deques), and the partition the window belongs to. The playback
// clock and nextEmitTime travel with them, so a restored query continues exactly where the
// snapshot was taken.
//
// Blob: "SHQ1" | u32 version | u64 descriptor fingerprint | u32 kind | sections (host scalars and
// device buffers copied through the host, in a fixed order).
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>
#include <vector>

#include "sh_internal.h"
#include "sh_runtime.h"
#include "sh_wide.h"

using namespace shd;

#define RCHK(x)            \
    do {                   \
        int _r = (x);      \
        if (_r) return _r; \
    } while (0)

namespace {

constexpr uint32_t kVersion = 7;  // 5: band key mode, sharded aggregation sections; 6: timeout / limiter in the fingerprint; 7: replaceTimestampWithBatchEndTime

struct Writer {
    std::vector<uint8_t> b;
    void put(const void* p, size_t n) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n); }
    template <typename T> void val(const T& x) { put(&x, sizeof(T)); }
    int dev(const void* d, size_t n, hipStream_t s) {
        val<uint64_t>(n);
        size_t o = b.size();
        b.resize(o + n);
        if (n && (hipMemcpyAsync(b.data() + o, d, n, hipMemcpyDeviceToHost, s) != hipSuccess ||
                  hipStreamSynchronize(s) != hipSuccess))
            return sh_fail(SH_ERR_DEVICE, "snapshot: device read failed");
        return SH_OK;
    }
};

struct Reader {
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
    // device section into `buf` (grown to at least `min_cap` bytes)
    int dev(DevBuf& buf, size_t min_cap, hipStream_t s) {
        uint64_t len = val<uint64_t>();
        if (!ok || o + len > n) { ok = false; return sh_fail(SH_ERR_INVALID, "snapshot blob truncated"); }
        RCHK(buf.reserve(std::max<size_t>({len, min_cap, 8}), false));
        if (len && (hipMemcpyAsync(buf.p, p + o, len, hipMemcpyHostToDevice, s) != hipSuccess ||
                    hipStreamSynchronize(s) != hipSuccess))
            return sh_fail(SH_ERR_DEVICE, "restore: device write failed");
        o += len;
        return SH_OK;
    }
};

uint64_t fnv(uint64_t h, const void* p, size_t n) {
    const uint8_t* c = (const uint8_t*)p;
    for (size_t i = 0; i < n; i++) h = (h ^ c[i]) * 1099511628211ull;
    return h;
}

// the query's semantics: a blob only restores into a query built from the same descriptor
uint64_t fingerprint(const sh_query* q) {
    const sh_query_desc& d = q->d;
    uint64_t h = 1469598103934665603ull;
    int32_t ints[] = {d.n_cols, d.window, d.stream_current, d.has_start_time, d.n_group_by, d.n_aggs, d.current_on,
                      d.expired_on, d.partition_col, d.ts_col, d.start_col};
    h = fnv(h, ints, sizeof(ints));
    h = fnv(h, d.col_types, sizeof(int32_t) * d.n_cols);
    h = fnv(h, &d.window_param, 8);
    h = fnv(h, &d.start_time, 8);
    h = fnv(h, d.group_by, sizeof(int32_t) * d.n_group_by);
    h = fnv(h, d.aggs, sizeof(sh_agg_spec) * d.n_aggs);
    // set after creation but part of the blob's layout: the externalTimeBatch timeout (its scheduler
    // section) and the output rate limiter's kind / per-partition form (their sections)
    const int64_t extra[] = {q->xt_timeout, q->rate.kind, q->rate.N, q->rate.part, q->rate.pkey, q->rate.lkey,
                             q->xt_replace};
    h = fnv(h, extra, sizeof(extra));
    h = fnv(h, &q->fp_orig.n, sizeof(int));
    for (int i = 0; i < q->fp_orig.n; i++) {
        const FilterOpD& o = q->fp_orig.ops[i];
        int32_t oi[] = {o.op, o.type, o.col};
        h = fnv(h, oi, sizeof(oi));
        h = fnv(h, &o.ival, 8);
        h = fnv(h, &o.dval, 8);
    }
    return h;
}

// the key table's insert counter after a restore (stream-ordered, from pinned memory)
int set_key_count(sh_query* q, int64_t nk) {
    PinnedBuf h;
    RCHK(h.reserve(16));
    uint32_t* c = h.as<uint32_t>();
    c[0] = (uint32_t)nk; c[1] = c[2] = c[3] = 0;
    if (hipMemcpyAsync(q->kt.ctrl.p, c, 16, hipMemcpyHostToDevice, q->ctx->stream) != hipSuccess ||
        hipStreamSynchronize(q->ctx->stream) != hipSuccess)
        return sh_fail(SH_ERR_DEVICE, "restore: key table counter");
    return SH_OK;
}

}  // namespace

// ---- per-kind sections (batch windows: sh_window.cpp; sliding: sh_sliding.cpp) -----------------
int batch_snapshot(sh_query* q, Writer& w);
int batch_restore(sh_query* q, Reader& r);
int sliding_snapshot(sh_query* q, Writer& w);
int sliding_restore(sh_query* q, Reader& r);

int batch_snapshot(sh_query* q, Writer& w) {
    hipStream_t s = q->ctx->stream;
    w.val<uint8_t>(q->clock_valid);
    w.val<int64_t>(q->clock);
    w.val<uint8_t>(q->e0_valid);
    w.val<int64_t>(q->E0);
    w.val<int64_t>(q->W_open);
    w.val<int64_t>(q->xm);
    w.val<uint8_t>(q->p0_known);
    w.val<int64_t>(q->p0);
    // group-key table: the queued events refer to its slots
    // key mode: 0 open addressing, 1 dictionary ids, 2 band (an aggregation root's (bucket, id) rows)
    w.val<uint8_t>(q->kt.lk ? 2 : q->kt.dense ? 1 : 0);
    w.val<uint64_t>(q->kt.size_);
    if (q->kt.lk) {
        w.val<uint32_t>(q->kt.lk);
        w.val<uint32_t>(q->kt.rows);
        w.val<int64_t>(q->kt.band_base);
    }
    RCHK(q->kt.check(s));
    w.val<int64_t>(q->kt.n_keys);
    RCHK(w.dev(q->kt.keys.p, q->kt.dense ? 0 : q->kt.size_ * 8, s));
    // the open window's queued events (currentEventQueue / count)
    const int64_t n = q->n_pend;
    w.val<int64_t>(n);
    RCHK(w.dev(q->pend_pos.p, n * 4, s));
    RCHK(w.dev(q->pend_ts.p, n * 8, s));
    w.val<int32_t>(q->ap.n_vcols);
    for (int j = 0; j < q->ap.n_vcols; j++) RCHK(w.dev(q->pend_vals.as<char>() + (size_t)j * q->pend_cap * 8, n * 8, s));
    // stream numbering (sh_out.rep): the queued events' indices and the next event's
    RCHK(w.dev(q->pend_gidx.p, n * 8, s));
    // expired / all-events output: the last flushed batch's keys and representative events, carried
    // until the batch after it closes (sh_expired.cpp)
    w.val<uint8_t>(q->xmode);
    if (q->xmode) {
        const int64_t xn = q->xc_valid ? q->xc_n : 0;
        w.val<uint8_t>(q->xc_valid);
        w.val<int64_t>(xn);
        w.val<int64_t>(q->xc_W);
        RCHK(w.dev(q->xc_keys.p, (size_t)q->kp.n * xn * 8, s));
        RCHK(w.dev(q->xc_rep.p, (size_t)xn * 8, s));
        if (q->given) RCHK(w.dev(q->xc_order.p, (size_t)xn * 8, s));  // (a sharded owner's rows' global order)
    }
    w.val<int64_t>(q->seq);
    // externalTimeBatch timeout: lastScheduledTime and the open batch's events not yet sent
    if (q->xt_timeout > 0) {
        w.val<uint8_t>(q->xt_Lvalid);
        w.val<int64_t>(q->xt_L);
        w.val<int64_t>(q->xt_nnew);
    }
    // replaceTimestampWithBatchEndTime: the last windows' first events (the batch of a later row's
    // representative event)
    if (q->xt_replace) {
        w.val<uint64_t>(q->xr_starts.size());
        for (auto& e : q->xr_starts) { w.val<int64_t>(e.first); w.val<int64_t>(e.second); }
    }
    return SH_OK;
}

int query_resize_for_restore(sh_query* q, size_t table_size, int64_t n_pend, const KeyBand* band);
int query_set_partition(sh_query* q, int64_t p0);

int batch_restore(sh_query* q, Reader& r) {
    hipStream_t s = q->ctx->stream;
    q->clock_valid = r.val<uint8_t>();
    q->clock = r.val<int64_t>();
    q->e0_valid = r.val<uint8_t>();
    q->E0 = r.val<int64_t>();
    q->W_open = r.val<int64_t>();
    q->xm = r.val<int64_t>();
    bool p0k = r.val<uint8_t>();
    int64_t p0 = r.val<int64_t>();
    const int mode = r.val<uint8_t>();
    uint64_t size = r.val<uint64_t>();
    KeyBand band{};
    if (mode == 2) {
        band.lk = r.val<uint32_t>();
        band.rows = r.val<uint32_t>();
        band.base = r.val<int64_t>();
    }
    int64_t nk = r.val<int64_t>();
    // a band-keyed root may be in either of its modes; any other query in the one it was created with
    const bool fits = q->band_keys ? (mode == 0 || (mode == 2 && band.lk == q->band_lk && band.rows == q->band_rows))
                                   : mode == (q->kt.dense ? 1 : 0);
    if (!r.ok || !fits) return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
    const bool dense = mode != 0;
    // table of the snapshot's size, then its keys
    int64_t n_pend_peek;
    {
        Reader t = r;
        uint64_t klen = t.val<uint64_t>();
        t.o += klen;
        n_pend_peek = t.val<int64_t>();
        if (!t.ok || n_pend_peek < 0) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    }
    RCHK(query_resize_for_restore(q, size, n_pend_peek, mode == 2 ? &band : nullptr));
    RCHK(r.dev(q->kt.keys, dense ? 8 : size * 8, s));
    RCHK(set_key_count(q, nk));
    q->kt.n_keys = nk;
    const int64_t n = r.val<int64_t>();
    q->n_pend = n;
    // pending buffers were sized by query_resize_for_restore; copy the sections into them
    DevBuf tmp;
    RCHK(r.dev(tmp, 8, s));
    if (n && hipMemcpyAsync(q->pend_pos.p, tmp.p, n * 4, hipMemcpyDeviceToDevice, s) != hipSuccess) return sh_fail(SH_ERR_DEVICE, "restore");
    RCHK(r.dev(tmp, 8, s));
    if (n && hipMemcpyAsync(q->pend_ts.p, tmp.p, n * 8, hipMemcpyDeviceToDevice, s) != hipSuccess) return sh_fail(SH_ERR_DEVICE, "restore");
    int32_t nv = r.val<int32_t>();
    if (nv != q->ap.n_vcols) { tmp.release(); return sh_fail(SH_ERR_INVALID, "snapshot does not match this query"); }
    for (int j = 0; j < nv; j++) {
        RCHK(r.dev(tmp, 8, s));
        if (n && (hipMemcpyAsync(q->pend_vals.as<char>() + (size_t)j * q->pend_cap * 8, tmp.p, n * 8,
                                 hipMemcpyDeviceToDevice, s) != hipSuccess ||
                  hipStreamSynchronize(s) != hipSuccess))
            return sh_fail(SH_ERR_DEVICE, "restore");
    }
    RCHK(r.dev(tmp, 8, s));
    if (n && (hipMemcpyAsync(q->pend_gidx.p, tmp.p, n * 8, hipMemcpyDeviceToDevice, s) != hipSuccess ||
              hipStreamSynchronize(s) != hipSuccess))
        return sh_fail(SH_ERR_DEVICE, "restore");
    if ((bool)r.val<uint8_t>() != q->xmode || !r.ok) return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
    if (q->xmode) {
        q->xc_valid = r.val<uint8_t>();
        q->xc_n = r.val<int64_t>();
        q->xc_W = r.val<int64_t>();
        if (!r.ok || q->xc_n < 0) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        RCHK(r.dev(q->xc_keys, 8, s));
        RCHK(r.dev(q->xc_rep, 8, s));
        if (q->given) RCHK(r.dev(q->xc_order, 8, s));
    }
    q->seq = r.val<int64_t>();
    if (q->xt_timeout > 0) {
        q->xt_Lvalid = r.val<uint8_t>();
        q->xt_L = r.val<int64_t>();
        q->xt_nnew = r.val<int64_t>();
    }
    if (q->xt_replace) {
        const uint64_t ns = r.val<uint64_t>();
        if (!r.ok || ns > (r.n - r.o) / 16) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        q->xr_starts.clear();
        for (uint64_t i = 0; i < ns; i++) {
            const int64_t a = r.val<int64_t>(), b = r.val<int64_t>();
            q->xr_starts.emplace_back(a, b);
        }
    }
    tmp.release();
    if (!r.ok) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    q->p0_known = false;
    if (p0k) RCHK(query_set_partition(q, p0));
    return SH_OK;
}

int query_out_keys(sh_query* q);

// Output rate limiter (sh_rate.cpp; the reference limiters' State: counters, the carried rows of an
// open group, the FirstGroupBy key -> count table, `first every <t>`'s output time / key table)
static int rate_snapshot(sh_query* q, Writer& w) {
    auto& r = q->rate;
    hipStream_t s = q->ctx->stream;
    const int nk = query_out_keys(q), na = q->ap.n;
    w.val<int32_t>(r.kind);
    w.val<int64_t>(r.N);
    if (r.kind == SH_RATE_NONE) return SH_OK;
    w.val<int64_t>(r.seq);
    w.val<int64_t>(r.nc);
    const size_t n = (size_t)r.nc;
    RCHK(w.dev(r.c_ts.p, n * 8, s));
    RCHK(w.dev(r.c_exp.p, n, s));
    RCHK(w.dev(r.c_rep.p, n * 8, s));
    RCHK(w.dev(r.c_keys.p, (size_t)nk * n * 8, s));
    RCHK(w.dev(r.c_vals.p, (size_t)na * n * 8, s));
    RCHK(w.dev(r.c_nulls.p, (size_t)na * n, s));
    w.val<int64_t>(r.t_cap);
    w.val<int64_t>(r.t_keys);
    RCHK(w.dev(r.tk.p, (size_t)r.t_cap * 8, s));
    RCHK(w.dev(r.tc.p, (size_t)r.t_cap * 8, s));
    w.val<uint8_t>(r.ft_has);
    w.val<int64_t>(r.ft_last);
    w.val<int64_t>(r.ft_cap);
    w.val<int64_t>(r.ft_keys);
    RCHK(w.dev(r.ftk.p, (size_t)r.ft_cap * 8, s));
    RCHK(w.dev(r.ftt.p, (size_t)r.ft_cap * 8, s));
    if (r.part) {  // one limiter per partition: the carried rows' partitions and every partition's state
        const size_t np = (size_t)r.nparts;
        RCHK(w.dev(r.c_part.p, n * 4, s));
        RCHK(w.dev(r.pseq.p, np * 8, s));
        RCHK(w.dev(r.pft_has.p, np, s));
        RCHK(w.dev(r.pft_last.p, np * 8, s));
    }
    return SH_OK;
}

static int rate_restore(sh_query* q, Reader& rd) {
    auto& r = q->rate;
    hipStream_t s = q->ctx->stream;
    const int32_t kind = rd.val<int32_t>();
    const int64_t N = rd.val<int64_t>();
    if (!rd.ok) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    if (kind != r.kind || N != r.N)
        return sh_fail(SH_ERR_INVALID, "snapshot's output rate limiting differs from this query's (set it before restoring)");
    if (kind == SH_RATE_NONE) return SH_OK;
    r.seq = rd.val<int64_t>();
    r.nc = rd.val<int64_t>();
    if (!rd.ok || r.nc < 0) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    for (DevBuf* b : {&r.c_ts, &r.c_exp, &r.c_rep, &r.c_keys, &r.c_vals, &r.c_nulls}) RCHK(rd.dev(*b, 8, s));
    r.t_cap = rd.val<int64_t>();
    r.t_keys = rd.val<int64_t>();
    RCHK(rd.dev(r.tk, 8, s));
    RCHK(rd.dev(r.tc, 8, s));
    r.ft_has = rd.val<uint8_t>();
    r.ft_last = rd.val<int64_t>();
    r.ft_cap = rd.val<int64_t>();
    r.ft_keys = rd.val<int64_t>();
    RCHK(rd.dev(r.ftk, 8, s));
    RCHK(rd.dev(r.ftt, 8, s));
    if (r.part) {
        RCHK(rd.dev(r.c_part, 8, s));
        RCHK(rd.dev(r.pseq, 8, s));
        RCHK(rd.dev(r.pft_has, 8, s));
        RCHK(rd.dev(r.pft_last, 8, s));
    }
    if (!rd.ok) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    return SH_OK;
}

static int query_snapshot_blob(sh_query* q, Writer& w) {
    if (q->given) return sh_fail(SH_ERR_UNSUPPORTED, "snapshot of a sharded owner: snapshot the sh_shard instead");
    RCHK(query_drain_async(q));
    w.put("SHQ1", 4);
    w.val<uint32_t>(kVersion);
    w.val<uint64_t>(fingerprint(q));
    w.val<uint32_t>((uint32_t)q->kind);
    RCHK(q->kind == 1 ? sliding_snapshot(q, w) : batch_snapshot(q, w));
    RCHK(rate_snapshot(q, w));
    if (q->wide) {  // the interned group keys (the window's key ids)
        std::vector<uint8_t> kb;
        RCHK(q->wide->save(kb, q->ctx->stream));
        w.val<uint64_t>(kb.size());
        w.put(kb.data(), kb.size());
    }
    return SH_OK;
}

extern "C" int sh_query_snapshot(sh_query* q, void* buf, int64_t cap, int64_t* len) {
    SH_RANGE("sh_query_snapshot");
    StreamScope _ss(q && q->ctx ? q->ctx->stream : nullptr);
    if (!q || !len) return sh_fail(SH_ERR_INVALID, "sh_query_snapshot: NULL argument");
    Writer w;
    RCHK(query_snapshot_blob(q, w));
    *len = (int64_t)w.b.size();
    if (buf) {
        if (cap < *len) return sh_fail(SH_ERR_INVALID, "sh_query_snapshot: buffer too small (call with buf=NULL for the size)");
        std::memcpy(buf, w.b.data(), w.b.size());
    }
    return SH_OK;
}

static int query_restore_blob(sh_query* q, const void* buf, int64_t len) {
    if (q->given) return sh_fail(SH_ERR_UNSUPPORTED, "restore of a sharded owner: restore the sh_shard instead");
    Reader r{(const uint8_t*)buf, (size_t)len};
    if (std::memcmp(buf, "SHQ1", 4) != 0) return sh_fail(SH_ERR_INVALID, "not a siddhi_hip query snapshot");
    r.o = 4;
    if (r.val<uint32_t>() != kVersion) return sh_fail(SH_ERR_INVALID, "snapshot version mismatch");
    if (r.val<uint64_t>() != fingerprint(q)) return sh_fail(SH_ERR_INVALID, "snapshot was taken from a different query");
    if (r.val<uint32_t>() != (uint32_t)q->kind) return sh_fail(SH_ERR_INVALID, "snapshot kind mismatch");
    RCHK(query_drain_async(q));  // a queued report must not land on the restored counters
    (void)hipStreamSynchronize(q->ctx->stream);
    RCHK(q->kind == 1 ? sliding_restore(q, r) : batch_restore(q, r));
    RCHK(rate_restore(q, r));
    if (q->wide) {
        const uint64_t kn = r.val<uint64_t>();
        if (!r.ok || r.o + kn > r.n) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        size_t off = 0;
        RCHK(q->wide->load(r.p + r.o, (size_t)kn, off, q->ctx->stream));
        r.o += kn;
    }
    return SH_OK;
}

// A restore either applies the whole blob or leaves the query as it was: the current state is
// snapshotted first and put back when the blob fails part-way (truncated, wrong sections, device
// error), keeping the first failure's message.
template <class Snap, class Rest>
static int restore_or_roll_back(Snap snap, Rest rest, const void* buf, int64_t len) {
    Writer backup;
    const bool have = snap(backup) == SH_OK;
    const int rc = rest(buf, len);
    if (rc != SH_OK && have) {
        const std::string msg = sh_last_error();
        (void)rest(backup.b.data(), (int64_t)backup.b.size());
        return sh_fail(rc, msg);
    }
    return rc;
}

extern "C" int sh_query_restore(sh_query* q, const void* buf, int64_t len) {
    SH_RANGE("sh_query_restore");
    StreamScope _ss(q && q->ctx ? q->ctx->stream : nullptr);
    if (!q || !buf || len < 20) return sh_fail(SH_ERR_INVALID, "sh_query_restore: bad arguments");
    return restore_or_roll_back([&](Writer& w) { return query_snapshot_blob(q, w); },
                                [&](const void* b, int64_t n) { return query_restore_blob(q, b, n); }, buf, len);
}

// ---- sliding window (state in SlidingImpl, sh_sliding.cpp) ---------------------------------------
struct SlidingImpl;
int sliding_state_buffers(sh_query* q, std::vector<std::pair<DevBuf*, size_t>>& bufs, int64_t* scalars, int n_scalars,
                          bool set, int64_t new_rc);
int sliding_fifo_state(sh_query* q, std::vector<std::pair<DevBuf*, size_t>>& bufs, int64_t* sc, bool set, int* kind);
void plane_state_buffers(sh_query* q, std::vector<std::pair<DevBuf*, size_t>>& bufs);
int plane_host_save(sh_query* q, std::vector<uint8_t>& out);
int plane_host_load(sh_query* q, const uint8_t* p, size_t n, size_t* used);

int sliding_snapshot(sh_query* q, Writer& w) {
    hipStream_t s = q->ctx->stream;
    w.val<uint8_t>(q->clock_valid);
    w.val<int64_t>(q->clock);
    w.val<uint64_t>(q->kt.size_);
    RCHK(q->kt.check(s));
    w.val<int64_t>(q->kt.n_keys);
    RCHK(w.dev(q->kt.keys.p, q->kt.dense ? 0 : q->kt.size_ * 8, s));
    int64_t sc[4];
    std::vector<std::pair<DevBuf*, size_t>> bufs;
    RCHK(sliding_state_buffers(q, bufs, sc, 4, false, 0));
    for (int i = 0; i < 4; i++) w.val<int64_t>(sc[i]);
    for (auto& b : bufs) RCHK(w.dev(b.first->p, b.second, s));
    // the expiry FIFO of expired / all-events output and pass-through windows
    int64_t fs[5] = {0, 0, 0, 0, 0};
    int fk = 0;
    RCHK(sliding_fifo_state(q, bufs, fs, false, &fk));
    w.val<int32_t>(fk);
    if (fk == 1) {
        for (int i = 0; i < 5; i++) w.val<int64_t>(fs[i]);
        for (auto& b : bufs) RCHK(w.dev(b.first->p, b.second, s));
    } else if (fk == 2) {
        // the partition lanes: their per-slot device state and the host-side Scheduler
        plane_state_buffers(q, bufs);
        for (auto& b : bufs) RCHK(w.dev(b.first->p, b.second, s));
        std::vector<uint8_t> hs;
        RCHK(plane_host_save(q, hs));
        w.val<uint64_t>(hs.size());
        w.put(hs.data(), hs.size());
    }
    w.val<int64_t>(q->seq);
    return SH_OK;
}

int sliding_restore(sh_query* q, Reader& r) {
    hipStream_t s = q->ctx->stream;
    q->clock_valid = r.val<uint8_t>();
    q->clock = r.val<int64_t>();
    uint64_t size = r.val<uint64_t>();
    int64_t nk = r.val<int64_t>();
    if (!r.ok || size != q->kt.size_) return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
    RCHK(r.dev(q->kt.keys, q->kt.dense ? 8 : size * 8, s));
    RCHK(set_key_count(q, nk));
    q->kt.n_keys = nk;
    int64_t sc[4];
    for (int i = 0; i < 4; i++) sc[i] = r.val<int64_t>();
    if (!r.ok) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    std::vector<std::pair<DevBuf*, size_t>> bufs;
    RCHK(sliding_state_buffers(q, bufs, sc, 4, true, sc[1]));
    for (auto& b : bufs) RCHK(r.dev(*b.first, b.second, s));
    int64_t fs[5] = {0, 0, 0, 0, 0};
    int fk = 0;
    RCHK(sliding_fifo_state(q, bufs, fs, false, &fk));
    if (r.val<int32_t>() != fk || !r.ok) return sh_fail(SH_ERR_INVALID, "snapshot does not match this query");
    if (fk == 1) {
        for (int i = 0; i < 5; i++) fs[i] = r.val<int64_t>();
        if (!r.ok) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        RCHK(sliding_fifo_state(q, bufs, fs, true, &fk));
        for (auto& b : bufs) RCHK(r.dev(*b.first, b.second, s));
    } else if (fk == 2) {
        plane_state_buffers(q, bufs);
        for (auto& b : bufs) RCHK(r.dev(*b.first, b.second, s));
        const uint64_t hn = r.val<uint64_t>();
        if (!r.ok || r.o + hn > r.n) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        size_t used = 0;
        RCHK(plane_host_load(q, r.p + r.o, (size_t)hn, &used));
        r.o += hn;
    }
    q->seq = r.val<int64_t>();
    if (!r.ok) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    return SH_OK;
}

// ---- sharded query (sh_shard.cpp): the shard's global stream state + its owner query -------------
// (a sharded aggregation's roll-up executors and tables follow as one length-prefixed section)
int shard_checkpoint_state(sh_shard* s, int64_t* sc, int n, bool set, sh_query** owner);
sh_aggregation* shard_aggregation(sh_shard* s);
int agg_shard_state_write(sh_aggregation* a, std::vector<uint8_t>& out);
int agg_shard_state_read(sh_aggregation* a, const uint8_t* p, size_t n);

static int shard_snapshot_blob(sh_shard* sd, sh_query* q, Writer& w) {
    int64_t sc[14];
    RCHK(shard_checkpoint_state(sd, sc, 14, false, &q));
    w.put("SHS1", 4);
    w.val<uint32_t>(kVersion);
    w.val<uint64_t>(fingerprint(q));
    w.val<uint32_t>((uint32_t)q->kind);
    for (int i = 0; i < 14; i++) w.val<int64_t>(sc[i]);
    RCHK(q->kind == 1 ? sliding_snapshot(q, w) : batch_snapshot(q, w));
    if (q->wide) {  // an owner's interned group keys (its window's key ids)
        std::vector<uint8_t> kb;
        RCHK(q->wide->save(kb, q->ctx->stream));
        w.val<uint64_t>(kb.size());
        w.put(kb.data(), kb.size());
    }
    sh_aggregation* a = shard_aggregation(sd);
    w.val<uint8_t>(a ? 1 : 0);
    if (a) {
        std::vector<uint8_t> ab;
        RCHK(agg_shard_state_write(a, ab));
        w.val<uint64_t>(ab.size());
        w.put(ab.data(), ab.size());
    }
    return SH_OK;
}

extern "C" int sh_shard_snapshot(sh_shard* sd, void* buf, int64_t cap, int64_t* len) {
    SH_RANGE("sh_shard_snapshot");
    if (!sd || !len) return sh_fail(SH_ERR_INVALID, "sh_shard_snapshot: NULL argument");
    int64_t sc[14];
    sh_query* q = nullptr;
    RCHK(shard_checkpoint_state(sd, sc, 14, false, &q));
    StreamScope _ss(q->ctx->stream);
    Writer w;
    RCHK(shard_snapshot_blob(sd, q, w));
    *len = (int64_t)w.b.size();
    if (buf) {
        if (cap < *len) return sh_fail(SH_ERR_INVALID, "sh_shard_snapshot: buffer too small (call with buf=NULL for the size)");
        std::memcpy(buf, w.b.data(), w.b.size());
    }
    return SH_OK;
}

// The owner's windows are restored before the rank's global stream state is applied, and both only
// after the blob's header checked out; a failure part-way rolls the shard back (restore_or_roll_back).
static int shard_restore_blob(sh_shard* sd, sh_query* q, const void* buf, int64_t len) {
    Reader r{(const uint8_t*)buf, (size_t)len};
    if (len < 20 || std::memcmp(buf, "SHS1", 4) != 0) return sh_fail(SH_ERR_INVALID, "not a siddhi_hip shard snapshot");
    r.o = 4;
    if (r.val<uint32_t>() != kVersion) return sh_fail(SH_ERR_INVALID, "snapshot version mismatch");
    if (r.val<uint64_t>() != fingerprint(q)) return sh_fail(SH_ERR_INVALID, "snapshot was taken from a different query");
    if (r.val<uint32_t>() != (uint32_t)q->kind) return sh_fail(SH_ERR_INVALID, "snapshot kind mismatch");
    int64_t sc[14];
    for (int i = 0; i < 14; i++) sc[i] = r.val<int64_t>();
    if (!r.ok) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
    (void)hipStreamSynchronize(q->ctx->stream);
    // the owner takes its events already filtered by the ingest: keep its own (empty) filter
    const FilterProg keep = q->fp;
    const int rc = q->kind == 1 ? sliding_restore(q, r) : batch_restore(q, r);
    q->fp = keep;
    RCHK(rc);
    if (q->wide) {
        const uint64_t kn = r.val<uint64_t>();
        if (!r.ok || r.o + kn > r.n) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        size_t off = 0;
        RCHK(q->wide->load(r.p + r.o, (size_t)kn, off, q->ctx->stream));
        r.o += kn;
    }
    sh_aggregation* a = shard_aggregation(sd);
    const bool has_agg = r.val<uint8_t>() != 0;
    if (!r.ok || has_agg != (a != nullptr)) return sh_fail(SH_ERR_INVALID, "snapshot does not match this shard");
    if (a) {
        const uint64_t n = r.val<uint64_t>();
        if (!r.ok || r.o + n > r.n) return sh_fail(SH_ERR_INVALID, "snapshot blob truncated");
        RCHK(agg_shard_state_read(a, r.p + r.o, (size_t)n));
        r.o += n;
    }
    return shard_checkpoint_state(sd, sc, 14, true, &q);
}

extern "C" int sh_shard_restore(sh_shard* sd, const void* buf, int64_t len) {
    SH_RANGE("sh_shard_restore");
    if (!sd || !buf || len < 20) return sh_fail(SH_ERR_INVALID, "sh_shard_restore: bad arguments");
    int64_t cur[14];
    sh_query* q = nullptr;
    RCHK(shard_checkpoint_state(sd, cur, 14, false, &q));
    StreamScope _ss(q->ctx->stream);
    return restore_or_roll_back([&](Writer& w) { return shard_snapshot_blob(sd, q, w); },
                                [&](const void* b, int64_t n) { return shard_restore_blob(sd, q, b, n); }, buf, len);
}
