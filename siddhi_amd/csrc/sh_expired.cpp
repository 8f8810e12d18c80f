// sh_expired.cpp — `insert expired events` / `insert all events` output of lengthBatch and timeBatch
// windows (LengthBatchWindowProcessor.processFullBatchEvents :206-243, TimeBatchWindowProcessor.process
// :297-333, QuerySelector.processInBatchGroupBy :315-374 / processNoGroupBy :161-205).
//
// The batch pipeline (sh_window.cpp) produces the current rows of every closed batch as usual; this
// step turns them into the reference's output flushes. The flush that closes window X carries the
// expired copies of window X-1's events (only if X-1 was flushed with events: an empty window's close
// clears the expired queue) and the current events of X; its clock is the clock X closes at. Expired
// rows need no aggregation (sh_expired_kernels.hip): they are window X-1's current rows with constant
// values. A batch whose successor has not closed yet is carried to the next call.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "sh_runtime.h"

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

// window w closes at the first window start above w recorded by this call
static bool close_clock(const sh_query* q, int64_t w, int64_t* clock) {
    for (const auto& c : q->x_closes)
        if (c.first > w) { *clock = c.second; return true; }
    return false;
}

static int copy_cols(hipStream_t s, void* dst, size_t dst_stride, const void* src, size_t src_stride, size_t n, int cols,
                     size_t elem) {
    for (int c = 0; c < cols; c++)
        if (n) HIPCHK(hipMemcpyAsync((char*)dst + c * dst_stride * elem, (const char*)src + c * src_stride * elem, n * elem,
                                     hipMemcpyDeviceToDevice, s));
    return SH_OK;
}

int xout_finish(sh_query* q, bool host_out, const sh_out** out) {
    hipStream_t s = q->ctx->stream;
    const int nk = q->kp.n, na = q->ap.n;
    // lengthBatch and externalTimeBatch never close an empty batch: the expired copies of flush j go
    // out with flush j + 1 (ExternalTimeBatchWindowProcessor.flushToOutputChunk :336-383), stamped
    // with the attribute time that closed it (its running max, x_stamps) instead of the clock
    const bool ext = q->d.window == SH_WIN_EXT_TIME_BATCH;
    // (a sharded owner's lengthBatch windows are global batches: they close at the global window
    // starts, like timeBatch windows; its rows carry their global order)
    const bool lb = (q->d.window == SH_WIN_LENGTH_BATCH && !q->given) || ext;
    const bool ord = q->given;
    const int m = (int)q->dev_flush_clock.size();
    const int64_t nr = q->dev_flush_offsets.back();
    const int64_t nc = q->xc_valid ? q->xc_n : 0;
    const int64_t S = nc + nr;
    const int off = q->xc_valid ? 1 : 0;
    struct Src { int64_t lo, n, W; };
    std::vector<Src> src;
    if (q->xc_valid) src.push_back({0, nc, lb ? -1 : q->xc_W});
    for (int j = 0; j < m; j++)
        src.push_back({nc + q->dev_flush_offsets[j], q->dev_flush_offsets[j + 1] - q->dev_flush_offsets[j],
                       lb ? (int64_t)j : q->flush_window[j]});
    // output flushes keyed by the window they close
    struct It { int p = -1, c = -1; int64_t clock = 0; };
    std::map<int64_t, It> plan;
    for (int j = 0; j < m; j++) {
        It& it = plan[src[j + off].W];
        it.c = j + off;
        it.clock = q->dev_flush_clock[j];
    }
    int pending = -1;
    for (int si = 0; si < (int)src.size(); si++) {
        const int64_t w1 = src[si].W + 1;
        int64_t clk = 0;
        bool known;
        if (lb) {
            known = w1 < m;
            if (known) clk = q->dev_flush_clock[w1];
        } else {
            known = close_clock(q, w1, &clk);
        }
        if (known) {
            It& it = plan[w1];
            it.p = si;
            if (it.c < 0) it.clock = clk;
        } else {
            if (si != (int)src.size() - 1) return sh_fail(SH_ERR_INVALID, "expired output: window close order");
            pending = si;
        }
    }
    const bool merge_ok = !(nk == 0 && na == 0);  // pass-through rows are never merged
    // one dictionary-id key (dense, ids below the table's capacity): a flush's table is indexed by the id
    // itself when it is at most 4x the hashed table's size (no hashing, no key column, no probing)
    const int64_t dense_cap = (nk == 1 && q->kp.n == 1 && q->kt.dense && q->kt.dmul == 1 && q->kt.dadd == 0 && !q->wide)
                                  ? (int64_t)q->kt.size_ : 0;
    std::vector<XItem> items;
    std::vector<int64_t> item_w;
    int64_t tab_total = 0;
    for (auto& kv : plan) {
        const It& it = kv.second;
        XItem x{};
        x.clock = it.clock;
        x.xts = ext && kv.first >= 0 && kv.first < (int64_t)q->x_stamps.size() ? q->x_stamps[kv.first] : it.clock;
        if (it.p >= 0) { x.p_lo = src[it.p].lo; x.p_n = src[it.p].n; }
        if (it.c >= 0 && q->d.current_on) { x.c_lo = src[it.c].lo; x.c_n = src[it.c].n; }
        if (x.p_n + x.c_n == 0) continue;
        if (x.p_n > 0 && x.c_n > 0 && merge_ok) {
            int64_t ts = 2;
            while (ts < 2 * x.c_n) ts <<= 1;
            if (dense_cap > 0 && dense_cap <= 4 * ts) {
                ts = std::max<int64_t>(ts, dense_cap);
                x.pad = 1;  // (direct: slot = the id)
            }
            x.tab_off = tab_total;
            x.tab_size = ts;
            tab_total += ts;
        }
        items.push_back(x);
        item_w.push_back(kv.first);
    }
    const int ni = (int)items.size();
    // the source array: [carried rows] + [this call's current rows]
    const int NK = std::max(1, nk), NA = std::max(1, na);
    if (S > 0) {
        RCHK(q->xs_ts.reserve(S * 8, false));
        RCHK(q->xs_rep.reserve(S * 8, false));
        RCHK(q->xs_keys.reserve((size_t)NK * S * 8, false));
        RCHK(q->xs_vals.reserve((size_t)NA * S * 8, false));
        RCHK(q->xs_nulls.reserve((size_t)NA * S, false));
        if (ord) RCHK(q->xs_order.reserve(S * 8, false));
        if (nc) {
            RCHK(copy_cols(s, q->xs_keys.p, S, q->xc_keys.p, nc, nc, nk, 8));
            RCHK(copy_cols(s, q->xs_rep.p, S, q->xc_rep.p, nc, nc, 1, 8));
            if (ord) RCHK(copy_cols(s, q->xs_order.p, S, q->xc_order.p, nc, nc, 1, 8));
        }
        if (nr && ord) RCHK(copy_cols(s, q->xs_order.as<int64_t>() + nc, S, q->out_order.p, nr, nr, 1, 8));
        if (nr) {
            RCHK(copy_cols(s, q->xs_ts.as<int64_t>() + nc, S, q->out_ts.p, nr, nr, 1, 8));
            RCHK(copy_cols(s, q->xs_rep.as<int64_t>() + nc, S, q->out_rep.p, nr, nr, 1, 8));
            RCHK(copy_cols(s, q->xs_keys.as<int64_t>() + nc, S, q->out_keys.p, nr, nr, nk, 8));
            RCHK(copy_cols(s, q->xs_vals.as<uint64_t>() + nc, S, q->out_vals.p, nr, nr, na, 8));
            RCHK(copy_cols(s, q->xs_nulls.as<unsigned char>() + nc, S, q->out_nulls.p, nr, nr, na, 1));
        }
    }
    std::vector<int64_t> cum_c(ni + 1, 0), cum_p(ni + 1, 0), cum_o(ni + 1, 0);
    for (int i = 0; i < ni; i++) {
        const bool mg = items[i].tab_size > 0;
        cum_c[i + 1] = cum_c[i] + (mg ? items[i].c_n : 0);
        cum_p[i + 1] = cum_p[i] + (mg ? items[i].p_n : 0);
        cum_o[i + 1] = cum_o[i] + items[i].p_n + items[i].c_n;
    }
    // one upload: [items][cum_c][cum_p][cum_o]
    const size_t items_bytes = (size_t)ni * sizeof(XItem), up = items_bytes + (size_t)3 * (ni + 1) * 8;
    auto upload = [&]() -> int {
        RCHK(q->x_items.reserve(std::max<size_t>(up, 64), false));
        RCHK(q->x_h.reserve(std::max<size_t>(up, 64) + (size_t)ni * 4 + 64));
        char* h = q->x_h.as<char>();
        std::memcpy(h, items.data(), items_bytes);
        int64_t* hc = (int64_t*)(h + items_bytes);
        std::memcpy(hc, cum_c.data(), (ni + 1) * 8);
        std::memcpy(hc + (ni + 1), cum_p.data(), (ni + 1) * 8);
        std::memcpy(hc + 2 * (ni + 1), cum_o.data(), (ni + 1) * 8);
        HIPCHK(hipMemcpyAsync(q->x_items.p, h, up, hipMemcpyHostToDevice, s));
        return SH_OK;
    };
    const XItem* d_items = nullptr;
    const int64_t *d_cum_c = nullptr, *d_cum_p = nullptr, *d_cum_o = nullptr;
    int64_t T = 0;
    const bool merging = ni > 0 && cum_c[ni] > 0;
    if (!merging) {
        for (int i = 0; i < ni; i++) {
            items[i].out_base = T;
            T += items[i].p_n + items[i].c_n;
        }
    }
    if (ni > 0) {
        RCHK(upload());
        d_items = q->x_items.as<XItem>();
        d_cum_c = (const int64_t*)(q->x_items.as<char>() + items_bytes);
        d_cum_p = d_cum_c + (ni + 1);
        d_cum_o = d_cum_p + (ni + 1);
        RCHK(q->x_keep.reserve((size_t)(S + 1) * 4, false));
        RCHK(q->x_rank.reserve((size_t)(S + 1) * 4, false));
        RCHK(q->x_match.reserve((size_t)std::max<int64_t>(S, 1) * 4, false));
        RCHK(q->x_tmp.reserve((size_t)((S + 1 + kTile - 1) / kTile + 16) * 8, false));
        RCHK(q->x_matched.reserve((size_t)ni * 4 + 16, false));
        // keep = 1 for this call's current rows (carried rows are never current)
        HIPCHK(hipMemsetAsync(q->x_keep.p, 0, (size_t)(S + 1) * 4, s));
        if (nr) HIPCHK(hipMemsetD32Async((hipDeviceptr_t)(q->x_keep.as<uint32_t>() + nc), 1, (size_t)nr, s));
        HIPCHK(hipMemsetAsync(q->x_matched.p, 0, (size_t)ni * 4, s));
        if (merging) {
            RCHK(q->x_trow.reserve((size_t)tab_total * 4, false));
            RCHK(q->x_tkey.reserve((size_t)tab_total * 8, false));
            HIPCHK(hipMemsetAsync(q->x_trow.p, 0xff, (size_t)tab_total * 4, s));
            launch_x_merge(s, d_items, d_cum_c, d_cum_p, ni, cum_c[ni], cum_p[ni], q->xs_keys.as<int64_t>(), S, nk,
                           q->x_trow.as<uint32_t>(), q->x_tkey.as<u64>(), q->x_match.as<int>(),
                           q->x_keep.as<uint32_t>(), q->x_matched.as<uint32_t>());
            HIPCHK(hipGetLastError());
            uint32_t* hm = (uint32_t*)(q->x_h.as<char>() + up);
            HIPCHK(hipMemcpyAsync(hm, q->x_matched.p, (size_t)ni * 4, hipMemcpyDeviceToHost, s));
            HIPCHK(hipStreamSynchronize(s));
            std::vector<uint32_t> mt(hm, hm + ni);
            for (int i = 0; i < ni; i++) {
                items[i].out_base = T;
                T += items[i].p_n + items[i].c_n - (int64_t)mt[i];
            }
            RCHK(upload());  // the output bases (after the synchronisation: the pinned area is free)
        }
        HIPCHK(hipMemcpyAsync(q->x_rank.p, q->x_keep.p, (size_t)(S + 1) * 4, hipMemcpyDeviceToDevice, s));
        launch_scan_sum_large_u32(s, q->x_rank.as<uint32_t>(), S + 1, q->x_tmp.as<int64_t>());
        const int64_t TC = std::max<int64_t>(T, 1);
        RCHK(q->x_ts.reserve(TC * 8, false));
        RCHK(q->x_rep.reserve(TC * 8, false));
        RCHK(q->x_expired.reserve(TC, false));
        RCHK(q->x_keys.reserve((size_t)NK * TC * 8, false));
        RCHK(q->x_vals.reserve((size_t)NA * TC * 8, false));
        RCHK(q->x_nulls.reserve((size_t)NA * TC, false));
        uint32_t count_mask = 0;
        for (int a = 0; a < na; a++) if (q->ap.kind[a] == AK_COUNT) count_mask |= 1u << a;
        if (ord) RCHK(q->x_order.reserve(TC * 8, false));
        XOut xo{q->x_ts.as<int64_t>(), q->x_expired.as<unsigned char>(), q->x_keys.as<int64_t>(), q->x_vals.as<u64>(),
                q->x_nulls.as<unsigned char>(), q->x_rep.as<int64_t>(), ord ? q->x_order.as<int64_t>() : nullptr,
                ord ? q->xs_order.as<int64_t>() : nullptr};
        launch_x_scatter(s, d_items, d_cum_o, ni, cum_o[ni], q->xs_ts.as<int64_t>(), q->xs_keys.as<int64_t>(),
                         q->xs_vals.as<u64>(), q->xs_nulls.as<unsigned char>(), q->xs_rep.as<int64_t>(), S, nk, na,
                         count_mask, q->x_match.as<int>(), q->x_keep.as<uint32_t>(), q->x_rank.as<uint32_t>(), T, xo);
        HIPCHK(hipGetLastError());
    }
    // the batch whose successor has not closed is carried (its keys and representative events)
    if (pending < 0) {
        q->xc_valid = false;
        q->xc_n = 0;
    } else if (!(q->xc_valid && pending == 0)) {
        const Src& ps = src[pending];
        RCHK(q->xc_keys2.reserve((size_t)NK * std::max<int64_t>(ps.n, 1) * 8, false));
        RCHK(q->xc_rep2.reserve((size_t)std::max<int64_t>(ps.n, 1) * 8, false));
        RCHK(copy_cols(s, q->xc_keys2.p, ps.n, q->xs_keys.as<int64_t>() + ps.lo, S, ps.n, nk, 8));
        RCHK(copy_cols(s, q->xc_rep2.p, ps.n, q->xs_rep.as<int64_t>() + ps.lo, S, ps.n, 1, 8));
        std::swap(q->xc_keys, q->xc_keys2);
        std::swap(q->xc_rep, q->xc_rep2);
        if (ord) {
            RCHK(q->xc_order2.reserve((size_t)std::max<int64_t>(ps.n, 1) * 8, false));
            RCHK(copy_cols(s, q->xc_order2.p, ps.n, q->xs_order.as<int64_t>() + ps.lo, S, ps.n, 1, 8));
            std::swap(q->xc_order, q->xc_order2);
        }
        q->xc_valid = true;
        q->xc_n = ps.n;
        q->xc_W = ps.W;
    }
    // output flushes, and the window each closes (a sharded merge matches the owners' flushes by it)
    std::vector<int64_t> fo(1, 0), fc;
    q->flush_window.clear();
    for (int i = 0; i < ni; i++) {
        const int64_t next = i + 1 < ni ? items[i + 1].out_base : T;
        if (next == items[i].out_base) continue;
        fo.push_back(next);
        fc.push_back(items[i].clock);
        q->flush_window.push_back(item_w[i]);
    }
    if (host_out) {
        OutHost& o = q->out;
        o.reset();
        o.flush_offsets.assign(fo.begin(), fo.end());
        o.flush_clock.assign(fc.begin(), fc.end());
        o.ts.resize(T);
        o.expired.resize(T);
        o.rep.resize(T);
        o.keys.resize((size_t)nk * T);
        o.vals.resize((size_t)na * T);
        o.nulls.resize((size_t)na * T);
        if (ord) {
            q->order_host.resize(T);
            if (T > 0) HIPCHK(hipMemcpyAsync(q->order_host.data(), q->x_order.p, T * 8, hipMemcpyDeviceToHost, s));
        }
        if (T > 0) {
            HIPCHK(hipMemcpyAsync(o.ts.data(), q->x_ts.p, T * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(o.expired.data(), q->x_expired.p, T, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(o.rep.data(), q->x_rep.p, T * 8, hipMemcpyDeviceToHost, s));
            // device columns have stride T (the output row count)
            if (nk) HIPCHK(hipMemcpyAsync(o.keys.data(), q->x_keys.p, (size_t)nk * T * 8, hipMemcpyDeviceToHost, s));
            if (na) {
                HIPCHK(hipMemcpyAsync(o.vals.data(), q->x_vals.p, (size_t)na * T * 8, hipMemcpyDeviceToHost, s));
                HIPCHK(hipMemcpyAsync(o.nulls.data(), q->x_nulls.p, (size_t)na * T, hipMemcpyDeviceToHost, s));
            }
        }
        HIPCHK(hipStreamSynchronize(s));
        *out = o.view(nk, na, q->vtypes);
    } else {
        HIPCHK(hipStreamSynchronize(s));
        q->dev_flush_offsets.assign(fo.begin(), fo.end());
        q->dev_flush_clock.assign(fc.begin(), fc.end());
        sh_out& o = q->dev_out;
        o = sh_out{};
        o.n_flushes = (int64_t)fc.size();
        o.n_rows = T;
        o.n_keys = nk;
        o.n_vals = na;
        for (int i = 0; i < na; i++) o.val_types[i] = q->vtypes[i];
        o.flush_offsets = q->dev_flush_offsets.data();
        o.flush_clock = q->dev_flush_clock.data();
        o.ts = q->x_ts.as<int64_t>();
        o.expired = q->x_expired.as<uint8_t>();
        o.keys = q->x_keys.as<int64_t>();
        o.vals = q->x_vals.as<uint64_t>();
        o.nulls = q->x_nulls.as<uint8_t>();
        o.rep = q->x_rep.as<int64_t>();
        RCHK(flush_layout_to_device(q, o));
        *out = &o;
    }
    q->x_closes.clear();
    return SH_OK;
}
