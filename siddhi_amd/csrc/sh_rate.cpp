// sh_rate.cpp — output rate limiting `output [all|first|last] every N events`
// (OutputParser.constructOutputRateLimiter :288-303; core/query/output/ratelimit/event/
// AllPerEvent, FirstPerEvent, LastPerEvent, FirstGroupByPerEvent, LastGroupByPerEventOutputRateLimiter).
//
// The limiter sits after the selector: every flush a call produces is one process() chunk. A call
// runs the query with device output, then this step keeps the rows the limiter sends on
// (sh_rate_kernels.hip) and groups them by the input flush that emits them; that flush's clock is the
// output flush's clock, and input flushes that emit nothing send no chunk.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "sh_agg.h"
#include "sh_plane_group.h"
#include "sh_runtime.h"

using namespace shd;

// the partition lanes (sh_plane.cpp): partition slots, and the partition slot of every output row
int64_t plane_slots(sh_query* q);
const u32* plane_out_part(sh_query* q);

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

extern "C" int sh_query_set_output_rate(sh_query* q, int32_t kind, int64_t n) {
    if (!q) return sh_fail(SH_ERR_INVALID, "sh_query_set_output_rate: NULL query");
    if (kind < SH_RATE_NONE || kind > SH_RATE_FIRST_TIME) return sh_fail(SH_ERR_INVALID, "unknown output rate kind");
    if (kind != SH_RATE_NONE && kind != SH_RATE_FIRST_TIME && n < 1)
        return sh_fail(SH_ERR_INVALID, "output rate needs every >= 1 events");
    if (kind == SH_RATE_FIRST_TIME && n < 0) return sh_fail(SH_ERR_INVALID, "output rate needs a time >= 0");
    if (n > (int64_t)1 << 30) return sh_fail(SH_ERR_UNSUPPORTED, "output rate above 2^30 events");
    if (q->seq > 0 || q->clock_valid) return sh_fail(SH_ERR_INVALID, "output rate must be set before the first push");
    // a partitioned query holds one limiter per partition instance (PartitionRuntime clones the query);
    // the GPU's partitioned timeBatch flushes only partition p0 (R12), so its one limiter is p0's
    if (kind != SH_RATE_NONE && q->given)
        return sh_fail(SH_ERR_UNSUPPORTED, "a sharded query's limiter runs over the merged output (sh_rate_apply_merged)");
    if (kind != SH_RATE_NONE && q->kp.n > 2) return sh_fail(SH_ERR_UNSUPPORTED, "output rate with more than 2 group-by keys");
    // the partition lanes (sh_plane.cpp): one limiter per partition instance. Grouped by the partition
    // key, a partition's limiter sees one key, so the keyed First variants equal the global keyed ones
    // (their state is per key) and LastGroupBy is the positional LastPerEvent of the partition.
    const bool lanes = q->kind == 1 && q->d.partition_col >= 0;
    if (lanes && kind != SH_RATE_NONE && q->xt_replace)
        return sh_fail(SH_ERR_UNSUPPORTED,
                       "replaceTimestampWithBatchEndTime of a partitioned query with an output rate limiter");
    bool gb = (lanes ? q->d.n_group_by > 0 : q->kp.n > 0) && kind != SH_RATE_ALL;
    bool part = false;
    if (lanes && kind != SH_RATE_NONE) {
        // grouped by other columns, each partition's keyed First limiter is the global one keyed by
        // (partition, group key) — one 32-bit group column packs beside the partition slot
        const int gc = q->d.n_group_by == 1 ? q->d.group_by[0] : -1;
        const bool k32 = gc >= 0 && (q->d.col_types[gc] == SH_T_INT || q->d.col_types[gc] == SH_T_STRID ||
                                     q->d.col_types[gc] == SH_T_BOOL);
        if (gb && q->group_other && !k32)
            return sh_fail(SH_ERR_UNSUPPORTED,
                           "keyed output rate limiting of a partitioned window grouped by a long / floating / two-column "
                           "key: `output all every`, a limiter keyed by one int / string group column, or no group-by");
        q->rate.pkey = gb && q->group_other;
        // LastGroupBy grouped by other columns: the per-partition positional windows, keyed inside them
        q->rate.lkey = kind == SH_RATE_LAST && gb && q->group_other;
        part = kind == SH_RATE_ALL || kind == SH_RATE_LAST || !gb;
        if (part) gb = false;
        const int64_t np = plane_slots(q);
        auto& r = q->rate;
        RCHK(r.pseq.reserve((size_t)np * 8, false));
        RCHK(r.pft_has.reserve((size_t)np, false));
        RCHK(r.pft_last.reserve((size_t)np * 8, false));
        HIPCHK(hipMemsetAsync(r.pseq.p, 0, (size_t)np * 8, q->ctx->stream));
        HIPCHK(hipMemsetAsync(r.pft_has.p, 0, (size_t)np, q->ctx->stream));
        HIPCHK(hipMemsetAsync(r.pft_last.p, 0, (size_t)np * 8, q->ctx->stream));
        HIPCHK(hipStreamSynchronize(q->ctx->stream));
        r.nparts = np;
    }
    if (!lanes) q->rate.pkey = q->rate.lkey = false;
    q->rate.part = part;
    q->rate.kind = kind;
    q->rate.N = n;
    q->rate.gb = gb;
    q->rate.seq = 0;
    q->rate.nc = 0;
    q->rate.t_cap = 0;
    q->rate.t_keys = 0;
    q->rate.ft_has = false;
    q->rate.ft_cap = 0;
    q->rate.ft_keys = 0;
    return SH_OK;
}

// `output first every <t>` group-by table: room for `need` keys at load <= 1/2
static int grow_ftime_table(sh_query* q, int64_t need) {
    auto& r = q->rate;
    hipStream_t s = q->ctx->stream;
    int64_t cap = 64;
    while (cap < 2 * need) cap <<= 1;
    if (cap > ((int64_t)1 << 31)) return sh_fail(SH_ERR_UNSUPPORTED, "output rate: too many group keys");
    if (cap <= r.ft_cap) return SH_OK;
    RCHK(r.ftk2.reserve((size_t)cap * 8, false));
    RCHK(r.ftt2.reserve((size_t)cap * 8, false));
    // kEmptyKey (0x8000000000000001) in every slot
    std::vector<uint64_t> empty((size_t)cap, kEmptyKey);
    HIPCHK(hipMemcpyAsync(r.ftk2.p, empty.data(), (size_t)cap * 8, hipMemcpyHostToDevice, s));
    if (r.ft_cap > 0)
        launch_rate_ftime_rehash(s, r.ft_cap, r.ftk.as<u64>(), r.ftt.as<i64>(), r.ftk2.as<u64>(), r.ftt2.as<i64>(),
                                 (u32)(cap - 1));
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));  // `empty` is pageable host memory
    std::swap(r.ftk, r.ftk2);
    std::swap(r.ftt, r.ftt2);
    r.ft_cap = cap;
    return SH_OK;
}

static int copy_cols(hipStream_t s, void* dst, size_t dst_stride, const void* src, size_t src_stride, size_t n, int cols,
                     size_t elem) {
    for (int c = 0; c < cols; c++)
        if (n) HIPCHK(hipMemcpyAsync((char*)dst + c * dst_stride * elem, (const char*)src + c * src_stride * elem, n * elem,
                                     hipMemcpyDeviceToDevice, s));
    return SH_OK;
}

static int reserve_rows(DevBuf* b, int64_t rows, int cols, size_t elem) {
    return b->reserve((size_t)std::max<int64_t>(rows, 1) * std::max(cols, 1) * elem, false);
}

// rows [lo, lo + n) of a row set with the given stride -> a row set of stride n
static int copy_rows(hipStream_t s, RateRows dst, int64_t dst_stride, RateRows src, int64_t src_stride, int64_t lo,
                     int64_t n, int nk, int na) {
    if (n <= 0) return SH_OK;
    RCHK(copy_cols(s, dst.ts, dst_stride, src.ts + lo, src_stride, n, 1, 8));
    RCHK(copy_cols(s, dst.expired, dst_stride, src.expired + lo, src_stride, n, 1, 1));
    RCHK(copy_cols(s, dst.rep, dst_stride, src.rep + lo, src_stride, n, 1, 8));
    RCHK(copy_cols(s, dst.keys, dst_stride, src.keys + lo, src_stride, n, nk, 8));
    RCHK(copy_cols(s, dst.vals, dst_stride, src.vals + lo, src_stride, n, na, 8));
    RCHK(copy_cols(s, dst.nulls, dst_stride, src.nulls + lo, src_stride, n, na, 1));
    return SH_OK;
}

static int reserve_set(DevBuf& ts, DevBuf& ex, DevBuf& rep, DevBuf& keys, DevBuf& vals, DevBuf& nulls, int64_t n, int nk,
                       int na, RateRows* r) {
    RCHK(reserve_rows(&ts, n, 1, 8));
    RCHK(reserve_rows(&ex, n, 1, 1));
    RCHK(reserve_rows(&rep, n, 1, 8));
    RCHK(reserve_rows(&keys, n, nk, 8));
    RCHK(reserve_rows(&vals, n, na, 8));
    RCHK(reserve_rows(&nulls, n, na, 1));
    *r = RateRows{ts.as<i64>(), ex.as<unsigned char>(), rep.as<i64>(), keys.as<i64>(), vals.as<u64>(),
                  nulls.as<unsigned char>()};
    return SH_OK;
}

// FirstGroupBy table: room for `need` keys at load <= 1/2 (existing entries rehashed on growth)
static int grow_table(sh_query* q, int64_t need) {
    auto& r = q->rate;
    hipStream_t s = q->ctx->stream;
    int64_t cap = 64;
    while (cap < 2 * need) cap <<= 1;
    if (cap > ((int64_t)1 << 31)) return sh_fail(SH_ERR_UNSUPPORTED, "output rate: too many group keys");
    if (cap <= r.t_cap) return SH_OK;
    RCHK(r.tk2.reserve((size_t)cap * 8, false));
    RCHK(r.tc2.reserve((size_t)cap * 8, false));
    HIPCHK(hipMemsetAsync(r.tc2.p, 0xff, (size_t)cap * 8, s));
    if (r.t_cap > 0)
        launch_rate_rehash(s, r.t_cap, r.tk.as<u64>(), r.tc.as<i64>(), r.tk2.as<u64>(), r.tc2.as<i64>(), (u32)(cap - 1));
    HIPCHK(hipGetLastError());
    std::swap(r.tk, r.tk2);
    std::swap(r.tc, r.tc2);
    r.t_cap = cap;
    return SH_OK;
}

// the kept rows (o, T of them, o_flush = their emitting input flushes) -> output flushes and the
// host or device view
static int rate_finish(sh_query* q, const RateRows& o, int64_t T, int nk, int na, bool host_out, const sh_out** out) {
    auto& r = q->rate;
    hipStream_t s = q->ctx->stream;
    // output flushes: runs of equal emitting flush
    r.h_flush.resize(std::max<int64_t>(T, 1));
    if (T > 0) HIPCHK(hipMemcpyAsync(r.h_flush.data(), r.o_flush.p, (size_t)T * 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    r.flush_offsets.assign(1, 0);
    r.flush_clock.clear();
    for (int64_t i = 0; i < T; i++) {
        if (i + 1 == T || r.h_flush[i + 1] != r.h_flush[i]) {
            r.flush_offsets.push_back(i + 1);
            r.flush_clock.push_back(r.h_clk[r.h_flush[i]]);
        }
    }
    if (host_out) {
        OutHost& ho = q->out;
        ho.reset();
        ho.flush_offsets.assign(r.flush_offsets.begin(), r.flush_offsets.end());
        ho.flush_clock.assign(r.flush_clock.begin(), r.flush_clock.end());
        ho.ts.resize(T);
        ho.expired.resize(T);
        ho.rep.resize(T);
        ho.keys.resize((size_t)nk * T);
        ho.vals.resize((size_t)na * T);
        ho.nulls.resize((size_t)na * T);
        if (T > 0) {
            HIPCHK(hipMemcpyAsync(ho.ts.data(), o.ts, T * 8, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(ho.expired.data(), o.expired, T, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(ho.rep.data(), o.rep, T * 8, hipMemcpyDeviceToHost, s));
            if (nk) HIPCHK(hipMemcpyAsync(ho.keys.data(), o.keys, (size_t)nk * T * 8, hipMemcpyDeviceToHost, s));
            if (na) {
                HIPCHK(hipMemcpyAsync(ho.vals.data(), o.vals, (size_t)na * T * 8, hipMemcpyDeviceToHost, s));
                HIPCHK(hipMemcpyAsync(ho.nulls.data(), o.nulls, (size_t)na * T, hipMemcpyDeviceToHost, s));
            }
            HIPCHK(hipStreamSynchronize(s));
        }
        *out = ho.view(nk, na, q->vtypes);
    } else {
        sh_out& d = r.dev_out;
        d = sh_out{};
        d.n_flushes = (int64_t)r.flush_clock.size();
        d.n_rows = T;
        d.n_keys = nk;
        d.n_vals = na;
        for (int i = 0; i < na; i++) d.val_types[i] = q->vtypes[i];
        d.flush_offsets = r.flush_offsets.data();
        d.flush_clock = r.flush_clock.data();
        d.ts = o.ts;
        d.expired = o.expired;
        d.keys = o.keys;
        d.vals = (const uint64_t*)o.vals;
        d.nulls = o.nulls;
        d.rep = o.rep;
        *out = &d;
    }
    return SH_OK;
}

static int rate_part(sh_query* q, const sh_out* in, const i64* foff, int nf, bool host_out, const sh_out** out);

int rate_apply(sh_query* q, const sh_out* in, bool flush_dev, bool host_out, const sh_out** out) {
    auto& r = q->rate;
    hipStream_t s = q->ctx->stream;
    const int nk = (int)in->n_keys, na = (int)in->n_vals;
    const int64_t n = in->n_rows;
    const int nf = (int)in->n_flushes;
    const int64_t N = r.N;
    if (n == 0) {  // no chunk reaches the limiter
        r.flush_offsets.assign(1, 0);
        r.flush_clock.clear();
        if (host_out) {
            q->out.reset();
            *out = q->out.view(nk, na, q->vtypes);
        } else {
            r.dev_out = sh_out{};
            r.dev_out.n_keys = nk;
            r.dev_out.n_vals = na;
            for (int i = 0; i < na; i++) r.dev_out.val_types[i] = q->vtypes[i];
            r.dev_out.flush_offsets = r.flush_offsets.data();
            r.dev_out.flush_clock = r.flush_clock.data();
            *out = &r.dev_out;
        }
        return SH_OK;
    }
    // the input's flush layout on the host (clocks of the output flushes) and offsets on the device
    r.h_off.resize(nf + 1);
    r.h_clk.resize(std::max(nf, 1));
    if (flush_dev) {
        HIPCHK(hipMemcpyAsync(r.h_off.data(), in->flush_offsets, (size_t)(nf + 1) * 8, hipMemcpyDeviceToHost, s));
        if (nf) HIPCHK(hipMemcpyAsync(r.h_clk.data(), in->flush_clock, (size_t)nf * 8, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
    } else {
        std::memcpy(r.h_off.data(), in->flush_offsets, (size_t)(nf + 1) * 8);
        if (nf) std::memcpy(r.h_clk.data(), in->flush_clock, (size_t)nf * 8);
    }
    if (nf == 0) r.h_off[0] = 0;
    RCHK(r.foff.reserve((size_t)(nf + 1) * 8, false));
    HIPCHK(hipMemcpyAsync(r.foff.p, r.h_off.data(), (size_t)(nf + 1) * 8, hipMemcpyHostToDevice, s));
    const i64* foff = r.foff.as<i64>();
    if (r.part) return rate_part(q, in, foff, nf, host_out, out);

    // the source rows: [carried rows | this call's rows]
    const bool carries = r.kind == SH_RATE_ALL || (r.kind == SH_RATE_LAST && r.gb);
    const int64_t nc = carries ? r.nc : 0;
    const int64_t S = nc + n;
    RateRows inr{(i64*)in->ts, (unsigned char*)in->expired, (i64*)in->rep, (i64*)in->keys, (u64*)in->vals,
                 (unsigned char*)in->nulls};
    RateRows src = inr;
    int64_t sstride = n;
    if (nc > 0) {
        RCHK(reserve_set(r.s_ts, r.s_exp, r.s_rep, r.s_keys, r.s_vals, r.s_nulls, S, nk, na, &src));
        RateRows car{r.c_ts.as<i64>(), r.c_exp.as<unsigned char>(), r.c_rep.as<i64>(), r.c_keys.as<i64>(),
                     r.c_vals.as<u64>(), r.c_nulls.as<unsigned char>()};
        RCHK(copy_rows(s, src, S, car, nc, 0, nc, nk, na));
        RateRows tail = src;
        tail.ts += nc; tail.expired += nc; tail.rep += nc; tail.keys += nc; tail.vals += nc; tail.nulls += nc;
        RCHK(copy_rows(s, tail, S, inr, n, 0, n, nk, na));
        sstride = S;
    }
    const int64_t E = carries ? S / N * N : S;  // rows [E, S) wait for their group
    RCHK(r.flag.reserve((size_t)(S + 1) * 4, false));
    RCHK(r.pre.reserve((size_t)(S + 1) * 4, false));
    RCHK(r.src.reserve((size_t)std::max<int64_t>(S, 1) * 4, false));
    RCHK(r.eflush.reserve((size_t)std::max<int64_t>(S, 1) * 4, false));
    RCHK(r.tmp.reserve((size_t)((S + 1 + kTile - 1) / kTile + 16) * 8, false));
    RCHK(r.h_small.reserve(64));
    if (r.kind == SH_RATE_FIRST_TIME && !r.gb) {
        // FirstPerTimeOutputRateLimiter :54-78, flush by flush in order (a flush = one process() chunk)
        std::vector<unsigned char> chosen((size_t)std::max(nf, 1), 0);
        for (int f = 0; f < nf; f++) {
            if (r.h_off[f + 1] <= r.h_off[f]) continue;
            if (!r.ft_has || r.ft_last + N <= r.h_clk[f]) {
                chosen[f] = 1;
                r.ft_has = true;
                r.ft_last = r.h_clk[f];
            }
        }
        RCHK(r.chosen.reserve(chosen.size(), false));
        HIPCHK(hipMemcpyAsync(r.chosen.p, chosen.data(), chosen.size(), hipMemcpyHostToDevice, s));
        launch_rate_ftime_rows(s, S, foff, nf, r.chosen.as<unsigned char>(), r.flag.as<u32>(), r.eflush.as<int>(),
                               r.src.as<u32>());
        HIPCHK(hipStreamSynchronize(s));  // `chosen` is pageable host memory
    } else if (r.kind == SH_RATE_FIRST_TIME) {
        // FirstGroupByPerTimeOutputRateLimiter :54-80: rows sorted stably by key, one walker per key
        RCHK(r.fclk.reserve((size_t)std::max(nf, 1) * 8, false));
        if (nf) HIPCHK(hipMemcpyAsync(r.fclk.p, r.h_clk.data(), (size_t)nf * 8, hipMemcpyHostToDevice, s));
        launch_rate_ftime_rows(s, S, foff, nf, nullptr, r.flag.as<u32>(), r.eflush.as<int>(), r.src.as<u32>());
        const int64_t m = S;
        RCHK(r.skey.reserve((size_t)m * 8, false));
        RCHK(r.skey2.reserve((size_t)m * 8, false));
        RCHK(r.idx.reserve((size_t)m * 4, false));
        RCHK(r.idx2.reserve((size_t)m * 4, false));
        RCHK(r.hd.reserve((size_t)(m + 1) * 4, false));
        RCHK(r.pos.reserve((size_t)(m + 1) * 4, false));
        RCHK(r.starts.reserve((size_t)(m + 1) * 4, false));
        RCHK(r.tmp.reserve((size_t)((m + 1 + kTile - 1) / kTile + 16) * 8, false));
        if (r.pkey) launch_ratep_pkey(s, m, src.keys, plane_out_part(q), r.skey.as<u64>(), r.idx.as<u32>());
        else launch_rate_pack(s, m, src.keys, sstride, nk, r.skey.as<u64>(), r.idx.as<u32>());
        size_t tb = 0;
        if (sort_u64_pairs(nullptr, &tb, nullptr, nullptr, nullptr, nullptr, m, s))
            return sh_fail(SH_ERR_DEVICE, "output rate: sort sizing");
        RCHK(r.sort_tmp.reserve(std::max<size_t>(tb, 16), false));
        if (sort_u64_pairs(r.sort_tmp.p, &tb, r.skey.as<u64>(), r.skey2.as<u64>(), r.idx.as<u32>(), r.idx2.as<u32>(), m, s))
            return sh_fail(SH_ERR_DEVICE, "output rate: sort failed");
        launch_rate_segments(s, m, r.skey2.as<u64>(), r.idx2.as<u32>(), 1, 0, r.hd.as<u32>(), r.pos.as<u32>(),
                             r.starts.as<u32>(), r.tmp.as<i64>());
        HIPCHK(hipMemcpyAsync(r.h_small.as<char>() + 16, r.pos.as<u32>() + m, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        RCHK(grow_ftime_table(q, r.ft_keys + *(const uint32_t*)(r.h_small.as<char>() + 16)));
        RCHK(r.n_keys.reserve(16, false));
        HIPCHK(hipMemsetAsync(r.n_keys.p, 0, 4, s));
        launch_rate_ftime_walk(s, m, r.hd.as<u32>(), r.pos.as<u32>(), r.starts.as<u32>(), r.skey2.as<u64>(),
                               r.idx2.as<u32>(), foff, r.fclk.as<i64>(), nf, N, r.ftk.as<u64>(), r.ftt.as<i64>(),
                               (u32)(r.ft_cap - 1), r.flag.as<u32>(), r.n_keys.as<u32>());
        HIPCHK(hipMemcpyAsync(r.h_small.as<char>() + 24, r.n_keys.p, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        r.ft_keys += *(const uint32_t*)(r.h_small.as<char>() + 24);
    } else if (!r.gb) {
        launch_rate_pos(s, S, nc, r.kind, N, r.seq, foff, nf, r.flag.as<u32>(), r.eflush.as<int>(), r.src.as<u32>());
    } else {
        launch_rate_clear(s, S, r.src.as<u32>(), r.flag.as<u32>());
        const int64_t m = r.kind == SH_RATE_FIRST ? S : E;  // rows the segments cover
        if (m > 0) {
            RCHK(r.skey.reserve((size_t)m * 8, false));
            RCHK(r.skey2.reserve((size_t)m * 8, false));
            RCHK(r.idx.reserve((size_t)m * 4, false));
            RCHK(r.idx2.reserve((size_t)m * 4, false));
            RCHK(r.hd.reserve((size_t)(m + 1) * 4, false));
            RCHK(r.pos.reserve((size_t)(m + 1) * 4, false));
            RCHK(r.starts.reserve((size_t)(m + 1) * 4, false));
            RCHK(r.tmp.reserve((size_t)((m + 1 + kTile - 1) / kTile + 16) * 8, false));
            if (r.pkey) launch_ratep_pkey(s, m, src.keys, plane_out_part(q), r.skey.as<u64>(), r.idx.as<u32>());
            else launch_rate_pack(s, m, src.keys, sstride, nk, r.skey.as<u64>(), r.idx.as<u32>());
            size_t tb = 0;
            if (sort_u64_pairs(nullptr, &tb, nullptr, nullptr, nullptr, nullptr, m, s))
                return sh_fail(SH_ERR_DEVICE, "output rate: sort sizing");
            RCHK(r.sort_tmp.reserve(std::max<size_t>(tb, 16), false));
            if (sort_u64_pairs(r.sort_tmp.p, &tb, r.skey.as<u64>(), r.skey2.as<u64>(), r.idx.as<u32>(),
                               r.idx2.as<u32>(), m, s))
                return sh_fail(SH_ERR_DEVICE, "output rate: sort failed");
            launch_rate_segments(s, m, r.skey2.as<u64>(), r.idx2.as<u32>(), N, r.kind == SH_RATE_LAST ? 1 : 0,
                                 r.hd.as<u32>(), r.pos.as<u32>(), r.starts.as<u32>(), r.tmp.as<i64>());
            if (r.kind == SH_RATE_FIRST) {
                // the table holds distinct keys: size it by the call's segments (its distinct keys,
                // pos[m] after the head scan), not by its rows
                HIPCHK(hipMemcpyAsync(r.h_small.as<char>() + 16, r.pos.as<u32>() + m, 4, hipMemcpyDeviceToHost, s));
                HIPCHK(hipStreamSynchronize(s));
                const int64_t n_seg = *(const uint32_t*)(r.h_small.as<char>() + 16);
                RCHK(grow_table(q, r.t_keys + n_seg));
                RCHK(r.seg_c0.reserve((size_t)m * 8, false));
                RCHK(r.seg_new.reserve((size_t)m * 4, false));
                RCHK(r.n_keys.reserve(16, false));
                HIPCHK(hipMemsetAsync(r.n_keys.p, 0, 4, s));
                launch_rate_first(s, m, r.hd.as<u32>(), r.pos.as<u32>(), r.starts.as<u32>(), r.skey2.as<u64>(),
                                  r.idx2.as<u32>(), N, r.tk.as<u64>(), r.tc.as<i64>(), (u32)(r.t_cap - 1),
                                  r.seg_c0.as<i64>(), r.seg_new.as<u32>(), r.n_keys.as<u32>(), foff, nf, r.flag.as<u32>(),
                                  r.eflush.as<int>());
                HIPCHK(hipMemcpyAsync(r.h_small.as<char>() + 8, r.n_keys.p, 4, hipMemcpyDeviceToHost, s));
            } else {
                launch_rate_last(s, m, r.hd.as<u32>(), r.pos.as<u32>(), r.starts.as<u32>(), r.idx2.as<u32>(), N, nc,
                                 foff, nf, r.flag.as<u32>(), r.src.as<u32>(), r.eflush.as<int>());
            }
        }
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(r.pre.p, r.flag.p, (size_t)(S + 1) * 4, hipMemcpyDeviceToDevice, s));
    launch_scan_sum_large_u32(s, r.pre.as<u32>(), S + 1, r.tmp.as<i64>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(r.h_small.p, r.pre.as<u32>() + S, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const int64_t T = *r.h_small.as<uint32_t>();
    if (r.gb && r.kind == SH_RATE_FIRST && S > 0) r.t_keys += *(uint32_t*)(r.h_small.as<char>() + 8);
    RateRows o{};
    RCHK(reserve_set(r.o_ts, r.o_exp, r.o_rep, r.o_keys, r.o_vals, r.o_nulls, T, nk, na, &o));
    RCHK(r.o_flush.reserve((size_t)std::max<int64_t>(T, 1) * 4, false));
    launch_rate_gather(s, S, r.flag.as<u32>(), r.pre.as<u32>(), r.src.as<u32>(), r.eflush.as<int>(), src, sstride, o, T,
                       nk, na, r.o_flush.as<int>());
    HIPCHK(hipGetLastError());
    // rows of the open group wait for the next call
    if (carries) {
        const int64_t nn = S - E;
        if (nn > 0) {
            RateRows c2{};
            // the new carry is written to the source buffers' twin: stage it in the output-free area first
            DevBuf t_ts, t_exp, t_rep, t_keys, t_vals, t_nulls;
            RCHK(reserve_set(t_ts, t_exp, t_rep, t_keys, t_vals, t_nulls, nn, nk, na, &c2));
            RCHK(copy_rows(s, c2, nn, src, sstride, E, nn, nk, na));
            std::swap(r.c_ts, t_ts);
            std::swap(r.c_exp, t_exp);
            std::swap(r.c_rep, t_rep);
            std::swap(r.c_keys, t_keys);
            std::swap(r.c_vals, t_vals);
            std::swap(r.c_nulls, t_nulls);
        }
        r.nc = nn;
    }
    r.seq += n;
    return rate_finish(q, o, T, nk, na, host_out, out);
}

static unsigned bits_of(int64_t n) {  // bits needed for values < n
    unsigned b = 1;
    while (b < 63 && ((int64_t)1 << b) < n) b++;
    return b;
}

// One limiter per partition instance (PartitionRuntimeImpl clones the query and its OutputRateLimiter):
// `output all / first / last every N events` and `output first every <t>` without group-by run on each
// partition's own row sequence. A flush of the lanes is one chunk of one partition, so the rows a
// flush emits come from one partition; the kept rows leave ordered by their emitting flush.
static int rate_part(sh_query* q, const sh_out* in, const i64* foff, int nf, bool host_out, const sh_out** out) {
    auto& r = q->rate;
    hipStream_t s = q->ctx->stream;
    const int nk = (int)in->n_keys, na = (int)in->n_vals;
    const int64_t n = in->n_rows, N = r.N;
    const u32* in_part = plane_out_part(q);
    const bool carries = r.kind == SH_RATE_ALL || r.lkey;
    const int64_t nc = carries ? r.nc : 0, S = nc + n;
    RateRows inr{(i64*)in->ts, (unsigned char*)in->expired, (i64*)in->rep, (i64*)in->keys, (u64*)in->vals,
                 (unsigned char*)in->nulls};
    RateRows src = inr;
    int64_t sstride = n;
    const u32* sp = in_part;
    if (nc > 0) {
        RCHK(reserve_set(r.s_ts, r.s_exp, r.s_rep, r.s_keys, r.s_vals, r.s_nulls, S, nk, na, &src));
        RateRows car{r.c_ts.as<i64>(), r.c_exp.as<unsigned char>(), r.c_rep.as<i64>(), r.c_keys.as<i64>(),
                     r.c_vals.as<u64>(), r.c_nulls.as<unsigned char>()};
        RCHK(copy_rows(s, src, S, car, nc, 0, nc, nk, na));
        RateRows tail = src;
        tail.ts += nc; tail.expired += nc; tail.rep += nc; tail.keys += nc; tail.vals += nc; tail.nulls += nc;
        RCHK(copy_rows(s, tail, S, inr, n, 0, n, nk, na));
        sstride = S;
        RCHK(r.s_part.reserve((size_t)S * 4, false));
        HIPCHK(hipMemcpyAsync(r.s_part.p, r.c_part.p, (size_t)nc * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(hipMemcpyAsync(r.s_part.as<u32>() + nc, in_part, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
        sp = r.s_part.as<u32>();
    }
    const int64_t m = std::max<int64_t>(S, nf);
    RCHK(r.flag.reserve((size_t)(S + 1) * 4, false));
    RCHK(r.keep.reserve((size_t)(S + 1) * 4, false));
    RCHK(r.pre.reserve((size_t)(S + 1) * 4, false));
    RCHK(r.src.reserve((size_t)std::max<int64_t>(S, 1) * 4, false));
    RCHK(r.eflush.reserve((size_t)std::max<int64_t>(S, 1) * 4, false));
    RCHK(r.tmp.reserve((size_t)((m + 1 + kTile - 1) / kTile + 16) * 8, false));
    RCHK(r.skey.reserve((size_t)std::max<int64_t>(m, 1) * 8, false));
    RCHK(r.skey2.reserve((size_t)std::max<int64_t>(m, 1) * 8, false));
    RCHK(r.idx.reserve((size_t)std::max<int64_t>(m, 1) * 4, false));
    RCHK(r.idx2.reserve((size_t)std::max<int64_t>(m, 1) * 4, false));
    RCHK(r.hd.reserve((size_t)(m + 1) * 4, false));
    RCHK(r.pos.reserve((size_t)(m + 1) * 4, false));
    RCHK(r.starts.reserve((size_t)(m + 1) * 4, false));
    RCHK(r.h_small.reserve(64));
    const unsigned pbits = bits_of(r.nparts + 1);
    size_t tb = 0;
    if (r.kind == SH_RATE_FIRST_TIME) {
        // the partitions' flushes in order, one walker per partition
        RCHK(r.fclk.reserve((size_t)std::max(nf, 1) * 8, false));
        RCHK(r.chosen.reserve((size_t)std::max(nf, 1), false));
        if (nf) HIPCHK(hipMemcpyAsync(r.fclk.p, r.h_clk.data(), (size_t)nf * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemsetAsync(r.chosen.p, 0, (size_t)std::max(nf, 1), s));
        const u32 none = (u32)r.nparts;
        launch_ratep_fparts(s, nf, foff, in_part, none, r.skey.as<u64>(), r.idx.as<u32>());
        if (sort_u64_pairs_bits(nullptr, &tb, r.skey.as<u64>(), nullptr, r.idx.as<u32>(), nullptr, nf, pbits, s))
            return sh_fail(SH_ERR_DEVICE, "output rate: sort sizing");
        RCHK(r.sort_tmp.reserve(std::max<size_t>(tb, 16), false));
        if (sort_u64_pairs_bits(r.sort_tmp.p, &tb, r.skey.as<u64>(), r.skey2.as<u64>(), r.idx.as<u32>(), r.idx2.as<u32>(),
                                nf, pbits, s))
            return sh_fail(SH_ERR_DEVICE, "output rate: sort failed");
        launch_rate_segments(s, nf, r.skey2.as<u64>(), r.idx2.as<u32>(), 1, 0, r.hd.as<u32>(), r.pos.as<u32>(),
                             r.starts.as<u32>(), r.tmp.as<i64>());
        launch_ratep_ftime(s, nf, r.hd.as<u32>(), r.pos.as<u32>(), r.starts.as<u32>(), r.skey2.as<u64>(), r.idx2.as<u32>(),
                           r.fclk.as<i64>(), none, N, r.pft_has.as<unsigned char>(), r.pft_last.as<i64>(),
                           r.chosen.as<unsigned char>());
        launch_rate_ftime_rows(s, S, foff, nf, r.chosen.as<unsigned char>(), r.flag.as<u32>(), r.eflush.as<int>(),
                               r.src.as<u32>());
    } else {
        // every row's ordinal in its partition's sequence (carried rows first)
        launch_ratep_pack(s, S, nc, r.c_part.as<u32>(), in_part, r.skey.as<u64>(), r.idx.as<u32>());
        if (sort_u64_pairs_bits(nullptr, &tb, r.skey.as<u64>(), nullptr, r.idx.as<u32>(), nullptr, S, pbits, s))
            return sh_fail(SH_ERR_DEVICE, "output rate: sort sizing");
        RCHK(r.sort_tmp.reserve(std::max<size_t>(tb, 16), false));
        if (sort_u64_pairs_bits(r.sort_tmp.p, &tb, r.skey.as<u64>(), r.skey2.as<u64>(), r.idx.as<u32>(), r.idx2.as<u32>(),
                                S, pbits, s))
            return sh_fail(SH_ERR_DEVICE, "output rate: sort failed");
        launch_rate_segments(s, S, r.skey2.as<u64>(), r.idx2.as<u32>(), 1, 0, r.hd.as<u32>(), r.pos.as<u32>(),
                             r.starts.as<u32>(), r.tmp.as<i64>());
        if (r.lkey) {
            // windows of N rows per partition; inside a complete one, per group key its last row at its
            // first row's place (LastGroupByPerEventOutputRateLimiter :51-83)
            RCHK(r.lk_ord.reserve((size_t)std::max<int64_t>(S, 1) * 8, false));
            RCHK(r.lk_cidx.reserve((size_t)std::max<int64_t>(S, 1) * 4, false));
            RCHK(r.lk_key.reserve((size_t)std::max<int64_t>(S, 1) * 8, false));
            RCHK(r.lk_key2.reserve((size_t)std::max<int64_t>(S, 1) * 8, false));
            RCHK(r.lk_idx.reserve((size_t)std::max<int64_t>(S, 1) * 4, false));
            RCHK(r.lk_idx2.reserve((size_t)std::max<int64_t>(S, 1) * 4, false));
            launch_ratep_last_keyed(s, S, r.hd.as<u32>(), r.pos.as<u32>(), r.starts.as<u32>(), r.idx2.as<u32>(), N, src.keys,
                                    sstride, sp, r.lk_ord.as<i64>(), r.lk_cidx.as<u32>(), r.keep.as<u32>(),
                                    r.lk_key.as<u64>(), r.lk_idx.as<u32>());
            tb = 0;
            if (sort_u64_pairs(nullptr, &tb, r.lk_key.as<u64>(), nullptr, r.lk_idx.as<u32>(), nullptr, S, s))
                return sh_fail(SH_ERR_DEVICE, "output rate: sort sizing");
            RCHK(r.sort_tmp.reserve(std::max<size_t>(tb, 16), false));
            if (sort_u64_pairs(r.sort_tmp.p, &tb, r.lk_key.as<u64>(), r.lk_key2.as<u64>(), r.lk_idx.as<u32>(),
                               r.lk_idx2.as<u32>(), S, s))
                return sh_fail(SH_ERR_DEVICE, "output rate: sort failed");
            // (src = identity first: only the runs' first rows get another source)
            launch_rate_clear(s, S, r.src.as<u32>(), r.flag.as<u32>());
            launch_ratep_last_keyed_rows(s, S, r.lk_key2.as<u64>(), r.lk_idx2.as<u32>(), r.lk_cidx.as<u32>(),
                                         r.lk_ord.as<i64>(), N, nc, foff, nf, r.hd.as<u32>(), r.pos.as<u32>(),
                                         r.flag.as<u32>(), r.src.as<u32>(), r.eflush.as<int>());
        } else {
            launch_ratep_flags(s, S, r.hd.as<u32>(), r.pos.as<u32>(), r.starts.as<u32>(), r.skey2.as<u64>(),
                               r.idx2.as<u32>(), r.kind, N, nc, r.pseq.as<i64>(), foff, nf, r.flag.as<u32>(),
                               r.eflush.as<int>(), r.src.as<u32>(), r.keep.as<u32>());
        }
    }
    HIPCHK(hipGetLastError());
    // kept rows, ordered by their emitting flush (stable: a group leaves in its own order)
    HIPCHK(hipMemcpyAsync(r.pre.p, r.flag.p, (size_t)(S + 1) * 4, hipMemcpyDeviceToDevice, s));
    launch_scan_sum_large_u32(s, r.pre.as<u32>(), S + 1, r.tmp.as<i64>());
    HIPCHK(hipMemcpyAsync(r.h_small.p, r.pre.as<u32>() + S, 4, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    const int64_t T = *r.h_small.as<uint32_t>();
    const int64_t tc = std::max<int64_t>(T, 1);
    RCHK(r.okey.reserve((size_t)tc * 8, false));
    RCHK(r.okey2.reserve((size_t)tc * 8, false));
    RCHK(r.olist.reserve((size_t)tc * 4, false));
    RCHK(r.olist2.reserve((size_t)tc * 4, false));
    launch_ratep_list(s, S, r.flag.as<u32>(), r.pre.as<u32>(), r.eflush.as<int>(), r.src.as<u32>(), r.okey.as<u64>(),
                      r.olist.as<u32>());
    if (T > 0) {
        const unsigned fbits = bits_of((int64_t)nf + 1);
        tb = 0;
        if (sort_u64_pairs_bits(nullptr, &tb, r.okey.as<u64>(), nullptr, r.olist.as<u32>(), nullptr, T, fbits, s))
            return sh_fail(SH_ERR_DEVICE, "output rate: sort sizing");
        RCHK(r.sort_tmp.reserve(std::max<size_t>(tb, 16), false));
        if (sort_u64_pairs_bits(r.sort_tmp.p, &tb, r.okey.as<u64>(), r.okey2.as<u64>(), r.olist.as<u32>(),
                                r.olist2.as<u32>(), T, fbits, s))
            return sh_fail(SH_ERR_DEVICE, "output rate: sort failed");
    }
    RateRows o{};
    RCHK(reserve_set(r.o_ts, r.o_exp, r.o_rep, r.o_keys, r.o_vals, r.o_nulls, T, nk, na, &o));
    RCHK(r.o_flush.reserve((size_t)tc * 4, false));
    launch_ratep_gather(s, T, r.olist2.as<u32>(), r.okey2.as<u64>(), src, sstride, sp, o, nk, na, r.o_flush.as<int>(),
                        nullptr);
    HIPCHK(hipGetLastError());
    if (carries) {
        // the partitions' open groups wait for their next rows (source order kept)
        HIPCHK(hipMemcpyAsync(r.pre.p, r.keep.p, (size_t)(S + 1) * 4, hipMemcpyDeviceToDevice, s));
        launch_scan_sum_large_u32(s, r.pre.as<u32>(), S + 1, r.tmp.as<i64>());
        HIPCHK(hipMemcpyAsync(r.h_small.as<char>() + 8, r.pre.as<u32>() + S, 4, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        const int64_t nn = *(const uint32_t*)(r.h_small.as<char>() + 8);
        if (nn > 0) {
            RCHK(r.olist.reserve((size_t)nn * 4, false));
            RCHK(r.okey.reserve((size_t)nn * 8, false));
            launch_ratep_list(s, S, r.keep.as<u32>(), r.pre.as<u32>(), r.eflush.as<int>(), nullptr, r.okey.as<u64>(),
                              r.olist.as<u32>());
            RateRows c2{};
            DevBuf t_ts, t_exp, t_rep, t_keys, t_vals, t_nulls;
            RCHK(reserve_set(t_ts, t_exp, t_rep, t_keys, t_vals, t_nulls, nn, nk, na, &c2));
            RCHK(r.t_part.reserve((size_t)nn * 4, false));
            launch_ratep_gather(s, nn, r.olist.as<u32>(), nullptr, src, sstride, sp, c2, nk, na, nullptr, r.t_part.as<u32>());
            HIPCHK(hipGetLastError());
            std::swap(r.c_ts, t_ts);
            std::swap(r.c_exp, t_exp);
            std::swap(r.c_rep, t_rep);
            std::swap(r.c_keys, t_keys);
            std::swap(r.c_vals, t_vals);
            std::swap(r.c_nulls, t_nulls);
            std::swap(r.c_part, r.t_part);
        }
        r.nc = nn;
    }
    r.seq += n;
    return rate_finish(q, o, T, nk, na, host_out, out);
}

// A sharded query's limiter (OutputRateLimiter.process after the selector: it sees the merged
// single-stream output). The merged rows come from the host; they go to the device once and run through
// the same limiter kernels as an unsharded query's output.
extern "C" int sh_rate_apply_merged(sh_query* q, const sh_out* in, const sh_out** out) {
    StreamScope _ss(q && q->ctx ? q->ctx->stream : nullptr);
    if (!q || !in || !out) return sh_fail(SH_ERR_INVALID, "sh_rate_apply_merged: NULL argument");
    if (q->rate.kind == SH_RATE_NONE) return sh_fail(SH_ERR_INVALID, "sh_rate_apply_merged: the query has no output rate");
    if (q->seq > 0 || q->clock_valid)
        return sh_fail(SH_ERR_INVALID, "sh_rate_apply_merged: the limiter's query must never be pushed");
    if (q->wide || q->kind == 1 && q->d.partition_col >= 0)
        return sh_fail(SH_ERR_UNSUPPORTED, "sh_rate_apply_merged: a query the sharded ingest does not run");
    if (in->n_keys != q->kp.n || in->n_vals != q->ap.n || in->n_rows < 0 || in->n_flushes < 0 ||
        (in->n_rows > 0 && (!in->ts || !in->expired || (in->n_keys && !in->keys) || (in->n_vals && (!in->vals || !in->nulls)))))
        return sh_fail(SH_ERR_INVALID, "sh_rate_apply_merged: rows do not match the query's keys / aggregators");
    if (in->n_rows > 0 && (!in->flush_offsets || in->flush_offsets[in->n_flushes] != in->n_rows))
        return sh_fail(SH_ERR_INVALID, "sh_rate_apply_merged: the merged output needs its flush offsets");
    auto& r = q->rate;
    hipStream_t s = q->ctx->stream;
    const int nk = (int)in->n_keys, na = (int)in->n_vals;
    const int64_t n = in->n_rows;
    RateRows d{};
    RCHK(reserve_set(r.m_ts, r.m_exp, r.m_rep, r.m_keys, r.m_vals, r.m_nulls, n, nk, na, &d));
    if (n > 0) {
        HIPCHK(hipMemcpyAsync(d.ts, in->ts, (size_t)n * 8, hipMemcpyHostToDevice, s));
        HIPCHK(hipMemcpyAsync(d.expired, in->expired, (size_t)n, hipMemcpyHostToDevice, s));
        if (in->rep) HIPCHK(hipMemcpyAsync(d.rep, in->rep, (size_t)n * 8, hipMemcpyHostToDevice, s));
        else HIPCHK(hipMemsetAsync(d.rep, 0xFF, (size_t)n * 8, s));
        if (nk) HIPCHK(hipMemcpyAsync(d.keys, in->keys, (size_t)nk * n * 8, hipMemcpyHostToDevice, s));
        if (na) {
            HIPCHK(hipMemcpyAsync(d.vals, in->vals, (size_t)na * n * 8, hipMemcpyHostToDevice, s));
            HIPCHK(hipMemcpyAsync(d.nulls, in->nulls, (size_t)na * n, hipMemcpyHostToDevice, s));
        }
        HIPCHK(hipStreamSynchronize(s));  // (the caller's host arrays may go once this returns)
    }
    sh_out dv = *in;
    dv.ts = d.ts;
    dv.expired = d.expired;
    dv.rep = d.rep;
    dv.keys = d.keys;
    dv.vals = (const uint64_t*)d.vals;
    dv.nulls = d.nulls;
    return rate_apply(q, &dv, false, true, out);
}
