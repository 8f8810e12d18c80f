// sh_plane_kernels.hip — `partition with (p of S)` around lengthBatch(L) and time(T) windows whose
// group key is the partition key (or that have no group-by), on gfx950.
//
// PartitionStreamReceiver.receive (core/partition/PartitionStreamReceiver.java:176-272) cuts every
// send into runs of consecutive events with one partition key and sends each run through the query
// under that partition's flow: the window state (LengthBatchWindowProcessor.WindowState :302-350,
// TimeWindowProcessor.WindowState :196-222) and every aggregator state are per partition. With the
// group key equal to the partition key every selector chunk holds one key, so a partition's whole
// behaviour is a sequential walk over its own events (and, for time windows, its TIMER calls):
// one lane per partition replays exactly the reference's per-partition sequence.
#include "sh_device.h"
#include "sh_sliding.h"

namespace shd {

namespace {

__device__ __forceinline__ bool p_worse(int kind, u64 cur, u64 v) {
    switch (kind) {
        case AK_MIN_L: return (i64)cur > (i64)v;
        case AK_MAX_L: return (i64)cur < (i64)v;
        case AK_MIN_D: return __longlong_as_double((i64)cur) > __longlong_as_double((i64)v);
        case AK_MAX_D: return __longlong_as_double((i64)cur) < __longlong_as_double((i64)v);
        case AK_MIN_F: return (float)__longlong_as_double((i64)cur) > (float)__longlong_as_double((i64)v);
        default: return (float)__longlong_as_double((i64)cur) < (float)__longlong_as_double((i64)v);
    }
}

__device__ __forceinline__ bool p_eq(int kind, u64 a, u64 b) {
    if (kind == AK_MIN_L || kind == AK_MAX_L) return a == b;
    const double x = __longlong_as_double((i64)a), y = __longlong_as_double((i64)b);
    if (kind == AK_MIN_F || kind == AK_MAX_F) {
        const float fx = (float)x, fy = (float)y;
        if (fx != fx && fy != fy) return true;
        return __float_as_uint(fx) == __float_as_uint(fy);
    }
    if (x != x && y != y) return true;
    return a == b;
}

__device__ __forceinline__ double p_num(const AggPlan& ap, int a, u64 x) {
    return (ap.kind[a] == AK_AVG && !is_fp(ap.vcol_type[ap.vcol[a]])) ? (double)(i64)x : __longlong_as_double((i64)x);
}

// the row of a chunk: aggregates of the lane's state (count / sum / avg / min / max; null at count 0)
template <int NA>
__device__ __forceinline__ void p_row_vals(const AggPlan& ap, i64 cnt, const u64 (&f)[NA], const u64 (&mm)[NA],
                                           const unsigned char (&mmh)[NA], u64 (&rv)[NA], unsigned char (&rn)[NA]) {
#pragma unroll
    for (int a = 0; a < NA; a++) {
        rv[a] = 0;
        rn[a] = 0;
        if (a >= ap.n) continue;
        const int kind = ap.kind[a];
        if (kind == AK_COUNT) rv[a] = (u64)cnt;
        else if (kind == AK_SUM_L || kind == AK_SUM_D) { rn[a] = cnt == 0; rv[a] = cnt == 0 ? 0 : f[a]; }
        else if (kind == AK_AVG) {
            rn[a] = cnt == 0;
            if (cnt) rv[a] = (u64)__double_as_longlong(__longlong_as_double((i64)f[a]) / (double)cnt);
        } else { rn[a] = mmh[a] ? 0 : 1; rv[a] = mmh[a] ? mm[a] : 0; }
    }
}

template <int NA>
__device__ __forceinline__ void p_write_row(SlxRows rows, const AggPlan& ap, i64 pos, i64 ts, i64 rep, u32 slot, i64 clk,
                                            unsigned char exp, const u64 (&rv)[NA], const unsigned char (&rn)[NA]) {
    rows.ts[pos] = ts;
    rows.rep[pos] = rep;
    rows.slot[pos] = slot;
    rows.ch[pos] = pos;
    rows.clk[pos] = clk;
    rows.exp[pos] = exp;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (a < ap.n) {
            rows.vals[(size_t)a * rows.cap + pos] = rv[a];
            rows.nulls[(size_t)a * rows.cap + pos] = rn[a];
        }
    }
}

}  // namespace

// ---- partitioned lengthBatch(L): one lane per partition. The open batch is a running fold (a batch
// is add-only: RESET before its events, LengthBatchWindowProcessor.processFullBatchEvents :206-243);
// the batch completed by a partition's L-th event is its own flush (one chunk per completed batch),
// at that event's position in the stream. With expired output the chunk begins with the previous
// batch's events as EXPIRED: the key's row then is that batch removed again (count 0, the others
// null), re-stamped with the flush clock and represented by its last event — unless current events
// follow, whose row replaces it (LinkedHashMap.put keeps one row per key). ----------------------------
//
// lengthBatch(L, true) (stream.current.event, processStreamCurrentEvents :245-274): every event is a chunk
// of its own and emits the partition's running aggregates; the (L + 1)-th event of a batch starts the
// next one — its chunk is [the previous batch's events as EXPIRED, RESET, the event], and the selector
// without group-by (or grouped by the partition key: one key) keeps the chunk's last qualifying event
// (processInBatchNoGroupBy :271-313): the current one, or with `insert expired events` the batch's last
// event removed again (count 0, the others null, stamped with the send's clock).
template <int NA, int NV>
__global__ __launch_bounds__(64) void k_pl_walk_lb(const u32* __restrict__ key_off, const u32* __restrict__ sorted_rank,
                                                   u32 nslots, SlRecords rec, i64 L, i64 seq_base, SlState S,
                                                   i64* last_ts, i64* last_seq, i64* prev_seq, AggPlan ap, int cur_on,
                                                   int exp_on, int sc, SlxRows rows, unsigned char* flags) {
    const u32 k = blockIdx.x * 64 + threadIdx.x;
    if (k >= nslots) return;
    const u32 lo = key_off[k], hi = key_off[k + 1];
    if (lo == hi) return;
    i64 cnt = S.cnt[k], lts = last_ts[k], lseq = last_seq[k], pseq = prev_seq[k];
    u64 f[NA], mm[NA];
    unsigned char mmh[NA];
#pragma unroll
    for (int a = 0; a < NA; a++) {
        f[a] = 0; mm[a] = 0; mmh[a] = 0;
        if (a >= ap.n || ap.kind[a] == AK_COUNT) continue;
        const size_t fi = (size_t)ap.field[a] * S.nslots + k;
        f[a] = S.f[fi];
        if (ap.kind[a] >= AK_MIN_L) { mm[a] = S.mm[fi]; mmh[a] = S.mm_has[fi]; }
    }
    for (u32 i = lo; i < hi; i++) {
        const u32 r = sorted_rank[i];
        const bool newb = sc && cnt == L;  // (stream.current) this event starts the next batch
        if (newb) cnt = 0;
        if (cnt == 0) {  // RESET: the batch starts from fresh states
#pragma unroll
            for (int a = 0; a < NA; a++) { f[a] = 0; mm[a] = 0; mmh[a] = 0; }
        }
        cnt++;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            if (a >= ap.n) continue;
            const int kind = ap.kind[a];
            if (kind == AK_COUNT) continue;
            u64 x = rec.vals[r];
#pragma unroll
            for (int q = 1; q < NV; q++)
                if (ap.vcol[a] == q) x = rec.vals[(size_t)q * rec.cap + r];
            if (kind == AK_SUM_L) f[a] = (u64)((i64)f[a] + (i64)x);
            else if (kind == AK_SUM_D || kind == AK_AVG)
                f[a] = (u64)__double_as_longlong(__longlong_as_double((i64)f[a]) + p_num(ap, a, x));
            else {
                const bool take = !mmh[a] || p_worse(kind, mm[a], x);
                mm[a] = take ? x : mm[a];
                mmh[a] = 1;
            }
        }
        lts = rec.ts[r];
        if (sc) {
            u64 rv[NA];
            unsigned char rn[NA];
            if (cur_on) {
                p_row_vals<NA>(ap, cnt, f, mm, mmh, rv, rn);
                p_write_row<NA>(rows, ap, r, lts, seq_base + (i64)rec.raw[r], k, rec.clock[r], 0, rv, rn);
                flags[r] = 1;
            } else if (newb) {
                const u64 z[NA] = {};
                const unsigned char zh[NA] = {};
                p_row_vals<NA>(ap, 0, z, z, zh, rv, rn);
                p_write_row<NA>(rows, ap, r, rec.clock[r], lseq, k, rec.clock[r], 1, rv, rn);
                flags[r] = 1;
            }
            lseq = seq_base + (i64)rec.raw[r];
            continue;
        }
        lseq = seq_base + (i64)rec.raw[r];
        if (cnt == L) {
            u64 rv[NA];
            unsigned char rn[NA];
            if (cur_on) {
                p_row_vals<NA>(ap, cnt, f, mm, mmh, rv, rn);
                p_write_row<NA>(rows, ap, r, lts, lseq, k, rec.clock[r], 0, rv, rn);
                flags[r] = 1;
            } else if (pseq >= 0) {
                const u64 z[NA] = {};
                const unsigned char zh[NA] = {};
                p_row_vals<NA>(ap, 0, z, z, zh, rv, rn);
                p_write_row<NA>(rows, ap, r, rec.clock[r], pseq, k, rec.clock[r], 1, rv, rn);
                flags[r] = 1;
            }
            pseq = exp_on ? lseq : -1;
            cnt = 0;
        }
    }
    S.cnt[k] = cnt;
    last_ts[k] = lts;
    last_seq[k] = lseq;
    prev_seq[k] = pseq;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (a >= ap.n || ap.kind[a] == AK_COUNT) continue;
        const size_t fi = (size_t)ap.field[a] * S.nslots + k;
        S.f[fi] = f[a];
        if (ap.kind[a] >= AK_MIN_L) { S.mm[fi] = mm[a]; S.mm_has[fi] = mmh[a]; }
    }
}

void launch_pl_walk_lb(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, SlRecords rec, i64 L,
                       i64 seq_base, SlState S, i64* last_ts, i64* last_seq, i64* prev_seq, AggPlan ap, int cur_on,
                       int exp_on, int sc, SlxRows rows, unsigned char* flags) {
    const unsigned grid = (unsigned)((nslots + 63) / 64);
    if (!grid) return;
#define SH_PL_LB(A, V)                                                                                               \
    hipLaunchKernelGGL((k_pl_walk_lb<A, V>), dim3(grid), dim3(64), 0, s, key_off, sorted_rank, (u32)nslots, rec, L,  \
                       seq_base, S, last_ts, last_seq, prev_seq, ap, cur_on, exp_on, sc, rows, flags)
    const int nv = ap.n_vcols < 1 ? 1 : ap.n_vcols;
    if (ap.n <= 4 && nv <= 1) SH_PL_LB(4, 1);
    else if (nv <= 2) SH_PL_LB(8, 2);
    else SH_PL_LB(8, 8);
#undef SH_PL_LB
}

// ---- runs: an event starts a run at a send's first event or where the partition key changes
// (PartitionStreamReceiver.receive :176-213 over every event of the send, filtered or not) --------------
__global__ __launch_bounds__(kBlock) void k_pl_run_start(ColSet cols, int pcol, i64 N, i64 send_size,
                                                        unsigned char* start) {
    const i64 e = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (e >= N) return;
    const i64 sl = send_size > 0 ? send_size : N;
    // (the partitions' String.valueOf equality: float / double keys by their bits, every NaN one key)
    auto key = [&](i64 i) -> i64 {
        const i64 v = load_raw(cols, pcol, i);
        return (is_fp(cols.type[pcol]) && __longlong_as_double(v) != __longlong_as_double(v)) ? 0x7FF8000000000000ll : v;
    };
    start[e] = (e % sl == 0) || key(e) != key(e - 1);
}

// run number of every event: inclusive count of run starts - 1 (tile prefix from launch_scan_sum)
__global__ __launch_bounds__(kBlock) void k_pl_run_id(const unsigned char* __restrict__ start, i64 N,
                                                     const i64* __restrict__ blk_pre, i64* run) {
    const i64 tile = (i64)blockIdx.x * kTile;
    i64 acc = blk_pre[blockIdx.x];
    for (int it = 0; it < kItems; it++) {
        const i64 e = tile + (i64)it * kBlock + threadIdx.x;
        const i64 v = e < N ? start[e] : 0;
        i64 tot;
        const i64 ex = block_excl_scan(v, SumOp(), 0, &tot);
        if (e < N) run[e] = acc + ex + v - 1;
        acc += tot;
    }
}

__global__ __launch_bounds__(kBlock) void k_pl_count(const unsigned char* __restrict__ f, i64 n, i64* blk) {
    const i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 c = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++)
        if (base + i < n) c += f[base + i];
    const i64 t = block_reduce(c, SumOp(), 0);
    if (threadIdx.x == 0) blk[blockIdx.x] = t;
}

void launch_pl_runs(hipStream_t s, ColSet cols, int pcol, i64 N, i64 send_size, unsigned char* start, i64* blk,
                    i64* run) {
    if (N <= 0) return;
    const int nb = (int)((N + kTile - 1) / kTile);
    hipLaunchKernelGGL(k_pl_run_start, dim3((unsigned)((N + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, cols, pcol, N,
                       send_size, start);
    hipLaunchKernelGGL(k_pl_count, dim3(nb), dim3(kBlock), 0, s, start, N, blk);
    launch_scan_sum(s, blk, nb);
    hipLaunchKernelGGL(k_pl_run_id, dim3(nb), dim3(kBlock), 0, s, start, N, blk, run);
}

// ---- the partition key of every slot, as sh_out reports it (int64 widening): the host names the
// partition String.valueOf(key) for the Scheduler's HashMap order (sh_jmap.h). Every event of a slot
// carries the same key, so concurrent stores write one value -------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_pl_slot_key(ColSet cols, KeyPlan kp, KeyTable kt, i64 N, i64* slot_key) {
    const i64 e = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (e >= N) return;
    const u64 key = make_key(kp, cols, e);
    i64 v;
    unpack_key(kp, key, &v, 0);
    slot_key[key_slot(kt, key)] = v;
}

// externalTime lanes: every record's timestamp attribute
__global__ __launch_bounds__(kBlock) void k_pl_xattr(ColSet cols, int xcol, const u32* __restrict__ raw, i64 M, i64* x) {
    const i64 r = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (r < M) x[r] = load_raw(cols, xcol, raw[r]);
}

void launch_pl_xattr(hipStream_t s, ColSet cols, int xcol, const u32* raw, i64 M, i64* x) {
    if (M > 0) hipLaunchKernelGGL(k_pl_xattr, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, cols, xcol, raw, M, x);
}

void launch_pl_slot_key(hipStream_t s, ColSet cols, KeyPlan kp, KeyTable kt, i64 N, i64* slot_key) {
    if (N <= 0) return;
    hipLaunchKernelGGL(k_pl_slot_key, dim3((unsigned)((N + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, cols, kp, kt, N,
                       slot_key);
}

// ---- notify registrations of partitioned time windows: Scheduler.notifyAt(ts + T) whenever an event
// raises its partition's lastTimestamp (TimeWindowProcessor :157-160) -----------------------------------
__global__ __launch_bounds__(64) void k_pl_notify(const u32* __restrict__ key_off, const u32* __restrict__ sorted_rank,
                                                 u32 nslots, const i64* __restrict__ ts, i64* last_ts,
                                                 unsigned char* reg) {
    const u32 k = blockIdx.x * 64 + threadIdx.x;
    if (k >= nslots) return;
    const u32 lo = key_off[k], hi = key_off[k + 1];
    if (lo == hi) return;
    i64 lt = last_ts[k];
    for (u32 i = lo; i < hi; i++) {
        const u32 r = sorted_rank[i];
        const i64 t = ts[r];
        reg[r] = t > lt;
        lt = max(lt, t);
    }
    last_ts[k] = lt;
}

void launch_pl_notify(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, const i64* ts, i64* last_ts,
                      unsigned char* reg) {
    const unsigned grid = (unsigned)((nslots + 63) / 64);
    if (grid) hipLaunchKernelGGL(k_pl_notify, dim3(grid), dim3(64), 0, s, key_off, sorted_rank, (u32)nslots, ts, last_ts, reg);
}

// ---- partitioned time(T): one lane per partition merges its TIMER calls (the calls where the
// scheduler fires its notify times, host-simulated) with its events. At every point the partition's
// queue head expires while ts + T <= now (re-stamped with now, inserted before the event); each run of
// the partition's events is one chunk, each TIMER call another. Positions (= output order):
// timer t (calls sorted by send) at K_t + t, record r at r + #timers at calls <= its send. --------------
template <int NA, int NV>
__global__ __launch_bounds__(64) void k_pl_walk_tm(const u32* __restrict__ key_off, const u32* __restrict__ sorted_rank,
                                                   u32 nslots, SlRecords rec, const i64* __restrict__ run, i64 T,
                                                   i64 seq_base, i64 send_size, const i64* __restrict__ t_off,
                                                   const i64* __restrict__ t_send, const i64* __restrict__ t_clk,
                                                   const i64* __restrict__ t_pos, const i64* __restrict__ f_send,
                                                   i64 nF, SlState S, i64* rseq, AggPlan ap, int cur_on, int exp_on,
                                                   SlxRows rows, unsigned char* flags, const i64* __restrict__ xattr) {
    const u32 k = blockIdx.x * 64 + threadIdx.x;
    if (k >= nslots) return;
    const u32 lo = key_off[k], hi = key_off[k + 1];
    const i64 tlo = t_off ? t_off[k] : 0, thi = t_off ? t_off[k + 1] : 0;
    if (lo == hi && tlo == thi) return;
    const i64 rc = S.rc, rm = rc - 1;
    i64 rh = S.rhead[k], rlen = S.rlen[k], cnt = S.cnt[k];
    u64 f[NA], mm[NA];
    unsigned char mmh[NA];
    i64 dqh[NA], dql[NA];
#pragma unroll
    for (int a = 0; a < NA; a++) {
        f[a] = 0; mm[a] = 0; mmh[a] = 0; dqh[a] = 0; dql[a] = 0;
        if (a >= ap.n || ap.kind[a] == AK_COUNT) continue;
        const size_t fi = (size_t)ap.field[a] * S.nslots + k;
        f[a] = S.f[fi];
        if (ap.kind[a] >= AK_MIN_L) {
            mm[a] = S.mm[fi]; mmh[a] = S.mm_has[fi]; dqh[a] = S.dq_head[fi]; dql[a] = S.dq_len[fi];
        }
    }
    i64 row_pos = -1, row_ts = 0, row_rep = 0, row_clk = 0;
    unsigned char row_exp = 0;
    u64 rv[NA];
    unsigned char rn[NA];
#pragma unroll
    for (int a = 0; a < NA; a++) { rv[a] = 0; rn[a] = 0; }
    u32 i = lo;
    i64 t = tlo;
    i64 cur_run = -1, run_pos = 0;
    while (i < hi || t < thi) {
        const i64 rsend = i < hi ? (send_size > 0 ? (i64)rec.raw[sorted_rank[i]] / send_size : 0) : INT64_MAX;
        const bool timer = t < thi && t_send[t] <= rsend;
        i64 now, pos, clk;
        u32 r = 0;
        if (timer) {
            now = t_clk[t];
            pos = t_pos[t];
            clk = now;
        } else {
            r = sorted_rank[i];
            clk = rec.clock[r];
            // externalTime (ExternalTimeWindowProcessor :126-161): `now` is the event's attribute
            now = xattr ? xattr[r] : clk;
            const i64 rn_ = run[rec.raw[r]];
            if (rn_ != cur_run) {
                cur_run = rn_;
                // f_send: sends of the global timer list (ascending); timers at calls <= this send precede
                i64 lo2 = 0, hi2 = nF;
                while (lo2 < hi2) {
                    const i64 m = (lo2 + hi2) >> 1;
                    if (f_send[m] <= rsend) lo2 = m + 1;
                    else hi2 = m;
                }
                run_pos = (i64)r + lo2;
            }
            pos = run_pos;
        }
        if (pos != row_pos && row_pos >= 0 && flags[row_pos]) {
            p_write_row<NA>(rows, ap, row_pos, row_ts, row_rep, k, row_clk, row_exp, rv, rn);
        }
        if (pos != row_pos) row_pos = pos;
        // expiry of the queue head (TimeWindowProcessor :137-149)
        while (rlen > 0) {
            const i64 sl = rh & rm;
            const i64 hts = S.rpm[(size_t)k * rc + sl];
            if (hts - now + T > 0) break;
            u64 v[NV];
#pragma unroll
            for (int q = 0; q < NV; q++) v[q] = q < ap.n_vcols ? S.rval[((size_t)q * S.nslots + k) * rc + sl] : 0;
            const i64 seq = rseq[(size_t)k * rc + sl];
            rh++;
            rlen--;
            cnt--;
#pragma unroll
            for (int a = 0; a < NA; a++) {
                if (a >= ap.n) continue;
                const int kind = ap.kind[a];
                if (kind == AK_COUNT) continue;
                u64 x = v[0];
#pragma unroll
                for (int q = 1; q < NV; q++)
                    if (ap.vcol[a] == q) x = v[q];
                if (kind == AK_SUM_L) {
                    f[a] = (u64)java_d2l((double)(i64)f[a] - (double)(i64)x);
                } else if (kind == AK_SUM_D || kind == AK_AVG) {
                    double rr = __longlong_as_double((i64)f[a]) - p_num(ap, a, x);
                    if (cnt == 0 && rr == 0.0) rr = 0.0;
                    f[a] = (u64)__double_as_longlong(rr);
                } else {
                    u64* d = S.dq + ((size_t)ap.field[a] * S.nslots + k) * rc;
                    const i64 h = dqh[a];
                    i64 len = dql[a], found = -1;
                    for (i64 j = 0; j < len; j++)
                        if (p_eq(kind, d[(h + j) & rm], x)) { found = j; break; }
                    if (found == 0) { dqh[a] = h + 1; len--; }
                    else if (found > 0) {
                        for (i64 j = found; j + 1 < len; j++) d[(h + j) & rm] = d[(h + j + 1) & rm];
                        len--;
                    }
                    dql[a] = len;
                    mm[a] = len > 0 ? d[dqh[a] & rm] : 0;
                    mmh[a] = len > 0 ? 1 : 0;
                }
            }
            if (exp_on) {
                p_row_vals<NA>(ap, cnt, f, mm, mmh, rv, rn);
                row_ts = now;
                row_rep = seq;
                row_clk = clk;
                row_exp = 1;
                flags[pos] = 1;
            }
        }
        if (timer) {
            t++;
            continue;
        }
        // the event joins the queue (TimeWindowProcessor :150-163) and the aggregators
        {
            u64 v[NV];
#pragma unroll
            for (int q = 0; q < NV; q++) v[q] = q < ap.n_vcols ? rec.vals[(size_t)q * rec.cap + r] : 0;
            const i64 sl = (rh + rlen) & rm;
            S.rpm[(size_t)k * rc + sl] = xattr ? xattr[r] : rec.ts[r];
            rseq[(size_t)k * rc + sl] = seq_base + (i64)rec.raw[r];
#pragma unroll
            for (int q = 0; q < NV; q++)
                if (q < ap.n_vcols) S.rval[((size_t)q * S.nslots + k) * rc + sl] = v[q];
            rlen++;
            cnt++;
#pragma unroll
            for (int a = 0; a < NA; a++) {
                if (a >= ap.n) continue;
                const int kind = ap.kind[a];
                if (kind == AK_COUNT) continue;
                u64 x = v[0];
#pragma unroll
                for (int q = 1; q < NV; q++)
                    if (ap.vcol[a] == q) x = v[q];
                if (kind == AK_SUM_L) f[a] = (u64)((i64)f[a] + (i64)x);
                else if (kind == AK_SUM_D || kind == AK_AVG)
                    f[a] = (u64)__double_as_longlong(__longlong_as_double((i64)f[a]) + p_num(ap, a, x));
                else {
                    u64* d = S.dq + ((size_t)ap.field[a] * S.nslots + k) * rc;
                    const i64 h = dqh[a];
                    i64 len = dql[a];
                    while (len > 0 && p_worse(kind, d[(h + len - 1) & rm], x)) len--;
                    d[(h + len) & rm] = x;
                    dql[a] = len + 1;
                    // minValue = value when strictly better (MinAttributeAggregatorExecutor.processAdd :187):
                    // the deque's front except past a NaN, which no comparison pops
                    const bool take = !mmh[a] || p_worse(kind, mm[a], x);
                    mm[a] = take ? x : mm[a];  // (a select: see k_slx_walk)
                    mmh[a] = 1;
                }
            }
            if (cur_on) {
                p_row_vals<NA>(ap, cnt, f, mm, mmh, rv, rn);
                row_ts = rec.ts[r];
                row_rep = seq_base + (i64)rec.raw[r];
                row_clk = clk;
                row_exp = 0;
                flags[pos] = 1;
            }
            i++;
        }
    }
    if (row_pos >= 0 && flags[row_pos]) p_write_row<NA>(rows, ap, row_pos, row_ts, row_rep, k, row_clk, row_exp, rv, rn);
    S.cnt[k] = cnt;
    S.rhead[k] = rh;
    S.rlen[k] = rlen;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (a >= ap.n || ap.kind[a] == AK_COUNT) continue;
        const size_t fi = (size_t)ap.field[a] * S.nslots + k;
        S.f[fi] = f[a];
        if (ap.kind[a] >= AK_MIN_L) {
            S.mm[fi] = mm[a]; S.mm_has[fi] = mmh[a]; S.dq_head[fi] = dqh[a]; S.dq_len[fi] = dql[a];
        }
    }
}

void launch_pl_walk_tm(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, SlRecords rec,
                       const i64* run, i64 T, i64 seq_base, i64 send_size, const i64* t_off, const i64* t_send,
                       const i64* t_clk, const i64* t_pos, const i64* f_send, i64 nF, SlState S, i64* rseq, AggPlan ap,
                       int cur_on, int exp_on, SlxRows rows, unsigned char* flags, const i64* xattr) {
    const unsigned grid = (unsigned)((nslots + 63) / 64);
    if (!grid) return;
#define SH_PL_TM(A, V)                                                                                               \
    hipLaunchKernelGGL((k_pl_walk_tm<A, V>), dim3(grid), dim3(64), 0, s, key_off, sorted_rank, (u32)nslots, rec, run, \
                       T, seq_base, send_size, t_off, t_send, t_clk, t_pos, f_send, nF, S, rseq, ap, cur_on, exp_on,  \
                       rows, flags, xattr)
    const int nv = ap.n_vcols < 1 ? 1 : ap.n_vcols;
    if (ap.n <= 4 && nv <= 1) SH_PL_TM(4, 1);
    else if (nv <= 2) SH_PL_TM(8, 2);
    else SH_PL_TM(8, 8);
#undef SH_PL_TM
}

// ---- emission: one row per flagged position, each its own flush; output keys from the slot (nk = 0:
// no group-by, the partition key is internal) -----------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_pl_emit(const unsigned char* __restrict__ flags, i64 n,
                                                   const i64* __restrict__ blk_pre, SlxRows rows, int n_aggs, int nk,
                                                   KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys,
                                                   u64* out_vals, unsigned char* out_nulls, unsigned char* out_exp,
                                                   i64* out_ch, i64* out_clock, i64* out_rep, u32* out_part) {
    const i64 tile = (i64)blockIdx.x * kTile;
    i64 acc = blk_pre[blockIdx.x];
    for (int it = 0; it < kItems; it++) {
        const i64 j = tile + (i64)it * kBlock + threadIdx.x;
        const i64 fl = j < n ? flags[j] : 0;
        i64 tot;
        const i64 r = acc + block_excl_scan(fl, SumOp(), 0, &tot);
        acc += tot;
        if (!fl) continue;
        out_ts[r] = rows.ts[j];
        if (nk > 0) unpack_key(kp, slot_key(kt, rows.slot[j]), out_keys + r, out_cap);
        for (int a = 0; a < n_aggs; a++) {
            out_vals[(size_t)a * out_cap + r] = rows.vals[(size_t)a * rows.cap + j];
            out_nulls[(size_t)a * out_cap + r] = rows.nulls[(size_t)a * rows.cap + j];
        }
        out_exp[r] = rows.exp[j];
        out_ch[r] = j;
        out_clock[r] = rows.clk[j];
        out_rep[r] = rows.rep[j];
        out_part[r] = rows.slot[j];
    }
}

void launch_pl_emit(hipStream_t s, const unsigned char* flags, i64 n, const i64* blk_pre, int nblk, SlxRows rows,
                    int n_aggs, int nk, KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals,
                    unsigned char* out_nulls, unsigned char* out_exp, i64* out_ch, i64* out_clock, i64* out_rep,
                    u32* out_part) {
    if (nblk <= 0) return;
    hipLaunchKernelGGL(k_pl_emit, dim3(nblk), dim3(kBlock), 0, s, flags, n, blk_pre, rows, n_aggs, nk, kt, kp, out_cap,
                       out_ts, out_keys, out_vals, out_nulls, out_exp, out_ch, out_clock, out_rep, out_part);
}

}  // namespace shd
