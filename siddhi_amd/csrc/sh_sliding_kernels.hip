// sh_sliding_kernels.hip — gfx950 kernels of the sliding `#window.time(T)` group-by path.
//
// TimeWindowProcessor.process (core/query/processor/stream/window/TimeWindowProcessor.java:132-169)
// expires, before each event, the longest queue prefix whose events satisfy ts + T <= now. For the
// j-th passing event that prefix condition is PM(j) + T <= clock, PM(j) = max ts of passing events
// 0..j. Per key, an expiry only has to be applied before the key's next add (its state is only
// observed at its own events), so each key's window is a ring of (value, PM) and expiry is applied
// lazily when the key is next touched. Aggregators run in SLIDE mode: sums with Java's sequential
// add/remove (residue included), min/max with the reference's monotone deque and its
// removeFirstOccurrence(value) quirk (MinAttributeAggregatorExecutor.java:170-205).
#include "sh_device.h"
#include "sh_sliding.h"

namespace shd {

// ------------------------------------------------------------------------------------------------
// s_blockagg: per workgroup pass count, max send-last ts, max ts over passing events.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_sl_blockagg(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                       WinParams wp, i64* blk_pass, i64* blk_tl, i64* blk_pm) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 cnt = 0, tl = INT64_MIN, pm = INT64_MIN;
    bool pass[kItems];
    filter_items(f, cols, base, wp.N, pass);
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        if (e < wp.N) {
            i64 t = ts[e];
            if (pass[i]) { cnt++; pm = max(pm, t); }
            if (is_send_last(wp, e)) tl = max(tl, t);
        }
    }
    i64 c = block_reduce(cnt, SumOp(), 0);
    i64 t = block_reduce(tl, MaxOp(), INT64_MIN);
    i64 p = block_reduce(pm, MaxOp(), INT64_MIN);
    if (threadIdx.x == 0) { blk_pass[blockIdx.x] = c; blk_tl[blockIdx.x] = t; blk_pm[blockIdx.x] = p; }
}

__global__ __launch_bounds__(1024) void k_sl_scan(i64* blk_pass, i64* blk_tl, i64* blk_pm, int nblk, SlInfo* info) {
    __shared__ i64 a[1024], b[1024], c[1024];
    int t = threadIdx.x;
    int per = (nblk + 1023) / 1024;
    int lo = t * per, hi = min(nblk, lo + per);
    i64 s = 0, m = INT64_MIN, p = INT64_MIN;
    for (int i = lo; i < hi; i++) { s += blk_pass[i]; m = max(m, blk_tl[i]); p = max(p, blk_pm[i]); }
    a[t] = s; b[t] = m; c[t] = p;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        i64 x = t >= d ? a[t - d] : 0, y = t >= d ? b[t - d] : INT64_MIN, z = t >= d ? c[t - d] : INT64_MIN;
        __syncthreads();
        a[t] += x; b[t] = max(b[t], y); c[t] = max(c[t], z);
        __syncthreads();
    }
    i64 rs = t ? a[t - 1] : 0, rm = t ? b[t - 1] : INT64_MIN, rp = t ? c[t - 1] : INT64_MIN;
    for (int i = lo; i < hi; i++) {
        i64 x = blk_pass[i], y = blk_tl[i], z = blk_pm[i];
        blk_pass[i] = rs; blk_tl[i] = rm; blk_pm[i] = rp;
        rs += x; rm = max(rm, y); rp = max(rp, z);
    }
    if (t == 1023) { info->total_pass = a[1023]; info->max_tl = b[1023]; info->max_pm = c[1023]; }
}

void launch_sl_prefix(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp, i64* blk_pass,
                      i64* blk_tl, i64* blk_pm, int nblk, SlInfo* info) {
    hipLaunchKernelGGL(k_sl_blockagg, dim3(nblk), dim3(kBlock), 0, s, ts, cols, f, wp, blk_pass, blk_tl, blk_pm);
    hipLaunchKernelGGL(k_sl_scan, dim3(1), dim3(1024), 0, s, blk_pass, blk_tl, blk_pm, nblk, info);
}

// ------------------------------------------------------------------------------------------------
// s_records: passing events -> rank-indexed records {raw idx, slot, clock, PM, ts, values} and the
// per-slot count of new events (for ring sizing).
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_sl_records(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                      WinParams wp, KeyPlan kp, KeyTable kt, AggPlan ap,
                                                      const i64* blk_pass_pre, const i64* blk_tl_pre,
                                                      const i64* blk_pm_pre, i64 pm0, SlRecords rec, u32* slot_cnt) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    bool pass[kItems];
    i64 cnt = 0, tl = INT64_MIN, pm = INT64_MIN;
    filter_items(f, cols, base, wp.N, pass);
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        if (e < wp.N) {
            i64 t = ts[e];
            cnt += pass[i];
            if (pass[i]) pm = max(pm, t);
            if (is_send_last(wp, e)) tl = max(tl, t);
        }
    }
    i64 r = block_excl_scan(cnt, SumOp(), 0, nullptr) + blk_pass_pre[blockIdx.x];
    i64 cm = max(block_excl_scan(tl, MaxOp(), INT64_MIN, nullptr), blk_tl_pre[blockIdx.x]);
    i64 pmx = max(max(block_excl_scan(pm, MaxOp(), INT64_MIN, nullptr), blk_pm_pre[blockIdx.x]), pm0);
    const i64 c0 = wp.clock_valid ? wp.clock0 : INT64_MIN;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        if (e >= wp.N) break;
        i64 t = ts[e];
        if (pass[i]) {
            pmx = max(pmx, t);
            i64 clk = max(c0, max(cm, ts[send_last_of(wp, e)]));
            u32 pos = key_slot(kt, make_key(kp, cols, e));
            rec.raw[r] = (u32)e;
            rec.slot[r] = pos;
            rec.clock[r] = clk;
            rec.pm[r] = pmx;
            rec.ts[r] = t;
            for (int j = 0; j < ap.n_vcols; j++) rec.vals[(size_t)j * rec.cap + r] = (u64)load_raw(cols, ap.vcol_src[j], e);
            atomicAdd(&slot_cnt[pos], 1u);
            r++;
        }
        if (is_send_last(wp, e)) cm = max(cm, t);
    }
}

void launch_sl_records(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp, KeyPlan kp,
                       KeyTable kt, AggPlan ap, const i64* blk_pass_pre, const i64* blk_tl_pre, const i64* blk_pm_pre,
                       i64 pm0, SlRecords rec, u32* slot_cnt, int nblk) {
    hipLaunchKernelGGL(k_sl_records, dim3(nblk), dim3(kBlock), 0, s, ts, cols, f, wp, kp, kt, ap, blk_pass_pre,
                       blk_tl_pre, blk_pm_pre, pm0, rec, slot_cnt);
}

// max over slots of (ring length + new events): the ring capacity this push needs
__global__ __launch_bounds__(kBlock) void k_sl_need(const u32* slot_cnt, const i64* rlen, i64 n, i64* out) {
    i64 m = 0;
    for (i64 i = (i64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (i64)gridDim.x * kBlock)
        if (slot_cnt[i]) m = max(m, rlen[i] + (i64)slot_cnt[i]);
    i64 t = block_reduce(m, MaxOp(), 0);
    if (threadIdx.x == 0) atomicMax((unsigned long long*)out, (unsigned long long)t);
}

void launch_sl_need(hipStream_t s, const u32* slot_cnt, const i64* rlen, i64 n, i64* out) {
    hipLaunchKernelGGL(k_sl_need, dim3(256), dim3(kBlock), 0, s, slot_cnt, rlen, n, out);
}

// ------------------------------------------------------------------------------------------------
// stable multisplit of the records by key partition p = slot & (P-1): rank lists per partition.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_sl_ms_count(const u32* __restrict__ slot, i64 n, int P, i64* counts,
                                                       int nblk) {
    extern __shared__ __attribute__((aligned(16))) u32 hist[];
    for (int i = threadIdx.x; i < P; i += kBlock) hist[i] = 0;
    __syncthreads();
    i64 t0 = (i64)blockIdx.x * kTile;
    for (int r = 0; r < kItems; r++) {
        i64 e = t0 + (i64)r * kBlock + threadIdx.x;
        if (e < n) atomicAdd(&hist[slot[e] & (P - 1)], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < P; i += kBlock) counts[(i64)i * nblk + blockIdx.x] = hist[i];
}

__global__ __launch_bounds__(kBlock) void k_sl_ms_scatter(const u32* __restrict__ slot, i64 n, int P,
                                                         const i64* __restrict__ offsets, int nblk, u32* out_rank) {
    __shared__ u32 stage[kTile];
    extern __shared__ __attribute__((aligned(16))) u32 dyn[];
    u32* hist = dyn;
    u32* local_start = hist + P;
    u32* running = local_start + P;
    u32* wave_cnt = running + P;  // [4][P]
    u32* stage_p = wave_cnt + 4 * P;  // [kTile]
    for (int i = threadIdx.x; i < P; i += kBlock) {
        hist[i] = 0; running[i] = 0;
        for (int w = 0; w < 4; w++) wave_cnt[w * P + i] = 0;
    }
    __syncthreads();
    const i64 t0 = (i64)blockIdx.x * kTile;
    u32 my_p[kItems];
    bool ok_[kItems];
#pragma unroll
    for (int r = 0; r < kItems; r++) {
        i64 e = t0 + (i64)r * kBlock + threadIdx.x;
        ok_[r] = e < n;
        my_p[r] = ok_[r] ? (slot[e] & (P - 1)) : 0;
        if (ok_[r]) atomicAdd(&hist[my_p[r]], 1u);
    }
    __syncthreads();
    {
        int per = (P + kBlock - 1) / kBlock;
        int a = threadIdx.x * per, b = min(P, a + per);
        i64 sum = 0;
        for (int i = a; i < b; i++) sum += hist[i];
        i64 pre = block_excl_scan(sum, SumOp(), 0, nullptr);
        for (int i = a; i < b; i++) { local_start[i] = (u32)pre; pre += hist[i]; }
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 lt_mask = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    int bits = 0;
    while ((1 << bits) < P) bits++;
    for (int r = 0; r < kItems; r++) {
        bool ok = ok_[r];
        u32 p = my_p[r];
        u64 peers = __ballot(ok);
        for (int bt = 0; bt < bits; bt++) {
            u64 m = __ballot((p >> bt) & 1);
            peers &= ((p >> bt) & 1) ? m : ~m;
        }
        u32 lrank = __popcll(peers & lt_mask);
        bool leader = ok && lrank == 0;
        if (leader) wave_cnt[wave * P + p] = __popcll(peers);
        __syncthreads();
        if (ok) {
            u32 before = running[p];
            for (int w = 0; w < wave; w++) before += wave_cnt[w * P + p];
            u32 sl = local_start[p] + before + lrank;
            stage[sl] = (u32)(t0 + (i64)r * kBlock + threadIdx.x);
            stage_p[sl] = p;
        }
        __syncthreads();
        if (leader) { atomicAdd(&running[p], wave_cnt[wave * P + p]); wave_cnt[wave * P + p] = 0; }
        __syncthreads();
    }
    u32 n_tile = local_start[P - 1] + hist[P - 1];
    for (u32 j = threadIdx.x; j < n_tile; j += kBlock) {
        u32 p = stage_p[j];
        out_rank[offsets[(i64)p * nblk + blockIdx.x] + (j - local_start[p])] = stage[j];
    }
}

void launch_sl_multisplit(hipStream_t s, const u32* slot, i64 n, int P, i64* counts, i64* tmp, u32* out_rank,
                          i64* part_off) {
    int nblk = (int)((n + kTile - 1) / kTile);
    if (nblk == 0) return;
    hipLaunchKernelGGL(k_sl_ms_count, dim3(nblk), dim3(kBlock), P * 4, s, slot, n, P, counts, nblk);
    i64 ncnt = (i64)P * nblk;
    (void)hipMemsetAsync(counts + ncnt, 0, 8, s);
    launch_scan_sum_large(s, counts, ncnt + 1, tmp);
    size_t lds = (size_t)P * 4 * 7 + (size_t)kTile * 4 + 16;
    hipLaunchKernelGGL(k_sl_ms_scatter, dim3(nblk), dim3(kBlock), lds, s, slot, n, P, counts, nblk, out_rank);
    launch_part_off(s, counts, nblk, P, part_off);
}

// ------------------------------------------------------------------------------------------------
// k_sliding: one wave per key partition walks its records in event order. Lanes sharing a key are
// resolved in rounds (lowest lane first), so each key's adds / removes run in the reference's order.
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ bool mm_worse(int kind, u64 cur, u64 v) {
    // `next > value` (min) / `next < value` (max) on unboxed values of the input type
    switch (kind) {
        case AK_MIN_L: return (i64)cur > (i64)v;
        case AK_MAX_L: return (i64)cur < (i64)v;
        case AK_MIN_D: return __longlong_as_double((i64)cur) > __longlong_as_double((i64)v);
        case AK_MAX_D: return __longlong_as_double((i64)cur) < __longlong_as_double((i64)v);
        case AK_MIN_F: return (float)__longlong_as_double((i64)cur) > (float)__longlong_as_double((i64)v);
        default: return (float)__longlong_as_double((i64)cur) < (float)__longlong_as_double((i64)v);
    }
}

// Double.equals / Float.equals (bit equality, NaN == NaN) and Integer/Long.equals
__device__ __forceinline__ bool boxed_eq(int kind, u64 a, u64 b) {
    if (kind == AK_MIN_L || kind == AK_MAX_L) return a == b;
    double x = __longlong_as_double((i64)a), y = __longlong_as_double((i64)b);
    if (kind == AK_MIN_F || kind == AK_MAX_F) {
        float fx = (float)x, fy = (float)y;
        if (fx != fx && fy != fy) return true;
        return __float_as_uint(fx) == __float_as_uint(fy);
    }
    if (x != x && y != y) return true;
    return a == b;
}

__device__ __forceinline__ void sl_remove(const SlState& S, const AggPlan& ap, u32 k, const u64* v) {
    i64 c = S.cnt[k] - 1;
    S.cnt[k] = c;
    for (int a = 0; a < ap.n; a++) {
        int kind = ap.kind[a];
        if (kind == AK_COUNT) continue;
        u64 x = v[ap.vcol[a]];
        size_t fi = (size_t)ap.field[a] * S.nslots + k;
        switch (kind) {
            case AK_SUM_L: S.f[fi] = (u64)java_d2l((double)(i64)S.f[fi] - (double)(i64)x); break;
            case AK_SUM_D: case AK_AVG: {
                double xv = (kind == AK_AVG && !(ap.vcol_type[ap.vcol[a]] == SH_T_FLOAT ||
                                                 ap.vcol_type[ap.vcol[a]] == SH_T_DOUBLE))
                                ? (double)(i64)x : __longlong_as_double((i64)x);
                double r = __longlong_as_double((i64)S.f[fi]) - xv;
                // state destroyed when count == 0 && sum == 0.0 (PartitionStateHolder.returnState):
                // a fresh state restarts from +0.0
                if (c == 0 && r == 0.0) r = 0.0;
                S.f[fi] = (u64)__double_as_longlong(r);
                break;
            }
            default: {
                // removeFirstOccurrence(value) on the deque ring; then minValue = peekFirst()
                u64* dq = S.dq + ((size_t)ap.field[a] * S.nslots + k) * S.rc;
                i64 h = S.dq_head[fi], len = S.dq_len[fi];
                i64 found = -1;
                for (i64 i = 0; i < len; i++) {
                    if (boxed_eq(kind, dq[(h + i) & (S.rc - 1)], x)) { found = i; break; }
                }
                if (found >= 0) {
                    for (i64 i = found; i + 1 < len; i++) dq[(h + i) & (S.rc - 1)] = dq[(h + i + 1) & (S.rc - 1)];
                    len--;
                    S.dq_len[fi] = len;
                }
                if (len > 0) { S.mm[fi] = dq[h & (S.rc - 1)]; S.mm_has[fi] = 1; }
                else S.mm_has[fi] = 0;
            }
        }
    }
}

__device__ __forceinline__ void sl_add(const SlState& S, const AggPlan& ap, u32 k, const u64* v) {
    i64 c = S.cnt[k] + 1;
    S.cnt[k] = c;
    for (int a = 0; a < ap.n; a++) {
        int kind = ap.kind[a];
        if (kind == AK_COUNT) continue;
        u64 x = v[ap.vcol[a]];
        size_t fi = (size_t)ap.field[a] * S.nslots + k;
        switch (kind) {
            case AK_SUM_L: S.f[fi] = (u64)((i64)S.f[fi] + (i64)x); break;
            case AK_SUM_D: case AK_AVG: {
                double xv = (kind == AK_AVG && !(ap.vcol_type[ap.vcol[a]] == SH_T_FLOAT ||
                                                 ap.vcol_type[ap.vcol[a]] == SH_T_DOUBLE))
                                ? (double)(i64)x : __longlong_as_double((i64)x);
                S.f[fi] = (u64)__double_as_longlong(__longlong_as_double((i64)S.f[fi]) + xv);
                break;
            }
            default: {
                u64* dq = S.dq + ((size_t)ap.field[a] * S.nslots + k) * S.rc;
                i64 h = S.dq_head[fi], len = S.dq_len[fi];
                while (len > 0 && mm_worse(kind, dq[(h + len - 1) & (S.rc - 1)], x)) len--;
                dq[(h + len) & (S.rc - 1)] = x;
                S.dq_len[fi] = len + 1;
                if (!S.mm_has[fi] || mm_worse(kind, S.mm[fi], x)) { S.mm[fi] = x; S.mm_has[fi] = 1; }
            }
        }
    }
}

__global__ __launch_bounds__(64) void k_sliding(const u32* __restrict__ rank_list, const i64* __restrict__ part_off,
                                                int P, SlRecords rec, SlState S, AggPlan ap, i64 T, i64 send_size,
                                                i64 send_base, SlRows rows, unsigned char* flags) {
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    const i64 lo = part_off[p], hi = part_off[p + 1];
    for (i64 b = lo; b < hi; b += 64) {
        i64 idx = b + lane;
        bool pend = idx < hi;
        u32 r = 0, k = 0;
        if (pend) { r = rank_list[idx]; k = rec.slot[r]; }
        while (__ballot(pend)) {
            // lowest pending lane per key wins this round:
            // find, for each pending lane, whether an earlier pending lane has the same key
            bool win = pend;
            for (int j = 0; j < 64; j++) {
                u32 kj = __shfl(k, j, 64);
                bool pj = __shfl((int)pend, j, 64);
                if (j < lane && pj && kj == k) win = false;
            }
            if (win) {
                i64 clk = rec.clock[r];
                // lazy expiry: ring head events with PM + T <= clock
                i64 h = S.rhead[k], len = S.rlen[k];
                while (len > 0) {
                    i64 slot = (h & (S.rc - 1));
                    i64 pmj = S.rpm[(size_t)k * S.rc + slot];
                    if (pmj + T > clk) break;
                    u64 v[SH_MAX_AGGS];
                    for (int j = 0; j < ap.n_vcols; j++) v[j] = S.rval[((size_t)j * S.nslots + k) * S.rc + slot];
                    sl_remove(S, ap, k, v);
                    h++; len--;
                }
                // add the event to the key's ring and aggregators
                u64 v[SH_MAX_AGGS];
                for (int j = 0; j < ap.n_vcols; j++) v[j] = rec.vals[(size_t)j * rec.cap + r];
                i64 slot = (h + len) & (S.rc - 1);
                S.rpm[(size_t)k * S.rc + slot] = rec.pm[r];
                for (int j = 0; j < ap.n_vcols; j++) S.rval[((size_t)j * S.nslots + k) * S.rc + slot] = v[j];
                len++;
                S.rhead[k] = h; S.rlen[k] = len;
                sl_add(S, ap, k, v);
                // output row of (send, key): first occurrence position, last event's values
                i64 send = send_base + (send_size > 0 ? (i64)rec.raw[r] / send_size : 0);
                i64 first;
                if (S.cur_send[k] != send) { S.cur_send[k] = send; S.cur_first[k] = r; first = r; flags[r] = 1; }
                else first = S.cur_first[k];
                rows.ts[first] = rec.ts[r];
                rows.slot[first] = k;
                rows.send[first] = send;
                rows.clock[first] = clk;
                i64 c = S.cnt[k];
                for (int a = 0; a < ap.n; a++) {
                    int kind = ap.kind[a];
                    u64 o; unsigned char nl = 0;
                    if (kind == AK_COUNT) o = (u64)c;
                    else {
                        size_t fi = (size_t)ap.field[a] * S.nslots + k;
                        if (kind == AK_SUM_L || kind == AK_SUM_D) o = S.f[fi];
                        else if (kind == AK_AVG) o = (u64)__double_as_longlong(__longlong_as_double((i64)S.f[fi]) / (double)c);
                        else { o = S.mm[fi]; nl = S.mm_has[fi] ? 0 : 1; }
                    }
                    rows.vals[(size_t)a * rows.cap + first] = o;
                    rows.nulls[(size_t)a * rows.cap + first] = nl;
                }
                pend = false;
            }
            __builtin_amdgcn_wave_barrier();
            __threadfence_block();
        }
    }
}

void launch_sliding(hipStream_t s, const u32* rank_list, const i64* part_off, int P, SlRecords rec, SlState S,
                    AggPlan ap, i64 T, i64 send_size, i64 send_base, SlRows rows, unsigned char* flags) {
    hipLaunchKernelGGL(k_sliding, dim3(P), dim3(64), 0, s, rank_list, part_off, P, rec, S, ap, T, send_size,
                       send_base, rows, flags);
}

// ------------------------------------------------------------------------------------------------
// emit: flagged ranks -> output rows in rank order; flush starts where the send changes.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_sl_emit(const unsigned char* __restrict__ flags, i64 n,
                                                   const i64* __restrict__ blk_pre, SlRows rows, int n_aggs,
                                                   KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys,
                                                   u64* out_vals, unsigned char* out_nulls, i64* out_send,
                                                   i64* out_clock) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    unsigned char fl[kItems];
    i64 c = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) { fl[i] = base + i < n ? flags[base + i] : 0; c += fl[i]; }
    i64 r = block_excl_scan(c, SumOp(), 0, nullptr) + blk_pre[blockIdx.x];
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        if (!fl[i]) continue;
        i64 j = base + i;
        out_ts[r] = rows.ts[j];
        unpack_key(kp, slot_key(kt, rows.slot[j]), out_keys + r, out_cap);
        for (int a = 0; a < n_aggs; a++) {
            out_vals[(size_t)a * out_cap + r] = rows.vals[(size_t)a * rows.cap + j];
            out_nulls[(size_t)a * out_cap + r] = rows.nulls[(size_t)a * rows.cap + j];
        }
        out_send[r] = rows.send[j];
        out_clock[r] = rows.clock[j];
        r++;
    }
}

__global__ __launch_bounds__(kBlock) void k_flush_starts(const i64* __restrict__ out_send, i64 n, i64* blk_cnt) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 c = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 r = base + i;
        if (r < n && (r == 0 || out_send[r] != out_send[r - 1])) c++;
    }
    i64 t = block_reduce(c, SumOp(), 0);
    if (threadIdx.x == 0) blk_cnt[blockIdx.x] = t;
}

__global__ __launch_bounds__(kBlock) void k_flush_write(const i64* __restrict__ out_send, const i64* __restrict__ out_clock,
                                                       i64 n, const i64* blk_pre, i64* flush_off, i64* flush_clock) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 c = 0;
    bool st[kItems];
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 r = base + i;
        st[i] = r < n && (r == 0 || out_send[r] != out_send[r - 1]);
        c += st[i];
    }
    i64 f = block_excl_scan(c, SumOp(), 0, nullptr) + blk_pre[blockIdx.x];
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        if (!st[i]) continue;
        flush_off[f] = base + i;
        flush_clock[f] = out_clock[base + i];
        f++;
    }
}

void launch_sl_emit(hipStream_t s, const unsigned char* flags, i64 n, const i64* blk_pre, int nblk, SlRows rows,
                    int n_aggs, KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals,
                    unsigned char* out_nulls, i64* out_send, i64* out_clock) {
    hipLaunchKernelGGL(k_sl_emit, dim3(nblk), dim3(kBlock), 0, s, flags, n, blk_pre, rows, n_aggs, kt, kp, out_cap,
                       out_ts, out_keys, out_vals, out_nulls, out_send, out_clock);
}

void launch_flush_starts(hipStream_t s, const i64* out_send, i64 n_rows, i64* blk_cnt, int nb) {
    hipLaunchKernelGGL(k_flush_starts, dim3(nb), dim3(kBlock), 0, s, out_send, n_rows, blk_cnt);
}

void launch_flush_write(hipStream_t s, const i64* out_send, const i64* out_clock, i64 n_rows, const i64* blk_pre,
                        int nb, i64* flush_off, i64* flush_clock) {
    hipLaunchKernelGGL(k_flush_write, dim3(nb), dim3(kBlock), 0, s, out_send, out_clock, n_rows, blk_pre, flush_off,
                       flush_clock);
}

// grow the per-key rings / deques to a new capacity (power of two), preserving contents
__global__ void k_sl_regrow(const u64* old_buf, u64* new_buf, const i64* head, const i64* len, i64 nslots, int nsub,
                            i64 old_rc, i64 new_rc, const i64* hsel) {
    // one thread per (sub-array, slot): copies len elements starting at head into [0, len)
    i64 t = (i64)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nslots * nsub) return;
    i64 k = t % nslots;
    i64 h = head[hsel ? (t) : k], l = len[hsel ? (t) : k];
    const u64* src = old_buf + (size_t)t * old_rc;
    u64* dst = new_buf + (size_t)t * new_rc;
    for (i64 i = 0; i < l; i++) dst[i] = src[(h + i) & (old_rc - 1)];
}

void launch_sl_regrow(hipStream_t s, const u64* old_buf, u64* new_buf, const i64* head, const i64* len, i64 nslots,
                      int nsub, i64 old_rc, i64 new_rc, bool per_sub) {
    i64 n = nslots * nsub;
    if (n == 0) return;
    hipLaunchKernelGGL(k_sl_regrow, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, old_buf, new_buf, head, len,
                       nslots, nsub, old_rc, new_rc, per_sub ? head : nullptr);
}

}  // namespace shd
