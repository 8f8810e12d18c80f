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
    // externalTime: PM runs over the timestamp attribute instead of the event timestamps
    const bool ext = wp.kind == SH_WIN_EXT_TIME;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        if (e < wp.N) {
            i64 t = ts[e];
            if (pass[i]) { cnt++; pm = max(pm, ext ? load_raw(cols, wp.ts_col, e) : t); }
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
// The per-slot count through a workgroup table in LDS: the tile's events add to their slot's LDS
// counter and each distinct slot of the tile makes one global atomic at the end. A Zipf-hot key
// (partition lanes over 10M Zipf keys: the hottest holds ~10% of the events) otherwise sends millions
// of same-address atomics into one L2 channel, which serialises them (43 ms per 33.5M-event push).
constexpr int kSlotTab = 2 * kTile;  // at most kTile distinct slots per tile: never full
__device__ __forceinline__ void slot_tab_add(u32* tk, u32* tc, u32 pos) {
    u32 h = (pos * 2654435761u) & (kSlotTab - 1);
    for (;;) {
        const u32 old = atomicCAS(&tk[h], 0xFFFFFFFFu, pos);
        if (old == 0xFFFFFFFFu || old == pos) { atomicAdd(&tc[h], 1u); return; }
        h = (h + 1) & (kSlotTab - 1);
    }
}

__global__ __launch_bounds__(kBlock) void k_sl_records(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                      WinParams wp, KeyPlan kp, KeyTable kt, AggPlan ap,
                                                      const i64* blk_pass_pre, const i64* blk_tl_pre,
                                                      const i64* blk_pm_pre, i64 pm0, SlRecords rec, u32* slot_cnt,
                                                      i64* send_clock) {
    __shared__ u32 tk[kSlotTab], tc[kSlotTab];
    for (int i = threadIdx.x; i < kSlotTab; i += kBlock) { tk[i] = 0xFFFFFFFFu; tc[i] = 0; }
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    bool pass[kItems];
    i64 cnt = 0, tl = INT64_MIN, pm = INT64_MIN;
    filter_items(f, cols, base, wp.N, pass);
    const bool ext = wp.kind == SH_WIN_EXT_TIME;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        if (e < wp.N) {
            i64 t = ts[e];
            cnt += pass[i];
            if (pass[i]) pm = max(pm, ext ? load_raw(cols, wp.ts_col, e) : t);
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
        const bool in = e < wp.N;
        const bool valid = in && pass[i];
        u32 pos = 0;
        i64 t = in ? ts[e] : 0;
        if (valid) {
            // externalTime (ExternalTimeWindowProcessor :126-161): an event expires the queue head
            // while headTime + T <= its own attribute, so event j has left the window at event i iff
            // PMa(j) + T <= PMa(i) (PMa = running max of the attribute): clock = PMa(i)
            pmx = max(pmx, ext ? load_raw(cols, wp.ts_col, e) : t);
            const i64 sclk = max(c0, max(cm, ts[send_last_of(wp, e)]));
            i64 clk = ext ? pmx : sclk;
            if (send_clock) send_clock[r] = sclk;  // the flush clock of an externalTime row
            pos = key_slot(kt, make_key(kp, cols, e));
            rec.raw[r] = (u32)e;
            rec.slot[r] = pos;
            if (rec.aos) {
                ulonglong2* o = (ulonglong2*)(rec.aos + (size_t)r * kSlAosWords);
                o[0] = make_ulonglong2((u64)clk, (u64)pmx);
                o[1] = make_ulonglong2((u64)t, (u64)load_raw(cols, ap.vcol_src[0], e));
                o[2] = make_ulonglong2((u64)e, 0ull);
            } else {
                rec.clock[r] = clk;
                rec.pm[r] = pmx;
                rec.ts[r] = t;
                for (int j = 0; j < ap.n_vcols; j++) rec.vals[(size_t)j * rec.cap + r] = (u64)load_raw(cols, ap.vcol_src[j], e);
            }
            slot_tab_add(tk, tc, pos);
            r++;
        }
        if (in && is_send_last(wp, e)) cm = max(cm, t);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < kSlotTab; i += kBlock)
        if (tc[i]) atomicAdd(&slot_cnt[tk[i]], tc[i]);
}

// The common case of k_sl_records — no filter, one event per send, time(T) — with the tile's events
// taken lane-strided (round i: events tile + i * kBlock + lane), so consecutive lanes write consecutive
// records (whole lines; the thread-contiguous form stored 48-byte records 8 apart per lane, and PMC saw
// 2.3x the record bytes written). Every event passes and ends its own send, so its clock and PM are the
// running maximum of the timestamps (a block max-scan per round, carried across rounds).
template <bool COUNT>
__global__ __launch_bounds__(kBlock) void k_sl_records_seq(const i64* __restrict__ ts, ColSet cols, WinParams wp,
                                                          KeyPlan kp, KeyTable kt, AggPlan ap,
                                                          const i64* blk_pass_pre, const i64* blk_tl_pre,
                                                          const i64* blk_pm_pre, i64 pm0, SlRecords rec,
                                                          u32* slot_cnt, i64* send_clock) {
    // (without the slot table the block needs 12 KB of LDS instead of 45: 8 resident waves, not 3)
    __shared__ u32 tk[COUNT ? kSlotTab : 1], tc[COUNT ? kSlotTab : 1];
    // the wave's 64 records staged in LDS, then stored as contiguous 16-byte pieces (each store
    // instruction covers 1 KB of whole lines instead of one piece of 64 records 48 bytes apart)
    __shared__ ulonglong2 stg[kBlock * 3];
    // slot_cnt null: the caller takes the per-slot counts from the sorted slots instead (k_counts_sorted:
    // r05, the tile's LDS table and its global atomics were 1.2 of the kernel's 1.9 ms at C3)
    constexpr bool count = COUNT;
    if (count)
        for (int i = threadIdx.x; i < kSlotTab; i += kBlock) { tk[i] = 0xFFFFFFFFu; tc[i] = 0; }
    const i64 tile0 = (i64)blockIdx.x * kTile;
    const i64 r0 = blk_pass_pre[blockIdx.x];
    i64 carry_cm = blk_tl_pre[blockIdx.x];
    i64 carry_pm = max(blk_pm_pre[blockIdx.x], pm0);
    const i64 c0 = wp.clock_valid ? wp.clock0 : INT64_MIN;
    const int lane = threadIdx.x & 63, wb = threadIdx.x & ~63;
    for (int it = 0; it < kItems; it++) {
        const i64 e = tile0 + (i64)it * kBlock + threadIdx.x;
        const bool in = e < wp.N;
        const i64 t = in ? ts[e] : INT64_MIN;
        const u32 pos = in ? key_slot(kt, make_key(kp, cols, e)) : 0u;
        const u64 v = in ? (u64)load_raw(cols, ap.vcol_src[0], e) : 0ull;
        i64 tot;
        const i64 incl = max(block_excl_scan(t, MaxOp(), INT64_MIN, &tot), t);
        if (rec.aos) {
            // (every event of the tile passes: record r0 + it * kBlock + thread; the wave's run is whole
            // records r_w .. r_w + 63, fewer at the push's end)
            const i64 pmx = max(carry_pm, incl);
            const i64 sclk = max(c0, max(carry_cm, incl));
            const i64 r = r0 + (i64)it * kBlock + threadIdx.x;
            if (in) {
                if (send_clock) send_clock[r] = sclk;
                rec.raw[r] = (u32)e;
                rec.slot[r] = pos;
                if (count) slot_tab_add(tk, tc, pos);
            }
            stg[threadIdx.x * 3 + 0] = make_ulonglong2((u64)sclk, (u64)pmx);
            stg[threadIdx.x * 3 + 1] = make_ulonglong2((u64)t, v);
            stg[threadIdx.x * 3 + 2] = make_ulonglong2((u64)e, 0ull);
            __syncthreads();
            const i64 rw = r0 + (i64)it * kBlock + wb;  // the wave's first record
            const i64 ew = tile0 + (i64)it * kBlock + wb;
            const int nw = (int)max((i64)0, min((i64)64, wp.N - ew));
            ulonglong2* dst = (ulonglong2*)(rec.aos + (size_t)rw * kSlAosWords);
            for (int q = lane; q < nw * 3; q += 64) dst[q] = stg[wb * 3 + q];
            __syncthreads();
        } else if (in) {
            const i64 pmx = max(carry_pm, incl);
            const i64 sclk = max(c0, max(carry_cm, incl));
            const i64 r = r0 + (i64)it * kBlock + threadIdx.x;
            if (send_clock) send_clock[r] = sclk;
            rec.raw[r] = (u32)e;
            rec.slot[r] = pos;
            {
                rec.clock[r] = sclk;
                rec.pm[r] = pmx;
                rec.ts[r] = t;
                for (int j = 0; j < ap.n_vcols; j++) rec.vals[(size_t)j * rec.cap + r] = (u64)load_raw(cols, ap.vcol_src[j], e);
            }
            if (count) slot_tab_add(tk, tc, pos);
        }
        carry_pm = max(carry_pm, tot);
        carry_cm = max(carry_cm, tot);
    }
    __syncthreads();
    if (count)
        for (int i = threadIdx.x; i < kSlotTab; i += kBlock)
            if (tc[i]) atomicAdd(&slot_cnt[tk[i]], tc[i]);
}

bool sl_records_seq_applies(FilterProg f, WinParams wp, AggPlan ap) {
    return filter_kind(f) == 0 && wp.send_size == 1 && wp.kind == SH_WIN_TIME && ap.n_vcols >= 1 && wp.rec_seq;
}

void launch_sl_records(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp, KeyPlan kp,
                       KeyTable kt, AggPlan ap, const i64* blk_pass_pre, const i64* blk_tl_pre, const i64* blk_pm_pre,
                       i64 pm0, SlRecords rec, u32* slot_cnt, int nblk, i64* send_clock) {
    if (sl_records_seq_applies(f, wp, ap)) {
        if (slot_cnt)
            hipLaunchKernelGGL(k_sl_records_seq<true>, dim3(nblk), dim3(kBlock), 0, s, ts, cols, wp, kp, kt, ap,
                               blk_pass_pre, blk_tl_pre, blk_pm_pre, pm0, rec, slot_cnt, send_clock);
        else
            hipLaunchKernelGGL(k_sl_records_seq<false>, dim3(nblk), dim3(kBlock), 0, s, ts, cols, wp, kp, kt, ap,
                               blk_pass_pre, blk_tl_pre, blk_pm_pre, pm0, rec, nullptr, send_clock);
        return;
    }
    hipLaunchKernelGGL(k_sl_records, dim3(nblk), dim3(kBlock), 0, s, ts, cols, f, wp, kp, kt, ap, blk_pass_pre,
                       blk_tl_pre, blk_pm_pre, pm0, rec, slot_cnt, send_clock);
}

// Sharded owner (sh_shard.cpp): the records arrive filtered and re-keyed, with the global clock of
// their send and the global PM computed by the source slice (sh_shard_kernels.hip k_shard_sl_assign);
// raw = position in the global push, so send = send_base + raw / send_size as in the single stream.
__device__ __forceinline__ void sl_record_given(i64 r, const i64* __restrict__ ts, ColSet cols, KeyPlan kp, KeyTable kt,
                                                AggPlan ap, const i64* __restrict__ gclk, const i64* __restrict__ gpm,
                                                const u64* __restrict__ gidx, i64 raw_base, SlRecords rec, u32* tk,
                                                u32* tc) {
    const u32 pos = key_slot(kt, make_key(kp, cols, r));
    const u32 raw = (u32)((i64)gidx[r] - raw_base);
    rec.raw[r] = raw;
    rec.slot[r] = pos;
    if (rec.aos) {
        ulonglong2* o = (ulonglong2*)(rec.aos + (size_t)r * kSlAosWords);
        o[0] = make_ulonglong2((u64)gclk[r], (u64)gpm[r]);
        o[1] = make_ulonglong2((u64)ts[r], (u64)load_raw(cols, ap.vcol_src[0], r));
        o[2] = make_ulonglong2((u64)raw, 0ull);
    } else {
        rec.clock[r] = gclk[r];
        rec.pm[r] = gpm[r];
        rec.ts[r] = ts[r];
        for (int j = 0; j < ap.n_vcols; j++) rec.vals[(size_t)j * rec.cap + r] = (u64)load_raw(cols, ap.vcol_src[j], r);
    }
    slot_tab_add(tk, tc, pos);
}

__global__ __launch_bounds__(kBlock) void k_sl_records_given(i64 M, const i64* __restrict__ ts, ColSet cols,
                                                            KeyPlan kp, KeyTable kt, AggPlan ap,
                                                            const i64* __restrict__ gclk, const i64* __restrict__ gpm,
                                                            const u64* __restrict__ gidx, i64 raw_base,
                                                            SlRecords rec, u32* slot_cnt) {
    __shared__ u32 tk[kSlotTab], tc[kSlotTab];
    for (int i = threadIdx.x; i < kSlotTab; i += kBlock) { tk[i] = 0xFFFFFFFFu; tc[i] = 0; }
    __syncthreads();
    const i64 r = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (r < M) sl_record_given(r, ts, cols, kp, kt, ap, gclk, gpm, gidx, raw_base, rec, tk, tc);
    __syncthreads();
    for (int i = threadIdx.x; i < kSlotTab; i += kBlock)
        if (tc[i]) atomicAdd(&slot_cnt[tk[i]], tc[i]);
}


void launch_sl_records_given(hipStream_t s, i64 M, const i64* ts, ColSet cols, KeyPlan kp, KeyTable kt, AggPlan ap,
                             const i64* gclk, const i64* gpm, const u64* gidx, i64 raw_base, SlRecords rec,
                             u32* slot_cnt) {
    if (M <= 0) return;
    hipLaunchKernelGGL(k_sl_records_given, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, M, ts,
                       cols, kp, kt, ap, gclk, gpm, gidx, raw_base, rec, slot_cnt);
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

// Per-slot counts from the slot-sorted records: the first position of a slot's run subtracts its index,
// the last adds its index + 1 (two atomics per run, each on its own slot: no contention), so
// slot_cnt[k] = the run's length; zeroed by the caller. (Writing the key offsets directly from the run
// starts loops over every absent slot in between: with sparse slots — 231k Zipf partitions in a 10M-slot
// dictionary — single lanes filled gaps of thousands, plb 20 -> 103 ms per push.)
__global__ __launch_bounds__(kBlock) void k_counts_sorted(const u32* __restrict__ ps, i64 M, u32* slot_cnt) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= M) return;
    const u32 cur = ps[i];
    if (i == 0 || ps[i - 1] != cur) atomicAdd(&slot_cnt[cur], (u32)(-(i64)i));
    if (i == M - 1 || ps[i + 1] != cur) atomicAdd(&slot_cnt[cur], (u32)(i + 1));
}

void launch_counts_sorted(hipStream_t s, const u32* ps, i64 M, u32* slot_cnt) {
    if (M > 0)
        hipLaunchKernelGGL(k_counts_sorted, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, ps, M,
                           slot_cnt);
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

// ------------------------------------------------------------------------------------------------
// k_sl_own: one wave per key partition, lane ownership. Local key li = slot >> logP belongs to lane
// li & 63 (with NL <= 64 local keys every lane owns at most one key, whose state — counts, sums,
// min/max values, ring and deque heads — stays in registers for the whole push). The partition's
// records (event order) are taken in chunks; each chunk is split stably in LDS into 64 per-lane
// lists, and every lane replays its key's events in order: lazy expiry from the ring head, add, row.
// No conflict rounds. Latency is what bounds it (one dependent chain per key), so:
//  - the next record's fields and the next ring-head entry are loaded one step ahead;
//  - the min/max deques (MinAttributeAggregatorExecutor's LinkedList with removeFirstOccurrence)
//    live in LDS, kDqL entries per (key, aggregator); a deque that outgrows that spills to its ring
//    in global memory for the rest of the push (sorted input makes deques as long as the window).
// ------------------------------------------------------------------------------------------------
constexpr int kSlCh = 2048;
#ifndef SH_SL_KL
#define SH_SL_KL 8
#endif
// records staged per chunk of k_sl_own_d. Measured on MI355X, C3 (10k keys, 16.7M events per
// push): CH 512 -> 23.9 ms at KL 8 with CH 256, 20.2 ms at CH 128, 20.1 ms at CH 64; KL 4/8/16
// within 10% at CH 256, KL 2 31 ms (the ~11 KB LDS footprint at CH 128 keeps ~14 waves per CU)
#ifndef SH_SL_CH
#define SH_SL_CH 128
#endif
constexpr int kSlKeyLanes = SH_SL_KL;  // key-owning lanes per wave of k_sl_own_d
constexpr int kDqL = 32;

template <int NA, int NV>
struct LaneKey {
    u32 k;  // cached slot (kNoPos: none)
    i64 cnt, rh, rlen, cur_send, cur_first;
    u64 f[NA], mm[NA], dqf[NA], dqb[NA];
    i64 dqh[NA], dql[NA];
    unsigned char mmh[NA];
    bool spill[NA];
    bool hvalid;
    i64 hpm;
    u64 hval[NV];
    i64 hb_base;  // ring index of the first entry in the lane's LDS head cache
    int hb_n;     // valid entries there
};
constexpr int kHb = 8;  // ring-head entries fetched per refill (one latency per kHb expiries)

__device__ __forceinline__ bool is_mm(int kind) { return kind >= AK_MIN_L; }

// v[i] with a run-time i, as a select chain over the unrolled slots (keeps v in registers)
template <int NV>
__device__ __forceinline__ u64 pick(const u64 (&v)[NV], int i) {
    u64 x = v[0];
#pragma unroll
    for (int q = 1; q < NV; q++) x = (i == q) ? v[q] : x;
    return x;
}

// deque storage of aggregator a for the lane's key: LDS ring (kDqL) or, spilled, the global ring
struct DqView {
    u64* g;
    u64* l;
    i64 gm;
    bool spill;
    __device__ __forceinline__ u64 get(i64 i) const { return spill ? g[i & gm] : l[i & (kDqL - 1)]; }
    __device__ __forceinline__ void set(i64 i, u64 v) const {
        if (spill) g[i & gm] = v;
        else l[i & (kDqL - 1)] = v;
    }
};

template <int NA, int NV>
__device__ __forceinline__ DqView dq_view(const LaneKey<NA, NV>& L, const SlState& S, const AggPlan& ap, u64* lds_dq,
                                          const int (&mmi)[NA], int a) {
    DqView d;
    d.g = S.dq + ((size_t)ap.field[a] * S.nslots + L.k) * S.rc;
    d.l = lds_dq + ((size_t)mmi[a] * 64 + threadIdx.x) * kDqL;
    d.gm = S.rc - 1;
    d.spill = L.spill[a];
    return d;
}

template <int NA, int NV>
__device__ __forceinline__ void lk_load(LaneKey<NA, NV>& L, const SlState& S, const AggPlan& ap, u64* lds_dq,
                                        const int (&mmi)[NA], u32 k) {
    L.k = k;
    L.cnt = S.cnt[k];
    L.rh = S.rhead[k];
    L.rlen = S.rlen[k];
    L.cur_send = S.cur_send[k];
    L.cur_first = S.cur_first[k];
    L.hvalid = false;
    L.hb_n = 0;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (a >= ap.n) break;
        const int kind = ap.kind[a];
        if (kind == AK_COUNT) continue;
        const size_t fi = (size_t)ap.field[a] * S.nslots + k;
        L.f[a] = S.f[fi];
        if (is_mm(kind)) {
            L.mm[a] = S.mm[fi];
            L.mmh[a] = S.mm_has[fi];
            L.dqh[a] = S.dq_head[fi];
            L.dql[a] = S.dq_len[fi];
            L.spill[a] = L.dql[a] >= kDqL;
            const DqView d = dq_view(L, S, ap, lds_dq, mmi, a);
            const i64 h = L.dqh[a], len = L.dql[a];
            if (!d.spill)
                for (i64 i = 0; i < len; i++) d.l[(h + i) & (kDqL - 1)] = d.g[(h + i) & d.gm];
            if (len > 0) {
                L.dqf[a] = d.get(h);
                L.dqb[a] = d.get(h + len - 1);
            }
        }
    }
}

template <int NA, int NV>
__device__ __forceinline__ void lk_store(const LaneKey<NA, NV>& L, const SlState& S, const AggPlan& ap, u64* lds_dq,
                                         const int (&mmi)[NA]) {
    const u32 k = L.k;
    S.cnt[k] = L.cnt;
    S.rhead[k] = L.rh;
    S.rlen[k] = L.rlen;
    S.cur_send[k] = L.cur_send;
    S.cur_first[k] = L.cur_first;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (a >= ap.n) break;
        const int kind = ap.kind[a];
        if (kind == AK_COUNT) continue;
        const size_t fi = (size_t)ap.field[a] * S.nslots + k;
        S.f[fi] = L.f[a];
        if (is_mm(kind)) {
            S.mm[fi] = L.mm[a];
            S.mm_has[fi] = L.mmh[a];
            S.dq_head[fi] = L.dqh[a];
            S.dq_len[fi] = L.dql[a];
            const DqView d = dq_view(L, S, ap, lds_dq, mmi, a);
            if (!d.spill)
                for (i64 i = 0; i < L.dql[a]; i++) d.g[(L.dqh[a] + i) & d.gm] = d.l[(L.dqh[a] + i) & (kDqL - 1)];
        }
    }
}

// the ring head entry (index rh) into registers, from the lane's LDS cache of the next kHb
// entries; a refill loads up to kHb entries (never past the current tail) in one round trip
template <int NA, int NV>
__device__ __forceinline__ void lk_head(LaneKey<NA, NV>& L, const SlState& S, const AggPlan& ap, i64* hb_pm,
                                        u64* hb_v) {
    const int lane = threadIdx.x;
    if (!(L.rh >= L.hb_base && L.rh < L.hb_base + L.hb_n)) {
        const int n = (int)min<i64>(kHb, L.rlen);
        i64 pm[kHb];
        u64 vv[NV][kHb];
#pragma unroll
        for (int e = 0; e < kHb; e++) {
            if (e < n) {
                const i64 sl = (L.rh + e) & (S.rc - 1);
                pm[e] = S.rpm[(size_t)L.k * S.rc + sl];
#pragma unroll
                for (int j = 0; j < NV; j++)
                    if (j < ap.n_vcols) vv[j][e] = S.rval[((size_t)j * S.nslots + L.k) * S.rc + sl];
            }
        }
#pragma unroll
        for (int e = 0; e < kHb; e++) {
            if (e < n) {
                hb_pm[lane * kHb + e] = pm[e];
#pragma unroll
                for (int j = 0; j < NV; j++)
                    if (j < ap.n_vcols) hb_v[(j * 64 + lane) * kHb + e] = vv[j][e];
            }
        }
        L.hb_base = L.rh;
        L.hb_n = n;
    }
    const int e = (int)(L.rh - L.hb_base);
    L.hpm = hb_pm[lane * kHb + e];
#pragma unroll
    for (int j = 0; j < NV; j++) {
        if (j >= ap.n_vcols) break;
        L.hval[j] = hb_v[(j * 64 + lane) * kHb + e];
    }
    L.hvalid = true;
}

// AttributeAggregatorExecutor.processRemove for every aggregator (same arithmetic as sl_remove)
template <int NA, int NV>
__device__ __forceinline__ void lk_remove(LaneKey<NA, NV>& L, const SlState& S, const AggPlan& ap, u64* lds_dq,
                                          const int (&mmi)[NA], const u64 (&v)[NV]) {
    const i64 c = L.cnt - 1;
    L.cnt = c;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (a >= ap.n) break;
        const int kind = ap.kind[a];
        if (kind == AK_COUNT) continue;
        const u64 x = pick(v, ap.vcol[a]);
        if (kind == AK_SUM_L) {
            L.f[a] = (u64)java_d2l((double)(i64)L.f[a] - (double)(i64)x);
        } else if (kind == AK_SUM_D || kind == AK_AVG) {
            const double xv = (kind == AK_AVG && !(ap.vcol_type[ap.vcol[a]] == SH_T_FLOAT ||
                                                   ap.vcol_type[ap.vcol[a]] == SH_T_DOUBLE))
                                  ? (double)(i64)x : __longlong_as_double((i64)x);
            double r = __longlong_as_double((i64)L.f[a]) - xv;
            if (c == 0 && r == 0.0) r = 0.0;  // destroyed state restarts from +0.0 (canDestroy)
            L.f[a] = (u64)__double_as_longlong(r);
        } else {
            // removeFirstOccurrence(value): the front in the common case, else a scan
            const DqView d = dq_view(L, S, ap, lds_dq, mmi, a);
            i64 h = L.dqh[a], len = L.dql[a];
            if (len > 0 && boxed_eq(kind, L.dqf[a], x)) {
                h++;
                len--;
                if (len > 0) L.dqf[a] = d.get(h);
            } else if (len > 1) {
                i64 found = -1;
                for (i64 i = 1; i < len; i++)
                    if (boxed_eq(kind, d.get(h + i), x)) { found = i; break; }
                if (found >= 0) {
                    for (i64 i = found; i + 1 < len; i++) d.set(h + i, d.get(h + i + 1));
                    len--;
                    L.dqb[a] = d.get(h + len - 1);
                }
            }
            L.dqh[a] = h;
            L.dql[a] = len;
            if (len > 0) { L.mm[a] = L.dqf[a]; L.mmh[a] = 1; }
            else L.mmh[a] = 0;
        }
    }
}

// processAdd (same arithmetic as sl_add)
template <int NA, int NV>
__device__ __forceinline__ void lk_add(LaneKey<NA, NV>& L, const SlState& S, const AggPlan& ap, u64* lds_dq,
                                       const int (&mmi)[NA], const u64 (&v)[NV]) {
    L.cnt = L.cnt + 1;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (a >= ap.n) break;
        const int kind = ap.kind[a];
        if (kind == AK_COUNT) continue;
        const u64 x = pick(v, ap.vcol[a]);
        if (kind == AK_SUM_L) {
            L.f[a] = (u64)((i64)L.f[a] + (i64)x);
        } else if (kind == AK_SUM_D || kind == AK_AVG) {
            const double xv = (kind == AK_AVG && !(ap.vcol_type[ap.vcol[a]] == SH_T_FLOAT ||
                                                   ap.vcol_type[ap.vcol[a]] == SH_T_DOUBLE))
                                  ? (double)(i64)x : __longlong_as_double((i64)x);
            L.f[a] = (u64)__double_as_longlong(__longlong_as_double((i64)L.f[a]) + xv);
        } else {
            DqView d = dq_view(L, S, ap, lds_dq, mmi, a);
            const i64 h = L.dqh[a];
            i64 len = L.dql[a];
            while (len > 0 && mm_worse(kind, L.dqb[a], x)) {
                len--;
                if (len > 0) L.dqb[a] = d.get(h + len - 1);
            }
            if (!d.spill && len == kDqL) {  // the LDS ring is full: move to the global ring
                for (i64 i = 0; i < len; i++) d.g[(h + i) & d.gm] = d.l[(h + i) & (kDqL - 1)];
                L.spill[a] = true;
                d.spill = true;
            }
            d.set(h + len, x);
            len++;
            L.dqb[a] = x;
            if (len == 1) L.dqf[a] = x;
            L.dql[a] = len;
            if (!L.mmh[a] || mm_worse(kind, L.mm[a], x)) { L.mm[a] = x; L.mmh[a] = 1; }
        }
    }
}

template <int NV>
struct SlRec {
    i64 clk, pm, ts;
    u32 raw;
    u64 v[NV];
};

template <int NV>
__device__ __forceinline__ void sl_rec_load(SlRec<NV>& o, const SlRecords& rec, const AggPlan& ap, i64 r) {
    o.clk = rec.clock[r];
    o.pm = rec.pm[r];
    o.ts = rec.ts[r];
    o.raw = rec.raw[r];
#pragma unroll
    for (int q = 0; q < NV; q++) {
        if (q >= ap.n_vcols) break;
        o.v[q] = rec.vals[(size_t)q * rec.cap + r];
    }
}

// Chunk split shared by the k_sl_own kernels: records [c0, c0+n) of the partition (event order)
// into 64 stable per-lane lists (lane = (slot >> logP) & 63). Returns this lane's count and start.
// BYRANK: slot is indexed by record rank (records not gathered into partition order).
template <int KL = 64, bool BYRANK = false>
__device__ __forceinline__ void sl_chunk_split(const u32* __restrict__ rank_list, const u32* __restrict__ slot, i64 c0,
                                               int n, int logP, u32* ch_rank, u32* ch_slot, unsigned short* list,
                                               u32* run, u32& mine_out, u32& start_out) {
    constexpr int B = KL == 64 ? 6 : KL == 32 ? 5 : KL == 16 ? 4 : KL == 8 ? 3 : KL == 4 ? 2 : 1;
    const int lane = threadIdx.x;
    const u64 lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    u32 mine = 0;
    for (int g = 0; g < n; g += 64) {
        const int j = g + lane;
        u32 o = 0;
        if (j < n) {
            const u32 rk = rank_list[c0 + j];
            const u32 k = BYRANK ? slot[rk] : slot[c0 + j];
            o = (k >> logP) & (KL - 1);
            ch_rank[j] = rk;
            ch_slot[j] = k;
        }
        u64 mask = __ballot(j < n);
#pragma unroll
        for (int bt = 0; bt < B; bt++) {
            const u64 b = __ballot((o >> bt) & 1);
            mask &= ((lane >> bt) & 1) ? b : ~b;
        }
        if (lane < KL) mine += (u32)__popcll(mask);
    }
    u32 incl = mine;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    const u32 start = incl - mine;
    run[lane] = start;
    __syncthreads();
    for (int g = 0; g < n; g += 64) {
        const int j = g + lane;
        const bool ok = j < n;
        const u32 o = ok ? ((ch_slot[j] >> logP) & (KL - 1)) : 0;
        u64 peers = __ballot(ok);
#pragma unroll
        for (int bt = 0; bt < B; bt++) {
            const bool bit = (o >> bt) & 1;
            const u64 b = __ballot(bit);
            peers &= bit ? b : ~b;
        }
        const u32 lr = (u32)__popcll(peers & lt_mask);
        u32 base = 0;
        if (ok) base = run[o];
        __syncthreads();
        if (ok) list[base + lr] = (unsigned short)j;
        if (ok && lr == 0) run[o] = base + (u32)__popcll(peers);
        __syncthreads();
    }
    mine_out = mine;
    start_out = start;
}

// ---- k_sl_own_d: the same replay specialised for the common shape — every aggregator is count or
// reads one DOUBLE column with sum / avg / min / max (each at most once). Sum and avg perform the
// identical += / -= sequence (with the same canDestroy reset), so they share one running sum; the
// min and max deques use plain double comparisons and Double.equals. Far fewer instructions per
// event than the generic kernel, whose run-time aggregator dispatch dominated its chain latency.
struct DFields {
    int sum, avg, mn, mx;  // field index of each (-1: absent)
};

struct DDeque {
    i64 h, len;
    u64 f, b, mm;
    bool mmh, spill;
    bool nan;  // a NaN may be in the deque (Java comparisons with NaN are false: order no longer holds)
};

__device__ __forceinline__ bool d_eq(u64 a, u64 b) {
    const double x = __longlong_as_double((i64)a), y = __longlong_as_double((i64)b);
    return a == b || (x != x && y != y);
}

template <bool MIN>
__device__ __forceinline__ bool d_worse(u64 cur, u64 x) {
    const double c = __longlong_as_double((i64)cur), v = __longlong_as_double((i64)x);
    return MIN ? (c > v) : (c < v);
}

__device__ __forceinline__ bool d_isnan(u64 a) {
    const double x = __longlong_as_double((i64)a);
    return x != x;
}

// The deque of the lane's key lives in its LDS ring `l` (kDqL entries) unless it outgrew that
// (`spill`): then in its global ring `g`. The two paths are separate so each uses plain LDS or
// global instructions (a pointer select would compile to FLAT accesses that wait on both counters).
template <int LS = 1>
__device__ __forceinline__ void dd_load(DDeque& q, const SlState& S, int field, u32 k, u64* l) {
    const size_t fi = (size_t)field * S.nslots + k;
    q.mm = S.mm[fi];
    q.mmh = S.mm_has[fi];
    q.h = S.dq_head[fi];
    q.len = S.dq_len[fi];
    q.spill = q.len >= kDqL;
    q.nan = q.spill;
    const u64* g = S.dq + fi * S.rc;
    const i64 gm = S.rc - 1;
    if (!q.spill) {
        for (i64 i = 0; i < q.len; i++) {
            const u64 v = g[(q.h + i) & gm];
            l[((q.h + i) & (kDqL - 1)) * LS] = v;
            q.nan |= d_isnan(v);
        }
    }
    if (q.len > 0) {
        q.f = g[q.h & gm];
        q.b = g[(q.h + q.len - 1) & gm];
    }
}

template <int LS = 1>
__device__ __forceinline__ void dd_store(const DDeque& q, const SlState& S, int field, u32 k, const u64* l) {
    const size_t fi = (size_t)field * S.nslots + k;
    S.mm[fi] = q.mm;
    S.mm_has[fi] = q.mmh;
    S.dq_head[fi] = q.h;
    S.dq_len[fi] = q.len;
    u64* g = S.dq + fi * S.rc;
    const i64 gm = S.rc - 1;
    if (!q.spill)
        for (i64 i = 0; i < q.len; i++) g[(q.h + i) & gm] = l[((q.h + i) & (kDqL - 1)) * LS];
}

// removeFirstOccurrence(x) then minValue = peekFirst() (Min/MaxAttributeAggregatorExecutor).
// The front is the common case. Otherwise, while no NaN is in the deque it is monotone (min:
// non-decreasing, max: non-increasing), so an x beyond the back cannot be in it and needs no scan.
template <bool MIN, bool GLOBAL, int LS = 1>
__device__ __forceinline__ void dd_remove_t(DDeque& q, u64* g, i64 gm, u64* l, u64 x) {
    auto at = [&](i64 i) -> u64 { return GLOBAL ? g[i & gm] : l[(i & (kDqL - 1)) * LS]; };
    if (q.len > 0 && d_eq(q.f, x)) {
        q.h++;
        q.len--;
        if (q.len > 0) q.f = at(q.h);
    } else if (q.len > 1 && (q.nan || !d_worse<MIN>(x, q.b))) {
        i64 found = -1;
        for (i64 i = 1; i < q.len; i++)
            if (d_eq(at(q.h + i), x)) { found = i; break; }
        if (found >= 0) {
            for (i64 i = found; i + 1 < q.len; i++) {
                const u64 v = at(q.h + i + 1);
                if (GLOBAL) g[(q.h + i) & gm] = v;
                else l[((q.h + i) & (kDqL - 1)) * LS] = v;
            }
            q.len--;
            q.b = at(q.h + q.len - 1);
        }
    }
    if (q.len > 0) { q.mm = q.f; q.mmh = true; }
    else { q.mmh = false; q.nan = q.spill; }
}

template <bool MIN, int LS = 1>
__device__ __forceinline__ void dd_remove(DDeque& q, u64* g, i64 gm, u64* l, u64 x) {
    if (q.spill) dd_remove_t<MIN, true, LS>(q, g, gm, l, x);
    else dd_remove_t<MIN, false, LS>(q, g, gm, l, x);
}

template <bool MIN, bool GLOBAL, int LS = 1>
__device__ __forceinline__ void dd_add_t(DDeque& q, u64* g, i64 gm, u64* l, u64 x) {
    while (q.len > 0 && d_worse<MIN>(q.b, x)) {
        q.len--;
        if (q.len > 0) q.b = GLOBAL ? g[(q.h + q.len - 1) & gm] : l[((q.h + q.len - 1) & (kDqL - 1)) * LS];
    }
}

template <bool MIN, int LS = 1>
__device__ __forceinline__ void dd_add(DDeque& q, u64* g, i64 gm, u64* l, u64 x) {
    if (q.spill) dd_add_t<MIN, true, LS>(q, g, gm, l, x);
    else dd_add_t<MIN, false, LS>(q, g, gm, l, x);
    if (!q.spill && q.len == kDqL) {  // the LDS ring is full: move to the global ring
        for (i64 i = 0; i < q.len; i++) g[(q.h + i) & gm] = l[((q.h + i) & (kDqL - 1)) * LS];
        q.spill = true;
        q.nan = true;  // the global path always scans
    }
    if (q.spill) g[(q.h + q.len) & gm] = x;
    else l[((q.h + q.len) & (kDqL - 1)) * LS] = x;
    q.len++;
    q.b = x;
    q.nan |= d_isnan(x);
    if (q.len == 1) q.f = x;
    if (!q.mmh || d_worse<MIN>(q.mm, x)) { q.mm = x; q.mmh = true; }
}

// BYRANK: `rec` is the push's records in rank order (no k_sl_gather pass): the chunk's fields are
// read through the partition's rank list, and their latency overlaps the other waves' replay
template <bool HSUM, bool HMIN, bool HMAX, bool BYRANK>
__global__ __launch_bounds__(64) void k_sl_own_d(const u32* __restrict__ rank_list, const i64* __restrict__ part_off,
                                                int logP, SlRecords rec, SlState S, AggPlan ap, DFields fd, i64 T,
                                                i64 send_size, i64 send_base, SlRows rows, unsigned char* flags) {
    // KL key lanes per wave (one key each when the partition has <= KL local keys): few lanes keep
    // the divergence of the per-key chains low, and the small LDS footprint (≈ 11 KB) lets many
    // waves share a CU, which is what hides each chain's instruction latency
    constexpr int KL = kSlKeyLanes;
    constexpr int CH = SH_SL_CH;
    __shared__ u32 ch_rank[CH];
    __shared__ u32 ch_slot[CH];
    __shared__ unsigned short list[CH];
    __shared__ i64 ch_clk[CH];
    __shared__ i64 ch_pm[CH];
    __shared__ i64 ch_ts[CH];
    __shared__ u32 ch_raw[CH];
    __shared__ u64 ch_v[CH];
    __shared__ u32 run[64];
    __shared__ i64 hb_pm[KL * kHb];
    __shared__ u64 hb_v[KL * kHb];
    __shared__ u64 dq_min[KL * kDqL];
    __shared__ u64 dq_max[KL * kDqL];
    const int lane = threadIdx.x;
    const int kl = lane & (KL - 1);
    u64* lmin = dq_min + kl * kDqL;
    u64* lmax = dq_max + kl * kDqL;
    const i64 lo = part_off[blockIdx.x], hi = part_off[blockIdx.x + 1];
    const i64 gm = S.rc - 1;
    // lane state
    u32 K = kNoPos;
    i64 cnt = 0, rh = 0, rlen = 0, cur_send = 0, cur_first = 0, hb_base = 0;
    int hb_n = 0;
    u64 sum = 0;
    DDeque qn{}, qx{};
    u64* gmin = nullptr;
    u64* gmax = nullptr;
    auto store_key = [&]() {
        S.cnt[K] = cnt;
        S.rhead[K] = rh;
        S.rlen[K] = rlen;
        S.cur_send[K] = cur_send;
        S.cur_first[K] = cur_first;
        if (HSUM) {
            if (fd.sum >= 0) S.f[(size_t)fd.sum * S.nslots + K] = sum;
            if (fd.avg >= 0) S.f[(size_t)fd.avg * S.nslots + K] = sum;
        }
        if (HMIN) dd_store(qn, S, fd.mn, K, lmin);
        if (HMAX) dd_store(qx, S, fd.mx, K, lmax);
    };
    for (i64 c0 = lo; c0 < hi; c0 += CH) {
        const int n = (int)min<i64>(CH, hi - c0);
        u32 mine, start;
        if (!BYRANK) {
            // the chunk's fields, coalesced (the records are in partition order), into LDS
#pragma unroll 4
            for (int g = 0; g < CH; g += 64) {
                const int j = g + lane;
                if (j < n) {
                    ch_clk[j] = rec.clock[c0 + j];
                    ch_pm[j] = rec.pm[c0 + j];
                    ch_ts[j] = rec.ts[c0 + j];
                    ch_raw[j] = rec.raw[c0 + j];
                    ch_v[j] = rec.vals[c0 + j];
                }
            }
        }
        sl_chunk_split<KL, BYRANK>(rank_list, rec.slot, c0, n, logP, ch_rank, ch_slot, list, run, mine, start);
        if (BYRANK) {
            // each thread fetches the fields of the records whose rank it staged in the split
#pragma unroll 4
            for (int g = 0; g < CH; g += 64) {
                const int j = g + lane;
                if (j < n) {
                    const u32 rk = ch_rank[j];
                    ch_clk[j] = rec.clock[rk];
                    ch_pm[j] = rec.pm[rk];
                    ch_ts[j] = rec.ts[rk];
                    ch_raw[j] = rec.raw[rk];
                    ch_v[j] = rec.vals[rk];
                }
            }
            __syncthreads();
        }
        for (u32 i = 0; i < mine; i++) {
            const int j = list[start + i];
            const u32 r = ch_rank[j], k = ch_slot[j];
            const i64 clk = ch_clk[j], pmr = ch_pm[j], tsr = ch_ts[j];
            const u32 raw = ch_raw[j];
            const u64 x = ch_v[j];
            if (k != K) {
                if (K != kNoPos) store_key();
                K = k;
                cnt = S.cnt[k];
                rh = S.rhead[k];
                rlen = S.rlen[k];
                cur_send = S.cur_send[k];
                cur_first = S.cur_first[k];
                hb_n = 0;
                if (HSUM) sum = S.f[(size_t)(fd.sum >= 0 ? fd.sum : fd.avg) * S.nslots + k];
                if (HMIN) { dd_load(qn, S, fd.mn, k, lmin); gmin = S.dq + ((size_t)fd.mn * S.nslots + k) * S.rc; }
                if (HMAX) { dd_load(qx, S, fd.mx, k, lmax); gmax = S.dq + ((size_t)fd.mx * S.nslots + k) * S.rc; }
            }
            // lazy expiry: ring head events with PM + T <= clock (TimeWindowProcessor.java:132-169)
            while (rlen > 0) {
                if (!(rh >= hb_base && rh < hb_base + hb_n)) {  // refill the head cache
                    const int m = (int)min<i64>(kHb, rlen);
                    i64 pm8[kHb];
                    u64 v8[kHb];
#pragma unroll
                    for (int e = 0; e < kHb; e++) {
                        if (e < m) {
                            const i64 sl = (rh + e) & gm;
                            pm8[e] = S.rpm[(size_t)k * S.rc + sl];
                            v8[e] = S.rval[(size_t)k * S.rc + sl];
                        }
                    }
#pragma unroll
                    for (int e = 0; e < kHb; e++)
                        if (e < m) { hb_pm[kl * kHb + e] = pm8[e]; hb_v[kl * kHb + e] = v8[e]; }
                    hb_base = rh;
                    hb_n = m;
                }
                const int e = (int)(rh - hb_base);
                if (hb_pm[kl * kHb + e] + T > clk) break;
                const u64 y = hb_v[kl * kHb + e];
                cnt--;
                if (HSUM) {
                    double rr = __longlong_as_double((i64)sum) - __longlong_as_double((i64)y);
                    if (cnt == 0 && rr == 0.0) rr = 0.0;  // destroyed state restarts from +0.0
                    sum = (u64)__double_as_longlong(rr);
                }
                if (HMIN) dd_remove<true>(qn, gmin, gm, lmin, y);
                if (HMAX) dd_remove<false>(qx, gmax, gm, lmax, y);
                rh++;
                rlen--;
            }
            // the event joins the ring and the aggregators
            const i64 sl = (rh + rlen) & gm;
            S.rpm[(size_t)k * S.rc + sl] = pmr;
            S.rval[(size_t)k * S.rc + sl] = x;
            rlen++;
            cnt++;
            if (HSUM) sum = (u64)__double_as_longlong(__longlong_as_double((i64)sum) + __longlong_as_double((i64)x));
            if (HMIN) dd_add<true>(qn, gmin, gm, lmin, x);
            if (HMAX) dd_add<false>(qx, gmax, gm, lmax, x);
            // output row of (send, key): first occurrence position, last event's values
            const i64 send = send_base + (send_size > 0 ? (i64)raw / send_size : 0);
            i64 first;
            if (cur_send != send) { cur_send = send; cur_first = r; first = r; flags[r] = 1; }
            else first = cur_first;
#ifdef SH_SL_EXP_NOROWS
            if (first != 0x7fffffff) continue;  // timing experiment only: no row stores
#endif
            rows.ts[first] = tsr;
            rows.rep[first] = raw;
            rows.slot[first] = k;
            rows.send[first] = send;
            rows.clock[first] = clk;
            for (int a = 0; a < ap.n; a++) {
                const int kind = ap.kind[a];
                u64 o = 0;
                unsigned char nl = 0;
                if (kind == AK_COUNT) o = (u64)cnt;
                else if (kind == AK_SUM_D) o = sum;
                else if (kind == AK_AVG) o = (u64)__double_as_longlong(__longlong_as_double((i64)sum) / (double)cnt);
                else if (kind == AK_MIN_D) { o = qn.mm; nl = qn.mmh ? 0 : 1; }
                else { o = qx.mm; nl = qx.mmh ? 0 : 1; }
                rows.vals[(size_t)a * rows.cap + first] = o;
                rows.nulls[(size_t)a * rows.cap + first] = nl;
            }
        }
        __syncthreads();
    }
    if (K != kNoPos) store_key();
}

template <int NA, int NV>
__global__ __launch_bounds__(64) void k_sl_own(const u32* __restrict__ rank_list, const i64* __restrict__ part_off,
                                              int logP, SlRecords rec, SlState S, AggPlan ap, i64 T, i64 send_size,
                                              i64 send_base, SlRows rows, unsigned char* flags) {
    __shared__ u32 ch_rank[kSlCh];
    __shared__ u32 ch_slot[kSlCh];
    __shared__ unsigned short list[kSlCh];
    __shared__ u32 run[64];
    __shared__ i64 hb_pm[64 * kHb];
    __shared__ u64 hb_v[NV * 64 * kHb];
    extern __shared__ __attribute__((aligned(16))) u64 lds_dq[];  // [min/max aggregator][lane][kDqL]
    const int p = blockIdx.x;
    const int lane = threadIdx.x;
    const u64 lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    const i64 lo = part_off[p], hi = part_off[p + 1];
    int mmi[NA];
    {
        int c = 0;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            mmi[a] = c;
            if (a < ap.n && is_mm(ap.kind[a])) c++;
        }
    }
    LaneKey<NA, NV> L;
    L.k = kNoPos;
    L.hvalid = false;
    L.hb_n = 0;
    L.hb_base = 0;
    for (i64 c0 = lo; c0 < hi; c0 += kSlCh) {
        const int n = (int)min<i64>(kSlCh, hi - c0);
        // per-lane counts of the chunk
        u32 mine = 0;
        for (int g = 0; g < n; g += 64) {
            const int j = g + lane;
            u32 o = 64;
            if (j < n) {
                const u32 r = rank_list[c0 + j];
                const u32 k = rec.slot[c0 + j];
                o = (k >> logP) & 63;
                ch_rank[j] = r;
                ch_slot[j] = k;
            }
            // how many of this group's records go to my lane
            u64 mask = __ballot(j < n);
#pragma unroll
            for (int bt = 0; bt < 6; bt++) {
                const u64 b = __ballot((o >> bt) & 1);
                mask &= ((lane >> bt) & 1) ? b : ~b;
            }
            mine += (u32)__popcll(mask);
        }
        // exclusive scan of the lane counts -> list starts
        u32 incl = mine;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u32 y = __shfl_up(incl, d, 64);
            if (lane >= d) incl += y;
        }
        const u32 start = incl - mine;
        run[lane] = start;
        __syncthreads();
        // stable placement: rank among the group's same-owner records + that owner's running count
        for (int g = 0; g < n; g += 64) {
            const int j = g + lane;
            const bool ok = j < n;
            const u32 o = ok ? ((ch_slot[j] >> logP) & 63) : 0;
            u64 peers = __ballot(ok);
#pragma unroll
            for (int bt = 0; bt < 6; bt++) {
                const bool bit = (o >> bt) & 1;
                const u64 b = __ballot(bit);
                peers &= bit ? b : ~b;
            }
            const u32 lr = (u32)__popcll(peers & lt_mask);
            u32 base = 0;
            if (ok) base = run[o];
            __syncthreads();
            if (ok) list[base + lr] = (unsigned short)j;
            if (ok && lr == 0) run[o] = base + (u32)__popcll(peers);
            __syncthreads();
        }
        // replay: my key's events in order, the next record's fields loaded one step ahead
        SlRec<NV> nx;
        if (mine > 0) sl_rec_load(nx, rec, ap, c0 + list[start]);
        for (u32 i = 0; i < mine; i++) {
            const int j = list[start + i];
            const u32 r = ch_rank[j], k = ch_slot[j];
            const SlRec<NV> cur = nx;
            if (i + 1 < mine) sl_rec_load(nx, rec, ap, c0 + list[start + i + 1]);
            if (k != L.k) {
                if (L.k != kNoPos) lk_store(L, S, ap, lds_dq, mmi);
                lk_load(L, S, ap, lds_dq, mmi, k);
            }
            const i64 clk = cur.clk;
            // lazy expiry: ring head events with PM + T <= clock (TimeWindowProcessor.java:132-169)
            while (L.rlen > 0) {
                if (!L.hvalid) lk_head(L, S, ap, hb_pm, hb_v);
                if (L.hpm + T > clk) break;
                lk_remove(L, S, ap, lds_dq, mmi, L.hval);
                L.rh++;
                L.rlen--;
                L.hvalid = false;
                if (L.rlen > 0) lk_head(L, S, ap, hb_pm, hb_v);
            }
            // the event joins the ring and the aggregators
            const i64 sl = (L.rh + L.rlen) & (S.rc - 1);
            S.rpm[(size_t)k * S.rc + sl] = cur.pm;
#pragma unroll
            for (int q = 0; q < NV; q++) {
                if (q >= ap.n_vcols) break;
                S.rval[((size_t)q * S.nslots + k) * S.rc + sl] = cur.v[q];
            }
            if (L.rlen == 0) {
                L.hpm = cur.pm;
#pragma unroll
                for (int q = 0; q < NV; q++) {
                    if (q >= ap.n_vcols) break;
                    L.hval[q] = cur.v[q];
                }
                L.hvalid = true;
            }
            L.rlen++;
            lk_add(L, S, ap, lds_dq, mmi, cur.v);
            // output row of (send, key): first occurrence position, last event's values
            const i64 send = send_base + (send_size > 0 ? (i64)cur.raw / send_size : 0);
            i64 first;
            if (L.cur_send != send) { L.cur_send = send; L.cur_first = r; first = r; flags[r] = 1; }
            else first = L.cur_first;
            rows.ts[first] = cur.ts;
            rows.rep[first] = cur.raw;
            rows.slot[first] = k;
            rows.send[first] = send;
            rows.clock[first] = clk;
            const i64 c = L.cnt;
#pragma unroll
            for (int a = 0; a < NA; a++) {
                if (a >= ap.n) break;
                const int kind = ap.kind[a];
                u64 o;
                unsigned char nl = 0;
                if (kind == AK_COUNT) o = (u64)c;
                else if (kind == AK_SUM_L || kind == AK_SUM_D) o = L.f[a];
                else if (kind == AK_AVG) o = (u64)__double_as_longlong(__longlong_as_double((i64)L.f[a]) / (double)c);
                else { o = L.mm[a]; nl = L.mmh[a] ? 0 : 1; }
                rows.vals[(size_t)a * rows.cap + first] = o;
                rows.nulls[(size_t)a * rows.cap + first] = nl;
            }
        }
        __syncthreads();
    }
    if (L.k != kNoPos) lk_store(L, S, ap, lds_dq, mmi);
}

// rank-indexed records -> partition order (position q of the multisplit's rank list), so the
// per-key replay reads each partition's records from one contiguous range
__global__ __launch_bounds__(kBlock) void k_sl_gather(const u32* __restrict__ ranks, i64 M, SlRecords rec, SlRecords out,
                                                     int nv) {
    const i64 q = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (q >= M) return;
    const u32 r = ranks[q];
    out.raw[q] = rec.raw[r];
    out.slot[q] = rec.slot[r];
    out.clock[q] = rec.clock[r];
    out.pm[q] = rec.pm[r];
    out.ts[q] = rec.ts[r];
    for (int j = 0; j < nv; j++) out.vals[(size_t)j * out.cap + q] = rec.vals[(size_t)j * rec.cap + r];
}

void launch_sl_gather(hipStream_t s, const u32* ranks, i64 M, SlRecords rec, SlRecords out, int nv) {
    if (M <= 0) return;
    hipLaunchKernelGGL(k_sl_gather, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, ranks, M, rec, out,
                       nv);
}

// the double-column shape (C3): count + at most one each of sum / avg / min / max of one DOUBLE
static bool own_d_fields(const AggPlan& ap, DFields& fd) {
    fd = DFields{-1, -1, -1, -1};
    bool ok = ap.n_vcols == 1 && ap.vcol_type[0] == SH_T_DOUBLE;
    for (int a = 0; ok && a < ap.n; a++) {
        int* slotp = nullptr;
        switch (ap.kind[a]) {
            case AK_COUNT: continue;
            case AK_SUM_D: slotp = &fd.sum; break;
            case AK_AVG: slotp = &fd.avg; break;
            case AK_MIN_D: slotp = &fd.mn; break;
            case AK_MAX_D: slotp = &fd.mx; break;
            default: ok = false; continue;
        }
        if (*slotp >= 0) ok = false;
        else *slotp = ap.field[a];
    }
    return ok;
}

// keys a key partition should hold so that every key gets a lane of its own in the replay kernel
// (k_sl_own_d: kSlKeyLanes per wave; k_sl_own: 64). A lane owning several keys switches per-key
// state (global loads and stores) whenever consecutive records of its list change key.
// ---- key-sorted replay: the records of a push sorted stably by key slot (sh_sort.hip), so each key's
// events form one contiguous run in event order, walked by one wave per key (k_sl_wkey). The key's
// window is its carried ring (events of earlier pushes) followed by the run itself; only the entries
// still in the window at the end of the push go to the ring. Rows are written in key order as one record
// each (full-line stores) and put in stream order by the emit kernel. ------------------------------------
// resident waves per SIMD the wave-per-key replays are compiled for: k_sl_wkey at 4 (128 VGPRs, 8 bytes
// of spill; left alone the compiler takes 131 and 3 waves: C3 8.29 -> 7.53 ms per push, r05_wpe; 5
// spills 412 bytes and runs 3x slower); timing experiments override it
#ifndef SH_WK_WPE
#define SH_WK_WPE 4
#endif
#define SH_WK_ATTR __attribute__((amdgpu_waves_per_eu(SH_WK_WPE)))
#ifdef SH_XW_WPE
#define SH_XW_ATTR __attribute__((amdgpu_waves_per_eu(SH_XW_WPE)))
#else
#define SH_XW_ATTR
#endif
constexpr int kDqK = 64;  // LDS min/max deque entries per lane (longer deques continue in global memory)
constexpr u32 kFirstBit = 0x80000000u;

__global__ void k_sl_keyoff(const u32* __restrict__ slot_cnt, i64 nslots, u32* key_off) {
    const i64 k = (i64)blockIdx.x * blockDim.x + threadIdx.x;
    if (k <= nslots) key_off[k] = k < nslots ? slot_cnt[k] : 0u;
}

// Wait for this wave's vector-memory loads right where a rare path issued them. The replay step keeps
// the next step's loads and this step's row stores in flight; a load result that flows out of a
// rare branch would otherwise make the compiler wait for every outstanding vector-memory operation
// at the merge point, on every record, taken or not (the counter retires in order).
__device__ __forceinline__ void wait_vm_here() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0)

// a lane's min or max deque (MinAttributeAggregatorExecutor's LinkedList with removeFirstOccurrence):
// ring `l` in LDS (kDqK entries, lane-interleaved) or, once longer, ring `g` in global memory
struct KDq {
    int h, len;
    u64 f, b, mm;
    bool mmh, spill, nan;
};

// GLOBAL: the deque lives in its global ring; otherwise in LDS. Separate instances, so each uses plain
// LDS or global instructions (no pointer select)
template <bool MIN, bool GLOBAL, int KL>
__device__ __forceinline__ void kdq_remove_t(KDq& q, u64* g, int gm, u64* l, u64 x) {
    auto at = [&](int i) -> u64 {
        if (!GLOBAL) return l[(i & (kDqK - 1)) * KL];
        const u64 v = g[i & gm];
        wait_vm_here();
        return v;
    };
    if (q.len > 0 && d_eq(q.f, x)) {
        q.h++;
        q.len--;
        if (q.len > 0) q.f = at(q.h);
    } else if (q.len > 1 && (q.nan || !d_worse<MIN>(x, q.b))) {
        int found = -1;
        if (!q.nan) {
            // NaN-free: the deque is monotone (min: non-decreasing), so the first entry not better
            // than x is found by bisection; x is present iff that entry equals it
            int lo = 1, hi = q.len;  // answer in [lo, hi]
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (d_worse<MIN>(x, at(q.h + mid))) lo = mid + 1;
                else hi = mid;
            }
            // among numerically equal entries (0.0 / -0.0) Double.equals wants the same bits
            for (int i = lo; i < q.len; i++) {
                const u64 e = at(q.h + i);
                if (d_eq(e, x)) { found = i; break; }
                if (d_worse<MIN>(e, x)) break;  // past every entry equal to x
            }
        } else {
            for (int i = 1; i < q.len; i++)
                if (d_eq(at(q.h + i), x)) { found = i; break; }
        }
        if (found >= 0) {
            for (int i = found; i + 1 < q.len; i++) {
                const u64 v = at(q.h + i + 1);
                if (GLOBAL) g[(q.h + i) & gm] = v;
                else l[((q.h + i) & (kDqK - 1)) * KL] = v;
            }
            q.len--;
            q.b = at(q.h + q.len - 1);
        }
    }
    if (q.len > 0) { q.mm = q.f; q.mmh = true; }
    else { q.mmh = false; q.nan = q.spill; }
}

template <bool MIN, int KL>
__device__ __forceinline__ void kdq_remove(KDq& q, u64* g, int gm, u64* l, u64 x) {
    if (q.spill) kdq_remove_t<MIN, true, KL>(q, g, gm, l, x);
    else kdq_remove_t<MIN, false, KL>(q, g, gm, l, x);
}

template <bool MIN, bool GLOBAL, int KL>
__device__ __forceinline__ void kdq_pop_t(KDq& q, const u64* g, int gm, const u64* l, u64 x) {
    while (q.len > 0 && d_worse<MIN>(q.b, x)) {
        q.len--;
        if (q.len > 0) {
            if (GLOBAL) { q.b = g[(q.h + q.len - 1) & gm]; wait_vm_here(); }
            else q.b = l[((q.h + q.len - 1) & (kDqK - 1)) * KL];
        }
    }
}

template <bool MIN, int KL>
__device__ __forceinline__ void kdq_add(KDq& q, u64* g, int gm, u64* l, u64 x) {
    if (q.spill) kdq_pop_t<MIN, true, KL>(q, g, gm, l, x);
    else kdq_pop_t<MIN, false, KL>(q, g, gm, l, x);
    if (!q.spill && q.len == kDqK) {  // the LDS ring is full: the deque moves to its global ring
        for (int i = 0; i < q.len; i++) g[(q.h + i) & gm] = l[((q.h + i) & (kDqK - 1)) * KL];
        q.spill = true;
        q.nan = true;  // the global path always scans
    }
    if (q.spill) g[(q.h + q.len) & gm] = x;
    else l[((q.h + q.len) & (kDqK - 1)) * KL] = x;
    q.len++;
    q.b = x;
    q.nan |= d_isnan(x);
    if (q.len == 1) q.f = x;
    if (!q.mmh || d_worse<MIN>(q.mm, x)) { q.mm = x; q.mmh = true; }
}

template <int KL>
__device__ __forceinline__ void kdq_load(KDq& q, const SlState& S, int field, u32 k, u64* l) {
    const size_t fi = (size_t)field * S.nslots + k;
    q.mm = S.mm[fi];
    q.mmh = S.mm_has[fi];
    q.len = (int)S.dq_len[fi];
    q.h = (int)(S.dq_head[fi] & (S.rc - 1));
    q.spill = q.len > kDqK;
    q.nan = q.spill;
    const u64* g = S.dq + fi * S.rc;
    const int gm = (int)(S.rc - 1);
    if (!q.spill) {
        for (int i = 0; i < q.len; i++) {
            const u64 v = g[(q.h + i) & gm];
            l[((q.h + i) & (kDqK - 1)) * KL] = v;
            q.nan |= d_isnan(v);
        }
    }
    if (q.len > 0) {
        q.f = g[q.h & gm];
        q.b = g[(q.h + q.len - 1) & gm];
    }
}

template <int KL>
__device__ __forceinline__ void kdq_store(const KDq& q, const SlState& S, int field, u32 k, const u64* l) {
    const size_t fi = (size_t)field * S.nslots + k;
    S.mm[fi] = q.mm;
    S.mm_has[fi] = q.mmh;
    const int gm = (int)(S.rc - 1);
    S.dq_head[fi] = q.h & gm;
    S.dq_len[fi] = q.len;
    u64* g = S.dq + fi * S.rc;
    if (!q.spill)
        for (int i = 0; i < q.len; i++) g[(q.h + i) & gm] = l[((q.h + i) & (kDqK - 1)) * KL];
}

// output aggregator sources of the keyed replay: 0 count, 1 sum, 2 avg, 3 min, 4 max
struct KOut {
    int n;
    int src[SH_MAX_AGGS];
};

// ---- one wave per key (round 3): the 64 lanes of a wave share one key's run, 64 records at a time.
// Everything per record that does not depend on the running aggregates is computed lane-parallel:
// the expiry prefix (the heads with PM + T <= the record's clock form a prefix, PM and the clock both
// being non-decreasing along a key's events — one binary search per lane over the staged heads), the
// count, the row position and the row stores. The Java-order double sum runs sequentially, by the whole
// wave in lockstep on wave-uniform state, reading the records' values and expiry points from the lanes'
// registers (readlane). With a wave per key a SIMD holds several keys' waves, whose sequential parts
// interleave. TimeWindowProcessor.java:132-169; QuerySelector.processInBatchGroupBy :315-374.
//
// Min / max off the sequential chain (round 4). MinAttributeAggregatorExecutor (:187-236) keeps a
// LinkedList deque: processAdd pops the back while it is strictly worse, processRemove calls
// removeFirstOccurrence(value) and reads the front. The expiring event is the window's oldest, so when it
// is in the deque it is the front and leaves; the result differs from the window's true minimum only if
// it was popped earlier and a bit-equal value sits in the deque (the reference's quirk), or once a NaN
// breaks the order. While neither can happen the deque after every event is the monotone deque of the
// window and minValue is the window's range minimum (the older entry on ties, which the front and the
// strict `minValue > value` both keep). So per chunk the lanes check that no expiring head meets a
// bit-equal value among the deque (entries carry their window index) or the chunk's records and that no
// NaN is in sight, then compute each record's result in parallel: the first deque entry at or after the
// record's first unexpired head, against the leftmost best of the chunk's records in its window. The
// deque after the chunk is the old entries still unexpired and not worse than the chunk's best, then the
// chunk's suffix bests. A chunk that fails the check or would outgrow the LDS ring runs the sequential
// deque (kdq_*), and its key stays sequential for the rest of the push (the indices are not kept there).
constexpr int kWS = 128;  // window-head entries staged per chunk (two per lane)

// The quirk check compares every expiring head with each of the chunk's records; bit-equal pairs are
// rare, so the records first go into a 32K-bit filter in LDS and a head runs the exact comparison only
// on a hit (about 0.2% of heads on distinct values). One wave per block: its LDS accesses are in order.
constexpr int kBfWords = 1024;
__device__ __forceinline__ u32 bf_hash(u64 v) { return (u32)((v * 0x9E3779B97F4A7C15ull) >> 49); }
__device__ __forceinline__ void bf_init(u32* bf, int lane) {
    for (int i = lane; i < kBfWords; i += 64) bf[i] = 0;
}
__device__ __forceinline__ bool bf_hit(const u32* bf, u64 v) {
    const u32 h = bf_hash(v);
    return (bf[h >> 5] >> (h & 31)) & 1u;
}

// lane l's value of a 64-bit register (l wave-uniform)
__device__ __forceinline__ u64 rl64(u64 v, int l) {
    const u32 lo = (u32)__builtin_amdgcn_readlane((int)(u32)v, l);
    const u32 hi = (u32)__builtin_amdgcn_readlane((int)(u32)(v >> 32), l);
    return ((u64)hi << 32) | lo;
}

__device__ __forceinline__ u64 shfl64(u64 v, int src) {
    const u32 lo = (u32)__shfl((int)(u32)v, src, 64), hi = (u32)__shfl((int)(u32)(v >> 32), src, 64);
    return ((u64)hi << 32) | lo;
}

// a (value, present) pair's leftmost-best combination: the right one only when strictly better
template <bool MIN>
__device__ __forceinline__ void best_comb(u64& bv, bool& bh, u64 v, bool h) {
    if (h && (!bh || d_worse<MIN>(bv, v))) { bv = v; bh = true; }
}

// The window indices of the deque loaded from the carried state: it must be the suffix-best chain of
// the carried ring (no quirk in its history), entry by entry, with minValue at its front; false leaves
// the key sequential.
template <bool MIN>
__device__ bool dq_index_init(const KDq& q, const u64* dv, int* di, const u64* rval, int rh0, int gm, int H0,
                              int lane) {
    if (q.spill || q.nan) return false;
    if (q.len == 0) return H0 == 0;
    if (!q.mmh || q.mm != dv[q.h & (kDqK - 1)]) return false;
    int seen = 0;      // chain entries found in the blocks after the current one
    u64 after = 0;     // best value after the current block
    bool after_h = false, ok = true;
    for (int b1 = H0; b1 > 0 && ok; b1 -= 64) {
        const int b0 = b1 - 64 > 0 ? b1 - 64 : 0, h = b0 + lane;
        const bool in = h < b1;
        const u64 v = in ? rval[(rh0 + h) & gm] : 0;
        if (__any(in && d_isnan(v))) return false;
        // inclusive suffix best over the block's lanes (a numeric best: all the membership test needs)
        u64 t = v;
        bool th = in;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            // (every lane runs every shuffle: a lane that skipped one would leave its source register stale)
            const int src = lane + d < 64 ? lane + d : lane;
            const u64 ov = shfl64(t, src);
            const int oth = __shfl(th ? 1 : 0, src, 64);
            const bool oh = lane + d < 64 && oth != 0;
            if (oh && (!th || d_worse<MIN>(t, ov))) { t = ov; th = true; }
        }
        // best strictly after h: the next lane's suffix, then the later blocks
        const int nx = lane + 1 < 64 ? lane + 1 : lane;
        u64 nb = shfl64(t, nx);
        const int nth = __shfl(th ? 1 : 0, nx, 64);
        bool nh = lane + 1 < 64 && nth != 0;
        if (after_h && (!nh || d_worse<MIN>(nb, after))) { nb = after; nh = true; }
        const bool member = in && !(nh && d_worse<MIN>(v, nb));
        const unsigned long long bal = __ballot(member);
        const int above = lane == 63 ? 0 : __popcll(bal >> (lane + 1));
        const int pos = q.len - 1 - seen - above;
        bool bad = false;
        if (member) {
            if (pos < 0) bad = true;
            else {
                const int sl = (q.h + pos) & (kDqK - 1);
                if (dv[sl] != v) bad = true;
                else di[sl] = h;
            }
        }
        ok = !__any(bad);
        seen += __popcll(bal);
        const u64 bv = shfl64(t, 0);
        const bool bh = __shfl(th ? 1 : 0, 0, 64) != 0;
        if (bh && (!after_h || d_worse<MIN>(after, bv))) { after = bv; after_h = true; }
    }
    return ok && seen == q.len;
}

// per lane: the result after its record — the first deque entry at or after lo_eff against the chunk's
// records [max(lo_eff, S), S + lane] (leftmost best)
template <bool MIN>
__device__ __forceinline__ u64 par_best(const KDq& q, const u64* dv, const int* di, const u64* sx, u64 x, int lo_eff,
                                         int S, bool in_from0, int lane) {
    int a = 0, b = q.len;
    while (a < b) {
        const int mid = (a + b) >> 1;
        if (di[(q.h + mid) & (kDqK - 1)] < lo_eff) a = mid + 1;
        else b = mid;
    }
    u64 pv = a < q.len ? dv[(q.h + a) & (kDqK - 1)] : 0;
    bool ph = a < q.len;
    u64 cv;
    bool ch;
    if (in_from0) {
        // every lane's range starts at the chunk's first record: an inclusive prefix scan
        cv = x;
        ch = true;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const u64 ov = shfl64(cv, lane >= d ? lane - d : lane);
            const bool oh = lane >= d;
            // left operand (earlier lanes) wins ties
            if (oh && !d_worse<MIN>(ov, cv)) cv = ov;
        }
    } else {
        ch = false;
        cv = 0;
        for (int j = lo_eff - S > 0 ? lo_eff - S : 0; j <= lane; j++) best_comb<MIN>(cv, ch, sx[j], true);
    }
    best_comb<MIN>(pv, ph, cv, ch);
    return pv;
}

// the deque after the chunk (see above); false when it would not fit the LDS ring (nothing written)
struct DqPlan {
    int i0, i1, n_new;
};
template <bool MIN>
__device__ __forceinline__ DqPlan dq_plan(const KDq& q, const u64* dv, const int* di, u64 x, bool in, int S,
                                          int lo_end, int m, int lane, bool& surv) {
    // chunk's best over all its records
    u64 cb = x;
    bool chh = in;
    u64 sb = x;  // suffix best strictly after the lane
    bool sbh = false;
    {
        u64 t = x;
        bool th = in;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {  // inclusive suffix scan
            // (every lane runs every shuffle: a lane that skipped one would leave its source register stale)
            const int src = lane + d < 64 ? lane + d : lane;
            const u64 ov = shfl64(t, src);
            const int oth = __shfl(th ? 1 : 0, src, 64);
            const bool oh = lane + d < 64 && oth != 0;
            if (oh && (!th || d_worse<MIN>(t, ov))) { t = ov; th = true; }
        }
        cb = shfl64(t, 0);
        chh = __shfl(th ? 1 : 0, 0, 64) != 0;
        const int src = lane + 1 < 64 ? lane + 1 : lane;
        sb = shfl64(t, src);
        const int sth = __shfl(th ? 1 : 0, src, 64);
        sbh = lane + 1 < 64 && sth != 0;
    }
    surv = in && S + lane >= lo_end && !(sbh && d_worse<MIN>(x, sb));
    DqPlan p;
    int a = 0, b = q.len;
    while (a < b) {
        const int mid = (a + b) >> 1;
        if (di[(q.h + mid) & (kDqK - 1)] < lo_end) a = mid + 1;
        else b = mid;
    }
    p.i0 = a;
    int c = a;
    if (chh)
        while (c < q.len && !d_worse<MIN>(dv[(q.h + c) & (kDqK - 1)], cb)) c++;
    else
        c = q.len;
    p.i1 = c;
    p.n_new = __popcll(__ballot(surv));
    (void)m;
    return p;
}

template <bool MIN>
__device__ __forceinline__ void dq_commit(KDq& q, u64* dv, int* di, const DqPlan& p, u64 x, bool surv, int S,
                                          int lane, u64 last_best) {
    const unsigned long long bal = __ballot(surv);
    const int rank = __popcll(bal & ((1ull << lane) - 1ull));
    if (surv) {
        const int sl = (q.h + p.i1 + rank) & (kDqK - 1);
        dv[sl] = x;
        di[sl] = S + lane;
    }
    __syncthreads();
    q.h += p.i0;
    q.len = p.i1 - p.i0 + p.n_new;
    if (q.len > 0) {
        q.f = dv[q.h & (kDqK - 1)];
        q.b = dv[(q.h + q.len - 1) & (kDqK - 1)];
    }
    q.mm = last_best;
    q.mmh = true;
}

// AOS: the records are read in key order through the sort's rank list from the 48-byte records
// (SlRecords.aos); the lanes write the key-order (PM, value) columns the window-head reads use, and
// the first-record flags / key-order positions the emit needs.
template <bool HSUM, bool HMIN, bool HMAX>
__global__ __launch_bounds__(64) SH_WK_ATTR void k_sl_wkey(const u32* __restrict__ key_off, u32 nslots, i64* __restrict__ g_pm,
                                               u64* __restrict__ g_v, SlState S, DFields fd, KOut ko, i64 T,
                                               u32 send_size, i64 send_base, u64* __restrict__ rowsK, int RW,
                                               const u32* __restrict__ sorted_rank, const u64* __restrict__ aos,
                                               unsigned char* __restrict__ flags) {
    __shared__ u64 dq_min[HMIN ? kDqK : 1];
    __shared__ u64 dq_max[HMAX ? kDqK : 1];
    __shared__ int di_min[HMIN ? kDqK : 1];
    __shared__ int di_max[HMAX ? kDqK : 1];
    __shared__ i64 s_pm[kWS];
    __shared__ u64 s_x[64];
    // the order-dependent sum chain of a chunk as one operation list (kWS removes + 64 adds at most)
    __shared__ u64 s_op[kWS + 64];
    __shared__ int s_lo[64];
    __shared__ unsigned char s_fl[kWS + 64];
    __shared__ u32 s_bf[kBfWords];
    const u32 k = blockIdx.x;
    const int lane = threadIdx.x;
    if (k >= nslots) return;
    const u32 a = key_off[k], b = key_off[k + 1];
    if (a == b) return;
    const int gm = (int)(S.rc - 1);
    const i64* rpm = S.rpm + (size_t)k * S.rc;
    const u64* rval = S.rval + (size_t)k * S.rc;
    const int rh0 = (int)(S.rhead[k] & gm), H0 = (int)S.rlen[k];
    const int n = (int)(b - a), HN = H0 + n;
    // the records are read through the sort's rank list and the key-order PM / value columns written here
    // (a key-ordered copy of the records, k_sl_kgather in round 5, cost what it saved: r05_c3_kgather_*)
    auto run_pm = [&](u32 j) -> i64 { return g_pm[j]; };
    auto run_v = [&](u32 j) -> u64 { return g_v[j]; };
    auto head_pm = [&](int h) -> i64 { return h < H0 ? rpm[(rh0 + h) & gm] : run_pm(a + (u32)(h - H0)); };
    auto head_v = [&](int h) -> u64 { return h < H0 ? rval[(rh0 + h) & gm] : run_v(a + (u32)(h - H0)); };
    // the running state: the same in every lane (the sequential part runs wave-uniform)
    i64 cnt = 0;
    double sum = 0.0;
    KDq qn{}, qx{};
    u64* gmin = HMIN ? S.dq + ((size_t)fd.mn * S.nslots + k) * S.rc : nullptr;
    u64* gmax = HMAX ? S.dq + ((size_t)fd.mx * S.nslots + k) * S.rc : nullptr;
    {
        cnt = S.cnt[k];
        if (HSUM) sum = __longlong_as_double((i64)S.f[(size_t)(fd.sum >= 0 ? fd.sum : fd.avg) * S.nslots + k]);
        if (HMIN) kdq_load<1>(qn, S, fd.mn, k, dq_min);
        if (HMAX) kdq_load<1>(qx, S, fd.mx, k, dq_max);
    }
    if (HMIN || HMAX) bf_init(s_bf, lane);
    __syncthreads();
    // the parallel min / max needs the deque entries' window indices
    bool par = HMIN || HMAX;
    if (HMIN && par) par = dq_index_init<true>(qn, dq_min, di_min, rval, rh0, gm, H0, lane);
    if (HMAX && par) par = dq_index_init<false>(qx, dq_max, di_max, rval, rh0, gm, H0, lane);
    __syncthreads();
    int hj = 0;         // heads expired so far
    int open_row = 0;   // key-order index of the (send, key) row open at the chunk start
    i64 last_send = 0;
    u32 prev_raw = 0;   // the previous chunk's last record
    for (int o0 = 0; o0 < n; o0 += 64) {
        const int m = min(64, n - o0);
        const bool in = lane < m;
        const u32 i = a + (u32)(o0 + min(lane, m - 1));
        i64 clk, ts;
        u64 x;
        u32 raw, rk;
        {
            const u32 r = sorted_rank[i];  // the record's stream rank
            const ulonglong2* rp = (const ulonglong2*)(aos + (size_t)r * kSlAosWords);
            const ulonglong2 w0 = rp[0], w1 = rp[1], w2 = rp[2];
            clk = (i64)w0.x;
            ts = (i64)w1.x;
            x = w1.y;
            raw = (u32)w2.x;
            // a record opens a row when it is its key's first of its send (every record per-event)
            u32 pr = __shfl_up(raw, 1, 64);
            if (lane == 0) pr = prev_raw;
            const bool fst = send_size == 1 || (o0 + lane == 0) || (send_size == 0 ? false : pr / send_size != raw / send_size);
            rk = r | (fst ? kFirstBit : 0u);
            if (in) {
                g_pm[i] = (i64)w0.y;  // the window-head columns, in key order
                g_v[i] = x;
                if (flags) flags[r] = fst ? 1 : 0;  // (per-event sends: every record opens its row, no flags)
            }
            s_x[lane] = x;
            prev_raw = __shfl(raw, m - 1, 64);
#ifndef SH_WK_NOFENCE
            __threadfence_block();  // this chunk's own records may expire within it
#endif
            __syncthreads();
        }
        const int hb = hj;
        // the next kWS window heads: PM in LDS (the lanes' binary searches), values in two registers
        // per lane (entry d in lane d & 63 of hv0 / hv1, read back with readlane by the sequential part)
        u64 hv0 = 0, hv1 = 0;
        if (hb + lane < HN) { s_pm[lane] = head_pm(hb + lane); hv0 = head_v(hb + lane); }
        if (hb + 64 + lane < HN) { s_pm[64 + lane] = head_pm(hb + 64 + lane); hv1 = head_v(hb + 64 + lane); }
        __syncthreads();
        // heads expired before this record: the first h in [hb, added) whose PM + T exceeds its clock
        int lo = hb, hi = in ? H0 + o0 + lane : hb;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            const i64 pm = mid - hb < kWS ? s_pm[mid - hb] : head_pm(mid);
            if (pm + T <= clk) lo = mid + 1;
            else hi = mid;
        }
        // the effective expiry point of each record: the running max over the earlier lanes
        int lo_eff = in ? lo : hb;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int up = __shfl_up(lo_eff, d, 64);
            if (lane >= d) lo_eff = max(lo_eff, up);
        }
        const int Sx = H0 + o0;  // window index of the chunk's first record
        u64 r_mn = 0, r_mx = 0;
        u32 r_fl = 0;
#ifdef SH_WK_NOPAR
        bool pc = false;  // (timing experiment only)
        par = false;
#else
        bool pc = par;  // this chunk's min / max in parallel
#endif
        DqPlan pn{}, px{};
        bool sn = false, sx_ = false;
        if (pc) {
            const int lo_end = __builtin_amdgcn_readlane(lo_eff, m - 1);
            const int ne = lo_end - hb;
            pc = ne <= kWS && !__any(in && d_isnan(x));
            if (pc) {
                // the quirk check: an expiring head meeting a bit-equal value of another event among the
                // deque entries or the chunk's records
                bool dirty = false;
#ifndef SH_WK_NODIRTY
                // (the filter holds the chunk's records and the deques' entries)
                const u32 hx = bf_hash(x);
                const u32 hn = HMIN && lane < qn.len ? bf_hash(dq_min[(qn.h + lane) & (kDqK - 1)]) : 0u;
                const u32 hm = HMAX && lane < qx.len ? bf_hash(dq_max[(qx.h + lane) & (kDqK - 1)]) : 0u;
                if (in) atomicOr(&s_bf[hx >> 5], 1u << (hx & 31));
                if (HMIN && lane < qn.len) atomicOr(&s_bf[hn >> 5], 1u << (hn & 31));
                if (HMAX && lane < qx.len) atomicOr(&s_bf[hm >> 5], 1u << (hm & 31));
                __syncthreads();
#pragma unroll
                for (int t = 0; t < 2; t++) {
                    const int d = lane + 64 * t;
                    if (d >= ne) continue;
                    const u64 v = t ? hv1 : hv0;
                    const int idx = hb + d;
                    if (!bf_hit(s_bf, v)) continue;
                    if (HMIN)
                        for (int e = 0; e < qn.len; e++) {
                            const int sl = (qn.h + e) & (kDqK - 1);
                            dirty |= dq_min[sl] == v && di_min[sl] != idx;
                        }
                    if (HMAX)
                        for (int e = 0; e < qx.len; e++) {
                            const int sl = (qx.h + e) & (kDqK - 1);
                            dirty |= dq_max[sl] == v && di_max[sl] != idx;
                        }
                    for (int j = 0; j < m; j++) dirty |= s_x[j] == v && Sx + j != idx;
                }
                __syncthreads();
                // (after every lane's test)
                if (in) s_bf[hx >> 5] = 0;
                if (HMIN && lane < qn.len) s_bf[hn >> 5] = 0;
                if (HMAX && lane < qx.len) s_bf[hm >> 5] = 0;
#endif
                pc = !__any(dirty);
            }
            if (pc) {
                const bool from0 = !__any(in && lo_eff > Sx);
                if (HMIN) r_mn = par_best<true>(qn, dq_min, di_min, s_x, x, lo_eff, Sx, from0, lane);
                if (HMAX) r_mx = par_best<false>(qx, dq_max, di_max, s_x, x, lo_eff, Sx, from0, lane);
                if (HMIN) pn = dq_plan<true>(qn, dq_min, di_min, x, in, Sx, lo_end, m, lane, sn);
                if (HMAX) px = dq_plan<false>(qx, dq_max, di_max, x, in, Sx, lo_end, m, lane, sx_);
                pc = (!HMIN || pn.i1 - pn.i0 + pn.n_new <= kDqK) && (!HMAX || px.i1 - px.i0 + px.n_new <= kDqK);
            }
            if (pc) {
                if (HMIN) dq_commit<true>(qn, dq_min, di_min, pn, x, sn, Sx, lane, rl64(r_mn, m - 1));
                if (HMAX) dq_commit<false>(qx, dq_max, di_max, px, x, sx_, Sx, lane, rl64(r_mx, m - 1));
                r_fl = 3;
            } else {
                par = false;  // the sequential deque takes over for the rest of the push
            }
        }
        // The order-dependent part, run by the whole wave in lockstep on wave-uniform values (so the
        // compiler keeps the running state scalar): each record's expiry point and value, and the
        // expiring heads' values, come from other lanes' registers by readlane instead of LDS, and
        // record q's results land in lane q's registers (a select, no LDS store).
        i64 r_cnt = 0;
        u64 r_sum = 0;
        // Fast chain: with the min / max handled in parallel (or none), what stays sequential is the
        // Java-order double sum. Record q's removes are the heads [lo_eff(q-1), lo_eff(q)) and its add
        // follows them, so every operation's place in the chunk's list is known in parallel: add q at
        // (lo_eff(q) - hb) + q, head d at d + #{q : lo_eff(q) <= hb + d}. The lanes write the values
        // (a remove as the negated value: a - b is a + (-b) exactly in IEEE 754), the counts are
        // closed-form, and the wave then only adds the list up in order, reading it from LDS with a
        // uniform address (no readlane per value), capturing the running sum after each add.
        const int R = __builtin_amdgcn_readlane(lo_eff, m - 1) - hb;  // heads expiring in the chunk
        const bool fast = (pc || (!HMIN && !HMAX)) && R <= kWS;
        if (fast) {
            const int nops = R + m;
            if (in) s_lo[lane] = lo_eff;
            for (int j = lane; j < nops; j += 64) s_fl[j] = 0;
            __syncthreads();
            const int ap_q = (lo_eff - hb) + lane;  // this lane's add (lanes < m)
            if (in) {
                s_op[ap_q] = x;
                s_fl[ap_q] = 1;
            }
#pragma unroll
            for (int t = 0; t < 2; t++) {
                const int d = lane + 64 * t;
                if (d >= R) continue;
                // adds before head d: the records whose expiry point is at or below it
                int lo2 = 0, hi2 = m;
                while (lo2 < hi2) {
                    const int mid = (lo2 + hi2) >> 1;
                    if (s_lo[mid] <= hb + d) lo2 = mid + 1;
                    else hi2 = mid;
                }
                s_op[d + lo2] = (t ? hv1 : hv0) ^ 0x8000000000000000ull;  // -v
                // the count after this remove: zero -> the sum restarts from +0.0 (canDestroy)
                if (cnt + lo2 - (d + 1) == 0) s_fl[d + lo2] = 2;
            }
            __syncthreads();
            u64 czm[3];
#pragma unroll
            for (int wd = 0; wd < 3; wd++) {
                const int j = wd * 64 + lane;
                const unsigned char fv = j < nops ? s_fl[j] : 0;
                czm[wd] = __ballot(fv == 2);
            }
            if (HSUM) {
                // each lane keeps the running sum at its own add (position ap_q); the canDestroy restarts
                // are rare, so a chunk without one runs the loop without their check
                double sm = sum;
                const int myop = in ? ap_q : -1;
                if ((czm[0] | czm[1] | czm[2]) == 0) {
                    for (int j = 0; j < nops; j++) {
                        sm = sm + __longlong_as_double((i64)s_op[j]);
                        r_sum = j == myop ? (u64)__double_as_longlong(sm) : r_sum;
                    }
                } else {
                    for (int j = 0; j < nops; j++) {
                        sm = sm + __longlong_as_double((i64)s_op[j]);
                        const int wd = j >> 6;
                        const u64 cz = wd == 0 ? czm[0] : wd == 1 ? czm[1] : czm[2];
                        if ((cz >> (j & 63)) & 1ull) sm = sm == 0.0 ? 0.0 : sm;
                        r_sum = j == myop ? (u64)__double_as_longlong(sm) : r_sum;
                    }
                }
                sum = sm;
            }
            r_cnt = cnt + (lane + 1) - (lo_eff - hb);
            cnt = cnt + m - R;
            hj = hb + R;
            __syncthreads();  // (s_op / s_lo / s_fl are refilled by the next chunk)
        }
#ifdef SH_WK_NOSEQ
        // (timing experiment only: the order-dependent chain skipped, results wrong)
        hj = max(hb, __builtin_amdgcn_readlane(lo_eff, m - 1));
        r_cnt = 1;
        if (false)
#endif
        if (!fast) {
            int h = hb;
            for (int q = 0; q < m; q++) {
                const int e = max(__builtin_amdgcn_readlane(lo, q), h);
                for (; h < e; h++) {  // expired heads leave, oldest first (processRemove)
                    const int d = h - hb;
                    const u64 v = d < 64 ? rl64(hv0, d) : d < kWS ? rl64(hv1, d - 64) : head_v(h);
                    cnt--;
                    if (HSUM) {
                        sum = sum - __longlong_as_double((i64)v);
                        if (cnt == 0 && sum == 0.0) sum = 0.0;  // destroyed state restarts from +0.0 (canDestroy)
                    }
                    if (!pc) {
                        if (HMIN) kdq_remove<true, 1>(qn, gmin, gm, dq_min, v);
                        if (HMAX) kdq_remove<false, 1>(qx, gmax, gm, dq_max, v);
                    }
                }
                const u64 xq = rl64(x, q);  // the event joins the window (processAdd)
                cnt++;
                if (HSUM) sum = sum + __longlong_as_double((i64)xq);
                if (!pc) {
                    if (HMIN) kdq_add<true, 1>(qn, gmin, gm, dq_min, xq);
                    if (HMAX) kdq_add<false, 1>(qx, gmax, gm, dq_max, xq);
                }
                if (lane == q) {
                    r_cnt = cnt;
                    r_sum = (u64)__double_as_longlong(sum);
                    if (!pc) {
                        r_mn = qn.mm;
                        r_mx = qx.mm;
                        r_fl = (qn.mmh ? 1u : 0u) | (qx.mmh ? 2u : 0u);
                    }
                }
            }
            hj = h;
        }
        // the row of (send, key): opened by the group's first record (its key-order position), written
        // with the values after the group's last record of this chunk (a later chunk overwrites it)
        const bool first = in && (rk & kFirstBit);
        int grp = first ? o0 + lane : -1;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const int up = __shfl_up(grp, d, 64);
            if (lane >= d) grp = max(grp, up);
        }
        grp = max(grp, open_row);
        // (the shuffle runs on every lane: a lane may only read a lane that executes it)
        const u32 rk_next = __shfl_down(rk, 1, 64);
        const bool next_first = lane + 1 < m ? (rk_next & kFirstBit) != 0 : true;
        const i64 send = send_base + (send_size == 1 ? (i64)raw : send_size ? (i64)(raw / send_size) : 0);
#ifdef SH_WK_NOROWS
        if (false) {  // (timing experiment only: no row stores)
#else
        if (in && next_first) {
#endif
            u64 w[4 + SH_MAX_AGGS];
            u32 nulls = 0;
            const i64 c = r_cnt;
            const u64 sb = r_sum;
            const u32 fl = r_fl;
            w[0] = (u64)ts;
            w[1] = (u64)raw | ((u64)k << 32);
            w[2] = (u64)clk;
#pragma unroll
            for (int o = 0; o < SH_MAX_AGGS; o++) {
                if (o >= ko.n) break;
                const int src = ko.src[o];
                u64 v = 0;
                if (src == 0) v = (u64)c;
                else if (src == 1) v = sb;
                else if (src == 2) v = (u64)__double_as_longlong(__longlong_as_double((i64)sb) / (double)c);
                else if (src == 3) { v = r_mn; nulls |= ((fl & 1) ? 0u : 1u) << o; }
                else { v = r_mx; nulls |= ((fl & 2) ? 0u : 1u) << o; }
                w[4 + o] = v;
            }
            w[3] = (u64)send | ((u64)nulls << 56);
            // the row lands at the stream rank of its first record, so the emission reads the rows in
            // stream order (whole lines) instead of gathering them from key order
            const u32 row_rank = grp == o0 + lane ? (rk & ~kFirstBit)
                                 : sorted_rank[a + (u32)grp];
            ulonglong2* dst = (ulonglong2*)(rowsK + (size_t)row_rank * RW);
            if (!flags) {
                // per-event sends: every record's row follows its own add (count >= 1, no nulls) and the
                // emission takes ts / clock / event / slot from the stream-order records, so the row is
                // its values alone — half the bytes of the random stores (r05: 2.4 ms of the replay)
#pragma unroll
                for (int o = 0; o < SH_MAX_AGGS / 2; o++)
                    if (2 * o < RW) dst[o] = make_ulonglong2(w[4 + 2 * o], w[4 + 2 * o + 1]);
            } else {
#pragma unroll
                for (int o = 0; o < (4 + SH_MAX_AGGS) / 2; o++)
                    if (2 * o < RW) dst[o] = make_ulonglong2(w[2 * o], w[2 * o + 1]);
            }
        }
        open_row = __shfl(grp, m - 1, 64);
        last_send = __shfl(send, m - 1, 64);
        __syncthreads();  // the staging arrays are refilled by the next chunk
    }
    // the window after the push: heads [hj, HN) — ring entries keep their place, the run's follow
    const int keep = hj < H0 ? H0 - hj : 0;
    const int rh = (rh0 + (hj < H0 ? hj : H0)) & gm;
    const int j0 = hj > H0 ? hj : H0;
    i64* wpm = S.rpm + (size_t)k * S.rc;
    u64* wval = S.rval + (size_t)k * S.rc;
    for (int j = j0 + lane; j < HN; j += 64) {
        const int sl = (rh + keep + (j - j0)) & gm;
        wpm[sl] = run_pm(a + (u32)(j - H0));
        wval[sl] = run_v(a + (u32)(j - H0));
    }
    if (lane == 0) {
        S.cnt[k] = cnt;
        S.rhead[k] = rh;
        S.rlen[k] = keep + (HN - j0);
        S.cur_send[k] = last_send;
        S.cur_first[k] = 0;
        if (HSUM) {
            const u64 sb = (u64)__double_as_longlong(sum);
            if (fd.sum >= 0) S.f[(size_t)fd.sum * S.nslots + k] = sb;
            if (fd.avg >= 0) S.f[(size_t)fd.avg * S.nslots + k] = sb;
        }
        if (HMIN) kdq_store<1>(qn, S, fd.mn, k, dq_min);
        if (HMAX) kdq_store<1>(qx, S, fd.mx, k, dq_max);
    }
}

// emit of the keyed replay: flagged ranks in stream order, each row read from its record at that rank
__global__ __launch_bounds__(kBlock) void k_slk_emit(const unsigned char* __restrict__ flags, i64 n,
                                                    const i64* __restrict__ blk_pre,
                                                    const u64* __restrict__ rowsK, int RW, int n_aggs, KeyTable kt,
                                                    KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals,
                                                    unsigned char* out_nulls, i64* out_send, i64* out_clock,
                                                    const u32* __restrict__ rank_raw, i64 raw_base, i64* out_order,
                                                    i64* out_rep, const u64* __restrict__ aos,
                                                    const u32* __restrict__ rank_slot) {
    const i64 tile = (i64)blockIdx.x * kTile;
    if (!flags) {
        // per-event sends: row j is record j's (compact: values only); the rest from the record itself
        for (int it = 0; it < kItems; it++) {
            const i64 j = tile + (i64)it * kBlock + threadIdx.x;
            if (j >= n) continue;
            const ulonglong2* rp = (const ulonglong2*)(aos + (size_t)j * kSlAosWords);
            const ulonglong2 w0 = rp[0], w1 = rp[1], w2 = rp[2];
            const u64* src = rowsK + (size_t)j * RW;
            out_ts[j] = (i64)w1.x;
            unpack_key(kp, slot_key(kt, rank_slot[j]), out_keys + j, out_cap);
            for (int a = 0; a < n_aggs; a++) {
                out_vals[(size_t)a * out_cap + j] = src[a];
                out_nulls[(size_t)a * out_cap + j] = 0;
            }
            out_clock[j] = (i64)w0.x;
            if (out_order) out_order[j] = raw_base + (i64)rank_raw[j];
            out_rep[j] = raw_base + (i64)(u32)w2.x;
        }
        return;
    }
    i64 run = flags ? blk_pre[blockIdx.x] : tile;
    for (int it = 0; it < kItems; it++) {
        const i64 j = tile + (i64)it * kBlock + threadIdx.x;
        i64 r = j;
        if (flags) {
            const i64 fl = j < n ? flags[j] : 0;
            i64 tot;
            r = run + block_excl_scan(fl, SumOp(), 0, &tot);
            run += tot;
            if (!fl) continue;
        } else if (j >= n) {
            continue;  // (per-event sends: every record's rank holds a row)
        }
        const u64* src = rowsK + (size_t)j * RW;
        u64 w[4 + SH_MAX_AGGS];
#pragma unroll
        for (int o = 0; o < (4 + SH_MAX_AGGS) / 2; o++) {
            if (2 * o >= RW) break;
            const ulonglong2 v = ((const ulonglong2*)src)[o];
            w[2 * o] = v.x;
            w[2 * o + 1] = v.y;
        }
        out_ts[r] = (i64)w[0];
        unpack_key(kp, slot_key(kt, (u32)(w[1] >> 32)), out_keys + r, out_cap);
        const u32 nulls = (u32)(w[3] >> 56);
        for (int a = 0; a < n_aggs; a++) {
            out_vals[(size_t)a * out_cap + r] = w[4 + a];
            out_nulls[(size_t)a * out_cap + r] = (nulls >> a) & 1u;
        }
        if (out_send) out_send[r] = (i64)(w[3] & ((1ull << 56) - 1));  // (per-event sends: the flushes are the rows)
        out_clock[r] = (i64)w[2];
        if (out_order) out_order[r] = raw_base + (i64)rank_raw[j];
        out_rep[r] = raw_base + (i64)(u32)w[1];
    }
}

void launch_slk_emit(hipStream_t s, const unsigned char* flags, i64 n, const i64* blk_pre, int nblk,
                     const u64* rowsK, int RW, int n_aggs, KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts,
                     i64* out_keys, u64* out_vals, unsigned char* out_nulls, i64* out_send, i64* out_clock,
                     const u32* rank_raw, i64 raw_base, i64* out_order, i64* out_rep, const u64* aos,
                     const u32* rank_slot) {
    hipLaunchKernelGGL(k_slk_emit, dim3(nblk), dim3(kBlock), 0, s, flags, n, blk_pre, rowsK, RW, n_aggs, kt, kp,
                       out_cap, out_ts, out_keys, out_vals, out_nulls, out_send, out_clock, rank_raw, raw_base,
                       out_order, out_rep, aos, rank_slot);
}

// The keyed replay is used where it measured faster than the key-partition replay (k_sl_own_d): with
// a min or max deque (C3's count/min/max/avg: 18.5 vs 20.7 ms per 16.7M-event push on MI355X);
// count/sum/avg alone stay on k_sl_own_d (5.5 vs 6.1 ms).
bool sliding_keyed_ok(AggPlan ap) {
    DFields fd;
    return own_d_fields(ap, fd) && ap.n <= SH_MAX_AGGS && (fd.mn >= 0 || fd.mx >= 0);
}

int sliding_keyed_row_words(int n_aggs, bool compact) { return compact ? (n_aggs + 1) & ~1 : (4 + n_aggs + 1) & ~1; }

void launch_sliding_keyed(hipStream_t s, const u32* slot_cnt, u32* key_off, i64* tmp, const u32* sorted_rank,
                          SlRecords rec, i64* g_pm, u64* g_v, SlState S, AggPlan ap, i64 T,
                          i64 send_size, i64 send_base, u64* rowsK, unsigned char* flags) {
    DFields fd;
    own_d_fields(ap, fd);
    KOut ko{};
    ko.n = ap.n;
    for (int q = 0; q < ap.n; q++) {
        const int kind = ap.kind[q];
        ko.src[q] = kind == AK_COUNT ? 0 : kind == AK_SUM_D ? 1 : kind == AK_AVG ? 2 : kind == AK_MIN_D ? 3 : 4;
    }
    const i64 n = S.nslots;
    const u32 ss = send_size > 0 ? (u32)send_size : 0u;
    {
        hipLaunchKernelGGL(k_sl_keyoff, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, s, slot_cnt, n, key_off);
        launch_scan_sum_large_u32(s, key_off, n + 1, tmp);
    }
    const bool hs = fd.sum >= 0 || fd.avg >= 0, hn = fd.mn >= 0, hx = fd.mx >= 0;
    const int RW = sliding_keyed_row_words(ap.n, flags == nullptr);
#define SH_SL_W(A, B, C)                                                                                            \
    hipLaunchKernelGGL((k_sl_wkey<A, B, C>), dim3((unsigned)n), dim3(64), 0, s, key_off, (u32)n, g_pm, g_v, S, fd, ko, \
                       T, ss, send_base, rowsK, RW, sorted_rank, rec.aos, flags)
    if (hs && hn && hx) SH_SL_W(true, true, true);
    else if (hs && !hn && !hx) SH_SL_W(true, false, false);
    else if (!hs && hn && hx) SH_SL_W(false, true, true);
    else if (hs && hn) SH_SL_W(true, true, false);
    else if (hs && hx) SH_SL_W(true, false, true);
    else if (hn && !hx) SH_SL_W(false, true, false);
    else if (hx && !hn) SH_SL_W(false, false, true);
    else SH_SL_W(false, false, false);
#undef SH_SL_W
}

int sliding_keys_per_partition(AggPlan ap) {
    DFields fd;
    return own_d_fields(ap, fd) ? kSlKeyLanes : 64;
}

// ---- `insert expired / all events`, one wave per key (round 5) ----------------------------------------
// k_slx_walk gives every key one lane that merges its adds and removes one dependent load at a time
// (c3all: 148 ms per push). Here the 64 lanes of a wave take a key's next 64 operations at once: the
// next 64 adds (its records in arrival order, each with its operation index aop) and the next 64
// removes (its FIFO entries, each with the operation index xop of its expiry point, kNoOp when it
// stays) are staged, and every staged operation finds its place in the merged order by a binary
// search over the other list; the first 64 places form the chunk. Per operation t the window is the
// FIFO range [head(t), end(t)), both counted by ballots, so the count is closed-form; the Java-order
// double sum is one operation list added up from LDS (a remove as the negated value, the canDestroy
// restart where the count reaches 0); the min / max is the range best of [head(t), end(t)) while the
// reference's deque quirk cannot show (the same check and deque bookkeeping as k_sl_wkey), else the
// deque runs sequentially for the rest of the push. Rows: one per (chunk, key), opened by its first
// qualifying operation (the row's place = that operation's index) and holding the values after its last
// one — the lanes are segmented by their chunk, a row still open at the chunk's end is written and
// overwritten by the next chunk. TimeWindowProcessor.java:132-169; QuerySelector.java:315-374.
constexpr u64 kSlxNoOp = ~0ull;

template <bool HSUM, bool HMIN, bool HMAX>
__global__ __launch_bounds__(64) SH_XW_ATTR void k_slx_wkey(const u32* __restrict__ key_off, u32 nslots,
                                                const u32* __restrict__ sorted_rank, const u64* __restrict__ xa,
                                                const u64* __restrict__ xx, i64 n_u, i64 X0, i64 G0, i64 seq_base,
                                                i64 send_size, SlState S, i64* __restrict__ rg, DFields fd, KOut ko,
                                                int cur_on, int exp_on, SlxRows rows,
                                                unsigned char* __restrict__ flags) {
    __shared__ u64 dq_min[HMIN ? kDqK : 1];
    __shared__ u64 dq_max[HMAX ? kDqK : 1];
    __shared__ int di_min[HMIN ? kDqK : 1];
    __shared__ int di_max[HMAX ? kDqK : 1];
    __shared__ u64 s_aop[64], s_ax[64], s_xop[64], s_xx[64], s_val[64];
    __shared__ u64 s_pbn[HMIN ? 64 : 1], s_pbx[HMAX ? 64 : 1];
    __shared__ int s_sel[64];
    __shared__ u32 s_bf[kBfWords];
    const u32 k = blockIdx.x;
    const int lane = threadIdx.x;
    if (k >= nslots) return;
    const u32 lo = key_off[k];
    const int A = (int)(key_off[k + 1] - lo);
    const int H0 = (int)S.rlen[k];
    if (A == 0 && H0 == 0) return;
    const int gm = (int)(S.rc - 1);
    const int rh0 = (int)(S.rhead[k] & gm);
    const size_t kr = (size_t)k * S.rc;
    const int HN = H0 + A;
    i64 cnt = S.cnt[k];
    double sum = 0.0;
    if (HSUM) sum = __longlong_as_double((i64)S.f[(size_t)(fd.sum >= 0 ? fd.sum : fd.avg) * S.nslots + k]);
    KDq qn{}, qx{};
    u64* gmin = HMIN ? S.dq + ((size_t)fd.mn * S.nslots + k) * S.rc : nullptr;
    u64* gmax = HMAX ? S.dq + ((size_t)fd.mx * S.nslots + k) * S.rc : nullptr;
    if (HMIN) kdq_load<1>(qn, S, fd.mn, k, dq_min);
    if (HMAX) kdq_load<1>(qx, S, fd.mx, k, dq_max);
    if (HMIN || HMAX) bf_init(s_bf, lane);
    __syncthreads();
#ifdef SH_XW_SEQ
    bool par = false;  // (timing experiment only: the sequential deque throughout)
#else
    bool par = HMIN || HMAX;
#endif
#ifdef SH_XW_NOROWS
    u64 xw_chk = 0;
#endif
    if (HMIN && par) par = dq_index_init<true>(qn, dq_min, di_min, S.rval + kr, rh0, gm, H0, lane);
    if (HMAX && par) par = dq_index_init<false>(qx, dq_max, di_max, S.rval + kr, rh0, gm, H0, lane);
    __syncthreads();
    const u64 le = (2ull << lane) - 1ull;  // lanes <= this one (lane 63: all)
    int ia = 0, ie = 0;                    // adds / FIFO entries consumed
    i64 row_ch = -1, row_op = 0;           // the (chunk, key) row open at the chunk start
    // the staged adds / FIFO entries: lane l holds add ia + l and entry ie + l; after a chunk the
    // unconsumed ones move down (shuffles) and only the freed lanes load (each record read once)
    u64 a_op = kSlxNoOp, a_x = 0, a_ts = 0, a_clk = 0, a_ch = 0, a_rep = 0;
    u64 x_op = kSlxNoOp, x_x = 0, x_ts = 0, x_clk = 0, x_ch = 0, x_rep = 0;
    int a_keep = 0, x_keep = 0;  // lanes still holding a staged operation
    for (;;) {
        // ---- stage up to the next 64 adds and the next 64 FIFO entries: one 48-byte record each (xa
        // by record, xx by window position), the row fields kept in the staging lane's registers
        if (lane >= a_keep) {
            a_op = kSlxNoOp;
            a_x = a_ts = a_clk = a_ch = a_rep = 0;
        }
        if (lane >= x_keep) {
            x_op = kSlxNoOp;
            x_x = x_ts = x_clk = x_ch = x_rep = 0;
        }
        if (lane >= a_keep && ia + lane < A) {
            const u32 ar = sorted_rank[lo + (u32)(ia + lane)];
            const ulonglong2* q = (const ulonglong2*)(xa + (size_t)ar * kXaWords);
            const ulonglong2 w0 = q[0], w1 = q[1], w2 = q[2];
            a_op = w0.x;
            a_x = w0.y;
            a_ts = w1.x;
            a_clk = w1.y;
            a_ch = 2 * (send_size > 0 ? w2.x / (u64)send_size : 0) + 1;
            a_rep = (u64)seq_base + w2.x;
        }
        const int p = ie + lane;
        if (lane >= x_keep && p < HN) {
            i64 x_u;
            if (p < H0) {
                const size_t sl = kr + (size_t)((rh0 + p) & gm);
                x_u = rg[sl] - X0;
                x_x = S.rval[sl];
            } else {
                x_u = G0 + (i64)sorted_rank[lo + (u32)(p - H0)] - X0;
            }
            if (x_u >= 0 && x_u < n_u) {
                const ulonglong2* q = (const ulonglong2*)(xx + (size_t)x_u * kXaWords);
                const ulonglong2 w0 = q[0], w1 = q[1], w2 = q[2];
                x_op = w0.x;
                if (p >= H0) x_x = w0.y;
                x_ts = w1.x;
                x_clk = w1.y;
                x_rep = w2.x;
                x_ch = w2.y;
            }
        }
        if (!__any(a_op != kSlxNoOp || x_op != kSlxNoOp)) break;
        s_aop[lane] = a_op;
        s_ax[lane] = a_x;
        s_xop[lane] = x_op;
        s_xx[lane] = x_x;
        __syncthreads();
        // ---- places in the merged order (both lists ascend; kNoOp pads the ends)
        int pa = 64, px = 64;
        if (a_op != kSlxNoOp) {
            int l2 = 0, h2 = 64;
            while (l2 < h2) {
                const int mid = (l2 + h2) >> 1;
                if (s_xop[mid] < a_op) l2 = mid + 1;
                else h2 = mid;
            }
            pa = lane + l2;
        }
        if (x_op != kSlxNoOp) {
            int l2 = 0, h2 = 64;
            while (l2 < h2) {
                const int mid = (l2 + h2) >> 1;
                if (s_aop[mid] < x_op) l2 = mid + 1;
                else h2 = mid;
            }
            px = lane + l2;
        }
        if (pa < 64) s_sel[pa] = lane;
        if (px < 64) s_sel[px] = 64 | lane;
        const int na_c = __popcll(__ballot(pa < 64)), nx_c = __popcll(__ballot(px < 64));
        const int m = na_c + nx_c;
        __syncthreads();
        // ---- this lane's operation
        const bool in = lane < m;
        const int sel = in ? s_sel[lane] : 0;
        const bool is_add = in && !(sel & 64);
        const int si = sel & 63;
        const u64 op = in ? (is_add ? s_aop[si] : s_xop[si]) : 0;
        const u64 val = is_add ? s_ax[si] : s_xx[si];
        // (every lane runs every shuffle)
        const u64 sa_ts = shfl64(a_ts, si), sa_clk = shfl64(a_clk, si), sa_ch = shfl64(a_ch, si),
                  sa_rep = shfl64(a_rep, si);
        const u64 sx_ts = shfl64(x_ts, si), sx_clk = shfl64(x_clk, si), sx_ch = shfl64(x_ch, si),
                  sx_rep = shfl64(x_rep, si);
        const u64 am = __ballot(is_add), xm = __ballot(in && !is_add);
        const int adds_le = __popcll(am & le), rems_le = __popcll(xm & le);
        i64 r_cnt = cnt + adds_le - rems_le;
        const int S0 = H0 + ia;        // window index of the chunk's first add
        const int h_t = ie + rems_le;  // window head after this operation
        const int h_end = ie + nx_c;
        u64 r_sum = 0, r_mn = 0, r_mx = 0;
        u32 r_fl = 0;
        bool pc = par;
        if (pc) {
            // min / max in parallel: no NaN, no expiring value meeting a bit-equal one of another event
            const bool ain = lane < na_c;  // add-space lane c = add ia + c (its staged lane)
            pc = !__any(ain && d_isnan(a_x));
            if (pc) {
                bool dirty = false;
                const u32 hx = bf_hash(a_x);
                if (ain) atomicOr(&s_bf[hx >> 5], 1u << (hx & 31));
                __syncthreads();
                if (lane < nx_c) {
                    const int idx = ie + lane;
                    const u64 v = x_x;
                    if (HMIN)
                        for (int e = 0; e < qn.len; e++) {
                            const int sl = (qn.h + e) & (kDqK - 1);
                            dirty |= dq_min[sl] == v && di_min[sl] != idx;
                        }
                    if (HMAX)
                        for (int e = 0; e < qx.len; e++) {
                            const int sl = (qx.h + e) & (kDqK - 1);
                            dirty |= dq_max[sl] == v && di_max[sl] != idx;
                        }
                    if (bf_hit(s_bf, v))
                        for (int c = 0; c < na_c; c++) dirty |= s_ax[c] == v && S0 + c != idx;
                }
                __syncthreads();
                if (ain) s_bf[hx >> 5] = 0;  // (after every lane's test)
                pc = !__any(dirty);
            }
            DqPlan pn{}, px_{};
            bool sn = false, sx = false;
            if (pc) {
                const bool from0 = h_end <= S0;  // no add of the chunk leaves within it
                if (from0) {
                    // leftmost-best prefix of the chunk's adds
                    u64 bn = a_x, bx = a_x;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const int src = lane >= d ? lane - d : lane;
                        const u64 on = shfl64(bn, src), ox = shfl64(bx, src);
                        if (lane >= d) {
                            if (!d_worse<true>(on, bn)) bn = on;
                            if (!d_worse<false>(ox, bx)) bx = ox;
                        }
                    }
                    if (HMIN) s_pbn[lane] = bn;
                    if (HMAX) s_pbx[lane] = bx;
                }
                __syncthreads();
                if (in) {
                    const int c0 = h_t - S0 > 0 ? h_t - S0 : 0;
                    auto best = [&](const KDq& q, const u64* dv, const int* di, const u64* pb, bool MINB) -> u64 {
                        int a = 0, b = q.len;
                        while (a < b) {
                            const int mid = (a + b) >> 1;
                            if (di[(q.h + mid) & (kDqK - 1)] < h_t) a = mid + 1;
                            else b = mid;
                        }
                        u64 bv = a < q.len ? dv[(q.h + a) & (kDqK - 1)] : 0;
                        bool bh = a < q.len;
                        u64 cv = 0;
                        bool chh = false;
                        if (from0) {
                            if (adds_le > 0) { cv = pb[adds_le - 1]; chh = true; }
                        } else {
                            for (int c = c0; c < adds_le; c++) {
                                const u64 v = s_ax[c];
                                if (!chh || (MINB ? d_worse<true>(cv, v) : d_worse<false>(cv, v))) { cv = v; chh = true; }
                            }
                        }
                        if (chh && (!bh || (MINB ? d_worse<true>(bv, cv) : d_worse<false>(bv, cv)))) bv = cv;
                        return bv;
                    };
                    if (HMIN) r_mn = best(qn, dq_min, di_min, s_pbn, true);
                    if (HMAX) r_mx = best(qx, dq_max, di_max, s_pbx, false);
                    r_fl = r_cnt > 0 ? 3u : 0u;
                }
                if (HMIN) pn = dq_plan<true>(qn, dq_min, di_min, a_x, ain, S0, h_end, na_c, lane, sn);
                if (HMAX) px_ = dq_plan<false>(qx, dq_max, di_max, a_x, ain, S0, h_end, na_c, lane, sx);
                pc = (!HMIN || pn.i1 - pn.i0 + pn.n_new <= kDqK) && (!HMAX || px_.i1 - px_.i0 + px_.n_new <= kDqK);
            }
            if (pc) {
                const bool live = cnt + na_c - nx_c > 0;
                if (HMIN) {
                    dq_commit<true>(qn, dq_min, di_min, pn, a_x, sn, S0, lane, rl64(r_mn, m - 1));
                    qn.mmh = live && qn.len > 0;
                }
                if (HMAX) {
                    dq_commit<false>(qx, dq_max, di_max, px_, a_x, sx, S0, lane, rl64(r_mx, m - 1));
                    qx.mmh = live && qx.len > 0;
                }
            } else {
                par = false;  // the sequential deque takes over for the rest of the push
            }
        }
        if (pc || (!HMIN && !HMAX)) {
            // the sum as one operation list: adds, negated removes, canDestroy restarts
            if (HSUM) {
                if (in) s_val[lane] = is_add ? val : val ^ 0x8000000000000000ull;
                const u64 czm = __ballot(in && !is_add && r_cnt == 0);
                __syncthreads();
                double sm = sum;
#ifdef SH_XW_NOSUM
                r_sum = s_val[lane] ^ czm;  // (timing experiment only: no sum chain)
#else
                if (czm == 0) {  // (the common chunk: no canDestroy restart to check)
                    for (int j = 0; j < m; j++) {
                        sm = sm + __longlong_as_double((i64)s_val[j]);
                        r_sum = lane == j ? (u64)__double_as_longlong(sm) : r_sum;
                    }
                } else {
                    for (int j = 0; j < m; j++) {
                        sm = sm + __longlong_as_double((i64)s_val[j]);
                        if ((czm >> j) & 1ull) sm = sm == 0.0 ? 0.0 : sm;
                        r_sum = lane == j ? (u64)__double_as_longlong(sm) : r_sum;
                    }
                }
#endif
                sum = sm;
            }
        } else {
            // sequential: every operation in order on wave-uniform state
            if (in) s_val[lane] = val;
            __syncthreads();
            i64 c = cnt;
            for (int j = 0; j < m; j++) {
                const bool ad = !(s_sel[j] & 64);
                const u64 v = s_val[j];
                if (ad) {
                    c++;
                    if (HSUM) sum = sum + __longlong_as_double((i64)v);
                    if (HMIN) kdq_add<true, 1>(qn, gmin, gm, dq_min, v);
                    if (HMAX) kdq_add<false, 1>(qx, gmax, gm, dq_max, v);
                } else {
                    c--;
                    if (HSUM) {
                        sum = sum - __longlong_as_double((i64)v);
                        if (c == 0 && sum == 0.0) sum = 0.0;  // destroyed state restarts from +0.0 (canDestroy)
                    }
                    if (HMIN) kdq_remove<true, 1>(qn, gmin, gm, dq_min, v);
                    if (HMAX) kdq_remove<false, 1>(qx, gmax, gm, dq_max, v);
                }
                if (lane == j) {
                    r_sum = (u64)__double_as_longlong(sum);
                    r_mn = qn.mm;
                    r_mx = qx.mm;
                    r_fl = (qn.mmh ? 1u : 0u) | (qx.mmh ? 2u : 0u);
                }
            }
        }
        cnt += na_c - nx_c;
        ia += na_c;
        ie += nx_c;
        {
            // the unconsumed staged operations move down to lane 0 (every lane runs every shuffle)
            const int sa = lane + na_c < 64 ? lane + na_c : 63, sx_ = lane + nx_c < 64 ? lane + nx_c : 63;
            a_op = shfl64(a_op, sa);
            a_x = shfl64(a_x, sa);
            a_ts = shfl64(a_ts, sa);
            a_clk = shfl64(a_clk, sa);
            a_ch = shfl64(a_ch, sa);
            a_rep = shfl64(a_rep, sa);
            x_op = shfl64(x_op, sx_);
            x_x = shfl64(x_x, sx_);
            x_ts = shfl64(x_ts, sx_);
            x_clk = shfl64(x_clk, sx_);
            x_ch = shfl64(x_ch, sx_);
            x_rep = shfl64(x_rep, sx_);
            a_keep = 64 - na_c;
            x_keep = 64 - nx_c;
        }
        // ---- rows: lanes segmented by their chunk among the qualifying operations
        const i64 ch = in ? (i64)(is_add ? sa_ch : sx_ch) : 0;
        const bool qual = in && (is_add ? cur_on : exp_on);
        const u64 qm = __ballot(qual);
        const u64 qb = qm & (le >> 1);  // qualifying lanes before this one
        const int pl = qb ? 63 - __clzll(qb) : lane;
        const i64 pch = (i64)shfl64((u64)ch, pl);
        const i64 prev_ch = qb ? pch : row_ch;
        const bool start = qual && ch != prev_ch;
        if (start) flags[op] = 1;
        const u64 stm = __ballot(start) & le;
        const int sl = stm ? 63 - __clzll(stm) : lane;
        const u64 sop = shfl64(op, sl);
        const i64 my_row = stm ? (i64)sop : row_op;
        const u64 qa = qm & ~le;  // qualifying lanes after this one
        const int nl = qa ? __ffsll((long long)qa) - 1 : lane;
        const i64 nch = (i64)shfl64((u64)ch, nl);
        const bool end = qual && (!qa || nch != ch);
        if (end) {
            const i64 ts = (i64)(is_add ? sa_ts : sx_ts), rep = (i64)(is_add ? sa_rep : sx_rep),
                      clk = (i64)(is_add ? sa_clk : sx_clk);
            u64 w[6 + SH_MAX_AGGS];
            u64 nulls = 0;
            w[0] = (u64)ts;
            w[1] = (u64)rep;
            w[2] = (u64)ch;
            w[3] = (u64)clk;
#pragma unroll
            for (int o = 0; o < SH_MAX_AGGS; o++) {
                w[5 + o] = 0;
                if (o >= ko.n) continue;
                const int src = ko.src[o];
                u64 v = 0;
                bool nul = false;
                if (src == 0) v = (u64)r_cnt;
                else if (src == 1) { nul = r_cnt == 0; v = r_sum; }
                else if (src == 2) {
                    nul = r_cnt == 0;
                    if (!nul) v = (u64)__double_as_longlong(__longlong_as_double((i64)r_sum) / (double)r_cnt);
                } else if (src == 3) { nul = (r_fl & 1u) == 0; v = r_mn; }
                else { nul = (r_fl & 2u) == 0; v = r_mx; }
                w[5 + o] = nul ? 0 : v;
                nulls |= (u64)(nul ? 1 : 0) << o;
            }
            w[4] = (u64)k | ((u64)(is_add ? 0 : 1) << 32) | (nulls << 40);
#ifdef SH_XW_NOROWS
#pragma unroll
            for (int o = 0; o < 5 + SH_MAX_AGGS; o++) xw_chk += w[o] ^ (u64)my_row;  // (timing experiment only)
#else
            ulonglong2* dst = (ulonglong2*)(rows.aos + (size_t)my_row * rows.rw);
#pragma unroll
            for (int o = 0; o < (6 + SH_MAX_AGGS) / 2; o++)
                if (2 * o < rows.rw) dst[o] = make_ulonglong2(w[2 * o], w[2 * o + 1]);
#endif
        }
        if (qm) {  // (wave-uniform)
            const int lq = 63 - __clzll(qm);
            row_ch = (i64)shfl64((u64)ch, lq);
            row_op = (i64)shfl64((u64)my_row, lq);
        }
        __syncthreads();  // the staging arrays are refilled by the next chunk
    }
    // ---- the window after the push: FIFO [ie, HN) — ring entries keep their place, new ones follow
    const int keep = ie < H0 ? H0 - ie : 0;
    const int rh = (rh0 + (ie < H0 ? ie : H0)) & gm;
    const int j0 = ie > H0 ? ie : H0;
    for (int j = j0 + lane; j < HN; j += 64) {
        const size_t sl = kr + (size_t)((rh + keep + (j - j0)) & gm);
        const u32 r = sorted_rank[lo + (u32)(j - H0)];
        const u64* q = xa + (size_t)r * kXaWords;
        S.rpm[sl] = (i64)q[5];
        S.rval[sl] = q[1];
        rg[sl] = G0 + (i64)r;
    }
#ifdef SH_XW_NOROWS
    if (xw_chk == 0x5A5A5A5A5A5A5A5Aull) flags[0] = 2;
#endif
    if (lane == 0) {
        S.cnt[k] = cnt;
        S.rhead[k] = rh;
        S.rlen[k] = keep + (HN - j0);
        if (HSUM) {
            const u64 sb = (u64)__double_as_longlong(sum);
            if (fd.sum >= 0) S.f[(size_t)fd.sum * S.nslots + k] = sb;
            if (fd.avg >= 0) S.f[(size_t)fd.avg * S.nslots + k] = sb;
        }
        if (HMIN) kdq_store<1>(qn, S, fd.mn, k, dq_min);
        if (HMAX) kdq_store<1>(qx, S, fd.mx, k, dq_max);
    }
}

// emission from the row records: flagged operation indices in order, each row read as one record
__global__ __launch_bounds__(kBlock) void k_slx_emit_aos(const unsigned char* __restrict__ flags, i64 n,
                                                        const i64* __restrict__ blk_pre, const u64* __restrict__ rows,
                                                        int rw, int n_aggs, KeyTable kt, KeyPlan kp, i64 out_cap,
                                                        i64* out_ts, i64* out_keys, u64* out_vals,
                                                        unsigned char* out_nulls, unsigned char* out_exp, i64* out_ch,
                                                        i64* out_clock, i64* out_rep) {
    const i64 tile = (i64)blockIdx.x * kTile;
    i64 run = blk_pre[blockIdx.x];
    for (int it = 0; it < kItems; it++) {
        const i64 j = tile + (i64)it * kBlock + threadIdx.x;
        const i64 fl = j < n ? flags[j] : 0;
        i64 tot;
        const i64 r = run + block_excl_scan(fl, SumOp(), 0, &tot);
        run += tot;
        if (!fl) continue;
        const ulonglong2* src = (const ulonglong2*)(rows + (size_t)j * rw);
        const ulonglong2 a0 = src[0], a1 = src[1], a2 = src[2];
        out_ts[r] = (i64)a0.x;
        out_rep[r] = (i64)a0.y;
        out_ch[r] = (i64)a1.x;
        out_clock[r] = (i64)a1.y;
        const u64 meta = a2.x;
        unpack_key(kp, slot_key(kt, (u32)meta), out_keys + r, out_cap);
        out_exp[r] = (unsigned char)((meta >> 32) & 1);
        for (int a = 0; a < n_aggs; a++) {
            out_vals[(size_t)a * out_cap + r] = a == 0 ? a2.y : rows[(size_t)j * rw + 5 + a];
            out_nulls[(size_t)a * out_cap + r] = (unsigned char)((meta >> (40 + a)) & 1);
        }
    }
}

void launch_slx_emit_aos(hipStream_t s, const unsigned char* flags, i64 n, const i64* blk_pre, int nblk, SlxRows rows,
                         int n_aggs, KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals,
                         unsigned char* out_nulls, unsigned char* out_exp, i64* out_ch, i64* out_clock, i64* out_rep) {
    if (nblk <= 0) return;
    hipLaunchKernelGGL(k_slx_emit_aos, dim3(nblk), dim3(kBlock), 0, s, flags, n, blk_pre, rows.aos, rows.rw, n_aggs, kt,
                       kp, out_cap, out_ts, out_keys, out_vals, out_nulls, out_exp, out_ch, out_clock, out_rep);
}

bool slx_keyed_ok(AggPlan ap) {
    DFields fd;
    return own_d_fields(ap, fd) && ap.n <= SH_MAX_AGGS;
}

void launch_slx_wkey(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, const u64* xa,
                     const u64* xx, i64 n_u, i64 X0, i64 G0, i64 seq_base, i64 send_size, SlState S, i64* rg,
                     AggPlan ap, int cur_on, int exp_on, SlxRows rows, unsigned char* flags) {
    if (nslots <= 0) return;
    DFields fd;
    own_d_fields(ap, fd);
    KOut ko{};
    ko.n = ap.n;
    for (int q = 0; q < ap.n; q++) {
        const int kind = ap.kind[q];
        ko.src[q] = kind == AK_COUNT ? 0 : kind == AK_SUM_D ? 1 : kind == AK_AVG ? 2 : kind == AK_MIN_D ? 3 : 4;
    }
    const bool hs = fd.sum >= 0 || fd.avg >= 0, hn = fd.mn >= 0, hx = fd.mx >= 0;
#define SH_SLX_K(A, B, C)                                                                                          \
    hipLaunchKernelGGL((k_slx_wkey<A, B, C>), dim3((unsigned)nslots), dim3(64), 0, s, key_off, (u32)nslots,       \
                       sorted_rank, xa, xx, n_u, X0, G0, seq_base, send_size, S, rg, fd, ko, cur_on, exp_on, rows,   \
                       flags)
    if (hs && hn && hx) SH_SLX_K(true, true, true);
    else if (hs && !hn && !hx) SH_SLX_K(true, false, false);
    else if (!hs && hn && hx) SH_SLX_K(false, true, true);
    else if (hs && hn) SH_SLX_K(true, true, false);
    else if (hs && hx) SH_SLX_K(true, false, true);
    else if (hn && !hx) SH_SLX_K(false, true, false);
    else if (hx && !hn) SH_SLX_K(false, false, true);
    else SH_SLX_K(false, false, false);
#undef SH_SLX_K
}

void launch_sliding_own(hipStream_t s, const u32* rank_list, const i64* part_off, int P, int logP, SlRecords rec,
                        SlState S, AggPlan ap, i64 T, i64 send_size, i64 send_base, SlRows rows,
                        unsigned char* flags, SlRecords rec_by_rank) {
    {
        DFields fd;
        const bool ok = own_d_fields(ap, fd);
        if (ok) {
            const bool hs = fd.sum >= 0 || fd.avg >= 0, hn = fd.mn >= 0, hx = fd.mx >= 0;
#define SH_SL_D(A, B, C)                                                                                      \
    hipLaunchKernelGGL((k_sl_own_d<A, B, C, true>), dim3(P), dim3(64), 0, s, rank_list, part_off, logP, rec_by_rank, S, \
                       ap, fd,                                                                                \
                       T, send_size, send_base, rows, flags)
            if (hs && hn && hx) SH_SL_D(true, true, true);
            else if (hs && !hn && !hx) SH_SL_D(true, false, false);
            else if (!hs && hn && hx) SH_SL_D(false, true, true);
            else if (hs && hn) SH_SL_D(true, true, false);
            else if (hs && hx) SH_SL_D(true, false, true);
            else if (hn && !hx) SH_SL_D(false, true, false);
            else if (hx && !hn) SH_SL_D(false, false, true);
            else SH_SL_D(false, false, false);
#undef SH_SL_D
            return;
        }
    }
    int n_mm = 0;
    for (int a = 0; a < ap.n; a++) n_mm += ap.kind[a] >= AK_MIN_L;
    const size_t lds = (size_t)std::max(1, n_mm) * 64 * kDqL * 8;
#define SH_SL_OWN(A, V)                                                                                        \
    hipLaunchKernelGGL((k_sl_own<A, V>), dim3(P), dim3(64), lds, s, rank_list, part_off, logP, rec, S, ap, T, \
                       send_size, send_base, rows, flags)
    const int nv = std::max(1, ap.n_vcols);
    if (ap.n <= 2 && nv <= 1) SH_SL_OWN(2, 1);
    else if (ap.n <= 4 && nv <= 1) SH_SL_OWN(4, 1);
    else if (ap.n <= 4 && nv <= 2) SH_SL_OWN(4, 2);
    else if (nv <= 2) SH_SL_OWN(8, 2);
    else SH_SL_OWN(8, 8);
#undef SH_SL_OWN
}

// ------------------------------------------------------------------------------------------------
// emit: flagged ranks -> output rows in rank order; flush starts where the send changes.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kBlock) void k_sl_emit(const unsigned char* __restrict__ flags, i64 n,
                                                   const i64* __restrict__ blk_pre, SlRows rows, int n_aggs,
                                                   KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys,
                                                   u64* out_vals, unsigned char* out_nulls, i64* out_send,
                                                   i64* out_clock, const u32* __restrict__ rank_raw, i64 raw_base,
                                                   i64* out_order, const i64* __restrict__ clock_by_rank,
                                                   i64* out_rep) {
    // striped over the tile (round it: elements tile + it * kBlock + lane), so every row read and
    // every output column store of a wave is one contiguous run; the tile's first output row is
    // blk_pre (k_count_flags counts whole tiles, whatever the order inside)
    const i64 tile = (i64)blockIdx.x * kTile;
    i64 run = blk_pre[blockIdx.x];
    for (int it = 0; it < kItems; it++) {
        const i64 j = tile + (i64)it * kBlock + threadIdx.x;
        const i64 fl = j < n ? flags[j] : 0;
        i64 tot;
        const i64 r = run + block_excl_scan(fl, SumOp(), 0, &tot);
        run += tot;
        if (!fl) continue;
        out_ts[r] = rows.ts[j];
        unpack_key(kp, slot_key(kt, rows.slot[j]), out_keys + r, out_cap);
        for (int a = 0; a < n_aggs; a++) {
            out_vals[(size_t)a * out_cap + r] = rows.vals[(size_t)a * rows.cap + j];
            out_nulls[(size_t)a * out_cap + r] = rows.nulls[(size_t)a * rows.cap + j];
        }
        out_send[r] = rows.send[j];
        out_clock[r] = clock_by_rank ? clock_by_rank[j] : rows.clock[j];
        if (out_order) out_order[r] = raw_base + (i64)rank_raw[j];
        out_rep[r] = raw_base + (i64)rows.rep[j];
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
                    unsigned char* out_nulls, i64* out_send, i64* out_clock, const u32* rank_raw, i64 raw_base,
                    i64* out_order, const i64* clock_by_rank, i64* out_rep) {
    hipLaunchKernelGGL(k_sl_emit, dim3(nblk), dim3(kBlock), 0, s, flags, n, blk_pre, rows, n_aggs, kt, kp, out_cap,
                       out_ts, out_keys, out_vals, out_nulls, out_send, out_clock, rank_raw, raw_base, out_order,
                       clock_by_rank, out_rep);
}

void launch_flush_starts(hipStream_t s, const i64* out_send, i64 n_rows, i64* blk_cnt, int nb) {
    hipLaunchKernelGGL(k_flush_starts, dim3(nb), dim3(kBlock), 0, s, out_send, n_rows, blk_cnt);
}

__global__ __launch_bounds__(kBlock) void k_iota_i64(i64* a, i64 n) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) a[i] = i;
}

void launch_iota_i64(hipStream_t s, i64* a, i64 n) {
    if (n > 0) hipLaunchKernelGGL(k_iota_i64, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a, n);
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


// ---- key-table rebuild of a sliding window (sh_sliding.cpp sliding_rekey): a key whose window holds
// no event that can still be in it for any later event (last ring entry's PM + T <= the clock every
// later record carries at least) is in the state the reference destroys (canDestroy): it is dropped;
// the live keys move to a fresh table and their state follows them to the new slots --------------------
__global__ __launch_bounds__(kBlock) void k_sl_rekey_map(i64 size, KeyTable old_kt, KeyTable new_kt,
                                                        const i64* __restrict__ rhead, const i64* __restrict__ rlen,
                                                        const i64* __restrict__ rpm, i64 rc, i64 T, i64 bound,
                                                        u32* map) {
    const i64 s = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (s > size) return;
    if (s == size) { map[s] = (u32)size; return; }  // the spare slot keeps its place
    map[s] = 0xFFFFFFFFu;
    const u64 key = old_kt.keys[s];
    if (key == kEmptyKey) return;
    const i64 n = rlen[s];
    if (n <= 0) return;
    const i64 last_pm = rpm[(size_t)s * rc + ((rhead[s] + n - 1) & (rc - 1))];
    if (last_pm + T <= bound) return;
    map[s] = key_slot(new_kt, key);
}

// dst[o][map[s]][.] = src[o][s][.] for live slots (unit-sized words; rings keep their head offsets)
__global__ __launch_bounds__(kBlock) void k_sl_rekey_copy(const unsigned char* __restrict__ src, unsigned char* dst,
                                                         i64 outer, i64 n, i64 inner, int unit,
                                                         const u32* __restrict__ map) {
    const i64 per = inner / unit;
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= outer * n * per) return;
    const i64 w = i % per, sl = (i / per) % n, o = i / (per * n);
    const u32 to = map[sl];
    if (to == 0xFFFFFFFFu) return;
    const size_t from_off = ((size_t)o * n + sl) * inner + (size_t)w * unit;
    const size_t to_off = ((size_t)o * n + to) * inner + (size_t)w * unit;
    if (unit == 8) *(u64*)(dst + to_off) = *(const u64*)(src + from_off);
    else dst[to_off] = src[from_off];
}

void launch_sl_rekey_map(hipStream_t s, i64 size, KeyTable old_kt, KeyTable new_kt, const i64* rhead, const i64* rlen,
                         const i64* rpm, i64 rc, i64 T, i64 bound, u32* map) {
    hipLaunchKernelGGL(k_sl_rekey_map, dim3((unsigned)((size + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, size,
                       old_kt, new_kt, rhead, rlen, rpm, rc, T, bound, map);
}

void launch_sl_rekey_copy(hipStream_t s, const void* src, void* dst, i64 outer, i64 n, i64 inner, const u32* map) {
    const int unit = inner % 8 == 0 ? 8 : 1;
    const i64 total = outer * n * (inner / unit);
    if (total <= 0) return;
    hipLaunchKernelGGL(k_sl_rekey_copy, dim3((unsigned)((total + kBlock - 1) / kBlock)), dim3(kBlock), 0, s,
                       (const unsigned char*)src, (unsigned char*)dst, outer, n, inner, unit, map);
}
}  // namespace shd
