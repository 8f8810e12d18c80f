// sh_kernels.hip — gfx950 kernels of the batch-window path (lengthBatch / timeBatch group-by).
//
// Pipeline of one push (DESIGN.md "Batch-window pipeline"):
//   k_blockagg      per-workgroup pass count + send clock maxima        (FilterProcessor, InputHandler clock)
//   k_scan_blocks   exclusive scans of those, nextEmitTime initialisation (TimeBatchWindowProcessor.process :266-276)
//   k_boundaries    window number per event, boundary list              (LengthBatch :206-243, TimeBatch :278-340, Scheduler)
//   k_ms_count/scatter  stable multisplit of closed-window events into key partitions (P > 1 only)
//   k_aggregate_*   ordered per-key aggregation of one (window, partition) (QuerySelector.processInBatchGroupBy :315-374)
//   k_bits_* + k_emit_rows   rows in first-occurrence order: rank of the first event's bit (LinkedHashMap order)
//   k_compact_pending        events of the still-open window carried to the next push
#include "sh_device.h"

namespace shd {

// Diagnostic phase stamps (make stamps -> libsiddhi_hip_stamps.so, read by scripts/stamps.py): thread 0
// of a workgroup records the shader clock at numbered points of a kernel. The product build has none.
#ifdef SH_STAMPS
constexpr int kStampKernels = 4, kStampBlocks = 32768, kStampPts = 16;
__device__ unsigned long long g_stamps[kStampKernels * kStampBlocks * kStampPts];
#define SH_STAMP(kern, pt)                                                                                   \
    do {                                                                                                     \
        if (threadIdx.x == 0 && blockIdx.x < kStampBlocks) {                                                 \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");                                      \
            g_stamps[((size_t)(kern) * kStampBlocks + blockIdx.x) * kStampPts + (pt)] = __builtin_amdgcn_s_memtime(); \
        }                                                                                                    \
    } while (0)
#else
#define SH_STAMP(kern, pt) do {} while (0)
#endif

// ================================================================================================
// k_blockagg: per workgroup (kTile events, blocked kItems per thread) the number of passing events,
// the max timestamp over send-last events and the first passing event.
// ================================================================================================
template <int FK>
__global__ __launch_bounds__(kBlock) void k_blockagg(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                    WinParams wp, i64* blk_pass, i64* blk_tl, i64* blk_first,
                                                    i64* blk_xm) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 cnt = 0, tl = INT64_MIN, first = INT64_MAX, xm = INT64_MIN;
    i64 tsv[kItems];
    load_items_i64(ts, base, wp.N, tsv, INT64_MIN);
    bool pass[kItems];
    filter_items<FK>(f, cols, base, wp.N, pass);
    SendCursor sc(wp, base);
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        if (e < wp.N) {
            if (pass[i]) {
                cnt++;
                if (first == INT64_MAX) first = e;
                if (blk_xm) xm = max(xm, load_raw(cols, wp.ts_col, e));
            }
            if (sc.last(wp, e)) tl = max(tl, tsv[i]);
        }
        sc.next();
    }
    i64 c = block_reduce(cnt, SumOp(), 0);
    i64 t = block_reduce(tl, MaxOp(), INT64_MIN);
    i64 fp = block_reduce(first, MinOp(), INT64_MAX);
    i64 x = blk_xm ? block_reduce(xm, MaxOp(), INT64_MIN) : INT64_MIN;
    if (threadIdx.x == 0) {
        blk_pass[blockIdx.x] = c; blk_tl[blockIdx.x] = t; blk_first[blockIdx.x] = fp;
        if (blk_xm) blk_xm[blockIdx.x] = x;
    }
}

void launch_blockagg(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, i64 N, i64 send_size,
                     i64* blk_pass, i64* blk_tl, i64* blk_first, int nblk, i64* blk_xm, int ts_col) {
    WinParams wp{};
    wp.N = N;
    wp.send_size = send_size;
    wp.ts_col = ts_col;
    i64* xm = ts_col >= 0 ? blk_xm : nullptr;
    switch (filter_kind(f)) {
        case 0: hipLaunchKernelGGL(k_blockagg<0>, dim3(nblk), dim3(kBlock), 0, s, ts, cols, f, wp, blk_pass, blk_tl, blk_first, xm); break;
        case 1: hipLaunchKernelGGL(k_blockagg<1>, dim3(nblk), dim3(kBlock), 0, s, ts, cols, f, wp, blk_pass, blk_tl, blk_first, xm); break;
        default: hipLaunchKernelGGL(k_blockagg<2>, dim3(nblk), dim3(kBlock), 0, s, ts, cols, f, wp, blk_pass, blk_tl, blk_first, xm);
    }
}

// ================================================================================================
// k_scan_blocks (one workgroup of 1024): exclusive prefix sum of pass counts, exclusive prefix max
// of send clocks, first passing event; initialises timeBatch's nextEmitTime on the first process()
// call: nextEmitTime = now + T, or getNextEmitTime(now) when start.time is given
// (TimeBatchWindowProcessor.java:266-276, 342-347).
// ================================================================================================
// 1024-thread exclusive scans of the tile partials, in coalesced passes of 1024 elements
// (thread t takes element c*1024 + t) carrying the running totals between passes.
struct Scan3 {
    i64 s, m, mn, x;  // sum, max, min, second max
};
template <bool XM = true>
__device__ __forceinline__ Scan3 block1024_excl(Scan3 v, Scan3* tot) {
    __shared__ i64 w_sum[16], w_max[16], w_min[16], w_x[16];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const i64 si = wave_incl_scan(v.s, SumOp());
    const i64 mi = wave_incl_scan(v.m, MaxOp());
    const i64 ni = wave_incl_scan(v.mn, MinOp());
    const i64 xi = XM ? wave_incl_scan(v.x, MaxOp()) : INT64_MIN;
    if (lane == 63) { w_sum[wv] = si; w_max[wv] = mi; w_min[wv] = ni; w_x[wv] = xi; }
    __syncthreads();
    Scan3 pre{0, INT64_MIN, INT64_MAX, INT64_MIN}, all{0, INT64_MIN, INT64_MAX, INT64_MIN};
    // not unrolled: all 64 LDS reads in flight at once would need 128 registers per thread
#pragma unroll 2
    for (int x = 0; x < 16; x++) {
        if (x < wv) { pre.s += w_sum[x]; pre.m = max(pre.m, w_max[x]); pre.x = max(pre.x, w_x[x]); }
        all.s += w_sum[x]; all.m = max(all.m, w_max[x]); all.mn = min(all.mn, w_min[x]); all.x = max(all.x, w_x[x]);
    }
    __syncthreads();
    i64 mex = __shfl_up(mi, 1, 64);
    i64 xex = XM ? __shfl_up(xi, 1, 64) : INT64_MIN;
    if (lane == 0) { mex = INT64_MIN; xex = INT64_MIN; }
    *tot = all;
    return Scan3{pre.s + si - v.s, max(pre.m, mex), 0, max(pre.x, xex)};
}

// Two launches of one workgroup per chunk of 1024 tiles (thread t takes tile c*1024 + t: coalesced).
// k_scan_chunks reduces each chunk to its totals {sum, max, min, second max}, stored after the
// tiles' first-event column (blk_first + nblk, see scan_blocks_first_bytes); k_scan_blocks scans
// each chunk offset by the totals of the chunks before it (uniform loads). A single workgroup looping
// over the chunks was latency-bound: its stores sat in the same in-order counter as the next
// chunk's loads.
template <bool XM>
__global__ __launch_bounds__(1024) void k_scan_chunks(const i64* blk_pass, const i64* blk_tl, i64* blk_first,
                                                     int nblk, const i64* blk_xm) {
    const int i = blockIdx.x * 1024 + threadIdx.x;
    const bool in = i < nblk;
    Scan3 v{in ? blk_pass[i] : 0, in ? blk_tl[i] : INT64_MIN, in ? blk_first[i] : INT64_MAX,
            (XM && in) ? blk_xm[i] : INT64_MIN};
    Scan3 all;
    block1024_excl<XM>(v, &all);
    if (threadIdx.x == 0) {
        i64* ct = blk_first + nblk + 4 * (i64)blockIdx.x;
        ct[0] = all.s; ct[1] = all.m; ct[2] = all.mn; ct[3] = all.x;
    }
}

template <bool XM>
__global__ __launch_bounds__(1024) void k_scan_blocks(i64* blk_pass, i64* blk_tl, const i64* blk_first, int nblk,
                                                     const i64* __restrict__ ts, WinParams wp, PushInfo* info,
                                                     i64* blk_xm, ColSet cols) {
    const int t = threadIdx.x, c = blockIdx.x, nch = (nblk + 1023) / 1024;
    const int i = c * 1024 + t;
    const bool in = i < nblk;
    Scan3 v{in ? blk_pass[i] : 0, in ? blk_tl[i] : INT64_MIN, INT64_MAX, (XM && in) ? blk_xm[i] : INT64_MIN};
    const i64* ct = blk_first + nblk;
    Scan3 pre{0, INT64_MIN, INT64_MAX, INT64_MIN}, all{0, INT64_MIN, INT64_MAX, INT64_MIN};
    for (int k = 0; k < nch; k++) {
        const i64 a0 = ct[4 * k], a1 = ct[4 * k + 1], a2 = ct[4 * k + 2], a3 = ct[4 * k + 3];
        if (k < c) { pre.s += a0; pre.m = max(pre.m, a1); pre.x = max(pre.x, a3); }
        all.s += a0; all.m = max(all.m, a1); all.mn = min(all.mn, a2); all.x = max(all.x, a3);
    }
    Scan3 call;
    const Scan3 ex = block1024_excl<XM>(v, &call);
    const i64 my_pm = max(pre.m, ex.m);  // exclusive prefix max of tile i
    if (in) {
        blk_pass[i] = pre.s + ex.s;
        blk_tl[i] = my_pm;
        if (XM) blk_xm[i] = max(pre.x, ex.x);
    }
    const i64 tot_s = all.s, tot_m = all.m, tot_mn = all.mn, tot_x = all.x;
    // the push info is written by one thread: the one holding the tile of the send that carries the
    // first passing event when that send's clock is needed, else thread 0 of chunk 0
    const bool init_e0 = wp.kind == SH_WIN_TIME_BATCH && !wp.e0_valid && !wp.wcol;
    const bool need_clk = tot_mn != INT64_MAX && (init_e0 || wp.want_first_clk);
    const i64 sl = wp.send_size > 0 ? wp.send_size : wp.N;
    const i64 start = need_clk ? (tot_mn / sl) * sl : 0;
    const int b0 = (int)(start / kTile);
    if (need_clk ? i == b0 : i == 0) {
        info->total_pass = tot_s;
        info->max_tl = tot_m;
        info->first_pass = tot_mn;
        info->e0_valid = wp.e0_valid;
        info->E0 = wp.E0;
        info->n_bounds = 0;
        info->first_clk = INT64_MIN;
        info->max_xm = tot_x;
        info->err = 0;
        info->first_key = (wp.pcol1 > 0 && tot_mn != INT64_MAX) ? load_raw(cols, wp.pcol1 - 1, tot_mn) : 0;
        // externalTimeBatch initTiming (:313-334): the start is the constant, the start attribute or
        // the timestamp attribute of the first event reaching the window
        if (wp.kind == SH_WIN_EXT_TIME_BATCH && !wp.e0_valid && tot_mn != INT64_MAX) {
            const i64 a = load_raw(cols, wp.ts_col, tot_mn);
            const i64 st = wp.has_start == 1 ? wp.start_time : wp.has_start == 2 ? load_raw(cols, wp.start_col, tot_mn) : a;
            info->E0 = st;
            info->e0_valid = 1;
            if (a < st || st < 0) info->err = 1;
        }
        if (need_clk) {
            // clock of the send that carries the first passing event (before the carried-in clock)
            const i64 last = min(wp.N - 1, start + sl - 1);
            i64 pm = my_pm;  // the exclusive prefix max of tile b0
            for (i64 e = (i64)b0 * kTile; e < start; e++)
                if (is_send_last(wp, e)) pm = max(pm, ts[e]);
            i64 cl = max(pm, ts[last]);
            info->first_clk = cl;
            if (init_e0) {
                if (wp.clock_valid) cl = max(cl, wp.clock0);
                i64 E0;
                if (wp.cal) {
                    E0 = cal_start_d(cal_idx_d(cl, wp.cal, wp.cal_tz) + 1, wp.cal, wp.cal_tz);
                } else if (wp.has_start) {
                    i64 elapsed = (cl - wp.start_time) % wp.T;  // Java % truncates like C++
                    E0 = cl + (wp.T - elapsed);
                } else {
                    E0 = cl + wp.T;
                }
                info->E0 = E0;
                info->e0_valid = 1;
            }
        }
    }
}

size_t scan_blocks_first_bytes(int nblk) { return ((size_t)nblk + 4 * (size_t)((nblk + 1023) / 1024)) * 8; }

void launch_scan_blocks(hipStream_t s, i64* blk_pass, i64* blk_tl, i64* blk_first, int nblk, const i64* ts,
                        WinParams wp, PushInfo* info, i64* blk_xm, ColSet cols) {
    const int nch = (nblk + 1023) / 1024;
    if (wp.kind == SH_WIN_EXT_TIME_BATCH) {
        hipLaunchKernelGGL(k_scan_chunks<true>, dim3(nch), dim3(1024), 0, s, blk_pass, blk_tl, blk_first, nblk, blk_xm);
        hipLaunchKernelGGL(k_scan_blocks<true>, dim3(nch), dim3(1024), 0, s, blk_pass, blk_tl, blk_first, nblk, ts, wp,
                           info, blk_xm, cols);
    } else {
        hipLaunchKernelGGL(k_scan_chunks<false>, dim3(nch), dim3(1024), 0, s, blk_pass, blk_tl, blk_first, nblk,
                           nullptr);
        hipLaunchKernelGGL(k_scan_blocks<false>, dim3(nch), dim3(1024), 0, s, blk_pass, blk_tl, blk_first, nblk, ts, wp,
                           info, nullptr, cols);
    }
}

// ================================================================================================
// k_boundaries: window number W(e) of every new event, and a boundary record wherever W rises.
//   lengthBatch: W = (n_pend + passing events before e) / L  (LengthBatchWindowProcessor :206-243:
//                a batch completes at its L-th event and is flushed as its own chunk);
//   timeBatch:   W = clock(e) < E0 ? 0 : (clock(e) - E0) / T + 1, clock(e) = the playback clock of
//                e's send. Due timers fire before the send is processed and catch up one period
//                each (Scheduler.sendTimerEvents :171-209), so the window boundaries sit at E0 + kT.
// ================================================================================================
// Single-pass form (SORTED, timeBatch once nextEmitTime is known): when the send-last timestamps do
// not decrease, the clock of an event's send is max(carried-in clock, the send's own last timestamp)
// — no prefix over earlier tiles is needed, so k_blockagg + k_scan_blocks are skipped. Every tile
// checks that ts never decreases across its events and into the next tile's first event; a tile
// that finds a decrease sets PushInfo.unsorted and the host redoes the window assignment with the
// prefix passes. The tile's passing-event count goes to blk_pass[tile] and each boundary records
// its tile and in-tile count; k_fix_bounds adds the scanned tile prefixes afterwards.
template <bool EXT, int FK, bool SORTED>
__global__ __launch_bounds__(kBlock) void k_boundaries(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                      WinParams wp, i64* blk_pass_pre, const i64* blk_tl_pre,
                                                      PushInfo* info, Bound* bounds, int max_bounds,
                                                      int* n_bounds, KeyPlan kp, KeyTable kt, u32* new_pos,
                                                      const i64* blk_xm_pre, u32* ms_counts, int P, int ms_nblk,
                                                      int ms_col0) {
    const int tile = blockIdx.x;
    i64 base = (i64)tile * kTile + (i64)threadIdx.x * kItems;
    // the timestamps are loaded first, so their latency overlaps the filter, key and histogram work
    i64 t[kItems];
    load_items_i64(ts, base, wp.N, t, INT64_MIN);
    bool pass[kItems];
    filter_items<FK>(f, cols, base, wp.N, pass);
    // group-key slot of every passing event, looked up once for the whole pipeline
    // (GroupByKeyGenerator.constructEventKey, QuerySelector.java:331-336)
    {
        u64 key[kItems];
        u32 pos[kItems];
        if (kp.n == 1 && kp.div[0] == 0 && kp.type[0] != SH_T_FLOAT && kp.type[0] != SH_T_DOUBLE) {
            i64 raw[kItems];
            load_items_raw(cols, kp.col[0], base, wp.N, raw);
#pragma unroll
            for (int i = 0; i < kItems; i++) key[i] = pass[i] ? (u64)raw[i] : 0;
        } else {
#pragma unroll
            for (int i = 0; i < kItems; i++) key[i] = pass[i] ? make_key(kp, cols, base + i) : 0;
        }
        key_slots<kItems>(kt, key, pass, pos);
#pragma unroll
        for (int i = 0; i < kItems; i++) pos[i] = pass[i] ? pos[i] : kNoPos;
        const i64 tile0 = (i64)tile * kTile;
        if (!new_pos) {
            // dictionary keys are their own slots (PosSrc reads the key column): no slot column
        } else if (tile0 + kTile <= wp.N && (((size_t)(new_pos + tile0)) & 15) == 0) {
            // transposed through LDS so every store instruction covers whole lines (a thread's own
            // 32-byte run would leave each 16-byte store half a line, written back twice)
            __shared__ uint4 tp[kTile / 4];
            tp[threadIdx.x * 2] = make_uint4(pos[0], pos[1], pos[2], pos[3]);
            tp[threadIdx.x * 2 + 1] = make_uint4(pos[4], pos[5], pos[6], pos[7]);
            __syncthreads();
            uint4* q = (uint4*)(new_pos + tile0);
            q[threadIdx.x] = tp[threadIdx.x];
            q[threadIdx.x + kBlock] = tp[threadIdx.x + kBlock];
        } else {
#pragma unroll
            for (int i = 0; i < kItems; i++)
                if (base + i < wp.N) new_pos[base + i] = pos[i];
        }
        // the multisplit's per-tile key-partition counts of this tile (k_ms_count's job for the
        // push's events when the split runs over the whole push)
        if (ms_counts) {
            extern __shared__ __attribute__((aligned(16))) u32 mhist[];
            for (int i = threadIdx.x; i < P; i += kBlock) mhist[i] = 0;
            __syncthreads();
#pragma unroll
            for (int i = 0; i < kItems; i++)
                if (pass[i]) atomicAdd(&mhist[pos[i] & (P - 1)], 1u);
            __syncthreads();
            // the tile's row of the [tile][partition] count matrix: one contiguous store per tile
            for (int i = threadIdx.x; i < P; i += kBlock)
                ms_counts[(i64)(ms_col0 + tile) * P + i] = mhist[i];
        }
    }
    i64 cnt = 0, tl = INT64_MIN;
    SendCursor sc(wp, base);
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        bool in = e < wp.N;
        cnt += pass[i];
        if (!SORTED && in && sc.last(wp, e)) tl = max(tl, t[i]);
        sc.next();
    }
    i64 pcb, pm = INT64_MIN;
    if (SORTED) {
        i64 tot_c;
        pcb = block_excl_scan(cnt, SumOp(), 0, &tot_c);  // in-tile: the tile prefix is added later
        if (threadIdx.x == 0) blk_pass_pre[tile] = tot_c;
        bool down = false;
#pragma unroll
        for (int i = 0; i + 1 < kItems; i++) down |= base + i + 1 < wp.N && t[i + 1] < t[i];
        if (base + kItems < wp.N) down |= ts[base + kItems] < t[kItems - 1];
        if (down) atomicOr(&info->unsorted, 1);
    } else {
        pcb = block_excl_scan(cnt, SumOp(), 0, nullptr) + blk_pass_pre[tile];
        pm = max(block_excl_scan(tl, MaxOp(), INT64_MIN, nullptr), blk_tl_pre[tile]);
    }
    // externalTimeBatch: running max of the timestamp attribute over the events reaching the window
    constexpr bool ext = EXT;  // externalTimeBatch (the running max M below)
    i64 av[kItems];
    i64 M = INT64_MIN;
    if (ext) {
        load_items_raw(cols, wp.ts_col, base, wp.N, av);
        i64 xm = INT64_MIN;
#pragma unroll
        for (int i = 0; i < kItems; i++) if (pass[i]) xm = max(xm, av[i]);
        M = max(wp.xm0, max(block_excl_scan(xm, MaxOp(), INT64_MIN, nullptr), blk_xm_pre[tile]));
    }
    const i64 c0 = wp.clock_valid ? wp.clock0 : INT64_MIN;
    const i64 E0 = SORTED ? wp.E0 : info->E0;
    const int e0v = SORTED ? wp.e0_valid : info->e0_valid;
    if (base >= wp.N) return;
    const bool per_event = send_len(wp) == 1;
    SendCursor sc2(wp, base);
    // previous event's window
    i64 Wprev, clock_prev;
    if (base == 0) {
        Wprev = wp.W_open;
        clock_prev = c0;
    } else {
        i64 ep = base - 1;
        bool pp = eval_filter<FK>(f, cols, ep);
        i64 pcb_prev = pcb - (pp ? 1 : 0);
        // ep and base in one send: ep's clock is that send's clock; else it closed the previous send
        if (SORTED) clock_prev = max(c0, ts[sc2.r != 0 ? sc2.last_of(wp, base) : ep]);
        else if (sc2.r != 0) clock_prev = max(c0, max(pm, ts[sc2.last_of(wp, base)]));
        else clock_prev = max(c0, pm);
        Wprev = wp.wcol ? wp.W_base + wp.wcol[ep] : wfun(wp, E0, e0v, pcb_prev, ext ? M : clock_prev);
    }
    WinCursor wc;
    wc.W = Wprev;
    wc.lim = INT64_MIN;  // first event recomputes
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        if (e >= wp.N) break;
        i64 tsl = per_event ? t[i] : ts[sc2.last_of(wp, e)];
        i64 clk = max(c0, max(pm, tsl));
        if (ext && pass[i]) M = max(M, av[i]);
        i64 W = wp.wcol ? wp.W_base + wp.wcol[e] : wc.at(wp, E0, e0v, pcb, ext ? M : clk);
        if (W > Wprev) {
            int k = atomicAdd(n_bounds, 1);
            if (k < max_bounds) {
                Bound b;
                b.idx = wp.n_pend + e; b.W = W; b.clock = clk; b.clock_prev = clock_prev; b.pcb = pcb;
                // (SORTED: pcb is in-tile until k_fix_bounds; externalTimeBatch: the attribute max M at
                // the closing event, the expired rows' timestamp)
                b.pad = SORTED ? tile : ext ? M : 0;
                bounds[k] = b;
            }
        }
        Wprev = W;
        clock_prev = clk;
        pcb += pass[i];
        if (!SORTED && sc2.last(wp, e)) pm = max(pm, t[i]);
        sc2.next();
    }
}

// two small regions zeroed by one launch (the push's info block and the tile-count tail)
__global__ void k_zero2(unsigned char* a, int na, unsigned char* b, int nb) {
    for (int i = threadIdx.x; i < na; i += blockDim.x) a[i] = 0;
    for (int i = threadIdx.x; i < nb; i += blockDim.x) b[i] = 0;
}

void launch_zero2(hipStream_t s, void* a, int na, void* b, int nb) {
    hipLaunchKernelGGL(k_zero2, dim3(1), dim3(256), 0, s, (unsigned char*)a, na, (unsigned char*)b, nb);
}

// SORTED form, after the scan of the tile counts (blk_pass[nblk] = total): the boundaries' pass
// counts become push-relative and the push totals go to PushInfo (the clock max of a sorted push is
// its last event's timestamp: the last event always ends a send).
__global__ __launch_bounds__(kBlock) void k_fix_bounds(Bound* bounds, int max_bounds, const i64* blk_pass_pre,
                                                      int nblk, const i64* __restrict__ ts, WinParams wp,
                                                      PushInfo* info) {
    const int n = min(info->n_bounds, max_bounds);
    for (int k = threadIdx.x; k < n; k += kBlock) bounds[k].pcb += blk_pass_pre[bounds[k].pad];
    if (threadIdx.x == 0) {
        info->total_pass = blk_pass_pre[nblk];
        info->max_tl = ts[wp.N - 1];
        info->first_pass = blk_pass_pre[nblk] ? 0 : INT64_MAX;
        info->E0 = wp.E0;
        info->e0_valid = wp.e0_valid;
        info->first_clk = INT64_MIN;
        info->max_xm = INT64_MIN;
    }
}

void launch_fix_bounds(hipStream_t s, Bound* bounds, int max_bounds, const i64* blk_pass_pre, int nblk, const i64* ts,
                       WinParams wp, PushInfo* info) {
    hipLaunchKernelGGL(k_fix_bounds, dim3(1), dim3(kBlock), 0, s, bounds, max_bounds, blk_pass_pre, nblk, ts, wp, info);
}

void launch_boundaries(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp,
                       i64* blk_pass_pre, const i64* blk_tl_pre, PushInfo* info, Bound* bounds,
                       int max_bounds, int nblk, KeyPlan kp, KeyTable kt, u32* new_pos, const i64* blk_xm_pre,
                       u32* ms_counts, int P, int ms_nblk, int ms_col0, bool sorted, i64* scan_tmp) {
    const size_t lds = ms_counts ? (size_t)P * 4 : 0;
    int* nb = &info->n_bounds;
#define SH_BOUNDS(EXT, FK, S)                                                                                     \
    hipLaunchKernelGGL((k_boundaries<EXT, FK, S>), dim3(nblk), dim3(kBlock), lds, s, ts, cols, f, wp, blk_pass_pre, \
                       blk_tl_pre, info, bounds, max_bounds, nb, kp, kt, new_pos, blk_xm_pre, ms_counts, P, ms_nblk,   \
                       ms_col0)
    const int fk = filter_kind(f);
    if (wp.kind == SH_WIN_EXT_TIME_BATCH) SH_BOUNDS(true, 2, false);
    else if (sorted) {
        if (fk == 0) SH_BOUNDS(false, 0, true);
        else if (fk == 1) SH_BOUNDS(false, 1, true);
        else SH_BOUNDS(false, 2, true);
    } else if (fk == 0) SH_BOUNDS(false, 0, false);
    else if (fk == 1) SH_BOUNDS(false, 1, false);
    else SH_BOUNDS(false, 2, false);
#undef SH_BOUNDS
    if (sorted) {
        // blk_pass[nblk] was zeroed with the info block: the scan leaves the total there
        launch_scan_sum_large(s, blk_pass_pre, nblk + 1, scan_tmp);
        hipLaunchKernelGGL(k_fix_bounds, dim3(1), dim3(kBlock), 0, s, bounds, max_bounds, blk_pass_pre, nblk, ts, wp,
                           info);
    }
}

// ================================================================================================
// Aggregation of the closed windows. One row per (window, key) with the aggregate values at the
// key's last event, folded in event order per key (QuerySelector.processInBatchGroupBy :315-374), so
// double sums are bit-identical to Java's sequential `sum += v`. State starts empty because each
// flush chunk begins with RESET (LengthBatch :222-226, TimeBatch :320-323;
// AttributeAggregatorExecutor.processReset :145-151).
//
// Rows are written as records of row_words(n_aggs) u64 words:
//   w0 = key slot | event count << 32, w1 = first | last << 32 (combined event index), w2.. = values
// and the row's first event is marked in a bitmap over the combined index space. The output position
// of a row is the rank of that bit (k_emit_rows): first-occurrence order inside a flush, and flushes
// in window order, because windows are consecutive index ranges.
// ================================================================================================
struct AggLds {
    u64* fields;  // [n_fields][NL]
    u32* cnt;
    u32* first;
    u32* last;
    u32* owner;
};

// value column j of an event held in registers (unrolled select: no dynamic register indexing)
template <int V>
__device__ __forceinline__ i64 pick(const i64 (&v)[V], int j) {
    i64 x = v[0];
#pragma unroll
    for (int i = 1; i < V; i++) if (j == i) x = v[i];
    return x;
}

// A key's aggregate fields held in registers while one of its events is folded, field j in register
// slot j: the per-event updates driven by the per-field op table (sums: sum += x / value += (double) x;
// min/max: replace when the state is new or x is smaller / larger in the column's type —
// MinAttributeAggregatorExecutor `minValue > value`).
// SIG != 0 is a compile-time op table (agg_sig): 4 bits per field, op + 1, so the folds of the common
// plans carry no per-field dispatch.
__host__ __device__ constexpr int sig_op(u32 sig, int j) { return (int)((sig >> (4 * j)) & 15u) - 1; }
__host__ __device__ constexpr int sig_fields(u32 sig) { return sig == 0 ? 0 : 1 + sig_fields(sig >> 4); }
constexpr u32 agg_sig3(int a, int b, int c) {
    return (u32)(a + 1) | ((u32)(b + 1) << 4) | ((u32)(c + 1) << 8);
}
// the plan's op table as a signature (0 when it has no field or more than 4)
inline u32 agg_sig(const AggPlan& ap) {
    if (ap.n_fields < 1 || ap.n_fields > 4) return 0;
    u32 s = 0;
    for (int j = 0; j < ap.n_fields; j++) s |= (u32)(ap.fop[j] + 1) << (4 * j);
    return s;
}

template <int V, int F = SH_MAX_AGGS, u32 SIG = 0>
__device__ __forceinline__ void fold_fields(const AggPlan& ap, u64 (&f)[F], bool first, const i64 (&v)[V]) {
#pragma unroll
    for (int j = 0; j < F; j++) {
        if (j >= (SIG ? sig_fields(SIG) : ap.n_fields)) break;
        const int op = SIG ? sig_op(SIG, j) : ap.fop[j];
        const i64 x = pick<V>(v, ap.fvcol[j]);
        const u64 cur = f[j];
        u64 r;
        if (op <= FOP_ADD_DI) {
            if (op == FOP_ADD_I) {
                r = (u64)((first ? 0 : (i64)cur) + x);
            } else {
                double xd = op == FOP_ADD_DI ? (double)x : __longlong_as_double(x);
                r = (u64)__double_as_longlong((first ? 0.0 : __longlong_as_double((i64)cur)) + xd);
            }
        } else {
            bool lt, gt;  // x < cur, x > cur in the column's type (false on NaN, as in Java)
            if (op <= FOP_MAX_I) {
                lt = x < (i64)cur; gt = x > (i64)cur;
            } else if (op <= FOP_MAX_D) {
                double a = __longlong_as_double(x), b = __longlong_as_double((i64)cur);
                lt = a < b; gt = a > b;
            } else {
                float a = (float)__longlong_as_double(x), b = (float)__longlong_as_double((i64)cur);
                lt = a < b; gt = a > b;
            }
            const bool is_min = op == FOP_MIN_I || op == FOP_MIN_D || op == FOP_MIN_F;
            r = (first || (is_min ? lt : gt)) ? (u64)x : cur;
        }
        f[j] = r;
    }
}

// The output values of a row: count, avg = value / count, the other fields as folded.
__device__ __forceinline__ u64 agg_out(const AggPlan& ap, int a, u32 c, u64 fv) {
    const int k = ap.kind[a];
    if (k == AK_COUNT) return (u64)(i64)c;
    if (k == AK_AVG) return (u64)__double_as_longlong(__longlong_as_double((i64)fv) / (double)(i64)c);
    return fv;
}

// one row record (see above) with 16-byte stores
template <int F = SH_MAX_AGGS>
__device__ __forceinline__ void write_row(const AggPlan& ap, u64* row, int RW, u32 pos, u32 c, u32 first, u32 last,
                                          const u64 (&f)[F], const EvSrc& es, bool have_last = false,
                                          i64 last_ts = 0, i64 last_seq = 0) {
    u64 w[4 + SH_MAX_AGGS];
    w[0] = (u64)pos | ((u64)c << 32);
    w[1] = (u64)first | ((u64)last << 32);
    // the last event's timestamp and stream index (prefetched by the caller when it could)
    w[2] = (u64)(have_last ? last_ts : ev_ts(es, last));
    w[3] = (u64)(have_last ? last_seq : ev_seq(es, last));
#pragma unroll
    for (int a = 0; a < SH_MAX_AGGS; a++) {
        u64 fv = f[0];
#pragma unroll
        for (int j = 1; j < F; j++) if (ap.field[a] == j) fv = f[j];
        w[4 + a] = a < ap.n ? agg_out(ap, a, c, fv) : 0;
    }
#pragma unroll
    for (int i = 0; i < (4 + SH_MAX_AGGS) / 2; i++) {
        if (2 * i >= RW) break;
        ((ulonglong2*)row)[i] = make_ulonglong2(w[2 * i], w[2 * i + 1]);
    }
}

__device__ __forceinline__ void mark_first(u32* first_bits, u32 first) {
    atomicOr(&first_bits[first >> 5], 1u << (first & 31));
}

__device__ __forceinline__ void lds_layout(unsigned char* smem_raw, const AggPlan& ap, int NL, AggLds& L) {
    // realign by pointer arithmetic on the LDS base (an int->pointer cast would lose the address space)
    unsigned char* smem = smem_raw + ((16u - ((unsigned)(size_t)smem_raw & 15u)) & 15u);
    L.fields = (u64*)smem;
    L.cnt = (u32*)(smem + (size_t)ap.n_fields * NL * 8);
    L.first = L.cnt + NL;
    L.last = L.first + NL;
    L.owner = L.last + NL;
}

template <int V>
__device__ __forceinline__ void apply_event(const AggPlan& ap, AggLds& L, int NL, u32 li, u32 idx, const i64 (&v)[V]) {
    const u32 c = L.cnt[li];
    u64 f[SH_MAX_AGGS];
#pragma unroll
    for (int j = 0; j < SH_MAX_AGGS; j++) f[j] = (j < ap.n_fields && c) ? L.fields[(size_t)j * NL + li] : 0;
    fold_fields<V>(ap, f, c == 0, v);
#pragma unroll
    for (int j = 0; j < SH_MAX_AGGS; j++) if (j < ap.n_fields) L.fields[(size_t)j * NL + li] = f[j];
    if (c == 0) L.first[li] = idx;
    L.last[li] = idx;
    L.cnt[li] = c + 1;
}

// Unpartitioned (P == 1, few keys, short windows): one workgroup per closed segment reads the events
// directly; the keys' state is in LDS and lanes that share a key resolve in ordered rounds (lowest
// lane first).
__global__ __launch_bounds__(kBlock) void k_aggregate_flat(const Segment* __restrict__ segs, int NL, i64 n_pend,
                                                          const u32* __restrict__ pend_pos,
                                                          const u64* __restrict__ pend_vals, i64 pend_cap,
                                                          const u32* __restrict__ new_pos, ColSet cols, AggPlan ap,
                                                          u64* rows, int RW, u32* unit_rows, u32* first_bits,
                                                          EvSrc es) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    AggLds L;
    lds_layout(smem_raw, ap, NL, L);
    const int seg = blockIdx.x;
    for (int i = threadIdx.x; i < NL; i += kBlock) { L.cnt[i] = 0; L.owner[i] = 0; }
    __syncthreads();
    i64 lo = segs[seg].lo, hi = segs[seg].hi;
    u32 round = 0;
    for (i64 b = lo; b < hi; b += kBlock) {
        i64 e = b + threadIdx.x;
        bool pend = false;
        u32 li = 0, idx = (u32)e;
        i64 v[SH_MAX_AGGS];
        if (e < hi) {
            if (e < n_pend) {
                li = pend_pos[e];
#pragma unroll
                for (int j = 0; j < SH_MAX_AGGS; j++)
                    if (j < ap.n_vcols) v[j] = (i64)pend_vals[(size_t)j * pend_cap + e];
                pend = true;
            } else {
                i64 x = e - n_pend;
                u32 pos = new_pos[x];
                if (pos != kNoPos) {
                    li = pos;
#pragma unroll
                    for (int j = 0; j < SH_MAX_AGGS; j++)
                        if (j < ap.n_vcols) v[j] = load_raw(cols, ap.vcol_src[j], x);
                    pend = true;
                }
            }
        }
        // ordered conflict rounds: owner = max(round<<9 | (511 - lane)) picks the lowest lane per key
        while (__syncthreads_or(pend)) {
            round++;
            u32 tag = (round << 9) | (511u - threadIdx.x);
            if (pend) atomicMax(&L.owner[li], tag);
            __syncthreads();
            if (pend && L.owner[li] == tag) {
                apply_event(ap, L, NL, li, idx, v);
                pend = false;
            }
        }
    }
    __syncthreads();
    int mine = 0;
    for (int i = threadIdx.x; i < NL; i += blockDim.x) mine += L.cnt[i] > 0;
    i64 tot;
    i64 pre = block_excl_scan_any((i64)mine, &tot);
    // the segment's rows fill its own region of NL row slots
    if (threadIdx.x == 0) unit_rows[seg] = (u32)tot;
    u32 r = (u32)seg * (u32)NL + (u32)pre;
    for (int i = threadIdx.x; i < NL; i += blockDim.x) {
        const u32 c = L.cnt[i];
        if (!c) continue;
        u64 f[SH_MAX_AGGS];
#pragma unroll
        for (int j = 0; j < SH_MAX_AGGS; j++) f[j] = j < ap.n_fields ? L.fields[(size_t)j * NL + i] : 0;
        write_row(ap, rows + (size_t)r * RW, RW, (u32)i, c, L.first[i], L.last[i], f, es);
        mark_first(first_bits, L.first[i]);
        r++;
    }
}

// Partitioned, thread ownership with register-resident state: thread t of the workgroup owns the
// local key t (local key = slot >> logP of key partition p = slot & (P - 1); with K == 2 also
// t + 512, which only the hash table's sentinel slot can be) and keeps its count, first/last event and
// aggregate fields in registers for the whole (window, partition). The partition's records (event
// order) are taken in chunks of CH = 512 * R; wave w loads the contiguous run [w * 64R, (w + 1) * 64R)
// of the chunk (coalesced), ranks each record among its run's records of the same owner (ballots over
// the 9 owner bits, a wave-private running count per owner), and after one workgroup scan per chunk
// every record has its slot in its owner's list, in event order. The owner then folds its list.
constexpr int kOwnT = 512;
template <int V, int K, int R, int F, u32 SIG, bool PACK>
__global__ __launch_bounds__(kOwnT, 4) void k_aggregate_own(const i64* __restrict__ seg_off, int P, int logP,
                                                           AggPlan ap, u64* rows, int RW, u32* unit_rows,
                                                           u32* first_bits, const Segment* __restrict__ segs,
                                                           const u32* __restrict__ rec_pos,
                                                           const u32* __restrict__ rec_idx,
                                                           const u64* __restrict__ rec_vals, i64 rec_cap, EvSrc es,
                                                           int dense) {
    constexpr int W = kOwnT / 64;
    constexpr int PW = 64 * R;   // records per wave and chunk
    constexpr int CH = kOwnT * R;
    __shared__ u32 st_idx[CH];
    __shared__ u64 st_v[V][CH];
    __shared__ unsigned char st_hi[K > 1 ? CH : 1];
    __shared__ u32 wcnt[W][kOwnT];  // per wave: running count per owner, then its offset
    __shared__ u32 bstart[kOwnT];
    __shared__ u32 lstart[CH / 32];  // bitmap: chunk positions where an owner's list starts
    constexpr u32 kNone = 0xFFFFFFFFu;
    const int seg = blockIdx.x / P;
    const int p = blockIdx.x - seg * P;
    const int t = threadIdx.x, lane = t & 63, w = t >> 6;
    const i64 lo = seg_off[(i64)seg * P + p], hi = seg_off[(i64)(seg + 1) * P + p];
    // packed records: the low kPackIdxBits of the event index, which lies in [seg_lo, seg_lo + 2^bits)
    const u32 seg_lo = PACK ? (u32)segs[seg].lo : 0u;
    SH_STAMP(0, 0);
    u32 cnt0 = 0, fst0 = 0, lst0 = 0, cnt1 = 0, fst1 = 0, lst1 = 0;
    i64 pf_ts = 0, pf_seq = 0;
    bool pf = false;
    u64 f0[F], f1[F];
#pragma unroll
    for (int j = 0; j < F; j++) { f0[j] = 0; f1[j] = 0; }
    for (i64 c0 = lo; c0 < hi; c0 += CH) {
        const int n = (int)min((i64)CH, hi - c0);
        // (a) the wave's run of the chunk, coalesced, into registers
        u32 li[R], ix[R];
        i64 v[R][V];
#pragma unroll
        for (int j = 0; j < R; j++) {
            const int r = w * PW + j * 64 + lane;
            const bool ok = r < n;
            if (PACK) {
                const u32 wd = ok ? rec_idx[c0 + r] : 0u;
                li[j] = ok ? (wd >> kPackIdxBits) : kNone;
                ix[j] = seg_lo + (((wd & kPackIdxMask) - seg_lo) & kPackIdxMask);
            } else {
                li[j] = ok ? (rec_pos[c0 + r] >> logP) : kNone;
                ix[j] = ok ? rec_idx[c0 + r] : 0;
            }
#pragma unroll
            for (int x = 0; x < V; x++) v[j][x] = (ok && x < ap.n_vcols) ? (i64)rec_vals[(size_t)x * rec_cap + c0 + r] : 0;
        }
        SH_STAMP(0, 1);
        // (b) rank among the run's records of the same owner: a wave-private running count per owner,
        // advanced by LDS atomics (the wave's rounds complete in program order; lanes of one round
        // that share an owner get distinct ranks, in an order (e) restores)
#pragma unroll
        for (int i = lane; i < kOwnT; i += 64) wcnt[w][i] = 0;
        for (int i = t; i < CH / 32; i += kOwnT) lstart[i] = 0;
#pragma unroll
        for (int j = 0; j < R; j++) {
            if (li[j] == kNone) continue;
            const u32 rk = atomicAdd(&wcnt[w][li[j] & (kOwnT - 1)], 1u);
            // local key (< 1024) and its rank (< CH <= 4096) share the register from here on
            li[j] |= rk << 10;
        }
        __syncthreads();
        SH_STAMP(0, 2);
        // (c) owner t: offsets of the waves' runs in its list, then its list's start in the chunk
        u32 tot = 0;
#pragma unroll
        for (int x = 0; x < W; x++) {
            const u32 c = wcnt[x][t];
            wcnt[x][t] = tot;
            tot += c;
        }
        i64 all;
        const u32 start = (u32)block_excl_scan_any((i64)tot, &all);
        bstart[t] = start;
        if (tot) atomicOr(&lstart[start >> 5], 1u << (start & 31));
        __syncthreads();
        // (d) every record into its owner's list
#pragma unroll
        for (int j = 0; j < R; j++) {
            if (li[j] == kNone) continue;
            const u32 b = li[j] & (kOwnT - 1);
            const u32 d = bstart[b] + wcnt[w][b] + (li[j] >> 10);
            st_idx[d] = ix[j];
#pragma unroll
            for (int x = 0; x < V; x++) st_v[x][d] = (u64)v[j][x];
            if (K > 1) st_hi[d] = (unsigned char)((li[j] >> 9) & 1);
        }
        __syncthreads();
        SH_STAMP(0, 3);
        // (e) the owner's list is in event order unless lanes of one round that shared the owner got
        // their ranks out of lane order (never seen on gfx950: scripts/probe/lds_atomic_order.hip);
        // checked in parallel over adjacent positions of one list, repaired by an insertion pass
        bool bad = false;
        for (int d = t; d + 1 < n; d += kOwnT)
            bad |= !((lstart[(d + 1) >> 5] >> ((d + 1) & 31)) & 1u) && st_idx[d + 1] < st_idx[d];
        if (__syncthreads_or(bad) && tot > 1) {
            u32 prev = st_idx[start];
            for (u32 k = 1; k < tot; k++) {
                const u32 e = st_idx[start + k];
                if (e > prev) { prev = e; continue; }
                u64 mv[V];
#pragma unroll
                for (int x = 0; x < V; x++) mv[x] = st_v[x][start + k];
                const unsigned char mh = K > 1 ? st_hi[start + k] : 0;
                u32 m = k;
                while (m > 0 && st_idx[start + m - 1] > e) {
                    st_idx[start + m] = st_idx[start + m - 1];
#pragma unroll
                    for (int x = 0; x < V; x++) st_v[x][start + m] = st_v[x][start + m - 1];
                    if (K > 1) st_hi[start + m] = st_hi[start + m - 1];
                    m--;
                }
                st_idx[start + m] = e;
#pragma unroll
                for (int x = 0; x < V; x++) st_v[x][start + m] = mv[x];
                if (K > 1) st_hi[start + m] = mh;
            }
        }
        SH_STAMP(0, 4);
        // the unit's last chunk: the owner's last event is its list's last entry (one key per owner
        // when K == 1), so the random reads of that event's timestamp and stream index for the row
        // are issued now and complete while the list is folded
        if (K == 1 && c0 + CH >= hi && tot) {
            const u32 el = st_idx[start + tot - 1];
            pf_ts = ev_ts(es, el);
            pf_seq = ev_seq(es, el);
            pf = true;
        }
        // then folds it; the next record's LDS loads are issued before the current one is folded, so
        // their latency overlaps the fold
        u32 e_nx = 0;
        i64 v_nx[V];
        unsigned char hi_nx = 0;
#pragma unroll
        for (int x = 0; x < V; x++) v_nx[x] = 0;
        if (tot) {
            e_nx = st_idx[start];
#pragma unroll
            for (int x = 0; x < V; x++) if (x < ap.n_vcols) v_nx[x] = (i64)st_v[x][start];
            if (K > 1) hi_nx = st_hi[start];
        }
        for (u32 k = 0; k < tot; k++) {
            const u32 e = e_nx;
            i64 vv[V];
#pragma unroll
            for (int x = 0; x < V; x++) vv[x] = v_nx[x];
            const unsigned char hi_cur = hi_nx;
            if (k + 1 < tot) {
                const u32 i = start + k + 1;
                e_nx = st_idx[i];
#pragma unroll
                for (int x = 0; x < V; x++) if (x < ap.n_vcols) v_nx[x] = (i64)st_v[x][i];
                if (K > 1) hi_nx = st_hi[i];
            }
            if (K > 1 && hi_cur) {
                fold_fields<V, F, SIG>(ap, f1, cnt1 == 0, vv);
                if (cnt1 == 0) fst1 = e;
                lst1 = e;
                cnt1++;
            } else {
                fold_fields<V, F, SIG>(ap, f0, cnt0 == 0, vv);
                if (cnt0 == 0) fst0 = e;
                lst0 = e;
                cnt0++;
            }
        }
    }
    SH_STAMP(0, 5);
    // one row per key with events, in the unit's own region of K * 512 row slots (no global counter:
    // a contended atomic on one address would serialise every workgroup of the launch)
    const int mine = (cnt0 > 0) + (K > 1 && cnt1 > 0);
    i64 tot;
    const i64 pre = block_excl_scan_any((i64)mine, &tot);
    if (t == 0) unit_rows[blockIdx.x] = (u32)tot;
    if (dense) {
        // rows at their local key's slot of the unit (K * kOwnT rows, holes where a key had no event):
        // the emission finds a row from its first event's key slot, no rank scatter (k_emit_gather)
        const u64 base = (u64)blockIdx.x * (u64)(K * kOwnT);
        if (K == 1 && (size_t)kOwnT * RW * 8 <= sizeof(st_v)) {
            u64* stg = &st_v[0][0];
            __shared__ unsigned char has[kOwnT];
            __syncthreads();
            has[t] = cnt0 > 0;
            if (cnt0) {
                write_row<F>(ap, stg + (size_t)t * RW, RW, ((u32)t << logP) | (u32)p, cnt0, fst0, lst0, f0, es, pf, pf_ts,
                             pf_seq);
                mark_first(first_bits, fst0);
            }
            __syncthreads();
            const int h = RW / 2, n2 = kOwnT * h;
            ulonglong2* dst = (ulonglong2*)(rows + base * RW);
            const ulonglong2* src = (const ulonglong2*)stg;
            for (int i = t; i < n2; i += kOwnT)
                if (has[i / h]) dst[i] = src[i];
            SH_STAMP(0, 6);
            return;
        }
        if (cnt0) {
            write_row<F>(ap, rows + (base + (u64)t) * RW, RW, ((u32)t << logP) | (u32)p, cnt0, fst0, lst0, f0, es, pf,
                         pf_ts, pf_seq);
            mark_first(first_bits, fst0);
        }
        if (K > 1 && cnt1) {
            write_row<F>(ap, rows + (base + (u64)(t + kOwnT)) * RW, RW, ((u32)(t + kOwnT) << logP) | (u32)p, cnt1, fst1,
                         lst1, f1, es);
            mark_first(first_bits, fst1);
        }
        SH_STAMP(0, 6);
        return;
    }
    u32 r = (u32)blockIdx.x * (u32)(K * kOwnT) + (u32)pre;
    if (K == 1 && (size_t)kOwnT * RW * 8 <= sizeof(st_v)) {
        // the unit's rows are one contiguous run: staged in LDS (the record staging is free now),
        // then stored with whole-line writes instead of each thread's strided 16-byte pieces
        u64* stg = &st_v[0][0];
        __syncthreads();
        if (cnt0)
            write_row<F>(ap, stg + (size_t)pre * RW, RW, ((u32)t << logP) | (u32)p, cnt0, fst0, lst0, f0, es, pf, pf_ts,
                         pf_seq);
        if (cnt0) mark_first(first_bits, fst0);
        __syncthreads();
        const int n2 = (int)tot * RW / 2;
        ulonglong2* dst = (ulonglong2*)(rows + (size_t)blockIdx.x * (K * kOwnT) * RW);
        const ulonglong2* src = (const ulonglong2*)stg;
        for (int i = t; i < n2; i += kOwnT) dst[i] = src[i];
        SH_STAMP(0, 6);
        return;
    }
    if (cnt0) {
        write_row<F>(ap, rows + (size_t)r * RW, RW, ((u32)t << logP) | (u32)p, cnt0, fst0, lst0, f0, es, pf, pf_ts,
                     pf_seq);
        mark_first(first_bits, fst0);
        r++;
    }
    if (K > 1 && cnt1) {
        write_row<F>(ap, rows + (size_t)r * RW, RW, ((u32)(t + kOwnT) << logP) | (u32)p, cnt1, fst1, lst1, f1, es);
        mark_first(first_bits, fst1);
    }
    SH_STAMP(0, 6);
}

int own_keys_per_thread(int NL) { return NL <= kOwnT ? 1 : 2; }

int agg_unit_rows(int P, int NL, bool own) { return own ? own_keys_per_thread(NL) * kOwnT : NL; }

void launch_aggregate(hipStream_t s, const Segment* segs, int nseg, int P, int logP, int NL, i64 n_pend,
                      const u32* pend_pos, const u64* pend_vals, i64 pend_cap, const u32* new_pos, ColSet cols,
                      AggPlan ap, u64* rows, int RW, u32* unit_rows, u32* first_bits,
                      const u32* rec_pos, const u32* rec_idx, const u64* rec_vals, i64 rec_cap, const i64* seg_off,
                      bool pack, EvSrc es, bool dense_rows) {
    const int dense = dense_rows ? 1 : 0;
    if (rec_idx) {  // multisplit records: thread-ownership kernel
        const int K = own_keys_per_thread(NL);
        const int F = ap.n_fields <= 2 ? 2 : ap.n_fields <= 4 ? 4 : 8;
#define SH_AGG_OWN(VV, KK, RR, FF, SG)                                                                          \
    do {                                                                                                        \
        if (pack)                                                                                               \
            hipLaunchKernelGGL((k_aggregate_own<VV, KK, RR, FF, SG, true>), dim3(nseg * P), dim3(kOwnT), 0, s,   \
                               seg_off, P, logP, ap, rows, RW, unit_rows, first_bits, segs, rec_pos, rec_idx,    \
                               rec_vals, rec_cap, es, dense);                                                   \
        else                                                                                                    \
            hipLaunchKernelGGL((k_aggregate_own<VV, KK, RR, FF, SG, false>), dim3(nseg * P), dim3(kOwnT), 0, s,  \
                               seg_off, P, logP, ap, rows, RW, unit_rows, first_bits, segs, rec_pos, rec_idx,    \
                               rec_vals, rec_cap, es, dense);                                                   \
    } while (0)
#define SH_AGG_OWN_F(VV, KK, RR)                          \
    do {                                                  \
        if (F == 2) SH_AGG_OWN(VV, KK, RR, 2, 0);         \
        else if (F == 4) SH_AGG_OWN(VV, KK, RR, 4, 0);    \
        else SH_AGG_OWN(VV, KK, RR, 8, 0);                \
    } while (0)
        // compile-time op tables of the common plans (one value column: sum / avg, min + max + avg;
        // two: long sum + double avg); anything else runs the table-driven fold
        constexpr u32 kMinMaxAvgD = agg_sig3(FOP_MIN_D, FOP_MAX_D, FOP_ADD_D), kSumD = agg_sig3(FOP_ADD_D, -1, -1),
                      kSumI = agg_sig3(FOP_ADD_I, -1, -1), kSumISumD = agg_sig3(FOP_ADD_I, FOP_ADD_D, -1),
                      kSumMinMaxD = agg_sig3(FOP_ADD_D, FOP_MIN_D, FOP_MAX_D);  // aggregation base values
        const u32 sig = agg_sig(ap);
        // (R = 4 — half-size chunks, 3 workgroups per CU — measured 349 vs 287 us per C2 push)
        // (values left in global memory and read back by their owner — 32 KB of LDS, four workgroups
        // per CU — measured 334 vs 310 us)
        if (K == 1 && ap.n_vcols <= 1 && sig == kMinMaxAvgD) SH_AGG_OWN(1, 1, 8, 4, kMinMaxAvgD);
        else if (K == 1 && ap.n_vcols <= 1 && sig == kSumD) SH_AGG_OWN(1, 1, 8, 2, kSumD);
        else if (K == 1 && ap.n_vcols <= 1 && sig == kSumI) SH_AGG_OWN(1, 1, 8, 2, kSumI);
        else if (K == 1 && ap.n_vcols == 2 && sig == kSumISumD) SH_AGG_OWN(2, 1, 4, 2, kSumISumD);
        else if (K == 2 && ap.n_vcols <= 1 && sig == kMinMaxAvgD) SH_AGG_OWN(1, 2, 8, 4, kMinMaxAvgD);
        else if (K == 2 && ap.n_vcols <= 1 && sig == kSumD) SH_AGG_OWN(1, 2, 8, 2, kSumD);
        else if (K == 1 && ap.n_vcols <= 1 && sig == kSumMinMaxD) SH_AGG_OWN(1, 1, 8, 4, kSumMinMaxD);
        else if (K == 2 && ap.n_vcols <= 1 && sig == kSumMinMaxD) SH_AGG_OWN(1, 2, 8, 4, kSumMinMaxD);
        else if (K == 1) {
            if (ap.n_vcols <= 1) SH_AGG_OWN_F(1, 1, 8);
            else if (ap.n_vcols <= 2) SH_AGG_OWN_F(2, 1, 4);
            else if (ap.n_vcols <= 4) SH_AGG_OWN_F(4, 1, 2);
            else SH_AGG_OWN_F(8, 1, 1);
        } else {
            if (ap.n_vcols <= 1) SH_AGG_OWN_F(1, 2, 8);
            else if (ap.n_vcols <= 2) SH_AGG_OWN_F(2, 2, 4);
            else if (ap.n_vcols <= 4) SH_AGG_OWN_F(4, 2, 2);
            else SH_AGG_OWN_F(8, 2, 1);
        }
#undef SH_AGG_OWN_F
#undef SH_AGG_OWN
    } else {
        size_t lds = (size_t)NL * (8 * ap.n_fields + 16) + 16;
        hipLaunchKernelGGL(k_aggregate_flat, dim3(nseg), dim3(kBlock), lds, s, segs, NL, n_pend, pend_pos, pend_vals,
                           pend_cap, new_pos, cols, ap, rows, RW, unit_rows, first_bits, es);
    }
}

// ================================================================================================
// Flag counts and single-workgroup scans (also used by the sliding path's row ordering).
// ================================================================================================
__global__ __launch_bounds__(kBlock) void k_count_flags(const unsigned char* __restrict__ flags, i64 n, i64* blk_cnt) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 c = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) if (base + i < n) c += flags[base + i];
    i64 t = block_reduce(c, SumOp(), 0);
    if (threadIdx.x == 0) blk_cnt[blockIdx.x] = t;
}

void launch_count_flags(hipStream_t s, const unsigned char* flags, i64 n, i64* blk_cnt, int nblk) {
    hipLaunchKernelGGL(k_count_flags, dim3(nblk), dim3(kBlock), 0, s, flags, n, blk_cnt);
}

__global__ __launch_bounds__(1024) void k_scan_sum(i64* a, int n) {
    if (n <= 0) return;
    constexpr int G = 8;
    i64 run = 0;
    for (int g0 = 0; g0 < n; g0 += G * 1024) {
        i64 va[G];
#pragma unroll
        for (int g = 0; g < G; g++) va[g] = a[min(g0 + g * 1024 + (int)threadIdx.x, n - 1)];
#pragma unroll
        for (int g = 0; g < G; g++) {
            if (g0 + g * 1024 >= n) break;
            const int i = g0 + g * 1024 + threadIdx.x;
            const bool in = i < n;
            Scan3 v{in ? va[g] : 0, INT64_MIN, INT64_MAX};
            Scan3 all;
            Scan3 ex = block1024_excl(v, &all);
            if (in) a[i] = run + ex.s;
            run += all.s;
        }
    }
}

void launch_scan_sum(hipStream_t s, i64* a, int n) {
    hipLaunchKernelGGL(k_scan_sum, dim3(1), dim3(1024), 0, s, a, n);
}

// Exclusive prefix of the popcounts of the first-occurrence bitmap, per 32-bit word.
__global__ __launch_bounds__(kBlock) void k_bits_tile(const u32* __restrict__ bits, i64 nw, i64* tile_sum) {
    const i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 c = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) if (base + i < nw) c += __popc(bits[base + i]);
    const i64 t = block_reduce(c, SumOp(), 0);
    if (threadIdx.x == 0) tile_sum[blockIdx.x] = t;
}

__global__ __launch_bounds__(kBlock) void k_bits_pre(const u32* __restrict__ bits, i64 nw, const i64* tile_pre,
                                                    u64* word_pre, u32* total) {
    const i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    u32 b[kItems];
    i64 c = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) { b[i] = base + i < nw ? bits[base + i] : 0; c += __popc(b[i]); }
    i64 r = block_excl_scan(c, SumOp(), 0, nullptr) + tile_pre[blockIdx.x];
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        if (base + i < nw) word_pre[base + i] = ((u64)b[i] << 32) | (u32)r;  // the word beside its prefix
        r += __popc(b[i]);
        if (base + i == nw - 1) *total = (u32)r;  // every row's first event has one bit: the row count
    }
}

void launch_bits_prefix(hipStream_t s, const u32* bits, i64 nw, i64* tile_sum, u64* word_pre, u32* total) {
    const int nb = (int)((nw + kTile - 1) / kTile);
    hipLaunchKernelGGL(k_bits_tile, dim3(nb), dim3(kBlock), 0, s, bits, nw, tile_sum);
    launch_scan_sum(s, tile_sum, nb);
    hipLaunchKernelGGL(k_bits_pre, dim3(nb), dim3(kBlock), 0, s, bits, nw, tile_sum, word_pre, total);
}

// Output rows are staged as records of stage_words(nk, na, order) u64 words at their output
// position — ts, keys, representative event, [first event], values — so the rank scatter writes
// whole 64-byte records and the column split (k_emit_soa) reads and writes contiguous runs.
__host__ __device__ constexpr int stage_words(int nk, int na, int order) { return (2 + nk + order + na + 1) & ~1; }

// Stage 1, one row record per thread: its output position is the rank of its first event's bit; the
// row's timestamp and representative event are those of the key's last event, the key comes from the
// slot. The records of a wave are then stored cooperatively through LDS: consecutive lanes write
// consecutive 16-byte pieces of one record, so each store instruction covers whole 64-byte records
// instead of one piece of 64 scattered ones.
constexpr int kStageMax = 2 + kKeyParts + 1 + SH_MAX_AGGS + 1;
__global__ __launch_bounds__(kBlock) void k_emit_rank(const u64* __restrict__ rows, int RW,
                                                     const u32* __restrict__ unit_rows, i64 n_units,
                                                     int unit_stride,
                                                     const u64* __restrict__ word_pre,
                                                     int n_aggs, KeyTable kt, KeyPlan kp, i64 n_pend,
                                                     const i64* __restrict__ pend_ts, const i64* __restrict__ ts,
                                                     const u64* __restrict__ pend_gidx,
                                                     const u64* __restrict__ new_gidx, int want_order, i64 seq_base,
                                                     u64* stage) {
    __shared__ ulonglong2 sw[kBlock][kStageMax / 2];
    __shared__ i64 so[kBlock];
    // thread (unit, j): the j-th row of a unit's region, if the unit produced that many
    const int t = threadIdx.x;
    // XCD-aware: each XCD takes a contiguous run of blocks (a few windows), so the random reads of
    // its rows' last-event timestamps stay inside a window-sized range its own L2 holds
    const int nb = gridDim.x, per = (nb + 7) >> 3;
    const int lb = (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
    const i64 r = (i64)lb * kBlock + t;
    const i64 u = r / unit_stride;
    const bool valid = u < n_units && (u32)(r - u * unit_stride) < unit_rows[u];
    const int nk = kp.n, SW = stage_words(nk, n_aggs, want_order);
    so[t] = -1;
    if (valid) {
        const u64* row = rows + (size_t)r * RW;
        const ulonglong2 h = *(const ulonglong2*)row;
        const u32 pos = (u32)h.x, first = (u32)h.y;
        const u32 wd = first >> 5;
        const u64 wp2 = word_pre[wd];  // one read: the bitmap word and the rows before it
        const i64 o = (i64)(u32)wp2 + __popc((u32)(wp2 >> 32) & ((1u << (first & 31)) - 1u));
        // stream index of an event of the combined (queued + new) sequence
        auto sidx = [&](u32 c) -> i64 {
            if (c < n_pend) return (i64)pend_gidx[c];
            return new_gidx ? (i64)new_gidx[c - n_pend] : seq_base + (i64)(c - n_pend);
        };
        u64 w[kStageMax + 1];
        const ulonglong2 tr = *(const ulonglong2*)(row + 2);  // the last event's timestamp and stream index
        w[0] = tr.x;
        i64 kv[kKeyParts] = {0, 0};
        unpack_key(kp, slot_key(kt, pos), kv, 1);
        w[1] = tr.y;
        w[2] = (u64)kv[0];
        w[3] = (u64)kv[1];
        int c = 2 + nk;
        if (want_order) w[c++] = (u64)sidx(first);
#pragma unroll
        for (int a = 0; a < SH_MAX_AGGS; a++) if (a < n_aggs) w[c + a] = row[4 + a];
#pragma unroll
        for (int i = 0; i < kStageMax / 2; i++) {
            if (2 * i >= SW) break;
            sw[t][i] = make_ulonglong2(w[2 * i], w[2 * i + 1]);
        }
        so[t] = o;
    }
    __syncthreads();
    // the wave's 64 records as SW / 2 pieces each, piece-major across lanes
    const int pcs = SW / 2, wb = t & ~63, lane = t & 63;
    for (int q = lane; q < 64 * pcs; q += 64) {
        const int rec = q / pcs, pc = q - rec * pcs;
        const i64 o = so[wb + rec];
        if (o >= 0) ((ulonglong2*)(stage + (size_t)o * SW))[pc] = sw[wb + rec][pc];
    }
}

// Stage 2, one output row per thread: the staged records split into the SoA output columns.
__global__ __launch_bounds__(kBlock) void k_emit_soa(const u64* __restrict__ stage, const u32* __restrict__ n_rows_dev,
                                                    int nk, int n_aggs, int want_order, i64 out_cap, i64* out_ts,
                                                    i64* out_keys, u64* out_vals, i64* out_order, i64* out_rep) {
    const i64 o = (i64)blockIdx.x * kBlock + threadIdx.x;
    const i64 n = (i64)*n_rows_dev;  // the column stride of the output: [k][n_rows] as sh_out states
    if (o >= n) return;
    (void)out_cap;
    const int SW = stage_words(nk, n_aggs, want_order);
    const u64* src = stage + (size_t)o * SW;
    u64 w[2 + kKeyParts + 1 + SH_MAX_AGGS + 1];
#pragma unroll
    for (int i = 0; i < (2 + kKeyParts + 1 + SH_MAX_AGGS + 1) / 2; i++) {
        if (2 * i >= SW) break;
        const ulonglong2 v = ((const ulonglong2*)src)[i];
        w[2 * i] = v.x;
        w[2 * i + 1] = v.y;
    }
    out_ts[o] = (i64)w[0];
    out_rep[o] = (i64)w[1];
    for (int k = 0; k < nk; k++) out_keys[(size_t)k * n + o] = (i64)w[2 + k];
    int c = 2 + nk;
    if (want_order) out_order[o] = (i64)w[c++];
    for (int a = 0; a < n_aggs; a++) out_vals[(size_t)a * n + o] = w[c + a];
}

void launch_emit_rows(hipStream_t s, const u64* rows, int RW, const u32* unit_rows, i64 n_units, int unit_stride,
                      i64 row_cap, const u32* n_rows_dev, const u64* word_pre, int n_aggs, KeyTable kt,
                      KeyPlan kp, i64 n_pend, const i64* pend_ts, const i64* ts, i64 out_cap, i64* out_ts,
                      i64* out_keys, u64* out_vals, const u64* pend_gidx, const u64* new_gidx, i64* out_order,
                      i64 seq_base, i64* out_rep, u64* stage) {
    if (row_cap <= 0 || n_units <= 0) return;
    const int want_order = out_order ? 1 : 0;
    // (rounded to a multiple of 8 for the XCD-aware block order; surplus blocks find no row)
    const unsigned g1 = (unsigned)(((n_units * unit_stride + kBlock - 1) / kBlock + 7) / 8 * 8);
    hipLaunchKernelGGL(k_emit_rank, dim3(g1), dim3(kBlock), 0, s, rows, RW, unit_rows, n_units, unit_stride, word_pre,
                       n_aggs, kt, kp, n_pend, pend_ts, ts, pend_gidx, new_gidx, want_order, seq_base, stage);
    const unsigned g2 = (unsigned)((row_cap + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_emit_soa, dim3(g2), dim3(kBlock), 0, s, stage, n_rows_dev, kp.n, n_aggs, want_order, out_cap,
                       out_ts, out_keys, out_vals, out_order, out_rep);
}

size_t emit_stage_bytes(int nk, int na, int order, i64 n_rows) { return (size_t)stage_words(nk, na, order) * 8 * n_rows; }

// One-pass emission for rows the fold left at their key's slot (dense rows, k_aggregate_own `dense`).
// A wave takes 512 events of the combined index space (16 words of the first-occurrence bitmap): every
// set bit is a row's first event e. The lanes load the key slots of their 8 events (the slot column or
// the dictionary ids, coalesced) and compact the set ones into LDS in event order; the chunk's rows have
// consecutive output ranks from the first word's prefix. Then each lane takes every 64th entry: its
// segment (the closed window holding e) and slot name the unit and local key, the row is read where the
// fold wrote it and its columns are stored at the rank — consecutive lanes, consecutive ranks. Replaces
// the rank scatter of whole records and the column split (k_emit_rank + k_emit_soa): one read of every
// row instead of two, no staged copy.
constexpr int kGatherEv = 512;  // events per wave
__global__ __launch_bounds__(kBlock) void k_emit_gather(const u64* __restrict__ word_pre, i64 nw,
                                                       const Segment* __restrict__ segs, int nseg, int P, int logP,
                                                       int unit_stride, const u64* __restrict__ rows, int RW,
                                                       PosSrc ps, const u32* __restrict__ pend_pos, i64 n_pend,
                                                       const u32* __restrict__ n_rows_dev, int n_aggs, KeyTable kt,
                                                       KeyPlan kp, i64* out_ts, i64* out_keys, u64* out_vals,
                                                       const u64* __restrict__ pend_gidx,
                                                       const u64* __restrict__ new_gidx, i64* out_order, i64 seq_base,
                                                       i64* out_rep) {
    __shared__ u32 ent_e[kBlock / 64][kGatherEv], ent_s[kBlock / 64][kGatherEv];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const i64 e_base = ((i64)blockIdx.x * (kBlock / 64) + wv) * kGatherEv;
    const i64 n_ev = nw * 32;
    const bool act = e_base < n_ev;
    const i64 w0 = e_base >> 5;
    // the lane's 8 events: bits (lane & 3) * 8 .. + 8 of word w0 + lane / 4
    const i64 w = w0 + (lane >> 2);
    u32 bits8 = 0;
    if (act && w < nw) bits8 = ((u32)(word_pre[w] >> 32) >> ((lane & 3) * 8)) & 0xFFu;
    const int cnt = __popc(bits8);
    int pre = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int up = __shfl_up(pre, d, 64);
        if (lane >= d) pre += up;
    }
    const int total = __shfl(pre, 63, 64);
    pre -= cnt;
    for (int k = 0; bits8; k++) {
        const int b = __ffs(bits8) - 1;
        bits8 &= bits8 - 1;
        const int off = lane * 8 + b;
        const i64 e = e_base + off;
        ent_e[wv][pre + k] = (u32)off;
        ent_s[wv][pre + k] = e < n_pend ? pend_pos[e] : pos_at(ps, e - n_pend);
    }
    __syncthreads();
    if (!act || total == 0) return;
    const i64 o0 = (i64)(u32)word_pre[w0];  // the rank of the chunk's first row
    const i64 n = (i64)*n_rows_dev;         // the output columns' stride ([k][n_rows])
    // the segment holding the chunk's first event (segments are consecutive, sorted by lo)
    int s0 = 0, hi = nseg - 1;
    while (s0 < hi) {
        const int mid = (s0 + hi + 1) >> 1;
        if (segs[mid].lo <= e_base) s0 = mid;
        else hi = mid - 1;
    }
    const int nk = kp.n;
    for (int j = lane; j < total; j += 64) {
        const i64 e = e_base + ent_e[wv][j];
        const u32 slot = ent_s[wv][j];
        int sg = s0;
        while (sg + 1 < nseg && e >= segs[sg].hi) sg++;
        const i64 unit = (i64)sg * P + (slot & (u32)(P - 1));
        const u64* row = rows + ((size_t)unit * unit_stride + (slot >> logP)) * RW;
        const ulonglong2 h0 = ((const ulonglong2*)row)[1];  // the last event's timestamp and stream index
        u64 av[SH_MAX_AGGS];
#pragma unroll
        for (int a = 0; a < SH_MAX_AGGS / 2; a++) {
            if (2 * a >= n_aggs) break;
            const ulonglong2 v = ((const ulonglong2*)row)[2 + a];
            av[2 * a] = v.x;
            av[2 * a + 1] = v.y;
        }
        const i64 o = o0 + j;
        out_ts[o] = (i64)h0.x;
        out_rep[o] = (i64)h0.y;
        i64 kv[kKeyParts] = {0, 0};
        unpack_key(kp, slot_key(kt, slot), kv, 1);
        for (int k = 0; k < nk; k++) out_keys[(size_t)k * n + o] = kv[k];
        if (out_order)
            out_order[o] = e < n_pend ? (i64)pend_gidx[e] : new_gidx ? (i64)new_gidx[e - n_pend] : seq_base + (e - n_pend);
#pragma unroll
        for (int a = 0; a < SH_MAX_AGGS; a++)
            if (a < n_aggs) out_vals[(size_t)a * n + o] = av[a];
    }
}

void launch_emit_gather(hipStream_t s, const u64* word_pre, i64 nw, const Segment* segs, int nseg, int P, int logP,
                        int unit_stride, const u64* rows, int RW, PosSrc ps, const u32* pend_pos, i64 n_pend,
                        const u32* n_rows_dev, int n_aggs, KeyTable kt, KeyPlan kp, i64* out_ts, i64* out_keys,
                        u64* out_vals, const u64* pend_gidx, const u64* new_gidx, i64* out_order, i64 seq_base,
                        i64* out_rep) {
    if (nw <= 0 || nseg <= 0) return;
    const i64 per_block = (i64)(kBlock / 64) * kGatherEv / 32;  // words per block
    hipLaunchKernelGGL(k_emit_gather, dim3((unsigned)((nw + per_block - 1) / per_block)), dim3(kBlock), 0, s, word_pre, nw,
                       segs, nseg, P, logP, unit_stride, rows, RW, ps, pend_pos, n_pend, n_rows_dev, n_aggs, kt, kp,
                       out_ts, out_keys, out_vals, pend_gidx, new_gidx, out_order, seq_base, out_rep);
}

// ================================================================================================
// k_compact_pending: passing events of the open window [e_lo, N) appended to the pending buffer
// (the window's queued events, LengthBatch WindowState.currentEventQueue / TimeBatch queue).
// ================================================================================================
__global__ __launch_bounds__(kBlock) void k_compact_pending(const i64* __restrict__ ts, ColSet cols,
                                                           PosSrc new_pos, AggPlan ap, i64 e_lo,
                                                           i64 N, i64 pcb_lo, i64 dst_base, const i64* blk_pass_pre,
                                                           int blk0, u32* pend_pos, i64* pend_ts, u64* pend_vals,
                                                           i64 pend_cap, const u64* __restrict__ new_gidx,
                                                           u64* pend_gidx, i64 seq_base) {
    // the tile's events taken lane-strided (round i: events tile + i * kBlock + thread), one block scan
    // per round: consecutive lanes read and write consecutive entries (the thread-contiguous form's
    // stores were 64 pieces 8 entries apart per instruction; r05: 1.9 ms of c2cur's push)
    const int blk = blk0 + blockIdx.x;
    const i64 tile = (i64)blk * kTile;
    i64 run = blk_pass_pre[blk];
    for (int it = 0; it < kItems; it++) {
        const i64 e = tile + (i64)it * kBlock + threadIdx.x;
        const u32 p = e < N ? pos_at(new_pos, e) : kNoPos;
        const i64 fl = p != kNoPos;
        i64 tot;
        const i64 pcb = run + block_excl_scan(fl, SumOp(), 0, &tot);
        run += tot;
        if (fl && e >= e_lo) {
            const i64 d = dst_base + (pcb - pcb_lo);
            pend_pos[d] = p;
            pend_ts[d] = ts[e];
            for (int j = 0; j < ap.n_vcols; j++) pend_vals[(size_t)j * pend_cap + d] = (u64)load_raw(cols, ap.vcol_src[j], e);
            pend_gidx[d] = new_gidx ? new_gidx[e] : (u64)(seq_base + e);
        }
    }
}

void launch_compact_pending(hipStream_t s, const i64* ts, ColSet cols, PosSrc new_pos, AggPlan ap, i64 e_lo,
                            i64 N, i64 pcb_lo, i64 base, const i64* blk_pass_pre, u32* pend_pos, i64* pend_ts,
                            u64* pend_vals, i64 pend_cap, const u64* new_gidx, u64* pend_gidx, i64 seq_base) {
    if (e_lo >= N) return;
    int blk0 = (int)(e_lo / kTile);
    int blk1 = (int)((N + kTile - 1) / kTile);
    hipLaunchKernelGGL(k_compact_pending, dim3(blk1 - blk0), dim3(kBlock), 0, s, ts, cols, new_pos, ap, e_lo, N,
                       pcb_lo, base, blk_pass_pre, blk0, pend_pos, pend_ts, pend_vals, pend_cap, new_gidx,
                       pend_gidx, seq_base);
}

}  // namespace shd

namespace shd {

// ================================================================================================
// Multisplit: stable partition of the closed events (pending records + new events) by key
// partition p = pos & (P - 1). Partition p's list stays in event order, so every (window, p)
// work item sees its events in the order the reference's selector sees them.
// ================================================================================================
struct EvLoad {
    bool ok;
    u32 pos;
};

// combined index space: pending events [0, n_pend), then the push's events
__device__ __forceinline__ EvLoad load_pos(i64 e, i64 n_pend, const u32* pend_pos, const PosSrc& new_pos) {
    u32 p = e < n_pend ? pend_pos[e] : pos_at(new_pos, e - n_pend);
    return EvLoad{p != kNoPos, p};
}

// XCD-aware tile order: workgroups are dealt to the 8 XCDs round-robin, so give each XCD a
// contiguous run of tiles; a partition's consecutive record runs are then written through one L2.
__device__ __forceinline__ int xcd_tile(int nblk) {
    int per = (nblk + 7) >> 3;
    return (int)(blockIdx.x & 7) * per + (int)(blockIdx.x >> 3);
}

__global__ __launch_bounds__(kBlock) void k_ms_count(TileMap m, int n_count, i64 n_pend, const u32* __restrict__ pend_pos,
                                                    PosSrc new_pos, int P, u32* counts) {
    extern __shared__ __attribute__((aligned(16))) u32 hist[];
    const int tile = xcd_tile(n_count);
    if (tile >= n_count) return;
    for (int i = threadIdx.x; i < P; i += kBlock) hist[i] = 0;
    __syncthreads();
    const i64 t0 = tile_lo(m, tile), t1 = tile_hi(m, tile);
    for (int r = 0; r < kItems; r++) {
        i64 e = t0 + (i64)r * kBlock + threadIdx.x;
        if (e < t1) {
            EvLoad ev = load_pos(e, n_pend, pend_pos, new_pos);
            if (ev.ok) atomicAdd(&hist[ev.pos & (P - 1)], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < P; i += kBlock) counts[(i64)tile * P + i] = hist[i];
}

void launch_ms_count(hipStream_t s, TileMap m, int n_count, i64 n_pend, const u32* pend_pos, PosSrc new_pos, int P,
                     u32* counts) {
    int grid = std::max(1, ((n_count + 7) >> 3) * 8);
    hipLaunchKernelGGL(k_ms_count, dim3(grid), dim3(kBlock), P * 4, s, m, n_count, n_pend, pend_pos, new_pos, P, counts);
}

// Stable multisplit of one tile of kTile closed events into the P key partitions. Wave w takes
// the tile's events [w*512, w*512+512) in 8 rounds of 64; all 8 rounds' positions and values are
// loaded first (one memory latency per tile). An event's rank inside its partition is the wave's
// running count for that partition plus its rank among the round's lanes of the same partition
// (ballots over the partition bits). One barrier, a scan over (partition, wave) gives every event
// its staging slot (partition-major, event order inside a partition), and the staged tile is
// written out as one contiguous run per partition.
// LDS: stage_vals[V][kTile] | stage_pos[kTile] | stage_idx[kTile] | start[P] | gbase[P] (i64) | run[4][P] (u16)
template <int V, bool PACK>
__global__ __launch_bounds__(kBlock) void k_ms_scatter(TileMap m, i64 n_pend, const u32* __restrict__ pend_pos,
                                                      const u64* __restrict__ pend_vals, i64 pend_cap,
                                                      PosSrc new_pos, ColSet cols, AggPlan ap, int P,
                                                      int logP, const u32* __restrict__ offsets, u32* rec_pos,
                                                      u32* rec_idx, u64* rec_vals, i64 rec_cap) {
    const int nblk = m.nblk;
    const int tile = xcd_tile(nblk);
    if (tile >= nblk) return;
    constexpr int NW = kBlock / 64;
    constexpr int PER_WAVE = kTile / NW;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    unsigned char* sm = smem_raw + ((16u - ((unsigned)(size_t)smem_raw & 15u)) & 15u);
    u64* stage_vals = (u64*)sm;
    u32* stage_pos = (u32*)(stage_vals + (size_t)V * kTile);
    u32* stage_idx = stage_pos + kTile;
    u32* start = stage_idx + kTile;
    i64* gbase = (i64*)(start + P + (P & 1));                // [P] global position of the tile's run - start
    unsigned short* run = (unsigned short*)(gbase + P);  // [NW][P]
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const i64 t0 = tile_lo(m, tile) + (i64)w * PER_WAVE, hi = tile_hi(m, tile);
    // every round's position and values, and the tile's run offsets (one per partition, strided by
    // nblk in the [p][tile] scan), requested before anything waits on them
    u32 my_pos[kItems];
    u64 my_val[kItems][V];
#pragma unroll
    for (int r = 0; r < kItems; r++) {
        const i64 e = t0 + (i64)r * 64 + lane;
        u32 pos = kNoPos;
#pragma unroll
        for (int j = 0; j < V; j++) my_val[r][j] = 0;
        if (e < hi) {
            if (e < n_pend) {
                pos = pend_pos[e];
#pragma unroll
                for (int j = 0; j < V; j++)
                    if (j < ap.n_vcols) my_val[r][j] = pend_vals[(size_t)j * pend_cap + e];
            } else {
                pos = pos_at(new_pos, e - n_pend);
#pragma unroll
                for (int j = 0; j < V; j++)
                    if (j < ap.n_vcols) my_val[r][j] = (u64)load_raw(cols, ap.vcol_src[j], e - n_pend);
            }
        }
        my_pos[r] = pos;
    }
    constexpr int kOffRegs = 4;
    i64 off_reg[kOffRegs];
#pragma unroll
    for (int k = 0; k < kOffRegs; k++) {
        const int i = threadIdx.x + k * kBlock;
        off_reg[k] = i < P ? (i64)offsets[(i64)tile * P + i] : 0;
    }
    for (int i = threadIdx.x; i < NW * P; i += kBlock) run[i] = 0;
    __syncthreads();
    // rank = the wave's running count of its partition, advanced by LDS atomics on the 16-bit
    // counters (two per 32-bit word); the wave's rounds complete in program order, and lanes of one
    // round that hit the same counter receive their values in lane order on gfx950
    // (scripts/probe/lds_atomic_order.hip) — the check after staging repairs the order if not
    u32* wrun32 = (u32*)run;
    unsigned short* wrun = run + w * P;
    u32 my_rank[kItems];
#pragma unroll
    for (int r = 0; r < kItems; r++) {
        my_rank[r] = 0;
        if (my_pos[r] == kNoPos) continue;
        const u32 c = (u32)(w * P) + (my_pos[r] & (P - 1));
        const u32 sh = (c & 1) * 16;
        my_rank[r] = (atomicAdd(&wrun32[c >> 1], 1u << sh) >> sh) & 0xFFFFu;
    }
    __syncthreads();
    // partition starts in the tile (p-major), then each wave's offset inside its partition
    __shared__ u32 s_total;
    {
        int per = (P + kBlock - 1) / kBlock;
        int a = threadIdx.x * per, b = min(P, a + per);
        i64 sum = 0;
        for (int i = a; i < b; i++)
            for (int x = 0; x < NW; x++) sum += run[x * P + i];
        i64 tot;
        i64 pre = block_excl_scan(sum, SumOp(), 0, &tot);
        if (threadIdx.x == 0) s_total = (u32)tot;
        for (int i = a; i < b; i++) {
            const i64 st = pre;
            start[i] = (u32)st;
            for (int x = 0; x < NW; x++) {
                u32 c = run[x * P + i];
                run[x * P + i] = (unsigned short)(pre - st);  // wave x's offset inside partition i
                pre += c;
            }
        }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kOffRegs; k++) {
        const int i = threadIdx.x + k * kBlock;
        if (i < P) gbase[i] = off_reg[k] - (i64)start[i];
    }
    for (int i = threadIdx.x + kOffRegs * kBlock; i < P; i += kBlock) gbase[i] = (i64)offsets[(i64)tile * P + i] - (i64)start[i];
#pragma unroll
    for (int r = 0; r < kItems; r++) {
        if (my_pos[r] == kNoPos) continue;
        const u32 p = my_pos[r] & (P - 1);
        const u32 slot = start[p] + wrun[p] + my_rank[r];
        stage_pos[slot] = my_pos[r];
        stage_idx[slot] = (u32)(t0 + (i64)r * 64 + lane);
#pragma unroll
        for (int j = 0; j < V; j++)
            if (j < ap.n_vcols) stage_vals[(size_t)j * kTile + slot] = my_val[r][j];
    }
    __syncthreads();
    const u32 n_tile = s_total;
    // stability check: inside each partition's run the events must be in stream order
    bool bad = false;
    for (u32 j = threadIdx.x; j + 1 < n_tile; j += kBlock)
        bad |= stage_idx[j + 1] < stage_idx[j] && ((stage_pos[j + 1] ^ stage_pos[j]) & (P - 1)) == 0;
    if (__syncthreads_or(bad)) {
        for (int p = threadIdx.x; p < P; p += kBlock) {
            const u32 a = start[p], b = p + 1 < P ? start[p + 1] : n_tile;
            for (u32 k = a + 1; k < b; k++) {
                const u32 e = stage_idx[k], pos = stage_pos[k];
                u64 mv[V];
#pragma unroll
                for (int j = 0; j < V; j++) mv[j] = j < ap.n_vcols ? stage_vals[(size_t)j * kTile + k] : 0;
                u32 m = k;
                while (m > a && stage_idx[m - 1] > e) {
                    stage_idx[m] = stage_idx[m - 1];
                    stage_pos[m] = stage_pos[m - 1];
#pragma unroll
                    for (int j = 0; j < V; j++)
                        if (j < ap.n_vcols) stage_vals[(size_t)j * kTile + m] = stage_vals[(size_t)j * kTile + m - 1];
                    m--;
                }
                stage_idx[m] = e;
                stage_pos[m] = pos;
#pragma unroll
                for (int j = 0; j < V; j++)
                    if (j < ap.n_vcols) stage_vals[(size_t)j * kTile + m] = mv[j];
            }
        }
        __syncthreads();
    }
    // write every partition's run of this tile contiguously
    for (u32 j = threadIdx.x; j < n_tile; j += kBlock) {
        const u32 pp = stage_pos[j] & (P - 1);
        const i64 dst = gbase[pp] + j;
        if (PACK) {
            rec_idx[dst] = ((stage_pos[j] >> logP) << kPackIdxBits) | (stage_idx[j] & kPackIdxMask);
        } else {
            rec_pos[dst] = stage_pos[j];
            rec_idx[dst] = stage_idx[j];
        }
#pragma unroll
        for (int v = 0; v < V; v++)
            if (v < ap.n_vcols) rec_vals[(size_t)v * rec_cap + dst] = stage_vals[(size_t)v * kTile + j];
    }
}

void launch_ms_scatter(hipStream_t s, TileMap m, i64 n_pend, const u32* pend_pos, const u64* pend_vals,
                       i64 pend_cap, PosSrc new_pos, ColSet cols, AggPlan ap, int P, int logP, const u32* offsets,
                       u32* rec_pos, u32* rec_idx, u64* rec_vals, i64 rec_cap, bool pack) {
    const int nblk = m.nblk;
    const int V = ap.n_vcols <= 1 ? 1 : ap.n_vcols <= 2 ? 2 : ap.n_vcols <= 4 ? 4 : 8;
    size_t lds = (size_t)V * kTile * 8 + (size_t)kTile * 8 + (size_t)P * 4 + 4 + (size_t)P * 8 +
                 (size_t)P * 2 * (kBlock / 64) + 32;
    int grid = ((nblk + 7) >> 3) * 8;
#define SH_MS(VV)                                                                                                   \
    do {                                                                                                            \
        if (pack)                                                                                                   \
            hipLaunchKernelGGL((k_ms_scatter<VV, true>), dim3(grid), dim3(kBlock), lds, s, m, n_pend, pend_pos,       \
                               pend_vals, pend_cap, new_pos, cols, ap, P, logP, offsets, rec_pos, rec_idx, rec_vals,  \
                               rec_cap);                                                                            \
        else                                                                                                        \
            hipLaunchKernelGGL((k_ms_scatter<VV, false>), dim3(grid), dim3(kBlock), lds, s, m, n_pend, pend_pos,      \
                               pend_vals, pend_cap, new_pos, cols, ap, P, logP, offsets, rec_pos, rec_idx, rec_vals,  \
                               rec_cap);                                                                            \
    } while (0)
    if (V == 1) SH_MS(1);
    else if (V == 2) SH_MS(2);
    else if (V == 4) SH_MS(4);
    else SH_MS(8);
#undef SH_MS
}

// three-phase exclusive scan for long arrays (i64, or u32 counts whose total stays below 2^32): each
// thread takes kItems consecutive elements with 16-byte loads and stores
template <typename T>
__device__ __forceinline__ void load_run(const T* a, i64 base, i64 n, T (&v)[kItems]) {
    constexpr int PER16 = 16 / sizeof(T);
    if (base + kItems <= n && (((size_t)(a + base)) & 15) == 0) {
#pragma unroll
        for (int j = 0; j < kItems / PER16; j++) {
            const uint4 q = ((const uint4*)(a + base))[j];
            const T* e = (const T*)&q;
#pragma unroll
            for (int k = 0; k < PER16; k++) v[j * PER16 + k] = e[k];
        }
    } else {
#pragma unroll
        for (int i = 0; i < kItems; i++) v[i] = base + i < n ? a[base + i] : (T)0;
    }
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_reduce_tiles(const T* a, i64 n, i64* tmp) {
    const i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    T v[kItems];
    load_run(a, base, n, v);
    i64 s = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) s += (i64)v[i];
    i64 t = block_reduce(s, SumOp(), 0);
    if (threadIdx.x == 0) tmp[blockIdx.x] = t;
}

template <typename T>
__global__ __launch_bounds__(kBlock) void k_scan_tiles(T* a, i64 n, const i64* tmp) {
    const i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    T v[kItems];
    load_run(a, base, n, v);
    i64 s = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) s += (i64)v[i];
    i64 pre = block_excl_scan(s, SumOp(), 0, nullptr) + tmp[blockIdx.x];
    T o[kItems];
#pragma unroll
    for (int i = 0; i < kItems; i++) { o[i] = (T)pre; pre += (i64)v[i]; }
    constexpr int PER16 = 16 / sizeof(T);
    if (base + kItems <= n && (((size_t)(a + base)) & 15) == 0) {
#pragma unroll
        for (int j = 0; j < kItems / PER16; j++) ((uint4*)(a + base))[j] = *(const uint4*)&o[j * PER16];
    } else {
#pragma unroll
        for (int i = 0; i < kItems; i++) if (base + i < n) a[base + i] = o[i];
    }
}

void launch_scan_sum_large(hipStream_t s, i64* a, i64 n, i64* tmp) {
    if (n <= 16384) {  // (one workgroup's loop: one launch instead of three, e.g. a push's tile counts)
        launch_scan_sum(s, a, (int)n);
        return;
    }
    int nb = (int)((n + kTile - 1) / kTile);
    hipLaunchKernelGGL(k_reduce_tiles<i64>, dim3(nb), dim3(kBlock), 0, s, a, n, tmp);
    launch_scan_sum(s, tmp, nb);
    hipLaunchKernelGGL(k_scan_tiles<i64>, dim3(nb), dim3(kBlock), 0, s, a, n, tmp);
}

void launch_scan_sum_large_u32(hipStream_t s, u32* a, i64 n, i64* tmp) {
    int nb = (int)((n + kTile - 1) / kTile);
    hipLaunchKernelGGL(k_reduce_tiles<u32>, dim3(nb), dim3(kBlock), 0, s, a, n, tmp);
    launch_scan_sum(s, tmp, nb);
    hipLaunchKernelGGL(k_scan_tiles<u32>, dim3(nb), dim3(kBlock), 0, s, a, n, tmp);
}

__global__ void k_part_off(const i64* counts, int nblk, int P, i64* part_off) {
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p <= P) part_off[p] = counts[(i64)p * nblk];
}

void launch_part_off(hipStream_t s, const i64* counts, int nblk, int P, i64* part_off) {
    hipLaunchKernelGGL(k_part_off, dim3((P + 1 + 255) / 256), dim3(256), 0, s, counts, nblk, P, part_off);
}

// Record offsets of the [tile][partition] count matrix, in place: offset(t, p) = (records of the
// partitions before p) + (records of p in the tiles before t) — the stable multisplit's layout
// (partition-major, tile order inside a partition). Row nblk gets each partition's end. Three passes
// over coalesced rows: per block of kColT tiles the per-partition sums, per partition the exclusive
// scan over the blocks (+ its total), the scan of the totals over the partitions, then the rows.
constexpr int kColT = 16;
__global__ __launch_bounds__(kBlock) void k_col_reduce(const u32* __restrict__ c, int nblk, int P, i64* bsum,
                                                      u32* ticket) {
    const int b = blockIdx.y;
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (b == 0 && p == 0) *ticket = 0;  // k_col_blocks' completion count
    if (p >= P) return;
    const int t0 = b * kColT, t1 = min(nblk, t0 + kColT);
    i64 acc = 0;
    for (int t = t0; t < t1; t++) acc += c[(i64)t * P + p];
    bsum[(i64)b * P + p] = acc;
}

// One workgroup per partition: the exclusive scan of its column of block sums, kBlock blocks at a
// time (a thread per column walking every block serialised nb dependent loads: 63 us at C2 size).
// The last workgroup to finish also turns the partitions' totals into their bases (an exclusive scan
// over P), so no separate copy + scan launches.
__global__ __launch_bounds__(kBlock) void k_col_blocks(i64* bsum, int nb, int P, i64* total, i64* base, u32* ticket) {
    const int p = blockIdx.x;
    i64 run = 0;
    for (int b0 = 0; b0 < nb; b0 += kBlock) {
        const int b = b0 + threadIdx.x;
        const i64 x = b < nb ? bsum[(i64)b * P + p] : 0;
        i64 tot;
        const i64 pre = block_excl_scan(x, SumOp(), 0, &tot);
        if (b < nb) bsum[(i64)b * P + p] = run + pre;
        run += tot;
    }
    __shared__ bool last;
    if (threadIdx.x == 0) {
        total[p] = run;
        __threadfence();
        last = atomicAdd(ticket, 1u) == (u32)(P - 1);
    }
    __syncthreads();
    if (!last) return;
    __threadfence();
    i64 carry = 0;
    for (int q0 = 0; q0 < P; q0 += kBlock) {
        const int q = q0 + threadIdx.x;
        const i64 x = q < P ? __atomic_load_n(&total[q], __ATOMIC_RELAXED) : 0;
        i64 tot;
        const i64 pre = block_excl_scan(x, SumOp(), 0, &tot);
        if (q < P) base[q] = carry + pre;
        carry += tot;
    }
}

// Many partitions over few block rows (C4's band-keyed roots: 16k partitions, ~64 rows): a thread per
// partition walks its column (coalesced across the partitions; the rows are loaded 8 at a time) and
// the partitions' totals are scanned by k_scan_sum — k_col_blocks' one workgroup per partition plus
// its last workgroup's P / kBlock serial block scans cost ~95 us there.
__global__ __launch_bounds__(kBlock) void k_col_walk(i64* __restrict__ bsum, int nb, int P, i64* __restrict__ total,
                                                    i64* __restrict__ base) {
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= P) return;
    i64 run = 0;
    for (int b0 = 0; b0 < nb; b0 += 8) {
        i64 x[8];
#pragma unroll
        for (int k = 0; k < 8; k++) x[k] = b0 + k < nb ? bsum[(i64)(b0 + k) * P + p] : 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            if (b0 + k < nb) bsum[(i64)(b0 + k) * P + p] = run;
            run += x[k];
        }
    }
    total[p] = run;
    base[p] = run;  // (exclusive-scanned in place next)
}

__global__ __launch_bounds__(kBlock) void k_col_apply(u32* c, int nblk, int P, const i64* __restrict__ bpre,
                                                     const i64* __restrict__ base, const i64* __restrict__ total) {
    const int b = blockIdx.y;
    const int p = blockIdx.x * kBlock + threadIdx.x;
    if (p >= P) return;
    const int t0 = b * kColT, t1 = min(nblk, t0 + kColT);
    i64 run = base[p] + bpre[(i64)b * P + p];
    for (int t = t0; t < t1; t++) {
        const u32 x = c[(i64)t * P + p];
        c[(i64)t * P + p] = (u32)run;
        run += x;
    }
    if (t1 == nblk) c[(i64)nblk * P + p] = (u32)(base[p] + total[p]);
}

size_t ms_offsets_tmp_bytes(int nblk, int P) {
    const size_t nb = (size_t)(std::max(nblk, 1) + kColT - 1) / kColT;
    return (nb * P + 2 * (size_t)P + 16) * 8;
}

void launch_ms_offsets(hipStream_t s, u32* counts, int nblk, int P, i64* tmp) {
    const int nb = (std::max(nblk, 1) + kColT - 1) / kColT;
    i64* bsum = tmp;
    i64* total = tmp + (size_t)nb * P;
    i64* base = total + P;
    u32* ticket = (u32*)(base + P);
    const dim3 g((P + kBlock - 1) / kBlock, nb);
    // (nblk == 0: the reduce pass still runs — zero block sums over no tiles — and zeroes the ticket)
    hipLaunchKernelGGL(k_col_reduce, g, dim3(kBlock), 0, s, counts, nblk, P, bsum, ticket);
    if (P >= 2048 && nb <= 256) {
        hipLaunchKernelGGL(k_col_walk, dim3((P + kBlock - 1) / kBlock), dim3(kBlock), 0, s, bsum, nb, P, total, base);
        launch_scan_sum(s, base, P);
    } else {
        hipLaunchKernelGGL(k_col_blocks, dim3(P), dim3(kBlock), 0, s, bsum, nb, P, total, base, ticket);
    }
    if (nblk > 0) hipLaunchKernelGGL(k_col_apply, g, dim3(kBlock), 0, s, counts, nblk, P, bsum, base, total);
    else hipLaunchKernelGGL(k_col_apply, dim3((P + kBlock - 1) / kBlock, 1), dim3(kBlock), 0, s, counts, nblk, P, bsum,
                            base, total);
}

// Record offset of every segment boundary in every partition's list: boundary b lies in tile
// t = b / kTile; offset = (scanned count of p before tile t) + (p-records of tile t before b).
__global__ __launch_bounds__(kBlock) void k_seg_offsets(const Segment* __restrict__ segs, int nseg, i64 n_pend,
                                                       const u32* __restrict__ pend_pos,
                                                       PosSrc new_pos, int P,
                                                       const u32* __restrict__ counts, TileMap m, i64* seg_off) {
    extern __shared__ __attribute__((aligned(16))) u32 hist[];
    const int k = blockIdx.x;
    const i64 b = k < nseg ? segs[k].lo : segs[nseg - 1].hi;
    const int t = tile_of(m, b);
    for (int i = threadIdx.x; i < P; i += kBlock) hist[i] = 0;
    __syncthreads();
    for (i64 e = tile_lo(m, t) + threadIdx.x; e < b; e += kBlock) {
        EvLoad ev = load_pos(e, n_pend, pend_pos, new_pos);
        if (ev.ok) atomicAdd(&hist[ev.pos & (P - 1)], 1u);
    }
    __syncthreads();
    for (int p = threadIdx.x; p < P; p += kBlock) seg_off[(i64)k * P + p] = (i64)counts[(i64)t * P + p] + hist[p];
}

void launch_seg_offsets(hipStream_t s, const Segment* segs, int nseg, i64 n_pend, const u32* pend_pos,
                        PosSrc new_pos, int P, const u32* counts, TileMap m, i64* seg_off) {
    hipLaunchKernelGGL(k_seg_offsets, dim3(nseg + 1), dim3(kBlock), P * 4, s, segs, nseg, n_pend, pend_pos, new_pos, P,
                       counts, m, seg_off);
}

#ifdef SH_STAMPS
}  // namespace shd
extern "C" int sh_debug_stamps(unsigned long long* out, long long n, int clear) {
    const long long cap = (long long)shd::kStampKernels * shd::kStampBlocks * shd::kStampPts;
    if (n > cap) n = cap;
    if (out && hipMemcpyFromSymbol(out, HIP_SYMBOL(shd::g_stamps), n * 8, 0, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (clear) {
        static unsigned long long* zero = nullptr;
        if (!zero) zero = (unsigned long long*)calloc(cap, 8);
        if (hipMemcpyToSymbol(HIP_SYMBOL(shd::g_stamps), zero, cap * 8, 0, hipMemcpyHostToDevice) != hipSuccess) return -1;
    }
    return 0;
}
namespace shd {
#endif

// ---- key-table rebuild: the open window's keys move to a fresh table (drops dead keys / grows) ------
__global__ __launch_bounds__(kBlock) void k_rekey(i64 n, u32* pos, KeyTable old_kt, KeyTable new_kt) {
    i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    pos[i] = key_slot(new_kt, slot_key(old_kt, pos[i]));
}

void launch_rekey(hipStream_t s, i64 n, u32* pos, KeyTable old_kt, KeyTable new_kt) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_rekey, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, pos, old_kt, new_kt);
}


// ================================================================================================
// stream.current.event batch windows (sh_stream_current.cpp)
// ================================================================================================
// sh_sc_kernels.hip — `#window.lengthBatch(L, true)` / `#window.timeBatch(T, true)` (stream.current.event)
// with current-events output. The window emits every arriving event at once and resets the aggregators
// when a batch ends (LengthBatchWindowProcessor.processStreamCurrentEvents :245-274, TimeBatchWindow-
// Processor.process :262-340 in RESET mode); the selector groups each chunk by key (QuerySelector
// :315-374: a key's row is the value after its last event of the chunk, at its first position). A row's
// values are therefore the running aggregates of its (window, key) up to that event.
//
// The pending buffer holds [the open window's earlier events | this push's passing events]; the
// entries are stably sorted by (window, key slot), each (window, key) run is folded in event order by
// one thread (the Java order of the double sums), and the last entry of every (chunk, key) group writes
// the group's row values at the group's first entry. A scan over those heads gives the output order.


// The row values (sval) are one record of n_aggs words per row head ([row][agg]): the walk's rows land
// at scattered heads, and one record is one store where [agg][row] columns were n_aggs scattered
// partial-line stores (r05: c2cur's walk).
// window of entry m (0 = the window open before the push; a new entry j is in window #{pcb <= j})
// and its chunk: lengthBatch sends every event on its own (:160-182), timeBatch the whole send
__global__ __launch_bounds__(kBlock) void k_sc_keys(i64 M, i64 n_old, const i64* __restrict__ pcb, int nb,
                                                   const u32* __restrict__ pend_pos, const u64* __restrict__ pend_gidx,
                                                   int per_event, i64 send_size, i64 seq0, u64* skey, u32* idx,
                                                   i64* chunk, i64* send, int by_entry) {
    const i64 m = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (m >= M) return;
    u32 w = 0;
    if (m >= n_old) {
        const i64 j = m - n_old;
        int lo = 0, hi = nb;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (pcb[mid] <= j) lo = mid + 1; else hi = mid;
        }
        w = (u32)lo;
        const i64 e = (i64)pend_gidx[m] - seq0;  // the event's index in the push
        const i64 sd = send_size > 0 ? e / send_size : 0;
        if (chunk) chunk[m] = per_event ? j : sd;  // (null: every entry its own chunk)
        // (a sharded owner: the chunk is the global send, the clock is looked up per record — by_entry)
        send[m] = by_entry ? j : sd;
    } else {
        if (chunk) chunk[m] = -1;
        send[m] = -1;
    }
    skey[m] = ((u64)w << 32) | (u64)pend_pos[m];
    idx[m] = (u32)m;
}

__global__ __launch_bounds__(kBlock) void k_sc_pack_keys(i64 M, unsigned kb, u64* skey) {
    const i64 m = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (m >= M) return;
    const u64 k = skey[m];
    skey[m] = ((k >> 32) << kb) | (k & 0xFFFFFFFFull);
}

void launch_sc_pack_keys(hipStream_t s, i64 M, unsigned kb, u64* skey) {
    if (M <= 0) return;
    hipLaunchKernelGGL(k_sc_pack_keys, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, M, kb, skey);
}

// one thread per (window, key) run of the sorted entries, the runs packed onto the first threads (pos[M]
// runs: a thread per entry that returned unless it was a head left ~9 of 10 lanes idle, C2's runs being
// ~10 entries long)
__global__ __launch_bounds__(kBlock) void k_sc_walk(i64 M, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                   const u32* __restrict__ starts, const u32* __restrict__ idx,
                                                   const i64* __restrict__ chunk, const u64* __restrict__ pend_vals,
                                                   i64 pend_cap, AggPlan ap, i64 n_old, u32* ghead, u64* sval,
                                                   u32* slast) {
    (void)hd;
    const i64 sg = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (sg >= (i64)pos[M]) return;
    const i64 i = starts[sg], hi = starts[sg + 1];
    u64 f[SH_MAX_AGGS];
#pragma unroll
    for (int j = 0; j < SH_MAX_AGGS; j++) f[j] = 0;
    u32 c = 0;
    i64 head = -1;
    // each entry's chunk is read once and carried (the previous / next entry's chunk decide the group's
    // first and last event): one random chunk load per entry instead of three
    // (every new entry its own chunk — ghead null —: the entry's own index names its chunk, no load)
    const bool ah = ghead == nullptr;
    u32 m_nx = idx[i];
    i64 ch_nx = (i64)m_nx < n_old ? -1 : ah ? (i64)m_nx : chunk[m_nx], ch_prev = -2;
    for (i64 t = i; t < hi; t++) {
        const u32 m = m_nx;
        const i64 ch = ch_nx;
        if (t + 1 < hi) {
            m_nx = idx[t + 1];
            ch_nx = (i64)m_nx < n_old ? -1 : ah ? (i64)m_nx : chunk[m_nx];
        }
        i64 v[SH_MAX_AGGS];
#pragma unroll
        for (int j = 0; j < SH_MAX_AGGS; j++) v[j] = j < ap.n_vcols ? (i64)pend_vals[(size_t)j * pend_cap + m] : 0;
        fold_fields<SH_MAX_AGGS>(ap, f, c == 0, v);
        c++;
        const i64 cp = ch_prev;
        ch_prev = ch;
        if ((i64)m < n_old) continue;
        if (head < 0 || cp != ch) {
            head = m;
            if (ghead) ghead[m] = 1;  // (null: every new entry is its own chunk, so its own row)
        }
        if (t + 1 == hi || ch_nx != ch) {  // the group's last event: its row values
#pragma unroll
            for (int a = 0; a < SH_MAX_AGGS; a++) {
                if (a >= ap.n) break;
                u64 fv = f[0];
#pragma unroll
                for (int j = 1; j < SH_MAX_AGGS; j++) if (ap.field[a] == j) fv = f[j];
                sval[(size_t)head * ap.n + a] = agg_out(ap, a, c, fv);  // (one record per row: see k_sc_keys)
            }
            if (ghead) slast[head] = m;
        }
    }
}

// rows in output order (heads of the new entries, scanned): ts / representative event of the group's
// last event, the key of its slot, the values
__global__ __launch_bounds__(kBlock) void k_sc_emit(i64 M, i64 n_old, const u32* __restrict__ ghead,
                                                   const u32* __restrict__ pre, const u32* __restrict__ slast,
                                                   const u64* __restrict__ sval, const u32* __restrict__ pend_pos,
                                                   const i64* __restrict__ pend_ts, const u64* __restrict__ pend_gidx,
                                                   const i64* __restrict__ chunk, const i64* __restrict__ send,
                                                   KeyTable kt, KeyPlan kp, int na, i64 T, i64* out_ts, i64* out_keys,
                                                   u64* out_vals, i64* out_rep, i64* out_chunk, i64* out_send,
                                                   i64* out_order) {
    const i64 m = n_old + (i64)blockIdx.x * kBlock + threadIdx.x;
    if (m >= M || (ghead && !ghead[m])) return;
    // (ghead null: every new entry is its own chunk — per-event sends — so row o is entry m itself)
    const i64 o = ghead ? (i64)pre[m - n_old] : m - n_old;
    const u32 l = ghead ? slast[m] : (u32)m;
    out_ts[o] = pend_ts[l];
    out_rep[o] = (i64)pend_gidx[l];
    i64 kv[kKeyParts] = {0, 0};
    unpack_key(kp, slot_key(kt, pend_pos[m]), kv, 1);
    for (int k = 0; k < kp.n; k++) out_keys[(size_t)k * T + o] = kv[k];
    for (int a = 0; a < na; a++) out_vals[(size_t)a * T + o] = sval[(size_t)m * na + a];
    if (out_chunk) out_chunk[o] = chunk[m];  // (null: every row its own chunk and flush)
    out_send[o] = send[m];
    if (out_order) out_order[o] = (i64)pend_gidx[m];  // (the group's first event in the chunk: merge order)
}

// the last timestamp of every send of the push (the send's playback clock before the prefix max)
__global__ __launch_bounds__(kBlock) void k_sc_send_last(const i64* __restrict__ ts, i64 N, i64 send_size, i64 n_sends,
                                                        i64* out) {
    const i64 s = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (s >= n_sends) return;
    const i64 e = send_size > 0 ? min((s + 1) * send_size, N) - 1 : N - 1;
    out[s] = ts[e];
}

static inline unsigned sc_grid(i64 n) { return (unsigned)((n + kBlock - 1) / kBlock); }

void launch_sc_keys(hipStream_t s, i64 M, i64 n_old, const i64* pcb, int nb, const u32* pend_pos, const u64* pend_gidx,
                    int per_event, i64 send_size, i64 seq0, u64* skey, u32* idx, i64* chunk, i64* send,
                    int by_entry) {
    if (M <= 0) return;
    hipLaunchKernelGGL(k_sc_keys, dim3(sc_grid(M)), dim3(kBlock), 0, s, M, n_old, pcb, nb, pend_pos, pend_gidx, per_event,
                       send_size, seq0, skey, idx, chunk, send, by_entry);
}

void launch_sc_walk(hipStream_t s, i64 M, const u32* hd, const u32* pos, const u32* starts, const u32* idx,
                    const i64* chunk, const u64* pend_vals, i64 pend_cap, AggPlan ap, i64 n_old, u32* ghead, u64* sval,
                    u32* slast) {
    if (M <= 0) return;
    hipLaunchKernelGGL(k_sc_walk, dim3(sc_grid(M)), dim3(kBlock), 0, s, M, hd, pos, starts, idx, chunk, pend_vals,
                       pend_cap, ap, n_old, ghead, sval, slast);
}

void launch_sc_emit(hipStream_t s, i64 M, i64 n_old, const u32* ghead, const u32* pre, const u32* slast, const u64* sval,
                    const u32* pend_pos, const i64* pend_ts, const u64* pend_gidx, const i64* chunk, const i64* send,
                    KeyTable kt, KeyPlan kp, int na, i64 T, i64* out_ts, i64* out_keys, u64* out_vals, i64* out_rep,
                    i64* out_chunk, i64* out_send, i64* out_order) {
    if (M <= n_old || T <= 0) return;
    hipLaunchKernelGGL(k_sc_emit, dim3(sc_grid(M - n_old)), dim3(kBlock), 0, s, M, n_old, ghead, pre, slast, sval,
                       pend_pos, pend_ts, pend_gidx, chunk, send, kt, kp, na, T, out_ts, out_keys, out_vals, out_rep,
                       out_chunk, out_send, out_order);
}

void launch_sc_send_last(hipStream_t s, const i64* ts, i64 N, i64 send_size, i64 n_sends, i64* out) {
    if (n_sends <= 0) return;
    hipLaunchKernelGGL(k_sc_send_last, dim3(sc_grid(n_sends)), dim3(kBlock), 0, s, ts, N, send_size, n_sends, out);
}


// ---- lengthBatch(L, true) with expired / all-events output: the event that starts batch w + 1 (the
// reference's count == length + 1, :249-266) carries batch w's events as EXPIRED before the RESET; the
// selector groups that chunk by key, so batch w's keys show their empty state (count 0, the others
// null) at their first-occurrence position, each with ts = the chunk's clock and the representative
// event of the key's last event in w; with `all events` the new event's own row replaces its key's
// expired row (LinkedHashMap.put) or follows them.
__device__ __forceinline__ i64 sc_wstart(i64 w, i64 n_old, const i64* pcb) { return w == 0 ? 0 : n_old + pcb[w - 1]; }

// fe[m] = 1 at the first entry (stream order) of every (window, key) run; lastidx[first] = its last entry
__global__ __launch_bounds__(kBlock) void k_scx_first(i64 M, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                     const u32* __restrict__ starts, const u32* __restrict__ idx,
                                                     u32* fe, u32* fpre, u32* lastidx) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i > M) return;
    if (i == M) { fpre[M] = 0; return; }
    u32 f = 0;
    if (hd[i]) {
        const u32 m = idx[i];
        fe[m] = 1;
        lastidx[m] = idx[starts[pos[i] + 1] - 1];
    }
    (void)f;
}

// rows of every new entry's chunk and, at batch starts, the new event's key rank in the closing batch
__global__ __launch_bounds__(kBlock) void k_scx_count(i64 M, i64 n_old, const i64* __restrict__ pcb,
                                                     const u64* __restrict__ skey, const u64* __restrict__ skey2,
                                                     const u32* __restrict__ idx2, const u32* __restrict__ fpre,
                                                     int cur_on, int exp_on, u32* rows, i64* rank_e) {
    const i64 j = (i64)blockIdx.x * kBlock + threadIdx.x;
    const i64 m = n_old + j;
    if (m > M) return;
    if (m == M) { rows[j] = 0; return; }
    const u64 key = skey[m];
    const i64 w = (i64)(key >> 32);
    i64 re = -1;
    u32 r = cur_on ? 1u : 0u;
    if (w >= 1 && m == sc_wstart(w, n_old, pcb)) {
        const i64 ws0 = sc_wstart(w - 1, n_old, pcb);
        const i64 nprev = (i64)fpre[m] - (i64)fpre[ws0];
        // the new event's key among batch w - 1's keys: lower bound of (w - 1, slot) in the sorted keys
        const u64 want = ((u64)(w - 1) << 32) | (key & 0xFFFFFFFFull);
        i64 lo = 0, hi = M;
        while (lo < hi) {
            const i64 mid = (lo + hi) >> 1;
            if (skey2[mid] < want) lo = mid + 1; else hi = mid;
        }
        if (lo < M && skey2[lo] == want) re = (i64)fpre[idx2[lo]] - (i64)fpre[ws0];
        if (exp_on) r = (u32)nprev + ((cur_on && re < 0) ? 1u : 0u);
    }
    rows[j] = r;
    rank_e[j] = re;
}

// the expired rows: one per (batch, key) run whose batch closes in this push
__global__ __launch_bounds__(kBlock) void k_scx_expired(i64 M, i64 n_old, const i64* __restrict__ pcb, int nb,
                                                       const u64* __restrict__ skey, const u32* __restrict__ fe,
                                                       const u32* __restrict__ fpre, const u32* __restrict__ lastidx,
                                                       const u32* __restrict__ base, const i64* __restrict__ rank_e,
                                                       const i64* __restrict__ send, const i64* __restrict__ send_clock,
                                                       const i64* __restrict__ bclk,
                                                       const u64* __restrict__ pend_gidx, KeyTable kt, KeyPlan kp,
                                                       AggPlan ap, int cur_on, int tb, i64 T, i64* out_ts, i64* out_keys,
                                                       u64* out_vals, unsigned char* out_nulls, unsigned char* out_exp,
                                                       i64* out_rep, i64* out_chunk, i64* out_send) {
    const i64 m = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (m >= M || !fe[m]) return;
    const u64 key = skey[m];
    const i64 w = (i64)(key >> 32);
    if (w >= nb) return;  // batch w has not closed yet
    const i64 mb = n_old + pcb[w];  // the event starting batch w + 1
    const i64 jb = mb - n_old;
    const i64 rank = (i64)fpre[m] - (i64)fpre[sc_wstart(w, n_old, pcb)];
    if (cur_on && rank == rank_e[jb]) return;  // the new event's current row takes this position
    const i64 o = base[jb] + rank;
    out_ts[o] = tb ? bclk[w] : send_clock[send[mb]];  // (timeBatch: mb may be past the push's entries)
    out_rep[o] = (i64)pend_gidx[lastidx[m]];
    i64 kv[kKeyParts] = {0, 0};
    unpack_key(kp, slot_key(kt, (u32)key), kv, 1);
    for (int k = 0; k < kp.n; k++) out_keys[(size_t)k * T + o] = kv[k];
    for (int a = 0; a < ap.n; a++) {
        out_vals[(size_t)a * T + o] = 0;
        out_nulls[(size_t)a * T + o] = ap.kind[a] == AK_COUNT ? 0 : 1;
    }
    out_exp[o] = 1;
    out_chunk[o] = tb ? -(w + 1) : jb;  // timeBatch: the closing TIMER chunk precedes the send's own
    out_send[o] = tb ? -(w + 1) : send[mb];
}

// the current rows (per-event chunks): at a batch start after the batch's expired rows, or in place
// of the key's expired row
__global__ __launch_bounds__(kBlock) void k_scx_current(i64 M, i64 n_old, const i64* __restrict__ pcb,
                                                       const u64* __restrict__ skey, const u32* __restrict__ fpre,
                                                       const u32* __restrict__ base, const i64* __restrict__ rank_e,
                                                       const u64* __restrict__ sval, const i64* __restrict__ send,
                                                       const i64* __restrict__ pend_ts, const u64* __restrict__ pend_gidx,
                                                       KeyTable kt, KeyPlan kp, int na, int exp_on, i64 T, i64* out_ts,
                                                       i64* out_keys, u64* out_vals, unsigned char* out_nulls,
                                                       unsigned char* out_exp, i64* out_rep, i64* out_chunk,
                                                       i64* out_send) {
    const i64 j = (i64)blockIdx.x * kBlock + threadIdx.x;
    const i64 m = n_old + j;
    if (m >= M) return;
    const u64 key = skey[m];
    const i64 w = (i64)(key >> 32);
    i64 o = base[j];
    if (exp_on && w >= 1 && m == sc_wstart(w, n_old, pcb)) {
        const i64 nprev = (i64)fpre[m] - (i64)fpre[sc_wstart(w - 1, n_old, pcb)];
        o += rank_e[j] >= 0 ? rank_e[j] : nprev;
    }
    out_ts[o] = pend_ts[m];
    out_rep[o] = (i64)pend_gidx[m];
    i64 kv[kKeyParts] = {0, 0};
    unpack_key(kp, slot_key(kt, (u32)key), kv, 1);
    for (int k = 0; k < kp.n; k++) out_keys[(size_t)k * T + o] = kv[k];
    for (int a = 0; a < na; a++) {
        out_vals[(size_t)a * T + o] = sval[(size_t)m * na + a];
        out_nulls[(size_t)a * T + o] = 0;
    }
    out_exp[o] = 0;
    out_chunk[o] = j;
    out_send[o] = send[m];
}

void launch_scx_first(hipStream_t s, i64 M, const u32* hd, const u32* pos, const u32* starts, const u32* idx, u32* fe,
                      u32* fpre, u32* lastidx) {
    hipLaunchKernelGGL(k_scx_first, dim3(sc_grid(M + 1)), dim3(kBlock), 0, s, M, hd, pos, starts, idx, fe, fpre,
                       lastidx);
}

void launch_scx_count(hipStream_t s, i64 M, i64 n_old, const i64* pcb, const u64* skey, const u64* skey2,
                      const u32* idx2, const u32* fpre, int cur_on, int exp_on, u32* rows, i64* rank_e) {
    hipLaunchKernelGGL(k_scx_count, dim3(sc_grid(M - n_old + 1)), dim3(kBlock), 0, s, M, n_old, pcb, skey, skey2, idx2,
                       fpre, cur_on, exp_on, rows, rank_e);
}

void launch_scx_rows(hipStream_t s, i64 M, i64 n_old, const i64* pcb, int nb, const u64* skey, const u32* fe,
                     const u32* fpre, const u32* lastidx, const u32* base, const i64* rank_e, const u64* sval,
                     const i64* send, const i64* send_clock, const i64* pend_ts, const u64* pend_gidx, KeyTable kt,
                     KeyPlan kp, AggPlan ap, int cur_on, int exp_on, i64 T, i64* out_ts, i64* out_keys, u64* out_vals,
                     unsigned char* out_nulls, unsigned char* out_exp, i64* out_rep, i64* out_chunk, i64* out_send) {
    if (T <= 0) return;
    if (exp_on)
        hipLaunchKernelGGL(k_scx_expired, dim3(sc_grid(M)), dim3(kBlock), 0, s, M, n_old, pcb, nb, skey, fe, fpre,
                           lastidx, base, rank_e, send, send_clock, (const i64*)nullptr, pend_gidx, kt, kp, ap, cur_on, 0, T, out_ts,
                           out_keys, out_vals, out_nulls, out_exp, out_rep, out_chunk, out_send);
    if (cur_on && M > n_old)
        hipLaunchKernelGGL(k_scx_current, dim3(sc_grid(M - n_old)), dim3(kBlock), 0, s, M, n_old, pcb, skey, fpre, base,
                           rank_e, sval, send, pend_ts, pend_gidx, kt, kp, ap.n, exp_on, T, out_ts, out_keys, out_vals,
                           out_nulls, out_exp, out_rep, out_chunk, out_send);
}

// ---- timeBatch(T, true) with expired / all-events output: a window closes in the scheduler's TIMER
// chunk, which runs before the crossing send's own chunk (Scheduler.onTimeChange at the send's
// set_clock): its keys' EXPIRED rows (empty state) form a flush of their own, in the window's
// first-occurrence order, followed by the send's CURRENT rows (one per (send, key) group) ----------
// keys of the window that closes right before entry m (m == M: after the push's last entry), if
// entry m - 1's window closes in this push (w < nb) and entry m starts a later window (or there is none)
__device__ __forceinline__ i64 sc_closing_keys(i64 m, i64 M, i64 n_old, const i64* pcb, int nb, const u64* skey,
                                               const u32* fpre) {
    if (m < 1) return 0;
    const i64 wp = (i64)(skey[m - 1] >> 32);
    if (wp >= nb) return 0;
    if (m < M && (i64)(skey[m] >> 32) <= wp) return 0;
    return (i64)fpre[m] - (i64)fpre[sc_wstart(wp, n_old, pcb)];
}

__global__ __launch_bounds__(kBlock) void k_scxt_count(i64 M, i64 n_old, const i64* __restrict__ pcb, int nb,
                                                      const u64* __restrict__ skey, const u32* __restrict__ fpre,
                                                      const u32* __restrict__ ghead, int cur_on, u32* rows) {
    const i64 j = (i64)blockIdx.x * kBlock + threadIdx.x;
    const i64 m = n_old + j;
    if (m > M + 1) return;
    if (m == M + 1) { rows[j] = 0; return; }  // (rows[nn] counts windows closing after the last entry)
    u32 r = (m < M && cur_on && ghead[m]) ? 1u : 0u;
    r += (u32)sc_closing_keys(m, M, n_old, pcb, nb, skey, fpre);
    rows[j] = r;
}

__global__ __launch_bounds__(kBlock) void k_scxt_current(i64 M, i64 n_old, const i64* __restrict__ pcb, int nb,
                                                        const u64* __restrict__ skey, const u32* __restrict__ fpre,
                                                        const u32* __restrict__ ghead, const u32* __restrict__ base,
                                                        const u32* __restrict__ slast, const u64* __restrict__ sval,
                                                        const i64* __restrict__ chunk, const i64* __restrict__ send,
                                                        const i64* __restrict__ pend_ts, const u64* __restrict__ pend_gidx,
                                                        KeyTable kt, KeyPlan kp, int na, i64 T, i64* out_ts,
                                                        i64* out_keys, u64* out_vals, unsigned char* out_nulls,
                                                        unsigned char* out_exp, i64* out_rep, i64* out_chunk,
                                                        i64* out_send) {
    const i64 j = (i64)blockIdx.x * kBlock + threadIdx.x;
    const i64 m = n_old + j;
    if (m >= M || !ghead[m]) return;
    const u64 key = skey[m];
    const i64 o = base[j] + sc_closing_keys(m, M, n_old, pcb, nb, skey, fpre);
    const u32 l = slast[m];
    out_ts[o] = pend_ts[l];
    out_rep[o] = (i64)pend_gidx[l];
    i64 kv[kKeyParts] = {0, 0};
    unpack_key(kp, slot_key(kt, (u32)key), kv, 1);
    for (int k = 0; k < kp.n; k++) out_keys[(size_t)k * T + o] = kv[k];
    for (int a = 0; a < na; a++) {
        out_vals[(size_t)a * T + o] = sval[(size_t)m * na + a];
        out_nulls[(size_t)a * T + o] = 0;
    }
    out_exp[o] = 0;
    out_chunk[o] = chunk[m];
    out_send[o] = send[m];
}

// the open window closed by a TIMER without events (sh_advance_time): its keys' EXPIRED rows
__global__ __launch_bounds__(kBlock) void k_scx_pending_rows(i64 M, const u32* __restrict__ fe,
                                                            const u32* __restrict__ fpre, const u32* __restrict__ lastidx,
                                                            const u32* __restrict__ pend_pos,
                                                            const u64* __restrict__ pend_gidx, KeyTable kt, KeyPlan kp,
                                                            AggPlan ap, i64 now, i64 T, i64* out_ts, i64* out_keys,
                                                            u64* out_vals, unsigned char* out_nulls,
                                                            unsigned char* out_exp, i64* out_rep) {
    const i64 m = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (m >= M || !fe[m]) return;
    const i64 o = fpre[m];
    out_ts[o] = now;
    out_rep[o] = (i64)pend_gidx[lastidx[m]];
    i64 kv[kKeyParts] = {0, 0};
    unpack_key(kp, slot_key(kt, pend_pos[m]), kv, 1);
    for (int k = 0; k < kp.n; k++) out_keys[(size_t)k * T + o] = kv[k];
    for (int a = 0; a < ap.n; a++) {
        out_vals[(size_t)a * T + o] = 0;
        out_nulls[(size_t)a * T + o] = ap.kind[a] == AK_COUNT ? 0 : 1;
    }
    out_exp[o] = 1;
}

void launch_scxt_count(hipStream_t s, i64 M, i64 n_old, const i64* pcb, int nb, const u64* skey, const u32* fpre,
                       const u32* ghead, int cur_on, u32* rows) {
    hipLaunchKernelGGL(k_scxt_count, dim3(sc_grid(M - n_old + 2)), dim3(kBlock), 0, s, M, n_old, pcb, nb, skey, fpre,
                       ghead, cur_on, rows);
}

void launch_scxt_rows(hipStream_t s, i64 M, i64 n_old, const i64* pcb, int nb, const u64* skey, const u32* fe,
                      const u32* fpre, const u32* lastidx, const u32* ghead, const u32* base, const u32* slast,
                      const u64* sval, const i64* chunk, const i64* send, const i64* bclk, const i64* pend_ts,
                      const u64* pend_gidx, KeyTable kt, KeyPlan kp, AggPlan ap, int cur_on, i64 T, i64* out_ts,
                      i64* out_keys, u64* out_vals, unsigned char* out_nulls, unsigned char* out_exp, i64* out_rep,
                      i64* out_chunk, i64* out_send) {
    if (T <= 0) return;
    hipLaunchKernelGGL(k_scx_expired, dim3(sc_grid(M)), dim3(kBlock), 0, s, M, n_old, pcb, nb, skey, fe, fpre, lastidx,
                       base, (const i64*)nullptr, send, (const i64*)nullptr, bclk, pend_gidx, kt, kp, ap, 0, 1, T,
                       out_ts, out_keys, out_vals, out_nulls, out_exp, out_rep, out_chunk, out_send);
    if (cur_on && M > n_old)
        hipLaunchKernelGGL(k_scxt_current, dim3(sc_grid(M - n_old)), dim3(kBlock), 0, s, M, n_old, pcb, nb, skey, fpre,
                           ghead, base, slast, sval, chunk, send, pend_ts, pend_gidx, kt, kp, ap.n, T, out_ts, out_keys,
                           out_vals, out_nulls, out_exp, out_rep, out_chunk, out_send);
}

void launch_scx_pending_rows(hipStream_t s, i64 M, const u32* fe, const u32* fpre, const u32* lastidx,
                             const u32* pend_pos, const u64* pend_gidx, KeyTable kt, KeyPlan kp, AggPlan ap, i64 now,
                             i64 T, i64* out_ts, i64* out_keys, u64* out_vals, unsigned char* out_nulls,
                             unsigned char* out_exp, i64* out_rep) {
    if (T <= 0) return;
    hipLaunchKernelGGL(k_scx_pending_rows, dim3(sc_grid(M)), dim3(kBlock), 0, s, M, fe, fpre, lastidx, pend_pos,
                       pend_gidx, kt, kp, ap, now, T, out_ts, out_keys, out_vals, out_nulls, out_exp, out_rep);
}
}  // namespace shd

namespace shd {

// ================================================================================================
// Small pushes (send(Event[n]) with n <= kSmallMax): the common case closes no window — the events
// only join the open window's queue (LengthBatch currentEventQueue / TimeBatch queue). One workgroup
// does what k_boundaries + k_compact_pending do for it: the filter, the key slots, the window test
// (timeBatch: the push's last send clock still below nextEmitTime, timestamps non-decreasing;
// lengthBatch: the queue stays below L) and the append, then reports to pinned host memory, so the
// host learns the outcome without a stream synchronisation. Any push that closes a window (or has
// decreasing timestamps) appends nothing and reports `fallback`: the full pipeline runs it.
// ================================================================================================
template <int FK>
__global__ __launch_bounds__(kSmallT) void k_small_push(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                       WinParams wp, KeyPlan kp, KeyTable kt, AggPlan ap,
                                                       u32* pend_pos, i64* pend_ts, u64* pend_vals, i64 pend_cap,
                                                       u64* pend_gidx, i64 seq_base, SmallRes* res, u64 token,
                                                       int force) {
    const int t = threadIdx.x;
    const i64 base = (i64)t * kItems;
    bool pass[kItems];
    filter_items<FK>(f, cols, base, wp.N, pass);
    u32 pos[kItems];
    {
        u64 key[kItems];
#pragma unroll
        for (int i = 0; i < kItems; i++) key[i] = pass[i] ? make_key(kp, cols, base + i) : 0;
        key_slots<kItems>(kt, key, pass, pos);
    }
    i64 tv[kItems];
    load_items_i64(ts, base, wp.N, tv, INT64_MAX);
    bool down = false;
    i64 cnt = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        cnt += pass[i];
        if (i + 1 < kItems) down |= base + i + 1 < wp.N && tv[i + 1] < tv[i];
    }
    if (base + kItems < wp.N) down |= ts[base + kItems] < tv[kItems - 1];
    i64 tot;
    i64 pre = block_excl_scan_any(cnt, &tot);
    const bool any_down = __syncthreads_or(down);
    bool fallback = any_down;
    if (wp.kind == SH_WIN_LENGTH_BATCH) {
        fallback |= wp.n_pend + tot >= wp.L;
    } else {
        // sorted: the last send's clock is the push's largest; its window must still be the open one
        const i64 clk = max(wp.clock_valid ? wp.clock0 : INT64_MIN, ts[wp.N - 1]);
        fallback |= wfun(wp, wp.E0, wp.e0_valid, 0, clk) > wp.W_open;
    }
    if (force) fallback = false;
    if (!fallback) {
#pragma unroll
        for (int i = 0; i < kItems; i++) {
            if (!pass[i]) continue;
            const i64 e = base + i, d = wp.n_pend + pre;
            pend_pos[d] = pos[i];
            pend_ts[d] = tv[i];
            for (int j = 0; j < ap.n_vcols; j++) pend_vals[(size_t)j * pend_cap + d] = (u64)load_raw(cols, ap.vcol_src[j], e);
            pend_gidx[d] = (u64)(seq_base + e);
            pre++;
        }
    }
    __syncthreads();
    if (t == 0) {
        __threadfence();
        SmallRes r;
        r.total_pass = tot;
        r.max_tl = ts[wp.N - 1];
        r.fallback = fallback ? 1 : 0;
        r.pad = 0;
        const volatile u32* c = (const volatile u32*)kt.n_keys;  // the key table's control words
        for (int i = 0; i < 4; i++) r.ctrl[i] = c[i];
        res->total_pass = r.total_pass;
        res->max_tl = r.max_tl;
        res->fallback = r.fallback;
        for (int i = 0; i < 4; i++) res->ctrl[i] = r.ctrl[i];
        __threadfence_system();
        ((volatile u64*)&res->token)[0] = token;
        __threadfence_system();
    }
}

void launch_small_push(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp, KeyPlan kp, KeyTable kt,
                       AggPlan ap, u32* pend_pos, i64* pend_ts, u64* pend_vals, i64 pend_cap, u64* pend_gidx,
                       i64 seq_base, SmallRes* res, u64 token, bool force) {
    const int fo = force ? 1 : 0;
    switch (filter_kind(f)) {
        case 0: hipLaunchKernelGGL(k_small_push<0>, dim3(1), dim3(kSmallT), 0, s, ts, cols, f, wp, kp, kt, ap, pend_pos, pend_ts, pend_vals, pend_cap, pend_gidx, seq_base, res, token, fo); break;
        case 1: hipLaunchKernelGGL(k_small_push<1>, dim3(1), dim3(kSmallT), 0, s, ts, cols, f, wp, kp, kt, ap, pend_pos, pend_ts, pend_vals, pend_cap, pend_gidx, seq_base, res, token, fo); break;
        default: hipLaunchKernelGGL(k_small_push<2>, dim3(1), dim3(kSmallT), 0, s, ts, cols, f, wp, kp, kt, ap, pend_pos, pend_ts, pend_vals, pend_cap, pend_gidx, seq_base, res, token, fo);
    }
}

// ---- stream.current.event flushes on the device: a flush ends where the row's chunk changes; its
// clock is its send's playback clock (the running max of the sends' last timestamps, with the clock
// carried in) or, for a TIMER chunk (osd < 0), its window start's clock ---------------------------------
__global__ __launch_bounds__(kBlock) void k_sc_flush_flags(i64 T, const i64* __restrict__ och, u32* flag) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i > T) return;
    flag[i] = i < T && (i + 1 == T || och[i + 1] != och[i]) ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void k_sc_flushes(i64 T, const i64* __restrict__ osd, const u32* __restrict__ pre,
                                                      const i64* __restrict__ slp, int cv0, i64 clock0,
                                                      const i64* __restrict__ bclk, i64* fo1, i64* fc) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= T || (pre && pre[i + 1] == pre[i])) return;
    const u32 k = pre ? pre[i] : (u32)i;  // (pre null: every row ends its own flush)
    const i64 sd = osd[i];
    fo1[k] = i + 1;
    fc[k] = sd >= 0 ? (cv0 ? max(clock0, slp[sd]) : slp[sd]) : bclk[-sd - 1];
}

void launch_sc_flush_flags(hipStream_t s, i64 T, const i64* och, u32* flag) {
    hipLaunchKernelGGL(k_sc_flush_flags, dim3((unsigned)((T + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, T, och, flag);
}

void launch_sc_flushes(hipStream_t s, i64 T, const i64* osd, const u32* pre, const i64* slp, int cv0, i64 clock0,
                       const i64* bclk, i64* fo1, i64* fc) {
    if (T <= 0) return;
    hipLaunchKernelGGL(k_sc_flushes, dim3((unsigned)((T + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, T, osd, pre, slp,
                       cv0, clock0, bclk, fo1, fc);
}

// compact flushes (sh_query_set_compact_flushes): ok[0] stays 1 iff every flush's clock equals its one
// row's timestamp (the caller has checked one row per flush); plain stores of one value, no atomics
__global__ __launch_bounds__(kBlock) void k_flush_clock_is_ts(i64 n, const i64* __restrict__ fc,
                                                             const i64* __restrict__ ts, u32* ok) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i < n && fc[i] != ts[i]) ok[0] = 0u;
}

// the same for stream.current rows that are their own flushes, the clocks taken from the sends' clocks
__global__ __launch_bounds__(kBlock) void k_sc_clock_is_ts(i64 n, const i64* __restrict__ osd, const i64* __restrict__ slp,
                                                          int cv0, i64 clock0, const i64* __restrict__ ts, u32* ok) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const i64 c = cv0 ? max(clock0, slp[osd[i]]) : slp[osd[i]];
    if (c != ts[i]) ok[0] = 0u;
}

void launch_sc_clock_is_ts(hipStream_t s, i64 n, const i64* osd, const i64* slp, int cv0, i64 clock0, const i64* ts,
                           u32* ok) {
    (void)hipMemsetD32Async((hipDeviceptr_t)ok, 1, 1, s);
    if (n > 0)
        hipLaunchKernelGGL(k_sc_clock_is_ts, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, osd, slp,
                           cv0, clock0, ts, ok);
}

void launch_flush_clock_is_ts(hipStream_t s, i64 n, const i64* fc, const i64* ts, u32* ok) {
    (void)hipMemsetD32Async((hipDeviceptr_t)ok, 1, 1, s);
    if (n > 0)
        hipLaunchKernelGGL(k_flush_clock_is_ts, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, fc,
                           ts, ok);
}

// ---- externalTimeBatch timeout: where the push's clock passes lastScheduledTime --------------------
// First send whose last event's timestamp reaches L (InputHandler.send sets the clock from it, and
// every earlier send's clock stays below L): out[0] = its index (u64 max: none).
__global__ __launch_bounds__(kBlock) void k_xt_first_send(const i64* __restrict__ ts, i64 N, i64 send_size, i64 L,
                                                          unsigned long long* out) {
    const i64 n_sends = send_size > 0 ? (N + send_size - 1) / send_size : 1;
    i64 first = INT64_MAX;  // this thread's first qualifying send (j grows along the stride)
    for (i64 j = (i64)blockIdx.x * kBlock + threadIdx.x; j < n_sends; j += (i64)gridDim.x * kBlock) {
        const i64 last = send_size > 0 ? min((j + 1) * send_size, N) - 1 : N - 1;
        if (ts[last] >= L) { first = j; break; }
    }
    // one atomic per block (per send, every send past the crossing queued on one address)
    first = block_reduce(first, MinOp(), INT64_MAX);
    if (threadIdx.x == 0 && first != INT64_MAX) atomicMin(out, (unsigned long long)first);
}

// passing events of the push in [0, hi): the open batch's events before a timeout's send, and (xcol >=
// 0) the largest timestamp attribute among them — lastCurrentEventTime at the timeout (the expired rows'
// stamp, flushToOutputChunk :341-348)
__global__ __launch_bounds__(kBlock) void k_xt_count_pass(ColSet cols, FilterProg f, i64 hi, unsigned long long* out,
                                                          int xcol, long long* xmax) {
    i64 c = 0, m = INT64_MIN;
    for (i64 e = (i64)blockIdx.x * kBlock + threadIdx.x; e < hi; e += (i64)gridDim.x * kBlock)
        if (eval_filter(f, cols, e)) {
            c++;
            if (xcol >= 0) m = max(m, load_raw(cols, xcol, e));
        }
    c = block_reduce(c, [](i64 a, i64 b) { return a + b; }, 0);
    if (threadIdx.x == 0 && c) atomicAdd(out, (unsigned long long)c);
    if (xcol >= 0) {
        m = block_reduce(m, MaxOp(), INT64_MIN);
        if (threadIdx.x == 0 && m != INT64_MIN) atomicMax(xmax, (long long)m);
    }
}

void launch_xt_first_send(hipStream_t s, const i64* ts, i64 N, i64 send_size, i64 L, unsigned long long* out) {
    const i64 n_sends = send_size > 0 ? (N + send_size - 1) / send_size : 1;
    const unsigned g = (unsigned)std::min<i64>((n_sends + kBlock - 1) / kBlock, 2048);
    hipLaunchKernelGGL(k_xt_first_send, dim3(std::max(1u, g)), dim3(kBlock), 0, s, ts, N, send_size, L, out);
}

void launch_xt_count_pass(hipStream_t s, ColSet cols, FilterProg f, i64 hi, unsigned long long* out, int xcol,
                          long long* xmax) {
    if (hi <= 0) return;
    const unsigned g = (unsigned)std::min<i64>((hi + kBlock - 1) / kBlock, 2048);
    hipLaunchKernelGGL(k_xt_count_pass, dim3(g), dim3(kBlock), 0, s, cols, f, hi, out, xcol, xmax);
}

}  // namespace shd
