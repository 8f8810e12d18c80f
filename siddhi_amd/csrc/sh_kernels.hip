// sh_kernels.hip — gfx950 kernels of the batch-window path (lengthBatch / timeBatch group-by).
//
// Pipeline of one push (DESIGN.md "Batch-window pipeline"):
//   k_blockagg      per-workgroup pass count + send clock maxima        (FilterProcessor, InputHandler clock)
//   k_scan_blocks   exclusive scans of those, nextEmitTime initialisation (TimeBatchWindowProcessor.process :266-276)
//   k_boundaries    window number per event, boundary list              (LengthBatch :206-243, TimeBatch :278-340, Scheduler)
//   k_ms_count/scatter  stable multisplit of closed-window events into key partitions (P > 1 only)
//   k_aggregate     ordered per-key aggregation of one (window, partition) in LDS (QuerySelector.processInBatchGroupBy :315-374)
//   k_count_flags + k_emit   rows in first-occurrence order                (LinkedHashMap insertion order)
//   k_compact_pending        events of the still-open window carried to the next push
#include "sh_device.h"

namespace shd {

// ================================================================================================
// k_blockagg: per workgroup (kTile events, blocked kItems per thread) the number of passing events,
// the max timestamp over send-last events and the first passing event.
// ================================================================================================
__global__ __launch_bounds__(kBlock) void k_blockagg(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                    WinParams wp, i64* blk_pass, i64* blk_tl, i64* blk_first) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 cnt = 0, tl = INT64_MIN, first = INT64_MAX;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        if (e < wp.N) {
            if (eval_filter(f, cols, e)) { cnt++; if (first == INT64_MAX) first = e; }
            if (is_send_last(wp, e)) tl = max(tl, ts[e]);
        }
    }
    i64 c = block_reduce(cnt, SumOp(), 0);
    i64 t = block_reduce(tl, MaxOp(), INT64_MIN);
    i64 fp = block_reduce(first, MinOp(), INT64_MAX);
    if (threadIdx.x == 0) { blk_pass[blockIdx.x] = c; blk_tl[blockIdx.x] = t; blk_first[blockIdx.x] = fp; }
}

void launch_blockagg(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, i64 N, i64 send_size,
                     i64* blk_pass, i64* blk_tl, i64* blk_first, int nblk) {
    WinParams wp{};
    wp.N = N;
    wp.send_size = send_size;
    hipLaunchKernelGGL(k_blockagg, dim3(nblk), dim3(kBlock), 0, s, ts, cols, f, wp, blk_pass, blk_tl, blk_first);
}

// ================================================================================================
// k_scan_blocks (one workgroup of 1024): exclusive prefix sum of pass counts, exclusive prefix max
// of send clocks, first passing event; initialises timeBatch's nextEmitTime on the first process()
// call: nextEmitTime = now + T, or getNextEmitTime(now) when start.time is given
// (TimeBatchWindowProcessor.java:266-276, 342-347).
// ================================================================================================
__global__ __launch_bounds__(1024) void k_scan_blocks(i64* blk_pass, i64* blk_tl, i64* blk_first, int nblk,
                                                     const i64* __restrict__ ts, WinParams wp, PushInfo* info) {
    __shared__ i64 sh_sum[1024], sh_max[1024], sh_min[1024];
    int t = threadIdx.x;
    int per = (nblk + 1023) / 1024;
    int lo = t * per, hi = min(nblk, lo + per);
    i64 s = 0, m = INT64_MIN, mn = INT64_MAX;
    for (int i = lo; i < hi; i++) { s += blk_pass[i]; m = max(m, blk_tl[i]); mn = min(mn, blk_first[i]); }
    sh_sum[t] = s; sh_max[t] = m; sh_min[t] = mn;
    __syncthreads();
    // Hillis-Steele inclusive scans over 1024 partials
    for (int d = 1; d < 1024; d <<= 1) {
        i64 a = t >= d ? sh_sum[t - d] : 0;
        i64 b = t >= d ? sh_max[t - d] : INT64_MIN;
        __syncthreads();
        sh_sum[t] += a;
        sh_max[t] = max(sh_max[t], b);
        __syncthreads();
    }
    for (int d = 512; d > 0; d >>= 1) {
        if (t < d) sh_min[t] = min(sh_min[t], sh_min[t + d]);
        __syncthreads();
    }
    i64 run_s = t > 0 ? sh_sum[t - 1] : 0;
    i64 run_m = t > 0 ? sh_max[t - 1] : INT64_MIN;
    for (int i = lo; i < hi; i++) {
        i64 c = blk_pass[i], x = blk_tl[i];
        blk_pass[i] = run_s; blk_tl[i] = run_m;
        run_s += c; run_m = max(run_m, x);
    }
    __syncthreads();
    if (t == 0) {
        info->total_pass = sh_sum[1023];
        info->max_tl = sh_max[1023];
        info->first_pass = sh_min[0];
        info->e0_valid = wp.e0_valid;
        info->E0 = wp.E0;
        info->n_bounds = 0;
        if (wp.kind == SH_WIN_TIME_BATCH && !wp.e0_valid && sh_min[0] != INT64_MAX) {
            // clock of the send that carries the first passing event
            i64 e0 = sh_min[0];
            i64 sl = wp.send_size > 0 ? wp.send_size : wp.N;
            i64 start = (e0 / sl) * sl;
            i64 last = min(wp.N - 1, start + sl - 1);
            int b0 = (int)(start / kTile);
            i64 pm = blk_tl[b0];  // now the exclusive prefix max of block b0
            for (i64 e = (i64)b0 * kTile; e < start; e++)
                if (is_send_last(wp, e)) pm = max(pm, ts[e]);
            i64 c = max(pm, ts[last]);
            if (wp.clock_valid) c = max(c, wp.clock0);
            i64 E0;
            if (wp.has_start) {
                i64 elapsed = (c - wp.start_time) % wp.T;  // Java % truncates like C++
                E0 = c + (wp.T - elapsed);
            } else {
                E0 = c + wp.T;
            }
            info->E0 = E0;
            info->e0_valid = 1;
        }
    }
}

void launch_scan_blocks(hipStream_t s, i64* blk_pass, i64* blk_tl, i64* blk_first, int nblk, const i64* ts,
                        WinParams wp, PushInfo* info) {
    hipLaunchKernelGGL(k_scan_blocks, dim3(1), dim3(1024), 0, s, blk_pass, blk_tl, blk_first, nblk, ts, wp, info);
}

// ================================================================================================
// k_boundaries: window number W(e) of every new event, and a boundary record wherever W rises.
//   lengthBatch: W = (n_pend + passing events before e) / L  (LengthBatchWindowProcessor :206-243:
//                a batch completes at its L-th event and is flushed as its own chunk);
//   timeBatch:   W = clock(e) < E0 ? 0 : (clock(e) - E0) / T + 1, clock(e) = the playback clock of
//                e's send. Due timers fire before the send is processed and catch up one period
//                each (Scheduler.sendTimerEvents :171-209), so the window boundaries sit at E0 + kT.
// ================================================================================================
__device__ __forceinline__ i64 wfun(const WinParams& wp, i64 E0, int e0_valid, i64 pcb, i64 clock) {
    if (wp.kind == SH_WIN_LENGTH_BATCH) return (wp.n_pend + pcb) / wp.L;
    if (!e0_valid) return wp.W_open;
    return clock < E0 ? 0 : (clock - E0) / wp.T + 1;
}

__global__ __launch_bounds__(kBlock) void k_boundaries(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                      WinParams wp, const i64* blk_pass_pre, const i64* blk_tl_pre,
                                                      const PushInfo* info, Bound* bounds, int max_bounds,
                                                      int* n_bounds) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    bool pass[kItems];
    i64 cnt = 0, tl = INT64_MIN;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        pass[i] = e < wp.N && eval_filter(f, cols, e);
        cnt += pass[i];
        if (e < wp.N && is_send_last(wp, e)) tl = max(tl, ts[e]);
    }
    i64 pcb = block_excl_scan(cnt, SumOp(), 0, nullptr) + blk_pass_pre[blockIdx.x];
    i64 pm = max(block_excl_scan(tl, MaxOp(), INT64_MIN, nullptr), blk_tl_pre[blockIdx.x]);
    const i64 c0 = wp.clock_valid ? wp.clock0 : INT64_MIN;
    const i64 E0 = info->E0;
    const int e0v = info->e0_valid;
    if (base >= wp.N) return;
    // previous event's window
    i64 Wprev, clock_prev;
    if (base == 0) {
        Wprev = wp.W_open;
        clock_prev = c0;
    } else {
        i64 ep = base - 1;
        bool pp = eval_filter(f, cols, ep);
        i64 pcb_prev = pcb - (pp ? 1 : 0);
        i64 sl = send_len(wp);
        if (ep / sl == base / sl) clock_prev = max(c0, max(pm, ts[send_last_of(wp, base)]));
        else clock_prev = max(c0, pm);
        Wprev = wfun(wp, E0, e0v, pcb_prev, clock_prev);
    }
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        if (e >= wp.N) break;
        i64 clk = max(c0, max(pm, ts[send_last_of(wp, e)]));
        i64 W = wfun(wp, E0, e0v, pcb, clk);
        if (W > Wprev) {
            int k = atomicAdd(n_bounds, 1);
            if (k < max_bounds) {
                Bound b;
                b.idx = wp.n_pend + e; b.W = W; b.clock = clk; b.clock_prev = clock_prev; b.pcb = pcb; b.pad = 0;
                bounds[k] = b;
            }
        }
        Wprev = W;
        clock_prev = clk;
        pcb += pass[i];
        if (is_send_last(wp, e)) pm = max(pm, ts[e]);
    }
}

void launch_boundaries(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp,
                       const i64* blk_pass_pre, const i64* blk_tl_pre, const PushInfo* info, Bound* bounds,
                       int max_bounds, int nblk) {
    hipLaunchKernelGGL(k_boundaries, dim3(nblk), dim3(kBlock), 0, s, ts, cols, f, wp, blk_pass_pre, blk_tl_pre,
                       info, bounds, max_bounds, (int*)&((PushInfo*)info)->n_bounds);
}

// ================================================================================================
// k_aggregate: one workgroup per (closed segment, key partition). Events are applied to the key's
// LDS state strictly in event order — each step takes 256 consecutive events; lanes that share a
// key resolve in rounds (the lowest lane of each key wins a round), so every per-key update runs
// in the order the reference's selector runs it (QuerySelector.processInBatchGroupBy :315-374).
// Double sums are therefore bit-identical to Java's sequential `sum += v`.
// State starts empty because each flush chunk begins with RESET (LengthBatch :222-226,
// TimeBatch :320-323; AttributeAggregatorExecutor.processReset :145-151).
// ================================================================================================
struct AggLds {
    u64* fields;  // [n_fields][NL]
    u32* cnt;
    u32* first;
    u32* last;
    u32* owner;
};

__device__ __forceinline__ void apply_event(const AggPlan& ap, AggLds& L, int NL, u32 li, u32 idx, const i64* v) {
    u32 c = L.cnt[li];
    if (c == 0) L.first[li] = idx;
    L.cnt[li] = c + 1;
    L.last[li] = idx;
    for (int a = 0; a < ap.n; a++) {
        int k = ap.kind[a];
        if (k == AK_COUNT) continue;
        u64* fp = L.fields + (size_t)ap.field[a] * NL + li;
        i64 x = v[ap.vcol[a]];
        switch (k) {
            case AK_SUM_L: *fp = (u64)((c == 0 ? 0 : (i64)*fp) + x); break;  // SumAttributeAggregatorExecutor long: sum += data
            case AK_SUM_D:                                                // double: sum += data
            case AK_AVG: {                                               // Avg*: value += (double) data
                double cur = c == 0 ? 0.0 : __longlong_as_double((i64)*fp);
                double xv = (k == AK_AVG && !(ap.vcol_type[ap.vcol[a]] == SH_T_FLOAT ||
                                              ap.vcol_type[ap.vcol[a]] == SH_T_DOUBLE))
                                ? (double)x : __longlong_as_double(x);
                *fp = (u64)__double_as_longlong(cur + xv);
                break;
            }
            case AK_MIN_L: if (c == 0 || (i64)*fp > x) *fp = (u64)x; break;  // minValue > value
            case AK_MAX_L: if (c == 0 || (i64)*fp < x) *fp = (u64)x; break;
            case AK_MIN_D: if (c == 0 || __longlong_as_double((i64)*fp) > __longlong_as_double(x)) *fp = (u64)x; break;
            case AK_MAX_D: if (c == 0 || __longlong_as_double((i64)*fp) < __longlong_as_double(x)) *fp = (u64)x; break;
            case AK_MIN_F: if (c == 0 || (float)__longlong_as_double((i64)*fp) > (float)__longlong_as_double(x)) *fp = (u64)x; break;
            case AK_MAX_F: if (c == 0 || (float)__longlong_as_double((i64)*fp) < (float)__longlong_as_double(x)) *fp = (u64)x; break;
        }
    }
}

template <bool PARTITIONED>
__global__ __launch_bounds__(kBlock) void k_aggregate(const Segment* __restrict__ segs, int P, int logP, int NL,
                                                     i64 n_pend, const u32* __restrict__ pend_pos,
                                                     const u64* __restrict__ pend_vals, i64 pend_cap,
                                                     const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                     KeyPlan kp, KeyTable kt, AggPlan ap, RowTmp* rows,
                                                     u64* row_vals, u32* row_counter, unsigned char* flags,
                                                     u32* rowref, i64* seg_rows, const u32* __restrict__ rec_pos,
                                                     const u32* __restrict__ rec_idx,
                                                     const u64* __restrict__ rec_vals, i64 rec_cap,
                                                     const i64* __restrict__ part_off) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    // static __shared__ of the scan helpers precede the dynamic region; realign it to 16 bytes
    unsigned char* smem = (unsigned char*)(((uintptr_t)smem_raw + 15) & ~(uintptr_t)15);
    AggLds L;
    L.fields = (u64*)smem;
    L.cnt = (u32*)(smem + (size_t)ap.n_fields * NL * 8);
    L.first = L.cnt + NL;
    L.last = L.first + NL;
    L.owner = L.last + NL;
    const int seg = blockIdx.x / P;
    const int p = blockIdx.x % P;
    for (int i = threadIdx.x; i < NL; i += kBlock) { L.cnt[i] = 0; L.owner[i] = 0; }
    __syncthreads();

    i64 lo = segs[seg].lo, hi = segs[seg].hi;
    if (PARTITIONED) {
        // binary search the partition's record list (sorted by combined index) for [lo, hi)
        i64 a0 = part_off[p], a1 = part_off[p + 1];
        i64 l = a0, r = a1;
        while (l < r) { i64 m = (l + r) >> 1; if ((i64)rec_idx[m] < lo) l = m + 1; else r = m; }
        i64 s0 = l;
        l = s0; r = a1;
        while (l < r) { i64 m = (l + r) >> 1; if ((i64)rec_idx[m] < hi) l = m + 1; else r = m; }
        lo = s0; hi = l;
    }
    u32 round = 0;
    for (i64 b = lo; b < hi; b += kBlock) {
        i64 e = b + threadIdx.x;
        bool pend = false;
        u32 li = 0, idx = 0;
        i64 v[SH_MAX_AGGS];
        if (e < hi) {
            if (PARTITIONED) {
                u32 pos = rec_pos[e];
                li = pos >> logP;
                idx = rec_idx[e];
                for (int j = 0; j < ap.n_vcols; j++) v[j] = (i64)rec_vals[(size_t)j * rec_cap + e];
                pend = true;
            } else if (e < n_pend) {
                li = pend_pos[e] >> logP;
                idx = (u32)e;
                for (int j = 0; j < ap.n_vcols; j++) v[j] = (i64)pend_vals[(size_t)j * pend_cap + e];
                pend = true;
            } else {
                i64 x = e - n_pend;
                if (eval_filter(f, cols, x)) {
                    u32 pos = key_slot(kt, make_key(kp, cols, x));
                    li = pos >> logP;
                    idx = (u32)e;
                    for (int j = 0; j < ap.n_vcols; j++) v[j] = load_raw(cols, ap.vcol_src[j], x);
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

    // emit one row per touched key
    int mine = 0;
    for (int i = threadIdx.x; i < NL; i += kBlock) mine += L.cnt[i] > 0;
    i64 tot;
    i64 pre = block_excl_scan((i64)mine, SumOp(), 0, &tot);
    __shared__ u32 base_row;
    if (threadIdx.x == 0) {
        base_row = tot ? atomicAdd(row_counter, (u32)tot) : 0;
        if (tot) atomicAdd((unsigned long long*)&seg_rows[seg], (unsigned long long)tot);
    }
    __syncthreads();
    u32 r = base_row + (u32)pre;
    for (int i = threadIdx.x; i < NL; i += kBlock) {
        u32 c = L.cnt[i];
        if (!c) continue;
        RowTmp t;
        t.pos = ((u32)i << logP) | (u32)p;
        t.first = L.first[i];
        t.last = L.last[i];
        t.pad = c;
        rows[r] = t;
        for (int a = 0; a < ap.n; a++) {
            u64 out;
            int k = ap.kind[a];
            if (k == AK_COUNT) out = (u64)(i64)c;
            else {
                u64 fv = L.fields[(size_t)ap.field[a] * NL + i];
                if (k == AK_AVG) out = (u64)__double_as_longlong(__longlong_as_double((i64)fv) / (double)(i64)c);
                else out = fv;
            }
            row_vals[(size_t)r * ap.n + a] = out;
        }
        flags[t.first] = 1;
        rowref[t.first] = r;
        r++;
    }
}

void launch_aggregate(hipStream_t s, const Segment* segs, int nseg, int P, int logP, int NL, i64 n_pend,
                      const u32* pend_pos, const u64* pend_vals, i64 pend_cap, const i64* ts, ColSet cols,
                      FilterProg f, KeyPlan kp, KeyTable kt, AggPlan ap, RowTmp* rows, u64* row_vals,
                      u32* row_counter, unsigned char* flags, u32* rowref, i64* seg_rows, const u32* rec_pos,
                      const u32* rec_idx, const u64* rec_vals, i64 rec_cap, const i64* part_off) {
    size_t lds = (size_t)NL * (8 * ap.n_fields + 16) + 16;
    dim3 grid(nseg * P);
    if (P > 1)
        hipLaunchKernelGGL(k_aggregate<true>, grid, dim3(kBlock), lds, s, segs, P, logP, NL, n_pend, pend_pos,
                           pend_vals, pend_cap, ts, cols, f, kp, kt, ap, rows, row_vals, row_counter, flags, rowref,
                           seg_rows, rec_pos, rec_idx, rec_vals, rec_cap, part_off);
    else
        hipLaunchKernelGGL(k_aggregate<false>, grid, dim3(kBlock), lds, s, segs, P, logP, NL, n_pend, pend_pos,
                           pend_vals, pend_cap, ts, cols, f, kp, kt, ap, rows, row_vals, row_counter, flags, rowref,
                           seg_rows, rec_pos, rec_idx, rec_vals, rec_cap, part_off);
}

// ================================================================================================
// Ordering: a row's position is the rank of its first-occurrence index among all first indices.
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
    __shared__ i64 sh[1024];
    int t = threadIdx.x;
    int per = (n + 1023) / 1024;
    int lo = t * per, hi = min(n, lo + per);
    i64 s = 0;
    for (int i = lo; i < hi; i++) s += a[i];
    sh[t] = s;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        i64 x = t >= d ? sh[t - d] : 0;
        __syncthreads();
        sh[t] += x;
        __syncthreads();
    }
    i64 run = t > 0 ? sh[t - 1] : 0;
    for (int i = lo; i < hi; i++) { i64 c = a[i]; a[i] = run; run += c; }
}

void launch_scan_sum(hipStream_t s, i64* a, int n) {
    hipLaunchKernelGGL(k_scan_sum, dim3(1), dim3(1024), 0, s, a, n);
}

__global__ __launch_bounds__(kBlock) void k_emit(const unsigned char* __restrict__ flags, const u32* __restrict__ rowref,
                                                i64 n, const i64* __restrict__ blk_pre, const RowTmp* __restrict__ rows,
                                                const u64* __restrict__ row_vals, int n_aggs, KeyTable kt, KeyPlan kp,
                                                i64 n_pend, const i64* __restrict__ pend_ts, const i64* __restrict__ ts,
                                                i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals,
                                                unsigned char* out_nulls) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    unsigned char fl[kItems];
    i64 c = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) { fl[i] = base + i < n ? flags[base + i] : 0; c += fl[i]; }
    i64 r = block_excl_scan(c, SumOp(), 0, nullptr) + blk_pre[blockIdx.x];
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        if (!fl[i]) continue;
        u32 row = rowref[base + i];
        RowTmp t = rows[row];
        out_ts[r] = t.last < n_pend ? pend_ts[t.last] : ts[t.last - n_pend];
        unpack_key(kp, slot_key(kt, t.pos), out_keys + r, out_cap);
        for (int a = 0; a < n_aggs; a++) {
            out_vals[(size_t)a * out_cap + r] = row_vals[(size_t)row * n_aggs + a];
            out_nulls[(size_t)a * out_cap + r] = 0;
        }
        r++;
    }
}

void launch_emit(hipStream_t s, const unsigned char* flags, const u32* rowref, i64 n, const i64* blk_pre, int nblk,
                 const RowTmp* rows, const u64* row_vals, int n_aggs, KeyTable kt, KeyPlan kp, i64 n_pend,
                 const i64* pend_ts, const i64* ts, i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals,
                 unsigned char* out_nulls) {
    hipLaunchKernelGGL(k_emit, dim3(nblk), dim3(kBlock), 0, s, flags, rowref, n, blk_pre, rows, row_vals, n_aggs,
                       kt, kp, n_pend, pend_ts, ts, out_cap, out_ts, out_keys, out_vals, out_nulls);
}

// ================================================================================================
// k_compact_pending: passing events of the open window [e_lo, N) appended to the pending buffer
// (the window's queued events, LengthBatch WindowState.currentEventQueue / TimeBatch queue).
// ================================================================================================
__global__ __launch_bounds__(kBlock) void k_compact_pending(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                           KeyPlan kp, KeyTable kt, AggPlan ap, i64 e_lo, i64 N,
                                                           i64 pcb_lo, i64 dst_base, const i64* blk_pass_pre,
                                                           int blk0, u32* pend_pos, i64* pend_ts, u64* pend_vals,
                                                           i64 pend_cap) {
    int blk = blk0 + blockIdx.x;
    i64 base = (i64)blk * kTile + (i64)threadIdx.x * kItems;
    bool pass[kItems];
    i64 cnt = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        pass[i] = e < N && eval_filter(f, cols, e);
        cnt += pass[i];
    }
    i64 pcb = block_excl_scan(cnt, SumOp(), 0, nullptr) + blk_pass_pre[blk];
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        if (pass[i]) {
            if (e >= e_lo) {
                i64 d = dst_base + (pcb - pcb_lo);
                pend_pos[d] = key_slot(kt, make_key(kp, cols, e));
                pend_ts[d] = ts[e];
                for (int j = 0; j < ap.n_vcols; j++) pend_vals[(size_t)j * pend_cap + d] = (u64)load_raw(cols, ap.vcol_src[j], e);
            }
            pcb++;
        }
    }
}

void launch_compact_pending(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, KeyPlan kp, KeyTable kt,
                            AggPlan ap, i64 e_lo, i64 N, i64 pcb_lo, i64 base, const i64* blk_pass_pre,
                            u32* pend_pos, i64* pend_ts, u64* pend_vals, i64 pend_cap) {
    if (e_lo >= N) return;
    int blk0 = (int)(e_lo / kTile);
    int blk1 = (int)((N + kTile - 1) / kTile);
    hipLaunchKernelGGL(k_compact_pending, dim3(blk1 - blk0), dim3(kBlock), 0, s, ts, cols, f, kp, kt, ap, e_lo, N,
                       pcb_lo, base, blk_pass_pre, blk0, pend_pos, pend_ts, pend_vals, pend_cap);
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

__device__ __forceinline__ EvLoad load_pos(i64 e, i64 n_pend, const u32* pend_pos, const ColSet& cols,
                                           const FilterProg& f, const KeyPlan& kp, const KeyTable& kt) {
    EvLoad r{false, 0};
    if (e < n_pend) { r.ok = true; r.pos = pend_pos[e]; return r; }
    i64 x = e - n_pend;
    if (eval_filter(f, cols, x)) { r.ok = true; r.pos = key_slot(kt, make_key(kp, cols, x)); }
    return r;
}

__global__ __launch_bounds__(kBlock) void k_ms_count(i64 lo, i64 hi, i64 n_pend, const u32* __restrict__ pend_pos,
                                                    ColSet cols, FilterProg f, KeyPlan kp, KeyTable kt, int P,
                                                    i64* counts, int nblk) {
    extern __shared__ __attribute__((aligned(16))) u32 hist[];
    for (int i = threadIdx.x; i < P; i += kBlock) hist[i] = 0;
    __syncthreads();
    i64 t0 = lo + (i64)blockIdx.x * kTile;
    for (int r = 0; r < kItems; r++) {
        i64 e = t0 + (i64)r * kBlock + threadIdx.x;
        if (e < hi) {
            EvLoad ev = load_pos(e, n_pend, pend_pos, cols, f, kp, kt);
            if (ev.ok) atomicAdd(&hist[ev.pos & (P - 1)], 1u);
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < P; i += kBlock) counts[(i64)i * nblk + blockIdx.x] = hist[i];
}

void launch_ms_count(hipStream_t s, i64 lo, i64 hi, i64 n_pend, const u32* pend_pos, const i64* ts, ColSet cols,
                     FilterProg f, KeyPlan kp, KeyTable kt, int P, i64* counts, int nblk) {
    (void)ts;
    hipLaunchKernelGGL(k_ms_count, dim3(nblk), dim3(kBlock), P * 4, s, lo, hi, n_pend, pend_pos, cols, f, kp, kt, P,
                       counts, nblk);
}

// LDS: hist[P] (u32) | local_start[P] (u32) | running[P] (u32) | wave_cnt[4][P] (u32) |
//      stage_pos[kTile] | stage_idx[kTile] | stage_p[kTile] | stage_vals[V][kTile] (u64)
__global__ __launch_bounds__(kBlock) void k_ms_scatter(i64 lo, i64 hi, i64 n_pend, const u32* __restrict__ pend_pos,
                                                      const u64* __restrict__ pend_vals, i64 pend_cap, ColSet cols,
                                                      FilterProg f, KeyPlan kp, KeyTable kt, AggPlan ap, int P,
                                                      const i64* __restrict__ offsets, int nblk, u32* rec_pos,
                                                      u32* rec_idx, u64* rec_vals, i64 rec_cap) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    unsigned char* sm = (unsigned char*)(((uintptr_t)smem_raw + 15) & ~(uintptr_t)15);
    u64* stage_vals = (u64*)sm;
    u32* stage_pos = (u32*)(stage_vals + (size_t)ap.n_vcols * kTile);
    u32* stage_idx = stage_pos + kTile;
    u32* stage_p = stage_idx + kTile;
    u32* hist = stage_p + kTile;
    u32* local_start = hist + P;
    u32* running = local_start + P;
    u32* wave_cnt = running + P;  // [4][P]
    for (int i = threadIdx.x; i < P; i += kBlock) {
        hist[i] = 0; running[i] = 0;
        for (int w = 0; w < 4; w++) wave_cnt[w * P + i] = 0;
    }
    __syncthreads();
    const i64 t0 = lo + (i64)blockIdx.x * kTile;
    // pass 1: histogram of this tile
    u32 my_pos[kItems];
    bool my_ok[kItems];
#pragma unroll
    for (int r = 0; r < kItems; r++) {
        i64 e = t0 + (i64)r * kBlock + threadIdx.x;
        my_ok[r] = false;
        if (e < hi) {
            EvLoad ev = load_pos(e, n_pend, pend_pos, cols, f, kp, kt);
            my_ok[r] = ev.ok;
            my_pos[r] = ev.pos;
            if (ev.ok) atomicAdd(&hist[ev.pos & (P - 1)], 1u);
        }
    }
    __syncthreads();
    // exclusive scan of hist -> local_start (each thread scans a contiguous chunk of P)
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
    // pass 2: ordered ranks per sub-round of kBlock events
    for (int r = 0; r < kItems; r++) {
        bool ok = my_ok[r];
        u32 p = ok ? (my_pos[r] & (P - 1)) : 0;
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
            u32 slot = local_start[p] + before + lrank;
            i64 e = t0 + (i64)r * kBlock + threadIdx.x;
            stage_pos[slot] = my_pos[r];
            stage_idx[slot] = (u32)e;
            stage_p[slot] = p;
            if (e < n_pend) {
                for (int j = 0; j < ap.n_vcols; j++) stage_vals[(size_t)j * kTile + slot] = pend_vals[(size_t)j * pend_cap + e];
            } else {
                for (int j = 0; j < ap.n_vcols; j++)
                    stage_vals[(size_t)j * kTile + slot] = (u64)load_raw(cols, ap.vcol_src[j], e - n_pend);
            }
        }
        __syncthreads();
        if (leader) { atomicAdd(&running[p], wave_cnt[wave * P + p]); wave_cnt[wave * P + p] = 0; }
        __syncthreads();
    }
    // pass 3: write each partition's run of this tile contiguously
    i64 total = 0;
    for (int i = 0; i < P; i++) {}
    u32 n_tile = 0;
    {
        // total valid = local_start[P-1] + hist[P-1]
        n_tile = local_start[P - 1] + hist[P - 1];
    }
    for (u32 j = threadIdx.x; j < n_tile; j += kBlock) {
        u32 p = stage_p[j];
        i64 dst = offsets[(i64)p * nblk + blockIdx.x] + (j - local_start[p]);
        rec_pos[dst] = stage_pos[j];
        rec_idx[dst] = stage_idx[j];
        for (int v = 0; v < ap.n_vcols; v++) rec_vals[(size_t)v * rec_cap + dst] = stage_vals[(size_t)v * kTile + j];
    }
    (void)total;
}

void launch_ms_scatter(hipStream_t s, i64 lo, i64 hi, i64 n_pend, const u32* pend_pos, const u64* pend_vals,
                       i64 pend_cap, const i64* ts, ColSet cols, FilterProg f, KeyPlan kp, KeyTable kt, AggPlan ap,
                       int P, const i64* offsets, int nblk, u32* rec_pos, u32* rec_idx, u64* rec_vals, i64 rec_cap) {
    (void)ts;
    size_t lds = (size_t)ap.n_vcols * kTile * 8 + (size_t)kTile * 12 + (size_t)P * 4 * 7 + 16;
    hipLaunchKernelGGL(k_ms_scatter, dim3(nblk), dim3(kBlock), lds, s, lo, hi, n_pend, pend_pos, pend_vals, pend_cap,
                       cols, f, kp, kt, ap, P, offsets, nblk, rec_pos, rec_idx, rec_vals, rec_cap);
}

// three-phase exclusive scan for long arrays
__global__ __launch_bounds__(kBlock) void k_reduce_tiles(const i64* a, i64 n, i64* tmp) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 s = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) if (base + i < n) s += a[base + i];
    i64 t = block_reduce(s, SumOp(), 0);
    if (threadIdx.x == 0) tmp[blockIdx.x] = t;
}
__global__ __launch_bounds__(kBlock) void k_scan_tiles(i64* a, i64 n, const i64* tmp) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 v[kItems];
    i64 s = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) { v[i] = base + i < n ? a[base + i] : 0; s += v[i]; }
    i64 pre = block_excl_scan(s, SumOp(), 0, nullptr) + tmp[blockIdx.x];
#pragma unroll
    for (int i = 0; i < kItems; i++) if (base + i < n) { a[base + i] = pre; pre += v[i]; }
}

void launch_scan_sum_large(hipStream_t s, i64* a, i64 n, i64* tmp) {
    int nb = (int)((n + kTile - 1) / kTile);
    hipLaunchKernelGGL(k_reduce_tiles, dim3(nb), dim3(kBlock), 0, s, a, n, tmp);
    launch_scan_sum(s, tmp, nb);
    hipLaunchKernelGGL(k_scan_tiles, dim3(nb), dim3(kBlock), 0, s, a, n, tmp);
}

__global__ void k_part_off(const i64* counts, int nblk, int P, i64* part_off) {
    int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p <= P) part_off[p] = counts[(i64)p * nblk];
}

void launch_part_off(hipStream_t s, const i64* counts, int nblk, int P, i64* part_off) {
    hipLaunchKernelGGL(k_part_off, dim3((P + 1 + 255) / 256), dim3(256), 0, s, counts, nblk, P, part_off);
}

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

}  // namespace shd
