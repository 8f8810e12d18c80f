// sh_slx_kernels.hip — `insert expired events` / `insert all events` of the sliding time(T) and
// externalTime(ts, T) windows on gfx950.
//
// TimeWindowProcessor.process (core/query/processor/stream/window/TimeWindowProcessor.java:132-169)
// keeps ONE expiry queue in arrival order. Before every event it removes the longest queue prefix
// whose heads satisfy ts + T <= now, re-stamps each with now and inserts it into the chunk before
// the event (insertBeforeCurrent); TIMER events (Scheduler.notifyAt(ts + T) at every new maximum ts,
// fired before a send whose clock reached them, Scheduler.java:71-104, 171-209) do the same in a
// chunk of their own. The selector (QuerySelector.processInBatchGroupBy :315-374) then emits per
// chunk one row per key in first-occurrence order with the aggregates after the key's last
// qualifying event — for an EXPIRED event after its processRemove.
//
// Everything is a function of two monotone sequences: PM(g) = max ts of the passing events up to
// arrival g (the queue head blocks, so event g has expired at a point p iff PM(g) + T <= now(p)) and
// the points' clocks. With m(now) = #{g : PM(g) + T <= now}, the expired prefix after point p is
// min(inserted(p), m(now(p))). So every event's expiry point is found by binary search, every
// operation (add at its own point, remove at its expiry point) gets its position in the push's
// operation sequence arithmetically, and one lane per key replays its adds and removes in that order.
#include "sh_device.h"
#include "sh_sliding.h"

namespace shd {

namespace {

constexpr u64 kNoOp = ~0ull;

__device__ __forceinline__ i64 sat_add(i64 a, i64 b) { return a > INT64_MAX - b ? INT64_MAX : a + b; }

// first index in [lo, hi) with a[i] >= x (a non-decreasing); hi when none
__device__ __forceinline__ i64 lb_ge(const i64* __restrict__ a, i64 lo, i64 hi, i64 x) {
    while (lo < hi) {
        const i64 m = (lo + hi) >> 1;
        if (a[m] < x) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// first u in [0, n) with A[u] + T > c (A non-decreasing): the number of events whose PM + T <= c
__device__ __forceinline__ i64 n_expirable(const i64* __restrict__ A, i64 n, i64 T, i64 c) {
    i64 lo = 0, hi = n;
    while (lo < hi) {
        const i64 m = (lo + hi) >> 1;
        if (sat_add(A[m], T) <= c) lo = m + 1;
        else hi = m;
    }
    return lo;
}

// `next > value` (min) / `next < value` (max) on the input type (MinAttributeAggregatorExecutor :86-236)
__device__ __forceinline__ bool x_worse(int kind, u64 cur, u64 v) {
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
__device__ __forceinline__ bool x_eq(int kind, u64 a, u64 b) {
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

}  // namespace

// ---- per send: records before it, clock before it, its last timestamp ---------------------------
// (InputHandler.send sets the clock from the send's last event, TimestampGeneratorImpl :104-122;
// a send whose last ts is below the clock does not move it and fires no timer)
__global__ __launch_bounds__(kBlock) void k_slx_sends(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                     WinParams wp, const i64* blk_pass_pre, const i64* blk_tl_pre,
                                                     i64* sK, i64* scb, i64* slast) {
    // the tile's events lane-strided (round i: tile + i * kBlock + thread), a block scan per round, so
    // consecutive lanes write consecutive sends (per-event sends: the thread-contiguous stores were 64
    // pieces 8 entries apart per instruction; r05: 1.2 ms of c3all's push)
    const i64 tile = (i64)blockIdx.x * kTile;
    i64 run = blk_pass_pre[blockIdx.x], run_cm = blk_tl_pre[blockIdx.x];
    const i64 c0 = wp.clock_valid ? wp.clock0 : INT64_MIN;
    const i64 sl = send_len(wp);
    for (int it = 0; it < kItems; it++) {
        const i64 e = tile + (i64)it * kBlock + threadIdx.x;
        const bool in = e < wp.N;
        const bool pass = in && eval_filter(f, cols, e);
        const i64 t = in ? ts[e] : INT64_MIN;
        const i64 tl = in && is_send_last(wp, e) ? t : INT64_MIN;
        i64 tot, mx;
        const i64 r = run + block_excl_scan(pass ? (i64)1 : (i64)0, SumOp(), 0, &tot);
        const i64 cm = max(run_cm, block_excl_scan(tl, MaxOp(), INT64_MIN, &mx));
        run += tot;
        run_cm = max(run_cm, mx);
        if (in && e % sl == 0) {
            const i64 s = e / sl;
            sK[s] = r;
            scb[s] = max(c0, cm);
            slast[s] = sl == 1 ? t : ts[send_last_of(wp, e)];
        }
    }
}

void launch_slx_sends(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp, const i64* blk_pass_pre,
                      const i64* blk_tl_pre, int nblk, i64* sK, i64* scb, i64* slast) {
    hipLaunchKernelGGL(k_slx_sends, dim3(nblk), dim3(kBlock), 0, s, ts, cols, f, wp, blk_pass_pre, blk_tl_pre, sK, scb,
                       slast);
}

// ---- stream compaction helpers (striped over tiles of kTile, tile prefix from launch_scan_sum) ----
// kind 0: calls (slast >= scb) -> (cK, cC = slast, cS = send); kind 1: u8 flags -> index list
__global__ __launch_bounds__(kBlock) void k_slx_count(int kind, const unsigned char* __restrict__ flags,
                                                     const i64* __restrict__ scb, const i64* __restrict__ slast, i64 n,
                                                     i64* blk_cnt) {
    const i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 c = 0;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        const i64 j = base + i;
        if (j < n) c += kind == 0 ? (slast[j] >= scb[j]) : flags[j] != 0;
    }
    const i64 t = block_reduce(c, SumOp(), 0);
    if (threadIdx.x == 0) blk_cnt[blockIdx.x] = t;
}

__global__ __launch_bounds__(kBlock) void k_slx_compact(int kind, const unsigned char* __restrict__ flags,
                                                       const i64* __restrict__ sK, const i64* __restrict__ scb,
                                                       const i64* __restrict__ slast, i64 n,
                                                       const i64* __restrict__ blk_pre, i64* oK, i64* oC, i64* oS) {
    const i64 tile = (i64)blockIdx.x * kTile;
    i64 run = blk_pre[blockIdx.x];
    for (int it = 0; it < kItems; it++) {
        const i64 j = tile + (i64)it * kBlock + threadIdx.x;
        const i64 fl = j < n ? (kind == 0 ? (slast[j] >= scb[j]) : flags[j] != 0) : 0;
        i64 tot;
        const i64 r = run + block_excl_scan(fl, SumOp(), 0, &tot);
        run += tot;
        if (!fl) continue;
        if (kind == 0) {
            oK[r] = sK[j];
            oC[r] = slast[j];
            oS[r] = j;
        } else {
            oS[r] = j;
        }
    }
}

// n entries -> compacted; blk (nblk + 1 entries) ends with the total
void launch_slx_compact(hipStream_t s, int kind, const unsigned char* flags, const i64* sK, const i64* scb,
                        const i64* slast, i64 n, i64* blk, i64* oK, i64* oC, i64* oS) {
    const int nblk = (int)((n + kTile - 1) / kTile);
    if (n <= 0) {
        (void)hipMemsetAsync(blk, 0, 8, s);
        return;
    }
    hipLaunchKernelGGL(k_slx_count, dim3(nblk), dim3(kBlock), 0, s, kind, flags, scb, slast, n, blk);
    (void)hipMemsetAsync(blk + nblk, 0, 8, s);
    launch_scan_sum(s, blk, nblk + 1);
    hipLaunchKernelGGL(k_slx_compact, dim3(nblk), dim3(kBlock), 0, s, kind, flags, sK, scb, slast, n, blk, oK, oC, oS);
}

// ---- timers: Scheduler.notifyAt(ts + T) at every new maximum ts (TimeWindowProcessor :157-160); a
// notify time fires at the first call (clock set by a send, Scheduler.onTimeChange :71-104) made after
// it was registered whose clock reached it. A call fires a TIMER chunk iff some notify time fires
// there. Candidates: the carried pending times (registered before the push), then the push's records
// that raise the max. keep = the candidate stays pending after the push.
__global__ __launch_bounds__(kBlock) void k_slx_notify(const i64* __restrict__ pend, i64 n_pend,
                                                      const i64* __restrict__ pm, i64 M, i64 pm0,
                                                      const i64* __restrict__ cK, const i64* __restrict__ cC, i64 nC,
                                                      i64 T, unsigned char* fire, unsigned char* keep) {
    const i64 t = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (t >= n_pend + M) return;
    i64 v, j1 = 0;
    if (t < n_pend) {
        v = pend[t];
    } else {
        const i64 r = t - n_pend;
        const i64 prev = r ? pm[r - 1] : pm0;
        if (pm[r] <= prev) { keep[t] = 0; return; }
        v = pm[r];
        j1 = lb_ge(cK, 0, nC, r + 1);  // a call after the record was processed
    }
    const i64 j2 = lb_ge(cC, 0, nC, sat_add(v, T));
    const i64 j = max(j1, j2);
    if (j < nC) {
        fire[j] = 1;
        keep[t] = 0;
    } else {
        keep[t] = 1;
    }
}

void launch_slx_notify(hipStream_t s, const i64* pend, i64 n_pend, const i64* pm, i64 M, i64 pm0, const i64* cK,
                       const i64* cC, i64 nC, i64 T, unsigned char* fire, unsigned char* keep) {
    const i64 n = n_pend + M;
    if (n <= 0) return;
    hipLaunchKernelGGL(k_slx_notify, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, pend, n_pend, pm,
                       M, pm0, cK, cC, nC, T, fire, keep);
}

// gathers of compacted index lists
__global__ __launch_bounds__(kBlock) void k_slx_gather_calls(const i64* __restrict__ idx, i64 n, const i64* cK,
                                                            const i64* cC, const i64* cS, i64* fK, i64* fC, i64* fS) {
    const i64 j = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (j >= n) return;
    const i64 c = idx[j];
    fK[j] = cK[c];
    fC[j] = cC[c];
    fS[j] = cS[c];
}

__global__ __launch_bounds__(kBlock) void k_slx_gather_pend(const i64* __restrict__ idx, i64 n, const i64* pend,
                                                           i64 n_pend, const i64* pm, i64* out) {
    const i64 j = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (j >= n) return;
    const i64 c = idx[j];
    out[j] = c < n_pend ? pend[c] : pm[c - n_pend];
}

void launch_slx_gather_calls(hipStream_t s, const i64* idx, i64 n, const i64* cK, const i64* cC, const i64* cS, i64* fK,
                             i64* fC, i64* fS) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_slx_gather_calls, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, idx, n, cK,
                       cC, cS, fK, fC, fS);
}

void launch_slx_gather_pend(hipStream_t s, const i64* idx, i64 n, const i64* pend, i64 n_pend, const i64* pm,
                            i64* out) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_slx_gather_pend, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, idx, n, pend,
                       n_pend, pm, out);
}

// ---- the window FIFO: U = [carried unexpired events | this push's records] (PM and stream index) ----
__global__ __launch_bounds__(kBlock) void k_slx_append(const i64* __restrict__ pm, const u32* __restrict__ raw, i64 M,
                                                      i64 seq_base, i64* upm, i64* useq) {
    const i64 r = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (r >= M) return;
    upm[r] = pm[r];
    useq[r] = seq_base + (i64)raw[r];
}

void launch_slx_append(hipStream_t s, const i64* pm, const u32* raw, i64 M, i64 seq_base, i64* upm, i64* useq) {
    if (M <= 0) return;
    hipLaunchKernelGGL(k_slx_append, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, pm, raw, M,
                       seq_base, upm, useq);
}

// ---- expiry point and operation index of every window event --------------------------------------
// u = the event's position in U (global arrival = X0 + u). Its expiry point is the first point after
// its arrival whose clock reaches PM + T: an event point i (record i, clock rclk[i]; points of the
// push's records start at local index max(0, u - W0 + 1)) or a firing call f (fK[f] records before
// it). The timer of call f precedes event point fK[f]. Operation index = u + records before the point.
// one event's expiry point (see above); true when it has one
// The searches are monotone in u (PM and u - W0 grow with u), so a block's answers lie between those of
// its first and last event: [ie0, ie1] and [f0, f1] bound every thread's search (a few steps over lines
// the block shares instead of 25 over the whole push).
struct XBounds {
    i64 ie0, ie1, fa0, fa1, fb0, fb1;
};
__device__ __forceinline__ bool slx_expiry_one(i64 u, const i64* __restrict__ upm, i64 W0, i64 M,
                                               const i64* __restrict__ rclk, const i64* __restrict__ rsclk,
                                               const u32* __restrict__ raw, i64 send_size, const i64* __restrict__ fK,
                                               const i64* __restrict__ fC, const i64* __restrict__ fS, i64 nF, i64 T,
                                               u64* xop, i64* xch, i64* xts, i64* xclk, const XBounds& B,
                                               u64* xx, const i64* __restrict__ useq, const u64* __restrict__ rvals) {
    const i64 th = sat_add(upm[u], T);
    const i64 lo_i = max((i64)0, u - W0 + 1);
    const i64 ie = lb_ge(rclk, max(lo_i, B.ie0), B.ie1, th);
    const i64 f = max(lb_ge(fK, B.fa0, B.fa1, u - W0 + 1), lb_ge(fC, B.fb0, B.fb1, th));
    u64 op = kNoOp;
    i64 c_ch = 0, c_ts = 0, c_clk = 0;
    if (f < nF && (ie >= M || fK[f] <= ie)) {
        op = (u64)(u + fK[f]);
        c_ch = 2 * fS[f];
        c_ts = fC[f];
        c_clk = fC[f];
    } else if (ie < M) {
        op = (u64)(u + ie);
        c_ch = 2 * (send_size > 0 ? (i64)raw[ie] / send_size : 0) + 1;
        c_ts = rclk[ie];
        c_clk = rsclk ? rsclk[ie] : rclk[ie];
    }
    if (xx) {
        ulonglong2* o = (ulonglong2*)(xx + (size_t)u * kXaWords);
        o[0] = make_ulonglong2(op, u >= W0 ? rvals[u - W0] : 0ull);
        o[1] = make_ulonglong2((u64)c_ts, (u64)c_clk);
        o[2] = make_ulonglong2((u64)useq[u], (u64)c_ch);
    } else {
        if (op != kNoOp) {
            xch[u] = c_ch;
            xts[u] = c_ts;
            xclk[u] = c_clk;
        }
        xop[u] = op;
    }
    return op != kNoOp;
}

__global__ __launch_bounds__(kBlock) void k_slx_expiry(const i64* __restrict__ upm, i64 n_u, i64 W0, i64 M,
                                                      const i64* __restrict__ rclk, const i64* __restrict__ rsclk,
                                                      const u32* __restrict__ raw, i64 send_size,
                                                      const i64* __restrict__ fK, const i64* __restrict__ fC,
                                                      const i64* __restrict__ fS, i64 nF, i64 T, u64* xop, i64* xch,
                                                      i64* xts, i64* xclk, unsigned long long* n_exp, u64* xx,
                                                      const i64* __restrict__ useq, const u64* __restrict__ rvals,
                                                      const i64* __restrict__ bnd) {
    // the block's bounds: the full searches of its first event and of the next block's (k_slx_xbounds)
    const int bk = blockIdx.x;
    const XBounds B{bnd[3 * bk], bnd[3 * bk + 3], bnd[3 * bk + 1], bnd[3 * bk + 4], bnd[3 * bk + 2], bnd[3 * bk + 5]};
    const i64 u = (i64)bk * kBlock + threadIdx.x;
    const bool has = u < n_u && slx_expiry_one(u, upm, W0, M, rclk, rsclk, raw, send_size, fK, fC, fS, nF, T, xop,
                                               xch, xts, xclk, B, xx, useq, rvals);
    // The events with an expiry point form a prefix of U (PM and the first eligible point both grow with
    // u), so n_exp is written once, by the last of them: the lane whose successor has none. (r04 took one
    // atomicMax per wave on one address: 680k serialised L2 atomics, 5.4 of the 6 ms of c3all's kernel.)
    __shared__ unsigned char s_has[kBlock + 1];
    s_has[threadIdx.x] = has ? 1 : 0;
    if (threadIdx.x == kBlock - 1) {
        // the next block's first event: its full searches are the bounds' upper entries
        bool hn = false;
        if (u + 1 < n_u) {
            const i64 f = max(B.fa1, B.fb1);
            hn = (f < nF && (B.ie1 >= M || fK[f] <= B.ie1)) || B.ie1 < M;
        }
        s_has[kBlock] = hn ? 1 : 0;
    }
    __syncthreads();
    if (has && !s_has[threadIdx.x + 1]) *n_exp = (unsigned long long)(u + 1);
}

// the full searches at every block start u = b * kBlock (and at n_u - 1 past the last block): entry b
// bounds block b from below, entry b + 1 from above; one thread each, all in parallel
__global__ __launch_bounds__(kBlock) void k_slx_xbounds(const i64* __restrict__ upm, i64 n_u, i64 W0, i64 M,
                                                       const i64* __restrict__ rclk, const i64* __restrict__ fK,
                                                       const i64* __restrict__ fC, i64 nF, i64 T, int nb, i64* bnd) {
    const int b = blockIdx.x * kBlock + threadIdx.x;
    if (b > nb) return;
    const i64 u = b < nb ? (i64)b * kBlock : n_u - 1;
    const i64 th = sat_add(upm[u], T);
    bnd[3 * b] = lb_ge(rclk, max((i64)0, u - W0 + 1), M, th);
    bnd[3 * b + 1] = lb_ge(fK, 0, nF, u - W0 + 1);
    bnd[3 * b + 2] = lb_ge(fC, 0, nF, th);
}

void launch_slx_expiry(hipStream_t s, const i64* upm, i64 n_u, i64 W0, i64 M, const i64* rclk, const i64* rsclk,
                       const u32* raw, i64 send_size, const i64* fK, const i64* fC, const i64* fS, i64 nF, i64 T,
                       u64* xop, i64* xch, i64* xts, i64* xclk, unsigned long long* n_exp, u64* xx, const i64* useq,
                       const u64* rvals, i64* bnd) {
    if (n_u <= 0) return;
    const int nb = (int)((n_u + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_slx_xbounds, dim3((unsigned)((nb + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, upm, n_u, W0,
                       M, rclk, fK, fC, nF, T, nb, bnd);
    hipLaunchKernelGGL(k_slx_expiry, dim3((unsigned)nb), dim3(kBlock), 0, s, upm, n_u, W0, M, rclk, rsclk, raw,
                       send_size, fK, fC, fS, nF, T, xop, xch, xts, xclk, n_exp, xx, useq, rvals, bnd);
}

// add of record i: after the removes of every point up to and including its own
// (X(i) - X0 = min(W0 + i, #{u : PM(u) + T <= clock_i}))
__global__ __launch_bounds__(kBlock) void k_slx_aop(const i64* __restrict__ rclk, i64 M, const i64* __restrict__ upm,
                                                   i64 n_u, i64 W0, i64 T, u64* aop, u64* xa, SlRecords rec,
                                                   const i64* __restrict__ rsclk, const i64* __restrict__ bnd) {
    // (monotone in i: the full searches at this block's start and the next one's bound every thread's)
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= M) return;
    i64 lo = bnd[blockIdx.x], hi = bnd[blockIdx.x + 1];
    const i64 c = rclk[i];
    while (lo < hi) {
        const i64 m = (lo + hi) >> 1;
        if (sat_add(upm[m], T) <= c) lo = m + 1;
        else hi = m;
    }
    const u64 op = (u64)(i + min(W0 + i, lo));
    if (xa) {
        ulonglong2* o = (ulonglong2*)(xa + (size_t)i * kXaWords);
        o[0] = make_ulonglong2(op, rec.vals[i]);
        o[1] = make_ulonglong2((u64)rec.ts[i], (u64)(rsclk ? rsclk[i] : c));
        o[2] = make_ulonglong2((u64)rec.raw[i], (u64)rec.pm[i]);
    } else {
        aop[i] = op;
    }
}

__global__ __launch_bounds__(kBlock) void k_slx_abounds(const i64* __restrict__ rclk, i64 M, const i64* __restrict__ upm,
                                                       i64 n_u, i64 T, int nb, i64* bnd) {
    const int b = blockIdx.x * kBlock + threadIdx.x;
    if (b > nb) return;
    bnd[b] = n_expirable(upm, n_u, T, rclk[b < nb ? (i64)b * kBlock : M - 1]);
}

void launch_slx_aop(hipStream_t s, const i64* rclk, i64 M, const i64* upm, i64 n_u, i64 W0, i64 T, u64* aop, u64* xa,
                    SlRecords rec, const i64* rsclk, i64* bnd) {
    if (M <= 0) return;
    const int nb = (int)((M + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_slx_abounds, dim3((unsigned)((nb + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rclk, M, upm,
                       n_u, T, nb, bnd);
    hipLaunchKernelGGL(k_slx_aop, dim3((unsigned)nb), dim3(kBlock), 0, s, rclk, M, upm, n_u, W0, T, aop, xa, rec, rsclk,
                       bnd);
}

// ---- the replay: one lane per key slot walks its adds (records sorted stably by slot) and the
// removes of its ring entries, merged by operation index. Rows: one per (chunk, key), opened at the
// first qualifying operation of the key in the chunk (its operation index is the row's position) and
// carrying the aggregates after the key's last qualifying operation there. ------------------------------
template <int NA, int NV>
__global__ __launch_bounds__(64) void k_slx_walk(const u32* __restrict__ key_off, const u32* __restrict__ sorted_rank,
                                                 u32 nslots, SlRecords rec, const u64* __restrict__ aop,
                                                 const u64* __restrict__ xop, const i64* __restrict__ xch,
                                                 const i64* __restrict__ xts, const i64* __restrict__ xclk,
                                                 const i64* __restrict__ useq, i64 n_u, i64 X0, i64 G0, i64 seq_base,
                                                 i64 send_size, SlState S, i64* rg, AggPlan ap, int cur_on, int exp_on,
                                                 SlxRows rows, unsigned char* flags, const i64* __restrict__ rsclk) {
    const u32 k = blockIdx.x * 64 + threadIdx.x;
    if (k >= nslots) return;
    const u32 lo = key_off[k], hi = key_off[k + 1];
    i64 rlen = S.rlen[k];
    if (lo == hi && rlen == 0) return;
    const i64 rc = S.rc, rm = rc - 1;
    i64 rh = S.rhead[k];
    i64 cnt = S.cnt[k];
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
            mm[a] = S.mm[fi];
            mmh[a] = S.mm_has[fi];
            dqh[a] = S.dq_head[fi];
            dql[a] = S.dq_len[fi];
        }
    }
    // open row
    i64 row_ch = -1, row_op = 0, row_ts = 0, row_rep = 0, row_clk = 0;
    unsigned char row_exp = 0;
    u64 rv[NA];
    unsigned char rn[NA];
#pragma unroll
    for (int a = 0; a < NA; a++) { rv[a] = 0; rn[a] = 0; }
#define SLX_WRITE_ROW()                                                   \
    do {                                                                  \
        rows.ts[row_op] = row_ts;                                         \
        rows.rep[row_op] = row_rep;                                       \
        rows.slot[row_op] = k;                                            \
        rows.ch[row_op] = row_ch;                                         \
        rows.clk[row_op] = row_clk;                                       \
        rows.exp[row_op] = row_exp;                                       \
        _Pragma("unroll") for (int a = 0; a < NA; a++) {                  \
            if (a < ap.n) {                                               \
                rows.vals[(size_t)a * rows.cap + row_op] = rv[a];         \
                rows.nulls[(size_t)a * rows.cap + row_op] = rn[a];        \
            }                                                             \
        }                                                                 \
    } while (0)
    u32 ai = lo;
    u64 a_op = ai < hi ? aop[sorted_rank[ai]] : kNoOp;
    for (;;) {
        u64 x_op = kNoOp;
        i64 u = -1;
        if (rlen > 0) {
            u = rg[(size_t)k * rc + (rh & rm)] - X0;
            if (u >= 0 && u < n_u) x_op = xop[u];
        }
        if (a_op == kNoOp && x_op == kNoOp) break;
        i64 op, ch, ts_row, rep, clk;
        bool is_exp;
        if (x_op < a_op) {
            // processRemove of the ring head (AttributeAggregatorExecutor.processRemove)
            const i64 sl = rh & rm;
            u64 v[NV];
#pragma unroll
            for (int q = 0; q < NV; q++) v[q] = q < ap.n_vcols ? S.rval[((size_t)q * S.nslots + k) * rc + sl] : 0;
            rh++;
            rlen--;
            cnt--;
#pragma unroll
            for (int a = 0; a < NA; a++) {
                if (a >= ap.n) break;
                const int kind = ap.kind[a];
                if (kind == AK_COUNT) continue;
                u64 x = v[0];
#pragma unroll
                for (int q = 1; q < NV; q++) x = ap.vcol[a] == q ? v[q] : x;
                if (kind == AK_SUM_L) {
                    f[a] = (u64)java_d2l((double)(i64)f[a] - (double)(i64)x);
                } else if (kind == AK_SUM_D || kind == AK_AVG) {
                    const double xv = (kind == AK_AVG && !is_fp(ap.vcol_type[ap.vcol[a]])) ? (double)(i64)x
                                                                                           : __longlong_as_double((i64)x);
                    double r = __longlong_as_double((i64)f[a]) - xv;
                    if (cnt == 0 && r == 0.0) r = 0.0;  // destroyed state restarts from +0.0 (canDestroy)
                    f[a] = (u64)__double_as_longlong(r);
                } else {
                    // removeFirstOccurrence(value)
                    u64* d = S.dq + ((size_t)ap.field[a] * S.nslots + k) * rc;
                    const i64 h = dqh[a];
                    i64 len = dql[a], found = -1;
                    for (i64 j = 0; j < len; j++)
                        if (x_eq(kind, d[(h + j) & rm], x)) { found = j; break; }
                    if (found == 0) {
                        dqh[a] = h + 1;
                        len--;
                    } else if (found > 0) {
                        for (i64 j = found; j + 1 < len; j++) d[(h + j) & rm] = d[(h + j + 1) & rm];
                        len--;
                    }
                    dql[a] = len;
                    mm[a] = len > 0 ? d[dqh[a] & rm] : 0;
                    mmh[a] = len > 0 ? 1 : 0;
                }
            }
            op = (i64)x_op;
            ch = xch[u];
            ts_row = xts[u];
            clk = xclk[u];
            rep = useq[u];
            is_exp = true;
        } else {
            // processAdd of the record; it joins the ring
            const u32 r = sorted_rank[ai];
            u64 v[NV];
#pragma unroll
            for (int q = 0; q < NV; q++) v[q] = q < ap.n_vcols ? rec.vals[(size_t)q * rec.cap + r] : 0;
            const i64 sl = (rh + rlen) & rm;
            S.rpm[(size_t)k * rc + sl] = rec.pm[r];
            rg[(size_t)k * rc + sl] = G0 + r;
#pragma unroll
            for (int q = 0; q < NV; q++)
                if (q < ap.n_vcols) S.rval[((size_t)q * S.nslots + k) * rc + sl] = v[q];
            rlen++;
            cnt++;
#pragma unroll
            for (int a = 0; a < NA; a++) {
                if (a >= ap.n) break;
                const int kind = ap.kind[a];
                if (kind == AK_COUNT) continue;
                u64 x = v[0];
#pragma unroll
                for (int q = 1; q < NV; q++) x = ap.vcol[a] == q ? v[q] : x;
                if (kind == AK_SUM_L) {
                    f[a] = (u64)((i64)f[a] + (i64)x);
                } else if (kind == AK_SUM_D || kind == AK_AVG) {
                    const double xv = (kind == AK_AVG && !is_fp(ap.vcol_type[ap.vcol[a]])) ? (double)(i64)x
                                                                                           : __longlong_as_double((i64)x);
                    f[a] = (u64)__double_as_longlong(__longlong_as_double((i64)f[a]) + xv);
                } else {
                    u64* d = S.dq + ((size_t)ap.field[a] * S.nslots + k) * rc;
                    const i64 h = dqh[a];
                    i64 len = dql[a];
                    while (len > 0 && x_worse(kind, d[(h + len - 1) & rm], x)) len--;
                    d[(h + len) & rm] = x;
                    dql[a] = len + 1;
                    // minValue = value when strictly better (MinAttributeAggregatorExecutor.processAdd): the
                    // deque's front except past a NaN, which no comparison pops
                    {
                        // (a select, not a conditional store: hipcc for gfx950 dropped the store of the
                        // `if` form in this divergent branch — r05, tests/test_gpu_sliding_expired.py)
                        const bool take = !mmh[a] || x_worse(kind, mm[a], x);
                        mm[a] = take ? x : mm[a];
                    }
                    mmh[a] = 1;
                }
            }
            op = (i64)a_op;
            const i64 send = send_size > 0 ? (i64)rec.raw[r] / send_size : 0;
            ch = 2 * send + 1;
            ts_row = rec.ts[r];
            clk = rsclk ? rsclk[r] : rec.clock[r];  // externalTime: the send's playback clock
            rep = seq_base + (i64)rec.raw[r];
            is_exp = false;
            ai++;
            a_op = ai < hi ? aop[sorted_rank[ai]] : kNoOp;
        }
        if (is_exp ? !exp_on : !cur_on) continue;
        if (ch != row_ch) {
            if (row_ch >= 0) SLX_WRITE_ROW();
            row_ch = ch;
            row_op = op;
            flags[op] = 1;
        }
        row_ts = ts_row;
        row_rep = rep;
        row_clk = clk;
        row_exp = is_exp ? 1 : 0;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            if (a >= ap.n) break;
            const int kind = ap.kind[a];
            u64 o = 0;
            unsigned char nl = 0;
            if (kind == AK_COUNT) o = (u64)cnt;
            else if (kind == AK_SUM_L || kind == AK_SUM_D) { o = f[a]; nl = cnt == 0; }
            else if (kind == AK_AVG) {
                nl = cnt == 0;
                if (!nl) o = (u64)__double_as_longlong(__longlong_as_double((i64)f[a]) / (double)cnt);
            } else { o = mm[a]; nl = mmh[a] ? 0 : 1; }
            rv[a] = nl ? 0 : o;
            rn[a] = nl;
        }
    }
    if (row_ch >= 0) SLX_WRITE_ROW();
#undef SLX_WRITE_ROW
    S.cnt[k] = cnt;
    S.rhead[k] = rh;
    S.rlen[k] = rlen;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (a >= ap.n || ap.kind[a] == AK_COUNT) continue;
        const size_t fi = (size_t)ap.field[a] * S.nslots + k;
        S.f[fi] = f[a];
        if (ap.kind[a] >= AK_MIN_L) {
            S.mm[fi] = mm[a];
            S.mm_has[fi] = mmh[a];
            S.dq_head[fi] = dqh[a];
            S.dq_len[fi] = dql[a];
        }
    }
}

void launch_slx_walk(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, SlRecords rec,
                     const u64* aop, const u64* xop, const i64* xch, const i64* xts, const i64* xclk, const i64* useq,
                     i64 n_u, i64 X0, i64 G0, i64 seq_base, i64 send_size, SlState S, i64* rg, AggPlan ap, int cur_on,
                     int exp_on, SlxRows rows, unsigned char* flags, const i64* rsclk) {
    const unsigned grid = (unsigned)((nslots + 63) / 64);
    if (grid == 0) return;
#define SH_SLX_W(A, V)                                                                                            \
    hipLaunchKernelGGL((k_slx_walk<A, V>), dim3(grid), dim3(64), 0, s, key_off, sorted_rank, (u32)nslots, rec, aop, \
                       xop, xch, xts, xclk, useq, n_u, X0, G0, seq_base, send_size, S, rg, ap, cur_on, exp_on, rows,  \
                       flags, rsclk)
    const int nv = ap.n_vcols < 1 ? 1 : ap.n_vcols;
    if (ap.n <= 4 && nv <= 1) SH_SLX_W(4, 1);
    else if (nv <= 2) SH_SLX_W(8, 2);
    else SH_SLX_W(8, 8);
#undef SH_SLX_W
}

// pass-through (`select *`, no aggregators, no group-by: QuerySelector.processNoGroupBy :161-205): every
// qualifying operation is a row of its own at its operation index
__global__ __launch_bounds__(kBlock) void k_slx_pass(SlRecords rec, i64 M, const u64* __restrict__ aop,
                                                    const u64* __restrict__ xop, const i64* __restrict__ xch,
                                                    const i64* __restrict__ xts, const i64* __restrict__ xclk,
                                                    const i64* __restrict__ useq, i64 n_u, i64 seq_base, i64 send_size,
                                                    int cur_on, int exp_on, SlxRows rows, unsigned char* flags,
                                                    const i64* __restrict__ rsclk) {
    const i64 t = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (t < M) {
        if (!cur_on) return;
        const i64 op = (i64)aop[t];
        const i64 send = send_size > 0 ? (i64)rec.raw[t] / send_size : 0;
        rows.ts[op] = rec.ts[t];
        rows.rep[op] = seq_base + (i64)rec.raw[t];
        rows.slot[op] = 0;
        rows.ch[op] = 2 * send + 1;
        rows.clk[op] = rsclk ? rsclk[t] : rec.clock[t];
        rows.exp[op] = 0;
        flags[op] = 1;
    } else if (t < M + n_u) {
        const i64 u = t - M;
        const u64 op = xop[u];
        if (!exp_on || op == kNoOp) return;
        rows.ts[op] = xts[u];
        rows.rep[op] = useq[u];
        rows.slot[op] = 0;
        rows.ch[op] = xch[u];
        rows.clk[op] = xclk[u];
        rows.exp[op] = 1;
        flags[op] = 1;
    }
}

void launch_slx_pass(hipStream_t s, SlRecords rec, i64 M, const u64* aop, const u64* xop, const i64* xch, const i64* xts,
                     const i64* xclk, const i64* useq, i64 n_u, i64 seq_base, i64 send_size, int cur_on, int exp_on,
                     SlxRows rows, unsigned char* flags, const i64* rsclk) {
    const i64 n = M + n_u;
    if (n <= 0) return;
    hipLaunchKernelGGL(k_slx_pass, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rec, M, aop, xop, xch,
                       xts, xclk, useq, n_u, seq_base, send_size, cur_on, exp_on, rows, flags, rsclk);
}

// per slot key offsets of the slot-sorted records (exclusive scan of the per-slot counts)
__global__ void k_slx_keyoff(const u32* __restrict__ slot_cnt, i64 nslots, u32* key_off) {
    const i64 i = (i64)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= nslots) key_off[i] = i < nslots ? slot_cnt[i] : 0;
}

void launch_slx_keyoff(hipStream_t s, const u32* slot_cnt, i64 nslots, u32* key_off, i64* tmp) {
    hipLaunchKernelGGL(k_slx_keyoff, dim3((unsigned)((nslots + 1 + 255) / 256)), dim3(256), 0, s, slot_cnt, nslots,
                       key_off);
    launch_scan_sum_large_u32(s, key_off, nslots + 1, tmp);
}

// ---- emission: flagged operation indices -> output rows in operation order -------------------------
__global__ __launch_bounds__(kBlock) void k_slx_emit(const unsigned char* __restrict__ flags, i64 n,
                                                    const i64* __restrict__ blk_pre, SlxRows rows, int n_aggs,
                                                    KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys,
                                                    u64* out_vals, unsigned char* out_nulls, unsigned char* out_exp,
                                                    i64* out_ch, i64* out_clock, i64* out_rep) {
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
        out_exp[r] = rows.exp[j];
        out_ch[r] = rows.ch[j];
        out_clock[r] = rows.clk[j];
        out_rep[r] = rows.rep[j];
    }
}

void launch_slx_emit(hipStream_t s, const unsigned char* flags, i64 n, const i64* blk_pre, int nblk, SlxRows rows,
                     int n_aggs, KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals,
                     unsigned char* out_nulls, unsigned char* out_exp, i64* out_ch, i64* out_clock, i64* out_rep) {
    if (nblk <= 0) return;
    hipLaunchKernelGGL(k_slx_emit, dim3(nblk), dim3(kBlock), 0, s, flags, n, blk_pre, rows, n_aggs, kt, kp, out_cap,
                       out_ts, out_keys, out_vals, out_nulls, out_exp, out_ch, out_clock, out_rep);
}

// the unexpired tail of U moves to the front (the window FIFO carried to the next push)
__global__ __launch_bounds__(kBlock) void k_slx_shift(const i64* __restrict__ upm, const i64* __restrict__ useq,
                                                     i64 from, i64 n, i64* opm, i64* oseq) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    opm[i] = upm[from + i];
    oseq[i] = useq[from + i];
}

void launch_slx_shift(hipStream_t s, const i64* upm, const i64* useq, i64 from, i64 n, i64* opm, i64* oseq) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_slx_shift, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, upm, useq, from, n,
                       opm, oseq);
}

// Key-table rebuild with expired output: a key is only dropped once its window is empty and every
// aggregator state of it is the one canDestroy removes (count 0, sums exactly 0.0 / 0) — a double sum
// left with a rounding residue keeps the reference's state alive (SumAttributeAggregatorExecutor
// canDestroy), and a key with window events still has expired rows to emit.
__global__ __launch_bounds__(kBlock) void k_slx_rekey_map(i64 size, KeyTable old_kt, KeyTable new_kt,
                                                         const i64* __restrict__ rlen, const i64* __restrict__ cnt,
                                                         const u64* __restrict__ f, i64 nslots, AggPlan ap, u32* map) {
    const i64 s = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (s > size) return;
    if (s == size) { map[s] = (u32)size; return; }
    map[s] = 0xFFFFFFFFu;
    const u64 key = old_kt.keys[s];
    if (key == kEmptyKey) return;
    bool dead = rlen[s] == 0 && cnt[s] == 0;
    for (int a = 0; dead && a < ap.n; a++) {
        const int kind = ap.kind[a];
        const u64 x = kind == AK_COUNT || kind >= AK_MIN_L ? 0 : f[(size_t)ap.field[a] * nslots + s];
        if (kind == AK_SUM_L) dead = x == 0;
        else if (kind == AK_SUM_D || kind == AK_AVG) dead = __longlong_as_double((i64)x) == 0.0;
    }
    if (dead) return;
    map[s] = key_slot(new_kt, key);
}

void launch_slx_rekey_map(hipStream_t s, i64 size, KeyTable old_kt, KeyTable new_kt, const i64* rlen, const i64* cnt,
                          const u64* f, i64 nslots, AggPlan ap, u32* map) {
    hipLaunchKernelGGL(k_slx_rekey_map, dim3((unsigned)((size + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, size,
                       old_kt, new_kt, rlen, cnt, f, nslots, ap, map);
}

}  // namespace shd
