// sh_expired_kernels.hip — expired / all-events output of the batch windows, and pass-through
// (no aggregator, no group-by) batch queries.
//
// A batch flush in the reference is the chunk [expired copies of the previous batch] + RESET +
// [current batch] (LengthBatchWindowProcessor.processFullBatchEvents :206-243,
// TimeBatchWindowProcessor.process :297-333). The selector removes the previous batch's events from
// the aggregator states, so every key of the previous batch ends empty: count 0, every other
// aggregator null (Sum/Avg return null at count 0, Min/Max at an empty deque). Its expired row is
// therefore the previous flush's current row of that key with ts = the flush clock and constant
// values — nothing needs re-aggregating. With `all events`, QuerySelector.processInBatchGroupBy
// (:315-374) keeps one row per key (LinkedHashMap.put: the LAST event's row at the FIRST
// occurrence's position), so a key present in both batches shows its current row at its position in
// the expired part; keys new in the current batch follow in their first-occurrence order.
// The kernels below assemble the output flushes from one source array = [carried rows of the last
// flush of an earlier call] + [this call's current rows].
#include <hip/hip_runtime.h>

#include "sh_device.h"
#include "sh_internal.h"

namespace shd {

constexpr u32 kXEmpty = 0xFFFFFFFFu;

__device__ __forceinline__ u64 x_packed_key(const i64* keys, i64 stride, int nk, i64 r) {
    if (nk == 0) return 0;
    if (nk == 1) return (u64)keys[r];
    return ((u64)(u32)keys[r] << 32) | (u64)(u32)keys[stride + r];
}

// largest i with cum[i] <= g (cum[0] = 0, non-decreasing)
__device__ __forceinline__ int x_find(const i64* cum, int n, i64 g) {
    int lo = 0, hi = n - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (cum[mid] <= g) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Current rows of the merged flushes into their flush's open-addressing table (keys within one
// flush are distinct, so an insert only claims the first free slot).
__global__ __launch_bounds__(kBlock) void k_x_insert(const XItem* items, const i64* cum, int n_items, i64 total,
                                                     const i64* s_keys, i64 S, int nk, u32* trow, u64* tkey) {
    const i64 g = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (g >= total) return;
    const int i = x_find(cum, n_items + 1, g);
    const XItem it = items[i];
    const i64 r = it.c_lo + (g - cum[i]);
    const u64 key = x_packed_key(s_keys, S, nk, r);
    if (it.pad) {  // (a dense id below the table size: its own slot, distinct within the flush)
        if (key < (u64)it.tab_size) trow[it.tab_off + (i64)key] = (u32)r;
        return;
    }
    const u32 mask = (u32)it.tab_size - 1;
    u32 h = (u32)mix64(key) & mask;
    for (;;) {
        if (atomicCAS(&trow[it.tab_off + h], kXEmpty, (u32)r) == kXEmpty) {
            tkey[it.tab_off + h] = key;
            return;
        }
        h = (h + 1) & mask;
    }
}

// Expired rows of the merged flushes look up their key among the flush's current rows: match[r] =
// that current row (or -1); the matched current row is not emitted a second time.
__global__ __launch_bounds__(kBlock) void k_x_probe(const XItem* items, const i64* cum, int n_items, i64 total,
                                                    const i64* s_keys, i64 S, int nk, const u32* trow, const u64* tkey,
                                                    int* match, u32* keep, u32* item_matched) {
    const i64 g = (i64)blockIdx.x * kBlock + threadIdx.x;
    const bool valid = g < total;
    int i = 0;
    bool mt = false;
    if (valid) {
        i = x_find(cum, n_items + 1, g);
        const XItem it = items[i];
        const i64 r = it.p_lo + (g - cum[i]);
        const u64 key = x_packed_key(s_keys, S, nk, r);
        int m = -1;
        if (it.pad) {  // (direct table: the id is the slot)
            const u32 t = key < (u64)it.tab_size ? trow[it.tab_off + (i64)key] : kXEmpty;
            m = t == kXEmpty ? -1 : (int)t;
        } else {
            const u32 mask = (u32)it.tab_size - 1;
            u32 h = (u32)mix64(key) & mask;
            for (;;) {
                const u32 t = trow[it.tab_off + h];
                if (t == kXEmpty) break;
                if (tkey[it.tab_off + h] == key) { m = (int)t; break; }
                h = (h + 1) & mask;
            }
        }
        match[r] = m;
        if (m >= 0) {
            keep[m] = 0;
            mt = true;
        }
    }
    // the matched count per flush: one atomic per block when the block's rows belong to one flush (the
    // usual case: a flush has ~100k rows) — per-row, even per-wave atomics on a few counters serialise at
    // the L2 (C2 `insert all events`: ~1600 waves per flush counter)
    __shared__ int s_item[kBlock / 64];
    __shared__ u32 s_cnt[kBlock / 64];
    const int w = threadIdx.x >> 6;
    const int i0 = __shfl(i, 0, 64);  // lane 0 holds the wave's smallest g: valid if any lane is
    const u64 same = __ballot(!valid || i == i0);
    const u64 b = __ballot(mt);
    if (same == ~0ull) {
        if ((threadIdx.x & 63) == 0) { s_item[w] = b ? i0 : -1; s_cnt[w] = (u32)__popcll(b); }
    } else {
        if ((threadIdx.x & 63) == 0) { s_item[w] = -1; s_cnt[w] = 0; }
        if (mt) atomicAdd(&item_matched[i], 1u);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        int cur = -1;
        u32 acc = 0;
        for (int x = 0; x < kBlock / 64; x++) {
            if (s_item[x] < 0) continue;
            if (s_item[x] != cur) {
                if (cur >= 0 && acc) atomicAdd(&item_matched[cur], acc);
                cur = s_item[x];
                acc = 0;
            }
            acc += s_cnt[x];
        }
        if (cur >= 0 && acc) atomicAdd(&item_matched[cur], acc);
    }
}

__device__ __forceinline__ void x_copy_current(i64 r, i64 o, i64 S, i64 T, int nk, int na, const i64* s_ts,
                                               const i64* s_keys, const u64* s_vals, const unsigned char* s_nulls,
                                               const i64* s_rep, XOut out) {
    out.ts[o] = s_ts[r];
    out.expired[o] = 0;
    out.rep[o] = s_rep[r];
    for (int k = 0; k < nk; k++) out.keys[(size_t)k * T + o] = s_keys[(size_t)k * S + r];
    for (int a = 0; a < na; a++) {
        out.vals[(size_t)a * T + o] = s_vals[(size_t)a * S + r];
        out.nulls[(size_t)a * T + o] = s_nulls[(size_t)a * S + r];
    }
}

// One output row per thread: position k of flush i is an expired row (k < p_n: the previous
// batch's row, or the matched current row when merged) or a current row in first-occurrence order.
__global__ __launch_bounds__(kBlock) void k_x_scatter(const XItem* items, const i64* cum, int n_items, i64 total,
                                                      const i64* s_ts, const i64* s_keys, const u64* s_vals,
                                                      const unsigned char* s_nulls, const i64* s_rep, i64 S, int nk,
                                                      int na, u32 count_mask, const int* match, const u32* keep,
                                                      const u32* rank, i64 T, XOut out) {
    const i64 g = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (g >= total) return;
    const int i = x_find(cum, n_items + 1, g);
    const XItem it = items[i];
    const i64 k = g - cum[i];
    if (k < it.p_n) {
        const i64 r = it.p_lo + k;
        const i64 o = it.out_base + k;
        const int m = it.tab_size > 0 ? match[r] : -1;
        if (out.order) out.order[o] = out.s_order[r];  // (a merged current row takes this place)
        if (m >= 0) {
            x_copy_current(m, o, S, T, nk, na, s_ts, s_keys, s_vals, s_nulls, s_rep, out);
            return;
        }
        out.ts[o] = it.xts;
        out.expired[o] = 1;
        out.rep[o] = s_rep[r];
        for (int kk = 0; kk < nk; kk++) out.keys[(size_t)kk * T + o] = s_keys[(size_t)kk * S + r];
        for (int a = 0; a < na; a++) {
            const bool cnt = (count_mask >> a) & 1u;
            out.vals[(size_t)a * T + o] = 0;
            out.nulls[(size_t)a * T + o] = cnt ? 0 : 1;
        }
        return;
    }
    const i64 r = it.c_lo + (k - it.p_n);
    if (!keep[r]) return;
    const i64 o = it.out_base + it.p_n + (i64)(rank[r] - rank[it.c_lo]);
    if (out.order) out.order[o] = out.s_order[r];
    x_copy_current(r, o, S, T, nk, na, s_ts, s_keys, s_vals, s_nulls, s_rep, out);
}

void launch_x_merge(hipStream_t s, const XItem* items, const i64* cum_c, const i64* cum_p, int n_items, i64 tot_c,
                    i64 tot_p, const i64* s_keys, i64 S, int nk, u32* trow, u64* tkey, int* match, u32* keep,
                    u32* item_matched) {
    if (tot_c > 0)
        hipLaunchKernelGGL(k_x_insert, dim3((unsigned)((tot_c + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, items, cum_c,
                           n_items, tot_c, s_keys, S, nk, trow, tkey);
    if (tot_p > 0)
        hipLaunchKernelGGL(k_x_probe, dim3((unsigned)((tot_p + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, items, cum_p,
                           n_items, tot_p, s_keys, S, nk, trow, tkey, match, keep, item_matched);
}

void launch_x_scatter(hipStream_t s, const XItem* items, const i64* cum, int n_items, i64 total, const i64* s_ts,
                      const i64* s_keys, const u64* s_vals, const unsigned char* s_nulls, const i64* s_rep, i64 S,
                      int nk, int na, u32 count_mask, const int* match, const u32* keep, const u32* rank, i64 T,
                      XOut out) {
    if (total <= 0) return;
    hipLaunchKernelGGL(k_x_scatter, dim3((unsigned)((total + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, items, cum,
                       n_items, total, s_ts, s_keys, s_vals, s_nulls, s_rep, S, nk, na, count_mask, match, keep, rank,
                       T, out);
}

// ---- pass-through batch queries (`select *`, QuerySelector.processNoGroupBy :161-205): every
// passing event of a closed batch is a row --------------------------------------------------------
__device__ __forceinline__ bool pass_at(i64 c, i64 n_pend, const u32* new_pos) {
    return c < n_pend || new_pos[c - n_pend] != kNoPos;
}

// (segments sorted and disjoint; they cover [0, hi) but where an externalTimeBatch timeout left a
// batch's events out: those are in no segment)
__device__ __forceinline__ bool in_segs(i64 c, const Segment* segs, int nseg) {
    int a = 0, b = nseg;  // first segment with lo > c
    while (a < b) {
        const int m = (a + b) >> 1;
        if (segs[m].lo <= c) a = m + 1; else b = m;
    }
    return a > 0 && c < segs[a - 1].hi;
}

__global__ __launch_bounds__(kBlock) void k_pass_flags(i64 hi, i64 n_pend, const u32* new_pos, const Segment* segs,
                                                       int nseg, u32* f) {
    const i64 c = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (c > hi) return;
    f[c] = c < hi && pass_at(c, n_pend, new_pos) && in_segs(c, segs, nseg) ? 1u : 0u;
}

__global__ __launch_bounds__(kBlock) void k_pass_rows(i64 hi, i64 n_pend, const u32* new_pos, const u32* pos,
                                                      const i64* pend_ts, const u64* pend_gidx, const i64* ts,
                                                      i64 seq_base, i64* out_ts, i64* out_rep) {
    const i64 c = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (c >= hi || pos[c + 1] == pos[c]) return;  // (not passing, or in no segment)
    const i64 o = pos[c];
    out_ts[o] = c < n_pend ? pend_ts[c] : ts[c - n_pend];
    out_rep[o] = c < n_pend ? (i64)pend_gidx[c] : seq_base + (c - n_pend);
}

__global__ void k_pass_seg_rows(const Segment* segs, int nseg, const u32* pos, u32* seg_rows, u32* n_rows) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nseg) seg_rows[i] = pos[segs[i].hi] - pos[segs[i].lo];
    if (i == nseg - 1) *n_rows = pos[segs[i].hi];
}

void launch_pass_rows(hipStream_t s, i64 hi, i64 n_pend, const u32* new_pos, u32* pos, i64* tmp, const i64* pend_ts,
                      const u64* pend_gidx, const i64* ts, i64 seq_base, const Segment* segs, int nseg, i64* out_ts,
                      i64* out_rep, u32* seg_rows, u32* n_rows) {
    const unsigned g = (unsigned)((hi + 1 + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_pass_flags, dim3(g), dim3(kBlock), 0, s, hi, n_pend, new_pos, segs, nseg, pos);
    launch_scan_sum_large_u32(s, pos, hi + 1, tmp);
    hipLaunchKernelGGL(k_pass_rows, dim3(g), dim3(kBlock), 0, s, hi, n_pend, new_pos, pos, pend_ts, pend_gidx, ts,
                       seq_base, out_ts, out_rep);
    hipLaunchKernelGGL(k_pass_seg_rows, dim3((nseg + 255) / 256), dim3(256), 0, s, segs, nseg, pos, seg_rows, n_rows);
}

}  // namespace shd
