// sh_rate_kernels.hip — `output [all|first|last] every N events` on the GPU: the output rate limiters
// of a query (core/query/output/ratelimit/event/*OutputRateLimiter.java) over the rows the selector
// emitted, in stream order. A row's fate depends only on its position in the output sequence (and
// on its group key for the group-by variants), so each limiter is a flag per row, a prefix over the
// flags and a gather of the kept rows; rows waiting for their group of N travel to the next call.
//
// Rows of one call: the source array [carried rows | this call's rows] (ALL and LAST group-by carry
// the rows of their open group). Every kept row records the input flush whose processing emits it
// (the flush holding the row whose arrival completes its group), which gives the output flushes.
#include <hip/hip_runtime.h>

#include "sh_device.h"
#include "sh_internal.h"

namespace shd {

__device__ __forceinline__ int rate_flush_of(const i64* off, int nf, i64 r) {  // largest f with off[f] <= r
    int lo = 0, hi = nf - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (off[mid] <= r) lo = mid; else hi = mid - 1;
    }
    return lo;
}

__device__ __forceinline__ u64 rate_key(const i64* keys, i64 stride, int nk, i64 r) {
    if (nk == 0) return 0;
    if (nk == 1) return (u64)keys[r];
    return ((u64)(u32)keys[r] << 32) | (u64)(u32)keys[stride + r];
}

// Positional limiters (no group key), one thread per source row; flag[n_src] = 0 closes the scan.
//  ALL (AllPerEvent :48-77): rows leave in groups of N when the group's N-th row arrives.
//  FIRST (FirstPerEvent :48-72): counter 1 emits, counter N resets; N = 1 never resets (only the
//   stream's first row is kept), as the reference's `else if` ordering implies.
//  LAST (LastPerEvent :47-71): the N-th of every N.
__global__ __launch_bounds__(kBlock) void k_rate_pos(i64 n_src, i64 n_carry, int mode, i64 N, i64 seq0,
                                                    const i64* __restrict__ flush_off, int nf, u32* flag, int* eflush,
                                                    u32* src) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i > n_src) return;
    if (i == n_src) { flag[i] = 0; return; }
    u32 f;
    i64 at = i;  // the row whose arrival emits row i
    if (mode == SH_RATE_ALL) {
        at = (i / N) * N + N - 1;
        f = at < n_src ? 1u : 0u;
    } else if (mode == SH_RATE_FIRST) {
        const i64 s = seq0 + i;
        f = N == 1 ? (s == 0) : (s % N == 0);
    } else {
        f = (seq0 + i) % N == N - 1;
    }
    flag[i] = f;
    src[i] = (u32)i;
    eflush[i] = f ? rate_flush_of(flush_off, nf, at - n_carry) : 0;
}

// ---- group-by limiters over the rows sorted (stably) by packed key --------------------------------
__global__ __launch_bounds__(kBlock) void k_rate_pack(i64 n, const i64* __restrict__ keys, i64 stride, int nk,
                                                     u64* skey, u32* idx) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    skey[i] = rate_key(keys, stride, nk, i);
    idx[i] = (u32)i;
}

// hd[i] = 1 where a segment of equal (key[, window of N rows]) starts in sorted order; hd[n] = 0
__global__ __launch_bounds__(kBlock) void k_rate_heads(i64 n, const u64* __restrict__ skey, const u32* __restrict__ idx,
                                                      i64 N, int with_win, u32* hd, u32* pos) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i > n) return;
    u32 h = 0;
    if (i < n) {
        h = i == 0 || skey[i - 1] != skey[i] || (with_win && idx[i - 1] / N != idx[i] / N);
    }
    hd[i] = h;
    pos[i] = h;
}

// starts[g] = first sorted position of segment g (pos = exclusive scan of hd); starts[n_seg] = n
__global__ __launch_bounds__(kBlock) void k_rate_starts(i64 n, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                       u32* starts) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i > n) return;
    if (i == n) starts[pos[n]] = (u32)n;
    else if (hd[i]) starts[pos[i]] = (u32)i;
}

// FirstGroupByPerEvent :48-77, per key: the stored count c (absent = 0) goes 0 -> 1 (emit), c ->
// c + 1, and N - 1 -> absent; so an occurrence emits when (c0 + j) % N == 0, and with N = 1 only the
// key's very first occurrence emits (the count then grows without reset). The table maps a packed key
// to its count across calls; tc < 0 marks a free slot. One thread per segment (the call's distinct
// keys): a lookup pass over the keys published by earlier calls (a found slot belongs to this key
// alone), then the new keys claim free slots with a CAS on the count word and never compare keys, so
// no thread reads a slot another thread of the same kernel is filling.
__device__ __forceinline__ i64 rate_first_next(i64 c0, i64 len, i64 N) { return N == 1 ? c0 + len : (c0 + len) % N; }

__global__ __launch_bounds__(kBlock) void k_rate_first_lookup(i64 n, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                             const u32* __restrict__ starts, const u64* __restrict__ skey,
                                                             i64 N, const u64* __restrict__ tk, i64* tc, u32 tmask,
                                                             i64* seg_c0, u32* seg_new) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || !hd[i]) return;
    const u32 g = pos[i];
    const i64 len = (i64)starts[g + 1] - i;
    const u64 key = skey[i];
    u32 h = (u32)mix64(key) & tmask;
    for (;;) {
        const i64 c = tc[h];
        if (c < 0) {  // absent: inserted by k_rate_first_insert
            seg_c0[g] = 0;
            seg_new[g] = 1;
            return;
        }
        if (tk[h] == key) {
            seg_c0[g] = c;
            seg_new[g] = 0;
            tc[h] = rate_first_next(c, len, N);
            return;
        }
        h = (h + 1) & tmask;
    }
}

__global__ __launch_bounds__(kBlock) void k_rate_first_insert(i64 n, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                             const u32* __restrict__ starts, const u64* __restrict__ skey,
                                                             const u32* __restrict__ seg_new, i64 N, u64* tk, i64* tc,
                                                             u32 tmask, u32* n_keys) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || !hd[i]) return;
    const u32 g = pos[i];
    if (!seg_new[g]) return;
    const i64 len = (i64)starts[g + 1] - i;
    const u64 key = skey[i];
    const unsigned long long cnt = (unsigned long long)rate_first_next(0, len, N);
    u32 h = (u32)mix64(key) & tmask;
    for (;;) {
        if (atomicCAS((unsigned long long*)&tc[h], ~0ull, cnt) == ~0ull) {
            tk[h] = key;
            atomicAdd(n_keys, 1u);
            return;
        }
        h = (h + 1) & tmask;
    }
}

// the table lives across calls: concurrent claims in a rehash are atomic on the count word
__global__ __launch_bounds__(kBlock) void k_rate_rehash(i64 old_cap, const u64* __restrict__ otk,
                                                       const i64* __restrict__ otc, u64* tk, i64* tc, u32 tmask) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= old_cap || otc[i] < 0) return;
    const u64 key = otk[i];
    u32 h = (u32)mix64(key) & tmask;
    for (;;) {
        if (atomicCAS((unsigned long long*)&tc[h], ~0ull, (unsigned long long)otc[i]) == ~0ull) {
            tk[h] = key;
            return;
        }
        h = (h + 1) & tmask;
    }
}

__global__ __launch_bounds__(kBlock) void k_rate_first_rows(i64 n, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                           const u32* __restrict__ starts, const u32* __restrict__ idx,
                                                           const i64* __restrict__ seg_c0, i64 N,
                                                           const i64* __restrict__ flush_off, int nf, u32* flag,
                                                           int* eflush) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const u32 g = pos[i] + hd[i] - 1;
    const i64 j = i - (i64)starts[g];
    const i64 c0 = seg_c0[g];
    const bool emit = N == 1 ? (c0 == 0 && j == 0) : ((c0 + j) % N == 0);
    if (!emit) return;
    const u32 q = idx[i];
    flag[q] = 1;
    eflush[q] = rate_flush_of(flush_off, nf, (i64)q);
}

// LastGroupByPerEvent :51-83: within each complete window of N rows, a key's first position (the
// LinkedHashMap keeps the first insertion's slot) shows its last row of the window.
__global__ __launch_bounds__(kBlock) void k_rate_last_seg(i64 n, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                         const u32* __restrict__ starts, const u32* __restrict__ idx,
                                                         i64 N, i64 n_carry, const i64* __restrict__ flush_off, int nf,
                                                         u32* flag, u32* src, int* eflush) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || !hd[i]) return;
    const u32 g = pos[i];
    const u32 r = idx[i];
    flag[r] = 1;
    src[r] = idx[starts[g + 1] - 1];
    eflush[r] = rate_flush_of(flush_off, nf, ((i64)r / N + 1) * N - 1 - n_carry);
}

__global__ void k_rate_clear(i64 n, u32* src, u32* flag) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i <= n) flag[i] = 0;
    if (i < n) src[i] = (u32)i;
}

// kept rows gathered in source order: out[o] = source[src[i]] for flagged i (o = prefix of flags),
// with the index of the input flush whose processing emits them
__global__ __launch_bounds__(kBlock) void k_rate_gather(i64 n, const u32* __restrict__ flag, const u32* __restrict__ pre,
                                                       const u32* __restrict__ src, const int* __restrict__ eflush,
                                                       RateRows in, i64 in_stride, RateRows out, i64 T, int nk, int na,
                                                       int* out_flush) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || !flag[i]) return;
    const i64 o = pre[i];
    const u32 s = src[i];
    out.ts[o] = in.ts[s];
    out.expired[o] = in.expired[s];
    out.rep[o] = in.rep[s];
    for (int k = 0; k < nk; k++) out.keys[(size_t)k * T + o] = in.keys[(size_t)k * in_stride + s];
    for (int a = 0; a < na; a++) {
        out.vals[(size_t)a * T + o] = in.vals[(size_t)a * in_stride + s];
        out.nulls[(size_t)a * T + o] = in.nulls[(size_t)a * in_stride + s];
    }
    out_flush[o] = eflush[i];
}

static inline unsigned grid_of(i64 n) { return (unsigned)((n + kBlock - 1) / kBlock); }

void launch_rate_pos(hipStream_t s, i64 n_src, i64 n_carry, int mode, i64 N, i64 seq0, const i64* flush_off, int nf,
                     u32* flag, int* eflush, u32* src) {
    hipLaunchKernelGGL(k_rate_pos, dim3(grid_of(n_src + 1)), dim3(kBlock), 0, s, n_src, n_carry, mode, N, seq0, flush_off,
                       nf, flag, eflush, src);
}

void launch_rate_clear(hipStream_t s, i64 n, u32* src, u32* flag) {
    hipLaunchKernelGGL(k_rate_clear, dim3(grid_of(n + 1)), dim3(kBlock), 0, s, n, src, flag);
}

void launch_rate_pack(hipStream_t s, i64 n, const i64* keys, i64 stride, int nk, u64* skey, u32* idx) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_rate_pack, dim3(grid_of(n)), dim3(kBlock), 0, s, n, keys, stride, nk, skey, idx);
}

void launch_rate_segments(hipStream_t s, i64 n, const u64* skey, const u32* idx, i64 N, int with_win, u32* hd, u32* pos,
                          u32* starts, i64* tmp) {
    hipLaunchKernelGGL(k_rate_heads, dim3(grid_of(n + 1)), dim3(kBlock), 0, s, n, skey, idx, N, with_win, hd, pos);
    launch_scan_sum_large_u32(s, pos, n + 1, tmp);
    hipLaunchKernelGGL(k_rate_starts, dim3(grid_of(n + 1)), dim3(kBlock), 0, s, n, hd, pos, starts);
}

void launch_rate_first(hipStream_t s, i64 n, const u32* hd, const u32* pos, const u32* starts, const u64* skey,
                       const u32* idx, i64 N, u64* tk, i64* tc, u32 tmask, i64* seg_c0, u32* seg_new, u32* n_keys,
                       const i64* flush_off, int nf, u32* flag, int* eflush) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_rate_first_lookup, dim3(grid_of(n)), dim3(kBlock), 0, s, n, hd, pos, starts, skey, N, tk, tc,
                       tmask, seg_c0, seg_new);
    hipLaunchKernelGGL(k_rate_first_insert, dim3(grid_of(n)), dim3(kBlock), 0, s, n, hd, pos, starts, skey, seg_new, N, tk,
                       tc, tmask, n_keys);
    hipLaunchKernelGGL(k_rate_first_rows, dim3(grid_of(n)), dim3(kBlock), 0, s, n, hd, pos, starts, idx, seg_c0, N,
                       flush_off, nf, flag, eflush);
}

void launch_rate_rehash(hipStream_t s, i64 old_cap, const u64* otk, const i64* otc, u64* tk, i64* tc, u32 tmask) {
    if (old_cap <= 0) return;
    hipLaunchKernelGGL(k_rate_rehash, dim3(grid_of(old_cap)), dim3(kBlock), 0, s, old_cap, otk, otc, tk, tc, tmask);
}

void launch_rate_last(hipStream_t s, i64 n, const u32* hd, const u32* pos, const u32* starts, const u32* idx, i64 N,
                      i64 n_carry, const i64* flush_off, int nf, u32* flag, u32* src, int* eflush) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_rate_last_seg, dim3(grid_of(n)), dim3(kBlock), 0, s, n, hd, pos, starts, idx, N, n_carry,
                       flush_off, nf, flag, src, eflush);
}

void launch_rate_gather(hipStream_t s, i64 n, const u32* flag, const u32* pre, const u32* src, const int* eflush,
                        RateRows in, i64 in_stride, RateRows out, i64 T, int nk, int na, int* out_flush) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_rate_gather, dim3(grid_of(n)), dim3(kBlock), 0, s, n, flag, pre, src, eflush, in, in_stride,
                       out, T, nk, na, out_flush);
}

// ---- `output first every <t>` (core/query/output/ratelimit/time/): the playback clock of the chunk
// (the input flush) decides. FirstPerTimeOutputRateLimiter.process :54-78 sends a chunk's FIRST event
// when no output happened yet or outputTime + t <= now (chosen per flush on the host, in order), then
// outputTime = now. Every row also gets its emitting flush and source index here.
__global__ __launch_bounds__(kBlock) void k_rate_ftime_rows(i64 n, const i64* __restrict__ foff, int nf,
                                                           const unsigned char* __restrict__ chosen, u32* flag,
                                                           int* eflush, u32* src) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i > n) return;
    if (i == n) { flag[n] = 0; return; }
    const int f = rate_flush_of(foff, nf, i);
    eflush[i] = f;
    src[i] = (u32)i;
    flag[i] = chosen ? (chosen[f] && foff[f] == i) : 0u;
}

void launch_rate_ftime_rows(hipStream_t s, i64 n, const i64* foff, int nf, const unsigned char* chosen, u32* flag,
                            int* eflush, u32* src) {
    hipLaunchKernelGGL(k_rate_ftime_rows, dim3(grid_of(n + 1)), dim3(kBlock), 0, s, n, foff, nf, chosen, flag, eflush,
                       src);
}

// FirstGroupByPerTimeOutputRateLimiter.process :54-80: per group key the time of its last output row
// (groupByOutputTime); a row is sent when its key has none or that time + t <= the chunk's clock. One
// thread per key segment of the call (rows of one key in stream order); the key -> time table keeps
// the keys of earlier calls (tk == kEmptyKey: free; a thread only ever claims or reads its own key's slot).
__global__ __launch_bounds__(kBlock) void k_rate_ftime_walk(i64 n, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                           const u32* __restrict__ starts, const u64* __restrict__ skey,
                                                           const u32* __restrict__ idx, const i64* __restrict__ foff,
                                                           const i64* __restrict__ fclk, int nf, i64 T, u64* tk, i64* tt,
                                                           u32 tmask, u32* flag, u32* n_new) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n || !hd[i]) return;
    const u32 g = pos[i];
    const i64 end = starts[g + 1];
    const u64 key = skey[i];
    u32 h = (u32)mix64(key) & tmask;
    bool has = true;
    for (;;) {
        const u64 k0 = tk[h];
        if (k0 == key) break;
        if (k0 == kEmptyKey) {
            const u64 old = atomicCAS(&tk[h], kEmptyKey, key);
            if (old == kEmptyKey) { has = false; atomicAdd(n_new, 1u); break; }
            if (old == key) break;
        }
        h = (h + 1) & tmask;
    }
    i64 last = has ? tt[h] : 0;
    for (i64 j = i; j < end; j++) {
        const u32 r = idx[j];
        const i64 c = fclk[rate_flush_of(foff, nf, r)];
        if (!has || last + T <= c) {
            flag[r] = 1;
            has = true;
            last = c;
        }
    }
    tt[h] = last;
}

__global__ __launch_bounds__(kBlock) void k_rate_ftime_rehash(i64 old_cap, const u64* __restrict__ otk,
                                                             const i64* __restrict__ ott, u64* tk, i64* tt, u32 tmask) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= old_cap) return;
    const u64 key = otk[i];
    if (key == kEmptyKey) return;
    u32 h = (u32)mix64(key) & tmask;
    while (atomicCAS(&tk[h], kEmptyKey, key) != kEmptyKey) h = (h + 1) & tmask;
    tt[h] = ott[i];
}

void launch_rate_ftime_walk(hipStream_t s, i64 n, const u32* hd, const u32* pos, const u32* starts, const u64* skey,
                            const u32* idx, const i64* foff, const i64* fclk, int nf, i64 T, u64* tk, i64* tt, u32 tmask,
                            u32* flag, u32* n_new) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_rate_ftime_walk, dim3(grid_of(n)), dim3(kBlock), 0, s, n, hd, pos, starts, skey, idx, foff, fclk,
                       nf, T, tk, tt, tmask, flag, n_new);
}

void launch_rate_ftime_rehash(hipStream_t s, i64 old_cap, const u64* otk, const i64* ott, u64* tk, i64* tt, u32 tmask) {
    if (old_cap <= 0) return;
    hipLaunchKernelGGL(k_rate_ftime_rehash, dim3(grid_of(old_cap)), dim3(kBlock), 0, s, old_cap, otk, ott, tk, tt, tmask);
}

// ---- one limiter per partition instance (PartitionRuntimeImpl clones the query, so each partition
// has its own OutputRateLimiter): the partition lanes' rows carry their partition slot. Rows sorted
// stably by partition (carried rows first) give every row its ordinal within its partition's
// sequence; the positional limiters run on those ordinals with a per-partition counter. ---------------
__global__ __launch_bounds__(kBlock) void k_ratep_pack(i64 S, i64 nc, const u32* __restrict__ c_part,
                                                      const u32* __restrict__ in_part, u64* skey, u32* idx) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= S) return;
    skey[i] = i < nc ? c_part[i] : in_part[i - nc];
    idx[i] = (u32)i;
}

// per sorted position i (segment = one partition's rows in source order): ordinal o, the partition's
// row count tot. ALL: complete groups of N leave at their last row (keep = the open group's rows);
// FIRST / LAST: the partition's running count pseq decides.
__global__ __launch_bounds__(kBlock) void k_ratep_flags(i64 S, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                       const u32* __restrict__ starts, const u64* __restrict__ skey,
                                                       const u32* __restrict__ idx, int mode, i64 N, i64 nc,
                                                       const i64* __restrict__ pseq, const i64* __restrict__ flush_off,
                                                       int nf, u32* flag, int* eflush, u32* src, u32* keep) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i > S) return;
    if (i == S) { flag[S] = 0; keep[S] = 0; return; }
    const u32 g = pos[i] + hd[i] - 1;
    const i64 lo = starts[g], o = i - lo, tot = (i64)starts[g + 1] - lo;
    const u32 r = idx[i];
    u32 f = 0, k = 0;
    i64 at = r;
    if (mode == SH_RATE_ALL) {
        if (o < tot / N * N) {
            f = 1;
            at = idx[lo + (o / N + 1) * N - 1];
        } else {
            k = 1;
        }
    } else {
        const i64 sq = pseq[skey[i]] + o;
        f = mode == SH_RATE_FIRST ? (N == 1 ? sq == 0 : sq % N == 0) : (sq % N == N - 1);
    }
    flag[r] = f;
    keep[r] = k;
    src[r] = r;
    eflush[r] = f ? rate_flush_of(flush_off, nf, at - nc) : 0;
}

// after the flags: the partitions' counters advance by their rows of the call (FIRST with N == 1 keeps
// the count growing: only the partition's very first row is ever sent)
__global__ __launch_bounds__(kBlock) void k_ratep_advance(i64 S, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                         const u32* __restrict__ starts, const u64* __restrict__ skey,
                                                         int mode, i64 N, i64* pseq) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= S || !hd[i]) return;
    const u32 g = pos[i];
    const i64 tot = (i64)starts[g + 1] - i;
    const i64 v = pseq[skey[i]] + tot;
    pseq[skey[i]] = (mode == SH_RATE_FIRST && N == 1) ? v : v % N;
}

// `output first every <t>` without group-by, per partition: a flush (one chunk, one partition) sends its
// first row when the partition has no output time yet or that time + t <= the flush's clock. Flushes
// sorted stably by partition; one thread walks a partition's flushes in order.
__global__ __launch_bounds__(kBlock) void k_ratep_fparts(int nf, const i64* __restrict__ foff, const u32* __restrict__ in_part,
                                                        u32 none, u64* fkey, u32* fidx) {
    const int f = blockIdx.x * kBlock + threadIdx.x;
    if (f >= nf) return;
    fkey[f] = foff[f + 1] > foff[f] ? in_part[foff[f]] : none;
    fidx[f] = (u32)f;
}

__global__ __launch_bounds__(kBlock) void k_ratep_ftime(int nf, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                       const u32* __restrict__ starts, const u64* __restrict__ fkey,
                                                       const u32* __restrict__ fidx, const i64* __restrict__ fclk, u32 none,
                                                       i64 T, unsigned char* has, i64* last, unsigned char* chosen) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nf || !hd[i]) return;
    const u32 g = pos[i];
    const u64 p = fkey[i];
    if (p == none) return;
    unsigned char h = has[p];
    i64 t = last[p];
    for (u32 j = (u32)i; j < starts[g + 1]; j++) {
        const u32 f = fidx[j];
        if (!h || t + T <= fclk[f]) {
            chosen[f] = 1;
            h = 1;
            t = fclk[f];
        }
    }
    has[p] = h;
    last[p] = t;
}

// flagged source rows -> (emitting flush, row to show) lists, in source order (src: the row whose data
// the flagged place shows; null = itself)
__global__ __launch_bounds__(kBlock) void k_ratep_list(i64 S, const u32* __restrict__ flag, const u32* __restrict__ pre,
                                                      const int* __restrict__ eflush, const u32* __restrict__ src,
                                                      u64* okey, u32* olist) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= S || !flag[i]) return;
    okey[pre[i]] = (u64)(u32)eflush[i];
    olist[pre[i]] = src ? src[i] : (u32)i;
}

// rows of a list (source indices) -> a row set of stride T; out_flush from okey when given
__global__ __launch_bounds__(kBlock) void k_ratep_gather(i64 T, const u32* __restrict__ list, const u64* __restrict__ okey,
                                                        RateRows in, i64 in_stride, const u32* __restrict__ in_part,
                                                        RateRows out, int nk, int na, int* out_flush, u32* out_part) {
    const i64 o = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (o >= T) return;
    const u32 s = list[o];
    out.ts[o] = in.ts[s];
    out.expired[o] = in.expired[s];
    out.rep[o] = in.rep[s];
    for (int k = 0; k < nk; k++) out.keys[(size_t)k * T + o] = in.keys[(size_t)k * in_stride + s];
    for (int a = 0; a < na; a++) {
        out.vals[(size_t)a * T + o] = in.vals[(size_t)a * in_stride + s];
        out.nulls[(size_t)a * T + o] = in.nulls[(size_t)a * in_stride + s];
    }
    if (out_flush) out_flush[o] = (int)okey[o];
    if (out_part) out_part[o] = in_part[s];
}

// (partition slot, 32-bit group key) as one sort key: the per-partition keyed limiters as one keyed limiter
__global__ __launch_bounds__(kBlock) void k_ratep_pkey(i64 n, const i64* __restrict__ keys, const u32* __restrict__ part,
                                                      u64* skey, u32* idx) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    skey[i] = ((u64)part[i] << 32) | (u64)(u32)keys[i];
    idx[i] = (u32)i;
}

void launch_ratep_pkey(hipStream_t s, i64 n, const i64* keys, const u32* part, u64* skey, u32* idx) {
    if (n > 0) hipLaunchKernelGGL(k_ratep_pkey, dim3(grid_of(n)), dim3(kBlock), 0, s, n, keys, part, skey, idx);
}

// LastGroupByPerEvent per partition instance (grouped by another column): every row's ordinal in its
// partition's sequence (carried rows first) names its window of N; rows of complete windows are keyed
// (partition, group key) for the second sort, the open window's rows are carried
__global__ __launch_bounds__(kBlock) void k_ratep_lk_ord(i64 S, const u32* __restrict__ hd, const u32* __restrict__ pos,
                                                        const u32* __restrict__ starts, const u32* __restrict__ idx, i64 N,
                                                        const i64* __restrict__ keys, i64 kstride, const u32* __restrict__ sp,
                                                        i64* ord, u32* cidx, u32* keep, u64* skey, u32* sidx) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i > S) return;
    if (i == S) { keep[S] = 0; return; }
    const u32 g = pos[i] + hd[i] - 1;
    const i64 lo = starts[g], o = i - lo, tot = (i64)starts[g + 1] - lo;
    const u32 r = idx[i];
    ord[r] = o;
    const bool complete = o < tot / N * N;
    keep[r] = complete ? 0u : 1u;
    cidx[r] = complete ? idx[lo + (o / N + 1) * N - 1] : 0u;
    skey[r] = complete ? (((u64)sp[r] << 32) | (u64)(u32)keys[r]) : ~0ull;
    sidx[r] = r;
}

// heads of the (partition, key, window) runs of the key-sorted rows (source order inside a run)
__global__ __launch_bounds__(kBlock) void k_ratep_lk_heads(i64 n, const u64* __restrict__ skey, const u32* __restrict__ idx,
                                                          const i64* __restrict__ ord, i64 N, u32* hd, u32* pos) {
    const i64 j = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (j > n) return;
    u32 h = 0;
    if (j < n && skey[j] != ~0ull)
        h = j == 0 || skey[j] != skey[j - 1] || ord[idx[j]] / N != ord[idx[j - 1]] / N;
    hd[j] = h;
    pos[j] = h;
}

// per run: the flag at its first row, the data of its last row, emitted by the window's completing row
__global__ __launch_bounds__(kBlock) void k_ratep_lk_rows(i64 n, const u64* __restrict__ skey, const u32* __restrict__ hd,
                                                         const u32* __restrict__ idx, const u32* __restrict__ cidx,
                                                         const i64* __restrict__ ord, i64 N, i64 nc,
                                                         const i64* __restrict__ flush_off, int nf, u32* flag, u32* src,
                                                         int* eflush) {
    const i64 j = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (j >= n || !hd[j]) return;
    i64 e = j + 1;
    while (e < n && !hd[e] && skey[e] != ~0ull) e++;
    const u32 r = idx[j];
    flag[r] = 1;
    src[r] = idx[e - 1];
    eflush[r] = rate_flush_of(flush_off, nf, (i64)cidx[r] - nc);
}

void launch_ratep_last_keyed(hipStream_t s, i64 S, const u32* hd, const u32* pos, const u32* starts, const u32* idx, i64 N,
                             const i64* keys, i64 kstride, const u32* sp, i64* ord, u32* cidx, u32* keep, u64* skey,
                             u32* sidx) {
    hipLaunchKernelGGL(k_ratep_lk_ord, dim3(grid_of(S + 1)), dim3(kBlock), 0, s, S, hd, pos, starts, idx, N, keys, kstride,
                       sp, ord, cidx, keep, skey, sidx);
}

void launch_ratep_last_keyed_rows(hipStream_t s, i64 S, const u64* skey, const u32* idx, const u32* cidx, const i64* ord,
                                  i64 N, i64 nc, const i64* flush_off, int nf, u32* hd, u32* pos, u32* flag, u32* src,
                                  int* eflush) {
    hipLaunchKernelGGL(k_ratep_lk_heads, dim3(grid_of(S + 1)), dim3(kBlock), 0, s, S, skey, idx, ord, N, hd, pos);
    if (S > 0)
        hipLaunchKernelGGL(k_ratep_lk_rows, dim3(grid_of(S)), dim3(kBlock), 0, s, S, skey, hd, idx, cidx, ord, N, nc,
                           flush_off, nf, flag, src, eflush);
}

void launch_ratep_pack(hipStream_t s, i64 S, i64 nc, const u32* c_part, const u32* in_part, u64* skey, u32* idx) {
    if (S > 0) hipLaunchKernelGGL(k_ratep_pack, dim3(grid_of(S)), dim3(kBlock), 0, s, S, nc, c_part, in_part, skey, idx);
}

void launch_ratep_flags(hipStream_t s, i64 S, const u32* hd, const u32* pos, const u32* starts, const u64* skey,
                        const u32* idx, int mode, i64 N, i64 nc, i64* pseq, const i64* flush_off, int nf, u32* flag,
                        int* eflush, u32* src, u32* keep) {
    hipLaunchKernelGGL(k_ratep_flags, dim3(grid_of(S + 1)), dim3(kBlock), 0, s, S, hd, pos, starts, skey, idx, mode, N, nc,
                       pseq, flush_off, nf, flag, eflush, src, keep);
    if (mode != SH_RATE_ALL && S > 0)
        hipLaunchKernelGGL(k_ratep_advance, dim3(grid_of(S)), dim3(kBlock), 0, s, S, hd, pos, starts, skey, mode, N, pseq);
}

void launch_ratep_fparts(hipStream_t s, int nf, const i64* foff, const u32* in_part, u32 none, u64* fkey, u32* fidx) {
    if (nf > 0) hipLaunchKernelGGL(k_ratep_fparts, dim3(grid_of(nf)), dim3(kBlock), 0, s, nf, foff, in_part, none, fkey, fidx);
}

void launch_ratep_ftime(hipStream_t s, int nf, const u32* hd, const u32* pos, const u32* starts, const u64* fkey,
                        const u32* fidx, const i64* fclk, u32 none, i64 T, unsigned char* has, i64* last,
                        unsigned char* chosen) {
    if (nf > 0)
        hipLaunchKernelGGL(k_ratep_ftime, dim3(grid_of(nf)), dim3(kBlock), 0, s, nf, hd, pos, starts, fkey, fidx, fclk, none,
                           T, has, last, chosen);
}

void launch_ratep_list(hipStream_t s, i64 S, const u32* flag, const u32* pre, const int* eflush, const u32* src, u64* okey,
                       u32* olist) {
    if (S > 0) hipLaunchKernelGGL(k_ratep_list, dim3(grid_of(S)), dim3(kBlock), 0, s, S, flag, pre, eflush, src, okey, olist);
}

void launch_ratep_gather(hipStream_t s, i64 T, const u32* list, const u64* okey, RateRows in, i64 in_stride,
                         const u32* in_part, RateRows out, int nk, int na, int* out_flush, u32* out_part) {
    if (T > 0)
        hipLaunchKernelGGL(k_ratep_gather, dim3(grid_of(T)), dim3(kBlock), 0, s, T, list, okey, in, in_stride, in_part, out,
                           nk, na, out_flush, out_part);
}

}  // namespace shd
