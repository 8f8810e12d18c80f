// sh_plane_group_kernels.hip — `partition with (p of S) begin from S#window.lengthBatch(L) select g…,
// aggs group by g… insert [current|all|expired] events into O; end` with a group key other than the
// partition key, on gfx950.
//
// Every partition owns its own lengthBatch window (PartitionRuntimeImpl.initPartition :346-367). A batch
// the partition completes is one selector chunk (LengthBatchWindowProcessor.processFullBatchEvents
// :206-243): [the previous batch's events as EXPIRED, RESET, the batch's L events], and
// QuerySelector.processInBatchGroupBy (:315-374) keeps one row per group key in first-insertion order
// (LinkedHashMap.put). The RESET clears every group state, so a group's current row folds only its own
// events of the batch; its expired row is its previous-batch events removed again (count 0, the others
// null). Nothing here is sequential per partition: a partition's batches are fixed windows of L events
// of its run in stream order, so
//   1. the records of the push are appended to the carried ones (the partitions' open batches and,
//      with expired output, their last completed batch) and sorted stably by partition slot;
//   2. every sorted position knows its batch from its offset in the run (k_pg_assign) and emits up to
//      two entries — EXPIRED into the chunk of the next batch, CURRENT into its own — keyed
//      (chunk, group slot), where a chunk is named by the combined index of the event completing it;
//   3. the entries are sorted stably by that key (rocPRIM), a segment is one output row (k_pg_fold);
//   4. the rows are sorted by (chunk, first entry) and written in that order (k_pg_emit).
// The records of incomplete batches (and the last completed batch, for expired output) are carried to
// the next push in stream order (k_pg_assign marks them, k_pg_gather compacts them).
#include <rocprim/device/device_scan_by_key.hpp>

#include "sh_device.h"
#include "sh_sliding.h"
#include "sh_plane_group.h"

namespace shd {

// a row slot from one counter for every active lane of the wave: one atomic per wave (the rows' order is
// set by a later sort; per-row atomics on one counter serialise at the L2)
__device__ __forceinline__ u32 wave_row_slot(u32* ctr) {
    const u64 act = __ballot(1);
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __ffsll((long long)act) - 1;
    u32 base = 0;
    if (lane == leader) base = atomicAdd(ctr, (u32)__popcll(act));
    base = __shfl(base, leader, 64);
    return base + (u32)__popcll(act & ((1ull << lane) - 1ull));
}

namespace {

__device__ __forceinline__ bool g_worse(int kind, u64 cur, u64 v) {
    switch (kind) {
        case AK_MIN_L: return (i64)cur > (i64)v;
        case AK_MAX_L: return (i64)cur < (i64)v;
        case AK_MIN_D: return __longlong_as_double((i64)cur) > __longlong_as_double((i64)v);
        case AK_MAX_D: return __longlong_as_double((i64)cur) < __longlong_as_double((i64)v);
        case AK_MIN_F: return (float)__longlong_as_double((i64)cur) > (float)__longlong_as_double((i64)v);
        default: return (float)__longlong_as_double((i64)cur) < (float)__longlong_as_double((i64)v);
    }
}

__device__ __forceinline__ double g_num(const AggPlan& ap, int a, u64 x) {
    return (ap.kind[a] == AK_AVG && !is_fp(ap.vcol_type[ap.vcol[a]])) ? (double)(i64)x : __longlong_as_double((i64)x);
}

}  // namespace

// ---- 1. the push's records appended after the n_old carried ones (partition slot from the records
// kernel, group slot looked up here), and the carried ones counted into the per-partition totals ----
__global__ __launch_bounds__(kBlock) void k_pg_append(SlRecords rec, i64 M, i64 n_old, i64 seq_base, ColSet cols,
                                                     KeyPlan gkp, KeyTable gkt, int nv, PgRecs C, int xcol, int scol,
                                                     i64* xs) {
    const i64 r = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (r >= M) return;
    const i64 c = n_old + r;
    const u32 e = rec.raw[r];
    if (xcol >= 0) {
        C.x[c] = load_raw(cols, xcol, e);
        xs[c] = scol >= 0 ? load_raw(cols, scol, e) : 0;
    }
    C.ps[c] = rec.slot[r];
    C.gs[c] = key_slot(gkt, make_key(gkp, cols, e));
    C.ts[c] = rec.ts[r];
    C.seq[c] = seq_base + (i64)e;
    C.clk[c] = rec.clock[r];
    C.prev[c] = 0;
    for (int v = 0; v < nv; v++) C.vals[(size_t)v * C.cap + c] = rec.vals[(size_t)v * rec.cap + r];
}

__global__ __launch_bounds__(kBlock) void k_pg_count_old(PgRecs C, i64 n_old, u32* slot_cnt, u32* prev_cnt,
                                                        u32* pend_cnt) {
    const i64 c = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (c >= n_old) return;
    const u32 p = C.ps[c];
    if (slot_cnt) atomicAdd(&slot_cnt[p], 1u);  // (null: the offsets come from the sorted slots)
    if (C.prev[c]) atomicAdd(&prev_cnt[p], 1u);
    else if (pend_cnt) atomicAdd(&pend_cnt[p], 1u);
}

void launch_pg_append(hipStream_t s, SlRecords rec, i64 M, i64 n_old, i64 seq_base, ColSet cols, KeyPlan gkp,
                      KeyTable gkt, int nv, PgRecs C, u32* slot_cnt, u32* prev_cnt, int xcol, int scol, i64* xs,
                      u32* pend_cnt) {
    if (M > 0)
        hipLaunchKernelGGL(k_pg_append, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rec, M, n_old,
                           seq_base, cols, gkp, gkt, nv, C, xcol, scol, xs);
    if (n_old > 0)
        hipLaunchKernelGGL(k_pg_count_old, dim3((unsigned)((n_old + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, C,
                           n_old, slot_cnt, prev_cnt, pend_cnt);
}

// ---- externalTimeBatch (ExternalTimeBatchWindowProcessor.process :238-311 per partition): an event
// appends while its attribute t < endTime, else it flushes the batch and sets endTime =
// findEndTime(lastCurrentEventTime) (:297, :440-444) = start + T((M - start) / T + 1), M the running max
// of t. So an event starts a new batch exactly when (M - start) / T grows: the bucket of a partition's
// running max names its batch, and the event crossing into a higher bucket closes the batch before it
// (that event is the chunk's name; the expired rows are stamped with M there, flushToOutputChunk :341-348).
__global__ __launch_bounds__(kBlock) void k_pg_xgather(const u32* __restrict__ ranks, PgRecs C, i64 n, i64* xv) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) xv[i] = C.x[ranks[i]];
}

struct MaxI64 {
    __device__ __host__ i64 operator()(i64 a, i64 b) const { return a > b ? a : b; }
};

int launch_pg_ext_scan(hipStream_t s, const u32* ranks, const u32* p_sorted, PgRecs C, i64 n, i64* xv, i64* ms,
                       void* temp, size_t* temp_bytes) {
    if (temp && n > 0)
        hipLaunchKernelGGL(k_pg_xgather, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, ranks, C, n, xv);
    const hipError_t e = rocprim::inclusive_scan_by_key(temp, *temp_bytes, p_sorted, xv, ms, (size_t)n, MaxI64(),
                                                        rocprim::equal_to<u32>(), s);
    return e == hipSuccess ? 0 : -1;
}

namespace {
// a partition's run: [lo, lo + np) carried previous batch, [lo + np, a) carried open batch (bucket
// bopen), [a, hi) the push's events
struct ExtRun {
    i64 lo, hi, np, a, Mcar, start, bopen;
    bool has;
};

__device__ __forceinline__ ExtRun ext_run(const u32* key_off, const u32* ranks, const u32* prev_cnt, const u32* pend_cnt,
                                          const PgRecs& C, const i64* xs, const PgExt& X, u32 p) {
    ExtRun R;
    R.lo = key_off[p];
    R.hi = key_off[p + 1];
    R.np = prev_cnt[p];
    R.a = R.lo + R.np + pend_cnt[p];
    R.has = X.has[p] != 0;
    R.Mcar = R.has ? X.M[p] : INT64_MIN;
    R.bopen = X.bopen[p];
    if (R.has) {
        R.start = X.start[p];
    } else if (R.a >= R.hi) {
        R.start = 0;  // no event of the partition yet
    } else {
        // initTiming (:313-334) at the partition's first event
        const u32 c = ranks[R.a];
        R.start = X.has_start == 1 ? X.start_time : X.has_start == 2 ? xs[c] : C.x[c];
    }
    return R;
}

// bucket of sorted position pos >= R.a (the push's events); -1 flags an event before the start
__device__ __forceinline__ i64 ext_bucket(const ExtRun& R, const PgExt& X, const i64* ms, i64 pos, i64* m_out) {
    const i64 m = max(R.Mcar, ms[pos]);
    if (m_out) *m_out = m;
    return m < R.start ? -1 : (m - R.start) / X.T;
}

__device__ __forceinline__ i64 ext_b(const ExtRun& R, const PgExt& X, const i64* ms, i64 pos) {
    return pos < R.a ? R.bopen : ext_bucket(R, X, ms, pos, nullptr);
}

// first position in [from, R.hi) whose bucket exceeds b (buckets do not decrease along the run)
__device__ __forceinline__ i64 ext_after(const ExtRun& R, const PgExt& X, const i64* ms, i64 from, i64 b) {
    i64 lo = from, hi = R.hi;
    while (lo < hi) {
        const i64 mid = (lo + hi) >> 1;
        if (ext_b(R, X, ms, mid) > b) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}
}  // namespace

__global__ __launch_bounds__(kBlock) void k_pg_assign_ext(const u32* __restrict__ key_off, const u32* __restrict__ ranks,
                                                         const u32* __restrict__ prev_cnt, const u32* __restrict__ pend_cnt,
                                                         PgRecs C, const i64* __restrict__ xs, const i64* __restrict__ ms,
                                                         PgExt X, i64 n, int cur_on, int exp_on, int gbits, u64 none,
                                                         u64* ekey, u32* eval, unsigned char* keep,
                                                         unsigned long long* n_entries, i64* chunk_ts, int* err) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    int made = 0;
    if (i < n) {
        const u32 c = ranks[i];
        const u32 p = C.ps[c];
        const ExtRun R = ext_run(key_off, ranks, prev_cnt, pend_cnt, C, xs, X, p);
        const u64 g = C.gs[c];
        u64 kx = none, kc = none;
        unsigned char kp = 0;
        if (i >= R.a) {
            i64 m;
            const i64 bk = ext_bucket(R, X, ms, i, &m);
            if (bk < 0 || R.start < 0) atomicExch(err, 1);
            chunk_ts[c] = m;  // lastCurrentEventTime once this event is in (the expired rows' stamp)
            C.xe[c] = R.start + X.T * (bk + 1);  // endTime when the event was appended (findEndTime :440-444)
            C.xm[c] = m;
        }
        if (i < R.lo + R.np) {
            // the last completed batch: EXPIRED into the chunk that closes the open batch, else kept
            const i64 x2 = ext_after(R, X, ms, R.lo + R.np, R.bopen);
            if (x2 < R.hi) kx = ((u64)ranks[x2] << gbits) | g;
            else kp = 1;
        } else {
            const i64 b = ext_b(R, X, ms, i);
            const i64 x1 = ext_after(R, X, ms, i + 1, b);  // the event closing this batch
            if (x1 < R.hi) {
                if (cur_on) kc = ((u64)ranks[x1] << gbits) | g;
                if (exp_on) {
                    const i64 x2 = ext_after(R, X, ms, x1 + 1, ext_b(R, X, ms, x1));
                    if (x2 < R.hi) kx = ((u64)ranks[x2] << gbits) | g;
                    else kp = 1;
                }
            } else {
                kp = 2;
            }
        }
        if (!exp_on) kx = none;
        if (exp_on) {
            ekey[2 * i] = kx;
            ekey[2 * i + 1] = kc;
            eval[2 * i] = (u32)i;
            eval[2 * i + 1] = (u32)i | 0x80000000u;
        } else {  // current rows only: one entry per event (the sort takes n entries, not 2n)
            ekey[i] = kc;
            eval[i] = (u32)i | 0x80000000u;
        }
        keep[c] = kp;
        made = (kx != none) + (kc != none);
    }
    const i64 tot = block_reduce((i64)made, SumOp(), 0);
    if (threadIdx.x == 0 && tot) atomicAdd(n_entries, (unsigned long long)tot);
}

void launch_pg_assign_ext(hipStream_t s, const u32* key_off, const u32* ranks, const u32* prev_cnt, const u32* pend_cnt,
                          PgRecs C, const i64* xs, const i64* ms, PgExt X, i64 n, int cur_on, int exp_on, int gbits,
                          u64 none, u64* ekey, u32* eval, unsigned char* keep, unsigned long long* n_entries, i64* chunk_ts,
                          int* err) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_pg_assign_ext, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, key_off, ranks,
                       prev_cnt, pend_cnt, C, xs, ms, X, n, cur_on, exp_on, gbits, none, ekey, eval, keep, n_entries,
                       chunk_ts, err);
}

// after the entries: every partition with events in the push keeps its running max, start and the
// bucket of its open batch
__global__ __launch_bounds__(kBlock) void k_pg_ext_state(const u32* __restrict__ key_off, const u32* __restrict__ ranks,
                                                        const u32* __restrict__ prev_cnt, const u32* __restrict__ pend_cnt,
                                                        PgRecs C, const i64* __restrict__ xs, const i64* __restrict__ ms,
                                                        PgExt X, i64 nslots) {
    const i64 p = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (p >= nslots) return;
    const ExtRun R = ext_run(key_off, ranks, prev_cnt, pend_cnt, C, xs, X, (u32)p);
    if (R.a >= R.hi) return;  // no event of the push
    i64 m;
    const i64 b = ext_bucket(R, X, ms, R.hi - 1, &m);
    X.M[p] = m;
    X.start[p] = R.start;
    X.has[p] = 1;
    X.bopen[p] = b;
}

void launch_pg_ext_state(hipStream_t s, const u32* key_off, const u32* ranks, const u32* prev_cnt, const u32* pend_cnt,
                         PgRecs C, const i64* xs, const i64* ms, PgExt X, i64 nslots) {
    if (nslots > 0)
        hipLaunchKernelGGL(k_pg_ext_state, dim3((unsigned)((nslots + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, key_off,
                           ranks, prev_cnt, pend_cnt, C, xs, ms, X, nslots);
}

// ---- externalTimeBatch(ts, T, start, timeout) under `partition with`. Which batch every event joins is
// still the bucket of its partition's running max, but when a batch goes out is the Scheduler's: a timeout
// re-sends a partition's open batch whenever the playback clock passes its lastScheduledTime, and ties
// between partitions due at the same time resolve in PartitionStateHolder's HashMap order — a sequential
// walk the host runs (sh_plane.cpp xt_walk) over these per-event flags; the emissions it finds are then
// expanded into (emission, group) entries and folded like the batches above.
__global__ __launch_bounds__(kBlock) void k_pg_xt_flags(const u32* __restrict__ key_off, const u32* __restrict__ ranks,
                                                       const u32* __restrict__ prev_cnt, const u32* __restrict__ pend_cnt,
                                                       PgRecs C, const i64* __restrict__ xs, const i64* __restrict__ ms,
                                                       PgExt X, i64 n, unsigned char* flag, int* err) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const u32 c = ranks[i];
    const ExtRun R = ext_run(key_off, ranks, prev_cnt, pend_cnt, C, xs, X, C.ps[c]);
    if (i < R.a) return;  // (a carried record)
    i64 m;
    const i64 bk = ext_bucket(R, X, ms, i, &m);
    if (bk < 0 || R.start < 0) atomicExch(err, 1);
    C.xm[c] = m;
    C.xe[c] = R.start + X.T * (bk + 1);
    unsigned char f = 0;
    if (!R.has && i == R.a) {
        // initTiming (:313-334); with the start from an attribute the first event may already be past
        // endTime = start + T: it "crosses" an empty batch (no output, but a reschedule)
        f = 2 | (bk > 0 ? 1 : 0);
    } else {
        const i64 pb = i == R.a ? R.bopen : ext_bucket(R, X, ms, i - 1, nullptr);
        f = bk > pb ? 1 : 0;
    }
    flag[c] = f;
}

void launch_pg_xt_flags(hipStream_t s, const u32* key_off, const u32* ranks, const u32* prev_cnt, const u32* pend_cnt,
                        PgRecs C, const i64* xs, const i64* ms, PgExt X, i64 n, unsigned char* flag, int* err) {
    if (n > 0)
        hipLaunchKernelGGL(k_pg_xt_flags, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, key_off, ranks,
                           prev_cnt, pend_cnt, C, xs, ms, X, n, flag, err);
}

__global__ __launch_bounds__(kBlock) void k_pg_xt_expand(const PgXtEmit* __restrict__ em, i64 ne, i64 n_ent,
                                                        const u32* __restrict__ key_off, const u32* __restrict__ ranks,
                                                        PgRecs C, int gbits, int cur_on, int exp_on, u64* ekey, u32* eval,
                                                        u32* epos) {
    const i64 t = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (t >= n_ent) return;
    i64 lo = 0, hi = ne;  // the last emission whose first entry is at or before t
    while (hi - lo > 1) {
        const i64 mid = (lo + hi) >> 1;
        if (em[mid].off <= t) lo = mid;
        else hi = mid;
    }
    const PgXtEmit E = em[lo];
    const i64 k = t - E.off, nx = exp_on ? E.xhi - E.xlo : 0;
    const bool cur = k >= nx;
    const u32 pos = key_off[E.p] + (u32)(cur ? E.lo + (k - nx) : E.xlo + k);
    const u32 c = ranks[pos];
    (void)cur_on;
    ekey[t] = ((u64)lo << gbits) | (u64)C.gs[c];
    eval[t] = (u32)t | (cur ? 0x80000000u : 0u);
    epos[t] = pos;
}

void launch_pg_xt_expand(hipStream_t s, const PgXtEmit* em, i64 ne, i64 n_ent, const u32* key_off, const u32* ranks,
                         PgRecs C, int gbits, int cur_on, int exp_on, u64* ekey, u32* eval, u32* epos) {
    if (n_ent > 0)
        hipLaunchKernelGGL(k_pg_xt_expand, dim3((unsigned)((n_ent + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, em, ne,
                           n_ent, key_off, ranks, C, gbits, cur_on, exp_on, ekey, eval, epos);
}

__global__ __launch_bounds__(kBlock) void k_pg_xt_keep(const u32* __restrict__ key_off, const u32* __restrict__ ranks,
                                                      PgRecs C, i64 n, const u32* __restrict__ kf, unsigned char* keep) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const u32 c = ranks[i];
    const u32 p = C.ps[c];
    keep[c] = (u32)(i - key_off[p]) >= kf[p] ? 2 : 0;
}

void launch_pg_xt_keep(hipStream_t s, const u32* key_off, const u32* ranks, PgRecs C, i64 n, const u32* kf,
                       unsigned char* keep) {
    if (n > 0)
        hipLaunchKernelGGL(k_pg_xt_keep, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, key_off, ranks,
                           C, n, kf, keep);
}

__global__ __launch_bounds__(kBlock) void k_pg_xt_kf(const u32* __restrict__ slots, const u32* __restrict__ vals, i64 n,
                                                    u32* kf) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) kf[slots[i]] = vals ? vals[i] : 0u;
}

void launch_pg_xt_kf(hipStream_t s, const u32* slots, const u32* vals, i64 n, u32* kf) {
    if (n > 0)
        hipLaunchKernelGGL(k_pg_xt_kf, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, slots, vals, n,
                           kf);
}

// ---- 2. batch of every sorted position. Partition p's run [lo, hi) of the sorted order holds its
// np carried previous-batch records first, then its open batch and the push's events in stream order.
// Position j = i - lo - np >= 0 is in batch j / L, complete iff the run holds all of it; the chunk of
// batch b is named by the combined index of its last event. Entries (2 per position, key ~0 = none):
//   [2i]     EXPIRED of position i into the chunk of the following batch (expired output only);
//   [2i + 1] CURRENT of position i into its own batch's chunk (current output only);
// value = i | (1 << 31) for CURRENT. keep[c]: 1 = carried as the last completed batch, 2 = open batch.
__global__ __launch_bounds__(kBlock) void k_pg_assign(const u32* __restrict__ key_off, const u32* __restrict__ ranks,
                                                     const u32* __restrict__ p_sorted,
                                                     const u32* __restrict__ prev_cnt, PgRecs C, i64 n, i64 L,
                                                     int cur_on, int exp_on, int gbits, u64 none, u64* ekey, u32* eval,
                                                     unsigned char* keep, unsigned long long* n_entries) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    int made = 0;
    if (i < n) {
        const u32 c = ranks[i];
        const u32 p = p_sorted[i];  // (= C.ps[c]: the sort's keys, read coalesced instead of through c)
        const i64 lo = key_off[p], hi = key_off[p + 1], np = prev_cnt[p];
        const i64 run = hi - lo - np, nfull = run / L;
        const i64 j = i - lo - np;
        const u64 g = C.gs[c];
        u64 kx = none, kc = none;
        unsigned char kp = 0;
        if (j < 0) {
            // a carried record of the last completed batch: EXPIRED into batch 0's chunk, else kept
            if (nfull > 0) kx = ((u64)ranks[lo + np + L - 1] << gbits) | g;
            else kp = 1;
        } else {
            const i64 b = j / L;
            if (b < nfull) {
                if (cur_on) kc = ((u64)ranks[lo + np + (b + 1) * L - 1] << gbits) | g;
                if (exp_on) {
                    if (b + 1 < nfull) kx = ((u64)ranks[lo + np + (b + 2) * L - 1] << gbits) | g;
                    else kp = 1;
                }
            } else {
                kp = 2;
            }
        }
        if (!exp_on) kx = none;
        if (exp_on) {
            ekey[2 * i] = kx;
            ekey[2 * i + 1] = kc;
            eval[2 * i] = (u32)i;
            eval[2 * i + 1] = (u32)i | 0x80000000u;
        } else {  // current rows only: one entry per event (the sort takes n entries, not 2n)
            ekey[i] = kc;
            eval[i] = (u32)i | 0x80000000u;
        }
        keep[c] = kp;
        made = (kx != none) + (kc != none);
    }
    const i64 tot = block_reduce((i64)made, SumOp(), 0);
    if (threadIdx.x == 0 && tot) atomicAdd(n_entries, (unsigned long long)tot);
}

void launch_pg_assign(hipStream_t s, const u32* key_off, const u32* ranks, const u32* p_sorted, const u32* prev_cnt,
                      PgRecs C, i64 n, i64 L, int cur_on, int exp_on, int gbits, u64 none, u64* ekey, u32* eval,
                      unsigned char* keep, unsigned long long* n_entries) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_pg_assign, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, key_off, ranks,
                       p_sorted, prev_cnt, C, n, L, cur_on, exp_on, gbits, none, ekey, eval, keep, n_entries);
}

// ---- lengthBatch(L, true) grouped by other columns (stream.current.event, current output): every event
// is a chunk of its own (LengthBatchWindowProcessor.processStreamCurrentEvents :245-274: the event passes
// through, a RESET before the partition's (L + 1)-th event of the batch clears the group states), so its
// row is its group's fold over the partition's batch up to it. One entry per sorted position, keyed
// (the batch's first combined index, group slot); the carried events of the open batches fold without
// emitting (their rows went out with their own push). keep: the events of a run's last batch unless it
// is complete (the next event of the partition resets).
__global__ __launch_bounds__(kBlock) void k_pg_sc_assign(const u32* __restrict__ key_off, const u32* __restrict__ ranks,
                                                        const u32* __restrict__ p_sorted, PgRecs C, i64 n, i64 L,
                                                        int gbits, u64* ekey, u32* eval, unsigned char* keep) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const u32 c = ranks[i];
    const u32 p = p_sorted[i];
    const i64 lo = key_off[p], run = (i64)key_off[p + 1] - lo;
    const i64 j = i - lo, b = j / L;
    ekey[i] = ((u64)ranks[lo + b * L] << gbits) | (u64)C.gs[c];
    eval[i] = (u32)i;
    keep[c] = (b == (run - 1) / L && run % L != 0) ? 2 : 0;
}

void launch_pg_sc_assign(hipStream_t s, const u32* key_off, const u32* ranks, const u32* p_sorted, PgRecs C, i64 n,
                         i64 L, int gbits, u64* ekey, u32* eval, unsigned char* keep) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_pg_sc_assign, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, key_off, ranks,
                       p_sorted, C, n, L, gbits, ekey, eval, keep);
}

// one thread per (batch, group) segment folds its events in stream order; every event of this push
// (combined index >= n_old) writes its row at its own place among the push's events (stream order)
template <int NA>
__global__ __launch_bounds__(64) void k_pg_sc_fold(const i64* __restrict__ seg_start, i64 n_seg, i64 n_e,
                                                  const u64* __restrict__ ekey, const u32* __restrict__ eval,
                                                  const u32* __restrict__ ranks, PgRecs C, AggPlan ap, int gbits,
                                                  i64 n_old, SlxRows rows, u32* row_part) {
    const i64 sidx = (i64)blockIdx.x * 64 + threadIdx.x;
    if (sidx >= n_seg) return;
    const i64 lo = seg_start[sidx], hi = sidx + 1 < n_seg ? seg_start[sidx + 1] : n_e;
    const u32 g = (u32)(ekey[lo] & ((1ull << gbits) - 1));
    u64 f[NA], mm[NA];
    unsigned char mmh[NA];
#pragma unroll
    for (int a = 0; a < NA; a++) { f[a] = 0; mm[a] = 0; mmh[a] = 0; }
    i64 cnt = 0;
    for (i64 t = lo; t < hi; t++) {
        const u32 c = ranks[eval[t]];
        cnt++;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            if (a >= ap.n) continue;
            const int kind = ap.kind[a];
            if (kind == AK_COUNT) continue;
            const u64 x = C.vals[(size_t)ap.vcol[a] * C.cap + c];
            if (kind == AK_SUM_L) f[a] = (u64)((i64)f[a] + (i64)x);
            else if (kind == AK_SUM_D || kind == AK_AVG)
                f[a] = (u64)__double_as_longlong(__longlong_as_double((i64)f[a]) + g_num(ap, a, x));
            else {
                const bool take = !mmh[a] || g_worse(kind, mm[a], x);
                mm[a] = take ? x : mm[a];
                mmh[a] = 1;
            }
        }
        if ((i64)c < n_old) continue;  // carried: its row went out with its own push
        const i64 r = (i64)c - n_old;
        rows.ts[r] = C.ts[c];
        rows.rep[r] = C.seq[c];
        rows.slot[r] = g;
        rows.ch[r] = C.seq[c];
        rows.clk[r] = C.clk[c];
        rows.exp[r] = 0;
        row_part[r] = C.ps[c];
#pragma unroll
        for (int a = 0; a < NA; a++) {
            if (a >= ap.n) continue;
            const int kind = ap.kind[a];
            u64 rv = 0;
            unsigned char rn = 0;
            if (kind == AK_COUNT) rv = (u64)cnt;
            else if (kind == AK_SUM_L || kind == AK_SUM_D) rv = f[a];
            else if (kind == AK_AVG) rv = (u64)__double_as_longlong(__longlong_as_double((i64)f[a]) / (double)cnt);
            else { rn = mmh[a] ? 0 : 1; rv = mmh[a] ? mm[a] : 0; }
            rows.vals[(size_t)a * rows.cap + r] = rv;
            rows.nulls[(size_t)a * rows.cap + r] = rn;
        }
    }
}

void launch_pg_sc_fold(hipStream_t s, const i64* seg_start, i64 n_seg, i64 n_e, const u64* ekey, const u32* eval,
                       const u32* ranks, PgRecs C, AggPlan ap, int gbits, i64 n_old, SlxRows rows, u32* row_part) {
    if (n_seg <= 0) return;
    const unsigned grid = (unsigned)((n_seg + 63) / 64);
    if (ap.n <= 4) hipLaunchKernelGGL(k_pg_sc_fold<4>, dim3(grid), dim3(64), 0, s, seg_start, n_seg, n_e, ekey, eval,
                                      ranks, C, ap, gbits, n_old, rows, row_part);
    else hipLaunchKernelGGL(k_pg_sc_fold<8>, dim3(grid), dim3(64), 0, s, seg_start, n_seg, n_e, ekey, eval, ranks, C,
                            ap, gbits, n_old, rows, row_part);
}

// segment heads of the sorted entries
__global__ __launch_bounds__(kBlock) void k_pg_heads(const u64* __restrict__ key, i64 n, unsigned char* head) {
    const i64 j = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (j < n) head[j] = j == 0 || key[j] != key[j - 1];
}

void launch_pg_heads(hipStream_t s, const u64* key, i64 n, unsigned char* head) {
    if (n > 0)
        hipLaunchKernelGGL(k_pg_heads, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, key, n, head);
}

// ---- 3. one row per (chunk, group) segment. EXPIRED entries come first (the previous batch), then
// CURRENT ones, each in stream order. With current entries the row is the group's last current event
// carrying the fold of the group's current events (the RESET cleared the state); with expired entries
// only, the last expired event with the state emptied (count 0, the others null), stamped with the
// chunk's clock. Row order key: (chunk, the segment's first sorted position).
template <int NA>
__global__ __launch_bounds__(64) void k_pg_fold(const i64* __restrict__ seg_start, i64 n_seg, i64 n_e,
                                               const u64* __restrict__ ekey, const u32* __restrict__ eval,
                                               const u32* __restrict__ ranks, PgRecs C, AggPlan ap, int gbits,
                                               SlxRows rows, u64* row_key, u32* row_part,
                                               const i64* __restrict__ chunk_ts, const PgXtEmit* __restrict__ xem,
                                               const u32* __restrict__ epos, const u32* __restrict__ key_off) {
    const i64 sidx = (i64)blockIdx.x * 64 + threadIdx.x;
    if (sidx >= n_seg) return;
    const i64 lo = seg_start[sidx], hi = sidx + 1 < n_seg ? seg_start[sidx + 1] : n_e;
    const u64 key = ekey[lo];
    const u32 chunk = (u32)(key >> gbits);
    const u32 g = (u32)(key & ((1ull << gbits) - 1));
    u64 f[NA], mm[NA];
    unsigned char mmh[NA];
#pragma unroll
    for (int a = 0; a < NA; a++) { f[a] = 0; mm[a] = 0; mmh[a] = 0; }
    i64 cnt = 0, last_c = -1, last_x = -1;
    for (i64 t = lo; t < hi; t++) {
        const u32 v = eval[t];
        const u32 c = ranks[epos ? epos[v & 0x7FFFFFFFu] : v & 0x7FFFFFFFu];
        if (!(v >> 31)) { last_x = c; continue; }
        last_c = c;
        cnt++;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            if (a >= ap.n) continue;
            const int kind = ap.kind[a];
            if (kind == AK_COUNT) continue;
            const u64 x = C.vals[(size_t)ap.vcol[a] * C.cap + c];
            if (kind == AK_SUM_L) f[a] = (u64)((i64)f[a] + (i64)x);
            else if (kind == AK_SUM_D || kind == AK_AVG)
                f[a] = (u64)__double_as_longlong(__longlong_as_double((i64)f[a]) + g_num(ap, a, x));
            else {
                const bool take = !mmh[a] || g_worse(kind, mm[a], x);
                mm[a] = take ? x : mm[a];
                mmh[a] = 1;
            }
        }
    }
    const bool cur = last_c >= 0;
    const i64 rc = cur ? last_c : last_x;
    if (xem) {
        // a timeout-path emission: its own clock, partition and lastCurrentEventTime stamp
        const PgXtEmit E = xem[chunk];
        rows.ts[sidx] = cur ? C.ts[rc] : C.xm[ranks[key_off[E.p] + (u32)E.sidx]];
        rows.ch[sidx] = (i64)chunk;
        rows.clk[sidx] = E.clock;
        row_part[sidx] = E.p;
    } else {
        rows.ts[sidx] = cur ? C.ts[rc] : chunk_ts ? chunk_ts[chunk] : C.clk[chunk];
        rows.ch[sidx] = C.seq[chunk];
        rows.clk[sidx] = C.clk[chunk];
        row_part[sidx] = C.ps[chunk];
    }
    rows.rep[sidx] = C.seq[rc];
    if (rows.xa) rows.xa[sidx] = C.xe[rc];
    rows.slot[sidx] = g;
    rows.exp[sidx] = cur ? 0 : 1;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (a >= ap.n) continue;
        const int kind = ap.kind[a];
        u64 rv = 0;
        unsigned char rn = 0;
        if (kind == AK_COUNT) rv = (u64)cnt;
        else if (kind == AK_SUM_L || kind == AK_SUM_D) { rn = cnt == 0; rv = cnt == 0 ? 0 : f[a]; }
        else if (kind == AK_AVG) {
            rn = cnt == 0;
            if (cnt) rv = (u64)__double_as_longlong(__longlong_as_double((i64)f[a]) / (double)cnt);
        } else { rn = mmh[a] ? 0 : 1; rv = mmh[a] ? mm[a] : 0; }
        rows.vals[(size_t)a * rows.cap + sidx] = rv;
        rows.nulls[(size_t)a * rows.cap + sidx] = rn;
    }
    row_key[sidx] = ((u64)chunk << 32) | (u64)(eval[lo] & 0x7FFFFFFFu);
}

void launch_pg_fold(hipStream_t s, const i64* seg_start, i64 n_seg, i64 n_e, const u64* ekey, const u32* eval,
                    const u32* ranks, PgRecs C, AggPlan ap, int gbits, SlxRows rows, u64* row_key, u32* row_part,
                    const i64* chunk_ts, const PgXtEmit* xem, const u32* epos, const u32* key_off) {
    if (n_seg <= 0) return;
    const unsigned grid = (unsigned)((n_seg + 63) / 64);
    if (ap.n <= 4) hipLaunchKernelGGL(k_pg_fold<4>, dim3(grid), dim3(64), 0, s, seg_start, n_seg, n_e, ekey, eval, ranks,
                                      C, ap, gbits, rows, row_key, row_part, chunk_ts, xem, epos, key_off);
    else hipLaunchKernelGGL(k_pg_fold<8>, dim3(grid), dim3(64), 0, s, seg_start, n_seg, n_e, ekey, eval, ranks, C, ap,
                            gbits, rows, row_key, row_part, chunk_ts, xem, epos, key_off);
}

// ---- 4. the rows in (chunk, first entry) order -> the push's output columns
__global__ __launch_bounds__(kBlock) void k_pg_emit(const u32* __restrict__ order, i64 n, SlxRows rows, int n_aggs,
                                                   int nk, KeyTable kt, KeyPlan kp, i64 out_cap, i64* out_ts,
                                                   i64* out_keys, u64* out_vals, unsigned char* out_nulls,
                                                   unsigned char* out_exp, i64* out_ch, i64* out_clock, i64* out_rep,
                                                   const u32* __restrict__ row_part, u32* out_part, i64* out_xa) {
    const i64 r = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (r >= n) return;
    const u32 j = order ? order[r] : (u32)r;  // (null: the rows are already in output order)
    out_ts[r] = rows.ts[j];
    if (nk > 0) unpack_key(kp, slot_key(kt, rows.slot[j]), out_keys + r, out_cap);
    for (int a = 0; a < n_aggs; a++) {
        out_vals[(size_t)a * out_cap + r] = rows.vals[(size_t)a * rows.cap + j];
        out_nulls[(size_t)a * out_cap + r] = rows.nulls[(size_t)a * rows.cap + j];
    }
    out_exp[r] = rows.exp[j];
    out_ch[r] = rows.ch[j];
    out_clock[r] = rows.clk[j];
    out_rep[r] = rows.rep[j];
    out_part[r] = row_part[j];
    if (out_xa) out_xa[r] = rows.xa[j];
}

void launch_pg_emit(hipStream_t s, const u32* order, i64 n, SlxRows rows, int n_aggs, int nk, KeyTable kt, KeyPlan kp,
                    i64 out_cap, i64* out_ts, i64* out_keys, u64* out_vals, unsigned char* out_nulls,
                    unsigned char* out_exp, i64* out_ch, i64* out_clock, i64* out_rep, const u32* row_part,
                    u32* out_part, i64* out_xa) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_pg_emit, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, order, n, rows,
                       n_aggs, nk, kt, kp, out_cap, out_ts, out_keys, out_vals, out_nulls, out_exp, out_ch, out_clock,
                       out_rep, row_part, out_part, out_xa);
}

// ---- carried records: the kept ones (keep != 0) of the combined order, gathered in that (stream)
// order into the other buffer set
__global__ __launch_bounds__(kBlock) void k_pg_gather(const i64* __restrict__ idx, i64 n, const unsigned char* keep,
                                                     PgRecs C, PgRecs D, int nv) {
    const i64 k = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (k >= n) return;
    const i64 c = idx[k];
    D.ps[k] = C.ps[c];
    D.gs[k] = C.gs[c];
    D.ts[k] = C.ts[c];
    D.seq[k] = C.seq[c];
    D.clk[k] = C.clk[c];
    D.prev[k] = keep[c] == 1;
    if (C.x) D.x[k] = C.x[c];
    if (C.xe) D.xe[k] = C.xe[c];
    if (C.xm) D.xm[k] = C.xm[c];
    for (int v = 0; v < nv; v++) D.vals[(size_t)v * D.cap + k] = C.vals[(size_t)v * C.cap + c];
}

void launch_pg_gather(hipStream_t s, const i64* idx, i64 n, const unsigned char* keep, PgRecs C, PgRecs D, int nv) {
    if (n > 0)
        hipLaunchKernelGGL(k_pg_gather, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, idx, n, keep, C,
                           D, nv);
}

// ==== time / externalTime windows under `partition with`, grouped by other columns ==========================
// TimeWindowProcessor (:132-169) per partition: at every point of the partition (a run of its events in a
// send, or a TIMER call the Scheduler fires for it) the queue head expires while ts + T <= now, then the
// event joins. Each EXPIRED / CURRENT event updates its group's aggregator state (partition, group) in
// chunk order and the selector keeps one row per group per chunk (QuerySelector :315-374). Stage 1: one
// lane per partition walks its points exactly like the time lanes but, instead of folding, writes the
// partition's operations (add / remove, group, event) in order into its own region of an operation list.
// Stage 2: the operations sorted stably by (partition, group) state slot; one thread per state replays
// its operations in order (the double sums in Java's add / remove order) and emits a row per chunk:
// placed at the chunk's first qualifying operation, valued after its last one.
template <int NV>
__global__ __launch_bounds__(64) void k_pg_walk_ops(const u32* __restrict__ key_off, const u32* __restrict__ sorted_rank,
                                                   u32 nslots, SlRecords rec, const i64* __restrict__ run, i64 T,
                                                   i64 seq_base, i64 send_size, const i64* __restrict__ t_off,
                                                   const i64* __restrict__ t_send, const i64* __restrict__ t_clk,
                                                   const i64* __restrict__ t_pos, const i64* __restrict__ f_send, i64 nF,
                                                   SlState S, i64* rseq, int nv, const i64* __restrict__ xattr,
                                                   KeyTable pgkt, const i64* __restrict__ obase, PgOps O, u32* o_cnt) {
    const u32 k = blockIdx.x * 64 + threadIdx.x;
    if (k >= nslots) return;
    const u32 lo = key_off[k], hi = key_off[k + 1];
    const i64 tlo = t_off ? t_off[k] : 0, thi = t_off ? t_off[k + 1] : 0;
    if (lo == hi && tlo == thi) return;
    const i64 rc = S.rc, rm = rc - 1;
    i64 rh = S.rhead[k], rlen = S.rlen[k];
    i64 o = obase[k];
    const i64 o0 = o;
    u32 i = lo;
    i64 t = tlo;
    i64 cur_run = -1, run_pos = 0;
    const int gcol = nv;  // the group slot travels as the last value column
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
            now = xattr ? xattr[r] : clk;
            const i64 rn_ = run[rec.raw[r]];
            if (rn_ != cur_run) {
                cur_run = rn_;
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
        while (rlen > 0) {
            const i64 sl = rh & rm;
            if (S.rpm[(size_t)k * rc + sl] - now + T > 0) break;
            const u32 g = (u32)S.rval[((size_t)gcol * S.nslots + k) * rc + sl];
            O.pos[o] = pos;
            O.pg[o] = key_slot(pgkt, ((u64)k << 32) | g);
            O.kind[o] = 2;
            O.seq[o] = rseq[(size_t)k * rc + sl];
            O.ts[o] = now;
            O.clk[o] = clk;
#pragma unroll
            for (int q = 0; q < NV; q++)
                if (q < nv) O.vals[(size_t)q * O.cap + o] = S.rval[((size_t)q * S.nslots + k) * rc + sl];
            o++;
            rh++;
            rlen--;
        }
        if (timer) {
            t++;
            continue;
        }
        {
            const i64 sl = (rh + rlen) & rm;
            const u32 g = (u32)rec.vals[(size_t)gcol * rec.cap + r];
            S.rpm[(size_t)k * rc + sl] = xattr ? xattr[r] : rec.ts[r];
            rseq[(size_t)k * rc + sl] = seq_base + (i64)rec.raw[r];
            for (int q = 0; q <= nv; q++) S.rval[((size_t)q * S.nslots + k) * rc + sl] = rec.vals[(size_t)q * rec.cap + r];
            rlen++;
            O.pos[o] = pos;
            O.pg[o] = key_slot(pgkt, ((u64)k << 32) | g);
            O.kind[o] = 1;
            O.seq[o] = seq_base + (i64)rec.raw[r];
            O.ts[o] = rec.ts[r];
            O.clk[o] = clk;
#pragma unroll
            for (int q = 0; q < NV; q++)
                if (q < nv) O.vals[(size_t)q * O.cap + o] = rec.vals[(size_t)q * rec.cap + r];
            o++;
            i++;
        }
    }
    S.rhead[k] = rh;
    S.rlen[k] = rlen;
    o_cnt[k] = (u32)(o - o0);
}

void launch_pg_walk_ops(hipStream_t s, const u32* key_off, const u32* sorted_rank, i64 nslots, SlRecords rec,
                        const i64* run, i64 T, i64 seq_base, i64 send_size, const i64* t_off, const i64* t_send,
                        const i64* t_clk, const i64* t_pos, const i64* f_send, i64 nF, SlState S, i64* rseq, int nv,
                        const i64* xattr, KeyTable pgkt, const i64* obase, PgOps O, u32* o_cnt) {
    const unsigned grid = (unsigned)((nslots + 63) / 64);
    if (!grid) return;
    if (nv <= 1)
        hipLaunchKernelGGL(k_pg_walk_ops<1>, dim3(grid), dim3(64), 0, s, key_off, sorted_rank, (u32)nslots, rec, run, T,
                           seq_base, send_size, t_off, t_send, t_clk, t_pos, f_send, nF, S, rseq, nv, xattr, pgkt, obase, O,
                           o_cnt);
    else
        hipLaunchKernelGGL(k_pg_walk_ops<8>, dim3(grid), dim3(64), 0, s, key_off, sorted_rank, (u32)nslots, rec, run, T,
                           seq_base, send_size, t_off, t_send, t_clk, t_pos, f_send, nF, S, rseq, nv, xattr, pgkt, obase, O,
                           o_cnt);
}

// each partition's operation region: room for its queued events' removes and its new events' adds and
// removes
__global__ __launch_bounds__(kBlock) void k_pg_ops_room(const u32* __restrict__ slot_cnt, const i64* __restrict__ rlen,
                                                       i64 n, i64* room) {
    const i64 k = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (k < n) room[k] = rlen[k] + 2 * (i64)slot_cnt[k];
}

void launch_pg_ops_room(hipStream_t s, const u32* slot_cnt, const i64* rlen, i64 n, i64* room) {
    if (n > 0) hipLaunchKernelGGL(k_pg_ops_room, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, slot_cnt, rlen, n, room);
}

// the group slot of every record, as its extra value column
__global__ __launch_bounds__(kBlock) void k_pg_rec_group(SlRecords rec, i64 M, ColSet cols, KeyPlan gkp, KeyTable gkt,
                                                        int nv) {
    const i64 r = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (r < M) rec.vals[(size_t)nv * rec.cap + r] = key_slot(gkt, make_key(gkp, cols, rec.raw[r]));
}

void launch_pg_rec_group(hipStream_t s, SlRecords rec, i64 M, ColSet cols, KeyPlan gkp, KeyTable gkt, int nv) {
    if (M > 0) hipLaunchKernelGGL(k_pg_rec_group, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rec, M, cols, gkp, gkt, nv);
}

// stage 2: one thread per (partition, group) state replays its operations (sorted stably by state slot).
// Min / max keep MinAttributeAggregatorExecutor's deque (:86-236, removeFirstOccurrence on expiry) per
// state: carried between pushes in a pool (PgDeques: per (field, state) offset and length), worked on in
// the segment's own scratch area — room for its carried entries plus one per add of the push — and
// gathered back into a fresh pool afterwards (k_pg_dq_pool).
__device__ __forceinline__ bool g_eq(int kind, u64 a, u64 b) {
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

// scratch words a segment needs: per min / max field its carried deque plus its adds
__global__ __launch_bounds__(kBlock) void k_pg_dq_need(const i64* __restrict__ seg_start, i64 n_seg, i64 n_ops,
                                                      const u32* __restrict__ skey, const u32* __restrict__ sidx, PgOps O,
                                                      PgDeques D, i64* need) {
    const i64 sg = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (sg > n_seg) return;
    if (sg == n_seg) { need[sg] = 0; return; }
    const i64 lo = seg_start[sg], hi = sg + 1 < n_seg ? seg_start[sg + 1] : n_ops;
    const u32 pg = skey[lo];
    i64 adds = 0;
    for (i64 j = lo; j < hi; j++) adds += O.kind[sidx[j]] == 1;
    i64 w = 0;
    for (int f = 0; f < D.nf; f++) w += D.len[(size_t)D.field[f] * D.n + pg] + adds;
    need[sg] = w;
}

void launch_pg_dq_need(hipStream_t s, const i64* seg_start, i64 n_seg, i64 n_ops, const u32* skey, const u32* sidx,
                       PgOps O, PgDeques D, i64* need) {
    hipLaunchKernelGGL(k_pg_dq_need, dim3((unsigned)((n_seg + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, seg_start,
                       n_seg, n_ops, skey, sidx, O, D, need);
}

template <int NA>
__global__ __launch_bounds__(64) void k_pg_replay(const i64* __restrict__ seg_start, i64 n_seg, i64 n_ops,
                                                 const u32* __restrict__ skey, const u32* __restrict__ sidx, PgOps O,
                                                 KeyTable pgkt, i64* st_cnt, u64* st_f, i64 st_n, AggPlan ap, int cur_on,
                                                 int exp_on, SlxRows rows, u64* row_key, u32* row_part,
                                                 unsigned int* n_rows, PgDeques D, const i64* __restrict__ scr_off) {
    const i64 sg = (i64)blockIdx.x * 64 + threadIdx.x;
    if (sg >= n_seg) return;
    const i64 lo = seg_start[sg], hi = sg + 1 < n_seg ? seg_start[sg + 1] : n_ops;
    const u32 pg = skey[lo];
    const u64 pk = slot_key(pgkt, pg);
    i64 cnt = st_cnt[pg];
    u64 f[NA];
    // min / max: the deque of aggregator a in scratch [dqb[a] + dqh[a], + dql[a])
    i64 dqb[NA], dqh[NA], dql[NA];
    i64 adds = 0;
    if (D.nf > 0)
        for (i64 j = lo; j < hi; j++) adds += O.kind[sidx[j]] == 1;
    i64 base = D.nf > 0 ? scr_off[sg] : 0;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        f[a] = 0;
        dqb[a] = dqh[a] = dql[a] = 0;
        if (a >= ap.n) continue;
        const int kind = ap.kind[a];
        if (kind == AK_COUNT) continue;
        if (kind >= AK_MIN_L) {
            // (aggregators of one field share its deque: the first one loads it)
            int first = a;
            for (int b = 0; b < a; b++)
                if (ap.kind[b] >= AK_MIN_L && ap.field[b] == ap.field[a]) { first = b; break; }
            if (first != a) { dqb[a] = dqb[first]; dql[a] = dql[first]; continue; }
            const size_t fi = (size_t)ap.field[a] * D.n + pg;
            const i64 L = D.len[fi];
            dqb[a] = base;
            for (i64 e = 0; e < L; e++) D.scratch[base + e] = D.pool[D.off[fi] + e];
            dql[a] = L;
            base += L + adds;
        } else {
            f[a] = st_f[(size_t)ap.field[a] * st_n + pg];
        }
    }
    i64 chunk = -1, first = -1, q_ts = 0, q_seq = 0, q_clk = 0;
    unsigned char q_exp = 0;
    u64 rv[NA];
    unsigned char rn[NA];
#pragma unroll
    for (int a = 0; a < NA; a++) { rv[a] = 0; rn[a] = 0; }
    auto flush_row = [&]() {
        if (first < 0) return;
        const u32 slot = wave_row_slot(n_rows);
        rows.ts[slot] = q_ts;
        rows.rep[slot] = q_seq;
        rows.slot[slot] = (u32)pk;
        rows.ch[slot] = chunk;
        rows.clk[slot] = q_clk;
        rows.exp[slot] = q_exp;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            if (a >= ap.n) continue;
            rows.vals[(size_t)a * rows.cap + slot] = rv[a];
            rows.nulls[(size_t)a * rows.cap + slot] = rn[a];
        }
        row_key[slot] = ((u64)chunk << 32) | (u64)(u32)first;
        row_part[slot] = (u32)(pk >> 32);
    };
    for (i64 j = lo; j < hi; j++) {
        const u32 oi = sidx[j];
        const i64 pos = O.pos[oi];
        if (pos != chunk) {
            flush_row();
            chunk = pos;
            first = -1;
        }
        const bool add = O.kind[oi] == 1;
        add ? cnt++ : cnt--;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            if (a >= ap.n) continue;
            const int kind = ap.kind[a];
            if (kind == AK_COUNT) continue;
            const u64 x = O.vals[(size_t)ap.vcol[a] * O.cap + oi];
            if (kind >= AK_MIN_L) {
                bool owner = true;
                for (int b = 0; b < a; b++)
                    if (ap.kind[b] >= AK_MIN_L && ap.field[b] == ap.field[a]) owner = false;
                if (!owner) continue;  // the field's deque moves once per operation
                u64* d = D.scratch + dqb[a];
                i64 h = dqh[a], len = dql[a];
                if (add) {
                    // MinAttributeAggregatorExecutor.processAdd: drop worse entries from the back
                    while (len > 0 && g_worse(kind, d[h + len - 1], x)) len--;
                    d[h + len] = x;
                    len++;
                } else {
                    // processRemove: removeFirstOccurrence(value)
                    i64 found = -1;
                    for (i64 e = 0; e < len; e++)
                        if (g_eq(kind, d[h + e], x)) { found = e; break; }
                    if (found == 0) { h++; len--; }
                    else if (found > 0) {
                        for (i64 e = found; e + 1 < len; e++) d[h + e] = d[h + e + 1];
                        len--;
                    }
                }
                dqh[a] = h;
                dql[a] = len;
                for (int b = a + 1; b < NA; b++)
                    if (b < ap.n && ap.kind[b] >= AK_MIN_L && ap.field[b] == ap.field[a]) { dqh[b] = h; dql[b] = len; }
            } else if (kind == AK_SUM_L) {
                f[a] = add ? (u64)((i64)f[a] + (i64)x) : (u64)java_d2l((double)(i64)f[a] - (double)(i64)x);
            } else {
                const double v = g_num(ap, a, x);
                double rr = __longlong_as_double((i64)f[a]) + (add ? v : -v);
                if (!add && cnt == 0 && rr == 0.0) rr = 0.0;
                f[a] = (u64)__double_as_longlong(rr);
            }
        }
        if ((add && cur_on) || (!add && exp_on)) {
            if (first < 0) first = oi;
            q_ts = O.ts[oi];
            q_seq = O.seq[oi];
            q_clk = O.clk[oi];
            q_exp = add ? 0 : 1;
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
                } else {
                    rn[a] = dql[a] > 0 ? 0 : 1;
                    rv[a] = dql[a] > 0 ? D.scratch[dqb[a] + dqh[a]] : 0;
                }
            }
        }
    }
    flush_row();
    st_cnt[pg] = cnt;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (a >= ap.n || ap.kind[a] == AK_COUNT) continue;
        if (ap.kind[a] >= AK_MIN_L) {
            const size_t fi = (size_t)ap.field[a] * D.n + pg;
            D.new_at[fi] = dqb[a] + dqh[a];
            D.new_len[fi] = dql[a];
        } else {
            st_f[(size_t)ap.field[a] * st_n + pg] = f[a];
        }
    }
    if (D.nf > 0) D.active[pg] = 1;
}

void launch_pg_replay(hipStream_t s, const i64* seg_start, i64 n_seg, i64 n_ops, const u32* skey, const u32* sidx,
                      PgOps O, KeyTable pgkt, i64* st_cnt, u64* st_f, i64 st_n, AggPlan ap, int cur_on, int exp_on,
                      SlxRows rows, u64* row_key, u32* row_part, unsigned int* n_rows, PgDeques D, const i64* scr_off) {
    if (n_seg <= 0) return;
    const unsigned grid = (unsigned)((n_seg + 63) / 64);
    if (ap.n <= 4)
        hipLaunchKernelGGL(k_pg_replay<4>, dim3(grid), dim3(64), 0, s, seg_start, n_seg, n_ops, skey, sidx, O, pgkt, st_cnt,
                           st_f, st_n, ap, cur_on, exp_on, rows, row_key, row_part, n_rows, D, scr_off);
    else
        hipLaunchKernelGGL(k_pg_replay<8>, dim3(grid), dim3(64), 0, s, seg_start, n_seg, n_ops, skey, sidx, O, pgkt, st_cnt,
                           st_f, st_n, ap, cur_on, exp_on, rows, row_key, row_part, n_rows, D, scr_off);
}

// the deques after the push, (field, state)-major, into a fresh pool: lengths (then their scan) ...
__global__ __launch_bounds__(kBlock) void k_pg_dq_len(PgDeques D, i64* out_len) {
    const i64 t = (i64)blockIdx.x * kBlock + threadIdx.x;
    const i64 total = (i64)D.nf * D.n;
    if (t > total) return;
    if (t == total) { out_len[t] = 0; return; }
    const i64 fi = (i64)D.field[t / D.n] * D.n + t % D.n;
    out_len[t] = D.active[t % D.n] ? D.new_len[fi] : D.len[fi];
}

// ... and the copies (pool_out gets every state's deque at off_out[t])
__global__ __launch_bounds__(kBlock) void k_pg_dq_pool(PgDeques D, const i64* __restrict__ off_out, u64* pool_out,
                                                      i64* new_off) {
    const i64 t = (i64)blockIdx.x * kBlock + threadIdx.x;
    const i64 total = (i64)D.nf * D.n;
    if (t >= total) return;
    const i64 st = t % D.n;
    const i64 fi = (i64)D.field[t / D.n] * D.n + st;
    const bool act = D.active[st] != 0;
    const i64 L = act ? D.new_len[fi] : D.len[fi];
    const u64* src = act ? D.scratch + D.new_at[fi] : D.pool + D.off[fi];
    u64* dst = pool_out + off_out[t];
    for (i64 e = 0; e < L; e++) dst[e] = src[e];
    new_off[fi] = off_out[t];
    D.len[fi] = L;
}

void launch_pg_dq_len(hipStream_t s, PgDeques D, i64* out_len) {
    const i64 total = (i64)D.nf * D.n;
    hipLaunchKernelGGL(k_pg_dq_len, dim3((unsigned)((total + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, D, out_len);
}

void launch_pg_dq_pool(hipStream_t s, PgDeques D, const i64* off_out, u64* pool_out, i64* new_off) {
    const i64 total = (i64)D.nf * D.n;
    if (total > 0)
        hipLaunchKernelGGL(k_pg_dq_pool, dim3((unsigned)((total + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, D, off_out,
                           pool_out, new_off);
}

// sorted operation keys: heads of the (partition, group) runs among the first n valid ones
__global__ __launch_bounds__(kBlock) void k_pg_heads32(const u32* __restrict__ key, i64 n, unsigned char* head) {
    const i64 j = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (j < n) head[j] = j == 0 || key[j] != key[j - 1];
}

void launch_pg_heads32(hipStream_t s, const u32* key, i64 n, unsigned char* head) {
    if (n > 0) hipLaunchKernelGGL(k_pg_heads32, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, key, n, head);
}

__global__ __launch_bounds__(kBlock) void k_pg_sum_u32(const u32* __restrict__ a, i64 n, unsigned long long* out) {
    const i64 k = (i64)blockIdx.x * kBlock + threadIdx.x;
    const i64 t = block_reduce(k < n ? (i64)a[k] : 0, SumOp(), 0);
    if (threadIdx.x == 0 && t) atomicAdd(out, (unsigned long long)t);
}

void launch_pg_sum_u32(hipStream_t s, const u32* a, i64 n, unsigned long long* out) {
    if (n > 0) hipLaunchKernelGGL(k_pg_sum_u32, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, a, n, out);
}

// ---- rebuild of the (partition, group) pair table (time lanes grouped by other columns) -----------
// PartitionStateHolder drops a group's state once every aggregator can be destroyed (returnState /
// canDestroy); here a state that is all zero — count, fields and deque lengths — is exactly what a fresh
// pair starts from, so the rebuild keeps the others and drops those. Slot n - 1 is the table's sentinel
// (mask + 1), which maps to the new table's sentinel.
__device__ __forceinline__ bool pg_live(i64 n, i64 s, const i64* cnt, const u64* f, const i64* dql, int F) {
    bool live = cnt[s] != 0;
    for (int j = 0; j < F && !live; j++) live = f[(size_t)j * n + s] != 0 || dql[(size_t)j * n + s] != 0;
    return live;
}

__global__ __launch_bounds__(kBlock) void k_pg_count_live(KeyTable kt, i64 n, const i64* __restrict__ cnt,
                                                         const u64* __restrict__ f, const i64* __restrict__ dql, int F,
                                                         unsigned long long* n_live) {
    const i64 s = (i64)blockIdx.x * kBlock + threadIdx.x;
    bool live = false;
    if (s < n && (s == n - 1 || kt.keys[s] != kEmptyKey)) live = pg_live(n, s, cnt, f, dql, F);
    const unsigned long long b = __ballot(live);
    if ((threadIdx.x & 63) == 0 && b) atomicAdd(n_live, (unsigned long long)__popcll(b));
}

__global__ __launch_bounds__(kBlock) void k_pg_rehash(KeyTable okt, i64 on, const i64* __restrict__ cnt,
                                                     const u64* __restrict__ f, const i64* __restrict__ dqo,
                                                     const i64* __restrict__ dql, int F, KeyTable nkt, i64 nn,
                                                     i64* ncnt, u64* nf, i64* ndqo, i64* ndql) {
    const i64 s = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (s >= on) return;
    const bool sentinel = s == on - 1;
    if (!sentinel && okt.keys[s] == kEmptyKey) return;
    if (!pg_live(on, s, cnt, f, dql, F)) return;
    const i64 d = sentinel ? nn - 1 : (i64)key_slot(nkt, okt.keys[s]);
    ncnt[d] = cnt[s];
    for (int j = 0; j < F; j++) {
        nf[(size_t)j * nn + d] = f[(size_t)j * on + s];
        ndqo[(size_t)j * nn + d] = dqo[(size_t)j * on + s];
        ndql[(size_t)j * nn + d] = dql[(size_t)j * on + s];
    }
}

void launch_pg_count_live(hipStream_t s, KeyTable kt, i64 n, const i64* cnt, const u64* f, const i64* dql, int F,
                          unsigned long long* n_live) {
    hipLaunchKernelGGL(k_pg_count_live, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, kt, n, cnt, f,
                       dql, F, n_live);
}

void launch_pg_rehash(hipStream_t s, KeyTable okt, i64 on, const i64* cnt, const u64* f, const i64* dqo, const i64* dql,
                      int F, KeyTable nkt, i64 nn, i64* ncnt, u64* nf, i64* ndqo, i64* ndql) {
    hipLaunchKernelGGL(k_pg_rehash, dim3((unsigned)((on + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, okt, on, cnt, f,
                       dqo, dql, F, nkt, nn, ncnt, nf, ndqo, ndql);
}

}  // namespace shd

namespace shd {

// ==== partitioned timeBatch(T, true) — stream.current.event, current output (lane 4) ==================
// TimeBatchWindowProcessor.process (:262-340) per partition: every partition chunk (its run of events
// in a send, PartitionStreamReceiver.receive :176-272) goes out at once with the running aggregates of
// its groups; a partition's state is RESET only when its own chunk or TIMER finds the playback clock
// past the shared nextEmitTime (a processor field, :128) — the host walks those calls (sh_plane.cpp
// tbsc_walk) and gives every chunk its partition's batch number. Here: per record its chunk, its
// (partition, group) state slot; one thread per state folds its records in stream order from the
// carried state (a new batch number starts fresh) and writes a row per (chunk, group) after the group's
// last record of the chunk.

// a chunk starts at the first passing record of a partition run (runs: k_pl_run_start over all events)
__global__ __launch_bounds__(kBlock) void k_tb_chunk_flags(SlRecords rec, i64 M, const i64* __restrict__ run,
                                                          unsigned char* flag) {
    const i64 r = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (r >= M) return;
    flag[r] = r == 0 || run[rec.raw[r]] != run[rec.raw[r - 1]];
}

void launch_tb_chunk_flags(hipStream_t s, SlRecords rec, i64 M, const i64* run, unsigned char* flag) {
    if (M > 0)
        hipLaunchKernelGGL(k_tb_chunk_flags, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rec, M,
                           run, flag);
}

// per chunk (its first record r): partition slot, send number, clock
__global__ __launch_bounds__(kBlock) void k_tb_chunk_info(SlRecords rec, const i64* __restrict__ first, i64 nch,
                                                         i64 send_size, u32* slot, i64* send, i64* clock) {
    const i64 k = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (k >= nch) return;
    const i64 r = first[k];
    slot[k] = rec.slot[r];
    send[k] = send_size > 0 ? (i64)rec.raw[r] / send_size : 0;
    clock[k] = rec.clock[r];
}

void launch_tb_chunk_info(hipStream_t s, SlRecords rec, const i64* first, i64 nch, i64 send_size, u32* slot, i64* send,
                          i64* clock) {
    if (nch > 0)
        hipLaunchKernelGGL(k_tb_chunk_info, dim3((unsigned)((nch + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rec,
                           first, nch, send_size, slot, send, clock);
}

// per record its chunk: the last chunk whose first record is at or before it
__global__ __launch_bounds__(kBlock) void k_tb_chunk_of(const i64* __restrict__ first, i64 nch, i64 M, i64* chunk_of) {
    const i64 r = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (r >= M) return;
    i64 lo = 0, hi = nch;
    while (hi - lo > 1) {
        const i64 mid = (lo + hi) >> 1;
        if (first[mid] <= r) lo = mid;
        else hi = mid;
    }
    chunk_of[r] = lo;
}

void launch_tb_chunk_of(hipStream_t s, const i64* first, i64 nch, i64 M, i64* chunk_of) {
    if (M > 0)
        hipLaunchKernelGGL(k_tb_chunk_of, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, first, nch, M,
                           chunk_of);
}

// per record: its chunk (inclusive count of chunk starts - 1, from the flags' scan), its group slot and
// its (partition, group) state slot
__global__ __launch_bounds__(kBlock) void k_tb_pairs(SlRecords rec, i64 M, ColSet cols, KeyPlan gkp, KeyTable gkt,
                                                    KeyTable pgkt, u32* pair, u32* gslot) {
    const i64 r = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (r >= M) return;
    const u32 g = gkp.n ? key_slot(gkt, make_key(gkp, cols, rec.raw[r])) : 0u;
    gslot[r] = g;
    pair[r] = key_slot(pgkt, ((u64)rec.slot[r] << 32) | g);
}

void launch_tb_pairs(hipStream_t s, SlRecords rec, i64 M, ColSet cols, KeyPlan gkp, KeyTable gkt, KeyTable pgkt,
                     u32* pair, u32* gslot) {
    if (M > 0)
        hipLaunchKernelGGL(k_tb_pairs, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, rec, M, cols, gkp,
                           gkt, pgkt, pair, gslot);
}

// one thread per state segment of the records sorted stably by state slot (sidx: record indices)
template <int NA>
__global__ __launch_bounds__(64) void k_tb_fold(const i64* __restrict__ seg_start, i64 n_seg, i64 M,
                                               const u32* __restrict__ skey, const u32* __restrict__ sidx, SlRecords rec,
                                               const i64* __restrict__ chunk_of, const i64* __restrict__ chunk_bid,
                                               const u32* __restrict__ gslot, AggPlan ap, TbState S, i64 chunk_base,
                                               SlxRows rows, u64* row_key, u32* row_part, unsigned int* n_rows,
                                               i64 seq_base) {
    const i64 t = (i64)blockIdx.x * 64 + threadIdx.x;
    if (t >= n_seg) return;
    const i64 lo = seg_start[t], hi = t + 1 < n_seg ? seg_start[t + 1] : M;
    const u32 st = skey[lo];
    i64 cnt = S.cnt[st], bid = S.bid[st];
    u64 f[NA];
    unsigned char h[NA];
#pragma unroll
    for (int a = 0; a < NA; a++) {
        f[a] = a < ap.n ? S.f[(size_t)a * S.n + st] : 0;
        h[a] = a < ap.n ? S.has[(size_t)a * S.n + st] : 0;
    }
    i64 first_r = -1;
    for (i64 i = lo; i < hi; i++) {
        const u32 r = sidx[i];
        const i64 ch = chunk_of[r];
        const i64 b = chunk_bid[ch];
        if (b != bid) {  // a RESET of the partition since the state's last event: fresh state
            bid = b;
            cnt = 0;
#pragma unroll
            for (int a = 0; a < NA; a++) { f[a] = 0; h[a] = 0; }
        }
        if (first_r < 0) first_r = r;
        cnt++;
#pragma unroll
        for (int a = 0; a < NA; a++) {
            if (a >= ap.n) continue;
            const int kind = ap.kind[a];
            if (kind == AK_COUNT) continue;
            const u64 x = rec.vals[(size_t)ap.vcol[a] * rec.cap + r];
            if (kind == AK_SUM_L) {
                f[a] = (u64)((i64)f[a] + (i64)x);
                h[a] = 1;
            } else if (kind == AK_SUM_D || kind == AK_AVG) {
                f[a] = (u64)__double_as_longlong((h[a] ? __longlong_as_double((i64)f[a]) : 0.0) + g_num(ap, a, x));
                h[a] = 1;
            } else {
                const bool take = !h[a] || g_worse(kind, f[a], x);
                f[a] = take ? x : f[a];
                h[a] = 1;
            }
        }
        const bool last = i + 1 == hi || chunk_of[sidx[i + 1]] != ch;
        if (!last) continue;
        // the group's row of this chunk: its last event carrying the running values (QuerySelector
        // .processInBatchGroupBy :315-374: LinkedHashMap.put keeps the group's first position)
        const u32 o = wave_row_slot(n_rows);
        rows.ts[o] = rec.ts[r];
        rows.rep[o] = seq_base + (i64)rec.raw[r];
        rows.slot[o] = gslot[r];
        rows.ch[o] = chunk_base + ch;
        rows.clk[o] = rec.clock[r];
        rows.exp[o] = 0;
        row_part[o] = rec.slot[r];
#pragma unroll
        for (int a = 0; a < NA; a++) {
            if (a >= ap.n) continue;
            const int kind = ap.kind[a];
            u64 rv = 0;
            unsigned char rn = 0;
            if (kind == AK_COUNT) rv = (u64)cnt;
            else if (kind == AK_AVG) rv = (u64)__double_as_longlong(__longlong_as_double((i64)f[a]) / (double)cnt);
            else { rv = f[a]; rn = h[a] ? 0 : 1; }
            rows.vals[(size_t)a * rows.cap + o] = rv;
            rows.nulls[(size_t)a * rows.cap + o] = rn;
        }
        row_key[o] = ((u64)ch << 32) | (u64)(u32)first_r;
        first_r = -1;
    }
    S.cnt[st] = cnt;
    S.bid[st] = bid;
#pragma unroll
    for (int a = 0; a < NA; a++) {
        if (a >= ap.n) continue;
        S.f[(size_t)a * S.n + st] = f[a];
        S.has[(size_t)a * S.n + st] = h[a];
    }
}

void launch_tb_fold(hipStream_t s, const i64* seg_start, i64 n_seg, i64 M, const u32* skey, const u32* sidx,
                    SlRecords rec, const i64* chunk_of, const i64* chunk_bid, const u32* gslot, AggPlan ap, TbState S,
                    i64 chunk_base, SlxRows rows, u64* row_key, u32* row_part, unsigned int* n_rows, i64 seq_base) {
    if (n_seg <= 0) return;
    const unsigned grid = (unsigned)((n_seg + 63) / 64);
    if (ap.n <= 4)
        hipLaunchKernelGGL(k_tb_fold<4>, dim3(grid), dim3(64), 0, s, seg_start, n_seg, M, skey, sidx, rec, chunk_of,
                           chunk_bid, gslot, ap, S, chunk_base, rows, row_key, row_part, n_rows, seq_base);
    else
        hipLaunchKernelGGL(k_tb_fold<8>, dim3(grid), dim3(64), 0, s, seg_start, n_seg, M, skey, sidx, rec, chunk_of,
                           chunk_bid, gslot, ap, S, chunk_base, rows, row_key, row_part, n_rows, seq_base);
}

}  // namespace shd
