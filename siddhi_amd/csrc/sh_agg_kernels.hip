// sh_agg_kernels.hip — gfx950 kernels of the incremental-aggregation roll-up levels (minutes ... years).
//
// The root duration runs on the batch-window pipeline (sh_kernels.hip). Every dispatch of a level's
// store sends one row per (bucket, key) to the next duration (IncrementalExecutor.dispatchEvent,
// core/aggregation/IncrementalExecutor.java:201-258), whose BaseIncrementalValueStore folds them with
// sum / min / max executors (BaseIncrementalValueStore.process :141-160). Here a level's store is a
// device hash table keyed by (bucket, key) with one 8-byte state per base value.
#include "sh_device.h"
#include "sh_agg.h"

namespace shd {

// (the GMT calendar helpers floor_div_d / days_from_civil_d / civil_from_days_d are in sh_device.h)

// getStartTimeOfAggregates (IncrementalTimeConverterUtil.java:52-69); sec/min use `t - t % d`
__device__ __forceinline__ i64 start_of_gmt(i64 t, int dur) {
    switch (dur) {
        case SH_DUR_SECONDS: return t - t % 1000;
        case SH_DUR_MINUTES: return t - t % 60000;
        case SH_DUR_HOURS: return floor_div_d(t, 3600000) * 3600000;
        case SH_DUR_DAYS: return floor_div_d(t, 86400000) * 86400000;
        default: {
            i64 days = floor_div_d(t, 86400000);
            i64 y; unsigned m, d;
            civil_from_days_d(days, y, m, d);
            if (dur == SH_DUR_MONTHS) return days_from_civil_d(y, m, 1) * 86400000;
            return days_from_civil_d(y, 1, 1) * 86400000;
        }
    }
}

// in the aggregation's time zone (a fixed offset): hours and longer start at the zone's local boundaries
__device__ __forceinline__ i64 start_of_dev(i64 t, int dur, i64 tz) {
    return dur >= SH_DUR_HOURS ? start_of_gmt(t + tz, dur) - tz : start_of_gmt(t, dur);
}

__device__ __forceinline__ u64 level_key(int has_bucket, i64 bucket, i64 key) {
    if (!has_bucket) return (u64)key;
    return ((u64)(u32)(bucket / 1000) << 32) | (u64)(u32)key;
}

// one lookup per incoming row; `first_seq` keeps the arrival index of a slot's first row since the last
// dispatch so extraction can restore insertion order (the oracle's store order)
__global__ __launch_bounds__(kBlock) void k_level_lookup(i64 n, const i64* __restrict__ bucket_in,
                                                        const i64* __restrict__ key_in, int has_bucket, int dur,
                                                        LevelDev L, u32 epoch, u32 seq0, u32* slot_out, int* dup, i64 tz) {
    i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    i64 cb = has_bucket ? start_of_dev(bucket_in[i], dur, tz) : 0;
    u32 pos = key_slot(L.kt, level_key(has_bucket, cb, key_in ? key_in[i] : 0));
    slot_out[i] = pos;
    atomicMin(&L.first_seq[pos], seq0 + (u32)i);
    u32 old = atomicExch(&L.tag[pos], epoch);
    if (old == epoch) atomicExch(dup, (int)epoch);  // this merge's epoch: no reset between merges
}

__device__ __forceinline__ void level_fold(const LevelDev& L, const BasePlan& bp, u32 pos, const u64* vin,
                                           i64 stride, i64 i) {
    u64* rec = L.vals + (size_t)pos * L.vs;  // the slot's values and has-mask share a line
    const u64 has = rec[bp.n];
    for (int b = 0; b < bp.n; b++) {
        u64 x = vin[(size_t)b * stride + i];
        const bool first = !((has >> b) & 1);
        u64 cur = rec[b], r = cur;
        switch (bp.kind[b]) {
            case AK_SUM_L: case AK_COUNT: r = (u64)((first ? 0 : (i64)cur) + (i64)x); break;  // sum += v
            case AK_SUM_D:
                r = (u64)__double_as_longlong((first ? 0.0 : __longlong_as_double((i64)cur)) + __longlong_as_double((i64)x));
                break;
            case AK_MIN_L: if (first || (i64)cur > (i64)x) r = x; break;
            case AK_MAX_L: if (first || (i64)cur < (i64)x) r = x; break;
            case AK_MIN_D: if (first || __longlong_as_double((i64)cur) > __longlong_as_double((i64)x)) r = x; break;
            case AK_MAX_D: if (first || __longlong_as_double((i64)cur) < __longlong_as_double((i64)x)) r = x; break;
            case AK_MIN_F: if (first || (float)__longlong_as_double((i64)cur) > (float)__longlong_as_double((i64)x)) r = x; break;
            case AK_MAX_F: if (first || (float)__longlong_as_double((i64)cur) < (float)__longlong_as_double((i64)x)) r = x; break;
        }
        rec[b] = r;
    }
    rec[bp.n] = (1ull << bp.n) - 1;
}

// The merge of one batch of rows: rows with distinct slots fold in parallel; when the lookup saw two
// rows share a slot (late events) one lane folds them all in row order. The choice is made on the
// device from the lookup's flag, so the host does not wait between the two kernels.
__global__ __launch_bounds__(kBlock) void k_level_fold(i64 n, const u32* __restrict__ slots,
                                                      const u64* __restrict__ vin, i64 stride, LevelDev L,
                                                      BasePlan bp, const int* __restrict__ dup, u32 epoch) {
    if (*dup == (int)epoch) {
        if (blockIdx.x != 0 || threadIdx.x != 0) return;
        for (i64 i = 0; i < n; i++) level_fold(L, bp, slots[i], vin, stride, i);
        return;
    }
    i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    level_fold(L, bp, slots[i], vin, stride, i);
}

void launch_level_merge(hipStream_t s, i64 n, const i64* bucket_in, const i64* key_in, int has_bucket, int dur,
                        const u64* vin, i64 stride, LevelDev L, BasePlan bp, u32 epoch, u32 seq0, u32* slots,
                        int* dup_dev, i64 tz) {
    if (n == 0) return;
    unsigned g = (unsigned)((n + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_level_lookup, dim3(g), dim3(kBlock), 0, s, n, bucket_in, key_in, has_bucket, dur, L, epoch,
                       seq0, slots, dup_dev, tz);
    hipLaunchKernelGGL(k_level_fold, dim3(g), dim3(kBlock), 0, s, n, slots, vin, stride, L, bp, dup_dev, epoch);
}

__global__ __launch_bounds__(kBlock) void k_table_append(i64 n, const i64* __restrict__ bucket,
                                                        const i64* __restrict__ key, const u64* __restrict__ vals,
                                                        i64 vstride, int nb, i64* t_bucket, i64* t_key, u64* t_vals,
                                                        i64 t_cap) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    t_bucket[i] = bucket[i];
    t_key[i] = key[i];
    for (int b = 0; b < nb; b++) t_vals[(size_t)b * t_cap + i] = vals[(size_t)b * vstride + i];
}

void launch_table_append(hipStream_t s, i64 n, const i64* bucket, const i64* key, const u64* vals, i64 vstride,
                         int nb, i64* t_bucket, i64* t_key, u64* t_vals, i64 t_cap) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_table_append, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, bucket,
                       key, vals, vstride, nb, t_bucket, t_key, t_vals, t_cap);
}

// ---- extraction of a level's store (dispatch) -----------------------------------------------------
// order[first_seq[slot]] = slot, so walking `order` visits the slots in first-arrival order
// reset = false: the retrieval's read of the in-progress store (the store stays as it is)
__global__ __launch_bounds__(kBlock) void k_level_mark(LevelDev L, int reset) {
    i64 p = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (p >= L.nslots) return;
    u32 f = L.first_seq[p];
    if (f != 0xFFFFFFFFu) {
        L.order[f] = (u32)p;
        if (reset) L.first_seq[p] = 0xFFFFFFFFu;
    }
}

__global__ __launch_bounds__(kBlock) void k_level_count(LevelDev L, i64 n_in, i64* blk_cnt) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    i64 c = 0;
    for (int i = 0; i < kItems; i++) {
        i64 q = base + i;
        if (q < n_in && L.order[q] != 0xFFFFFFFFu) c++;
    }
    i64 t = block_reduce(c, SumOp(), 0);
    if (threadIdx.x == 0) blk_cnt[blockIdx.x] = t;
}

__global__ __launch_bounds__(kBlock) void k_level_extract(LevelDev L, BasePlan bp, int has_bucket, i64 store_ts,
                                                         i64 n_in, const i64* blk_pre, i64 cap, i64* out_bucket,
                                                         i64* out_key, u64* out_vals, int clear) {
    i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    u32 slot[kItems];
    i64 c = 0;
    for (int i = 0; i < kItems; i++) {
        i64 q = base + i;
        slot[i] = q < n_in ? L.order[q] : 0xFFFFFFFFu;
        c += slot[i] != 0xFFFFFFFFu;
    }
    i64 r = block_excl_scan(c, SumOp(), 0, nullptr) + blk_pre[blockIdx.x];
    for (int i = 0; i < kItems; i++) {
        if (slot[i] == 0xFFFFFFFFu) continue;
        u32 p = slot[i];
        u64 k = slot_key(L.kt, p);
        if (has_bucket) {
            out_bucket[r] = (i64)(u32)(k >> 32) * 1000;
            out_key[r] = (i64)(int)(u32)k;
        } else {
            out_bucket[r] = store_ts;
            out_key[r] = (i64)k;
        }
        u64* rec = L.vals + (size_t)p * L.vs;
        for (int b = 0; b < bp.n; b++) out_vals[(size_t)b * cap + r] = rec[b];
        if (clear) rec[bp.n] = 0;
        if (clear && p <= L.kt.mask) L.kt.keys[p] = kEmptyKey;  // BaseIncrementalValueStore.clearValues (:73-78)
        r++;
    }
}

void launch_level_mark(hipStream_t s, LevelDev L, i64 n_in, bool reset) {
    (void)hipMemsetAsync(L.order, 0xFF, (size_t)n_in * 4, s);
    unsigned g = (unsigned)((L.nslots + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_level_mark, dim3(g), dim3(kBlock), 0, s, L, reset ? 1 : 0);
}

void launch_level_count(hipStream_t s, LevelDev L, i64 n_in, i64* blk, int nblk) {
    hipLaunchKernelGGL(k_level_count, dim3(nblk), dim3(kBlock), 0, s, L, n_in, blk);
}

void launch_level_extract(hipStream_t s, LevelDev L, BasePlan bp, int has_bucket, i64 store_ts, i64 n_in, i64* blk,
                          int nblk, i64 cap, i64* out_bucket, i64* out_key, u64* out_vals, bool clear) {
    hipLaunchKernelGGL(k_level_extract, dim3(nblk), dim3(kBlock), 0, s, L, bp, has_bucket, store_ts, n_in, blk, cap,
                       out_bucket, out_key, out_vals, clear ? 1 : 0);
}

// ---- retrieval (sh_aggregation_find) ---------------------------------------------------------------
// rows re-bucketed to the `per` duration; rows outside [start, end) get bucket -1 (sorted last, dropped)
__global__ __launch_bounds__(kBlock) void k_find_rebucket(i64 n, const i64* __restrict__ bucket_in, int per, i64 start,
                                                         i64 end, i64* bucket_out, u32* idx, i64 tz) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const i64 b = start_of_dev(bucket_in[i], per, tz);
    bucket_out[i] = (b >= start && b < end) ? b : -1;
    idx[i] = (u32)i;
}

__global__ __launch_bounds__(kBlock) void k_find_gather_u64(i64 n, const u32* __restrict__ idx, const i64* __restrict__ src,
                                                           u64* dst, u64 flip) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) dst[i] = (u64)src[idx[i]] ^ flip;
}

// group starts in (bucket, key) order; out-of-range rows (bucket -1) start no group
__global__ __launch_bounds__(kBlock) void k_find_starts(i64 n, const u32* __restrict__ idx, const i64* __restrict__ bucket,
                                                       const i64* __restrict__ key, u32* flag) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i > n) return;
    if (i == n) { flag[i] = 0; return; }
    const u32 r = idx[i];
    bool st = bucket[r] >= 0;
    if (st && i > 0) {
        const u32 q = idx[i - 1];
        st = bucket[q] != bucket[r] || key[q] != key[r];
    }
    flag[i] = st ? 1u : 0u;
}

// one thread per group: its rows folded in input order with the base executors' semantics
// (sum / count: 0 + v1 + v2 ..., min / max: first value then compares; OutOfOrderEventsDataAggregator,
// IncrementalDataAggregator)
__global__ __launch_bounds__(kBlock) void k_find_fold(i64 n, const u32* __restrict__ idx, const u32* __restrict__ flag,
                                                     const u32* __restrict__ pre, const i64* __restrict__ bucket,
                                                     const i64* __restrict__ key, const u64* __restrict__ vals,
                                                     i64 vstride, BasePlan bp, i64 cap, i64* out_bucket, i64* out_key,
                                                     u64* out_vals) {
    const i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    if (!flag[i]) return;  // not a group's first row
    const u32 r = idx[i];
    const i64 o = pre[i];
    u64 acc[SH_MAX_AGGS];
    for (int b = 0; b < bp.n; b++) acc[b] = vals[(size_t)b * vstride + r];
    for (int b = 0; b < bp.n; b++)
        if (bp.kind[b] == AK_SUM_D) acc[b] = (u64)__double_as_longlong(0.0 + __longlong_as_double((i64)acc[b]));
    for (i64 j = i + 1; j < n && !flag[j]; j++) {
        const u32 q = idx[j];
        if (bucket[q] < 0) break;  // the out-of-range rows sorted last
        for (int b = 0; b < bp.n; b++) {
            const u64 x = vals[(size_t)b * vstride + q];
            switch (bp.kind[b]) {
                case AK_SUM_L: case AK_COUNT: acc[b] = (u64)((i64)acc[b] + (i64)x); break;
                case AK_SUM_D:
                    acc[b] = (u64)__double_as_longlong(__longlong_as_double((i64)acc[b]) + __longlong_as_double((i64)x));
                    break;
                case AK_MIN_L: if ((i64)acc[b] > (i64)x) acc[b] = x; break;
                case AK_MAX_L: if ((i64)acc[b] < (i64)x) acc[b] = x; break;
                case AK_MIN_D: if (__longlong_as_double((i64)acc[b]) > __longlong_as_double((i64)x)) acc[b] = x; break;
                case AK_MAX_D: if (__longlong_as_double((i64)acc[b]) < __longlong_as_double((i64)x)) acc[b] = x; break;
                case AK_MIN_F: if ((float)__longlong_as_double((i64)acc[b]) > (float)__longlong_as_double((i64)x)) acc[b] = x; break;
                case AK_MAX_F: if ((float)__longlong_as_double((i64)acc[b]) < (float)__longlong_as_double((i64)x)) acc[b] = x; break;
            }
        }
    }
    out_bucket[o] = bucket[r];
    out_key[o] = key[r];
    for (int b = 0; b < bp.n; b++) out_vals[(size_t)b * cap + o] = acc[b];
}

void launch_find_rebucket(hipStream_t s, i64 n, const i64* bucket_in, int per, i64 start, i64 end, i64* bucket_out,
                          u32* idx, i64 tz) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_find_rebucket, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, bucket_in,
                       per, start, end, bucket_out, idx, tz);
}

void launch_find_gather_u64(hipStream_t s, i64 n, const u32* idx, const i64* src, u64* dst, u64 flip) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_find_gather_u64, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, idx,
                       src, dst, flip);
}

void launch_find_starts(hipStream_t s, i64 n, const u32* idx, const i64* bucket, const i64* key, u32* flag) {
    hipLaunchKernelGGL(k_find_starts, dim3((unsigned)((n + 1 + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, idx,
                       bucket, key, flag);
}

void launch_find_fold(hipStream_t s, i64 n, const u32* idx, const u32* flag, const u32* pre, const i64* bucket,
                      const i64* key, const u64* vals, i64 vstride, BasePlan bp, i64 cap, i64* out_bucket,
                      i64* out_key, u64* out_vals) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_find_fold, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, n, idx, flag,
                       pre, bucket, key, vals, vstride, bp, cap, out_bucket, out_key, out_vals);
}

// min / max of an int64 column (event-time span of a push -> root key-table bound)
// min / max of an i64 column in two passes: per-block partials (16-byte loads), then one block
// folds them (a single pair of global atomics hit by every block serialised at the L2)
constexpr int kMinmaxBlocks = 512;
__global__ __launch_bounds__(kBlock) void k_minmax_i64(const i64* __restrict__ x, i64 n, i64* part) {
    i64 lo = INT64_MAX, hi = INT64_MIN;
    const i64 n2 = n >> 1;
    const longlong2* x2 = (const longlong2*)x;
    for (i64 i = (i64)blockIdx.x * kBlock + threadIdx.x; i < n2; i += (i64)gridDim.x * kBlock) {
        const longlong2 v = x2[i];
        lo = min(lo, (i64)min(v.x, v.y));
        hi = max(hi, (i64)max(v.x, v.y));
    }
    if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
        lo = min(lo, x[n - 1]);
        hi = max(hi, x[n - 1]);
    }
    lo = block_reduce(lo, MinOp(), INT64_MAX);
    hi = block_reduce(hi, MaxOp(), INT64_MIN);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = lo;
        part[2 * blockIdx.x + 1] = hi;
    }
}

__global__ __launch_bounds__(kBlock) void k_minmax_final(const i64* __restrict__ part, int nb, i64* out) {
    i64 lo = INT64_MAX, hi = INT64_MIN;
    for (int i = threadIdx.x; i < nb; i += kBlock) {
        lo = min(lo, part[2 * i]);
        hi = max(hi, part[2 * i + 1]);
    }
    lo = block_reduce(lo, MinOp(), INT64_MAX);
    hi = block_reduce(hi, MaxOp(), INT64_MIN);
    if (threadIdx.x == 0) {
        out[0] = lo;
        out[1] = hi;
    }
}

__global__ void k_minmax_init(i64* out) {
    out[0] = INT64_MAX;
    out[1] = INT64_MIN;
}

size_t minmax_scratch_bytes() { return 16 + (size_t)kMinmaxBlocks * 16; }

// a column that is not 16-byte aligned: scalar loads
__global__ __launch_bounds__(kBlock) void k_minmax_i64_s(const i64* __restrict__ x, i64 n, i64* part) {
    i64 lo = INT64_MAX, hi = INT64_MIN;
    for (i64 i = (i64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (i64)gridDim.x * kBlock) {
        lo = min(lo, x[i]);
        hi = max(hi, x[i]);
    }
    lo = block_reduce(lo, MinOp(), INT64_MAX);
    hi = block_reduce(hi, MaxOp(), INT64_MIN);
    if (threadIdx.x == 0) {
        part[2 * blockIdx.x] = lo;
        part[2 * blockIdx.x + 1] = hi;
    }
}

void launch_minmax_i64(hipStream_t s, const i64* x, i64 n, i64* out) {
    if (n <= 0) {
        hipLaunchKernelGGL(k_minmax_init, dim3(1), dim3(1), 0, s, out);
        return;
    }
    const unsigned g = (unsigned)std::max<i64>(1, std::min<i64>(kMinmaxBlocks, (n / 2 + kBlock - 1) / kBlock));
    if (((uintptr_t)x & 15) == 0)
        hipLaunchKernelGGL(k_minmax_i64, dim3(g), dim3(kBlock), 0, s, x, n, out + 2);
    else
        hipLaunchKernelGGL(k_minmax_i64_s, dim3(g), dim3(kBlock), 0, s, x, n, out + 2);
    hipLaunchKernelGGL(k_minmax_final, dim3(1), dim3(kBlock), 0, s, out + 2, (int)g, out);
}

__global__ __launch_bounds__(kBlock) void k_pend_bucket_range(const u32* __restrict__ pos, i64 n, KeyTable kt,
                                                              u32 ref, i64* out) {
    i64 lo = INT64_MAX, hi = INT64_MIN;
    for (i64 i = (i64)blockIdx.x * kBlock + threadIdx.x; i < n; i += (i64)gridDim.x * kBlock) {
        // band keys: the bucket's signed distance from the band's row 0; otherwise the whole u32 bucket
        const u32 b = (u32)(slot_key(kt, pos[i]) >> 32);
        const i64 d = kt.lk ? (i64)(int)(b - ref) : (i64)b;
        lo = d < lo ? d : lo;
        hi = d > hi ? d : hi;
    }
    lo = block_reduce(lo, MinOp(), INT64_MAX);
    hi = block_reduce(hi, MaxOp(), INT64_MIN);
    if (threadIdx.x == 0) {
        atomicMin((long long*)&out[0], (long long)lo);
        atomicMax((long long*)&out[1], (long long)hi);
    }
}

void launch_pend_bucket_range(hipStream_t s, const u32* pos, i64 n, KeyTable kt, u32 ref, i64* out) {
    hipLaunchKernelGGL(k_minmax_init, dim3(1), dim3(1), 0, s, out);
    if (n <= 0) return;
    const i64 g = std::min<i64>((n + kBlock - 1) / kBlock, 1024);
    hipLaunchKernelGGL(k_pend_bucket_range, dim3((unsigned)g), dim3(kBlock), 0, s, pos, n, kt, ref, out);
}

__global__ __launch_bounds__(kBlock) void k_fill_i64(i64* p, i64 n, i64 v) {
    i64 i = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (i < n) p[i] = v;
}

void launch_fill_i64(hipStream_t s, i64* p, i64 n, i64 v) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_fill_i64, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, p, n, v);
}

}  // namespace shd

namespace shd {

}  // namespace shd
