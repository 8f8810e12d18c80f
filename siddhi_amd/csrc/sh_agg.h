// sh_agg.h — device structures of the incremental-aggregation roll-up levels.
#pragma once
#include "sh_internal.h"

namespace shd {

// base values of a duration's store (AggregationParser.populateFinalBaseAggregators :693-728):
// SUM_L / SUM_D (sum of convert(v, 'long'|'double')), COUNT (sum of 1L), MIN_* / MAX_*.
struct BasePlan {
    int n;
    int pad;
    int kind[SH_MAX_AGGS];
};

struct LevelDev {
    KeyTable kt;         // (bucket, key) -> slot
    i64 nslots;          // mask + 2
    u64* vals;           // [nslots][vs]: the slot's base values, then a word whose bit b = base b is set
    int vs;              // n_bases + 1
    u32* tag;            // [nslots] duplicate detection epoch
    u32* first_seq;      // [nslots] arrival index of the slot's first row since the last dispatch
    u32* order;          // [rows since the last dispatch] slot by first arrival
};

void launch_level_merge(hipStream_t s, i64 n, const i64* bucket_in, const i64* key_in, int has_bucket, int dur,
                        const u64* vin, i64 stride, LevelDev L, BasePlan bp, u32 epoch, u32 seq0, u32* slots,
                        int* dup_dev, i64 tz);
// rows appended to a duration table: bucket, key and every base column in one launch
void launch_table_append(hipStream_t s, i64 n, const i64* bucket, const i64* key, const u64* vals, i64 vstride,
                         int nb, i64* t_bucket, i64* t_key, u64* t_vals, i64 t_cap);
void launch_level_mark(hipStream_t s, LevelDev L, i64 n_in, bool reset = true);
void launch_level_count(hipStream_t s, LevelDev L, i64 n_in, i64* blk, int nblk);
void launch_level_extract(hipStream_t s, LevelDev L, BasePlan bp, int has_bucket, i64 store_ts, i64 n_in, i64* blk,
                          int nblk, i64 cap, i64* out_bucket, i64* out_key, u64* out_vals, bool clear = true);
// retrieval (sh_aggregation_find)
void launch_find_rebucket(hipStream_t s, i64 n, const i64* bucket_in, int per, i64 start, i64 end, i64* bucket_out,
                          u32* idx, i64 tz);
// dst[i] = src[idx[i]] ^ flip (flip = the sign bit: signed order as unsigned)
void launch_find_gather_u64(hipStream_t s, i64 n, const u32* idx, const i64* src, u64* dst, u64 flip = 0);
void launch_find_starts(hipStream_t s, i64 n, const u32* idx, const i64* bucket, const i64* key, u32* flag);
void launch_find_fold(hipStream_t s, i64 n, const u32* idx, const u32* flag, const u32* pre, const i64* bucket,
                      const i64* key, const u64* vals, i64 vstride, BasePlan bp, i64 cap, i64* out_bucket,
                      i64* out_key, u64* out_vals);
int sort_u64_pairs(void* temp, size_t* bytes, const u64* keys, u64* keys_out, const u32* vals, u32* vals_out, i64 n,
                   hipStream_t s);
int sort_u64_pairs_bits(void* temp, size_t* bytes, const u64* keys, u64* keys_out, const u32* vals, u32* vals_out,
                        i64 n, unsigned end_bit, hipStream_t s);
void launch_fill_i64(hipStream_t s, i64* p, i64 n, i64 v);
void launch_minmax_i64(hipStream_t s, const i64* x, i64 n, i64* out);  // out: minmax_scratch_bytes()
size_t minmax_scratch_bytes();
// time buckets of the root's queued events, relative to `ref` (out[0] = min, out[1] = max)
void launch_pend_bucket_range(hipStream_t s, const u32* pos, i64 n, KeyTable kt, u32 ref, i64* out);

}  // namespace shd
