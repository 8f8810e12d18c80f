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
    u64* vals;           // [n_bases][nslots]
    unsigned char* has;  // [n_bases][nslots]
    u32* tag;            // [nslots] duplicate detection epoch
    u32* first_seq;      // [nslots] arrival index of the slot's first row since the last dispatch
    u32* order;          // [rows since the last dispatch] slot by first arrival
};

void launch_level_merge(hipStream_t s, i64 n, const i64* bucket_in, const i64* key_in, int has_bucket, int dur,
                        const u64* vin, i64 stride, LevelDev L, BasePlan bp, u32 epoch, u32 seq0, u32* slots,
                        int* dup_dev, int* dup_host);
void launch_level_mark(hipStream_t s, LevelDev L, i64 n_in);
void launch_level_count(hipStream_t s, LevelDev L, i64 n_in, i64* blk, int nblk);
void launch_level_extract(hipStream_t s, LevelDev L, BasePlan bp, int has_bucket, i64 store_ts, i64 n_in, i64* blk,
                          int nblk, i64 cap, i64* out_bucket, i64* out_key, u64* out_vals);
void launch_fill_i64(hipStream_t s, i64* p, i64 n, i64 v);
void launch_minmax_i64(hipStream_t s, const i64* x, i64 n, i64* out);

}  // namespace shd
