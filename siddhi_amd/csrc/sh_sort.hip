// sh_sort.hip — stable device radix sort of the sliding window's records by key slot (rocPRIM
// onesweep), so that every key's records of a push form one contiguous run in event order.
#include <hip/hip_runtime.h>

#include <cstring>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/device/device_scan.hpp>

#include "sh_internal.h"

namespace shd {

// bits needed for slots < nslots
static unsigned slot_bits(i64 nslots) {
    unsigned b = 1;
    while (b < 32 && ((i64)1 << b) < nslots) b++;
    return b;
}

// temp == nullptr: *bytes = the temporary storage needed. Sorts keys (slots) stably, values = the
// records' ranks 0..M-1.
int sort_slot_ranks(void* temp, size_t* bytes, const u32* slot, u32* slot_out, u32* rank_out, i64 M, i64 nslots,
                    hipStream_t s) {
    rocprim::counting_iterator<u32> iota(0u);
    hipError_t e = rocprim::radix_sort_pairs(temp, *bytes, slot, slot_out, iota, rank_out, (unsigned)M, 0u,
                                             slot_bits(nslots), s);
    return e == hipSuccess ? 0 : -1;
}

// stable sort of (u64 key, u32 value) pairs over all 64 key bits (aggregation retrieval)
int sort_u64_pairs(void* temp, size_t* bytes, const u64* keys, u64* keys_out, const u32* vals, u32* vals_out, i64 n,
                   hipStream_t s) {
    hipError_t e = rocprim::radix_sort_pairs(temp, *bytes, keys, keys_out, vals, vals_out, (unsigned)n, 0u, 64u, s);
    return e == hipSuccess ? 0 : -1;
}

// the same over key bits [0, end_bit) only (the partition lanes' (chunk, group) entry keys)
int sort_u64_pairs_bits(void* temp, size_t* bytes, const u64* keys, u64* keys_out, const u32* vals, u32* vals_out,
                        i64 n, unsigned end_bit, hipStream_t s) {
    hipError_t e =
        rocprim::radix_sort_pairs(temp, *bytes, keys, keys_out, vals, vals_out, (unsigned)n, 0u, end_bit, s);
    return e == hipSuccess ? 0 : -1;
}

// the same over key bits [begin_bit, end_bit) (keys whose low bits follow from the high ones)
int sort_u64_pairs_range(void* temp, size_t* bytes, const u64* keys, u64* keys_out, const u32* vals, u32* vals_out,
                         i64 n, unsigned begin_bit, unsigned end_bit, hipStream_t s) {
    hipError_t e = rocprim::radix_sort_pairs(temp, *bytes, keys, keys_out, vals, vals_out, (unsigned)n, begin_bit, end_bit, s);
    return e == hipSuccess ? 0 : -1;
}

// stable sort of u64 keys over bits [0, end_bit), values = the keys' input positions
int sort_u64_iota_bits(void* temp, size_t* bytes, const u64* keys, u64* keys_out, u32* vals_out, i64 n,
                       unsigned end_bit, hipStream_t s) {
    rocprim::counting_iterator<u32> iota(0u);
    hipError_t e = rocprim::radix_sort_pairs(temp, *bytes, keys, keys_out, iota, vals_out, (unsigned)n, 0u, end_bit, s);
    return e == hipSuccess ? 0 : -1;
}

// inclusive running maximum (the playback clock over the sends' last timestamps)
int scan_max_i64(void* temp, size_t* bytes, const i64* in, i64* out, i64 n, hipStream_t s) {
    return rocprim::inclusive_scan(temp, *bytes, in, out, (size_t)n, rocprim::maximum<i64>(), s) != hipSuccess;
}

}  // namespace shd
