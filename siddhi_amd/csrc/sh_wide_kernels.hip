// sh_wide_kernels.hip — interning levels and the decode walk of wide group keys (sh_wide.h).
#include "sh_device.h"
#include "sh_wide.h"

namespace shd {

// one level over every event: the level's key from its 2-column view, interned into its table. A level
// over stream columns only evaluates the filter; one over an earlier level's ids follows that level
// (kNoId = dropped). The chain's last level writes 0 for dropped events (the window's key column).
__global__ __launch_bounds__(kBlock) void k_wide_level(ColSet full, FilterProg f, int first, ColSet cs2, KeyPlan kp,
                                                      KeyTable t, const u32* __restrict__ prev, int last, i64 n,
                                                      u32* ids) {
    const i64 e = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (e >= n) return;
    const bool pass = first ? eval_filter(f, full, e) : prev[e] != kNoId;
    ids[e] = pass ? key_slot(t, make_key(kp, cs2, e)) : (last ? 0u : kNoId);
}

void launch_wide_level(hipStream_t s, ColSet full, FilterProg f, int first, ColSet cs2, const WideLevel& lv,
                       const u32* prev, int last, i64 n, u32* ids) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_wide_level, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, full, f, first,
                       cs2, lv.kp, lv.t, prev, last, n, ids);
}

// ids -> the group-by values ([group column][n], as sh_out reports keys): from the last level back along
// the chain; a component that is an earlier level's id is walked too (a 64-bit column's own level)
__global__ __launch_bounds__(kBlock) void k_wide_decode(WideDev w, const i64* __restrict__ idv, i64 n, i64* out) {
    const i64 r = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (r >= n) return;
    int lvl_stack[kWideLevels];
    u32 id_stack[kWideLevels];
    int sp = 0;
    lvl_stack[sp] = w.last;
    id_stack[sp] = (u32)idv[r];
    sp++;
    while (sp > 0) {
        sp--;
        const WideLevel& L = w.lv[lvl_stack[sp]];
        const u64 key = slot_key(L.t, id_stack[sp]);
        if (L.kp.n == 1) {
            // a one-column key is the value's 8-byte raw form already (ints sign-extended, floats widened
            // to double bits with NaN canonical): as sh_out reports it
            if (L.out[0] >= 0) out[(i64)L.out[0] * n + r] = (i64)key;
            continue;
        }
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const u32 x = j == 0 ? (u32)(key >> 32) : (u32)key;
            if (L.out[j] >= 0) {
                out[(i64)L.out[j] * n + r] = unpack_part(L.kp, j, x);
            } else if (sp < kWideLevels) {
                lvl_stack[sp] = -L.out[j] - 1;
                id_stack[sp] = x;
                sp++;
            }
        }
    }
}

void launch_wide_decode(hipStream_t s, const WideDev& w, const i64* ids, i64 n, i64* out) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_wide_decode, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, w, ids, n, out);
}

}  // namespace shd
