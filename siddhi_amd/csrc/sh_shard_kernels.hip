// sh_shard_kernels.hip — gfx950 kernels of the sharded ingest: every rank holds a
// contiguous slice of the global stream, assigns each event its GLOBAL window (the playback clock
// and nextEmitTime are global, TimeBatchWindowProcessor.java:262-347) and re-keys it to the GPU that
// owns its group key. The all-to-all itself is done by the caller over RCCL/xGMI.
//
//   k_shard_assign  window of every event (clock carried in from the slices before), owner =
//                   mix64(key) % G, per-(owner, tile) histogram, window starts of the slice (and, for
//                   stream.current.event, every passing event's send clock: its row's flush clock)
//   k_shard_pack    stable multisplit of the passing events into per-owner runs of AoS records
//                   {key, slice position, ts, values...} (event order kept inside every run)
//   k_shard_unpack  received records -> SoA columns of the owner's pipeline (given-window mode)
#include "sh_device.h"

namespace shd {

// owner GPU of a group key: dictionary ids (dense keys) round-robin, so every owner's ids stay dense
// as id / G; other keys by a 64-bit mix (independent of the owner's Fibonacci slot hash)
__device__ __forceinline__ u32 owner_of(const KeyPlan& kp, u64 key, int G) {
    if (kp.dense) return (u32)key % (u32)G;
    return (u32)(mix64(key ^ 0x5851F42D4C957F2Dull) % (u64)G);
}

// code of a passing event: (W - W_base) << 4 | owner; kNoPos when it is filtered out
constexpr int kOwnerBits = 4;

// lengthBatch (LengthBatchWindowProcessor :206-243): the window of a passing event is
// (carry + global passing events before it) / L — wp.n_pend holds the carry plus the passing events
// of the slices before this one, blk_pass_pre the slice's tile prefix. A window start is recorded at
// the event after every L-th passing event, with the clock of the L-th event's send (the flush clock).
__global__ __launch_bounds__(kBlock) void k_shard_assign(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                        WinParams wp, const i64* __restrict__ blk_tl_pre,
                                                        const i64* __restrict__ blk_pass_pre, KeyPlan kp,
                                                        int G, int nblk, u32* code, i64* counts, Bound* bounds,
                                                        int max_bounds, int* n_bounds, i64* clk_out) {
    __shared__ u32 hist[kMaxShards];
    if (threadIdx.x < kMaxShards) hist[threadIdx.x] = 0;
    const i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    bool pass[kItems];
    i64 t[kItems];
    i64 tl = INT64_MIN;
    SendCursor sc(wp, base);
    load_items_i64(ts, base, wp.N, t, INT64_MIN);
    filter_items(f, cols, base, wp.N, pass);
    // one 32-bit key column (the usual wire key): the thread's keys in vector loads, codes stored as two
    // 16-byte words below (a lane's 8 scalar stores at a 32-byte stride otherwise)
    const bool vkey = kp.n == 1 && kp.div[0] == 0 && (kp.type[0] == SH_T_INT || kp.type[0] == SH_T_STRID);
    i64 kv[kItems];
    if (vkey) load_items_raw(cols, kp.col[0], base, wp.N, kv);
    u32 cd[kItems];
#pragma unroll
    for (int i = 0; i < kItems; i++) cd[i] = kNoPos;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        i64 e = base + i;
        bool in = e < wp.N;
        if (in && sc.last(wp, e)) tl = max(tl, t[i]);
        sc.next();
    }
    i64 pm = max(block_excl_scan(tl, MaxOp(), INT64_MIN, nullptr), blk_tl_pre[blockIdx.x]);
    const i64 c0 = wp.clock_valid ? wp.clock0 : INT64_MIN;
    const bool lb = wp.kind == SH_WIN_LENGTH_BATCH;
    if (lb) {
        i64 cnt = 0;
#pragma unroll
        for (int i = 0; i < kItems; i++) cnt += pass[i];
        i64 pcb = block_excl_scan(cnt, SumOp(), 0, nullptr) + blk_pass_pre[blockIdx.x] + wp.n_pend;
        SendCursor sc2(wp, base);
#pragma unroll
        for (int i = 0; i < kItems; i++) {
            i64 e = base + i;
            if (e >= wp.N) break;
            u32 c = kNoPos;
            if (pass[i] && clk_out) {  // (stream.current.event: the send's global clock, the row's flush clock)
                const i64 tsl = sc2.s == 1 ? t[i] : ts[sc2.last_of(wp, e)];
                clk_out[e] = max(c0, max(pm, tsl));
            }
            if (pass[i]) {
                const i64 Wr = pcb / wp.L;
                if ((pcb + 1) % wp.L == 0) {
                    const i64 tsl = sc2.s == 1 ? t[i] : ts[sc2.last_of(wp, e)];
                    int k = atomicAdd(n_bounds, 1);
                    if (k < max_bounds) {
                        Bound b;
                        b.idx = e + 1; b.W = wp.W_base + Wr + 1; b.clock = max(c0, max(pm, tsl));
                        b.clock_prev = b.clock; b.pcb = 0; b.pad = 0;
                        bounds[k] = b;
                    }
                }
                u32 o = owner_of(kp, vkey ? (u64)kv[i] : make_key(kp, cols, e), G);
                c = ((u32)Wr << kOwnerBits) | o;
                atomicAdd(&hist[o], 1u);
                pcb++;
            }
            cd[i] = c;
            if (sc2.last(wp, e)) pm = max(pm, t[i]);
            sc2.next();
        }
    }
    const i64 E0 = wp.E0;
    const int e0v = wp.e0_valid;
    if (!lb && base < wp.N) {
        SendCursor sc2(wp, base);
        i64 Wprev, clock_prev;
        if (base == 0) {
            Wprev = wp.W_open;
            clock_prev = c0;
        } else {
            if (sc2.r != 0) clock_prev = max(c0, max(pm, ts[sc2.last_of(wp, base)]));
            else clock_prev = max(c0, pm);
            Wprev = max(wp.W_open, wfun(wp, E0, e0v, 0, clock_prev));
        }
        WinCursor wc;
        wc.W = Wprev;
        wc.lim = INT64_MIN;
#pragma unroll
        for (int i = 0; i < kItems; i++) {
            i64 e = base + i;
            if (e >= wp.N) break;
            i64 tsl = sc2.s == 1 ? t[i] : ts[sc2.last_of(wp, e)];
            i64 clk = max(c0, max(pm, tsl));
            if (clk_out && pass[i]) clk_out[e] = clk;
            i64 W = max(wp.W_open, wc.at(wp, E0, e0v, 0, clk));
            if (W > Wprev) {
                int k = atomicAdd(n_bounds, 1);
                if (k < max_bounds) {
                    Bound b;
                    b.idx = e; b.W = W; b.clock = clk; b.clock_prev = clock_prev; b.pcb = 0; b.pad = 0;
                    bounds[k] = b;
                }
            }
            u32 c = kNoPos;
            if (pass[i]) {
                u32 o = owner_of(kp, vkey ? (u64)kv[i] : make_key(kp, cols, e), G);
                c = ((u32)(W - wp.W_base) << kOwnerBits) | o;
                atomicAdd(&hist[o], 1u);
            }
            cd[i] = c;
            Wprev = W;
            clock_prev = clk;
            if (sc2.last(wp, e)) pm = max(pm, t[i]);
            sc2.next();
        }
    }
    static_assert(kItems == 8, "two 16-byte code stores per thread");
    if (base + kItems <= wp.N) {
        uint4* q = (uint4*)(code + base);
        q[0] = make_uint4(cd[0], cd[1], cd[2], cd[3]);
        q[1] = make_uint4(cd[4], cd[5], cd[6], cd[7]);
    } else {
#pragma unroll
        for (int i = 0; i < kItems; i++)
            if (base + i < wp.N) code[base + i] = cd[i];
    }
    __syncthreads();
    if (threadIdx.x < G) counts[(i64)threadIdx.x * nblk + blockIdx.x] = hist[threadIdx.x];
}

void launch_shard_assign(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp, const i64* blk_tl_pre,
                         const i64* blk_pass_pre, const PushInfo* info, KeyPlan kp, int G, int nblk, u32* code,
                         i64* counts, Bound* bounds, int max_bounds, int* n_bounds, i64* clk_out) {
    (void)info;
    hipLaunchKernelGGL(k_shard_assign, dim3(nblk), dim3(kBlock), 0, s, ts, cols, f, wp, blk_tl_pre, blk_pass_pre, kp,
                       G, nblk, code, counts, bounds, max_bounds, n_bounds, clk_out);
}

// Sliding time(T) (TimeWindowProcessor :132-169): the owner needs, per passing event, the global
// clock of its send and PM = max ts over the passing events of the whole stream up to it (its expiry
// key, sh_sliding_kernels.hip); both are prefix quantities of the slice (blk_*_pre from the sliding
// prefix scan) continued from the slices before (wp.clock0, pm0). They travel as two extra raw
// columns of the record; code = owner (no window bits).
__global__ __launch_bounds__(kBlock) void k_shard_sl_assign(const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                           WinParams wp, const i64* __restrict__ blk_tl_pre,
                                                           const i64* __restrict__ blk_pm_pre, i64 pm0, KeyPlan kp,
                                                           int G, int nblk, u32* code, i64* counts, i64* clk_out,
                                                           i64* pm_out) {
    __shared__ u32 hist[kMaxShards];
    if (threadIdx.x < kMaxShards) hist[threadIdx.x] = 0;
    __syncthreads();
    const i64 base = (i64)blockIdx.x * kTile + (i64)threadIdx.x * kItems;
    bool pass[kItems];
    i64 tl = INT64_MIN, pm = INT64_MIN;
    filter_items(f, cols, base, wp.N, pass);
    const bool vkey = kp.n == 1 && kp.div[0] == 0 && (kp.type[0] == SH_T_INT || kp.type[0] == SH_T_STRID);
    i64 kv[kItems];
    if (vkey) load_items_raw(cols, kp.col[0], base, wp.N, kv);
    u32 cd[kItems];
#pragma unroll
    for (int i = 0; i < kItems; i++) cd[i] = kNoPos;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        const i64 e = base + i;
        if (e < wp.N) {
            const i64 t = ts[e];
            if (pass[i]) pm = max(pm, t);
            if (is_send_last(wp, e)) tl = max(tl, t);
        }
    }
    i64 cm = max(block_excl_scan(tl, MaxOp(), INT64_MIN, nullptr), blk_tl_pre[blockIdx.x]);
    i64 pmx = max(max(block_excl_scan(pm, MaxOp(), INT64_MIN, nullptr), blk_pm_pre[blockIdx.x]), pm0);
    const i64 c0 = wp.clock_valid ? wp.clock0 : INT64_MIN;
#pragma unroll
    for (int i = 0; i < kItems; i++) {
        const i64 e = base + i;
        if (e >= wp.N) break;
        const i64 t = ts[e];
        u32 c = kNoPos;
        if (pass[i]) {
            pmx = max(pmx, t);
            clk_out[e] = max(c0, max(cm, ts[send_last_of(wp, e)]));
            pm_out[e] = pmx;
            c = owner_of(kp, vkey ? (u64)kv[i] : make_key(kp, cols, e), G);
            atomicAdd(&hist[c], 1u);
        }
        cd[i] = c;
        if (is_send_last(wp, e)) cm = max(cm, t);
    }
    if (base + kItems <= wp.N) {
        uint4* q = (uint4*)(code + base);
        q[0] = make_uint4(cd[0], cd[1], cd[2], cd[3]);
        q[1] = make_uint4(cd[4], cd[5], cd[6], cd[7]);
    } else {
#pragma unroll
        for (int i = 0; i < kItems; i++)
            if (base + i < wp.N) code[base + i] = cd[i];
    }
    __syncthreads();
    if (threadIdx.x < G) counts[(i64)threadIdx.x * nblk + blockIdx.x] = hist[threadIdx.x];
}

void launch_shard_sl_assign(hipStream_t s, const i64* ts, ColSet cols, FilterProg f, WinParams wp,
                            const i64* blk_tl_pre, const i64* blk_pm_pre, i64 pm0, KeyPlan kp, int G, int nblk,
                            u32* code, i64* counts, i64* clk_out, i64* pm_out) {
    hipLaunchKernelGGL(k_shard_sl_assign, dim3(nblk), dim3(kBlock), 0, s, ts, cols, f, wp, blk_tl_pre, blk_pm_pre, pm0,
                       kp, G, nblk, code, counts, clk_out, pm_out);
}

// Stable multisplit by owner. Tile events are taken in kItems rounds of kBlock consecutive events;
// inside a round, the rank of an event among the same owner's events is (waves before) + (lanes
// before), so every owner's run keeps event order. offsets = exclusive scan of counts[o][tile].
__global__ __launch_bounds__(kBlock) void k_shard_pack(ColSet cols, const i64* __restrict__ ts,
                                                      const u32* __restrict__ code, KeyPlan kp, RawPlan rp, int G,
                                                      i64 N, int nblk, const i64* __restrict__ offsets, u32* out,
                                                      int rec_words, int key32, int narrow, i64 tsbase) {
    __shared__ u32 running[kMaxShards];
    __shared__ u32 wave_cnt[kBlock / 64][kMaxShards];
    const int tile = blockIdx.x;
    if (threadIdx.x < kMaxShards) running[threadIdx.x] = 0;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 lt_mask = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    __syncthreads();
    for (int r = 0; r < kItems; r++) {
        const i64 e = (i64)tile * kTile + (i64)r * kBlock + threadIdx.x;
        u32 c = e < N ? code[e] : kNoPos;
        bool ok = c != kNoPos;
        u32 o = ok ? (c & ((1u << kOwnerBits) - 1)) : 0;
        u64 peers = __ballot(ok);
#pragma unroll
        for (int bt = 0; bt < kOwnerBits; bt++) {
            bool bit = (o >> bt) & 1;
            u64 m = __ballot(bit);
            peers &= bit ? m : ~m;
        }
        u32 lrank = (u32)__popcll(peers & lt_mask);
        if (lane < G) wave_cnt[wave][lane] = 0;
        __syncthreads();
        if (ok && lrank == 0) wave_cnt[wave][o] = (u32)__popcll(peers);
        __syncthreads();
        if (ok) {
            u32 before = running[o];
            for (int w = 0; w < wave; w++) before += wave_cnt[w][o];
            i64 dst = offsets[(i64)o * nblk + tile] + before + lrank;
            u32* rec = out + dst * rec_words;
            const u64 key = make_key(kp, cols, e);
            int w8;  // first 8-byte word
            if (key32) {
                rec[0] = (u32)key;
                rec[1] = (u32)e;
                w8 = 2;
            } else {
                *(u64*)rec = key;
                rec[2] = (u32)e;
                rec[3] = 0;
                w8 = 4;
            }
            if (narrow) {
                // (32-bit wire key only) ts as its offset from the push's minimum, the raw words as
                // 4-byte-aligned pairs: 20 bytes for C2 instead of 24
                rec[2] = (u32)((u64)ts[e] - (u64)tsbase);
                for (int j = 0; j < rp.n; j++) {
                    const u64 v = (u64)load_raw(cols, rp.src[j], e);
                    rec[3 + 2 * j] = (u32)v;
                    rec[4 + 2 * j] = (u32)(v >> 32);
                }
            } else {
                u64* r8 = (u64*)(rec + w8);
                r8[0] = (u64)ts[e];
                for (int j = 0; j < rp.n; j++) r8[1 + j] = (u64)load_raw(cols, rp.src[j], e);
            }
        }
        __syncthreads();
        if (threadIdx.x < G) {
            u32 add = 0;
            for (int w = 0; w < kBlock / 64; w++) add += wave_cnt[w][threadIdx.x];
            running[threadIdx.x] += add;
        }
        __syncthreads();
    }
}

void launch_shard_pack(hipStream_t s, ColSet cols, const i64* ts, const u32* code, KeyPlan wkp, RawPlan rp, int G,
                       i64 N, int nblk, const i64* offsets, unsigned char* out, int rec_words, int key32, int narrow,
                       i64 tsbase) {
    hipLaunchKernelGGL(k_shard_pack, dim3(nblk), dim3(kBlock), 0, s, cols, ts, code, wkp, rp, G, N, nblk, offsets,
                       (u32*)out, rec_words, key32, narrow, tsbase);
}

// Received records -> the owner's SoA columns (8-byte raw form for every referenced column).
// role[c]: -1 unused, 0..15 raw slot, 16 + g component g of the wire key (kp = the wire key plan). The global index of a record is
// its source slice's base + its slice position; its window is that of the last global window start
// at or before it (binary search over the all-gathered starts), W_base before the first.
__global__ __launch_bounds__(kBlock) void k_shard_unpack(const u32* __restrict__ rec, i64 M, int rec_words, KeyPlan kp,
                                                        ColRoles roles, ShardSrc src,
                                                        const i64* __restrict__ bound_gidx,
                                                        const i64* __restrict__ bound_W, int n_bounds, i64 W_base,
                                                        i64* ts, ColPtrs cols, int* wcol, u64* gidx) {
    i64 m = (i64)blockIdx.x * kBlock + threadIdx.x;
    if (m >= M) return;
    const u32* r = rec + m * rec_words;
    u64 key;
    u32 pos;
    int w8;
    if (src.key32) { key = (u64)(i64)(int)r[0]; pos = r[1]; w8 = 2; }
    else { key = *(const u64*)r; pos = r[2]; w8 = 4; }
    const u64* r8 = (const u64*)(r + w8);
    ts[m] = src.narrow ? (i64)((u64)src.tsbase + (u64)r[2]) : (i64)r8[0];
    int g = 0;
    while (g + 1 < src.G && m >= src.start[g + 1]) g++;
    const i64 gi = src.gbase[g] + (i64)pos;
    gidx[m] = (u64)gi;
    int lo = 0, hi = n_bounds;  // first bound with gidx > gi
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (bound_gidx[mid] <= gi) lo = mid + 1; else hi = mid;
    }
    wcol[m] = (int)((lo > 0 ? bound_W[lo - 1] : W_base) - W_base);
    for (int c = 0; c < roles.n; c++) {
        int role = roles.role[c];
        if (role < 0) continue;
        u64 v;
        if (role < 16) v = src.narrow ? ((u64)r[3 + 2 * role] | ((u64)r[4 + 2 * role] << 32)) : r8[1 + role];
        else if (kp.n == 1) v = key;
        else if (role == 16) v = (u64)(i64)(int)(u32)(key >> 32);
        else v = (u64)(i64)(int)(u32)key;
        cols.p[c][m] = v;
    }
}

void launch_shard_unpack(hipStream_t s, const unsigned char* rec, i64 M, int rec_words, KeyPlan kp, ColRoles roles,
                         ShardSrc src, const i64* bound_gidx, const i64* bound_W, int n_bounds, i64 W_base, i64* ts,
                         ColPtrs cols, int* wcol, u64* gidx) {
    if (M <= 0) return;
    hipLaunchKernelGGL(k_shard_unpack, dim3((unsigned)((M + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, (const u32*)rec,
                       M, rec_words, kp, roles, src, bound_gidx, bound_W, n_bounds, W_base, ts, cols, wcol, gidx);
}

}  // namespace shd
