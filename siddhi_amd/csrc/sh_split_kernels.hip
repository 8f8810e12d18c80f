// sh_split_kernels.hip — one-sweep window assignment + key-partition multisplit of a timeBatch push
// (round 4), on gfx950.
//
// The batch pipeline's first two passes (k_boundaries: window numbers, key slots, per-tile partition
// counts; then the column scan and k_ms_scatter: the stable multisplit) read the push twice and hand a
// slot column from one to the other. For the steady state of a timeBatch query — nextEmitTime known,
// one InputHandler.send per event (TimeBatchWindowProcessor.process :262-340 on a PER_EVENT clock) —
// k_split_sweep reads every event's timestamp, key and values once and:
//  * assigns windows exactly as k_boundaries' SORTED form: the clock of a per-event send is
//    max(clock before the push, ts) while timestamps do not decrease (checked here; a decrease sets
//    PushInfo.unsorted and the host redoes the assignment with the prefix passes), a boundary where
//    the window number grows (pass counts in-tile: k_fix_bounds adds the tile prefixes);
//  * splits the queued events (pending tiles) and the push's passing events stably by key partition
//    (pos & (P - 1)), writing the packed records into fixed-capacity per-partition buckets. A tile's
//    offset in each bucket comes from a decoupled look-back over the tiles: it publishes its counts
//    (flag AGG), adds its predecessors' published values back to the first inclusive prefix and
//    publishes its own (flag INCL). Tiles take their index from a ticket, so a tile only waits on tiles
//    already running. The status words are the whole hand-off (agent-scope stores and loads that
//    bypass L1, no payload behind them); the records are read only by later kernels.
//  * writes the [tile][partition] record offsets the segment offsets (k_seg_offsets) and the fold read,
//    and the new tiles' exclusive pass-count prefix (k_fix_bounds, k_compact_pending).
// A bucket that would overflow reports PushInfo.ms_overflow: nothing is written past it and the host
// redoes the split with the counting passes (and keeps them for the query).
#include "sh_device.h"

namespace shd {

constexpr u32 kStAgg = 1u << 30, kStIncl = 2u << 30, kStVal = (1u << 30) - 1u;

__device__ __forceinline__ void st_publish(u32* p, u32 v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ u32 st_poll(const u32* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// LDS: stage_vals[V][kTile] | stage_pos[kTile] | stage_idx[kTile] | start[P] | excl[P] | run[NW][P] (u16)
template <int V, int FK>
__global__ __launch_bounds__(kBlock) void k_split_sweep(TileMap m, i64 n_pend, const u32* __restrict__ pend_pos,
                                                       const u64* __restrict__ pend_vals, i64 pend_cap,
                                                       const i64* __restrict__ ts, ColSet cols, FilterProg f,
                                                       WinParams wp, KeyPlan kp, KeyTable kt, AggPlan ap, int P,
                                                       int logP, i64 cap_p, u32* status, u32* ticket, u32* ms_off,
                                                       u32* rec_idx, u64* rec_vals, i64 rec_cap, u32* new_pos,
                                                       i64* blk_pass_pre, PushInfo* info, Bound* bounds,
                                                       int max_bounds) {
    constexpr int NW = kBlock / 64;
    constexpr int PER_WAVE = kTile / NW;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
    unsigned char* sm = smem_raw + ((16u - ((unsigned)(size_t)smem_raw & 15u)) & 15u);
    u64* stage_vals = (u64*)sm;
    u32* stage_pos = (u32*)(stage_vals + (size_t)V * kTile);
    u32* stage_idx = stage_pos + kTile;
    u32* start = stage_idx + kTile;
    u32* excl = start + P;
    unsigned short* run = (unsigned short*)(excl + P);  // [NW][P]
    __shared__ u32 s_tile, s_total;
    __shared__ i64 s_wave_pass[NW];
    if (threadIdx.x == 0) s_tile = atomicAdd(ticket, 1u);
    __syncthreads();
    const int tile = (int)s_tile;
    if (tile >= m.nblk) return;
    const bool pend_tile = tile < m.np_t;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const i64 t0 = tile_lo(m, tile) + (i64)w * PER_WAVE, hi = tile_hi(m, tile);
    // every round's position, values and (push events) timestamp, requested before anything waits
    u32 my_pos[kItems];
    u64 my_val[kItems][V];
    i64 my_ts[kItems];
#pragma unroll
    for (int r = 0; r < kItems; r++) {
        const i64 e = t0 + (i64)r * 64 + lane;
        u32 pos = kNoPos;
        my_ts[r] = INT64_MAX;
#pragma unroll
        for (int j = 0; j < V; j++) my_val[r][j] = 0;
        if (e < hi) {
            if (pend_tile) {
                pos = pend_pos[e];
#pragma unroll
                for (int j = 0; j < V; j++)
                    if (j < ap.n_vcols) my_val[r][j] = pend_vals[(size_t)j * pend_cap + e];
            } else {
                const i64 en = e - n_pend;
                my_ts[r] = ts[en];
                if (eval_filter<FK>(f, cols, en)) pos = key_slot(kt, make_key(kp, cols, en));
#pragma unroll
                for (int j = 0; j < V; j++)
                    if (j < ap.n_vcols) my_val[r][j] = (u64)load_raw(cols, ap.vcol_src[j], en);
            }
        }
        my_pos[r] = pos;
    }
    if (new_pos && !pend_tile) {  // the slot column for the pending carry (hashed keys)
#pragma unroll
        for (int r = 0; r < kItems; r++) {
            const i64 e = t0 + (i64)r * 64 + lane;
            if (e < hi) new_pos[e - n_pend] = my_pos[r];
        }
    }
    for (int i = threadIdx.x; i < NW * P; i += kBlock) run[i] = 0;
    __syncthreads();
    // rank inside the wave's run of the partition (16-bit LDS counters, two per word; lanes of a round
    // that hit one counter receive their values in lane order on gfx950 — the stability check repairs
    // the order otherwise)
    u32* wrun32 = (u32*)run;
    unsigned short* wrun = run + w * P;
    u32 my_rank[kItems];
#pragma unroll
    for (int r = 0; r < kItems; r++) {
        my_rank[r] = 0;
        if (my_pos[r] == kNoPos) continue;
        const u32 c = (u32)(w * P) + (my_pos[r] & (P - 1));
        const u32 sh = (c & 1) * 16;
        my_rank[r] = (atomicAdd(&wrun32[c >> 1], 1u << sh) >> sh) & 0xFFFFu;
    }
    __syncthreads();
    {
        int per = (P + kBlock - 1) / kBlock;
        int a = threadIdx.x * per, b = min(P, a + per);
        i64 sum = 0;
        for (int i = a; i < b; i++)
            for (int x = 0; x < NW; x++) sum += run[x * P + i];
        i64 tot;
        i64 pre = block_excl_scan(sum, SumOp(), 0, &tot);
        if (threadIdx.x == 0) s_total = (u32)tot;
        for (int i = a; i < b; i++) {
            const i64 st = pre;
            start[i] = (u32)st;
            for (int x = 0; x < NW; x++) {
                u32 c = run[x * P + i];
                run[x * P + i] = (unsigned short)(pre - st);
                pre += c;
            }
        }
    }
    __syncthreads();
    const u32 n_tile = s_total;
    // ---- decoupled look-back: the tile's offset in every partition bucket
    for (int p = threadIdx.x; p < P; p += kBlock) {
        const u32 c = (p + 1 < P ? start[p + 1] : n_tile) - start[p];
        u32* me = status + (size_t)tile * P + p;
        u32 pre = 0;
        if (tile == 0) {
            st_publish(me, kStIncl | c);
        } else {
            st_publish(me, kStAgg | c);
            // predecessors read kLb at a time (independent loads, one latency per batch), summed back to
            // the first inclusive prefix; a not-yet-published one is polled again from there
            constexpr int kLb = 16;
            int t = tile - 1;
            for (bool done = false; !done;) {
                u32 v[kLb];
#pragma unroll
                for (int j = 0; j < kLb; j++) v[j] = t - j >= 0 ? st_poll(status + (size_t)(t - j) * P + p) : kStIncl;
                int j = 0;
                for (; j < kLb; j++) {
                    const u32 fl = v[j] & ~kStVal;
                    if (fl == 0) break;
                    pre += v[j] & kStVal;
                    if (fl == kStIncl) { done = true; break; }
                }
                if (done) break;
                t -= j;
                if (j < kLb) __builtin_amdgcn_s_sleep(1);
            }
            st_publish(me, kStIncl | ((pre + c) & kStVal));
        }
        excl[p] = pre;
        ms_off[(size_t)tile * P + p] = (u32)((i64)p * cap_p + pre);
        if (tile == m.nblk - 1) ms_off[(size_t)m.nblk * P + p] = (u32)((i64)p * cap_p + pre + c);
        if ((i64)pre + c > cap_p) atomicOr(&info->ms_overflow, 1);
    }
    __syncthreads();
    // ---- windows of the push's events (SORTED form of k_boundaries, per-event sends)
    if (!pend_tile) {
        const int nt = tile - m.np_t;  // new-event tile
        // passing events before this tile (new events): every record before it, minus the queue
        i64 my_pre = 0;
        for (int p = threadIdx.x; p < P; p += kBlock) my_pre += excl[p];
        const i64 pre_all = block_reduce(my_pre, SumOp(), 0);
        if (threadIdx.x == 0) {
            blk_pass_pre[nt] = pre_all - n_pend;
            if (tile == m.nblk - 1) blk_pass_pre[nt + 1] = pre_all + n_tile - n_pend;
        }
        // the tile's passing events before each event: per wave, per round (ballots)
        i64 wave_cnt = 0;
#pragma unroll
        for (int r = 0; r < kItems; r++) wave_cnt += __popcll(__ballot(my_pos[r] != kNoPos));
        if (lane == 0) s_wave_pass[w] = wave_cnt;
        // the timestamps never decrease: within the wave's rounds, and into the next event of the tile
        const i64 N = wp.N;
        bool down = false;
#pragma unroll
        for (int r = 0; r < kItems; r++) {
            const i64 e = t0 + (i64)r * 64 + lane;
            const i64 sh = __shfl_down(my_ts[r], 1, 64);  // (every lane takes part in the shuffle)
            if (e >= hi) continue;
            const i64 en = e - n_pend;
            // the next event: the next lane's, or (wave / round / tile end) read again
            const i64 nxt = (lane < 63 && e + 1 < hi) ? sh : (en + 1 < N ? ts[en + 1] : INT64_MAX);
            down |= nxt < my_ts[r];
        }
        if (__any(down)) atomicOr(&info->unsorted, 1);
        __syncthreads();
        i64 pcb = 0;  // passing events of the tile before this wave
        for (int x = 0; x < w; x++) pcb += s_wave_pass[x];
        const i64 c0 = wp.clock_valid ? wp.clock0 : INT64_MIN;
        const i64 E0 = wp.E0, T = wp.T;
        auto W_of = [&](i64 clk) -> i64 { return clk < E0 ? 0 : (clk - E0) / T + 1; };
        // windows change rarely: a tile whose first and last clocks share a window has no boundary
        // (the window of the event before the tile is the first event's, or a boundary is at the tile's
        // first event, found below)
        const i64 tile_first = tile_lo(m, tile) - n_pend;
        const i64 last_clk = max(c0, ts[hi - 1 - n_pend]);
        const i64 prev_clk = tile_first > 0 ? max(c0, ts[tile_first - 1]) : c0;
        const i64 W_prev_tile = tile_first > 0 ? W_of(prev_clk) : wp.W_open;
        if (W_of(last_clk) > W_prev_tile) {
#pragma unroll
            for (int r = 0; r < kItems; r++) {
                const i64 e = t0 + (i64)r * 64 + lane;
                const bool pass = my_pos[r] != kNoPos;
                const u64 bal = __ballot(pass);
                const i64 before = pcb + __popcll(bal & (lane == 0 ? 0ull : (~0ull >> (64 - lane))));
                pcb += __popcll(bal);
                if (e >= hi) continue;
                const i64 en = e - n_pend;
                const i64 clk = max(c0, my_ts[r]);
                const i64 pclk = en > 0 ? max(c0, ts[en - 1]) : c0;
                const i64 W = W_of(clk), Wp = en > 0 ? W_of(pclk) : wp.W_open;
                if (W > Wp) {
                    const int k = atomicAdd(&info->n_bounds, 1);
                    if (k < max_bounds) {
                        Bound bd;
                        bd.idx = n_pend + en;
                        bd.W = W;
                        bd.clock = clk;
                        bd.clock_prev = pclk;
                        bd.pcb = before;  // in-tile: k_fix_bounds adds the tile prefix
                        bd.pad = nt;
                        bounds[k] = bd;
                    }
                }
            }
        }
    }
    // ---- stage the tile partition-major (event order inside a partition) and write the runs
#pragma unroll
    for (int r = 0; r < kItems; r++) {
        if (my_pos[r] == kNoPos) continue;
        const u32 p = my_pos[r] & (P - 1);
        const u32 slot = start[p] + wrun[p] + my_rank[r];
        stage_pos[slot] = my_pos[r];
        stage_idx[slot] = (u32)(t0 + (i64)r * 64 + lane);
#pragma unroll
        for (int j = 0; j < V; j++)
            if (j < ap.n_vcols) stage_vals[(size_t)j * kTile + slot] = my_val[r][j];
    }
    __syncthreads();
    bool bad = false;
    for (u32 j = threadIdx.x; j + 1 < n_tile; j += kBlock)
        bad |= stage_idx[j + 1] < stage_idx[j] && ((stage_pos[j + 1] ^ stage_pos[j]) & (P - 1)) == 0;
    if (__syncthreads_or(bad)) {
        for (int p = threadIdx.x; p < P; p += kBlock) {
            const u32 a = start[p], b = p + 1 < P ? start[p + 1] : n_tile;
            for (u32 k = a + 1; k < b; k++) {
                const u32 e = stage_idx[k], pos = stage_pos[k];
                u64 mv[V];
#pragma unroll
                for (int j = 0; j < V; j++) mv[j] = j < ap.n_vcols ? stage_vals[(size_t)j * kTile + k] : 0;
                u32 q = k;
                while (q > a && stage_idx[q - 1] > e) {
                    stage_idx[q] = stage_idx[q - 1];
                    stage_pos[q] = stage_pos[q - 1];
#pragma unroll
                    for (int j = 0; j < V; j++)
                        if (j < ap.n_vcols) stage_vals[(size_t)j * kTile + q] = stage_vals[(size_t)j * kTile + q - 1];
                    q--;
                }
                stage_idx[q] = e;
                stage_pos[q] = pos;
#pragma unroll
                for (int j = 0; j < V; j++)
                    if (j < ap.n_vcols) stage_vals[(size_t)j * kTile + q] = mv[j];
            }
        }
        __syncthreads();
    }
    for (u32 j = threadIdx.x; j < n_tile; j += kBlock) {
        const u32 pp = stage_pos[j] & (P - 1);
        const i64 in_p = (i64)excl[pp] + (j - start[pp]);
        if (in_p >= cap_p) continue;  // overflow: reported above, the host redoes the split
        const i64 dst = (i64)pp * cap_p + in_p;
        rec_idx[dst] = ((stage_pos[j] >> logP) << kPackIdxBits) | (stage_idx[j] & kPackIdxMask);
#pragma unroll
        for (int v = 0; v < V; v++)
            if (v < ap.n_vcols) rec_vals[(size_t)v * rec_cap + dst] = stage_vals[(size_t)v * kTile + j];
    }
}

size_t split_sweep_lds(int n_vcols, int P) {
    const int V = n_vcols <= 1 ? 1 : n_vcols <= 2 ? 2 : n_vcols <= 4 ? 4 : 8;
    return (size_t)V * kTile * 8 + (size_t)kTile * 8 + (size_t)P * 8 + (size_t)P * 2 * (kBlock / 64) + 32;
}

void launch_split_sweep(hipStream_t s, TileMap m, i64 n_pend, const u32* pend_pos, const u64* pend_vals, i64 pend_cap,
                        const i64* ts, ColSet cols, FilterProg f, WinParams wp, KeyPlan kp, KeyTable kt, AggPlan ap,
                        int P, int logP, i64 cap_p, u32* status, u32* ticket, u32* ms_off, u32* rec_idx, u64* rec_vals,
                        i64 rec_cap, u32* new_pos, i64* blk_pass_pre, PushInfo* info, Bound* bounds, int max_bounds) {
    const int V = ap.n_vcols <= 1 ? 1 : ap.n_vcols <= 2 ? 2 : ap.n_vcols <= 4 ? 4 : 8;
    const int fk = filter_kind(f);
    const size_t lds = split_sweep_lds(ap.n_vcols, P);
#define SH_SW(VV, FKK)                                                                                               \
    hipLaunchKernelGGL((k_split_sweep<VV, FKK>), dim3(m.nblk), dim3(kBlock), lds, s, m, n_pend, pend_pos, pend_vals,  \
                       pend_cap, ts, cols, f, wp, kp, kt, ap, P, logP, cap_p, status, ticket, ms_off, rec_idx, rec_vals, \
                       rec_cap, new_pos, blk_pass_pre, info, bounds, max_bounds)
#define SH_SWV(VV)                        \
    do {                                  \
        if (fk == 0) SH_SW(VV, 0);        \
        else if (fk == 1) SH_SW(VV, 1);   \
        else SH_SW(VV, 2);                \
    } while (0)
    if (V == 1) SH_SWV(1);
    else if (V == 2) SH_SWV(2);
    else if (V == 4) SH_SWV(4);
    else SH_SWV(8);
#undef SH_SWV
#undef SH_SW
}

}  // namespace shd
