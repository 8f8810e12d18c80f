// sh_device.h — device helpers for the gfx950 kernels: Java value semantics, filter evaluation,
// group-key hashing, wave64 / workgroup scans.
#pragma once

#include "sh_internal.h"

namespace shd {

// ---- column access ---------------------------------------------------------------------------
// Raw 8-byte form: integral types sign-extended to int64, FLOAT widened exactly to double bits,
// DOUBLE bits. Same convention as the oracle (oracle/siddhi_oracle.cpp load_event).
__device__ __forceinline__ i64 load_raw(const ColSet& cs, int c, i64 e) {
    switch (cs.type[c]) {
        case SH_T_INT:
        case SH_T_STRID: return (i64)((const int*)cs.ptr[c])[e];
        case SH_T_LONG: return ((const i64*)cs.ptr[c])[e];
        case SH_T_BOOL: return ((const unsigned char*)cs.ptr[c])[e] ? 1 : 0;
        case SH_T_FLOAT: return __double_as_longlong((double)((const float*)cs.ptr[c])[e]);
        default: return __double_as_longlong(((const double*)cs.ptr[c])[e]);
    }
}

// kItems consecutive 8-byte values p[base..base+kItems) of one thread's blocked run: four 16-byte
// loads when the run is aligned and inside [0, N), else element loads (`fill` past N).
__device__ __forceinline__ void load_items_i64(const i64* __restrict__ p, i64 base, i64 N, i64 (&out)[kItems],
                                               i64 fill) {
    if (base + kItems <= N && (((size_t)(p + base)) & 15) == 0) {
        const longlong2* q = (const longlong2*)(p + base);
#pragma unroll
        for (int j = 0; j < kItems / 2; j++) {
            longlong2 v = q[j];
            out[2 * j] = v.x;
            out[2 * j + 1] = v.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < kItems; j++) out[j] = base + j < N ? p[base + j] : fill;
    }
}

// Raw values of column c for one thread's kItems consecutive events (vector loads for 4- and
// 8-byte integral columns when aligned; load_raw otherwise).
__device__ __forceinline__ void load_items_raw(const ColSet& cs, int c, i64 base, i64 N, i64 (&out)[kItems]) {
    const int t = cs.type[c];
    if ((t == SH_T_INT || t == SH_T_STRID) && base + kItems <= N &&
        (((size_t)((const int*)cs.ptr[c] + base)) & 15) == 0) {
        const int4* q = (const int4*)((const int*)cs.ptr[c] + base);
#pragma unroll
        for (int j = 0; j < kItems / 4; j++) {
            int4 v = q[j];
            out[4 * j] = v.x; out[4 * j + 1] = v.y; out[4 * j + 2] = v.z; out[4 * j + 3] = v.w;
        }
    } else if (t == SH_T_LONG || t == SH_T_DOUBLE) {  // DOUBLE: the bit patterns
        load_items_i64((const i64*)cs.ptr[c], base, N, out, 0);
    } else if (t == SH_T_FLOAT && base + kItems <= N && (((size_t)((const float*)cs.ptr[c] + base)) & 15) == 0) {
        const float4* q = (const float4*)((const float*)cs.ptr[c] + base);
#pragma unroll
        for (int j = 0; j < kItems / 4; j++) {
            float4 v = q[j];
            out[4 * j] = __double_as_longlong((double)v.x);
            out[4 * j + 1] = __double_as_longlong((double)v.y);
            out[4 * j + 2] = __double_as_longlong((double)v.z);
            out[4 * j + 3] = __double_as_longlong((double)v.w);
        }
    } else {
#pragma unroll
        for (int j = 0; j < kItems; j++) out[j] = base + j < N ? load_raw(cs, c, base + j) : 0;
    }
}

// Java (long) cast of a double (JLS 5.1.3): NaN -> 0, saturating, truncation toward zero
__device__ __forceinline__ i64 java_d2l(double x) {
    if (x != x) return 0;
    if (x >= 9.2233720368547758e18) return INT64_MAX;
    if (x <= -9.2233720368547758e18) return INT64_MIN;
    return (i64)x;
}

__device__ __forceinline__ bool is_fp(int t) { return t == SH_T_FLOAT || t == SH_T_DOUBLE; }
__device__ __forceinline__ int prank(int t) { return t == SH_T_LONG ? 2 : t == SH_T_FLOAT ? 3 : t == SH_T_DOUBLE ? 4 : 1; }

// Compare executors (core/executor/condition/compare/**): binary numeric promotion, except ==/!=
// between FLOAT and LONG which compare doubleValue() of both sides (EqualCompare...FloatLong.java).
__device__ __forceinline__ bool java_cmp(int op, int ta, i64 a, int tb, i64 b) {
    int r = max(prank(ta), prank(tb));
    bool eq = (op == SH_OP_EQ || op == SH_OP_NE);
    if (eq && ((ta == SH_T_FLOAT && tb == SH_T_LONG) || (ta == SH_T_LONG && tb == SH_T_FLOAT))) r = 4;
    if (r >= 3) {
        double x = is_fp(ta) ? __longlong_as_double(a) : (double)a;
        double y = is_fp(tb) ? __longlong_as_double(b) : (double)b;
        if (r == 3) {
            float fx = is_fp(ta) ? (float)x : (float)a;
            float fy = is_fp(tb) ? (float)y : (float)b;
            switch (op) {
                case SH_OP_GT: return fx > fy; case SH_OP_GE: return fx >= fy;
                case SH_OP_LT: return fx < fy; case SH_OP_LE: return fx <= fy;
                case SH_OP_EQ: return fx == fy; default: return fx != fy;
            }
        }
        switch (op) {
            case SH_OP_GT: return x > y; case SH_OP_GE: return x >= y;
            case SH_OP_LT: return x < y; case SH_OP_LE: return x <= y;
            case SH_OP_EQ: return x == y; default: return x != y;
        }
    }
    switch (op) {
        case SH_OP_GT: return a > b; case SH_OP_GE: return a >= b;
        case SH_OP_LT: return a < b; case SH_OP_LE: return a <= b;
        case SH_OP_EQ: return a == b; default: return a != b;
    }
}

// FilterProcessor.process (core/query/processor/filter/FilterProcessor.java:47-60): a postfix
// program over column refs and constants; the result must be TRUE to keep the event.
__device__ __forceinline__ void filter_const(const FilterOpD& o, int& t, i64& v) {
    t = o.type;
    if (o.type == SH_T_FLOAT) v = __double_as_longlong((double)(float)o.dval);
    else if (o.type == SH_T_DOUBLE) v = __double_as_longlong(o.dval);
    else if (o.type == SH_T_INT) v = (i64)(int)o.ival;
    else v = o.ival;
}

__device__ __forceinline__ bool is_leaf(const FilterProg& f, int i) {
    return f.ops[i].op == SH_OP_COL && f.ops[i + 1].op == SH_OP_CONST && f.ops[i + 2].op >= SH_OP_GT &&
           f.ops[i + 2].op <= SH_OP_NE;
}

// `col <cmp> const` (ops i .. i+2) in registers
__device__ __forceinline__ bool eval_leaf(const FilterProg& f, int i, const ColSet& cs, i64 e) {
    int tc;
    i64 vc;
    filter_const(f.ops[i + 1], tc, vc);
    const int c = f.ops[i].col;
    return java_cmp(f.ops[i + 2].op, cs.type[c], load_raw(cs, c, e), tc, vc);
}

// FK narrows the program forms a kernel instance handles (filter_kind on the host): 0 no filter,
// 1 the register-only forms below, 2 any program. The narrow instances do not carry the stack
// machine's registers.
template <int FK = 2>
__device__ __forceinline__ bool eval_filter(const FilterProg& f, const ColSet& cs, i64 e) {
    if (FK == 0 || f.n == 0) return true;
    // register-only forms of the common programs (the branch is uniform: f is a kernel argument);
    // the general stack machine below keeps its operand stack in scratch memory
    if (f.n == 3 && is_leaf(f, 0)) return eval_leaf(f, 0, cs, e);
    if (f.n == 7 && is_leaf(f, 0) && is_leaf(f, 3)) {
        if (f.ops[6].op == SH_OP_AND) return eval_leaf(f, 0, cs, e) && eval_leaf(f, 3, cs, e);
        if (f.ops[6].op == SH_OP_OR) return eval_leaf(f, 0, cs, e) || eval_leaf(f, 3, cs, e);
    }
    if (FK < 2) return false;  // not reached: filter_kind picked FK 1 for a register form
    i64 sv[16];
    int st[16];
    int sp = 0;
    for (int i = 0; i < f.n; i++) {
        const FilterOpD& o = f.ops[i];
        switch (o.op) {
            case SH_OP_COL: sv[sp] = load_raw(cs, o.col, e); st[sp] = cs.type[o.col]; sp++; break;
            case SH_OP_CONST:
                st[sp] = o.type;
                if (o.type == SH_T_FLOAT) sv[sp] = __double_as_longlong((double)(float)o.dval);
                else if (o.type == SH_T_DOUBLE) sv[sp] = __double_as_longlong(o.dval);
                else if (o.type == SH_T_INT) sv[sp] = (i64)(int)o.ival;
                else sv[sp] = o.ival;
                sp++;
                break;
            case SH_OP_AND: sp--; sv[sp - 1] = (sv[sp - 1] && sv[sp]) ? 1 : 0; st[sp - 1] = SH_T_BOOL; break;
            case SH_OP_OR: sp--; sv[sp - 1] = (sv[sp - 1] || sv[sp]) ? 1 : 0; st[sp - 1] = SH_T_BOOL; break;
            case SH_OP_NOT: sv[sp - 1] = sv[sp - 1] ? 0 : 1; st[sp - 1] = SH_T_BOOL; break;
            case kOpKeyEq: {
                sp--;
                auto canon = [](int t, i64 v) -> i64 {
                    return (is_fp(t) && __longlong_as_double(v) != __longlong_as_double(v)) ? 0x7FF8000000000000ll : v;
                };
                sv[sp - 1] = canon(st[sp - 1], sv[sp - 1]) == canon(st[sp], sv[sp]) ? 1 : 0;
                st[sp - 1] = SH_T_BOOL;
                break;
            }
            default: {
                sp--;
                bool r = java_cmp(o.op, st[sp - 1], sv[sp - 1], st[sp], sv[sp]);
                sv[sp - 1] = r ? 1 : 0;
                st[sp - 1] = SH_T_BOOL;
            }
        }
    }
    return sp > 0 && sv[sp - 1] != 0;
}

// The filter over one thread's kItems consecutive events: the leaf forms load their columns with
// the blocked vector loads (16-byte loads per thread) instead of one scattered element load per item.
__device__ __forceinline__ void leaf_items(const FilterProg& f, int i, const ColSet& cs, i64 base, i64 N,
                                          bool (&r)[kItems]) {
    int tc;
    i64 vc;
    filter_const(f.ops[i + 1], tc, vc);
    const int c = f.ops[i].col, op = f.ops[i + 2].op, ta = cs.type[c];
    i64 x[kItems];
    load_items_raw(cs, c, base, N, x);
#pragma unroll
    for (int j = 0; j < kItems; j++) r[j] = java_cmp(op, ta, x[j], tc, vc);
}

template <int FK = 2>
__device__ __forceinline__ void filter_items(const FilterProg& f, const ColSet& cs, i64 base, i64 N,
                                            bool (&pass)[kItems]) {
    if (FK == 0) {
#pragma unroll
        for (int j = 0; j < kItems; j++) pass[j] = true;
    } else if (f.n == 3 && is_leaf(f, 0)) {
        leaf_items(f, 0, cs, base, N, pass);
    } else if (f.n == 7 && is_leaf(f, 0) && is_leaf(f, 3) && (f.ops[6].op == SH_OP_AND || f.ops[6].op == SH_OP_OR)) {
        bool a[kItems], b[kItems];
        leaf_items(f, 0, cs, base, N, a);
        leaf_items(f, 3, cs, base, N, b);
        const bool conj = f.ops[6].op == SH_OP_AND;
#pragma unroll
        for (int j = 0; j < kItems; j++) pass[j] = conj ? (a[j] && b[j]) : (a[j] || b[j]);
    } else {
#pragma unroll
        for (int j = 0; j < kItems; j++) pass[j] = base + j < N && eval_filter<FK>(f, cs, base + j);
    }
#pragma unroll
    for (int j = 0; j < kItems; j++) pass[j] = pass[j] && base + j < N;
}

// ---- group keys ---------------------------------------------------------------------------------
// GroupByKeyGenerator.constructEventKey (core/query/selector/GroupByKeyGenerator.java:63-73) keys
// by the values' string form; for the integral key columns string equality is value equality.
// Floating-point keys: String.valueOf(double / float) names every value apart (0.0 and -0.0 too)
// except NaN, whose payloads all print "NaN" — so the key is the value's bits with NaN made canonical.
// A float alone is keyed by its value widened to double (an injective map); as one of two 32-bit
// components by its own (canonical) bits.
// ---- GMT calendar (IncrementalTimeConverterUtil with ZoneId "GMT") ------------------------------
__device__ __forceinline__ i64 floor_div_d(i64 a, i64 b) {
    i64 q = a / b;
    if ((a % b != 0) && ((a < 0) != (b < 0))) q--;
    return q;
}
__device__ __forceinline__ i64 days_from_civil_d(i64 y, unsigned m, unsigned d) {
    y -= m <= 2;
    const i64 era = (y >= 0 ? y : y - 399) / 400;
    const unsigned yoe = (unsigned)(y - era * 400);
    const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + d - 1;
    const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + (i64)doe - 719468;
}
__device__ __forceinline__ void civil_from_days_d(i64 z, i64& y, unsigned& m, unsigned& d) {
    z += 719468;
    const i64 era = (z >= 0 ? z : z - 146096) / 146097;
    const unsigned doe = (unsigned)(z - era * 146097);
    const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    y = (i64)yoe + era * 400;
    const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const unsigned mp = (5 * doy + 2) / 153;
    d = doy - (153 * mp + 2) / 5 + 1;
    m = mp + (mp < 10 ? 3 : -9);
    y += (m <= 2);
}

// Calendar buckets (aggregation roots `every month` / `every year`, IncrementalTimeConverterUtil with
// a fixed-offset zone tz): cal 1 = months, 2 = years; the bucket index of t and the start of index i
__device__ __forceinline__ i64 cal_idx_d(i64 t, int cal, i64 tz) {
    i64 y; unsigned m, d;
    civil_from_days_d(floor_div_d(t + tz, 86400000), y, m, d);
    return cal == 1 ? y * 12 + (i64)(m - 1) : y;
}
__device__ __forceinline__ i64 cal_start_d(i64 i, int cal, i64 tz) {
    if (cal == 1) {
        const i64 y = floor_div_d(i, 12);
        return days_from_civil_d(y, (unsigned)(i - y * 12 + 1), 1) * 86400000 - tz;
    }
    return days_from_civil_d(i, 1, 1) * 86400000 - tz;
}

__device__ __forceinline__ i64 key_part(const KeyPlan& kp, const ColSet& cs, int g, i64 e) {
    i64 v = load_raw(cs, kp.col[g], e);
    const int t = kp.type[g];
    if (t == SH_T_FLOAT || t == SH_T_DOUBLE) return __longlong_as_double(v) != __longlong_as_double(v) ? 0x7FF8000000000000ll : v;
    // aggregation time bucket: getStartTimeOfAggregates (IncrementalTimeConverterUtil.java:52-69);
    // div < 0: a calendar bucket (-1 months, -2 years) in the zone offset `add`
    if (kp.div[g] > 0) v = (v + kp.add[g]) / kp.div[g];
    else if (kp.div[g] < 0) v = cal_idx_d(v, (int)-kp.div[g], kp.add[g]);
    return v;
}

__device__ __forceinline__ u32 key_part32(const KeyPlan& kp, const ColSet& cs, int g, i64 e) {
    if (kp.type[g] == SH_T_FLOAT) {
        // (a column loaded in its raw 8-byte form holds the value widened to double)
        const float f = cs.type[kp.col[g]] == SH_T_FLOAT ? ((const float*)cs.ptr[kp.col[g]])[e]
                                                         : (float)__longlong_as_double(load_raw(cs, kp.col[g], e));
        return f != f ? 0x7FC00000u : __float_as_uint(f);
    }
    return (u32)key_part(kp, cs, g, e);
}

__device__ __forceinline__ u64 make_key(const KeyPlan& kp, const ColSet& cs, i64 e) {
    if (kp.n == 0) return 0;
    if (kp.n == 1) return (u64)key_part(kp, cs, 0, e);
    u64 a = (u64)key_part32(kp, cs, 0, e);
    u64 b = (u64)key_part32(kp, cs, 1, e);
    return (a << 32) | b;
}

// a component as sh_out reports it: int64 widening; floats as the bits of the value widened to double
__device__ __forceinline__ i64 unpack_part(const KeyPlan& kp, int g, u32 x) {
    if (kp.type[g] == SH_T_FLOAT) return __double_as_longlong((double)__uint_as_float(x));
    if (kp.div[g] < 0) return cal_start_d((i64)x, (int)-kp.div[g], kp.add[g]);
    return kp.div[g] > 0 ? (i64)x * kp.div[g] - kp.add[g] : (i64)(int)x;
}

__device__ __forceinline__ void unpack_key(const KeyPlan& kp, u64 key, i64* out, i64 stride) {
    if (kp.n == 1) out[0] = kp.div[0] > 0 ? (i64)key * kp.div[0] - kp.add[0]
                            : kp.div[0] < 0 ? cal_start_d((i64)key, (int)-kp.div[0], kp.add[0]) : (i64)key;
    else if (kp.n == 2) {
        out[0] = unpack_part(kp, 0, (u32)(key >> 32));
        out[stride] = unpack_part(kp, 1, (u32)key);
    }
}

__device__ __forceinline__ u64 mix64(u64 z) {
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

// Home slot: Fibonacci (multiplicative) hashing, top log2(size) bits of key * 2^64/phi. Dense key
// ranges (dictionary ids, small integers) land on distinct slots (three-gap theorem), so most
// lookups take one probe; other keys are spread like any multiplicative hash.
__device__ __forceinline__ u32 key_home(const KeyTable& kt, u64 key) {
    return (u32)((key * 0x9E3779B97F4A7C15ull) >> kt.shift) & kt.mask;
}

// Open-addressing lookup-or-insert (linear probing). The position is the group slot. A plain load
// that sees a stale EMPTY (another CU inserted meanwhile) is corrected by the CAS, which reads the
// line at the memory side; a non-EMPTY key never changes, so it can't be stale.
__device__ __forceinline__ bool probe_step(const KeyTable& kt, u64 key, u64 k, u32& h) {
    if (k == key) return true;
    if (k == kEmptyKey) {
        u64 old = atomicCAS(&kt.keys[h], kEmptyKey, key);
        if (old == kEmptyKey) { atomicAdd(kt.n_keys, 1u); return true; }
        if (old == key) return true;
    }
    h = (h + 1) & kt.mask;
    return false;
}

// Dense mode: a dictionary id maps to its slot directly (the sharded owner of ids = dadd mod dmul
// keeps them compact as (id - dadd) / dmul); an id outside the table fails the push loudly.
__device__ __forceinline__ u32 dense_slot(const KeyTable& kt, u64 key) {
    u32 id = (u32)key;
    u32 s = kt.dmul == 1 ? id - kt.dadd : (id - kt.dadd) / kt.dmul;
    if (kt.lk) {
        // band: the bucket's row (the host placed every live bucket inside the band) and the id's slot
        const u32 row = (u32)(key >> 32) - kt.b0;
        if (row >= kt.rows) { atomicExch(kt.overflow, 3); return 0; }
        if ((int)id < 0 || (s >> kt.lk) != 0) { atomicExch(kt.overflow, 2); return 0; }
        return (row << kt.lk) | s;
    }
    if ((i64)key < 0 || s > kt.mask) { atomicExch(kt.overflow, 2); return 0; }
    return s;
}

__device__ __forceinline__ u32 key_slot(const KeyTable& kt, u64 key) {
    if (kt.dense) return dense_slot(kt, key);
    if (key == kEmptyKey) return kt.mask + 1;
    u32 h = key_home(kt, key);
    for (u32 probe = 0; probe <= kt.mask; probe++)
        if (probe_step(kt, key, kt.keys[h], h)) return h;
    atomicExch(kt.overflow, 1);
    return 0;
}

// K independent lookups advanced together: each probe round issues the loads of every unresolved
// lookup back to back, so their latencies overlap.
template <int K>
__device__ __forceinline__ void key_slots(const KeyTable& kt, const u64* key, const bool* valid, u32* out) {
    u32 h[K];
    bool done[K];
    if (kt.dense) {
#pragma unroll
        for (int i = 0; i < K; i++) if (valid[i]) out[i] = dense_slot(kt, key[i]);
        return;
    }
#pragma unroll
    for (int i = 0; i < K; i++) {
        done[i] = !valid[i] || key[i] == kEmptyKey;
        if (valid[i] && key[i] == kEmptyKey) out[i] = kt.mask + 1;
        h[i] = key_home(kt, key[i]);
    }
    for (u32 probe = 0; probe <= kt.mask; probe++) {
        u64 k[K];
#pragma unroll
        for (int i = 0; i < K; i++) k[i] = done[i] ? 0 : kt.keys[h[i]];
        bool left = false;
#pragma unroll
        for (int i = 0; i < K; i++) {
            if (done[i]) continue;
            if (probe_step(kt, key[i], k[i], h[i])) { out[i] = h[i]; done[i] = true; }
            left |= !done[i];
        }
        if (!left) return;
    }
    atomicExch(kt.overflow, 1);
#pragma unroll
    for (int i = 0; i < K; i++) if (!done[i]) out[i] = 0;
}

__device__ __forceinline__ u64 slot_key(const KeyTable& kt, u32 pos) {
    if (kt.lk) {
        const u32 s = pos & ((1u << kt.lk) - 1u);
        return ((u64)(kt.b0 + (pos >> kt.lk)) << 32) | (u64)(s * kt.dmul + kt.dadd);
    }
    if (kt.dense) return (u64)(pos * kt.dmul + kt.dadd);
    return pos > kt.mask ? kEmptyKey : kt.keys[pos];
}

// ---- scans --------------------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

template <typename T, typename Op>
__device__ __forceinline__ T wave_incl_scan(T v, Op op) {
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T o = __shfl_up(v, d, 64);
        if (lane_id() >= d) v = op(v, o);
    }
    return v;
}

struct SumOp { __device__ i64 operator()(i64 a, i64 b) const { return a + b; } };
struct MaxOp { __device__ i64 operator()(i64 a, i64 b) const { return a > b ? a : b; } };
struct MinOp { __device__ i64 operator()(i64 a, i64 b) const { return a < b ? a : b; } };

// Workgroup exclusive scan (kBlock threads); returns exclusive prefix, *total gets the reduction.
template <typename Op>
__device__ __forceinline__ i64 block_excl_scan(i64 v, Op op, i64 identity, i64* total) {
    __shared__ i64 wsum[kBlock / 64];
    i64 incl = wave_incl_scan(v, op);
    int w = threadIdx.x >> 6;
    if (lane_id() == 63) wsum[w] = incl;
    __syncthreads();
    i64 pre = identity;
    for (int i = 0; i < w; i++) pre = op(pre, wsum[i]);
    i64 tot = identity;
    for (int i = 0; i < kBlock / 64; i++) tot = op(tot, wsum[i]);
    __syncthreads();
    if (total) *total = tot;
    i64 excl = __shfl_up(incl, 1, 64);
    if (lane_id() == 0) excl = identity;
    return op(pre, excl);
}

// Sum scan for any workgroup size that is a multiple of 64 (up to 1024 threads).
__device__ __forceinline__ i64 block_excl_scan_any(i64 v, i64* total) {
    __shared__ i64 wsum_any[16];
    i64 incl = wave_incl_scan(v, SumOp());
    int w = threadIdx.x >> 6, nw = (int)(blockDim.x >> 6);
    if (lane_id() == 63) wsum_any[w] = incl;
    __syncthreads();
    i64 pre = 0, tot = 0;
    for (int i = 0; i < nw; i++) { if (i < w) pre += wsum_any[i]; tot += wsum_any[i]; }
    __syncthreads();
    if (total) *total = tot;
    return pre + incl - v;
}

template <typename Op>
__device__ __forceinline__ i64 block_reduce(i64 v, Op op, i64 identity) {
    i64 t;
    block_excl_scan(v, op, identity, &t);
    return t;
}

// Send bookkeeping: InputHandler.send(Event[]) sets the playback clock from the last event of
// each send (core/stream/input/InputHandler.java:85-96).
__device__ __forceinline__ i64 send_len(const WinParams& wp) { return wp.send_size > 0 ? wp.send_size : wp.N; }
__device__ __forceinline__ bool is_send_last(const WinParams& wp, i64 e) {
    i64 s = send_len(wp);
    return ((e + 1) % s == 0) || (e == wp.N - 1);
}
__device__ __forceinline__ i64 send_last_of(const WinParams& wp, i64 e) {
    i64 s = send_len(wp);
    i64 l = (e / s) * s + s - 1;
    return l < wp.N - 1 ? l : wp.N - 1;
}

// Send bookkeeping of a thread's kItems consecutive events with one division: r = e % send_len.
struct SendCursor {
    i64 s, r;
    __device__ __forceinline__ SendCursor(const WinParams& wp, i64 base) {
        s = send_len(wp);
        r = s == 1 ? 0 : base % s;
    }
    __device__ __forceinline__ bool last(const WinParams& wp, i64 e) const { return r == s - 1 || e == wp.N - 1; }
    __device__ __forceinline__ i64 last_of(const WinParams& wp, i64 e) const { return min(e - r + s - 1, wp.N - 1); }
    __device__ __forceinline__ void next() { if (++r == s) r = 0; }
};

// Window number of an event. lengthBatch: from the passing-event count; timeBatch: from the
// playback clock; externalTimeBatch: `clock` is the running max M of the timestamp attribute and
// E0 the start time — the batch end is findEndTime(M) = E0 + T * ((M - E0) / T + 1)
// (ExternalTimeBatchWindowProcessor :440-444), so the window is (M - E0) / T.
__device__ __forceinline__ i64 wfun(const WinParams& wp, i64 E0, int e0_valid, i64 pcb, i64 clock) {
    if (wp.kind == SH_WIN_LENGTH_BATCH) return (wp.n_pend + pcb) / wp.L;
    if (!e0_valid) return wp.W_open;
    if (wp.kind == SH_WIN_EXT_TIME_BATCH) return clock < E0 ? 0 : (clock - E0) / wp.T;
    if (wp.cal) return clock < E0 ? 0 : cal_idx_d(clock, wp.cal, wp.cal_tz) - cal_idx_d(E0, wp.cal, wp.cal_tz) + 1;
    return clock < E0 ? 0 : (clock - E0) / wp.T + 1;
}

// W of successive events with at most one division per window change: `lim` is the smallest pcb
// (lengthBatch) or clock (timeBatch) at which W grows.
struct WinCursor {
    i64 W, lim;
    __device__ __forceinline__ void set(const WinParams& wp, i64 E0, int e0v, i64 pcb, i64 clk) {
        W = wfun(wp, E0, e0v, pcb, clk);
        if (wp.kind == SH_WIN_LENGTH_BATCH) lim = (W + 1) * wp.L - wp.n_pend;
        else if (!e0v) lim = INT64_MAX;
        else if (wp.kind == SH_WIN_EXT_TIME_BATCH) lim = E0 + (W + 1) * wp.T;
        else if (wp.cal) lim = cal_start_d(cal_idx_d(E0, wp.cal, wp.cal_tz) + W, wp.cal, wp.cal_tz);
        else lim = E0 + W * wp.T;
    }
    __device__ __forceinline__ i64 at(const WinParams& wp, i64 E0, int e0v, i64 pcb, i64 clk) {
        i64 x = wp.kind == SH_WIN_LENGTH_BATCH ? pcb : clk;
        if (x >= lim) set(wp, E0, e0v, pcb, clk);
        return W;
    }
};

}  // namespace shd
