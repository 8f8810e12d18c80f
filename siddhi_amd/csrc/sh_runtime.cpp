// sh_runtime.cpp — host runtime behind include/siddhi_hip.h: query objects, device buffers,
// launch sequencing and output assembly. Runs only the HIP path; any feature without a GPU
// implementation is refused with SH_ERR_UNSUPPORTED (there is no CPU fallback).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "sh_agg.h"
#include "sh_internal.h"
#include "sh_runtime.h"

#include <chrono>

using namespace shd;

thread_local std::string g_last_error;

int sh_fail(int code, const std::string& msg) {
    g_last_error = msg;
    SH_TRACE("error %d: %s", code, msg.c_str());
    return code;
}

namespace {
struct HostTiming {
    static constexpr int kPts = 16;
    std::vector<double> d[kPts];
    std::chrono::steady_clock::time_point last;
    int last_pt = -1;
    ~HostTiming() {
        if (!sh_timing_on()) return;
        for (int p = 1; p < kPts; p++) {
            if (d[p].empty()) continue;
            std::vector<double> v = d[p];
            std::sort(v.begin(), v.end());
            fprintf(stderr, "[sh timing] ->%d: %zu x, median %.1f us, min %.1f, max %.1f\n", p, v.size(), v[v.size() / 2],
                    v.front(), v.back());
        }
    }
};
HostTiming g_timing;
}  // namespace

template <typename Q, typename W>
static hipError_t poll_then_wait(Q query, W wait) {
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; it++) {
        const hipError_t e = query();
        if (e != hipErrorNotReady) return e;
        if ((it & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) return wait();
    }
}

hipError_t sh_wait_stream(hipStream_t s) {
    return poll_then_wait([&] { return hipStreamQuery(s); }, [&] { return hipStreamSynchronize(s); });
}

hipError_t sh_wait_event(hipEvent_t e) {
    return poll_then_wait([&] { return hipEventQuery(e); }, [&] { return hipEventSynchronize(e); });
}

bool sh_timing_on() {
    static const bool on = getenv("SH_TIMING") != nullptr;
    return on;
}

// point 0 starts a push; point p > 0 adds the time since the previous point to slot p
void sh_timing_mark(int p) {
    const auto now = std::chrono::steady_clock::now();
    if (p > 0 && g_timing.last_pt >= 0 && p < HostTiming::kPts) {
        g_timing.d[p].push_back(std::chrono::duration<double, std::micro>(now - g_timing.last).count());
    }
    g_timing.last = now;
    g_timing.last_pt = p;
}

bool sh_trace_on() {
    static const bool on = [] {
        const char* e = getenv("SH_TRACE");
        return e && *e && *e != '0';
    }();
    return on;
}

#define HIPCHK(x)                                                                                          \
    do {                                                                                                   \
        hipError_t _e = (x);                                                                               \
        if (_e != hipSuccess) return sh_fail(SH_ERR_DEVICE, std::string(#x) + ": " + hipGetErrorString(_e)); \
    } while (0)

// ---------------------------------------------------------------------------------------------
// device buffer helpers
// ---------------------------------------------------------------------------------------------
thread_local hipStream_t g_stream = nullptr;

// Growth on the calling context's stream, with plain (not stream-ordered) allocations: the stream is
// drained before the old block is copied and freed. hipMallocAsync / hipFreeAsync pool reuse was seen
// to hand a block back while a copy out of it was still pending (the sliding window's FIFO came back
// corrupted at C3 size, nondeterministically); growth is rare (x1.5 steps), so two waits per growth
// cost nothing in steady state. Outside any API scope (g_stream null) the whole device is drained.
static hipError_t drain() { return g_stream ? hipStreamSynchronize(g_stream) : hipDeviceSynchronize(); }

int DevBuf::reserve(size_t n, bool keep) {
    if (n <= cap) return SH_OK;
    size_t ncap = std::max(n, cap + cap / 2);
    void* np = nullptr;
    static const bool trace = getenv("SH_ALLOC_TRACE") != nullptr;  // (diagnostics: growth in a push)
    if (trace && ncap >= (1u << 20))
        fprintf(stderr, "[sh alloc] %zu -> %zu bytes (keep %d)\n", cap, ncap, (int)keep);
    hipError_t e = hipMalloc(&np, ncap);
    if (e != hipSuccess) return sh_fail(SH_ERR_OOM, "device allocation failed: " + std::string(hipGetErrorString(e)));
    if (p) {
        if (keep && used) {
            e = hipMemcpyAsync(np, p, used, hipMemcpyDeviceToDevice, g_stream);
            if (e != hipSuccess) {
                (void)drain();
                (void)hipFree(np);
                return sh_fail(SH_ERR_DEVICE, "device copy (grow) failed");
            }
        }
        release();
    }
    p = np;
    cap = ncap;
    return SH_OK;
}

void DevBuf::release() {
    if (p) {
        (void)drain();  // kernels and copies queued on the block have finished
        (void)hipFree(p);
    }
    p = nullptr;
    cap = used = 0;
}

int PinnedBuf::reserve(size_t n) {
    if (n <= cap) return SH_OK;
    release();
    size_t ncap = std::max<size_t>(n, 4096);
    if (hipHostMalloc(&p, ncap, hipHostMallocDefault) != hipSuccess) {
        p = nullptr;
        return sh_fail(SH_ERR_OOM, "pinned host allocation failed");
    }
    cap = ncap;
    return SH_OK;
}

void PinnedBuf::release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
}

// ---------------------------------------------------------------------------------------------
// context
// ---------------------------------------------------------------------------------------------
extern "C" int sh_init(int32_t device, sh_ctx** out) {
    if (!out) return sh_fail(SH_ERR_INVALID, "sh_init: out is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0) return sh_fail(SH_ERR_DEVICE, "no HIP device visible (this library has no CPU path)");
    if (device < 0 || device >= n) return sh_fail(SH_ERR_INVALID, "sh_init: bad device ordinal");
    HIPCHK(hipSetDevice(device));
    hipDeviceProp_t prop;
    HIPCHK(hipGetDeviceProperties(&prop, device));
    if (std::string(prop.gcnArchName).find("gfx950") == std::string::npos)
        return sh_fail(SH_ERR_DEVICE, std::string("built for gfx950, found ") + prop.gcnArchName);
    // stream-ordered buffers come from the device's default pool; keep what it has reserved instead
    // of handing it back at every synchronisation (a grown buffer's old block is reused, not re-mapped)
    hipMemPool_t pool = nullptr;
    if (hipDeviceGetDefaultMemPool(&pool, device) == hipSuccess && pool) {
        uint64_t keep = UINT64_MAX;
        (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep);
    }
    sh_ctx* c = new sh_ctx();
    c->device = device;
    c->num_cus = prop.multiProcessorCount;
    c->max_lds = (int)prop.sharedMemPerBlock;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c->copy_stream, hipStreamNonBlocking) != hipSuccess) {
        if (c->stream) (void)hipStreamDestroy(c->stream);
        delete c;
        return sh_fail(SH_ERR_DEVICE, "hipStreamCreate failed");
    }
    *out = c;
    return SH_OK;
}

extern "C" int sh_ctx_destroy(sh_ctx* c) {
    if (!c) return SH_OK;
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->copy_stream);
    (void)hipStreamDestroy(c->stream);
    (void)hipStreamDestroy(c->copy_stream);
    delete c;
    return SH_OK;
}

extern "C" int sh_alloc_pinned(int64_t bytes, void** out) {
    if (!out || bytes < 0) return sh_fail(SH_ERR_INVALID, "sh_alloc_pinned: bad arguments");
    HIPCHK(hipHostMalloc(out, (size_t)std::max<int64_t>(bytes, 1), hipHostMallocDefault));
    return SH_OK;
}

extern "C" int sh_free_pinned(void* p) {
    if (p) HIPCHK(hipHostFree(p));
    return SH_OK;
}

extern "C" const char* sh_last_error(void) { return g_last_error.c_str(); }
extern "C" int32_t sh_abi_version(void) { return SH_ABI_VERSION; }

Tuning Tuning::from_env() {
    Tuning t;
    auto on = [](const char* n) { const char* v = getenv(n); return v && *v && strcmp(v, "0") != 0; };
    t.direct_pos = on("SH_DIRECT_POS");
    t.part_keys_1024 = getenv("SH_PART_KEYS") && atoi(getenv("SH_PART_KEYS")) == 1024;
    t.no_async_small = on("SH_NO_ASYNC_SMALL");
    // measured faster on MI355X (3.12 vs 3.03 G events/s on C3, profiles/r04_c3_records_seq.txt): default,
    // SH_SL_RECORDS_SEQ=0 restores the one-pass form
    t.sl_records_seq = !getenv("SH_SL_RECORDS_SEQ") || on("SH_SL_RECORDS_SEQ");
    // sorted chunks for partitioned lengthBatch keyed by the partition: 5.5e8 vs 8.2e6 events/s over
    // C5's Zipf partitions (one sequential lane per partition serialises the hot one); SH_PL_SORT=0 walks
    t.pl_sort = !getenv("SH_PL_SORT") || on("SH_PL_SORT");
    if (getenv("SH_AGG_BAND_ROWS")) t.agg_band_rows = atoi(getenv("SH_AGG_BAND_ROWS"));
    t.slx_wave = !getenv("SH_SLX_WAVE") || on("SH_SLX_WAVE");
    return t;
}

extern "C" int sh_query_set_strings(sh_query* q, int32_t col, int64_t first_id, int64_t n, const uint16_t* units,
                                    const int64_t* offsets) {
    if (!q) return sh_fail(SH_ERR_INVALID, "sh_query_set_strings: NULL query");
    if (col < 0 || col >= q->d.n_cols || q->d.col_types[col] != SH_T_STRID)
        return sh_fail(SH_ERR_INVALID, "sh_query_set_strings: not a string column");
    if (first_id < 0 || n < 0 || first_id + n > ((int64_t)1 << 31) || (n > 0 && (!units || !offsets)))
        return sh_fail(SH_ERR_INVALID, "sh_query_set_strings: bad id range");
    for (int64_t i = 0; i < n; i++)
        if (offsets[i + 1] < offsets[i] || offsets[i] < 0)
            return sh_fail(SH_ERR_INVALID, "sh_query_set_strings: offsets must be non-decreasing");
    auto& v = q->strings[col];
    auto& set = q->strings_set[col];
    if ((int64_t)v.size() < first_id + n) {
        v.resize((size_t)(first_id + n));
        set.resize((size_t)(first_id + n), 0);
    }
    for (int64_t i = 0; i < n; i++) {
        const size_t id = (size_t)(first_id + i);
        if (set[id] && v[id].compare(0, std::u16string::npos, (const char16_t*)units + offsets[i],
                                     (size_t)(offsets[i + 1] - offsets[i])) != 0)
            return sh_fail(SH_ERR_INVALID, "sh_query_set_strings: id " + std::to_string(id) + " already has another text");
        v[id].assign((const char16_t*)units + offsets[i], (const char16_t*)units + offsets[i + 1]);
        set[id] = 1;
    }
    return SH_OK;
}

// ---------------------------------------------------------------------------------------------
// descriptor compilation
// ---------------------------------------------------------------------------------------------
static bool integral(int t) { return t == SH_T_INT || t == SH_T_LONG || t == SH_T_STRID || t == SH_T_BOOL; }
static bool numeric(int t) { return t == SH_T_INT || t == SH_T_LONG || t == SH_T_FLOAT || t == SH_T_DOUBLE; }

int compile_filter(int n_ops, const sh_filter_op* ops, int n_cols, const int32_t* types, FilterProg& fp) {
    if (n_ops < 0 || n_ops > kMaxFilterOps) return sh_fail(SH_ERR_UNSUPPORTED, "filter program longer than 32 ops");
    fp = FilterProg{};
    fp.n = n_ops;
    int depth = 0;
    for (int i = 0; i < n_ops; i++) {
        const sh_filter_op& o = ops[i];
        FilterOpD d{o.op, o.type, o.col, 0, o.ival, o.dval};
        switch (o.op) {
            case SH_OP_COL:
                if (o.col < 0 || o.col >= n_cols) return sh_fail(SH_ERR_INVALID, "filter column out of range");
                if (types[o.col] == SH_T_STRID && false) {}
                depth++;
                break;
            case SH_OP_CONST: depth++; break;
            case SH_OP_NOT: if (depth < 1) return sh_fail(SH_ERR_INVALID, "filter stack underflow"); break;
            case SH_OP_GT: case SH_OP_GE: case SH_OP_LT: case SH_OP_LE: case SH_OP_EQ: case SH_OP_NE:
            case SH_OP_AND: case SH_OP_OR:
                if (depth < 2) return sh_fail(SH_ERR_INVALID, "filter stack underflow");
                depth--;
                break;
            default: return sh_fail(SH_ERR_INVALID, "unknown filter opcode");
        }
        if (depth > 16) return sh_fail(SH_ERR_UNSUPPORTED, "filter stack deeper than 16");
        fp.ops[i] = d;
    }
    if (n_ops > 0 && depth != 1) return sh_fail(SH_ERR_INVALID, "filter program leaves stack depth != 1");
    return SH_OK;
}

int compile_aggs(int n_aggs, const sh_agg_spec* aggs, int n_cols, const int32_t* types, AggPlan& ap,
                 int32_t* out_types) {
    ap = AggPlan{};
    ap.n = n_aggs;
    for (int a = 0; a < n_aggs; a++) {
        int fn = aggs[a].fn, col = aggs[a].col;
        if (fn == SH_AGG_COUNT) {
            ap.kind[a] = AK_COUNT; ap.field[a] = -1; ap.vcol[a] = -1;
            out_types[a] = SH_T_LONG;
            continue;
        }
        if (col < 0 || col >= n_cols) return sh_fail(SH_ERR_INVALID, "aggregator column out of range");
        int t = types[col];
        if (!numeric(t)) return sh_fail(SH_ERR_INVALID, "aggregator over a non-numeric attribute");
        int v = -1;
        for (int j = 0; j < ap.n_vcols; j++) if (ap.vcol_src[j] == col) v = j;
        if (v < 0) { v = ap.n_vcols++; ap.vcol_src[v] = col; ap.vcol_type[v] = t; }
        ap.vcol[a] = v;
        ap.field[a] = ap.n_fields++;
        bool fp = t == SH_T_FLOAT || t == SH_T_DOUBLE;
        switch (fn) {
            case SH_AGG_SUM: ap.kind[a] = fp ? AK_SUM_D : AK_SUM_L; out_types[a] = fp ? SH_T_DOUBLE : SH_T_LONG; break;
            case SH_AGG_AVG: ap.kind[a] = AK_AVG; out_types[a] = SH_T_DOUBLE; break;
            case SH_AGG_MIN:
                ap.kind[a] = t == SH_T_DOUBLE ? AK_MIN_D : t == SH_T_FLOAT ? AK_MIN_F : AK_MIN_L;
                out_types[a] = t;
                break;
            case SH_AGG_MAX:
                ap.kind[a] = t == SH_T_DOUBLE ? AK_MAX_D : t == SH_T_FLOAT ? AK_MAX_F : AK_MAX_L;
                out_types[a] = t;
                break;
            default: return sh_fail(SH_ERR_INVALID, "unknown aggregator");
        }
    }
    for (int a = 0; a < n_aggs; a++) {
        if (ap.kind[a] == AK_COUNT) continue;
        int f = ap.field[a], v = ap.vcol[a];
        bool fpcol = ap.vcol_type[v] == SH_T_FLOAT || ap.vcol_type[v] == SH_T_DOUBLE;
        ap.fvcol[f] = v;
        switch (ap.kind[a]) {
            case AK_SUM_L: ap.fop[f] = FOP_ADD_I; break;
            case AK_SUM_D: ap.fop[f] = FOP_ADD_D; break;
            case AK_AVG: ap.fop[f] = fpcol ? FOP_ADD_D : FOP_ADD_DI; break;
            case AK_MIN_L: ap.fop[f] = FOP_MIN_I; break;
            case AK_MAX_L: ap.fop[f] = FOP_MAX_I; break;
            case AK_MIN_D: ap.fop[f] = FOP_MIN_D; break;
            case AK_MAX_D: ap.fop[f] = FOP_MAX_D; break;
            case AK_MIN_F: ap.fop[f] = FOP_MIN_F; break;
            case AK_MAX_F: ap.fop[f] = FOP_MAX_F; break;
        }
    }
    return SH_OK;
}

int compile_keys(int n_group, const int32_t* group, int n_cols, const int32_t* types, KeyPlan& kp) {
    kp = KeyPlan{};
    kp.n = n_group;
    if (n_group < 0 || n_group > SH_MAX_GROUP) return sh_fail(SH_ERR_INVALID, "bad group-by count");
    if (n_group > kKeyParts)
        return sh_fail(SH_ERR_UNSUPPORTED, "more than two group-by columns key this window only interned (sh_wide.h)");
    for (int g = 0; g < n_group; g++) {
        int c = group[g];
        if (c < 0 || c >= n_cols) return sh_fail(SH_ERR_INVALID, "group-by column out of range");
        if (!integral(types[c]) && types[c] != SH_T_FLOAT && types[c] != SH_T_DOUBLE)
            return sh_fail(SH_ERR_INVALID, "unknown group-by column type");
        kp.col[g] = c;
        kp.type[g] = types[c];
    }
    // one column of any type, or two 32-bit ones (int / string id / bool / float): the key is one u64
    if (n_group == 2 && (kp.type[0] == SH_T_LONG || kp.type[1] == SH_T_LONG || kp.type[0] == SH_T_DOUBLE ||
                         kp.type[1] == SH_T_DOUBLE))
        return sh_fail(SH_ERR_UNSUPPORTED, "two group-by columns must both be 32-bit (int, string, bool, float)");
    // string keys arrive as dictionary ids the host assigns densely from 0: the id is the slot
    kp.dense = n_group == 1 && kp.type[0] == SH_T_STRID;
    return SH_OK;
}

int KeyTableHost::init(int64_t capacity) {
    int64_t want = std::max<int64_t>(16, 2 * std::max<int64_t>(1, capacity));
    size_t ts = 16;
    while ((int64_t)ts < want) ts <<= 1;
    return init_size(ts);
}

int KeyTableHost::init_dense(int64_t capacity, uint32_t mul, uint32_t add) {
    size_t ts = 16;
    while ((int64_t)ts < capacity) ts <<= 1;
    dense = true;
    lk = 0;
    dmul = mul;
    dadd = add;
    size_ = ts;
    n_keys = 0;
    int rc = keys.reserve(64, false);
    if (rc) return rc;
    rc = ctrl.reserve(64, false);
    if (rc) return rc;
    if (hipMemsetAsync(ctrl.p, 0, 64, g_stream) != hipSuccess) return sh_fail(SH_ERR_DEVICE, "key table init failed");
    return SH_OK;
}

int KeyTableHost::init_band(uint32_t lg, uint32_t nrows, int64_t base, uint32_t mul, uint32_t add) {
    int rc = init_dense((int64_t)nrows << lg, mul, add);
    if (rc) return rc;
    lk = lg;
    rows = nrows;
    band_base = base;
    b0 = (uint32_t)base;
    return SH_OK;
}

int KeyTableHost::init_size(size_t ts) {
    dense = false;
    lk = 0;
    size_ = ts;
    n_keys = 0;
    int rc = keys.reserve(ts * 8, false);
    if (rc) return rc;
    rc = ctrl.reserve(64, false);
    if (rc) return rc;
    // EMPTY sentinels written on the device, in the calling context's stream order
    launch_fill_i64(g_stream, (int64_t*)keys.p, (int64_t)ts, (int64_t)kEmptyKey);
    if (hipGetLastError() != hipSuccess || hipMemsetAsync(ctrl.p, 0, 64, g_stream) != hipSuccess)
        return sh_fail(SH_ERR_DEVICE, "key table init failed");
    return SH_OK;
}

KeyTable KeyTableHost::dev() const {
    KeyTable kt;
    kt.keys = (u64*)keys.p;
    kt.mask = (u32)(size_ - 1);
    int lg = 0;
    while (((size_t)1 << lg) < size_) lg++;
    kt.shift = (u32)(64 - lg);
    kt.n_keys = (u32*)ctrl.p;
    kt.overflow = (int*)((char*)ctrl.p + 8);
    kt.dense = dense ? 1 : 0;
    kt.dmul = dmul;
    kt.dadd = dadd;
    kt.lk = lk;
    kt.b0 = b0;
    kt.rows = rows;
    return kt;
}

int KeyTableHost::check_async(hipStream_t s, uint32_t* pinned4) {
    if (hipMemcpyAsync(pinned4, ctrl.p, 16, hipMemcpyDeviceToHost, s) != hipSuccess)
        return sh_fail(SH_ERR_DEVICE, "key table check failed");
    return SH_OK;
}

int KeyTableHost::check_result(const uint32_t* c) {
    n_keys = c[0];
    if (c[2] == 2) return sh_fail(SH_ERR_INVALID, "dictionary id outside [0, key_capacity): raise key_capacity");
    if (c[2] == 3) return sh_fail(SH_ERR_DEVICE, "aggregation time bucket outside the root key band");
    if (c[2]) return sh_fail(SH_ERR_INVALID, "group key table full: raise key_capacity");
    return SH_OK;
}

int KeyTableHost::check(hipStream_t s) {
    int rc = h_ctrl.reserve(16);
    if (rc) return rc;
    if ((rc = check_async(s, h_ctrl.as<uint32_t>()))) return rc;
    if (hipStreamSynchronize(s) != hipSuccess) return sh_fail(SH_ERR_DEVICE, "key table check failed");
    return check_result(h_ctrl.as<uint32_t>());
}
