// siddhi_oracle.cpp — CPU restatement of the reference's filtered windowed group-by aggregation
// and incremental aggregation semantics.
//
// TEST INFRASTRUCTURE ONLY. This file is the parity checker: only tests/, __graft_entry__.smoke()
// and bench.py's cpu_baseline leg may load it. The product library (siddhi_amd/csrc) never links
// or calls it, and has no CPU fallback.
//
// The reference is Java (Arshardh/siddhi @ 5.1.21-SNAPSHOT) and cannot be built or run in this
// image (no JVM), so this restatement follows the Java sources line by line. Parity is pinned by
// the known-answer vectors transcribed from the reference's own TestNG cases into
// tests/golden/kat_*.json (see tests/test_oracle_kat.py). Citations:
//   core/ = /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/
//
// Every function below names the Java method it restates.

#include "../include/siddhi_hip.h"
#include "oracle.h"
#include "jhashmap.h"

#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <deque>
#include <list>
#include <map>
#include <memory>
#include <set>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

thread_local std::string g_err;

// ------------------------------------------------------------------------------------------
// Java value model. A column value is kept as raw 8 bytes: int64 for INT/LONG/STRID/BOOL,
// double for FLOAT/DOUBLE (a float is held exactly as its double widening).
// ------------------------------------------------------------------------------------------
struct JVal {
    int t = 0;       // SH_T_*; 0 = null
    int64_t i = 0;   // integral value
    double d = 0.0;  // floating value
};

inline bool is_fp(int t) { return t == SH_T_FLOAT || t == SH_T_DOUBLE; }

// Java (long) cast of a double: NaN -> 0, saturating, truncation toward zero (JLS 5.1.3).
inline int64_t java_d2l(double x) {
    if (std::isnan(x)) return 0;
    if (x >= 9.2233720368547758e18) return INT64_MAX;
    if (x <= -9.2233720368547758e18) return INT64_MIN;
    return (int64_t)x;
}

// Promotion rank INT(1) < LONG(2) < FLOAT(3) < DOUBLE(4); STRID/BOOL compare as INT.
inline int rank_of(int t) {
    switch (t) {
        case SH_T_LONG: return 2;
        case SH_T_FLOAT: return 3;
        case SH_T_DOUBLE: return 4;
        default: return 1;
    }
}

// Compare executors, core/executor/condition/compare/**: relational ops use binary numeric
// promotion ((Float) l > (Long) r compares as float); ==/!= use the same except FloatLong and
// LongFloat which call doubleValue() on both sides
// (equal/EqualCompareConditionExpressionExecutorFloatLong.java, ...LongFloat.java).
bool java_compare(int op, const JVal& a, const JVal& b) {
    // CompareConditionExpressionExecutor.execute: null operand -> false (line 36-40)
    if (a.t == 0 || b.t == 0) return false;
    int ra = rank_of(a.t), rb = rank_of(b.t);
    int r = std::max(ra, rb);
    bool eqop = (op == SH_OP_EQ || op == SH_OP_NE);
    if (eqop && ((a.t == SH_T_FLOAT && b.t == SH_T_LONG) || (a.t == SH_T_LONG && b.t == SH_T_FLOAT))) r = 4;
    auto as_d = [](const JVal& v) { return is_fp(v.t) ? v.d : (double)v.i; };
    auto as_f = [](const JVal& v) { return is_fp(v.t) ? (float)v.d : (float)v.i; };
    if (r == 4) {
        double x = as_d(a), y = as_d(b);
        switch (op) {
            case SH_OP_GT: return x > y; case SH_OP_GE: return x >= y;
            case SH_OP_LT: return x < y; case SH_OP_LE: return x <= y;
            case SH_OP_EQ: return x == y; default: return x != y;
        }
    } else if (r == 3) {
        float x = as_f(a), y = as_f(b);
        switch (op) {
            case SH_OP_GT: return x > y; case SH_OP_GE: return x >= y;
            case SH_OP_LT: return x < y; case SH_OP_LE: return x <= y;
            case SH_OP_EQ: return x == y; default: return x != y;
        }
    } else {
        int64_t x = a.i, y = b.i;  // int promoted to long is exact; int-int compares equal
        switch (op) {
            case SH_OP_GT: return x > y; case SH_OP_GE: return x >= y;
            case SH_OP_LT: return x < y; case SH_OP_LE: return x <= y;
            case SH_OP_EQ: return x == y; default: return x != y;
        }
    }
}

// ------------------------------------------------------------------------------------------
// Events. core/event/stream/StreamEvent.java; types from core/event/ComplexEvent.java:48-53.
// ------------------------------------------------------------------------------------------
enum EvType { CURRENT = 0, EXPIRED = 1, TIMER = 2, RESET = 3 };

struct OEvent {
    int64_t ts = 0;
    int type = CURRENT;
    int64_t seq = -1;  // stream index (arrival order over every pushed event): sh_out.rep
    std::array<int64_t, SH_MAX_COLS> raw{};  // column values, raw 8-byte form
};

using Chunk = std::vector<OEvent>;

struct Schema {
    int n = 0;
    int types[SH_MAX_COLS]{};
    JVal get(const OEvent& e, int c) const {
        JVal v;
        v.t = types[c];
        if (is_fp(v.t)) std::memcpy(&v.d, &e.raw[c], 8);
        else v.i = e.raw[c];
        return v;
    }
};

// Read event i of a batch into raw form.
void load_event(const Schema& s, const sh_batch* b, int64_t i, OEvent& e) {
    e.ts = b->ts[i];
    e.type = CURRENT;
    for (int c = 0; c < s.n; c++) {
        switch (s.types[c]) {
            case SH_T_INT: case SH_T_STRID: e.raw[c] = ((const int32_t*)b->cols[c])[i]; break;
            case SH_T_LONG: e.raw[c] = ((const int64_t*)b->cols[c])[i]; break;
            case SH_T_BOOL: e.raw[c] = ((const uint8_t*)b->cols[c])[i] ? 1 : 0; break;
            case SH_T_FLOAT: { double d = ((const float*)b->cols[c])[i]; std::memcpy(&e.raw[c], &d, 8); break; }
            case SH_T_DOUBLE: { double d = ((const double*)b->cols[c])[i]; std::memcpy(&e.raw[c], &d, 8); break; }
        }
    }
}

// FilterProcessor.process + condition executors (And/Or/Not short-circuit,
// core/executor/condition/AndConditionExpressionExecutor.java:65-74 etc.).
bool eval_filter(const Schema& s, const std::vector<sh_filter_op>& prog, const OEvent& e) {
    if (prog.empty()) return true;
    JVal st[64];
    int sp = 0;
    for (const auto& op : prog) {
        switch (op.op) {
            case SH_OP_COL: st[sp++] = s.get(e, op.col); break;
            case SH_OP_CONST: {
                JVal v; v.t = op.type;
                if (is_fp(op.type)) v.d = (op.type == SH_T_FLOAT) ? (double)(float)op.dval : op.dval;
                else v.i = (op.type == SH_T_INT) ? (int64_t)(int32_t)op.ival : op.ival;
                st[sp++] = v;
                break;
            }
            case SH_OP_GT: case SH_OP_GE: case SH_OP_LT: case SH_OP_LE: case SH_OP_EQ: case SH_OP_NE: {
                JVal b = st[--sp], a = st[--sp];
                JVal r; r.t = SH_T_BOOL; r.i = java_compare(op.op, a, b) ? 1 : 0;
                st[sp++] = r;
                break;
            }
            case SH_OP_AND: { JVal b = st[--sp], a = st[--sp]; JVal r; r.t = SH_T_BOOL; r.i = (a.i && b.i) ? 1 : 0; st[sp++] = r; break; }
            case SH_OP_OR: { JVal b = st[--sp], a = st[--sp]; JVal r; r.t = SH_T_BOOL; r.i = (a.i || b.i) ? 1 : 0; st[sp++] = r; break; }
            case SH_OP_NOT: { st[sp - 1].i = st[sp - 1].i ? 0 : 1; st[sp - 1].t = SH_T_BOOL; break; }
        }
    }
    return sp > 0 ? st[sp - 1].i != 0 : true;
}

// ------------------------------------------------------------------------------------------
// Aggregator states. Each restates the Java State subclass; `result` returns Java null as
// has=false. canDestroy() drives PartitionStateHolder.returnState removal
// (core/util/snapshot/state/PartitionStateHolder.java:50-69).
// ------------------------------------------------------------------------------------------
struct AggOut { bool has = false; int64_t i = 0; double d = 0.0; };

struct AggState {
    virtual ~AggState() {}
    virtual AggOut add(const JVal& v) = 0;
    virtual AggOut remove(const JVal& v) = 0;
    virtual bool can_destroy() const = 0;
};

// SumAttributeAggregatorExecutor.AggregatorStateDouble / Float (:164-254)
struct SumDouble : AggState {
    double sum = 0.0; int64_t count = 0;
    AggOut add(const JVal& v) override { sum += v.d; count++; AggOut o; o.has = true; o.d = sum; return o; }
    AggOut remove(const JVal& v) override {
        sum -= v.d; count--; AggOut o;
        if (count == 0) return o;
        o.has = true; o.d = sum; return o;
    }
    bool can_destroy() const override { return count == 0 && sum == 0.0; }
};
// SumAttributeAggregatorExecutor.AggregatorStateLong / Int (:256-342). processRemove goes through
// processRemove(double): `sum -= data` is `sum = (long)(sum - data)` (:283-291).
struct SumLong : AggState {
    int64_t sum = 0; int64_t count = 0;
    AggOut add(const JVal& v) override { sum += v.i; count++; AggOut o; o.has = true; o.i = sum; return o; }
    AggOut remove(const JVal& v) override {
        sum = java_d2l((double)sum - (double)v.i); count--; AggOut o;
        if (count == 0) return o;
        o.has = true; o.i = sum; return o;
    }
    bool can_destroy() const override { return count == 0 && sum == 0; }
};
// AvgAttributeAggregatorExecutor states (:143-378): double value, long count.
struct AvgState : AggState {
    double value = 0.0; int64_t count = 0;
    static double num(const JVal& v) { return is_fp(v.t) ? v.d : (double)v.i; }
    AggOut add(const JVal& v) override {
        count++; value += num(v); AggOut o;
        if (count == 0) return o;
        o.has = true; o.d = value / (double)count; return o;
    }
    AggOut remove(const JVal& v) override {
        count--; value -= num(v); AggOut o;
        if (count == 0) return o;
        o.has = true; o.d = value / (double)count; return o;
    }
    bool can_destroy() const override { return value == 0.0 && count == 0; }
};
// CountAttributeAggregatorExecutor (:96-146)
struct CountState : AggState {
    int64_t count = 0;
    AggOut add(const JVal&) override { count++; AggOut o; o.has = true; o.i = count; return o; }
    AggOut remove(const JVal&) override { count--; AggOut o; o.has = true; o.i = count; return o; }
    bool can_destroy() const override { return count == 0; }
};

// Min/Max: MinAttributeAggregatorExecutor (:86-483), MaxAttributeAggregatorExecutor (:85-475).
// trackFutureStates (SLIDE mode or expired output) keeps a LinkedList deque; processRemove calls
// removeFirstOccurrence(value) (Double.equals / Float.equals / Integer.equals / Long.equals).
template <bool IS_MIN>
struct MinMaxState : AggState {
    int t;                     // input type
    bool track;
    std::list<JVal> dq;        // Deque<T>
    bool has = false;          // volatile T minValue != null
    JVal val;
    MinMaxState(int type, bool tr) : t(type), track(tr) {}
    // `iterator.next() > value` / `<` on unboxed values of the same type
    bool worse(const JVal& cur, const JVal& v) const {
        if (is_fp(t)) {
            if (t == SH_T_FLOAT) { float a = (float)cur.d, b = (float)v.d; return IS_MIN ? (a > b) : (a < b); }
            return IS_MIN ? (cur.d > v.d) : (cur.d < v.d);
        }
        return IS_MIN ? (cur.i > v.i) : (cur.i < v.i);
    }
    // Boxed equals: Double.equals compares doubleToLongBits (NaN == NaN, 0.0 != -0.0);
    // Float.equals compares floatToIntBits.
    bool boxed_equals(const JVal& a, const JVal& b) const {
        if (t == SH_T_DOUBLE) {
            double x = a.d, y = b.d;
            if (std::isnan(x) && std::isnan(y)) return true;
            uint64_t bx, by; std::memcpy(&bx, &x, 8); std::memcpy(&by, &y, 8); return bx == by;
        }
        if (t == SH_T_FLOAT) {
            float x = (float)a.d, y = (float)b.d;
            if (std::isnan(x) && std::isnan(y)) return true;
            uint32_t bx, by; std::memcpy(&bx, &x, 4); std::memcpy(&by, &y, 4); return bx == by;
        }
        return a.i == b.i;
    }
    AggOut out() const { AggOut o; if (!has) return o; o.has = true; if (is_fp(t)) o.d = val.d; else o.i = val.i; return o; }
    AggOut add(const JVal& v) override {
        if (track) {
            // for (descendingIterator) { if (next > value) remove; else break; } addLast(value)
            while (!dq.empty() && worse(dq.back(), v)) dq.pop_back();
            dq.push_back(v);
        }
        if (!has || worse(val, v)) { has = true; val = v; }
        return out();
    }
    AggOut remove(const JVal& v) override {
        if (track) {
            for (auto it = dq.begin(); it != dq.end(); ++it) {
                if (boxed_equals(*it, v)) { dq.erase(it); break; }
            }
            if (dq.empty()) has = false; else { has = true; val = dq.front(); }
        } else {
            if (has && boxed_equals(val, v)) has = false;
        }
        return out();
    }
    bool can_destroy() const override { return dq.empty() && !has; }
};

struct AggDef {
    int fn; int col; int in_type; int out_type; bool track;
};

std::unique_ptr<AggState> make_state(const AggDef& a) {
    switch (a.fn) {
        case SH_AGG_SUM:
            if (is_fp(a.in_type)) return std::unique_ptr<AggState>(new SumDouble());
            return std::unique_ptr<AggState>(new SumLong());
        case SH_AGG_AVG: return std::unique_ptr<AggState>(new AvgState());
        case SH_AGG_COUNT: return std::unique_ptr<AggState>(new CountState());
        case SH_AGG_MIN: return std::unique_ptr<AggState>(new MinMaxState<true>(a.in_type, a.track));
        default: return std::unique_ptr<AggState>(new MinMaxState<false>(a.in_type, a.track));
    }
}

// Return types: Sum -> LONG/DOUBLE (:92-104), Avg -> DOUBLE, Count -> LONG, Min/Max -> input type.
int agg_out_type(int fn, int in_type) {
    switch (fn) {
        case SH_AGG_SUM: return is_fp(in_type) ? SH_T_DOUBLE : SH_T_LONG;
        case SH_AGG_AVG: return SH_T_DOUBLE;
        case SH_AGG_COUNT: return SH_T_LONG;
        default: return (in_type == SH_T_STRID || in_type == SH_T_BOOL) ? SH_T_INT : in_type;
    }
}

// Group key: GroupByKeyGenerator.constructEventKey (core/query/selector/GroupByKeyGenerator.java:
// 63-73) concatenates toString()+":-:"; for the integral columns used as keys, string equality is
// value equality, so the key is the tuple of raw values.
struct GKey {
    int64_t k[SH_MAX_GROUP + 1] = {};
    bool operator==(const GKey& o) const { return k[0] == o.k[0] && k[1] == o.k[1] && k[2] == o.k[2]; }
};
struct GKeyHash {
    size_t operator()(const GKey& g) const {
        uint64_t h = 1469598103934665603ull;
        for (int i = 0; i < SH_MAX_GROUP + 1; i++) { h ^= (uint64_t)g.k[i]; h *= 1099511628211ull; h ^= h >> 29; }
        return (size_t)h;
    }
};

// Canonical raw key of a column value: NaN canonicalised for floating keys.
int64_t key_raw(const Schema& s, const OEvent& e, int c) {
    if (is_fp(s.types[c])) {
        double d; std::memcpy(&d, &e.raw[c], 8);
        if (std::isnan(d)) d = NAN;
        int64_t r; std::memcpy(&r, &d, 8); return r;
    }
    return e.raw[c];
}

// Output collection: one flush per selector output chunk.
struct OutRow {
    int64_t ts; uint8_t expired; int64_t keys[SH_MAX_GROUP + 1];  // (+1: an aggregation table's bucket)
    uint64_t vals[SH_MAX_AGGS]; uint8_t nulls[SH_MAX_AGGS];
    int64_t rep;  // stream index of the event the row was built from
    int64_t rep_attr;  // externalTimeBatch: that event's timestamp attribute as the window holds it
};
struct OutBuf {
    std::vector<int64_t> flush_offsets{0};
    std::vector<int64_t> flush_clock;
    std::vector<OutRow> rows;
    // flattened views for sh_out
    std::vector<int64_t> ts, keys, rep, rep_attr; std::vector<uint8_t> expired, nulls; std::vector<uint64_t> vals;
    bool with_rep = true;  // aggregation tables carry no representative event (sh_out.rep NULL)
    sh_out out{};
    void clear() { flush_offsets.assign(1, 0); flush_clock.clear(); rows.clear(); }
    void close_flush(int64_t clock) { flush_offsets.push_back((int64_t)rows.size()); flush_clock.push_back(clock); }
    const sh_out* view(int nk, int nv, const int* vtypes) {
        int64_t n = (int64_t)rows.size();
        ts.resize(n); expired.resize(n); keys.assign((size_t)nk * n, 0); rep.resize(n); rep_attr.resize(n);
        vals.assign((size_t)nv * n, 0); nulls.assign((size_t)nv * n, 0);
        for (int64_t r = 0; r < n; r++) {
            ts[r] = rows[r].ts; expired[r] = rows[r].expired; rep[r] = rows[r].rep; rep_attr[r] = rows[r].rep_attr;
            for (int k = 0; k < nk; k++) keys[k * n + r] = rows[r].keys[k];
            for (int v = 0; v < nv; v++) { vals[v * n + r] = rows[r].vals[v]; nulls[v * n + r] = rows[r].nulls[v]; }
        }
        out.n_flushes = (int64_t)flush_clock.size();
        out.n_rows = n; out.n_keys = nk; out.n_vals = nv;
        for (int v = 0; v < nv; v++) out.val_types[v] = vtypes[v];
        out.flush_offsets = flush_offsets.data(); out.flush_clock = flush_clock.data();
        out.ts = ts.data(); out.expired = expired.data(); out.keys = keys.data();
        out.vals = vals.data(); out.nulls = nulls.data();
        out.rep = with_rep ? rep.data() : nullptr;
        return &out;
    }
};

// ==========================================================================================
// Output rate limiting `output [all|first|last] every N events` (OutputParser.java:288-303 picks the
// limiter; core/query/output/ratelimit/event/*.java). Each selector output chunk (one flush here) is
// one process() call; a call that emits rows sends one chunk with the flush's clock.
// ==========================================================================================
struct RateLimiter {
    int kind = SH_RATE_NONE;
    int64_t value = 0;
    bool group_by = false;
    int64_t counter = 0;                          // All/First/Last(GroupBy)PerEvent: state.counter
    std::vector<OutRow> all_chunk;                // AllPerEvent: state.allComplexEventChunk
    std::map<std::vector<int64_t>, int64_t> first_count;  // FirstGroupByPerEvent: groupByOutputTime
    std::vector<std::vector<int64_t>> last_order;  // LastGroupByPerEvent: allGroupByKeyEvents (LinkedHashMap)
    std::map<std::vector<int64_t>, OutRow> last_rows;
    int nk = 0;

    bool has_out_time = false;                     // FirstPerTime: state.outputTime != null
    int64_t out_time = 0;
    std::map<std::vector<int64_t>, int64_t> first_time;  // FirstGroupByPerTime: groupByOutputTime

    std::vector<int64_t> key_of(const OutRow& r) const { return std::vector<int64_t>(r.keys, r.keys + nk); }

    // one selector output chunk at playback clock `now`
    void process(const OutRow* rows, int64_t n, std::vector<OutRow>& out, int64_t now) {
        if (kind == SH_RATE_FIRST_TIME) {
            if (!group_by) {  // FirstPerTimeOutputRateLimiter.process :54-78: the chunk's first event
                if (n > 0 && (!has_out_time || out_time + value <= now)) {
                    has_out_time = true;
                    out_time = now;
                    out.push_back(rows[0]);
                }
                return;
            }
            for (int64_t i = 0; i < n; i++) {  // FirstGroupByPerTimeOutputRateLimiter.process :54-80
                const std::vector<int64_t> k = key_of(rows[i]);
                auto it = first_time.find(k);
                if (it == first_time.end() || it->second + value <= now) {
                    first_time[k] = now;
                    out.push_back(rows[i]);
                }
            }
            return;
        }
        for (int64_t i = 0; i < n; i++) {
            const OutRow& ev = rows[i];
            if (kind == SH_RATE_ALL) {  // AllPerEventOutputRateLimiter.process :48-77
                all_chunk.push_back(ev);
                if (++counter == value) {
                    out.insert(out.end(), all_chunk.begin(), all_chunk.end());
                    all_chunk.clear();
                    counter = 0;
                }
            } else if (kind == SH_RATE_FIRST && !group_by) {  // FirstPerEventOutputRateLimiter :48-72
                counter++;
                if (counter == 1) out.push_back(ev);
                else if (counter == value) counter = 0;
            } else if (kind == SH_RATE_LAST && !group_by) {  // LastPerEventOutputRateLimiter :47-71
                if (++counter == value) {
                    out.push_back(ev);
                    counter = 0;
                }
            } else if (kind == SH_RATE_FIRST) {  // FirstGroupByPerEventOutputRateLimiter :48-77
                const std::vector<int64_t> k = key_of(ev);
                auto it = first_count.find(k);
                if (it == first_count.end()) {
                    first_count[k] = 1;
                    out.push_back(ev);
                } else if (it->second == value - 1) {
                    first_count.erase(it);
                } else {
                    it->second++;
                }
            } else {  // LastGroupByPerEventOutputRateLimiter :51-83
                const std::vector<int64_t> k = key_of(ev);
                if (!last_rows.count(k)) last_order.push_back(k);
                last_rows[k] = ev;
                if (++counter == value) {
                    counter = 0;
                    for (const auto& kk : last_order) out.push_back(last_rows[kk]);
                    last_order.clear();
                    last_rows.clear();
                }
            }
        }
    }
};

// ==========================================================================================
// Window query engine
// ==========================================================================================
struct PartitionState {
    // LengthBatchWindowProcessor.WindowState (:302-350)
    int count = 0;
    Chunk current_queue, expired_queue;
    bool has_reset = false; OEvent reset_event;
    // TimeWindowProcessor.WindowState (:196-222)
    std::deque<OEvent> time_queue;
    int64_t last_timestamp = INT64_MIN;
    // per-aggregator group states: PartitionStateHolder states.get(partitionFlowId)
    std::vector<std::unordered_map<GKey, std::unique_ptr<AggState>, GKeyHash>> agg_states;
    // Scheduler.SchedulerState (core/util/Scheduler.java:330-367): toNotifyQueue
    std::deque<int64_t> notify_queue;
    // ExternalTimeBatchWindowProcessor.WindowState (:495-517): endTime = -1, startTime = the constant
    // start (commonStartTime, 0 when absent), lastCurrentEventTime = 0 (Java default)
    int64_t ext_end = -1, ext_start = 0, ext_last = 0;
    int64_t ext_sched = 0;     // lastScheduledTime (timeout form)
    bool ext_flushed = false;  // flushed (timeout form)
    Chunk ext_current, ext_expired;
    bool ext_has_reset = false; OEvent ext_reset;
    int64_t key = 0;
    // the partition flow id: String.valueOf of the partition key (ValuePartitionExecutor.execute :34-40)
    std::u16string flow_id;
    bool front_indexed = false;  // (front due time, key) is in Query::fronts
    int64_t indexed_front = 0;
    // the query's output rate limiter: one per partition instance (PartitionRuntime clones the query
    // with its OutputRateLimiter, PartitionRuntimeImpl)
    RateLimiter rl;
    bool rl_init = false;
};

struct Query {
    Schema schema;
    sh_query_desc d{};
    std::vector<sh_filter_op> filter;
    std::vector<AggDef> aggs;
    int vtypes[SH_MAX_AGGS]{};
    bool grouped_states = true;  // PartitionStateHolder vs SingleStateHolder
    bool output_expects_expired = false;
    // playback clock: TimestampGeneratorImpl.lastEventTimestamp (:104-122)
    int64_t clock = INT64_MIN;
    bool clock_set = false;
    // TimeBatchWindowProcessor.nextEmitTime is a processor field shared by all partitions (:128)
    int64_t next_emit_time = -1;
    int64_t ext_timeout = 0;  // externalTimeBatch(ts, T, start, timeout): schedulerTimeout
    bool ext_replace = false;  // externalTimeBatch(ts, T, start, timeout, true): replaceTimestampWithBatchEndTime
    int64_t seq_base = 0;  // stream index of the current push's first event
    std::unordered_map<int64_t, std::unique_ptr<PartitionState>> parts;  // partition flow id -> state
    // Scheduler.stateHolder (PartitionSyncStateHolder -> PartitionStateHolder.states, a
    // HashMap<String, …> keyed by the partition flow id, :36): the partitions whose notify queue is
    // non-empty, in java.util.HashMap order (jhashmap.h); fronts = their due times, to skip calls
    // with nothing due (onTimeChange then puts nothing into its TreeMultimap)
    jhm::HashMap<int64_t> sched_states;
    std::set<std::pair<int64_t, int64_t>> fronts;
    // text of dictionary ids per string column (sh_query_set_strings), UTF-16 as Java holds it
    std::unordered_map<int, std::vector<std::u16string>> strings;
    std::unordered_map<int, std::vector<uint8_t>> has_string;
    OutBuf out;
    RateLimiter rate;

    // the scheduler's tie rule decides output only for partitioned time windows with expired output
    // (and for externalTimeBatch's timeout, whose TIMER calls act on the window)
    bool tie_rule_matters() const {
        return d.partition_col >= 0 &&
               ((d.window == SH_WIN_TIME && d.expired_on) || (d.window == SH_WIN_EXT_TIME_BATCH && ext_timeout > 0));
    }

    // String.valueOf(partition key): Integer/Long/Float/Double.toString, Boolean.toString, the string itself
    std::u16string flow_id_of(int64_t key) const {
        const int c = d.partition_col;
        if (c < 0) return std::u16string();
        switch (schema.types[c]) {
            case SH_T_INT: case SH_T_LONG: return jhm::decimal(key);
            case SH_T_FLOAT: case SH_T_DOUBLE: {  // the key is the value's bits widened to double
                double v; std::memcpy(&v, &key, 8);
                return jhm::fp_decimal(v, schema.types[c] == SH_T_FLOAT);
            }
            case SH_T_BOOL: return key ? u"true" : u"false";
            case SH_T_STRID: {
                auto it = strings.find(c);
                if (it != strings.end() && key >= 0 && key < (int64_t)it->second.size() && has_string.at(c)[(size_t)key])
                    return it->second[(size_t)key];
                break;
            }
            default: break;
        }
        if (tie_rule_matters())
            throw std::runtime_error(schema.types[c] == SH_T_STRID
                                         ? "partition key string id " + std::to_string(key) +
                                               " has no text (sh_query_set_strings): the Scheduler's tie rule needs it"
                                         : "partition key type without a String.valueOf restatement");
        return jhm::decimal(key);  // order irrelevant to the output: any stable text
    }

    PartitionState& part(int64_t key) {
        auto it = parts.find(key);
        if (it != parts.end()) return *it->second;
        auto ps = std::unique_ptr<PartitionState>(new PartitionState());
        ps->agg_states.resize(aggs.size());
        if (d.window == SH_WIN_EXT_TIME_BATCH && d.has_start_time == 1) ps->ext_start = d.start_time;
        ps->key = key;
        ps->flow_id = flow_id_of(key);
        PartitionState& r = *ps;
        parts.emplace(key, std::move(ps));
        return r;
    }

    // Scheduler.notifyAt (core/util/Scheduler.java:113-127): stateHolder.getState() is
    // states.computeIfAbsent(partitionFlowId, …) (PartitionStateHolder.java:46), then the time joins
    // the state's queue; returnState keeps it (the queue is not empty)
    void notify_at(PartitionState& ps, int64_t t) {
        sched_states.compute_if_absent(ps.flow_id, ps.key);
        ps.notify_queue.push_back(t);
        index_front(ps);
    }
    void index_front(PartitionState& ps) {
        if (ps.front_indexed) fronts.erase({ps.indexed_front, ps.key});
        ps.front_indexed = !ps.notify_queue.empty();
        if (ps.front_indexed) fronts.insert({ps.indexed_front = ps.notify_queue.front(), ps.key});
    }

    // ---- selector: QuerySelector.processInBatchGroupBy (core/query/selector/QuerySelector.java:315-374)
    // one selector output chunk -> the partition's rate limiter -> one flush (if it sends anything)
    void close_chunk(PartitionState& ps, size_t start) {
        if (rate.kind == SH_RATE_NONE) { out.close_flush(clock); return; }
        if (!ps.rl_init) { ps.rl = rate; ps.rl_init = true; }
        std::vector<OutRow> chunk(out.rows.begin() + (int64_t)start, out.rows.end()), kept;
        out.rows.resize(start);
        ps.rl.process(chunk.data(), (int64_t)chunk.size(), kept, clock);
        if (kept.empty()) return;
        out.rows.insert(out.rows.end(), kept.begin(), kept.end());
        out.close_flush(clock);
    }

    void selector(PartitionState& ps, const Chunk& chunk) {
        const size_t start = out.rows.size();
        if (aggs.empty() && d.n_group_by == 0) {
            // QuerySelector.processNoGroupBy (:161-205): every qualifying event passes through
            bool any = false;
            for (const OEvent& ev : chunk) {
                if (ev.type != CURRENT && ev.type != EXPIRED) continue;
                bool q = (ev.type == CURRENT && d.current_on) || (ev.type == EXPIRED && d.expired_on);
                if (!q) continue;
                OutRow row{}; row.ts = ev.ts; row.expired = ev.type == EXPIRED; row.rep = ev.seq;
                row.rep_attr = d.window == SH_WIN_EXT_TIME_BATCH ? ev.raw[d.ts_col] : 0;
                out.rows.push_back(row); any = true;
            }
            if (any) close_chunk(ps, start);
            return;
        }
        std::vector<GKey> order;
        std::unordered_map<GKey, OutRow, GKeyHash> grouped;
        for (const OEvent& ev : chunk) {
            if (ev.type == CURRENT || ev.type == EXPIRED) {
                GKey key;
                for (int g = 0; g < d.n_group_by; g++) key.k[g] = key_raw(schema, ev, d.group_by[g]);
                OutRow row{};
                row.ts = ev.ts; row.expired = ev.type == EXPIRED; row.rep = ev.seq;
                row.rep_attr = d.window == SH_WIN_EXT_TIME_BATCH ? ev.raw[d.ts_col] : 0;
                for (int g = 0; g < d.n_group_by; g++) row.keys[g] = key.k[g];
                for (size_t a = 0; a < aggs.size(); a++) {
                    auto& states = ps.agg_states[a];
                    // AttributeAggregatorExecutor.processAdd/processRemove: getState -> op -> returnState
                    auto it = states.find(key);
                    if (it == states.end()) it = states.emplace(key, make_state(aggs[a])).first;
                    JVal v;
                    if (aggs[a].fn != SH_AGG_COUNT) v = schema.get(ev, aggs[a].col);
                    AggOut o = (ev.type == CURRENT) ? it->second->add(v) : it->second->remove(v);
                    if (grouped_states && it->second->can_destroy()) states.erase(it);
                    row.nulls[a] = o.has ? 0 : 1;
                    if (o.has) {
                        if (is_fp(aggs[a].out_type)) std::memcpy(&row.vals[a], &o.d, 8);
                        else row.vals[a] = (uint64_t)o.i;
                    }
                }
                bool qualifies = (ev.type == CURRENT && d.current_on) || (ev.type == EXPIRED && d.expired_on);
                if (qualifies) {
                    auto it = grouped.find(key);
                    if (it == grouped.end()) { order.push_back(key); grouped.emplace(key, row); }
                    else it->second = row;  // LinkedHashMap.put keeps the first-insertion position
                }
            } else if (ev.type == RESET) {
                // AttributeAggregatorExecutor.processReset -> stateHolder.cleanGroupByStates()
                for (auto& st : ps.agg_states) st.clear();
            }
            // TIMER: ignored (:344-345)
        }
        if (!order.empty()) {
            for (const GKey& k : order) out.rows.push_back(grouped[k]);
            close_chunk(ps, start);
        }
    }

    // ---- windows ------------------------------------------------------------------------
    // LengthBatchWindowProcessor.process (:153-187) with processFullBatchEvents (:206-243) and
    // processStreamCurrentEvents (:245-274). Each completed batch is its own downstream chunk.
    void length_batch(PartitionState& ps, Chunk& in) {
        std::vector<Chunk> outs;
        Chunk cur;
        int64_t length = d.window_param;
        int64_t now = clock;
        for (OEvent& ev : in) {
            if (length == 0) {
                // processLengthZeroBatch (:189-204)
                cur.push_back(ev);
                if (output_expects_expired) { OEvent x = ev; x.type = EXPIRED; x.ts = now; cur.push_back(x); }
                OEvent r = ev; r.type = RESET; r.ts = now; cur.push_back(r);
            } else {
                if (!ps.has_reset) { ps.reset_event = ev; ps.reset_event.type = RESET; ps.has_reset = true; }
                if (d.stream_current) {
                    ps.count++;
                    if (ps.count == length + 1) {
                        if (output_expects_expired && !ps.expired_queue.empty()) {
                            for (auto& x : ps.expired_queue) { x.ts = now; cur.push_back(x); }
                            ps.expired_queue.clear();
                        }
                        if (ps.has_reset) { ps.reset_event.ts = now; cur.push_back(ps.reset_event); ps.has_reset = false; }
                        ps.count = 1;
                    }
                    cur.push_back(ev);
                    if (output_expects_expired) { OEvent x = ev; x.type = EXPIRED; ps.expired_queue.push_back(x); }
                } else {
                    ps.current_queue.push_back(ev);
                    ps.count++;
                    if (ps.count == length) {
                        if (output_expects_expired && !ps.expired_queue.empty()) {
                            for (auto& x : ps.expired_queue) { x.ts = now; cur.push_back(x); }
                            ps.expired_queue.clear();
                        }
                        if (ps.has_reset) { ps.reset_event.ts = now; cur.push_back(ps.reset_event); ps.has_reset = false; }
                        if (!ps.current_queue.empty()) {
                            if (output_expects_expired)
                                for (auto& c : ps.current_queue) { OEvent x = c; x.type = EXPIRED; ps.expired_queue.push_back(x); }
                            for (auto& c : ps.current_queue) cur.push_back(c);
                            ps.current_queue.clear();
                        }
                        ps.count = 0;
                    }
                }
            }
            if (!cur.empty()) { outs.push_back(std::move(cur)); cur = Chunk(); }
        }
        for (auto& c : outs) selector(ps, c);
    }

    // TimeBatchWindowProcessor.process (:262-340); getNextEmitTime (:342-347).
    void time_batch(PartitionState& ps, Chunk& in) {
        int64_t T = d.window_param;
        if (next_emit_time == -1) {
            if (d.has_start_time) {
                int64_t elapsed = (clock - d.start_time) % T;  // Java % truncates like C++
                next_emit_time = clock + (T - elapsed);
            } else {
                next_emit_time = clock + T;
            }
            notify_at(ps, next_emit_time);
        }
        bool send = false;
        if (clock >= next_emit_time) { next_emit_time += T; notify_at(ps, next_emit_time); send = true; }
        Chunk outc;
        for (OEvent& ev : in) {
            if (ev.type != CURRENT) continue;
            if (!ps.has_reset) { ps.reset_event = ev; ps.reset_event.type = RESET; ps.has_reset = true; }
            if (!d.stream_current) ps.current_queue.push_back(ev);
            else if (output_expects_expired) { OEvent x = ev; x.type = EXPIRED; ps.expired_queue.push_back(x); }
        }
        if (!d.stream_current) in.clear();
        else { Chunk kept; for (auto& e : in) if (e.type != TIMER) kept.push_back(e); in.swap(kept); }
        // when streamCurrent, the incoming CURRENT events stay in the chunk ahead of the flush
        outc = in;
        if (send) {
            if (output_expects_expired && !ps.expired_queue.empty()) {
                for (auto& x : ps.expired_queue) { x.ts = clock; outc.push_back(x); }
                ps.expired_queue.clear();
            }
            if (ps.has_reset) { outc.push_back(ps.reset_event); ps.has_reset = false; }
            if (!ps.current_queue.empty()) {
                if (output_expects_expired)
                    for (auto& c : ps.current_queue) { OEvent x = c; x.type = EXPIRED; ps.expired_queue.push_back(x); }
                for (auto& c : ps.current_queue) outc.push_back(c);
                ps.current_queue.clear();
            }
        }
        if (!outc.empty()) selector(ps, outc);
    }

    // TimeWindowProcessor.process (:132-169)
    void time_window(PartitionState& ps, Chunk& in) {
        int64_t T = d.window_param;
        Chunk outc;
        for (OEvent& ev : in) {
            int64_t now = clock;
            while (!ps.time_queue.empty()) {
                OEvent& x = ps.time_queue.front();
                if (x.ts - now + T <= 0) {
                    OEvent e2 = x; e2.ts = now; e2.type = EXPIRED;
                    ps.time_queue.pop_front();
                    outc.push_back(e2);  // insertBeforeCurrent
                } else break;
            }
            if (ev.type == CURRENT) {
                OEvent c = ev; c.type = EXPIRED;
                ps.time_queue.push_back(c);
                if (ps.last_timestamp < c.ts) { notify_at(ps, c.ts + T); ps.last_timestamp = c.ts; }
                outc.push_back(ev);
            }
            // TIMER and others removed from the chunk
        }
        selector(ps, outc);
    }

    // ExternalTimeWindowProcessor.process (:126-161): sliding over the attribute ts_col; each event
    // expires the queue head while expiredTime - currentTime + timeToKeep <= 0 (currentTime = the
    // event's attribute, not the playback clock), expired events re-stamped with currentTime
    void ext_time_window(PartitionState& ps, Chunk& in) {
        const int64_t T = d.window_param;
        Chunk outc;
        for (OEvent& ev : in) {
            const int64_t now = ext_attr(ev, d.ts_col);
            while (!ps.time_queue.empty()) {
                OEvent& x = ps.time_queue.front();
                if (ext_attr(x, d.ts_col) - now + T <= 0) {
                    OEvent e2 = x; e2.ts = now; e2.type = EXPIRED;
                    ps.time_queue.pop_front();
                    outc.push_back(e2);  // insertBeforeCurrent
                } else break;
            }
            if (ev.type == CURRENT) {
                OEvent c = ev; c.type = EXPIRED;
                ps.time_queue.push_back(c);
                outc.push_back(ev);
            }
        }
        selector(ps, outc);
    }

    // ExternalTimeBatchWindowProcessor.process (:238-311) without a timeout (no TIMER events reach it):
    // initTiming (:313-334), flushToOutputChunk (:336-383), findEndTime (:440-444), cloneAppend
    // (:446-456). Every batch an event closes is its own downstream chunk, emitted after the whole
    // incoming chunk is consumed (:308-310).
    int64_t ext_attr(const OEvent& e, int col) const { return e.raw[col]; }
    static int64_t find_end_time(int64_t current, int64_t start, int64_t T) {
        int64_t elapsed = (current - start) % T;  // Java % truncates like C++
        return current + (T - elapsed);
    }
    // the expired chunk exists when expired events are output or a timeout is set (WindowState :507-517)
    bool ext_keeps_expired() const { return output_expects_expired || ext_timeout > 0; }
    void ext_flush(PartitionState& ps, std::vector<Chunk>& outs, int64_t current_time) {
        Chunk c;
        if (output_expects_expired && !ps.ext_expired.empty()) {
            for (auto& x : ps.ext_expired) { x.ts = current_time; c.push_back(x); }
        }
        ps.ext_expired.clear();
        if (!ps.ext_current.empty()) {
            ps.ext_reset.ts = current_time;
            c.push_back(ps.ext_reset);
            ps.ext_has_reset = false;
            if (ext_keeps_expired())
                for (auto& e : ps.ext_current) { OEvent x = e; x.type = EXPIRED; ps.ext_expired.push_back(x); }
            for (auto& e : ps.ext_current) c.push_back(e);
        }
        ps.ext_current.clear();
        if (!c.empty()) outs.push_back(std::move(c));
    }
    // appendToOutputChunk (:385-438): after a timeout flush the batch goes out again, whole — its
    // flushed part re-sent as CURRENT behind a RESET (expired copies first when expired events are
    // output), then the new events; the expired chunk keeps growing until the batch's real flush
    void ext_append(PartitionState& ps, std::vector<Chunk>& outs, int64_t current_time) {
        if (ps.ext_current.empty()) return;
        Chunk c, sent;
        for (const auto& x : ps.ext_expired) {
            if (output_expects_expired) { OEvent e = x; e.ts = current_time; c.push_back(e); }
            OEvent s2 = x; s2.type = CURRENT; sent.push_back(s2);
        }
        OEvent r = ps.ext_reset; r.type = RESET; r.ts = current_time;
        c.push_back(r);
        for (auto& e : sent) c.push_back(e);
        for (auto& e : ps.ext_current) { OEvent x = e; x.type = EXPIRED; ps.ext_expired.push_back(x); }
        for (auto& e : ps.ext_current) c.push_back(e);
        ps.ext_current.clear();
        outs.push_back(std::move(c));
    }
    void ext_schedule(PartitionState& ps) {
        ps.ext_sched = clock + ext_timeout;
        notify_at(ps, ps.ext_sched);
    }
    // cloneAppend (:446-456): the window's copy carries endTime in the timestamp attribute when
    // replaceTimestampWithBatchEndTime is set (the RESET event is a copy of the original)
    void ext_append(PartitionState& ps, const OEvent& ev) {
        ps.ext_current.push_back(ev);
        if (ext_replace) ps.ext_current.back().raw[d.ts_col] = ps.ext_end;
        if (!ps.ext_has_reset) { ps.ext_reset = ev; ps.ext_reset.type = RESET; ps.ext_has_reset = true; }
    }
    void ext_time_batch(PartitionState& ps, Chunk& in) {
        if (in.empty()) return;
        const int64_t T = d.window_param;
        if (ps.ext_end < 0 && in.front().type == CURRENT) {
            const OEvent& f = in.front();
            if (d.has_start_time == 1) {
                ps.ext_end = find_end_time(ext_attr(f, d.ts_col), ps.ext_start, T);
            } else if (d.has_start_time == 2) {
                ps.ext_start = ext_attr(f, d.start_col);
                ps.ext_end = ps.ext_start + T;
            } else {
                ps.ext_start = ext_attr(f, d.ts_col);
                ps.ext_end = ps.ext_start + T;
            }
            if (ext_timeout > 0) ext_schedule(ps);  // initTiming :328-332
        }
        std::vector<Chunk> outs;
        for (OEvent& ev : in) {
            if (ev.type == TIMER) {
                // :256-275: the timeout of the last scheduled time flushes the batch so far (once; a
                // later timeout re-sends it whole with its new events), then reschedules
                if (ext_timeout > 0 && ps.ext_sched <= ev.ts) {
                    if (!ps.ext_flushed) {
                        ext_flush(ps, outs, ps.ext_last);
                        ps.ext_flushed = true;
                    } else {
                        ext_append(ps, outs, ps.ext_last);
                    }
                    ext_schedule(ps);
                }
                continue;
            }
            if (ev.type != CURRENT) continue;
            int64_t t = ext_attr(ev, d.ts_col);
            if (ps.ext_last < t) ps.ext_last = t;
            if (t < ps.ext_end) {
                ext_append(ps, ev);
            } else {
                if (ps.ext_flushed) {
                    ext_append(ps, outs, ps.ext_last);
                    ps.ext_flushed = false;
                } else {
                    ext_flush(ps, outs, ps.ext_last);
                }
                ps.ext_end = find_end_time(ps.ext_last, ps.ext_start, T);
                ext_append(ps, ev);
                if (ext_timeout > 0) ext_schedule(ps);
            }
        }
        for (auto& c : outs) selector(ps, c);
    }

    void window(PartitionState& ps, Chunk& c) {
        switch (d.window) {
            case SH_WIN_EXT_TIME_BATCH: ext_time_batch(ps, c); break;
            case SH_WIN_EXT_TIME: ext_time_window(ps, c); break;
            case SH_WIN_NONE: { Chunk k; for (auto& e : c) if (e.type != TIMER) k.push_back(e); if (!k.empty()) selector(ps, k); break; }
            case SH_WIN_LENGTH_BATCH: length_batch(ps, c); break;
            case SH_WIN_TIME_BATCH: time_batch(ps, c); break;
            default: time_window(ps, c); break;
        }
    }

    // Scheduler.onTimeChange (core/util/Scheduler.java:71-104) + sendTimerEvents (:171-209).
    // getAllStates() is walked in HashMap order and every due state is put into a
    // TreeMultimap<Long, SchedulerState> whose values compare equal (:363-366): per distinct due time
    // only the first state put is kept. returnAllStates (PartitionStateHolder.java:132-161) then
    // removes, in iteration order, the states whose queue is empty (canDestroy, :343-346).
    void on_time_change() {
        if (fronts.empty() || fronts.begin()->first > clock) return;
        std::map<int64_t, int64_t> sorted;  // due time -> partition key (first put wins)
        sched_states.for_each([&](const std::u16string&, int64_t key) {
            PartitionState& ps = *parts[key];
            if (!ps.notify_queue.empty() && ps.notify_queue.front() <= clock) sorted.emplace(ps.notify_queue.front(), key);
        });
        for (auto& kv : sorted) {
            PartitionState& ps = *parts[kv.second];
            while (!ps.notify_queue.empty() && ps.notify_queue.front() - clock <= 0) {
                int64_t t = ps.notify_queue.front();
                ps.notify_queue.pop_front();
                OEvent timer; timer.type = TIMER; timer.ts = t;
                Chunk c{timer};
                window(ps, c);  // EntryValveProcessor -> window
            }
            index_front(ps);
        }
        std::vector<std::u16string> gone;
        sched_states.for_each([&](const std::u16string& k, int64_t key) {
            if (parts[key]->notify_queue.empty()) gone.push_back(k);
        });
        for (auto& k : gone) sched_states.remove(k);
    }

    void set_clock(int64_t ts) {
        // TimestampGeneratorImpl.setCurrentTimestamp: only moves forward (>=), then notifies
        if (!clock_set || ts >= clock) {
            clock = ts; clock_set = true;
            on_time_change();
        }
    }

    // InputHandler.send(Event[]) (core/stream/input/InputHandler.java:85-96) ->
    // [PartitionStreamReceiver.receive (core/partition/PartitionStreamReceiver.java:176-213)] ->
    // FilterProcessor -> window.
    void send(const sh_batch* b, int64_t lo, int64_t hi) {
        if (hi <= lo) return;
        set_clock(b->ts[hi - 1]);
        if (d.partition_col < 0) {
            Chunk c;
            c.reserve((size_t)(hi - lo));
            OEvent e;
            for (int64_t i = lo; i < hi; i++) {
                load_event(schema, b, i, e);
                e.seq = seq_base + i;
                if (eval_filter(schema, filter, e)) c.push_back(e);
            }
            if (!c.empty()) window(part(0), c);
        } else {
            // runs of consecutive equal partition keys (ValuePartitionExecutor: expr.toString())
            int64_t i = lo;
            OEvent e;
            while (i < hi) {
                load_event(schema, b, i, e);
                int64_t key = key_raw(schema, e, d.partition_col);
                Chunk c;
                int64_t j = i;
                while (j < hi) {
                    OEvent f; load_event(schema, b, j, f);
                    f.seq = seq_base + j;
                    if (key_raw(schema, f, d.partition_col) != key) break;
                    if (eval_filter(schema, filter, f)) c.push_back(f);
                    j++;
                }
                if (!c.empty()) window(part(key), c);
                else part(key);  // PartitionRuntimeImpl.initPartition
                i = j;
            }
        }
    }
};

// ==========================================================================================
// Incremental aggregation engine
// ==========================================================================================
// GMT civil calendar (IncrementalTimeConverterUtil with ZoneId "GMT").
int64_t days_from_civil(int64_t y, unsigned m, unsigned dd) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const unsigned yoe = (unsigned)(y - era * 400);
    const unsigned doy = (153 * (m + (m > 2 ? -3 : 9)) + 2) / 5 + dd - 1;
    const unsigned doe = yoe * 365 + yoe / 4 - yoe / 100 + doy;
    return era * 146097 + (int64_t)doe - 719468;
}
void civil_from_days(int64_t z, int64_t& y, unsigned& m, unsigned& dd) {
    z += 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const unsigned doe = (unsigned)(z - era * 146097);
    const unsigned yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    y = (int64_t)yoe + era * 400;
    const unsigned doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const unsigned mp = (5 * doy + 2) / 153;
    dd = doy - (153 * mp + 2) / 5 + 1;
    m = mp + (mp < 10 ? 3 : -9);
    y += (m <= 2);
}
int64_t floor_div(int64_t a, int64_t b) { int64_t q = a / b; if ((a % b != 0) && ((a < 0) != (b < 0))) q--; return q; }

// ZonedDateTime.of(y, m, d, h, 0, 0, 0, GMT).toEpochSecond() * 1000
int64_t epoch_ms(int64_t y, int64_t m, int64_t dd, int64_t h) {
    return (days_from_civil(y, (unsigned)m, (unsigned)dd) * 86400 + h * 3600) * 1000;
}
struct Civil { int64_t y; unsigned m, d; int64_t h; };
Civil civil(int64_t ms) {
    int64_t days = floor_div(ms, 86400000);
    int64_t rem = ms - days * 86400000;
    Civil c; civil_from_days(days, c.y, c.m, c.d); c.h = rem / 3600000; return c;
}
// Month.length(leapYear) with the reference's `year % 4 == 0` leap test
int month_len(unsigned m, bool leap) {
    static const int L[13] = {0, 31, 28, 31, 30, 31, 30, 31, 31, 30, 31, 30, 31};
    return (m == 2 && leap) ? 29 : L[m];
}

// IncrementalTimeConverterUtil.getStartTimeOfAggregates (:52-69)
int64_t start_time_of(int64_t t, int dur) {
    switch (dur) {
        case SH_DUR_SECONDS: return t - t % 1000;
        case SH_DUR_MINUTES: return t - t % 60000;
        case SH_DUR_HOURS: { Civil c = civil(t); return epoch_ms(c.y, c.m, c.d, c.h); }
        case SH_DUR_DAYS: { Civil c = civil(t); return epoch_ms(c.y, c.m, c.d, 0); }
        case SH_DUR_MONTHS: { Civil c = civil(t); return epoch_ms(c.y, c.m, 1, 0); }
        default: { Civil c = civil(t); return epoch_ms(c.y, 1, 1, 0); }
    }
}
// IncrementalTimeConverterUtil.getNextEmitTime (:33-50) and the per-duration helpers (:89-160)
int64_t next_emit_of(int64_t t, int dur) {
    switch (dur) {
        case SH_DUR_SECONDS: return t - t % 1000 + 1000;
        case SH_DUR_MINUTES: return t - t % 60000 + 60000;
        case SH_DUR_HOURS: {
            Civil c = civil(t);
            if (c.h == 23) {
                if ((int)c.d + 1 > month_len(c.m, c.y % 4 == 0)) {
                    if (c.m == 12) return epoch_ms(c.y + 1, 1, 1, 0);
                    return epoch_ms(c.y, c.m + 1, 1, 0);
                }
                return epoch_ms(c.y, c.m, c.d + 1, 0);
            }
            return epoch_ms(c.y, c.m, c.d, c.h + 1);
        }
        case SH_DUR_DAYS: {
            Civil c = civil(t);
            if ((int)c.d + 1 > month_len(c.m, c.y % 4 == 0)) {
                if (c.m == 12) return epoch_ms(c.y + 1, 1, 1, 0);
                return epoch_ms(c.y, c.m + 1, 1, 0);
            }
            return epoch_ms(c.y, c.m, c.d + 1, 0);
        }
        case SH_DUR_MONTHS: {
            Civil c = civil(t);
            if (c.m == 12) return epoch_ms(c.y + 1, 1, 1, 0);
            return epoch_ms(c.y, c.m + 1, 1, 0);
        }
        default: { Civil c = civil(t); return epoch_ms(c.y + 1, 1, 1, 0); }
    }
}

// Base value kinds (AggregationParser.populateFinalBaseAggregators :693-728).
enum BaseKind { B_SUM = 0, B_COUNT = 1, B_MIN = 2, B_MAX = 3 };
struct BaseDef { int kind; int col; int type; };  // type: LONG or DOUBLE for sums, input type for min/max

// One row of a duration's value store: BaseIncrementalValueStore.ValueState.values, where each
// base executor is sum()/min()/max() in BATCH mode over the per-key rows.
struct BaseRow {
    int64_t ext = 0;  // AGG_EXTERNAL_TIMESTAMP bucket at this duration (or 0)
    int64_t keys[SH_MAX_GROUP] = {};
    std::vector<std::unique_ptr<AggState>> st;  // per base value
    std::vector<AggOut> val;                    // last value returned by each executor
};

struct AggRuntime;

// IncrementalExecutor (core/aggregation/IncrementalExecutor.java)
struct IncExec {
    int dur;
    bool root;
    IncExec* next = nullptr;
    int64_t next_emit_time = -1;        // ExecutorState.nextEmitTime
    int64_t start_time_of_aggs = -1;    // ExecutorState.startTimeOfAggregates
    bool timer_started = false;
    int64_t store_ts = -1;              // BaseIncrementalValueStore StoreState.timestamp
    bool processed = false;             // StoreState.isProcessed
    std::vector<GKey> order;            // insertion order (the reference's HashMap order differs)
    std::unordered_map<GKey, BaseRow, GKeyHash> store;
    AggRuntime* rt = nullptr;
};

struct InRow {  // an event or a dispatched row entering an executor
    int type;           // CURRENT or TIMER
    int64_t ts;         // AGG_TIMESTAMP (row) / event timestamp (TIMER)
    int64_t ext;        // external timestamp (raw event ts at root; bucket at children)
    int64_t keys[SH_MAX_GROUP];
    std::vector<JVal> base;  // base values (root: initial values; child: parent's outputs)
};

struct AggRuntime {
    Schema schema;
    sh_aggregation_desc d{};
    std::vector<sh_filter_op> filter;
    std::vector<BaseDef> bases;
    std::vector<std::unique_ptr<IncExec>> execs;
    int64_t clock = INT64_MIN; bool clock_set = false;
    std::deque<int64_t> notify_queue;  // root scheduler (AggregationParser.java:431-437)
    // table rows per duration, appended on dispatch; `history` keeps every row (retrieval)
    std::vector<std::vector<OutRow>> tables, history;
    std::vector<OutBuf> views;
    int vtypes[SH_MAX_AGGS]{};
    // aggTimeZone (IncrementalTimeConverterUtil.java:33-231 with a ZoneId): a fixed offset from GMT here,
    // hour / day / month / year buckets starting at the zone's local boundaries
    int64_t zst(int64_t t, int dur) const {
        return dur >= SH_DUR_HOURS ? start_time_of(t + d.tz_offset_ms, dur) - d.tz_offset_ms : start_time_of(t, dur);
    }
    int64_t zne(int64_t t, int dur) const {
        return dur >= SH_DUR_HOURS ? next_emit_of(t + d.tz_offset_ms, dur) - d.tz_offset_ms : next_emit_of(t, dur);
    }

    int base_out_type(const BaseDef& b) const {
        if (b.kind == B_COUNT) return SH_T_LONG;
        if (b.kind == B_SUM) return b.type;
        return b.type;
    }

    // IncrementalExecutor.execute (:110-139)
    void execute(IncExec& ex, std::vector<InRow>& chunk) {
        for (InRow& r : chunk) {
            int64_t timestamp;
            // getTimestamp (:152-169)
            if (r.type == CURRENT) {
                timestamp = r.ts;
                if (ex.root && !ex.timer_started) { notify_queue.push_back(zne(timestamp, ex.dur)); ex.timer_started = true; }
            } else {
                timestamp = r.ts;
                if (ex.root) notify_queue.push_back(zne(timestamp, ex.dur));
            }
            ex.start_time_of_aggs = zst(timestamp, ex.dur);
            if (timestamp >= ex.next_emit_time) {
                ex.next_emit_time = zne(timestamp, ex.dur);
                dispatch(ex, ex.start_time_of_aggs);
                // sendTimerEvent (:141-150)
                if (ex.next) {
                    InRow t{}; t.type = TIMER; t.ts = ex.start_time_of_aggs;
                    std::vector<InRow> tc{t};
                    execute(*ex.next, tc);
                }
            }
            if (r.type == CURRENT) process_aggregates(ex, r);
        }
    }

    // processAggregates (:183-198) -> BaseIncrementalValueStore.process (:141-160)
    void process_aggregates(IncExec& ex, const InRow& r) {
        GKey key;
        int off = 0;
        if (d.ts_col >= 0) key.k[off++] = zst(r.ext, ex.dur);  // getAggregationStartTime
        for (int g = 0; g < d.n_group_by; g++) key.k[off + g] = r.keys[g];
        auto it = ex.store.find(key);
        if (it == ex.store.end()) {
            BaseRow br;
            br.ext = d.ts_col >= 0 ? key.k[0] : 0;
            for (int g = 0; g < d.n_group_by; g++) br.keys[g] = r.keys[g];
            for (auto& b : bases) {
                AggDef ad;
                ad.fn = b.kind == B_SUM || b.kind == B_COUNT ? SH_AGG_SUM : (b.kind == B_MIN ? SH_AGG_MIN : SH_AGG_MAX);
                ad.in_type = b.kind == B_COUNT ? SH_T_LONG : b.type;
                ad.track = false; ad.col = 0; ad.out_type = 0;
                br.st.push_back(make_state(ad));
                br.val.push_back(AggOut());
            }
            it = ex.store.emplace(key, std::move(br)).first;
            ex.order.push_back(key);
        }
        for (size_t i = 0; i < bases.size(); i++) it->second.val[i] = it->second.st[i]->add(r.base[i]);
        ex.processed = true;
    }

    // dispatchEvent (:201-258) + cleanBaseIncrementalValueStore (:260-266)
    void dispatch(IncExec& ex, int64_t start_of_new) {
        if (ex.processed) {
            std::vector<InRow> rows;
            for (const GKey& k : ex.order) {
                BaseRow& br = ex.store[k];
                // getGroupedByEvents (:118-138): row timestamp = store timestamp
                InRow ir{}; ir.type = CURRENT; ir.ts = ex.store_ts; ir.ext = br.ext;
                for (int g = 0; g < d.n_group_by; g++) ir.keys[g] = br.keys[g];
                for (size_t i = 0; i < bases.size(); i++) {
                    JVal v; v.t = base_out_type(bases[i]);
                    const AggOut& o = br.val[i];
                    if (!o.has) v.t = 0; else if (is_fp(v.t)) v.d = o.d; else v.i = o.i;
                    ir.base.push_back(v);
                }
                record_table_row(ex.dur, ex.store_ts, br);
                rows.push_back(std::move(ir));
            }
            if (ex.next) execute(*ex.next, rows);
        }
        // BaseIncrementalValueStore.clearValues (:73-78)
        ex.store_ts = start_of_new;
        ex.processed = false;
        ex.store.clear(); ex.order.clear();
    }

    // table.addEvents of the dispatched rows. keys = [AGG_TIMESTAMP bucket, group-by value]; the
    // bucket is the event-time bucket (AGG_EXTERNAL_TIMESTAMP) when `aggregate by` is used.
    void record_table_row(int dur, int64_t store_ts, const BaseRow& br) {
        OutRow r{};
        r.ts = d.ts_col >= 0 ? br.ext : store_ts;
        r.keys[0] = r.ts;
        for (int g = 0; g < d.n_group_by; g++) r.keys[1 + g] = br.keys[g];
        for (size_t i = 0; i < bases.size(); i++) {
            const AggOut& o = br.val[i];
            r.nulls[i] = o.has ? 0 : 1;
            if (o.has) { if (is_fp(base_out_type(bases[i]))) std::memcpy(&r.vals[i], &o.d, 8); else r.vals[i] = (uint64_t)o.i; }
        }
        tables[dur].push_back(r);
        history[dur].push_back(r);
    }

    // Retrieval `from A within start, end per "<per>"`: AggregationRuntime.find ->
    // IncrementalAggregateCompileCondition.find (:180-290). The in-memory stores of the executors
    // per .. root are re-bucketed to `per` and folded per (bucket, key) in executor order
    // (IncrementalDataAggregator.aggregateInMemoryData :92-143), then merged with the `per` table's
    // rows by (AGG_TIMESTAMP, key), table rows first (OutOfOrderEventsDataAggregator), restricted to
    // start <= AGG_TIMESTAMP < end. Output order: (AGG_TIMESTAMP, key) (the reference's is a HashMap's).
    struct Acc { std::vector<std::unique_ptr<AggState>> st; std::vector<AggOut> val; };
    Acc new_acc() const {
        Acc a;
        for (auto& b : bases) {
            AggDef ad;
            ad.fn = b.kind == B_SUM || b.kind == B_COUNT ? SH_AGG_SUM : (b.kind == B_MIN ? SH_AGG_MIN : SH_AGG_MAX);
            ad.in_type = b.kind == B_COUNT ? SH_T_LONG : b.type;
            ad.track = false; ad.col = 0; ad.out_type = 0;
            a.st.push_back(make_state(ad));
            a.val.push_back(AggOut());
        }
        return a;
    }
    JVal as_jval(size_t i, const AggOut& o) const {
        JVal v; v.t = base_out_type(bases[i]);
        if (is_fp(v.t)) v.d = o.d; else v.i = o.i;
        return v;
    }
    void fold(Acc& a, const std::vector<AggOut>& vals) const {
        for (size_t i = 0; i < bases.size(); i++) if (vals[i].has) a.val[i] = a.st[i]->add(as_jval(i, vals[i]));
    }
    void find(int per, int64_t start, int64_t end, OutBuf& ob) {
        typedef std::array<int64_t, 1 + SH_MAX_GROUP> GK;  // (bucket, group-by values)
        std::map<GK, Acc> mem;
        const int ip = per - d.min_duration;
        for (int k = ip; k >= 0; k--) {
            IncExec& ex = *execs[k];
            for (const GKey& key : ex.order) {
                const BaseRow& br = ex.store[key];
                const int64_t b = zst(d.ts_col >= 0 ? br.ext : ex.store_ts, per);
                GK g{};
                g[0] = b;
                for (int x = 0; x < d.n_group_by; x++) g[1 + x] = br.keys[x];
                auto it = mem.find(g);
                if (it == mem.end()) it = mem.emplace(g, new_acc()).first;
                fold(it->second, br.val);
            }
        }
        std::map<GK, Acc> res;
        for (const OutRow& r : history[per]) {
            if (r.ts < start || r.ts >= end) continue;
            GK g{};
            g[0] = r.ts;
            for (int x = 0; x < d.n_group_by; x++) g[1 + x] = r.keys[1 + x];
            auto it = res.find(g);
            if (it == res.end()) it = res.emplace(g, new_acc()).first;
            std::vector<AggOut> v(bases.size());
            for (size_t i = 0; i < bases.size(); i++) {
                v[i].has = !r.nulls[i];
                if (is_fp(base_out_type(bases[i]))) std::memcpy(&v[i].d, &r.vals[i], 8); else v[i].i = (int64_t)r.vals[i];
            }
            fold(it->second, v);
        }
        for (auto& m : mem) {
            if (m.first[0] < start || m.first[0] >= end) continue;
            auto it = res.find(m.first);
            if (it == res.end()) it = res.emplace(m.first, new_acc()).first;
            fold(it->second, m.second.val);
        }
        ob.clear();
        ob.with_rep = false;
        for (auto& kv : res) {
            OutRow r{};
            r.ts = kv.first[0];
            for (int x = 0; x <= d.n_group_by; x++) r.keys[x] = kv.first[x];
            for (size_t i = 0; i < bases.size(); i++) {
                const AggOut& o = kv.second.val[i];
                r.nulls[i] = o.has ? 0 : 1;
                if (o.has) { if (is_fp(base_out_type(bases[i]))) std::memcpy(&r.vals[i], &o.d, 8); else r.vals[i] = (uint64_t)o.i; }
            }
            ob.rows.push_back(r);
        }
        if (!ob.rows.empty()) ob.close_flush(clock);
    }

    void on_time_change() {
        IncExec& root = *execs[0];
        while (!notify_queue.empty() && notify_queue.front() - clock <= 0) {
            int64_t t = notify_queue.front(); notify_queue.pop_front();
            InRow tr{}; tr.type = TIMER; tr.ts = t;
            std::vector<InRow> c{tr};
            execute(root, c);
        }
    }
    void set_clock(int64_t ts) {
        if (!clock_set || ts >= clock) { clock = ts; clock_set = true; on_time_change(); }
    }

    // InputHandler.send -> IncrementalAggregationProcessor.process (:66-101): per event
    // AGG_TIMESTAMP = currentTimeMillis() = playback clock; [ext ts]; group-by; base initial values
    // (convert(v,'double'|'long'), 1L for count, v for min/max).
    void send(const sh_batch* b, int64_t lo, int64_t hi) {
        if (hi <= lo) return;
        set_clock(b->ts[hi - 1]);
        std::vector<InRow> chunk;
        OEvent e;
        for (int64_t i = lo; i < hi; i++) {
            load_event(schema, b, i, e);
            if (!eval_filter(schema, filter, e)) continue;
            InRow r{};
            r.type = CURRENT; r.ts = clock;
            r.ext = d.ts_col >= 0 ? schema.get(e, d.ts_col).i : 0;
            for (int g = 0; g < d.n_group_by; g++) r.keys[g] = key_raw(schema, e, d.group_by[g]);
            for (auto& bd : bases) {
                JVal v;
                if (bd.kind == B_COUNT) { v.t = SH_T_LONG; v.i = 1; }
                else {
                    JVal x = schema.get(e, bd.col);
                    if (bd.kind == B_SUM) {
                        v.t = bd.type;
                        if (bd.type == SH_T_DOUBLE) v.d = is_fp(x.t) ? x.d : (double)x.i;
                        else v.i = x.i;
                    } else v = x;
                }
                r.base.push_back(v);
            }
            chunk.push_back(std::move(r));
        }
        if (!chunk.empty()) execute(*execs[0], chunk);
    }
};

}  // namespace

// ==========================================================================================
// C API (oracle.h)
// ==========================================================================================
extern "C" {

const char* or_last_error(void) { return g_err.c_str(); }

void* or_query_create(const sh_query_desc* desc) {
    if (!desc || desc->n_cols <= 0 || desc->n_cols > SH_MAX_COLS || desc->n_aggs < 0 ||
        desc->n_aggs > SH_MAX_AGGS || desc->n_group_by < 0 || desc->n_group_by > SH_MAX_GROUP) {
        g_err = "invalid descriptor"; return nullptr;
    }
    if (desc->window < SH_WIN_NONE || desc->window > SH_WIN_EXT_TIME) { g_err = "bad window"; return nullptr; }
    // ExternalTimeWindowProcessor.init (:108-116): the timestamp must be a LONG attribute
    if ((desc->window == SH_WIN_EXT_TIME || desc->window == SH_WIN_EXT_TIME_BATCH) &&
        (desc->ts_col < 0 || desc->ts_col >= desc->n_cols || desc->col_types[desc->ts_col] != SH_T_LONG)) {
        g_err = "external time windows need a long timestamp attribute";
        return nullptr;
    }
    Query* q = new Query();
    q->d = *desc;
    q->schema.n = desc->n_cols;
    for (int c = 0; c < desc->n_cols; c++) q->schema.types[c] = desc->col_types[c];
    if (desc->n_filter_ops > 0) q->filter.assign(desc->filter, desc->filter + desc->n_filter_ops);
    q->output_expects_expired = desc->expired_on != 0;
    // ProcessingMode: time window -> SLIDE; batch windows -> BATCH (RESET if streamCurrent)
    bool slide = desc->window == SH_WIN_TIME || desc->window == SH_WIN_EXT_TIME;
    for (int a = 0; a < desc->n_aggs; a++) {
        AggDef ad;
        ad.fn = desc->aggs[a].fn; ad.col = desc->aggs[a].col;
        ad.in_type = ad.fn == SH_AGG_COUNT ? SH_T_LONG : desc->col_types[ad.col];
        if (ad.in_type == SH_T_STRID || ad.in_type == SH_T_BOOL) ad.in_type = SH_T_INT;
        ad.out_type = agg_out_type(ad.fn, ad.in_type);
        ad.track = slide || q->output_expects_expired;
        q->aggs.push_back(ad);
        q->vtypes[a] = ad.out_type;
    }
    q->grouped_states = desc->n_group_by > 0 || desc->partition_col >= 0;
    return q;
}

void or_query_destroy(void* h) { delete (Query*)h; }

int or_query_set_strings(void* h, int32_t col, int64_t first_id, int64_t n, const uint16_t* units,
                         const int64_t* offsets) {
    Query* q = (Query*)h;
    if (col < 0 || col >= q->d.n_cols || q->d.col_types[col] != SH_T_STRID || first_id < 0 || n < 0 ||
        (n > 0 && (!units || !offsets))) {
        g_err = "sh_query_set_strings: bad column or range";
        return SH_ERR_INVALID;
    }
    auto& v = q->strings[col];
    auto& has = q->has_string[col];
    if ((int64_t)v.size() < first_id + n) { v.resize((size_t)(first_id + n)); has.resize((size_t)(first_id + n), 0); }
    for (int64_t i = 0; i < n; i++) {
        if (offsets[i + 1] < offsets[i]) { g_err = "sh_query_set_strings: offsets decrease"; return SH_ERR_INVALID; }
        v[(size_t)(first_id + i)].assign((const char16_t*)units + offsets[i], (const char16_t*)units + offsets[i + 1]);
        has[(size_t)(first_id + i)] = 1;
    }
    return SH_OK;
}

// externalTimeBatch's 4th parameter (ExternalTimeBatchWindowProcessor :196-207): scheduler timeout (ms)
int or_query_set_ext_timeout(void* h, int64_t ms) {
    Query* q = (Query*)h;
    if (q->d.window != SH_WIN_EXT_TIME_BATCH || ms < 0) {
        g_err = "a timeout needs an externalTimeBatch window and >= 0 ms";
        return SH_ERR_INVALID;
    }
    q->ext_timeout = ms;
    return SH_OK;
}

// externalTimeBatch's 5th parameter (ExternalTimeBatchWindowProcessor :210-220): replaceTimestampWithBatchEndTime
int or_query_set_ext_replace_ts(void* h, int32_t on) {
    Query* q = (Query*)h;
    if (q->d.window != SH_WIN_EXT_TIME_BATCH) {
        g_err = "replaceTimestampWithBatchEndTime needs an externalTimeBatch window";
        return SH_ERR_INVALID;
    }
    q->ext_replace = on != 0;
    return SH_OK;
}

// the timestamp attribute of every row's representative event in the last output (the batch end time
// under replaceTimestampWithBatchEndTime)
int or_query_rep_ts_attr(void* h, const int64_t** values, int64_t* n) {
    Query* q = (Query*)h;
    *values = q->out.rep_attr.data();
    *n = (int64_t)q->out.rep_attr.size();
    return SH_OK;
}

int or_query_set_output_rate(void* h, int32_t kind, int64_t n) {
    Query* q = (Query*)h;
    if (kind < SH_RATE_NONE || kind > SH_RATE_FIRST_TIME || (kind != SH_RATE_NONE && n < (kind == SH_RATE_FIRST_TIME ? 0 : 1))) {
        g_err = "invalid output rate";
        return SH_ERR_INVALID;
    }
    q->rate = RateLimiter{};
    q->rate.kind = kind;
    q->rate.value = n;
    q->rate.group_by = q->d.n_group_by > 0;
    q->rate.nk = q->d.n_group_by;
    return SH_OK;
}

int or_push(void* h, const sh_batch* b, const sh_out** out) {
    Query* q = (Query*)h;
    q->out.clear();
    int64_t step = b->send_size > 0 ? b->send_size : b->n;
    try {
        for (int64_t lo = 0; lo < b->n; lo += step) q->send(b, lo, std::min(b->n, lo + step));
    } catch (const std::exception& e) {
        g_err = e.what();
        return SH_ERR_INVALID;
    }
    q->seq_base += b->n;
    *out = q->out.view(q->d.n_group_by, (int)q->aggs.size(), q->vtypes);
    return SH_OK;
}

int or_advance_time(void* h, int64_t now, const sh_out** out) {
    Query* q = (Query*)h;
    q->out.clear();
    try {
        q->set_clock(now);
    } catch (const std::exception& e) {
        g_err = e.what();
        return SH_ERR_INVALID;
    }
    *out = q->out.view(q->d.n_group_by, (int)q->aggs.size(), q->vtypes);
    return SH_OK;
}

void* or_aggregation_create(const sh_aggregation_desc* desc) {
    if (!desc || desc->n_cols <= 0 || desc->n_cols > SH_MAX_COLS || desc->min_duration < 0 ||
        desc->max_duration > SH_DUR_YEARS || desc->min_duration > desc->max_duration ||
        desc->n_group_by < 0 || desc->n_group_by > SH_MAX_GROUP || desc->n_aggs <= 0 || desc->n_aggs > SH_MAX_AGGS) {
        g_err = "invalid aggregation descriptor"; return nullptr;
    }
    AggRuntime* a = new AggRuntime();
    a->d = *desc;
    a->schema.n = desc->n_cols;
    for (int c = 0; c < desc->n_cols; c++) a->schema.types[c] = desc->col_types[c];
    if (desc->n_filter_ops > 0) a->filter.assign(desc->filter, desc->filter + desc->n_filter_ops);
    // base attributes, de-duplicated by (kind, col) as finalBaseAttributes.contains does
    auto add_base = [&](int kind, int col) {
        int t = kind == B_COUNT ? SH_T_LONG : desc->col_types[col];
        if (kind == B_SUM) t = is_fp(t) ? SH_T_DOUBLE : SH_T_LONG;
        if (kind != B_SUM && kind != B_COUNT && (t == SH_T_STRID || t == SH_T_BOOL)) t = SH_T_INT;
        for (auto& b : a->bases) if (b.kind == kind && (kind == B_COUNT || b.col == col)) return;
        a->bases.push_back(BaseDef{kind, kind == B_COUNT ? -1 : col, t});
    };
    for (int i = 0; i < desc->n_aggs; i++) {
        int fn = desc->aggs[i].fn, col = desc->aggs[i].col;
        if (fn == SH_AGG_SUM) add_base(B_SUM, col);
        else if (fn == SH_AGG_AVG) { add_base(B_SUM, col); add_base(B_COUNT, -1); }
        else if (fn == SH_AGG_COUNT) add_base(B_COUNT, -1);
        else if (fn == SH_AGG_MIN) add_base(B_MIN, col);
        else add_base(B_MAX, col);
    }
    for (size_t i = 0; i < a->bases.size(); i++) a->vtypes[i] = a->base_out_type(a->bases[i]);
    // executor chain sec -> ... (AggregationParser.buildIncrementalExecutors :605-620)
    for (int dur = desc->min_duration; dur <= desc->max_duration; dur++) {
        auto ex = std::unique_ptr<IncExec>(new IncExec());
        ex->dur = dur; ex->root = dur == desc->min_duration; ex->rt = a;
        a->execs.push_back(std::move(ex));
    }
    for (size_t i = 0; i + 1 < a->execs.size(); i++) a->execs[i]->next = a->execs[i + 1].get();
    a->tables.resize(SH_DUR_YEARS + 1);
    a->history.resize(SH_DUR_YEARS + 1);
    a->views.resize(SH_DUR_YEARS + 2);
    return a;
}

void or_aggregation_destroy(void* h) { delete (AggRuntime*)h; }

int or_aggregation_push(void* h, const sh_batch* b) {
    AggRuntime* a = (AggRuntime*)h;
    int64_t step = b->send_size > 0 ? b->send_size : b->n;
    for (int64_t lo = 0; lo < b->n; lo += step) a->send(b, lo, std::min(b->n, lo + step));
    return SH_OK;
}

int or_aggregation_advance_time(void* h, int64_t now) {
    ((AggRuntime*)h)->set_clock(now);
    return SH_OK;
}

int or_aggregation_table(void* h, int32_t dur, const sh_out** out) {
    AggRuntime* a = (AggRuntime*)h;
    if (dur < 0 || dur > SH_DUR_YEARS) { g_err = "bad duration"; return SH_ERR_INVALID; }
    OutBuf& ob = a->views[dur];
    ob.clear();
    ob.with_rep = false;
    for (const OutRow& r : a->tables[dur]) ob.rows.push_back(r);
    if (!ob.rows.empty()) ob.close_flush(a->clock);
    *out = ob.view(1 + a->d.n_group_by, (int)a->bases.size(), a->vtypes);
    a->tables[dur].clear();
    return SH_OK;
}

int or_aggregation_find(void* h, int32_t per, int64_t start, int64_t end, const sh_out** out) {
    AggRuntime* a = (AggRuntime*)h;
    if (per < a->d.min_duration || per > a->d.max_duration) { g_err = "duration not aggregated"; return SH_ERR_INVALID; }
    OutBuf& ob = a->views[SH_DUR_YEARS + 1];
    a->find(per, start, end, ob);
    *out = ob.view(1 + a->d.n_group_by, (int)a->bases.size(), a->vtypes);
    return SH_OK;
}

// String.valueOf of a double / float (the partition flow id of such keys) as ASCII, for the tests
int or_fp_text(double v, int32_t is_float, char* out, int32_t cap) {
    const std::u16string t = jhm::fp_decimal(v, is_float != 0);
    if (!out || cap <= (int32_t)t.size()) return SH_ERR_INVALID;
    for (size_t i = 0; i < t.size(); i++) out[i] = (char)t[i];
    out[t.size()] = 0;
    return SH_OK;
}

}  // extern "C"
