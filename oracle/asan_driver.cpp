// asan_driver.cpp — TEST INFRASTRUCTURE ONLY. Drives the CPU restatement (siddhi_oracle.cpp) through
// every query shape it restates, on seeded synthetic streams, in a binary built with
// -fsanitize=address,undefined (oracle/Makefile `asan`), so the checker itself is run under the
// sanitizers (SURVEY.md §5's sanitizer build; tests/test_oracle_asan.py). Exit status 0 = every call
// returned OK and the sanitizers reported nothing (they abort the process otherwise).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#include "oracle.h"

namespace {

struct Rng {
    uint64_t s;
    uint64_t next() {
        s += 0x9E3779B97F4A7C15ull;
        uint64_t z = s;
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
};

// columns: k int, v double, x long, et long; ts non-decreasing with occasional late event times
struct Stream {
    std::vector<int64_t> ts, x, et;
    std::vector<int32_t> k;
    std::vector<double> v;
    Stream(int64_t n, uint64_t seed, int keys) {
        Rng r{seed};
        int64_t t = 1'700'000'000'000;
        for (int64_t i = 0; i < n; i++) {
            t += (int64_t)(r.next() % 3);
            ts.push_back(t);
            k.push_back((int32_t)(r.next() % (uint64_t)keys));
            v.push_back((double)((int64_t)(r.next() % 801) - 400) / 8.0);
            x.push_back((int64_t)(r.next() % 101) - 50);
            et.push_back(t - (int64_t)(r.next() % 500));
        }
    }
    sh_batch batch(int64_t lo, int64_t hi, int64_t send) const {
        sh_batch b{};
        b.n = hi - lo;
        b.send_size = send;
        b.ts = ts.data() + lo;
        b.cols[0] = k.data() + lo;
        b.cols[1] = v.data() + lo;
        b.cols[2] = x.data() + lo;
        b.cols[3] = et.data() + lo;
        return b;
    }
};

int fails = 0;

void check(int rc, const char* what) {
    if (rc != 0) {
        std::fprintf(stderr, "%s failed: %s\n", what, or_last_error());
        fails++;
    }
}

sh_query_desc base_desc(int window, int64_t param) {
    sh_query_desc d{};
    d.n_cols = 4;
    d.col_types[0] = SH_T_INT;
    d.col_types[1] = SH_T_DOUBLE;
    d.col_types[2] = SH_T_LONG;
    d.col_types[3] = SH_T_LONG;
    d.window = window;
    d.window_param = param;
    d.n_group_by = 1;
    d.group_by[0] = 0;
    d.n_aggs = 5;
    d.aggs[0] = {SH_AGG_COUNT, 0};
    d.aggs[1] = {SH_AGG_SUM, 1};
    d.aggs[2] = {SH_AGG_MIN, 1};
    d.aggs[3] = {SH_AGG_MAX, 2};
    d.aggs[4] = {SH_AGG_AVG, 2};
    d.current_on = 1;
    d.partition_col = -1;
    d.key_capacity = 256;
    d.ts_col = 3;
    d.start_col = -1;
    return d;
}

void run_query(const char* name, const sh_query_desc& d, const Stream& s, int64_t send, int rate_kind = SH_RATE_NONE,
               int64_t rate_n = 0) {
    void* q = or_query_create(&d);
    if (!q) {
        std::fprintf(stderr, "%s: create failed: %s\n", name, or_last_error());
        fails++;
        return;
    }
    if (rate_kind != SH_RATE_NONE) check(or_query_set_output_rate(q, rate_kind, rate_n), name);
    const int64_t n = (int64_t)s.ts.size();
    const int64_t cuts[] = {0, 1, 777, n / 3, n / 2 + 5, n};
    int64_t rows = 0;
    for (int i = 0; i + 1 < 6; i++) {
        sh_batch b = s.batch(cuts[i], cuts[i + 1], send);
        const sh_out* o = nullptr;
        check(or_push(q, &b, &o), name);
        if (o) rows += o->n_rows;
    }
    const sh_out* o = nullptr;
    check(or_advance_time(q, s.ts.back() + 100'000, &o), name);
    if (o) rows += o->n_rows;
    std::printf("%-28s rows %lld\n", name, (long long)rows);
    or_query_destroy(q);
}

}  // namespace

int main() {
    const Stream s(20'000, 0xA5A5, 97);
    sh_filter_op f[3] = {};
    f[0].op = SH_OP_COL; f[0].col = 1;
    f[1].op = SH_OP_CONST; f[1].type = SH_T_DOUBLE; f[1].dval = -20.0;
    f[2].op = SH_OP_GT;
    for (int out = 0; out < 3; out++) {
        const int cur = out != 2, exp = out != 0;
        const char* tag[] = {"current", "all", "expired"};
        char nm[64];
        // batch windows, filter, group-by
        sh_query_desc d = base_desc(SH_WIN_LENGTH_BATCH, 333);
        d.current_on = cur; d.expired_on = exp; d.n_filter_ops = 3; d.filter = f;
        std::snprintf(nm, sizeof nm, "lengthBatch %s", tag[out]); run_query(nm, d, s, 7);
        d = base_desc(SH_WIN_TIME_BATCH, 250);
        d.current_on = cur; d.expired_on = exp;
        std::snprintf(nm, sizeof nm, "timeBatch %s", tag[out]); run_query(nm, d, s, 1);
        d.stream_current = 1;
        std::snprintf(nm, sizeof nm, "timeBatch current %s", tag[out]); run_query(nm, d, s, 5);
        d = base_desc(SH_WIN_TIME, 300);
        d.current_on = cur; d.expired_on = exp;
        std::snprintf(nm, sizeof nm, "time %s", tag[out]); run_query(nm, d, s, 1);
        d = base_desc(SH_WIN_EXT_TIME, 300);
        d.current_on = cur; d.expired_on = exp;
        std::snprintf(nm, sizeof nm, "externalTime %s", tag[out]); run_query(nm, d, s, 3);
        d = base_desc(SH_WIN_EXT_TIME_BATCH, 400);
        d.current_on = cur; d.expired_on = exp;
        std::snprintf(nm, sizeof nm, "externalTimeBatch %s", tag[out]); run_query(nm, d, s, 1);
        // partitions (lanes for lengthBatch / time; the shared-timer quirk for timeBatch)
        d = base_desc(SH_WIN_LENGTH_BATCH, 5);
        d.current_on = cur; d.expired_on = exp; d.partition_col = 0;
        std::snprintf(nm, sizeof nm, "partition lengthBatch %s", tag[out]); run_query(nm, d, s, 4);
        d = base_desc(SH_WIN_TIME, 200);
        d.current_on = cur; d.expired_on = exp; d.partition_col = 0;
        std::snprintf(nm, sizeof nm, "partition time %s", tag[out]); run_query(nm, d, s, 1);
    }
    sh_query_desc d = base_desc(SH_WIN_TIME_BATCH, 500);
    d.partition_col = 0;
    run_query("partition timeBatch", d, s, 1);
    // output rate limiting (event-count and first-every-t forms, with and without group-by)
    const int kinds[] = {SH_RATE_ALL, SH_RATE_FIRST, SH_RATE_LAST, SH_RATE_FIRST_TIME};
    for (int g = 0; g < 2; g++)
        for (int kind : kinds) {
            d = base_desc(SH_WIN_LENGTH_BATCH, 50);
            d.n_group_by = g;
            char nm[64];
            std::snprintf(nm, sizeof nm, "rate %d group %d", kind, g);
            run_query(nm, d, s, 3, kind, kind == SH_RATE_FIRST_TIME ? 40 : 7);
        }
    // incremental aggregation sec ... year with late events, tables and retrievals
    sh_aggregation_desc ad{};
    ad.n_cols = 4;
    ad.col_types[0] = SH_T_INT; ad.col_types[1] = SH_T_DOUBLE; ad.col_types[2] = SH_T_LONG; ad.col_types[3] = SH_T_LONG;
    ad.n_group_by = 1;
    ad.group_by[0] = 0;
    ad.n_aggs = 4;
    ad.aggs[0] = {SH_AGG_SUM, 1}; ad.aggs[1] = {SH_AGG_AVG, 2}; ad.aggs[2] = {SH_AGG_MIN, 1}; ad.aggs[3] = {SH_AGG_COUNT, 0};
    ad.ts_col = 3;
    ad.min_duration = SH_DUR_SECONDS;
    ad.max_duration = SH_DUR_YEARS;
    ad.key_capacity = 128;
    void* a = or_aggregation_create(&ad);
    if (!a) { std::fprintf(stderr, "aggregation create failed: %s\n", or_last_error()); return 1; }
    const int64_t n = (int64_t)s.ts.size();
    for (int64_t lo = 0; lo < n; lo += 3001) {
        sh_batch b = s.batch(lo, lo + 3001 < n ? lo + 3001 : n, 9);
        check(or_aggregation_push(a, &b), "aggregation push");
    }
    check(or_aggregation_advance_time(a, s.ts.back() + 400LL * 86'400'000), "aggregation advance");
    int64_t rows = 0;
    for (int dur = SH_DUR_SECONDS; dur <= SH_DUR_YEARS; dur++) {
        const sh_out* o = nullptr;
        check(or_aggregation_table(a, dur, &o), "aggregation table");
        if (o) rows += o->n_rows;
        check(or_aggregation_find(a, dur, 0, INT64_MAX / 2, &o), "aggregation find");
    }
    std::printf("%-28s rows %lld\n", "aggregation sec..year", (long long)rows);
    or_aggregation_destroy(a);
    if (fails) std::fprintf(stderr, "%d calls failed\n", fails);
    return fails ? 1 : 0;
}
