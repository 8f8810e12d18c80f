"""Shared driver for the transcribed reference KATs (tests/golden/kat_reference.json): builds the
query / aggregation from a case, feeds its sends, and checks ONLY what the Java test asserted.
Used against the oracle (CPU) and the HIP library (GPU)."""
import json
import os

import numpy as np

from siddhi_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))


def load_cases():
    with open(os.path.join(HERE, "golden", "kat_reference.json")) as f:
        return json.load(f)["cases"]


class Dict:
    """Host string dictionary (the Java shim's String -> int32 id map)."""

    def __init__(self):
        self.ids = {}

    def id(self, s):
        return self.ids.setdefault(s, len(self.ids))

    def name(self, i):
        for k, v in self.ids.items():
            if v == i:
                return k
        raise KeyError(i)


def _conv_filter(expr, dic):
    if expr is None:
        return None
    if isinstance(expr, list):
        if len(expr) == 2 and expr[0] in abi.TYPE_NAMES:
            if expr[0] == "string":
                return ("string", dic.id(expr[1]))
            return (expr[0], expr[1])
        return tuple(_conv_filter(e, dic) for e in expr)
    return expr


def build(case, dic):
    schema = abi.Schema.parse(case["schema"])
    if case.get("kind") == "aggregation":
        a = case["aggregation"]
        spec = abi.AggregationSpec(schema, aggs=[tuple(x) for x in a["aggs"]], group_by=a.get("group_by", ()),
                                   ts=a.get("ts"), durations=tuple(a["durations"]),
                                   filter=_conv_filter(a.get("filter"), dic), tz_offset_ms=a.get("tz_offset_ms", 0))
        return schema, spec
    q = case["query"]
    spec = abi.QuerySpec(schema, q["window"], q.get("param", 0), group_by=q.get("group_by", ()),
                         aggs=[tuple(x) for x in q.get("aggs", [])], filter=_conv_filter(q.get("filter"), dic),
                         start_time=q.get("start_time"), stream_current=q.get("stream_current", False),
                         output=q.get("output", "current"), partition=q.get("partition"),
                         ts_attr=q.get("ts_attr"), start_attr=q.get("start_attr"), timeout=q.get("timeout"),
                         replace_ts=q.get("replace_ts", False),
                         rate=tuple(q["rate"]) if q.get("rate") else None)
    return schema, spec


def batch_of(schema, send, dic, send_size=0):
    rows = []
    for r in send:
        vals = [r[0]]
        for t, v in zip(schema.types, r[1:]):
            vals.append(dic.id(v) if t == abi.STRID else v)
        rows.append(tuple(vals))
    return abi.HostBatch.from_rows(schema, rows, send_size)


def run_query(case, make_query):
    """make_query(spec) -> object with push(HostBatch) and advance_time(now) returning flushes."""
    dic = Dict()
    schema, spec = build(case, dic)
    # the shim's dictionary holds every string it has seen; a string partition key's text goes with it
    # (sh_query_set_strings: the Scheduler's HashMap order hashes the partition key's String)
    for s in case["sends"]:
        if isinstance(s, list):
            batch_of(schema, s, dic)
    if spec.partition and schema.types[schema.col(spec.partition)] == abi.STRID:
        spec.strings = {spec.partition: [dic.name(i) for i in range(len(dic.ids))]}
    q = make_query(spec)
    flushes = []
    for s in case["sends"]:
        fl = q.advance_time(s["advance"]) if isinstance(s, dict) else q.push(batch_of(schema, s, dic))
        if spec.replace_ts:
            # replaceTimestampWithBatchEndTime: the representative events' timestamp attribute as the
            # window holds it (the batch end time), per row of this call
            ra, o = list(q.rep_ts_attr()), 0
            for f in fl:
                f.rep_attrs = ra[o:o + len(f.rows)]
                o += len(f.rows)
        flushes += fl
    return schema, spec, dic, flushes


def check_query(case, flushes, schema, dic):
    e = case["expect"]
    rows = [r for f in flushes for r in f.rows]
    ins = [r for r in rows if not r[1]]
    rem = [r for r in rows if r[1]]
    if "in_count" in e:
        assert len(ins) == e["in_count"], (len(ins), e)
    if "remove_count" in e:
        assert len(rem) == e["remove_count"], (len(rem), e)
    if "total_count" in e:
        assert len(rows) == e["total_count"], (len(rows), e)
    if "in_count_max" in e:
        assert len(ins) <= e["in_count_max"]
    if "min_in_count" in e:
        assert len(ins) >= e["min_in_count"]
    if "flush_sizes" in e:
        assert [len(f.rows) for f in flushes] == e["flush_sizes"], [len(f.rows) for f in flushes]
    if "values" in e:
        got = [list(r[3]) for r in rows]
        assert got == e["values"], (got, e["values"])
    if "flush_count" in e:
        assert len(flushes) == e["flush_count"], (len(flushes), e)
    if "flush_first_col" in e or "flush_last_col" in e:
        # rows carry their event timestamp, unique per send here: map it back to the sent column
        for key, pick in (("flush_first_col", 0), ("flush_last_col", -1)):
            if key not in e:
                continue
            col, want = e[key]
            c = schema.col(col)
            ts2v = {r[0]: r[1 + c] for s in case["sends"] if isinstance(s, list) for r in s}
            got = [ts2v[f.rows[pick][0]] for f in flushes[:len(want)]]
            assert got == want, (key, got, want)
    if "value_range" in e:
        idx, lo, hi = e["value_range"]
        for r in rows:
            assert lo <= r[3][idx] <= hi
    # non-aggregated select attributes come from the row's representative event (sh_out.rep, the
    # event QuerySelector keeps per key): in/remove order checks and transcribed attribute columns
    events = [r for s in case["sends"] if isinstance(s, list) for r in s]
    reps = [x for f in flushes for x in f.reps]
    if "in_order" in e or "remove_order" in e or "rep_cols" in e or "in_col_in" in e:
        assert len(reps) == len(rows), "output without representative events"

    replaced = [x for f in flushes for x in getattr(f, "rep_attrs", [])]
    ts_attr = case["query"].get("ts_attr") if case["query"].get("replace_ts") else None

    def attr(col, idx):
        if col == ts_attr:
            return int(replaced[idx])
        return events[reps[idx]][1 + schema.col(col)]
    if "in_order" in e:
        got = [attr(e["in_order_col"], i) for i, r in enumerate(rows) if not r[1]]
        assert got == e["in_order"], (got, e["in_order"])
    if "remove_order" in e:
        got = [attr(e.get("in_order_col", "volume"), i) for i, r in enumerate(rows) if r[1]]
        assert got == e["remove_order"], (got, e["remove_order"])
    if "in_col_in" in e:  # the Java callback asserts every (first) in-event's attribute is one of these
        col, allowed = e["in_col_in"]
        for i, r in enumerate(rows):
            if not r[1]:
                assert attr(col, i) in allowed, (col, attr(col, i), allowed)
    if "rep_cols" in e:
        for col, want in e["rep_cols"]:
            got = [attr(col, i) for i in range(len(rows))]
            assert got == want, (col, got, want)
    return rows


def run_aggregation(case, make_agg):
    dic = Dict()
    schema, spec = build(case, dic)
    a = make_agg(spec)
    for s in case["sends"]:
        if isinstance(s, dict):
            a.advance_time(s["advance"])
        else:
            a.push(batch_of(schema, s, dic))
    return schema, spec, dic, a


def check_aggregation_table(case, spec, dic, table_rows):
    """table_rows: [(ts, expired, keys, vals)] with keys = (bucket, group...) and vals = base values."""
    e = case["expect"]
    names = spec.base_names()
    got = []
    for ts, _, keys, vals in table_rows:
        base = dict(zip(names, vals))
        row = [keys[0]] + [dic.name(keys[1 + g]) for g in range(len(spec.group_by))]
        for fn, col in spec.aggs:
            if fn == "avg":
                row.append(base[f"sum_{col}"] / base["count"])
            elif fn == "sum":
                row.append(base[f"sum_{col}"])
            elif fn == "count":
                row.append(base["count"])
            else:
                row.append(base[f"{fn}_{col}"])
        got.append(row)
    exp = [list(r) for r in e["rows"]]
    key = lambda r: tuple(r[:1 + len(spec.group_by)])
    assert sorted(got, key=key) == sorted(exp, key=key), (sorted(got, key=key), sorted(exp, key=key))


def aggregation_rows(case, agg):
    """The rows a case checks: a retrieval (`within ... per`, expect.find) or a duration table."""
    e = case["expect"]
    if "find" in e:
        f = e["find"]
        return agg.find(abi.DUR_NAMES[f["per"]], f["start"], f["end"])
    return agg.table(abi.DUR_NAMES[e["table"]])
