"""CPU check of the oracle's output rate limiters: oracle(query with `output ... every n events`) must
equal a direct Python transcription of the five Java event limiters (core/query/output/ratelimit/event/*)
and of the two `output first every <t>` limiters (ratelimit/time/First[GroupBy]PerTimeOutputRateLimiter)
applied flush by flush to oracle(query without it), on random streams. Complements the 18
EventOutputRateLimitTestCase KATs that pin the counts."""
import numpy as np
import pytest

from oracle.oracle import OracleQuery
from siddhi_amd import abi
from tests.parity import run_pushes, split_batches

SCHEMA = abi.Schema.parse("k int, v double, ts long")


def py_limit(flushes, kind, n, group_by):
    """flushes: list of (clock, [rows]) with row = (key tuple, payload). Returns the limited flushes."""
    out, counter, chunk, counts, last = [], 0, [], {}, {}
    out_time = None
    for clock, rows in flushes:
        sent = []
        if kind == "first_time" and not group_by:  # FirstPerTimeOutputRateLimiter.process :54-78
            if rows and (out_time is None or out_time + n <= clock):
                out_time = clock
                sent.append(rows[0][1])
            if sent:
                out.append((clock, sent))
            continue
        for key, row in rows:
            if kind == "first_time":  # FirstGroupByPerTimeOutputRateLimiter.process :54-80
                t = counts.get(key)
                if t is None or t + n <= clock:
                    counts[key] = clock
                    sent.append(row)
                continue
            if kind == "all":  # AllPerEventOutputRateLimiter.process :48-77
                chunk.append(row)
                counter += 1
                if counter == n:
                    sent += chunk
                    chunk, counter = [], 0
            elif kind == "first" and not group_by:  # FirstPerEventOutputRateLimiter :48-72
                counter += 1
                if counter == 1:
                    sent.append(row)
                elif counter == n:
                    counter = 0
            elif kind == "last" and not group_by:  # LastPerEventOutputRateLimiter :47-71
                counter += 1
                if counter == n:
                    sent.append(row)
                    counter = 0
            elif kind == "first":  # FirstGroupByPerEventOutputRateLimiter :48-77
                c = counts.get(key)
                if c is None:
                    counts[key] = 1
                    sent.append(row)
                elif c == n - 1:
                    del counts[key]
                else:
                    counts[key] = c + 1
            else:  # LastGroupByPerEventOutputRateLimiter :51-83 (dict keeps first insertion order)
                last[key] = row
                counter += 1
                if counter == n:
                    counter = 0
                    sent += list(last.values())
                    last = {}
        if sent:
            out.append((clock, sent))
    return out


def flushes_of(a):
    res = []
    fo, fc = a["flush_offsets"], a["flush_clock"]
    for f in range(len(fc)):
        rows = []
        for r in range(fo[f], fo[f + 1]):
            key = tuple(int(x) for x in a["keys"][:, r])
            payload = (int(a["ts"][r]), int(a["expired"][r]), key, tuple(int(x) for x in a["vals"][:, r]),
                       tuple(int(x) for x in a["nulls"][:, r]), int(a["rep"][r]))
            rows.append((key, payload))
        res.append((int(fc[f]), rows))
    return res


@pytest.mark.parametrize("kind,n", [("all", 1), ("all", 4), ("first", 1), ("first", 3), ("last", 1), ("last", 5),
                                    ("first_time", 0), ("first_time", 37)])
@pytest.mark.parametrize("window,param,output", [("lengthBatch", 7, "current"), ("timeBatch", 50, "all"),
                                                 ("time", 40, "current")])
@pytest.mark.parametrize("group_by", [True, False])
def test_oracle_limiters_match_python(kind, n, window, param, output, group_by):
    rng = np.random.default_rng(hash((kind, n, window, group_by)) & 0xFFFF)
    m = 3_000
    ts = np.cumsum(rng.integers(0, 5, m)).astype(np.int64) + 1_000
    cols = [rng.integers(0, 12, m).astype(np.int32), rng.integers(-50, 50, m).astype(np.float64) / 4, ts.copy()]
    gb = ["k"] if group_by else ()
    base = abi.QuerySpec(SCHEMA, window, param, group_by=gb, aggs=[("count", None), ("sum", "v")], output=output)
    lim = abi.QuerySpec(SCHEMA, window, param, group_by=gb, aggs=[("count", None), ("sum", "v")], output=output,
                        rate=(kind, n))
    pushes = split_batches(SCHEMA, ts, cols, [500, 1_700], 3) + [("advance", int(ts[-1]) + 200)]
    qa, qb = OracleQuery(base), OracleQuery(lim)
    want = py_limit(flushes_of(run_pushes(qa, pushes)), kind, n, group_by)
    got = [(c, [p for _, p in rows]) for c, rows in flushes_of(run_pushes(qb, pushes))]
    assert got == want
    assert got or kind == "first"
