"""ctypes mirror of include/siddhi_hip.h plus helpers that build descriptors and batches and decode
sh_out into plain Python rows.

The structs here must match the C header field for field; tests/test_abi.py checks their sizes
against values the C compiler reports for the header.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np

# ---- constants (siddhi_hip.h) -------------------------------------------------------------
SH_OK = 0
SH_ERR_INVALID = -1
SH_ERR_UNSUPPORTED = -2
SH_ERR_DEVICE = -3
SH_ERR_OOM = -4
SH_ERR_STATE = -5

INT, LONG, FLOAT, DOUBLE, STRID, BOOL = 1, 2, 3, 4, 5, 6
TYPE_NAMES = {"int": INT, "long": LONG, "float": FLOAT, "double": DOUBLE, "string": STRID, "bool": BOOL}
NP_DTYPE = {INT: np.int32, LONG: np.int64, FLOAT: np.float32, DOUBLE: np.float64, STRID: np.int32, BOOL: np.uint8}

OP_COL, OP_CONST, OP_GT, OP_GE, OP_LT, OP_LE, OP_EQ, OP_NE, OP_AND, OP_OR, OP_NOT = range(1, 12)
CMP_OPS = {">": OP_GT, ">=": OP_GE, "<": OP_LT, "<=": OP_LE, "==": OP_EQ, "!=": OP_NE}

WIN_NONE, WIN_LENGTH_BATCH, WIN_TIME_BATCH, WIN_TIME, WIN_EXT_TIME_BATCH, WIN_EXT_TIME = 0, 1, 2, 3, 4, 5
AGG_SUM, AGG_AVG, AGG_COUNT, AGG_MIN, AGG_MAX = 1, 2, 3, 4, 5
AGG_NAMES = {"sum": AGG_SUM, "avg": AGG_AVG, "count": AGG_COUNT, "min": AGG_MIN, "max": AGG_MAX}
DUR_SECONDS, DUR_MINUTES, DUR_HOURS, DUR_DAYS, DUR_MONTHS, DUR_YEARS = range(6)
DUR_NAMES = {"sec": 0, "min": 1, "hour": 2, "day": 3, "month": 4, "year": 5}

MAX_COLS, MAX_AGGS, MAX_GROUP = 8, 8, 8


class FilterOp(C.Structure):
    _fields_ = [("op", C.c_int32), ("type", C.c_int32), ("col", C.c_int32), ("pad", C.c_int32),
                ("ival", C.c_int64), ("dval", C.c_double)]


class AggSpec(C.Structure):
    _fields_ = [("fn", C.c_int32), ("col", C.c_int32)]


class QueryDesc(C.Structure):
    _fields_ = [("n_cols", C.c_int32), ("col_types", C.c_int32 * MAX_COLS),
                ("n_filter_ops", C.c_int32), ("filter", C.POINTER(FilterOp)),
                ("window", C.c_int32), ("stream_current", C.c_int32), ("window_param", C.c_int64),
                ("has_start_time", C.c_int32), ("n_group_by", C.c_int32), ("start_time", C.c_int64),
                ("group_by", C.c_int32 * MAX_GROUP), ("n_aggs", C.c_int32), ("current_on", C.c_int32),
                ("aggs", AggSpec * MAX_AGGS), ("expired_on", C.c_int32), ("partition_col", C.c_int32),
                ("key_capacity", C.c_int64), ("ts_col", C.c_int32), ("start_col", C.c_int32)]


class AggregationDesc(C.Structure):
    _fields_ = [("n_cols", C.c_int32), ("col_types", C.c_int32 * MAX_COLS),
                ("n_filter_ops", C.c_int32), ("filter", C.POINTER(FilterOp)),
                ("n_group_by", C.c_int32), ("group_by", C.c_int32 * MAX_GROUP),
                ("n_aggs", C.c_int32), ("aggs", AggSpec * MAX_AGGS), ("ts_col", C.c_int32),
                ("min_duration", C.c_int32), ("max_duration", C.c_int32), ("key_capacity", C.c_int64),
                ("tz_offset_ms", C.c_int64)]


class Batch(C.Structure):
    _fields_ = [("n", C.c_int64), ("send_size", C.c_int64), ("ts", C.c_void_p),
                ("cols", C.c_void_p * MAX_COLS)]


class Out(C.Structure):
    _fields_ = [("n_flushes", C.c_int64), ("n_rows", C.c_int64), ("n_keys", C.c_int32),
                ("n_vals", C.c_int32), ("val_types", C.c_int32 * MAX_AGGS),
                ("flush_offsets", C.POINTER(C.c_int64)), ("flush_clock", C.POINTER(C.c_int64)),
                ("ts", C.POINTER(C.c_int64)), ("expired", C.POINTER(C.c_uint8)),
                ("keys", C.POINTER(C.c_int64)), ("vals", C.POINTER(C.c_uint64)),
                ("nulls", C.POINTER(C.c_uint8)), ("rep", C.POINTER(C.c_int64))]


class SliceSummary(C.Structure):
    _fields_ = [("n", C.c_int64), ("n_pass", C.c_int64), ("max_tl", C.c_int64), ("first_clock", C.c_int64),
                ("first_key", C.c_int64), ("ts_min", C.c_int64), ("ts_max", C.c_int64)]


class Bound(C.Structure):
    _fields_ = [("W", C.c_int64), ("clock", C.c_int64), ("gidx", C.c_int64), ("pad", C.c_int64)]


class Stats(C.Structure):
    _fields_ = [("push_ms", C.c_double), ("main_kernel_ms", C.c_double),
                ("main_kernel_bytes", C.c_int64), ("events", C.c_int64)]


# ---- descriptor builders ------------------------------------------------------------------

@dataclass
class Schema:
    names: List[str]
    types: List[int]

    @staticmethod
    def parse(spec: str) -> "Schema":
        """'symbol string, price double, volume long' -> Schema"""
        names, types = [], []
        for part in spec.split(","):
            n, t = part.split()
            names.append(n)
            types.append(TYPE_NAMES[t])
        return Schema(names, types)

    def col(self, name: str) -> int:
        return self.names.index(name)


def compile_filter(schema: Schema, expr) -> List[FilterOp]:
    """Compile a nested tuple expression into postfix FilterOps.

    expr := ('>', lhs, rhs) | ('and', e, e) | ('or', e, e) | ('not', e)
    operand := column name (str) | (type_name, value) constant | python int/float (int->INT, float->DOUBLE)
    """
    ops: List[FilterOp] = []

    def operand(x):
        if isinstance(x, str):
            ops.append(FilterOp(op=OP_COL, col=schema.col(x)))
        elif isinstance(x, tuple) and len(x) == 2 and x[0] in TYPE_NAMES:
            t = TYPE_NAMES[x[0]]
            if t in (FLOAT, DOUBLE):
                ops.append(FilterOp(op=OP_CONST, type=t, dval=float(x[1])))
            else:
                ops.append(FilterOp(op=OP_CONST, type=t, ival=int(x[1])))
        elif isinstance(x, bool):
            ops.append(FilterOp(op=OP_CONST, type=BOOL, ival=int(x)))
        elif isinstance(x, int):
            ops.append(FilterOp(op=OP_CONST, type=INT, ival=x))
        elif isinstance(x, float):
            ops.append(FilterOp(op=OP_CONST, type=DOUBLE, dval=x))
        else:
            walk(x)

    def walk(e):
        head = e[0]
        if head in CMP_OPS:
            operand(e[1]); operand(e[2]); ops.append(FilterOp(op=CMP_OPS[head]))
        elif head == "and":
            walk(e[1]); walk(e[2]); ops.append(FilterOp(op=OP_AND))
        elif head == "or":
            walk(e[1]); walk(e[2]); ops.append(FilterOp(op=OP_OR))
        elif head == "not":
            walk(e[1]); ops.append(FilterOp(op=OP_NOT))
        else:
            raise ValueError(f"bad filter expression {e!r}")

    if expr is not None:
        walk(expr)
    return ops


@dataclass
class QuerySpec:
    """`from S[filter]#window.kind(param...) select group..., aggs... group by group... insert ...`"""
    schema: Schema
    window: Optional[str]            # 'lengthBatch' | 'timeBatch' | 'time' | None (no window)
    param: int = 0
    group_by: Sequence[str] = ()
    aggs: Sequence[tuple] = ()       # (fn_name, column or None)
    filter: object = None
    start_time: Optional[int] = None
    stream_current: bool = False
    output: str = "current"          # 'current' | 'all' | 'expired'
    partition: Optional[str] = None
    key_capacity: int = 0
    rate: Optional[tuple] = None       # ('all'|'first'|'last', n): `output <kind> every n events`;
                                       # ('first_time', ms): `output first every <ms> milliseconds`
    strings: Optional[dict] = None     # {string column: [text of id 0, 1, ...]} (sh_query_set_strings)
    ts_attr: Optional[str] = None      # externalTimeBatch timestamp attribute
    start_attr: Optional[str] = None   # externalTimeBatch start time from this attribute
    timeout: Optional[int] = None      # externalTimeBatch(ts, T, start, timeout): scheduler timeout (ms)
    replace_ts: bool = False           # externalTimeBatch(..., timeout, true): replaceTimestampWithBatchEndTime
    _keep: list = field(default_factory=list, repr=False)

    def desc(self) -> QueryDesc:
        d = QueryDesc()
        d.n_cols = len(self.schema.types)
        for i, t in enumerate(self.schema.types):
            d.col_types[i] = t
        fops = compile_filter(self.schema, self.filter)
        arr = (FilterOp * max(1, len(fops)))(*fops)
        self._keep.append(arr)
        d.n_filter_ops = len(fops)
        d.filter = C.cast(arr, C.POINTER(FilterOp))
        d.window = {None: WIN_NONE, "lengthBatch": WIN_LENGTH_BATCH, "timeBatch": WIN_TIME_BATCH,
                    "time": WIN_TIME, "externalTimeBatch": WIN_EXT_TIME_BATCH,
                    "externalTime": WIN_EXT_TIME}[self.window]
        d.window_param = self.param
        d.stream_current = int(self.stream_current)
        d.has_start_time = int(self.start_time is not None)
        d.start_time = self.start_time or 0
        d.n_group_by = len(self.group_by)
        for i, g in enumerate(self.group_by):
            d.group_by[i] = self.schema.col(g)
        d.n_aggs = len(self.aggs)
        for i, (fn, col) in enumerate(self.aggs):
            d.aggs[i].fn = AGG_NAMES[fn]
            d.aggs[i].col = self.schema.col(col) if col is not None else 0
        d.current_on = int(self.output in ("current", "all"))
        d.expired_on = int(self.output in ("expired", "all"))
        d.partition_col = self.schema.col(self.partition) if self.partition else -1
        d.key_capacity = self.key_capacity
        d.ts_col = self.schema.col(self.ts_attr) if self.ts_attr else 0
        d.start_col = self.schema.col(self.start_attr) if self.start_attr else 0
        if self.start_attr:
            d.has_start_time = 2
        return d


@dataclass
class AggregationSpec:
    """`define aggregation A from S[filter] select g, aggs group by g aggregate [by ts] every a...b`"""
    schema: Schema
    aggs: Sequence[tuple]
    group_by: Sequence[str] = ()
    ts: Optional[str] = None
    durations: tuple = ("sec", "day")
    filter: object = None
    key_capacity: int = 0
    tz_offset_ms: int = 0  # aggTimeZone as a fixed offset from GMT (Asia/Singapore: 8 * 3600_000)
    _keep: list = field(default_factory=list, repr=False)

    def desc(self) -> AggregationDesc:
        d = AggregationDesc()
        d.n_cols = len(self.schema.types)
        for i, t in enumerate(self.schema.types):
            d.col_types[i] = t
        fops = compile_filter(self.schema, self.filter)
        arr = (FilterOp * max(1, len(fops)))(*fops)
        self._keep.append(arr)
        d.n_filter_ops = len(fops)
        d.filter = C.cast(arr, C.POINTER(FilterOp))
        d.n_group_by = len(self.group_by)
        for i, g in enumerate(self.group_by):
            d.group_by[i] = self.schema.col(g)
        d.n_aggs = len(self.aggs)
        for i, (fn, col) in enumerate(self.aggs):
            d.aggs[i].fn = AGG_NAMES[fn]
            d.aggs[i].col = self.schema.col(col) if col is not None else 0
        d.ts_col = self.schema.col(self.ts) if self.ts else -1
        d.min_duration = DUR_NAMES[self.durations[0]]
        d.max_duration = DUR_NAMES[self.durations[1]]
        d.key_capacity = self.key_capacity
        d.tz_offset_ms = self.tz_offset_ms
        return d

    def base_names(self) -> List[str]:
        """Base value order AggregationParser.populateFinalBaseAggregators produces."""
        names: List[str] = []
        for fn, col in self.aggs:
            want = {"sum": [f"sum_{col}"], "avg": [f"sum_{col}", "count"], "count": ["count"],
                    "min": [f"min_{col}"], "max": [f"max_{col}"]}[fn]
            for w in want:
                if w not in names:
                    names.append(w)
        return names


# ---- batches -------------------------------------------------------------------------------

class HostBatch:
    """SoA host arrays for one sh_batch; keeps numpy arrays alive while the struct is in use."""

    def __init__(self, schema: Schema, ts: np.ndarray, cols: Sequence[np.ndarray], send_size: int = 0):
        self.ts = np.ascontiguousarray(ts, dtype=np.int64)
        self.cols = [np.ascontiguousarray(c, dtype=NP_DTYPE[t]) for c, t in zip(cols, schema.types)]
        self.b = Batch()
        self.b.n = len(self.ts)
        self.b.send_size = send_size
        self.b.ts = self.ts.ctypes.data
        for i, c in enumerate(self.cols):
            self.b.cols[i] = c.ctypes.data

    @staticmethod
    def from_rows(schema: Schema, rows: Sequence[tuple], send_size: int = 0) -> "HostBatch":
        """rows: (ts, v0, v1, ...) with python values; strings must already be dictionary ids."""
        ts = np.array([r[0] for r in rows], dtype=np.int64)
        cols = [np.array([r[1 + i] for r in rows], dtype=NP_DTYPE[t]) for i, t in enumerate(schema.types)]
        return HostBatch(schema, ts, cols, send_size)


# ---- outputs -------------------------------------------------------------------------------

@dataclass
class Flush:
    clock: int
    rows: List[tuple]   # (ts, expired, keys tuple, values tuple with None for null)
    reps: List[int] = field(default_factory=list)  # stream index of each row's representative event


def flush_arrays(o, ts=None):
    """(flush_offsets, flush_clock) of an sh_out; a compact output (sh_query_set_compact_flushes: NULL arrays)
    is one flush per row at the row's timestamp (`ts`: the host copy of the rows' timestamps)."""
    if not o.n_flushes:
        return np.zeros(1, np.int64), np.zeros(0, np.int64)
    if not o.flush_offsets:
        if ts is None:
            ts = np.ctypeslib.as_array(o.ts, shape=(o.n_rows,))
        return np.arange(o.n_flushes + 1, dtype=np.int64), np.asarray(ts, np.int64)[:o.n_flushes].copy()
    return (np.ctypeslib.as_array(o.flush_offsets, shape=(o.n_flushes + 1,)).copy(),
            np.ctypeslib.as_array(o.flush_clock, shape=(o.n_flushes,)).copy())


def decode_out(out_ptr) -> List[Flush]:
    o = out_ptr.contents
    n = o.n_rows
    flushes: List[Flush] = []
    if o.n_flushes == 0:
        return flushes
    offs, clocks = flush_arrays(o)
    if n:
        ts = np.ctypeslib.as_array(o.ts, shape=(n,)).copy()
        exp = np.ctypeslib.as_array(o.expired, shape=(n,)).copy()
        keys = np.ctypeslib.as_array(o.keys, shape=(max(1, o.n_keys) * n,)).copy().reshape(max(1, o.n_keys), n) \
            if o.n_keys else np.zeros((0, n), np.int64)
        vals = np.ctypeslib.as_array(o.vals, shape=(max(1, o.n_vals) * n,)).copy().reshape(max(1, o.n_vals), n) \
            if o.n_vals else np.zeros((0, n), np.uint64)
        nulls = np.ctypeslib.as_array(o.nulls, shape=(max(1, o.n_vals) * n,)).copy().reshape(max(1, o.n_vals), n) \
            if o.n_vals else np.zeros((0, n), np.uint8)
        rep = np.ctypeslib.as_array(o.rep, shape=(n,)).copy() if o.rep else np.full(n, -1, np.int64)
    vt = [o.val_types[i] for i in range(o.n_vals)]
    for f in range(o.n_flushes):
        rows = []
        reps = [int(rep[r]) for r in range(int(offs[f]), int(offs[f + 1]))]
        for r in range(int(offs[f]), int(offs[f + 1])):
            vs = []
            for v in range(o.n_vals):
                if nulls[v, r]:
                    vs.append(None)
                elif vt[v] in (DOUBLE, FLOAT):
                    vs.append(float(np.array([vals[v, r]], dtype=np.uint64).view(np.float64)[0]))
                else:
                    vs.append(int(np.array([vals[v, r]], dtype=np.uint64).view(np.int64)[0]))
            rows.append((int(ts[r]), int(exp[r]), tuple(int(keys[k, r]) for k in range(o.n_keys)), tuple(vs)))
        flushes.append(Flush(int(clocks[f]), rows, reps))
    return flushes


def out_arrays(out_ptr) -> Dict[str, np.ndarray]:
    """Vectorised view of an sh_out (copies), for large parity comparisons."""
    o = out_ptr.contents
    n = o.n_rows
    fo, fc = flush_arrays(o)
    res: Dict[str, np.ndarray] = {
        "flush_offsets": fo, "flush_clock": fc,
        "val_types": np.array([o.val_types[i] for i in range(o.n_vals)], np.int32),
    }
    if n:
        res["ts"] = np.ctypeslib.as_array(o.ts, shape=(n,)).copy()
        res["expired"] = np.ctypeslib.as_array(o.expired, shape=(n,)).copy()
        res["keys"] = np.ctypeslib.as_array(o.keys, shape=(o.n_keys * n,)).copy().reshape(o.n_keys, n) \
            if o.n_keys else np.zeros((0, n), np.int64)
        res["vals"] = np.ctypeslib.as_array(o.vals, shape=(o.n_vals * n,)).copy().reshape(o.n_vals, n) \
            if o.n_vals else np.zeros((0, n), np.uint64)
        res["nulls"] = np.ctypeslib.as_array(o.nulls, shape=(o.n_vals * n,)).copy().reshape(o.n_vals, n) \
            if o.n_vals else np.zeros((0, n), np.uint8)
        res["rep"] = np.ctypeslib.as_array(o.rep, shape=(n,)).copy() if o.rep else np.full(n, -1, np.int64)
    else:
        res.update(ts=np.zeros(0, np.int64), expired=np.zeros(0, np.uint8),
                   keys=np.zeros((o.n_keys, 0), np.int64), vals=np.zeros((o.n_vals, 0), np.uint64),
                   nulls=np.zeros((o.n_vals, 0), np.uint8), rep=np.zeros(0, np.int64))
    return res


def concat_arrays(parts: List[Dict[str, np.ndarray]]) -> Dict[str, np.ndarray]:
    """Concatenate several out_arrays() results (e.g. one per push) into one stream."""
    if not parts:
        raise ValueError("no parts")
    offs = [np.zeros(1, np.int64)]
    base = 0
    for p in parts:
        offs.append(p["flush_offsets"][1:] + base)
        base += len(p["ts"])
    res = {"flush_offsets": np.concatenate(offs), "flush_clock": np.concatenate([p["flush_clock"] for p in parts]),
           "val_types": parts[0]["val_types"]}
    for k in ("ts", "expired", "rep"):
        res[k] = np.concatenate([p[k] for p in parts])
    if all("rep_attr" in p for p in parts):
        res["rep_attr"] = np.concatenate([p["rep_attr"] for p in parts])
    for k in ("keys", "vals", "nulls"):
        res[k] = np.concatenate([p[k] for p in parts], axis=1)
    return res


def setup_lib_prototypes(lib, prefix: str):
    """Declare argtypes for a library exposing the sh_* (prefix 'sh') ABI."""
    P = C.POINTER
    lib.sh_init.argtypes = [C.c_int32, P(C.c_void_p)]
    lib.sh_ctx_destroy.argtypes = [C.c_void_p]
    lib.sh_query_create.argtypes = [C.c_void_p, P(QueryDesc), P(C.c_void_p)]
    lib.sh_query_destroy.argtypes = [C.c_void_p]
    lib.sh_push.argtypes = [C.c_void_p, P(Batch), P(P(Out))]
    lib.sh_push_device.argtypes = [C.c_void_p, P(Batch), P(P(Out))]
    lib.sh_advance_time.argtypes = [C.c_void_p, C.c_int64, P(P(Out))]
    lib.sh_aggregation_create.argtypes = [C.c_void_p, P(AggregationDesc), P(C.c_void_p)]
    lib.sh_aggregation_destroy.argtypes = [C.c_void_p]
    lib.sh_aggregation_push.argtypes = [C.c_void_p, P(Batch)]
    lib.sh_aggregation_push_device.argtypes = [C.c_void_p, P(Batch)]
    lib.sh_aggregation_advance_time.argtypes = [C.c_void_p, C.c_int64]
    lib.sh_aggregation_table.argtypes = [C.c_void_p, C.c_int32, P(P(Out))]
    lib.sh_aggregation_find.argtypes = [C.c_void_p, C.c_int32, C.c_int64, C.c_int64, P(P(Out))]
    lib.sh_query_set_output_rate.argtypes = [C.c_void_p, C.c_int32, C.c_int64]
    lib.sh_rate_apply_merged.argtypes = [C.c_void_p, P(Out), P(P(Out))]
    lib.sh_query_set_ext_timeout.argtypes = [C.c_void_p, C.c_int64]
    lib.sh_query_set_ext_replace_ts.argtypes = [C.c_void_p, C.c_int32]
    lib.sh_query_set_compact_flushes.argtypes = [C.c_void_p, C.c_int32]
    lib.sh_query_set_device_flushes.argtypes = [C.c_void_p, C.c_int32]
    lib.sh_query_rep_ts_attr.argtypes = [C.c_void_p, P(P(C.c_int64)), P(C.c_int64)]
    lib.sh_aggregation_timing.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int32]
    lib.sh_shard_flush_windows.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    lib.sh_query_set_strings.argtypes = [C.c_void_p, C.c_int32, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p]
    lib.sh_aggregation_snapshot.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, P(C.c_int64)]
    lib.sh_aggregation_restore.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    lib.sh_alloc_pinned.argtypes = [C.c_int64, P(C.c_void_p)]
    lib.sh_stage.argtypes = [C.c_void_p, P(Batch), P(C.c_int32)]
    lib.sh_push_staged.argtypes = [C.c_void_p, C.c_int32, P(P(Out))]
    lib.sh_ingest_stats.argtypes = [C.c_void_p, P(C.c_double), P(C.c_int64)]
    lib.sh_free_pinned.argtypes = [C.c_void_p]
    lib.sh_query_stats.argtypes = [C.c_void_p, P(Stats)]
    lib.sh_aggregation_stats.argtypes = [C.c_void_p, P(Stats)]
    if hasattr(lib, "sh_query_snapshot"):
        lib.sh_query_snapshot.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, P(C.c_int64)]
        lib.sh_query_restore.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    lib.sh_last_error.restype = C.c_char_p
    lib.sh_abi_version.restype = C.c_int32
    if hasattr(lib, "sh_shard_create"):
        PI = P(C.c_int64)
        lib.sh_shard_create.argtypes = [C.c_void_p, P(QueryDesc), C.c_int32, C.c_int32, P(C.c_void_p)]
        lib.sh_shard_destroy.argtypes = [C.c_void_p]
        lib.sh_shard_record_bytes.argtypes = [C.c_void_p, PI]
        lib.sh_shard_summarize.argtypes = [C.c_void_p, P(Batch), P(SliceSummary)]
        lib.sh_shard_pack.argtypes = [C.c_void_p, P(SliceSummary), P(Batch), C.c_void_p, C.c_int64, PI,
                                      P(P(Bound)), PI]
        lib.sh_shard_consume.argtypes = [C.c_void_p, C.c_void_p, PI, P(Bound), C.c_int64, C.c_int32,
                                         P(P(Out)), P(PI)]
        lib.sh_shard_stats.argtypes = [C.c_void_p, P(Stats)]
        lib.sh_shard_advance_time.argtypes = [C.c_void_p, C.c_int64, C.c_int32, P(P(Out)), P(PI)]
        lib.sh_shard_snapshot.argtypes = [C.c_void_p, C.c_void_p, C.c_int64, PI]
        lib.sh_shard_restore.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
    if hasattr(lib, "sh_aggregation_shard_create"):
        lib.sh_aggregation_shard_create.argtypes = [C.c_void_p, P(AggregationDesc), C.c_int32, C.c_int32,
                                                    P(C.c_void_p), P(C.c_void_p)]


# every exported symbol include/siddhi_hip.h declares
ABI_SYMBOLS = [
    "sh_init", "sh_ctx_destroy", "sh_query_create", "sh_query_destroy", "sh_push", "sh_push_device",
    "sh_advance_time", "sh_aggregation_create", "sh_aggregation_destroy", "sh_aggregation_push",
    "sh_aggregation_push_device", "sh_aggregation_advance_time", "sh_aggregation_table",
    "sh_alloc_pinned", "sh_free_pinned", "sh_query_stats", "sh_last_error", "sh_abi_version",
    "sh_shard_create", "sh_shard_destroy", "sh_shard_record_bytes", "sh_shard_summarize", "sh_shard_pack",
    "sh_shard_consume", "sh_shard_advance_time", "sh_shard_stats", "sh_query_snapshot", "sh_query_restore",
    "sh_aggregation_shard_create", "sh_aggregation_stats", "sh_stage", "sh_push_staged", "sh_ingest_stats",
    "sh_aggregation_find", "sh_aggregation_snapshot", "sh_aggregation_restore", "sh_query_set_output_rate", "sh_query_set_ext_timeout", "sh_query_set_ext_replace_ts", "sh_query_set_compact_flushes", "sh_query_set_device_flushes", "sh_query_rep_ts_attr", "sh_aggregation_timing", "sh_shard_flush_windows",
    "sh_shard_snapshot", "sh_shard_restore", "sh_query_set_strings", "sh_rate_apply_merged",
]


def encode_strings(names):
    """UTF-16 code units + offsets (n + 1) of `names`: the sh_query_set_strings layout (a Java String's chars)."""
    parts = [np.frombuffer(str(s).encode("utf-16-le"), dtype=np.uint16) for s in names]
    offs = np.zeros(len(parts) + 1, dtype=np.int64)
    if parts:
        offs[1:] = np.cumsum([p.size for p in parts])
    units = np.concatenate(parts) if parts and offs[-1] > 0 else np.zeros(1, dtype=np.uint16)
    return np.ascontiguousarray(units), offs


def apply_strings(fn, h, spec, col, names, first_id=0):
    """fn = the library's set_strings entry point; registers `names` as ids first_id.. of column `col`."""
    units, offs = encode_strings(names)
    return fn(h, spec.schema.col(col), first_id, len(names), units.ctypes.data, offs.ctypes.data)

# output rate limiter kinds (SH_RATE_*)
RATE_KINDS = {"all": 1, "first": 2, "last": 3, "first_time": 4}
