"""Python loader for the CPU restatement (liboracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg, as the checker. The product path (siddhi_amd) never imports this module.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

from siddhi_amd import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.POINTER
        L.or_last_error.restype = C.c_char_p
        L.or_query_create.argtypes = [P(abi.QueryDesc)]
        L.or_query_create.restype = C.c_void_p
        L.or_query_destroy.argtypes = [C.c_void_p]
        L.or_query_set_output_rate.argtypes = [C.c_void_p, C.c_int32, C.c_int64]
        L.or_query_set_ext_timeout.argtypes = [C.c_void_p, C.c_int64]
        L.or_query_set_ext_replace_ts.argtypes = [C.c_void_p, C.c_int32]
        L.or_query_rep_ts_attr.argtypes = [C.c_void_p, P(P(C.c_int64)), P(C.c_int64)]
        L.or_query_set_strings.argtypes = [C.c_void_p, C.c_int32, C.c_int64, C.c_int64, C.c_void_p, C.c_void_p]
        L.or_push.argtypes = [C.c_void_p, P(abi.Batch), P(P(abi.Out))]
        L.or_advance_time.argtypes = [C.c_void_p, C.c_int64, P(P(abi.Out))]
        L.or_aggregation_create.argtypes = [P(abi.AggregationDesc)]
        L.or_aggregation_create.restype = C.c_void_p
        L.or_aggregation_destroy.argtypes = [C.c_void_p]
        L.or_aggregation_push.argtypes = [C.c_void_p, P(abi.Batch)]
        L.or_aggregation_advance_time.argtypes = [C.c_void_p, C.c_int64]
        L.or_aggregation_table.argtypes = [C.c_void_p, C.c_int32, P(P(abi.Out))]
        L.or_aggregation_find.argtypes = [C.c_void_p, C.c_int32, C.c_int64, C.c_int64, P(P(abi.Out))]
        L.or_fp_text.argtypes = [C.c_double, C.c_int32, C.c_char_p, C.c_int32]
        _lib = L
    return _lib


def fp_text(v: float, is_float: bool = False) -> str:
    """Double.toString / Float.toString of v as the restatement computes it (a partition flow id)."""
    buf = C.create_string_buffer(64)
    if lib().or_fp_text(float(v), int(is_float), buf, 64):
        raise ValueError("or_fp_text")
    return buf.value.decode()


class OracleQuery:
    """Window query run by the restatement. push()/advance_time() return decoded flushes."""

    def __init__(self, spec: abi.QuerySpec):
        self.spec = spec
        self._desc = spec.desc()
        self.h = lib().or_query_create(C.byref(self._desc))
        if not self.h:
            raise ValueError(lib().or_last_error().decode())
        if spec.rate and lib().or_query_set_output_rate(self.h, abi.RATE_KINDS[spec.rate[0]], int(spec.rate[1])):
            raise ValueError(lib().or_last_error().decode())
        if spec.timeout and lib().or_query_set_ext_timeout(self.h, int(spec.timeout)):
            raise ValueError(lib().or_last_error().decode())
        if spec.replace_ts and lib().or_query_set_ext_replace_ts(self.h, 1):
            raise ValueError(lib().or_last_error().decode())
        for col, names in (spec.strings or {}).items():
            self.set_strings(col, names)

    def set_strings(self, col, names, first_id=0):
        if abi.apply_strings(lib().or_query_set_strings, self.h, self.spec, col, list(names), first_id):
            raise ValueError(lib().or_last_error().decode())

    def push_raw(self, batch: abi.HostBatch):
        out = C.POINTER(abi.Out)()
        rc = lib().or_push(self.h, C.byref(batch.b), C.byref(out))
        if rc != 0:
            raise RuntimeError(lib().or_last_error().decode())
        return out

    def push(self, batch: abi.HostBatch):
        return abi.decode_out(self.push_raw(batch))

    def advance_time_raw(self, now: int):
        out = C.POINTER(abi.Out)()
        rc = lib().or_advance_time(self.h, now, C.byref(out))
        if rc != 0:
            raise RuntimeError(lib().or_last_error().decode())
        return out

    def advance_time(self, now: int):
        return abi.decode_out(self.advance_time_raw(now))

    def rep_ts_attr(self):
        """The timestamp attribute of every row's representative event in the last output."""
        import numpy as np
        v, n = C.POINTER(C.c_int64)(), C.c_int64()
        lib().or_query_rep_ts_attr(self.h, C.byref(v), C.byref(n))
        return np.ctypeslib.as_array(v, shape=(n.value,)).copy() if n.value else np.zeros(0, np.int64)

    def close(self):
        if self.h:
            lib().or_query_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class OracleAggregation:
    def __init__(self, spec: abi.AggregationSpec):
        self.spec = spec
        self._desc = spec.desc()
        self.h = lib().or_aggregation_create(C.byref(self._desc))
        if not self.h:
            raise ValueError(lib().or_last_error().decode())

    def push(self, batch: abi.HostBatch):
        rc = lib().or_aggregation_push(self.h, C.byref(batch.b))
        if rc != 0:
            raise RuntimeError(lib().or_last_error().decode())

    def advance_time(self, now: int):
        lib().or_aggregation_advance_time(self.h, now)

    def table_raw(self, duration: int):
        out = C.POINTER(abi.Out)()
        rc = lib().or_aggregation_table(self.h, duration, C.byref(out))
        if rc != 0:
            raise RuntimeError(lib().or_last_error().decode())
        return out

    def table(self, duration: int):
        fl = abi.decode_out(self.table_raw(duration))
        return [r for f in fl for r in f.rows]

    def find_raw(self, per: int, start: int, end: int):
        out = C.POINTER(abi.Out)()
        rc = lib().or_aggregation_find(self.h, per, start, end, C.byref(out))
        if rc != 0:
            raise RuntimeError(lib().or_last_error().decode())
        return out

    def find(self, per: int, start: int, end: int):
        fl = abi.decode_out(self.find_raw(per, start, end))
        return [r for f in fl for r in f.rows]

    def close(self):
        if self.h:
            lib().or_aggregation_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
