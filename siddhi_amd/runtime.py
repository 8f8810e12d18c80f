"""Host-side Python mirror of the reference's interface for the GPU path.

`GpuQuery` plays the role of a Siddhi query whose window / aggregator extensions run on the MI355X:
`send()` is `InputHandler.send(Event[])` (core/stream/input/InputHandler.java:85-96) and the
registered callbacks receive one list of rows per flush, as `StreamCallback.receive(Event[])` does
(core/stream/output/StreamCallback.java:93-129). Everything runs through libsiddhi_hip.so; there is
no CPU fallback — importing this module on a box without the built library raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import os
from typing import Callable, List, Optional

from . import abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SH_LIB", os.path.join(HERE, "libsiddhi_hip.so"))

_lib = None


def lib():
    """Load libsiddhi_hip.so (built in-tree by `make -C siddhi_amd/csrc`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make -C siddhi_amd/csrc` "
                              "(the GPU path has no CPU fallback)")
        L = C.CDLL(LIB_PATH)
        abi.setup_lib_prototypes(L, "sh")
        if L.sh_abi_version() != 16:
            raise ImportError("libsiddhi_hip ABI version mismatch")
        _lib = L
    return _lib


def device_out_arrays(out_ptr, device_flushes: bool = False):
    """abi.out_arrays for an sh_push_device result: its row arrays are copied out of HBM (hipMemcpy, a
    synchronising copy) into host arrays; flush offsets / clocks are on the host unless the query set the
    device flush layout (sh_query_set_device_flushes)."""
    o = out_ptr.contents
    n, nk, na = o.n_rows, o.n_keys, o.n_vals
    hip = C.CDLL("libamdhip64.so")
    host = {}
    if device_flushes and o.flush_offsets and o.n_flushes:
        fo = np.zeros(o.n_flushes + 1, np.int64)
        fc = np.zeros(o.n_flushes, np.int64)
        for a, p in ((fo, o.flush_offsets), (fc, o.flush_clock)):
            rc = hip.hipMemcpy(C.c_void_p(a.ctypes.data), C.cast(p, C.c_void_p), C.c_size_t(a.nbytes), 2)
            if rc != 0:
                raise SiddhiError(abi.SH_ERR_DEVICE, f"hipMemcpy of the flush layout failed ({rc})")
        host["flush"] = (fo, fc)
    for name, cnt, dt in (("ts", n, np.int64), ("expired", n, np.uint8), ("keys", nk * n, np.int64),
                          ("vals", na * n, np.uint64), ("nulls", na * n, np.uint8), ("rep", n, np.int64)):
        a = np.zeros(max(cnt, 1), dt)
        src = C.cast(getattr(o, name), C.c_void_p).value
        if cnt:
            rc = hip.hipMemcpy(C.c_void_p(a.ctypes.data), C.c_void_p(src), C.c_size_t(a.itemsize * cnt), 2)
            if rc != 0:
                raise SiddhiError(abi.SH_ERR_DEVICE, f"hipMemcpy of output column {name} failed ({rc})")
        host[name] = a[:cnt]
    fo, fc = host["flush"] if "flush" in host else abi.flush_arrays(o, host["ts"])
    return {
        "flush_offsets": fo, "flush_clock": fc,
        "val_types": np.array([o.val_types[i] for i in range(na)], np.int32),
        "ts": host["ts"], "expired": host["expired"], "rep": host["rep"],
        "keys": host["keys"].reshape(nk, n), "vals": host["vals"].reshape(na, n), "nulls": host["nulls"].reshape(na, n),
    }


class SiddhiError(RuntimeError):
    """SiddhiAppRuntimeException analogue: carries the library's error code and message."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def _check(rc: int):
    if rc != 0:
        raise SiddhiError(rc, lib().sh_last_error().decode())


class Context:
    def __init__(self, device: int = 0):
        self.h = C.c_void_p()
        _check(lib().sh_init(device, C.byref(self.h)))

    def close(self):
        if self.h:
            lib().sh_ctx_destroy(self.h)
            self.h = None


_default_ctx: Optional[Context] = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(int(os.environ.get("SH_DEVICE", "0")))
    return _default_ctx


class GpuQuery:
    """A window query on the GPU: `from S[cond]#window.<kind>(...) select k, aggs group by k insert into O`."""

    def __init__(self, spec: abi.QuerySpec, ctx: Optional[Context] = None):
        self.spec = spec
        self.ctx = ctx or default_context()
        self._desc = spec.desc()
        self.h = C.c_void_p()
        _check(lib().sh_query_create(self.ctx.h, C.byref(self._desc), C.byref(self.h)))
        self.callbacks: List[Callable] = []
        try:
            if spec.rate:
                _check(lib().sh_query_set_output_rate(self.h, abi.RATE_KINDS[spec.rate[0]], int(spec.rate[1])))
            if spec.timeout:
                _check(lib().sh_query_set_ext_timeout(self.h, int(spec.timeout)))
            if spec.replace_ts:
                _check(lib().sh_query_set_ext_replace_ts(self.h, 1))
            for col, names in (spec.strings or {}).items():
                self.set_strings(col, names)
        except Exception:
            self.close()
            raise

    def set_device_flushes(self, on: bool = True):
        """sh_query_set_device_flushes: sh_push_device leaves the flush layout in device memory too."""
        _check(lib().sh_query_set_device_flushes(self.h, 1 if on else 0))

    def set_compact_flushes(self, on: bool = True):
        """sh_query_set_compact_flushes: one-row flushes at their rows' timestamps leave the flush arrays NULL."""
        _check(lib().sh_query_set_compact_flushes(self.h, 1 if on else 0))

    def rate_apply_merged(self, merged: dict) -> dict:
        """sh_rate_apply_merged: this query (rate set, never pushed) as the output rate limiter of a sharded
        query; `merged` is one call's merged owner output (out_arrays layout), the result the limited rows."""
        n = int(merged["ts"].size)
        dt = {"flush_offsets": np.int64, "flush_clock": np.int64, "ts": np.int64, "expired": np.uint8,
              "keys": np.int64, "vals": np.uint64, "nulls": np.uint8, "rep": np.int64}
        keep = {k: np.ascontiguousarray(merged[k], dtype=t) for k, t in dt.items()}
        o = abi.Out()
        o.n_flushes = int(keep["flush_clock"].size)
        o.n_rows = n
        o.n_keys = int(keep["keys"].shape[0])
        o.n_vals = int(keep["vals"].shape[0])
        for i, t in enumerate(merged["val_types"]):
            o.val_types[i] = int(t)
        P = C.POINTER
        o.flush_offsets = keep["flush_offsets"].ctypes.data_as(P(C.c_int64))
        o.flush_clock = keep["flush_clock"].ctypes.data_as(P(C.c_int64))
        o.ts = keep["ts"].ctypes.data_as(P(C.c_int64))
        o.expired = keep["expired"].ctypes.data_as(P(C.c_uint8))
        o.keys = keep["keys"].ctypes.data_as(P(C.c_int64))
        o.vals = keep["vals"].ctypes.data_as(P(C.c_uint64))
        o.nulls = keep["nulls"].ctypes.data_as(P(C.c_uint8))
        o.rep = keep["rep"].ctypes.data_as(P(C.c_int64))
        out = C.POINTER(abi.Out)()
        _check(lib().sh_rate_apply_merged(self.h, C.byref(o), C.byref(out)))
        return abi.out_arrays(out)

    def set_strings(self, col: str, names, first_id: int = 0):
        """The text of string column `col`'s dictionary ids first_id.. (sh_query_set_strings)."""
        _check(abi.apply_strings(lib().sh_query_set_strings, self.h, self.spec, col, list(names), first_id))

    # -- reference-shaped API --------------------------------------------------------------
    def add_callback(self, fn: Callable[[List[tuple]], None]):
        """StreamCallback.receive(Event[]): fn(rows) once per flush."""
        self.callbacks.append(fn)

    def send(self, batch: abi.HostBatch):
        flushes = self.push(batch)
        for f in flushes:
            for cb in self.callbacks:
                cb(f.rows)
        return flushes

    # -- ABI-level API ---------------------------------------------------------------------
    def push_raw(self, batch: abi.HostBatch):
        out = C.POINTER(abi.Out)()
        _check(lib().sh_push(self.h, C.byref(batch.b), C.byref(out)))
        return out

    def push(self, batch: abi.HostBatch):
        return abi.decode_out(self.push_raw(batch))

    @staticmethod
    def device_batch(n: int, ts_ptr: int, col_ptrs: List[int], send_size: int = 0) -> abi.Batch:
        """An sh_batch descriptor of device-resident columns, built once and pushed any number of times
        (what a host shim keeps per buffer instead of rebuilding it per call)."""
        b = abi.Batch()
        b.n = n
        b.send_size = send_size
        b.ts = ts_ptr
        for i, p in enumerate(col_ptrs):
            b.cols[i] = p
        return b

    def push_device(self, n: int, ts_ptr: int, col_ptrs: List[int], send_size: int = 0):
        """Device-resident batch (HBM pointers, e.g. torch tensors' data_ptr()). Returns the sh_out
        pointer: flush metadata on the host, row arrays in device memory."""
        return self.push_device_batch(self.device_batch(n, ts_ptr, col_ptrs, send_size))

    def push_device_batch(self, b: abi.Batch):
        out = C.POINTER(abi.Out)()
        _check(lib().sh_push_device(self.h, C.byref(b), C.byref(out)))
        return out

    # -- double-buffered host ingest (sh_stage / sh_push_staged) -----------------------------
    def stage(self, batch) -> int:
        """Queue the H2D copy of a host batch (ideally a PinnedBatch) on the copy stream; returns the
        ticket for push_staged. The batch must stay alive and unchanged until its push returns."""
        t = C.c_int32()
        _check(lib().sh_stage(self.h, C.byref(batch.b), C.byref(t)))
        self._staged = getattr(self, "_staged", {})
        self._staged[t.value] = batch
        return t.value

    def push_staged_raw(self, ticket: int):
        out = C.POINTER(abi.Out)()
        _check(lib().sh_push_staged(self.h, ticket, C.byref(out)))
        getattr(self, "_staged", {}).pop(ticket, None)  # its copy has landed and been consumed
        return out

    def push_staged(self, ticket: int):
        return abi.decode_out(self.push_staged_raw(ticket))

    def ingest_stats(self):
        """(H2D copy ms, bytes) of the last pushed staged batch."""
        ms, nb = C.c_double(), C.c_int64()
        _check(lib().sh_ingest_stats(self.h, C.byref(ms), C.byref(nb)))
        return ms.value, nb.value

    def advance_time_raw(self, now: int):
        out = C.POINTER(abi.Out)()
        _check(lib().sh_advance_time(self.h, now, C.byref(out)))
        return out

    def advance_time(self, now: int):
        return abi.decode_out(self.advance_time_raw(now))

    def stats(self) -> abi.Stats:
        s = abi.Stats()
        _check(lib().sh_query_stats(self.h, C.byref(s)))
        return s

    def rep_ts_attr(self):
        """replaceTimestampWithBatchEndTime: the timestamp attribute of every row's representative event in
        the last output — its batch's end time (sh_query_rep_ts_attr)."""
        v, n = C.POINTER(C.c_int64)(), C.c_int64()
        _check(lib().sh_query_rep_ts_attr(self.h, C.byref(v), C.byref(n)))
        return np.ctypeslib.as_array(v, shape=(n.value,)).copy() if n.value else np.zeros(0, np.int64)

    def snapshot(self) -> bytes:
        """State.snapshot(): the query's device state as bytes (sh_query_snapshot)."""
        n = C.c_int64()
        _check(lib().sh_query_snapshot(self.h, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        _check(lib().sh_query_snapshot(self.h, buf, n.value, C.byref(n)))
        return buf.raw[:n.value]

    def restore(self, blob: bytes):
        """State.restore(): continue from a snapshot of a query built from the same descriptor."""
        _check(lib().sh_query_restore(self.h, blob, len(blob)))

    def close(self):
        if self.h:
            lib().sh_query_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class GpuAggregation:
    """`define aggregation ... every sec...year` on the GPU."""

    def __init__(self, spec: abi.AggregationSpec, ctx: Optional[Context] = None):
        self.spec = spec
        self.ctx = ctx or default_context()
        self._desc = spec.desc()
        self.h = C.c_void_p()
        _check(lib().sh_aggregation_create(self.ctx.h, C.byref(self._desc), C.byref(self.h)))

    def push(self, batch: abi.HostBatch):
        _check(lib().sh_aggregation_push(self.h, C.byref(batch.b)))

    def push_device(self, n: int, ts_ptr: int, col_ptrs: List[int], send_size: int = 0):
        b = abi.Batch()
        b.n = n
        b.send_size = send_size
        b.ts = ts_ptr
        for i, p in enumerate(col_ptrs):
            b.cols[i] = p
        _check(lib().sh_aggregation_push_device(self.h, C.byref(b)))

    def advance_time(self, now: int):
        _check(lib().sh_aggregation_advance_time(self.h, now))

    def stats(self) -> abi.Stats:
        s = abi.Stats()
        _check(lib().sh_aggregation_stats(self.h, C.byref(s)))
        return s

    def timing(self, reset: bool = False):
        """(device ms summed over the pushes since the last reset, pushes) — sh_aggregation_timing."""
        ms, n = C.c_double(), C.c_int64()
        _check(lib().sh_aggregation_timing(self.h, C.byref(ms), C.byref(n), int(reset)))
        return ms.value, n.value

    def table_raw(self, duration: int):
        out = C.POINTER(abi.Out)()
        _check(lib().sh_aggregation_table(self.h, duration, C.byref(out)))
        return out

    def find_raw(self, per: int, start: int, end: int):
        """`from A within start, end per <per>`: table + in-memory rows, (AGG_TIMESTAMP, key) order."""
        out = C.POINTER(abi.Out)()
        _check(lib().sh_aggregation_find(self.h, per, start, end, C.byref(out)))
        return out

    def find(self, per: int, start: int, end: int):
        fl = abi.decode_out(self.find_raw(per, start, end))
        return [r for f in fl for r in f.rows]

    def snapshot(self) -> bytes:
        n = C.c_int64()
        _check(lib().sh_aggregation_snapshot(self.h, None, 0, C.byref(n)))
        buf = C.create_string_buffer(n.value)
        _check(lib().sh_aggregation_snapshot(self.h, buf, n.value, C.byref(n)))
        return buf.raw[:n.value]

    def restore(self, blob: bytes):
        _check(lib().sh_aggregation_restore(self.h, blob, len(blob)))

    def table(self, duration: int):
        return [r for f in abi.decode_out(self.table_raw(duration)) for r in f.rows]

    def close(self):
        if self.h:
            lib().sh_aggregation_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class PinnedBatch:
    """An sh_batch whose SoA columns live in one pinned host block (sh_alloc_pinned): what the Java shim
    packs a ComplexEventChunk into. For n events the block holds ts[n], then every column's n values,
    each run 16-byte aligned — one contiguous region, so sh_stage moves it with a single H2D copy.
    `fill` copies numpy columns in (laying the block out for their length); `arrays` are the views of the
    current layout and are valid only until the next `fill` / `set_n` re-lays the block out. A caller that
    writes `arrays` directly (laid out for the capacity at construction) calls `set_n(n)` afterwards."""

    def __init__(self, schema: abi.Schema, capacity: int, send_size: int = 0):
        self.schema = schema
        self.capacity = capacity
        self._dts = [np.dtype(np.int64)] + [np.dtype(abi.NP_DTYPE[t]) for t in schema.types]
        self._ptrs = []
        p = C.c_void_p()
        _check(lib().sh_alloc_pinned(max(1, self._span(capacity)), C.byref(p)))
        self._ptrs.append(p)
        self.b = abi.Batch()
        self.b.send_size = send_size
        self._layout(capacity)
        self.b.n = 0

    @staticmethod
    def _a16(x):
        return (x + 15) & ~15

    def _span(self, n):
        off = 0
        for dt in self._dts:
            off = self._a16(off + n * dt.itemsize)
        return off

    def _layout(self, n):
        base, off = self._ptrs[0].value, 0
        self._laid = n
        self.arrays = []
        for dt in self._dts:
            buf = (C.c_char * max(1, n * dt.itemsize)).from_address(base + off)
            self.arrays.append(np.frombuffer(buf, dtype=dt, count=n))
            if len(self.arrays) == 1:
                self.b.ts = base + off
            else:
                self.b.cols[len(self.arrays) - 2] = base + off
            off = self._a16(off + n * dt.itemsize)

    def set_n(self, n: int):
        """The batch holds the first n events written into `arrays`: the columns move to their places in
        the n-event layout (nothing moves when the block is already laid out for n)."""
        assert n <= self.capacity
        if n != self._laid:
            keep = [a[:n].copy() for a in self.arrays]
            self._layout(n)
            for a, k in zip(self.arrays, keep):
                a[:] = k
        self.b.n = n

    def fill(self, ts, cols, send_size=None):
        n = len(ts)
        assert n <= self.capacity
        self._layout(n)
        self.arrays[0][:] = ts
        for a, c in zip(self.arrays[1:], cols):
            a[:] = c
        self.b.n = n
        if send_size is not None:
            self.b.send_size = send_size
        return self

    def close(self):
        for p in self._ptrs:
            if p.value:
                lib().sh_free_pinned(p)
        self._ptrs = []
        self.arrays = []

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
