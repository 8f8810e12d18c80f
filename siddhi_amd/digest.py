"""Canonical SHA-256 of a query's output stream ("a SHA-256 of the canonical output").

The digest covers, in this order and little-endian: the tag b"siddhi-out-v1", the flush sizes (int64)
and flush clocks (int64), then the rows' timestamps (int64), expired flags (uint8), group keys (int64,
[key][row]), aggregate values (their 8-byte patterns, [agg][row]), null flags (uint8, [agg][row]) and the
stream index of each row's representative event (int64). Doubles are hashed by their bits, so equal
digests mean bit-identical outputs, row order included. Works on the dicts abi.out_arrays /
abi.concat_arrays / runtime.device_out_arrays return.
"""
from __future__ import annotations

import hashlib

import numpy as np


def output_digest(a) -> str:
    h = hashlib.sha256(b"siddhi-out-v1")
    offs = np.asarray(a["flush_offsets"], dtype=np.int64)
    for arr, dt in ((np.diff(offs), "<i8"), (a["flush_clock"], "<i8"), (a["ts"], "<i8"), (a["expired"], "u1"),
                    (a["keys"], "<i8"), (a["vals"], "<u8"), (a["nulls"], "u1"), (a["rep"], "<i8")):
        b = np.ascontiguousarray(np.asarray(arr).astype(dt, copy=False))
        h.update(np.int64(b.size).tobytes())
        h.update(b.tobytes())
    return h.hexdigest()
