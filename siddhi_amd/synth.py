"""Seeded synthetic event streams for the BASELINE.json configurations.

PRNG: counter-based SplitMix64 — draw j of a stream with seed s is mix64(s + (j + 1) * GAMMA), so any
slice of a stream can be generated independently (used to shard streams across ranks and to build
bench batches without replaying the prefix). Each event consumes `width` consecutive draws.
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
T0 = 1_700_000_000_000  # event-time origin (ms)


def mix64(z: np.ndarray) -> np.ndarray:
    z = z.astype(np.uint64, copy=True)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def draws(seed: int, start: int, n: int, width: int) -> np.ndarray:
    """[n, width] uint64 draws for events start..start+n-1."""
    j = np.arange(start * width, (start + n) * width, dtype=np.uint64) + np.uint64(1)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + j * GAMMA
    return mix64(z).reshape(n, width)


def uniform_price(u: np.ndarray, quantized: bool = False) -> np.ndarray:
    """(u >> 11) * 2^-53 * 200 in [0, 200); quantized mode floors to multiples of 2^-6 (exactly summable)."""
    p = (u >> np.uint64(11)).astype(np.float64) * (2.0 ** -53) * 200.0
    if quantized:
        p = np.floor(p * 64.0) / 64.0
    return p


def c1_stock(start: int, n: int, seed: int = 0xC1, symbols: int = 1000, quantized: bool = False):
    """C1: StockStream(symbol string, price double, volume long, ts long); symbol 'S%04d' -> dict id."""
    d = draws(seed, start, n, 3)
    symbol = (d[:, 0] % np.uint64(symbols)).astype(np.int32)
    price = uniform_price(d[:, 1], quantized)
    volume = (np.uint64(1) + d[:, 2] % np.uint64(10000)).astype(np.int64)
    ts = T0 + np.arange(start, start + n, dtype=np.int64)
    return ts, [symbol, price, volume, ts.copy()]


def keyed_stream(start: int, n: int, seed: int, keys: int, events_per_ms: int, quantized: bool = False):
    """C2/C3/C4: (k int, v double, ts long) with `events_per_ms` events per event-time millisecond."""
    d = draws(seed, start, n, 2)
    k = (d[:, 0] % np.uint64(keys)).astype(np.int32)
    v = uniform_price(d[:, 1], quantized)
    ts = T0 + np.arange(start, start + n, dtype=np.int64) // events_per_ms
    return ts, [k, v, ts.copy()]


def zipf_keys(start: int, n: int, seed: int, keys: int, s: float = 1.1) -> np.ndarray:
    """C5: Zipf(s) keys over [0, keys) by inverse CDF on the continuous approximation."""
    d = draws(seed, start, n, 1)[:, 0]
    u = (d >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    # continuous inverse CDF of p(x) ~ x^-s on [1, keys+1)
    a = 1.0 - s
    hi = (keys + 1.0) ** a
    x = (1.0 + u * (hi - 1.0)) ** (1.0 / a)
    return np.minimum(np.floor(x) - 1, keys - 1).astype(np.int32)
