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


def hi53(u: np.ndarray) -> np.ndarray:
    """Top 53 bits of a draw (non-negative as int64, so the device generator can use signed ops)."""
    return u >> np.uint64(11)


def c1_stock(start: int, n: int, seed: int = 0xC1, symbols: int = 1000, quantized: bool = False):
    """C1: StockStream(symbol string, price double, volume long, ts long); symbol 'S%04d' -> dict id."""
    d = draws(seed, start, n, 3)
    symbol = (hi53(d[:, 0]) % np.uint64(symbols)).astype(np.int32)
    price = uniform_price(d[:, 1], quantized)
    volume = (np.uint64(1) + hi53(d[:, 2]) % np.uint64(10000)).astype(np.int64)
    ts = T0 + np.arange(start, start + n, dtype=np.int64)
    return ts, [symbol, price, volume, ts.copy()]


def keyed_stream(start: int, n: int, seed: int, keys: int, events_per_ms: int, quantized: bool = False):
    """C2/C3/C4: (k int, v double, ts long) with `events_per_ms` events per event-time millisecond."""
    d = draws(seed, start, n, 2)
    k = (hi53(d[:, 0]) % np.uint64(keys)).astype(np.int32)
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


# ---- the same streams generated on the GPU with torch (bench inputs resident in HBM) --------------
def _t_lsr(x, s):
    import torch
    return (x >> s) & ((1 << (64 - s)) - 1)


def _t_mix64(z):
    c1 = 0xBF58476D1CE4E5B9 - (1 << 64)
    c2 = 0x94D049BB133111EB - (1 << 64)
    z = (z ^ _t_lsr(z, 30)) * c1
    z = (z ^ _t_lsr(z, 27)) * c2
    return z ^ _t_lsr(z, 31)


def torch_draws(seed: int, start: int, n: int, width: int, device):
    """Same values as draws() (as int64 bit patterns), computed on `device`."""
    import torch
    g = 0x9E3779B97F4A7C15 - (1 << 64)
    j = torch.arange(start * width, (start + n) * width, dtype=torch.int64, device=device) + 1
    z = (seed - (1 << 64) if seed >= (1 << 63) else seed) + j * g
    return _t_mix64(z).reshape(n, width)


def torch_zipf_stream(start: int, n: int, seed: int, keys: int, events_per_ms: int, device, s: float = 1.1):
    """C5 on the GPU: Zipf(s) keys over [0, keys) (zipf_keys' inverse CDF, float64 on the device)
    and uniform [0, 200) values; returns (ts, [k int32, v float64, ts int64]) torch tensors."""
    import torch
    d = torch_draws(seed, start, n, 2, device)
    u = _t_lsr(d[:, 0], 11).to(torch.float64) * (2.0 ** -53)
    a = 1.0 - s
    hi = (keys + 1.0) ** a
    x = (1.0 + u * (hi - 1.0)) ** (1.0 / a)
    k = torch.clamp(torch.floor(x) - 1, max=keys - 1).to(torch.int32)
    v = _t_lsr(d[:, 1], 11).to(torch.float64) * (2.0 ** -53) * 200.0
    ts = T0 + torch.arange(start, start + n, dtype=torch.int64, device=device) // events_per_ms
    return ts, [k.contiguous(), v.contiguous(), ts.clone()]


def torch_keyed_stream(start: int, n: int, seed: int, keys: int, events_per_ms: int, device):
    """keyed_stream() on the GPU: returns (ts, [k int32, v float64, ts int64]) torch tensors."""
    import torch
    d = torch_draws(seed, start, n, 2, device)
    k = (_t_lsr(d[:, 0], 11) % keys).to(torch.int32)
    v = _t_lsr(d[:, 1], 11).to(torch.float64) * (2.0 ** -53) * 200.0
    ts = T0 + torch.arange(start, start + n, dtype=torch.int64, device=device) // events_per_ms
    return ts, [k.contiguous(), v.contiguous(), ts.clone()]
