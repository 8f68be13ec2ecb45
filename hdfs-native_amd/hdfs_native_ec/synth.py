"""Seeded synthetic stripe data for tests and bench (no datasets: the path's
input is raw file bytes, so synthetic bytes of the same shape are the
workload).

* splitmix64 byte streams, seed 0x5EED_EC00 + stripe;
* the reference bench's fill (rust/benches/ec.rs:19-27): shard i holds the
  big-endian i32 sequence v + i*slice_size for v in 0..slice_size/4.
"""
from __future__ import annotations

import numpy as np

SEED_BASE = 0x5EED_EC00
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64_bytes(seed: int, n: int) -> np.ndarray:
    """n bytes of the splitmix64 stream started at `seed` (little-endian words)."""
    words = (n + 7) // 8
    with np.errstate(over="ignore"):
        idx = np.arange(1, words + 1, dtype=np.uint64)
        z = np.uint64(seed) + idx * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z.astype("<u8").view(np.uint8)[:n].copy()


def stripe_data(stripe: int, units: int, cell: int) -> np.ndarray:
    """[units, cell] uint8 for one stripe."""
    return splitmix64_bytes(SEED_BASE + stripe, units * cell).reshape(units, cell)


def batch_data(stripes: int, units: int, cell: int, first: int = 0) -> np.ndarray:
    """[stripes, units, cell] uint8."""
    out = np.empty((stripes, units, cell), dtype=np.uint8)
    for s in range(stripes):
        out[s] = stripe_data(first + s, units, cell)
    return out


def bench_counter_shards(k: int, slice_size: int) -> np.ndarray:
    """rust/benches/ec.rs:19-27: buf.put_i32((v + i * slice_size) as i32),
    big-endian, for v in 0..slice_size/4."""
    out = np.empty((k, slice_size), dtype=np.uint8)
    v = np.arange(slice_size // 4, dtype=np.int64)
    for i in range(k):
        vals = ((v + i * slice_size) & 0xFFFFFFFF).astype(">u4")
        out[i] = vals.view(np.uint8)
    return out
