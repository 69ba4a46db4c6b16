"""Host (numpy) restatement of the device generators in csrc/synth.hip.

Element i of every synthetic stream is a pure function of (seed, stream, i),
SplitMix64-based, so tests can regenerate any sample of a
device-resident input on the host and check the two agree bit for bit.
"""
from __future__ import annotations

import numpy as np

GAMMA = np.uint64(0x9E3779B97F4A7C15)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = x + GAMMA
        x = (x ^ (x >> np.uint64(30))) * M1
        x = (x ^ (x >> np.uint64(27))) * M2
    return x ^ (x >> np.uint64(31))


def stream_key(seed: int, stream: int) -> np.uint64:
    return splitmix64(np.uint64(seed) ^ splitmix64(np.uint64(stream)))


def rnd(k, i):
    i = np.asarray(i, dtype=np.uint64)
    with np.errstate(over="ignore"):
        return splitmix64(np.uint64(k) + i * GAMMA)


_SPECIAL = np.array([0, 0x7FFFFFFFFFFFFFFF, 0x8000000000000000, 0xFFFFFFFFFFFFFFFF], dtype=np.uint64)


def counters(seed: int, stream: int, n: int, index_base: int = 0) -> np.ndarray:
    """G-Counter cells: 1/8 full-range, rest < 2^20, ~1/1024 planted edges."""
    k = stream_key(seed, stream)
    i = np.arange(index_base, index_base + n, dtype=np.uint64)
    x = rnd(k, i)
    out = (x >> np.uint64(20)) & np.uint64(0xFFFFF)
    full = (x >> np.uint64(61)) == 0
    out = np.where(full, rnd(k ^ np.uint64(0xA5A5A5A5A5A5A5A5), i), out)
    planted = (x & np.uint64(0x3FF)) == np.uint64(0x3FF)
    out = np.where(planted, _SPECIAL[((x >> np.uint64(10)) & np.uint64(3)).astype(np.int64)], out)
    return out.astype(np.uint64)


def vclock_pairs(seed: int, pairs: int, nodes: int, pair_base: int = 0):
    """(a, b) clocks [pairs x nodes]: 25% each of EQUAL/BEFORE/AFTER/CONCURRENT."""
    kb, kc = stream_key(seed, 10), stream_key(seed, 11)
    p = np.arange(pair_base, pair_base + pairs, dtype=np.uint64)[:, None]
    kk = np.arange(nodes, dtype=np.uint64)[None, :]
    with np.errstate(over="ignore"):
        base = rnd(kb, p * np.uint64(nodes) + kk) & np.uint64(0xFFFFFFFF)
    h = rnd(kc, p)
    cls = h & np.uint64(3)
    jj = (h >> np.uint64(8)) % np.uint64(nodes - 1) if nodes > 1 else np.zeros_like(h)
    big = ((h >> np.uint64(32)) & np.uint64(1023)) == 0
    base = np.where(big, np.uint64(0xFFFFFFFFFFFFFFFE) - (base & np.uint64(0xFF)), base)
    a = base.copy()
    b = base.copy()
    last = np.uint64(nodes - 1)
    one = np.uint64(1)
    is_last = kk == last
    b = np.where((cls == 1) & is_last, b + one, b)
    a = np.where((cls == 2) & is_last, a + one, a)
    b = np.where((cls == 3) & is_last, b + one, b)
    a = np.where((cls == 3) & (kk == jj), a + one, a)
    return a.astype(np.uint64), b.astype(np.uint64)


def set_tuples(seed: int, side: int, n: int, key_space: int):
    """Unsorted (key, ts, rep, tomb) tuples of one side (0 = A, 1 = B)."""
    s0 = side * 8
    i = np.arange(n, dtype=np.uint64)
    ks = np.uint64(key_space)
    key = rnd(stream_key(seed, 20 + s0), i) % ks
    ts = rnd(stream_key(seed, 21 + s0), i) & np.uint64(0xFFFFF)
    rep = (rnd(stream_key(seed, 22 + s0), i) & np.uint64(63)).astype(np.uint32)
    if side != 0:
        dup = rnd(stream_key(seed, 40), i) % np.uint64(20) == 0
        key = np.where(dup, rnd(stream_key(seed, 20), i) % ks, key)
        ts = np.where(dup, rnd(stream_key(seed, 21), i) & np.uint64(0xFFFFF), ts)
        rep = np.where(dup, (rnd(stream_key(seed, 22), i) & np.uint64(63)).astype(np.uint32), rep)
    tomb = (rnd(stream_key(seed, 23 + s0), i) % np.uint64(10) == 0).astype(np.uint8)
    return key.astype(np.uint64), ts.astype(np.uint64), rep.astype(np.uint32), tomb


def sort_tuples_np(key, ts, rep, tomb):
    """Stable (key, ts, rep) sort of numpy SoA tuples."""
    order = np.lexsort((rep, ts, key))  # lexsort is stable; last key is primary
    return key[order], ts[order], rep[order], tomb[order]
