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


ALPHABET = "abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ1234567890"   # main.go:274
_ODD_VALUES = ["+5", "007", "-0", "x", "", "9223372036854775807", "-9223372036854775808",
               "9223372036854775808", "1_0", " 3", "00000000000000000000042", "+", "--1"]


def refmerge_demo(seed: int, replicas: int = 5, entries: int = 10_000, multi_key: float = 0.0):
    """Config A (BASELINE configs[0]): the reference demo's workload shape.

    Per replica: a local Diff of `entries` ts with gaps U[1,4] (UnixMilli-like
    start), half local writes (*Command, main.go:187) and half previously
    merged remote maps; a RemoteDiff from a peer with ~5% ts collisions with
    the local log and ~10% of its ts above max(L).  Each entry holds one key
    of the 62-char alphabet (main.go:274) with a value in [-20, -11]
    (main.go:282), ~1% non-canonical / unparsable strings, and a
    `multi_key` fraction of entries hold 2-4 keys.
    Returns [(diff, remote), ...] with crdt_amd.refmerge.Command marking
    local writes.
    """
    from .refmerge import Command
    out = []
    for p in range(replicas):
        rng = np.random.default_rng([seed, p])

        def kv():
            nk = int(rng.integers(2, 5)) if rng.random() < multi_key else 1
            d = {}
            for _ in range(nk):
                k = ALPHABET[int(rng.integers(0, len(ALPHABET)))]
                if rng.random() < 0.01:
                    d[k] = _ODD_VALUES[int(rng.integers(0, len(_ODD_VALUES)))]
                else:
                    d[k] = str(int(rng.integers(0, 10)) + 2 * (-10))
            return d

        t0 = 1_700_000_000_000 + int(rng.integers(0, 1000))
        lts = t0 + np.cumsum(rng.integers(1, 5, size=entries))
        diff = {}
        for t in lts.tolist():
            diff[t] = Command(kv()) if rng.random() < 0.5 else kv()
        n_r = entries
        hi = int(lts[-1]) if entries else t0
        n_above = int(round(0.10 * n_r))
        n_coll = int(round(0.05 * n_r))
        rts = set((t0 + np.cumsum(rng.integers(1, 5, size=n_r - n_above - n_coll))).tolist())
        if entries:
            rts |= set(rng.choice(lts, size=min(n_coll, entries), replace=False).tolist())
        rts |= set((hi + np.cumsum(rng.integers(1, 5, size=n_above))).tolist())
        remote = {int(t): kv() for t in sorted(rts)}
        out.append((diff, remote))
    return out


def refmerge_packed(seed: int, replicas: int, entries: int):
    """Config A's workload shape at scale, generated directly in the packed
    CSR layout of crdt_refmerge_in (vectorised; one kv per entry as the
    reference's load generator sends, main.go:281-286).

    Per replica: L = `entries` ts with gaps U[1,4], origin local w.p. 1/2;
    R = `entries` ts: 85% own-clock, 5% colliding with L, 10% above max(L).
    Values: "-20".."-11" (main.go:282) plus ~1% odd strings; keys: 62 slots
    per replica (main.go:274).  Returns the dict Engine.refmerge_batch takes
    (numpy arrays; move with refmerge.to_device).
    """
    rng = np.random.default_rng(seed)
    P, E = replicas, entries
    strs = [str(v) for v in range(-20, -10)] + _ODD_VALUES
    blob = "".join(strs).encode()
    str_off = np.zeros(len(strs) + 1, np.int64)
    str_off[1:] = np.cumsum([len(s.encode()) for s in strs])
    t0 = 1_700_000_000_000 + rng.integers(0, 1000, size=(P, 1))
    l_ts = t0 + np.cumsum(rng.integers(1, 5, size=(P, E)), axis=1)
    l_origin = (rng.random((P, E)) < 0.5).astype(np.uint8)
    n_above, n_coll = E // 10, E // 20
    n_own = E - n_above - n_coll
    own = t0 + np.cumsum(rng.integers(1, 5, size=(P, n_own)), axis=1)
    coll = np.take_along_axis(l_ts, rng.integers(0, E, size=(P, n_coll)), axis=1)
    above = l_ts[:, -1:] + np.cumsum(rng.integers(1, 5, size=(P, n_above)), axis=1)
    r_all = np.sort(np.concatenate([own, coll, above], axis=1), axis=1)
    # unique per replica: bump duplicates by rebuilding each row's unique set
    r_rows = [np.unique(r) for r in r_all]
    r_off = np.zeros(P + 1, np.int64)
    r_off[1:] = np.cumsum([len(r) for r in r_rows])
    r_ts = np.concatenate(r_rows).astype(np.int64)
    n_l, n_r = P * E, int(r_off[-1])

    def vals(n):
        v = rng.integers(0, 10, size=n)
        odd = rng.random(n) < 0.01
        v[odd] = 10 + rng.integers(0, len(_ODD_VALUES), size=int(odd.sum()))
        return v.astype(np.uint32)

    l_rep = np.repeat(np.arange(P, dtype=np.int64), E)
    r_rep = np.repeat(np.arange(P, dtype=np.int64), np.diff(r_off))
    kv_key = np.concatenate([l_rep * 62 + rng.integers(0, 62, size=n_l),
                             r_rep * 62 + rng.integers(0, 62, size=n_r)]).astype(np.uint32)
    kv_val = np.concatenate([vals(n_l), vals(n_r)])
    return {
        "replicas": P, "n_slots": P * 62,
        "l_off": np.arange(0, n_l + 1, E, dtype=np.int64), "l_ts": l_ts.reshape(-1).astype(np.int64),
        "l_origin": l_origin.reshape(-1), "l_kv": np.arange(n_l + 1, dtype=np.int64),
        "r_off": r_off, "r_ts": r_ts, "r_kv": np.arange(n_l, n_l + n_r + 1, dtype=np.int64),
        "kv_key": kv_key.view(np.int32), "kv_val": kv_val.view(np.int32),
        "str_bytes": np.frombuffer(blob, np.uint8).copy(), "str_off": str_off,
    }


def sort_tuples_np(key, ts, rep, tomb):
    """Stable (key, ts, rep) sort of numpy SoA tuples."""
    order = np.lexsort((rep, ts, key))  # lexsort is stable; last key is primary
    return key[order], ts[order], rep[order], tomb[order]
