"""Fused D2 merge (crdt_lww_merge_unsorted / crdt_orset_merge_unsorted): one
device sort of both unsorted sides with a side bit, then a neighbour dedup.
Bit-exact against the oracle's merge of the numpy-lexsorted sides -- the same
expectation as the two-sort path (test_gpu_sort.py) -- across composite widths
of 1, 2 and 3 words, dedup tile edges, empty sides, cross-side duplicate tags
with differing tombs, and a full config-D pair checked by the two-sort path."""
import numpy as np
import pytest
from knobs import set_knob

from crdt_amd import synth
from crdt_amd.engine import TupleSet
from oracle import oracle

pytestmark = pytest.mark.gpu

MODES = [("lww", oracle.lww_merge), ("orset", oracle.orset_merge)]


def _np_sorted(t):
    o = np.lexsort((t[3], t[2], t[1], t[0]))
    return tuple(np.ascontiguousarray(x[o]) for x in t)


def _empty():
    return (np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.uint8))


def _check(eng, ua, ub):
    A = TupleSet.from_numpy(*ua, eng.device)
    B = TupleSet.from_numpy(*ub, eng.device)
    sa, sb = _np_sorted(ua), _np_sorted(ub)
    for name, ref in MODES:
        fn = getattr(eng, f"{name}_merge_unsorted")
        got = fn(A, B).to_numpy()
        exp = ref(sa, sb)
        for g, e, f in zip(got, exp, ("key", "ts", "rep", "tomb")):
            np.testing.assert_array_equal(g, e, err_msg=f"{name} {f}")
    assert eng.device_status() == 0


@pytest.mark.parametrize("na,nb", [(1, 0), (0, 1), (1, 1), (2047, 1), (1024, 1024), (1025, 1024),
                                   (4096, 4097), (30_000, 7), (100_000, 120_000)])
def test_unsorted_config_d_shape(eng, na, nb):
    ks = max(1, (na + nb) // 3)
    _check(eng, synth.set_tuples(5 + na, 0, na, ks), synth.set_tuples(5 + na, 1, nb, ks))


def test_unsorted_empty_both(eng):
    A = TupleSet.from_numpy(*_empty(), eng.device)
    for name, _ in MODES:
        out = getattr(eng, f"{name}_merge_unsorted")(A, A)
        assert len(out) == 0


def test_unsorted_cross_side_duplicates(eng):
    """Identical tags on both sides and within a side, tombs differing: the
    LWW winner's tomb comes from A's lowest-tomb copy; OR ORs every copy."""
    rng = np.random.default_rng(9)
    n = 20_000
    key = rng.integers(0, 300, n, dtype=np.uint64)
    ts = rng.integers(0, 4, n, dtype=np.uint64)
    rep = rng.integers(0, 3, n, dtype=np.uint64).astype(np.uint32)
    ta = rng.integers(0, 2, n, dtype=np.uint8)
    tb = rng.integers(0, 2, n, dtype=np.uint8)
    perm = rng.permutation(n)
    _check(eng, (key, ts, rep, ta), (key[perm], ts[perm], rep[perm], tb[perm]))


def test_unsorted_two_and_three_words(eng):
    rng = np.random.default_rng(10)
    n = 40_000
    for kbits, tbits, rbits in ((40, 30, 10), (64, 64, 32)):
        def side(m):
            key = rng.integers(0, 2**kbits, m, dtype=np.uint64)
            key[: m // 10] = key[m // 10: 2 * (m // 10)]          # key ties
            ts = rng.integers(0, 2**tbits, m, dtype=np.uint64)
            rep = rng.integers(0, 2**rbits, m, dtype=np.uint64).astype(np.uint32)
            return key, ts, rep, rng.integers(0, 2, m, dtype=np.uint8)
        a = side(n)
        b = side(n - 3)
        b[0][:500] = a[0][:500]                                    # cross-side equal tags
        b[1][:500] = a[1][:500]
        b[2][:500] = a[2][:500]
        _check(eng, a, b)


def test_unsorted_extremes(eng):
    key = np.array([0, 2**64 - 1, 2**63, 0, 2**64 - 1], np.uint64)
    ts = np.array([2**64 - 1, 0, 5, 2**64 - 1, 1], np.uint64)
    rep = np.array([2**32 - 1, 0, 1, 2**32 - 1, 0], np.uint32)
    tomb = np.array([1, 0, 1, 0, 1], np.uint8)
    _check(eng, (key, ts, rep, tomb), (key[::-1].copy(), ts[::-1].copy(), rep[::-1].copy(), tomb))


def test_unsorted_full_config_d_equals_two_sort_path(eng):
    n, ks = 10_000_000, 8_000_000
    UA = eng.synth_set_tuples(2024, 0, n, ks, sort=False)
    UB = eng.synth_set_tuples(2024, 1, n, ks, sort=False)
    A, B = eng.sort_tuples(UA), eng.sort_tuples(UB)
    for name in ("lww", "orset"):
        ref = getattr(eng, f"{name}_merge")(A, B)
        got = getattr(eng, f"{name}_merge_unsorted")(UA, UB)
        assert len(got) == len(ref)
        for g, e in zip((got.key, got.ts, got.rep, got.tomb), (ref.key, ref.ts, ref.rep, ref.tomb)):
            assert bool((g == e).all())


@pytest.mark.parametrize("n", [1, 5000])
def test_unsorted_single_tag(eng, n):
    """Every tuple the same tag (only side and tomb differ): no tag bit to sort
    on, one composing pass; LWW takes A's least tomb, OR-Set ORs them all."""
    rng = np.random.default_rng(n)
    k = np.full(n, 7, np.uint64)
    t = np.full(n, 2**40, np.uint64)
    r = np.full(n, 3, np.uint32)
    _check(eng, (k, t, r, rng.integers(0, 2, n, dtype=np.uint8)), (k.copy(), t.copy(), r.copy(),
                                                                  rng.integers(0, 2, n, dtype=np.uint8)))
    _check(eng, (k[:0], t[:0], r[:0], np.zeros(0, np.uint8)), (k, t, r, np.ones(n, np.uint8)))


def test_unsorted_run_lengths_around_the_mark_limit(eng):
    """OR-Set D2 marks runs of up to 32 tuples element-wise (unsorted) and
    rank-sorts longer ones in LDS first: key runs of 1..70 tuples (so 32 / 33
    on both sides of the limit, and runs crossing the 2048-tuple tile
    nominal edges), duplicate tags with differing tombs and sides inside
    every run, shuffled."""
    rng = np.random.default_rng(33)
    lens = np.concatenate([np.arange(1, 71), rng.integers(1, 40, 3000)])
    key = np.repeat(np.arange(len(lens), dtype=np.uint64) * 7, lens)
    m = len(key)
    ts = rng.integers(0, 5, m, dtype=np.uint64)
    rep = rng.integers(0, 3, m, dtype=np.uint64).astype(np.uint32)
    tomb = rng.integers(0, 2, m, dtype=np.uint8)
    side = rng.integers(0, 2, m).astype(bool)
    p = rng.permutation(m)
    key, ts, rep, tomb, side = key[p], ts[p], rep[p], tomb[p], side[p]
    a = tuple(np.ascontiguousarray(x[~side]) for x in (key, ts, rep, tomb))
    b = tuple(np.ascontiguousarray(x[side]) for x in (key, ts, rep, tomb))
    _check(eng, a, b)


@pytest.mark.diag
@pytest.mark.parametrize("mode", [0, 1, 2])
def test_unsorted_orset_sort_modes(eng, mode):
    """sort.or_key_only: 0 the full tag sort + neighbour dedup; 1 key bits only,
    key runs marked in LDS; 2 (default) the key and one more tag digit, groups
    of equal sorted bits marked in LDS.  All == the oracle."""
    from crdt_amd import _lib
    set_knob(b"sort.or_key_only", mode)
    set_knob(b"sort.or_table", 0)
    try:
        ks = 30_000
        _check(eng, synth.set_tuples(71, 0, 100_000, ks), synth.set_tuples(71, 1, 90_000, ks))
        test_unsorted_cross_side_duplicates(eng)
        test_unsorted_run_lengths_around_the_mark_limit(eng)
        test_unsorted_single_tag(eng, 5000)
    finally:
        set_knob(b"sort.or_key_only", 2)
        set_knob(b"sort.or_table", 1)


@pytest.mark.diag
@pytest.mark.parametrize("kbits,tbits", [(11, 20), (12, 20), (16, 20), (20, 8), (23, 20), (24, 20),
                                         (16, 40), (22, 40), (23, 40)])
def test_unsorted_lww_key_tables(eng, kbits, tbits):
    """LWW D2 by key-bucket LDS tables (sort.lww_table; taken when the key
    offsets span 12..23 bits with tags of <= 31 bits, 12..22 bits with wider
    tags; 11 / 24 key bits and 23 bits with wide tags keep the key-only
    sort) and OR-Set D2 by key chunks sorted in LDS (sort.or_table; 16..25
    key bits, <= 1280 tuples per 2^9-key chunk on average): with both on and off == the
    oracle.  Keys offset far from 0 and spanning their full width, 80 % of
    the tuples in one key bucket, cross-side equal tags with differing
    tombs, one side shorter."""
    from crdt_amd import _lib
    rng = np.random.default_rng(kbits * 100 + tbits)

    def side(m):
        key = rng.integers(0, 2**kbits, m, dtype=np.uint64)
        hot = rng.random(m) < 0.8                                  # one hot bucket (top key byte 0)
        key[hot] = rng.integers(0, 2**max(kbits - 8, 1), int(hot.sum()), dtype=np.uint64)
        key[:2] = [0, 2**kbits - 1]
        ts = rng.integers(0, 2**tbits, m, dtype=np.uint64)
        ts[:2] = [0, 2**tbits - 1]
        rep = rng.integers(0, 40, m, dtype=np.uint64).astype(np.uint32)
        tomb = rng.integers(0, 2, m, dtype=np.uint8)
        return key + np.uint64(2**61), ts + np.uint64(12345), rep + np.uint32(7), tomb

    a, b = side(150_000), side(130_000)
    for f in range(3):                                            # cross-side equal tags
        b[f][:5000] = a[f][:5000]
    try:
        for on in (1, 0):
            set_knob(b"sort.lww_table", on)
            set_knob(b"sort.or_table", on)
            _check(eng, a, b)
            _check(eng, a, tuple(x[:0] for x in b))
    finally:
        set_knob(b"sort.lww_table", 1)
        set_knob(b"sort.or_table", 1)


def _keyed(rng, keys, tbits=6):
    m = len(keys)
    ts = rng.integers(0, 2**tbits, m, dtype=np.uint64)
    rep = rng.integers(0, 3, m, dtype=np.uint64).astype(np.uint32)
    tomb = rng.integers(0, 2, m, dtype=np.uint8)
    side = rng.integers(0, 2, m).astype(bool)
    p = rng.permutation(m)
    keys, ts, rep, tomb, side = keys[p], ts[p], rep[p], tomb[p], side[p]
    a = tuple(np.ascontiguousarray(x[~side]) for x in (keys, ts, rep, tomb))
    b = tuple(np.ascontiguousarray(x[side]) for x in (keys, ts, rep, tomb))
    return a, b


@pytest.mark.diag
@pytest.mark.parametrize("case", ["long_keys", "key_of_2000", "too_many_long_keys", "chunk_over_cap"])
def test_unsorted_orset_tables_long_keys(eng, case):
    """OR-Set key chunks sorted in LDS around their limits (20 key bits:
    2048 chunks of 2^9 keys, 1536 tuples and 64 keys of over 32 tuples per
    chunk in LDS): keys of 9..60 tuples (the insertion-sorted and the
    workgroup's long-key paths, few ts values so tags repeat within a key), a
    key of 2000 tuples, 300 keys of 9 tuples in one chunk and one chunk of
    9000+ tuples: the last three chunks are over the LDS capacity and fall
    back to the radix sort.  All == the oracle: chunks with look-back
    offsets, chunks with the scan + emit pass, and the radix path."""
    from crdt_amd import _lib
    rng = np.random.default_rng({"long_keys": 1, "key_of_2000": 2, "too_many_long_keys": 3, "chunk_over_cap": 4}[case])
    bg = rng.integers(0, 2**20, 150_000, dtype=np.uint64)
    if case == "long_keys":
        extra = np.repeat(rng.choice(2**20, 400, replace=False).astype(np.uint64), rng.integers(9, 61, 400))
    elif case == "key_of_2000":
        extra = np.full(2000, 77, np.uint64)
    elif case == "too_many_long_keys":
        extra = np.repeat(np.arange(300, dtype=np.uint64), 9)
    else:
        extra = np.full(9000, 5, np.uint64)
    a, b = _keyed(rng, np.concatenate([bg, extra, np.array([2**20 - 1], np.uint64)]))
    try:
        for on, lb in ((1, 1), (1, 0), (0, 1)):
            set_knob(b"sort.or_table", on)
            set_knob(b"sort.or_lookback", lb)
            _check(eng, a, b)
    finally:
        set_knob(b"sort.or_table", 1)
        set_knob(b"sort.or_lookback", 1)


@pytest.mark.diag
@pytest.mark.parametrize("outlier", [False, True])
def test_unsorted_sampled_plans(eng, outlier):
    """The dense-key D2 paths from a sampled plan (sort.sample_plan; forced on
    these small calls by sort.sample_min = 0): 200k / 180k tuples, keys in
    2^20, ts in 2^24, cross-side equal tags.  With an outlier key and ts at
    an index the sample (256 runs of 64 tuples per side) skips, the upsweep
    flags the miss and the call is redone from the exact plan (the wide ts
    then keeps LWW off its tables).  == the oracle, sampling on and off."""
    from crdt_amd import _lib
    rng = np.random.default_rng(77 + outlier)

    def side(m):
        return (rng.integers(0, 2**20, m, dtype=np.uint64), rng.integers(0, 2**24, m, dtype=np.uint64),
                rng.integers(0, 50, m, dtype=np.uint64).astype(np.uint32), rng.integers(0, 2, m, dtype=np.uint8))

    a, b = side(200_000), side(180_000)
    for f in range(3):
        b[f][:3000] = a[f][:3000]
    if outlier:
        a[0][100] = 2**22          # (sampled: 256 runs of 64 tuples per side, ~784 / ~706 apart from index 0)
        b[1][100] = 2**40
    try:
        set_knob(b"sort.sample_min", 0)
        for on in (1, 0):
            set_knob(b"sort.sample_plan", on)
            _check(eng, a, b)
    finally:
        set_knob(b"sort.sample_plan", 1)
        set_knob(b"sort.sample_min", 1 << 20)



def test_unsorted_refuses_out_aliasing_an_input(eng):
    """The dense-key D2 forms store into out before they know whether the
    call is redone from the inputs, so out may not overlap a or b: refused
    with CRDT_E_INVAL, the inputs untouched; a disjoint view of
    the same allocation is fine."""
    from crdt_amd import _lib
    ua = synth.set_tuples(91, 0, 3000, 1000)
    ub = synth.set_tuples(91, 1, 2000, 1000)
    n = 5000
    big = TupleSet.from_numpy(*(np.concatenate([x, y, x, y]) for x, y in zip(ua, ub)), eng.device)
    A = TupleSet(big.key[:3000], big.ts[:3000], big.rep[:3000], big.tomb[:3000])
    B = TupleSet(big.key[3000:n], big.ts[3000:n], big.rep[3000:n], big.tomb[3000:n])
    sa, sb = _np_sorted(ua), _np_sorted(ub)
    for name, ref in MODES:
        fn = getattr(eng, f"{name}_merge_unsorted")
        for lo in (0, 2000, 4999):                       # out over a, over both, over b's last tuple
            out = TupleSet(big.key[lo:lo + n], big.ts[lo:lo + n], big.rep[lo:lo + n], big.tomb[lo:lo + n])
            with pytest.raises(_lib.CrdtError):
                fn(A, B, out=out)
        np.testing.assert_array_equal(A.to_numpy()[0], ua[0])
        np.testing.assert_array_equal(B.to_numpy()[0], ub[0])
        out = TupleSet(big.key[n:], big.ts[n:], big.rep[n:], big.tomb[n:])   # disjoint: the second copy
        got = fn(A, B, out=out).to_numpy()
        for g, e in zip(got, ref(sa, sb)):
            np.testing.assert_array_equal(g, e)


@pytest.mark.diag
def test_unsorted_plan_cache_shape_changes(eng):
    """sort.plan_cache: a sampled dense-key call launches from the last such
    call's plan shape with no read-back, the device checking the fresh plan
    against it.  Calls of one size whose key / ts widths change between calls
    (a shape mismatch: the call is redone from the exact plan and the cache
    dropped), alternating modes, and a repeat of each == the oracle."""
    from crdt_amd import _lib
    rng = np.random.default_rng(123)

    def side(m, kbits, tbits):
        return (rng.integers(0, 2**kbits, m, dtype=np.uint64), rng.integers(0, 2**tbits, m, dtype=np.uint64),
                rng.integers(0, 50, m, dtype=np.uint64).astype(np.uint32), rng.integers(0, 2, m, dtype=np.uint8))

    try:
        set_knob(b"sort.sample_min", 0)
        for kbits, tbits in ((20, 20), (20, 20), (21, 20), (18, 24), (18, 24), (20, 20)):
            a, b = side(120_000, kbits, tbits), side(120_000, kbits, tbits)
            for f in range(3):
                b[f][:2000] = a[f][:2000]
            _check(eng, a, b)
    finally:
        set_knob(b"sort.sample_min", 1 << 20)
