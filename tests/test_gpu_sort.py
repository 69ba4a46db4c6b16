"""GPU tuple sort (crdt_tuples_sort, config D2): bit-exact against numpy's
lexsort on (key, ts, rep, tomb), across composite widths of 1, 2 and 3
words, tile edges, duplicates and a full config-D side; plus the D2 path
end to end (sort both unsorted sides, then merge) against the oracle."""
import numpy as np
import pytest

from crdt_amd import synth
from crdt_amd.engine import TupleSet
from oracle import oracle

pytestmark = pytest.mark.gpu


def _np_sorted(key, ts, rep, tomb):
    o = np.lexsort((tomb, rep, ts, key))
    return key[o], ts[o], rep[o], tomb[o]


def _check(eng, t):
    got = eng.sort_tuples(TupleSet.from_numpy(*t, eng.device)).to_numpy()
    exp = _np_sorted(*t)
    for g, e, f in zip(got, exp, ("key", "ts", "rep", "tomb")):
        np.testing.assert_array_equal(g, e, err_msg=f)
    assert eng.device_status() == 0


@pytest.mark.parametrize("n", [1, 2, 255, 4095, 4096, 4097, 12_289, 200_000])
def test_sort_config_d_shape(eng, n):
    _check(eng, synth.set_tuples(11 + n, 1, n, max(1, n // 2)))


def test_sort_wide_fields_three_words(eng):
    """Full-range 64-bit keys and ts and 32-bit reps: a 161-bit composite."""
    rng = np.random.default_rng(3)
    n = 50_000
    key = rng.integers(0, 2**64, n, dtype=np.uint64)
    key[:100] = key[100:200]                        # key ties
    ts = rng.integers(0, 2**64, n, dtype=np.uint64)
    ts[0], ts[1] = 0, 2**64 - 1
    rep = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    tomb = rng.integers(0, 2, n, dtype=np.uint8)
    _check(eng, (key, ts, rep, tomb))


def test_sort_two_words(eng):
    rng = np.random.default_rng(4)
    n = 30_000
    key = rng.integers(0, 2**40, n, dtype=np.uint64)
    ts = rng.integers(0, 2**30, n, dtype=np.uint64)
    rep = rng.integers(0, 2**10, n, dtype=np.uint64).astype(np.uint32)
    tomb = rng.integers(0, 2, n, dtype=np.uint8)
    _check(eng, (key, ts, rep, tomb))


def test_sort_duplicates_and_single_pass(eng):
    """Identical tags differing only in tomb; and a composite of <= 8 bits."""
    n = 9_000
    key = np.full(n, 7, np.uint64)
    ts = np.full(n, 2**63, np.uint64)
    rep = (np.arange(n) % 5).astype(np.uint32)
    tomb = (np.arange(n) % 2).astype(np.uint8)
    _check(eng, (key, ts, rep, tomb))


def test_sort_full_config_d_side(eng):
    n, ks = 10_000_000, 8_000_000
    t = synth.set_tuples(2024, 1, n, ks)
    got = eng.sort_tuples(TupleSet.from_numpy(*t, eng.device))
    assert eng.count_unsorted(got) == 0
    g = got.to_numpy()
    e = _np_sorted(*t)
    for a, b in zip(g, e):
        np.testing.assert_array_equal(a, b)


def test_d2_unsorted_merge_end_to_end(eng):
    """Config D2: unsorted sides -> device sort -> LWW / OR-Set merge."""
    n, ks = 300_000, 200_000
    ua = synth.set_tuples(77, 0, n, ks)
    ub = synth.set_tuples(77, 1, n, ks)
    A = eng.sort_tuples(TupleSet.from_numpy(*ua, eng.device))
    B = eng.sort_tuples(TupleSet.from_numpy(*ub, eng.device))
    sa, sb = _np_sorted(*ua), _np_sorted(*ub)
    for fn, ref in ((eng.lww_merge, oracle.lww_merge), (eng.orset_merge, oracle.orset_merge)):
        got = fn(A, B).to_numpy()
        exp = ref(sa, sb)
        for g, e in zip(got, exp):
            np.testing.assert_array_equal(g, e)
