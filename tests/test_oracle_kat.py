"""CPU: the oracle's build-defined CRDT joins against hand-derived KATs,
plus algebraic properties (idempotence, commutativity, associativity) on
seeded inputs -- the oracle is the checker every GPU parity test trusts."""
import numpy as np
import pytest

from crdt_amd import synth
from kat_util import load, tuples, tuples_list, u64
from oracle import oracle

K = load()


@pytest.mark.parametrize("i", range(len(K["gcounter_join"])))
def test_join_kat(i):
    k = K["gcounter_join"][i]
    np.testing.assert_array_equal(oracle.gcounter_join(u64(k["a"]), u64(k["b"])), u64(k["out"]))


@pytest.mark.parametrize("i", range(len(K["gcounter_fold"])))
def test_fold_kat(i):
    k = K["gcounter_fold"][i]
    np.testing.assert_array_equal(oracle.gcounter_fold(u64(k["a"])), u64(k["out"]))


@pytest.mark.parametrize("i", range(len(K["pncounter_value"])))
def test_pn_kat(i):
    k = K["pncounter_value"][i]
    np.testing.assert_array_equal(oracle.pncounter_value(u64(k["p"]), u64(k["n"])), np.array(k["out"], np.int64))


@pytest.mark.parametrize("i", range(len(K["vclock_classify"])))
def test_vclock_kat(i):
    k = K["vclock_classify"][i]
    np.testing.assert_array_equal(oracle.vclock_classify(u64(k["a"]), u64(k["b"])), np.array(k["out"], np.uint8))


@pytest.mark.parametrize("kind", ["lww_merge", "orset_merge"])
def test_set_kats(kind):
    fn = getattr(oracle, kind)
    for k in K[kind]:
        assert tuples_list(fn(tuples(k["a"]), tuples(k["b"]))) == k["out"], k


def test_join_lattice_properties():
    n = 64 * 2000
    a, b, c = (synth.counters(4, s, n).reshape(-1, 64) for s in (1, 2, 3))
    j = oracle.gcounter_join
    np.testing.assert_array_equal(j(a, a), a)                       # idempotent
    np.testing.assert_array_equal(j(a, b), j(b, a))                 # commutative
    np.testing.assert_array_equal(j(j(a, b), c), j(a, j(b, c)))     # associative
    np.testing.assert_array_equal(oracle.gcounter_fold(np.vstack([a, b])),
                                  j(oracle.gcounter_fold(a)[None], oracle.gcounter_fold(b)[None])[0])
    np.testing.assert_array_equal(j(a, b, threads=4), j(a, b))


def test_vclock_antisymmetry_and_distribution():
    a, b = synth.vclock_pairs(8, 4000, 128)
    f = oracle.vclock_classify(a, b)
    r = oracle.vclock_classify(b, a)
    np.testing.assert_array_equal(r, np.array([0, 2, 1, 3], np.uint8)[f])
    np.testing.assert_array_equal(oracle.vclock_classify(a, a), np.zeros(4000, np.uint8))
    assert np.all(np.abs(np.bincount(f, minlength=4) / 4000 - 0.25) < 0.05)
    np.testing.assert_array_equal(oracle.vclock_classify(a, b, threads=3), f)


def test_set_merge_properties():
    sa = synth.sort_tuples_np(*synth.set_tuples(9, 0, 20000, 5000))
    sb = synth.sort_tuples_np(*synth.set_tuples(9, 1, 20000, 5000))
    empty = tuples([])
    lww_ab = oracle.lww_merge(sa, sb)
    # LWW output: one tuple per distinct key, keys strictly increasing
    assert np.all(np.diff(lww_ab[0].astype(np.float64)) > 0)
    assert len(lww_ab[0]) == len(np.unique(np.concatenate([sa[0], sb[0]])))
    # idempotence: merging a canonical state with itself changes nothing
    np.testing.assert_array_equal(oracle.lww_merge(lww_ab, lww_ab)[0], lww_ab[0])
    # OR-Set: union of tags; merging with an empty side dedupes only
    or_ab = oracle.orset_merge(sa, sb)
    tags = set(zip(*[x.tolist() for x in sa[:3]])) | set(zip(*[x.tolist() for x in sb[:3]]))
    assert len(or_ab[0]) == len(tags)
    or_a = oracle.orset_merge(sa, empty)
    for x, y in zip(oracle.orset_merge(or_a, or_a), or_a):
        np.testing.assert_array_equal(x, y)
    # commutativity of the OR-Set (tombs OR-ed; no tie rule involved)
    for x, y in zip(oracle.orset_merge(sb, sa), or_ab):
        np.testing.assert_array_equal(x, y)


def test_synth_set_dup_fraction():
    ka, ta, ra, _ = synth.set_tuples(3, 0, 100000, 8_000_000)
    kb, tb, rb, _ = synth.set_tuples(3, 1, 100000, 8_000_000)
    same = (ka == kb) & (ta == tb) & (ra == rb)
    assert abs(same.mean() - 0.05) < 0.01
