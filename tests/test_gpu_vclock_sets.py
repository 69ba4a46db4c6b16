"""GPU parity: vector-clock classification and LWW / OR-Set merges vs the oracle.

Build-defined types (no reference code): bit-exact against
oracle/crdt_oracle.c, whose semantics are pinned by tests/golden KATs.
"""
import numpy as np
import pytest
from knobs import set_knob
import torch

from crdt_amd import synth
from crdt_amd.engine import TupleSet, as_u64, u64_tensor
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("pairs,nodes", [(1, 128), (7, 128), (20_000, 128), (5000, 64), (3000, 32),
                                         (1000, 100), (100, 1), (50, 3), (10, 513)])
def test_vclock_matches_oracle(eng, pairs, nodes):
    a, b = synth.vclock_pairs(21, pairs, nodes)
    cls = eng.vclock_classify(u64_tensor(a, eng.device), u64_tensor(b, eng.device))
    exp = oracle.vclock_classify(a, b)
    np.testing.assert_array_equal(cls.cpu().numpy(), exp)
    # antisymmetry: classify(b, a) swaps BEFORE/AFTER
    rev = eng.vclock_classify(u64_tensor(b, eng.device), u64_tensor(a, eng.device)).cpu().numpy()
    np.testing.assert_array_equal(rev, np.array([0, 2, 1, 3], np.uint8)[exp])


def test_vclock_full_config_c_sample(eng):
    """configs[2]-shaped (128 nodes) at 2M pairs (16 MB per 1k... 4 GB total)."""
    pairs, nodes = 2_000_000, 128
    ta, tb = eng.synth_vclock_pairs(99, pairs, nodes)
    cls = eng.vclock_classify(ta, tb).cpu().numpy()
    a, b = as_u64(ta), as_u64(tb)
    np.testing.assert_array_equal(cls, oracle.vclock_classify(a, b, threads=8))
    ha, hb = synth.vclock_pairs(99, 1000, nodes, pair_base=pairs - 1000)
    np.testing.assert_array_equal(a[-1000:], ha)
    np.testing.assert_array_equal(b[-1000:], hb)
    frac = np.bincount(cls, minlength=4) / pairs
    assert np.all(np.abs(frac - 0.25) < 0.01), frac


def test_vclock_edges(eng):
    M = 2**64 - 1
    rows = [
        ([0, 0], [0, 0], 0), ([M, 0], [M, 0], 0), ([0, M], [1, M], 1), ([M, 1], [M - 1, 1], 2),
        ([2**63, 0], [2**63 - 1, 1], 3), ([2**63, 5], [2**63, 5], 0),
    ]
    a = np.array([r[0] for r in rows], dtype=np.uint64)
    b = np.array([r[1] for r in rows], dtype=np.uint64)
    cls = eng.vclock_classify(u64_tensor(a, eng.device), u64_tensor(b, eng.device)).cpu().numpy()
    np.testing.assert_array_equal(cls, [r[2] for r in rows])


def _sets(seed, na, nb, key_space):
    sa = synth.sort_tuples_np(*synth.set_tuples(seed, 0, na, key_space))
    sb = synth.sort_tuples_np(*synth.set_tuples(seed, 1, nb, key_space))
    return sa, sb


def _check(eng, sa, sb):
    A = TupleSet.from_numpy(*sa, eng.device)
    B = TupleSet.from_numpy(*sb, eng.device)
    for fn, ref in ((eng.lww_merge, oracle.lww_merge), (eng.orset_merge, oracle.orset_merge)):
        got = fn(A, B).to_numpy()
        exp = ref(sa, sb)
        for g, e, f in zip(got, exp, ("key", "ts", "rep", "tomb")):
            np.testing.assert_array_equal(g, e, err_msg=f"{fn.__name__}.{f}")


@pytest.mark.parametrize("na,nb,key_space", [
    (1, 1, 1), (0, 10, 5), (10, 0, 5), (2048, 2048, 100), (2047, 2049, 10), (5000, 3, 1000),
    (100_000, 100_000, 1), (100_000, 100_000, 7), (100_000, 100_000, 50_000), (300_000, 200_000, 10**9),
])
def test_sets_match_oracle(eng, na, nb, key_space):
    _check(eng, *_sets(31 + na + nb, na, nb, key_space))


def test_sets_identical_inputs_idempotent(eng):
    sa, _ = _sets(5, 50_000, 1, 20_000)
    _check(eng, sa, sa)
    A = TupleSet.from_numpy(*sa, eng.device)
    got = eng.orset_merge(A, A).to_numpy()
    dedup = oracle.orset_merge(sa, (sa[0][:0], sa[1][:0], sa[2][:0], sa[3][:0]))
    for g, e in zip(got, dedup):
        np.testing.assert_array_equal(g, e)


def test_sets_long_runs_cross_tiles(eng):
    # one key with 20k versions on each side: key runs and equal-tag runs cross many tiles
    n = 20_000
    ka = np.zeros(n, np.uint64)
    ta = np.repeat(np.arange(n // 4, dtype=np.uint64), 4)
    ra = np.tile(np.array([0, 0, 1, 1], np.uint32), n // 4)
    tomba = (np.arange(n) % 3 == 0).astype(np.uint8)
    sa = (ka, ta, ra, tomba)
    sb = (ka.copy(), ta.copy(), ra.copy(), (np.arange(n) % 5 == 0).astype(np.uint8))
    _check(eng, sa, sb)


def test_sets_uint64_extremes(eng):
    key = np.array([0, 5, 2**63, 2**64 - 1], np.uint64)
    ts = np.array([2**64 - 1, 0, 2**63, 1], np.uint64)
    rep = np.array([0, 2**32 - 1, 7, 7], np.uint32)
    tomb = np.array([0, 1, 0, 1], np.uint8)
    sa = (key, ts, rep, tomb)
    sb = (key.copy(), ts.copy(), rep.copy(), 1 - tomb)
    _check(eng, sa, sb)


def test_sets_full_config_d(eng):
    """configs[3] at full size: 10M tuples per side, device generated + sorted."""
    n, ks = 10_000_000, 8_000_000
    A = eng.synth_set_tuples(2024, 0, n, ks)
    B = eng.synth_set_tuples(2024, 1, n, ks)
    assert eng.count_unsorted(A) == 0 and eng.count_unsorted(B) == 0
    sa, sb = A.to_numpy(), B.to_numpy()
    ha = synth.sort_tuples_np(*synth.set_tuples(2024, 0, n, ks))
    for g, e in zip(sa, ha):
        np.testing.assert_array_equal(g, e)
    for fn, ref in ((eng.lww_merge, oracle.lww_merge), (eng.orset_merge, oracle.orset_merge)):
        got = fn(A, B).to_numpy()
        exp = ref(sa, sb)
        for g, e in zip(got, exp):
            np.testing.assert_array_equal(g, e)
    torch.cuda.synchronize()


@pytest.mark.parametrize("tiles", [8192, 8193, 9216, 16385])
def test_sets_tile_count_scan_shapes(eng, tiles):
    """The tile-count scan's shapes (k_chunk_scan): up to 8k counts a run per
    thread, above that striped rows (16 per thread), and past kScanMax
    (16384) a second scan chunk on top of the first's total.  OR-Set tiles
    are 2048 merge items, LWW tiles 4096: `tiles` OR tiles (half as many
    LWW ones) plus one item, device-generated sorted sides == the oracle."""
    n = tiles * 2048 + 1
    na, ks = n // 2 + 1, n // 3
    A = eng.synth_set_tuples(77 + tiles, 0, na, ks)
    B = eng.synth_set_tuples(77 + tiles, 1, n - na, ks)
    sa, sb = A.to_numpy(), B.to_numpy()
    for fn, ref in ((eng.orset_merge, oracle.orset_merge), (eng.lww_merge, oracle.lww_merge)):
        got = fn(A, B).to_numpy()
        exp = ref(sa, sb)
        for g, e, f in zip(got, exp, ("key", "ts", "rep", "tomb")):
            np.testing.assert_array_equal(g, e, err_msg=f"{fn.__name__}.{f}")
    torch.cuda.synchronize()


@pytest.mark.parametrize("na,nb", [(1535, 1), (1536, 1536), (1537, 1535), (3071, 3073), (4608, 0), (0, 4609)])
def test_sets_tile_boundaries(eng, na, nb):
    """Sizes around the 1536-element merge tile."""
    _check(eng, *_sets(900 + na + nb, na, nb, max(1, (na + nb) // 3)))


@pytest.mark.parametrize("off_a,off_b", [(1, 0), (3, 5), (7, 2), (13, 11)])
def test_sets_unaligned_views(eng, off_a, off_b):
    """Inputs that start mid-allocation: every segment the LDS-DMA loader
    copies then begins off a 16-byte boundary (and tombs off a 4-byte one)."""
    n = 20_000
    sa = _sets(41 + off_a, n + off_a, 0, 9_000)[0]
    sb = _sets(43 + off_b, n + off_b, 0, 9_000)[0]
    Afull = TupleSet.from_numpy(*sa, eng.device)
    Bfull = TupleSet.from_numpy(*sb, eng.device)
    A = TupleSet(Afull.key[off_a:], Afull.ts[off_a:], Afull.rep[off_a:], Afull.tomb[off_a:])
    B = TupleSet(Bfull.key[off_b:], Bfull.ts[off_b:], Bfull.rep[off_b:], Bfull.tomb[off_b:])
    ha = tuple(x[off_a:] for x in sa)
    hb = tuple(x[off_b:] for x in sb)
    for fn, ref in ((eng.lww_merge, oracle.lww_merge), (eng.orset_merge, oracle.orset_merge)):
        got = fn(A, B).to_numpy()
        exp = ref(ha, hb)
        for g, e, f in zip(got, exp, ("key", "ts", "rep", "tomb")):
            np.testing.assert_array_equal(g, e, err_msg=f"{fn.__name__}.{f}")


@pytest.mark.diag
@pytest.mark.parametrize("chunk", [0, 1, 3, 7, 64])
def test_sets_chunked_schedules(eng, chunk):
    """The count / write passes over chunks of tiles (sets.lww_chunk,
    sets.or_chunk; 0 = one chunk of up to 16384 tiles, the schedule of any
    larger call): chunk edges inside key runs, tile edges, unaligned views;
    == the oracle."""
    for name, v in ((b"sets.lww_chunk", chunk), (b"sets.or_chunk", chunk)):
        set_knob(name, v)
    try:
        _check(eng, *_sets(77, 100_000, 100_000, 50_000))
        _check(eng, *_sets(78, 4097, 4095, 1000))
        _check(eng, *_sets(79, 40_000, 1, 100))                 # long key runs across chunk edges
        test_sets_long_runs_cross_tiles(eng)
        test_sets_unaligned_views(eng, 3, 5)
        assert eng.device_status(clear=True) == 0
    finally:
        for name, v in ((b"sets.lww_chunk", 0), (b"sets.or_chunk", 0)):
            set_knob(name, v)


@pytest.mark.diag
def test_sets_inconsistent_bitmaps_raise_range(eng):
    """fail.zero_bits: the merge bitmaps zeroed between the count and write
    passes (the GPU fault of DESIGN.md §5.4's timing build): every write-pass
    workgroup finds them inconsistent with its tile and raises CRDT_DEV_RANGE
    instead of staging a run past the end of an input; the next merge is
    exact again."""
    from crdt_amd import _lib
    from crdt_amd._lib import CrdtLibraryError
    sa, sb = _sets(81, 50_000, 30_000, 20_000)
    A = TupleSet.from_numpy(*sa, eng.device)
    B = TupleSet.from_numpy(*sb, eng.device)
    for fn in (eng.lww_merge, eng.orset_merge):
        set_knob(b"fail.zero_bits", 1)
        with pytest.raises(CrdtLibraryError, match="0x2"):
            fn(A, B)
        assert eng.device_status(clear=True) == 0
    _check(eng, sa, sb)


@pytest.mark.diag
@pytest.mark.parametrize("parts", [2, 8, 16])
def test_lww_write_parts(eng, parts):
    """The LWW write pass at every workgroup shape (sets.lww_parts: 1/parts of
    a 4096-item tile per workgroup; default 4): tile and part edges, long key
    runs across parts, unaligned views (register staging)."""
    from crdt_amd import _lib
    set_knob(b"sets.lww_parts", parts)
    try:
        _check(eng, *_sets(91, 100_000, 90_000, 40_000))
        for na, nb in ((4095, 1), (4096, 4096), (1023, 1025), (255, 257), (0, 5000)):
            _check(eng, *_sets(92 + na, na, nb, max(1, (na + nb) // 3)))
        test_sets_long_runs_cross_tiles(eng)
        test_sets_unaligned_views(eng, 3, 5)
    finally:
        set_knob(b"sets.lww_parts", 4)


@pytest.mark.diag
@pytest.mark.parametrize("parts", [1, 2, 4])
def test_orset_write_parts(eng, parts):
    """The OR-Set write pass at every workgroup shape (sets.or_parts: 1/parts
    of a 2048-item tile per workgroup): tile and part edges, tag copies that
    run past a part (the global-memory walk), unaligned views."""
    from crdt_amd import _lib
    set_knob(b"sets.or_parts", parts)
    try:
        _check(eng, *_sets(93, 100_000, 90_000, 40_000))
        for na, nb in ((2047, 1), (2048, 2048), (511, 513), (1023, 1025), (0, 3000)):
            _check(eng, *_sets(94 + na, na, nb, max(1, (na + nb) // 3)))
        test_sets_long_runs_cross_tiles(eng)
        test_sets_identical_inputs_idempotent(eng)
        test_sets_unaligned_views(eng, 3, 5)
        test_sets_unaligned_views(eng, 13, 11)
    finally:
        set_knob(b"sets.or_parts", 2)
