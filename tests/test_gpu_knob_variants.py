"""GPU: every measured alternative of the round-5 D2 and population paths
stays bit-exact.  Each knob's non-default value is what DESIGN.md's A/B
records compare against; the default runs in the rest of the suite.  Per
knob value: a sampled dense-key D2 merge of both modes (400k + 399k tuples,
config D's key density, called twice so the plan cache is used) == the
oracle's merge of the lexsorted sides, and (pop.* knobs) two population
rounds == the same rounds with the knob at its default."""
import numpy as np
import pytest
from knobs import set_knob

from crdt_amd import _lib, gossip, synth
from crdt_amd.engine import TupleSet
from oracle import oracle

pytestmark = [pytest.mark.gpu, pytest.mark.diag]

D2_KNOBS = [("sort.plan_cache", 0), ("sort.plan_cache", 1), ("sort.group_tile", 8192), ("sort.up_threads", 256),
            ("sort.or_sub_hist", 0), ("sort.or_place_batch", 0), ("sort.or_bucket", 0), ("sort.lww_gather", 0),
            ("sort.or_pair", 0), ("sort.or_narrow", 0), ("ctx.read_poll", 0)]
DEFAULTS = {"sort.plan_cache": 2, "sort.group_tile": 4096, "sort.up_threads": 512, "sort.or_sub_hist": 1,
            "sort.or_place_batch": 1, "sort.or_bucket": 1, "sort.lww_gather": 1, "sort.or_pair": 1,
            "sort.or_narrow": 1, "ctx.read_poll": 1, "pop.direct": 1, "pop.wire_early": 1}


def _set(name, v):
    set_knob(name.encode(), v)


def _np_sorted(t):
    o = np.lexsort((t[3], t[2], t[1], t[0]))
    return tuple(np.ascontiguousarray(x[o]) for x in t)


@pytest.fixture(scope="module")
def d2_case(eng):
    n, ks = 400_000, 320_000                              # config D's 1.25 tuples per key per side
    ua, ub = synth.set_tuples(31, 0, n, ks), synth.set_tuples(31, 1, n - 1000, ks)
    A, B = TupleSet.from_numpy(*ua, eng.device), TupleSet.from_numpy(*ub, eng.device)
    sa, sb = _np_sorted(ua), _np_sorted(ub)
    return A, B, {True: oracle.lww_merge(sa, sb), False: oracle.orset_merge(sa, sb)}


@pytest.mark.parametrize("knob,value", D2_KNOBS)
def test_d2_knob_variant_matches_oracle(eng, d2_case, knob, value):
    A, B, exp = d2_case
    try:
        _set("sort.sample_min", 0)                        # the sampled dense-key forms at this size
        _set(knob, value)
        for lww in (True, False):
            fn = eng.lww_merge_unsorted if lww else eng.orset_merge_unsorted
            for _ in range(2):                            # the second call: the context's plan cache
                got = fn(A, B).to_numpy()
                assert len(got[0]) == len(exp[lww][0])
                for g, e in zip(got, exp[lww]):
                    np.testing.assert_array_equal(g, e)
        assert eng.device_status() == 0
    finally:
        _set(knob, DEFAULTS[knob])
        _set("sort.sample_min", 1 << 20)


@pytest.mark.parametrize("knob", ["pop.direct"])
def test_population_knob_variant_rounds(eng, knob):
    """Two local rounds with the knob off == with it on (Diffs, kv pairs,
    CurrentState), and undo restores the first round's result either way."""
    P, E, K = 40, 2500, 62
    h = synth.refmerge_packed(77, P, E)
    n_l = len(h["l_ts"])
    host = dict(h, replicas=P, kv_key=h["kv_key"].view(np.uint32)[:n_l], kv_val=h["kv_val"].view(np.uint32)[:n_l])
    rng = np.random.default_rng(3)
    draws = [gossip.random_peers(rng, P, 0, P) for _ in range(2)]
    reads = {}
    try:
        for v in (DEFAULTS[knob], 0):
            _set(knob, v)
            pop = gossip.NativePopulation(eng, host, K)
            try:
                pop.round(draws[0])
                first = pop.read()
                pop.round(draws[1])
                second = pop.read()
                pop.undo()
                back = pop.read()
                for k in first:
                    np.testing.assert_array_equal(back[k], first[k], err_msg=f"undo {k}")
                reads[v] = (first, second)
            finally:
                pop.close()
    finally:
        _set(knob, DEFAULTS[knob])
    for a, b in zip(reads[DEFAULTS[knob]], reads[0]):
        for k in a:
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
