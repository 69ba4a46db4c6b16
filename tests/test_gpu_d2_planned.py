"""GPU: stream-ordered D2 merges -- crdt_set_merge_plan once, then
crdt_{lww,orset}_merge_unsorted_planned with no host synchronisation, so a
HIP graph can capture the whole merge (VERDICT r04 "Next round" item 3).

* eager planned calls == the oracle's merge of the lexsorted sides, on the
  dense-key forms (LWW key-bucket tables, OR-Set key chunks) and on the
  general radix path (2-word composites);
* the planned call captured in a graph (torch.cuda.graph on the context's
  stream), replayed, == the oracle; new inputs of the same shape copied into
  the captured buffers, replayed again == the oracle of the new inputs;
* a tuple outside the plan: the replay raises CRDT_DEV_PLAN and the count
  reads 2^64 - 1; the unplanned call on the same inputs is exact;
* refusals: a plan of another shape or mode."""
import numpy as np
import pytest
import torch
from knobs import set_knob

from crdt_amd import _lib, synth
from crdt_amd.engine import TupleSet, as_u64
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV_PLAN = 4


def _np_sorted(t):
    o = np.lexsort((t[3], t[2], t[1], t[0]))
    return tuple(np.ascontiguousarray(x[o]) for x in t)


def _expect(lww, ua, ub):
    return (oracle.lww_merge if lww else oracle.orset_merge)(_np_sorted(ua), _np_sorted(ub))


def _same(out, count, exp):
    n = int(as_u64(count)[0])
    assert n == len(exp[0])
    for g, e, f in zip(out.slice(n).to_numpy(), exp, ("key", "ts", "rep", "tomb")):
        np.testing.assert_array_equal(g, e, err_msg=f)


def _load(dst: TupleSet, src):
    for t, x in zip((dst.key, dst.ts, dst.rep, dst.tomb), src):
        t.copy_(torch.from_numpy(np.ascontiguousarray(x).view(np.int64 if x.dtype == np.uint64 else
                                                               np.int32 if x.dtype == np.uint32 else np.uint8)))


def _dense(seed, n, ks):
    return synth.set_tuples(seed, 0, n, ks), synth.set_tuples(seed, 1, n - 1000, ks)


def _wide(seed, n):
    rng = np.random.default_rng(seed)

    def side(m):
        return (rng.integers(0, 2**40, m, dtype=np.uint64), rng.integers(0, 2**30, m, dtype=np.uint64),
                rng.integers(0, 2**10, m, dtype=np.uint64).astype(np.uint32), rng.integers(0, 2, m, dtype=np.uint8))
    a, b = side(n), side(n - 7)
    for f in range(3):
        b[f][:500] = a[f][:500]                          # cross-side equal tags
    return a, b


@pytest.mark.parametrize("lww", [True, False])
@pytest.mark.parametrize("shape", ["dense", "wide"])
def test_planned_eager_and_graph_replays(eng, lww, shape):
    ua, ub = _dense(11, 400_000, 300_000) if shape == "dense" else _wide(12, 200_000)
    A = TupleSet.from_numpy(*ua, eng.device)
    B = TupleSet.from_numpy(*ub, eng.device)
    out = TupleSet.empty(len(A) + len(B), eng.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=eng.device)
    plan = eng.set_merge_plan(lww, A, B, widen=True)
    exp = _expect(lww, ua, ub)
    eng.merge_unsorted_planned(lww, plan, A, B, out, cnt)          # eager, stream-ordered
    torch.cuda.synchronize()
    _same(out, cnt, exp)
    assert eng.device_status() == 0
    # the same call captured in a graph
    out.key.fill_(-1)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, capture_error_mode="thread_local"):
        eng.merge_unsorted_planned(lww, plan, A, B, out, cnt)
    g.replay()
    torch.cuda.synchronize()
    _same(out, cnt, exp)
    # new inputs of the same shape, inside the plan: the captured buffers refilled
    rng = np.random.default_rng(5)
    pa, pb = rng.permutation(len(A)), rng.permutation(len(B))
    na_ = tuple(x[pa] for x in ua)
    nb_ = tuple(x[pb] for x in ub)
    na_[3][:] = rng.integers(0, 2, len(A), dtype=np.uint8)
    _load(A, na_)
    _load(B, nb_)
    g.replay()
    torch.cuda.synchronize()
    _same(out, cnt, _expect(lww, na_, nb_))
    assert eng.device_status() == 0
    # a tuple outside the plan: flagged, never silently wrong
    bad = tuple(np.array(x, copy=True) for x in na_)
    bad[0][len(A) // 2] = np.uint64(2**63 + 12345)
    _load(A, bad)
    g.replay()
    torch.cuda.synchronize()
    assert int(as_u64(cnt)[0]) == 2**64 - 1
    assert eng.device_status(clear=True) & DEV_PLAN
    fn = eng.lww_merge_unsorted if lww else eng.orset_merge_unsorted
    got = fn(A, B).to_numpy()
    for g_, e in zip(got, _expect(lww, bad, nb_)):
        np.testing.assert_array_equal(g_, e)
    del g


@pytest.mark.diag
@pytest.mark.parametrize("lww", [True, False])
def test_device_plan_changed_behind_the_launch(eng, lww):
    """VERDICT r05 item 6 (the fault of commit 01a0e59): the device plan's
    shape differs from the one the passes were launched for (failpoint
    fail.d2_plan: more key bits in device memory).  Every pass compares the
    device plan with its launch shape first and stores nothing: the planned
    call raises CRDT_DEV_PLAN with count 2^64 - 1, the unplanned call
    (sampled plan, then the context's cached plan) redoes from the exact plan
    == the oracle, and the next planned call == the oracle."""
    ua, ub = _dense(17, 400_000, 300_000)
    A = TupleSet.from_numpy(*ua, eng.device)
    B = TupleSet.from_numpy(*ub, eng.device)
    out = TupleSet.empty(len(A) + len(B), eng.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=eng.device)
    exp = _expect(lww, ua, ub)
    plan = eng.set_merge_plan(lww, A, B, widen=True)
    assert eng.device_status() == 0
    try:
        set_knob(b"fail.d2_plan", 1)
        eng.merge_unsorted_planned(lww, plan, A, B, out, cnt)
        torch.cuda.synchronize()
        assert int(as_u64(cnt)[0]) == 2**64 - 1
        assert eng.device_status(clear=True) & DEV_PLAN
        set_knob(b"sort.sample_min", 0)                  # the sampled / cached dense-key forms at this size
        fn = eng.lww_merge_unsorted if lww else eng.orset_merge_unsorted
        for _ in range(2):                               # a fresh sampled plan, then the context's cached one
            set_knob(b"fail.d2_plan", 1)
            got = fn(A, B).to_numpy()
            assert len(got[0]) == len(exp[0])
            for g, e in zip(got, exp):
                np.testing.assert_array_equal(g, e)
            assert eng.device_status() == 0              # (the redo is silent)
    finally:
        set_knob(b"fail.d2_plan", 0)
        set_knob(b"sort.sample_min", 1 << 20)
    eng.merge_unsorted_planned(lww, plan, A, B, out, cnt)
    torch.cuda.synchronize()
    _same(out, cnt, exp)
    assert eng.device_status() == 0


def test_planned_refuses_another_shape(eng):
    ua, ub = _dense(13, 50_000, 40_000)
    A = TupleSet.from_numpy(*ua, eng.device)
    B = TupleSet.from_numpy(*ub, eng.device)
    out = TupleSet.empty(len(A) + len(B), eng.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=eng.device)
    plan = eng.set_merge_plan(True, A, B)
    with pytest.raises(_lib.CrdtError):
        eng.merge_unsorted_planned(False, plan, A, B, out, cnt)     # an LWW plan for an OR-Set merge
    with pytest.raises(_lib.CrdtError):
        eng.merge_unsorted_planned(True, plan, A.slice(len(A) - 2), B, out, cnt)
    eng.merge_unsorted_planned(True, plan, A, B, out, cnt)
    torch.cuda.synchronize()
    _same(out, cnt, _expect(True, ua, ub))


def test_planned_full_config_d(eng):
    """configs[3] D2 at full size (10M + 10M unsorted, key space 8M) through
    the planned calls == the unplanned calls, both modes."""
    n, ks = 10_000_000, 8_000_000
    UA = eng.synth_set_tuples(2024, 0, n, ks, sort=False)
    UB = eng.synth_set_tuples(2024, 1, n, ks, sort=False)
    for lww in (True, False):
        ref = (eng.lww_merge_unsorted if lww else eng.orset_merge_unsorted)(UA, UB)
        plan = eng.set_merge_plan(lww, UA, UB, widen=True)
        out = TupleSet.empty(2 * n, eng.device)
        cnt = torch.zeros(1, dtype=torch.int64, device=eng.device)
        eng.merge_unsorted_planned(lww, plan, UA, UB, out, cnt)
        torch.cuda.synchronize()
        m = int(cnt.item())
        assert m == len(ref)
        got = out.slice(m)
        for g, e in zip((got.key, got.ts, got.rep, got.tomb), (ref.key, ref.ts, ref.rep, ref.tomb)):
            assert bool((g == e).all())
        assert eng.device_status() == 0
