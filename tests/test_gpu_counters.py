"""GPU parity: G-Counter / PN-Counter / vector-clock join kernels vs the oracle.

Bit-exact (integer) comparisons through the C-ABI.  Reference parity is
unpinned for these build-defined types; the oracle
restatement is pinned by tests/golden/counters_kat.json.
"""
import numpy as np
import pytest
import torch

from crdt_amd import synth
from crdt_amd.engine import as_u64, u64_tensor
from oracle import oracle

pytestmark = pytest.mark.gpu

EDGE = np.array([0, 1, 2**63 - 1, 2**63, 2**64 - 2, 2**64 - 1], dtype=np.uint64)


def _edge_pairs(nodes):
    a = np.repeat(EDGE, len(EDGE))
    b = np.tile(EDGE, len(EDGE))
    n = (len(a) + nodes - 1) // nodes * nodes
    a = np.resize(a, n).reshape(-1, nodes)
    b = np.resize(b, n).reshape(-1, nodes)
    return a, b


@pytest.mark.parametrize("rows,nodes", [(1, 64), (3, 64), (1000, 64), (777, 63), (5, 1), (100, 128), (33, 7)])
def test_join_matches_oracle(eng, rows, nodes):
    a = synth.counters(1, 1, rows * nodes).reshape(rows, nodes)
    b = synth.counters(1, 2, rows * nodes).reshape(rows, nodes)
    out = eng.gcounter_join(u64_tensor(a, eng.device), u64_tensor(b, eng.device))
    np.testing.assert_array_equal(as_u64(out), oracle.gcounter_join(a, b))


def test_join_edge_values_unsigned(eng):
    a, b = _edge_pairs(64)
    out = as_u64(eng.gcounter_join(u64_tensor(a, eng.device), u64_tensor(b, eng.device)))
    np.testing.assert_array_equal(out, np.maximum(a, b))


def test_join_in_place_alias(eng):
    a = synth.counters(3, 1, 4096 * 64).reshape(4096, 64)
    b = synth.counters(3, 2, 4096 * 64).reshape(4096, 64)
    ta = u64_tensor(a, eng.device)
    eng.gcounter_join(ta, u64_tensor(b, eng.device), out=ta)
    np.testing.assert_array_equal(as_u64(ta), oracle.gcounter_join(a, b))


def test_join_full_config_b(eng):
    """configs[1] at full size: 1M replicas x 64 nodes, device-generated."""
    rows, nodes = 1_000_000, 64
    ta = eng.synth_counters(7, 1, rows, nodes)
    tb = eng.synth_counters(7, 2, rows, nodes)
    out = eng.gcounter_join(ta, tb)
    a, b, o = as_u64(ta), as_u64(tb), as_u64(out)
    # device generator == host generator on a head and a tail window
    flat = a.reshape(-1)
    np.testing.assert_array_equal(flat[:64000], synth.counters(7, 1, 64000))
    np.testing.assert_array_equal(flat[-64000:], synth.counters(7, 1, 64000, rows * nodes - 64000))
    np.testing.assert_array_equal(o, oracle.gcounter_join(a, b, threads=8))
    # idempotent / commutative
    np.testing.assert_array_equal(as_u64(eng.gcounter_join(out, out)), o)
    np.testing.assert_array_equal(as_u64(eng.gcounter_join(tb, ta)), o)


def test_device_generator_matches_host(eng):
    n = 64 * 5000
    dev = as_u64(eng.synth_counters(11, 3, 5000, 64)).reshape(-1)
    np.testing.assert_array_equal(dev, synth.counters(11, 3, n))
    base = 123457
    dev2 = as_u64(eng.synth_counters(11, 3, 10, 64, row_base=base)).reshape(-1)
    np.testing.assert_array_equal(dev2, synth.counters(11, 3, 640, base * 64))


@pytest.mark.parametrize("rows,nodes", [(1, 64), (1000, 64), (100_003, 64), (999, 63), (10, 1024), (4, 3), (257, 128)])
def test_fold_matches_oracle(eng, rows, nodes):
    a = synth.counters(5, 4, rows * nodes).reshape(rows, nodes)
    out = eng.gcounter_fold(u64_tensor(a, eng.device))
    np.testing.assert_array_equal(as_u64(out), oracle.gcounter_fold(a))


def test_fold_empty_rows_is_identity(eng):
    a = torch.empty(0, 64, dtype=torch.int64, device=eng.device)
    out = eng.gcounter_fold(a)
    assert (as_u64(out) == 0).all()


@pytest.mark.parametrize("rows,nodes", [(1, 64), (5000, 64), (333, 128), (77, 32), (50, 16), (40, 5), (9, 200)])
def test_pncounter_value_and_join(eng, rows, nodes):
    p = synth.counters(9, 1, rows * nodes).reshape(rows, nodes)
    n = synth.counters(9, 2, rows * nodes).reshape(rows, nodes)
    tp, tn = u64_tensor(p, eng.device), u64_tensor(n, eng.device)
    v = eng.pncounter_value(tp, tn)
    np.testing.assert_array_equal(v.cpu().numpy(), oracle.pncounter_value(p, n))
    g = eng.gcounter_value(tp)
    np.testing.assert_array_equal(as_u64(g), oracle.pncounter_value(p, np.zeros_like(p)).view(np.uint64))
    p2 = synth.counters(9, 3, rows * nodes).reshape(rows, nodes)
    n2 = synth.counters(9, 4, rows * nodes).reshape(rows, nodes)
    po, no = eng.pncounter_join(tp, tn, u64_tensor(p2, eng.device), u64_tensor(n2, eng.device))
    np.testing.assert_array_equal(as_u64(po), oracle.gcounter_join(p, p2))
    np.testing.assert_array_equal(as_u64(no), oracle.gcounter_join(n, n2))


def test_ordered_i64_roundtrip(eng):
    x = np.concatenate([EDGE, synth.counters(2, 2, 1000)])
    t = u64_tensor(x, eng.device)
    o = eng.u64_to_ordered_i64(t)
    # signed order of the mapped values == unsigned order of the originals
    assert (np.argsort(o.cpu().numpy(), kind="stable") == np.argsort(x, kind="stable")).all()
    np.testing.assert_array_equal(as_u64(eng.ordered_i64_to_u64(o)), x)


def test_stream_peak_kernels(eng):
    """The bench's self-measured peak kernels: the copy
    reproduces its input, the read sweep touches every word (xor of the
    per-workgroup sinks = xor of the input)."""
    n = (1 << 20) + 6                                   # not a multiple of the grid stride
    src = torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device=eng.device)
    for unroll in (1, 2, 4, 8):
        dst = torch.zeros_like(src)
        eng.stream_copy(src, dst, unroll, 2)
        assert torch.equal(dst, src)
        sink = torch.zeros(1 << 16, dtype=torch.int64, device=eng.device)
        eng.stream_read(src, sink, unroll, 1)
        x = np.bitwise_xor.reduce(sink.cpu().numpy().view(np.uint64))
        assert x == np.bitwise_xor.reduce(src.cpu().numpy().view(np.uint64))


def test_ctx_set_stream_orders_work_across_streams(eng):
    """crdt_ctx_set_stream: work queued on the old stream
    finishes before the new stream's work touches its outputs -- a 512-MB
    join on stream 1, then (no host sync) the fold of its output on stream 2
    == the oracle; and the context's workspace is not freed under a set
    merge still running on the old stream."""
    from crdt_amd import synth
    from crdt_amd.engine import TupleSet
    rows, nodes = 1_000_000, 64
    a = eng.synth_counters(77, 1, rows, nodes)
    b = eng.synth_counters(77, 2, rows, nodes)
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = torch.empty_like(a)
    with torch.cuda.stream(s1):
        eng.gcounter_join(a, b, out=out)
    with torch.cuda.stream(s2):
        fold = eng.gcounter_fold(out)          # the context switches to s2 on this call
    torch.cuda.synchronize()
    exp = oracle.gcounter_fold(np.maximum(as_u64(a).reshape(rows, nodes), as_u64(b).reshape(rows, nodes)))
    np.testing.assert_array_equal(as_u64(fold), exp)
    # a set merge on s1, then a bigger one on s2 (the workspace grows: ws_reserve frees the old one)
    sa = synth.sort_tuples_np(*synth.set_tuples(3, 0, 200_000, 100_000))
    sb = synth.sort_tuples_np(*synth.set_tuples(3, 1, 200_000, 100_000))
    A, B = TupleSet.from_numpy(*sa, eng.device), TupleSet.from_numpy(*sb, eng.device)
    big_a = eng.synth_set_tuples(4, 0, 3_000_000, 2_000_000)
    big_b = eng.synth_set_tuples(4, 1, 3_000_000, 2_000_000)
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        small, _ = eng.lww_merge(A, B, trim=False)
    with torch.cuda.stream(s2):
        eng.lww_merge(big_a, big_b, trim=False)
    torch.cuda.synchronize()
    got = small.slice(len(oracle.lww_merge(sa, sb)[0])).to_numpy()
    for g, e in zip(got, oracle.lww_merge(sa, sb)):
        np.testing.assert_array_equal(g, e)
