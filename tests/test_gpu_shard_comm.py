"""GPU: the C-ABI's own RCCL communicator (crdt_shard_*, csrc/shard.hip) on
the one-GPU box: a 1-device ncclCommInitAll communicator and a 1-rank
ncclCommInitRank one.  Outputs are checked against the oracle
(oc_gcounter_fold, oc_lww_merge, oc_orset_merge)."""
import numpy as np
import pytest
from knobs import set_knob
import torch

from crdt_amd import shard, synth
from crdt_amd.engine import TupleSet, as_u64, u64_tensor
from oracle import oracle

pytestmark = pytest.mark.gpu

EDGE = np.array([0, 1, 2**63 - 1, 2**63, 2**64 - 2, 2**64 - 1], dtype=np.uint64)


@pytest.fixture(scope="module")
def comm():
    c = shard.Comm.create([0])
    yield c
    c.close()


def test_comm_info(comm):
    assert (comm.members, comm.nranks, comm.rank0) == (1, 1, 0)


@pytest.mark.parametrize("rows,nodes", [(100_003, 64), (1, 64), (4097, 128), (999, 63)])
def test_fold_allreduce_max_matches_oracle(comm, rows, nodes):
    a = synth.counters(21, 1, rows * nodes).reshape(rows, nodes)
    a.reshape(-1)[: len(EDGE)] = EDGE                    # the unsigned edges ride through ncclUint64 max
    t = u64_tensor(a, "cuda:0")
    torch.cuda.synchronize()
    out = comm.fold_max([t])
    comm.sync()
    np.testing.assert_array_equal(as_u64(out[0]), oracle.gcounter_fold(a))


def test_allreduce_max_u64_single_rank_is_identity(comm):
    x = np.concatenate([EDGE, synth.counters(4, 4, 10_000)])
    t = u64_tensor(x, "cuda:0")
    torch.cuda.synchronize()
    comm.allreduce_max_u64([t])
    comm.sync()
    np.testing.assert_array_equal(as_u64(t), x)


@pytest.mark.parametrize("lww", [True, False])
@pytest.mark.parametrize("n,ks", [(200_000, 150_000), (5000, 50), (0, 10)])
def test_sharded_set_merge_matches_oracle(comm, lww, n, ks):
    sa = synth.sort_tuples_np(*synth.set_tuples(31, 0, n, ks))
    sb = synth.sort_tuples_np(*synth.set_tuples(31, 1, n + 7, ks))
    A = TupleSet.from_numpy(*sa, "cuda:0")
    B = TupleSet.from_numpy(*sb, "cuda:0")
    torch.cuda.synchronize()
    got = comm.set_merge([A], [B], lww=lww)[0].to_numpy()
    exp = (oracle.lww_merge if lww else oracle.orset_merge)(sa, sb)
    for g, e in zip(got, exp):
        np.testing.assert_array_equal(g, e)


def test_set_allgather_v_single_rank_copies(comm):
    s = synth.sort_tuples_np(*synth.set_tuples(3, 0, 1234, 999))
    loc = TupleSet.from_numpy(*s, "cuda:0")
    out = TupleSet.empty(2000, "cuda:0")
    torch.cuda.synchronize()
    n = comm.set_allgather_v([loc], [out], 2000)
    comm.sync()
    assert n == 1234
    for g, e in zip(out.slice(n).to_numpy(), s):
        np.testing.assert_array_equal(g, e)
    with pytest.raises(Exception):
        comm.set_allgather_v([loc], [out], 1000)       # CRDT_E_RANGE: capacity too small


def test_init_rank_single_process(eng):
    """ncclCommInitRank with nranks = 1 on the engine's own context/stream."""
    c = shard.Comm.init_rank(eng)
    try:
        rows, nodes = 50_000, 64
        a = eng.synth_counters(8, 1, rows, nodes)
        out = c.fold_max([a])
        np.testing.assert_array_equal(as_u64(out[0]), oracle.gcounter_fold(as_u64(a).reshape(rows, nodes)))
    finally:
        c.close()


# ---------------------------------------------------------------- one-call sharded RefMerge
def _check_refmerge_vs_oracle(h, out):
    from refmerge_util import assert_batch_matches_oracle
    assert_batch_matches_oracle(h, out)


@pytest.mark.parametrize("replicas,entries", [(48, 3000), (5, 10_000), (1, 1)])
def test_comm_refmerge_matches_oracle(comm, eng, replicas, entries):
    """crdt_shard_refmerge through a 1-device ncclCommInitAll communicator:
    the whole protocol (max(L) all-reduce, local merge, accumulator
    all-reduces, finalize) in one C-ABI call == oc_refmerge per replica."""
    from crdt_amd import refmerge
    h = synth.refmerge_packed(61 + replicas, replicas, entries)
    d = refmerge.to_device(h, "cuda:0")
    torch.cuda.synchronize()
    out = comm.refmerge([eng], [d])[0]
    comm.sync()
    _check_refmerge_vs_oracle(h, out)


@pytest.mark.diag
def test_init_rank_refmerge_and_local_sets(eng):
    """The same calls through ncclCommInitRank (nranks = 1) on the engine's
    own context and stream: crdt_shard_refmerge == oracle, and the
    distributed set merge == the plain merge's oracle."""
    from crdt_amd import refmerge
    c = shard.Comm.init_rank(eng)
    try:
        h = synth.refmerge_packed(71, 32, 4000)
        d = refmerge.to_device(h, eng.device)
        out = c.refmerge([eng], [d])[0]
        eng.sync()
        _check_refmerge_vs_oracle(h, out)
        sa = synth.sort_tuples_np(*synth.set_tuples(72, 0, 30_000, 20_000))
        sb = synth.sort_tuples_np(*synth.set_tuples(72, 1, 25_000, 20_000))
        A, B = TupleSet.from_numpy(*sa, eng.device), TupleSet.from_numpy(*sb, eng.device)
        from crdt_amd import _lib
        for lww in (True, False):
            set_knob(b"shard.exchange_always", 1)
            try:
                got = c.set_merge_local([A], [B], lww=lww)[0].to_numpy()
            finally:
                set_knob(b"shard.exchange_always", 0)
            exp = (oracle.lww_merge if lww else oracle.orset_merge)(sa, sb)
            for g, e in zip(got, exp):
                np.testing.assert_array_equal(g, e)
    finally:
        c.close()


@pytest.mark.diag
@pytest.mark.parametrize("lww", [True, False])
@pytest.mark.parametrize("gather", [True, False])
@pytest.mark.parametrize("na,nb", [(200_000, 180_000), (0, 5000), (7, 0), (0, 0)])
@pytest.mark.parametrize("exchange", [0, 1])
def test_comm_set_merge_local_matches_oracle(comm, lww, gather, na, nb, exchange):
    """crdt_shard_{lww,orset}_merge_local on a 1-member communicator, with the
    one-rank shortcut and (shard.exchange_always) through the whole protocol:
    sample block, splitters, count matrix, the all-to-all (a self send), the
    tree of merges and the all-gather -- == the oracle's merge."""
    from crdt_amd import _lib
    sa = synth.sort_tuples_np(*synth.set_tuples(91, 0, na, 50_000))
    sb = synth.sort_tuples_np(*synth.set_tuples(91, 1, nb, 50_000))
    A, B = TupleSet.from_numpy(*sa, "cuda:0"), TupleSet.from_numpy(*sb, "cuda:0")
    torch.cuda.synchronize()
    set_knob(b"shard.exchange_always", exchange)
    try:
        got = comm.set_merge_local([A], [B], lww=lww, gather=gather)[0].to_numpy()
    finally:
        set_knob(b"shard.exchange_always", 0)
    exp = (oracle.lww_merge if lww else oracle.orset_merge)(sa, sb)
    for g, e in zip(got, exp):
        np.testing.assert_array_equal(g, e)


def test_comm_alltoallv_single_rank_copies(comm):
    x = torch.arange(1000, dtype=torch.int64, device="cuda:0")
    y = torch.zeros(1000, dtype=torch.int64, device="cuda:0")
    torch.cuda.synchronize()
    comm.alltoallv([x], [[1000]], [y], [[1000]], 8)
    comm.sync()
    assert torch.equal(x, y)
