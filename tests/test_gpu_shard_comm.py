"""GPU: the C-ABI's own RCCL communicator (crdt_shard_*, csrc/shard.hip) on
the one-GPU box: a 1-device ncclCommInitAll communicator and a 1-rank
ncclCommInitRank one.  Outputs are checked against the oracle
(oc_gcounter_fold, oc_lww_merge, oc_orset_merge)."""
import numpy as np
import pytest
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
