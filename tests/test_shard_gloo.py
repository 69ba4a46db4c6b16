"""CPU, world_size 2 (gloo): the multi-GPU exchange protocol of crdt_amd.shard.

The per-rank compute here is the oracle (no GPU in this container); what is
under test is the exchange: shard planning, the order-preserving uint64 MAX
all-reduce, and the key-range all-gather-v assembling a sorted merged set.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from crdt_amd import shard, synth
from oracle import oracle


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    try:
        _worker_body(rank, world, port, q)
    except Exception:                        # surface the failure instead of a queue timeout
        import traceback
        q.put((rank, "ERROR", traceback.format_exc()))


def _worker_body(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # --- counters: 10_001 rows x 64 sharded, fold + all-reduce(max)
        rows, nodes = 10_001, 64
        b, e = shard.shard_range(rows, world, rank)
        full = synth.counters(3, 1, rows * nodes).reshape(rows, nodes)
        full[5, 7] = np.uint64(2**64 - 1) if rank == 1 else full[5, 7]   # unsigned edge on one rank
        local = oracle.gcounter_fold(full[b:e])
        t = torch.from_numpy(local.view(np.int64).copy())
        shard.allreduce_max_u64(t)
        got_fold = t.numpy().view(np.uint64).copy()
        full[5, 7] = np.uint64(2**64 - 1)
        exp_fold = oracle.gcounter_fold(full)

        # --- sets: key-range partition, local merge, all-gather-v
        ks = 5000
        sa = synth.sort_tuples_np(*synth.set_tuples(8, 0, 20000, ks))
        sb = synth.sort_tuples_np(*synth.set_tuples(8, 1, 20000, ks))
        # sampled splitters (shard.sample_splitters: one all-gather of samples)
        from crdt_amd.engine import TupleSet
        spl = shard.sample_splitters(TupleSet.from_numpy(*sa, "cpu"), TupleSet.from_numpy(*sb, "cpu"), world,
                                     per=64)
        lo, hi = spl[rank], spl[rank + 1]

        def part(s):
            i = np.searchsorted(s[0], np.uint64(lo))
            j = np.searchsorted(s[0], np.uint64(hi)) if hi < shard.KEY_END else len(s[0])
            return tuple(x[i:j] for x in s)

        m = oracle.lww_merge(part(sa), part(sb))
        keys = shard.allgather_v(torch.from_numpy(m[0].view(np.int64).copy())).numpy().view(np.uint64)
        tss = shard.allgather_v(torch.from_numpy(m[1].view(np.int64).copy())).numpy().view(np.uint64)
        full_m = oracle.lww_merge(sa, sb)
        q.put((rank, np.array_equal(got_fold, exp_fold), np.array_equal(keys, full_m[0]),
               np.array_equal(tss, full_m[1]), (b, e), spl))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_sharded_exchange(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort(key=lambda r: r[0])
    for r in res:
        assert r[1] != "ERROR", r[2]
    for rank, fold_ok, keys_ok, ts_ok, _, _ in res:
        assert fold_ok, f"rank {rank}: sharded fold != oracle fold"
        assert keys_ok and ts_ok, f"rank {rank}: gathered LWW merge != oracle"
    assert res[0][4][1] == res[1][4][0]      # contiguous shards
    assert res[0][5] == res[1][5]            # every rank derives the same splitters
    assert res[0][5][0] == 0 and res[0][5][-1] == shard.KEY_END and len(res[0][5]) == world + 1


# ---------------------------------------------------------------- distributed keyed sets
def rank_sets(seed, rank, n_a, n_b, key_space):
    """Rank `rank`'s own sorted tuples (A and B) of a distributed population."""
    a = synth.sort_tuples_np(*synth.set_tuples(seed * 100 + rank, 0, n_a, key_space))
    b = synth.sort_tuples_np(*synth.set_tuples(seed * 100 + rank, 1, n_b, key_space))
    return a, b


def stable_rank_merge(parts):
    """The population's side: every rank's sorted tuples merged stably in rank
    order (equal tags keep rank order) -- the input order
    crdt_shard_*_merge_local defines."""
    cat = [np.concatenate([p[f] for p in parts]) for f in range(4)]
    rec = np.empty(len(cat[0]), dtype=[("k", np.uint64), ("t", np.uint64), ("r", np.uint32)])
    rec["k"], rec["t"], rec["r"] = cat[0], cat[1], cat[2]
    o = np.argsort(rec, order=["k", "t", "r"], kind="stable")
    return tuple(x[o] for x in cat)


def _oracle_merge(lww):
    from crdt_amd.engine import TupleSet
    fn = oracle.lww_merge if lww else oracle.orset_merge

    def merge(x, y):
        return TupleSet.from_numpy(*fn(x.to_numpy(), y.to_numpy()), "cpu")
    return merge


SIZES = [(3000, 2500), (0, 4000), (5000, 1), (2200, 2700)]     # per rank: uneven, one empty side


def _local_worker(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        try:
            from crdt_amd.engine import TupleSet
            res = []
            for lww in (True, False):
                na, nb = SIZES[rank]
                a, b = rank_sets(7, rank, na, nb, 3000)
                A, B = TupleSet.from_numpy(*a, "cpu"), TupleSet.from_numpy(*b, "cpu")
                got = shard.sharded_set_merge_local(None, A, B, lww=lww, merge=_oracle_merge(lww), per=32)
                mine = shard.sharded_set_merge_local(None, A, B, lww=lww, merge=_oracle_merge(lww), per=32,
                                                     gather=False)
                everyone = [rank_sets(7, p, *SIZES[p], 3000) for p in range(world)]
                pa = stable_rank_merge([e[0] for e in everyone])
                pb = stable_rank_merge([e[1] for e in everyone])
                exp = (oracle.lww_merge if lww else oracle.orset_merge)(pa, pb)
                g = got.to_numpy()
                res.append(all(np.array_equal(x, y) for x, y in zip(g, exp)))
                res.append(len(mine))
            q.put((rank, res))
        finally:
            dist.destroy_process_group()
    except Exception:
        import traceback
        q.put((rank, "ERROR", traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_distributed_set_merge(world):
    """The all-to-all protocol of crdt_shard_{lww,orset}_merge_local over gloo:
    weighted splitters, key-range exchange, rank-order tree merge, all-gather
    -- == the oracle's merge of the rank-order stable merges of every rank's
    own tuples; the per-rank ranges (gather=False) partition the result."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_local_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert r[1] != "ERROR", r[2]
    res.sort(key=lambda r: r[0])
    for rank, (lww_ok, lww_n, or_ok, or_n) in res:
        assert lww_ok, f"rank {rank}: distributed LWW merge != oracle"
        assert or_ok, f"rank {rank}: distributed OR-Set merge != oracle"


def test_weighted_splitters_rule():
    """The splitter rule shared with csrc/shard.hip: weights are the ranks'
    side sizes; an empty side contributes nothing; no data: all zero."""
    per = 4
    blocks = np.zeros((2, 2 + 2 * per), np.uint64)
    blocks[0, :2] = (100, 0)
    blocks[0, 2:2 + per] = (10, 20, 30, 40)
    blocks[1, :2] = (300, 0)
    blocks[1, 2:2 + per] = (15, 25, 35, 45)
    # weights: 100 each for 10..40, 300 each for 15..45; total 1600; 10+15+20+25 reach 800
    assert shard.weighted_splitters(blocks, 2, per) == [0, 25, shard.KEY_END]
    assert shard.weighted_splitters(np.zeros((3, 2 + 2 * per), np.uint64), 3, per) == [0, 0, 0, shard.KEY_END]
