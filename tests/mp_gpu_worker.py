"""One rank of tests/test_gpu_multirank.py (not a test module itself).

Runs the multi-rank paths through a REAL torch.distributed process group
(gloo: every rank uses cuda:0 of the one-GPU box; RCCL refuses two ranks on
one GPU) and checks them against the oracle, not against another GPU path:

  1. shard.sharded_refmerge -- a ts-range-sharded batch (rank r holds the
     r-th ts range of every replica): this rank's slice of the new Diff must
     equal the oracle's new Diff restricted to the rank's ts range, and the
     all-reduced CurrentState must equal the oracle's, replica by replica
     (oracle/crdt_oracle.c oc_refmerge, main.go:35-100);
  2. gossip.sharded_round -- replicas partitioned over the ranks; every
     round each rank fetches only the Diffs its replicas pull (all-to-all-v)
     and each replica pulls its peer (self-pulls and dead peers included);
     the rank's block must equal a host simulation of the reference's rounds
     on oracle/pyref.py (main.go:226-258);
  3. shard.sharded_set_merge_local with the HIP set merges as the per-rank
     compute -- the gathered state must equal the oracle's merge of the
     rank-order stable merges of every rank's own tuples.

Env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT.  Prints one line
"RANK r OK <checks>" and exits 0, or raises.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def check_sharded_refmerge(eng, rank, world):
    from crdt_amd import refmerge, shard, synth
    from refmerge_util import oracle_packed_replica, split_ts_range, ts_splitters
    h = synth.refmerge_packed(41, 48, 3000)
    spl = ts_splitters(h, world)
    lo, hi = spl[rank], spl[rank + 1]
    part = split_ts_range(h, lo, hi)
    dev = refmerge.to_device({k: v for k, v in part.items() if not k.endswith("_sel")}, eng.device)
    out = shard.sharded_refmerge(eng, dev)
    off = out["off"].cpu().numpy()
    ts, org, src = (out[k].cpu().numpy() for k in ("ts", "origin", "src"))
    kind, sstr, ssum = (out[k].cpu().numpy() for k in ("st_kind", "st_str", "st_sum"))
    n_rows = 0
    for p in range(h["replicas"]):
        o_ts, o_or, o_src, k, s, v = oracle_packed_replica(h, p)
        keep = (o_ts >= lo) & (o_ts < hi) if hi != spl[-1] else (o_ts >= lo)
        a, b = int(off[p]), int(off[p + 1])
        np.testing.assert_array_equal(ts[a:b], o_ts[keep])
        np.testing.assert_array_equal(org[a:b], o_or[keep])
        loc = src[a:b]                                   # rank-local L / R index -> global
        glob = np.where(loc >= 0, part["l_sel"][np.maximum(loc, 0)], -part["r_sel"][np.maximum(-loc - 1, 0)] - 1)
        np.testing.assert_array_equal(glob, o_src[keep])
        sl = slice(p * 62, (p + 1) * 62)
        np.testing.assert_array_equal(kind[sl], k)
        np.testing.assert_array_equal(sstr[sl].view(np.uint32)[k == 1], s[k == 1])
        np.testing.assert_array_equal(ssum[sl][k == 2], v[k == 2])
        n_rows += b - a
    # the slices partition the new Diff: their lengths sum to the oracle's
    tot = torch.tensor([n_rows], dtype=torch.int64)
    dist.all_reduce(tot)
    assert int(tot) == sum(len(oracle_packed_replica(h, p)[0]) for p in range(h["replicas"]))
    return "sharded_refmerge"


def check_sharded_gossip(eng, rank, world):
    from crdt_amd import gossip, shard
    from gossip_util import K, _host_round, _local_writes, _pack, _rand_diff, _same_diffs, _state, _unpack
    rng = np.random.default_rng(17)                      # identical stream on every rank
    P = 7
    diffs = [_rand_diff(rng, 2_000 + 11 * i, int(rng.integers(3, 35))) for i in range(P)]
    b, e = shard.shard_range(P, world, rank)
    pop = gossip.Population(eng, _pack(diffs[b:e]), K, first=b)
    states = [{} for _ in range(P)]
    for rnd in range(5):
        # odd rounds draw like the reference: self-pulls and dead peers (-1)
        peers = gossip.random_peers(rng, P, 0, P) if rnd % 2 == 0 else gossip.reference_peers(rng, P, 0, P)
        gossip.sharded_round(pop, peers)
        diffs, states = _host_round(diffs, peers, states)
        _same_diffs(_unpack(pop), diffs[b:e])
        assert _state(pop) == states[b:e], f"round {rnd}: state"
        if rnd == 1:                                     # local writes between rounds (main.go:187)
            blk = _local_writes(rng, diffs)
            sel = slice(int(blk["off"][b]), int(blk["off"][e]))
            ksel = slice(int(blk["kv_off"][blk["off"][b]]), int(blk["kv_off"][blk["off"][e]]))
            mine = {"off": blk["off"][b:e + 1] - blk["off"][b], "ts": blk["ts"][sel],
                    "kv_off": blk["kv_off"][blk["off"][b]:blk["off"][e] + 1] - blk["kv_off"][blk["off"][b]],
                    "kv_key": blk["kv_key"][ksel] - np.uint32(b * K), "kv_val": blk["kv_val"][ksel]}
            pop.append_local(mine)
            _same_diffs(_unpack(pop), diffs[b:e])
    return "sharded_round"


def check_sharded_set_merge_local(eng, rank, world):
    """shard.sharded_set_merge_local with the HIP LWW / OR-Set merge as the
    per-rank compute (the default): the gathered state == the oracle's merge
    of the rank-order stable merges of every rank's own tuples, and the
    ungathered per-rank ranges partition it."""
    from crdt_amd import shard
    from crdt_amd.engine import TupleSet
    from oracle import oracle
    from test_shard_gloo import SIZES, rank_sets, stable_rank_merge
    done = []
    for lww in (True, False):
        sizes = [SIZES[p % len(SIZES)] for p in range(world)]
        a, b = rank_sets(13, rank, *sizes[rank], 3000)
        A, B = TupleSet.from_numpy(*a, eng.device), TupleSet.from_numpy(*b, eng.device)
        got = shard.sharded_set_merge_local(eng, A, B, lww=lww)
        mine = shard.sharded_set_merge_local(eng, A, B, lww=lww, gather=False)
        everyone = [rank_sets(13, p, *sizes[p], 3000) for p in range(world)]
        exp = (oracle.lww_merge if lww else oracle.orset_merge)(stable_rank_merge([e[0] for e in everyone]),
                                                                 stable_rank_merge([e[1] for e in everyone]))
        for g, e in zip(got.to_numpy(), exp):
            np.testing.assert_array_equal(g, e)
        tot = torch.tensor([len(mine)], dtype=torch.int64)
        dist.all_reduce(tot)
        assert int(tot) == len(exp[0])
        done.append("lww" if lww else "orset")
    return "sharded_set_merge_local(" + ",".join(done) + ")"


def main():
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from crdt_amd.engine import Engine
    eng = Engine(0)
    try:
        done = [check_sharded_refmerge(eng, rank, world), check_sharded_gossip(eng, rank, world),
                check_sharded_set_merge_local(eng, rank, world)]
        torch.cuda.synchronize()
        dist.barrier()
        print(f"RANK {rank} OK {' '.join(done)}", flush=True)
    finally:
        eng.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
