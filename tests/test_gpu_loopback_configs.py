"""GPU: the multi-rank protocols at BASELINE config size, R = 8 ranks on the
loopback transport (crdt_shard_comm_create_loopback: eight ranks on one GPU,
each with its own context and stream -- the same planning, count matrices,
offsets, capacities and tree merges the RCCL transport runs on an 8-GPU
node), each against the oracle (oracle/crdt_oracle.c), never against another
GPU path (VERDICT r04 "Next round" item 2).  Reference analog: the
cross-replica exchange of main.go:226-258.

* configs[3] as a distributed population: 10M + 10M tuples (key space 8M)
  split over 8 ranks, each rank holding its own sorted share of both sides,
  through crdt_shard_{lww,orset}_merge_local with and without the final
  all-gather == oc_lww_merge / oc_orset_merge of the rank-order stable
  merges of the sides;
* crdt_population_round_sharded at the gossip bench's 1000 replicas x 10k
  entries over 8 ranks, two rounds (a random live draw, then the
  reference's draw with self-pulls and dead peers) == oc_refmerge of each
  replica's Diff with its peer's pulled Diff;
(configs[4]'s 100M x 64 population over 8 loopback ranks through fold_max
lives in test_gpu_configs4.py, beside the 51.2-GB population it reuses.)"""
import numpy as np
import pytest
import torch

from crdt_amd import gossip, shard, synth
from oracle import oracle

pytestmark = pytest.mark.gpu

R = 8
K = 62


@pytest.fixture(scope="module")
def comm8():
    c = shard.Comm.loopback(0, R)
    yield c
    c.close()


def _rank_merge(parts):
    """The population's side: every rank's sorted tuples merged stably in
    rank order (np.lexsort is stable) -- the order crdt_shard_*_merge_local
    defines for a distributed population."""
    cat = [np.concatenate([p[f] for p in parts]) for f in range(4)]
    o = np.lexsort((cat[2], cat[1], cat[0]))
    return tuple(np.ascontiguousarray(x[o]) for x in cat)


@pytest.fixture(scope="module")
def configs3_population(eng):
    n, ks = 10_000_000, 8_000_000
    A, B = [], []
    for r in range(R):
        b, e = shard.shard_range(n, R, r)
        A.append(eng.synth_set_tuples(202_400 + r, 0, e - b, ks))
        B.append(eng.synth_set_tuples(202_400 + r, 1, e - b, ks))
    torch.cuda.synchronize()
    pa = _rank_merge([a.to_numpy() for a in A])
    pb = _rank_merge([b.to_numpy() for b in B])
    yield A, B, pa, pb
    del A, B
    torch.cuda.empty_cache()


@pytest.mark.parametrize("lww", [True, False])
def test_configs3_distributed_population_r8(comm8, configs3_population, lww):
    A, B, pa, pb = configs3_population
    assert len(pa[0]) == len(pb[0]) == 10_000_000
    exp = (oracle.lww_merge if lww else oracle.orset_merge)(pa, pb)
    n_exp = len(exp[0])
    got = comm8.set_merge_local(A, B, lww=lww, gather=True)
    for i, g in enumerate(got):                          # every rank holds the whole merged state
        assert len(g) == n_exp, f"member {i}"
        for x, e, f in zip(g.to_numpy(), exp, ("key", "ts", "rep", "tomb")):
            np.testing.assert_array_equal(x, e, err_msg=f"member {i} {f}")
    del got
    mine = comm8.set_merge_local(A, B, lww=lww, gather=False)   # each rank its key range, in rank order
    assert sum(len(m) for m in mine) == n_exp
    assert all(len(m) > 0 for m in mine)                # the weighted splitters spread the key space
    cat = [np.concatenate([m.to_numpy()[f] for m in mine]) for f in range(4)]
    for x, e in zip(cat, exp):
        np.testing.assert_array_equal(x, e)
    del mine
    torch.cuda.empty_cache()


# ---------------------------------------------------------------- sharded gossip rounds at the bench's size
def _slice_population(h, b, e):
    """Replicas [b, e) of a packed population (kv slots made local: i*K + k)."""
    lb, le = int(h["l_off"][b]), int(h["l_off"][e])
    kb, ke = int(h["l_kv"][lb]), int(h["l_kv"][le])
    return {"replicas": e - b, "l_off": h["l_off"][b:e + 1] - lb, "l_ts": h["l_ts"][lb:le],
            "l_origin": h["l_origin"][lb:le], "l_kv": h["l_kv"][lb:le + 1] - kb,
            "kv_key": (h["kv_key"][kb:ke].astype(np.int64) - b * K).astype(np.uint32),
            "kv_val": h["kv_val"][kb:ke], "str_bytes": h["str_bytes"], "str_off": h["str_off"]}


def _gather(pops, cuts):
    """Every member's read() concatenated into one population (global slots)."""
    parts = [p.read() for p in pops]
    off, kvo, ts, org, kk, kv, kind, sstr, ssum = [np.zeros(1, np.int64)], [np.zeros(1, np.int64)], [], [], [], [], \
        [], [], []
    for (b, e), x in zip(cuts, parts):
        off.append(x["off"][1:].astype(np.int64) + off[-1][-1])
        kvo.append(x["kv_off"][1:].astype(np.int64) + kvo[-1][-1])
        ts.append(x["ts"])
        org.append(x["origin"])
        kk.append(x["kv_key"].astype(np.int64) + b * K)
        kv.append(x["kv_val"])
        kind.append(x["st_kind"])
        sstr.append(x["st_str"])
        ssum.append(x["st_sum"])
    c = np.concatenate
    return {"off": c(off), "kv_off": c(kvo), "ts": c(ts), "origin": c(org), "kv_key": c(kk), "kv_val": c(kv),
            "st_kind": c(kind), "st_str": c(sstr), "st_sum": c(ssum)}


def _check_round(before, after, peers, h):
    """after == oc_refmerge of every replica's Diff (before) with its peer's
    whole Diff as remote maps (main.go:245-256); a dead peer (-1) leaves the
    replica's Diff and CurrentState as they were (main.go:234-239)."""
    off, kvo, ts, org, kvk, kvv = (before[k] for k in ("off", "kv_off", "ts", "origin", "kv_key", "kv_val"))
    aoff, akvo = after["off"], after["kv_off"]
    for p in range(len(peers)):
        a0, a1 = int(aoff[p]), int(aoff[p + 1])
        sl = slice(p * K, (p + 1) * K)
        q = int(peers[p])
        lb, le = int(off[p]), int(off[p + 1])
        if q < 0:
            np.testing.assert_array_equal(after["ts"][a0:a1], ts[lb:le])
            np.testing.assert_array_equal(after["origin"][a0:a1], org[lb:le])
            exp_idx, exp_base = np.arange(lb, le), np.full(le - lb, p)
            for k in ("st_kind", "st_str", "st_sum"):
                np.testing.assert_array_equal(after[k][sl], before[k][sl], err_msg=f"replica {p} {k}")
        else:
            qb, qe = int(off[q]), int(off[q + 1])
            lk0, lk1, qk0, qk1 = int(kvo[lb]), int(kvo[le]), int(kvo[qb]), int(kvo[qe])
            kv_key = np.concatenate([kvk[lk0:lk1] - p * K, kvk[qk0:qk1] - q * K]).astype(np.uint32)
            kv_val = np.concatenate([kvv[lk0:lk1], kvv[qk0:qk1]]).astype(np.uint32)
            l_kv = (kvo[lb:le + 1] - lk0).astype(np.uint32)
            r_kv = (kvo[qb:qe + 1] - qk0 + (lk1 - lk0)).astype(np.uint32)
            o_ts, o_or, o_src, kind, s, v = oracle.refmerge_packed(
                ts[lb:le], org[lb:le], l_kv, ts[qb:qe], r_kv, kv_key, kv_val, h["str_bytes"], h["str_off"], K)
            np.testing.assert_array_equal(after["ts"][a0:a1], o_ts, err_msg=f"replica {p}")
            np.testing.assert_array_equal(after["origin"][a0:a1], o_or, err_msg=f"replica {p}")
            exp_idx = np.where(o_src >= 0, lb + o_src, qb + (-o_src - 1))
            exp_base = np.where(o_src >= 0, p, q)
            np.testing.assert_array_equal(after["st_kind"][sl], kind, err_msg=f"replica {p}")
            np.testing.assert_array_equal(after["st_str"][sl][kind == 1], s[kind == 1], err_msg=f"replica {p}")
            np.testing.assert_array_equal(after["st_sum"][sl][kind == 2], v[kind == 2], err_msg=f"replica {p}")
        # the new Diff's kv pairs: each kept entry's pairs, key slots re-based to replica p
        cnt = kvo[exp_idx + 1] - kvo[exp_idx]
        np.testing.assert_array_equal(np.diff(akvo[a0:a1 + 1]), cnt, err_msg=f"replica {p} pair counts")
        tot = int(cnt.sum())
        starts = np.repeat(kvo[exp_idx] - np.concatenate([[0], np.cumsum(cnt)[:-1]]), cnt)
        idx = starts + np.arange(tot)
        base = np.repeat(exp_base, cnt)
        k0 = int(akvo[a0])
        np.testing.assert_array_equal(after["kv_key"][k0:k0 + tot], kvk[idx] - base * K + p * K,
                                      err_msg=f"replica {p} kv keys")
        np.testing.assert_array_equal(after["kv_val"][k0:k0 + tot], kvv[idx], err_msg=f"replica {p} kv vals")


def test_population_round_sharded_r8_bench_size(comm8):
    """1000 replicas x 10k entries (the gossip_round bench's population) over
    8 loopback ranks: two sharded rounds, each == the oracle per replica."""
    P, E = 1000, 10_000
    h = synth.refmerge_packed(2024, P, E)
    n_l = len(h["l_ts"])
    h = dict(h, kv_key=h["kv_key"].view(np.uint32)[:n_l], kv_val=h["kv_val"].view(np.uint32)[:n_l])
    cuts = [shard.shard_range(P, R, r) for r in range(R)]
    pops = [gossip.NativePopulation.on_member(comm8, i, _slice_population(h, b, e), K, b)
            for i, (b, e) in enumerate(cuts)]
    rng = np.random.default_rng(5)
    try:
        cur = _gather(pops, cuts)
        np.testing.assert_array_equal(cur["ts"], h["l_ts"])
        np.testing.assert_array_equal(cur["kv_key"], h["kv_key"].astype(np.int64))
        for rnd, draw in enumerate((gossip.random_peers, gossip.reference_peers)):
            peers = draw(rng, P, 0, P)
            if rnd == 1:
                assert np.any(peers < 0) and np.any(peers == np.arange(P))
            gossip.NativePopulation.round_sharded(comm8, pops, peers)
            nxt = _gather(pops, cuts)
            _check_round(cur, nxt, peers, h)
            cur = nxt
    finally:
        for p in pops:
            p.close()
