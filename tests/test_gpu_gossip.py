"""GPU: anti-entropy rounds (crdt_amd.gossip) against a
host simulation of the reference's rounds with the Python restatement of
merge() (oracle/pyref.py): every replica pulls its peer's whole Diff as
remote maps (main.go:159, :245-256) and merges (main.go:257); local writes
(*Command, main.go:187) between rounds.  Synchronous rounds; one GPU, and a
2-rank split emulated in one process through the import-block path."""
import numpy as np
import pytest

from crdt_amd import gossip
from gossip_util import K, _host_round, _local_writes, _pack, _rand_diff, _same_diffs, _state, _unpack

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("mode", ["inplace_kv", "assembled_kv", "assembled_gather"])
@pytest.mark.parametrize("seed", [1, 2])
def test_gossip_rounds_match_reference_simulation(eng, seed, mode):
    """inplace: the merge reads the peers' Diffs where they lie
    (crdt_refmerge_batch_pull, the default) / assembled: RemoteDiffs built by
    segmented copies first; kv: the new Diff's kv pairs copied by the merge's
    tile pass (the default) / gather: gathered by src afterwards (assembled
    pulls only: the gather does not re-base the pulled key slots)."""
    rng = np.random.default_rng(seed)
    P = 7
    diffs = [_rand_diff(rng, 1_000 + 13 * i, int(rng.integers(0, 40))) for i in range(P)]
    pop = gossip.Population(eng, _pack(diffs), K)
    pop.pull_inplace = mode.startswith("inplace")
    pop.kv_fused = mode.endswith("_kv")
    for rnd in range(5):
        peers = gossip.random_peers(rng, P, 0, P)
        pop.round(peers)
        diffs, states = _host_round(diffs, peers)
        _same_diffs(_unpack(pop), diffs)
        assert _state(pop) == states
        if rnd % 2 == 0:
            pop.append_local(_local_writes(rng, diffs))
            _same_diffs(_unpack(pop), diffs)


def test_gossip_two_rank_import_block(eng):
    """Replicas split over two 'ranks' (two populations on one GPU); every
    round each pulls from the import block built from both ranks' exports
    (the all-gather of gossip.sharded_round, done in-process)."""
    rng = np.random.default_rng(5)
    P, cut = 6, 4
    diffs = [_rand_diff(rng, 5_000 + 7 * i, int(rng.integers(5, 30))) for i in range(P)]
    pops = [gossip.Population(eng, _pack(diffs[:cut]), K, first=0),
            gossip.Population(eng, _pack(diffs[cut:]), K, first=cut)]
    owner_first = np.array([0] * cut + [cut] * (P - cut))
    for _ in range(4):
        peers = gossip.random_peers(rng, P, 0, P)
        blocks = [p.export_block() for p in pops]
        imps = [p.import_from_blocks(blocks) for p in pops]
        for p, imp in zip(pops, imps):
            mine = peers[p.first:p.first + p.P]
            p.round(mine, imp=imp, peer_first=owner_first[mine])
        diffs, states = _host_round(diffs, peers)
        _same_diffs(_unpack(pops[0]) + _unpack(pops[1]), diffs)
        assert _state(pops[0]) + _state(pops[1]) == states


def test_random_peers_never_self():
    rng = np.random.default_rng(0)
    for _ in range(50):
        p = gossip.random_peers(rng, 9, 0, 9)
        assert np.all(p != np.arange(9)) and np.all((p >= 0) & (p < 9))


@pytest.mark.parametrize("seed", [3, 4])
def test_reference_friend_list_rounds(eng, seed):
    """Peers drawn like the reference (main.go:219-222, :230): a friend list
    holding every replica -- itself included -- and as many dead ports.  A
    self-pull still merges and rebuilds CurrentState from the remote entries
    (main.go:76), dropping what local writes applied to it; a dead pick skips
    the round (main.go:234-239) and keeps the local writes' state.  Local
    writes go through the device AddCommand (Population.apply_local) between
    rounds.  == the pyref simulation."""
    from oracle import pyref
    from test_gpu_local_apply import _cmd_block
    from gossip_util import KEYS, STRS
    rng = np.random.default_rng(seed)
    P = 8
    diffs = [_rand_diff(rng, 1_000 + 13 * i, int(rng.integers(0, 30))) for i in range(P)]
    pop = gossip.Population(eng, _pack(diffs), K)
    states = [{} for _ in range(P)]
    saw_self = saw_dead = False
    for rnd in range(6):
        cmds, exp = [], []
        for i in range(P):
            t0 = max(diffs[i]) if diffs[i] else 1_000
            mine = [(t0 + int(rng.integers(1, 6)), {KEYS[int(rng.integers(0, K))]: STRS[int(rng.integers(0, 10))]})
                    for _ in range(int(rng.integers(0, 3)))]
            exp += [pyref.add_command(diffs[i], states[i], t, d) for t, d in mine]
            cmds.append(mine)
        np.testing.assert_array_equal(pop.apply_local(_cmd_block(cmds)), exp)
        peers = gossip.reference_peers(rng, P, 0, P)
        saw_self |= bool(np.any(peers == np.arange(P)))
        saw_dead |= bool(np.any(peers < 0))
        pop.round(peers)
        diffs, states = _host_round(diffs, peers, states)
        _same_diffs(_unpack(pop), diffs)
        assert _state(pop) == states, f"round {rnd}"
    assert saw_self and saw_dead


def test_reference_peers_distribution():
    rng = np.random.default_rng(1)
    d = np.concatenate([gossip.reference_peers(rng, 5, 0, 5) for _ in range(2000)])
    assert d.min() == -1 and d.max() == 4
    assert 0.45 < np.mean(d < 0) < 0.55                 # 5 of the 10 friends are dead (main.go:219-222)
