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


@pytest.mark.parametrize("seed", [1, 2])
def test_gossip_rounds_match_reference_simulation(eng, seed):
    rng = np.random.default_rng(seed)
    P = 7
    diffs = [_rand_diff(rng, 1_000 + 13 * i, int(rng.integers(0, 40))) for i in range(P)]
    pop = gossip.Population(eng, _pack(diffs), K)
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
