"""GPU: anti-entropy rounds behind the C-ABI (crdt_population_*,
csrc/population.hip) against the host simulation of the
reference's rounds on oracle/pyref.py (main.go:226-258): every replica pulls
its peer's whole Diff as remote maps and merges; self-pulls rebuild
CurrentState, dead peers (-1) skip the round.

* crdt_population_round on one population;
* crdt_population_round_sharded over a 1-member RCCL communicator and over
  loopback communicators of 2, 3 and 5 ranks on the one GPU (replicas split
  by crdt_shard_range; every rank receives only the Diffs its replicas pull).
"""
import numpy as np
import pytest
from knobs import set_knob

from crdt_amd import gossip, shard
from gossip_util import K, KEYS, STRS, _host_round, _pack, _rand_diff, _same_diffs
from oracle import pyref

pytestmark = pytest.mark.gpu


def _unpack_native(h, P, strs=STRS):
    out = []
    for i in range(P):
        d = {}
        for e in range(int(h["off"][i]), int(h["off"][i + 1])):
            kv = {KEYS[int(h["kv_key"][q]) - i * K]: strs[int(h["kv_val"][q])]
                  for q in range(int(h["kv_off"][e]), int(h["kv_off"][e + 1]))}
            d[int(h["ts"][e])] = pyref.Command(kv) if h["origin"][e] else kv
        out.append(d)
    return out


def _state_native(h, P, strs=STRS):
    out = []
    for i in range(P):
        st = {}
        for k in range(K):
            s = i * K + k
            if h["st_kind"][s] == 1:
                st[KEYS[k]] = strs[int(h["st_str"][s])]
            elif h["st_kind"][s] == 2:
                st[KEYS[k]] = str(int(h["st_sum"][s]))
        out.append(st)
    return out


@pytest.mark.parametrize("draw", ["random", "reference"])
@pytest.mark.parametrize("seed", [1, 2])
def test_population_rounds_match_reference_simulation(eng, seed, draw):
    rng = np.random.default_rng(seed)
    P = 9
    diffs = [_rand_diff(rng, 1_000 + 13 * i, int(rng.integers(0, 40))) for i in range(P)]
    pop = gossip.NativePopulation(eng, _pack(diffs), K)
    states = [{} for _ in range(P)]
    try:
        saw = set()
        for rnd in range(6):
            peers = (gossip.random_peers if draw == "random" else gossip.reference_peers)(rng, P, 0, P)
            saw |= {"self"} if np.any(peers == np.arange(P)) else set()
            saw |= {"dead"} if np.any(peers < 0) else set()
            pop.round(peers)
            diffs, states = _host_round(diffs, peers, states)
            h = pop.read()
            _same_diffs(_unpack_native(h, P), diffs)
            assert _state_native(h, P) == states, f"round {rnd}"
        if draw == "reference":
            assert saw == {"self", "dead"}
    finally:
        pop.close()


def test_population_round_rejects_remote_peer(eng):
    from crdt_amd import _lib
    rng = np.random.default_rng(3)
    diffs = [_rand_diff(rng, 100, 5) for _ in range(3)]
    pop = gossip.NativePopulation(eng, _pack(diffs), K, first=10)
    try:
        with pytest.raises(_lib.CrdtError):
            pop.round([10, 11, 3])                       # replica 3 lives on another rank
    finally:
        pop.close()


def _sharded_rounds(comm, total, seed, rounds=5):
    rng = np.random.default_rng(seed)
    diffs = [_rand_diff(rng, 2_000 + 11 * i, int(rng.integers(0, 35))) for i in range(total)]
    R = comm.nranks
    cuts = [shard.shard_range(total, R, r) for r in range(R)]
    pops = []
    for i in range(comm.members):
        b, e = cuts[comm.rank0 + i]
        pops.append(gossip.NativePopulation.on_member(comm, i, _pack(diffs[b:e]), K, b))
    states = [{} for _ in range(total)]
    try:
        for rnd in range(rounds):
            peers = (gossip.random_peers if rnd % 2 == 0 else gossip.reference_peers)(rng, total, 0, total)
            gossip.NativePopulation.round_sharded(comm, pops, peers)
            diffs, states = _host_round(diffs, peers, states)
            for i, p in enumerate(pops):
                b, e = cuts[comm.rank0 + i]
                h = p.read()
                _same_diffs(_unpack_native(h, e - b), diffs[b:e])
                assert _state_native(h, e - b) == states[b:e], f"round {rnd}, member {i}"
    finally:
        for p in pops:
            p.close()


@pytest.mark.parametrize("world,total", [(2, 7), (3, 10), (5, 4)])
def test_population_sharded_rounds_loopback(world, total):
    """R ranks on the loopback transport (5 ranks over 4 replicas: one rank
    holds none)."""
    comm = shard.Comm.loopback(0, world)
    try:
        _sharded_rounds(comm, total, 40 + world)
    finally:
        comm.close()


def test_population_sharded_round_rccl_one_rank(eng):
    """The same protocol through a 1-member RCCL communicator (ncclCommInitRank)
    -- self sends / receives of the point-to-point group."""
    comm = shard.Comm.init_rank(eng)
    try:
        _sharded_rounds(comm, 6, 77, rounds=3)
    finally:
        comm.close()


def test_population_undo_restores_the_previous_round(eng):
    """crdt_population_undo: the Diffs and CurrentState of before the last
    round, once; repeating the round then gives the same result."""
    from crdt_amd import _lib
    rng = np.random.default_rng(9)
    P = 6
    diffs = [_rand_diff(rng, 3_000 + 5 * i, int(rng.integers(1, 30))) for i in range(P)]
    pop = gossip.NativePopulation(eng, _pack(diffs), K)
    try:
        peers = gossip.reference_peers(rng, P, 0, P)
        pop.round(gossip.random_peers(rng, P, 0, P))
        before = pop.read()
        pop.round(peers)
        after = pop.read()
        pop.undo()
        back = pop.read()
        for k in before:
            np.testing.assert_array_equal(back[k], before[k], err_msg=k)
        with pytest.raises(_lib.CrdtError):
            pop.undo()                                   # once only
        pop.round(peers)
        again = pop.read()
        for k in after:
            np.testing.assert_array_equal(again[k], after[k], err_msg=k)
    finally:
        pop.close()


@pytest.mark.diag
def test_population_failed_round_leaves_nothing_to_undo(eng):
    """A round that fails after the previous round succeeded (fault injection
    "fail.refmerge": its merge call returns an error) leaves the population
    as it was, and undo is refused: the spare buffers no longer hold a
    consistent snapshot (population.hip)."""
    from crdt_amd import _lib
    rng = np.random.default_rng(19)
    P = 5
    diffs = [_rand_diff(rng, 4_000 + 7 * i, int(rng.integers(1, 25))) for i in range(P)]
    pop = gossip.NativePopulation(eng, _pack(diffs), K)
    try:
        pop.round(gossip.random_peers(rng, P, 0, P))
        after = pop.read()
        set_knob(b"fail.refmerge", 1)
        try:
            with pytest.raises(_lib.CrdtError):
                pop.round(gossip.random_peers(rng, P, 0, P))
        finally:
            set_knob(b"fail.refmerge", 0)
        with pytest.raises(_lib.CrdtError):
            pop.undo()
        now = pop.read()
        for k in after:
            np.testing.assert_array_equal(now[k], after[k], err_msg=k)
        eng.check_device()
    finally:
        pop.close()


@pytest.mark.parametrize("seed", [3, 4])
def test_population_commands_and_rounds(eng, seed):
    """AddCommand on every replica through crdt_population_add_commands
    (main.go:173-215: same-ms replaces, early return after a new key, 500 on
    an unparsable value) between reference-drawn rounds == pyref: statuses,
    Diffs and CurrentState."""
    from test_gpu_local_apply import _cmd_block
    rng = np.random.default_rng(seed)
    P = 8
    diffs = [_rand_diff(rng, 1_000 + 13 * i, int(rng.integers(0, 30))) for i in range(P)]
    pop = gossip.NativePopulation(eng, _pack(diffs), K)
    states = [{} for _ in range(P)]
    try:
        for rnd in range(5):
            cmds, exp = [], []
            for i in range(P):
                t0 = max(diffs[i]) if diffs[i] else 1_000
                mine = [(t0 + int(rng.integers(-3, 6)), {KEYS[int(rng.integers(0, K))]: STRS[int(rng.integers(0, 12))]})
                        for _ in range(int(rng.integers(0, 4)))]
                exp += [pyref.add_command(diffs[i], states[i], t, d) for t, d in mine]
                cmds.append(mine)
            np.testing.assert_array_equal(pop.add_commands(_cmd_block(cmds)), exp)
            h = pop.read()
            _same_diffs(_unpack_native(h, P), diffs)
            assert _state_native(h, P) == states, f"after commands, round {rnd}"
            peers = gossip.reference_peers(rng, P, 0, P)
            pop.round(peers)
            diffs, states = _host_round(diffs, peers, states)
            h = pop.read()
            _same_diffs(_unpack_native(h, P), diffs)
            assert _state_native(h, P) == states, f"round {rnd}"
    finally:
        pop.close()


def test_population_commands_over_the_per_call_limit(eng):
    """5000 commands on one replica (past crdt_local_apply's 4096 per call):
    chunked in arrival order == pyref."""
    from test_gpu_local_apply import _cmd_block
    rng = np.random.default_rng(12)
    P = 3
    diffs = [_rand_diff(rng, 100 + i, 3) for i in range(P)]
    pop = gossip.NativePopulation(eng, _pack(diffs), K)
    states = [{} for _ in range(P)]
    try:
        cmds, exp = [], []
        for i in range(P):
            n = 5000 if i == 1 else 7
            mine = [(10_000 + j // 2, {KEYS[int(rng.integers(0, K))]: STRS[int(rng.integers(0, 10))]}) for j in range(n)]
            exp += [pyref.add_command(diffs[i], states[i], t, d) for t, d in mine]
            cmds.append(mine)
        np.testing.assert_array_equal(pop.add_commands(_cmd_block(cmds)), exp)
        h = pop.read()
        _same_diffs(_unpack_native(h, P), diffs)
        assert _state_native(h, P) == states
    finally:
        pop.close()


def _wire_tables(eng):
    from crdt_amd import codec
    keys, vals = codec.StrTab(eng), codec.StrTab(eng)
    assert keys.intern(KEYS).tolist() == list(range(K))            # key id = KEYS index
    assert vals.intern(STRS).tolist() == list(range(len(STRS)))    # value id = the population's string id
    return keys, vals


@pytest.mark.parametrize("one", [False, True], ids=["pairs", "one_pair"])
@pytest.mark.parametrize("seed", [5, 6])
def test_population_wire_rounds_match_reference_simulation(eng, seed, one):
    """crdt_population_round_wire: every replica's pull arrives as a binary
    gossip body in HBM (main.go:159, :245-256), decoded on the device and
    merged == the pyref simulation; failed GETs (empty bodies) skip the
    round, self-pulls rebuild CurrentState, a value the tables have not seen
    is interned and lands in the population's arena (adopted from vals),
    and AddCommand between wire rounds uses the same ids.  one: every
    entry holds one pair (the one-pair kv passes, kept through the rounds)."""
    from test_gpu_codec import _serve, _upload
    from test_gpu_local_apply import _cmd_block
    rng = np.random.default_rng(seed)
    P = 7
    gen = _rand_diff_one if one else _rand_diff
    diffs = [gen(rng, 1_000 + 13 * i, int(rng.integers(0, 30))) for i in range(P)]
    keys, vals = _wire_tables(eng)
    pop = gossip.NativePopulation(eng, _pack(diffs), K)
    states = [{} for _ in range(P)]
    try:
        for rnd in range(6):
            peers = (gossip.random_peers if rnd % 2 else gossip.reference_peers)(rng, P, 0, P)
            pulls = [dict(diffs[q]) if q >= 0 else None for q in peers]
            if rnd == 2:                                 # a value no table holds yet
                t = 50_000 + rnd
                pulls[0] = dict(pulls[0] or {})
                pulls[0][t] = {KEYS[1]: "fresh-" + str(seed)}
            bodies = [_serve(pl) if pl is not None else b"" for pl in pulls]
            data, off = _upload(eng, bodies)
            pop.round_wire(data, off, keys, vals)
            strs = [x.decode() for x in vals.strings()]
            for i in range(P):
                if pulls[i] is None:
                    continue                             # a failed GET: no merge (main.go:234-239)
                diffs[i], states[i] = pyref.merge(diffs[i], {t: dict(v) for t, v in pulls[i].items()})
            h = pop.read()
            _same_diffs(_unpack_native(h, P, strs), diffs)
            assert _state_native(h, P, strs) == states, f"round {rnd}"
            if rnd == 3:                                 # AddCommand between wire rounds (main.go:173-215)
                cmds, exp = [], []
                for i in range(P):
                    t0 = max(diffs[i]) if diffs[i] else 1_000
                    mine = [(t0 + 1 + j, {KEYS[int(rng.integers(0, K))]: STRS[int(rng.integers(0, 12))]})
                            for j in range(int(rng.integers(0, 3)))]
                    exp += [pyref.add_command(diffs[i], states[i], t, d) for t, d in mine]
                    cmds.append(mine)
                np.testing.assert_array_equal(pop.add_commands(_cmd_block(cmds)), exp)
    finally:
        pop.close()


def test_population_wire_round_refusals(eng):
    """A body the device decode does not take (here: a nil map, and one
    truncated) fails the round with CRDT_E_UNSORTED and its status, the
    population unchanged; a value table that does not hold the population's
    strings at their ids is refused before anything is decoded."""
    from crdt_amd import _lib, codec
    from test_gpu_codec import _raw_body, _serve, _upload
    rng = np.random.default_rng(8)
    P = 3
    diffs = [_rand_diff(rng, 100 + i, 5) for i in range(P)]
    keys, vals = _wire_tables(eng)
    pop = gossip.NativePopulation(eng, _pack(diffs), K)
    try:
        before = pop.read()
        good = _serve(diffs[1])
        for bad in (_raw_body([(7, None)]), good[:-1]):
            data, off = _upload(eng, [good, bad, good])
            with pytest.raises(_lib.CrdtError) as ei:
                pop.round_wire(data, off, keys, vals)
            assert ei.value.body_status[1] != 0 and ei.value.body_status[0] == 0
            after = pop.read()
            for k in before:
                np.testing.assert_array_equal(after[k], before[k], err_msg=k)
        other = codec.StrTab(eng)
        other.intern(list(reversed(STRS)))               # the same strings at other ids
        data, off = _upload(eng, [good, good, good])
        with pytest.raises(_lib.CrdtError):
            pop.round_wire(data, off, keys, other)
    finally:
        pop.close()


@pytest.mark.parametrize("how", ["refused_first", "shared_vals"])
def test_population_first_wire_round_with_strings_past_the_arena(eng, how):
    """ADVICE r05 (population.hip, pop.wire_early): on a population's FIRST
    wire round vals may already hold strings past the population's own
    arena -- interned by a refused earlier round's good bodies, or by another
    user of a shared table.  A pulled value resolving to such an id must take
    part in the replay fold (main.go:75-98) == pyref."""
    from crdt_amd import _lib
    from test_gpu_codec import _raw_body, _serve, _upload
    rng = np.random.default_rng(31)
    P = 3
    diffs = [_rand_diff(rng, 100 + 7 * i, 6) for i in range(P)]
    keys, vals = _wire_tables(eng)
    pop = gossip.NativePopulation(eng, _pack(diffs), K)
    try:
        # below every puller's max(L) (t0 >= 100), new strings only
        pull = {50: {KEYS[2]: "17"}, 51: {KEYS[2]: "past-the-arena"}, 52: {KEYS[3]: "40"}, 53: {KEYS[3]: "2"}}
        if how == "shared_vals":
            vals.intern([b"40", b"past-the-arena", b"2", b"17"])
        else:
            good = _serve(pull)
            data, off = _upload(eng, [good, _raw_body([(7, None)]), good])
            with pytest.raises(_lib.CrdtError):
                pop.round_wire(data, off, keys, vals)
        if how == "shared_vals":
            assert len(vals) > len(STRS)
        pulls = [pull, None, pull]
        data, off = _upload(eng, [_serve(p) if p is not None else b"" for p in pulls])
        pop.round_wire(data, off, keys, vals)
        strs = [x.decode() for x in vals.strings()]
        states = [{} for _ in range(P)]
        for i in range(P):
            if pulls[i] is not None:
                diffs[i], states[i] = pyref.merge(diffs[i], {t: dict(v) for t, v in pulls[i].items()})
        h = pop.read()
        _same_diffs(_unpack_native(h, P, strs), diffs)
        assert _state_native(h, P, strs)[0] == states[0]
        assert _state_native(h, P, strs) == states
    finally:
        pop.close()


def _rand_diff_one(rng, t0, n):
    """A Diff whose every entry holds exactly one pair (the reference's load
    generator: one key per command, main.go:282)."""
    d, t = {}, t0
    for _ in range(n):
        t += int(rng.integers(1, 5))
        kv = {KEYS[int(rng.integers(0, K))]: STRS[int(rng.integers(0, len(STRS)))]}
        d[t] = pyref.Command(kv) if rng.random() < 0.5 else kv
    return d


@pytest.mark.parametrize("seed", [21, 22])
def test_population_one_pair_rounds(eng, seed):
    """Populations whose entries all hold one pair take the one-pair kv
    passes (refmerge_batch_pull_one_pair: tile pair counts from the emitted
    counts): rounds (self-pulls, dead peers), undo, one-pair AddCommands, then
    multi-pair AddCommands (which drop the invariant) and more rounds -- all
    == pyref."""
    from test_gpu_local_apply import _cmd_block
    rng = np.random.default_rng(seed)
    P = 9
    diffs = [_rand_diff_one(rng, 1_000 + 17 * i, int(rng.integers(0, 60))) for i in range(P)]
    pop = gossip.NativePopulation(eng, _pack(diffs), K)
    states = [{} for _ in range(P)]
    try:
        for rnd in range(8):
            if rnd in (3, 6):                            # AddCommand: one pair each, then (round 6) several
                cmds, exp = [], []
                for i in range(P):
                    t0 = max(diffs[i]) if diffs[i] else 1_000
                    npairs = 1 if rnd == 3 else 2
                    mine = [(t0 + 1 + j, {KEYS[int(q)]: STRS[int(rng.integers(0, 12))]
                                          for q in rng.choice(K, npairs, replace=False)})
                            for j in range(int(rng.integers(0, 3)))]
                    exp += [pyref.add_command(diffs[i], states[i], t, d) for t, d in mine]
                    cmds.append(mine)
                np.testing.assert_array_equal(pop.add_commands(_cmd_block(cmds)), exp)
            peers = (gossip.random_peers if rnd % 2 else gossip.reference_peers)(rng, P, 0, P)
            if rnd == 1:                                 # a round undone and drawn again
                pop.round(gossip.random_peers(rng, P, 0, P))
                pop.undo()
            pop.round(peers)
            diffs, states = _host_round(diffs, peers, states)
            h = pop.read()
            _same_diffs(_unpack_native(h, P), diffs)
            assert _state_native(h, P) == states, f"round {rnd}"
    finally:
        pop.close()
