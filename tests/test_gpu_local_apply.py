"""GPU: batched local apply (crdt_local_apply) -- AddCommand
(main.go:173-215) for a whole population in one device call, against the
Python restatement oracle/pyref.add_command (itself pinned by the hand-derived
KATs of tests/test_oracle_add_command.py): same new Diffs (*Command entries,
same-ms replacement), same CurrentState, same HTTP status per command."""
import numpy as np
import pytest
import torch

from crdt_amd import gossip
from gossip_util import K, KEYS, STRS, _pack, _rand_diff, _same_diffs, _state, _unpack
from oracle import pyref
from test_oracle_add_command import KATS

pytestmark = pytest.mark.gpu


def _cmd_block(cmds_per_replica, keys=KEYS, strs=STRS, k=K):
    """[(ts, {key: val}), ...] per replica -> crdt_local_in host arrays
    (pairs in key order: the restatement's -- one of Go's legal orders)."""
    off, ts, kvo, kk, kv = [0], [], [0], [], []
    for i, cmds in enumerate(cmds_per_replica):
        for t, data in cmds:
            ts.append(t)
            for key in sorted(data):
                kk.append(i * k + keys.index(key))
                kv.append(strs.index(data[key]))
            kvo.append(len(kk))
        off.append(len(ts))
    return {"off": np.array(off), "ts": np.array(ts, np.int64), "kv_off": np.array(kvo),
            "kv_key": np.array(kk, np.uint32), "kv_val": np.array(kv, np.uint32)}


def _set_state(pop, states, keys=KEYS, strs=STRS, k=K):
    st = pop.empty_state()
    kind = np.zeros(pop.P * k, np.uint8)
    sstr = np.zeros(pop.P * k, np.int32)
    for i, s in enumerate(states):
        for key, v in s.items():
            kind[i * k + keys.index(key)] = 1
            sstr[i * k + keys.index(key)] = strs.index(v)
    st["st_kind"].copy_(torch.from_numpy(kind))
    st["st_str"].copy_(torch.from_numpy(sstr))
    pop.state = st


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_local_apply_matches_restatement(eng, seed):
    rng = np.random.default_rng(seed)
    P = 9
    diffs = [_rand_diff(rng, 1_000 + 7 * i, int(rng.integers(0, 40))) for i in range(P)]
    pop = gossip.Population(eng, _pack(diffs), K)
    states = [{} for _ in range(P)]
    for rnd in range(3):
        cmds, exp_status = [], []
        for i in range(P):
            lo = min(diffs[i]) if diffs[i] else 1_000
            hi = max(diffs[i]) if diffs[i] else 1_050
            mine = []
            for _ in range(int(rng.integers(0, 25))):
                t = int(rng.integers(lo - 5, hi + 20))           # on / between / after Diff entries, same-ms repeats
                data = {KEYS[int(q)]: STRS[int(rng.integers(0, len(STRS)))]
                        for q in rng.choice(K, int(rng.integers(0, 4)), replace=False)}
                mine.append((t, data))
                exp_status.append(pyref.add_command(diffs[i], states[i], t, data))
            cmds.append(mine)
        got_status = pop.apply_local(_cmd_block(cmds))
        np.testing.assert_array_equal(got_status, exp_status)
        _same_diffs(_unpack(pop), diffs)
        assert _state(pop) == states, f"round {rnd}"


def test_local_apply_then_gossip_round(eng):
    """Local writes, then a pull round (merge rebuilds CurrentState from the
    remote entries only, main.go:76-80), then more local writes."""
    from gossip_util import _host_round
    rng = np.random.default_rng(8)
    P = 6
    diffs = [_rand_diff(rng, 3_000 + 5 * i, int(rng.integers(5, 30))) for i in range(P)]
    pop = gossip.Population(eng, _pack(diffs), K)
    states = [{} for _ in range(P)]
    for step in range(4):
        cmds, exp = [], []
        for i in range(P):
            t0 = max(diffs[i]) if diffs[i] else 3_000
            mine = [(t0 + int(rng.integers(-3, 6)), {KEYS[int(rng.integers(0, K))]: STRS[int(rng.integers(0, 10))]})
                    for _ in range(int(rng.integers(1, 6)))]
            exp += [pyref.add_command(diffs[i], states[i], t, d) for t, d in mine]
            cmds.append(mine)
        np.testing.assert_array_equal(pop.apply_local(_cmd_block(cmds)), exp)
        _same_diffs(_unpack(pop), diffs)
        assert _state(pop) == states
        peers = gossip.random_peers(rng, P, 0, P)
        pop.round(peers)
        diffs, states = _host_round(diffs, peers)
        _same_diffs(_unpack(pop), diffs)
        assert _state(pop) == states


def test_local_apply_kats(eng):
    """The hand-derived AddCommand KATs, one replica each, in ONE device call."""
    keys = sorted({k for kat in KATS for c in kat[3] for k in c[1]} | {k for kat in KATS for k in kat[2]} |
                  {k for kat in KATS for v in kat[1].values() for k in v})
    strs = sorted({v for kat in KATS for c in kat[3] for v in c[1].values()} |
                  {v for kat in KATS for v in kat[2].values()} | {v for kat in KATS for d in kat[1].values()
                                                                 for v in d.values()})
    k = len(keys)
    blob = "".join(strs).encode()
    so = np.zeros(len(strs) + 1, np.int64)
    so[1:] = np.cumsum([len(s.encode()) for s in strs])
    off, ts, org, kvo, kk, kv = [0], [], [], [0], [], []
    for i, kat in enumerate(KATS):
        for t in sorted(kat[1]):
            ts.append(t)
            org.append(0)
            for key, v in sorted(kat[1][t].items()):
                kk.append(i * k + keys.index(key))
                kv.append(strs.index(v))
            kvo.append(len(kk))
        off.append(len(ts))
    host = {"replicas": len(KATS), "l_off": np.array(off), "l_ts": np.array(ts, np.int64),
            "l_origin": np.array(org, np.uint8), "l_kv": np.array(kvo), "kv_key": np.array(kk, np.uint32),
            "kv_val": np.array(kv, np.uint32), "str_bytes": np.frombuffer(blob, np.uint8).copy(), "str_off": so}
    pop = gossip.Population(eng, host, k)
    _set_state(pop, [kat[2] for kat in KATS], keys, strs, k)
    status = pop.apply_local(_cmd_block([kat[3] and [(c[0], c[1]) for c in kat[3]] for kat in KATS], keys, strs, k))
    np.testing.assert_array_equal(status, [c[2] for kat in KATS for c in kat[3]])
    h = pop.to_host()
    kind, sstr, ssum = (pop.state[x].cpu().numpy() for x in ("st_kind", "st_str", "st_sum"))
    for i, kat in enumerate(KATS):
        assert h["ts"][h["off"][i]:h["off"][i + 1]].tolist() == kat[4], kat[0]
        assert all(h["origin"][h["off"][i]:h["off"][i + 1]] == 1), kat[0]
        st = {}
        for j, key in enumerate(keys):
            s = i * k + j
            if kind[s] == 1:
                st[key] = strs[int(sstr[s])]
            elif kind[s] == 2:
                st[key] = str(int(ssum[s]))
        assert st == kat[5], kat[0]


def test_local_apply_over_the_per_call_limit(eng):
    """More than 4096 commands for one replica (crdt_local_apply's per-call
    limit): Population.apply_local runs them as several device
    calls in arrival order, == the restatement; a raw over-limit call raises
    CRDT_DEV_RANGE and applies nothing of that replica."""
    rng = np.random.default_rng(11)
    P = 3
    diffs = [_rand_diff(rng, 1_000 + 7 * i, 20) for i in range(P)]
    pop = gossip.Population(eng, _pack(diffs), K)
    states = [{} for _ in range(P)]
    cmds, exp = [], []
    for i, n in enumerate((9000, 5, 4097)):
        lo = min(diffs[i])
        mine = []
        for _ in range(n):
            t = int(rng.integers(lo - 5, lo + 6000))
            data = {KEYS[int(rng.integers(0, K))]: STRS[int(rng.integers(0, len(STRS)))]}
            mine.append((t, data))
            exp.append(pyref.add_command(diffs[i], states[i], t, data))
        cmds.append(mine)
    np.testing.assert_array_equal(pop.apply_local(_cmd_block(cmds)), exp)
    _same_diffs(_unpack(pop), diffs)
    assert _state(pop) == states
    # one device call over the limit: flagged, and the replica's Diff range / state untouched
    before = pop.to_host()
    st_before = {k: v.clone() for k, v in pop.state.items()}
    blk = _cmd_block([[(5_000_000 + j, {KEYS[0]: STRS[1]}) for j in range(4097)], [], []])
    with pytest.raises(Exception, match="device-side failure"):
        pop._apply_local_once(blk)
    after = pop.to_host()
    for k in ("off", "ts", "origin"):
        np.testing.assert_array_equal(before[k], after[k])
    for k, v in st_before.items():
        assert torch.equal(v, pop.state[k]), k
