"""GPU: the device-resident Server (server.hip) through the reference-shaped
API -- Diffs stay in HBM between merges, pulls are decoded on the device,
local writes are queued for crdt_local_apply, and the host view is rebuilt
only when read.  Checked over mixed multi-round schedules against the Python
restatement of merge() / AddCommand (oracle/pyref.py, main.go:35-100,
:173-215) and the JSON restatement of the wire (oracle/gojson.py)."""
import numpy as np
import pytest

from crdt_amd.refmerge import Command
from crdt_amd.server import Server, merge_servers
from oracle import gojson, pyref

pytestmark = pytest.mark.gpu

KEYS = [f"k{i}" for i in range(6)] + ["zz"]
VALS = [str(v) for v in range(-20, -10)] + ["x", "007", "+3"]


def _rand_value(rng):
    return {KEYS[int(q)]: VALS[int(rng.integers(0, len(VALS)))] for q in rng.choice(len(KEYS), int(rng.integers(1, 3)),
                                                                                  replace=False)}


def _sig(diff):
    return [[t, "local" if isinstance(v, (Command, pyref.Command)) else "remote"] for t, v in sorted(diff.items())]


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_resident_servers_match_restatement(eng, seed):
    rng = np.random.default_rng(seed)
    P = 4
    model = [({}, {}) for _ in range(P)]                       # (diff, state) per replica
    srv = [Server(eng, 8080 + i) for i in range(P)]
    clock = [1_000 + 37 * i for i in range(P)]
    for i in range(P):                                         # some history before the first merge
        for _ in range(int(rng.integers(5, 25))):
            clock[i] += int(rng.integers(1, 4))
            v = _rand_value(rng)
            if rng.random() < 0.5:
                srv[i].Diff.Put(clock[i], Command(v))
                model[i][0][clock[i]] = pyref.Command(v)
            else:
                srv[i].Diff.Put(clock[i], v)
                model[i][0][clock[i]] = dict(v)
    for rnd in range(6):
        # local writes (AddCommand, main.go:173-215), some at an existing ts (same-ms overwrite)
        for i in range(P):
            for _ in range(int(rng.integers(0, 4))):
                clock[i] += int(rng.integers(0, 3))
                v = _rand_value(rng)
                assert srv[i].AddCommand(clock[i], v) == pyref.add_command(model[i][0], model[i][1], clock[i], v)
        # pulls: a random peer's whole Diff, binary (device decode) or JSON (host parse)
        peers = [int((i + 1 + rng.integers(0, P - 1)) % P) for i in range(P)]
        bodies = []
        for i, q in enumerate(peers):
            if rng.random() < 0.7:
                st, body = srv[q].GossipBinary()
                bodies.append(("bin", body))
            else:
                st, body = srv[q].Gossip()
                assert body == gojson.marshal_diff(model[q][0])          # the served JSON, byte for byte
                bodies.append(("json", body))
            assert st == 200
        remotes = [{t: dict(v) for t, v in model[q][0].items()} for q in peers]
        for (kind, body), s in zip(bodies, srv):
            assert (s.IngestBinary(body) if kind == "bin" else s.IngestGossip(body)) == 0
        if rnd % 2 == 0:
            merge_servers(srv)                                   # one batched device merge
        else:
            for s in srv:
                s.merge()
        for i in range(P):
            model[i] = pyref.merge(model[i][0], remotes[i])
        for i in range(P):
            assert srv[i].CurrentState == model[i][1], f"round {rnd} replica {i}"
            if rnd % 3 == 2:                                     # host view rebuilt from HBM on read
                assert srv[i].DiffSignature == _sig(model[i][0]), f"round {rnd} replica {i}"
    for s in srv:
        s.close()


def test_resident_diff_put_and_remote_put_between_merges(eng):
    """Host-side mutations (Diff.Put / RemoteDiff.Put) on a device-resident
    server: the Diff is rebuilt on the host, re-uploaded at the next merge."""
    s = Server(eng, 8080)
    diff = {10: pyref.Command({"a": "1"}), 20: {"b": "2"}}
    s.Diff.Put(10, Command({"a": "1"}))
    s.Diff.Put(20, {"b": "2"})
    remote = {5: {"a": "3"}, 15: {"b": "4"}, 25: {"c": "9"}}
    for t, v in remote.items():
        s.RemoteDiff.Put(t, v)
    s.merge()
    diff, st = pyref.merge(diff, remote)
    assert s.CurrentState == st and s.DiffSignature == _sig(diff)
    s.Diff.Put(30, {"a": "7"})                                    # a remote-form entry put directly
    diff[30] = {"a": "7"}
    s.RemoteDiff.Put(12, {"a": "1"})
    assert s.RemoteDiff.Size() == 1
    s.merge()
    diff, st = pyref.merge(diff, {12: {"a": "1"}})
    assert s.CurrentState == st and s.DiffSignature == _sig(diff)
    assert s.RemoteDiff.Size() == 0
    s.close()


def test_resident_server_many_queued_writes(eng):
    """More than 4096 distinct-ts local writes queued between merges of a
    device-resident server: they are applied to the device Diff in
    chunks and none is lost."""
    rng = np.random.default_rng(5)
    s = Server(eng, 8080)
    diff, state = {}, {}
    for t in range(10, 400, 7):
        v = _rand_value(rng)
        s.Diff.Put(t, v)
        diff[t] = dict(v)
    s.RemoteDiff.Put(3, {"k1": "-12"})
    s.merge()                                                     # device-resident from here on
    diff, state = pyref.merge(diff, {3: {"k1": "-12"}})
    assert s.CurrentState == state
    for j in range(9000):
        t = 500 + j + (j // 3)                                    # distinct ms, a few gaps
        v = _rand_value(rng)
        assert s.AddCommand(t, v) == pyref.add_command(diff, state, t, v)
    remote = {1: {"k2": "-15"}, 600: {"k2": "-11"}, 20_000: {"k3": "x"}}
    for t, v in remote.items():
        s.RemoteDiff.Put(t, v)
    s.merge()
    diff, state = pyref.merge(diff, remote)
    assert s.CurrentState == state
    assert s.DiffSignature == _sig(diff)
    s.close()


@pytest.mark.parametrize("wire", ["json", "bin"])
def test_self_pull_round_trip(eng, wire):
    """A server that pulls ITSELF (the reference's friend list holds its own
    port, main.go:219-222, :230): its Diff -- local *Command entries included
    -- goes out through Gossip (main.go:159), comes back as remote maps
    (main.go:245-256) and merges (main.go:257).  Nothing is inserted (every
    ts is already local, local wins, main.go:54-65) and CurrentState is
    rebuilt from the remote-origin entries only (main.go:76-80), dropping the
    local writes' direct applies.  == pyref, twice (resident on the second)."""
    rng = np.random.default_rng(9)
    s = Server(eng, 8080)
    diff, state = {}, {}
    for t in range(100, 160, 3):
        v = _rand_value(rng)
        if rng.random() < 0.5:
            s.Diff.Put(t, v)
            diff[t] = dict(v)
        else:
            assert s.AddCommand(t, v) == pyref.add_command(diff, state, t, v)
    for _ in range(2):
        st, body = s.Gossip() if wire == "json" else s.GossipBinary()
        assert st == 200
        assert (s.IngestGossip(body) if wire == "json" else s.IngestBinary(body)) == 0
        remote = {t: dict(v) for t, v in diff.items()}
        s.merge()
        diff, state = pyref.merge(diff, remote)
        assert s.CurrentState == state
        assert s.DiffSignature == _sig(diff)
        assert s.AddCommand(200, {"k1": "-13"}) == pyref.add_command(diff, state, 200, {"k1": "-13"})
        assert s.CurrentState == state
    s.close()


@pytest.mark.parametrize("seed", [5, 6])
def test_resident_state_updates_and_double_pulls(eng, seed):
    """Merges with no AddCommand in between (CurrentState updated only where
    the device's per-key words changed, server.hip apply_state), pulls that
    grow the key set, a second pull before the merge (the first one's upload
    started at ingest, then parsed on the host) and empty pulls: CurrentState
    and the Diff == pyref after every merge."""
    rng = np.random.default_rng(seed)
    P = 3
    keys = KEYS + [f"n{i}" for i in range(8)]
    model = [({}, {}) for _ in range(P)]
    srv = [Server(eng, 8080 + i) for i in range(P)]
    peers_src = [Server(None, 9100 + i) for i in range(P)]           # host-only peers serving pulls
    clock = 5_000
    for rnd in range(8):
        remotes = []
        for i in range(P):
            pulls = []
            for _ in range(1 if rnd % 3 else 2):                     # every third round: two pulls before the merge
                p = peers_src[i] if rnd != 4 else Server(None, 9200)   # round 4: empty pulls
                for _ in range(int(rng.integers(0, 6)) if rnd != 4 else 0):
                    clock += int(rng.integers(1, 4))
                    ks = rng.choice(len(keys) if rnd > 2 else 6, int(rng.integers(1, 3)), replace=False)
                    p.Diff.Put(clock, {keys[int(q)]: VALS[int(rng.integers(0, len(VALS)))] for q in ks})
                st, body = p.GossipBinary()
                assert st == 200
                assert srv[i].IngestBinary(body) == 0
                pulls.append({t: dict(p.Diff.Get(t)[0]) for t in p.Diff.Keys()})
                if rnd == 4:
                    p.close()
            rem = {}
            for pl in pulls:                                         # RemoteDiff.Put: the later pull wins
                rem.update(pl)
            remotes.append(rem)
        if rnd % 2 == 0:
            merge_servers(srv)
        else:
            for s in srv:
                s.merge()
        for i in range(P):
            model[i] = pyref.merge(model[i][0], remotes[i])
            assert srv[i].CurrentState == model[i][1], f"round {rnd} replica {i}"
        if rnd % 4 == 3:
            for i in range(P):
                assert srv[i].DiffSignature == _sig(model[i][0]), f"round {rnd} replica {i}"
    for s in srv + peers_src:
        s.close()
