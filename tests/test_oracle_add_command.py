"""CPU: the AddCommand restatement (oracle/pyref.add_command, main.go:173-215)
on hand-derived known answers, and the host Server mirror
(crdt_server_add_command) against it on random command streams."""
import random

import pytest

from crdt_amd.server import Server
from oracle import pyref

# (start diff, start state, [(ts, data, status)], end diff signature, end state) -- derived by hand from main.go
KATS = [
    ("new key inserted verbatim, early return",
     {}, {}, [(100, {"a": "5"}, 200)], [100], {"a": "5"}),
    ("existing key: Atoi both sides, Itoa(sum)",
     {}, {"a": "5"}, [(101, {"a": "-3"}, 200)], [101], {"a": "2"}),
    ("Atoi(value) fails: 500, state untouched, Diff still written",
     {}, {"a": "2"}, [(102, {"a": "x"}, 500)], [102], {"a": "2"}),
    ("Atoi(current) fails: 500",
     {}, {"a": "007x"}, [(5, {"a": "1"}, 500)], [5], {"a": "007x"}),
    ("first NEW key returns: later keys (key order) not applied",
     {}, {"a": "1"}, [(7, {"a": "1", "b": "2", "c": "3"}, 200)], [7], {"a": "2", "b": "2"}),
    ("same-ms write replaces the Diff entry, both applied to the state",
     {}, {}, [(9, {"k": "1"}, 200), (9, {"k": "4"}, 200)], [9], {"k": "5"}),
    ("int64 wrap",
     {}, {"w": "9223372036854775807"}, [(3, {"w": "1"}, 200)], [3], {"w": "-9223372036854775808"}),
    ("leading zeros and + parse; result re-formatted",
     {}, {"z": "007"}, [(4, {"z": "+3"}, 200)], [4], {"z": "10"}),
    ("empty command: 200, Diff written",
     {}, {}, [(8, {}, 200)], [8], {}),
    ("a Put on an existing remote entry's ts replaces it with a local *Command",
     {8: {"q": "1"}}, {}, [(8, {"q": "2"}, 200)], [8], {"q": "2"}),
]


@pytest.mark.parametrize("kat", KATS, ids=[k[0] for k in KATS])
def test_pyref_add_command_kats(kat):
    _, d0, s0, cmds, sig, st = kat
    diff, state = dict(d0), dict(s0)
    for ts, data, status in cmds:
        assert pyref.add_command(diff, state, ts, data) == status
    assert sorted(diff) == sig
    assert all(isinstance(diff[t], pyref.Command) for t, *_ in cmds)
    assert state == st


def test_pyref_dead_replica_502():
    diff, state = {}, {}
    assert pyref.add_command(diff, state, 1, {"a": "1"}, alive=False) == 502
    assert diff == {} and state == {}


def test_host_mirror_matches_restatement_random():
    rng = random.Random(5)
    vals = ["1", "-3", "x", "007", "+2", "9223372036854775807", "-20", ""]
    for _ in range(20):
        s = Server(None, 8080)
        diff, state = {}, {}
        for _ in range(rng.randrange(1, 40)):
            ts = rng.randrange(0, 30)
            data = {rng.choice("abcde"): rng.choice(vals) for _ in range(rng.randrange(0, 4))}
            assert s.AddCommand(ts, data) == pyref.add_command(diff, state, ts, data)
        assert [t for t, _ in s._diff_entries()] == sorted(diff)
        assert s.CurrentState == state
        s.close()
