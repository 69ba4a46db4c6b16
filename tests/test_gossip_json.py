"""Gossip wire codec: the C++ Server mirror's
Diff.ToJSON serve (main.go:153-170) and JSON pull decode (main.go:245-256).

Host-only (no GPU, no kernel): the codec runs in libcrdt_amd.so on a Server
built without an engine.  Checked three ways: against the hand-written KATs
in tests/golden/gossip_json_kat.json (Go 1.18 encoding/json semantics,
derived from the reference's source -- no Go toolchain or reference run
exists here, so these are the pin), the test-only restatement in
oracle/gojson.py against the same KATs, and library vs restatement on seeded
random diffs / bodies."""
import json
import os
import random

import pytest

from crdt_amd.refmerge import Command
from crdt_amd.server import Server
from oracle import gojson

_KAT = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "gossip_json_kat.json")))
_B = lambda s: s.encode("latin-1")                       # KAT strings: one char per byte


def _dec(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")


def _srv(diff=()):
    s = Server(None, 8080)
    for ts, local, kv in diff:
        v = {_B(k): _B(x) for k, x in kv.items()}
        s.Diff.Put(ts, Command(v) if local else v)
    return s


@pytest.mark.parametrize("case", _KAT["marshal"], ids=[c["name"] for c in _KAT["marshal"]])
def test_marshal_kat(case):
    s = _srv(case["diff"])
    st, body = s.Gossip()
    assert st == 200
    assert body == _B(case["body"])
    assert gojson.marshal_diff({ts: {_B(k): _B(x) for k, x in kv.items()}
                                for ts, _, kv in case["diff"]}) == _B(case["body"])
    s.close()


@pytest.mark.parametrize("case", _KAT["ingest"], ids=[c["name"] for c in _KAT["ingest"]])
def test_ingest_kat(case):
    s = _srv()
    out = s.IngestGossip(_B(case["body"]))
    assert out == case["outcome"]
    exp = {ts: {_dec(_B(k)): _dec(_B(v)) for k, v in kv.items()} for ts, kv in case["remote"]}
    assert s.RemoteDiff.Keys() == sorted(exp)
    assert s.RemoteDiff.Size() == len(exp)
    for ts, kv in exp.items():
        got, found = s.RemoteDiff.Get(ts)
        assert found and got == kv
    try:
        _B(case["body"]).decode("utf-8")
    except UnicodeDecodeError:
        return                                            # raw invalid bytes: KAT only
    o_out, o_remote = gojson.ingest(_B(case["body"]))
    assert o_out == case["outcome"]
    assert o_remote == exp
    s.close()


def test_unreachable_when_not_alive():
    s = _srv([(1, False, {"a": "1"})])
    s.SetAlive(False)
    assert s.Gossip() == (502, b"Unreachable")          # main.go:166
    s.SetAlive(True)
    assert s.Gossip() == (200, b'{"1":{"a":"1"}}')
    s.close()


def test_failed_round_leaves_remote_untouched():
    s = _srv()
    assert s.IngestGossip(b'{"3":{"a":"x"}}') == 0
    assert s.IngestGossip(b'{"4":{"a":"y"},"bad":{}}') == 2      # Atoi fails: nothing from this body
    assert s.IngestGossip(b'{"5":{"a":"y"}') == 1                 # truncated
    assert s.RemoteDiff.Keys() == [3]
    assert s.IngestGossip(b'{"3":{"b":"z"}}') == 0               # Put replaces the entry
    assert s.RemoteDiff.Get(3) == ({"b": "z"}, True)
    assert s.RemoteDiff.Get(4) == (None, False)
    s.close()


def _rand_str(rng, alphabet):
    return "".join(rng.choice(alphabet) for _ in range(rng.randrange(0, 6)))


_ALPHA = list("ab01<>&\"\\/ \n\t\x00\x1f\x7f") + ["é", " ", " ", "\U0001F600", "�"]


@pytest.mark.parametrize("seed", range(6))
def test_serve_then_pull_roundtrip_random(seed):
    """Random Diffs: library body == restatement body, and pulling that body
    into a fresh server's RemoteDiff reproduces every entry (the wire path a
    friend takes, main.go:159 -> :245-256)."""
    rng = random.Random(seed)
    diff = {}
    for _ in range(rng.randrange(0, 40)):
        ts = rng.choice([rng.randrange(-2**63, 2**63), rng.randrange(-20, 20)])
        diff[ts] = {_rand_str(rng, _ALPHA): _rand_str(rng, _ALPHA) for _ in range(rng.randrange(0, 4))}
    a = _srv()
    for ts, kv in diff.items():
        a.Diff.Put(ts, Command(kv) if rng.random() < 0.5 else kv)
    st, body = a.Gossip()
    assert st == 200
    assert body == gojson.marshal_diff(diff)
    assert json.loads(body) == {str(t): v for t, v in diff.items()}
    b = _srv()
    assert b.IngestGossip(body) == 0
    assert b.RemoteDiff.Keys() == sorted(diff)
    for ts, kv in diff.items():
        assert b.RemoteDiff.Get(ts) == (kv, True)
    a.close()
    b.close()


def _rand_body(rng):
    """Mostly-valid JSON bodies with mutations: wrong types, bad keys,
    escapes, whitespace, truncation."""
    def key():
        return rng.choice([str(rng.randrange(-50, 50)), "0" + str(rng.randrange(9)), "+7", "x", "", "1e3",
                           str(2**63), "\\u0031" + str(rng.randrange(9)), "-0"])

    def sval():
        return rng.choice(['"v"', '"\\u00e9\\n"', '"\\ud83d\\ude00"', '"\\ud800"', 'null', '1', 'true', '"a\\/b"',
                           '"\\uDC00x"', '[]', '{}'])

    def inner():
        if rng.random() < 0.1:
            return "null"
        if rng.random() < 0.05:
            return rng.choice(["[]", "3", '"s"'])
        members = ['"%s":%s' % (rng.choice(["a", "b", "c", "\\u0061"]), sval()) for _ in range(rng.randrange(0, 4))]
        return "{" + ",".join(members) + "}"

    ws = lambda: rng.choice(["", "", " ", "\n\t "])
    body = "{" + ",".join(ws() + '"%s"' % key() + ws() + ":" + ws() + inner() + ws()
                          for _ in range(rng.randrange(0, 6))) + "}"
    r = rng.random()
    if r < 0.05:
        body = body[: rng.randrange(len(body) + 1)]
    elif r < 0.08:
        body += rng.choice([" x", ",", "}"])
    elif r < 0.1:
        body = rng.choice(["null", " null ", "[]", "", "nul", "{}"])
    return body.encode()


def test_ingest_random_bodies_match_restatement():
    rng = random.Random(1234)
    seen = {0: 0, 1: 0, 2: 0}
    for _ in range(3000):
        body = _rand_body(rng)
        s = _srv()
        out = s.IngestGossip(body)
        o_out, o_remote = gojson.ingest(body)
        assert out == o_out, body
        seen[out] += 1
        got = {ts: s.RemoteDiff.Get(ts)[0] for ts in s.RemoteDiff.Keys()}
        assert got == o_remote, body
        s.close()
    assert all(v > 50 for v in seen.values()), seen


# ---------------------------------------------------------------- binary SoA codec
def test_binary_roundtrip_equals_json_roundtrip():
    """serve binary -> pull binary puts exactly what serve JSON -> pull JSON
    puts (random Diffs, every byte value in keys and values)."""
    rng = random.Random(77)
    for _ in range(30):
        a = _srv()
        diff = {}
        for _ in range(rng.randrange(0, 25)):
            ts = rng.choice([rng.randrange(-2**63, 2**63), rng.randrange(-9, 9)])
            kv = {_rand_str(rng, _ALPHA): _rand_str(rng, _ALPHA) for _ in range(rng.randrange(0, 4))}
            diff[ts] = kv
            a.Diff.Put(ts, Command(kv) if rng.random() < 0.5 else kv)
        st, body = a.GossipBinary()
        assert st == 200 and body[:8] == b"CRDTSOA1"
        bj, bb = _srv(), _srv()
        assert bj.IngestGossip(a.Gossip()[1]) == 0
        assert bb.IngestBinary(body) == 0
        assert bb.RemoteDiff.Keys() == bj.RemoteDiff.Keys() == sorted(diff)
        for ts in diff:
            assert bb.RemoteDiff.Get(ts) == bj.RemoteDiff.Get(ts) == (diff[ts], True)
        for s in (a, bj, bb):
            s.close()


def test_binary_raw_bytes_survive():
    """Unlike JSON (invalid UTF-8 -> U+FFFD), the binary codec is byte-exact."""
    a = _srv([(3, False, {"k": "\xff\x00"})])                # latin-1 -> bytes ff 00
    b = _srv()
    assert b.IngestBinary(a.GossipBinary()[1]) == 0
    got, found = b.RemoteDiff.Get(3)
    assert found and got == {"k": _dec(b"\xff\x00")}


def test_binary_malformed_bodies_rejected():
    a = _srv([(1, False, {"a": "1"}), (2, True, {"b": "22", "c": "3"})])
    body = a.GossipBinary()[1]
    b = _srv()
    for bad in [b"", b"CRDTSOA1", body[:-1], body + b"x", b"CRDTSOA2" + body[8:],
                body[:8] + (2**62).to_bytes(8, "little") + body[16:],      # n_entries too large
                body[:16] + (99).to_bytes(8, "little") + body[24:]]:        # n_pairs inconsistent
        assert b.IngestBinary(bad) == 1
    assert b.RemoteDiff.Size() == 0
    a.SetAlive(False)
    assert a.GossipBinary() == (502, b"Unreachable")
