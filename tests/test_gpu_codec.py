"""GPU: the gossip pull decoded on the device (SURVEY §8(f) row 2,
crdt_gossip_decode) -- binary SoA bodies served by the host mirror
(crdt_server_gossip_binary, the wire form of Diff.ToJSON, main.go:159) are
decoded in HBM into RemoteDiff arrays (main.go:245-256).  Checked against
the host ingest of the same bodies (crdt_server_ingest_binary, itself pinned
to the JSON codec and its Go encoding/json KATs by tests/test_gossip_json.py)
and, through whole pull rounds, against the pyref simulation of the
reference's rounds."""
import struct

import numpy as np
import pytest
from knobs import set_knob
import torch

from crdt_amd import codec, gossip
from crdt_amd.refmerge import Command
from crdt_amd.server import Server
from gossip_util import K, KEYS, STRS, _host_round, _pack, _rand_diff, _same_diffs, _state, _unpack

pytestmark = [pytest.mark.gpu, pytest.mark.diag]


@pytest.fixture(params=[1, 2, 0, 3], ids=["auto", "one_pass", "multi_pass", "one_pass_coalesced"], autouse=True)
def decode_form(request, eng):
    """Every test under each decode form: the product's choice by size
    (codec.small = 1), the one-pass small-body kernel (2: always), the multi-pass form (0) and the one-pass form
    with coalesced accesses (3)."""
    from crdt_amd import _lib
    set_knob(b"codec.small", request.param)
    yield request.param
    set_knob(b"codec.small", 1)


def _serve(diff) -> bytes:
    """The binary gossip body of a Diff (host-only Server: main.go:153-170)."""
    s = Server(None, 8080)
    for ts, v in diff.items():
        s.Diff.Put(ts, v)
    st, body = s.GossipBinary()
    s.close()
    assert st == 200
    return body


def _raw_body(entries):
    """Hand-built binary body: entries = [(ts, [(k, v), ...] or None)] in the
    given order (None: a nil map)."""
    ts, pairs, kl, vl, by = [], [], [], [], b""
    for t, kv in entries:
        ts.append(t)
        pairs.append(0xFFFFFFFF if kv is None else len(kv))
        for k, v in kv or []:
            kl.append(len(k))
            vl.append(len(v))
            by += k + v
    n = len(kl)
    return (b"CRDTSOA1" + struct.pack("<QQQ", len(ts), n, len(by)) + struct.pack(f"<{len(ts)}q", *ts) +
            struct.pack(f"<{len(ts)}I", *pairs) + struct.pack(f"<{n}I", *kl) + struct.pack(f"<{n}I", *vl) + by)


def _upload(eng, bodies):
    off = np.zeros(len(bodies) + 1, np.int64)
    off[1:] = np.cumsum([len(b) for b in bodies])
    blob = b"".join(bodies) or b"\0"
    return torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(eng.device), off.tolist()


def _decode(eng, bodies, keys, vals, key_cap=1 << 20, kv_base=3):
    data, off = _upload(eng, bodies)
    ne = sum(codec.body_counts(b)[0] for b in bodies)
    npairs = sum(codec.body_counts(b)[1] for b in bodies)
    kk = torch.full((kv_base + npairs + 1,), -1, dtype=torch.int32, device=eng.device)
    kv = torch.full_like(kk, -1)
    dec, st = codec.decode(eng, data, off, [1000 * i for i in range(len(bodies))], key_cap, keys, vals, kv_base,
                           kk, kv, ne)
    return dec, st, kk.cpu().numpy(), kv.cpu().numpy()


_ODD = ["", "x", "\xff\x00", "é", "007", "-0", "\n\t\"<>&", "9223372036854775808"]


def test_decode_matches_host_ingest(eng):
    rng = np.random.default_rng(4)
    diffs = []
    for b in range(11):
        d, t = {}, int(rng.integers(-50, 50))
        for _ in range(int(rng.integers(0, 60))):
            t += int(rng.integers(1, 9))
            kv = {f"k{int(q)}".encode() if q % 3 else _ODD[int(q) % len(_ODD)].encode("latin-1"):
                  (str(int(rng.integers(-30, 30))) if rng.random() < 0.8 else _ODD[int(rng.integers(0, len(_ODD)))])
                  .encode("latin-1") for q in rng.choice(20, int(rng.integers(0, 5)), replace=False)}
            d[t] = Command(kv) if rng.random() < 0.5 else kv
        diffs.append(d)
    bodies = [_serve(d) for d in diffs]
    keys, vals = codec.StrTab(eng, 4, 64), codec.StrTab(eng, 4, 64)       # tiny: forces growth + rehash
    dec, st, kk, kv = _decode(eng, bodies, keys, vals)
    assert not st.any(), st
    r_off, r_ts, r_kv = (dec[x].cpu().numpy() for x in ("r_off", "r_ts", "r_kv"))
    ks, vs = keys.strings(), vals.strings()
    assert len(set(ks)) == len(ks) and len(set(vs)) == len(vs)          # interned: each string once
    for b, body in enumerate(bodies):
        host = Server(None, 9000)
        assert host.IngestBinary(body) == 0
        exp_ts = host.RemoteDiff.Keys()
        got_ts = r_ts[r_off[b]:r_off[b + 1]].tolist()
        assert got_ts == exp_ts
        for e, t in zip(range(r_off[b], r_off[b + 1]), exp_ts):
            got = {}
            for q in range(r_kv[e], r_kv[e + 1]):
                got[ks[kk[q] - 1000 * b].decode("utf-8", "surrogateescape")] = \
                    vs[kv[q]].decode("utf-8", "surrogateescape")
            assert got == host.RemoteDiff.Get(t)[0]
        host.close()
    # a second decode re-uses the interned strings (no new ids for seen strings)
    n_k, n_v = len(keys), len(vals)
    _, st2, _, _ = _decode(eng, bodies[:3], keys, vals)
    assert not st2.any() and (len(keys), len(vals)) == (n_k, n_v)


def test_decode_flags(eng):
    keys, vals = codec.StrTab(eng), codec.StrTab(eng)
    good = _raw_body([(1, [(b"a", b"1")]), (2, [(b"a", b"2"), (b"b", b"3")])])
    bodies = [
        good,
        good[:-1],                                                   # truncated: malformed (header sizes)
        _raw_body([(1, [(b"a", b"1")]), (5, None)]),                 # nil map: host path (keeps the nil flag)
        _raw_body([(3, [(b"a", b"1")]), (2, [(b"a", b"1")])]),       # ts not ascending: host path
        _raw_body([(1, [(b"b", b"1"), (b"a", b"2")])]),              # keys not ascending: host path
        _raw_body([(1, [(b"a", b"1"), (b"a", b"2")])]),              # duplicate key: host path
    ]
    bad_count = bytearray(good)
    struct.pack_into("<I", bad_count, 32 + 16, 5)                    # pairs[0] = 5 != header n_pairs
    bodies.append(bytes(bad_count))
    _, st, _, _ = _decode(eng, bodies, keys, vals)
    assert st.tolist() == [0, 1, 2, 2, 2, 2, 1], st
    # a valid body AFTER a body whose pair counts disagree with its header
    # decodes exactly (its kv ranges are rebased per body), and the rejected
    # body's strings never enter the tables
    bad = bytearray(_raw_body([(1, [(b"qq", b"77")]), (2, [(b"rr", b"88"), (b"ss", b"99")])]))
    struct.pack_into("<I", bad, 32 + 16, 7)                          # pairs[0] = 7 != header n_pairs
    good2 = _raw_body([(4, [(b"a", b"5"), (b"c", b"6")]), (9, [(b"b", b"x")])])
    k3, v3 = codec.StrTab(eng), codec.StrTab(eng)
    dec, st, kk, kv = _decode(eng, [good, bytes(bad), good2], k3, v3)
    assert st.tolist() == [0, 1, 0], st
    r_off, r_ts, r_kv = (dec[x].cpu().numpy() for x in ("r_off", "r_ts", "r_kv"))
    ks, vs = k3.strings(), v3.strings()
    assert not {b"qq", b"rr", b"ss"} & set(ks) and not {b"77", b"88", b"99"} & set(vs)
    for b, body in ((0, good), (2, good2)):
        host = Server(None, 9000)
        assert host.IngestBinary(body) == 0
        assert r_ts[r_off[b]:r_off[b + 1]].tolist() == host.RemoteDiff.Keys()
        for e, t in zip(range(r_off[b], r_off[b + 1]), host.RemoteDiff.Keys()):
            got = {ks[kk[q] - 1000 * b].decode(): vs[kv[q]].decode() for q in range(r_kv[e], r_kv[e + 1])}
            assert got == host.RemoteDiff.Get(t)[0]
        host.close()
    # a key id past the replica's slot range takes the host path
    k2, v2 = codec.StrTab(eng), codec.StrTab(eng)
    _, st, _, _ = _decode(eng, [_raw_body([(1, [(b"a", b"1"), (b"b", b"1"), (b"c", b"1")])])], k2, v2, key_cap=2)
    assert st.tolist() == [2]


@pytest.mark.parametrize("seed", [1, 2])
def test_wire_rounds_match_reference_simulation(eng, seed):
    """Pull rounds whose pulls arrive as binary bodies (decoded on the device,
    Population.round_wire) == the pyref simulation of the reference's
    rounds (main.go:226-258)."""
    rng = np.random.default_rng(seed)
    P = 7
    diffs = [_rand_diff(rng, 1_000 + 13 * i, int(rng.integers(0, 40))) for i in range(P)]
    pop = gossip.Population(eng, _pack(diffs), K)
    keys, vals = codec.StrTab(eng), codec.StrTab(eng)
    assert keys.intern(KEYS).tolist() == list(range(K))                  # key id = KEYS index
    assert vals.intern(STRS).tolist() == list(range(len(STRS)))          # string id = STRS index
    for rnd in range(5):
        peers = gossip.random_peers(rng, P, 0, P)
        bodies = [_serve(diffs[q]) for q in peers]
        data, off = _upload(eng, bodies)
        ne = sum(codec.body_counts(b)[0] for b in bodies)
        npairs = sum(codec.body_counts(b)[1] for b in bodies)
        pop.round_wire(data, off, keys, vals, ne, npairs)
        diffs, states = _host_round(diffs, peers)
        _same_diffs(_unpack(pop), diffs)
        assert _state(pop) == states, f"round {rnd}"
    assert len(keys) == K and len(vals) == len(STRS)                     # nothing new was interned


def test_decode_short_string_order_and_interning(eng):
    """The claim pass packs strings of <= 8 bytes into one word (hash, table
    compares, the keys-ascending check): NUL bytes, prefixes, 8 / 9-byte
    strings and strings that straddle an 8-byte word of the body all intern
    to the host decode's strings, and the ascending check orders them like
    Go strings (a prefix first; "a" < "a\\x00" < "a\\x01" < "b")."""
    keys, vals = codec.StrTab(eng), codec.StrTab(eng)
    ok = _raw_body([(1, [(b"a", b""), (b"a\x00", b"\x00"), (b"a\x01", b"12345678"), (b"b", b"123456789")]),
                    (2, [(b"x" * 7, b"y" * 7), (b"x" * 8, b"y" * 8), (b"x" * 9, b"y" * 9)]),
                    (3, [(b"\x00", b"\x00\x00"), (b"\x00\x00", b"\xff" * 3)])])
    # (host-path bodies may still intern their strings: these reuse body 0's)
    bad1 = _raw_body([(1, [(b"a\x00", b""), (b"a", b"\x00")])])      # prefix after the longer key: not ascending
    bad2 = _raw_body([(1, [(b"x" * 8, b""), (b"x" * 7, b"\x00")])])
    pad = _raw_body([(1, [(b"q", b"r")])])                           # shifts the next bodies' byte alignment
    dec, st, kk, kv = _decode(eng, [ok, bad1, pad, ok, bad2], keys, vals)
    assert st.tolist() == [0, 2, 0, 0, 2], st
    ks, vs = keys.strings(), vals.strings()
    want_k = [b"a", b"a\x00", b"a\x01", b"b", b"x" * 7, b"x" * 8, b"x" * 9, b"\x00", b"\x00\x00", b"q"]
    want_v = [b"", b"\x00", b"12345678", b"123456789", b"y" * 7, b"y" * 8, b"y" * 9, b"\x00\x00", b"\xff" * 3, b"r"]
    assert set(ks) == set(want_k) and len(ks) == len(want_k), ks
    assert set(vs) == set(want_v) and len(vs) == len(want_v), vs
    # body 3 (the same strings as body 0, at another alignment) resolves to the same ids
    r_kv = dec["r_kv"].cpu().numpy()
    r_off = dec["r_off"].cpu().numpy()
    b0 = slice(int(r_kv[r_off[0]]), int(r_kv[r_off[1]]))
    b3 = slice(int(r_kv[r_off[3]]), int(r_kv[r_off[4]]))
    assert np.array_equal(kv[b0], kv[b3])
    assert np.array_equal(kk[b0] - 0, kk[b3] - 3000)               # key ids rebased into each body's slot range


def test_decode_large_bodies_both_forms_agree(eng, decode_form):
    """Bodies past one chunk of the one-pass kernel (8192 items per round of
    its scans; 20k entries / ~60k pairs) and a body at an odd byte offset:
    the same ids, ranges and flags from every form (multi-pass, one-pass,
    coalesced one-pass at 4 and 8 items per thread)."""
    from crdt_amd import _lib
    rng = np.random.default_rng(11)
    bodies = []
    for n in (20_000, 3, 9_000):
        d, t = {}, 5
        for _ in range(n):
            t += int(rng.integers(1, 4))
            d[t] = {f"k{int(q)}": str(int(rng.integers(-99, 99))) for q in rng.choice(40, int(rng.integers(0, 6)), replace=False)}
        bodies.append(_serve(d))
    bodies.insert(1, _raw_body([(1, [(b"a", b"1")])]) + b"")     # shifts the next body off 8-byte alignment
    out = []
    # (3, 8): the coalesced one-pass form with 8 items per thread per chunk
    # (codec.big_r = 8, k_dec_big8)
    for form, big_r in ((0, 4), (2, 4), (3, 4), (3, 8)):
        set_knob(b"codec.small", form)
        set_knob(b"codec.big_r", big_r)
        keys, vals = codec.StrTab(eng), codec.StrTab(eng)
        dec, st, kk, kv = _decode(eng, bodies, keys, vals)
        h = {x: dec[x].cpu().numpy() for x in ("r_off", "r_ts", "r_kv")}
        ks, vs = keys.strings(), vals.strings()
        # ids follow the claim races: compare the strings they resolve to
        pairs = [(ks[kk[q] - 1000 * bi], vs[kv[q]]) for bi in range(len(bodies))
                 for q in range(h["r_kv"][h["r_off"][bi]], h["r_kv"][h["r_off"][bi + 1]])]
        out.append((st.tolist(), h, pairs, sorted(ks), sorted(vs)))
    set_knob(b"codec.small", decode_form)
    set_knob(b"codec.big_r", 4)
    a = out[0]
    assert a[0] == [0, 0, 0, 0]
    for b in out[1:]:
        assert b[0] == a[0]
        for x in a[1]:
            np.testing.assert_array_equal(a[1][x], b[1][x], err_msg=x)
        assert a[2] == b[2] and a[3] == b[3] and a[4] == b[4]
    r_off, r_ts = a[1]["r_off"], a[1]["r_ts"]
    host = Server(None, 9000)
    assert host.IngestBinary(bodies[0]) == 0
    assert r_ts[r_off[0]:r_off[1]].tolist() == host.RemoteDiff.Keys()
    host.close()


@pytest.mark.parametrize("short_tab", [2, 3, 4, 1, 0])
def test_decode_resolved_short_forms_across_calls_and_rehash(eng, short_tab):
    """Strings of <= 7 bytes resolved in an earlier call are found by the
    short form stored beside their table entry (codec.short_tab, written with
    the id and again by a rehash; form 2 probes a pair's two home entries at
    once and lists the rest for the claim loop): a later call -- before and after the table
    grows -- maps every string to the id the first call gave it, NUL bytes
    and equal-padded strings of different lengths ("a" / "a\\x00") apart,
    8-byte and longer strings by the byte walk, and interns nothing new."""
    from crdt_amd import _lib
    set_knob(b"codec.short_tab", short_tab)
    try:
        keys, vals = codec.StrTab(eng, 4, 64), codec.StrTab(eng, 4, 64)       # tiny: grows in the first call
        strs = [b"", b"a", b"a\x00", b"a\x00\x00", b"\x00", b"x" * 7, b"x" * 8, b"x" * 9, b"7", b"-12", b"\xff" * 6]
        body = _raw_body([(i + 1, [(b"k%02d" % i, s)]) for i, s in enumerate(strs)] +
                         [(100 + i, [(s, b"v")]) for i, s in enumerate(sorted(set(strs) - {b""}))])
        dec1, st1, kk1, kv1 = _decode(eng, [body], keys, vals)
        assert st1.tolist() == [0]
        n_k, n_v = len(keys), len(vals)
        for step in range(2):
            if step:                                                     # grow both tables: a rehash
                keys.intern([b"g%d" % i for i in range(300)])
                vals.intern([b"h%d" % i for i in range(300)])
                n_k, n_v = n_k + 300, n_v + 300
            dec2, st2, kk2, kv2 = _decode(eng, [body], keys, vals)
            assert st2.tolist() == [0]
            assert (len(keys), len(vals)) == (n_k, n_v)                 # nothing new interned
            assert np.array_equal(kk1, kk2) and np.array_equal(kv1, kv2)
        ks, vs = keys.strings(), vals.strings()
        n = len(strs)
        assert [vs[kv1[3 + i]] for i in range(n)] == strs              # kv_base 3: pair i of entry i
        assert [ks[kk1[3 + n + i]] for i in range(n - 1)] == sorted(set(strs) - {b""})
    finally:
        set_knob(b"codec.short_tab", 3)
