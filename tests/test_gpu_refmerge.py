"""GPU parity for RefMerge: the bit-exact (*Server).merge() of main.go:35-100.

Pinned twice: every hand-derived KAT (tests/golden/refmerge_kat.json) must
come out of the GPU path exactly, and seeded config-A workloads must match the
C oracle (oracle/crdt_oracle.c) replica by replica -- same new Diff (same
keys, same value objects), same CurrentState strings.
"""
import numpy as np
import pytest
from knobs import set_knob
import torch

from crdt_amd import refmerge, synth
from crdt_amd.server import Command, NewServer, Server, merge_servers
from oracle import oracle, pyref
from refmerge_util import diff_signature, kat_inputs, load_kats, oracle_merge

pytestmark = pytest.mark.gpu
KATS = load_kats()


def _server_from(eng, diff, remote, port=8080):
    s = Server(eng, port)
    for ts, v in diff.items():
        s.Diff.Put(ts, v)
    for ts, v in remote.items():
        s.RemoteDiff.Put(ts, v)
    return s


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_server_merge_kat(eng, kat):
    diff, remote = kat_inputs(kat)
    s = _server_from(eng, diff, remote)
    s.merge()
    assert s.DiffSignature == kat["diff"]
    assert s.CurrentState == kat["state"]
    assert s.RemoteDiff.Size() == 0          # RemoteDiff.Clear() (main.go:75)
    s.close()


def test_all_kats_in_one_batch(eng):
    res = refmerge.merge_batch(eng, [kat_inputs(k) for k in KATS])
    for k, (d, st) in zip(KATS, res):
        assert diff_signature(d) == k["diff"], k["name"]
        assert st == k["state"], k["name"]


@pytest.mark.parametrize("seed", [1, 2])
def test_config_a_demo_matches_oracle(eng, seed):
    reps = synth.refmerge_demo(seed, replicas=5, entries=10_000, multi_key=0.1)
    res = refmerge.merge_batch(eng, reps)
    for (diff, remote), (d_gpu, s_gpu) in zip(reps, res):
        d_or, s_or = oracle_merge(diff, remote)
        assert list(d_gpu) == list(d_or)
        assert all(d_gpu[t] is d_or[t] for t in d_or)
        assert s_gpu == s_or


def test_large_batch_matches_oracle(eng):
    reps = synth.refmerge_demo(77, replicas=400, entries=600, multi_key=0.3)
    res = refmerge.merge_batch(eng, reps)
    for (diff, remote), (d_gpu, s_gpu) in zip(reps, res):
        d_or, s_or = oracle_merge(diff, remote)
        assert list(d_gpu) == list(d_or)
        assert s_gpu == s_or


def _big_string_table(h, n_str, seed):
    """Re-point every kv value at one of n_str strings (numbers, Atoi edge
    cases and words): the fold stages tables of <= 256 strings in LDS, larger
    ones take the global Atoi lookup."""
    rng = np.random.default_rng(seed)
    base = ["-9223372036854775808", "9223372036854775807", "9223372036854775808", "+7", "007", "-0", "x1", ""]
    strs = base + [str(int(v)) if i % 5 else f"w{i}" for i, v in
                   enumerate(rng.integers(-2**62, 2**62, size=n_str - len(base)))]
    blob = "".join(strs).encode()
    so = np.zeros(len(strs) + 1, np.int64)
    so[1:] = np.cumsum([len(x.encode()) for x in strs])
    h = dict(h)
    h["kv_val"] = rng.integers(0, n_str, size=len(h["kv_val"])).astype(np.uint32).view(np.int32)
    h["str_bytes"], h["str_off"] = np.frombuffer(blob, np.uint8).copy(), so
    return h


@pytest.mark.parametrize("n_str", [0, 256, 257, 5000])
def test_packed_batch_matches_oracle(eng, n_str):
    """The bench's packed config-A-at-scale batch: every replica checked
    (n_str 0: the generator's own ten values plus odd strings)."""
    from refmerge_util import oracle_packed_replica
    h = synth.refmerge_packed(11, 48, 5000)
    if n_str:
        h = _big_string_table(h, n_str, n_str)
    out = eng.refmerge_batch(refmerge.to_device(h, eng.device))
    off = out["off"].cpu().numpy()
    ts, org, src = (out[k].cpu().numpy() for k in ("ts", "origin", "src"))
    kind, sstr, ssum = (out[k].cpu().numpy() for k in ("st_kind", "st_str", "st_sum"))
    for p in range(h["replicas"]):
        o_ts, o_or, o_src, k, s, v = oracle_packed_replica(h, p)
        a, b = int(off[p]), int(off[p + 1])
        np.testing.assert_array_equal(ts[a:b], o_ts)
        np.testing.assert_array_equal(org[a:b], o_or)
        np.testing.assert_array_equal(src[a:b], o_src)
        sl = slice(p * 62, (p + 1) * 62)
        np.testing.assert_array_equal(kind[sl], k)
        m = k > 0
        np.testing.assert_array_equal(sstr[sl].view(np.uint32)[k == 1], s[k == 1])
        np.testing.assert_array_equal(ssum[sl][k == 2], v[k == 2])
        assert m.sum() > 0


def test_many_replicas_multi_kernel_plan(eng):
    """> 65536 replicas (and tiles): the planning and tile-count scan take the
    multi-kernel device-scan path instead of the single-workgroup one.
    Replicas sampled across the batch are checked against the oracle, and
    the new-Diff ranges against a host recount."""
    from refmerge_util import oracle_packed_replica
    h = synth.refmerge_packed(23, 70_000, 12)
    out = eng.refmerge_batch(refmerge.to_device(h, eng.device))
    off = out["off"].cpu().numpy()
    ts, org, src = (out[k].cpu().numpy() for k in ("ts", "origin", "src"))
    kind = out["st_kind"].cpu().numpy()
    assert off[0] == 0 and np.all(np.diff(off) >= np.diff(h["l_off"]))
    for p in list(range(0, 70_000, 997)) + [69_999]:
        o_ts, o_or, o_src, k, _, _ = oracle_packed_replica(h, p)
        a, b = int(off[p]), int(off[p + 1])
        np.testing.assert_array_equal(ts[a:b], o_ts)
        np.testing.assert_array_equal(org[a:b], o_or)
        np.testing.assert_array_equal(src[a:b], o_src)
        np.testing.assert_array_equal(kind[p * 62:(p + 1) * 62], k)


def test_servers_batched_equals_single(eng):
    reps = synth.refmerge_demo(5, replicas=6, entries=2000, multi_key=0.2)
    batch = [_server_from(eng, d, r, 8080 + i) for i, (d, r) in enumerate(reps)]
    single = [_server_from(eng, d, r, 9080 + i) for i, (d, r) in enumerate(reps)]
    merge_servers(batch)
    for s in single:
        s.merge()
    for a, b, (d, r) in zip(batch, single, reps):
        _, st = pyref.merge(d, r)
        assert a.DiffSignature == b.DiffSignature
        assert a.CurrentState == b.CurrentState == st


def test_merge_idempotent_and_empty(eng):
    diff, remote = synth.refmerge_demo(9, replicas=1, entries=3000)[0]
    s = _server_from(eng, diff, remote)
    s.merge()
    sig, st = s.DiffSignature, s.CurrentState
    for ts, v in remote.items():            # re-gossip the same R (KAT-5 at scale)
        s.RemoteDiff.Put(ts, v)
    s.merge()
    assert s.DiffSignature == sig and s.CurrentState == st
    e = Server(eng, 1)
    e.merge()                               # empty Diff and RemoteDiff
    assert e.DiffSignature == [] and e.CurrentState == {}


def test_add_command_local_apply(eng):
    s = NewServer(8080, {}, [], eng=eng)
    assert s.AddCommand(100, {"a": "5"}) == 200          # new key: inserted, early return
    assert s.CurrentState == {"a": "5"}
    assert s.AddCommand(101, {"a": "-3"}) == 200
    assert s.CurrentState == {"a": "2"}
    assert s.AddCommand(102, {"a": "x"}) == 500          # Atoi(value) error
    assert s.AddCommand(103, {"b": "1", "c": "2"}) == 200  # returns after the first new key
    assert s.CurrentState == {"a": "2", "b": "1"}
    assert s.AddCommand(103, {"a": "1"}) == 200          # same-ms write overwrites the Diff entry
    assert s.DiffSignature == [[100, "local"], [101, "local"], [102, "local"], [103, "local"]]
    s.merge()                                            # local entries are excluded from the replay
    assert s.CurrentState == {}


def test_device_atoi_matches_go(eng):
    cases = ["0", "-0", "+7", "007", "9223372036854775807", "-9223372036854775808", "9223372036854775808",
             "", "+", "-", "1_0", "0x1", " 1", "1 ", "18446744073709551616", "00000000000000000000000000042",
             "-00000000000000000000001", "--1", "12a", "99999999999999999999", "-9223372036854775809"]
    blob = b"".join(c.encode() for c in cases)
    off = np.concatenate([[0], np.cumsum([len(c.encode()) for c in cases])]).astype(np.int64)
    ok, val = eng.atoi_batch(torch.from_numpy(np.frombuffer(blob, np.uint8).copy()).to(eng.device),
                             torch.from_numpy(off).to(eng.device))
    for c, o, v in zip(cases, ok.cpu().tolist(), val.cpu().tolist()):
        assert (bool(o), v if o else 0) == oracle.go_atoi(c), c


def test_many_keys_per_replica_matches_oracle(eng):
    """Replicas with ~2500 distinct keys overflow the replay fold's 512-entry
    per-tile LDS table, so part of their pairs go straight to the global slot
    accumulators; mixed in one batch with small replicas that stay in LDS."""
    rng = np.random.default_rng(5)
    reps = []
    for r, nkeys in enumerate((2500, 40, 3000)):
        diff, remote, ts = {}, {}, 0
        for _ in range(4000):
            ts += int(rng.integers(1, 4))
            m = {}
            for _ in range(int(rng.integers(1, 4))):
                v = int(rng.integers(-50, 50))
                m[f"key{int(rng.integers(0, nkeys))}"] = str(v) if rng.random() > 0.05 else f"x{v}"
            if rng.random() < 0.5:
                diff[ts] = Command(m) if rng.random() < 0.3 else m
            else:
                remote[ts] = m
        reps.append((diff, remote))
    res = refmerge.merge_batch(eng, reps)
    for (diff, remote), (d_gpu, s_gpu) in zip(reps, res):
        d_or, s_or = oracle_merge(diff, remote)
        assert list(d_gpu) == list(d_or)
        assert s_gpu == s_or


def test_slice_write_without_slots(eng):
    """n_slots = 0 (no replay): the new Diff comes from the standalone slice
    write (k_rm_write) instead of the fused fold pass -- same slices."""
    h = synth.refmerge_packed(12, 40, 4000)
    full = eng.refmerge_batch(refmerge.to_device(h, eng.device))
    bare = eng.refmerge_batch(refmerge.to_device(dict(h, n_slots=0), eng.device))
    n = int(full["off"][-1])
    np.testing.assert_array_equal(bare["off"].cpu().numpy(), full["off"].cpu().numpy())
    for k in ("ts", "origin", "src"):
        np.testing.assert_array_equal(bare[k][:n].cpu().numpy(), full[k][:n].cpu().numpy())


@pytest.mark.diag
def test_count_pass_register_staging(eng):
    """refmerge.count_dma=0: the count pass stages the tile's ts through
    registers instead of LDS-DMA (also the path for logs that are not 8-byte
    aligned); same outputs on the packed batch and the KATs."""
    from crdt_amd import _lib
    set_knob(b"refmerge.count_dma", 0)
    try:
        test_packed_batch_matches_oracle(eng, 0)
        test_all_kats_in_one_batch(eng)
    finally:
        set_knob(b"refmerge.count_dma", 1)


def _expected_kv(h, src, n_out):
    """The new Diff's kv pairs by definition: entry i's pairs are its source
    entry's (src >= 0: L index, < 0: R index -src-1), ranges clamped to the
    arena like the device does; offsets are their running sum."""
    n_kv = len(h["kv_key"])
    kk, vv = np.asarray(h["kv_key"]).view(np.uint32), np.asarray(h["kv_val"]).view(np.uint32)
    off, keys, vals = [0], [], []
    for s in src[:n_out].tolist():
        kvo = h["l_kv"] if s >= 0 else h["r_kv"]
        j = s if s >= 0 else -s - 1
        b, e = int(kvo[j]), min(int(kvo[j + 1]), n_kv)
        if b < e:
            keys.append(kk[b:e])
            vals.append(vv[b:e])
        off.append(off[-1] + max(e - b, 0))
    cat = lambda xs: np.concatenate(xs) if xs else np.zeros(0, np.uint32)
    return np.array(off, np.int64), cat(keys), cat(vals)


def _run_kv(eng, h, cap=None):
    d = refmerge.to_device(h, eng.device)
    n = len(h["l_ts"]) + len(h["r_ts"])
    cap = 2 * max(len(h["kv_key"]), 1) if cap is None else cap
    kv = {"off": torch.full((n + 1,), -1, dtype=torch.int64, device=eng.device),
          "key": torch.zeros(max(cap, 1), dtype=torch.int32, device=eng.device),
          "val": torch.zeros(max(cap, 1), dtype=torch.int32, device=eng.device)}
    if cap == 0:
        kv["key"], kv["val"] = kv["key"][:0], kv["val"][:0]
    return eng.refmerge_batch(d, kv=kv), eng.refmerge_batch(d), kv


def _assert_kv_output(h, out, plain, kv):
    """crdt_refmerge_batch_kv: the merge outputs equal the plain call's
    (themselves oracle-checked above) and the kv pairs equal the host gather."""
    for k in ("off", "ts", "origin", "src", "st_kind", "st_str", "st_sum"):
        n = int(plain["off"][-1]) if k in ("ts", "origin", "src") else None
        assert torch.equal(out[k][:n], plain[k][:n]), k
    n_out = int(plain["off"][-1])
    e_off, e_key, e_val = _expected_kv(h, plain["src"].cpu().numpy(), n_out)
    np.testing.assert_array_equal(kv["off"][: n_out + 1].cpu().numpy(), e_off)
    m = int(e_off[-1])
    np.testing.assert_array_equal(kv["key"][:m].cpu().numpy().view(np.uint32), e_key)
    np.testing.assert_array_equal(kv["val"][:m].cpu().numpy().view(np.uint32), e_val)


@pytest.mark.parametrize("case", ["packed", "multi_key", "ragged_ranges", "many_replicas"])
def test_batch_kv_output(eng, case):
    """The new Diff's kv pairs out of the merge's own passes (count pass:
    pairs per tile; tile pass: offsets and copies) == a host gather by src:
    the bench's packed batch (one pair per entry), multi-pair entries, empty
    / overlapping / past-the-arena ranges, and > 65536 tiles (the
    multi-kernel scan path)."""
    if case == "packed":
        h = synth.refmerge_packed(11, 48, 5000)
    elif case == "many_replicas":
        h = synth.refmerge_packed(23, 70_000, 12)
    else:
        pk = refmerge.Packer()
        for d, r in synth.refmerge_demo(31, replicas=40, entries=700, multi_key=0.4):
            pk.add_replica(d, r)
        h = pk.arrays()
        if case == "ragged_ranges":
            rng = np.random.default_rng(5)
            n_kv = len(h["kv_key"])
            for a in ("l_kv", "r_kv"):
                x = h[a].copy()
                i = rng.choice(len(x), size=len(x) // 7, replace=False)
                # shifted ends: empty, reversed, overlapping and past-the-arena ranges
                x[i] = np.clip(x[i] + rng.integers(-3, 4, size=len(i)), 0, n_kv + 5)
                h[a] = x
    out, plain, kv = _run_kv(eng, h)
    assert eng.device_status(clear=True) == 0
    _assert_kv_output(h, out, plain, kv)


def test_batch_kv_output_capacity(eng):
    """A kv total over kv_cap raises CRDT_DEV_RANGE (nothing written past
    the arena); an exact-size arena is enough."""
    h = synth.refmerge_packed(7, 9, 3000)
    _, plain, _ = _run_kv(eng, h)
    total = len(_expected_kv(h, plain["src"].cpu().numpy(), int(plain["off"][-1]))[1])
    out, _, kv = _run_kv(eng, h, cap=total)
    assert eng.device_status(clear=True) == 0
    _assert_kv_output(h, out, plain, kv)
    _run_kv(eng, h, cap=total - 1)
    assert eng.device_status(clear=True) == 2


def test_batch_pull_in_place_equals_assembled(eng):
    """crdt_refmerge_batch_pull: every replica's R is a peer's L read in
    place (overlapping ranges, self-pulls, key slots re-based by
    r_slot_delta) == the same batch with each RemoteDiff assembled as a copy
    (the peer's entries, its pairs' slots re-based) through
    crdt_refmerge_batch_kv: same new Diffs, kv pairs and CurrentState."""
    h = synth.refmerge_packed(13, 24, 3000)
    P, S = h["replicas"], h["n_slots"] // h["replicas"]
    q = (np.arange(P) * 7 + 3) % P                      # peers (replica 5: itself)
    l_off, l_kv = h["l_off"], h["l_kv"]
    kk, kv_val = np.asarray(h["kv_key"]).view(np.uint32), np.asarray(h["kv_val"])
    sd = ((np.arange(P) - q) * S) % (1 << 32)
    # assembled: R_p = a copy of L_q, its pairs appended to the arena with re-based slots
    r_off, r_ts, r_kv, ek, ev = [0], [], [], [], []
    base = len(kk)
    for p in range(P):
        a, b = int(l_off[q[p]]), int(l_off[q[p] + 1])
        r_ts.append(h["l_ts"][a:b])
        for e in range(a, b):
            r_kv.append(base)
            x, y = int(l_kv[e]), int(l_kv[e + 1])
            ek.append(((kk[x:y].astype(np.int64) + int(sd[p])) % (1 << 32)).astype(np.uint32))
            ev.append(kv_val[x:y])
            base += y - x
        r_off.append(r_off[-1] + b - a)
    r_kv.append(base)
    ha = dict(h, r_off=np.array(r_off, np.int64), r_ts=np.concatenate(r_ts), r_kv=np.array(r_kv, np.int64),
              kv_key=np.concatenate([kk] + ek).view(np.int32), kv_val=np.concatenate([kv_val] + ev))
    out_a, _, kv_a = _run_kv(eng, ha)
    # in place: R ranges of the L arrays
    hi = dict(h, r_off=l_off[q].copy(), r_ts=h["l_ts"], r_kv=l_kv)
    d = refmerge.to_device(hi, eng.device)
    d["n_r"] = int(r_off[-1])
    n = len(h["l_ts"]) + d["n_r"]
    kv_i = {"off": torch.full((n + 1,), -1, dtype=torch.int64, device=eng.device),
            "key": torch.zeros(2 * base, dtype=torch.int32, device=eng.device),
            "val": torch.zeros(2 * base, dtype=torch.int32, device=eng.device)}
    pull = {"r_end": torch.from_numpy(l_off[q + 1].copy()).to(eng.device),
            "r_slot_delta": torch.from_numpy(sd.astype(np.uint32).view(np.int32)).to(eng.device)}
    out_i = eng.refmerge_batch(d, kv=kv_i, pull=pull)
    assert eng.device_status(clear=True) == 0
    n_out = int(out_a["off"][-1])
    for k in ("off", "st_kind", "st_str", "st_sum"):
        assert torch.equal(out_i[k], out_a[k]), k
    for k in ("ts", "origin"):
        assert torch.equal(out_i[k][:n_out], out_a[k][:n_out]), k
    # src: an R entry's index in the assembled R <-> its L index in place
    sa, si = out_a["src"][:n_out].cpu().numpy(), out_i["src"][:n_out].cpu().numpy()
    np.testing.assert_array_equal(si >= 0, sa >= 0)
    np.testing.assert_array_equal(si[sa >= 0], sa[sa >= 0])
    ra = np.array(r_off, np.int64)
    j = -sa[sa < 0] - 1
    p_of = np.searchsorted(ra, j, side="right") - 1
    np.testing.assert_array_equal(-si[sa < 0] - 1, l_off[q[p_of]] + (j - ra[p_of]))
    m = int(kv_a["off"][n_out])
    assert int(kv_i["off"][n_out]) == m and int(kv_i["off"][n]) == m
    assert torch.equal(kv_i["off"][: n_out + 1], kv_a["off"][: n_out + 1])
    assert torch.equal(kv_i["key"][:m], kv_a["key"][:m]) and torch.equal(kv_i["val"][:m], kv_a["val"][:m])


def _pull_batch(eng, seed=19, P=12):
    h = synth.refmerge_packed(seed, P, 2000)
    q = (np.arange(P) * 5 + 1) % P
    l_off = h["l_off"]
    hi = dict(h, r_off=l_off[q].copy(), r_ts=h["l_ts"], r_kv=h["l_kv"])
    d = refmerge.to_device(hi, eng.device)
    d["n_r"] = int((l_off[q + 1] - l_off[q]).sum())
    n = len(h["l_ts"]) + d["n_r"]
    kv = {"off": torch.zeros(n + 1, dtype=torch.int64, device=eng.device),
          "key": torch.zeros(2 * len(h["kv_key"]) + 2, dtype=torch.int32, device=eng.device),
          "val": torch.zeros(2 * len(h["kv_key"]) + 2, dtype=torch.int32, device=eng.device)}
    sd = ((np.arange(P) - q) * (h["n_slots"] // P)) % (1 << 32)
    pull = {"r_end": torch.from_numpy(l_off[q + 1].copy()).to(eng.device),
            "r_slot_delta": torch.from_numpy(sd.astype(np.uint32).view(np.int32)).to(eng.device)}
    return d, kv, pull, q


def test_batch_pull_slot_delta_requires_kv_output(eng):
    """crdt_refmerge_batch_pull with re-based key slots (r_slot_delta) but no
    fused kv output is CRDT_E_INVAL: a gather of the new Diff's pairs by src
    afterwards could not re-base the pulled slots (the boundary hazard of a
    cgo caller, include/crdt_amd.h)."""
    from crdt_amd import _lib
    d, kv, pull, _ = _pull_batch(eng)
    with pytest.raises(_lib.CrdtError) as ei:
        eng.refmerge_batch(d, pull=pull)
    assert ei.value.status == -1                         # CRDT_E_INVAL
    eng.refmerge_batch(d, pull={"r_end": pull["r_end"], "r_slot_delta": None})   # no re-basing: allowed
    assert eng.device_status(clear=True) == 0
    eng.refmerge_batch(d, kv=kv, pull=pull)
    assert eng.device_status(clear=True) == 0


@pytest.mark.parametrize("bad", ["reversed", "past_n_r"])
def test_batch_pull_bad_ranges_raise_range_flag(eng, bad):
    """R ranges the call was not sized for -- a reversed range (r_end < r_off)
    or ranges summing past n_r -- raise CRDT_DEV_RANGE on the device instead
    of reading / writing out of range (the planning passes clamp and the
    offset passes write nothing)."""
    d, kv, pull, q = _pull_batch(eng, seed=23)
    if bad == "reversed":
        r_end = pull["r_end"].clone()
        r_end[3] = d["r_off"][3] - 1 if int(d["r_off"][3]) > 0 else 0
        d["r_off"][3] = r_end[3] + 1
        pull = dict(pull, r_end=r_end)
    else:
        d["n_r"] = d["n_r"] // 3
        kv["off"] = kv["off"][: len(d["l_ts"]) + d["n_r"] + 1].clone()
    eng.refmerge_batch(d, kv=kv, pull=pull)
    assert eng.device_status(clear=True) & 2            # CRDT_DEV_RANGE
