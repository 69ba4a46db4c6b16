"""GPU: incremental replay -- crdt_refmerge_delta with a
carried ts-keyed state must equal the full re-fold of crdt_refmerge_batch
(itself pinned to the oracle by test_gpu_refmerge.py), merge after merge,
and the carried state must equal a fresh crdt_replay_state_init of the new
Diff."""
import numpy as np
import pytest

from crdt_amd import refmerge, synth
from refmerge_util import kat_inputs, load_kats

pytestmark = pytest.mark.gpu


def _np(out, k, n=None):
    a = out[k].cpu().numpy()
    return a if n is None else a[:n]


def _same_merge(full, delta):
    n = int(full["off"][-1])
    for k in ("off",):
        np.testing.assert_array_equal(_np(delta, k), _np(full, k))
    for k in ("ts", "origin", "src"):
        np.testing.assert_array_equal(_np(delta, k, n), _np(full, k, n))
    kind = _np(full, "st_kind")
    np.testing.assert_array_equal(_np(delta, "st_kind"), kind)
    np.testing.assert_array_equal(_np(delta, "st_str")[kind == 1], _np(full, "st_str")[kind == 1])
    np.testing.assert_array_equal(_np(delta, "st_sum")[kind == 2], _np(full, "st_sum")[kind == 2])


def _same_state(a, b):
    present = a["nhold"].cpu().numpy() > 0
    np.testing.assert_array_equal(b["nhold"].cpu().numpy(), a["nhold"].cpu().numpy())
    for k in ("best_key", "best_str", "sum", "npar"):
        np.testing.assert_array_equal(a[k].cpu().numpy()[present], b[k].cpu().numpy()[present])


def _next_round(h, out, rng, slots_per_replica=62):
    """Host batch for the next merge: L = the new Diff (kvs carried along by
    src), R = fresh remote entries (some on L's ts, some new, some above
    max(L))."""
    n = int(out["off"][-1].item())
    off = _np(out, "off")
    ts, org, src = _np(out, "ts", n), _np(out, "origin", n), _np(out, "src", n)
    kvs = []
    for s in src.tolist():
        if s >= 0:
            a, b = int(h["l_kv"][s]), int(h["l_kv"][s + 1])
        else:
            g = -s - 1
            a, b = int(h["r_kv"][g]), int(h["r_kv"][g + 1])
        kvs.append((h["kv_key"][a:b], h["kv_val"][a:b]))
    l_kv = np.zeros(n + 1, np.int64)
    l_kv[1:] = np.cumsum([len(k) for k, _ in kvs])
    r_rows, r_keys, r_vals = [], [], []
    nstr = len(h["str_off"]) - 1
    for p in range(h["replicas"]):
        lt = ts[off[p]:off[p + 1]]
        hi = int(lt[-1]) if len(lt) else 0
        lo = int(lt[0]) if len(lt) else 0
        m = int(rng.integers(50, 400))
        cand = np.concatenate([rng.integers(lo - 5, hi + 50, m),
                               rng.choice(lt, min(len(lt), 20)) if len(lt) else np.zeros(0, np.int64)])
        row = np.unique(cand.astype(np.int64))
        r_rows.append(row)
        for _ in row:
            k = int(rng.integers(1, 3))
            # a map: distinct keys within one entry
            r_keys.append((p * slots_per_replica + rng.choice(slots_per_replica, k, replace=False)).astype(np.uint32))
            r_vals.append(rng.integers(0, nstr, k).astype(np.uint32))
    r_off = np.zeros(h["replicas"] + 1, np.int64)
    r_off[1:] = np.cumsum([len(r) for r in r_rows])
    nl_kv = int(l_kv[-1])
    r_kv = np.zeros(int(r_off[-1]) + 1, np.int64)
    r_kv[1:] = np.cumsum([len(k) for k in r_keys])
    r_kv += nl_kv
    kv_key = np.concatenate([k for k, _ in kvs] + r_keys).astype(np.uint32) if (kvs or r_keys) else \
        np.zeros(0, np.uint32)
    kv_val = np.concatenate([v for _, v in kvs] + r_vals).astype(np.uint32) if (kvs or r_vals) else \
        np.zeros(0, np.uint32)
    return {"replicas": h["replicas"], "n_slots": h["n_slots"], "l_off": off.astype(np.int64),
            "l_ts": ts.astype(np.int64), "l_origin": org.astype(np.uint8), "l_kv": l_kv,
            "r_off": r_off, "r_ts": np.concatenate(r_rows).astype(np.int64), "r_kv": r_kv,
            "kv_key": kv_key.view(np.int32), "kv_val": kv_val.view(np.int32),
            "str_bytes": h["str_bytes"], "str_off": h["str_off"]}


def test_delta_equals_full_single_merge(eng):
    h = synth.refmerge_packed(3, 64, 3000)
    d = refmerge.to_device(h, eng.device)
    full = eng.refmerge_batch(d)
    st = eng.replay_state_init(d)
    _same_merge(full, eng.refmerge_delta(d, st))


def test_delta_chained_merges(eng):
    rng = np.random.default_rng(9)
    h = synth.refmerge_packed(4, 32, 2000)
    h["kv_key"] = h["kv_key"].view(np.uint32)
    h["kv_val"] = h["kv_val"].view(np.uint32)
    d = refmerge.to_device({**h, "kv_key": h["kv_key"].view(np.int32), "kv_val": h["kv_val"].view(np.int32)},
                           eng.device)
    st = eng.replay_state_init(d)
    for _ in range(3):
        full = eng.refmerge_batch(d)
        out = eng.refmerge_delta(d, st)
        _same_merge(full, out)
        h = _next_round(h, out, rng)
        d = refmerge.to_device(h, eng.device)
        h["kv_key"] = h["kv_key"].view(np.uint32)
        h["kv_val"] = h["kv_val"].view(np.uint32)
        _same_state(eng.replay_state_init(d), st)       # carried state == fresh fold of the new Diff


def test_delta_on_kats(eng):
    """Every hand-derived KAT in one batch, through init + delta."""
    kats = load_kats()
    pk = refmerge.Packer()
    for k in kats:
        pk.add_replica(*kat_inputs(k))
    d = refmerge.to_device(pk.arrays(), eng.device)
    full = eng.refmerge_batch(d)
    st = eng.replay_state_init(d)
    _same_merge(full, eng.refmerge_delta(d, st))


def test_delta_table_overflow(eng):
    """Replicas with thousands of distinct keys overflow the delta fold's
    512-entry per-tile LDS table (pairs go straight to the carried state and
    the holder pass walks every inserted entry); mixed with a small replica."""
    from crdt_amd.server import Command
    rng = np.random.default_rng(6)
    pk = refmerge.Packer()
    for nkeys in (2500, 40, 3000):
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
        pk.add_replica(diff, remote)
    d = refmerge.to_device(pk.arrays(), eng.device)
    full = eng.refmerge_batch(d)
    st = eng.replay_state_init(d)
    _same_merge(full, eng.refmerge_delta(d, st))


def test_delta_large_batch_then_overflow(eng):
    """A candidate-path delta merge followed by an overflow-path one on the
    same engine: the overflow flag is reset per merge."""
    h = synth.refmerge_packed(8, 16, 3000)
    d = refmerge.to_device(h, eng.device)
    st = eng.replay_state_init(d)
    _same_merge(eng.refmerge_batch(d), eng.refmerge_delta(d, st))
    test_delta_table_overflow(eng)
    h = synth.refmerge_packed(9, 16, 3000)
    d = refmerge.to_device(h, eng.device)
    st = eng.replay_state_init(d)
    _same_merge(eng.refmerge_batch(d), eng.refmerge_delta(d, st))


# ---- pinned to the oracle / the hand-derived KATs directly (not only to the full GPU refold)
def test_delta_kats_match_expected(eng):
    """Every KAT through crdt_replay_state_init + crdt_refmerge_delta: the new
    Diff and CurrentState equal the hand-derived expectations."""
    from refmerge_util import diff_signature
    kats = load_kats()
    pk = refmerge.Packer()
    for k in kats:
        pk.add_replica(*kat_inputs(k))
    arrs = pk.arrays()
    d = refmerge.to_device(arrs, eng.device)
    st = eng.replay_state_init(d)
    res = refmerge.unpack_batch(pk, arrs, eng.refmerge_delta(d, st))
    for k, (diff, state) in zip(kats, res):
        assert diff_signature(diff) == k["diff"], k["name"]
        assert state == k["state"], k["name"]


def test_delta_chained_merges_match_oracle(eng):
    """Three chained delta merges (the carried state is never rebuilt): every
    replica's new Diff and CurrentState == oc_refmerge of that merge's
    (L, R), main.go:35-100."""
    from refmerge_util import assert_batch_matches_oracle
    rng = np.random.default_rng(19)
    h = synth.refmerge_packed(14, 24, 2500)
    d = refmerge.to_device(h, eng.device)
    st = eng.replay_state_init(d)
    for _ in range(3):
        out = eng.refmerge_delta(d, st)
        assert_batch_matches_oracle(h, out)
        h = _next_round({**h, "kv_key": h["kv_key"].view(np.uint32), "kv_val": h["kv_val"].view(np.uint32)},
                        out, rng)
        d = refmerge.to_device(h, eng.device)
