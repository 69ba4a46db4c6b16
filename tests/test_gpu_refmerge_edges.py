"""GPU: RefMerge on adversarial batch shapes -- replica logs sized around the
tile (4096 merge items; 2048 before) and its bitmap words (64 items):
n-1 / n / n+1 / many tiles / one side empty / both
empty), ts at the int64 extremes and negative, heavy L/R collisions at tile
edges, 1-2 kv pairs per entry -- replica by replica against the C oracle,
through the full re-fold and through the incremental replay."""
import numpy as np
import pytest

from crdt_amd import refmerge
from oracle import oracle

pytestmark = pytest.mark.gpu

K = 16
I64 = np.iinfo(np.int64)
STRS = [str(v) for v in range(-5, 6)] + ["x", "007", "+3", "9223372036854775807", "-9223372036854775808", ""]
SHAPES = [(0, 0), (0, 5), (5, 0), (2047, 1), (1, 2047), (2048, 2048), (2049, 0), (0, 2049), (3000, 3000),
          (1, 1), (6000, 10), (10, 6000), (4095, 4097), (0, 0), (700, 700),
          (4095, 1), (1, 4095), (4096, 1), (4097, 0), (0, 4097), (8193, 3), (63, 1), (64, 64), (65, 0)]


def _batch(seed):
    rng = np.random.default_rng(seed)
    l_ts, l_org, r_ts, l_off, r_off = [], [], [], [0], [0]
    for nl, nr in SHAPES:
        span = max(nl, nr) * 2 + 4
        base = int(rng.integers(-10**6, 10**6))
        L = np.unique(rng.integers(base, base + span, nl * 2 + 1))[:nl] if nl else np.zeros(0, np.int64)
        if nl and rng.random() < 0.3:
            L[0] = I64.min                                  # extremes at the ends of the order
        if nl > 1 and rng.random() < 0.3:
            L[-1] = I64.max
        L = np.unique(L)
        coll = rng.choice(L, min(len(L), nr // 3)) if len(L) else np.zeros(0, np.int64)
        R = np.unique(np.concatenate([rng.integers(base - 3, base + span + 3, nr), coll]))[:nr] if nr else \
            np.zeros(0, np.int64)
        l_ts.append(L)
        r_ts.append(R)
        l_org.append((rng.random(len(L)) < 0.4).astype(np.uint8))
        l_off.append(l_off[-1] + len(L))
        r_off.append(r_off[-1] + len(R))
    nL, nR = l_off[-1], r_off[-1]
    P = len(SHAPES)
    l_rep = np.repeat(np.arange(P), np.diff(l_off))
    r_rep = np.repeat(np.arange(P), np.diff(r_off))
    keys, vals, cnt = [], [], []
    for rep in np.concatenate([l_rep, r_rep]):
        k = int(rng.integers(1, 3))
        keys.append(rep * K + rng.choice(K, k, replace=False))
        vals.append(rng.integers(0, len(STRS), k))
        cnt.append(k)
    kv_off = np.zeros(nL + nR + 1, np.int64)
    kv_off[1:] = np.cumsum(cnt)
    blob = "".join(STRS).encode()
    so = np.zeros(len(STRS) + 1, np.int64)
    so[1:] = np.cumsum([len(s.encode()) for s in STRS])
    return {"replicas": P, "n_slots": P * K,
            "l_off": np.array(l_off, np.int64), "l_ts": np.concatenate(l_ts).astype(np.int64),
            "l_origin": np.concatenate(l_org), "l_kv": kv_off[:nL + 1].copy(),
            "r_off": np.array(r_off, np.int64), "r_ts": np.concatenate(r_ts).astype(np.int64),
            "r_kv": kv_off[nL:].copy(),
            "kv_key": np.concatenate(keys).astype(np.uint32).view(np.int32),
            "kv_val": np.concatenate(vals).astype(np.uint32).view(np.int32),
            "str_bytes": np.frombuffer(blob, np.uint8).copy(), "str_off": so}


def _check(h, out):
    off = out["off"].cpu().numpy()
    ts, org, src = (out[k].cpu().numpy() for k in ("ts", "origin", "src"))
    kind, sstr, ssum = (out[k].cpu().numpy() for k in ("st_kind", "st_str", "st_sum"))
    kvk_all = h["kv_key"].view(np.uint32).astype(np.int64)
    for p in range(h["replicas"]):
        lb, le = int(h["l_off"][p]), int(h["l_off"][p + 1])
        rb, re_ = int(h["r_off"][p]), int(h["r_off"][p + 1])
        o_ts, o_or, o_src, k, s, v = oracle.refmerge_packed(
            h["l_ts"][lb:le], h["l_origin"][lb:le], h["l_kv"][lb:le + 1].astype(np.uint32),
            h["r_ts"][rb:re_], h["r_kv"][rb:re_ + 1].astype(np.uint32), (kvk_all - p * K).astype(np.uint32),
            h["kv_val"].view(np.uint32), h["str_bytes"], h["str_off"], K)
        a, b = int(off[p]), int(off[p + 1])
        np.testing.assert_array_equal(ts[a:b], o_ts, err_msg=f"replica {p} ts")
        np.testing.assert_array_equal(org[a:b], o_or, err_msg=f"replica {p} origin")
        np.testing.assert_array_equal(src[a:b], np.where(o_src >= 0, o_src + lb, o_src - rb), err_msg=f"replica {p}")
        sl = slice(p * K, (p + 1) * K)
        np.testing.assert_array_equal(kind[sl], k, err_msg=f"replica {p} kind")
        np.testing.assert_array_equal(sstr[sl].view(np.uint32)[k == 1], s[k == 1], err_msg=f"replica {p} str")
        np.testing.assert_array_equal(ssum[sl][k == 2], v[k == 2], err_msg=f"replica {p} sum")


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_edge_shapes_full_refold(eng, seed):
    h = _batch(seed)
    _check(h, eng.refmerge_batch(refmerge.to_device(h, eng.device)))


@pytest.mark.parametrize("seed", [4, 5])
def test_edge_shapes_incremental_replay(eng, seed):
    h = _batch(seed)
    d = refmerge.to_device(h, eng.device)
    st = eng.replay_state_init(d)
    _check(h, eng.refmerge_delta(d, st))
