"""Test helpers for the anti-entropy rounds (crdt_amd.gossip): host dict
Diffs <-> Population arrays, and the host simulation of a round on the
Python restatement of merge() (oracle/pyref.py, main.go:35-100)."""
import numpy as np

from oracle import pyref

K = 8
KEYS = [f"k{i}" for i in range(K)]
STRS = [str(v) for v in range(-20, -10)] + ["x", "007", "+3", "9223372036854775807"]


def _arena():
    blob = "".join(STRS).encode()
    off = np.zeros(len(STRS) + 1, np.int64)
    off[1:] = np.cumsum([len(s.encode()) for s in STRS])
    return np.frombuffer(blob, np.uint8).copy(), off


def _pack(diffs, first=0):
    """Host dict Diffs of replicas [first, first+len) -> Population host arrays."""
    sb, so = _arena()
    off, ts, org, kvo, kk, kv = [0], [], [], [0], [], []
    for i, d in enumerate(diffs):
        for t in sorted(d):
            v = d[t]
            ts.append(t)
            org.append(1 if isinstance(v, pyref.Command) else 0)
            for k, s in v.items():
                kk.append(i * K + KEYS.index(k))
                kv.append(STRS.index(s))
            kvo.append(len(kk))
        off.append(len(ts))
    return {"replicas": len(diffs), "l_off": np.array(off), "l_ts": np.array(ts, np.int64),
            "l_origin": np.array(org, np.uint8), "l_kv": np.array(kvo), "kv_key": np.array(kk, np.uint32),
            "kv_val": np.array(kv, np.uint32), "str_bytes": sb, "str_off": so}


def _unpack(pop):
    h = pop.to_host()
    out = []
    for i in range(pop.P):
        d = {}
        for e in range(int(h["off"][i]), int(h["off"][i + 1])):
            kv = {KEYS[int(h["kv_key"][q]) - i * K]: STRS[int(h["kv_val"][q])]
                  for q in range(int(h["kv_off"][e]), int(h["kv_off"][e + 1]))}
            d[int(h["ts"][e])] = pyref.Command(kv) if h["origin"][e] else kv
        out.append(d)
    return out


def _state(pop):
    kind = pop.state["st_kind"].cpu().numpy()
    sstr = pop.state["st_str"].cpu().numpy()
    ssum = pop.state["st_sum"].cpu().numpy()
    out = []
    for i in range(pop.P):
        st = {}
        for k in range(K):
            s = i * K + k
            if kind[s] == 1:
                st[KEYS[k]] = STRS[int(sstr[s])]
            elif kind[s] == 2:
                st[KEYS[k]] = str(int(ssum[s]))
        out.append(st)
    return out


def _same_diffs(got, exp):
    assert len(got) == len(exp)
    for g, e in zip(got, exp):
        assert sorted(g) == sorted(e)
        for t in e:
            assert isinstance(g[t], pyref.Command) == isinstance(e[t], pyref.Command), t
            assert dict(g[t]) == dict(e[t]), t


def _rand_diff(rng, t0, n):
    d, t = {}, t0
    for _ in range(n):
        t += int(rng.integers(1, 5))
        kv = {KEYS[int(k)]: STRS[int(rng.integers(0, len(STRS)))] for k in rng.choice(K, int(rng.integers(1, 3)),
                                                                                     replace=False)}
        d[t] = pyref.Command(kv) if rng.random() < 0.5 else kv
    return d


def _local_writes(rng, diffs):
    """1-3 local writes per replica after its last ts: host dicts updated,
    the device block returned."""
    off, ts, kvo, kk, kv = [0], [], [0], [], []
    for i, d in enumerate(diffs):
        t = max(d) if d else 1_000
        for _ in range(int(rng.integers(1, 4))):
            t += int(rng.integers(1, 5))
            k = KEYS[int(rng.integers(0, K))]
            s = STRS[int(rng.integers(0, len(STRS)))]
            d[t] = pyref.Command({k: s})
            ts.append(t)
            kk.append(i * K + KEYS.index(k))
            kv.append(STRS.index(s))
            kvo.append(len(kk))
        off.append(len(ts))
    return {"off": np.array(off), "ts": np.array(ts, np.int64), "kv_off": np.array(kvo),
            "kv_key": np.array(kk, np.uint32), "kv_val": np.array(kv, np.uint32)}


def _host_round(diffs, peers, states=None):
    """One synchronous round on pyref: replica i pulls diffs[peers[i]] (its
    own Diff on a self-pull); peers[i] < 0 is a dead peer, the round is
    skipped (main.go:234-239): Diff and CurrentState (from `states`, {} when
    not given) stay as they were."""
    pulled = [{t: dict(v) for t, v in diffs[q].items()} if q >= 0 else None for q in peers]   # ToJSON -> maps
    res = [pyref.merge(d, r) if r is not None else (d, (states[i] if states else {}))
           for i, (d, r) in enumerate(zip(diffs, pulled))]
    return [r[0] for r in res], [r[1] for r in res]
