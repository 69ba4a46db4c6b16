"""Test helpers for RefMerge: KAT loading and the C-oracle driver."""
import json
import os

import numpy as np

from crdt_amd.refmerge import Command, Packer
from oracle import oracle

HERE = os.path.dirname(os.path.abspath(__file__))


def load_kats():
    with open(os.path.join(HERE, "golden", "refmerge_kat.json")) as f:
        return json.load(f)["kats"]


def kat_inputs(k):
    diff = {ts: (Command(kv) if origin == "local" else dict(kv)) for ts, origin, kv in k["L"]}
    remote = {ts: dict(kv) for ts, kv in k["R"]}
    return diff, remote


def diff_signature(diff):
    return [[ts, "local" if type(v).__name__ == "Command" else "remote"] for ts, v in sorted(diff.items())]


def oracle_packed_replica(h, p, slots_per_replica=62):
    """Oracle merge of replica p of a packed batch (crdt_amd.synth.refmerge_packed).
    Returns (diff_ts, diff_origin, diff_src_global, kind, str, sum) with src
    rebased to the batch's global L / R indices like the device output."""
    lb, le = int(h["l_off"][p]), int(h["l_off"][p + 1])
    rb, re_ = int(h["r_off"][p]), int(h["r_off"][p + 1])
    kv_key = (h["kv_key"].view(np.uint32).astype(np.int64) - p * slots_per_replica).astype(np.uint32)
    o_ts, o_or, o_src, kind, sstr, ssum = oracle.refmerge_packed(
        h["l_ts"][lb:le], h["l_origin"][lb:le], h["l_kv"][lb:le + 1].astype(np.uint32),
        h["r_ts"][rb:re_], h["r_kv"][rb:re_ + 1].astype(np.uint32), kv_key, h["kv_val"].view(np.uint32),
        h["str_bytes"], h["str_off"], slots_per_replica)
    src = np.where(o_src >= 0, o_src + lb, o_src - rb)
    return o_ts, o_or, src, kind, sstr, ssum


def oracle_merge(diff, remote):
    """(new_diff, state) of one replica through oracle/crdt_oracle.c."""
    pk = Packer()
    pk.add_replica(diff, remote)
    a = pk.arrays()
    n_l = len(a["l_ts"])
    o_ts, o_or, o_src, kind, sstr, ssum = oracle.refmerge_packed(
        a["l_ts"], a["l_origin"], a["l_kv"][: n_l + 1].astype(np.uint32), a["r_ts"],
        a["r_kv"].astype(np.uint32), a["kv_key"].view(np.uint32), a["kv_val"].view(np.uint32),
        a["str_bytes"], a["str_off"], a["n_slots"])
    new_diff = {}
    for t, s in zip(o_ts.tolist(), o_src.tolist()):
        new_diff[t] = pk.l_vals[s] if s >= 0 else pk.r_vals[-s - 1]
    state = {}
    for slot in range(a["n_slots"]):
        if kind[slot] == 1:
            state[pk.slot_names[slot]] = pk.strings[int(sstr[slot])].decode("utf-8", "surrogatepass")
        elif kind[slot] == 2:
            state[pk.slot_names[slot]] = str(int(ssum[slot]))
    return new_diff, state


def assert_batch_matches_oracle(h, out, slots_per_replica=62, replicas=None):
    """Every replica (or the listed ones) of a packed batch's device output
    == oracle_packed_replica: new Diff ts / origin / src and CurrentState."""
    off = out["off"].cpu().numpy()
    ts, org, src = (out[k].cpu().numpy() for k in ("ts", "origin", "src"))
    kind, sstr, ssum = (out[k].cpu().numpy() for k in ("st_kind", "st_str", "st_sum"))
    for p in (range(h["replicas"]) if replicas is None else replicas):
        o_ts, o_or, o_src, k, s, v = oracle_packed_replica(h, p, slots_per_replica)
        a, b = int(off[p]), int(off[p + 1])
        np.testing.assert_array_equal(ts[a:b], o_ts)
        np.testing.assert_array_equal(org[a:b], o_or)
        np.testing.assert_array_equal(src[a:b], o_src)
        sl = slice(p * slots_per_replica, (p + 1) * slots_per_replica)
        np.testing.assert_array_equal(kind[sl], k)
        np.testing.assert_array_equal(sstr[sl].view(np.uint32)[k == 1], s[k == 1])
        np.testing.assert_array_equal(ssum[sl][k == 2], v[k == 2])


def split_ts_range(h, lo, hi):
    """The [lo, hi) ts slice of every replica of a host packed batch (kv pairs
    carried along), plus the global L / R index of each kept entry
    (`l_sel` / `r_sel`): one rank's share of a ts-range-sharded batch."""
    P = h["replicas"]
    kvk, kvv = h["kv_key"], h["kv_val"]
    out = {"replicas": P, "n_slots": h["n_slots"], "str_bytes": h["str_bytes"], "str_off": h["str_off"]}
    keys, vals = [], []
    nkv = 0
    for side in ("l", "r"):
        off, ts, kv = h[f"{side}_off"], h[f"{side}_ts"], h[f"{side}_kv"]
        sel = []
        noff = [0]
        for p in range(P):
            b, e = int(off[p]), int(off[p + 1])
            i = b + int(np.searchsorted(ts[b:e], lo, side="left"))
            j = b + int(np.searchsorted(ts[b:e], hi, side="left"))
            sel.append(np.arange(i, j))
            noff.append(noff[-1] + (j - i))
        sel = np.concatenate(sel).astype(np.int64) if sel else np.zeros(0, np.int64)
        cnt = (kv[sel + 1] - kv[sel]).astype(np.int64)
        nkvo = np.zeros(len(sel) + 1, np.int64)
        nkvo[1:] = np.cumsum(cnt)
        idx = np.concatenate([np.arange(kv[s], kv[s + 1]) for s in sel]).astype(np.int64) if len(sel) else \
            np.zeros(0, np.int64)
        keys.append(kvk[idx])
        vals.append(kvv[idx])
        out[f"{side}_off"] = np.array(noff, np.int64)
        out[f"{side}_ts"] = ts[sel].copy()
        out[f"{side}_kv"] = nkvo + nkv
        out[f"{side}_sel"] = sel
        if side == "l":
            out["l_origin"] = h["l_origin"][sel].copy()
        nkv += int(nkvo[-1])
    out["kv_key"] = np.concatenate(keys)
    out["kv_val"] = np.concatenate(vals)
    return out


def ts_splitters(h, world):
    """world + 1 ts splitters: quantiles of every L and R ts, open ends."""
    allts = np.sort(np.concatenate([h["l_ts"], h["r_ts"]]))
    return [int(np.iinfo(np.int64).min)] + [int(allts[(r * len(allts)) // world]) for r in range(1, world)] + \
        [int(np.iinfo(np.int64).max)]
