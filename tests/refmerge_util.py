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
