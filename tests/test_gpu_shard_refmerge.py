"""GPU: the ts-range-sharded RefMerge emulated in one process.

A packed batch is split by ts range into W shards (every replica's Diff and
RemoteDiff cut at the same ts splitters, kv pairs carried along); each shard
runs the per-rank steps of crdt_amd.shard.sharded_refmerge, with the
all-reduces done here across the W shard results; the concatenated new-Diff
slices and the reduced CurrentState must equal the unsharded merge bit for
bit, and that unsharded merge == the oracle per replica in the same test."""
import numpy as np
import pytest
import torch

from crdt_amd import refmerge, synth
from refmerge_util import assert_batch_matches_oracle, split_ts_range as _split, ts_splitters

pytestmark = pytest.mark.gpu


def _run_sharded(eng, shards):
    """The per-rank steps of shard.sharded_refmerge with the all-reduces done
    across the in-process shards."""
    devs = [refmerge.to_device({k: v for k, v in s.items() if not k.endswith("_sel")}, eng.device) for s in shards]
    n_slots = int(shards[0]["n_slots"])
    maxl = torch.stack([eng.refmerge_local_maxl(d) for d in devs]).max(0).values
    accs = [eng.refmerge_acc_new(n_slots) for _ in devs]
    outs = [eng.refmerge_batch(d, maxl=maxl.clone(), acc=a) for d, a in zip(devs, accs)]
    cs = [eng.refmerge_acc_rank(a, n_slots, r) for r, a in enumerate(accs)]
    cmax = torch.stack(cs).max(0).values
    v = sum(eng.refmerge_acc_owner_str(a, n_slots, c, cmax) for a, c in zip(accs, cs))
    acc = {"best": accs[0]["best"], "sum": sum(a["sum"] for a in accs), "npar": sum(a["npar"] for a in accs)}
    eng.refmerge_acc_set_best(acc, n_slots, cmax, v)
    state = eng.refmerge_finalize(devs[0], acc, outs[0])
    return outs, state


@pytest.mark.parametrize("world", [2, 3, 5])
def test_ts_range_sharded_refmerge_equals_unsharded(eng, world):
    h = synth.refmerge_packed(41, 64, 3000)
    full = eng.refmerge_batch(refmerge.to_device(h, eng.device))
    assert_batch_matches_oracle(h, full)                     # the reference result itself == the oracle
    spl = ts_splitters(h, world)
    shards = [_split(h, spl[r], spl[r + 1]) for r in range(world)]
    # the top shard's exclusive end must not lose ts == INT64_MAX (none in this data)
    assert sum(len(s["l_ts"]) for s in shards) == len(h["l_ts"])
    assert sum(len(s["r_ts"]) for s in shards) == len(h["r_ts"])
    outs, state = _run_sharded(eng, shards)
    f_off = full["off"].cpu().numpy()
    f_ts, f_org, f_src = (full[k].cpu().numpy() for k in ("ts", "origin", "src"))
    so = [o["off"].cpu().numpy() for o in outs]
    sts = [o["ts"].cpu().numpy() for o in outs]
    sorg = [o["origin"].cpu().numpy() for o in outs]
    ssrc = [o["src"].cpu().numpy() for o in outs]
    for p in range(h["replicas"]):
        ts_p, org_p, src_p = [], [], []
        for r, s in enumerate(shards):
            a, b = int(so[r][p]), int(so[r][p + 1])
            ts_p.append(sts[r][a:b])
            org_p.append(sorg[r][a:b])
            loc = ssrc[r][a:b]                                 # shard-local L / R index -> global
            src_p.append(np.where(loc >= 0, s["l_sel"][np.maximum(loc, 0)],
                                  -s["r_sel"][np.maximum(-loc - 1, 0)] - 1))
        a, b = int(f_off[p]), int(f_off[p + 1])
        np.testing.assert_array_equal(np.concatenate(ts_p), f_ts[a:b])
        np.testing.assert_array_equal(np.concatenate(org_p), f_org[a:b])
        np.testing.assert_array_equal(np.concatenate(src_p), f_src[a:b])
    for k in ("st_kind", "st_str", "st_sum"):
        f = full[k].cpu().numpy()
        g = state[k].cpu().numpy()
        kind = full["st_kind"].cpu().numpy()
        if k == "st_kind":
            np.testing.assert_array_equal(g, f)
        elif k == "st_str":
            np.testing.assert_array_equal(g[kind == 1], f[kind == 1])
        else:
            np.testing.assert_array_equal(g[kind == 2], f[kind == 2])


def test_sharded_refmerge_single_rank_is_plain_merge(eng):
    from crdt_amd import shard
    h = synth.refmerge_packed(5, 16, 2000)
    d = refmerge.to_device(h, eng.device)
    full = eng.refmerge_batch(d)
    assert_batch_matches_oracle(h, full)
    got = shard.sharded_refmerge(eng, d)
    for k in ("off", "ts", "origin", "src", "st_kind"):
        n = int(full["off"][-1]) if k in ("ts", "origin", "src") else None
        np.testing.assert_array_equal(got[k].cpu().numpy()[:n], full[k].cpu().numpy()[:n])
    kind = full["st_kind"].cpu().numpy()
    np.testing.assert_array_equal(got["st_str"].cpu().numpy()[kind == 1], full["st_str"].cpu().numpy()[kind == 1])
    np.testing.assert_array_equal(got["st_sum"].cpu().numpy()[kind == 2], full["st_sum"].cpu().numpy()[kind == 2])
