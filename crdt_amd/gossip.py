"""Anti-entropy rounds on the GPU.

The reference runs one gossip goroutine per Server (main.go:226-261): every
round it picks a random friend, GETs its /gossip (the friend's whole Diff,
main.go:159), decodes it into RemoteDiff (every pulled entry becomes a remote
map, main.go:245-256) and merges (main.go:257).  Here a population of
replicas lives in HBM in the crdt_refmerge_in layout and a whole round runs
as device passes:

  1. RemoteDiff of replica p := the Diff segment of its peer q -- per-replica
     segmented copies (crdt_seg_copy2): q's ts and kv offsets (re-based by
     one per-replica delta), then q's kv pairs with the key slots re-based
     from q's slot range to p's;
  2. the bit-exact merge of every replica at once (crdt_refmerge_batch);
  3. the next Diff := the merge's new Diff, its kv offsets scanned and kv
     pairs gathered by `src` from the L / R arena in one pass
     (crdt_seg_gather2 with the merge's own +/- coding).

Rounds are synchronous (every replica pulls the Diffs as of the round's
start), one legal schedule of the reference's asynchronous goroutines.
Across GPUs (one process per GPU, replicas partitioned by contiguous
ranges) each rank all-gathers the population's Diffs once per round over
RCCL and pulls any peer from that import block.

Key slots: local replica i's key k is slot i*K + k (K keys per replica).
"""
from __future__ import annotations

import ctypes as C
from typing import Dict, List, Sequence

import numpy as np
import torch
import torch.distributed as dist

from . import shard
from .engine import Engine


def _p(t: torch.Tensor | None):
    return None if t is None else t.data_ptr()


class Population:
    """P replicas' Diffs (this rank's block of a population) on one GPU."""

    def __init__(self, eng: Engine, host: dict, keys_per_replica: int, first: int = 0):
        """host: numpy arrays {replicas, l_off, l_ts, l_origin, l_kv, kv_key
        (local slot ids), kv_val, str_bytes, str_off}; `first` = global id of
        local replica 0."""
        self.eng, self.K, self.first = eng, int(keys_per_replica), int(first)
        self.P = int(host["replicas"])
        dev = eng.device
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(dev)
        self.off = t(host["l_off"], np.int64)
        self.ts = t(host["l_ts"], np.int64)
        self.origin = t(host["l_origin"], np.uint8)
        self.kv_off = t(host["l_kv"], np.int64)
        kk = np.asarray(host["kv_key"]).view(np.uint32).view(np.int32)
        kvv = np.asarray(host["kv_val"]).view(np.uint32).view(np.int32)
        # the kv pairs live at the front of an arena with room for a round's pulled pairs
        cap = 2 * max(len(kk), 1)
        ak = torch.empty(cap, dtype=torch.int32, device=dev)
        av = torch.empty(cap, dtype=torch.int32, device=dev)
        ak[: len(kk)].copy_(t(kk, np.int32))
        av[: len(kvv)].copy_(t(kvv, np.int32))
        self.kv_key, self.kv_val = ak[: len(kk)], av[: len(kvv)]
        self.str_bytes = t(host["str_bytes"], np.uint8)
        self.str_off = t(host["str_off"], np.int64)
        self.state = None
        # kv arena of the next round: the current Diff's kv pairs are its
        # prefix (written there by the last round's gather), spare capacity
        # behind them takes the pulled pairs -- no copy of the Diff's pairs
        self._arena = (ak, av)

    def snapshot(self) -> tuple:
        """The population's Diffs (device views; a round never writes them)."""
        return (self.off, self.ts, self.origin, self.kv_off, self.kv_key, self.kv_val, self._arena)

    def restore(self, snap: tuple) -> None:
        (self.off, self.ts, self.origin, self.kv_off, self.kv_key, self.kv_val, self._arena) = snap

    # ---------------------------------------------------------------- helpers
    def _call(self, fn, *args):
        self.eng._call(fn, *args)

    def _seg_offsets(self, codes, a_off, b_off, base=0):
        out = torch.empty(codes.numel() + 1, dtype=torch.int64, device=self.eng.device)
        self._call("crdt_seg_offsets", codes.numel(), _p(codes), _p(a_off), _p(b_off), int(base), _p(out))
        return out

    def _seg_copy(self, codes, a_off, b_off, dst_off, a, b, n_out, delta=None, wide=0):
        dst = torch.empty(max(int(n_out), 1), dtype=a.dtype, device=self.eng.device)
        self._call("crdt_seg_copy", codes.numel(), _p(codes), _p(a_off), _p(b_off), _p(dst_off), a.element_size(),
                   _p(a), _p(b), _p(dst), _p(delta), wide)
        return dst[: int(n_out)]

    def _counts(self, off):
        c = torch.empty(max(off.numel() - 1, 1), dtype=torch.int32, device=self.eng.device)
        self._call("crdt_offsets_to_counts", _p(off), off.numel() - 1, _p(c))
        return c[: off.numel() - 1]

    def _offsets(self, counts, base=0):
        o = torch.empty(counts.numel() + 1, dtype=torch.int64, device=self.eng.device)
        self._call("crdt_counts_to_offsets", _p(counts), counts.numel(), int(base), _p(o))
        return o

    def _iota(self, n, negative=False):
        a = torch.arange(n, dtype=torch.int64, device=self.eng.device)
        return -(a + 1) if negative else a

    # ---------------------------------------------------------------- exchange
    def export_block(self) -> List[torch.Tensor]:
        """This rank's Diffs as the 5 flat arrays an import block is built
        from: entries per replica, ts, kv pairs per entry, kv keys, values."""
        return [self._counts(self.off), self.ts, self._counts(self.kv_off), self.kv_key, self.kv_val]

    def import_from_blocks(self, blocks: Sequence[List[torch.Tensor]]) -> dict:
        """Concatenate every rank's exported block (rank order = global
        replica order) into one import block (the 'B' source of a round)."""
        cat = [torch.cat([b[i] for b in blocks]) for i in range(5)]
        return self._make_import(*cat)

    def gather_import(self, group=None) -> dict:
        """All-gather the population's Diffs (one all-gather-v per array)."""
        blk = self.export_block()
        return self._make_import(*[shard.allgather_v(x, group) for x in blk])

    def _make_import(self, ecnt, ts, kvcnt, kkey, kval) -> dict:
        return {"off": self._offsets(ecnt.contiguous()), "ts": ts.contiguous(),
                "kv_off": self._offsets(kvcnt.contiguous()), "kv_key": kkey.contiguous(),
                "kv_val": kval.contiguous()}

    # ---------------------------------------------------------------- rounds
    def round(self, peers: Sequence[int], imp: dict | None = None, peer_first: Sequence[int] | None = None) -> dict:
        """One pull round: local replica i pulls the Diff of global replica
        peers[i] and merges.  imp = None: every peer is local (this rank);
        else peers index the import block (global ids) and peer_first[i] is
        the global id of the first replica on the peer's rank (for the slot
        re-basing).  Returns the merge output (new-Diff ranges and state)."""
        eng, dev, K = self.eng, self.eng.device, self.K
        peers = np.asarray(peers, dtype=np.int64)
        assert len(peers) == self.P
        if imp is None:
            lq = peers - self.first
            assert np.all((lq >= 0) & (lq < self.P)), "peer not on this rank: pass an import block"
            codes_np = lq
            b = {"off": None, "ts": None, "kv_off": None, "kv_key": None, "kv_val": None}
        else:
            codes_np = -(peers + 1)
            b = imp
            lq = peers - np.asarray(peer_first if peer_first is not None else np.zeros_like(peers), dtype=np.int64)
        # the slot re-basing of each pulled pair: (i - local index of q) * K, mod 2^32
        delta_np = ((np.arange(self.P, dtype=np.int64) - lq) * K) % (1 << 32)
        codes = torch.from_numpy(codes_np.copy()).to(dev)
        delta = torch.from_numpy(delta_np.astype(np.uint32).view(np.int32)).to(dev)

        # 1. RemoteDiff: entries, then their kv pairs behind the Diff's kv pairs in one arena.
        # A pulled Diff is one contiguous entry range and one contiguous kv range of its
        # source, so every copy is per replica: R's kv offsets are the source's offsets
        # plus a per-replica delta (no per-entry scan).
        a_kr = self.kv_off[self.off]                       # kv range of each local replica's Diff
        b_kr = b["kv_off"][b["off"]] if imp is not None else None
        r_off = self._seg_offsets(codes, self.off, b["off"])
        n_lkv = self.kv_key.numel()
        r_kb = self._seg_offsets(codes, a_kr, b_kr, base=n_lkv)   # where each replica's pulled kv pairs go
        n_r, n_kv_end = (int(x) for x in torch.stack([r_off[-1], r_kb[-1]]).cpu())
        n_rkv = n_kv_end - n_lkv
        n_b = b["ts"].numel() if b["ts"] is not None else 0
        src_kr = a_kr[codes.clamp(min=0)] if imp is None else b_kr[(-codes - 1).clamp(min=0)]
        kdelta = r_kb[:-1] - src_kr
        r_kv = torch.empty(n_r + 1, dtype=torch.int64, device=dev)
        r_ts = torch.empty(n_r, dtype=torch.int64, device=dev)
        r_kv[n_r:].copy_(r_kb[-1:])
        arena_k, arena_v = self._kv_arena(n_lkv, n_rkv)   # the Diff's pairs are already its prefix
        if n_r:
            bo = b["kv_off"] if n_b else self.kv_off
            bt = b["ts"] if n_b else self.ts
            self._call("crdt_seg_copy2", self.P, _p(codes), _p(self.off), _p(b["off"]), _p(r_off), 8,
                       _p(self.kv_off), _p(bo), _p(r_kv), _p(kdelta), _p(self.ts), _p(bt), _p(r_ts), 1)
            bk = b["kv_key"] if n_b else self.kv_key
            bv = b["kv_val"] if n_b else self.kv_val
            self._call("crdt_seg_copy2", self.P, _p(codes), _p(a_kr), _p(b_kr), _p(r_kb), 4,
                       _p(self.kv_key), _p(bk), _p(arena_k), _p(delta), _p(self.kv_val), _p(bv), _p(arena_v), 1)
        return self._merge_round(r_off, r_ts, r_kv, arena_k, arena_v, n_lkv, n_rkv)

    def _kv_arena(self, n_lkv: int, n_more: int):
        """A kv arena whose prefix is the Diff's pairs, with room for n_more."""
        ar = self._arena
        if (ar is not None and ar[0].numel() >= n_lkv + n_more and n_lkv > 0
                and ar[0].data_ptr() == self.kv_key.data_ptr() and ar[1].data_ptr() == self.kv_val.data_ptr()):
            return ar
        dev = self.eng.device
        arena_k = torch.empty(max(n_lkv + n_more, 1), dtype=torch.int32, device=dev)
        arena_v = torch.empty_like(arena_k)
        arena_k[:n_lkv].copy_(self.kv_key)
        arena_v[:n_lkv].copy_(self.kv_val)
        return arena_k, arena_v

    def round_wire(self, data: torch.Tensor, body_off: Sequence[int], keys, vals, n_entries: int,
                   n_pairs: int) -> dict:
        """One pull round whose pulls arrive on the wire: body i (bytes
        data[body_off[i]:body_off[i+1]] in HBM, the binary form of a peer's
        Diff.ToJSON, main.go:159) is replica i's RemoteDiff.  The device
        decode (crdt_gossip_decode, main.go:245-256) interns keys into `keys`
        (key id k -> slot i*K + k) and values into `vals`, whose arena becomes
        the population's string arena; then the batched merge and the next
        Diffs as in round().  n_entries / n_pairs: totals of the bodies'
        headers (codec.body_counts)."""
        from . import codec
        n_lkv = self.kv_key.numel()
        arena_k, arena_v = self._kv_arena(n_lkv, n_pairs)
        dec, st = codec.decode(self.eng, data, body_off, [i * self.K for i in range(self.P)], self.K, keys, vals,
                               n_lkv, arena_k, arena_v, n_entries)
        if st.any():
            raise ValueError(f"bodies not taken by the device decode (status {st[st != 0][:8].tolist()}): "
                             "decode those on the host")
        self.str_bytes, self.str_off = vals.arena()
        return self._merge_round(dec["r_off"], dec["r_ts"], dec["r_kv"], arena_k, arena_v, n_lkv, n_pairs)

    def _merge_round(self, r_off, r_ts, r_kv, arena_k, arena_v, n_lkv: int, n_rkv: int) -> dict:
        eng, dev, K = self.eng, self.eng.device, self.K
        # 2. the merge of every local replica
        packed = {"replicas": self.P, "n_slots": self.P * K, "l_off": self.off, "l_ts": self.ts,
                  "l_origin": self.origin, "l_kv": self.kv_off, "r_off": r_off, "r_ts": r_ts, "r_kv": r_kv,
                  "kv_key": arena_k[: n_lkv + n_rkv], "kv_val": arena_v[: n_lkv + n_rkv],
                  "str_bytes": self.str_bytes, "str_off": self.str_off}
        out = eng.refmerge_batch(packed)
        # 3. the next Diff: entries from the merge, kv pairs gathered by src
        n_out = int(out["off"][-1].item())
        src = out["src"][:n_out].contiguous()
        # offsets and kv gather in one pass; the arena size bounds the new Diff's kv count
        # into fresh buffers with room behind the pairs for the next round's pulled pairs
        # (a pull round moves about one population's worth of pairs; short capacity
        # falls back to a copy into a new arena)
        new_kv = torch.empty(n_out + 1, dtype=torch.int64, device=dev)
        cap = 2 * max(n_lkv + n_rkv, 1)
        nk = torch.empty(cap, dtype=torch.int32, device=dev)
        nv = torch.empty(cap, dtype=torch.int32, device=dev)
        self._call("crdt_seg_gather2", n_out, _p(src), _p(self.kv_off), _p(r_kv), 0, _p(new_kv), 4, _p(arena_k),
                   _p(arena_k), _p(nk), _p(arena_v), _p(arena_v), _p(nv))
        n_kv = int(new_kv[-1].item())
        self.kv_key, self.kv_val = nk[:n_kv], nv[:n_kv]
        self._arena = (nk, nv)
        self.kv_off = new_kv
        self.off = out["off"]
        self.ts = out["ts"][:n_out]
        self.origin = out["origin"][:n_out]
        self.state = {k: out[k] for k in ("st_kind", "st_str", "st_sum")}
        return out

    def append_local(self, host_new: dict) -> None:
        """Local writes (AddCommand's Diff.Put of a *Command, main.go:187)
        appended after each replica's Diff: host_new = {off (P+1), ts,
        kv_off, kv_key (local slot ids), kv_val}; every new ts must exceed
        its replica's current last ts."""
        dev = self.eng.device
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(dev)
        b_off, b_ts = t(host_new["off"], np.int64), t(host_new["ts"], np.int64)
        b_kv = t(host_new["kv_off"], np.int64)
        b_key = t(np.asarray(host_new["kv_key"]).astype(np.uint32).view(np.int32), np.int32)
        b_val = t(np.asarray(host_new["kv_val"]).astype(np.uint32).view(np.int32), np.int32)
        n_b = b_ts.numel()
        codes_np = np.empty(2 * self.P, np.int64)
        codes_np[0::2] = np.arange(self.P)
        codes_np[1::2] = -(np.arange(self.P) + 1)
        codes = torch.from_numpy(codes_np).to(dev)
        d_off = self._seg_offsets(codes, self.off, b_off)
        n = int(d_off[-1].item())
        ecodes = self._seg_copy(codes, self.off, b_off, d_off, self._iota(self.ts.numel()),
                                self._iota(max(n_b, 1), True), n, wide=1)
        ts = self._seg_copy(codes, self.off, b_off, d_off, self.ts, b_ts, n, wide=1)
        org = self._seg_copy(codes, self.off, b_off, d_off, self.origin,
                             torch.ones(max(n_b, 1), dtype=torch.uint8, device=dev), n, wide=1)
        kv = self._seg_offsets(ecodes, self.kv_off, b_kv)
        m = int(kv[-1].item())
        self.kv_key = self._seg_copy(ecodes, self.kv_off, b_kv, kv, self.kv_key, b_key, m)
        self.kv_val = self._seg_copy(ecodes, self.kv_off, b_kv, kv, self.kv_val, b_val, m)
        self.kv_off, self.ts, self.origin = kv, ts, org
        self.off = d_off[0::2].contiguous()

    def empty_state(self) -> dict:
        """CurrentState with every key slot absent (NewServer with an empty
        initialState, main.go:102-105)."""
        n = max(self.P * self.K, 1)
        dev = self.eng.device
        return {"st_kind": torch.zeros(n, dtype=torch.uint8, device=dev),
                "st_str": torch.zeros(n, dtype=torch.int32, device=dev),
                "st_sum": torch.zeros(n, dtype=torch.int64, device=dev)}

    def apply_local(self, host_cmds: dict) -> np.ndarray:
        """POST /data on every replica at once (AddCommand, main.go:173-215;
        crdt_local_apply): host_cmds = {off (P+1), ts, kv_off, kv_key (local
        slot ids), kv_val}, commands in arrival order per replica, pairs in
        apply order.  The Diffs get the *Command entries (a same-ms write
        replaces, main.go:187), CurrentState the local apply; returns the
        HTTP status of each command (200 / 500)."""
        dev = self.eng.device
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(dev)
        cmds = {"off": t(host_cmds["off"], np.int64), "ts": t(host_cmds["ts"], np.int64),
                "kv_off": t(host_cmds["kv_off"], np.int64),
                "kv_key": t(np.asarray(host_cmds["kv_key"]).astype(np.uint32).view(np.int32), np.int32),
                "kv_val": t(np.asarray(host_cmds["kv_val"]).astype(np.uint32).view(np.int32), np.int32)}
        if self.state is None:
            self.state = self.empty_state()
        out = self.eng.local_apply({"off": self.off, "ts": self.ts, "origin": self.origin}, cmds, self.state,
                                   self.str_bytes, self.str_off, self.P * self.K)
        n_out = int(out["off"][-1].item())
        src = out["src"][:n_out].contiguous()
        new_kv = torch.empty(n_out + 1, dtype=torch.int64, device=dev)
        cap = 2 * max(self.kv_key.numel() + cmds["kv_key"].numel(), 1)
        nk = torch.empty(cap, dtype=torch.int32, device=dev)
        nv = torch.empty(cap, dtype=torch.int32, device=dev)
        # the Diff's kv pairs: from the old Diff (src >= 0) or the command (src < 0); command
        # slots are local slot ids re-based to the replica's range by the caller's layout
        self._call("crdt_seg_gather2", n_out, _p(src), _p(self.kv_off), _p(cmds["kv_off"]), 0, _p(new_kv), 4,
                   _p(self.kv_key), _p(cmds["kv_key"]), _p(nk), _p(self.kv_val), _p(cmds["kv_val"]), _p(nv))
        n_kv = int(new_kv[-1].item())
        self.kv_key, self.kv_val = nk[:n_kv], nv[:n_kv]
        self._arena = (nk, nv)
        self.kv_off = new_kv
        self.off = out["off"]
        self.ts = out["ts"][:n_out]
        self.origin = out["origin"][:n_out]
        return out["status"][: cmds["ts"].numel()].cpu().numpy().astype(np.int64)

    # ---------------------------------------------------------------- readback
    def to_host(self) -> dict:
        g = lambda x: x.cpu().numpy()
        return {"off": g(self.off), "ts": g(self.ts), "origin": g(self.origin), "kv_off": g(self.kv_off),
                "kv_key": g(self.kv_key).view(np.uint32), "kv_val": g(self.kv_val).view(np.uint32)}


def random_peers(rng: np.random.Generator, total: int, first: int, count: int) -> np.ndarray:
    """A random peer other than itself for each of replicas [first, first+count).

    The reference draws uniformly from friendList (main.go:230), which is
    ports 8080..8089 (main.go:219-222): that list holds the server itself
    and ports no server listens on (the demo starts 8080..8084,
    main.go:319-321), so some of its rounds fail the request and skip
    (main.go:234-237: no merge) and some pull its own Diff.  A self-pull
    inserts nothing (every key equal, the local entry kept, main.go:54-65)
    but merge() still runs (main.go:257) and rebuilds CurrentState from the
    remote-origin entries (main.go:76), dropping what local writes applied
    to it directly (main.go:188-207) -- the same rebuild every merge ends
    with.  This schedule draws uniformly over the OTHER live replicas only:
    the Diffs it reaches are the reference's, and its CurrentState is the
    rebuild after each round's merge; it never produces the reference's
    merge-without-new-data rounds, so per-round pull rates differ."""
    r = rng.integers(0, total - 1, size=total)
    ids = np.arange(total)
    peers = np.where(r >= ids, r + 1, r)
    return peers[first:first + count]


def sharded_round(pop: Population, peers_all: np.ndarray, group=None) -> dict:
    """One round across the ranks of `group`: every rank all-gathers the
    population's Diffs, then pulls its replicas' peers from that block."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return pop.round(peers_all[pop.first:pop.first + pop.P])
    P_all = len(peers_all)
    firsts = [shard.shard_range(P_all, world, r)[0] for r in range(world)]
    owner_first = np.array([max(f for f in firsts if f <= q) for q in range(P_all)], dtype=np.int64)
    imp = pop.gather_import(group)
    mine = peers_all[pop.first:pop.first + pop.P]
    return pop.round(mine, imp=imp, peer_first=owner_first[mine])
