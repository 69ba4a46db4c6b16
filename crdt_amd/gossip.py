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
ranges) each rank fetches only the Diffs its replicas pull, by one
all-to-all-v per array (sharded_round), and merges from that import block.

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

LOCAL_MAX_CMD = 4096        # crdt_local_apply: commands per replica per call (its LDS sort)


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
        self.kv_fused = True                  # new Diff's kv pairs from the merge's tile pass
        self.pull_inplace = True              # local rounds: the merge reads the peers' Diffs in place
        # per-replica entry / kv-pair counts of the Diffs on the host: a round
        # sizes the pulled arrays from them (no host round trip up front) and
        # refreshes them in its one read-back at the end; None = unknown (after
        # a local write), the round then reads the sizes back first
        l_off = np.asarray(host["l_off"], dtype=np.int64)
        l_kv = np.asarray(host["l_kv"], dtype=np.int64)
        self._cnt = np.diff(l_off)
        self._kvcnt = np.diff(l_kv[l_off])
        # the fast path rebuilds entry / kv offsets as cumulative sums from 0
        if (len(l_off) and l_off[0] != 0) or (len(l_kv) and len(l_off) and l_kv[l_off[0]] != 0):
            self._cnt = self._kvcnt = None
        self._pin = None                                   # pinned staging of a round's per-replica arrays
        # kv arena of the next round: the current Diff's kv pairs are its
        # prefix (written there by the last round's gather), spare capacity
        # behind them takes the pulled pairs -- no copy of the Diff's pairs
        self._arena = (ak, av)

    def snapshot(self) -> tuple:
        """The population's Diffs (device views; a round never writes them)."""
        return (self.off, self.ts, self.origin, self.kv_off, self.kv_key, self.kv_val, self._arena, self._cnt,
                self._kvcnt)

    def restore(self, snap: tuple) -> None:
        (self.off, self.ts, self.origin, self.kv_off, self.kv_key, self.kv_val, self._arena, self._cnt,
         self._kvcnt) = snap

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
    def round(self, peers: Sequence[int], imp: dict | None = None, peer_first: Sequence[int] | None = None,
              peer_index: Sequence[int] | None = None) -> dict:
        """One pull round: local replica i pulls the Diff of global replica
        peers[i] and merges (main.go:230-257).  peers[i] == the replica itself
        is a self-pull (merge() still runs and rebuilds CurrentState,
        main.go:76); peers[i] < 0 is a dead peer: the request fails and the
        replica skips the round -- no merge, Diff and CurrentState unchanged
        (main.go:234-239).  imp = None: every peer is on this rank; else the
        pulled Diffs come from the import block: peer_index[i] (default
        peers[i]) is the peer's replica in the block and peer_first[i] the
        global id of the first replica on the peer's rank (for the slot
        re-basing).  Returns the merge output (new-Diff ranges and state)."""
        eng, dev, K = self.eng, self.eng.device, self.K
        peers = np.asarray(peers, dtype=np.int64)
        assert len(peers) == self.P
        skip = peers < 0
        if imp is None and self._cnt is not None and not skip.any():
            return self._round_local(peers - self.first)
        if imp is None:
            lq = np.where(skip, np.arange(self.P) + self.first, peers) - self.first
            assert np.all((lq >= 0) & (lq < self.P)), "peer not on this rank: pass an import block"
            codes_np = lq.copy()
            b = {"off": None, "ts": None, "kv_off": None, "kv_key": None, "kv_val": None}
        else:
            idx = np.asarray(peer_index if peer_index is not None else peers, dtype=np.int64)
            codes_np = -(idx + 1)
            b = imp
            pf = np.asarray(peer_first if peer_first is not None else np.zeros_like(peers), dtype=np.int64)
            lq = np.where(skip, np.arange(self.P), peers - pf)
        if skip.any():
            # a skipped replica "pulls" an empty segment appended to the B block
            if b["off"] is None:
                z = torch.zeros(2, dtype=torch.int64, device=dev)
                e = torch.zeros(0, dtype=torch.int64, device=dev)
                e32 = torch.zeros(0, dtype=torch.int32, device=dev)
                b = {"off": z, "ts": e, "kv_off": z[:1], "kv_key": e32, "kv_val": e32}
            else:
                b = dict(b, off=torch.cat([b["off"], b["off"][-1:]]))
            codes_np[skip] = -(b["off"].numel() - 1)       # B's last (empty) segment
            prev_state = self.state if self.state is not None else self.empty_state()
            prev_state = {k: v.clone() for k, v in prev_state.items()}
        # the slot re-basing of each pulled pair: (i - local index of q) * K, mod 2^32
        delta_np = ((np.arange(self.P, dtype=np.int64) - lq) * K) % (1 << 32)
        codes = torch.from_numpy(codes_np.copy()).to(dev)
        delta = torch.from_numpy(delta_np.astype(np.uint32).view(np.int32)).to(dev)

        # 1. RemoteDiff: entries, then their kv pairs behind the Diff's kv pairs in one arena.
        # A pulled Diff is one contiguous entry range and one contiguous kv range of its
        # source, so every copy is per replica: R's kv offsets are the source's offsets
        # plus a per-replica delta (no per-entry scan).
        a_kr = self.kv_off[self.off]                       # kv range of each local replica's Diff
        b_kr = b["kv_off"][b["off"]] if b["off"] is not None else None
        r_off = self._seg_offsets(codes, self.off, b["off"])
        n_lkv = self.kv_key.numel()
        r_kb = self._seg_offsets(codes, a_kr, b_kr, base=n_lkv)   # where each replica's pulled kv pairs go
        if imp is None and self._cnt is not None:          # sizes from the host counts: no read-back
            pull = np.where(skip, 0, 1)
            n_r = int((self._cnt[lq] * pull).sum())
            n_rkv = int((self._kvcnt[lq] * pull).sum())
        else:
            n_r, n_kv_end = (int(x) for x in torch.stack([r_off[-1], r_kb[-1]]).cpu())
            n_rkv = n_kv_end - n_lkv
        n_b = b["ts"].numel() if b["ts"] is not None else 0
        src_kr = torch.where(codes >= 0, a_kr[codes.clamp(min=0)],
                             b_kr[(-codes - 1).clamp(min=0)] if b_kr is not None else a_kr[0])
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
        out = self._merge_round(r_off, r_ts, r_kv, arena_k, arena_v, n_lkv, n_rkv)
        if skip.any():                                     # no merge ran for these: CurrentState as it was
            sl = torch.from_numpy((np.flatnonzero(skip)[:, None] * K + np.arange(K)[None, :]).reshape(-1)).to(dev)
            for k in ("st_kind", "st_str", "st_sum"):
                self.state[k][sl] = prev_state[k][sl]
        return out

    def _round_local(self, lq: np.ndarray) -> dict:
        """round() when every peer is on this rank, none is dead, and the
        per-replica counts are on the host: the per-replica arrays of the
        pull assembly (source codes, R entry and kv offsets, kv re-basing
        deltas, slot deltas) are computed on the host and uploaded in one
        pinned asynchronous copy -- no scans or index kernels on the device,
        no host round trip before the merge."""
        P, K, dev = self.P, self.K, self.eng.device
        assert np.all((lq >= 0) & (lq < P)), "peer not on this rank: pass an import block"
        n_lkv = self.kv_key.numel()
        cnt, kvc = self._cnt[lq], self._kvcnt[lq]
        n_r, n_rkv = int(cnt.sum()), int(kvc.sum())
        if self.pull_inplace and self.kv_fused:             # (the gather by src cannot re-base slots)
            # every replica's RemoteDiff is its peer's Diff where it lies in
            # HBM: the merge reads R ranges (r_off, r_end) of the population's
            # own arrays and re-bases the pulled key slots (r_slot_delta), so
            # nothing is assembled.  int64 fields: r_off P | r_end P | delta (int32, P)
            n64 = 2 * P + (P + 1) // 2
            if self._pin is None or self._pin.numel() < n64:
                self._pin = torch.empty(n64, dtype=torch.int64).pin_memory()
            h = self._pin.numpy()
            l_off = np.zeros(P + 1, np.int64)
            np.cumsum(self._cnt, out=l_off[1:])
            h[:P] = l_off[lq]
            h[P:2 * P] = l_off[lq + 1]
            h[2 * P:n64].view(np.int32)[:P] = (((np.arange(P, dtype=np.int64) - lq) * K) % (1 << 32)).astype(
                np.uint32).view(np.int32)
            d = self._pin[:n64].to(dev, non_blocking=True)
            pull = {"r_end": d[P:2 * P], "r_slot_delta": d[2 * P:].view(torch.int32)[:P]}
            return self._merge_round(d[:P], self.ts, self.kv_off, self.kv_key, self.kv_val, n_lkv, 0,
                                     pull=pull, n_r=n_r, n_pull_kv=n_rkv)
        # int64 fields: codes P | a_kr P+1 | r_off P+1 | r_kb P+1 | kdelta P | delta (int32, P)
        n64 = 5 * P + 3 + (P + 1) // 2
        if self._pin is None or self._pin.numel() < n64:
            self._pin = torch.empty(n64, dtype=torch.int64).pin_memory()
        h = self._pin.numpy()
        h[:P] = lq
        a_kr = h[P:2 * P + 1]
        a_kr[0] = 0
        np.cumsum(self._kvcnt, out=a_kr[1:])
        r_off = h[2 * P + 1:3 * P + 2]
        r_off[0] = 0
        np.cumsum(cnt, out=r_off[1:])
        r_kb = h[3 * P + 2:4 * P + 3]
        r_kb[0] = n_lkv
        np.cumsum(kvc, out=r_kb[1:])
        r_kb[1:] += n_lkv
        h[4 * P + 3:5 * P + 3] = r_kb[:-1] - a_kr[lq]
        h[5 * P + 3:].view(np.int32)[:P] = (((np.arange(P, dtype=np.int64) - lq) * K) % (1 << 32)).astype(
            np.uint32).view(np.int32)
        d = self._pin[:n64].to(dev, non_blocking=True)
        codes, a_kr_d, r_off_d, r_kb_d = d[:P], d[P:2 * P + 1], d[2 * P + 1:3 * P + 2], d[3 * P + 2:4 * P + 3]
        kdelta = d[4 * P + 3:5 * P + 3]
        delta = d[5 * P + 3:].view(torch.int32)[:P]
        r_kv = torch.empty(n_r + 1, dtype=torch.int64, device=dev)
        r_ts = torch.empty(n_r, dtype=torch.int64, device=dev)
        r_kv[n_r:].copy_(r_kb_d[-1:])
        arena_k, arena_v = self._kv_arena(n_lkv, n_rkv)
        if n_r:
            self._call("crdt_seg_copy2", P, _p(codes), _p(self.off), None, _p(r_off_d), 8,
                       _p(self.kv_off), None, _p(r_kv), _p(kdelta), _p(self.ts), None, _p(r_ts), 1)
            self._call("crdt_seg_copy2", P, _p(codes), _p(a_kr_d), None, _p(r_kb_d), 4,
                       _p(self.kv_key), None, _p(arena_k), _p(delta), _p(self.kv_val), None, _p(arena_v), 1)
        return self._merge_round(r_off_d, r_ts, r_kv, arena_k, arena_v, n_lkv, n_rkv)

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

    def _merge_round(self, r_off, r_ts, r_kv, arena_k, arena_v, n_lkv: int, n_rkv: int, pull: dict | None = None,
                     n_r: int | None = None, n_pull_kv: int = 0) -> dict:
        """pull: in-place R ranges (crdt_refmerge_batch_pull; r_ts / r_kv /
        the arena are the population's own arrays, n_r the total of the
        ranges, n_pull_kv their kv pairs)."""
        eng, dev, K = self.eng, self.eng.device, self.K
        # 2. the merge of every local replica
        packed = {"replicas": self.P, "n_slots": self.P * K, "l_off": self.off, "l_ts": self.ts,
                  "l_origin": self.origin, "l_kv": self.kv_off, "r_off": r_off, "r_ts": r_ts, "r_kv": r_kv,
                  "kv_key": arena_k[: n_lkv + n_rkv], "kv_val": arena_v[: n_lkv + n_rkv],
                  "str_bytes": self.str_bytes, "str_off": self.str_off}
        if n_r is not None:
            packed["n_r"] = n_r
        n_rkv += n_pull_kv
        # 3. the next Diff: entries from the merge, kv pairs copied by the
        # merge's own tile pass (crdt_refmerge_batch_kv; kv_fused = False:
        # a segmented gather by src after the merge, crdt_seg_gather2_n).
        # The entry count stays on the device; the arrays are sized for its
        # upper bound |L| + |R|; ONE read-back at the end brings the new
        # Diffs' entry and kv offsets per replica (the next round's sizes).
        # The fresh kv arena has room behind the pairs for the next round's
        # pulled pairs.
        n_max = self.ts.numel() + (r_ts.numel() if n_r is None else n_r)
        new_kv = torch.empty(n_max + 1, dtype=torch.int64, device=dev)
        cap = 2 * max(n_lkv + n_rkv, 1)
        nk = torch.empty(cap, dtype=torch.int32, device=dev)
        nv = torch.empty(cap, dtype=torch.int32, device=dev)
        if self.kv_fused:
            out = eng.refmerge_batch(packed, kv={"off": new_kv, "key": nk, "val": nv}, pull=pull)
        else:
            out = eng.refmerge_batch(packed, pull=pull)
            self._call("crdt_seg_gather2_n", n_max, _p(out["off"][self.P:]), _p(out["src"]), _p(self.kv_off),
                       _p(r_kv), _p(new_kv), _p(arena_k), _p(arena_k), _p(nk), _p(arena_v), _p(arena_v), _p(nv))
        ho = torch.cat([out["off"], new_kv[out["off"]]]).cpu().numpy()
        n_out, n_kv = int(ho[self.P]), int(ho[-1])
        self._cnt, self._kvcnt = np.diff(ho[: self.P + 1]), np.diff(ho[self.P + 1:])
        new_kv = new_kv[: n_out + 1]
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
        self._cnt = self._kvcnt = None

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
        HTTP status of each command (200 / 500).  More than LOCAL_MAX_CMD
        commands for one replica run as several device calls, each taking the
        next LOCAL_MAX_CMD of every replica's commands in arrival order."""
        off = np.asarray(host_cmds["off"], dtype=np.int64)
        cnt = np.diff(off)
        if cnt.size == 0 or int(cnt.max()) <= LOCAL_MAX_CMD:
            return self._apply_local_once(host_cmds)
        kv_off = np.asarray(host_cmds["kv_off"], dtype=np.int64)
        ts = np.asarray(host_cmds["ts"], dtype=np.int64)
        kk, kv = np.asarray(host_cmds["kv_key"]), np.asarray(host_cmds["kv_val"])
        status = np.zeros(int(off[-1]), dtype=np.int64)
        for r in range(-(-int(cnt.max()) // LOCAL_MAX_CMD)):
            lo = np.minimum(off[:-1] + r * LOCAL_MAX_CMD, off[1:])
            hi = np.minimum(lo + LOCAL_MAX_CMD, off[1:])
            idx = np.concatenate([np.arange(a, b) for a, b in zip(lo, hi)]).astype(np.int64)
            sub_off = np.concatenate([[0], np.cumsum(hi - lo)])
            pcnt = kv_off[idx + 1] - kv_off[idx]
            pidx = np.concatenate([np.arange(kv_off[j], kv_off[j + 1]) for j in idx] or [np.zeros(0, np.int64)])
            pidx = pidx.astype(np.int64)
            sub = {"off": sub_off, "ts": ts[idx], "kv_off": np.concatenate([[0], np.cumsum(pcnt)]),
                   "kv_key": kk[pidx], "kv_val": kv[pidx]}
            status[idx] = self._apply_local_once(sub)
        return status

    def _apply_local_once(self, host_cmds: dict) -> np.ndarray:
        dev = self.eng.device
        t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a).astype(dt)).to(dev)
        cmds = {"off": t(host_cmds["off"], np.int64), "ts": t(host_cmds["ts"], np.int64),
                "kv_off": t(host_cmds["kv_off"], np.int64),
                "kv_key": t(np.asarray(host_cmds["kv_key"]).astype(np.uint32).view(np.int32), np.int32),
                "kv_val": t(np.asarray(host_cmds["kv_val"]).astype(np.uint32).view(np.int32), np.int32)}
        # the apply updates CurrentState in place: run it on a copy and commit
        # the copy only after the device status is clean, so a raised flag
        # leaves CurrentState and the Diffs of the population consistent
        state = {k: v.clone() for k, v in (self.state or self.empty_state()).items()}
        out = self.eng.local_apply({"off": self.off, "ts": self.ts, "origin": self.origin}, cmds, state,
                                   self.str_bytes, self.str_off, self.P * self.K)
        self.eng.check_device()        # CRDT_DEV_RANGE: nothing of an over-limit replica was applied
        self.state = state
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
        self._cnt = self._kvcnt = None
        return out["status"][: cmds["ts"].numel()].cpu().numpy().astype(np.int64)

    # ---------------------------------------------------------------- readback
    def to_host(self) -> dict:
        g = lambda x: x.cpu().numpy()
        return {"off": g(self.off), "ts": g(self.ts), "origin": g(self.origin), "kv_off": g(self.kv_off),
                "kv_key": g(self.kv_key).view(np.uint32), "kv_val": g(self.kv_val).view(np.uint32)}


def random_peers(rng: np.random.Generator, total: int, first: int, count: int) -> np.ndarray:
    """A random peer other than itself for each of replicas [first, first+count).

    A schedule that only pulls live peers: every round of every replica
    reaches new data.  reference_peers draws like the reference instead."""
    r = rng.integers(0, total - 1, size=total)
    ids = np.arange(total)
    peers = np.where(r >= ids, r + 1, r)
    return peers[first:first + count]


def reference_peers(rng: np.random.Generator, total: int, first: int, count: int,
                    dead: int | None = None) -> np.ndarray:
    """The reference's draw (main.go:230): uniform over friendList, which
    holds EVERY replica -- the server itself included -- and ports no server
    listens on (main.go:219-222: 8080..8089 against the 8080..8084 the demo
    starts, main.go:319-321; `dead` defaults to `total`, the same ratio).  A
    dead pick is -1: the request fails and the round is skipped (main.go:234-
    239, Population.round leaves that replica alone); a self pick is a
    self-pull, whose merge() inserts nothing and rebuilds CurrentState
    (main.go:76)."""
    dead = total if dead is None else dead
    r = rng.integers(0, total + dead, size=total)
    peers = np.where(r < total, r, -1)
    return peers[first:first + count]


def pull_plan(peers_all: np.ndarray, world: int) -> tuple:
    """Who pulls what in a round over `world` ranks (replicas partitioned by
    contiguous ranges, shard.shard_range): firsts[r] = rank r's first global
    replica (firsts[world] = total) and need[r] = the sorted distinct live
    peers rank r's replicas pull.  Every rank derives the same plan from the
    round's draw (no exchange)."""
    total = len(peers_all)
    firsts = [shard.shard_range(total, world, r)[0] for r in range(world)] + [total]
    need = []
    for r in range(world):
        mine = np.asarray(peers_all[firsts[r]:firsts[r + 1]], dtype=np.int64)
        need.append(np.unique(mine[mine >= 0]))
    return firsts, need


def sharded_round(pop: Population, peers_all: np.ndarray, group=None, comm=None) -> dict:
    """One round across the ranks of `group` (main.go:226-258 over xGMI):
    every rank fetches ONLY the Diffs its replicas pull -- rank p sends rank
    r the Diffs of the replicas p owns among need[r] (pull_plan), as one
    all-to-all-v per array (the native RCCL communicator `comm`'s
    crdt_shard_alltoallv when given, else torch.distributed) -- then the
    round merges as on one GPU.  peers_all: every replica's draw (global
    ids, -1 = dead peer), identical on every rank."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    if world == 1:
        return pop.round(peers_all[pop.first:pop.first + pop.P])
    rank = dist.get_rank(group)
    dev = pop.eng.device
    firsts, need = pull_plan(peers_all, world)
    f0, f1 = firsts[rank], firsts[rank + 1]
    # what this rank sends: for each destination r, the replicas of need[r] it owns
    send_ids = [need[r][(need[r] >= f0) & (need[r] < f1)] - f0 for r in range(world)]
    n_rep = [len(x) for x in send_ids]
    codes = torch.from_numpy(np.concatenate(send_ids).astype(np.int64)).to(dev)
    ecnt = pop._counts(pop.off)
    kvcnt = pop._counts(pop.kv_off)
    a_kr = pop.kv_off[pop.off]
    e_off = pop._seg_offsets(codes, pop.off, None)
    k_off = pop._seg_offsets(codes, a_kr, None)
    cut = np.concatenate([[0], np.cumsum(n_rep)]).astype(np.int64)
    eb, kb = (x[torch.from_numpy(cut).to(dev)].cpu().numpy() for x in (e_off, k_off))
    n_e, n_k = int(eb[-1]), int(kb[-1])
    s_ecnt = ecnt[codes] if codes.numel() else ecnt[:0]
    s_ts = pop._seg_copy(codes, pop.off, None, e_off, pop.ts, None, n_e, wide=1) if n_e else pop.ts[:0]
    s_kvcnt = pop._seg_copy(codes, pop.off, None, e_off, kvcnt, None, n_e, wide=1) if n_e else kvcnt[:0]
    s_key = pop._seg_copy(codes, a_kr, None, k_off, pop.kv_key, None, n_k) if n_k else pop.kv_key[:0]
    s_val = pop._seg_copy(codes, a_kr, None, k_off, pop.kv_val, None, n_k) if n_k else pop.kv_val[:0]
    # per-destination entry / pair counts, all-gathered (replica counts follow from the plan)
    se = np.diff(eb).tolist()
    sk = np.diff(kb).tolist()
    # (device tensors: the collective runs on NCCL / RCCL as well as gloo)
    mat = [torch.zeros(2 * world, dtype=torch.int64, device=dev) for _ in range(world)]
    dist.all_gather(mat, torch.tensor(se + sk, dtype=torch.int64, device=dev), group=group)
    mat = torch.stack(mat).cpu().numpy()
    r_rep = [int(((need[rank] >= firsts[p]) & (need[rank] < firsts[p + 1])).sum()) for p in range(world)]
    r_e, r_k = mat[:, rank].tolist(), mat[:, world + rank].tolist()

    def xchg(t, s_counts, r_counts):
        if comm is not None:
            out = torch.empty(max(sum(r_counts), 1), dtype=t.dtype, device=dev)
            src = t if t.numel() else torch.empty(1, dtype=t.dtype, device=dev)
            torch.cuda.synchronize(dev)
            comm.alltoallv([src], [s_counts], [out], [r_counts], t.element_size())
            comm.sync()
            return out[:sum(r_counts)]
        return shard.alltoallv(t, s_counts, r_counts, group)

    imp = pop._make_import(xchg(s_ecnt, n_rep, r_rep), xchg(s_ts, se, r_e), xchg(s_kvcnt, se, r_e),
                           xchg(s_key, sk, r_k), xchg(s_val, sk, r_k))
    mine = np.asarray(peers_all[pop.first:pop.first + pop.P], dtype=np.int64)
    live = mine >= 0
    idx = np.where(live, np.searchsorted(need[rank], np.maximum(mine, 0)), -1)
    owner = np.searchsorted(np.asarray(firsts), np.maximum(mine, 0), side="right") - 1
    pf = np.where(live, np.asarray(firsts)[owner], 0)
    return pop.round(mine, imp=imp, peer_first=pf, peer_index=idx)


# ---------------------------------------------------------------- the C-ABI population
class NativePopulation:
    """A replica population whose anti-entropy rounds run entirely behind the
    C-ABI (crdt_population_*, csrc/population.hip) -- what a cgo host of the
    gossip loop (main.go:226-261) binds.  Same rounds as :class:`Population`
    (in-place pulls, kv pairs from the merge's passes, dead peers skipped),
    with the per-replica planning in C++.

    * ``NativePopulation(eng, host, K, first)``: on an Engine's context;
    * ``NativePopulation.on_member(comm, i, host, K, first)``: on member i of
      a shard.Comm, for :meth:`round_sharded`.
    ``host``: the Population host arrays (replicas, l_off, l_ts, l_origin,
    l_kv, kv_key as local slot ids, kv_val, str_bytes, str_off)."""

    def __init__(self, eng, host: dict, keys_per_replica: int, first: int = 0, _ctx=None, _owner=None):
        from ._lib import crdt_population_init
        self._owner = eng if eng is not None else _owner
        ctx = eng.ctx if eng is not None else _ctx
        if eng is not None:
            eng._bind()
        self.K, self.first = int(keys_per_replica), int(first)
        self.P = int(host["replicas"])
        a = lambda x, dt: np.ascontiguousarray(np.asarray(x).astype(dt) if np.asarray(x).dtype != dt
                                               else np.asarray(x))
        self._keep = [a(host["l_off"], np.uint64), a(host["l_ts"], np.int64), a(host["l_origin"], np.uint8),
                      a(host["l_kv"], np.uint64), a(np.asarray(host["kv_key"]).view(np.uint32), np.uint32),
                      a(np.asarray(host["kv_val"]).view(np.uint32), np.uint32), a(host["str_bytes"], np.uint8),
                      a(host["str_off"], np.uint64)]
        ptr = lambda x: x.ctypes.data if x.size else None
        ini = crdt_population_init(self.P, self.K, self.first, len(self._keep[7]) - 1,
                                   *[ptr(x) for x in self._keep])
        h = C.c_void_p()
        from . import _lib
        _lib.call("crdt_population_create", ctx, C.byref(ini), C.byref(h), ctx=ctx)
        self._h = h
        self._ctx = ctx
        if eng is not None:
            eng._depend(self)                  # eng.close() destroys the population first

    @classmethod
    def on_member(cls, comm, member: int, host: dict, keys_per_replica: int, first: int):
        from . import _lib
        ctx = C.c_void_p()
        _lib.call("crdt_shard_member_ctx", comm._h, member, C.byref(ctx))
        pop = cls(None, host, keys_per_replica, first, _ctx=ctx, _owner=comm)
        comm._depend(pop)                      # (the member context dies with the communicator)
        return pop

    def close(self) -> None:
        from . import _lib
        if getattr(self, "_h", None):
            _lib.lib().crdt_population_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def round(self, peers) -> None:
        """One round, every peer on this population (global ids, -1 = dead)."""
        from . import _lib
        pk = np.ascontiguousarray(np.asarray(peers, dtype=np.int64))
        assert len(pk) == self.P
        if hasattr(self._owner, "_bind"):
            self._owner._bind()
        _lib.call("crdt_population_round", self._h, pk.ctypes.data, ctx=self._ctx)

    def sizes(self):
        """(replicas, Diff entries, kv pairs) of the current Diffs."""
        from . import _lib
        P, n_e, n_kv = C.c_uint32(), C.c_size_t(), C.c_size_t()
        _lib.call("crdt_population_info", self._h, C.byref(P), C.byref(n_e), C.byref(n_kv))
        return P.value, n_e.value, n_kv.value

    def add_commands(self, host_cmds: dict) -> np.ndarray:
        """POST /data on every replica at once (AddCommand, main.go:173-215;
        crdt_population_add_commands): host_cmds = {off (P+1), ts, kv_off,
        kv_key (local slot ids), kv_val}, commands in arrival order per
        replica.  Returns every command's HTTP status (200 / 500)."""
        from . import _lib
        from ._lib import crdt_population_cmds
        a = lambda x, dt: np.ascontiguousarray(np.asarray(x).astype(dt))
        keep = [a(host_cmds["off"], np.uint64), a(host_cmds["ts"], np.int64), a(host_cmds["kv_off"], np.uint64),
                a(np.asarray(host_cmds["kv_key"]).astype(np.uint32), np.uint32),
                a(np.asarray(host_cmds["kv_val"]).astype(np.uint32), np.uint32)]
        ptr = lambda x: x.ctypes.data if x.size else None
        cmds = crdt_population_cmds(*[ptr(x) for x in keep])
        status = np.zeros(max(len(keep[1]), 1), np.uint16)
        _lib.call("crdt_population_add_commands", self._h, C.byref(cmds), status.ctypes.data, ctx=self._ctx)
        return status[:len(keep[1])].astype(np.int64)

    def round_wire(self, data, body_off, keys, vals) -> None:
        """One round whose pulls arrive on the wire (crdt_population_round_wire):
        body i = data[body_off[i]:body_off[i+1]] (a device uint8 tensor) is
        replica i's pulled Diff in the binary gossip form, an empty body a
        failed GET.  keys / vals: codec.StrTab of the key ids (< K) and value
        ids (vals must hold this population's strings at their ids).
        Raises CrdtError (CRDT_E_UNSORTED) with .body_status when a body is
        not taken by the device decode; nothing is merged then."""
        from . import _lib
        bo = np.ascontiguousarray(np.asarray(body_off, dtype=np.uint64))
        assert len(bo) == self.P + 1
        st = np.zeros(max(self.P, 1), np.uint32)
        if hasattr(self._owner, "_bind"):
            self._owner._bind()
        self._vtab = vals                      # (the population borrows its arena from now on)
        try:
            _lib.call("crdt_population_round_wire", self._h, keys._h, vals._h, data.data_ptr() if data.numel() else None,
                      bo.ctypes.data, st.ctypes.data, ctx=self._ctx)
        except _lib.CrdtError as err:
            err.body_status = st[:self.P].copy()
            raise

    def undo(self) -> None:
        """Back to the Diffs and CurrentState before the last round."""
        from . import _lib
        _lib.call("crdt_population_undo", self._h, ctx=self._ctx)

    @staticmethod
    def round_sharded(comm, pops, peers_all) -> None:
        """One round over the communicator: pops[i] = member i's population."""
        from . import _lib
        pk = np.ascontiguousarray(np.asarray(peers_all, dtype=np.int64))
        arr = (C.c_void_p * len(pops))(*[p._h.value for p in pops])
        comm._call("crdt_population_round_sharded", arr, pk.ctypes.data, len(pk))

    def read(self) -> dict:
        """The Diffs (Population.to_host layout) and CurrentState, on the host."""
        from . import _lib
        P, n_e, n_kv = C.c_uint32(), C.c_size_t(), C.c_size_t()
        _lib.call("crdt_population_info", self._h, C.byref(P), C.byref(n_e), C.byref(n_kv))
        ns = self.P * self.K
        out = {"off": np.empty(self.P + 1, np.uint64), "ts": np.empty(n_e.value, np.int64),
               "origin": np.empty(n_e.value, np.uint8), "kv_off": np.empty(n_e.value + 1, np.uint64),
               "kv_key": np.empty(n_kv.value, np.uint32), "kv_val": np.empty(n_kv.value, np.uint32),
               "st_kind": np.empty(ns, np.uint8), "st_str": np.empty(ns, np.uint32), "st_sum": np.empty(ns, np.int64)}
        ptr = lambda x: x.ctypes.data if x.size else None
        _lib.call("crdt_population_read", self._h, *[ptr(out[k]) for k in
                                                      ("off", "ts", "origin", "kv_off", "kv_key", "kv_val",
                                                       "st_kind", "st_str", "st_sum")], ctx=self._ctx)
        return out
