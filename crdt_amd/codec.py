"""Device gossip decode over the C-ABI (csrc/codec.hip).

A pulled Diff travels as the binary SoA body of crdt_server_gossip_binary
(the wire form of Diff.ToJSON, main.go:159); crdt_gossip_decode turns a batch
of such bodies, already in HBM, into the RemoteDiff arrays of a batched merge
(main.go:245-256), interning keys and values into device string tables.
"""
from __future__ import annotations

import ctypes as C
import struct
from typing import List, Sequence

import numpy as np
import torch

from . import _lib
from ._lib import call

MAGIC = b"CRDTSOA1"
BODY_OK, BODY_MALFORMED, BODY_HOST, BODY_FULL = 0, 1, 2, 4


class RawBuf:
    """A device pointer that quacks like a tensor for the packers (data_ptr/numel)."""

    def __init__(self, ptr: int, n: int):
        self._p, self._n = int(ptr), int(n)

    def data_ptr(self) -> int:
        return self._p

    def numel(self) -> int:
        return self._n


class StrTab:
    """crdt_strtab: string -> dense id (first-seen order), device arena +
    host mirror."""

    def __init__(self, eng, cap_strings: int = 1024, cap_bytes: int = 1 << 16):
        self.eng = eng
        h = C.c_void_p()
        eng._bind()
        call("crdt_strtab_create", eng.ctx, cap_strings, cap_bytes, C.byref(h), ctx=eng.ctx)
        self._h = h
        eng._depend(self)

    def close(self) -> None:
        if getattr(self, "_h", None):
            _lib.lib().crdt_strtab_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        n, nb, b, o = C.c_uint64(), C.c_uint64(), C.c_void_p(), C.c_void_p()
        call("crdt_strtab_info", self._h, C.byref(n), C.byref(nb), C.byref(b), C.byref(o))
        return n.value, nb.value, b.value, o.value

    def __len__(self) -> int:
        return self.info()[0]

    def arena(self):
        """(str_bytes, str_off) as device buffers for crdt_refmerge_in."""
        n, nb, b, o = self.info()
        return RawBuf(b, max(nb, 1)), RawBuf(o, n + 1)

    def get(self, i: int) -> bytes:
        p, n = C.c_void_p(), C.c_size_t()
        call("crdt_strtab_get", self._h, i, C.byref(p), C.byref(n))
        return C.string_at(p.value, n.value) if n.value else b""

    def strings(self) -> List[bytes]:
        return [self.get(i) for i in range(len(self))]

    def intern(self, strs: Sequence[bytes]) -> np.ndarray:
        """Ids of the given strings (new ones appended)."""
        strs = [s if isinstance(s, bytes) else s.encode() for s in strs]
        off = np.zeros(len(strs) + 1, np.uint64)
        off[1:] = np.cumsum([len(s) for s in strs])
        blob = b"".join(strs) or b"\0"
        dev = torch.frombuffer(bytearray(blob), dtype=torch.uint8).to(self.eng.device)
        ids = torch.empty(max(len(strs), 1), dtype=torch.int32, device=self.eng.device)
        self.eng._bind()
        call("crdt_strtab_intern", self.eng.ctx, self._h, dev.data_ptr(), off.ctypes.data_as(C.c_void_p), len(strs),
             ids.data_ptr(), ctx=self.eng.ctx)
        return ids[: len(strs)].cpu().numpy().view(np.uint32)


def body_counts(body: bytes):
    """(n_entries, n_pairs) from a binary body's header; (0, 0) if malformed."""
    if len(body) < 32 or body[:8] != MAGIC:
        return 0, 0
    ne, np_, nb = struct.unpack_from("<QQQ", body, 8)
    if 32 + 12 * ne + 8 * np_ + nb != len(body):
        return 0, 0
    return ne, np_


def decode(eng, data: torch.Tensor, body_off: Sequence[int], slot_base: Sequence[int], key_cap: int,
           keys: StrTab, vals: StrTab, kv_base: int, kv_key: torch.Tensor, kv_val: torch.Tensor, n_entries: int):
    """crdt_gossip_decode of the bodies data[body_off[b]:body_off[b+1]] (device
    uint8).  kv_key / kv_val (int32, capacity >= kv_base + pairs) receive the
    pairs.  Returns ({r_off, r_ts, r_kv}, body_status)."""
    nb = len(body_off) - 1
    dev = eng.device
    out = {"r_off": torch.empty(nb + 1, dtype=torch.int64, device=dev),
           "r_ts": torch.empty(max(n_entries, 1), dtype=torch.int64, device=dev),
           "r_kv": torch.empty(n_entries + 1, dtype=torch.int64, device=dev)}
    boff = (C.c_uint64 * (nb + 1))(*body_off)
    sbase = (C.c_uint32 * max(nb, 1))(*slot_base)
    gb = _lib.crdt_gossip_bodies(nb, key_cap, kv_base, data.data_ptr(), C.cast(boff, C.c_void_p),
                                 C.cast(sbase, C.c_void_p))
    go = _lib.crdt_gossip_decoded(out["r_off"].data_ptr(), out["r_ts"].data_ptr(), out["r_kv"].data_ptr(),
                                  kv_key.data_ptr(), kv_val.data_ptr())
    st = (C.c_uint32 * max(nb, 1))()
    eng._bind()
    call("crdt_gossip_decode", eng.ctx, C.byref(gb), keys._h, vals._h, C.byref(go), st, ctx=eng.ctx)
    out["r_ts"] = out["r_ts"][:n_entries]
    return out, np.array(st[:nb], dtype=np.uint32)


def encode_packed_diffs(h: dict, key_names: Sequence[bytes], slots_per_replica: int):
    """Binary gossip bodies (crdt_server_gossip_binary's format) of every
    replica's Diff in a packed batch (crdt_amd.synth.refmerge_packed layout:
    one kv per entry, key slot p * slots_per_replica + k -> key_names[k]),
    vectorised.  Returns (blob, offsets) with body p = blob[off[p]:off[p+1]]."""
    P = h["replicas"]
    l_off = np.asarray(h["l_off"], np.int64)
    ts = np.asarray(h["l_ts"], np.int64)
    kv_key = np.asarray(h["kv_key"]).view(np.uint32).astype(np.int64)[: len(ts)]
    kv_val = np.asarray(h["kv_val"]).view(np.uint32).astype(np.int64)[: len(ts)]
    if not np.array_equal(np.asarray(h["l_kv"], np.int64), np.arange(len(ts) + 1)):
        raise ValueError("one kv per entry expected")
    sb = np.asarray(h["str_bytes"], np.uint8)
    so = np.asarray(h["str_off"], np.int64)
    names = [bytes(k) for k in key_names]
    if any(len(k) != 1 for k in names):
        raise ValueError("single-byte key names expected (the reference's alphabet, main.go:274)")
    kbyte = np.frombuffer(b"".join(names), np.uint8)
    rep = np.repeat(np.arange(P, dtype=np.int64), np.diff(l_off))
    kidx = kv_key - rep * slots_per_replica
    vlen = (so[kv_val + 1] - so[kv_val]).astype(np.int64)
    rec = 1 + vlen                                        # key byte + value bytes per entry
    rec_off = np.zeros(len(ts) + 1, np.int64)
    rec_off[1:] = np.cumsum(rec)
    data = np.empty(int(rec_off[-1]), np.uint8)
    data[rec_off[:-1]] = kbyte[kidx]
    # value bytes: for byte t of entry e, source so[v_e] + t, destination rec_off[e] + 1 + t
    e_of = np.repeat(np.arange(len(ts)), vlen)
    within = np.arange(int(vlen.sum())) - np.repeat(np.cumsum(vlen) - vlen, vlen)
    data[rec_off[e_of] + 1 + within] = sb[so[kv_val[e_of]] + within]
    bodies = []
    for p in range(P):
        a, b = int(l_off[p]), int(l_off[p + 1])
        ne = b - a
        nby = int(rec_off[b] - rec_off[a])
        hdr = MAGIC + struct.pack("<QQQ", ne, ne, nby)
        bodies.append(hdr + ts[a:b].astype("<i8").tobytes() + np.ones(ne, "<u4").tobytes() +
                      np.ones(ne, "<u4").tobytes() + vlen[a:b].astype("<u4").tobytes() +
                      data[rec_off[a]:rec_off[b]].tobytes())
    off = np.zeros(P + 1, np.int64)
    off[1:] = np.cumsum([len(x) for x in bodies])
    return b"".join(bodies), off
