"""Batched bit-exact (*Server).merge() -- host side.

Packs many replicas' `Diff` / `RemoteDiff` treemaps (main.go:26-27) into the
CSR structure-of-arrays layout of `crdt_refmerge_in` (include/crdt_amd.h),
runs ONE device call for the whole batch, and unpacks the new Diff and the
rebuilt CurrentState of every replica.

Reference data model, mirrored with Python types:
  * `Data` / `Command` are `map[string]string` (main.go:19-21).  A Diff value
    that is a :class:`Command` is a local write (`*Command`, main.go:187):
    the replay skips it (main.go:80).  Any other dict is a remote map
    (main.go:245-255).
  * Keys are int64 Unix-millisecond timestamps ordered by the signed
    Int64Comparator (main.go:106-107).
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

INT64_MIN, INT64_MAX = -(2**63), 2**63 - 1


class Command(dict):
    """`type Command map[string]string` (main.go:21): a local write."""


Data = dict  # `type Data map[string]string` (main.go:19)


def _check_ts(ts):
    if not isinstance(ts, (int, np.integer)) or not (INT64_MIN <= int(ts) <= INT64_MAX):
        # the reference comparator panics on non-int64 keys (main.go:106)
        raise TypeError(f"Diff keys must be int64 timestamps, got {ts!r}")


class Packer:
    """Interns strings and builds the CSR arrays for a batch of replicas."""

    def __init__(self):
        self.strings: List[bytes] = []
        self._sid: Dict[bytes, int] = {}
        self.slot_names: List[str] = []          # slot id -> key string
        self.slot_off: List[int] = [0]           # replica -> slot range
        self.l_ts: List[int] = []
        self.l_origin: List[int] = []
        self.l_vals: List[object] = []
        self.l_kv: List[int] = [0]
        self.l_off: List[int] = [0]
        self.r_ts: List[int] = []
        self.r_vals: List[object] = []
        self.r_kv: List[int] = [0]
        self.r_off: List[int] = [0]
        self.kv_key: List[int] = []
        self.kv_val: List[int] = []
        self._l_kv_items: List[Tuple[int, int]] = []

    def _str(self, s: str) -> int:
        b = s.encode("utf-8", "surrogatepass")
        i = self._sid.get(b)
        if i is None:
            i = self._sid[b] = len(self.strings)
            self.strings.append(b)
        return i

    def add_replica(self, diff: dict, remote: dict) -> None:
        base = len(self.slot_names)
        local: Dict[str, int] = {}

        def slot(k: str) -> int:
            s = local.get(k)
            if s is None:
                s = local[k] = base + len(local)
                self.slot_names.append(k)
            return s

        # kv arena order: every L entry's pairs, then every R entry's pairs
        # (per replica); the L/R kv offset arrays index one shared arena.
        l_pairs, r_pairs = [], []
        for ts in sorted(diff):
            _check_ts(ts)
            v = diff[ts]
            self.l_ts.append(int(ts))
            self.l_origin.append(1 if isinstance(v, Command) else 0)
            self.l_vals.append(v)
            l_pairs.append([(slot(k), self._str(x)) for k, x in v.items()])
        for ts in sorted(remote):
            _check_ts(ts)
            v = remote[ts]
            self.r_ts.append(int(ts))
            self.r_vals.append(v)
            r_pairs.append([(slot(k), self._str(x)) for k, x in v.items()])
        self._pending = getattr(self, "_pending", [])
        self._pending.append((l_pairs, r_pairs))
        self.l_off.append(len(self.l_ts))
        self.r_off.append(len(self.r_ts))
        self.slot_off.append(len(self.slot_names))

    def arrays(self) -> dict:
        """numpy arrays of the packed batch (host)."""
        kv_key, kv_val = [], []
        l_kv, r_kv = [], []
        for l_pairs, _ in getattr(self, "_pending", []):
            for pairs in l_pairs:
                l_kv.append(len(kv_key))
                for s, v in pairs:
                    kv_key.append(s)
                    kv_val.append(v)
        l_kv.append(len(kv_key))
        for _, r_pairs in getattr(self, "_pending", []):
            for pairs in r_pairs:
                r_kv.append(len(kv_key))
                for s, v in pairs:
                    kv_key.append(s)
                    kv_val.append(v)
        r_kv.append(len(kv_key))
        blob = b"".join(self.strings)
        str_off = np.zeros(len(self.strings) + 1, dtype=np.int64)
        if self.strings:
            str_off[1:] = np.cumsum([len(s) for s in self.strings])
        if len(self.slot_names) >= 2**32 or len(self.strings) >= 2**32:
            raise OverflowError("more than 2^32 key slots or strings in one batch")
        return {
            "replicas": len(self.l_off) - 1,
            "n_slots": len(self.slot_names),
            "l_off": np.array(self.l_off, np.int64), "l_ts": np.array(self.l_ts, np.int64),
            "l_origin": np.array(self.l_origin, np.uint8), "l_kv": np.array(l_kv, np.int64),
            "r_off": np.array(self.r_off, np.int64), "r_ts": np.array(self.r_ts, np.int64),
            "r_kv": np.array(r_kv, np.int64),
            "kv_key": np.array(kv_key, np.uint32).view(np.int32), "kv_val": np.array(kv_val, np.uint32).view(np.int32),
            "str_bytes": np.frombuffer(blob if blob else b"\0", dtype=np.uint8).copy(),
            "str_off": str_off,
        }


def to_device(arrs: dict, device) -> dict:
    out = {}
    for k, v in arrs.items():
        if isinstance(v, np.ndarray):
            out[k] = torch.from_numpy(np.ascontiguousarray(v)).to(device)
        else:
            out[k] = v
    return out


def unpack_batch(pk: Packer, arrs: dict, out: dict):
    """Device outputs of a packed batch -> [(new_diff, current_state), ...]
    with the Diff values being the Packer's own value objects."""
    off = out["off"].cpu().numpy()
    n_out = int(off[-1])
    ts = out["ts"][:n_out].cpu().numpy()
    src = out["src"][:n_out].cpu().numpy()
    ns = arrs["n_slots"]
    kind = out["st_kind"][:ns].cpu().numpy()
    sstr = out["st_str"][:ns].cpu().numpy().view(np.uint32)
    ssum = out["st_sum"][:ns].cpu().numpy()
    results = []
    for p in range(arrs["replicas"]):
        new_diff = {}
        for o in range(int(off[p]), int(off[p + 1])):
            s = int(src[o])
            new_diff[int(ts[o])] = pk.l_vals[s] if s >= 0 else pk.r_vals[-s - 1]
        state = {}
        for slot in range(pk.slot_off[p], pk.slot_off[p + 1]):
            k = int(kind[slot])
            if k == 1:
                state[pk.slot_names[slot]] = pk.strings[int(sstr[slot])].decode("utf-8", "surrogatepass")
            elif k == 2:
                state[pk.slot_names[slot]] = str(int(ssum[slot]))        # strconv.Itoa (main.go:96)
        results.append((new_diff, state))
    return results


def merge_batch(eng, replicas: Sequence[Tuple[dict, dict]]):
    """Bit-exact (*Server).merge() of every (Diff, RemoteDiff) pair in ONE
    device call.  Returns [(new_diff, current_state), ...]."""
    pk = Packer()
    for diff, remote in replicas:
        pk.add_replica(diff, remote)
    arrs = pk.arrays()
    out = eng.refmerge_batch(to_device(arrs, eng.device))
    return unpack_batch(pk, arrs, out)
