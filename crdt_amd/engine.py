"""Device-level host API over the C-ABI (include/crdt_amd.h).

PyTorch is plumbing here: it owns device memory (tensors in HBM) and the
stream; every merge/compare computation runs in libcrdt_amd.so's gfx950 HIP
kernels.  uint64 state is carried in int64 tensors (same bits); use
:func:`as_u64` to view a host copy as numpy uint64.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib
from ._lib import (call, crdt_local_in, crdt_local_out, crdt_refmerge_acc, crdt_refmerge_in, crdt_refmerge_kv_out,
                   crdt_refmerge_out, crdt_refmerge_pull, crdt_replay_state, crdt_tuples)

VC_EQUAL, VC_BEFORE, VC_AFTER, VC_CONCURRENT = 0, 1, 2, 3


def as_u64(t: torch.Tensor) -> np.ndarray:
    """Host numpy uint64 view of an 8-byte integer tensor (any device)."""
    return t.detach().cpu().contiguous().numpy().view(np.uint64)


def u64_tensor(a, device) -> torch.Tensor:
    """numpy uint64 (or int64) array -> int64 tensor with the same bits."""
    a = np.ascontiguousarray(a)
    if a.dtype != np.int64:
        a = a.view(np.int64) if a.dtype.itemsize == 8 else a.astype(np.int64)
    return torch.from_numpy(a.copy()).to(device)


def _ptr(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


@dataclass
class TupleSet:
    """SoA (key u64, ts u64, rep u32, tomb u8) tuples, sorted by (key, ts, rep)."""

    key: torch.Tensor   # int64 storage of uint64 keys
    ts: torch.Tensor    # int64 storage of uint64 timestamps
    rep: torch.Tensor   # int32 storage of uint32 replica ids
    tomb: torch.Tensor  # uint8 0/1

    def __len__(self) -> int:
        return int(self.key.numel())

    @staticmethod
    def empty(n: int, device) -> "TupleSet":
        return TupleSet(torch.empty(n, dtype=torch.int64, device=device),
                        torch.empty(n, dtype=torch.int64, device=device),
                        torch.empty(n, dtype=torch.int32, device=device),
                        torch.empty(n, dtype=torch.uint8, device=device))

    def c(self) -> crdt_tuples:
        return crdt_tuples(self.key.data_ptr(), self.ts.data_ptr(), self.rep.data_ptr(), self.tomb.data_ptr())

    def slice(self, n: int) -> "TupleSet":
        return TupleSet(self.key[:n], self.ts[:n], self.rep[:n], self.tomb[:n])

    def to_numpy(self):
        return (as_u64(self.key), as_u64(self.ts), self.rep.cpu().numpy().view(np.uint32),
                self.tomb.cpu().numpy())

    @staticmethod
    def from_numpy(key, ts, rep, tomb, device) -> "TupleSet":
        return TupleSet(u64_tensor(key, device), u64_tensor(ts, device),
                        torch.from_numpy(np.ascontiguousarray(rep).view(np.int32).copy()).to(device),
                        torch.from_numpy(np.ascontiguousarray(tomb).astype(np.uint8)).to(device))


class Engine:
    """One crdt_ctx bound to one GPU and to torch's current stream."""

    def __init__(self, device: int | torch.device = 0):
        if not torch.cuda.is_available():
            raise _lib.CrdtLibraryError("no GPU visible: the crdt_amd engine has no CPU path")
        self.device = torch.device("cuda", device if isinstance(device, int) else device.index or 0)
        lib = _lib.lib()
        self._stream = torch.cuda.current_stream(self.device).cuda_stream
        ctx = C.c_void_p()
        call("crdt_ctx_create", self.device.index, self._stream, C.byref(ctx))
        self.ctx = ctx
        self._lib = lib
        self._dependents = []              # weakrefs to objects borrowing ctx (shard.Comm)

    def _depend(self, obj) -> None:
        import weakref
        self._dependents.append(weakref.ref(obj))

    def close(self) -> None:
        for r in getattr(self, "_dependents", []):   # borrowers first: they use ctx in their teardown
            o = r()
            if o is not None:
                o.close()
        self._dependents = []
        if getattr(self, "ctx", None):
            self._lib.crdt_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _bind(self) -> None:
        s = torch.cuda.current_stream(self.device).cuda_stream
        if s != self._stream:
            call("crdt_ctx_set_stream", self.ctx, s, ctx=self.ctx)
            self._stream = s

    def _call(self, fn: str, *args) -> None:
        self._bind()
        call(fn, self.ctx, *args, ctx=self.ctx)

    def _check(self, *ts: torch.Tensor, itemsize: int | None = None) -> None:
        for t in ts:
            if t.device != self.device:
                raise ValueError(f"tensor on {t.device}, engine on {self.device}")
            if not t.is_contiguous():
                raise ValueError("tensors must be contiguous")
            if itemsize is not None and t.element_size() != itemsize:
                raise ValueError(f"expected {itemsize}-byte elements, got {t.dtype}")

    def sync(self) -> None:
        self._call("crdt_ctx_sync")

    def device_status(self, clear: bool = True) -> int:
        """Kernel-raised failure flags (CRDT_DEV_*) since the last clear; syncs."""
        v = C.c_uint32()
        self._call("crdt_ctx_device_status", C.byref(v), 1 if clear else 0)
        return v.value

    def check_device(self) -> None:
        """Raise if a kernel reported a device-side failure (its output is invalid)."""
        flags = self.device_status(clear=True)
        if flags:
            raise _lib.CrdtLibraryError(f"device-side failure flags 0x{flags:x} (CRDT_DEV_*): output invalid")

    def reserve(self, nbytes: int) -> None:
        self._call("crdt_ctx_reserve", nbytes)

    # ------------------------------------------------------------ counters (a6)
    def gcounter_join(self, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """out = max(a, b) elementwise (uint64); a, b: [rows, nodes]."""
        if a.shape != b.shape or a.dim() != 2:
            raise ValueError("a and b must be [rows, nodes] of equal shape")
        out = torch.empty_like(a) if out is None else out
        self._check(a, b, out, itemsize=8)
        if out.shape != a.shape:
            raise ValueError("out shape mismatch")
        self._call("crdt_gcounter_join", a.data_ptr(), b.data_ptr(), out.data_ptr(), a.shape[0], a.shape[1])
        return out

    vclock_join = gcounter_join

    def gcounter_fold(self, a: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """out[n] = max over rows of a[:, n]."""
        rows, nodes = a.shape
        out = torch.empty(nodes, dtype=torch.int64, device=self.device) if out is None else out
        self._check(a, out, itemsize=8)
        self._call("crdt_gcounter_fold", a.data_ptr(), rows, nodes, out.data_ptr())
        return out

    def stream_copy(self, src: torch.Tensor, dst: torch.Tensor, unroll: int = 4, blocks_per_cu: int = 2) -> None:
        """dst = src with the library's streaming copy kernel (peak measurement)."""
        self._check(src, dst)
        n = min(src.numel() * src.element_size(), dst.numel() * dst.element_size())
        self._call("crdt_stream_copy", src.data_ptr(), dst.data_ptr(), n & ~15, unroll, blocks_per_cu)

    def stream_read(self, src: torch.Tensor, sink: torch.Tensor, unroll: int = 4, blocks_per_cu: int = 2) -> None:
        """Read all of src (one word per workgroup to sink): read-only streaming peak."""
        self._check(src)
        self._check(sink, itemsize=8)
        n = src.numel() * src.element_size()
        self._call("crdt_stream_read", src.data_ptr(), n & ~15, sink.data_ptr(), sink.numel(), unroll, blocks_per_cu)

    def gcounter_value(self, a: torch.Tensor) -> torch.Tensor:
        rows, nodes = a.shape
        out = torch.empty(rows, dtype=torch.int64, device=self.device)
        self._check(a, out, itemsize=8)
        self._call("crdt_gcounter_value", a.data_ptr(), rows, nodes, out.data_ptr())
        return out

    def pncounter_join(self, pa, na, pb, nb, pout=None, nout=None):
        pout = torch.empty_like(pa) if pout is None else pout
        nout = torch.empty_like(na) if nout is None else nout
        for t in (na, pb, nb, pout, nout):
            if t.shape != pa.shape:
                raise ValueError("PN-Counter operands must share one [rows, nodes] shape")
        self._check(pa, na, pb, nb, pout, nout, itemsize=8)
        rows, nodes = pa.shape
        self._call("crdt_pncounter_join", pa.data_ptr(), na.data_ptr(), pb.data_ptr(), nb.data_ptr(),
                   pout.data_ptr(), nout.data_ptr(), rows, nodes)
        return pout, nout

    def pncounter_value(self, p: torch.Tensor, n: torch.Tensor) -> torch.Tensor:
        if p.shape != n.shape:
            raise ValueError("P and N must share one shape")
        rows, nodes = p.shape
        out = torch.empty(rows, dtype=torch.int64, device=self.device)
        self._check(p, n, out, itemsize=8)
        self._call("crdt_pncounter_value", p.data_ptr(), n.data_ptr(), out.data_ptr(), rows, nodes)
        return out

    # ------------------------------------------------------------ vector clocks (a7)
    def vclock_classify(self, a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        if a.shape != b.shape or a.dim() != 2:
            raise ValueError("a and b must be [pairs, nodes] of equal shape")
        pairs, nodes = a.shape
        out = torch.empty(pairs, dtype=torch.uint8, device=self.device) if out is None else out
        self._check(a, b, itemsize=8)
        self._check(out, itemsize=1)
        self._call("crdt_vclock_classify", a.data_ptr(), b.data_ptr(), out.data_ptr(), pairs, nodes)
        return out

    # ------------------------------------------------------------ sets (a8)
    def _set_merge(self, fn: str, a: TupleSet, b: TupleSet, out: TupleSet | None,
                   count: torch.Tensor | None, trim: bool):
        na, nb = len(a), len(b)
        out = TupleSet.empty(max(na + nb, 1), self.device) if out is None else out
        count = torch.empty(1, dtype=torch.int64, device=self.device) if count is None else count
        for s in (a, b, out):
            self._check(s.key, s.ts, itemsize=8)
            self._check(s.rep, itemsize=4)
            self._check(s.tomb, itemsize=1)
        ca, cb, co = a.c(), b.c(), out.c()
        self._call(fn, C.byref(ca), na, C.byref(cb), nb, C.byref(co), count.data_ptr())
        if trim:                              # synchronises anyway: check the look-back's flag too
            self.check_device()
            return out.slice(int(count.item()))
        return out, count

    def lww_merge(self, a: TupleSet, b: TupleSet, out: TupleSet | None = None,
                  count: torch.Tensor | None = None, trim: bool = True):
        """LWW-Element-Set merge; a is the local (tie-winning) operand."""
        return self._set_merge("crdt_lww_merge", a, b, out, count, trim)

    def orset_merge(self, a: TupleSet, b: TupleSet, out: TupleSet | None = None,
                    count: torch.Tensor | None = None, trim: bool = True):
        """OR-Set merge: union of tags, tombstones OR-ed."""
        return self._set_merge("crdt_orset_merge", a, b, out, count, trim)

    def lww_merge_unsorted(self, a: TupleSet, b: TupleSet, out: TupleSet | None = None,
                           count: torch.Tensor | None = None, trim: bool = True):
        """LWW merge of UNSORTED sides (D2): one fused device sort + dedup;
        equal to sort_tuples of each side followed by lww_merge."""
        return self._set_merge("crdt_lww_merge_unsorted", a, b, out, count, trim)

    def orset_merge_unsorted(self, a: TupleSet, b: TupleSet, out: TupleSet | None = None,
                             count: torch.Tensor | None = None, trim: bool = True):
        """OR-Set merge of UNSORTED sides (D2): one fused device sort + dedup."""
        return self._set_merge("crdt_orset_merge_unsorted", a, b, out, count, trim)

    def set_merge_plan(self, lww: bool, a: TupleSet, b: TupleSet, widen: bool = False):
        """crdt_set_merge_plan: the exact plan of a D2 merge of this shape
        (one synchronisation); reserves the workspace its planned calls use."""
        from ._lib import crdt_set_plan
        plan = crdt_set_plan()
        ca, cb = a.c(), b.c()
        self._call("crdt_set_merge_plan", 0 if lww else 1, C.byref(ca), len(a), C.byref(cb), len(b),
                   1 if widen else 0, C.byref(plan))
        return plan

    def merge_unsorted_planned(self, lww: bool, plan, a: TupleSet, b: TupleSet, out: TupleSet,
                               count: torch.Tensor) -> None:
        """crdt_{lww,orset}_merge_unsorted_planned: the D2 merge enqueued with
        no host synchronisation (graph-capturable); *count = 2^64 - 1 and the
        CRDT_DEV_PLAN flag when the inputs left the plan."""
        for s in (a, b, out):
            self._check(s.key, s.ts, itemsize=8)
            self._check(s.rep, itemsize=4)
            self._check(s.tomb, itemsize=1)
        ca, cb, co = a.c(), b.c(), out.c()
        fn = "crdt_lww_merge_unsorted_planned" if lww else "crdt_orset_merge_unsorted_planned"
        self._call(fn, C.byref(plan), C.byref(ca), len(a), C.byref(cb), len(b), C.byref(co), count.data_ptr())

    def sort_tuples(self, t: TupleSet, out: TupleSet | None = None) -> TupleSet:
        """Device sort into ascending (key, ts, rep, tomb) order (config D2)."""
        n = len(t)
        out = TupleSet.empty(n, self.device) if out is None else out
        for s in (t, out):
            self._check(s.key, s.ts, itemsize=8)
            self._check(s.rep, itemsize=4)
            self._check(s.tomb, itemsize=1)
        ct, co = t.c(), out.c()
        self._call("crdt_tuples_sort", C.byref(ct), n, C.byref(co))
        return out

    def lower_bound_u64(self, sorted_u64: torch.Tensor, probes: torch.Tensor) -> torch.Tensor:
        """lower_bound of every probe in an ascending uint64 (int64-stored)
        device array, unsigned order (crdt_u64_lower_bound)."""
        self._check(sorted_u64, probes, itemsize=8)
        out = torch.empty(probes.numel(), dtype=torch.int64, device=self.device)
        self._call("crdt_u64_lower_bound", sorted_u64.data_ptr(), sorted_u64.numel(), probes.data_ptr(),
                   probes.numel(), out.data_ptr())
        return out

    def tuples_merge(self, a: TupleSet, b: TupleSet, out: TupleSet | None = None) -> TupleSet:
        """Stable merge of two sorted tuple arrays, every tuple kept (a's
        copies first on an equal tag): crdt_tuples_merge."""
        out = TupleSet.empty(max(len(a) + len(b), 1), self.device) if out is None else out
        for s in (a, b, out):
            self._check(s.key, s.ts, itemsize=8)
            self._check(s.rep, itemsize=4)
            self._check(s.tomb, itemsize=1)
        ca, cb, co = a.c(), b.c(), out.c()
        self._call("crdt_tuples_merge", C.byref(ca), len(a), C.byref(cb), len(b), C.byref(co))
        return out.slice(len(a) + len(b))

    def count_unsorted(self, t: TupleSet) -> int:
        bad = torch.empty(1, dtype=torch.int64, device=self.device)
        ct = t.c()
        self._call("crdt_tuples_count_unsorted", C.byref(ct), len(t), bad.data_ptr())
        return int(bad.item())

    # ------------------------------------------------------------ RefMerge (a1-a3)
    def _refmerge_in(self, d: dict) -> crdt_refmerge_in:
        return crdt_refmerge_in(
            d["replicas"], int(d["n_slots"]), d["l_ts"].numel(), int(d.get("n_r", d["r_ts"].numel())),
            d["kv_key"].numel(),
            d["str_off"].numel() - 1,
            _ptr(d["l_off"]), _ptr(d["l_ts"]), _ptr(d["l_origin"]), _ptr(d["l_kv"]),
            _ptr(d["r_off"]), _ptr(d["r_ts"]), _ptr(d["r_kv"]),
            _ptr(d["kv_key"]), _ptr(d["kv_val"]), _ptr(d["str_bytes"]), _ptr(d["str_off"]))

    def refmerge_batch(self, packed: dict, maxl: torch.Tensor | None = None,
                       acc: dict | None = None, _delta: dict | None = None, kv: dict | None = None,
                       pull: dict | None = None) -> dict:
        """Run the batched bit-exact reference merge on a packed batch.

        ``packed`` holds device tensors produced by
        :func:`crdt_amd.refmerge.pack_batch`; returns device output tensors.
        ``maxl`` / ``acc``: the ts-range-sharded form (crdt_refmerge_batch_ex;
        see :func:`crdt_amd.shard.sharded_refmerge`).
        ``kv`` = {"off": int64 [n_l + n_r + 1], "key", "val": int32 [cap]}:
        also the new Diff's kv pairs (crdt_refmerge_batch_kv): entry i owns
        key/val[off[i] .. off[i+1]), off[out["off"][-1]] = the total.
        ``pull`` = {"r_end": int64 [replicas], "r_slot_delta": int32
        [replicas] or None}: in-place pulls (crdt_refmerge_batch_pull) --
        replica p's R is r_ts[r_off[p] .. r_end[p]) (may alias L), and
        ``packed["n_r"]`` the total of the R ranges.
        """
        d = packed
        n_l, n_r = d["l_ts"].numel(), int(d.get("n_r", d["r_ts"].numel()))
        n_slots = int(d["n_slots"])
        dev = self.device
        out = {
            "off": torch.empty(d["replicas"] + 1, dtype=torch.int64, device=dev),
            "ts": torch.empty(max(n_l + n_r, 1), dtype=torch.int64, device=dev),
            "origin": torch.empty(max(n_l + n_r, 1), dtype=torch.uint8, device=dev),
            "src": torch.empty(max(n_l + n_r, 1), dtype=torch.int64, device=dev),
            "st_kind": torch.empty(max(n_slots, 1), dtype=torch.uint8, device=dev),
            "st_str": torch.empty(max(n_slots, 1), dtype=torch.int32, device=dev),
            "st_sum": torch.empty(max(n_slots, 1), dtype=torch.int64, device=dev),
        }
        cin = self._refmerge_in(d)
        cout = crdt_refmerge_out(*(out[k].data_ptr() for k in
                                   ("off", "ts", "origin", "src", "st_kind", "st_str", "st_sum")))
        if kv is not None:
            if _delta is not None or maxl is not None or acc is not None:
                raise ValueError("refmerge_batch: kv output only with the plain batch merge")
            self._check(kv["off"], itemsize=8)
            self._check(kv["key"], kv["val"], itemsize=4)
            if kv["off"].numel() < n_l + n_r + 1 or kv["val"].numel() < kv["key"].numel():
                raise ValueError("refmerge_batch: kv output too small")
            ckv = crdt_refmerge_kv_out(kv["off"].data_ptr(), kv["key"].data_ptr(), kv["val"].data_ptr(),
                                       kv["key"].numel())
        if pull is not None:
            if _delta is not None or maxl is not None or acc is not None:
                raise ValueError("refmerge_batch: in-place pulls only with the plain batch merge")
            self._check(pull["r_end"], itemsize=8)
            sd = pull.get("r_slot_delta")
            if sd is not None:
                self._check(sd, itemsize=4)
            cp = crdt_refmerge_pull(pull["r_end"].data_ptr(), sd.data_ptr() if sd is not None else None)
            self._call("crdt_refmerge_batch_pull", C.byref(cin), C.byref(cout), C.byref(cp),
                       C.byref(ckv) if kv is not None else None)
        elif kv is not None:
            self._call("crdt_refmerge_batch_kv", C.byref(cin), C.byref(cout), C.byref(ckv))
        elif _delta is not None:
            cs = self._rstate(_delta)
            self._call("crdt_refmerge_delta", C.byref(cin), C.byref(cout), C.byref(cs))
        elif maxl is None and acc is None:
            self._call("crdt_refmerge_batch", C.byref(cin), C.byref(cout))
        else:
            if maxl is not None:
                self._check(maxl, itemsize=8)
            cacc = self._acc(acc) if acc is not None else None
            self._call("crdt_refmerge_batch_ex", C.byref(cin), C.byref(cout),
                       maxl.data_ptr() if maxl is not None else None, C.byref(cacc) if cacc is not None else None)
        return out

    # -- incremental replay
    def replay_state_new(self, n_slots: int) -> dict:
        n = max(n_slots, 1)
        z = lambda dt: torch.zeros(n, dtype=dt, device=self.device)
        return {"best_key": z(torch.int64), "best_str": z(torch.int32), "sum": z(torch.int64),
                "npar": z(torch.int32), "nhold": z(torch.int32)}

    @staticmethod
    def _rstate(st: dict) -> crdt_replay_state:
        return crdt_replay_state(*(st[k].data_ptr() for k in ("best_key", "best_str", "sum", "npar", "nhold")))

    def replay_state_init(self, packed: dict, st: dict | None = None) -> dict:
        """Replay state of the batch's L logs (crdt_replay_state_init)."""
        st = self.replay_state_new(int(packed["n_slots"])) if st is None else st
        cin, cs = self._refmerge_in(packed), self._rstate(st)
        self._call("crdt_replay_state_init", C.byref(cin), C.byref(cs))
        return st

    def refmerge_delta(self, packed: dict, st: dict) -> dict:
        """crdt_refmerge_batch with the replay folded incrementally into
        ``st`` (the state of ``packed``'s L logs; updated in place)."""
        out = self.refmerge_batch(packed, _delta=st)
        return out

    # -- ts-range-sharded RefMerge steps
    def refmerge_acc_new(self, n_slots: int) -> dict:
        n = max(n_slots, 1)
        return {"best": torch.zeros(n, dtype=torch.int64, device=self.device),
                "sum": torch.zeros(n, dtype=torch.int64, device=self.device),
                "npar": torch.zeros(n, dtype=torch.int32, device=self.device)}

    @staticmethod
    def _acc(acc: dict) -> crdt_refmerge_acc:
        return crdt_refmerge_acc(acc["best"].data_ptr(), acc["sum"].data_ptr(), acc["npar"].data_ptr())

    def refmerge_local_maxl(self, packed: dict) -> torch.Tensor:
        out = torch.empty(max(packed["replicas"], 1), dtype=torch.int64, device=self.device)
        cin = self._refmerge_in(packed)
        self._call("crdt_refmerge_local_maxl", C.byref(cin), out.data_ptr())
        return out

    def refmerge_acc_rank(self, acc: dict, n_slots: int, shard: int) -> torch.Tensor:
        c = torch.empty(max(n_slots, 1), dtype=torch.int64, device=self.device)
        ca = self._acc(acc)
        self._call("crdt_refmerge_acc_rank", C.byref(ca), n_slots, shard, c.data_ptr())
        return c

    def refmerge_acc_owner_str(self, acc: dict, n_slots: int, c: torch.Tensor, cmax: torch.Tensor) -> torch.Tensor:
        v = torch.empty(max(n_slots, 1), dtype=torch.int64, device=self.device)
        ca = self._acc(acc)
        self._call("crdt_refmerge_acc_owner_str", C.byref(ca), n_slots, c.data_ptr(), cmax.data_ptr(), v.data_ptr())
        return v

    def refmerge_acc_set_best(self, acc: dict, n_slots: int, cmax: torch.Tensor, v: torch.Tensor) -> None:
        ca = self._acc(acc)
        self._call("crdt_refmerge_acc_set_best", C.byref(ca), n_slots, cmax.data_ptr(), v.data_ptr())

    def refmerge_finalize(self, packed: dict, acc: dict, out: dict) -> dict:
        ca = self._acc(acc)
        cout = crdt_refmerge_out(*(out[k].data_ptr() for k in
                                   ("off", "ts", "origin", "src", "st_kind", "st_str", "st_sum")))
        self._call("crdt_refmerge_finalize", C.byref(ca), int(packed["n_slots"]), _ptr(packed["str_bytes"]),
                   _ptr(packed["str_off"]), packed["str_off"].numel() - 1, C.byref(cout))
        return out

    # -- batched local apply
    def local_apply(self, diff: dict, cmds: dict, state: dict, str_bytes: torch.Tensor,
                    str_off: torch.Tensor, n_slots: int) -> dict:
        """AddCommand (main.go:173-215) for every replica at once
        (crdt_local_apply).  diff = {off, ts, origin} (device), cmds = {off,
        ts, kv_off, kv_key, kv_val} (device; arrival order per replica),
        state = {st_kind, st_str, st_sum} updated in place.  Returns the new
        Diff {off, ts, origin, src} (src < 0: command -(src+1)) and the
        per-command HTTP status."""
        dev = self.device
        n_l, n_c = diff["ts"].numel(), cmds["ts"].numel()
        P = diff["off"].numel() - 1
        out = {"off": torch.empty(P + 1, dtype=torch.int64, device=dev),
               "ts": torch.empty(max(n_l + n_c, 1), dtype=torch.int64, device=dev),
               "origin": torch.empty(max(n_l + n_c, 1), dtype=torch.uint8, device=dev),
               "src": torch.empty(max(n_l + n_c, 1), dtype=torch.int64, device=dev),
               "status": torch.empty(max(n_c, 1), dtype=torch.int16, device=dev)}
        cin = crdt_local_in(P, n_slots, n_l, n_c, cmds["kv_key"].numel(), str_off.numel() - 1,
                            _ptr(diff["off"]), _ptr(diff["ts"]), _ptr(diff["origin"]),
                            _ptr(cmds["off"]), _ptr(cmds["ts"]), _ptr(cmds["kv_off"]),
                            _ptr(cmds["kv_key"]), _ptr(cmds["kv_val"]), _ptr(str_bytes), _ptr(str_off))
        cout = crdt_local_out(*(out[k].data_ptr() for k in ("off", "ts", "origin", "src", "status")),
                              *(state[k].data_ptr() for k in ("st_kind", "st_str", "st_sum")))
        self._call("crdt_local_apply", C.byref(cin), C.byref(cout))
        return out

    def atoi_batch(self, str_bytes: torch.Tensor, str_off: torch.Tensor):
        n = str_off.numel() - 1
        ok = torch.empty(max(n, 1), dtype=torch.uint8, device=self.device)
        val = torch.empty(max(n, 1), dtype=torch.int64, device=self.device)
        self._call("crdt_atoi_batch", str_bytes.data_ptr(), str_off.data_ptr(), n, ok.data_ptr(), val.data_ptr())
        return ok[:n], val[:n]

    # ------------------------------------------------------------ sharding helpers (a9)
    def u64_to_ordered_i64(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        out = torch.empty_like(x) if out is None else out
        self._call("crdt_u64_to_ordered_i64", x.data_ptr(), out.data_ptr(), x.numel())
        return out

    def ordered_i64_to_u64(self, x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        out = torch.empty_like(x) if out is None else out
        self._call("crdt_ordered_i64_to_u64", x.data_ptr(), out.data_ptr(), x.numel())
        return out

    # ------------------------------------------------------------ synthetic state
    def synth_counters(self, seed: int, stream: int, rows: int, nodes: int, row_base: int = 0,
                       out: torch.Tensor | None = None) -> torch.Tensor:
        out = torch.empty(rows, nodes, dtype=torch.int64, device=self.device) if out is None else out
        self._call("crdt_synth_counters", seed, stream, out.data_ptr(), rows * nodes, row_base * nodes)
        return out

    def synth_vclock_pairs(self, seed: int, pairs: int, nodes: int, pair_base: int = 0):
        a = torch.empty(pairs, nodes, dtype=torch.int64, device=self.device)
        b = torch.empty(pairs, nodes, dtype=torch.int64, device=self.device)
        self._call("crdt_synth_vclock_pairs", seed, a.data_ptr(), b.data_ptr(), pairs, nodes, pair_base)
        return a, b

    def synth_set_tuples(self, seed: int, side: int, n: int, key_space: int, sort: bool = True) -> TupleSet:
        t = TupleSet.empty(n, self.device)
        ct = t.c()
        self._call("crdt_synth_set_tuples", seed, side, C.byref(ct), n, key_space)
        if sort:                                          # D1 inputs: the device tuple sort
            t = self.sort_tuples(t)
        return t
