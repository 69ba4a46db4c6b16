"""Replica-sharded joins across GPUs.

One process per GPU (torch.distributed; backend "nccl" is RCCL on ROCm,
"gloo" for the CPU tests).  The only data-path exchange steps:

  * counters / clocks: each rank folds its contiguous row shard on its GPU
    (crdt_gcounter_fold), then ONE all-reduce(MAX) of the `nodes`-long
    uint64 fold.  RCCL's MAX is signed on int64, so values travel through
    the order-preserving map x ^ 2^63 (crdt_u64_to_ordered_i64): exact, since
    max commutes with a monotone bijection.
  * keyed sets: ranks own disjoint, ordered key ranges (splitters), merge
    their ranges locally, and an all-gather-v concatenates the outputs in
    rank order -- already the globally sorted merged state, because LWW and
    OR-Set outputs for a key depend only on that key's tuples.

The reference's analog is pull gossip of the whole log over HTTP
(main.go:226-258); there is no reference collective to mirror.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from . import _lib

INT64_MIN = -(2**63)


def shard_range(rows: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous balanced row range of `rank` (crdt_shard_range)."""
    b, e = C.c_uint64(), C.c_uint64()
    _lib.call("crdt_shard_range", rows, world, rank, C.byref(b), C.byref(e))
    return b.value, e.value


def _to_ordered(t: torch.Tensor, eng=None) -> torch.Tensor:
    if t.is_cuda:
        return eng.u64_to_ordered_i64(t)
    return t ^ INT64_MIN          # gloo/CPU transport of the exchange (tests): same bijection


def _from_ordered(t: torch.Tensor, eng=None) -> torch.Tensor:
    if t.is_cuda:
        return eng.ordered_i64_to_u64(t)
    return t ^ INT64_MIN


def allreduce_max_u64(t: torch.Tensor, eng=None, group=None) -> torch.Tensor:
    """Unsigned-max all-reduce of an int64-stored uint64 tensor (in place)."""
    if t.dtype != torch.int64:
        raise TypeError("uint64 state travels in int64 tensors")
    o = _to_ordered(t, eng)
    dist.all_reduce(o, op=dist.ReduceOp.MAX, group=group)
    t.copy_(_from_ordered(o, eng))
    return t


def sharded_fold(eng, shard: torch.Tensor, group=None) -> torch.Tensor:
    """Whole-population join: GPU fold of this rank's [rows, nodes] shard,
    then all-reduce(max) across ranks.  Returns the global [nodes] fold."""
    local = eng.gcounter_fold(shard)
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        allreduce_max_u64(local, eng, group)
    return local


def allgather_v(t: torch.Tensor, group=None) -> torch.Tensor:
    """Concatenate variable-length 1-D tensors of every rank in rank order."""
    world = dist.get_world_size(group)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=t.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    pad = torch.zeros(m, dtype=t.dtype, device=t.device)
    pad[: t.numel()] = t
    bufs = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(bufs, pad, group=group)
    return torch.cat([b[:c] for b, c in zip(bufs, counts)])


def key_splitters(key_space: int, world: int) -> List[int]:
    """Equal-width key ranges [s_r, s_{r+1}) for `world` ranks (uint64 keys)."""
    return [key_space * r // world for r in range(world)] + [key_space]


# ---------------------------------------------------------------- keyed sets (§8(e) D)
KEY_END = 2**64                   # exclusive upper end of the uint64 key space


def sample_keys(t, per: int) -> torch.Tensor:
    """`per` keys at evenly spaced positions of a key-sorted TupleSet."""
    n = len(t)
    if n == 0 or per <= 0:
        return t.key[:0]
    idx = torch.arange(per, dtype=torch.int64, device=t.key.device) * n // per
    return t.key[idx]


def splitters_from_samples(samples: np.ndarray, world: int) -> List[int]:
    """Rank r owns keys [s[r], s[r+1]); s[0] = 0, s[world] = 2^64, the inner
    splitters are the world-quantiles of the pooled uint64 key sample."""
    s = np.sort(np.asarray(samples, dtype=np.uint64))
    inner = [int(s[(r * len(s)) // world]) if len(s) else 0 for r in range(1, world)]
    return [0] + inner + [KEY_END]


def sample_splitters(a, b, world: int, group=None, per: int = 256) -> List[int]:
    """Balanced key splitters for a sharded set merge: every rank samples its
    sorted inputs, the samples are all-gathered (one small exchange) and
    every rank derives the same splitters from the pooled sample."""
    loc = torch.cat([sample_keys(a, per), sample_keys(b, per)])
    if dist.is_initialized() and dist.get_world_size(group) > 1:
        loc = allgather_v(loc, group)
    return splitters_from_samples(loc.cpu().numpy().view(np.uint64), world)


def key_range(eng, t, lo: int, hi: int):
    """The tuples of a key-sorted TupleSet with lo <= key < hi (a view; one
    device lower_bound per end, crdt_u64_lower_bound)."""
    from .engine import TupleSet
    n = len(t)
    i, j = 0, n
    if n:
        probes = [lo] + ([hi] if hi < KEY_END else [])
        pr = torch.tensor(np.array(probes, dtype=np.uint64).view(np.int64), device=t.key.device)
        got = eng.lower_bound_u64(t.key, pr).cpu().tolist()
        i = got[0]
        j = got[1] if hi < KEY_END else n
    return TupleSet(t.key[i:j], t.ts[i:j], t.rep[i:j], t.tomb[i:j])


def merge_key_range(eng, a, b, lo: int, hi: int, lww: bool = True):
    """One rank's share of a key-range-sharded merge: the LWW / OR-Set merge
    of the [lo, hi) slices of both sorted inputs (outputs for a key depend
    only on that key's tuples, so the shards are independent)."""
    fn = eng.lww_merge if lww else eng.orset_merge
    return fn(key_range(eng, a, lo, hi), key_range(eng, b, lo, hi))


def sharded_set_merge(eng, a, b, lww: bool = True, group=None, gather: bool = True,
                      splitters: Sequence[int] | None = None):
    """Set merge of A and B (both key-sorted, present on every rank) sharded
    by key range over the ranks of `group`: sample splitters (unless given),
    merge this rank's range on its GPU, then (gather=True) an all-gather-v of
    the four SoA fields in rank order -- the globally sorted merged state.
    One rank (or no process group): the plain device merge."""
    from .engine import TupleSet
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return merge_key_range(eng, a, b, 0, KEY_END, lww)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    spl = list(splitters) if splitters is not None else sample_splitters(a, b, world, group)
    m = merge_key_range(eng, a, b, spl[rank], spl[rank + 1], lww)
    if not gather:
        return m
    return TupleSet(allgather_v(m.key, group), allgather_v(m.ts, group), allgather_v(m.rep, group),
                    allgather_v(m.tomb, group))



# ---------------------------------------------------------------- distributed keyed sets (§8(e) D)
SAMPLES_PER_SIDE = 256            # = kSamplesPerSide of csrc/shard.hip


def weighted_splitters(blocks: np.ndarray, world: int, per: int = SAMPLES_PER_SIDE) -> List[int]:
    """Splitters of a distributed key population (crdt_shard_*_merge_local's
    rule): blocks[p] = [n_a, n_b, per keys of A, per keys of B] of rank p; a
    non-empty side's samples each weigh its size, an empty side's none.  Inner
    splitter q = the first sample key (in key order) at which the cumulative
    weight reaches q / world of the total."""
    e = []
    for b in np.asarray(blocks, dtype=np.uint64).reshape(world, 2 + 2 * per):
        for side in range(2):
            n = int(b[side])
            if n:
                e += [(int(k), n) for k in b[2 + side * per: 2 + (side + 1) * per]]
    e.sort(key=lambda x: x[0])
    W = sum(w for _, w in e)
    spl, cum, k = [0], 0, 0
    for q in range(1, world):
        while k < len(e) and (cum + e[k][1]) * world < q * W:
            cum += e[k][1]
            k += 1
        spl.append(0 if W == 0 else (e[k][0] if k < len(e) else e[-1][0]))
    return spl + [KEY_END]


def _sample_block(t_a, t_b, per: int) -> torch.Tensor:
    out = torch.zeros(2 + 2 * per, dtype=torch.int64, device=t_a.key.device)
    out[0], out[1] = len(t_a), len(t_b)
    for side, t in ((0, t_a), (1, t_b)):
        n = len(t)
        if n:
            idx = torch.arange(per, dtype=torch.int64, device=t.key.device) * n // per
            out[2 + side * per: 2 + (side + 1) * per] = t.key[idx]
    return out


def _cuts(eng, t, spl: List[int]) -> List[int]:
    """0, lower_bound(spl[1]) .. lower_bound(spl[R-1]), n in t's sorted keys."""
    n, inner = len(t), spl[1:-1]
    if n == 0 or not inner:
        return [0] * (len(spl) - 1) + [n]
    pr = np.array(inner, dtype=np.uint64)
    if t.key.is_cuda:
        got = eng.lower_bound_u64(t.key, torch.from_numpy(pr.view(np.int64)).to(t.key.device)).cpu().tolist()
    else:
        got = np.searchsorted(t.key.numpy().view(np.uint64), pr, side="left").tolist()
    return [0] + [int(x) for x in got] + [n]


def alltoallv(t: torch.Tensor, send_counts: List[int], recv_counts: List[int], group=None) -> torch.Tensor:
    """All-to-all-v of a 1-D tensor: segment q of t (send_counts[q] elements,
    segments in rank order) goes to rank q; the result holds what every rank
    sent here, in rank order.  Paired isend / irecv (works on gloo and nccl)."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if t.is_cuda and dist.get_backend(group) == "gloo":      # gloo's send / recv take host tensors
        return alltoallv(t.cpu(), send_counts, recv_counts, group).to(t.device)
    out = torch.empty(sum(recv_counts), dtype=t.dtype, device=t.device)
    so = np.concatenate([[0], np.cumsum(send_counts)]).astype(np.int64)
    ro = np.concatenate([[0], np.cumsum(recv_counts)]).astype(np.int64)
    out[ro[rank]:ro[rank + 1]] = t[so[rank]:so[rank + 1]]
    reqs = []
    for q in range(world):
        if q == rank:
            continue
        peer = dist.get_global_rank(group, q) if group is not None else q
        if send_counts[q]:
            reqs.append(dist.isend(t[so[q]:so[q + 1]].contiguous(), peer, group=group))
        if recv_counts[q]:
            reqs.append(dist.irecv(out[ro[q]:ro[q + 1]], peer, group=group))
    for r in reqs:
        r.wait()
    return out


def _tree_merge(runs_a, runs_b, merge):
    """A's runs pairwise in rank order (lower rank left), B's likewise, then
    merge(A, B): the order crdt_shard_*_merge_local merges in."""
    def level(runs):
        return [merge(runs[k], runs[k + 1]) if k + 1 < len(runs) else merge(runs[k], runs[k].slice(0))
                for k in range(0, len(runs), 2)]
    while len(runs_a) > 1 or len(runs_b) > 1:
        runs_a, runs_b = level(runs_a), level(runs_b)
    return merge(runs_a[0], runs_b[0])


def sharded_set_merge_local(eng, a, b, lww: bool = True, group=None, gather: bool = True, merge=None,
                            per: int = SAMPLES_PER_SIDE):
    """Keyed-set merge of a DISTRIBUTED population over torch.distributed
    (crdt_shard_*_merge_local's protocol): a, b = THIS rank's sorted local
    tuples.  The population's A = stable rank-order merge of every rank's A
    (B likewise); returns the merge of the two -- the whole state (gather) or
    this rank's key range of it.  `merge` (default the engine's LWW / OR-Set
    merge) is the per-rank compute."""
    from .engine import TupleSet
    merge = merge or (eng.lww_merge if lww else eng.orset_merge)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return merge(a, b)
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    blk = _sample_block(a, b, per)
    blocks = [torch.zeros_like(blk) for _ in range(world)]
    dist.all_gather(blocks, blk, group=group)
    spl = weighted_splitters(torch.stack(blocks).cpu().numpy().view(np.uint64), world, per)
    ca, cb = _cuts(eng, a, spl), _cuts(eng, b, spl)
    sa = [ca[q + 1] - ca[q] for q in range(world)]
    sb = [cb[q + 1] - cb[q] for q in range(world)]
    cnt = torch.tensor(sa + sb, dtype=torch.int64, device=a.key.device)
    mat = [torch.zeros_like(cnt) for _ in range(world)]
    dist.all_gather(mat, cnt, group=group)
    mat = torch.stack(mat).cpu().numpy()
    ra, rb = mat[:, rank].tolist(), mat[:, world + rank].tolist()

    def xchg(t, s, r):
        return TupleSet(*(alltoallv(f, s, r, group) for f in (t.key, t.ts, t.rep, t.tomb)))

    ga, gb = xchg(a, sa, ra), xchg(b, sb, rb)

    def runs(t, counts):
        o = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
        return [TupleSet(t.key[o[p]:o[p + 1]], t.ts[o[p]:o[p + 1]], t.rep[o[p]:o[p + 1]], t.tomb[o[p]:o[p + 1]])
                for p in range(world)]

    m = _tree_merge(runs(ga, ra), runs(gb, rb), merge)
    if not gather:
        return m
    return TupleSet(allgather_v(m.key, group), allgather_v(m.ts, group), allgather_v(m.rep, group),
                    allgather_v(m.tomb, group))


# ---------------------------------------------------------------- RefMerge by ts range (§8(e))
def sharded_refmerge(eng, packed: dict, group=None) -> dict:
    """(*Server).merge() of one batch of replicas whose Diff/RemoteDiff logs
    are split by ts range over the ranks of `group` (rank r holds the r-th
    ts range of every replica, ranks in ascending ts order; `packed` is this
    rank's slice in the crdt_refmerge_in layout).  Exchange steps:
      1. all-reduce(MAX) of every replica's local max(L): remote ts at or
         above the GLOBAL max(L) are dropped (main.go:49);
      2. the local merge with that max -> this rank's slice of the new Diff
         (slices concatenate in rank order) + unreduced replay accumulators;
      3. all-reduce(MAX) of the cross-rank rank of each key's max-ts holder,
         all-reduce(SUM) of the owner's string id, of the wrapped sums and of
         the parsable counts (main.go:82-96);
      4. CurrentState from the reduced accumulators, identical on every rank.
    Integer reductions only: bit-exact for any world size.  Returns the
    refmerge_batch output dict (new-Diff slice + the full state)."""
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    n_slots = int(packed["n_slots"])
    maxl = eng.refmerge_local_maxl(packed)
    if world > 1:
        dist.all_reduce(maxl, op=dist.ReduceOp.MAX, group=group)     # int64 ts: signed MAX is exact
    acc = eng.refmerge_acc_new(n_slots)
    out = eng.refmerge_batch(packed, maxl=maxl, acc=acc)
    if world > 1 and n_slots:
        c = eng.refmerge_acc_rank(acc, n_slots, rank)
        cmax = c.clone()
        dist.all_reduce(cmax, op=dist.ReduceOp.MAX, group=group)
        v = eng.refmerge_acc_owner_str(acc, n_slots, c, cmax)
        dist.all_reduce(v, op=dist.ReduceOp.SUM, group=group)
        dist.all_reduce(acc["sum"], op=dist.ReduceOp.SUM, group=group)   # int64 add wraps (main.go:95)
        dist.all_reduce(acc["npar"], op=dist.ReduceOp.SUM, group=group)
        eng.refmerge_acc_set_best(acc, n_slots, cmax, v)
    return eng.refmerge_finalize(packed, acc, out)


# ---------------------------------------------------------------- native RCCL communicator
class Comm:
    """The C-ABI's own RCCL communicator (crdt_shard_*, csrc/shard.hip).

    * ``Comm.create(devices)``: one process drives every listed GPU
      (ncclCommInitAll); per-member inputs are lists indexed by member, each
      tensor on that member's GPU.  Member contexts run on streams the
      library owns: inputs must be ready (torch.cuda.synchronize) before a
      call, and :meth:`sync` before outputs are read.
    * ``Comm.init_rank(eng, group)``: one member per process (one process per
      GPU, as torchrun launches the bench); rank 0's RCCL unique id travels
      over the torch.distributed group once, after that every data-path
      collective is the library's own ncclAllReduce / ncclAllGather /
      grouped ncclSend-ncclRecv on the engine's stream.
    * ``Comm.loopback(device, members)``: ``members`` ranks on one GPU (the
      loopback transport), for the multi-rank protocols on a one-GPU box.

    uint64 state travels as ncclUint64 with ncclMax: RCCL's unsigned max is
    exactly the G-Counter / vector-clock join.
    """

    def __init__(self, handle: C.c_void_p, devices: Sequence[torch.device], owner=None):
        self._h = handle
        self.devices = list(devices)
        self._owner = owner                 # keeps a borrowed Engine alive
        m, n, r0 = C.c_int(), C.c_int(), C.c_int()
        _lib.call("crdt_shard_comm_info", handle, C.byref(m), C.byref(n), C.byref(r0))
        self.members, self.nranks, self.rank0 = m.value, n.value, r0.value

    @classmethod
    def create(cls, devices: Sequence[int]) -> "Comm":
        arr = (C.c_int * len(devices))(*devices)
        h = C.c_void_p()
        _lib.call("crdt_shard_comm_create", arr, len(devices), C.byref(h))
        return cls(h, [torch.device("cuda", d) for d in devices])

    @classmethod
    def loopback(cls, device: int, members: int) -> "Comm":
        """``members`` ranks on ONE GPU in this process (the loopback
        transport: device copies and a reduction kernel fenced by events
        against the member streams) -- the multi-rank protocols at R > 1 on a
        one-GPU machine, with the same compute as over RCCL."""
        h = C.c_void_p()
        _lib.call("crdt_shard_comm_create_loopback", device, members, C.byref(h))
        return cls(h, [torch.device("cuda", device)] * members)

    @property
    def transport(self) -> str:
        k = C.c_int()
        _lib.call("crdt_shard_comm_transport", self._h, C.byref(k))
        return {0: "rccl", 1: "loopback"}[k.value]

    @classmethod
    def init_rank(cls, eng, group=None) -> "Comm":
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        uid = C.create_string_buffer(128)
        if rank == 0:
            _lib.call("crdt_shard_unique_id", uid, 128)
        if world > 1:
            obj = [uid.raw if rank == 0 else None]
            dist.broadcast_object_list(obj, src=dist.get_global_rank(group, 0) if group is not None else 0,
                                       group=group)
            uid = C.create_string_buffer(obj[0], 128)
        eng._bind()
        h = C.c_void_p()
        _lib.call("crdt_shard_comm_init_rank", eng.ctx, uid, world, rank, C.byref(h), ctx=eng.ctx)
        c = cls(h, [eng.device], owner=eng)
        eng._depend(c)                      # eng.close() destroys the communicator first
        return c

    def _depend(self, obj) -> None:
        """obj (a population on a member context) is closed before the communicator."""
        import weakref
        if not hasattr(self, "_deps"):
            self._deps = []
        self._deps.append(weakref.ref(obj))

    def close(self) -> None:
        for r in getattr(self, "_deps", []):
            o = r()
            if o is not None:
                o.close()
        self._deps = []
        if getattr(self, "_h", None):
            if self._owner is not None and not getattr(self._owner, "ctx", None):
                raise RuntimeError("engine closed before its communicator")   # never reached via Engine.close
            _lib.lib().crdt_shard_comm_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def _call(self, fn: str, *args) -> None:
        if self._owner is not None:
            self._owner._bind()
        st = getattr(_lib.lib(), fn)(self._h, *args)
        if st < 0:
            raise _lib.CrdtError(fn, st, _lib.lib().crdt_shard_comm_last_error(self._h))

    def _ptrs(self, ts) -> C.Array:
        if len(ts) != self.members:
            raise ValueError(f"expected one tensor per member ({self.members})")
        for t, d in zip(ts, self.devices):
            if t.device != d or not t.is_contiguous():
                raise ValueError(f"member tensor must be contiguous on {d}")
        return (C.c_void_p * self.members)(*[t.data_ptr() for t in ts])

    def sync(self) -> None:
        self._call("crdt_shard_sync")

    def fold_max(self, shards: Sequence[torch.Tensor], outs: Sequence[torch.Tensor] | None = None):
        """Config E1: per-member fold of its [rows, nodes] shard, then
        ncclAllReduce(ncclUint64, ncclMax): every member's out = the global fold."""
        nodes = shards[0].shape[1]
        if outs is None:
            outs = [torch.empty(nodes, dtype=torch.int64, device=d) for d in self.devices]
        rows = (C.c_size_t * self.members)(*[s.shape[0] for s in shards])
        self._call("crdt_shard_fold_max_u64", self._ptrs(shards), rows, nodes, self._ptrs(outs))
        return outs

    def allreduce_max_u64(self, bufs: Sequence[torch.Tensor]):
        """Config E2: in-place ncclAllReduce(ncclUint64, ncclMax)."""
        self._call("crdt_shard_allreduce_max_u64", self._ptrs(bufs), bufs[0].numel())
        return bufs

    def allreduce(self, bufs: Sequence[torch.Tensor], op: str = "sum"):
        """In-place all-reduce of int64 / int32 tensors (signed), op 'sum' | 'max'."""
        t = {torch.int64: 0, torch.int32: 3}[bufs[0].dtype]
        self._call("crdt_shard_allreduce", self._ptrs(bufs), bufs[0].numel(), t, {"sum": 0, "max": 1}[op])
        return bufs

    @staticmethod
    def _tuples(sets) -> C.Array:
        from ._lib import crdt_tuples
        return (crdt_tuples * len(sets))(*[s.c() for s in sets])

    def set_allgather_v(self, locals_, outs, cap: int) -> int:
        """Every member's out <- all ranks' local tuples in rank order; returns the length."""
        n = (C.c_size_t * self.members)(*[len(s) for s in locals_])
        tot = C.c_size_t()
        self._call("crdt_shard_set_allgather_v", self._tuples(locals_), n, self._tuples(outs), cap, C.byref(tot))
        return tot.value

    def set_merge(self, a, b, lww: bool = True, outs=None):
        """Key-range-sharded LWW / OR-Set merge of inputs every member holds
        in full; returns per-member TupleSets (the whole merged state)."""
        from .engine import TupleSet
        na, nb = len(a[0]), len(b[0])
        cap = max(na + nb, 1)
        outs = [TupleSet.empty(cap, d) for d in self.devices] if outs is None else outs
        n = C.c_size_t()
        self._call("crdt_shard_lww_merge" if lww else "crdt_shard_orset_merge", self._tuples(a), na,
                   self._tuples(b), nb, self._tuples(outs), cap, C.byref(n))
        return [o.slice(n.value) for o in outs]

    def alltoallv(self, sends, send_counts, recvs, recv_counts, elem_size: int) -> None:
        """crdt_shard_alltoallv: counts are [members x nranks] nested lists."""
        flat = lambda x: (C.c_size_t * (self.members * self.nranks))(*[int(v) for row in x for v in row])
        self._call("crdt_shard_alltoallv", self._ptrs(sends), flat(send_counts), self._ptrs(recvs),
                   flat(recv_counts), elem_size)

    def set_merge_local(self, a, b, lww: bool = True, gather: bool = True, cap: int | None = None, outs=None):
        """Keyed-set merge of a distributed population: a[i], b[i] = member
        i's own sorted tuples (crdt_shard_*_merge_local).  Returns per-member
        TupleSets: the whole merged state (gather) or the member's key range."""
        from .engine import TupleSet
        na = (C.c_size_t * self.members)(*[len(x) for x in a])
        nb = (C.c_size_t * self.members)(*[len(x) for x in b])
        if cap is None:                     # a bound needs every rank's sizes: one process holding them all
            if self.members != self.nranks:
                raise ValueError("cap is required when other processes hold members")
            cap = max(sum(len(x) + len(y) for x, y in zip(a, b)), 1)
        outs = [TupleSet.empty(cap, d) for d in self.devices] if outs is None else outs
        n = (C.c_size_t * self.members)()
        self._call("crdt_shard_lww_merge_local" if lww else "crdt_shard_orset_merge_local", self._tuples(a), na,
                   self._tuples(b), nb, self._tuples(outs), cap, n, 1 if gather else 0)
        return [o.slice(n[i]) for i, o in enumerate(outs)]

    def set_merge_local_dev(self, a, b, lww: bool = True, cap: int | None = None, outs=None):
        """crdt_shard_*_merge_local_dev: each member's own key range, its
        length left on the device (no trailing synchronisation).  Returns
        (outs, counts): per-member TupleSets of capacity cap and int64[1]
        device counts."""
        from .engine import TupleSet
        na = (C.c_size_t * self.members)(*[len(x) for x in a])
        nb = (C.c_size_t * self.members)(*[len(x) for x in b])
        if cap is None:
            if self.members != self.nranks:
                raise ValueError("cap is required when other processes hold members")
            cap = max(sum(len(x) + len(y) for x, y in zip(a, b)), 1)
        outs = [TupleSet.empty(cap, d) for d in self.devices] if outs is None else outs
        counts = [torch.zeros(1, dtype=torch.int64, device=d) for d in self.devices]
        self._call("crdt_shard_lww_merge_local_dev" if lww else "crdt_shard_orset_merge_local_dev", self._tuples(a),
                   na, self._tuples(b), nb, self._tuples(outs), cap, self._ptrs(counts))
        return outs, counts

    def refmerge(self, engines, packed_list):
        """crdt_shard_refmerge: member i merges packed_list[i] (its ts-range
        slice of one batch, device tensors on member i's GPU; engines[i] only
        allocates the outputs).  Returns per-member refmerge output dicts
        (new-Diff slice + the whole CurrentState)."""
        from ._lib import crdt_refmerge_in, crdt_refmerge_out
        outs, cins, couts = [], [], []
        for eng, d in zip(engines, packed_list):
            n_l, n_r, ns = d["l_ts"].numel(), d["r_ts"].numel(), int(d["n_slots"])
            dev = eng.device
            o = {"off": torch.empty(d["replicas"] + 1, dtype=torch.int64, device=dev),
                 "ts": torch.empty(max(n_l + n_r, 1), dtype=torch.int64, device=dev),
                 "origin": torch.empty(max(n_l + n_r, 1), dtype=torch.uint8, device=dev),
                 "src": torch.empty(max(n_l + n_r, 1), dtype=torch.int64, device=dev),
                 "st_kind": torch.empty(max(ns, 1), dtype=torch.uint8, device=dev),
                 "st_str": torch.empty(max(ns, 1), dtype=torch.int32, device=dev),
                 "st_sum": torch.empty(max(ns, 1), dtype=torch.int64, device=dev)}
            outs.append(o)
            cins.append(eng._refmerge_in(d))
            couts.append(crdt_refmerge_out(*(o[k].data_ptr() for k in
                                             ("off", "ts", "origin", "src", "st_kind", "st_str", "st_sum"))))
        ci = (crdt_refmerge_in * self.members)(*cins)
        co = (crdt_refmerge_out * self.members)(*couts)
        self._call("crdt_shard_refmerge", ci, co)
        return outs
