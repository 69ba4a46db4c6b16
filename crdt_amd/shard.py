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
from typing import List, Tuple

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
