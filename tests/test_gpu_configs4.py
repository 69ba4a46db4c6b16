"""GPU: BASELINE configs[4] at FULL size on one MI355X -- a 100M-replica x
64-node uint64 G-Counter population (51.2 GB, device-generated), the
north_star's scaling config.

Checked against the oracle (oc_gcounter_fold) computed chunk-wise on the
host over 1-GB D2H slices of the same device population:
  * the one-GPU fold of the whole population;
  * an 8-way crdt_shard_range split (the 8-GPU sharding) folded per shard and
    max-combined -- the join the RCCL all-reduce(max) performs across GPUs;
  * the native communicator path crdt_shard_fold_max_u64 (1-rank RCCL
    ncclAllReduce(ncclUint64, ncclMax)) over the whole population;
  * the same protocol over 8 LOOPBACK ranks on the one GPU (each rank its
    crdt_shard_range shard, the all-reduce(max) a reduction kernel over the
    eight members' folds): every rank's result == the oracle.
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from crdt_amd import shard, synth
from crdt_amd.engine import as_u64
from oracle import oracle

pytestmark = pytest.mark.gpu

ROWS, NODES = 100_000_000, 64
CHUNK = 2_000_000                      # 1.024 GB per D2H slice


def _host_fold(t: torch.Tensor, threads: int = 16) -> np.ndarray:
    """oc_gcounter_fold over 1-GB slices of a device [rows, nodes] tensor,
    each slice split over host threads, max-combined."""
    acc = np.zeros(t.shape[1], np.uint64)
    pinned = torch.empty((CHUNK, t.shape[1]), dtype=torch.int64, pin_memory=True)
    with ThreadPoolExecutor(threads) as ex:
        for r0 in range(0, t.shape[0], CHUNK):
            n = min(CHUNK, t.shape[0] - r0)
            pinned[:n].copy_(t[r0:r0 + n])
            a = pinned[:n].numpy().view(np.uint64)
            parts = [a[i * n // threads:(i + 1) * n // threads] for i in range(threads)]
            acc = np.maximum.reduce([acc] + [f for f in ex.map(oracle.gcounter_fold, parts)])
    return acc


@pytest.fixture(scope="module")
def population(eng):
    t = eng.synth_counters(2024, 1, ROWS, NODES)       # the bench's shard_fold population (seed 2024, stream 1)
    torch.cuda.synchronize()
    yield t
    del t
    torch.cuda.empty_cache()


def test_configs4_population_generator(population):
    flat = population.view(-1)
    n = 64_000
    np.testing.assert_array_equal(as_u64(flat[:n]), synth.counters(2024, 1, n))
    np.testing.assert_array_equal(as_u64(flat[-n:]), synth.counters(2024, 1, n, ROWS * NODES - n))


@pytest.fixture(scope="module")
def expected_fold(population):
    return _host_fold(population)


def test_configs4_fold_and_8way_shards_match_oracle(eng, population, expected_fold):
    exp = expected_fold
    whole = as_u64(eng.gcounter_fold(population))
    np.testing.assert_array_equal(whole, exp)
    parts = []
    for r in range(8):
        b, e = shard.shard_range(ROWS, 8, r)
        parts.append(as_u64(eng.gcounter_fold(population[b:e])))
    np.testing.assert_array_equal(np.maximum.reduce(parts), exp)
    # the native RCCL path over the whole population (one rank)
    c = shard.Comm.init_rank(eng)
    try:
        got = c.fold_max([population])[0]
        np.testing.assert_array_equal(as_u64(got), exp)
    finally:
        c.close()


def test_configs4_fold_max_over_8_loopback_ranks(population, expected_fold):
    """configs[4] through crdt_shard_fold_max_u64 over R = 8 loopback ranks:
    the 8-GPU sharding of the north_star's scaling config, each rank's
    12.5M-row shard folded on its own stream, the 512-B folds all-reduced."""
    c = shard.Comm.loopback(0, 8)
    try:
        shards = []
        for r in range(8):
            b, e = shard.shard_range(ROWS, 8, r)
            shards.append(population[b:e])
        outs = c.fold_max(shards)
        c.sync()
        for r, o in enumerate(outs):
            np.testing.assert_array_equal(as_u64(o), expected_fold, err_msg=f"rank {r}")
    finally:
        c.close()
