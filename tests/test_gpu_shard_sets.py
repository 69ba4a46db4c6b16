"""GPU: key-range sharding of the set merges -- the device
lower_bound behind the shard slices, and the per-rank merges of a W-way
key-range split concatenated in rank order == the oracle's merge of the whole
sides, bit for bit (the all-gather-v step is covered on CPU by
test_shard_gloo.py)."""
import numpy as np
import pytest
import torch

from crdt_amd import shard, synth
from crdt_amd.engine import TupleSet, u64_tensor

from oracle import oracle
pytestmark = pytest.mark.gpu


def _cat(parts):
    return tuple(np.concatenate([p[i] for p in parts]) for i in range(4))


def test_lower_bound_u64_unsigned(eng):
    rng = np.random.default_rng(1)
    v = np.sort(np.concatenate([rng.integers(0, 2**64, 5000, dtype=np.uint64),
                                np.array([0, 0, 2**63, 2**63, 2**64 - 1], np.uint64)]))
    probes = np.concatenate([v[::37], rng.integers(0, 2**64, 300, dtype=np.uint64),
                             np.array([0, 1, 2**63 - 1, 2**63, 2**64 - 1], np.uint64)])
    got = eng.lower_bound_u64(u64_tensor(v, eng.device), u64_tensor(probes, eng.device)).cpu().numpy()
    np.testing.assert_array_equal(got, np.searchsorted(v, probes, side="left"))
    empty = eng.lower_bound_u64(u64_tensor(v[:0], eng.device), u64_tensor(probes[:3], eng.device))
    assert empty.cpu().tolist() == [0, 0, 0]


def _sets(kind):
    if kind == "config_d":
        n, ks = 200_000, 150_000
        return (synth.sort_tuples_np(*synth.set_tuples(31, 0, n, ks)),
                synth.sort_tuples_np(*synth.set_tuples(31, 1, n, ks)))
    rng = np.random.default_rng(7)

    def side(n):
        key = np.where(rng.random(n) < 0.4, np.uint64(2**63 + 5),          # one heavy key, high bit set
                       rng.integers(2**64 - 1000, 2**64, n, dtype=np.uint64))
        ts = rng.integers(0, 50, n, dtype=np.uint64)
        rep = rng.integers(0, 4, n, dtype=np.uint64).astype(np.uint32)
        tomb = rng.integers(0, 2, n, dtype=np.uint8)
        return synth.sort_tuples_np(key, ts, rep, tomb)
    return side(30_000), side(25_000)


@pytest.mark.parametrize("kind", ["config_d", "skewed_high_keys"])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("lww", [True, False])
def test_key_range_shards_concat_to_full_merge(eng, kind, world, lww):
    sa, sb = _sets(kind)
    A = TupleSet.from_numpy(*sa, eng.device)
    B = TupleSet.from_numpy(*sb, eng.device)
    full = (oracle.lww_merge if lww else oracle.orset_merge)(sa, sb)       # the oracle, not the unsharded GPU merge
    samples = torch.cat([shard.sample_keys(A, 256), shard.sample_keys(B, 256)]).cpu().numpy().view(np.uint64)
    spl = shard.splitters_from_samples(samples, world)
    parts = [shard.merge_key_range(eng, A, B, spl[r], spl[r + 1], lww).to_numpy() for r in range(world)]
    got = _cat(parts)
    for g, e in zip(got, full):
        np.testing.assert_array_equal(g, e)
    assert eng.device_status() == 0


def test_splitters_on_exact_keys_and_empty_ranges(eng):
    sa, sb = _sets("config_d")
    A = TupleSet.from_numpy(*sa, eng.device)
    B = TupleSet.from_numpy(*sb, eng.device)
    k = sa[0]
    spl = [0, int(k[1000]), int(k[1000]), int(k[50_000]) + 1, int(k[-1]), shard.KEY_END]   # equal + exact keys
    parts = [shard.merge_key_range(eng, A, B, spl[r], spl[r + 1]).to_numpy() for r in range(len(spl) - 1)]
    assert len(parts[1][0]) == 0
    for g, e in zip(_cat(parts), oracle.lww_merge(sa, sb)):
        np.testing.assert_array_equal(g, e)


def test_sharded_set_merge_single_rank(eng):
    sa, sb = _sets("config_d")
    A = TupleSet.from_numpy(*sa, eng.device)
    B = TupleSet.from_numpy(*sb, eng.device)
    got = shard.sharded_set_merge(eng, A, B, lww=False).to_numpy()
    for g, e in zip(got, oracle.orset_merge(sa, sb)):
        np.testing.assert_array_equal(g, e)
