"""GPU: BASELINE configs[2] and configs[3] D2 at FULL size against the oracle.

* configs[2]: 10M vector-clock pairs x 128 nodes (10.24 GB per operand, the
  bench's own device-generated population, seed 2024) classified on the GPU
  and by oc_vclock_classify over pinned D2H slices of the same pairs -- the
  full size crosses every 2^31-byte offset the 2M-pair sample does not.
* configs[3] D2: 10M + 10M UNSORTED tuples merged by the fused device sort +
  dedup (crdt_{lww,orset}_merge_unsorted) == oc_lww_merge / oc_orset_merge of
  the host-sorted sides ((key, ts, rep, tomb) order, the device sort's
  canonical order) -- directly against the oracle, not against the D1 path;
  and with tuples outside the sampled plan's ranges (the miss path at scale).
"""
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest
import torch

from oracle import oracle

pytestmark = pytest.mark.gpu

PAIRS, NODES = 10_000_000, 128
SLICE = 250_000                        # pairs per D2H slice: 256 MB per operand


def test_configs2_full_vclock_matches_oracle(eng):
    a, b = eng.synth_vclock_pairs(2024, PAIRS, NODES)   # bench.py VClockClassify's population (rank 0)
    cls = eng.vclock_classify(a, b).cpu().numpy()
    pa = torch.empty((SLICE, NODES), dtype=torch.int64, pin_memory=True)
    pb = torch.empty((SLICE, NODES), dtype=torch.int64, pin_memory=True)
    threads = 16
    with ThreadPoolExecutor(threads) as ex:
        for p0 in range(0, PAIRS, SLICE):
            n = min(SLICE, PAIRS - p0)
            pa[:n].copy_(a[p0:p0 + n])
            pb[:n].copy_(b[p0:p0 + n])
            ha, hb = pa[:n].numpy().view(np.uint64), pb[:n].numpy().view(np.uint64)
            cuts = [n * i // threads for i in range(threads + 1)]
            exp = np.concatenate(list(ex.map(lambda i: oracle.vclock_classify(ha[cuts[i]:cuts[i + 1]],
                                                                               hb[cuts[i]:cuts[i + 1]]),
                                              range(threads))))
            np.testing.assert_array_equal(cls[p0:p0 + n], exp, err_msg=f"pairs {p0}..{p0 + n}")
    frac = np.bincount(cls, minlength=4) / PAIRS
    assert np.all(np.abs(frac - 0.25) < 0.01), frac
    del a, b
    torch.cuda.empty_cache()


def _host_side(t):
    k, ts, r, m = t.to_numpy()
    o = np.lexsort((m, r, ts, k))                      # the device sort's (key, ts, rep, tomb) order
    return k[o], ts[o], r[o], m[o]


@pytest.mark.parametrize("lww", [True, False])
def test_configs3_full_d2_matches_oracle(eng, lww):
    n, ks = 10_000_000, 8_000_000                       # bench.py SetMergeUnsorted's population
    UA = eng.synth_set_tuples(2024, 0, n, ks, sort=False)
    UB = eng.synth_set_tuples(2024, 1, n, ks, sort=False)
    got = (eng.lww_merge_unsorted if lww else eng.orset_merge_unsorted)(UA, UB).to_numpy()
    sa, sb = _host_side(UA), _host_side(UB)
    ka = UA.key[:100_000].cpu().numpy().view(np.uint64)
    assert np.any(ka[1:] < ka[:-1])                    # the inputs really are unsorted
    exp = (oracle.lww_merge if lww else oracle.orset_merge)(sa, sb)
    assert len(got[0]) == len(exp[0])
    for g, e in zip(got, exp):
        np.testing.assert_array_equal(g, e)


def _sample_run_start(m, run):
    """First tuple of sampled run `run` (of 256, 64 tuples each) of a side of m
    tuples -- k_sample_minmax's spacing (sort.hip)."""
    return run * (m - 64) // 255


@pytest.mark.parametrize("lww", [True, False])
@pytest.mark.parametrize("outlier", ["key_unsampled", "key_sampled", "ts_rep_unsampled"])
def test_configs3_full_d2_plan_miss_matches_oracle(eng, lww, outlier):
    """configs[3] D2 at full size with a few tuples outside the dense-key
    plan's ranges (the sampled plan's miss path at scale).  The
    plan comes from 256 sampled runs of 64 tuples per side; a clean call first
    puts the shape in the context's plan cache, then:
    * *_unsampled: the far tuples lie between sampled runs -- the sample
      misses them, the composing pass's range check catches them, and the call
      is redone from the exact plan (a 2^40 key range: the general radix
      path; a wide ts / rep: wider composites);
    * key_sampled: the far key lies IN a sampled run -- the fresh sampled plan
      differs from the cached launch shape (k_plan_match: the passes keep the
      cached shape, the call is redone).
    The result == the oracle either way, and so is the next call."""
    n, ks = 10_000_000, 8_000_000
    UA = eng.synth_set_tuples(2024, 0, n, ks, sort=False)
    UB = eng.synth_set_tuples(2024, 1, n, ks, sort=False)
    fn = eng.lww_merge_unsorted if lww else eng.orset_merge_unsorted
    fn(UA, UB)                                           # the plan cache holds this shape now
    gap = _sample_run_start(n, 128) + 200                # between sampled runs 128 and 129
    if outlier == "key_unsampled":
        UA.key[gap] = 2**40 + 7
        UB.key[gap + 1000] = 2**40 + 7                   # the same key on both sides
    elif outlier == "key_sampled":
        UB.key[_sample_run_start(n, 85) + 5] = 2**40 + 7
    else:
        UB.ts[gap + 3] = 2**50 + 3
        UA.rep[gap + 5] = 0x7FFFFFF0
    got = fn(UA, UB).to_numpy()
    exp = (oracle.lww_merge if lww else oracle.orset_merge)(_host_side(UA), _host_side(UB))
    assert len(got[0]) == len(exp[0])
    for g, e in zip(got, exp):
        np.testing.assert_array_equal(g, e)
    again = fn(UA, UB).to_numpy()                        # the cache dropped on the miss: a fresh plan
    for g, e in zip(again, exp):
        np.testing.assert_array_equal(g, e)
