"""GPU: BASELINE configs[2] and configs[3] D2 at FULL size against the oracle.

* configs[2]: 10M vector-clock pairs x 128 nodes (10.24 GB per operand, the
  bench's own device-generated population, seed 2024) classified on the GPU
  and by oc_vclock_classify over pinned D2H slices of the same pairs -- the
  full size crosses every 2^31-byte offset the 2M-pair sample does not.
* configs[3] D2: 10M + 10M UNSORTED tuples merged by the fused device sort +
  dedup (crdt_{lww,orset}_merge_unsorted) == oc_lww_merge / oc_orset_merge of
  the host-sorted sides ((key, ts, rep, tomb) order, the device sort's
  canonical order) -- directly against the oracle, not against the D1 path.
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
