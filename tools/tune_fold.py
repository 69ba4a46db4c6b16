#!/usr/bin/env python3
"""Interleaved A/B sweep of the fold kernel knobs (one process), configs[4]
size by default: unroll x nontemporal x blocks_per_cu, median / min of the
per-launch HIP-event time (crdt_gcounter_fold, both kernels + the memset)."""
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crdt_amd import _lib  # noqa: E402
from crdt_amd.engine import Engine  # noqa: E402
from tune_join import timed  # noqa: E402


def main():
    rows, nodes = int(os.environ.get("ROWS", 100_000_000)), 64
    eng = Engine(0)
    a = eng.synth_counters(1, 1, rows, nodes)
    o = torch.empty(nodes, dtype=torch.int64, device=eng.device)
    nbytes = rows * nodes * 8
    variants = list(itertools.product([2, 4, 8, 16], [1], [1, 2, 3, 4]))
    res = {v: [] for v in variants}
    ref = None
    for rnd in range(3):
        for v in variants:
            u, nt, bpc = v
            _lib.call("crdt_set_option", b"fold.unroll", u)
            _lib.call("crdt_set_option", b"fold.nontemporal", nt)
            _lib.call("crdt_set_option", b"fold.blocks_per_cu", bpc)
            res[v] += timed(lambda: eng.gcounter_fold(a, out=o), reps=4)
            got = o.cpu()
            ref = got if ref is None else ref
            assert torch.equal(got, ref), v
        print(f"round {rnd} done", file=sys.stderr, flush=True)
    out = []
    for v, ts in res.items():
        med, mn = float(np.median(ts)), float(np.min(ts))
        out.append({"variant": "unroll,nt,bpc=" + str(v), "median_us": round(med, 1), "min_us": round(mn, 1),
                    "GBps_median": round(nbytes / med / 1e3, 1), "frac": round(nbytes / med / 1e3 / 8000, 4)})
    out.sort(key=lambda r: r["median_us"])
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
