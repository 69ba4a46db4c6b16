#!/usr/bin/env python3
"""Interleaved A/B sweep of the vector-clock classify knobs at configs[2]
size (10M pairs x 128 nodes): pairs_per_wave x blocks_per_cu."""
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
    pairs, nodes = int(os.environ.get("PAIRS", 10_000_000)), 128
    eng = Engine(0)
    a, b = eng.synth_vclock_pairs(2024, pairs, nodes)
    o = torch.empty(pairs, dtype=torch.uint8, device=eng.device)
    nbytes = pairs * (2 * nodes * 8 + 1)
    variants = list(itertools.product([1, 2, 4, 8], [1, 2, 4, 8, 16]))
    res = {v: [] for v in variants}
    ref = None
    for rnd in range(3):
        for v in variants:
            _lib.call("crdt_set_option", b"vclock.pairs_per_wave", v[0])
            _lib.call("crdt_set_option", b"vclock.blocks_per_cu", v[1])
            res[v] += timed(lambda: eng.vclock_classify(a, b, out=o), reps=4)
            got = o.cpu()
            ref = got if ref is None else ref
            assert torch.equal(got, ref), v
        print(f"round {rnd} done", file=sys.stderr, flush=True)
    out = []
    for v, ts in res.items():
        med, mn = float(np.median(ts)), float(np.min(ts))
        out.append({"variant": "ppw,bpc=" + str(v), "median_us": round(med, 1), "min_us": round(mn, 1),
                    "GBps_median": round(nbytes / med / 1e3, 1), "frac": round(nbytes / med / 1e3 / 8000, 4)})
    out.sort(key=lambda r: r["median_us"])
    for r in out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
