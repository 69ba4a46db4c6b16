#!/usr/bin/env python3
"""Interleaved A/B sweep of the G-Counter join kernel knobs (one process).

Methodology (cdna_hip_programming.md §5.4 rule 24): all variants run in
interleaved rounds on the same device and inputs; report median and min of
the per-launch HIP-event time.  Also times torch's device copy of the same
bytes as a self-measured streaming reference.
"""
import itertools
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crdt_amd import _lib  # noqa: E402
from crdt_amd.engine import Engine  # noqa: E402


def timed(fn, reps=10):
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(reps + 1)]
    ev[0].record(s)
    for i in range(reps):
        fn()
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    return [ev[i].elapsed_time(ev[i + 1]) * 1e3 for i in range(reps)]  # us


def main():
    rows, nodes = int(os.environ.get("ROWS", 1_000_000)), 64
    eng = Engine(0)
    a = eng.synth_counters(1, 1, rows, nodes)
    b = eng.synth_counters(1, 2, rows, nodes)
    o = torch.empty_like(a)
    nbytes = 3 * rows * nodes * 8
    variants = list(itertools.product([1, 2, 4, 8], [0, 1], [1, 2, 4, 8, 16, 32]))
    res = {v: [] for v in variants}
    res["torch_copy"] = []
    big = torch.empty(rows * nodes * 3 // 2, dtype=torch.int64, device=eng.device)
    big2 = torch.empty_like(big)
    for rnd in range(5):
        for v in variants:
            u, nt, bpc = v
            _lib.call("crdt_set_option", b"join.unroll", u)
            _lib.call("crdt_set_option", b"join.nontemporal", nt)
            _lib.call("crdt_set_option", b"join.blocks_per_cu", bpc)
            res[v] += timed(lambda: eng.gcounter_join(a, b, out=o))
        res["torch_copy"] += timed(lambda: big2.copy_(big))  # reads+writes 2 * 768 MB = same bytes
    rows_out = []
    for v, ts in res.items():
        med, mn = float(np.median(ts)), float(np.min(ts))
        rows_out.append({"variant": str(v), "median_us": round(med, 2), "min_us": round(mn, 2),
                         "GBps_median": round(nbytes / med / 1e3, 1)})
    rows_out.sort(key=lambda r: r["median_us"])
    for r in rows_out:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
