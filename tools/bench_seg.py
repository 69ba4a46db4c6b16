"""Micro-timing of the segmented primitives (gossip assembly) on a
gossip-shaped input: n length-1 segments whose codes walk two sources."""
import sys
import time

import numpy as np
import torch

from crdt_amd.engine import Engine


def _p(t):
    return None if t is None else t.data_ptr()


def main(n=16_000_000, reps=20):
    eng = Engine(0)
    dev = eng.device
    rng = np.random.default_rng(1)
    na = n // 2
    a_off = torch.arange(na + 1, dtype=torch.int64, device=dev)
    b_off = torch.arange(n - na + 1, dtype=torch.int64, device=dev)
    take_b = torch.from_numpy(rng.random(n) < 0.5).to(dev)
    ca = torch.cumsum(~take_b, 0) - 1
    cb = torch.cumsum(take_b, 0) - 1
    code = torch.where(take_b, -(cb + 1), ca.clamp(max=na - 1)).contiguous()
    a0 = torch.randint(0, 1 << 30, (n,), dtype=torch.int32, device=dev)
    a1 = torch.randint(0, 1 << 30, (n,), dtype=torch.int32, device=dev)
    off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    d0 = torch.empty(n + 1, dtype=torch.int32, device=dev)
    d1 = torch.empty_like(d0)
    cnt = torch.ones(n, dtype=torch.int32, device=dev)
    tests = {
        "counts_to_offsets": lambda: eng._call("crdt_counts_to_offsets", _p(cnt), n, 0, _p(off)),
        "seg_offsets": lambda: eng._call("crdt_seg_offsets", n, _p(code), _p(a_off), _p(b_off), 0, _p(off)),
        "seg_copy2_thread": lambda: eng._call("crdt_seg_copy2", n, _p(code), _p(a_off), _p(b_off), _p(off), 4,
                                              _p(a0), _p(a0), _p(d0), None, _p(a1), _p(a1), _p(d1), 0),
        "seg_gather2": lambda: eng._call("crdt_seg_gather2", n, _p(code), _p(a_off), _p(b_off), 0, _p(off), 4,
                                         _p(a0), _p(a0), _p(d0), _p(a1), _p(a1), _p(d1)),
    }
    from crdt_amd import _lib
    for items in (8, 4, 16):
        _lib.call("crdt_set_option", b"scan.items", items)
        print(f"-- scan.items={items}")
        run(tests, reps)


def run(tests, reps):
    for name, fn in tests.items():
        fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            fn()
        e.record()
        torch.cuda.synchronize()
        print(f"{name:20s} {s.elapsed_time(e) / reps * 1000:8.1f} us", flush=True)


if __name__ == "__main__":
    main(*[int(x) for x in sys.argv[1:]])
