#!/usr/bin/env python3
"""Phase breakdown of the set-merge kernel from in-kernel s_memtime stamps.

Diagnostic build path (crdt_set_option("sets.stamps", 1)): per tile, 8 stamps
at the phase boundaries of k_set_merge.  Prints the median / p90 cycles of
each phase and the tile start skew.  Read SHARES, not absolute time: the
stamp path adds a drain and a barrier at the end of every tile.
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crdt_amd import _lib  # noqa: E402
from crdt_amd.engine import Engine, TupleSet  # noqa: E402

# stamp index pairs per phase, in kernel order (see STAMP(i) in csrc/sets.hip)
PAIRS = {"merge": (0, 1), "emit+scan": (1, 2), "copy-out k-2": (2, 3), "resolve+stage": (3, 4),
         "hold+release": (4, 5)}


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else "lww"
    for opt in sys.argv[2:]:                      # name=value kernel knobs
        k, v = opt.split("=")
        _lib.call("crdt_set_option", k.encode(), int(v))
    n, ks = 10_000_000, 8_000_000
    eng = Engine(0)
    A = eng.synth_set_tuples(2024, 0, n, ks)
    B = eng.synth_set_tuples(2024, 1, n, ks)
    out = TupleSet.empty(2 * n, eng.device)
    cnt = torch.zeros(1, dtype=torch.int64, device=eng.device)
    fn = eng.lww_merge if mode == "lww" else eng.orset_merge
    for _ in range(3):
        fn(A, B, out=out, count=cnt, trim=False)
    _lib.call("crdt_set_option", b"sets.stamps", 1)
    fn(A, B, out=out, count=cnt, trim=False)
    torch.cuda.synchronize()
    m = C.c_size_t()
    _lib.call("crdt_debug_set_stamps", eng.ctx, None, 0, C.byref(m))
    buf = np.zeros(m.value, dtype=np.uint64)
    _lib.call("crdt_debug_set_stamps", eng.ctx, buf.ctypes.data, m.value, C.byref(m))
    _lib.call("crdt_set_option", b"sets.stamps", 0)
    g, o = C.c_size_t(), C.c_int()
    _lib.call("crdt_debug_set_grid", C.byref(g), C.byref(o))
    print(f"grid {g.value} workgroups (occupancy query {o.value} per CU)")
    st = buf.reshape(-1, 16).astype(np.int64)
    print(f"{mode}: tiles={st.shape[0]}")
    for p, (a, b) in PAIRS.items():
        d = st[:, b] - st[:, a]
        print(f"  {p:12s} median {np.median(d):9.0f}  p90 {np.percentile(d, 90):9.0f} cycles")
    lb = st[:, 9] - st[:, 8]
    print(f"  {'ctl look-back':12s} median {np.median(lb):9.0f}  p90 {np.percentile(lb, 90):9.0f} cycles; "
          f"rounds median {np.median(st[:, 11]):.0f} max {st[:, 11].max()}, spinning rounds median "
          f"{np.median(st[:, 10]):.0f} p90 {np.percentile(st[:, 10], 90):.0f}")
    for nm, (x, y) in {"loader DMA": (12, 13)}.items():
        d = st[:, y] - st[:, x]
        print(f"  {nm:12s} median {np.median(d):9.0f}  p90 {np.percentile(d, 90):9.0f}")
    tot = st[:, 5] - st[:, 0]
    print(f"  {'total':12s} median {np.median(tot):9.0f}  p90 {np.percentile(tot, 90):9.0f}")


if __name__ == "__main__":
    main()
