#!/usr/bin/env python3
"""Host-side time split of the server_merge bench step: the five pulls'
ingest (crdt_server_ingest_binary) vs the batched merge (crdt_servers_merge)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from crdt_amd import engine as E  # noqa: E402


def main():
    eng = E.Engine(0)
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    wl = bench.ServerMerge(eng, 0, 1, reps, 10_000)
    t_in, t_m = [], []
    for _ in range(30):
        t0 = time.perf_counter()
        for s, body in zip(wl.srv, wl.bodies):
            assert s.IngestBinary(body) == 0
        t1 = time.perf_counter()
        wl.server.merge_servers(wl.srv)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        t_in.append(t1 - t0)
        t_m.append(t2 - t1)
    print(f"ingest x5 median {np.median(t_in) * 1e6:.1f} us, merge median {np.median(t_m) * 1e6:.1f} us, "
          f"entries {wl.n_r}")
    for s in wl.srv:
        s.close()
    eng.close()


if __name__ == "__main__":
    main()
