#!/usr/bin/env python3
"""Where a bench step's wall time goes, from a rocprofv3 run with
--kernel-trace --memory-copy-trace --output-format csv:

    python tools/timeline.py <dir with run_kernel_trace.csv [, run_memory_copy_trace.csv]> [steps] [--seq]

Takes the last complete step (between the marker kernels bench.py launches
under CRDT_TRACE_MARK=1; else about the last 1/steps of the trace), and prints
its span, the time some kernel or copy was running (busy), the idle gaps,
the number of kernels / copies, and the top kernels and copy kinds by total
time in that window; --seq also lists the window's events in order (start
offset, idle gap before it, duration, name)."""
import collections
import csv
import os
import sys


def rows(path, kind):
    if not os.path.exists(path):
        return []
    out = []
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name") or r.get("Name") or r.get("Direction") or kind
        if kind == "copy":
            name = "copy " + (r.get("Direction") or r.get("Kind") or "?")
        out.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kind, name))
    return out


def main():
    args = [a for a in sys.argv[1:] if a != "--seq"]
    seq = "--seq" in sys.argv
    d = args[0]
    steps = int(args[1]) if len(args) > 1 else 10
    ev = rows(os.path.join(d, "run_kernel_trace.csv"), "kernel") + rows(os.path.join(d, "run_memory_copy_trace.csv"),
                                                                         "copy")
    ev.sort()
    if not ev:
        raise SystemExit("no trace rows")
    # steps are delimited by the marker kernel bench.py launches before each
    # timed step under CRDT_TRACE_MARK=1 (crdt_stream_copy of 512 B); the
    # window is the last complete step (marker to marker)
    marks = [e[0] for e in ev if "stream_copy" in e[3]]
    if len(marks) >= 2:
        w0, w1 = marks[-2], marks[-1]
    else:
        t_end = max(e[1] for e in ev)
        w0, w1 = t_end - (t_end - ev[0][0]) // (steps + 2), t_end + 1
    win = [e for e in ev if w0 <= e[0] < w1 and "stream_copy" not in e[3]]
    span = (w1 if len(marks) >= 2 else max(e[1] for e in win)) - w0
    busy, cur_s, cur_e = 0, None, None
    for s, e, _, _ in win:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    tot = collections.Counter()
    cnt = collections.Counter()
    for s, e, k, n in win:
        tot[n] += e - s
        cnt[n] += 1
    nk = sum(1 for e in win if e[2] == "kernel")
    nc = sum(1 for e in win if e[2] == "copy")
    print(f"window {span / 1e3:.1f} us: busy {busy / 1e3:.1f} us, idle {(span - busy) / 1e3:.1f} us; "
          f"{nk} kernels, {nc} copies")
    for n, t in tot.most_common(25):
        print(f"  {t / 1e3:9.1f} us  x{cnt[n]:<5} {n[:90]}")
    if seq:
        prev_end = w0
        for s, e, k, n in win:
            print(f"  +{(s - w0) / 1e3:8.1f} us  gap {(s - prev_end) / 1e3:7.1f}  {(e - s) / 1e3:8.1f} us  {n[:80]}")
            prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
