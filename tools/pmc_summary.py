#!/usr/bin/env python3
"""Fold a tools/profile.sh run into committed evidence under profiles/.

    python tools/pmc_summary.py <workload> <kernel-substrings> [round-tag] [launches-per-step]

<kernel-substrings>: one substring, or several separated by commas for a
multi-kernel step (the first names the anchor kernel: its launch count is
the number of steps profiled; the counters of every matching kernel are
summed and divided by it, so the traffic covers the whole step like the
bench's whole-op bytes_per_launch).

Reads gpurun_out/prof_<workload>/{trace,pmc_fetch,pmc_write} and
  * copies the rocprofv3 --stats kernel summary to
    profiles/<round>_<workload>_kernel_stats.csv,
  * writes profiles/<round>_<workload>_pmc.json with the per-launch counters,
  * updates profiles/traffic.json[<workload>] (read by bench.py's roofline).

HBM bytes per launch follow MI355X_MICROARCH.md §HBM for gfx950: FETCH_SIZE
and WRITE_SIZE are in KiB; FETCH_SIZE counts HALF the bytes of a coalesced
read, so it is doubled; WRITE_SIZE is exact.  The guide calibrates 16 B/lane
accesses only; round 3 calibrated every width the merge kernels use
(tools/mb/pmc_cal.hip: 1, 2, 4, 8, 16 B/lane reads and LDS-DMA reads -> factor
2.00; 2, 4, 8, 16 B/lane stores -> 1.00, 1 B/lane stores 0.99;
profiles/r03/pmc_calibration.json), so one correction holds for the whole
step.  Scattered single-element loads (merge-path probes) fetch whole lines:
their traffic is real, not a counter artefact.
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_launch(path, kernel, counter):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def per_step(path, kernels, counter):
    """(sum over every kernel matching one of `kernels`) / launches of kernels[0]."""
    anchor = per_launch(path, kernels[0], counter)
    tot = 0.0
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] == counter and any(k in row["Kernel_Name"] for k in kernels):
                tot += float(row["Counter_Value"])
    return [tot / len(anchor)] * len(anchor) if anchor else []


def main():
    wl, kernel = sys.argv[1], sys.argv[2]
    tag = sys.argv[3] if len(sys.argv) > 3 else "r01"
    lps = int(sys.argv[4]) if len(sys.argv) > 4 else 1     # launches of the kernel per bench step
    src = os.path.join(ROOT, "gpurun_out", f"prof_{wl}")
    prof = os.path.join(ROOT, "profiles")
    os.makedirs(prof, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(prof, f"{tag}_{wl}_kernel_stats.csv"))
    kernels = kernel.split(",")
    fetch = per_step(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), kernels, "FETCH_SIZE")
    write = per_step(os.path.join(src, "pmc_write", "run_counter_collection.csv"), kernels, "WRITE_SIZE")
    with open(os.path.join(src, "bench_trace.json")) as f:
        bench = json.loads(f.read().strip().splitlines()[-1])
    algo = bench["roofline"]["bytes_per_launch"]
    fk = sum(fetch) / len(fetch)
    wk = sum(write) / len(write)
    hbm = (2 * fk * 1024 + wk * 1024) * lps          # per bench step, like bytes_per_launch
    # average duration of the kernel in the --stats summary
    avg_ns = None
    with open(os.path.join(src, "trace", "run_kernel_stats.csv")) as f:
        for row in csv.DictReader(f):
            if kernels[0] in row["Name"]:
                avg_ns = float(row["AverageNs"])
                break
    rec = {
        "workload": wl, "kernel": kernel, "launches_fetch": len(fetch), "launches_write": len(write),
        "launches_per_step": lps,
        "FETCH_SIZE_KiB_per_launch": fk, "WRITE_SIZE_KiB_per_launch": wk,
        "hbm_bytes_per_launch": int(round(hbm)), "bytes_per_launch_algorithmic": algo,
        "traffic_over_algorithmic": round(hbm / algo, 4),
        "correction": ("hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950: FETCH_SIZE counts 1/2 of coalesced reads "
                       "of every width the kernels use, WRITE_SIZE exact; profiles/r03/pmc_calibration.json)"),
        "rocprof_avg_duration_us": None if avg_ns is None else round(avg_ns / 1e3, 2),
        "bench_event_avg_launch_us": bench["roofline"]["avg_launch_us"],
        "config": bench["config"],
    }
    with open(os.path.join(prof, f"{tag}_{wl}_pmc.json"), "w") as f:
        json.dump(rec, f, indent=1)
    tp = os.path.join(prof, "traffic.json")
    try:
        with open(tp) as f:
            traffic = json.load(f)
    except (OSError, ValueError):
        traffic = {}
    traffic[wl] = {k: rec[k] for k in ("kernel", "hbm_bytes_per_launch", "bytes_per_launch_algorithmic",
                                        "traffic_over_algorithmic", "correction")}
    traffic[wl]["source"] = f"profiles/{tag}_{wl}_pmc.json"
    with open(tp, "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
