#!/usr/bin/env python3
"""Calibration factors of rocprofv3 FETCH_SIZE / WRITE_SIZE per access width
(tools/mb/pmc_cal.hip under two separate --pmc passes).

    python tools/pmc_cal.py <fetch_counter_collection.csv> <write_counter_collection.csv> [out.json]

factor = true bytes / (counter KiB * 1024): multiply a kernel's counter by
the factor of its access width to get bytes.  Each kernel ran twice; the
second run is used (the first one also pays the page-table warm-up)."""
import csv
import json
import sys

BYTES = 1 << 30


def load(path, counter):
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"]
            out.setdefault(name, []).append(float(row["Counter_Value"]))
    return out


def width(name):
    if "read_lds_dma" in name:
        return "lds_dma16"
    for w in ("16", "8", "4", "2", "1"):
        if f"_w<{w}>" in name:
            return w
    return None


def main():
    fetch = load(sys.argv[1], "FETCH_SIZE")
    write = load(sys.argv[2], "WRITE_SIZE")
    res = {"bytes_per_kernel": BYTES, "read": {}, "write": {}}
    for name, v in fetch.items():
        if "read_" in name:
            kib = v[-1]
            res["read"][width(name)] = {"FETCH_SIZE_KiB": kib, "factor": round(BYTES / (kib * 1024), 4)}
    for name, v in write.items():
        if "write_w" in name:
            kib = v[-1]
            res["write"][width(name)] = {"WRITE_SIZE_KiB": kib, "factor": round(BYTES / (kib * 1024), 4)}
    res["note"] = ("factor = true bytes / counted bytes, per access width per lane (coalesced, 1 GiB, once); "
                   "MI355X_MICROARCH.md states 2.0 for 16 B/lane reads and 1.0 for 16 B/lane stores")
    out = sys.argv[3] if len(sys.argv) > 3 else None
    txt = json.dumps(res, indent=1, sort_keys=True)
    if out:
        with open(out, "w") as f:
            f.write(txt + "\n")
    print(txt)


if __name__ == "__main__":
    main()
