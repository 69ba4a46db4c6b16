"""Loading the build-defined CRDT KATs (tests/golden/crdt_kat.json)."""
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def load():
    with open(os.path.join(HERE, "golden", "crdt_kat.json")) as f:
        return json.load(f)["kats"]


def u64(rows):
    return np.array(rows, dtype=np.uint64)


def tuples(rows):
    rows = list(rows)
    if not rows:
        return (np.zeros(0, np.uint64), np.zeros(0, np.uint64), np.zeros(0, np.uint32), np.zeros(0, np.uint8))
    a = np.array(rows, dtype=object)
    return (a[:, 0].astype(np.uint64), a[:, 1].astype(np.uint64), a[:, 2].astype(np.uint32),
            a[:, 3].astype(np.uint8))


def tuples_list(t):
    return [[int(k), int(ts), int(r), int(tb)] for k, ts, r, tb in zip(*t)]
