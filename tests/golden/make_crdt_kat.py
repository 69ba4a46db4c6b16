#!/usr/bin/env python3
"""Writes tests/golden/crdt_kat.json: hand-derived known answers for the
build-defined CRDT joins (no reference code exists for them).

Expected values are written by hand from the definitions in DESIGN.md
(elementwise unsigned max; PN value with uint64 wrap read as int64; clock
classification; LWW max (ts, rep) with the left operand winning an exact tie,
mirroring main.go:54-65; OR-Set tag union with tombstones OR-ed).
"""
import json
import os

M = 2**64 - 1
H = 2**63

KATS = {
    "gcounter_join": [
        {"a": [[1, 5], [M, 0]], "b": [[3, 2], [7, H]], "out": [[3, 5], [M, H]]},
        {"a": [[0]], "b": [[0]], "out": [[0]]},
        {"a": [[H - 1, H]], "b": [[H, H - 1]], "out": [[H, H]]},
    ],
    "gcounter_fold": [
        {"a": [[1, 5], [3, 2], [0, 9]], "out": [3, 9]},
        {"a": [[H, 1], [H - 1, M]], "out": [H, M]},
    ],
    "pncounter_value": [
        {"p": [[5, 3]], "n": [[2, 10]], "out": [-4]},
        {"p": [[M, 2]], "n": [[0, 0]], "out": [1]},
        {"p": [[H, 0]], "n": [[0, 0]], "out": [-H]},
        {"p": [[0, 0]], "n": [[1, 0]], "out": [-1]},
    ],
    "vclock_classify": [
        {"a": [[1, 2]], "b": [[1, 2]], "out": [0]},
        {"a": [[1, 2]], "b": [[1, 3]], "out": [1]},
        {"a": [[2, 2]], "b": [[1, 2]], "out": [2]},
        {"a": [[2, 1]], "b": [[1, 2]], "out": [3]},
        {"a": [[H]], "b": [[5]], "out": [2]},
        {"a": [[M, 0, 0]], "b": [[M, 0, 1]], "out": [1]},
    ],
    # tuples: [key, ts, rep, tomb]
    "lww_merge": [
        {"a": [[1, 5, 0, 0]], "b": [[1, 5, 0, 1]], "out": [[1, 5, 0, 0]]},
        {"a": [[1, 5, 0, 0]], "b": [[1, 5, 1, 1]], "out": [[1, 5, 1, 1]]},
        {"a": [[1, 3, 0, 0], [2, 1, 0, 1]], "b": [[1, 4, 0, 1], [3, 0, 0, 0]],
         "out": [[1, 4, 0, 1], [2, 1, 0, 1], [3, 0, 0, 0]]},
        {"a": [[7, 1, 0, 0], [7, 9, 2, 1]], "b": [[7, 9, 2, 0]], "out": [[7, 9, 2, 1]]},
        {"a": [], "b": [[4, 1, 1, 1], [4, 1, 1, 0]], "out": [[4, 1, 1, 1]]},
        {"a": [[M, M, 2**32 - 1, 0]], "b": [[M, 0, 0, 1]], "out": [[M, M, 2**32 - 1, 0]]},
    ],
    "orset_merge": [
        {"a": [[1, 1, 0, 0], [1, 2, 0, 1]], "b": [[1, 1, 0, 1], [2, 1, 0, 0]],
         "out": [[1, 1, 0, 1], [1, 2, 0, 1], [2, 1, 0, 0]]},
        {"a": [[5, 5, 5, 0]], "b": [[5, 5, 5, 0]], "out": [[5, 5, 5, 0]]},
        {"a": [], "b": [], "out": []},
        {"a": [[3, 1, 0, 0], [3, 1, 0, 0]], "b": [[3, 1, 0, 1]], "out": [[3, 1, 0, 1]]},
    ],
}

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "crdt_kat.json")
    with open(out, "w") as f:
        json.dump({"source": "hand-derived (see make_crdt_kat.py)", "kats": KATS}, f, indent=1)
    print(f"wrote {sum(len(v) for v in KATS.values())} KATs to {out}")
