#!/usr/bin/env python3
"""Writes tests/golden/refmerge_kat.json: hand-derived known-answer tests for
(*Server).merge() (/root/reference/main.go:35-100).

Every expected value below was derived BY HAND from the reference source
(walk main.go:45-73, replay main.go:75-98, strconv.Atoi/Itoa semantics),
not computed by any restatement: these vectors pin the oracle.  KAT-1..6
are SURVEY.md §8(c); KAT-7..15 extend them to the signed comparator, the
multi-key entries and Atoi's edge cases.

Entry format:  L = [[ts, "local"|"remote", {k: v}], ...]  (local = *Command)
               R = [[ts, {k: v}], ...]
"""
import json
import os

KATS = [
    dict(name="KAT-1", pins="remote ts > max(L) dropped; equal ts keeps local; local entries excluded",
         L=[[10, "local", {"a": "1"}], [20, "local", {"b": "2"}]],
         R=[[5, {"a": "3"}], [15, {"a": "4"}], [20, {"b": "9"}], [25, {"c": "7"}]],
         diff=[[5, "remote"], [10, "local"], [15, "remote"], [20, "local"]], state={"a": "7"}),
    dict(name="KAT-2", pins="empty local log ingests nothing; state rebuilt from empty",
         L=[], R=[[1, {"a": "5"}]], diff=[], state={}),
    dict(name="KAT-3", pins="verbatim singleton, parse-skip, '+5' parses",
         L=[[100, "local", {"z": "0"}]],
         R=[[1, {"a": "007"}], [2, {"b": "x"}], [3, {"b": "5"}], [4, {"c": "+5"}], [5, {"c": "-2"}]],
         diff=[[1, "remote"], [2, "remote"], [3, "remote"], [4, "remote"], [5, "remote"], [100, "local"]],
         state={"a": "007", "b": "5", "c": "3"}),
    dict(name="KAT-3b", pins="a non-int base freezes the key",
         L=[[100, "local", {"z": "0"}]], R=[[1, {"b": "5"}], [2, {"b": "x"}]],
         diff=[[1, "remote"], [2, "remote"], [100, "local"]], state={"b": "x"}),
    dict(name="KAT-4", pins="int64 wraparound of the sum",
         L=[[3, "local", {}]], R=[[1, {"a": "9223372036854775807"}], [2, {"a": "1"}]],
         diff=[[1, "remote"], [2, "remote"], [3, "local"]], state={"a": "-9223372036854775808"}),
    dict(name="KAT-4b", pins="Atoi range error -> skipped",
         L=[[3, "local", {}]], R=[[1, {"a": "9223372036854775808"}], [2, {"a": "1"}]],
         diff=[[1, "remote"], [2, "remote"], [3, "local"]], state={"a": "1"}),
    dict(name="KAT-5", pins="idempotence: re-merging KAT-1's R into KAT-1's output",
         L=[[5, "remote", {"a": "3"}], [10, "local", {"a": "1"}], [15, "remote", {"a": "4"}],
            [20, "local", {"b": "2"}]],
         R=[[5, {"a": "3"}], [15, {"a": "4"}], [20, {"b": "9"}], [25, {"c": "7"}]],
         diff=[[5, "remote"], [10, "local"], [15, "remote"], [20, "local"]], state={"a": "7"}),
    dict(name="KAT-6", pins="equal ts -> local value kept",
         L=[[10, "remote", {"a": "1"}], [20, "local", {}]], R=[[10, {"a": "100"}]],
         diff=[[10, "remote"], [20, "local"]], state={"a": "1"}),
    dict(name="KAT-7", pins="empty R: replay of the remote-origin history alone",
         L=[[1, "remote", {"a": "2"}], [2, "remote", {"a": "3"}]], R=[],
         diff=[[1, "remote"], [2, "remote"]], state={"a": "5"}),
    dict(name="KAT-8", pins="keys held only by local entries are absent",
         L=[[1, "local", {"q": "9"}], [5, "remote", {"r": "1"}]], R=[[3, {"s": "2"}]],
         diff=[[1, "local"], [3, "remote"], [5, "remote"]], state={"r": "1", "s": "2"}),
    dict(name="KAT-9", pins="multi-key entries fold per key",
         L=[[10, "local", {}]], R=[[1, {"a": "1", "b": "2"}], [2, {"a": "3"}]],
         diff=[[1, "remote"], [2, "remote"], [10, "local"]], state={"a": "4", "b": "2"}),
    dict(name="KAT-10", pins="signed Int64Comparator order (main.go:106)",
         L=[[-5, "local", {}], [3, "local", {}]],
         R=[[-10, {"a": "1"}], [-7, {"a": "2"}], [0, {"a": "4"}], [3, {"a": "8"}], [4, {"a": "16"}]],
         diff=[[-10, "remote"], [-7, "remote"], [-5, "local"], [0, "remote"], [3, "local"]], state={"a": "7"}),
    dict(name="KAT-11", pins="'-0' base verbatim alone; canonicalised once summed",
         L=[[9, "local", {}]], R=[[1, {"a": "5", "b": "-0"}], [2, {"a": "-0"}]],
         diff=[[1, "remote"], [2, "remote"], [9, "local"]], state={"a": "5", "b": "-0"}),
    dict(name="KAT-12", pins="ParseInt slow path: >=19 chars with leading zeros",
         L=[[9, "local", {}]], R=[[1, {"a": "00000000000000000000042"}], [2, {"a": "1"}]],
         diff=[[1, "remote"], [2, "remote"], [9, "local"]], state={"a": "43"}),
    dict(name="KAT-13", pins="empty string never parses; as base it freezes the key",
         L=[[9, "local", {}]], R=[[1, {"a": "", "b": "3"}], [2, {"a": "3", "b": ""}]],
         diff=[[1, "remote"], [2, "remote"], [9, "local"]], state={"a": "3", "b": ""}),
    dict(name="KAT-14", pins="base-10 only: '1_0', '0x10', ' 5', '5 ', '--1' never parse",
         L=[[99, "local", {}]],
         R=[[1, {"a": "1_0"}], [2, {"a": "0x10"}], [3, {"a": " 5"}], [4, {"a": "5 "}], [5, {"a": "--1"}],
            [6, {"a": "2"}]],
         diff=[[1, "remote"], [2, "remote"], [3, "remote"], [4, "remote"], [5, "remote"], [6, "remote"],
               [99, "local"]], state={"a": "2"}),
    dict(name="KAT-15", pins="most negative int64 parses; sum wraps negative-to-positive",
         L=[[99, "local", {}]], R=[[1, {"a": "-9223372036854775808"}], [2, {"a": "-1"}]],
         diff=[[1, "remote"], [2, "remote"], [99, "local"]], state={"a": "9223372036854775807"}),
]

if __name__ == "__main__":
    out = os.path.join(os.path.dirname(os.path.abspath(__file__)), "refmerge_kat.json")
    with open(out, "w") as f:
        json.dump({"source": "hand-derived from /root/reference/main.go:35-100 (see make_refmerge_kat.py)",
                   "kats": KATS}, f, indent=1)
    print(f"wrote {len(KATS)} KATs to {out}")
