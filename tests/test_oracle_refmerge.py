"""CPU: the RefMerge oracle against the hand-derived KATs (pins the oracle).

Both restatements -- oracle/pyref.py (literal Python transliteration of
main.go:35-100) and oracle/crdt_oracle.c (the C checker the GPU tests use)
-- must reproduce every KAT in tests/golden/refmerge_kat.json, and agree
with each other on seeded config-A workloads.
"""
import pytest

from crdt_amd import synth
from oracle import oracle, pyref
from refmerge_util import diff_signature, kat_inputs, load_kats, oracle_merge

KATS = load_kats()


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_pyref_matches_kat(kat):
    diff, remote = kat_inputs(kat)
    new_diff, state = pyref.merge(diff, remote)
    assert diff_signature(new_diff) == kat["diff"]
    assert state == kat["state"]


@pytest.mark.parametrize("kat", KATS, ids=[k["name"] for k in KATS])
def test_c_oracle_matches_kat(kat):
    diff, remote = kat_inputs(kat)
    new_diff, state = oracle_merge(diff, remote)
    assert diff_signature(new_diff) == kat["diff"]
    assert state == kat["state"]


def test_kat5_is_kat1_remerged():
    k1 = next(k for k in KATS if k["name"] == "KAT-1")
    diff, remote = kat_inputs(k1)
    d1, s1 = pyref.merge(diff, remote)
    d2, s2 = pyref.merge(d1, remote)
    assert diff_signature(d2) == diff_signature(d1) and s2 == s1


@pytest.mark.parametrize("seed", [1, 2, 3])
def test_c_oracle_matches_pyref_on_demo(seed):
    for diff, remote in synth.refmerge_demo(seed, replicas=3, entries=1500, multi_key=0.2):
        d_py, s_py = pyref.merge(diff, remote)
        d_c, s_c = oracle_merge(diff, remote)
        assert diff_signature(d_c) == diff_signature(d_py)
        assert all(d_c[t] is d_py[t] for t in d_py)
        assert s_c == s_py


def test_refmerge_not_commutative():
    # the reference is asymmetric (truncation at max(L), local origin excluded)
    a = {1: {"x": "1"}, 5: {"x": "2"}}
    b = {2: {"x": "4"}, 9: {"x": "8"}}
    _, s_ab = pyref.merge(a, b)
    _, s_ba = pyref.merge(b, a)
    assert s_ab == {"x": "7"} and s_ba == {"x": "15"}


@pytest.mark.parametrize("s,ok,v", [
    ("0", True, 0), ("-0", True, 0), ("+7", True, 7), ("007", True, 7), ("9223372036854775807", True, 2**63 - 1),
    ("-9223372036854775808", True, -(2**63)), ("9223372036854775808", False, 0), ("", False, 0), ("+", False, 0),
    ("-", False, 0), ("1_0", False, 0), ("0x1", False, 0), (" 1", False, 0), ("1 ", False, 0),
    ("18446744073709551616", False, 0), ("00000000000000000000000000042", True, 42), ("-00000000000000000000001", True, -1),
    ("١", False, 0),
])
def test_go_atoi_edges(s, ok, v):
    assert oracle.go_atoi(s) == (ok, v)
    assert pyref.go_atoi(s) == (ok, v)
