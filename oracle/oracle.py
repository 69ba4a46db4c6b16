"""numpy/ctypes front end of the CPU restatement (oracle/crdt_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by crdt_amd.  See crdt_oracle.h for the
reference file:line each function restates and for the parity status.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_lib = None


def build() -> None:
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        P = C.c_void_p
        S = C.c_size_t
        _lib.oc_go_atoi.argtypes = [C.c_char_p, S, C.POINTER(C.c_int64)]
        _lib.oc_go_atoi.restype = C.c_int
        _lib.oc_go_itoa.argtypes = [C.c_int64, C.c_char_p]
        _lib.oc_go_itoa.restype = C.c_int
        _lib.oc_gcounter_join.argtypes = [P, P, P, S, S, C.c_int]
        _lib.oc_gcounter_fold.argtypes = [P, S, S, P]
        _lib.oc_pncounter_value.argtypes = [P, P, P, S, S]
        _lib.oc_vclock_classify.argtypes = [P, P, P, S, S, C.c_int]
        _lib.oc_lww_merge.argtypes = [P, S, P, S, P]
        _lib.oc_lww_merge.restype = S
        _lib.oc_orset_merge.argtypes = [P, S, P, S, P]
        _lib.oc_orset_merge.restype = S
        _lib.oc_refmerge.argtypes = [P, P, P, S, P, P, S, P, P, P, P, C.c_uint32, P, P, P,
                                     C.POINTER(S), P, P, P]
        _lib.oc_refmerge.restype = C.c_int
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def _u64(a):
    return np.ascontiguousarray(a, dtype=np.uint64)


# ---------------------------------------------------------------- Go strconv
def go_atoi(s: str | bytes):
    b = s.encode() if isinstance(s, str) else s
    out = C.c_int64()
    ok = lib().oc_go_atoi(b, len(b), C.byref(out))
    return (True, out.value) if ok else (False, 0)


def go_itoa(v: int) -> str:
    buf = C.create_string_buffer(24)
    n = lib().oc_go_itoa(v, buf)
    return buf.raw[:n].decode()


# ---------------------------------------------------------------- counters / clocks
def gcounter_join(a, b, threads: int = 1) -> np.ndarray:
    a, b = _u64(a), _u64(b)
    out = np.empty_like(a)
    rows, nodes = a.shape
    lib().oc_gcounter_join(_p(a), _p(b), _p(out), rows, nodes, threads)
    return out


def gcounter_fold(a) -> np.ndarray:
    a = _u64(a)
    rows, nodes = a.shape
    out = np.empty(nodes, dtype=np.uint64)
    lib().oc_gcounter_fold(_p(a), rows, nodes, _p(out))
    return out


def pncounter_value(p, n) -> np.ndarray:
    p, n = _u64(p), _u64(n)
    rows, nodes = p.shape
    out = np.empty(rows, dtype=np.int64)
    lib().oc_pncounter_value(_p(p), _p(n), _p(out), rows, nodes)
    return out


def vclock_classify(a, b, threads: int = 1) -> np.ndarray:
    a, b = _u64(a), _u64(b)
    pairs, nodes = a.shape
    out = np.empty(pairs, dtype=np.uint8)
    lib().oc_vclock_classify(_p(a), _p(b), _p(out), pairs, nodes, threads)
    return out


# ---------------------------------------------------------------- sets
class _Tuples(C.Structure):
    _fields_ = [("key", C.c_void_p), ("ts", C.c_void_p), ("rep", C.c_void_p), ("tomb", C.c_void_p)]


def _soa(key, ts, rep, tomb):
    arrs = (_u64(key), _u64(ts), np.ascontiguousarray(rep, dtype=np.uint32),
            np.ascontiguousarray(tomb, dtype=np.uint8))
    return arrs, _Tuples(*(a.ctypes.data for a in arrs))


def _set_merge(fn, a, b):
    (aa, ca), (bb, cb) = _soa(*a), _soa(*b)
    n = len(aa[0]) + len(bb[0])
    outs, co = _soa(np.empty(n, np.uint64), np.empty(n, np.uint64), np.empty(n, np.uint32), np.empty(n, np.uint8))
    m = fn(C.byref(ca), len(aa[0]), C.byref(cb), len(bb[0]), C.byref(co))
    return tuple(x[:m] for x in outs)


def lww_merge(a, b):
    """a, b: (key, ts, rep, tomb) numpy tuples sorted by (key, ts, rep)."""
    return _set_merge(lib().oc_lww_merge, a, b)


def orset_merge(a, b):
    return _set_merge(lib().oc_orset_merge, a, b)


# ---------------------------------------------------------------- RefMerge
def refmerge_packed(l_ts, l_origin, l_kv, r_ts, r_kv, kv_key, kv_val, str_bytes, str_off, n_keys):
    """One replica, packed arrays (see crdt_oracle.h).  Returns
    (diff_ts, diff_origin, diff_src, st_kind, st_str, st_sum)."""
    l_ts = np.ascontiguousarray(l_ts, dtype=np.int64)
    l_origin = np.ascontiguousarray(l_origin, dtype=np.uint8)
    l_kv = np.ascontiguousarray(l_kv, dtype=np.uint32)
    r_ts = np.ascontiguousarray(r_ts, dtype=np.int64)
    r_kv = np.ascontiguousarray(r_kv, dtype=np.uint32)
    kv_key = np.ascontiguousarray(kv_key, dtype=np.uint32)
    kv_val = np.ascontiguousarray(kv_val, dtype=np.uint32)
    str_bytes = np.frombuffer(bytes(str_bytes), dtype=np.uint8) if not isinstance(str_bytes, np.ndarray) \
        else np.ascontiguousarray(str_bytes, dtype=np.uint8)
    if str_bytes.size == 0:
        str_bytes = np.zeros(1, np.uint8)
    str_off = np.ascontiguousarray(str_off, dtype=np.uint64)
    nl, nr = len(l_ts), len(r_ts)
    n = nl + nr
    o_ts = np.empty(max(n, 1), np.int64)
    o_or = np.empty(max(n, 1), np.uint8)
    o_src = np.empty(max(n, 1), np.int64)
    nk = max(int(n_keys), 1)
    kind = np.empty(nk, np.uint8)
    sstr = np.empty(nk, np.uint32)
    ssum = np.empty(nk, np.int64)
    on = C.c_size_t()
    rc = lib().oc_refmerge(_p(l_ts), _p(l_origin), _p(l_kv), nl, _p(r_ts), _p(r_kv), nr,
                           _p(kv_key), _p(kv_val), _p(str_bytes), _p(str_off), int(n_keys),
                           _p(o_ts), _p(o_or), _p(o_src), C.byref(on), _p(kind), _p(sstr), _p(ssum))
    if rc != 0:
        raise ValueError(f"oc_refmerge failed: {rc}")
    m = on.value
    return o_ts[:m], o_or[:m], o_src[:m], kind[:n_keys], sstr[:n_keys], ssum[:n_keys]
