"""CPU: libcrdt_amd.so loads and exports every symbol include/crdt_amd.h
declares; host-only entry points behave; the product fails loudly without a
GPU (there is no CPU fallback)."""
import ctypes as C
import os
import re

import pytest

from crdt_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    with open(os.path.join(ROOT, "include", "crdt_amd.h")) as f:
        src = f.read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(crdt_\w+)\s*\(", src, flags=re.M)))


def test_header_declares_expected_surface():
    names = declared_functions()
    for must in ("crdt_gcounter_join", "crdt_vclock_classify", "crdt_lww_merge", "crdt_orset_merge",
                 "crdt_refmerge_batch", "crdt_compare_int64", "crdt_shard_range", "crdt_server_merge"):
        assert must in names, must


def test_library_exports_every_declared_symbol():
    lib = _lib.lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_table_matches_header():
    assert sorted(_lib.SIGNATURES) == declared_functions()


def test_abi_version_and_status_strings():
    lib = _lib.lib()
    assert lib.crdt_abi_version() == 1
    assert lib.crdt_status_str(0) == b"ok"
    assert lib.crdt_status_str(-5) == b"input not sorted"
    assert lib.crdt_status_str(-99) == b"unknown status"


@pytest.mark.parametrize("a,b,r", [(1, 2, -1), (2, 1, 1), (5, 5, 0), (-(2**63), 2**63 - 1, -1), (-1, 0, -1)])
def test_compare_is_signed_int64_comparator(a, b, r):
    # utils.Int64Comparator, main.go:106-107
    assert _lib.lib().crdt_compare_int64(a, b) == r


@pytest.mark.parametrize("rows,world", [(0, 1), (10, 3), (100_000_000, 8), (7, 8), (2**40 + 3, 7)])
def test_shard_range_partitions_rows(rows, world):
    lib = _lib.lib()
    prev = 0
    sizes = []
    for r in range(world):
        b, e = C.c_uint64(), C.c_uint64()
        assert lib.crdt_shard_range(rows, world, r, C.byref(b), C.byref(e)) == 0
        assert b.value == prev
        prev = e.value
        sizes.append(e.value - b.value)
    assert prev == rows and max(sizes) - min(sizes) <= 1


def test_shard_range_rejects_bad_args():
    lib = _lib.lib()
    b, e = C.c_uint64(), C.c_uint64()
    assert lib.crdt_shard_range(10, 0, 0, C.byref(b), C.byref(e)) == -1
    assert lib.crdt_shard_range(10, 2, 2, C.byref(b), C.byref(e)) == -1


def _diag_lib():
    path = os.path.join(ROOT, "crdt_amd", "libcrdt_amd_diag.so")
    lib = C.CDLL(path, mode=C.RTLD_LOCAL)
    lib.crdt_set_option.argtypes = [C.c_char_p, C.c_int64]
    lib.crdt_get_option.argtypes = [C.c_char_p, C.POINTER(C.c_int64)]
    return lib


def _knob_names():
    with open(os.path.join(ROOT, "crdt_amd", "csrc", "knobs.inc")) as f:
        return re.findall(r'^KNOB\(\w+, ([^,]+), "([\w.]+)"', f.read(), flags=re.M)


def test_product_refuses_every_option():
    """the product ABI carries no knobs, timing
    diagnostics or failpoints -- crdt_set_option refuses every name, even at
    the default value; crdt_get_option reports the compiled-in defaults."""
    lib = _lib.lib()
    assert _lib.get_option(b"build.diag") == 0
    knobs = _knob_names()
    assert len(knobs) > 40
    for default, name in knobs:
        assert _lib.get_option(name.encode()) == eval(default), name
        assert lib.crdt_set_option(name.encode(), eval(default)) == -1, name
    for name in (b"sort.rdd_diag", b"refmerge.diag_fold", b"fail.refmerge", b"fail.zero_bits", b"no.such.knob"):
        assert lib.crdt_set_option(name, 1) == -1
        assert lib.crdt_set_option(name, 0) == -1


def test_diag_build_option_validation():
    lib = _diag_lib()
    v = C.c_int64()
    assert lib.crdt_get_option(b"build.diag", C.byref(v)) == 0 and v.value == 1
    assert lib.crdt_set_option(b"join.unroll", 3) == -1
    assert lib.crdt_set_option(b"no.such.knob", 1) == -1
    assert lib.crdt_set_option(b"join.unroll", 2) == 0
    assert lib.crdt_get_option(b"join.unroll", C.byref(v)) == 0 and v.value == 2
    assert lib.crdt_set_option(b"join.unroll", 1) == 0
    assert lib.crdt_set_option(b"fail.refmerge", 1001) == -1
    assert lib.crdt_set_option(b"fail.refmerge", 0) == 0
    for default, name in _knob_names():          # every default is valid in its own table entry
        assert lib.crdt_set_option(name.encode(), eval(default)) == 0, name


def test_diag_build_d2_path_options():
    """The unsorted-merge forms' switches, diagnostic build:
    on / off accepted, anything else refused; each left at its default."""
    lib = _diag_lib()
    for name, default in ((b"sort.lww_table", 1), (b"sort.or_table", 1), (b"sort.or_lookback", 1),
                          (b"sort.sample_plan", 1)):
        assert lib.crdt_set_option(name, 2) == -1
        assert lib.crdt_set_option(name, -1) == -1
        assert lib.crdt_set_option(name, 1 - default) == 0
        assert lib.crdt_set_option(name, default) == 0
    assert lib.crdt_set_option(b"sort.sample_min", -1) == -1
    assert lib.crdt_set_option(b"sort.sample_min", 2**31) == -1
    assert lib.crdt_set_option(b"sort.sample_min", 1 << 20) == 0


def test_diag_build_exports_the_same_symbols():
    lib = _diag_lib()
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_null_context_is_invalid_not_a_crash():
    lib = _lib.lib()
    assert lib.crdt_gcounter_join(None, None, None, None, 1, 1) == -1
    assert lib.crdt_ctx_sync(None) == -1


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="needs a host without a GPU")
def test_no_gpu_fails_loudly():
    import torch  # noqa: F401
    from crdt_amd.engine import Engine
    with pytest.raises(_lib.CrdtLibraryError):
        Engine(0)
    ctx = C.c_void_p()
    assert _lib.lib().crdt_ctx_create(0, None, C.byref(ctx)) == -4   # CRDT_E_NODEV


def _ctx_functions():
    """(name, argtypes) of every declared entry point whose first parameter
    is the context."""
    with open(os.path.join(ROOT, "include", "crdt_amd.h")) as f:
        src = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    names = re.findall(r"^\s*int\s+(crdt_\w+)\s*\(\s*(?:const\s+)?crdt_ctx\s*\*", src, flags=re.M)
    return [(n, _lib.SIGNATURES[n][1]) for n in sorted(set(names))]


@pytest.mark.parametrize("name,argtypes", _ctx_functions(), ids=[n for n, _ in _ctx_functions()])
def test_every_device_entry_point_rejects_a_null_context(name, argtypes):
    """No entry point dereferences a NULL context: each returns a negative
    crdt_status (CRDT_E_INVAL) instead of crashing the host process."""
    zero = []
    for t in argtypes[1:]:
        zero.append(None if t in (C.c_void_p, C.c_char_p) or issubclass(t, C._Pointer) else 0)
    rc = getattr(_lib.lib(), name)(None, *zero)
    if name in ("crdt_ctx_destroy", "crdt_ctx_last_hip_error"):
        assert rc == 0                               # free(NULL)-like no-op / "no HIP error"
    else:
        assert rc < 0, f"{name} returned {rc}"


def _srv_functions():
    with open(os.path.join(ROOT, "include", "crdt_amd.h")) as f:
        src = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    names = re.findall(r"^\s*int\s+(crdt_server\w*)\s*\(\s*crdt_server\s*\*", src, flags=re.M)
    return [(n, _lib.SIGNATURES[n][1]) for n in sorted(set(names))]


@pytest.mark.parametrize("name,argtypes", _srv_functions(), ids=[n for n, _ in _srv_functions()])
def test_every_server_entry_point_rejects_a_null_server(name, argtypes):
    zero = [None if t in (C.c_void_p, C.c_char_p) or issubclass(t, C._Pointer) else 0 for t in argtypes[1:]]
    rc = getattr(_lib.lib(), name)(None, *zero)
    if name == "crdt_server_free":
        assert rc == 0                               # free(NULL)-like no-op
    elif name == "crdt_servers_merge":
        assert rc == 0                               # an empty batch
        assert _lib.lib().crdt_servers_merge(None, 1) == -1
    else:
        assert rc < 0, f"{name} returned {rc}"
