"""ctypes binding of libcrdt_amd.so -- the C-ABI declared in include/crdt_amd.h.

The shared library is built in-tree (``crdt_amd/libcrdt_amd.so``) by
``__graft_entry__.build()``.  There is deliberately NO fallback: if the
library is missing or cannot be loaded, every product entry point raises
:class:`CrdtLibraryError` (a CPU path would void the parity claims).

``torch`` is imported before the library is opened so that the library's
``libamdhip64.so.7`` dependency resolves to the HIP runtime torch already
loaded (same SONAME): one HIP runtime per process, so torch's device
pointers and streams are valid inside the library.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import torch  # noqa: F401  (load order: torch's HIP runtime first)

# CRDT_AMD_DIAG=1: the diagnostic build (libcrdt_amd_diag.so, -DCRDT_DIAG:
# settable kernel knobs, timing diagnostics, failpoints) -- the knob-variant
# tests (tests/test_gpu_diag_build.py runs them in a child process) and A/B
# tools.  CRDT_AMD_LIB: another build of the same library (A/B timing of two
# builds in one GPU call, tools/ab_build.sh).  Neither is set for the product
# tests, smoke or bench lines.
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CRDT_AMD_LIB") or os.path.join(
    _HERE, "libcrdt_amd_diag.so" if os.environ.get("CRDT_AMD_DIAG") == "1" else "libcrdt_amd.so")

CRDT_OK = 0
STATUS_NAMES = {
    0: "CRDT_OK",
    -1: "CRDT_E_INVAL",
    -2: "CRDT_E_HIP",
    -3: "CRDT_E_NOMEM",
    -4: "CRDT_E_NODEV",
    -5: "CRDT_E_UNSORTED",
    -6: "CRDT_E_RANGE",
    -7: "CRDT_E_COMM",
    -8: "CRDT_E_DEVICE",
}


class CrdtLibraryError(RuntimeError):
    """libcrdt_amd.so is missing or failed to load (no silent fallback)."""


class CrdtError(RuntimeError):
    """A C-ABI call returned a negative crdt_status."""

    def __init__(self, fn: str, status: int, hip_error: int = 0):
        self.status = status
        self.hip_error = hip_error
        name = STATUS_NAMES.get(status, str(status))
        msg = f"{fn} failed: {name}"
        if hip_error:
            msg += f" (hipError {hip_error})"
        super().__init__(msg)


class crdt_set_plan(C.Structure):
    """Opaque plan of a stream-ordered D2 merge (crdt_set_merge_plan)."""
    _fields_ = [("w", C.c_uint64 * 24)]


class crdt_tuples(C.Structure):
    _fields_ = [("key", C.c_void_p), ("ts", C.c_void_p), ("rep", C.c_void_p), ("tomb", C.c_void_p)]


class crdt_refmerge_in(C.Structure):
    _fields_ = [
        ("replicas", C.c_uint32), ("n_slots", C.c_uint32),
        ("n_l", C.c_uint64), ("n_r", C.c_uint64), ("n_kv", C.c_uint64), ("n_str", C.c_uint64),
        ("l_off", C.c_void_p), ("l_ts", C.c_void_p), ("l_origin", C.c_void_p), ("l_kv", C.c_void_p),
        ("r_off", C.c_void_p), ("r_ts", C.c_void_p), ("r_kv", C.c_void_p),
        ("kv_key", C.c_void_p), ("kv_val", C.c_void_p),
        ("str_bytes", C.c_void_p), ("str_off", C.c_void_p),
    ]


class crdt_refmerge_out(C.Structure):
    _fields_ = [
        ("off", C.c_void_p), ("ts", C.c_void_p), ("origin", C.c_void_p), ("src", C.c_void_p),
        ("st_kind", C.c_void_p), ("st_str", C.c_void_p), ("st_sum", C.c_void_p),
    ]


class crdt_refmerge_kv_out(C.Structure):
    _fields_ = [("kv_off", C.c_void_p), ("kv_key", C.c_void_p), ("kv_val", C.c_void_p), ("kv_cap", C.c_uint64)]


class crdt_refmerge_pull(C.Structure):
    _fields_ = [("r_end", C.c_void_p), ("r_slot_delta", C.c_void_p)]


class crdt_replay_state(C.Structure):
    _fields_ = [("best_key", C.c_void_p), ("best_str", C.c_void_p), ("sum", C.c_void_p), ("npar", C.c_void_p),
                ("nhold", C.c_void_p)]


class crdt_local_in(C.Structure):
    _fields_ = [
        ("replicas", C.c_uint32), ("n_slots", C.c_uint32),
        ("n_l", C.c_uint64), ("n_c", C.c_uint64), ("n_kv", C.c_uint64), ("n_str", C.c_uint64),
        ("l_off", C.c_void_p), ("l_ts", C.c_void_p), ("l_origin", C.c_void_p),
        ("c_off", C.c_void_p), ("c_ts", C.c_void_p), ("c_kv", C.c_void_p),
        ("kv_key", C.c_void_p), ("kv_val", C.c_void_p), ("str_bytes", C.c_void_p), ("str_off", C.c_void_p),
    ]


class crdt_local_out(C.Structure):
    _fields_ = [("off", C.c_void_p), ("ts", C.c_void_p), ("origin", C.c_void_p), ("src", C.c_void_p),
                ("status", C.c_void_p), ("st_kind", C.c_void_p), ("st_str", C.c_void_p), ("st_sum", C.c_void_p)]


class crdt_gossip_bodies(C.Structure):
    _fields_ = [("n_bodies", C.c_uint32), ("key_cap", C.c_uint32), ("kv_base", C.c_uint64), ("data", C.c_void_p),
                ("body_off", C.c_void_p), ("slot_base", C.c_void_p), ("host_hdr", C.c_void_p)]


class crdt_gossip_decoded(C.Structure):
    _fields_ = [("r_off", C.c_void_p), ("r_ts", C.c_void_p), ("r_kv", C.c_void_p), ("kv_key", C.c_void_p),
                ("kv_val", C.c_void_p)]


class crdt_refmerge_acc(C.Structure):
    _fields_ = [("best", C.c_void_p), ("sum", C.c_void_p), ("npar", C.c_void_p)]


class crdt_population_cmds(C.Structure):
    _fields_ = [("c_off", C.c_void_p), ("c_ts", C.c_void_p), ("c_kv", C.c_void_p), ("kv_key", C.c_void_p),
                ("kv_val", C.c_void_p)]


class crdt_population_init(C.Structure):
    _fields_ = [("replicas", C.c_uint32), ("keys_per_replica", C.c_uint32), ("first", C.c_uint64),
                ("n_str", C.c_uint64), ("l_off", C.c_void_p), ("l_ts", C.c_void_p), ("l_origin", C.c_void_p),
                ("l_kv", C.c_void_p), ("kv_key", C.c_void_p), ("kv_val", C.c_void_p), ("str_bytes", C.c_void_p),
                ("str_off", C.c_void_p)]


_P = C.c_void_p
_SZ = C.c_size_t
_U64 = C.c_uint64
_I = C.c_int
_CTX = C.c_void_p

# name -> (restype, argtypes); exactly the functions include/crdt_amd.h declares.
SIGNATURES = {
    "crdt_abi_version": (_I, []),
    "crdt_status_str": (C.c_char_p, [_I]),
    "crdt_device_count": (_I, [C.POINTER(_I)]),
    "crdt_ctx_create": (_I, [_I, _P, C.POINTER(_P)]),
    "crdt_ctx_destroy": (_I, [_CTX]),
    "crdt_ctx_set_stream": (_I, [_CTX, _P]),
    "crdt_stream_create": (_I, [_I, C.POINTER(_P)]),
    "crdt_stream_destroy": (_I, [_P]),
    "crdt_ctx_sync": (_I, [_CTX]),
    "crdt_ctx_device_status": (_I, [_CTX, C.POINTER(C.c_uint32), C.c_int]),
    "crdt_ctx_last_hip_error": (_I, [_CTX]),
    "crdt_ctx_reserve": (_I, [_CTX, _SZ]),
    "crdt_set_option": (_I, [C.c_char_p, C.c_int64]),
    "crdt_get_option": (_I, [C.c_char_p, C.POINTER(C.c_int64)]),
    "crdt_dev_alloc": (_I, [_CTX, _SZ, C.POINTER(_P)]),
    "crdt_dev_free": (_I, [_CTX, _P]),
    "crdt_memcpy_h2d": (_I, [_CTX, _P, _P, _SZ]),
    "crdt_memcpy_d2h": (_I, [_CTX, _P, _P, _SZ]),
    "crdt_memset": (_I, [_CTX, _P, _I, _SZ]),
    "crdt_compare_int64": (_I, [C.c_int64, C.c_int64]),
    "crdt_gcounter_join": (_I, [_CTX, _P, _P, _P, _SZ, _SZ]),
    "crdt_gcounter_fold": (_I, [_CTX, _P, _SZ, _SZ, _P]),
    "crdt_gcounter_value": (_I, [_CTX, _P, _SZ, _SZ, _P]),
    "crdt_stream_copy": (_I, [_CTX, _P, _P, _SZ, _I, _I]),
    "crdt_stream_read": (_I, [_CTX, _P, _SZ, _P, _SZ, _I, _I]),
    "crdt_pncounter_join": (_I, [_CTX, _P, _P, _P, _P, _P, _P, _SZ, _SZ]),
    "crdt_pncounter_value": (_I, [_CTX, _P, _P, _P, _SZ, _SZ]),
    "crdt_vclock_classify": (_I, [_CTX, _P, _P, _P, _SZ, _SZ]),
    "crdt_lww_merge": (_I, [_CTX, C.POINTER(crdt_tuples), _SZ, C.POINTER(crdt_tuples), _SZ,
                            C.POINTER(crdt_tuples), _P]),
    "crdt_orset_merge": (_I, [_CTX, C.POINTER(crdt_tuples), _SZ, C.POINTER(crdt_tuples), _SZ,
                              C.POINTER(crdt_tuples), _P]),
    "crdt_lww_merge_unsorted": (_I, [_CTX, C.POINTER(crdt_tuples), _SZ, C.POINTER(crdt_tuples), _SZ,
                                     C.POINTER(crdt_tuples), _P]),
    "crdt_orset_merge_unsorted": (_I, [_CTX, C.POINTER(crdt_tuples), _SZ, C.POINTER(crdt_tuples), _SZ,
                                       C.POINTER(crdt_tuples), _P]),
    "crdt_set_merge_plan": (_I, [_CTX, _I, C.POINTER(crdt_tuples), _SZ, C.POINTER(crdt_tuples), _SZ, C.c_uint32,
                                 C.POINTER(crdt_set_plan)]),
    "crdt_lww_merge_unsorted_planned": (_I, [_CTX, C.POINTER(crdt_set_plan), C.POINTER(crdt_tuples), _SZ,
                                             C.POINTER(crdt_tuples), _SZ, C.POINTER(crdt_tuples), _P]),
    "crdt_orset_merge_unsorted_planned": (_I, [_CTX, C.POINTER(crdt_set_plan), C.POINTER(crdt_tuples), _SZ,
                                               C.POINTER(crdt_tuples), _SZ, C.POINTER(crdt_tuples), _P]),
    "crdt_tuples_sort": (_I, [_CTX, C.POINTER(crdt_tuples), _SZ, C.POINTER(crdt_tuples)]),
    "crdt_u64_lower_bound": (_I, [_CTX, _P, _SZ, _P, _SZ, _P]),
    "crdt_tuples_count_unsorted": (_I, [_CTX, C.POINTER(crdt_tuples), _SZ, _P]),
    "crdt_tuples_merge": (_I, [_CTX, C.POINTER(crdt_tuples), _SZ, C.POINTER(crdt_tuples), _SZ,
                               C.POINTER(crdt_tuples)]),
    "crdt_refmerge_batch": (_I, [_CTX, C.POINTER(crdt_refmerge_in), C.POINTER(crdt_refmerge_out)]),
    "crdt_atoi_batch": (_I, [_CTX, _P, _P, _U64, _P, _P]),
    "crdt_local_apply": (_I, [_CTX, C.POINTER(crdt_local_in), C.POINTER(crdt_local_out)]),
    "crdt_refmerge_batch_kv": (_I, [_CTX, C.POINTER(crdt_refmerge_in), C.POINTER(crdt_refmerge_out),
                                    C.POINTER(crdt_refmerge_kv_out)]),
    "crdt_refmerge_batch_pull": (_I, [_CTX, C.POINTER(crdt_refmerge_in), C.POINTER(crdt_refmerge_out),
                                      C.POINTER(crdt_refmerge_pull), C.POINTER(crdt_refmerge_kv_out)]),
    "crdt_refmerge_batch_ex": (_I, [_CTX, C.POINTER(crdt_refmerge_in), C.POINTER(crdt_refmerge_out), _P,
                                    C.POINTER(crdt_refmerge_acc)]),
    "crdt_refmerge_local_maxl": (_I, [_CTX, C.POINTER(crdt_refmerge_in), _P]),
    "crdt_replay_state_init": (_I, [_CTX, C.POINTER(crdt_refmerge_in), C.POINTER(crdt_replay_state)]),
    "crdt_refmerge_delta": (_I, [_CTX, C.POINTER(crdt_refmerge_in), C.POINTER(crdt_refmerge_out),
                                 C.POINTER(crdt_replay_state)]),
    "crdt_refmerge_acc_rank": (_I, [_CTX, C.POINTER(crdt_refmerge_acc), _SZ, C.c_uint32, _P]),
    "crdt_refmerge_acc_owner_str": (_I, [_CTX, C.POINTER(crdt_refmerge_acc), _SZ, _P, _P, _P]),
    "crdt_refmerge_acc_set_best": (_I, [_CTX, C.POINTER(crdt_refmerge_acc), _SZ, _P, _P]),
    "crdt_refmerge_finalize": (_I, [_CTX, C.POINTER(crdt_refmerge_acc), _SZ, _P, _P, _U64,
                                    C.POINTER(crdt_refmerge_out)]),
    "crdt_server_new": (_I, [_CTX, _I, C.POINTER(_P)]),
    "crdt_server_free": (_I, [_P]),
    "crdt_server_init_state": (_I, [_P, _P, _P, _P, _P, _SZ]),
    "crdt_server_diff_put": (_I, [_P, C.c_int64, _I, _P, _P, _P, _P, _SZ]),
    "crdt_server_remote_put": (_I, [_P, C.c_int64, _P, _P, _P, _P, _SZ]),
    "crdt_server_add_command": (_I, [_P, C.c_int64, _P, _P, _P, _P, _SZ, C.POINTER(_I)]),
    "crdt_server_merge": (_I, [_P]),
    "crdt_servers_merge": (_I, [C.POINTER(_P), _SZ]),
    "crdt_server_diff_len": (_I, [_P, C.POINTER(_SZ)]),
    "crdt_server_remote_len": (_I, [_P, C.POINTER(_SZ)]),
    "crdt_server_diff_keys": (_I, [_P, _P, _P, _SZ, C.POINTER(_SZ)]),
    "crdt_seg_offsets": (_I, [_CTX, _SZ, _P, _P, _P, _U64, _P]),
    "crdt_seg_copy": (_I, [_CTX, _SZ, _P, _P, _P, _P, _SZ, _P, _P, _P, _P, _I]),
    "crdt_seg_copy2": (_I, [_CTX, _SZ, _P, _P, _P, _P, _SZ, _P, _P, _P, _P, _P, _P, _P, _I]),
    "crdt_seg_gather2": (_I, [_CTX, _SZ, _P, _P, _P, _U64, _P, _SZ, _P, _P, _P, _P, _P, _P]),
    "crdt_seg_gather2_n": (_I, [_CTX, _SZ, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "crdt_seg_fill_u32": (_I, [_CTX, _SZ, _P, _P, _P]),
    "crdt_counts_to_offsets": (_I, [_CTX, _P, _SZ, _U64, _P]),
    "crdt_offsets_to_counts": (_I, [_CTX, _P, _SZ, _P]),
    "crdt_server_gossip_json": (_I, [_P, C.c_char_p, _SZ, C.POINTER(_SZ), C.POINTER(C.c_int)]),
    "crdt_server_ingest_json": (_I, [_P, C.c_char_p, _SZ, C.POINTER(C.c_int)]),
    "crdt_server_gossip_binary": (_I, [_P, C.c_char_p, _SZ, C.POINTER(_SZ), C.POINTER(C.c_int)]),
    "crdt_server_ingest_binary": (_I, [_P, C.c_char_p, _SZ, C.POINTER(C.c_int)]),
    "crdt_server_set_alive": (_I, [_P, _I]),
    "crdt_strtab_create": (_I, [_CTX, _SZ, _SZ, C.POINTER(_P)]),
    "crdt_strtab_destroy": (_I, [_P]),
    "crdt_strtab_info": (_I, [_P, C.POINTER(_U64), C.POINTER(_U64), C.POINTER(_P), C.POINTER(_P)]),
    "crdt_strtab_get": (_I, [_P, _U64, C.POINTER(_P), C.POINTER(_SZ)]),
    "crdt_strtab_intern": (_I, [_CTX, _P, _P, _P, _SZ, _P]),
    "crdt_gossip_decode": (_I, [_CTX, C.POINTER(crdt_gossip_bodies), _P, _P, C.POINTER(crdt_gossip_decoded),
                                C.POINTER(C.c_uint32)]),
    "crdt_server_remote_keys": (_I, [_P, _P, _SZ, C.POINTER(_SZ)]),
    "crdt_server_entry_at": (_I, [_P, _I, C.c_int64, _SZ, C.POINTER(C.c_void_p), C.POINTER(_SZ),
                                 C.POINTER(C.c_void_p), C.POINTER(_SZ), C.POINTER(_SZ)]),
    "crdt_server_state_len": (_I, [_P, C.POINTER(_SZ)]),
    "crdt_server_state_at": (_I, [_P, _SZ, C.POINTER(C.c_void_p), C.POINTER(_SZ), C.POINTER(C.c_void_p),
                                  C.POINTER(_SZ)]),
    "crdt_shard_range": (_I, [_U64, _I, _I, C.POINTER(_U64), C.POINTER(_U64)]),
    "crdt_u64_to_ordered_i64": (_I, [_CTX, _P, _P, _SZ]),
    "crdt_ordered_i64_to_u64": (_I, [_CTX, _P, _P, _SZ]),
    "crdt_shard_unique_id": (_I, [_P, _SZ]),
    "crdt_shard_comm_create": (_I, [C.POINTER(_I), _I, C.POINTER(_P)]),
    "crdt_shard_comm_init_rank": (_I, [_CTX, _P, _I, _I, C.POINTER(_P)]),
    "crdt_shard_comm_create_loopback": (_I, [_I, _I, C.POINTER(_P)]),
    "crdt_shard_comm_transport": (_I, [_P, C.POINTER(_I)]),
    "crdt_rccl_info": (_I, [C.POINTER(_I), C.c_char_p, C.c_size_t]),
    "crdt_shard_comm_destroy": (_I, [_P]),
    "crdt_shard_comm_info": (_I, [_P, C.POINTER(_I), C.POINTER(_I), C.POINTER(_I)]),
    "crdt_shard_member_ctx": (_I, [_P, _I, C.POINTER(_P)]),
    "crdt_shard_comm_last_error": (_I, [_P]),
    "crdt_shard_sync": (_I, [_P]),
    "crdt_shard_fold_max_u64": (_I, [_P, C.POINTER(_P), C.POINTER(_SZ), _SZ, C.POINTER(_P)]),
    "crdt_shard_allreduce_max_u64": (_I, [_P, C.POINTER(_P), _SZ]),
    "crdt_shard_allreduce": (_I, [_P, C.POINTER(_P), _SZ, _I, _I]),
    "crdt_shard_set_allgather_v": (_I, [_P, C.POINTER(crdt_tuples), C.POINTER(_SZ), C.POINTER(crdt_tuples), _SZ,
                                        C.POINTER(_SZ)]),
    "crdt_shard_lww_merge": (_I, [_P, C.POINTER(crdt_tuples), _SZ, C.POINTER(crdt_tuples), _SZ,
                                  C.POINTER(crdt_tuples), _SZ, C.POINTER(_SZ)]),
    "crdt_shard_orset_merge": (_I, [_P, C.POINTER(crdt_tuples), _SZ, C.POINTER(crdt_tuples), _SZ,
                                    C.POINTER(crdt_tuples), _SZ, C.POINTER(_SZ)]),
    "crdt_shard_alltoallv": (_I, [_P, C.POINTER(_P), C.POINTER(_SZ), C.POINTER(_P), C.POINTER(_SZ), _SZ]),
    "crdt_shard_lww_merge_local": (_I, [_P, C.POINTER(crdt_tuples), C.POINTER(_SZ), C.POINTER(crdt_tuples),
                                        C.POINTER(_SZ), C.POINTER(crdt_tuples), _SZ, C.POINTER(_SZ), _I]),
    "crdt_shard_orset_merge_local": (_I, [_P, C.POINTER(crdt_tuples), C.POINTER(_SZ), C.POINTER(crdt_tuples),
                                          C.POINTER(_SZ), C.POINTER(crdt_tuples), _SZ, C.POINTER(_SZ), _I]),
    "crdt_shard_lww_merge_local_dev": (_I, [_P, C.POINTER(crdt_tuples), C.POINTER(_SZ), C.POINTER(crdt_tuples),
                                            C.POINTER(_SZ), C.POINTER(crdt_tuples), _SZ, C.POINTER(_P)]),
    "crdt_shard_orset_merge_local_dev": (_I, [_P, C.POINTER(crdt_tuples), C.POINTER(_SZ), C.POINTER(crdt_tuples),
                                              C.POINTER(_SZ), C.POINTER(crdt_tuples), _SZ, C.POINTER(_P)]),
    "crdt_shard_refmerge": (_I, [_P, C.POINTER(crdt_refmerge_in), C.POINTER(crdt_refmerge_out)]),
    "crdt_population_create": (_I, [_CTX, C.POINTER(crdt_population_init), C.POINTER(_P)]),
    "crdt_population_destroy": (_I, [_P]),
    "crdt_population_info": (_I, [_P, C.POINTER(C.c_uint32), C.POINTER(_SZ), C.POINTER(_SZ)]),
    "crdt_population_read": (_I, [_P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "crdt_population_round": (_I, [_P, _P]),
    "crdt_population_undo": (_I, [_P]),
    "crdt_population_add_commands": (_I, [_P, C.POINTER(crdt_population_cmds), _P]),
    "crdt_population_round_sharded": (_I, [_P, C.POINTER(_P), _P, _U64]),
    "crdt_population_round_wire": (_I, [_P, _P, _P, _P, _P, _P]),
    "crdt_synth_counters": (_I, [_CTX, _U64, C.c_uint32, _P, _SZ, _U64]),
    "crdt_synth_vclock_pairs": (_I, [_CTX, _U64, _P, _P, _SZ, _SZ, _U64]),
    "crdt_synth_set_tuples": (_I, [_CTX, _U64, C.c_uint32, C.POINTER(crdt_tuples), _SZ, _U64]),
}

_lib = None
_lock = threading.Lock()


def lib() -> C.CDLL:
    """Open libcrdt_amd.so once; raise CrdtLibraryError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise CrdtLibraryError(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(make -C crdt_amd/csrc). There is no CPU fallback.")
        try:
            handle = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        except OSError as e:  # pragma: no cover - depends on the box
            raise CrdtLibraryError(f"cannot load {LIB_PATH}: {e}") from e
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("CRDT_AMD_LIB") and not hasattr(handle, name):
                continue                      # an older A/B build lacks this round's entry points
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        _lib = handle
        return _lib


def check(fn: str, status: int, ctx=None) -> None:
    if status != CRDT_OK:
        hip = lib().crdt_ctx_last_hip_error(ctx) if ctx else 0
        raise CrdtError(fn, status, hip)


def call(fn: str, *args, ctx=None) -> int:
    st = getattr(lib(), fn)(*args)
    if isinstance(st, int) and st < 0:
        check(fn, st, ctx)
    return st


def use_diag_build() -> None:
    """Load libcrdt_amd_diag.so instead of the product (A/B tools, bench
    --option); must run before the library is first opened."""
    global LIB_PATH
    diag = os.path.join(_HERE, "libcrdt_amd_diag.so")
    if _lib is not None and LIB_PATH != diag:
        raise CrdtLibraryError(f"{LIB_PATH} is already loaded")
    LIB_PATH = diag


def get_option(name) -> int:
    """A kernel knob's value in the loaded build (crdt_get_option)."""
    v = C.c_int64(0)
    call("crdt_get_option", name if isinstance(name, bytes) else name.encode(), C.byref(v))
    return v.value


def is_diag() -> bool:
    """True when the diagnostic build (settable knobs, failpoints) is loaded."""
    return get_option(b"build.diag") == 1


def set_option(name, value: int) -> None:
    """crdt_set_option: diagnostic build only (the product refuses every name)."""
    call("crdt_set_option", name if isinstance(name, bytes) else name.encode(), int(value))


def rccl_info() -> dict:
    """The RCCL this process resolved (crdt_rccl_info): version and library path."""
    v = C.c_int(0)
    buf = C.create_string_buffer(512)
    call("crdt_rccl_info", C.byref(v), buf, 512)
    x = v.value
    return {"version": f"{x // 10000}.{x // 100 % 100}.{x % 100}", "code": x, "path": buf.value.decode()}
