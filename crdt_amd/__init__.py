"""crdt_amd -- MI355X-native batched CRDT merge engine.

Drop-in for the merge/compare path of anuragsarkar97/crdt
(/root/reference/main.go:35-113).  The product is libcrdt_amd.so (gfx950 HIP
kernels behind the C-ABI in include/crdt_amd.h); this package is the Python
host binding.  There is no CPU fallback: without the built library or a GPU
every entry point raises.
"""
from ._lib import CrdtError, CrdtLibraryError, LIB_PATH, lib  # noqa: F401

__all__ = ["CrdtError", "CrdtLibraryError", "LIB_PATH", "lib", "Engine", "TupleSet", "Server", "NewServer"]


def __getattr__(name):  # lazy: submodules load on first use
    if name in ("Engine", "TupleSet", "as_u64", "u64_tensor"):
        from . import engine
        return getattr(engine, name)
    if name in ("Server", "NewServer", "Command", "Data", "Int64Comparator"):
        from . import server
        return getattr(server, name)
    raise AttributeError(name)
