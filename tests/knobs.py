"""Kernel knobs and failpoints for the GPU tests.

The product library compiles every knob (crdt_amd/csrc/knobs.inc) as a
constant at its default and refuses crdt_set_option; the diagnostic build
(libcrdt_amd_diag.so) accepts them.  A test that needs a non-default knob or
a failpoint carries ``@pytest.mark.diag`` and calls :func:`set_knob`:

* under the product library a request for the compiled-in value is a no-op
  (the default variant of a parametrised test runs on the product), anything
  else skips the test here;
* tests/test_gpu_diag_build.py runs every ``diag`` test again in one child
  process with CRDT_AMD_DIAG=1, where every variant runs.
"""
import pytest

from crdt_amd import _lib


def set_knob(name, value: int) -> None:
    name = name if isinstance(name, bytes) else name.encode()
    if _lib.is_diag():
        _lib.set_option(name, value)
        return
    if name.startswith(b"fail."):
        current = 0                                   # failpoints: never armed in the product
    else:
        current = _lib.get_option(name)
    if current != int(value):
        pytest.skip(f"{name.decode()}={value}: diagnostic build only (tests/test_gpu_diag_build.py)")
