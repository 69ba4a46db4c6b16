"""GPU: the knob variants, timing-free diagnostics and failpoints, run under
the diagnostic build (libcrdt_amd_diag.so, -DCRDT_DIAG) in ONE child pytest
process.

The product library (the one the rest of this session loads) compiles every
kernel knob as a constant and refuses crdt_set_option, so the ``diag`` tests
run here only at the product's defaults and skip their other variants.  This
test starts a single child pytest over every ``gpu and diag`` test with
CRDT_AMD_DIAG=1: there every measured alternative (DESIGN.md's A/B records)
is checked against the oracle, and the failpoint tests raise their errors.
The child's progress streams to this session's terminal (capture suspended),
so a long child never looks hung.
"""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_diag_build_suite(request):
    lib = os.path.join(ROOT, "crdt_amd", "libcrdt_amd_diag.so")
    assert os.path.exists(lib), "build it: make -C crdt_amd/csrc (libcrdt_amd_diag.so)"
    if os.environ.get("CRDT_AMD_DIAG") == "1":
        pytest.skip("already the diagnostic build")
    env = dict(os.environ, CRDT_AMD_DIAG="1")
    env.pop("CRDT_AMD_LIB", None)
    cmd = [sys.executable, "-u", "-m", "pytest", os.path.join(ROOT, "tests"), "-m", "gpu and diag", "-x", "-q",
           "-p", "no:cacheprovider", "--timeout", "240", "--timeout-method", "thread"]
    capman = request.config.pluginmanager.getplugin("capturemanager")
    with capman.global_and_fixture_disabled():
        print("\n[diag build] " + " ".join(cmd[3:]), flush=True)
        rc = subprocess.run(cmd, cwd=ROOT, env=env, timeout=1500).returncode
    assert rc == 0, f"diagnostic-build suite failed (exit {rc})"
