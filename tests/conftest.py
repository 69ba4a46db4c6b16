import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libcrdt_amd.so")
    config.addinivalue_line("markers", "diag: sets kernel knobs or failpoints (tests/knobs.py): non-default variants "
                            "run under the diagnostic build, in the child suite of tests/test_gpu_diag_build.py")


@pytest.fixture(scope="session")
def eng():
    import torch
    from crdt_amd.engine import Engine
    assert torch.cuda.is_available(), "gpu-marked test without a GPU"
    e = Engine(0)
    # CRDT_TEST_OPTIONS="sets.lww_parts=2,join.unroll=2": run the GPU suite
    # under non-default kernel knobs (crdt_set_option)
    from knobs import set_knob
    for opt in filter(None, os.environ.get("CRDT_TEST_OPTIONS", "").split(",")):
        k, v = opt.split("=")
        set_knob(k.strip().encode(), int(v))
    yield e
    e.close()
