import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libcrdt_amd.so")


@pytest.fixture(scope="session")
def eng():
    import torch
    from crdt_amd.engine import Engine
    assert torch.cuda.is_available(), "gpu-marked test without a GPU"
    e = Engine(0)
    yield e
    e.close()
