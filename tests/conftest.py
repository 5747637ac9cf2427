import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libtmgpu.so)")


@pytest.fixture(scope="session")
def golden():
    import json

    def load(name):
        with open(os.path.join(GOLDEN, name)) as f:
            return json.load(f)
    return load


@pytest.fixture(scope="session")
def ctx():
    """One tmv context per test session on cuda:0 (GPU tests only)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tendermint_amd import _native
    c = _native.Context(1)
    yield c
    c.close()
