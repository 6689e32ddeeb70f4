import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "rust-crdt_amd"), os.path.join(ROOT, "oracle"), os.path.dirname(__file__)):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libcrdt_gpu.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def gpu_ctx():
    """The product context on cuda:0.  On a GPU box a missing library is a hard failure."""
    import torch
    import crdts_gpu

    assert torch.cuda.is_available(), "gpu-marked test on a host without a visible MI355X"
    torch.cuda.set_device(0)
    return crdts_gpu.Context.default(0)
