import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "parallel-ray-tracer_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the rt_* C-ABI in librt_hip.so)")
    config.addinivalue_line("markers", "slow: large frames")


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()
