import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "gym-po-taxi_amd"), os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run via gpurun)")
    config.addinivalue_line("markers", "slow: longer CPU test")
    config.addinivalue_line("markers", "gpu_first: runs before every other test (spawns GPU worker processes, which "
                                       "is only allowed before this process initialises the GPU)")


def pytest_collection_modifyitems(config, items):
    items.sort(key=lambda it: 0 if it.get_closest_marker("gpu_first") else 1)  # stable: the rest keep their order


@pytest.fixture(scope="session")
def gpu_device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
