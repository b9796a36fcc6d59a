import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nerf-replication_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden", "golden_v1.npz")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libnerf_amd.so)")


@pytest.fixture(scope="session")
def golden():
    return np.load(GOLDEN, allow_pickle=False)


@pytest.fixture(scope="session")
def seeded_state():
    from oracle import nerf_oracle as O
    return O.seeded_network_state(0)


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
