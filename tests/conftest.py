import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "active-perception-gym_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running")


def golden(name):
    import numpy as np

    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def oracle_mod():
    from oracle import oracle

    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ap_gym_amd

    ap_gym_amd._native.lib()
    return torch.device("cuda:0")
