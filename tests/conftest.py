"""Test configuration.  `-m gpu` tests need an MI355X (they call libmpcqp.so through its C
ABI); everything else runs on CPU.  The oracle (oracle/) is loaded only here, as the checker."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpc-limx-control_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X) and libmpcqp.so")


@pytest.fixture(scope="session")
def golden():
    def load(name):
        return np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    return load


@pytest.fixture(scope="session")
def orc():
    import oracle
    oracle.lib()
    return oracle


def rel_err(a, b):
    """norm-wise relative error max|a-b| / max(1, max|b|)"""
    a = np.asarray(a, float)
    b = np.asarray(b, float)
    return float(np.abs(a - b).max() / max(1.0, np.abs(b).max())) if b.size else 0.0


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu-marked test run without a HIP device")
    import mpcqp
    mpcqp.lib()  # raises loudly if libmpcqp.so is missing
    return torch
