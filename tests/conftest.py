import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libavsr_hip.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test requires a GPU (run with -m 'not gpu' on CPU)")
    from avsr_amd import _lib
    _lib.load()
    return torch.device("cuda:0")


@pytest.fixture
def lib_opt():
    """set a library kernel-selection option (avsr_set_option) for one test; restored after"""
    from avsr_amd import _lib
    saved = {}

    def set_(name, value):
        prev = _lib.set_option(name, value)
        saved.setdefault(name, prev)

    yield set_
    for name, value in saved.items():
        _lib.set_option(name, value)
