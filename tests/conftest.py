import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm GPU); run with -m gpu")


@pytest.fixture(scope="session")
def oracle_lib():
    import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected without a GPU (run -m 'not gpu' on CPU hosts)")
    return torch.device("cuda", 0)
