import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built _dls_hip extension")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def hip():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from distributed_learning_simulator_amd.ops import build

    build.build()
    from distributed_learning_simulator_amd.ops import hip as hipmod

    return hipmod
