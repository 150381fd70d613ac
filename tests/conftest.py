import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libnas.so on cuda:0)")


@pytest.fixture(scope="session")
def engine():
    """One Engine (nas_ctx on device 0) shared by the GPU tests."""
    from kubernetesnetawarescheduler_amd import Engine
    e = Engine(0)
    yield e
    e.close()
