import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def oracle():
    from tests import oracle_lib
    return oracle_lib.Oracle()


@pytest.fixture(scope="session")
def hip():
    """The product library; built in-tree if stale. GPU tests only."""
    from madraft_amd import build, sim
    if not os.path.exists(sim.LIB_PATH):
        build.build_hip()
    sim.lib()
    return sim
