import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def ctl():
    import cudatracerlib_amd
    cudatracerlib_amd.lib()
    return cudatracerlib_amd


@pytest.fixture(scope="session")
def orc():
    import oracle
    return oracle.load()
