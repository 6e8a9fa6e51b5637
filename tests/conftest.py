import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "babylon.js-pathtracing-renderer_amd")
for p in (os.path.join(PKG, "python"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLD = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device and the built libpt.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def gold():
    return GOLD


@pytest.fixture(scope="session")
def engine():
    import babylon_pt as bp
    e = bp.Engine(0)
    yield e
    e.dispose()
