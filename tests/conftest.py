import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


@pytest.fixture(scope="session")
def pg():
    import pgload
    return pgload.load()


@pytest.fixture(scope="session")
def O():
    """The CPU oracle (test infrastructure only)."""
    import oracle_py
    oracle_py.build()
    return oracle_py


GOLDEN = os.path.join(ROOT, "tests", "golden")
