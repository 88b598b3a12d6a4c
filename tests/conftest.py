import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP product path)")


@pytest.fixture(scope="session")
def built():
    """Build liburgym.so + the oracle once per session (no-op when up to date)."""
    import __graft_entry__
    __graft_entry__.build()
    return True
