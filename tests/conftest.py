import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libwasmedge_batch.so)")


def golden(name, mode="rb"):
    with open(os.path.join(GOLDEN, name), mode) as f:
        return f.read()


@pytest.fixture(scope="session")
def built():
    """Build the product library, the test emulator and the oracle (idempotent)."""
    import __graft_entry__
    __graft_entry__.build()
    return True
