import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def built():
    """Build the product library + oracle once (hipcc cross-compiles without a GPU)."""
    import __graft_entry__
    __graft_entry__.build()
    return True
