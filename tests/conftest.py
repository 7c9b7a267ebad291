import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; parity tests through the C ABI")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure the in-tree libraries exist (build() is idempotent and fast when up to date)."""
    import __graft_entry__ as g

    g.build()
    yield


GOLDEN = os.path.join(ROOT, "tests", "golden")
