import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))
GOLD = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libpygrid_hip on the GPU)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def gold():
    return GOLD


@pytest.fixture(scope="session")
def engine():
    """One GPU context for the whole GPU session (tests re-layout it as needed)."""
    from pygrid_amd import Engine

    eng = Engine(int(os.environ.get("PGH_DEVICE", "0")))
    yield eng
    eng.close()
