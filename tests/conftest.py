import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "gradient-compression_amd")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(autouse=True)
def _default_rng_mode():
    """Every test starts and ends with the package's default RNG mode (a test
    that switches the default generator's mode must not leak it)."""
    yield
    try:
        import gcodec
    except Exception:  # the package did not import: nothing to restore
        return
    g = gcodec.rng.default_generator
    if g.mode != gcodec.rng.DEFAULT_MODE:
        g.set_mode(gcodec.rng.DEFAULT_MODE)
