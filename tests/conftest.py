import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Make sure the oracle (checker) and the engine library exist (built in-tree)."""
    if not os.path.exists(os.path.join(ROOT, "oracle", "_build", "liboracle.so")):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(ROOT, "pipsort_amd", "lib", "libpipsort_engine.so")):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "pipsort_amd")], check=True)
    yield


@pytest.fixture(scope="session")
def gpu():
    # torch's bundled HIP runtime must load before the engine library (same
    # SONAME, one runtime for both), as in bench.py
    import torch  # noqa: F401
    from pipsort_amd import engine
    if engine.device_count() < 1:
        pytest.fail("GPU test on a host without a HIP device")
    return True
