import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Load the HIP engine library before anything imports torch, so the process
# has exactly one HIP runtime (ROCm 7.2 from /opt/rocm).
try:  # pragma: no cover - depends on the build state
    import sentinel_amd.engine  # noqa: F401
except Exception:
    pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def so():
    from oracle import oracle
    oracle.lib()
    return oracle
