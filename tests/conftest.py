import os
import sys

import pytest

# One HIP runtime per process: torch bundles its own libamdhip64/libhsa-runtime64 (same SONAME
# as ROCm's). Imported first, it is the runtime liboceanfft.so binds to as well, so torch streams
# and events (slab pipeline tests) and the library's launches share one runtime. Imported after
# the library, a second HSA runtime would be loaded beside ROCm's.
try:
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liboceanfft.so on the GPU)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    """The CPU checker (test infrastructure only)."""
    from oracle import oracle as O

    O.build()
    O.set_threads(min(16, os.cpu_count() or 1))
    return O
