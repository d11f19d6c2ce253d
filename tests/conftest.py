import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


def _native_or_none():
    try:
        from mxdesk import native

        return native()  # imports torch first (shared HIP runtime, see mxdesk.native)
    except ImportError:
        return None


@pytest.fixture(scope="session")
def native():
    """The compiled extension; built on demand (hipcc cross-compiles without a GPU)."""
    n = _native_or_none()
    if n is None:
        from mxdesk import _build

        _build.build()
        n = _native_or_none()
    assert n is not None, "native extension failed to build"
    return n


@pytest.fixture(scope="session")
def gpu(native):
    """Skip-proof GPU fixture: on a GPU run the device MUST be there (fail loudly)."""
    if native.device_count() < 1:
        pytest.fail("no HIP device visible but a gpu-marked test was selected")
    native.set_device(0)
    return native
