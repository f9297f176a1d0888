import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: multi-second CPU test")


@pytest.fixture(scope="session")
def gpu_ctx():
    from libhdfs3_amd.engine import CrcContext, device_count

    if device_count() < 1:
        pytest.fail("no GPU visible for a -m gpu test")
    ctx = CrcContext(0)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def lab_ctx():
    """A context of the measurement library (libhdfs3_crc_lab.so): the same production
    kernels plus the A/B variant knob (hdfs3x_set_variant). Variant tests run here, so the
    product library never carries the knob."""
    from libhdfs3_amd import _native
    from libhdfs3_amd.engine import CrcContext, device_count

    if device_count() < 1:
        pytest.fail("no GPU visible for a -m gpu test")
    ctx = CrcContext(0, lib=_native.lab())
    yield ctx
    ctx.close()
