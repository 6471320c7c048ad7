import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C ABI)")
    config.addinivalue_line("markers", "slow: long-running CPU check")


@pytest.fixture(autouse=True)
def _device_clean_after_gpu_test(request):
    """After every GPU test: wait for all device work the test left in flight
    and check it (rt_gpu_synchronize), so a device fault or a replayed-count
    mismatch fails the test whose work raised it instead of a later one."""
    yield
    if request.node.get_closest_marker("gpu") is None:
        return
    import helpers
    lib = helpers.rt580()._lib
    if lib is None:
        return
    if lib.rt_gpu_synchronize() != 0:
        msg = lib.rt_gpu_last_error()
        pytest.fail("device work left by this test failed: %s" % (msg.decode() if msg else "?"), pytrace=False)
