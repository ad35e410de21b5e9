"""C++ unit tests (ctest) of the native core: plain, ASan+UBSan, TSan.

The reference has no sanitizer or race coverage; its allocator
and health paths race under concurrent RPCs. test_core includes a 4-thread
concurrent allocate() on one shared allocator, which TSan checks here.
"""
import shutil

import pytest

from rocm_k8s_device_plugin_amd import _build

pytestmark = pytest.mark.slow


@pytest.mark.parametrize("sanitize", ["", "address,undefined", "thread"])
def test_ctest(sanitize):
    if not shutil.which("cmake"):
        pytest.skip("cmake not available")
    r = _build.run_ctest(sanitize)
    assert r.returncode == 0, r.stdout[-3000:]
    assert "100% tests passed" in r.stdout
