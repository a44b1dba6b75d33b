import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "zarr-java_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

# Plans of at most 64 inner chunks decode in one launch by default (ZH_SMALL_ONE: resolve and
# the generic paths per item, decode_small_kernel).  Most cases here are that small, so the
# suite keeps them on the multi-launch kernels (resolve, the fast kernels, the slow list) that
# large reads use; the tests parametrized with `small_one` run both forms.
os.environ.setdefault("ZH_SMALL_ONE", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def dev():
    """One DeviceContext for the whole GPU session (one process on the card)."""
    from zarrhip._lib import DeviceContext
    ctx = DeviceContext(0)
    yield ctx
    ctx.close()
