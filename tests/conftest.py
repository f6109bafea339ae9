import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "nim-raytracer_amd"), os.path.join(REPO, "oracle"), REPO):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle_mod():
    import oracle
    oracle.build()
    return oracle


@pytest.fixture(scope="session")
def gpu():
    """Skip-free GPU gate: on a GPU run the native library must load and see a
    gfx950 device, otherwise the test FAILS (no silent CPU fallback)."""
    from rtmi import renderer
    n = renderer.device_count()
    assert n > 0, "no GPU visible to librtmi.so"
    renderer.initRenderer(0)
    return 0
