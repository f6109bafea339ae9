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


@pytest.fixture(scope="session")
def c3_oracle_frame(oracle_mod):
    """The same-BVH oracle's WHOLE 1920x1080, 256-spp C3 frame (bunny + ground,
    bias 1e-4) and its Stats, computed once per session (~14 s on the GPU
    box's 16 host threads) and shared by the float32 whole-frame tolerance
    test and the float64 whole-frame bit-exact test."""
    import numpy as np
    from rtmi import Antialias, Options, Precision, akGrid, scenes
    opts = Options(width=1920, height=1080, antialias=Antialias(akGrid, 16), bias=1e-4, precision=Precision.fp64)
    fb = np.zeros((1080, 1920, 3), np.float32)
    _, st, _ = oracle_mod.OracleScene(scenes.mesh_bunny(), bvh=True).render(opts, rows=list(range(1080)), fb=fb,
                                                                            nthreads=16)
    return fb, st
