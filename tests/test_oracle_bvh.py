"""The oracle's same-BVH mode (the fair CPU baseline of SURVEY.md 8(d)) gives
exactly the brute-force reference loop's answers: same image bits, same Stats."""
import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, akGrid, akNone, scenes


@pytest.mark.parametrize("name,w,h,aa,m", [
    ("mesh-bunny", 40, 30, akNone, 1),
    ("mesh-mix", 48, 32, akGrid, 2),
    ("two-meshes", 48, 32, akNone, 1),
])
def test_bvh_equals_brute_force(oracle_mod, name, w, h, aa, m):
    scene = scenes.SCENES[name]()
    opts = Options(width=w, height=h, antialias=Antialias(aa, m), bias=1e-4, maxRayDepth=5,
                   precision=Precision.fp64)
    ref, rst, _ = oracle_mod.OracleScene(scene).render(opts, nthreads=8)
    got, gst, _ = oracle_mod.OracleScene(scene, bvh=True).render(opts, nthreads=8)
    assert np.array_equal(got, ref)
    assert gst == rst
