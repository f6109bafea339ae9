"""Stochastic samplers (sampling.nim:21-113) of the oracle over the counter
RNG: the structure each algorithm guarantees, determinism, and agreement of
the rendered image with the grid sampler's (same expectation)."""
import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, scenes
from rtmi.scene import akCorrelatedMultiJittered, akGrid, akJittered, akMultiJittered

KINDS = [akJittered, akMultiJittered, akCorrelatedMultiJittered]


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("m", [1, 2, 5, 16])
def test_sample_table_structure(oracle_mod, kind, m):
    sx, sy = oracle_mod.sample_table(kind, m, seed=12345, x=17, y=3)
    assert sx.shape == (m * m,) and ((sx >= 0) & (sx < 1) & (sy >= 0) & (sy < 1)).all()
    j, i = np.divmod(np.arange(m * m), m)
    # every entry p[j*m + i] stays in its 2D stratum (x cell i, y cell j)
    assert (np.floor(sx * m) == i).all() and (np.floor(sy * m) == j).all()
    if kind != akJittered:
        # n-rooks: the m*m x (and y) values occupy every 1D sub-stratum once
        assert sorted(np.floor(sx * m * m).astype(int)) == list(range(m * m))
        assert sorted(np.floor(sy * m * m).astype(int)) == list(range(m * m))


def test_sample_table_determinism(oracle_mod):
    a = oracle_mod.sample_table(akMultiJittered, 8, seed=1, x=5, y=6)
    b = oracle_mod.sample_table(akMultiJittered, 8, seed=1, x=5, y=6)
    c = oracle_mod.sample_table(akMultiJittered, 8, seed=2, x=5, y=6)
    d = oracle_mod.sample_table(akMultiJittered, 8, seed=1, x=6, y=5)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    assert not np.array_equal(a[0], c[0]) and not np.array_equal(a[0], d[0])


@pytest.mark.parametrize("kind", KINDS)
def test_stochastic_image_matches_grid_expectation(oracle_mod, kind):
    scene = scenes.spheres_warm(3)
    base = dict(width=48, height=32, bias=1e-4, precision=Precision.fp64, seed=7)
    g, gst, _ = oracle_mod.OracleScene(scene).render(Options(antialias=Antialias(akGrid, 4), **base))
    s, sst, _ = oracle_mod.OracleScene(scene).render(Options(antialias=Antialias(kind, 4), **base))
    assert sst.numPrimaryRays == gst.numPrimaryRays == 48 * 32 * 16
    err = np.abs(s.astype(np.float64) - g)
    assert err.mean() < 5e-3 and np.median(err) < 1e-3
