"""Reflection-ray compaction (k_render_wave, rt_fast.h; row n2).

With RT_FLAG_COMPACT, reflective scenes trace their reflected rays
(renderer.nim:104-124) in per-wave queues and full 64-ray passes; a queued ray's radiance is summed per
pixel in 32.32 fixed point and added after the kernel (k_sec_add). Checked
here:
  * against the default one-sample level loop: Stats identical,
    pixels equal to float rounding (the deeper levels are grouped
    differently: <= 2e-6 relative + 1e-6);
  * determinism: the fixed-point sums do not depend on which rays shared a
    pass, so repeated frames, row ranges and multi-GPU bands are bit-equal
    to the full frame;
  * against the float64 oracle (renderer.nim:71-159, oracle/rt_oracle.c) at
    1 spp (every camera ray's reflections in scattered passes) and 16 / 64
    spp, with the fp32 tolerance of tests/test_gpu_configs.py.
The float64 parity kernel does not compact (it keeps the reference's
recursive sum order) and stays bit-exact: tests/test_gpu_parity.py runs both
scenes through it.
"""
import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, akGrid, akNone, scenes
from rtmi.abi import RT_FLAG_COMPACT
from rtmi.renderer import DeviceScene, band_rows, unshard_bands_device

pytestmark = pytest.mark.gpu

BIAS = 1e-4
THREADS = 16


def _opts(w, h, m, flags=0, prec=Precision.fp32):
    return Options(width=w, height=h, antialias=Antialias(akGrid if m > 1 else akNone, m), bias=BIAS,
                   maxRayDepth=5, precision=prec, flags=flags)


def _render(ds, o, y0=0, y1=None):
    import torch
    fb = torch.zeros(o.width * o.height * 3, dtype=torch.float32, device="cuda")
    st = ds.render_device(o, fb, y0=y0, y1=y1)
    return fb, st


CASES = [("spheres-reflection", 320, 240, 1), ("spheres-reflection", 160, 120, 4),
         ("spheres-reflection", 96, 64, 8), ("mesh-mix", 320, 240, 1), ("mesh-mix", 160, 120, 4),
         ("mesh-mix", 96, 64, 8)]


@pytest.mark.parametrize("name,w,h,m", CASES)
def test_compact_matches_level_loop(gpu, name, w, h, m):
    import torch
    ds = DeviceScene(scenes.SCENES[name]())
    a, sa = _render(ds, _opts(w, h, m, RT_FLAG_COMPACT))
    assert ds.last_compacted()
    a2, sa2 = _render(ds, _opts(w, h, m, RT_FLAG_COMPACT))
    assert torch.equal(a, a2) and sa == sa2  # deterministic
    b, sb = _render(ds, _opts(w, h, m))
    assert not ds.last_compacted()
    assert sa == sb
    assert sa.numReflectionRays > 0
    err = (a - b).abs()
    bound = 2e-6 * b.abs() + 1e-6
    assert bool((err <= bound).all()), float((err - bound).max())


@pytest.mark.parametrize("name", ["spheres-reflection", "mesh-mix"])
def test_compact_rows_and_bands_match_full_frame(gpu, name):
    import torch
    w, h = 173, 131
    o = _opts(w, h, 4, RT_FLAG_COMPACT)
    ds = DeviceScene(scenes.SCENES[name]())
    full, _ = _render(ds, o)
    part, _ = _render(ds, o, 37, 90)
    img, pimg = full.view(h, w, 3), part.view(h, w, 3)
    assert torch.equal(pimg[37:90], img[37:90])
    assert float(pimg[:37].abs().max()) == 0.0 and float(pimg[90:].abs().max()) == 0.0
    for world, band_h in [(2, 16), (3, 7)]:
        rows = band_rows(h, band_h, world)
        gathered = torch.zeros(world * rows * w * 3, dtype=torch.float32, device="cuda")
        for r in range(world):
            ds.render_bands_device(o, gathered[r * rows * w * 3:(r + 1) * rows * w * 3], band_h, r, world)
            assert ds.last_compacted()
        fb = torch.zeros_like(full)
        unshard_bands_device(gathered, fb, w, h, band_h, world)
        torch.cuda.synchronize()
        assert torch.equal(fb, full), (world, band_h)


def _check(got, ref, what, frac=0.995, tol=2e-3, mean_tol=2e-4):
    err = np.abs(got.astype(np.float64) - ref.astype(np.float64)).max(axis=-1)
    ok = float((err <= tol).mean())
    assert ok >= frac, f"{what}: only {ok:.5f} of pixels within {tol} (max {err.max():.3g})"
    assert err.mean() <= mean_tol, f"{what}: mean abs err {err.mean():.3g}"


def _oracle_rows(scene, o, rows, bvh):
    import oracle
    ref = np.zeros((o.height, o.width, 3), np.float32)
    orc = oracle.OracleScene(scene, bvh=bvh)
    _, st, _ = orc.render(_opts(o.width, o.height, o.antialias.gridSize if o.antialias.kind != akNone else 1,
                                prec=Precision.fp64), rows=rows, fb=ref, nthreads=THREADS)
    return ref, st


@pytest.mark.parametrize("name,w,h,m,rows", [
    ("spheres-reflection", 1920, 1080, 1, [100, 330, 470, 540, 610, 700, 850, 1000]),
    ("spheres-reflection", 480, 270, 4, None),
    ("mesh-mix", 480, 270, 4, None),
    ("mesh-mix", 1920, 1080, 8, [420, 540, 600, 700]),
])
def test_compact_oracle(gpu, name, w, h, m, rows):
    sc = scenes.SCENES[name]()
    o = _opts(w, h, m, RT_FLAG_COMPACT)
    ds = DeviceScene(sc)
    fb, st = _render(ds, o)
    assert ds.last_compacted()
    got = fb.view(h, w, 3).cpu().numpy()
    rows = list(range(h)) if rows is None else rows
    ref, rst = _oracle_rows(sc, o, rows, bvh=name == "mesh-mix")
    _check(got[rows], ref[rows], f"{name} {w}x{h} {m * m} spp")
    if len(rows) == h:
        assert st.numPrimaryRays == rst.numPrimaryRays
        assert abs(st.numReflectionRays - rst.numReflectionRays) <= 1e-3 * rst.numReflectionRays + 2
        assert abs(st.numShadowRays - rst.numShadowRays) <= 1e-3 * rst.numShadowRays + 2
