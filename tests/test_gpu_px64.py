"""float64 parity mode, one pixel per wave (k_render_px64, rt_device.h).

akGrid frames of >= 64 samples per pixel render a pixel's 64 samples side by
side in one wave: the camera rays search the pixel's face list, the shadow
rays to distant lights their light-grid cells, and each pixel's samples are
summed in sample order (renderer.nim:149-159) from the wave's LDS rows. The
bar is the parity mode's: bit-exact framebuffer and identical Stats against
the fp64 oracle (oracle/rt_oracle.c), and bit-identical to the one-lane-per-
pixel kernel with the BVH for every ray (RT_FLAG_F64_PER_LANE).
"""
import ctypes as C

import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, Stats, akGrid, scenes
from rtmi._lib import lib
from rtmi.abi import RT_FLAG_F64_PER_LANE, RT_FLAG_NO_BINNING
from rtmi.renderer import DeviceScene, band_rows, unshard_bands_device

pytestmark = pytest.mark.gpu

BIAS = 1e-4


def _opts(w, h, m, flags=0, depth=5):
    return Options(width=w, height=h, antialias=Antialias(akGrid, m), bias=BIAS, maxRayDepth=depth,
                   precision=Precision.fp64, flags=flags)


def _dev(ds, opts, y0=0, y1=None, step=1, maxStep=1):
    import torch
    fb = torch.zeros(opts.width * opts.height * 3, dtype=torch.float32, device="cuda")
    st = ds.render_device(opts, fb, y0, y1, step, maxStep)
    return fb.view(opts.height, opts.width, 3).cpu().numpy(), st


# (scene, width, height, m): meshes with and without lists, reflection + a
# point light (BVH rays inside a one-pixel wave), analytic scenes, and
# m = 9 (81 spp: a partial second step of 17 samples)
CASES = [
    ("mesh-bunny", 48, 32, 8),
    ("mesh-bunny", 40, 24, 9),
    ("mesh-teapot", 40, 28, 8),  # the reference's live scene (mesh-bunny.nim loads teapot.obj)
    ("mesh-mix", 40, 28, 8),
    ("two-meshes", 36, 24, 8),
    ("spheres-reflection", 40, 30, 8),
    ("boxes2", 40, 24, 8),
    ("spheres-warm", 32, 24, 9),
]


@pytest.mark.parametrize("name,w,h,m", CASES)
def test_px64_bit_exact_against_oracle(gpu, oracle_mod, name, w, h, m):
    scene = scenes.SCENES[name]()
    opts = _opts(w, h, m)
    ref, rst, _ = oracle_mod.OracleScene(scene, bvh=True).render(opts)
    ds = DeviceScene(scene)
    got, gst = _dev(ds, opts)
    diff = np.argwhere(got != ref)
    assert diff.size == 0, f"{len(diff)} channels differ, first at {diff[:3].tolist()}"
    assert gst == rst


@pytest.mark.parametrize("name,w,h,m", CASES)
def test_px64_equals_per_lane_kernel(gpu, name, w, h, m):
    ds = DeviceScene(scenes.SCENES[name]())
    a, sa = _dev(ds, _opts(w, h, m))
    b, sb = _dev(ds, _opts(w, h, m, RT_FLAG_F64_PER_LANE))
    c, sc = _dev(ds, _opts(w, h, m, RT_FLAG_NO_BINNING))  # one pixel per wave, BVH for every ray
    assert np.array_equal(a, b) and np.array_equal(a, c)
    assert sa == sb == sc


def test_px64_progressive_and_row_ranges(gpu, oracle_mod):
    """step / maxStep passes (renderer.nim:166-209) and row ranges."""
    scene = scenes.mesh_bunny()
    opts = _opts(48, 36, 8)
    o = oracle_mod.OracleScene(scene, bvh=True)
    ds = DeviceScene(scene)
    ref = np.zeros((36, 48, 3), np.float32)
    got = np.zeros((36, 48, 3), np.float32)
    step = 4
    while step >= 1:
        _, rst, _ = o.render(opts, step=step, maxStep=4, fb=ref)
        gst = ds.render_lines(opts, got, 0, 36, step, 4)
        assert gst == rst
        step //= 2
    assert np.array_equal(got, ref)
    part = np.zeros_like(got)
    s1 = ds.render_lines(opts, part, 5, 23)
    assert np.array_equal(part[5:23], ref[5:23])
    _, rs = o.render(opts, rows=list(range(5, 23)))[:2]
    assert s1 == rs


def test_px64_bands_match_full_frame(gpu):
    """rt_render_bands_device layouts (multi-GPU shards) in float64."""
    import torch
    ds = DeviceScene(scenes.mesh_bunny())
    W, H, band_h = 40, 30, 4
    opts = _opts(W, H, 8)
    full, sfull = _dev(ds, opts)
    for world in (2, 3):
        rows = band_rows(H, band_h, world)
        gathered = torch.zeros(world * rows * W * 3, dtype=torch.float32, device="cuda")
        total = Stats()
        for rank in range(world):
            buf = gathered[rank * rows * W * 3:(rank + 1) * rows * W * 3]
            total += ds.render_bands_device(opts, buf, band_h, rank, world)
        fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
        unshard_bands_device(gathered, fb, W, H, band_h, world)
        assert np.array_equal(fb.view(H, W, 3).cpu().numpy(), full)
        assert total == sfull


@pytest.mark.parametrize("lg", [0, 2])
def test_px64_lists_past_their_slots_take_the_bvh(gpu, lg):
    """Pixels whose camera-ray list outgrows its 2^lg slots take the BVH in
    the one-pixel wave: the same frame and Stats."""
    ds = DeviceScene(scenes.mesh_bunny())
    opts = _opts(64, 36, 8)
    ref, sref = _dev(ds, opts)
    f = lib().rtmi_test_slot_lg
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int32]
    default = f(ds.h, -1)
    f(ds.h, lg)
    got, sgot = _dev(ds, opts)
    f(ds.h, default)
    assert np.array_equal(got, ref) and sgot == sref


def test_px64_full_c3_frame(gpu, c3_oracle_frame):
    """BASELINE config C3 at full size (1920x1080, 256 spp) in float64: EVERY
    row of the one-pixel-per-wave frame equals the oracle's whole frame bit
    for bit (same-BVH oracle, exact), with identical Stats — and the
    one-lane-per-pixel BVH kernel renders the same frame."""
    scene = scenes.mesh_bunny()
    opts = _opts(1920, 1080, 16)
    ds = DeviceScene(scene)
    a, sa = _dev(ds, opts)
    ref, rst = c3_oracle_frame
    diff = np.argwhere(a != ref)
    assert diff.size == 0, f"{len(diff)} channels differ, rows {sorted(set(diff[:, 0].tolist()))[:10]}"
    assert sa == rst
    b, sb = _dev(ds, _opts(1920, 1080, 16, RT_FLAG_F64_PER_LANE))
    assert sb == sa
    assert np.array_equal(a, b)
