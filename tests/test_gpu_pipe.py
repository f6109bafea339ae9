"""Pipelined per-call builds (rtmi.cpp rt_scene::pipe): a float32 call that
renders at most a third of the image (a multi-GPU rank's bands, a pool's
scanlines) builds its camera-dependent data on the scene's build stream into
the other of two buffer sets, overlapping the previous call's render. Calls
issued back to back without any host synchronisation must give the same
frames and Stats as the same calls made one at a time — the reference's pool
issues renderLine calls with no ordering among them (workerpool.nim:72-99,
raytracer.nim:25-32), and a rank issues frame after frame (raytracer.nim:67-70)."""
import ctypes as C
import os

import pytest

from rtmi import Antialias, Options, Precision, akGrid, scenes
from rtmi._lib import lib
from rtmi.dist import band_rows
from rtmi.glm import X_AXIS, degToRad, rotate, translate, mat4, vec3
from rtmi.renderer import DeviceScene
from rtmi.scene import Stats

pytestmark = pytest.mark.gpu

W, H, M = 480, 270, 16


def _opts(flags=0):
    return Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32, flags=flags)


def _scene(pipe):
    """pipe: "0" / "1" forces the pipelining off / on, None: by launch size."""
    old = os.environ.get("RTMI_PIPE")
    if pipe is None:
        os.environ.pop("RTMI_PIPE", None)
    else:
        os.environ["RTMI_PIPE"] = pipe  # read by rt_scene_create
    try:
        return DeviceScene(scenes.mesh_bunny())
    finally:
        if old is None:
            os.environ.pop("RTMI_PIPE", None)
        else:
            os.environ["RTMI_PIPE"] = old


def _pipelined(ds):
    f = lib().rtmi_test_last_pipelined
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
    s = C.c_int32()
    r = f(ds.h, C.byref(s))
    assert r >= 0
    return bool(r), int(s.value)


@pytest.mark.parametrize("pipe", [None, "1"])
@pytest.mark.parametrize("world", [4, 8])
def test_back_to_back_bands(gpu, pipe, world):
    """Every rank's bands, twice over, issued without a sync: each buffer
    equals the rank rendered alone with Stats (the serial path), and the last
    call's Stats equal its serial Stats."""
    import torch
    ref_ds = _scene("0")
    ds = _scene(pipe)
    rows = band_rows(H, 4, world)
    refs, ref_st = [], []
    for r in range(world):
        b = torch.full((rows * W * 3,), -7.0, dtype=torch.float32, device="cuda")
        ref_st.append(ref_ds.render_bands_device(_opts(), b, 4, r, world))
        assert _pipelined(ref_ds)[0] is False
        refs.append(b)
    outs = [torch.full((rows * W * 3,), -7.0, dtype=torch.float32, device="cuda") for _ in range(2 * world)]
    sets = []
    for k in range(2 * world):
        ds.render_bands_device(_opts(), outs[k], 4, k % world, world, stats=False)
        p, s = _pipelined(ds)
        assert p, k  # a rank's bands are <= 1/3 of the image
        sets.append(s)
    assert all(sets[k] != sets[k + 1] for k in range(len(sets) - 1)), sets
    torch.cuda.synchronize()
    for k in range(2 * world):
        assert torch.equal(outs[k], refs[k % world]), (k, float((outs[k] - refs[k % world]).abs().max()))
    st = ds.render_bands_device(_opts(), outs[0], 4, world - 1, world)
    assert st == ref_st[world - 1]


def test_back_to_back_scanlines(gpu):
    """renderLine per scanline (the pool's calls), all issued at once into one
    device frame: equals the whole frame rendered by one serial call, and the
    summed per-line Stats equal the frame's."""
    import torch
    ds = _scene(None)
    whole = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    st_whole = ds.render_device(_opts(), whole)
    assert _pipelined(ds)[0] is False  # a whole frame: the build in stream order
    fb = torch.full((W * H * 3,), -7.0, dtype=torch.float32, device="cuda")
    for y in range(0, H, 3):  # three-line calls
        ds.render_device(_opts(), fb, y0=y, y1=min(H, y + 3), stats=False)
        assert _pipelined(ds)[0]
    torch.cuda.synchronize()
    assert torch.equal(fb, whole), float((fb - whole).abs().max())
    tot = Stats()
    for y in range(0, H, 27):
        tot += ds.render_device(_opts(), fb, y0=y, y1=min(H, y + 27))
    assert (tot.numPrimaryRays, tot.numShadowRays, tot.numIntersectionHits, tot.numIntersectionTests) == (
        st_whole.numPrimaryRays, st_whole.numShadowRays, st_whole.numIntersectionHits, st_whole.numIntersectionTests)


def test_camera_change_between_pipelined_calls(gpu):
    """A camera change between two back-to-back pipelined calls: each call
    renders its own camera (the build reads the camera by value)."""
    import torch
    world = 4
    rows = band_rows(H, 4, world)
    cam2 = translate(rotate(mat4(1.0), X_AXIS, degToRad(-20.0)), vec3(0.7, 6.0, 2.5))
    ref_ds, ds = _scene("0"), _scene("1")
    want = []
    for cam in (None, cam2):
        if cam is not None:
            ref_ds.set_camera(cam)
        b = torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda")
        ref_ds.render_bands_device(_opts(), b, 4, 1, world)
        want.append(b)
    got = [torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda") for _ in range(2)]
    ds.render_bands_device(_opts(), got[0], 4, 1, world, stats=False)
    ds.set_camera(cam2)
    ds.render_bands_device(_opts(), got[1], 4, 1, world, stats=False)
    torch.cuda.synchronize()
    assert not torch.equal(want[0], want[1])
    for g, w in zip(got, want):
        assert torch.equal(g, w)


@pytest.mark.parametrize("world", [4, 8])
def test_pipelined_calls_on_two_streams(gpu, world):
    """Pipelined calls alternating between two streams A and B with no host
    sync: the library orders each call after the scene's previous one
    (render_device waits on `done` across streams), so every buffer equals
    the serial render and the Stats the last call left equal its serial
    Stats. (Letting call k + 1 render into call k's tail this way was
    measured and rejected: DESIGN.md (e), round 6.)"""
    import torch
    from rtmi import abi
    ref_ds = _scene("0")
    ds = _scene("1")
    rows = band_rows(H, 4, world)
    refs, ref_st = [], []
    for r in range(world):
        b = torch.full((rows * W * 3,), -7.0, dtype=torch.float32, device="cuda")
        ref_st.append(ref_ds.render_bands_device(_opts(), b, 4, r, world))
        refs.append(b)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs = [torch.full((rows * W * 3,), -7.0, dtype=torch.float32, device="cuda") for _ in range(3 * world)]
    torch.cuda.synchronize()
    for k in range(3 * world):
        ds.render_bands_device(_opts(), outs[k], 4, k % world, world, stream=streams[k % 2], stats=False)
        assert _pipelined(ds)[0], k
    # the last call's Stats (kept: no RT_FLAG_NO_STATS), read without a sync
    st = abi.rt_stats()
    assert lib().rt_scene_last_stats(ds.h, C.byref(st)) == 0
    assert Stats.from_c(st) == ref_st[(3 * world - 1) % world]
    torch.cuda.synchronize()
    for k in range(3 * world):
        assert torch.equal(outs[k], refs[k % world]), (k, float((outs[k] - refs[k % world]).abs().max()))
