"""Per-call camera-dependent data (rt_frame.h): every float32 render call
builds its pixels' camera-ray face lists, pixel records (list length + shadow
skip bits) and lean / general lists on the device; nothing that depends on
the camera survives from one call to the next (renderLine does all per-pixel
work on every call, renderer.nim:162-211).

* the device-built lists and records equal the host builders' (rt_bins.cpp,
  whose completeness test_bins_cpu.py checks against every face in float64):
  same faces per pixel, same records, for whole frames, band sets and row
  ranges;
* rt_scene_set_camera (Scene.cameraToWorld / fov, re-read by renderLine on
  every call, renderer.nim:135-136,150-153) changes the next frame to the
  oracle's for the new camera, and frames do not depend on what an earlier
  call rendered.
"""
import ctypes as C

import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, akGrid, scenes
from rtmi._lib import lib
from rtmi.abi import RT_FLAG_NO_REORDER
from rtmi.glm import X_AXIS, Y_AXIS, degToRad, mat4, rotate, translate, vec3
from rtmi.renderer import DeviceScene, band_rows

pytestmark = pytest.mark.gpu

BIAS = 1e-4


def _opts(w, h, m=16, prec=Precision.fp32, flags=RT_FLAG_NO_REORDER):
    return Options(width=w, height=h, antialias=Antialias(akGrid, m), bias=BIAS, precision=prec, flags=flags)


def _device_lists(ds, w, h):
    L = lib()
    f = L.rtmi_test_frame_lists
    f.restype = C.c_int64
    f.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    off = np.zeros(w * h + 1, dtype=np.int32)
    info = np.zeros(w * h, dtype=np.uint32)
    cap = 1 << 24
    ent = np.zeros(cap, dtype=np.int32)
    n = f(ds.h, off.ctypes.data, ent.ctypes.data, cap, info.ctypes.data)
    assert n >= 0, L.rt_last_error()
    return off, ent, info


def _host_lists(ds, w, h, bias=BIAS):
    L = lib()
    f = L.rtmi_test_host_lists
    f.restype = C.c_int64
    f.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_double, C.c_void_p, C.c_void_p, C.c_int64, C.c_void_p]
    off = np.zeros(w * h + 1, dtype=np.int32)
    info = np.zeros(w * h, dtype=np.uint32)
    cap = 1 << 24
    ent = np.zeros(cap, dtype=np.int32)
    n = f(ds.h, w, h, bias, off.ctypes.data, ent.ctypes.data, cap, info.ctypes.data)
    assert 0 <= n <= cap
    return off, ent, info


def _slot_lg(ds, lg=-1):
    f = lib().rtmi_test_slot_lg
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int32]
    r = f(ds.h, lg)
    assert r >= 0
    return r


def _compare(ds, w, h, pixels, records=True):
    """The device lists of the last call equal the host builders' on `pixels`
    (flat indices): same length and (for lists within their 2^lg slots —
    longer ones take the BVH) same face set per pixel, same record."""
    d_off, d_ent, d_info = _device_lists(ds, w, h)
    h_off, h_ent, h_info = _host_lists(ds, w, h)
    d_len = d_off[pixels + 1] - d_off[pixels]
    h_len = h_off[pixels + 1] - h_off[pixels]
    assert np.array_equal(d_len, h_len), int(np.count_nonzero(d_len != h_len))
    K = 1 << _slot_lg(ds)
    for p in pixels[(h_len > 0) & (h_len <= K)]:
        a = np.sort(d_ent[d_off[p]:d_off[p + 1]])
        b = np.sort(h_ent[h_off[p]:h_off[p + 1]])
        assert np.array_equal(a, b), int(p)
    if records:
        bad = np.flatnonzero(d_info[pixels] != h_info[pixels])
        assert bad.size == 0, (bad.size, [(int(pixels[i]), hex(d_info[pixels[i]]), hex(h_info[pixels[i]]))
                                          for i in bad[:5]])
    return int(h_len.sum()), int(np.count_nonzero(h_info[pixels] >> 24))


def _moved_camera():
    return translate(rotate(rotate(mat4(1.0), Y_AXIS, degToRad(14.0)), X_AXIS, degToRad(-9.0)), vec3(1.2, 3.9, 4.0))


@pytest.mark.parametrize("name", ["bunny", "bunny-moved", "torus", "mesh-mix"])
def test_device_lists_equal_host_builders(gpu, name):
    import torch
    if name.startswith("bunny"):
        sc = scenes.mesh_bunny()
    elif name == "torus":
        sc = scenes.torus_scene(U=200, V=100)
    else:
        sc = scenes.mesh_mix()
    ds = DeviceScene(sc)
    if name == "bunny-moved":
        ds.set_camera(_moved_camera(), 44.0)
    w, h = 480, 270
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    ds.render_device(_opts(w, h), fb)
    entries, skipped = _compare(ds, w, h, np.arange(w * h))
    assert entries > 0
    if name.startswith("bunny"):
        assert skipped > w * h // 2  # most ground / sky pixels carry skip bits
    lean, general = ds.last_split()
    if name != "mesh-mix":
        assert lean > 0 and general > 0 and lean + general == w * h


def test_device_lists_full_c3_frame(gpu):
    import torch
    ds = DeviceScene(scenes.mesh_bunny())
    w, h = 1920, 1080
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    ds.render_device(_opts(w, h, flags=0), fb, stats=False)
    _compare(ds, w, h, np.arange(w * h))


def test_device_lists_bands_and_rows(gpu):
    """A rank's band set and a row range build exactly their own pixels'
    lists (the multi-GPU setup is sharded: no rank bins the whole frame)."""
    import torch
    ds = DeviceScene(scenes.mesh_bunny())
    w, h, bh, world = 320, 180, 4, 3
    for rank in range(world):
        rows = band_rows(h, bh, world)
        buf = torch.zeros(rows * w * 3, dtype=torch.float32, device="cuda")
        ds.render_bands_device(_opts(w, h), buf, bh, rank, world)
        ys = [y for y in range(h) if (y // bh) % world == rank]
        pix = np.concatenate([np.arange(y * w, (y + 1) * w) for y in ys])
        _compare(ds, w, h, pix)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    ds.render_device(_opts(w, h), fb, y0=0, y1=h)
    ds.render_device(_opts(w, h), fb, y0=37, y1=121)
    pix = np.arange(37 * w, 121 * w)
    _compare(ds, w, h, pix)


def _oracle(scene, opts):
    import oracle
    fb, st, _ = oracle.OracleScene(scene).render(opts)
    return fb, st


@pytest.mark.parametrize("prec", [Precision.fp64, Precision.fp32])
def test_set_camera_renders_the_new_camera(gpu, prec):
    """A camera change through rt_scene_set_camera gives the oracle's frame
    for the new camera (float64 bit-exact, float32 within the parity
    tolerance) — the Nim binding's per-frame camera update."""
    import torch
    sc = scenes.mesh_bunny()
    ds = DeviceScene(sc)
    w, h = 96, 64
    o = _opts(w, h, m=2 if prec == Precision.fp64 else 16, prec=prec)
    fb0 = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    ds.render_device(o, fb0)
    sc.cameraToWorld = _moved_camera()
    sc.fov = 44.0
    ds.set_camera()  # re-read from the Scene, as the Nim binding does each frame
    fb1 = torch.zeros_like(fb0)
    st = ds.render_device(o, fb1)
    got = fb1.view(h, w, 3).cpu().numpy()
    ref, rst = _oracle(sc, o)
    assert not torch.equal(fb0, fb1)
    assert st.numPrimaryRays == rst.numPrimaryRays
    if prec == Precision.fp64:
        assert np.array_equal(got, ref) and st == rst
    else:
        err = np.abs(got - ref).max(axis=2)
        assert (err <= 2e-3).mean() >= 0.995 and err.mean() <= 2e-4, (float((err <= 2e-3).mean()), float(err.mean()))
        assert abs(st.numShadowRays - rst.numShadowRays) <= 1e-3 * rst.numShadowRays


def test_frames_do_not_depend_on_earlier_calls(gpu):
    """Camera A, camera B, camera A again: the two A frames are bit-identical,
    and the B frame equals a fresh scene created with camera B."""
    import torch
    sc = scenes.mesh_bunny()
    ds = DeviceScene(sc)
    w, h = 320, 180
    o = _opts(w, h, flags=0)
    a0 = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    sa0 = ds.render_device(o, a0)
    ds.set_camera(_moved_camera(), 44.0)
    b = torch.zeros_like(a0)
    sb = ds.render_device(o, b)
    ds.set_camera(sc.cameraToWorld, sc.fov)
    a1 = torch.zeros_like(a0)
    sa1 = ds.render_device(o, a1)
    assert torch.equal(a0, a1) and sa0 == sa1
    sc2 = scenes.mesh_bunny()
    sc2.cameraToWorld = _moved_camera()
    sc2.fov = 44.0
    ref = torch.zeros_like(a0)
    sref = DeviceScene(sc2).render_device(o, ref)
    assert torch.equal(b, ref) and sb == sref


def test_set_camera_rejects_bad_input(gpu):
    from rtmi._lib import RtmiError
    ds = DeviceScene(scenes.mesh_bunny())
    with pytest.raises(RtmiError):
        ds.set_camera(np.full((4, 4), np.nan), 50.0)
    with pytest.raises(RtmiError):
        ds.set_camera(mat4(1.0), 180.0)
