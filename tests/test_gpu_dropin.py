"""The drop-in renderLine under the reference's callers, and the boundary's
failure behaviour.

* renderLine is re-entrant: the reference's pool calls it from
  countProcessors() threads at once on disjoint rows of a shared read-only
  Scene (workerpool.nim:72-99, raytracer.nim:25-32). Here N threads call
  rtmi.renderer.renderLine with the reference's Scene object (the device copy
  is cached behind a lock and follows the Scene's camera, as the Nim binding
  in INTEGRATION.md does); a camera move and a box resized in y between
  frames render the oracle's frames for the new Scene.
* A render call whose camera-ray lists overflowed their entry capacity
  returns RT_E_DEVICE (never RT_OK with a truncated image): a test hook caps
  the capacity.
* rt_scene_last_split describes the last call, including a float64 call
  after a two-class float32 call.
"""
import ctypes as C
import threading

import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, akGrid, akNone, scenes
from rtmi._lib import RtmiError, lib
from rtmi.abi import RT_E_DEVICE
from rtmi.glm import X_AXIS, Y_AXIS, degToRad, mat4, rotate, translate, vec3
from rtmi.renderer import DeviceScene, deviceScene, invalidateScene, renderLine

pytestmark = pytest.mark.gpu

BIAS = 1e-4


def _pool_frame(scene, opts, nthreads=8):
    """raytracer.nim's scanline pool: nthreads workers pull rows and call
    renderLine(scene, ...) concurrently; Stats summed as raytracer.nim:95."""
    fb = np.zeros((opts.height, opts.width, 3), np.float32)
    rows = list(range(opts.height))
    lock = threading.Lock()
    tot = []
    errs = []

    def worker():
        from rtmi.scene import Stats
        mine = Stats()
        try:
            while True:
                with lock:
                    if not rows:
                        break
                    y = rows.pop()
                mine += renderLine(scene, opts, fb, y)
        except Exception as e:  # surfaced below
            errs.append(e)
        with lock:
            tot.append(mine)

    ts = [threading.Thread(target=worker) for _ in range(nthreads)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errs, errs
    from rtmi.scene import Stats
    st = Stats()
    for s in tot:
        st += s
    return fb, st


def _oracle(scene, opts):
    import oracle
    fb, st, _ = oracle.OracleScene(scene).render(opts, nthreads=16)
    return fb, st


def _moved_camera():
    return translate(rotate(rotate(mat4(1.0), Y_AXIS, degToRad(-11.0)), X_AXIS, degToRad(-7.0)), vec3(-0.8, 4.6, 3.0))


@pytest.mark.parametrize("name", ["boxes2", "mesh-bunny"])
def test_threaded_renderline_follows_scene_edits(gpu, name):
    """8 threads x disjoint rows through renderLine(Scene, ...): frame 1, then
    the camera moves (Scene.cameraToWorld / fov), then (boxes2) a box grows in
    y only: every frame is the oracle's, float64 bit-exact with equal Stats."""
    sc = scenes.SCENES[name]()
    opts = Options(width=72, height=40, antialias=Antialias(akGrid, 2), bias=BIAS, precision=Precision.fp64)
    try:
        got, gst = _pool_frame(sc, opts)
        ref, rst = _oracle(sc, opts)
        assert np.array_equal(got, ref) and gst == rst
        ds1 = deviceScene(sc)
        sc.cameraToWorld = _moved_camera()
        sc.fov = 47.0
        got, gst = _pool_frame(sc, opts)
        ref, rst = _oracle(sc, opts)
        assert np.array_equal(got, ref) and gst == rst
        assert deviceScene(sc) is ds1  # a camera move keeps the device scene (rt_scene_set_camera)
        if name == "boxes2":
            from rtmi.scene import Box
            box = next(o.geometry for o in sc.objects if isinstance(o.geometry, Box))
            box.vmax = box.vmax + np.array([0.0, 0.35, 0.0])  # y only: a fingerprint of x alone misses it
            got, gst = _pool_frame(sc, opts)
            ref, rst = _oracle(sc, opts)
            assert np.array_equal(got, ref) and gst == rst
            assert deviceScene(sc) is not ds1  # re-created for the new geometry
    finally:
        invalidateScene(sc)


def test_threaded_renderline_fp32_c3_scene(gpu):
    """The benchmark's scene and sampling (bunny, akGrid 16) through 8
    renderLine threads with a camera change: float32 within the parity
    tolerance of the oracle for both cameras."""
    sc = scenes.mesh_bunny()
    opts = Options(width=96, height=54, antialias=Antialias(akGrid, 16), bias=BIAS, precision=Precision.fp32)
    try:
        for cam in (None, _moved_camera()):
            if cam is not None:
                sc.cameraToWorld = cam
                sc.fov = 44.0
            got, gst = _pool_frame(sc, opts)
            ref, rst = _oracle(sc, opts)
            err = np.abs(got.astype(np.float64) - ref).max(axis=2)
            assert (err <= 2e-3).mean() >= 0.995 and err.mean() <= 2e-4
            assert gst.numPrimaryRays == rst.numPrimaryRays
            assert gst.numIntersectionTests == pytest.approx(rst.numIntersectionTests, rel=1e-4)
    finally:
        invalidateScene(sc)


def _entry_cap(ds, cap):
    f = lib().rtmi_test_entry_cap
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int64]
    assert f(ds.h, cap) == 0


def test_entry_overflow_fails_the_call(gpu):
    """A fill pass that runs out of entry capacity (forced by the test hook)
    fails the call with RT_E_DEVICE — host path and device path, including a
    device call without Stats (reported by the next call that reads them) —
    and the next call after the cap is lifted renders the right frame."""
    import torch
    sc = scenes.mesh_bunny()
    ds = DeviceScene(sc)
    opts = Options(width=160, height=90, antialias=Antialias(akGrid, 16), bias=BIAS)
    ref = torch.zeros(160 * 90 * 3, dtype=torch.float32, device="cuda")
    sref = ds.render_device(opts, ref)
    _entry_cap(ds, 16)
    fb = np.zeros((90, 160, 3), np.float32)
    with pytest.raises(RtmiError) as e:
        ds.render_lines(opts, fb, 0, 90)
    assert e.value.code == RT_E_DEVICE and "overflow" in str(e.value)
    d = torch.zeros_like(ref)
    with pytest.raises(RtmiError):
        ds.render_device(opts, d)
    ds.render_device(opts, d, stats=False)  # no wait, nothing read yet
    with pytest.raises(RtmiError):
        ds.last_split()  # the overflow is reported by the next read
    ds.last_split()  # ... once
    _entry_cap(ds, 0)
    out = torch.zeros_like(ref)
    assert ds.render_device(opts, out) == sref
    assert torch.equal(out, ref)
    got = np.zeros((90, 160, 3), np.float32)
    ds.render_lines(opts, got, 0, 90)
    assert np.array_equal(got, ref.view(90, 160, 3).cpu().numpy())


def test_last_split_describes_the_last_call(gpu):
    """fp32 two-class call, then an fp64 call: last_split / last_batch report
    the fp64 call (no lean pixels), not the earlier device counts."""
    import torch
    ds = DeviceScene(scenes.mesh_bunny())
    o32 = Options(width=128, height=72, antialias=Antialias(akGrid, 16), bias=BIAS)
    fb = torch.zeros(128 * 72 * 3, dtype=torch.float32, device="cuda")
    ds.render_device(o32, fb)
    lean, general = ds.last_split()
    assert lean > 0 and general > 0
    o64 = Options(width=128, height=72, antialias=Antialias(akNone, 1), bias=BIAS, precision=Precision.fp64)
    ds.render_device(o64, fb)
    lean64, general64 = ds.last_split()
    assert lean64 == 0 and general64 > 0 and general64 != general
    assert ds.last_batch()[0] == 0
    assert ds.last_lean_kernel() == 0
