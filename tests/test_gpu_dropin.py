"""The drop-in renderLine under the reference's callers, and the boundary's
failure behaviour.

* renderLine is re-entrant: the reference's pool calls it from
  countProcessors() threads at once on disjoint rows of a shared read-only
  Scene (workerpool.nim:72-99, raytracer.nim:25-32). Here N threads call
  rtmi.renderer.renderLine with the reference's Scene object (the device copy
  is cached behind a lock and follows the Scene's camera, as the Nim binding
  in INTEGRATION.md does); a camera move and a box resized in y between
  frames render the oracle's frames for the new Scene.
* A pixel whose camera-ray list outgrows its slots (a test hook shrinks
  them) renders exactly the same frame and Stats: its camera rays take the
  BVH. The per-call build has no failure mode that returns RT_OK with a
  wrong image.
* rt_scene_last_split describes the last call, including a float64 call
  after a two-class float32 call.
"""
import ctypes as C
import threading

import numpy as np
import pytest

from rtmi import Antialias, Options, Precision, akGrid, akNone, scenes
from rtmi._lib import lib
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


def test_invalidate_during_threaded_renderline(gpu):
    """invalidateScene / a geometry edit while pool threads are
    inside renderLine must not free the device copy under them. 6 threads
    render scanlines in a loop while the main thread invalidates the Scene
    and edits a box 20 times; every scanline either renders (the rows of the
    last pass equal the oracle's frame) or raises nothing — no fault, no
    error — and the replaced copies are all released."""
    import gc
    import weakref
    from rtmi import renderer
    from rtmi.scene import Box
    sc = scenes.boxes2()
    opts = Options(width=64, height=36, antialias=Antialias(akGrid, 2), bias=BIAS, precision=Precision.fp64)
    fb = np.zeros((36, 64, 3), np.float32)
    stop = threading.Event()
    errs = []
    copies = []

    def worker(k):
        try:
            while not stop.is_set():
                for y in range(k, 36, 6):
                    renderLine(sc, opts, fb, y)
        except Exception as e:  # noqa: BLE001
            errs.append(repr(e))

    ts = [threading.Thread(target=worker, args=(k,)) for k in range(6)]
    [t.start() for t in ts]
    box = next(o.geometry for o in sc.objects if isinstance(o.geometry, Box))
    try:
        for i in range(20):
            copies.append(weakref.ref(deviceScene(sc)))
            if i % 2:
                invalidateScene(sc)
            else:
                box.vmax = box.vmax + np.array([0.0, 0.01, 0.0])
    finally:
        stop.set()
        [t.join() for t in ts]
    assert not errs, errs[:3]
    fb[:] = 0
    for y in range(36):
        renderLine(sc, opts, fb, y)
    ref, _ = _oracle(sc, opts)
    assert np.array_equal(fb, ref)
    invalidateScene(sc)
    gc.collect()
    assert all(r() is None or not r().h.value for r in copies)  # every retired copy was destroyed
    n = len(renderer._cache)
    tmp = scenes.boxes2()
    renderLine(tmp, opts, fb, 0)
    assert len(renderer._cache) == n + 1
    del tmp
    gc.collect()
    assert len(renderer._cache) == n  # a collected Scene releases its device copy


def _slot_lg(ds, lg=-1):
    f = lib().rtmi_test_slot_lg
    f.restype = C.c_int
    f.argtypes = [C.c_void_p, C.c_int32]
    r = f(ds.h, lg)
    assert r >= 0
    return r


@pytest.mark.parametrize("lg", [0, 1, 3])
def test_list_past_its_slots_takes_the_bvh(gpu, lg):
    """A pixel whose camera-ray list holds more faces than its 2^lg slots
    (rt_frame.h) keeps its true length in the record, and its camera rays
    take the BVH — the same answers: frames and Stats bit-identical to the
    default slots, host path and device path (no failure mode). With 1 slot
    most bunny pixels overflow; with 8 a few do."""
    import torch
    sc = scenes.mesh_bunny()
    ds = DeviceScene(sc)
    opts = Options(width=160, height=90, antialias=Antialias(akGrid, 16), bias=BIAS)
    ref = torch.zeros(160 * 90 * 3, dtype=torch.float32, device="cuda")
    sref = ds.render_device(opts, ref)
    fb0 = ds.last_batch()[1]  # (at 160x90 the bunny's pixels list many faces: some overflow 32 slots too)
    default = _slot_lg(ds)
    _slot_lg(ds, lg)
    out = torch.zeros_like(ref)
    assert ds.render_device(opts, out) == sref
    assert torch.equal(out, ref)
    assert ds.last_batch()[1] > fb0  # more overflowed general pixels took the one-sample loop + BVH
    got = np.zeros((90, 160, 3), np.float32)
    assert ds.render_lines(opts, got, 0, 90) == sref
    assert np.array_equal(got, ref.view(90, 160, 3).cpu().numpy())
    _slot_lg(ds, default)
    again = torch.zeros_like(ref)
    assert ds.render_device(opts, again) == sref and torch.equal(again, ref)


def test_4k_frames_get_128_slots(gpu):
    """4K frames get 128 list slots per pixel (rtmi.cpp slot_lg_for; 1080p
    keeps 64): the C5 torus's fullest pixels (up to 99 camera-ray faces at
    4K, around row 1184) then stay in the batched kernel instead of taking the
    one-sample BVH loop at ~100x a pixel's cost, and the rows render the same
    frame and Stats as with 64 slots, where they overflow."""
    import torch
    ds = DeviceScene(scenes.torus_scene())
    opts = Options(width=3840, height=2160, antialias=Antialias(akGrid, 8), bias=BIAS)
    y0, y1 = 1176, 1192
    out = torch.zeros(3840 * 2160 * 3, dtype=torch.float32, device="cuda")
    st = ds.render_device(opts, out, y0=y0, y1=y1)
    assert _slot_lg(ds) == 7
    assert ds.last_batch()[1] == 0
    _slot_lg(ds, 6)
    ref = torch.zeros_like(out)
    assert ds.render_device(opts, ref, y0=y0, y1=y1) == st
    assert ds.last_batch()[1] > 0  # at 64 slots some of these pixels overflow
    assert torch.equal(out, ref)
    small = DeviceScene(scenes.mesh_bunny())
    o2 = Options(width=1920, height=1080, antialias=Antialias(akGrid, 16), bias=BIAS)
    fb = torch.zeros(1920 * 1080 * 3, dtype=torch.float32, device="cuda")
    small.render_device(o2, fb, y0=500, y1=508)
    assert _slot_lg(small) == 6


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
