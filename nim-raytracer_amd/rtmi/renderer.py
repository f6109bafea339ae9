"""Renderer API over librtmi.so, mirroring src/renderer/renderer.nim.

    initRenderer(device)                         renderer.nim:214-215
    renderLine(scene, opts, fb, y, step, maxStep) -> Stats
                                                 renderer.nim:162-211
plus the whole-frame and multi-GPU forms that replace the scanline worker
pool (src/raytracer.nim:25-109, src/concurrency/workerpool.nim) with one GPU
dispatch. `scene` is the reference's Scene (renderLine caches its device copy,
as the Nim binding in INTEGRATION.md does) or a DeviceScene: the Scene flattened and
uploaded once (BVH built) — the Nim shim in INTEGRATION.md does the same.
"""
import contextlib
import ctypes as C
import threading

import numpy as np

from . import abi, glm
from ._lib import RtmiError, check, lib
from .scene import Options, Scene, Stats, flatten


def initRenderer(device=0):
    """Bind this thread to GPU `device` (must be gfx950)."""
    check(lib().rt_init(int(device)))


def device_count():
    return int(lib().rt_device_count())


class DeviceScene:
    """A Scene resident in HBM on one GPU (objects, lights, BVH, triangles)."""

    def __init__(self, scene: Scene, device=0, bvh_builder=abi.RT_BVH_SAH):
        """bvh_builder: abi.RT_BVH_SAH (host binned SAH, default) or
        abi.RT_BVH_PLOC (built on the GPU); images and Stats are the same."""
        initRenderer(device)
        self.device = device
        self.scene = scene
        flat = flatten(scene)
        flat.desc.bvh_builder = int(bvh_builder)
        h = C.c_void_p()
        check(lib().rt_scene_create(C.byref(flat.desc), C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().rt_scene_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self):
        i = abi.rt_scene_info()
        check(lib().rt_scene_get_info(self.h, C.byref(i)))
        return i.as_dict()

    def set_camera(self, cameraToWorld=None, fov=None):
        """Scene.cameraToWorld / Scene.fov for the next render calls
        (renderLine re-reads them every call, renderer.nim:135-136,150-153);
        None: this DeviceScene's Scene's current values."""
        m = self.scene.cameraToWorld if cameraToWorld is None else cameraToWorld
        f = self.scene.fov if fov is None else fov
        arr = (C.c_double * 16)(*[float(x) for x in glm.flat(m)])
        check(lib().rt_scene_set_camera(self.h, arr, float(f)))

    # -- host framebuffer (the pool-compatible path) ----------------------
    def render_lines(self, opts: Options, fb, y0, y1, step=1, maxStep=1) -> Stats:
        """renderLine for every y in countup(y0, y1-1, step); fb is a
        C-contiguous float32 array of shape (h, w, 3) (framebuf.nim layout)."""
        if not (isinstance(fb, np.ndarray) and fb.dtype == np.float32 and fb.flags.c_contiguous
                and fb.shape == (opts.height, opts.width, 3)):
            raise ValueError("fb must be a C-contiguous float32 array of shape (height, width, 3)")
        o = opts.to_c()
        st = abi.rt_stats()
        check(lib().rt_render_lines(self.h, C.byref(o), fb.ctypes.data_as(C.POINTER(C.c_float)),
                                    opts.width, opts.height, int(y0), int(y1), int(step),
                                    int(maxStep), C.byref(st)))
        return Stats.from_c(st)

    # -- device framebuffer (the fast path) --------------------------------
    def render_device(self, opts: Options, d_fb, y0=0, y1=None, step=1, maxStep=1, stream=None,
                      stats=True):
        """Render rows into a device buffer (int pointer or torch tensor of
        height*width*3 float32). With stats=False nothing synchronises."""
        ptr = _ptr(d_fb, opts.width * opts.height * 3)
        o = opts.to_c()
        st = abi.rt_stats()
        check(lib().rt_render_lines_device(self.h, C.byref(o), C.c_void_p(ptr), int(y0),
                                           int(opts.height if y1 is None else y1), int(step),
                                           int(maxStep), _stream(stream),
                                           C.byref(st) if stats else None))
        return Stats.from_c(st) if stats else None

    def render_bands_device(self, opts: Options, d_bands, band_h, rank, world, stream=None,
                            stats=True):
        rows = band_rows(opts.height, band_h, world)
        ptr = _ptr(d_bands, rows * opts.width * 3)
        o = opts.to_c()
        st = abi.rt_stats()
        check(lib().rt_render_bands_device(self.h, C.byref(o), C.c_void_p(ptr), int(band_h), int(rank),
                                           int(world), _stream(stream), C.byref(st) if stats else None))
        return Stats.from_c(st) if stats else None

    def last_pipelined(self):
        """Whether the last render call was pipelined (its build on the
        scene's build stream, its own buffer set: rtmi.cpp rt_scene::pipe) —
        such calls on two alternating streams may render at once."""
        f = lib().rtmi_test_last_pipelined
        f.restype = C.c_int
        f.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
        s = C.c_int32()
        r = f(self.h, C.byref(s))
        if r < 0:
            raise RuntimeError("rtmi_test_last_pipelined failed")
        return bool(r)

    def last_split(self):
        """(lean, general) pixel groups of the last render call (two-class launches)."""
        a, b = C.c_int64(), C.c_int64()
        check(lib().rt_scene_last_split(self.h, C.byref(a), C.byref(b)))
        return int(a.value), int(b.value)

    def last_lean_kernel(self):
        """Kernels of the last call's two classes: bits 0-1 the lean pixels'
        (0 none, 1 k_render_lean, 2 k_render_lean1, 3 merged), bits 2-3 the
        general pixels' (0 k_render_fast, 1 k_render_gen, 2 k_render_gen1,
        3 merged: k_render_mix1)."""
        k = C.c_int32()
        check(lib().rt_scene_last_lean_kernel(self.h, C.byref(k)))
        return int(k.value) & 15

    def last_compacted(self):
        """Whether the last call traced its reflected rays in per-wave
        compacted passes (k_render_wave; reflective scenes with RT_FLAG_COMPACT)."""
        k = C.c_int32()
        check(lib().rt_scene_last_lean_kernel(self.h, C.byref(k)))
        return bool(int(k.value) & 16)

    def last_lean_lanes(self):
        """Lanes per lean pixel of the last two-class call (4 or 16:
        k_render_lean1q / k_render_mix1; 64: one pixel per wave), 0 if none."""
        k = C.c_int32()
        check(lib().rt_scene_last_lean_kernel(self.h, C.byref(k)))
        return int(k.value) >> 8

    def last_batch(self):
        """(batched, fallback) general pixel groups of the last render call:
        those the batched general kernel took, and of them those it
        re-rendered with the one-sample loop (as of the last call with Stats)."""
        a, b = C.c_int64(), C.c_int64()
        check(lib().rt_scene_last_batch(self.h, C.byref(a), C.byref(b)))
        return int(a.value), int(b.value)

    def last_timing(self):
        """(setup_ms, render_ms) of the last call made with RT_FLAG_TIMING:
        its per-call camera-dependent build and its render kernels (waits)."""
        a, b = C.c_double(), C.c_double()
        check(lib().rt_scene_last_timing(self.h, C.byref(a), C.byref(b)))
        return float(a.value), float(b.value)

    def last_counters(self):
        c = abi.rt_traversal_counters()
        check(lib().rt_scene_last_counters(self.h, C.byref(c)))
        return c.as_dict()


def band_rows(height, band_h, world):
    out = C.c_int32()
    check(lib().rt_band_rows(int(height), int(band_h), int(world), C.byref(out)))
    return out.value


def unshard_bands_device(d_gathered, d_fb, width, height, band_h, world, stream=None):
    rows = band_rows(height, band_h, world)
    check(lib().rt_unshard_bands_device(C.c_void_p(_ptr(d_gathered, world * rows * width * 3)),
                                        C.c_void_p(_ptr(d_fb, width * height * 3)), int(width),
                                        int(height), int(band_h), int(world), _stream(stream)))


def _shape_key(scene: Scene):
    """Everything of a Scene except the camera that the device copy holds:
    object transforms, materials, sphere radii, the FULL box bounds (all of
    vmin / vmax, geom.nim:169-170), mesh sizes, lights, background — the
    fingerprint INTEGRATION.md's Nim binding (shapeHash) keeps. Mesh vertices
    edited in place (same sizes) are not hashed per call: invalidateScene."""
    from .scene import Box, DistantLight, Sphere, TriangleMesh
    parts = []
    for o in scene.objects:
        g = o.geometry
        parts += [type(g).__name__, np.asarray(g.objectToWorld, np.float64).tobytes(),
                  np.asarray(g.worldToObject, np.float64).tobytes(),
                  np.asarray(o.material.albedo, np.float64).tobytes(), float(o.material.reflection)]
        if isinstance(g, Sphere):
            parts.append(g.r)
        elif isinstance(g, Box):
            parts += [g.vmin.tobytes(), g.vmax.tobytes()]
        elif isinstance(g, TriangleMesh):
            parts += [g.vertices.shape[0], g.faces.shape[0], id(g.vertices), id(g.faces)]
    for li in scene.lights:
        parts += [type(li).__name__, np.asarray(li.color, np.float64).tobytes(), float(li.intensity),
                  np.asarray(li.dir if isinstance(li, DistantLight) else li.pos, np.float64).tobytes()]
    parts.append(np.asarray(scene.bgColor, np.float64).tobytes())
    return tuple(parts)


class _Entry:
    """One cached device copy: the DeviceScene, what it was built from, and
    the renderLine calls running on it (renders happen outside the cache's
    lock, so a replaced or invalidated copy is closed by whichever comes
    last: the replacement, or the last of those calls)."""
    __slots__ = ("ds", "shape", "cam", "fov", "users", "retired")

    def __init__(self, ds, shape, cam, fov):
        self.ds, self.shape, self.cam, self.fov = ds, shape, cam, fov
        self.users = 0
        self.retired = False


class _DeviceCache:
    """The Nim binding's `deviceScene` in Python: one device
    copy per Scene, created on first use, re-created when the shape key
    changes, its camera pushed (rt_scene_set_camera) when Scene.cameraToWorld
    / fov moved — renderLine re-reads them on every call (renderer.nim:135-136,
    150-153). Re-entrant like renderLine (the pool calls it from
    countProcessors() threads at once, workerpool.nim:72-99): lookups,
    creation and camera pushes hold one lock; the render call itself runs
    outside it (the library serialises calls per scene), counted in its
    entry, and a copy that is replaced or invalidated meanwhile is destroyed
    only once its last call has returned (no use after free). Entries are
    keyed weakly: when a Scene is collected, its device copy is released
    (the cache no longer keeps every Scene and its GPU buffers
    alive)."""

    def __init__(self):
        # re-entrant: a Scene collected while this thread holds the lock runs
        # its weakref callback (_collected) on this thread
        self._lock = threading.RLock()
        self._entries = {}  # id(scene) -> (weakref to the scene, _Entry)

    def _drop(self, e):
        # under the lock: retire e; close it now if no call is running on it
        e.retired = True
        return e.ds if e.users == 0 else None

    def acquire(self, scene: Scene, device=0):
        """(DeviceScene, entry) with the entry's call count raised; pass the
        entry to release() when the call has returned."""
        import weakref
        shape = _shape_key(scene)
        cam = np.asarray(scene.cameraToWorld, np.float64).tobytes()
        fov = float(scene.fov)
        stale = None
        with self._lock:
            key = id(scene)
            item = self._entries.get(key)
            e = item[1] if item is not None and item[0]() is scene else None
            if e is not None and e.shape != shape:  # geometry / materials / lights changed
                stale = self._drop(e)
                e = None
            if e is None:
                ds = DeviceScene(scene, device)
                ds.scene = weakref.proxy(scene)  # the cache must not keep the Scene alive
                e = _Entry(ds, shape, cam, fov)
                self._entries[key] = (weakref.ref(scene, lambda _r, k=key: self._collected(k)), e)
            elif e.cam != cam or e.fov != fov:  # the camera moved: the next call renders it
                e.ds.set_camera(scene.cameraToWorld, fov)
                e.cam, e.fov = cam, fov
            e.users += 1
        if stale is not None:
            stale.close()
        return e.ds, e

    def release(self, e):
        with self._lock:
            e.users -= 1
            last = e.retired and e.users == 0
        if last:
            e.ds.close()

    def get(self, scene: Scene, device=0) -> "DeviceScene":
        """The device copy, NOT held: for single-threaded callers that keep
        it in step with invalidate() themselves. A concurrent
        invalidateScene, shape change or collection of the Scene may close
        the returned copy while it is in use; threaded callers use held()
        (or renderLine, which holds the copy for each call)."""
        ds, e = self.acquire(scene, device)
        self.release(e)
        return ds

    @contextlib.contextmanager
    def held(self, scene: Scene, device=0):
        """`with held(scene) as ds:` the device copy, kept open until the
        block ends (acquire / release around it) even if another thread
        invalidates or replaces it meanwhile."""
        ds, e = self.acquire(scene, device)
        try:
            yield ds
        finally:
            self.release(e)

    def invalidate(self, scene: Scene):
        with self._lock:
            item = self._entries.pop(id(scene), None)
            stale = self._drop(item[1]) if item is not None else None
        if stale is not None:
            stale.close()

    def _collected(self, key):
        with self._lock:
            item = self._entries.get(key)
            if item is None or item[0]() is not None:
                return
            del self._entries[key]
            stale = self._drop(item[1])
        if stale is not None:
            stale.close()

    def __len__(self):
        with self._lock:
            return len(self._entries)


_cache = _DeviceCache()


def deviceScene(scene: Scene, device=0) -> "DeviceScene":
    """The cached device copy of `scene` (INTEGRATION.md deviceScene).
    Single-threaded use only: the copy is not held (see heldDeviceScene)."""
    return _cache.get(scene, device)


def heldDeviceScene(scene: Scene, device=0):
    """Context manager: the cached device copy of `scene`, held open for the
    block (safe against a concurrent invalidateScene / Scene edit)."""
    return _cache.held(scene, device)


def invalidateScene(scene: Scene):
    """After editing mesh vertices / faces in place (same sizes)."""
    _cache.invalidate(scene)


def renderLine(scene, opts: Options, fb, y, step=1, maxStep=1) -> Stats:
    """renderer.nim:162-211 — one scanline (and its step x step blocks).
    `scene` is the reference's Scene (its device copy is cached and kept in
    step with the Scene's camera, as the Nim binding does) or a DeviceScene."""
    if isinstance(scene, DeviceScene):
        return scene.render_lines(opts, fb, y, y + 1, step, maxStep)
    ds, e = _cache.acquire(scene)
    try:
        return ds.render_lines(opts, fb, y, y + 1, step, maxStep)
    finally:
        _cache.release(e)


def render_frame(scene: DeviceScene, opts: Options, fb=None):
    """Whole frame through the host-framebuffer path. Returns (fb, Stats)."""
    if fb is None:
        fb = np.zeros((opts.height, opts.width, 3), dtype=np.float32)
    st = scene.render_lines(opts, fb, 0, opts.height, 1, 1)
    return fb, st


def ppm_encode_device(d_fb, width, height, bits=8, sRGB=True, stream=None):
    """writePpm's payload (framebuf.nim:55-93) of a device framebuffer,
    quantised on the GPU; returns (header bytes, uint8 CUDA tensor)."""
    import torch
    n = lib().rt_ppm_payload_bytes(int(width), int(height), int(bits))
    if n < 0:
        raise RtmiError(n, lib().rt_last_error().decode())
    out = torch.empty(n, dtype=torch.uint8, device=d_fb.device)
    check(lib().rt_ppm_encode_device(C.c_void_p(_ptr(d_fb, width * height * 3)), int(width), int(height),
                                     int(bits), 1 if sRGB else 0, C.c_void_p(int(out.data_ptr())),
                                     _stream(stream)))
    buf = C.create_string_buffer(64)
    hl = lib().rt_ppm_header(int(width), int(height), int(bits), buf, 64)
    if hl < 0:
        raise RtmiError(hl, lib().rt_last_error().decode())
    return buf.raw[:hl], out


class MultiDeviceScene:
    """One process, several GPUs (rt_multi_*, SURVEY.md 8(b)
    rt_render_frame_multi): the scene replicated on every listed device
    (repeats allowed), bands dealt round-robin, gathered on devices[0]."""

    def __init__(self, scene: Scene, devices=(0,), band_h=4):
        initRenderer(devices[0])
        self.devices = list(devices)
        flat = flatten(scene)
        arr = (C.c_int32 * len(self.devices))(*self.devices)
        h = C.c_void_p()
        check(lib().rt_multi_create(C.byref(flat.desc), arr, len(self.devices), int(band_h), C.byref(h)))
        self.h = h

    def set_camera(self, cameraToWorld, fov):
        """rt_scene_set_camera on every rank's scene."""
        arr = (C.c_double * 16)(*[float(x) for x in glm.flat(cameraToWorld)])
        check(lib().rt_multi_set_camera(self.h, arr, float(fov)))

    def render_frame(self, opts: Options, fb) -> Stats:
        """Whole frame into a host (h, w, 3) float32 array."""
        if not (isinstance(fb, np.ndarray) and fb.dtype == np.float32 and fb.flags.c_contiguous
                and fb.shape == (opts.height, opts.width, 3)):
            raise ValueError("fb must be a C-contiguous float32 array of shape (height, width, 3)")
        o = opts.to_c()
        st = abi.rt_stats()
        check(lib().rt_render_frame_multi(self.h, C.byref(o), fb.ctypes.data_as(C.POINTER(C.c_float)),
                                          opts.width, opts.height, C.byref(st)))
        return Stats.from_c(st)

    def render_frame_device(self, opts: Options, d_fb) -> Stats:
        """Whole frame into a device buffer on devices[0]; waits, returns Stats."""
        ptr = _ptr(d_fb, opts.width * opts.height * 3)
        o = opts.to_c()
        st = abi.rt_stats()
        check(lib().rt_render_frame_multi_device(self.h, C.byref(o), C.c_void_p(ptr), C.byref(st)))
        return Stats.from_c(st)

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            lib().rt_multi_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ResponseMsg:
    """ResponseMsg (raytracer.nim:21-23) plus the line it answers."""

    def __init__(self, line, stats):
        self.line = line
        self.stats = stats


class RenderQueue:
    """WorkerPool[WorkMsg, ResponseMsg] (src/concurrency/workerpool.nim) as
    raytracer.nim / gui.nim drive it, over the GPU (rt_queue_*): queued
    lines that form a run at one step become one launch; every line gets its
    response; a run's Stats ride on its last response (callers sum them)."""

    numActiveWorkers = 1  # one device "worker"; the pool size has no GPU meaning
    poolSize = 1

    def __init__(self, ds: DeviceScene):
        self.ds = ds
        h = C.c_void_p()
        check(lib().rt_queue_create(ds.h, C.byref(h)))
        self.h = h
        self._fbs = {}  # framebuffers the queue's thread may still write

    def state(self):
        return lib().rt_queue_state(self.h)

    def isReady(self):
        return lib().rt_queue_is_ready(self.h) == 1

    def waitForReady(self, timeout=1):
        """Commands complete before they return: always ready."""

    def start(self):
        return lib().rt_queue_start(self.h) == 1

    def stop(self):
        return lib().rt_queue_stop(self.h) == 1

    def queueWork(self, opts: Options, framebuf, line, step=0, maxStep=0):
        """WorkMsg{opts, framebuf, line, step, maxStep}: framebuf is the
        (h, w, 3) float32 array the line is rendered into."""
        if not (isinstance(framebuf, np.ndarray) and framebuf.dtype == np.float32 and framebuf.flags.c_contiguous
                and framebuf.shape == (opts.height, opts.width, 3)):
            raise ValueError("framebuf must be a C-contiguous float32 array of shape (height, width, 3)")
        o = opts.to_c()
        check(lib().rt_queue_work(self.h, C.byref(o), framebuf.ctypes.data_as(C.POINTER(C.c_float)),
                                  opts.width, opts.height, int(line), int(step), int(maxStep)))
        self._fbs[framebuf.ctypes.data] = framebuf

    def tryRecvResult(self):
        """(available, ResponseMsg); a failed line raises RtmiError."""
        r = abi.rt_response()
        n = lib().rt_queue_try_recv(self.h, C.byref(r))
        if n < 0:
            raise RtmiError(n, lib().rt_last_error().decode())
        if n == 0:
            return False, None
        if r.status != 0:
            raise RtmiError(r.status, r.error.decode(errors="replace"))
        if lib().rt_queue_pending(self.h) == 0:
            self._fbs.clear()
        return True, ResponseMsg(r.line, Stats.from_c(r.stats))

    def reset(self):
        return lib().rt_queue_reset(self.h) == 1

    def shutdown(self):
        return lib().rt_queue_shutdown(self.h) == 1

    def close(self):
        """workerpool.nim close: only after shutdown."""
        if self.h is None or self.state() != abi.RT_QUEUE_SHUTDOWN:
            return False
        check(lib().rt_queue_destroy(self.h))
        self.h = None
        self._fbs.clear()
        return True

    def __del__(self):
        try:
            if self.h is not None:
                lib().rt_queue_destroy(self.h)
                self.h = None
        except Exception:
            pass


def initRenderWorkers(ds: DeviceScene, numActiveWorkers=0, poolSize=0):
    """initRenderWorkers (raytracer.nim:35-38) -> a RenderQueue."""
    return RenderQueue(ds)


def rgba_encode_device(d_fb, width, height, alpha=0xFF, stream=None):
    """ImageRGBA.copyFrom (image.nim:45-54) of a device framebuffer on the
    GPU; returns a (height, width, 4) uint8 CUDA tensor."""
    import torch
    out = torch.empty((int(height), int(width), 4), dtype=torch.uint8, device=d_fb.device)
    check(lib().rt_rgba_encode_device(C.c_void_p(_ptr(d_fb, width * height * 3)), int(width), int(height),
                                      int(alpha) & 0xFF, C.c_void_p(int(out.data_ptr())), _stream(stream)))
    return out


def write_ppm_device(d_fb, width, height, filename, bits=8, sRGB=True, stream=None):
    """Framebuf.writePpm for a device framebuffer: the quantisation runs on
    the GPU and only the 8/16-bit payload crosses PCIe."""
    header, payload = ppm_encode_device(d_fb, width, height, bits, sRGB, stream)
    try:
        with open(filename, "wb") as f:
            f.write(header)
            f.write(payload.cpu().numpy().tobytes())
        return True
    except OSError:
        return False


def _ptr(buf, min_floats):
    if isinstance(buf, int):
        return buf
    try:  # torch tensor
        import torch  # noqa: F401
        if not buf.is_cuda or buf.dtype.itemsize != 4 or not buf.is_contiguous():
            raise ValueError("device buffer must be a contiguous 4-byte CUDA/HIP tensor")
        if buf.numel() < min_floats:
            raise ValueError(f"device buffer holds {buf.numel()} floats, need {min_floats}")
        return int(buf.data_ptr())
    except AttributeError:
        raise TypeError("device buffer must be an int pointer or a torch tensor") from None


def _stream(stream):
    """hipStream_t for the C-ABI. None = the current torch stream when torch
    is loaded (so torch ops and renders are ordered), else HIP's null stream."""
    if stream is None:
        import sys
        torch = sys.modules.get("torch")
        if torch is not None and torch.cuda.is_available() and torch.cuda.is_initialized():
            return C.c_void_p(int(torch.cuda.current_stream().cuda_stream) or None)
        return None
    if isinstance(stream, int):
        return C.c_void_p(stream or None)
    return C.c_void_p(int(stream.cuda_stream) or None)


__all__ = ["DeviceScene", "RtmiError", "band_rows", "device_count", "deviceScene", "heldDeviceScene", "initRenderer", "invalidateScene",
           "ppm_encode_device", "renderLine", "render_frame", "unshard_bands_device", "write_ppm_device"]
