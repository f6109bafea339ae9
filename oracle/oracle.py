"""ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes wrapper of oracle/build/liboracle_rt.so, the fp64 CPU restatement of the
reference's trace/shade path (rt_oracle.c). Imported only by tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg, always as the checker
or the CPU baseline — never by the product package (nim-raytracer_amd/rtmi).
"""
import ctypes as C
import os
import subprocess
import sys

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_HERE)
sys.path.insert(0, os.path.join(_REPO, "nim-raytracer_amd"))

from rtmi import abi  # noqa: E402  (shared struct layouts only)
from rtmi.scene import Options, Stats, flatten  # noqa: E402

LIB_PATH = os.path.join(_HERE, "build", "liboracle_rt.so")


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def _load():
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    P = C.c_void_p
    dp = C.POINTER(C.c_double)
    lib.oracle_scene_create.restype = P
    lib.oracle_scene_create.argtypes = [C.POINTER(abi.rt_scene_desc)]
    lib.oracle_scene_destroy.restype = None
    lib.oracle_scene_destroy.argtypes = [P]
    lib.oracle_scene_build_bvh.restype = C.c_int
    lib.oracle_scene_build_bvh.argtypes = [P]
    lib.oracle_sample_table.restype = None
    lib.oracle_sample_table.argtypes = [C.c_int32, C.c_int32, C.c_uint64, C.c_int32, C.c_int32, dp, dp]
    lib.oracle_render_line.restype = C.c_int
    lib.oracle_render_line.argtypes = [P, C.POINTER(abi.rt_options), C.POINTER(C.c_float),
                                       C.c_int32, C.c_int32, C.c_int32, C.POINTER(abi.rt_stats)]
    lib.oracle_render_rows_mt.restype = C.c_int
    lib.oracle_render_rows_mt.argtypes = [P, C.POINTER(abi.rt_options), C.POINTER(C.c_float),
                                          C.POINTER(C.c_int32), C.c_int32, C.c_int32, C.c_int32,
                                          C.c_int32, C.POINTER(abi.rt_stats), dp]
    lib.oracle_solve_quadratic.restype = None
    lib.oracle_solve_quadratic.argtypes = [C.c_double, C.c_double, C.c_double, dp, dp]
    lib.oracle_cast_primary_ray.restype = None
    lib.oracle_cast_primary_ray.argtypes = [C.c_int32, C.c_int32, C.c_double, C.c_double,
                                            C.c_double, dp, dp, dp]
    lib.oracle_ray_triangle.restype = C.c_double
    lib.oracle_ray_triangle.argtypes = [dp, dp, dp, dp, dp]
    lib.oracle_aabb_intersect.restype = C.c_double
    lib.oracle_aabb_intersect.argtypes = [dp, dp, dp, dp]
    lib.oracle_sphere_intersect.restype = C.c_double
    lib.oracle_sphere_intersect.argtypes = [C.c_double, dp, dp]
    lib.oracle_trace.restype = C.c_int32
    lib.oracle_trace.argtypes = [P, dp, dp, C.c_double, dp, C.POINTER(C.c_int64),
                                 C.POINTER(abi.rt_stats)]
    lib.oracle_calc_pixel.restype = None
    lib.oracle_calc_pixel.argtypes = [P, C.POINTER(abi.rt_options), C.c_int32, C.c_int32, dp,
                                      C.POINTER(abi.rt_stats)]
    lib.oracle_rgba_component.restype = C.c_uint8
    lib.oracle_rgba_component.argtypes = [C.c_float]
    lib.oracle_ppm_outvalue.restype = C.c_int32
    lib.oracle_ppm_outvalue.argtypes = [C.c_float, C.c_int32, C.c_int32]
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _dp(a):
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float64))
    return a, a.ctypes.data_as(C.POINTER(C.c_double))


def sample_table(kind, m, seed, x, y):
    """(sx, sy) of a stochastic antialias kind's m*m table for pixel (x, y)."""
    sx = np.zeros(m * m)
    sy = np.zeros(m * m)
    lib().oracle_sample_table(int(kind), int(m), int(seed), int(x), int(y),
                              sx.ctypes.data_as(C.POINTER(C.c_double)), sy.ctypes.data_as(C.POINTER(C.c_double)))
    return sx, sy


class OracleScene:
    """The reference algorithm over one flattened scene (fp64). bvh=False:
    the reference's brute-force face loop; bvh=True: the same answers from a
    per-ray fp64 BVH (the "CPU same-BVH" baseline)."""

    def __init__(self, scene, bvh=False):
        self.flat = flatten(scene)
        self.h = lib().oracle_scene_create(C.byref(self.flat.desc))
        if not self.h:
            raise ValueError("oracle rejected the scene description")
        if bvh:
            lib().oracle_scene_build_bvh(self.h)

    def close(self):
        if self.h:
            lib().oracle_scene_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def render_line(self, opts: Options, fb, y, step=1, maxStep=1):
        o = opts.to_c()
        st = abi.rt_stats()
        rc = lib().oracle_render_line(self.h, C.byref(o), fb.ctypes.data_as(C.POINTER(C.c_float)),
                                      y, step, maxStep, C.byref(st))
        if rc != 0:
            raise RuntimeError(f"oracle_render_line failed: {rc}")
        return Stats.from_c(st)

    def render(self, opts: Options, rows=None, step=1, maxStep=1, nthreads=None, fb=None):
        """Render `rows` (default all, in countup(0, h-1, step) order when
        step > 1) with the line-granular thread pool. Returns (fb, Stats, seconds)."""
        if fb is None:
            fb = np.zeros((opts.height, opts.width, 3), dtype=np.float32)
        if rows is None:
            rows = list(range(0, opts.height, step))
        rows_a = np.ascontiguousarray(np.asarray(rows, dtype=np.int32))
        o = opts.to_c()
        st = abi.rt_stats()
        secs = C.c_double(0.0)
        # the GPU box's CPU share is 16 threads (os.cpu_count() there is the whole machine's)
        nthreads = nthreads or min(16, os.cpu_count() or 1)
        rc = lib().oracle_render_rows_mt(self.h, C.byref(o), fb.ctypes.data_as(C.POINTER(C.c_float)),
                                         rows_a.ctypes.data_as(C.POINTER(C.c_int32)), len(rows_a),
                                         step, maxStep, nthreads, C.byref(st), C.byref(secs))
        if rc != 0:
            raise RuntimeError(f"oracle_render_rows_mt failed: {rc}")
        return fb, Stats.from_c(st), secs.value

    def trace(self, orig, dir, tnear=float("inf")):
        oa, op = _dp(orig)
        da, dpp = _dp(dir)
        t = C.c_double(0.0)
        tri = C.c_int64(-1)
        st = abi.rt_stats()
        obj = lib().oracle_trace(self.h, op, dpp, tnear, C.byref(t), C.byref(tri), C.byref(st))
        return obj, t.value, tri.value, Stats.from_c(st)

    def calc_pixel(self, opts: Options, x, y):
        o = opts.to_c()
        out = (C.c_double * 3)()
        st = abi.rt_stats()
        lib().oracle_calc_pixel(self.h, C.byref(o), x, y, out, C.byref(st))
        return np.array(list(out)), Stats.from_c(st)


def solve_quadratic(a, b, c):
    t1, t2 = C.c_double(), C.c_double()
    lib().oracle_solve_quadratic(a, b, c, C.byref(t1), C.byref(t2))
    return t1.value, t2.value


def cast_primary_ray(w, h, x, y, fov, c2w):
    c, cp = _dp(np.asarray(c2w, dtype=np.float64).reshape(16))
    o = (C.c_double * 4)()
    d = (C.c_double * 4)()
    lib().oracle_cast_primary_ray(w, h, x, y, fov, cp, o, d)
    return np.array(list(o)), np.array(list(d))


def ray_triangle(orig, dir, v0, v1, v2):
    arrs = [_dp(a) for a in (orig, dir, v0, v1, v2)]
    return lib().oracle_ray_triangle(*[p for _, p in arrs])


def aabb_intersect(vmin, vmax, orig, dir):
    arrs = [_dp(a) for a in (vmin, vmax, orig, dir)]
    return lib().oracle_aabb_intersect(*[p for _, p in arrs])


def sphere_intersect(r, orig, dir):
    (oa, op), (da, dpp) = _dp(orig), _dp(dir)
    return lib().oracle_sphere_intersect(r, op, dpp)


def rgba_component(v):
    """ImageRGBA.copyFrom's component (image.nim:45-54), oracle_rgba_component."""
    return lib().oracle_rgba_component(float(v))


def ppm_outvalue(v, bits=8, srgb=True):
    return lib().oracle_ppm_outvalue(float(v), bits, 1 if srgb else 0)
