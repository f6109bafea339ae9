"""Mesh ingestion.

- loadGeom: the .geom triangle soup written by src/loaders/objconv.nim:139-153
  and read by test/test.nim:14-26 — little-endian int32 N, then N triangles of
  3 vertices of 3 float32. (The reference's own src/loaders/geomloader.nim is
  broken: it reads no triangle data, geomloader.nim:38-45.)
- loadObj: the native OBJ reader (rt_load_obj, csrc/rt_obj.cpp) with
  src/loaders/obj.nim:87-126's semantics (1-based face indices, first three
  of each `f`, unparsable tokens -> 0), normals computed per face by the
  library exactly as calcNormals obj.nim:65-84.
- objconv: objconv.nim's OBJ -> .geom conversion (rt_write_geom).
"""
import os

import numpy as np

from .glm import mat4
from .scene import TriangleMesh


def readGeom(path):
    """Return (N, 3, 3) float32 triangle soup."""
    with open(path, "rb") as f:
        data = f.read()
    if len(data) < 4:
        raise ValueError(f"{path}: truncated .geom header")
    n = int(np.frombuffer(data[:4], dtype="<i4")[0])
    if n < 0 or len(data) < 4 + n * 36:
        raise ValueError(f"{path}: .geom claims {n} triangles, file has {len(data)} bytes")
    return np.frombuffer(data[4:4 + n * 36], dtype="<f4").reshape(n, 3, 3)


def loadGeom(path, objectToWorld=None, scale=1.0, offset=(0.0, 0.0, 0.0)):
    """TriangleMesh from a .geom soup; vertices baked as v*scale - offset (fp64)."""
    tris = readGeom(path).astype(np.float64)
    v = tris.reshape(-1, 3) * float(scale) - np.asarray(offset, dtype=np.float64)
    faces = np.arange(v.shape[0], dtype=np.int32).reshape(-1, 3)
    return TriangleMesh(v, faces, None, mat4(1.0) if objectToWorld is None else objectToWorld)


def writeGeom(path, vertices, faces):
    """objconv.nim writeGeom: int32 face count then float32 soup."""
    v = np.asarray(vertices, dtype=np.float64)
    f = np.asarray(faces, dtype=np.int64)
    with open(path, "wb") as fh:
        fh.write(np.int32(f.shape[0]).tobytes())
        fh.write(v[f].astype("<f4").tobytes())


def loadObjArrays(path, slash_indices=False):
    """obj.nim loadObj's vertex / face arrays through the native reader
    (rt_load_obj): (V, 3) float64, (F, 3) int32 0-based."""
    import ctypes as C

    from . import abi
    from ._lib import check, lib
    flags = abi.RT_OBJ_SLASH_INDICES if slash_indices else 0
    nv, nf = C.c_int64(0), C.c_int64(0)
    p = os.fsencode(path)
    check(lib().rt_load_obj(p, flags, C.byref(nv), None, C.byref(nf), None))
    v = np.zeros((max(nv.value, 1), 3), np.float64)
    f = np.zeros((max(nf.value, 1), 3), np.int32)
    check(lib().rt_load_obj(p, flags, C.byref(nv), v.ctypes.data_as(C.POINTER(C.c_double)), C.byref(nf),
                            f.ctypes.data_as(C.POINTER(C.c_int32))))
    return v[:nv.value], f[:nf.value]


def loadObj(path, objectToWorld=None, slash_indices=False):
    """obj.nim loadObj (87-126): a TriangleMesh of the file's `v` / `f`
    lines; face normals are computed by the library (calcNormals)."""
    v, f = loadObjArrays(path, slash_indices)
    return TriangleMesh(v, f, None, mat4(1.0) if objectToWorld is None else objectToWorld)


def objconv(obj_path, geom_path, slash_indices=False):
    """objconv.nim main: loadObj then writeGeom (native rt_write_geom)."""
    import ctypes as C

    from ._lib import check, lib
    v, f = loadObjArrays(obj_path, slash_indices)
    v = np.ascontiguousarray(v)
    f = np.ascontiguousarray(f)
    check(lib().rt_write_geom(os.fsencode(geom_path), v.ctypes.data_as(C.POINTER(C.c_double)), v.shape[0],
                              f.ctypes.data_as(C.POINTER(C.c_int32)), f.shape[0]))


def default_geom_path():
    """The committed copy of the reference's test/bunny.geom fixture."""
    here = os.path.dirname(os.path.abspath(__file__))
    return os.path.normpath(os.path.join(here, "..", "..", "tests", "golden", "bunny.geom"))
