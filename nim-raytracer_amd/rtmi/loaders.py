"""Mesh ingestion.

- loadGeom: the .geom triangle soup written by src/loaders/objconv.nim:139-153
  and read by test/test.nim:14-26 — little-endian int32 N, then N triangles of
  3 vertices of 3 float32. (The reference's own src/loaders/geomloader.nim is
  broken: it reads no triangle data, geomloader.nim:38-45.)
- loadObj: `v` / `f` OBJ subset of src/loaders/obj.nim:87-126 (1-based face
  indices, first three indices of each `f`, normals computed per face by the
  library exactly as calcNormals obj.nim:65-84).
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


def loadObj(path, objectToWorld=None):
    """obj.nim loadObj: vertices from `v x y z`, faces from `f a b c`."""
    verts, faces = [], []
    with open(path, "r") as fh:
        for line in fh:
            c = line.split()
            if not c:
                continue
            if c[0] == "v":
                verts.append([float(c[1]), float(c[2]), float(c[3])])
            elif c[0] == "f":
                faces.append([int(c[k].split("/")[0]) - 1 for k in (1, 2, 3)])
    return TriangleMesh(np.array(verts, dtype=np.float64), np.array(faces, dtype=np.int32), None,
                        mat4(1.0) if objectToWorld is None else objectToWorld)


def default_geom_path():
    """The committed copy of the reference's test/bunny.geom fixture."""
    here = os.path.dirname(os.path.abspath(__file__))
    return os.path.normpath(os.path.join(here, "..", "..", "tests", "golden", "bunny.geom"))
