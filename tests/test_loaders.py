"""Native mesh ingestion (csrc/rt_obj.cpp): the OBJ reader of
src/loaders/obj.nim:87-126 and objconv's .geom writer
(src/loaders/objconv.nim:139-153), on CPU. Edge-case fixtures are generated
here; two reference-held meshes are committed gzipped as data fixtures
(tests/golden/bunny.obj.gz, teapot.obj.gz = src/data/meshes/*.obj) and pin
the reader against the reference's own converted output (bunny.geom)."""
import ctypes as C
import os
import time

import numpy as np
import pytest

from rtmi import abi, scenes
from rtmi._lib import RtmiError, lib
from rtmi.loaders import loadObjArrays, objconv, readGeom


def _write_obj(path, v, f, newline="\n", extra=""):
    lines = ["# generated", "g mesh"] + [f"v {x!r} {y!r} {z!r}" for x, y, z in v.tolist()]
    lines += ["vn 0 1 0", "vt 0.5 0.5"] + [f"f {a + 1} {b + 1} {c + 1}" for a, b, c in f.tolist()]
    path.write_bytes((newline.join(lines) + newline + extra).encode())


def test_roundtrip_exact(tmp_path):
    m = scenes.torus_mesh(40, 20)
    p = tmp_path / "torus.obj"
    _write_obj(p, m.vertices, m.faces)
    v, f = loadObjArrays(str(p))
    assert np.array_equal(v, m.vertices) and np.array_equal(f, m.faces)
    g = tmp_path / "torus.geom"
    objconv(str(p), str(g))
    tris = readGeom(str(g))
    assert np.array_equal(tris, m.vertices[m.faces].astype(np.float32))


def test_reference_token_rules(tmp_path):
    """toVertex / toFaceIdx defaults, skipped line kinds, CRLF and tabs,
    quads (4th index ignored), 'v//vn' faces with and without the flag."""
    p = tmp_path / "edge.obj"
    p.write_bytes(b"v 1.5 abc 3\r\nv\t-2\t1e3\t0x\r\n  v 4 5 6  \r\n"
                  b"vn 1 0 0\r\nvt 0 0\r\n# f 9 9 9\r\nusemtl x\r\n"
                  b"f 3 1 2 9\r\nf 1//1 2//2 3//3\r\nf -1 +2 2.0\r\n\r\n")
    v, f = loadObjArrays(str(p))
    assert v.tolist() == [[1.5, 0.0, 3.0], [-2.0, 1000.0, 0.0], [4.0, 5.0, 6.0]]
    assert f.tolist() == [[2, 0, 1], [0, 0, 0], [-2, 1, 0]]
    _, fs = loadObjArrays(str(p), slash_indices=True)
    assert fs.tolist() == [[2, 0, 1], [0, 1, 2], [-2, 1, 0]]


def test_short_lines_and_missing_files_are_errors(tmp_path):
    p = tmp_path / "short.obj"
    p.write_text("v 1 2 3\nv 1 2\n")
    with pytest.raises(RtmiError, match="fewer than 3"):
        loadObjArrays(str(p))
    with pytest.raises(RtmiError):
        loadObjArrays(str(tmp_path / "missing.obj"))
    nv, nf = C.c_int64(0), C.c_int64(0)
    assert lib().rt_load_obj(None, 0, C.byref(nv), None, C.byref(nf), None) == abi.RT_E_INVALID
    v = np.zeros((1, 3))
    f = np.array([[0, 1, 2]], np.int32)
    assert lib().rt_write_geom(str(tmp_path / "x.geom").encode(), v.ctypes.data_as(C.POINTER(C.c_double)), 1,
                               f.ctypes.data_as(C.POINTER(C.c_int32)), 1) == abi.RT_E_INVALID


def test_empty_file(tmp_path):
    p = tmp_path / "empty.obj"
    p.write_text("# nothing\n")
    v, f = loadObjArrays(str(p))
    assert v.shape == (0, 3) and f.shape == (0, 3)


def test_large_obj_is_fast(tmp_path):
    """200k faces: the native reader is what makes million-face OBJ scenes
    practical."""
    m = scenes.torus_mesh(400, 250)
    p = tmp_path / "big.obj"
    _write_obj(p, m.vertices, m.faces)
    t0 = time.perf_counter()
    v, f = loadObjArrays(str(p))
    dt = time.perf_counter() - t0
    assert f.shape == (200000, 3) and np.array_equal(f, m.faces) and np.array_equal(v, m.vertices)
    assert dt < 5.0, dt


def test_bunny_obj_converts_to_the_reference_geom():
    """Reference-held pin: objconv.nim (loadObj 87-126 + writeGeom 139-153)
    turned src/data/meshes/bunny.obj into test/bunny.geom. Our reader of the
    same .obj, converted the same way (float64 parse, float32 soup), gives
    that file's 69,451 triangles bit for bit."""
    from rtmi import scenes
    from rtmi.loaders import default_geom_path
    v, f = loadObjArrays(scenes._golden_obj("bunny"))
    assert v.shape == (35947, 3) and f.shape == (69451, 3)
    assert f.min() == 0 and f.max() == 35946
    ref = readGeom(default_geom_path())
    assert np.array_equal(v[f].astype(np.float32), ref)


def test_teapot_obj_live_scene_mesh():
    """The mesh src/raytracer.nim's live scene (mesh-bunny.nim:1) loads:
    teapot.obj's 3,644 vertices / 6,320 faces, and the face normals the
    library computes as calcNormals (obj.nim:65-84) in float64."""
    from rtmi import scenes
    v, f = loadObjArrays(scenes._golden_obj("teapot"))
    assert v.shape == (3644, 3) and f.shape == (6320, 3)
    assert v.min(axis=0).tolist() == [-3.0, 0.0, -2.0] and v.max(axis=0).tolist() == [3.434, 3.15, 2.0]
    p0, p1, p2 = v[f[:, 0]], v[f[:, 1]], v[f[:, 2]]
    n = np.cross(p1 - p0, p2 - p0)
    assert np.isfinite(n).all()
