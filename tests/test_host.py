"""Host-side logic: glm semantics, scene data, flattening, loaders, band
mapping. CPU only."""
import math

import numpy as np
import pytest

from rtmi import abi, glm, scenes
from rtmi.dist import band_rows, rank_rows, unshard_host
from rtmi.loaders import loadObj, readGeom, writeGeom
from rtmi.scene import Box, Plane, Sphere, TriangleMesh, flatten


def test_glm_post_multiply_semantics():
    # m.rotate(X, a).translate(t) == R * T: the translation is rotated
    m = glm.translate(glm.rotate(glm.mat4(1.0), glm.X_AXIS, glm.degToRad(90.0)), glm.vec3(0.0, 1.0, 0.0))
    o = glm.mul(m, glm.point(0.0, 0.0, 0.0))
    assert o[:3] == pytest.approx([0.0, 0.0, 1.0], abs=1e-15)
    # translate then rotate: the translation is NOT rotated
    m2 = glm.rotate(glm.translate(glm.mat4(1.0), glm.vec3(0.0, 1.0, 0.0)), glm.X_AXIS, glm.degToRad(90.0))
    assert glm.mul(m2, glm.point(0.0, 0.0, 0.0))[:3] == pytest.approx([0.0, 1.0, 0.0])
    # columns: m[3] is the translation (column-major, glm layout)
    t = glm.translate(glm.mat4(1.0), glm.vec3(1.0, 2.0, 3.0))
    assert glm.flat(t)[12:15].tolist() == [1.0, 2.0, 3.0]


def test_glm_inverse():
    m = scenes.boxes2().objects[5].geometry.objectToWorld
    inv = glm.inverse(m)
    assert np.allclose(inv @ m, np.eye(4), atol=1e-14)  # (m[col][row] layout: inv*m == I)
    assert np.allclose(glm.inverse(glm.translate(glm.mat4(1.0), glm.vec3(1, 2, 3)))[3], [-1, -2, -3, 1])
    with pytest.raises(ValueError):
        glm.inverse(np.zeros((4, 4)))


def test_scene_inventory():
    b2 = scenes.boxes2()
    assert len(b2.objects) == 16
    assert [type(o.geometry) for o in b2.objects[:3]] == [Plane, Box, Sphere]
    c1 = scenes.spheres_warm(3)
    assert len(c1.objects) == 4 and len(c1.lights) == 2
    assert scenes.spheres_reflection().objects[0].material.reflection == 1.0
    for name, f in scenes.SCENES.items():
        if name != "torus":
            assert f().objects


def test_baked_bunny():
    m = scenes.baked_bunny()
    assert m.faces.shape == (69451, 3)
    v = m.vertices
    assert v[:, 1].min() == pytest.approx(scenes.BAKED_MIN_Y, abs=1e-12)
    assert 4.0 < v[:, 1].max() < 5.0                 # x30: ~4.6 units tall
    assert abs(v[:, 0].min() + v[:, 0].max()) < 1e-9  # centred in x
    # baking keeps the absolute det cull meaningful: |e1 x e2| well above 1e-6
    e1 = v[m.faces[:, 1]] - v[m.faces[:, 0]]
    e2 = v[m.faces[:, 2]] - v[m.faces[:, 0]]
    assert np.median(np.linalg.norm(np.cross(e1, e2), axis=1)) > 1e-3


@pytest.mark.parametrize("U,V", [(16, 8), (1000, 500)])
def test_torus_mesh(U, V):
    m = scenes.torus_mesh(U, V)
    assert m.faces.shape == (2 * U * V, 3)
    assert m.vertices.shape == (U * V, 3)
    assert m.faces.min() == 0 and m.faces.max() == U * V - 1
    assert m.vertices[:, 1].min() == pytest.approx(scenes.BAKED_MIN_Y)
    # closed, outward-wound surface: the divergence-theorem signed volume is
    # positive and close to the torus volume 2 pi^2 R r^2 (R = 3, r = 1)
    v = m.vertices
    f = m.faces
    vol = np.einsum("ij,ij->i", v[f[:, 0]], np.cross(v[f[:, 1]], v[f[:, 2]])).sum() / 6.0
    assert vol == pytest.approx(2 * math.pi ** 2 * 3.0, rel=0.2 if U < 100 else 0.01)


def test_flatten_descriptor():
    s = scenes.mesh_bunny()
    fl = flatten(s)
    d = fl.desc
    assert d.num_objects == 2 and d.num_lights == 2 and d.num_meshes == 1
    assert fl._objs[0].type == abi.RT_MESH and fl._objs[0].mesh == 0
    assert fl._objs[1].type == abi.RT_PLANE
    assert fl._mdesc[0].num_faces == 69451 and not fl._mdesc[0].normals
    assert d.fov == 50.0
    assert list(d.camera_to_world)[12:15] == pytest.approx([0.0, 5.5 * math.cos(math.radians(12)) + 1.5 * math.sin(math.radians(12)), 1.5 * math.cos(math.radians(12)) - 5.5 * math.sin(math.radians(12))], abs=1e-12)


def test_geom_roundtrip(tmp_path):
    v = np.array([[0, 1, -5], [-2, -1, -5], [2, -1, -5], [0, 0, 0]], dtype=np.float64)
    f = np.array([[0, 1, 2], [1, 2, 3]])
    p = tmp_path / "t.geom"
    writeGeom(str(p), v, f)
    tris = readGeom(str(p))
    assert tris.shape == (2, 3, 3)
    assert np.array_equal(tris[1], v[[1, 2, 3]].astype(np.float32))


def test_load_obj(tmp_path):
    p = tmp_path / "t.obj"
    p.write_text("# c\nv 0 1 -5\nv -2 -1 -5\nv 2 -1 -5\n\nf 1 2 3\nf 1/1/1 2/2/2 3/3/3\n")
    m = loadObj(str(p))
    assert isinstance(m, TriangleMesh)
    # obj.nim's parseInt("1/1/1") fails -> the index keeps its default 0
    assert m.vertices.shape == (3, 3) and m.faces.tolist() == [[0, 1, 2], [0, 0, 0]]
    assert loadObj(str(p), slash_indices=True).faces.tolist() == [[0, 1, 2], [0, 1, 2]]


@pytest.mark.parametrize("h,band_h,world", [(1080, 16, 1), (1080, 16, 2), (1080, 16, 8), (131, 7, 3),
                                            (10, 16, 4), (2160, 16, 8)])
def test_band_mapping_covers_every_row_once(h, band_h, world):
    rows = band_rows(h, band_h, world)
    seen = np.zeros(h, int)
    for r in range(world):
        ys = rank_rows(h, band_h, r, world)
        assert len(ys) == rows
        seen[ys[ys >= 0]] += 1
    assert (seen == 1).all()
    # unshard inverts the layout
    w = 5
    img = np.random.default_rng(0).random((h, w, 3)).astype(np.float32)
    g = np.zeros((world, rows, w, 3), np.float32)
    for r in range(world):
        ys = rank_rows(h, band_h, r, world)
        g[r, ys >= 0] = img[ys[ys >= 0]]
    assert np.array_equal(unshard_host(g, h, band_h), img)
