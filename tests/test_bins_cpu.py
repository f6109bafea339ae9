"""The float32 kernel's face bins (csrc/rt_bins.cpp) are conservative: every
face a camera ray of a pixel can hit is in that pixel's list, and every face
a distant light's shadow ray can hit is in its light-grid cell (a lane off
the grid hits nothing). Checked on the CPU against a float64 restatement of
the reference's single-sided Möller–Trumbore test (geom.nim:283-336) over
every face, for random rays of the families the bins serve — including
rays through pixel edges and corners and a rotated, scaled mesh. Exactness
of the GPU frames is tests/test_gpu_bins.py."""
import ctypes as C
import math

import numpy as np
import pytest

from rtmi import scenes
from rtmi._lib import lib
from rtmi.glm import X_AXIS, Y_AXIS, degToRad, inverse, mat4, rotate, scale, translate, vec3


def _m(a):
    """glm column-major 4x4 -> flat[16] (m[c*4 + r])."""
    return np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(16))


def _cols(a):
    """flat[16] column-major -> row-major 4x4 numpy matrix."""
    return np.asarray(a, dtype=np.float64).reshape(4, 4).T


def _faces(mesh):
    v = mesh.vertices[mesh.faces]  # (nf, 3, 3)
    return np.ascontiguousarray(v.reshape(-1, 9))


def _hits(v9, ro, rd):
    """Faces hit at t >= 0 by the ray (float64, single-sided, det < 1e-6 culled)."""
    v0, v1, v2 = v9[:, 0:3], v9[:, 3:6], v9[:, 6:9]
    e1, e2 = v1 - v0, v2 - v0
    p = np.cross(rd, e2)
    det = np.einsum("ij,ij->i", e1, p)
    ok = det >= 1e-6
    inv = np.where(ok, 1.0 / np.where(ok, det, 1.0), 0.0)
    tv = ro - v0
    u = np.einsum("ij,ij->i", tv, p) * inv
    q = np.cross(tv, e1)
    v = (q @ rd) * inv
    t = np.einsum("ij,ij->i", e2, q) * inv
    hit = ok & (u >= 0) & (u <= 1) & (v >= 0) & (u + v <= 1) & (t >= 0)
    return np.nonzero(hit)[0]


def _rotated_torus():
    mesh = scenes.torus_mesh(40, 20)
    m = translate(mat4(1.0), vec3(0.5, 1.2, -11.0))
    m = rotate(m, Y_AXIS, degToRad(35.0))
    m = rotate(m, X_AXIS, degToRad(-20.0))
    m = scale(m, vec3(1.3, 0.8, 1.1))
    mesh.objectToWorld = m
    mesh.worldToObject = inverse(m)
    return mesh


def _bunny():
    mesh = scenes.baked_bunny()
    mesh.objectToWorld = translate(mat4(1.0), vec3(0.0, 0.0001, -12.0))
    mesh.worldToObject = inverse(mesh.objectToWorld)
    return mesh


MESHES = {"bunny": _bunny, "rotated_torus": _rotated_torus}


@pytest.mark.parametrize("name", list(MESHES))
def test_pixel_lists_hold_every_hit_face(name):
    L = lib()
    f = L.rtmi_test_pixel_bins
    f.restype = C.c_int64
    mesh = MESHES[name]()
    v9 = _faces(mesh)
    nf = len(v9)
    o2w, w2o = _m(mesh.objectToWorld), _m(mesh.worldToObject)
    cam = scenes.mesh_bunny().cameraToWorld
    c2w = _m(cam)
    W, H, fov = 160, 90, 50.0
    off = np.zeros(W * H + 1, np.int32)
    cap = 4 * nf * 64 + 64
    ent = np.zeros(cap, np.int32)
    n = f(v9.ctypes.data_as(C.c_void_p), C.c_int64(nf), o2w.ctypes.data_as(C.c_void_p),
          w2o.ctypes.data_as(C.c_void_p), c2w.ctypes.data_as(C.c_void_p), C.c_double(fov), W, H,
          off.ctypes.data_as(C.c_void_p), ent.ctypes.data_as(C.c_void_p), C.c_int64(cap))
    assert n >= 0
    C2W, W2O = _cols(c2w), _cols(w2o)
    fo = math.tan(math.radians(fov) / 2)
    ca, cc = 2 * (W / H) * fo / W, 2 * fo / H
    rng = np.random.default_rng(7)
    origin = C2W[:3, 3]
    ro = W2O[:3, :3] @ origin + W2O[:3, 3]
    # random pixels on and around the mesh's projection, random and extreme
    # sub-pixel positions (edges / corners of the pixel square)
    checked = hits_total = 0
    listed = np.nonzero(np.diff(off) > 0)[0]
    assert len(listed) > 0
    for k in range(800):
        if k % 4:  # pixels with a non-empty list (the mesh's projection), or anywhere
            pix = int(listed[rng.integers(0, len(listed))])
            x, y = pix % W, pix // W
        else:
            x, y = int(rng.integers(0, W)), int(rng.integers(0, H))
        sx, sy = (rng.random(), rng.random()) if k % 3 else (float(rng.integers(0, 2)), float(rng.integers(0, 2)))
        px, py = x + min(sx, 0.999999), y + min(sy, 0.999999)
        dc = np.array([(px - W / 2) * ca, (H / 2 - py) * cc, -1.0])
        d = C2W[:3, :3] @ (dc / np.linalg.norm(dc))
        rd = W2O[:3, :3] @ d
        hit = _hits(v9, ro, rd)
        lst = set((ent[off[y * W + x]:off[y * W + x + 1]] // 64).tolist())
        missing = set(hit.tolist()) - lst
        assert not missing, (name, x, y, sorted(missing)[:5])
        checked += 1
        hits_total += len(hit)
    assert hits_total > 200  # the rays really meet the mesh


@pytest.mark.parametrize("name", list(MESHES))
def test_light_grid_cells_hold_every_hit_face(name):
    L = lib()
    f = L.rtmi_test_light_grid
    f.restype = C.c_int64
    mesh = MESHES[name]()
    v9 = _faces(mesh)
    nf = len(v9)
    w2o = _m(mesh.worldToObject)
    W2O = _cols(w2o)
    rng = np.random.default_rng(11)
    total_hits = 0
    for light in scenes.mesh_bunny().lights:
        dvec = np.asarray(light.dir[:3], np.float64)
        hdr = np.zeros(12, np.float32)
        offcap, entcap = 4096 * 4096 + 1, 64 * nf * 64
        off = np.zeros(min(offcap, 8_000_000), np.int32)
        ent = np.zeros(min(entcap, 16_000_000), np.int32)
        n = f(v9.ctypes.data_as(C.c_void_p), C.c_int64(nf), w2o.ctypes.data_as(C.c_void_p),
              dvec.ctypes.data_as(C.c_void_p), hdr.ctypes.data_as(C.c_void_p), off.ctypes.data_as(C.c_void_p),
              C.c_int64(len(off)), ent.ctypes.data_as(C.c_void_p), C.c_int64(len(ent)))
        assert n >= 0
        e1, u0, e2, v0 = hdr[0:3], hdr[3], hdr[4:7], hdr[7]
        inv_h, rmax, gu, gv = hdr[8], hdr[9], int(hdr[10]), int(hdr[11])
        sd = -dvec
        rd = W2O[:3, :3] @ sd
        # shadow-ray origins: ground points around the mesh (its shadow and
        # beyond) and points scattered through the mesh's box
        lo, hi = mesh.vertices.min(0), mesh.vertices.max(0)
        pts = []
        for _ in range(500):
            g = np.array([rng.uniform(-14, 14), 1e-4, rng.uniform(-26, 2)])
            pts.append(g)
        for _ in range(200):
            p = lo + (hi - lo) * rng.random(3)
            w = np.linalg.inv(W2O) @ np.append(p, 1.0)
            pts.append(w[:3] - sd * rng.uniform(0.0, 3.0))
        for o in pts:
            ro = W2O[:3, :3] @ o + W2O[:3, 3]
            hit = _hits(v9, ro, rd)
            total_hits += len(hit)
            ro32 = ro.astype(np.float32)
            uu = np.float32(ro32 @ e1.astype(np.float32))
            vv = np.float32(ro32 @ e2.astype(np.float32))
            fu, fv = np.float32((uu - u0) * inv_h), np.float32((vv - v0) * inv_h)
            if np.abs(ro32).max() > rmax:
                continue  # the kernel sends such lanes to the BVH
            if not (0 <= fu < gu and 0 <= fv < gv):
                assert len(hit) == 0, (name, o, hit[:5])
                continue
            cell = int(fv) * gu + int(fu)
            lst = set((ent[off[cell]:off[cell + 1]] // 64).tolist())
            missing = set(hit.tolist()) - lst
            assert not missing, (name, o, sorted(missing)[:5])
    assert total_hits > 100


def _tilted_plane():
    m = translate(mat4(1.0), vec3(0.0, -0.4, 0.0))
    m = rotate(m, X_AXIS, degToRad(4.0))
    m = rotate(m, Y_AXIS, degToRad(20.0))
    return m, inverse(m)


@pytest.mark.parametrize("name,tilted", [("bunny", False), ("rotated_torus", True)])
def test_shadow_skips_are_conservative(name, tilted):
    """A pixel's skip bit for a light (rt_bins.h build_shadow_skips) promises
    that no shadow ray to that light from a camera hit in the pixel meets a
    face: checked for random samples (and the pixel corners) of skipped
    pixels, against every face in float64."""
    L = lib()
    f = L.rtmi_test_shadow_skips
    f.restype = C.c_int64
    mesh = MESHES[name]()
    v9 = _faces(mesh)
    nf = len(v9)
    o2w, w2o = _m(mesh.objectToWorld), _m(mesh.worldToObject)
    sc = scenes.mesh_bunny()
    c2w = _m(sc.cameraToWorld)
    po2w, pw2o = _tilted_plane() if tilted else (mat4(1.0), mat4(1.0))
    planes = np.concatenate([_m(po2w), _m(pw2o)])
    dirs = np.ascontiguousarray(np.concatenate([np.asarray(l.dir[:3], np.float64) for l in sc.lights]))
    W, H, fov, bias = 480, 270, 50.0, 1e-4
    out = np.zeros((W * H + 3) // 4, np.uint32)
    n = f(v9.ctypes.data_as(C.c_void_p), C.c_int64(nf), o2w.ctypes.data_as(C.c_void_p),
          w2o.ctypes.data_as(C.c_void_p), c2w.ctypes.data_as(C.c_void_p), C.c_double(fov), W, H,
          planes.ctypes.data_as(C.c_void_p), 1, dirs.ctypes.data_as(C.c_void_p), len(sc.lights), C.c_double(bias),
          out.ctypes.data_as(C.c_void_p))
    assert n > 0.3 * W * H  # most ground pixels skip at least one light
    bits = (out.view(np.uint8)[:W * H]).astype(np.int64)
    C2W, W2O, P2W, W2P = _cols(c2w), _cols(w2o), _cols(_m(po2w)), _cols(_m(pw2o))
    N = P2W[:3, 1]
    fo = math.tan(math.radians(fov) / 2)
    ca, cc = 2 * (W / H) * fo / W, 2 * fo / H
    org = C2W[:3, 3]
    rng = np.random.default_rng(5)
    near = 0
    for li, light in enumerate(sc.lights):
        rd = W2O[:3, :3] @ -np.asarray(light.dir[:3], np.float64)
        sk = np.nonzero(bits >> li & 1)[0]
        # skipped pixels next to unskipped ones (the shadow's border) first
        edge = sk[(bits[np.clip(sk + 1, 0, W * H - 1)] >> li & 1) == 0]
        pick = np.concatenate([edge[rng.permutation(len(edge))[:400]], sk[rng.integers(0, len(sk), 200)]])
        for k, pix in enumerate(pick):
            x, y = int(pix % W), int(pix // W)
            sx, sy = (rng.random(), rng.random()) if k % 3 else (float(rng.integers(0, 2)), float(rng.integers(0, 2)))
            px, py = x + min(sx, 0.999999), y + min(sy, 0.999999)
            dc = np.array([(px - W / 2) * ca, (H / 2 - py) * cc, -1.0])
            d = C2W[:3, :3] @ (dc / np.linalg.norm(dc))
            oy = (W2P[:3, :3] @ org + W2P[:3, 3])[1]
            dy = (W2P[:3, :3] @ d)[1]
            t = -oy / dy
            if not (t >= 0):
                continue  # the sky: no shadow ray
            so = org + d * t + N * bias
            ro = W2O[:3, :3] @ so + W2O[:3, 3]
            hit = _hits(v9, ro, rd)
            assert len(hit) == 0, (name, li, x, y, hit[:5])
            near += k < len(edge)
    assert near > 100


@pytest.mark.parametrize("name,tilted", [("bunny", False), ("rotated_torus", True)])
def test_shadow_lists_hold_every_hit_face(name, tilted):
    """A pixel's shadow list for a light (rt_bins.h build_shadow_skips, sl)
    promises every face a shadow ray to that light from a camera hit in the
    pixel can meet: checked for random samples (and the pixel corners) of
    pixels with a list, against every face in float64."""
    L = lib()
    f = L.rtmi_test_shadow_lists
    f.restype = C.c_int64
    mesh = MESHES[name]()
    v9 = _faces(mesh)
    nf = len(v9)
    o2w, w2o = _m(mesh.objectToWorld), _m(mesh.worldToObject)
    sc = scenes.mesh_bunny()
    c2w = _m(sc.cameraToWorld)
    po2w, pw2o = _tilted_plane() if tilted else (mat4(1.0), mat4(1.0))
    planes = np.concatenate([_m(po2w), _m(pw2o)])
    dirs = np.ascontiguousarray(np.concatenate([np.asarray(l.dir[:3], np.float64) for l in sc.lights]))
    nl = len(sc.lights)
    W, H, fov, bias = 480, 270, 50.0, 1e-4
    sl = np.zeros(W * H * nl * 2, np.int32)
    cap = 1 << 22
    ent = np.zeros(cap, np.int32)
    n = f(v9.ctypes.data_as(C.c_void_p), C.c_int64(nf), o2w.ctypes.data_as(C.c_void_p),
          w2o.ctypes.data_as(C.c_void_p), c2w.ctypes.data_as(C.c_void_p), C.c_double(fov), W, H,
          planes.ctypes.data_as(C.c_void_p), 1, dirs.ctypes.data_as(C.c_void_p), nl, C.c_double(bias),
          sl.ctypes.data_as(C.c_void_p), ent.ctypes.data_as(C.c_void_p), C.c_int64(cap))
    assert n > 100, n
    sl = sl.reshape(W * H, nl, 2)
    C2W, W2O, P2W, W2P = _cols(c2w), _cols(w2o), _cols(_m(po2w)), _cols(_m(pw2o))
    N = P2W[:3, 1]
    fo = math.tan(math.radians(fov) / 2)
    ca, cc = 2 * (W / H) * fo / W, 2 * fo / H
    org = C2W[:3, 3]
    rng = np.random.default_rng(11)
    hits_seen = 0
    for li, light in enumerate(sc.lights):
        rd = W2O[:3, :3] @ -np.asarray(light.dir[:3], np.float64)
        have = np.nonzero(sl[:, li, 1] >= 0)[0]
        assert len(have) > 0
        for k, pix in enumerate(have[rng.permutation(len(have))[:500]]):
            x, y = int(pix % W), int(pix // W)
            lst = set((ent[sl[pix, li, 0]:sl[pix, li, 0] + sl[pix, li, 1]] // 64).tolist())
            for j in range(3):
                sx, sy = (rng.random(), rng.random()) if j else (float(rng.integers(0, 2)), float(rng.integers(0, 2)))
                px, py = x + min(sx, 0.999999), y + min(sy, 0.999999)
                dc = np.array([(px - W / 2) * ca, (H / 2 - py) * cc, -1.0])
                d = C2W[:3, :3] @ (dc / np.linalg.norm(dc))
                oy = (W2P[:3, :3] @ org + W2P[:3, 3])[1]
                dy = (W2P[:3, :3] @ d)[1]
                t = -oy / dy
                if not (t >= 0):
                    continue
                so = org + d * t + N * bias
                ro = W2O[:3, :3] @ so + W2O[:3, 3]
                hit = _hits(v9, ro, rd)
                hits_seen += len(hit)
                missing = set(hit.tolist()) - lst
                assert not missing, (name, li, x, y, sorted(missing)[:5])
    assert hits_seen > 50, hits_seen
