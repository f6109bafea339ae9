"""The per-light shadow-test records (rt_common.h LTri, rtmi.cpp make_ltri)
against the reference's Moller-Trumbore test (geom.nim:283-336, the oracle's
float64 restatement): evaluated as the kernels do — three float32 FMA chains
and min(u, v, 1 - (u + v)) >= 0 — a record gives the oracle's verdict on
every ray that is not within float32 rounding of an edge, and the oracle's t
to float32 precision; a face whose det for the light is below 1e-6
(single-sided cull, geom.nim:306) never hits. CPU only (no GPU)."""
import ctypes as C

import numpy as np

from rtmi._lib import lib


def _ltri(v, d, face=7):
    f = lib().rtmi_test_ltri
    out = np.zeros(16, np.uint32)
    v9 = np.ascontiguousarray(np.asarray(v, np.float64).reshape(9))
    dd = np.ascontiguousarray(np.asarray(d, np.float64))
    assert f(v9.ctypes.data_as(C.c_void_p), dd.ctypes.data_as(C.c_void_p), C.c_int32(face),
             out.ctypes.data_as(C.c_void_p)) == 0
    return out


def _eval(rec, o):
    """The kernel's ltri_t in float32 (fma chains)."""
    f = rec.view(np.float32)
    o = np.asarray(o, np.float32)

    def chain(a, c):
        return np.float32(np.float64(a[0]) * o[0] + np.float32(np.float64(a[1]) * o[1]
                                                               + np.float32(np.float64(a[2]) * o[2] + c)))
    u, v, t = chain(f[0:3], f[3]), chain(f[4:7], f[7]), chain(f[8:11], f[11])
    g = min(min(u, v), np.float32(1.0) - np.float32(u + v))
    return (float(t) if g >= 0 else -1.0), float(u), float(v)


def _mt(o, d, v):
    """geom.nim rayTriangleIntersectFast in float64 (the oracle's arithmetic)."""
    v0, v1, v2 = (np.asarray(x, np.float64) for x in v)
    e1, e2 = v1 - v0, v2 - v0
    p = np.cross(d, e2)
    det = float(np.dot(e1, p))
    if det < 1e-6:
        return None
    tv = o - v0
    u = float(np.dot(tv, p)) / det
    q = np.cross(tv, e1)
    w = float(np.dot(d, q)) / det
    if u < 0 or u > 1 or w < 0 or u + w > 1:
        return None
    return float(np.dot(e2, q)) / det, u, w


def test_ltri_matches_moller_trumbore():
    rng = np.random.default_rng(5)
    checked = hits = 0
    for _ in range(300):
        v = rng.normal(size=(3, 3)) * rng.uniform(0.05, 2.0)
        d = rng.normal(size=3)
        d /= np.linalg.norm(d)
        rec = _ltri(v, d)
        for _ in range(40):
            # origins behind the face along -d, around its centroid
            c = v.mean(axis=0) + rng.normal(size=3) * 0.6 * np.abs(v - v.mean(axis=0)).max()
            o = c - d * rng.uniform(0.5, 5.0)
            ref = _mt(o, d, v)
            t, u, w = _eval(rec, o)
            near_edge = ref is not None and min(ref[1], ref[2], 1 - ref[1] - ref[2]) < 1e-4
            if ref is None:
                # a miss: the record agrees unless the ray grazes an edge
                if t >= 0:
                    assert min(u, w, 1 - u - w) > -1e-4, (u, w)
                continue
            checked += 1
            if near_edge:
                continue
            hits += 1
            # (t may be negative: the face behind the origin, refused by trace's t >= 0 in both)
            assert t != -1.0 and abs(t - ref[0]) <= 2e-5 * (1 + abs(ref[0])), (t, ref)
    assert hits > 500 and checked >= hits


def test_ltri_culls_faces_below_det():
    v = np.array([[0.0, 1.0, -5.0], [-2.0, -1.0, -5.0], [2.0, -1.0, -5.0]])  # geomtest2.nim's triangle
    front = _ltri(v, np.array([0.0, 0.0, -1.0]))
    back = _ltri(v, np.array([0.0, 0.0, 1.0]))
    t, u, w = _eval(front, np.zeros(3))
    assert abs(t - 5.0) < 1e-6 and abs(u - 0.25) < 1e-7 and abs(w - 0.25) < 1e-7  # the reference's t, u, v
    assert _eval(back, np.array([0.0, 0.0, -10.0]))[0] == -1.0  # det < 1e-6 for this light: never a hit
    assert int(front[12]) == 7 and int(back[12]) == 7  # the face index rides along
