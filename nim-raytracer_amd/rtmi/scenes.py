"""The parity / benchmark scenes, re-expressed as data.

The reference's scenes are Nim source `include`d into main
(src/raytracer.nim:54); these builders restate them verbatim (same objects in
the same order, same materials, lights and cameras) as rtmi.scene.Scene.
"""
import math
import os

import numpy as np

from .glm import X_AXIS, Y_AXIS, degToRad, mat4, normalize, point, rotate, translate, vec, vec3
from .loaders import default_geom_path, loadGeom
from .scene import (DistantLight, Material, Object, PointLight, Scene, TriangleMesh, initBox,
                    initPlane, initSphere)

_WARM_BALLS = [  # src/data/scenes/spheres-warm.nim:2-50
    ("ball1", (-5.0, 2.0, -18.0), (0.9, 0.3, 0.2)),
    ("ball2", (0.5, 2.0, -8.0), (0.6, 0.9, 0.2)),
    ("ball3", (-5.0, 2.0, -10.0), (0.1, 0.7, 0.2)),
    ("ball4", (8.0, 2.0, -15.0), (0.2, 0.3, 0.9)),
    ("ball5", (4.0, 2.0, -16.0), (0.2, 0.5, 0.9)),
    ("ball6", (-2.0, 2.0, -42.0), (0.9, 0.5, 0.2)),
    ("ball7", (9.0, 2.0, -30.0), (0.6, 0.5, 0.9)),
]


def _warm_lights():
    # spheres-warm.nim:59-68 (also mesh-bunny.nim:21-30)
    return [
        DistantLight(color=vec3(1.0), intensity=4.0, dir=normalize(vec(-2.0, -0.8, -0.3))),
        DistantLight(color=vec3(0.8, 0.3, 0.0), intensity=1.0, dir=normalize(vec(2.0, -0.8, -1.3))),
    ]


def _std_camera(tx, ty, tz):
    return translate(rotate(mat4(1.0), X_AXIS, degToRad(-12.0)), vec3(tx, ty, tz))


def spheres_warm(num_balls=7):
    """src/data/scenes/spheres-warm.nim. num_balls=3 is BASELINE config C1
    (balls 1-3 + ground, both distant lights)."""
    objects = []
    for name, t, alb in _WARM_BALLS[:num_balls]:
        objects.append(Object(name, initSphere(r=2, objectToWorld=translate(mat4(1.0), vec3(*t))),
                              Material(albedo=vec3(*alb))))
    objects.append(Object("ground", initPlane(objectToWorld=mat4(1.0)), Material(albedo=vec3(0.4))))
    return Scene(objects=objects, lights=_warm_lights(), fov=50.0,
                 cameraToWorld=_std_camera(1.0, 5.5, 3.5), bgColor=vec3(0.01, 0.03, 0.05))


def boxes2():
    """src/data/scenes/boxes2.nim verbatim: 16 primitives, 1 distant light
    (BASELINE config C2)."""
    Z_DIST = -18.0
    objects = [
        Object("ground", initPlane(objectToWorld=mat4(1.0)), Material(albedo=vec3(0.3))),
        Object("platform", initBox(objectToWorld=translate(mat4(1.0), vec3(0.0, 0.0, Z_DIST)),
                                   vmin=vec(-6.3, 0.0, -6.3), vmax=vec(6.3, 0.5, 6.3)),
               Material(albedo=vec3(0.5))),
        Object("ball", initSphere(objectToWorld=translate(mat4(1.0), vec3(0.0, 4.8, Z_DIST)), r=1.5),
               Material(albedo=vec3(0.5))),
    ]
    N = 13
    rot = 0.0
    for i in range(N):
        m = translate(mat4(1.0), vec3(0.0, 1.0, Z_DIST))
        m = rotate(m, Y_AXIS, degToRad(rot))
        m = translate(m, vec3(0.0, 0.0, 5.0))
        objects.append(Object(f"box{i}", initBox(objectToWorld=m, vmin=vec(-0.5, -0.5, -0.5),
                                                 vmax=vec(0.5, 0.5, 0.5)),
                              Material(albedo=vec3(0.5))))
        rot += 360.0 / float(N)
    lights = [DistantLight(color=vec3(1.0, 1.0, 1.0), intensity=0.5,
                           dir=normalize(vec(3.0, -0.5, -4.0)))]
    cam = translate(rotate(mat4(1.0), X_AXIS, degToRad(-15.0)), vec3(0.0, 6.0, 20.0))
    return Scene(objects=objects, lights=lights, fov=20.0, cameraToWorld=cam,
                 bgColor=vec3(0.15, 0.07, 0.04))


def boxtest():
    """src/data/scenes/boxtest.nim (the NaN-slab KAT scene, test/boxtest.nim:31-41)."""
    objects = [
        Object("ground", initPlane(objectToWorld=mat4(1.0)), Material(albedo=vec3(0.4))),
        Object("box", initBox(objectToWorld=translate(mat4(1.0), vec3(0.0, 1.0, -10.0)),
                              vmin=vec(-1.0, -1.0, -1.0), vmax=vec(1.0, 1.0, 1.0)),
               Material(albedo=vec3(1.0))),
    ]
    lights = [
        DistantLight(color=vec3(1.0), intensity=9.0, dir=normalize(vec(-2.0, -0.8, -0.3))),
        DistantLight(color=vec3(0.8, 0.3, 0.0), intensity=2.0, dir=normalize(vec(2.0, -0.8, -1.3))),
    ]
    return Scene(objects=objects, lights=lights, fov=50.0, cameraToWorld=_std_camera(1.0, 5.5, 3.5),
                 bgColor=vec3(0.15, 0.09, 0.07))


def spheres_reflection():
    """src/data/scenes/spheres-reflection.nim: mirror balls (reflection 1.0,
    recursion to maxRayDepth), a point light and a distant light."""
    balls = [
        ("ball1", (-5.0, 2.0, -18.0), (1.0, 1.0, 1.0), 1.0),
        ("ball2", (0.5, 2.0, -8.0), (1.0, 1.0, 1.0), 1.0),
        ("ball3", (-5.0, 2.0, -10.0), (1.0, 1.0, 1.0), 1.0),
        ("ball4", (8.0, 2.0, -15.0), (0.2, 0.3, 0.9), 0.0),
        ("ball5", (4.0, 2.0, -16.0), (0.2, 0.5, 0.9), 0.0),
        ("ball6", (-2.0, 2.0, -42.0), (0.9, 0.5, 0.2), 1.0),
        ("ball7", (9.0, 2.0, -30.0), (0.6, 0.5, 0.9), 1.0),
    ]
    objects = [Object(n, initSphere(r=2, objectToWorld=translate(mat4(1.0), vec3(*t))),
                      Material(albedo=vec3(*a), reflection=r)) for n, t, a, r in balls]
    objects.append(Object("ground", initPlane(objectToWorld=mat4(1.0)),
                          Material(albedo=vec3(0.4), reflection=0.0)))
    objects.append(Object("ball-behind1", initSphere(r=2, objectToWorld=translate(mat4(1.0), vec3(-4.0, 2.0, 0.0))),
                          Material(albedo=vec3(0.2, 0.3, 0.6), reflection=0.0)))
    objects.append(Object("ball-behind2", initSphere(r=2, objectToWorld=translate(mat4(1.0), vec3(14.0, 2.0, 1.0))),
                          Material(albedo=vec3(0.4, 0.8, 1.0), reflection=0.0)))
    lights = [
        PointLight(color=vec3(1.0, 1.0, 1.0), intensity=3000.0, pos=point(3.0, 6.0, -12.0)),
        DistantLight(color=vec3(0.3, 0.4, 0.6), intensity=0.5, dir=normalize(vec(2.0, -0.8, -1.3))),
    ]
    return Scene(objects=objects, lights=lights, fov=50.0, cameraToWorld=_std_camera(1.0, 5.5, 3.5),
                 bgColor=vec3(0.25, 0.1, 0.2))


def spheres_pointlight1():
    """src/data/scenes/spheres-pointlight1.nim: the warm balls under one point light."""
    s = spheres_warm(7)
    s.lights = [PointLight(color=vec3(1.0, 0.8, 0.5), intensity=2000.0, pos=point(3.0, 6.0, -12.0))]
    s.bgColor = vec3(0.0, 0.0, 0.0)
    return s


BUNNY_SCALE = 30.0


BAKED_MIN_Y = 1e-3


def baked_bunny(path=None, scale=BUNNY_SCALE, min_y=BAKED_MIN_Y):
    """bunny.geom (69,451 triangles) baked into object space: v*scale, centred
    in x/z, lowest vertex at y = min_y. Baking (not an
    objectToWorld scale) keeps the reference's absolute det cull
    (geom.nim:306) meaningful: at native scale the median |e1 x e2| is 1.6e-6
    and most faces would be culled.

    min_y = 1e-3 keeps the mesh AABB's bottom face (world y = 1.1e-3 with the
    mesh-bunny.nim:3 translate) clear of ground shadow-ray origins (y = bias =
    1e-4): with the two coinciding, whether such a ray "starts inside" the box
    (the reference's mesh gate, geom.nim:340) is decided by the last ulp."""
    mesh = loadGeom(path or default_geom_path(), scale=1.0)
    v = mesh.vertices
    vmin, vmax = v.min(axis=0), v.max(axis=0)
    off = np.array([0.5 * (vmin[0] + vmax[0]) * scale, vmin[1] * scale - min_y,
                    0.5 * (vmin[2] + vmax[2]) * scale])
    mesh.vertices = np.ascontiguousarray(v * scale - off)
    return mesh


def _mesh_scene(mesh, name, albedo):
    """src/data/scenes/mesh-bunny.nim layout: mesh at translate(0, 0.0001, -12)
    (mesh-bunny.nim:3), ground plane, the two warm distant lights, camera
    rotate(X, -12deg).translate(0, 5.5, 1.5), fov 50."""
    mesh.objectToWorld = translate(mat4(1.0), vec3(0.0, 0.0001, -12.0))
    from .glm import inverse
    mesh.worldToObject = inverse(mesh.objectToWorld)
    objects = [
        Object(name, mesh, Material(albedo=vec3(*albedo))),
        Object("ground", initPlane(objectToWorld=mat4(1.0)), Material(albedo=vec3(0.4))),
    ]
    return Scene(objects=objects, lights=_warm_lights(), fov=50.0,
                 cameraToWorld=_std_camera(0.0, 5.5, 1.5), bgColor=vec3(0.01, 0.03, 0.05))


def mesh_bunny(path=None):
    """BASELINE configs C3/C4: baked bunny.geom + ground, mesh-bunny.nim lights/camera."""
    return _mesh_scene(baked_bunny(path), "bunny", (0.6, 0.9, 0.2))


def _golden_obj(name):
    """A reference mesh committed gzipped under tests/golden/ (data fixture),
    unpacked once per process for rt_load_obj, which reads a path."""
    import gzip
    import tempfile
    here = os.path.dirname(os.path.abspath(__file__))
    src = os.path.normpath(os.path.join(here, "..", "..", "tests", "golden", f"{name}.obj.gz"))
    dst = os.path.join(tempfile.gettempdir(), f"rtmi_{os.getpid()}_{name}.obj")
    if not os.path.exists(dst):
        with gzip.open(src, "rb") as fin:
            data = fin.read()
        tmp = dst + ".part"
        with open(tmp, "wb") as fout:
            fout.write(data)
        os.replace(tmp, dst)
    return dst


def mesh_teapot():
    """src/data/scenes/mesh-bunny.nim AS WRITTEN: despite its name it loads
    data/meshes/teapot.obj (mesh-bunny.nim:1) through obj.nim's loadObj
    (6,320 faces, normals by calcNormals, obj.nim:65-84) at native scale —
    the scene src/raytracer.nim:54 renders."""
    from .loaders import loadObj
    return _mesh_scene(loadObj(_golden_obj("teapot")), "teapot", (0.6, 0.9, 0.2))


def torus_mesh(U=1000, V=500, R=3.0, r=1.0, amp=0.08):
    """Procedural 2*U*V-triangle torus (U=1000, V=500 -> 1,000,000 triangles,
    BASELINE config C5) with a deterministic sinusoidal tube displacement, no
    RNG. Outward winding, so the single-sided test (geom.nim:306) sees the
    front faces."""
    u = np.arange(U, dtype=np.float64) * (2.0 * math.pi / U)
    w = np.arange(V, dtype=np.float64) * (2.0 * math.pi / V)
    uu, vv = np.meshgrid(u, w, indexing="ij")
    rr = r * (1.0 + amp * np.sin(6.0 * uu) * np.cos(5.0 * vv))
    A = R + rr * np.cos(vv)
    P = np.stack([A * np.cos(uu), rr * np.sin(vv), A * np.sin(uu)], axis=-1).reshape(-1, 3)
    i = np.arange(U)[:, None]
    j = np.arange(V)[None, :]
    i1 = (i + 1) % U
    j1 = (j + 1) % V
    p00 = (i * V + j).reshape(-1)
    p10 = (i1 * V + j).reshape(-1)
    p01 = (i * V + j1).reshape(-1)
    p11 = (i1 * V + j1).reshape(-1)
    t0 = np.stack([p00, p01, p10], axis=-1)
    t1 = np.stack([p10, p01, p11], axis=-1)
    faces = np.stack([t0, t1], axis=1).reshape(-1, 3).astype(np.int32)
    # stand the ring up at 60 degrees and lift it clear of the ground (baked)
    c, s = math.cos(math.radians(60.0)), math.sin(math.radians(60.0))
    y = P[:, 1] * c - P[:, 2] * s
    z = P[:, 1] * s + P[:, 2] * c
    P = np.stack([P[:, 0], y - y.min() + BAKED_MIN_Y, z], axis=-1)
    return TriangleMesh(P, faces, None, mat4(1.0))


def torus_scene(U=1000, V=500):
    """BASELINE config C5: 1M-triangle procedural mesh, same lights/ground/camera."""
    return _mesh_scene(torus_mesh(U, V), "torus", (0.9, 0.5, 0.2))


def _placed(mesh, t):
    from .glm import inverse
    mesh.objectToWorld = translate(mat4(1.0), vec3(*t))
    mesh.worldToObject = inverse(mesh.objectToWorld)
    return mesh


def mesh_mix():
    """Test scene (not one of the reference's): a small reflective mesh with
    analytic objects before AND after it in object order, lit by a point light
    above and a distant light. Shadow rays cross the mesh and then a later
    sphere (or a later sphere first), which exercises the exact shadow early
    exit's stop distance (rt_fast.h / rt_device.h trace) against the oracle's
    plain closest-hit loop."""
    objects = [
        Object("ballA", initSphere(r=1.0, objectToWorld=translate(mat4(1.0), vec3(-4.0, 1.0, -9.0))),
               Material(albedo=vec3(0.9, 0.3, 0.2))),
        Object("torus", _placed(torus_mesh(24, 12), (0.0, 0.0001, -12.0)),
               Material(albedo=vec3(0.9, 0.5, 0.2), reflection=0.5)),
        Object("ballB", initSphere(r=1.0, objectToWorld=translate(mat4(1.0), vec3(0.0, 9.0, -12.0))),
               Material(albedo=vec3(0.2, 0.5, 0.9))),
        Object("ballD", initSphere(r=0.8, objectToWorld=translate(mat4(1.0), vec3(2.5, 0.8, -10.0))),
               Material(albedo=vec3(0.6, 0.9, 0.2))),
        Object("boxC", initBox(objectToWorld=translate(mat4(1.0), vec3(4.0, 0.0, -13.0)),
                               vmin=vec(-1.0, 0.0, -1.0), vmax=vec(1.0, 2.0, 1.0)),
               Material(albedo=vec3(0.5))),
        Object("ground", initPlane(objectToWorld=mat4(1.0)), Material(albedo=vec3(0.4))),
    ]
    lights = [
        PointLight(color=vec3(1.0, 1.0, 1.0), intensity=4000.0, pos=point(0.5, 14.0, -12.0)),
        _warm_lights()[0],
    ]
    return Scene(objects=objects, lights=lights, fov=50.0, cameraToWorld=_std_camera(0.0, 5.5, 1.5),
                 bgColor=vec3(0.01, 0.03, 0.05))


def two_meshes():
    """Test scene: two mesh objects (the shadow early exit is off: with a
    second mesh later in object order its closest t is not known in advance)."""
    objects = [
        Object("torus1", _placed(torus_mesh(24, 12), (1.5, 0.0001, -12.0)), Material(albedo=vec3(0.9, 0.5, 0.2))),
        Object("torus2", _placed(torus_mesh(16, 8, R=1.5, r=0.5), (-3.0, 0.0001, -9.0)),
               Material(albedo=vec3(0.2, 0.5, 0.9))),
        Object("ground", initPlane(objectToWorld=mat4(1.0)), Material(albedo=vec3(0.4))),
    ]
    return Scene(objects=objects, lights=_warm_lights(), fov=50.0, cameraToWorld=_std_camera(0.0, 5.5, 1.5),
                 bgColor=vec3(0.01, 0.03, 0.05))


SCENES = {
    "spheres-warm": spheres_warm,
    "spheres-warm-3": lambda: spheres_warm(3),
    "boxes2": boxes2,
    "boxtest": boxtest,
    "spheres-reflection": spheres_reflection,
    "spheres-pointlight1": spheres_pointlight1,
    "mesh-bunny": mesh_bunny,
    "mesh-teapot": mesh_teapot,
    "torus": torus_scene,
    "mesh-mix": mesh_mix,
    "two-meshes": two_meshes,
}
