"""Host-side mirror of the reference's renderer data model.

Same names, fields and argument meaning as the Nim types so that scenes and
tests read like the reference's:
  Geometry/Sphere/Plane/Box/TriangleMesh + init*  src/renderer/geom.nim:137-198
  Material                                       src/renderer/material.nim:4-7
  Object / Scene                                 src/renderer/scene.nim:6-18
  Light / DistantLight / PointLight              src/renderer/light.nim:9-17
  AntialiasKind / Antialias / Options            src/renderer/renderer.nim:10-28
  Stats                                          src/renderer/stats.nim:4-13

`flatten(scene)` produces the rt_scene_desc the C-ABI consumes (one flattening,
done once per scene, as the Nim shim in INTEGRATION.md does).
"""
import ctypes as C
import enum
from dataclasses import dataclass, field

import numpy as np

from . import abi
from .glm import inverse, mat4, flat


class Geometry:
    def __init__(self, objectToWorld=None):
        self.objectToWorld = np.asarray(mat4(1.0) if objectToWorld is None else objectToWorld,
                                        dtype=np.float64)
        self.worldToObject = inverse(self.objectToWorld)


class Sphere(Geometry):
    def __init__(self, r, objectToWorld=None):
        super().__init__(objectToWorld)
        self.r = float(r)


class Plane(Geometry):
    pass


class Box(Geometry):
    def __init__(self, vmin, vmax, objectToWorld=None):
        super().__init__(objectToWorld)
        self.vmin = np.asarray(vmin, dtype=np.float64)[:3].copy()
        self.vmax = np.asarray(vmax, dtype=np.float64)[:3].copy()


class TriangleMesh(Geometry):
    """vertices (N,3) float64, faces (F,3) int32, normals (F,3) float64 or None
    (None = calcNormals of src/loaders/obj.nim:65-84, done by the library)."""

    def __init__(self, vertices, faces, normals=None, objectToWorld=None):
        super().__init__(objectToWorld)
        self.vertices = np.ascontiguousarray(np.asarray(vertices, dtype=np.float64).reshape(-1, 3))
        self.faces = np.ascontiguousarray(np.asarray(faces, dtype=np.int32).reshape(-1, 3))
        self.normals = (None if normals is None else
                        np.ascontiguousarray(np.asarray(normals, dtype=np.float64).reshape(-1, 3)))


def initSphere(r, objectToWorld):
    return Sphere(r, objectToWorld)


def initPlane(objectToWorld):
    return Plane(objectToWorld)


def initBox(vmin, vmax, objectToWorld):
    return Box(vmin, vmax, objectToWorld)


def initTriangleMesh(vertices, normals, faces, objectToWorld):
    return TriangleMesh(vertices, faces, normals, objectToWorld)


@dataclass
class Material:
    albedo: object = field(default_factory=lambda: np.zeros(3))
    reflection: float = 0.0


@dataclass
class Object:
    name: str
    geometry: Geometry
    material: Material


@dataclass
class DistantLight:
    color: object
    intensity: float
    dir: object


@dataclass
class PointLight:
    color: object
    intensity: float
    pos: object


@dataclass
class Scene:
    objects: list
    lights: list
    fov: float
    cameraToWorld: object
    bgColor: object


class AntialiasKind(enum.IntEnum):
    akNone = abi.RT_AA_NONE
    akGrid = abi.RT_AA_GRID
    akJittered = abi.RT_AA_JITTERED
    akMultiJittered = abi.RT_AA_MULTI_JITTERED
    akCorrelatedMultiJittered = abi.RT_AA_CORRELATED_MULTI_JITTERED


akNone = AntialiasKind.akNone
akGrid = AntialiasKind.akGrid
akJittered = AntialiasKind.akJittered
akMultiJittered = AntialiasKind.akMultiJittered
akCorrelatedMultiJittered = AntialiasKind.akCorrelatedMultiJittered


@dataclass
class Antialias:
    kind: AntialiasKind = akNone
    gridSize: int = 1


class Precision(enum.IntEnum):
    fp32 = abi.RT_FP32
    fp64 = abi.RT_FP64


@dataclass
class Options:
    width: int
    height: int
    antialias: Antialias = field(default_factory=Antialias)
    bias: float = 1e-8
    maxRayDepth: int = 5
    # device-path knobs (not in the reference's Options)
    precision: Precision = Precision.fp32
    flags: int = 0
    seed: int = 0x5EED

    @property
    def spp(self):
        if self.antialias.kind == akNone:
            return 1
        return self.antialias.gridSize * self.antialias.gridSize

    def to_c(self):
        o = abi.rt_options()
        o.width = int(self.width)
        o.height = int(self.height)
        o.aa_kind = int(self.antialias.kind)
        o.grid_size = int(self.antialias.gridSize)
        o.bias = float(self.bias)
        o.max_ray_depth = int(self.maxRayDepth)
        o.precision = int(self.precision)
        o.seed = int(self.seed)
        o.flags = int(self.flags)
        return o


@dataclass
class Stats:
    numPrimaryRays: int = 0
    numIntersectionTests: int = 0
    numIntersectionHits: int = 0
    numShadowRays: int = 0
    numReflectionRays: int = 0

    def __iadd__(self, o):
        self.numPrimaryRays += o.numPrimaryRays
        self.numIntersectionTests += o.numIntersectionTests
        self.numIntersectionHits += o.numIntersectionHits
        self.numShadowRays += o.numShadowRays
        self.numReflectionRays += o.numReflectionRays
        return self

    @classmethod
    def from_c(cls, s):
        return cls(int(s.num_primary_rays), int(s.num_intersection_tests),
                   int(s.num_intersection_hits), int(s.num_shadow_rays),
                   int(s.num_reflection_rays))

    @property
    def rays(self):
        """Primary + shadow rays: the numerator of the Mray/s metric."""
        return self.numPrimaryRays + self.numShadowRays


def _d(arr, n):
    a = (C.c_double * n)()
    for i, v in enumerate(np.asarray(arr, dtype=np.float64).reshape(-1)[:n]):
        a[i] = float(v)
    return a


class FlatScene:
    """rt_scene_desc plus the buffers it points into (kept alive together)."""

    def __init__(self, scene: Scene):
        objs = scene.objects
        self._meshes = []
        mesh_index = {}
        self._objs = (abi.rt_object_desc * max(1, len(objs)))()
        for i, ob in enumerate(objs):
            g = ob.geometry
            d = self._objs[i]
            d.object_to_world = _d(flat(g.objectToWorld), 16)
            d.world_to_object = _d(flat(g.worldToObject), 16)
            d.albedo = _d(ob.material.albedo, 3)
            d.reflection = float(ob.material.reflection)
            d.mesh = -1
            if isinstance(g, Sphere):
                d.type = abi.RT_SPHERE
                d.radius = g.r
            elif isinstance(g, Plane):
                d.type = abi.RT_PLANE
            elif isinstance(g, Box):
                d.type = abi.RT_BOX
                d.box_min = _d(g.vmin, 3)
                d.box_max = _d(g.vmax, 3)
            elif isinstance(g, TriangleMesh):
                d.type = abi.RT_MESH
                if id(g) not in mesh_index:
                    mesh_index[id(g)] = len(self._meshes)
                    self._meshes.append(g)
                d.mesh = mesh_index[id(g)]
            else:
                raise TypeError(f"unsupported geometry {type(g).__name__}")
        self._mdesc = (abi.rt_mesh_desc * max(1, len(self._meshes)))()
        for i, g in enumerate(self._meshes):
            m = self._mdesc[i]
            m.vertices = g.vertices.ctypes.data_as(C.POINTER(C.c_double))
            m.num_vertices = g.vertices.shape[0]
            m.faces = g.faces.ctypes.data_as(C.POINTER(C.c_int32))
            m.num_faces = g.faces.shape[0]
            m.normals = (None if g.normals is None else
                         g.normals.ctypes.data_as(C.POINTER(C.c_double)))
        self._lights = (abi.rt_light_desc * max(1, len(scene.lights)))()
        for i, l in enumerate(scene.lights):
            d = self._lights[i]
            d.color = _d(l.color, 3)
            d.intensity = float(l.intensity)
            if isinstance(l, DistantLight):
                d.type = abi.RT_DISTANT_LIGHT
                d.dir = _d(l.dir, 3)
            elif isinstance(l, PointLight):
                d.type = abi.RT_POINT_LIGHT
                d.pos = _d(l.pos, 3)
            else:
                raise TypeError(f"unsupported light {type(l).__name__}")
        desc = abi.rt_scene_desc()
        desc.objects = C.cast(self._objs, C.POINTER(abi.rt_object_desc))
        desc.num_objects = len(objs)
        desc.lights = C.cast(self._lights, C.POINTER(abi.rt_light_desc))
        desc.num_lights = len(scene.lights)
        desc.meshes = C.cast(self._mdesc, C.POINTER(abi.rt_mesh_desc))
        desc.num_meshes = len(self._meshes)
        desc.fov = float(scene.fov)
        desc.camera_to_world = _d(flat(scene.cameraToWorld), 16)
        desc.bg_color = _d(scene.bgColor, 3)
        self.desc = desc


def flatten(scene: Scene) -> FlatScene:
    return FlatScene(scene)
