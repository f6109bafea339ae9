"""rtmi — MI355X-native (gfx950) trace/shade backend for nim-raytracer.

Host-side mirror of the reference's renderer API (src/renderer/*.nim) over the
C-ABI library librtmi.so (include/rtmi.h). Importing the package is cheap; the
native library is loaded on first use and its absence is an error, never a
silent fallback.
"""
from . import abi, glm
from .scene import (Antialias, AntialiasKind, Box, DistantLight, Material, Object, Options,
                    Plane, PointLight, Precision, Scene, Sphere, Stats, TriangleMesh, akGrid,
                    akNone, flatten, initBox, initPlane, initSphere, initTriangleMesh)

__all__ = [
    "abi", "glm", "Antialias", "AntialiasKind", "Box", "DistantLight", "Material", "Object",
    "Options", "Plane", "PointLight", "Precision", "Scene", "Sphere", "Stats", "TriangleMesh",
    "akGrid", "akNone", "flatten", "initBox", "initPlane", "initSphere", "initTriangleMesh",
]
