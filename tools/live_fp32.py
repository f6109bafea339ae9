"""The float32 performance mode on the reference's live inputs
(src/raytracer.nim:43-54: teapot.obj via mesh-bunny.nim, 300x200, akNone,
bias 1e-8, depth 5) against the float64 oracle: per-pixel error
distribution and Stats, at the reference's bias and at 1e-4 (the bias the
benchmark configs use). Prints one JSON line per (scene, bias)."""
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path[:0] = [os.path.join(REPO, "nim-raytracer_amd"), os.path.join(REPO, "oracle")]
import numpy as np  # noqa: E402

import oracle  # noqa: E402
from rtmi import Antialias, Options, Precision, akNone, scenes  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

oracle.build()
for name in ("mesh-teapot", "boxes2", "spheres-warm"):
    sc = scenes.SCENES[name]()
    ds = DeviceScene(sc)
    for bias in (1e-8, 1e-4):
        o64 = Options(width=300, height=200, antialias=Antialias(akNone, 1), bias=bias, maxRayDepth=5,
                      precision=Precision.fp64)
        ref, rst, _ = oracle.OracleScene(sc).render(o64)
        o32 = Options(width=300, height=200, antialias=Antialias(akNone, 1), bias=bias, maxRayDepth=5,
                      precision=Precision.fp32)
        got = np.zeros_like(ref)
        gst = ds.render_lines(o32, got, 0, 200)
        err = np.abs(got.astype(np.float64) - ref).max(axis=-1)
        print(json.dumps({"scene": name, "bias": bias, "pixels": int(err.size), "max_err": float(err.max()),
                          "mean_err": float(err.mean()), "within_2e-3": float((err <= 2e-3).mean()),
                          "within_1e-4": float((err <= 1e-4).mean()), "gpu_stats": str(gst), "oracle_stats": str(rst)}),
              flush=True)
