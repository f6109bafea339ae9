"""Median C3 render_device time (HIP events) + Stats of this process's librtmi
build/environment; one JSON line. Env: REPS, CONFIG (C3|C2)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nim-raytracer_amd"))
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

cfg = os.environ.get("CONFIG", "C3")
scene, W, H, m = {"C3": (scenes.mesh_bunny, 1920, 1080, 16), "C2": (scenes.boxes2, 1920, 1080, 8),
                  "C4": (scenes.mesh_bunny, 3840, 2160, 32),
                  "C5": (scenes.torus_scene, 3840, 2160, 16)}[cfg]
ds = DeviceScene(scene())
info = ds.info()
opts = Options(width=W, height=H, antialias=Antialias(akGrid, m), bias=1e-4, precision=Precision.fp32,
               flags=int(os.environ.get("RTMI_FLAGS", "0"), 0))
fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
st = ds.render_device(opts, fb, stats=True)
ts = []
for _ in range(int(os.environ.get("REPS", "5"))):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    ds.render_device(opts, fb, stats=False)
    b.record()
    torch.cuda.synchronize()
    ts.append(a.elapsed_time(b))
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("RTMI_")}, "config": cfg,
                  "ms": round(sorted(ts)[len(ts) // 2], 3), "nodes": info["num_bvh_nodes"],
                  "depth": info["max_bvh_depth"], "stats": [st.numPrimaryRays, st.numIntersectionHits,
                                                             st.numShadowRays]}), flush=True)
