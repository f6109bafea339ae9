"""Host SAH vs device PLOC BVH: build time (rt_scene_info.build_ms = whole
scene setup) and the frame time of a trace through each tree.
  bunny: C3 (1920x1080, akGrid 16)      torus: C5 mesh (1M faces), 1080p akGrid 8"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nim-raytracer_amd"))
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.abi import RT_BVH_PLOC, RT_BVH_SAH  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402


def frame_ms(ds, opts, reps=3):
    fb = torch.zeros(opts.width * opts.height * 3, dtype=torch.float32, device="cuda")
    ds.render_device(opts, fb)
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ds.render_device(opts, fb, stats=False)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


cases = [("bunny", scenes.mesh_bunny(), 16), ("torus_1M", scenes.torus_scene(), 8)]
for name, scene, m in cases:
    opts = Options(width=1920, height=1080, antialias=Antialias(akGrid, m), bias=1e-4, precision=Precision.fp32)
    for builder, label in ((RT_BVH_SAH, "sah_host"), (RT_BVH_PLOC, "ploc_device")):
        DeviceScene(scene, bvh_builder=builder).close()  # warm (allocator, code objects)
        t0 = time.perf_counter()
        ds = DeviceScene(scene, bvh_builder=builder)
        wall = (time.perf_counter() - t0) * 1e3
        info = ds.info()
        print(json.dumps({"mesh": name, "builder": label, "faces": info["num_triangles"],
                          "nodes": info["num_bvh_nodes"], "depth": info["max_bvh_depth"],
                          "scene_setup_ms": round(info["build_ms"], 2), "create_wall_ms": round(wall, 2),
                          "frame_ms": round(frame_ms(ds, opts), 3), "spp": m * m}), flush=True)
        ds.close()
