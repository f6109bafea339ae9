"""Where a C3 frame's wave time goes, by pixel class (diagnostic).

    RTMI_COST_DUMP=gpurun_out/cost.bin python tools/cost_map.py

Every pixel group's duration (s_memtime cycles of the wave that rendered it,
rtmi.cpp RTMI_COST_DUMP) for the full C3 frame (one pixel per group at 256
spp), summed over: pixels whose camera rays hit the bunny, ground pixels the
bunny changes (its shadows), and the rest (ground / sky)."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, "nim-raytracer_amd")
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

W, H = 1920, 1080
path = os.environ["RTMI_COST_DUMP"]


def render(scene, m=16, flags=0):
    ds = DeviceScene(scene)
    o = Options(width=W, height=H, antialias=Antialias(akGrid, m), bias=1e-4, precision=Precision.fp32, flags=flags)
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    ds.render_device(o, fb)
    torch.cuda.synchronize()
    return fb.view(H, W, 3).cpu().numpy()


s = scenes.mesh_bunny(); s.objects = [s.objects[0]]
bunny = render(s, 2)
bg = np.array(scenes.mesh_bunny().bgColor[:3], np.float32)
A = np.abs(bunny - bg).max(axis=2) > 1e-6                # camera rays reach the bunny
s = scenes.mesh_bunny(); s.objects = [s.objects[1]]
ground = render(s)
out = {}
for name, flags in (("bvh", 0x8), ("binned", 0)):
    full = render(scenes.mesh_bunny(), flags=flags)       # last launch: its costs are in the dump
    cost = np.fromfile(path, dtype=np.uint32).astype(np.float64).reshape(H, W)
    B = (np.abs(full - ground).max(axis=2) > 1e-6) & ~A  # ground pixels the bunny changes
    C = ~A & ~B
    tot = cost.sum()
    out[name] = {k: {"pixels": int(m.sum()), "cost_share": round(float(cost[m].sum() / tot), 4),
                     "mean_cycles": round(float(cost[m].mean()), 1)}
                 for k, m in (("bunny", A), ("bunny_shadow", B), ("rest", C))}
    out[name]["total_cycles"] = tot
print(json.dumps(out, indent=1))
