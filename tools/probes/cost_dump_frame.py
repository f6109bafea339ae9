"""Save one config's whole-frame per-pixel cost map (the cost-dump build:
every pixel group's wave time in s_memtime cycles, one pixel per group at
>= 64 spp) as gpurun_out/costmap_<cfg>.npz, for scheduling simulations on
the CPU (tools/probes/sched_sim.py).

    RTMI_LIB=tools/ab/diag.so RTMI_COST_DUMP=/tmp/c.bin CONFIG=C3 python tools/probes/cost_dump_frame.py"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(REPO, "nim-raytracer_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from bench import CONFIGS, _scene  # noqa: E402
from rtmi import Antialias, Options, Precision, akGrid  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

CFG = os.environ.get("CONFIG", "C3")
name, W, H, M, _ = CONFIGS[CFG]
ds = DeviceScene(_scene(name))
o = Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32)
fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
ds.render_device(o, fb)
torch.cuda.synchronize()
cost = np.fromfile(os.environ["RTMI_COST_DUMP"], dtype=np.uint32).reshape(H, W)
# the two-class split of the same frame (normal build path: lean / general
# per pixel is not exposed, so the frame is re-rendered without the dump to
# read the counts only)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(REPO, "gpurun_out", f"costmap_{CFG.lower()}.npz"), cost=cost,
                    img=fb.view(H, W, 3).cpu().numpy())
print(CFG, cost.mean(), cost.max(), flush=True)
