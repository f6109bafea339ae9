"""Render the C3 frame whole (render_device) and as world-2 / world-4 band
sets (render_bands_device), REPS times each, for rocprofv3 --kernel-trace."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nim-raytracer_amd"))
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.dist import band_rows  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

W, H = 1920, 1080
ds = DeviceScene(scenes.mesh_bunny())
opts = Options(width=W, height=H, antialias=Antialias(akGrid, 16), bias=1e-4, precision=Precision.fp32)
fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
for _ in range(int(os.environ.get("REPS", "3"))):
    ds.render_device(opts, fb, stats=False)
    for world in (1, 2, 4):
        buf = torch.zeros(band_rows(H, 16, world) * W * 3, dtype=torch.float32, device="cuda")
        for rank in range(world):
            ds.render_bands_device(opts, buf, 16, rank, world, stats=False)
torch.cuda.synchronize()
