"""Per-launch overhead vs work: rank 0's band set of the C3 frame for
world = 1 .. 64 (render_bands_device, HIP events, median of REPS).
NO_REORDER=1: screen-order work queue (RT_FLAG_NO_REORDER) for comparison."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nim-raytracer_amd"))
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.abi import RT_FLAG_NO_REORDER  # noqa: E402
from rtmi.dist import band_rows  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

W, H = 1920, 1080
ds = DeviceScene(scenes.mesh_bunny())
flags = RT_FLAG_NO_REORDER if os.environ.get("NO_REORDER") else 0
opts = Options(width=W, height=H, antialias=Antialias(akGrid, 16), bias=1e-4, precision=Precision.fp32, flags=flags)
out = {"reorder": not flags}
for world in (1, 2, 4, 8, 16, 32, 64):
    rows = band_rows(H, 4, world)
    buf = torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda")
    ts = []
    for _ in range(int(os.environ.get("REPS", "5"))):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ds.render_bands_device(opts, buf, 4, 0, world, stats=False)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    out[world] = round(sorted(ts)[len(ts) // 2], 4)
print(json.dumps(out))
