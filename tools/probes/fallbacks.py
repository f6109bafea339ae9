"""General pixels the batched kernel re-renders with the one-sample (BVH)
loop because a shadow ray needed the BVH (rt_scene_last_batch), per config:
the whole frame and every rank of 8 (4-row bands), with each rank's call time.

    CONFIGS=C3,C4,C5 python tools/probes/fallbacks.py"""
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(REPO, "nim-raytracer_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from bench import CONFIGS, _scene  # noqa: E402
from rtmi import Antialias, Options, Precision, akGrid  # noqa: E402
from rtmi.dist import band_rows  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

for cfg in os.environ.get("CONFIGS", "C5").split(","):
    name, W, H, M, _ = CONFIGS[cfg]
    ds = DeviceScene(_scene(name))
    o = Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32)
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    ds.render_device(o, fb)
    out = {"config": cfg, "frame": list(ds.last_batch()), "ranks": []}
    rows = band_rows(H, 4, 8)
    buf = torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda")
    for r in range(8):
        ds.render_bands_device(o, buf, 4, r, 8)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ds.render_bands_device(o, buf, 4, r, 8)
        b.record()
        torch.cuda.synchronize()
        out["ranks"].append([r, list(ds.last_batch()), round(a.elapsed_time(b), 3)])
    print(json.dumps(out), flush=True)
