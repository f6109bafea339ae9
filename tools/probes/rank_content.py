"""Is a rank's band set dearer by content? (C5's ranks 0, 1, 7 of 8 run
~12 % longer than the others in every measurement order)

    RTMI_LIB=tools/ab/diag.so RTMI_COST_DUMP=gpurun_out/cost.bin CONFIG=C5 python tools/probes/rank_content.py

Renders the config's whole frame once with the per-group cost dump (every
pixel's wave time, s_memtime cycles; one pixel per group at >= 64 spp) and
sums it over each rank's rows for several band layouts: 4-row bands
round-robin (the shipped layout), 2 / 8 / 16-row bands, and a layout that
rotates the rank order every 8 bands. Prints one JSON line."""
import json
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

CFG = os.environ.get("CONFIG", "C5")
name, W, H, M, _ = CONFIGS[CFG]
path = os.environ["RTMI_COST_DUMP"]
ds = DeviceScene(_scene(name))
o = Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32)
fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
ds.render_device(o, fb)
torch.cuda.synchronize()
cost = np.fromfile(path, dtype=np.uint32).astype(np.float64)
assert cost.size == W * H, (cost.size, W * H)
row = cost.reshape(H, W).sum(axis=1)
bands = {"rr4": (4, lambda b, n: b % n), "rr2": (2, lambda b, n: b % n), "rr8": (8, lambda b, n: b % n),
         "rr16": (16, lambda b, n: b % n), "rot4": (4, lambda b, n: (b + b // n) % n)}
out = {"config": CFG, "total_cycles": float(row.sum()),
       "by_row_mod32": [round(float(row[k::32].sum() / row.sum() * 32), 4) for k in range(32)]}
for world in (4, 8):
    for key, (bh, f) in bands.items():
        r = np.zeros(world)
        for y in range(H):
            r[f(y // bh, world)] += row[y]
        out[f"w{world}_{key}"] = [round(float(x / r.mean()), 4) for x in r]
# the dearest pixels (a launch's tail is its last expensive item) and, per
# rank of 8 (4-row bands), its dearest pixel against the mean pixel
px = cost.reshape(H, W)
top = np.argsort(px, axis=None)[::-1][:40]
mean = float(px.mean())
out["mean_pixel_cycles"] = round(mean, 1)
out["top_pixels"] = [[int(i // W), int(i % W), int((i // W) // 4 % 8), round(float(px.flat[i]) / mean, 1)] for i in top]
out["w8_rr4_max_over_mean"] = [round(float(px[[y for y in range(H) if (y // 4) % 8 == r]].max()) / mean, 1)
                               for r in range(8)]
out["p999_over_mean"] = round(float(np.quantile(px, 0.999)) / mean, 1)
print(json.dumps(out), flush=True)
