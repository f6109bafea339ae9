"""Where does the per-launch fixed cost come from? Times rank 0's band set
(render_bands_device, HIP events, median of REPS) at world 1 and 64 for
scenes / sample counts of different per-item cost, with and without the
expensive-first order. overhead = t64 - t1/64 (ms)."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nim-raytracer_amd"))
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.abi import RT_FLAG_NO_REORDER  # noqa: E402
from rtmi.dist import band_rows  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

W, H = 1920, 1080
REPS = int(os.environ.get("REPS", "5"))


def t_band(ds, opts, world):
    rows = band_rows(H, 4, world)
    buf = torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda")
    ts = []
    for _ in range(REPS):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ds.render_bands_device(opts, buf, 4, 0, world, stats=False)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return sorted(ts)[len(ts) // 2]


bunny = scenes.mesh_bunny()
ground = scenes.mesh_bunny()
ground.objects = [o for o in ground.objects if o.name == "ground"]
nolight = scenes.mesh_bunny()
nolight.lights = []
cases = [("bunny", bunny, 16), ("bunny", bunny, 8), ("bunny", bunny, 4), ("ground", ground, 16),
         ("bunny_nolight", nolight, 16)]
only = os.environ.get("CASES")
if only:
    cases = [c for c in cases if f"{c[0]}:{c[2]}" in only.split(",")]
for name, sc, m in cases:
    ds = DeviceScene(sc)
    for flags in (0, RT_FLAG_NO_REORDER):
        opts = Options(width=W, height=H, antialias=Antialias(akGrid, m), bias=1e-4, precision=Precision.fp32,
                       flags=flags)
        res = {}
        for world in (1, 2, 4, 8, 16, 64):  # measuring launch + order build outside the timing
            t_band(ds, opts, world)
            t_band(ds, opts, world)
            res[world] = t_band(ds, opts, world)
        print(json.dumps({"policy": os.environ.get("RTMI_ORDER", "1"), "p": os.environ.get("RTMI_ORDER_P", ""),
                          "scene": name, "spp": m * m, "reorder": not flags,
                          **{f"t{w}": round(t, 4) for w, t in res.items()},
                          **{f"over{w}": round(t - res[1] / w, 4) for w, t in res.items() if w > 1}}), flush=True)
