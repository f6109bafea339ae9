"""Render-kernel time (RT_FLAG_TIMING: the build excluded) of the C3 frame
against launch size: rank 0 of a band-sharded frame (band heights 4 and 16)
and a contiguous run of H / world rows, for world = 1..16. Separates what a
smaller launch costs (ramp, tail) from what the band layout costs."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nim-raytracer_amd"))
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.abi import RT_FLAG_TIMING  # noqa: E402
from rtmi.dist import band_rows  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

W, H, M = 1920, 1080, 16
REPS = int(os.environ.get("REPS", "7"))
ds = DeviceScene(scenes.mesh_bunny())
opts = Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32,
               flags=RT_FLAG_TIMING | int(os.environ.get("RTMI_FLAGS", "0"), 0))
stream = torch.cuda.current_stream()
buf = torch.zeros((H + 16 * 16) * W * 3, dtype=torch.float32, device="cuda")  # (band buffers round up)


def med(fn):
    fn()
    fn()
    su, re = [], []
    for _ in range(REPS):
        fn()
        torch.cuda.synchronize()
        a, b = ds.last_timing()
        su.append(a)
        re.append(b)
    return round(sorted(su)[REPS // 2] * 1000, 1), round(sorted(re)[REPS // 2] * 1000, 1)


for world in [int(w) for w in os.environ.get("WORLDS", "1,2,4,8,16").split(",")]:
    res = {"world": world}
    for bh in (4, 16):
        s, r = med(lambda: ds.render_bands_device(opts, buf, bh, 0, world, stream=stream, stats=False))
        res[f"band{bh}_setup_us"], res[f"band{bh}_render_us"] = s, r
        res[f"band{bh}_split"] = list(ds.last_split())
    s, r = med(lambda: ds.render_device(opts, buf, 0, H // world, stream=stream, stats=False))
    res["rows_setup_us"], res["rows_render_us"] = s, r
    res["rows_split"] = list(ds.last_split())
    mid = (H - H // world) // 2
    s, r = med(lambda: ds.render_device(opts, buf, mid, mid + H // world, stream=stream, stats=False))
    res["midrows_setup_us"], res["midrows_render_us"] = s, r
    res["midrows_split"] = list(ds.last_split())
    print(json.dumps(res), flush=True)
