"""Per-rank render time of the band-sharded C3 frame, simulated on one GPU:
for N in 1,2,4,8 every rank's rt_render_bands_device call is timed (HIP
events, median of REPS) and the slowest rank is the N-GPU render time (the
all-gather + unshard come on top). Also each rank's back-to-back rate
(REPS calls issued without a host sync, total / REPS): a rank's step loop,
where a call's per-call build overlaps the previous call's render
(rt_scene bstream). Prints one JSON line per band height."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nim-raytracer_amd"))
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.dist import band_rows  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

W, H, M = 1920, 1080, 16
REPS = int(os.environ.get("REPS", "5"))
ds = DeviceScene(scenes.mesh_bunny())
opts = Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32,
               flags=int(os.environ.get("RTMI_FLAGS", "0"), 0))
stream = torch.cuda.current_stream()
for band_h in [int(b) for b in os.environ.get("BANDS", "16,8,4").split(",")]:
    res = {"band_h": band_h}
    for world in (1, 2, 4, 8):
        rows = band_rows(H, band_h, world)
        buf = torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda")
        per, b2b = [], []
        for rank in range(world):
            ts = []
            for _ in range(2):  # warm: the first launch of a mapping measures its launch order
                ds.render_bands_device(opts, buf, band_h, rank, world, stream=stream, stats=False)
            for _ in range(REPS):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record(stream)
                ds.render_bands_device(opts, buf, band_h, rank, world, stream=stream, stats=False)
                b.record(stream)
                torch.cuda.synchronize()
                ts.append(a.elapsed_time(b))
            per.append(sorted(ts)[len(ts) // 2])
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(stream)
            for _ in range(REPS):
                ds.render_bands_device(opts, buf, band_h, rank, world, stream=stream, stats=False)
            b.record(stream)
            torch.cuda.synchronize()
            b2b.append(a.elapsed_time(b) / REPS)
            if rank == 0:
                res[f"world{world}_split"] = list(ds.last_split())
        res[f"world{world}_max_ms"] = round(max(per), 3)
        res[f"world{world}_mean_ms"] = round(sum(per) / world, 3)
        res[f"world{world}_b2b_max_ms"] = round(max(b2b), 4)
    res["render_speedup_8"] = round(res["world1_max_ms"] / res["world8_max_ms"], 2)
    res["b2b_speedup_8"] = round(res["world1_b2b_max_ms"] / res["world8_b2b_max_ms"], 2)
    print(json.dumps(res), flush=True)
