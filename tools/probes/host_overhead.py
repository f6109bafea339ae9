"""Host cost of the per-frame render call at multi-GPU band sizes, on one GPU.

For world in 1,2,4,8 rank 0's band set of the C3 frame is rendered K times
back to back from Python exactly as bench.py's timed loop issues it
(render_bands_device, stats=False, no synchronisation in between). Printed
per world: the wall time per call, the GPU time per call (HIP events around
the whole loop / K), and the host time spent inside each call (ctypes +
rt_render_bands_device up to its return). Wall >> GPU means the launches,
not the kernels, pace the frame at that rank's share of the image."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nim-raytracer_amd"))
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.dist import band_rows  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

W, H, M, BAND = 1920, 1080, 16, 4
K = int(os.environ.get("K", "50"))
ds = DeviceScene(scenes.mesh_bunny())
opts = Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32)
stream = torch.cuda.current_stream()
for world in (1, 2, 4, 8):
    rows = band_rows(H, BAND, world)
    buf = torch.zeros(rows * W * 3, dtype=torch.float32, device="cuda")
    for _ in range(3):
        ds.render_bands_device(opts, buf, BAND, 0, world, stream=stream, stats=False)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    host = 0.0
    t0 = time.perf_counter()
    a.record(stream)
    for _ in range(K):
        c0 = time.perf_counter()
        ds.render_bands_device(opts, buf, BAND, 0, world, stream=stream, stats=False)
        host += time.perf_counter() - c0
    b.record(stream)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / K * 1e3
    # GPU-only reference: the same calls, each timed alone (idle gaps excluded)
    ts = []
    for _ in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ds.render_bands_device(opts, buf, BAND, 0, world, stream=stream, stats=False)
        e1.record(stream)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(json.dumps({"world": world, "wall_ms_per_call": round(wall, 4),
                      "loop_gpu_ms_per_call": round(a.elapsed_time(b) / K, 4),
                      "single_call_gpu_ms": round(sorted(ts)[2], 4),
                      "host_ms_in_call": round(host / K * 1e3, 4)}), flush=True)
