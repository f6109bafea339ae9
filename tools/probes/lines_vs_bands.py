"""The whole C3 frame through rt_render_lines_device (mapping mode 0) and
through rt_render_bands_device with world 1 (mode 1, 4-row bands: the same
rows in the same order), interleaved, back to back per rep; frames compared.

    python tools/probes/lines_vs_bands.py"""
import json
import os
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..")
sys.path.insert(0, os.path.join(REPO, "nim-raytracer_amd"))
sys.path.insert(0, REPO)
import torch  # noqa: E402

from bench import CONFIGS, _scene  # noqa: E402
from rtmi import Antialias, Options, Precision, akGrid  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

name, W, H, M, _ = CONFIGS[os.environ.get("CONFIG", "C3")]
ds = DeviceScene(_scene(name))
o = Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32)
a = torch.zeros(W * H * 3, device="cuda")
b = torch.zeros(W * H * 3, device="cuda")
st = torch.cuda.current_stream()
calls = {"lines": lambda: ds.render_device(o, a, stream=st, stats=False),
         "bands_w1": lambda: ds.render_bands_device(o, b, 4, 0, 1, stream=st, stats=False)}
for f in calls.values():
    f()
    f()
torch.cuda.synchronize()
res = {k: [] for k in calls}
for rep in range(int(os.environ.get("REPS", "8"))):
    for k, f in calls.items():
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            f()
        e1.record(st)
        torch.cuda.synchronize()
        res[k].append(e0.elapsed_time(e1) / 10)
out = {k: round(sorted(v)[len(v) // 2], 4) for k, v in res.items()}
out["identical"] = bool(torch.equal(a, b))
print(json.dumps(out), flush=True)
