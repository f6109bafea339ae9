"""One rank's band launch of the C3 frame, repeated (for a kernel trace of
the per-rank build and render at N > 1):

    rocprofv3 --kernel-trace --stats -- python3 tools/rank_prof.py   # WORLD=8 RANK=0 BAND=4 REPS=20 CONFIG=C3

CONFIG = a bench.py config (C3 default; C4 / C5 the 4K frames); WORLD=1 is
the whole frame through the band path.
"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nim-raytracer_amd"))
import torch  # noqa: E402

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bench import CONFIGS, _scene  # noqa: E402
from rtmi import Antialias, Options, Precision, akGrid  # noqa: E402
from rtmi.dist import band_rows  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

name, W, H, M, _ = CONFIGS[os.environ.get("CONFIG", "C3")]
world, rank = int(os.environ.get("WORLD", "8")), int(os.environ.get("RANK", "0"))
band_h, reps = int(os.environ.get("BAND", "4")), int(os.environ.get("REPS", "20"))
ds = DeviceScene(_scene(name))
opts = Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32)
stream = torch.cuda.current_stream()
buf = torch.zeros(band_rows(H, band_h, world) * W * 3, dtype=torch.float32, device="cuda")
for _ in range(reps):
    ds.render_bands_device(opts, buf, band_h, rank, world, stream=stream, stats=False)
torch.cuda.synchronize()
print("ok", world, rank, band_h, reps, ds.last_split())
