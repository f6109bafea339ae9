"""Stats and frame hashes of one scene under several rt_options flag sets,
each rendered twice (determinism + cross-path identity probe).

    RTMI_LIB=... SCENE=mesh-bunny W=200 H=120 M=16 FLAGS=0,0x400,0x100,0x8 python tools/flag_stats.py
"""
import hashlib
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nim-raytracer_amd"))
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.abi import RT_FLAG_NO_REORDER  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

W, H, M = int(os.environ.get("W", 200)), int(os.environ.get("H", 120)), int(os.environ.get("M", 16))
ds = DeviceScene(scenes.SCENES[os.environ.get("SCENE", "mesh-bunny")]())
ref = None
for f in [int(x, 0) for x in os.environ.get("FLAGS", "0,0x400,0x100,0x8").split(",")]:
    for rep in range(2):
        o = Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32,
                    flags=f | RT_FLAG_NO_REORDER)
        fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
        st = ds.render_device(o, fb)
        img = fb.cpu()
        h = hashlib.sha256(img.numpy().tobytes()).hexdigest()[:12]
        d = "" if ref is None else f" maxdiff {float((img - ref).abs().max()):.3g} ndiff {int(((img - ref) != 0).sum())}"
        ref = img if ref is None else ref
        print(f"flags {f:#x} rep {rep}: hits {st.numIntersectionHits} shadow {st.numShadowRays} frame {h}{d}", flush=True)
