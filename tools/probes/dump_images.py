"""Debug helper: render scenes on the GPU in both precisions, save npz."""
import sys, os
sys.path.insert(0, 'nim-raytracer_amd')
import numpy as np, torch
from rtmi import Antialias, Options, Precision, akGrid, akNone, scenes
from rtmi.renderer import DeviceScene
out = {}
CASES = [("mesh-bunny", 48, 32, akGrid, 2), ("spheres-warm-3", 160, 120, akNone, 1),
         ("boxes2", 160, 90, akGrid, 2), ("mesh-bunny", 96, 64, akNone, 1), ("boxtest", 120, 80, akNone, 1)]
sel = os.environ.get("DUMP", "")
for name, w, h, aa, m in CASES:
    if sel and name not in sel.split(","):
        continue
    ds = DeviceScene(scenes.SCENES[name]())
    for prec in (Precision.fp32, Precision.fp64):
        o = Options(width=w, height=h, antialias=Antialias(aa, m), bias=1e-4, precision=prec)
        fb = np.zeros((h, w, 3), np.float32)
        st = ds.render_lines(o, fb, 0, h)
        key = f"{name}_{w}x{h}_{int(prec)}"
        out[key] = fb
        print(key, st)
np.savez('gpurun_out/dump.npz', **out)
