"""Render-call times of several scenes (float32, device framebuffer): the
per-call camera-dependent build and the render kernels (RT_FLAG_TIMING), and
Mray/s (primary + shadow). Diagnostic for DESIGN.md's per-scene figures.

    python tools/scene_times.py [name:WxH:m ...]    (default: a fixed list)
"""
import json
import sys

sys.path.insert(0, "nim-raytracer_amd")
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, akNone, scenes  # noqa: E402
from rtmi.abi import RT_FLAG_TIMING  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

DEFAULT = ["boxes2:1920x1080:8", "spheres-reflection:1920x1080:8", "mesh-mix:1920x1080:8",
           "spheres-pointlight1:1920x1080:8", "mesh-bunny:1920x1080:16", "two-meshes:1920x1080:8"]


def main(args):
    out = {}
    for spec in args or DEFAULT:
        name, size, m = spec.split(":")
        w, h = (int(v) for v in size.split("x"))
        m = int(m)
        extra = 0
        if "+" in name:
            name, f = name.split("+")
            extra = int(f, 0)
        ds = DeviceScene(scenes.SCENES[name]())
        o = Options(width=w, height=h, antialias=Antialias(akGrid if m > 1 else akNone, m), bias=1e-4,
                    precision=Precision.fp32, flags=RT_FLAG_TIMING | extra)
        fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
        st = ds.render_device(o, fb)
        for _ in range(2):
            ds.render_device(o, fb, stats=False)
        setup, render = [], []
        for _ in range(5):
            ds.render_device(o, fb, stats=False)
            a, b = ds.last_timing()
            setup.append(a)
            render.append(b)
        s, r = min(setup), min(render)
        rays = st.numPrimaryRays + st.numShadowRays
        out[spec] = {"setup_ms": round(s, 4), "render_ms": round(r, 4), "call_ms": round(s + r, 4),
                     "mray_s": round(rays / (s + r) / 1e3, 1), "primary": st.numPrimaryRays,
                     "shadow": st.numShadowRays, "reflection": st.numReflectionRays,
                     "kernels": ds.last_lean_kernel(), "split": ds.last_split()}
        print(spec, out[spec], flush=True)
        ds.close()
    json.dump(out, open("gpurun_out/scene_times.json", "w"), indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
