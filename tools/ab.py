"""In-process A/B timing of several librtmi.so builds (interleaved reps).

    RTMI_LIBS=path/a.so,path/b.so ABLATE=c3_full,ground_nolights python tools/ab.py
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, "nim-raytracer_amd")
import torch  # noqa: E402  (one HIP runtime for all libraries)

from rtmi import abi, scenes  # noqa: E402
from rtmi.glm import inverse, mat4, translate, vec3  # noqa: E402
from rtmi.scene import Antialias, Options, Precision, akGrid, flatten  # noqa: E402


def load(path):
    return abi.bind(C.CDLL(path))


def variants():
    base = scenes.mesh_bunny()
    o = Options(width=1920, height=1080, antialias=Antialias(akGrid, 16), bias=1e-4,
                precision=Precision.fp32)
    v = {"c3_full": (base, o)}
    s = scenes.mesh_bunny(); s.objects = [s.objects[1]]; s.lights = []; v["ground_nolights"] = (s, o)
    s = scenes.mesh_bunny(); s.objects = [s.objects[1]]; v["ground_only"] = (s, o)
    s = scenes.mesh_bunny(); s.objects = [s.objects[0]]; v["bunny_only"] = (s, o)
    s = scenes.mesh_bunny(); s.lights = []; v["c3_nolights"] = (s, o)
    # every pixel lean (the bunny and its shadows off screen)
    s = scenes.mesh_bunny(); s.objects[0].geometry.objectToWorld = translate(mat4(1.0), vec3(200.0, 0.0001, -12.0))
    s.objects[0].geometry.worldToObject = inverse(s.objects[0].geometry.objectToWorld); v["lean_only"] = (s, o)
    s = scenes.mesh_bunny(); s.objects[0].geometry.objectToWorld = translate(mat4(1.0), vec3(200.0, 0.0001, -12.0))
    s.objects[0].geometry.worldToObject = inverse(s.objects[0].geometry.objectToWorld); s.lights = []
    v["lean_nolights"] = (s, o)
    v["boxes2_c2"] = (scenes.boxes2(), Options(width=1920, height=1080, antialias=Antialias(akGrid, 8),
                                               bias=1e-4, precision=Precision.fp32))
    # fallback-kernel scenes: mesh + spheres / boxes /
    # rotations + point light + reflection, two meshes
    for nm in ("mesh-mix", "two-meshes"):
        v[nm.replace("-", "_") + "_64"] = (scenes.SCENES[nm](), Options(width=1920, height=1080,
                                                                         antialias=Antialias(akGrid, 8), bias=1e-4,
                                                                         maxRayDepth=5, precision=Precision.fp32))
    # the other analytic scenes (feature subsets of their own), 1080p 64 spp
    for nm in ("spheres-warm", "spheres-reflection", "spheres-pointlight1", "boxtest"):
        v[nm.replace("-", "_") + "_64"] = (scenes.SCENES[nm](), Options(width=1920, height=1080,
                                                                         antialias=Antialias(akGrid, 8), bias=1e-4,
                                                                         maxRayDepth=5, precision=Precision.fp32))
    # C5 (only when asked for: 72 ms a frame)
    v["c5_full"] = (scenes.torus_scene(), Options(width=3840, height=2160, antialias=Antialias(akGrid, 64), bias=1e-4,
                                                  precision=Precision.fp32))
    sel = os.environ.get("ABLATE", "")
    return {k: x for k, x in v.items() if (not sel and k != "c5_full") or k in sel.split(",")}


def main():
    libs = os.environ["RTMI_LIBS"].split(",")
    reps = int(os.environ.get("REPS", "4"))
    L = [load(p) for p in libs]
    for lib in L:
        assert lib.rt_init(0) == 0, lib.rt_last_error()
    res = {}
    stream = torch.cuda.current_stream()
    for name, (scene, opts) in variants().items():
        flat = flatten(scene)
        hs = []
        for lib in L:
            h = C.c_void_p()
            assert lib.rt_scene_create(C.byref(flat.desc), C.byref(h)) == 0, lib.rt_last_error()
            hs.append(h)
        fb = torch.zeros(opts.width * opts.height * 3, dtype=torch.float32, device="cuda")
        o = opts.to_c()
        times = {p: [] for p in libs}
        ref_img = None
        for p, lib, h in zip(libs, L, hs):  # Stats + image agreement across builds
            st = abi.rt_stats()
            assert lib.rt_render_lines_device(h, C.byref(o), C.c_void_p(fb.data_ptr()), 0, opts.height, 1, 1,
                                              C.c_void_p(stream.cuda_stream or None), C.byref(st)) == 0
            torch.cuda.synchronize()
            img = fb.cpu()
            if ref_img is None:
                ref_img = img
            d = (img - ref_img).abs()
            print(f"  {os.path.basename(p)}: stats=({st.num_primary_rays},{st.num_intersection_tests},"
                  f"{st.num_intersection_hits},{st.num_shadow_rays},{st.num_reflection_rays}) "
                  f"maxdiff={d.max().item():.3g} frac>2e-3={(d > 2e-3).float().mean().item():.2e}", flush=True)
        for r in range(reps):
            for p, lib, h in zip(libs, L, hs):
                st = abi.rt_stats()
                lib.rt_render_lines_device(h, C.byref(o), C.c_void_p(fb.data_ptr()), 0, opts.height, 1, 1,
                                           C.c_void_p(stream.cuda_stream or None), C.byref(st))
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(3):
                    lib.rt_render_lines_device(h, C.byref(o), C.c_void_p(fb.data_ptr()), 0, opts.height, 1, 1,
                                               C.c_void_p(stream.cuda_stream or None), None)
                e1.record(stream)
                torch.cuda.synchronize()
                times[p].append(e0.elapsed_time(e1) / 3)
        for lib, h in zip(L, hs):
            lib.rt_scene_destroy(h)
        res[name] = {os.path.basename(p): round(min(t), 3) for p, t in times.items()}
        print(name, res[name], flush=True)
    json.dump(res, open("gpurun_out/ab.json", "w"), indent=1)


if __name__ == "__main__":
    main()
