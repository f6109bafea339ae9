"""In-process A/B timing of librtmi.so builds x option flag sets on one
scene (interleaved reps; frames and Stats checked equal across all runs).

    RTMI_LIBS=a.so,b.so FLAGSETS=0,0x20 CONFIG=C3 REPS=6 python tools/ab_flags.py
"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, "nim-raytracer_amd")
import torch  # noqa: E402  (one HIP runtime for all libraries)

from rtmi import abi, scenes  # noqa: E402
from rtmi.scene import Antialias, Options, Precision, akGrid, flatten  # noqa: E402

CONFIGS = {"C3": (scenes.mesh_bunny, 1920, 1080, 16), "C2": (scenes.boxes2, 1920, 1080, 8),
           "C4": (scenes.mesh_bunny, 3840, 2160, 32), "C5": (scenes.torus_scene, 3840, 2160, 16)}


def main():
    libs = os.environ["RTMI_LIBS"].split(",")
    flagsets = [int(x, 0) for x in os.environ.get("FLAGSETS", "0").split(",")]
    reps = int(os.environ.get("REPS", "6"))
    make, W, H, m = CONFIGS[os.environ.get("CONFIG", "C3")]
    flat = flatten(make())
    stream = torch.cuda.current_stream()
    sp = C.c_void_p(stream.cuda_stream or None)
    runs = []
    for path in libs:
        lib = abi.bind(C.CDLL(path))
        assert lib.rt_init(0) == 0, lib.rt_last_error()
        h = C.c_void_p()
        assert lib.rt_scene_create(C.byref(flat.desc), C.byref(h)) == 0, lib.rt_last_error()
        for f in flagsets:
            o = Options(width=W, height=H, antialias=Antialias(akGrid, m), bias=1e-4, precision=Precision.fp32,
                        flags=f).to_c()
            runs.append((os.path.basename(path), f, lib, h, o))
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    ref = None
    info = {}
    for name, f, lib, h, o in runs:
        st = abi.rt_stats()
        assert lib.rt_render_lines_device(h, C.byref(o), C.c_void_p(fb.data_ptr()), 0, H, 1, 1, sp, C.byref(st)) == 0
        torch.cuda.synchronize()
        img = fb.cpu()
        key = (st.num_primary_rays, st.num_intersection_hits, st.num_shadow_rays)
        if ref is None:
            ref = (img, key)
        same = bool(torch.equal(img, ref[0])) and key == ref[1]
        a, b = C.c_int64(), C.c_int64()
        extra = ""
        if hasattr(lib, "rt_scene_last_batch") and lib.rt_scene_last_batch(h, C.byref(a), C.byref(b)) == 0:
            extra = f" batched={a.value} fallback={b.value}"
        info[f"{name}/{f:#x}"] = {"same": same}
        print(f"  {name} flags={f:#x}: stats={key} identical={same}{extra}", flush=True)
    times = {f"{n}/{f:#x}": [] for n, f, *_ in runs}
    for _ in range(reps):
        for name, f, lib, h, o in runs:
            lib.rt_render_lines_device(h, C.byref(o), C.c_void_p(fb.data_ptr()), 0, H, 1, 1, sp, None)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(3):
                lib.rt_render_lines_device(h, C.byref(o), C.c_void_p(fb.data_ptr()), 0, H, 1, 1, sp, None)
            e1.record(stream)
            torch.cuda.synchronize()
            times[f"{name}/{f:#x}"].append(e0.elapsed_time(e1) / 3)
    res = {k: {"min_ms": round(min(v), 3), "med_ms": round(sorted(v)[len(v) // 2], 3), **info[k]}
           for k, v in times.items()}
    print(json.dumps(res, indent=1), flush=True)
    json.dump(res, open("gpurun_out/ab_flags.json", "w"), indent=1)


if __name__ == "__main__":
    main()
