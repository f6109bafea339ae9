"""Read the RTMI_STAMPS diagnostic build's cycle shares (slots 5..8).
    RTMI_LIB=tools/ab/stamps.so ABLATE=c3_full,ground_nolights python tools/stamps.py"""
import ctypes as C, os, sys, json
sys.path.insert(0, "nim-raytracer_amd")
import torch
from rtmi import abi, scenes
from rtmi.scene import Antialias, Options, Precision, akGrid, flatten
lib = abi.bind(C.CDLL(os.environ["RTMI_LIB"]))
assert lib.rt_init(0) == 0
out = {}
for name in os.environ.get("ABLATE", "c3_full").split(","):
    s = scenes.mesh_bunny()
    if name == "ground_only": s.objects = [s.objects[1]]
    if name == "c3_nolights": s.lights = []
    if name == "ground_nolights": s.objects = [s.objects[1]]; s.lights = []
    o = Options(width=1920, height=1080, antialias=Antialias(akGrid, 16), bias=1e-4, precision=Precision.fp32).to_c()
    flat = flatten(s); h = C.c_void_p()
    assert lib.rt_scene_create(C.byref(flat.desc), C.byref(h)) == 0
    fb = torch.zeros(1920 * 1080 * 3, device="cuda")
    st = abi.rt_stats()
    lib.rt_render_lines_device(h, C.byref(o), C.c_void_p(fb.data_ptr()), 0, 1080, 1, 1, None, C.byref(st))
    c = abi.rt_traversal_counters()
    lib.rt_scene_last_counters(h, C.byref(c))
    # wave-cycles (summed over waves) spent in: mesh traversal (slot 5),
    # trace() incl. analytic objects (6), shade_path per sample (7), whole
    # pixel-group items incl. placement, reduction and store (8)
    d = {"cyc_traverse": c.wave_node_fetches, "cyc_trace": c.wave_tri_fetches, "cyc_shade_path": c.lane_node_visits,
         "cyc_item": c.lane_tri_tests}
    d["share"] = {k: round(v / max(1, d["cyc_item"]), 3) for k, v in list(d.items())}
    print(name, d, flush=True)
    out[name] = d
json.dump(out, open("gpurun_out/stamps.json", "w"), indent=1)
