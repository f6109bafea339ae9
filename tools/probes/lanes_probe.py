"""Lane occupancy of the general pixels' face-list searches (row n2,
VERDICT r3): with a RTMI_DIAG_LANES build (tools/build_variant.sh lanes
"-DRTMI_DIAG_LANES") and RTMI_STAT_FLUSH=1, k_render_gen1 counts per face
test of each flagged sample the lanes still searching: shadow (light-grid
cell) searches in wave_node_fetches / lane_node_visits, camera (pixel list)
searches in wave_tri_fetches / lane_tri_tests. Occupancy = lanes / (64 x
tests). Prints one JSON line per scene.

    RTMI_LIB=tools/ab/lanes.so RTMI_STAT_FLUSH=1 python tools/lanes_probe.py
"""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nim-raytracer_amd"))
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

CASES = [("C3", scenes.mesh_bunny, 1920, 1080, 16), ("C5", scenes.torus_scene, 3840, 2160, 64)]
for name, mk, w, h, m in CASES:
    ds = DeviceScene(mk())
    o = Options(width=w, height=h, antialias=Antialias(akGrid, m), bias=1e-4, precision=Precision.fp32)
    fb = torch.zeros(w * h * 3, dtype=torch.float32, device="cuda")
    st = ds.render_device(o, fb)
    c = ds.last_counters()
    lean, gen = ds.last_split()
    out = {"config": name, "lean_pixels": lean, "general_pixels": gen, **c,
           "shadow_lane_occupancy": c["lane_node_visits"] / max(1, 64 * c["wave_node_fetches"]),
           "camera_lane_occupancy": c["lane_tri_tests"] / max(1, 64 * c["wave_tri_fetches"]),
           "primary": st.numPrimaryRays, "shadow": st.numShadowRays}
    print(json.dumps(out), flush=True)
