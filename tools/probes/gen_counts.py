"""Diagnostic (a -DRTMI_DIAG_GEN_COUNT build via RTMI_LIB): the batched general
kernel's shadow-search counters for one C3 frame."""
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "nim-raytracer_amd"))
import torch  # noqa: E402

from rtmi import Antialias, Options, Precision, akGrid, scenes  # noqa: E402
from rtmi.renderer import DeviceScene  # noqa: E402

ds = DeviceScene(scenes.mesh_bunny())
o = Options(width=1920, height=1080, antialias=Antialias(akGrid, 16), bias=1e-4, precision=Precision.fp32)
fb = torch.zeros(1920 * 1080 * 3, dtype=torch.float32, device="cuda")
ds.render_device(o, fb)
ds.render_device(o, fb)
c = ds.last_counters()
print(json.dumps({"split": ds.last_split(), "batch": ds.last_batch(), "cells_searched": c["wave_node_fetches"],
                  "face_x_samples": c["wave_tri_fetches"], "searched_visits": c["lane_node_visits"],
                  "batches": c["lane_tri_tests"]}))
