"""Which of two builds' float32 frames is closer to the float64 (oracle-exact)
frame where they differ.  RTMI_LIBS=a.so,b.so python tools/order_check.py"""
import ctypes as C
import json
import os
import sys

sys.path.insert(0, "nim-raytracer_amd")
import torch  # noqa: E402

from rtmi import abi, scenes  # noqa: E402
from rtmi.scene import Antialias, Options, Precision, akGrid, flatten  # noqa: E402

libs = os.environ["RTMI_LIBS"].split(",")
L = [abi.bind(C.CDLL(p)) for p in libs]
for lib in L:
    assert lib.rt_init(0) == 0
scene = scenes.mesh_bunny()
flat = flatten(scene)
W, H = 1920, 1080
out = {}


def render(lib, prec):
    h = C.c_void_p()
    assert lib.rt_scene_create(C.byref(flat.desc), C.byref(h)) == 0, lib.rt_last_error()
    o = Options(width=W, height=H, antialias=Antialias(akGrid, 16), bias=1e-4, precision=prec).to_c()
    fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
    st = abi.rt_stats()
    assert lib.rt_render_lines_device(h, C.byref(o), C.c_void_p(fb.data_ptr()), 0, H, 1, 1, None, C.byref(st)) == 0
    torch.cuda.synchronize()
    lib.rt_scene_destroy(h)
    return fb.view(H, W, 3).cpu(), st


ref, rst = render(L[0], Precision.fp64)
imgs = [render(lib, Precision.fp32) for lib in L]
a, b = imgs[0][0], imgs[1][0]
diff = (a - b).abs().amax(dim=2) > 1e-6
ys, xs = torch.nonzero(diff, as_tuple=True)
out["n_diff_pixels"] = int(diff.sum())
for name, (img, st) in zip(libs, imgs):
    e = (img - ref).abs().amax(dim=2)
    out[os.path.basename(name)] = {"hits": st.num_intersection_hits, "err_on_diff_pixels_mean": float(e[diff].mean()),
                                   "err_all_mean": float(e.mean()), "frac_err_gt_2e-3": float((e > 2e-3).float().mean())}
out["fp64_hits"] = rst.num_intersection_hits
out["sample_pixels"] = [(int(y), int(x)) for y, x in zip(ys[:20], xs[:20])]
print(json.dumps(out, indent=1))
