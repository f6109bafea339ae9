"""Debug: per library build, pixels where the binned frame differs from the
RT_FLAG_NO_BINNING frame (bunny scene, 200x120, akGrid m)."""
import ctypes as C
import os
import sys

sys.path.insert(0, "nim-raytracer_amd")
import torch  # noqa: E402

from rtmi import abi, scenes  # noqa: E402
from rtmi.scene import Antialias, Options, Precision, akGrid, flatten  # noqa: E402

W, H, M = 200, 120, int(os.environ.get("M", "16"))
for path in os.environ["RTMI_LIBS"].split(","):
    lib = abi.bind(C.CDLL(path))
    assert lib.rt_init(0) == 0
    flat = flatten(scenes.mesh_bunny())
    h = C.c_void_p()
    assert lib.rt_scene_create(C.byref(flat.desc), C.byref(h)) == 0, lib.rt_last_error()
    imgs = []
    for flags in (0, abi.RT_FLAG_NO_BINNING):
        o = Options(width=W, height=H, antialias=Antialias(akGrid, M), bias=1e-4, precision=Precision.fp32,
                    flags=flags).to_c()
        fb = torch.zeros(W * H * 3, dtype=torch.float32, device="cuda")
        st = abi.rt_stats()
        assert lib.rt_render_lines_device(h, C.byref(o), C.c_void_p(fb.data_ptr()), 0, H, 1, 1, None, C.byref(st)) == 0
        torch.cuda.synchronize()
        imgs.append(fb.view(H, W, 3).cpu())
    d = (imgs[0] - imgs[1]).abs().amax(dim=2)
    ys, xs = torch.nonzero(d > 0, as_tuple=True)
    print(os.path.basename(path), "differing pixels:", len(ys))
    for y, x in list(zip(ys.tolist(), xs.tolist()))[:12]:
        print("  ", (x, y), imgs[0][y, x].tolist(), imgs[1][y, x].tolist())
    lib.rt_scene_destroy(h)
