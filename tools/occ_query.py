"""Print the render kernel's resident blocks per CU (occupancy API) for each build."""
import ctypes as C
import glob
import sys

import torch  # noqa: F401  (one HIP runtime)

for p in sys.argv[1:] or sorted(glob.glob("tools/ab/*.so")):
    lib = C.CDLL(p)
    lib.rt_init(0)
    print(p, "blocks/CU:", lib.rtmi_render_f32_blocks_per_cu(0))
