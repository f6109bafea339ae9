import ctypes as C, os, sys
sys.path.insert(0, 'nim-raytracer_amd')
mode = sys.argv[1]
if mode == 'torch_first':
    import torch
    print('torch avail', torch.cuda.is_available(), torch.cuda.device_count())
from rtmi import _lib
l = _lib.lib()
print('rt_device_count', l.rt_device_count())
print('rt_init', l.rt_init(0), l.rt_last_error())
maps = open('/proc/self/maps').read()
print(sorted(set(ln.split()[-1] for ln in maps.splitlines() if 'amdhip' in ln or 'hsa-runtime' in ln)))
print('HIP_VISIBLE_DEVICES', os.environ.get('HIP_VISIBLE_DEVICES'), 'ROCR', os.environ.get('ROCR_VISIBLE_DEVICES'), 'CUDA', os.environ.get('CUDA_VISIBLE_DEVICES'))
