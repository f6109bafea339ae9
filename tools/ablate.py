"""Ablation timing of k_render on C3 variants (kernel time via HIP events)."""
import sys, os, json, dataclasses
sys.path.insert(0, 'nim-raytracer_amd')
import torch
from rtmi import Antialias, Options, Precision, akGrid, scenes
from rtmi.abi import RT_FLAG_COUNT_TRAVERSAL
from rtmi.renderer import DeviceScene

def timeit(ds, opts, n=5):
    fb = torch.zeros(opts.width * opts.height * 3, dtype=torch.float32, device='cuda')
    st = ds.render_device(opts, fb)
    ds.render_device(dataclasses.replace(opts, flags=opts.flags | RT_FLAG_COUNT_TRAVERSAL), fb)
    cnt = ds.last_counters()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(n):
        ds.render_device(opts, fb, stream=s, stats=False)
    e1.record(s); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    rays = st.numPrimaryRays + st.numShadowRays
    return dict(ms=round(ms, 3), grays=round(rays / ms / 1e6, 2), prim=st.numPrimaryRays, shadow=st.numShadowRays,
                tests=st.numIntersectionTests, **cnt)

base = scenes.mesh_bunny()
opts = Options(width=1920, height=1080, antialias=Antialias(akGrid, 16), bias=1e-4, precision=Precision.fp32)
variants = {}
variants['c3_full'] = (base, opts)
s = scenes.mesh_bunny(); s.lights = []; variants['c3_nolights'] = (s, opts)
s = scenes.mesh_bunny(); s.lights = s.lights[:1]; variants['c3_1light'] = (s, opts)
s = scenes.mesh_bunny(); s.objects = [s.objects[1]]; variants['ground_only'] = (s, opts)
s = scenes.mesh_bunny(); s.objects = [s.objects[0]]; variants['bunny_only'] = (s, opts)
s = scenes.mesh_bunny(); s.objects = [s.objects[1]]; s.lights = []; variants['ground_nolights'] = (s, opts)
variants['c3_1spp'] = (base, dataclasses.replace(opts, antialias=Antialias(akGrid, 1)))
variants['c3_64spp'] = (base, dataclasses.replace(opts, antialias=Antialias(akGrid, 8)))
sel = os.environ.get('ABLATE', '')
if sel:
    variants = {k: v for k, v in variants.items() if k in sel.split(',')}
out = {}
for k, (sc, o) in variants.items():
    ds = DeviceScene(sc)
    out[k] = timeit(ds, o)
    print(k, out[k], flush=True)
    ds.close()
json.dump(out, open('gpurun_out/ablate%s.json' % os.environ.get('TAG', ''), 'w'), indent=1)
