"""Summarise per-scene A/B logs (ab_<variant>_<rep>.log files of
`<scene> {scene_times dict}` lines, as tools/scene_times.py prints them): per
scene, each variant's minimum over the repetitions of one scene_times field
(default render_ms).

    python tools/ab_report.py gpurun_out/ab [render_ms|setup_ms|call_ms]
"""
import ast,glob,collections,sys
key=sys.argv[2] if len(sys.argv)>2 else 'render_ms'
r=collections.defaultdict(list); vs=[]
for f in sorted(glob.glob(sys.argv[1]+'/ab_*.log')):
    v=f.split('ab_')[1].rsplit('_',1)[0]
    if v not in vs: vs.append(v)
    for l in open(f):
        if 'amdgpu.ids' in l or not l.strip() or l.startswith('#'): continue
        k,d=l.split(' ',1); d=ast.literal_eval(d); r[(k,v)].append(d[key])
for k in sorted(set(k for k,_ in r)):
    print(f'{k:34s}', '  '.join(f"{v}:{min(r[(k,v)]):.4f}" for v in vs if (k,v) in r))
