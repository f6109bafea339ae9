"""Steady-state timeline of back-to-back render calls from a rocprofv3
kernel trace (tools/rank_prof.py): per call the render kernel's duration,
the period between consecutive render starts, and how much of each build
kernel ran while a render kernel was running (overlap).

    python tools/pipe_timeline.py <run_kernel_trace.csv> [skip]
"""
import csv
import sys

rows = [r for r in csv.DictReader(open(sys.argv[1]))]
skip = int(sys.argv[2]) if len(sys.argv) > 2 else 4
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows), key=lambda x: x[0])
ren = [(a, b) for a, b, n in ks if "k_render" in n][skip:]
bld = [(a, b, n) for a, b, n in ks if "k_frame_" in n]
if len(ren) < 2:
    sys.exit("no render kernels")
per = [(ren[i + 1][0] - ren[i][0]) / 1000 for i in range(len(ren) - 1)]
dur = [(b - a) / 1000 for a, b in ren]
t0, t1 = ren[0][0], ren[-1][1]
out = {"calls": len(ren), "period_us": round(sum(per) / len(per), 2), "render_us": round(sum(dur) / len(dur), 2)}
agg = {}
for a, b, n in bld:
    if a < t0 or b > t1:
        continue
    ov = sum(max(0, min(b, rb) - max(a, ra)) for ra, rb in ren)
    k = [x for x in n.replace("(", " ").replace("<", " ").split() if "k_" in x][0].split("::")[-1]
    d = agg.setdefault(k, [0, 0.0, 0.0])
    d[0] += 1
    d[1] += (b - a) / 1000
    d[2] += ov / 1000
for k, (c, d, o) in agg.items():
    out[k] = {"us": round(d / c, 2), "overlap_us": round(o / c, 2)}
gaps = [(ren[i + 1][0] - ren[i][1]) / 1000 for i in range(len(ren) - 1)]
out["gap_us"] = round(sum(gaps) / len(gaps), 2)
print(out)
