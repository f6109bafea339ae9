"""Scheduling simulation of one rank's render launch from a whole-frame cost
map (tools/probes/cost_dump_frame.py): does the order in which the general
pixels are handed out set the launch's tail?

    python tools/probes/sched_sim.py gpurun_out/costmap_c3.npz [rank] [world]

Model: W resident waves (7 per SIMD x 4 SIMDs x 256 CUs), dealt round robin
to SIMDs; a SIMD serves its active waves at a total rate min(n, SAT) / SAT
(latency-bound below SAT waves), shared equally; a pixel's measured cost
(wave cycles while 7 waves shared its SIMD) is 7 x its work at full rate.
Items: the rank's general pixels (cost above LEAN_X x the median: the
pixels a lean item could not hold), one per item, in the given order, then
the lean pixels in items of 16. Prints the makespan (cycles) per order."""
import json
import sys

import numpy as np

path = sys.argv[1]
rank = int(sys.argv[2]) if len(sys.argv) > 2 else 0
world = int(sys.argv[3]) if len(sys.argv) > 3 else 8
SAT, WPS, SIMDS, LEAN_X, DT = 3.0, 7, 1024, 3.0, 400.0
cost = np.load(path)["cost"].astype(np.float64)
H, W = cost.shape
rows = [y for y in range(H) if (y // 4) % world == rank]
sub = cost[rows]
med = float(np.median(sub))
# tile order: 64 x 4 tiles, row-major over tiles; the band's 4 rows = one tile row
ys, xs = np.meshgrid(np.arange(len(rows)), np.arange(W), indexing="ij")
tile = (ys // 4) * ((W + 63) // 64) + xs // 64
order = np.lexsort((xs.ravel(), (ys % 4).ravel(), tile.ravel()))  # tile, then row within tile, then x
flat = sub.ravel()[order]
gen = flat[flat > LEAN_X * med]
lean = flat[flat <= LEAN_X * med]
lean_items = np.add.reduceat(lean, np.arange(0, len(lean), 16)) if len(lean) else np.zeros(0)
NW = WPS * 4 * 256


def makespan(items):
    work = items / 7.0  # full-rate cycles
    rem = np.zeros(NW)
    nxt = 0
    t = 0.0
    simd = np.arange(NW) % SIMDS
    busy = np.zeros(NW, bool)
    while True:
        idle = np.flatnonzero(~busy)
        k = min(len(idle), len(work) - nxt)
        if k > 0:
            rem[idle[:k]] = work[nxt:nxt + k]
            busy[idle[:k]] = True
            nxt += k
        if not busy.any():
            return t
        n = np.bincount(simd[busy], minlength=SIMDS).astype(np.float64)
        rate = np.minimum(n, SAT) / SAT / np.maximum(n, 1.0)
        rem[busy] -= rate[simd[busy]] * DT
        done = busy & (rem <= 0)
        busy[done] = False
        t += DT


res = {"rank": rank, "world": world, "general": int(len(gen)), "lean_items": int(len(lean_items)),
       "median_cycles": med, "max_over_median": float(flat.max() / med)}
res["tile_order"] = makespan(np.concatenate([gen, lean_items]))
res["heavy_first_true"] = makespan(np.concatenate([np.sort(gen)[::-1], lean_items]))
q = np.quantile(gen, 0.75)
two = np.concatenate([gen[gen >= q], gen[gen < q]])  # top quarter first, tile order within
res["top_quarter_first"] = makespan(np.concatenate([two, lean_items]))
res["ideal_total_work_bound"] = float((gen.sum() + lean_items.sum()) / 7.0 / SIMDS)
print(json.dumps(res))
