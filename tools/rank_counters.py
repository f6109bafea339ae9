"""Per-kernel means of one tools/rank_prof.py run under rocprofv3 (kernel
trace + PMC passes, tools/ab-style job dirs): durations, issue counts, L2
hit rate and HBM fetch per call, to compare one rank of N with the whole
frame (the C5 per-rank efficiency).

    python tools/rank_counters.py <dir with trace/ fetch/ tcc/ sq/> [<dir> ...]
"""
import collections
import csv
import glob
import json
import os
import sys


def short(n):
    for k in ("k_render_mix1", "k_render_gen1", "k_render_lean1q", "k_render_fast", "k_frame_build1",
              "k_frame_build2", "k_frame_lists"):
        if k in n:
            return k
    return None


def pmc(path):
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            if k is None:
                continue
            agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
            disp[(k, r["Counter_Name"])].add(r["Dispatch_Id"])
    return {kc: v / len(disp[kc]) for kc, v in agg.items()}


def trace(path, skip=2):
    rows = []
    for f in glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    d = collections.defaultdict(list)
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        k = short(r["Kernel_Name"])
        if k:
            d[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: sum(v[skip:]) / max(1, len(v[skip:])) for k, v in d.items()}


def main(dirs):
    for dname in dirs:
        t = trace(os.path.join(dname, "trace"))
        c = {}
        for sub in ("fetch", "tcc", "sq"):
            c.update(pmc(os.path.join(dname, sub)))
        out = {"dir": dname, "kernels": {}}
        for k, us in sorted(t.items()):
            e = {"us": round(us, 2)}
            g = {cn: v for (kk, cn), v in c.items() if kk == k}
            if "FETCH_SIZE" in g:
                e["hbm_fetch_MB"] = round(2 * g["FETCH_SIZE"] * 1024 / 1e6, 2)  # gfx950: x2 (MI355X_MICROARCH.md)
            if "TCC_HIT_sum" in g and "TCC_MISS_sum" in g:
                e["l2_hit"] = round(g["TCC_HIT_sum"] / max(1.0, g["TCC_HIT_sum"] + g["TCC_MISS_sum"]), 4)
                e["l2_req_M"] = round((g["TCC_HIT_sum"] + g["TCC_MISS_sum"]) / 1e6, 2)
            for cn in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
                       "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAVES"):
                if cn in g:
                    e[cn] = round(g[cn] / 1e6, 3)
            out["kernels"][k] = e
        print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1:])
