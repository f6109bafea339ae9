"""Summarise rocprofv3 --pmc CSVs (one counter set per pass) into
profiles/pmc_summary.json: per render call, the per-dispatch means of every
render kernel (two-class launches: the lean-pixel k_render_lean and the
batched general k_render_gen or the general k_render_fast — one dispatch
each per call) summed over the
kernels, plus the per-kernel means.

HBM bytes per launch = (2 * FETCH_SIZE + WRITE_SIZE) * 1024: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE under-reports wide reads by 2x
(MI355X_MICROARCH.md "HBM"), so it is doubled as that guide prescribes.

    python tools/pmc_summary.py <pmc_dir> <workload_key> [note]
"""
import collections
import csv
import json
import os
import re
import sys

# the render call's kernels (a regex on the kernel name): the render kernels
# and the per-call camera-dependent builders (rt_frame.hip)
RENDER_RE = r"k_render_fast<false|k_render_lean|k_render_gen|k_render_mix1|k_render<double, false|k_render_px64"
KERNEL = RENDER_RE + r"|k_frame_"
RENDER = re.compile(RENDER_RE)


def means(path, kernel=None):
    """{kernel name: {counter: mean per dispatch}} of the matching kernels."""
    pat = re.compile(kernel or KERNEL)
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if not pat.search(r["Kernel_Name"]):
            continue
        agg[(r["Kernel_Name"], r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for (k, _, c), v in agg.items():
        per[k][c].append(v)
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in per.items()}


def main(pmc_dir, key, out="profiles/pmc_summary.json", note=""):
    per_kernel = collections.defaultdict(dict)
    for sub in sorted(os.listdir(pmc_dir)):
        f = os.path.join(pmc_dir, sub, "p_counter_collection.csv")
        if os.path.exists(f):
            for k, cs in means(f).items():
                per_kernel[k].update(cs)
    call = collections.defaultdict(float)    # the render kernels of one call
    setup = collections.defaultdict(float)   # the call's frame builders
    for k, cs in per_kernel.items():
        for c, v in cs.items():
            (call if RENDER.search(k) else setup)[c] += v
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "nim-raytracer_amd"))
    from rtmi._lib import kernel_source_hash
    d = json.load(open(out)) if os.path.exists(out) else {}
    e = {"counters_mean_per_dispatch": dict(call), "setup_counters_per_call": dict(setup),
         "per_kernel": per_kernel, "note": note, "source_hash": kernel_source_hash()}
    if "FETCH_SIZE" in call and "WRITE_SIZE" in call:
        e["hbm_bytes_per_launch"] = (2 * call["FETCH_SIZE"] + call["WRITE_SIZE"]) * 1024
        e["hbm_read_bytes_per_launch"] = 2 * call["FETCH_SIZE"] * 1024
        e["hbm_write_bytes_per_launch"] = call["WRITE_SIZE"] * 1024
    d[key] = e
    json.dump(d, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(e, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], note=sys.argv[3] if len(sys.argv) > 3 else "")
