"""Render-call spans from a rocprofv3 kernel trace (p_kernel_trace.csv).

A two-class launch is two kernels on two streams (the general kernel —
k_render_gen, or k_render_fast — on the caller's stream, k_render_lean on
the scene's aux stream, forked and joined
around the call), so their durations overlap and do not add up to the call;
what the bench's HIP events time is the span from the first kernel's start
to the last one's end. This pairs each k_render_fast<false,...> dispatch
with the k_render_lean dispatch that overlaps it and reports the spans.

    python tools/call_span.py <kernel_trace.csv> [out.json]
"""
import csv
import json
import sys


def spans(path):
    rows = [r for r in csv.DictReader(open(path)) if "k_render_fast<false" in r["Kernel_Name"]
            or "k_render_gen<" in r["Kernel_Name"] or "k_render_lean<" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    fast = [r for r in rows if "k_render_fast" in r["Kernel_Name"] or "k_render_gen" in r["Kernel_Name"]]
    lean = [r for r in rows if "k_render_lean" in r["Kernel_Name"]]
    out = []
    for f in fast:
        f0, f1 = int(f["Start_Timestamp"]), int(f["End_Timestamp"])
        partner = None
        for ln in lean:  # the lean dispatch overlapping (or right after) this one
            l0, l1 = int(ln["Start_Timestamp"]), int(ln["End_Timestamp"])
            if l1 >= f0 and l0 <= f1 + 50_000:
                partner = (l0, l1)
                break
        if partner:
            lean.remove(next(x for x in lean if int(x["Start_Timestamp"]) == partner[0]))
            s0, s1 = min(f0, partner[0]), max(f1, partner[1])
        else:
            s0, s1 = f0, f1
        out.append({"span_ms": (s1 - s0) / 1e6, "general_ms": (f1 - f0) / 1e6,
                    "lean_ms": None if not partner else (partner[1] - partner[0]) / 1e6})
    return out


def main():
    sp = spans(sys.argv[1])
    two = [s for s in sp if s["lean_ms"] is not None]
    res = {"calls": len(sp), "two_class_calls": len(two),
           "mean_span_ms": round(sum(s["span_ms"] for s in two) / max(1, len(two)), 4),
           "mean_general_ms": round(sum(s["general_ms"] for s in two) / max(1, len(two)), 4),
           "mean_lean_ms": round(sum(s["lean_ms"] for s in two) / max(1, len(two)), 4),
           "per_call": sp}
    print(json.dumps({k: v for k, v in res.items() if k != "per_call"}))
    if len(sys.argv) > 2:
        json.dump(res, open(sys.argv[2], "w"), indent=1)


if __name__ == "__main__":
    main()
