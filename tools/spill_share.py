"""Share of a kernel's VALU instructions that are SGPR-spill lane moves
(v_writelane / v_readlane), estimated from its gfx950 assembly: static
counts per loop depth (LLVM's "Loop Header: Depth=N" block comments),
weighted by an assumed trip count per loop level (4 and 8 per level). The
hot loops (depth >= 4: face tests, cell walks) hold almost none of the
spill code, so the weighted share bounds the dynamic one from above for
any loop whose trip count is at least that (report issue
net of spills).

    python tools/spill_share.py [out.json]   # compiles the float32 and float64 TUs (-S)
"""
import collections
import json
import os
import re
import subprocess
import sys

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
PKG = os.path.join(REPO, "nim-raytracer_amd")
F32 = ["-ffp-contract=fast", "-Xclang", "-target-feature", "-Xclang", "-packed-fp32-ops", "-mllvm",
       "-amdgpu-atomic-optimizer-strategy=None"]
KERNELS = {
    "csrc/rt_kernels_f32.hip": (F32, [r"k_render_mix1ILi2ELi4E"]),
    "csrc/rt_kernels_f64.hip": (["-ffp-contract=off"], [r"k_render_px64ILi4ELi1E"]),
}


def asm(src, flags):
    out = "/tmp/spill_share_%s.s" % os.path.basename(src)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S",
                    src, "-o", out] + flags, cwd=PKG, check=True, capture_output=True)
    return open(out).read().split("\n")


def analyse(lines, pat):
    st = next(i for i, l in enumerate(lines) if re.match(r"^_Z\w*%s\w*:" % pat, l))
    en = next(i for i in range(st, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    depth, cnt = 0, collections.defaultdict(collections.Counter)
    for l in lines[st:en]:
        t = l.strip()
        m = re.search(r"Depth=(\d+)", l)
        if t.startswith(".LBB"):
            depth = int(m.group(1)) if m else 0
        if t.startswith("v_"):
            op = t.split()[0]
            cnt[depth]["spill" if op.startswith(("v_readlane", "v_writelane")) else "other"] += 1
    res = {"by_loop_depth": {d: dict(c) for d, c in sorted(cnt.items())}}
    sp = sum(c["spill"] for c in cnt.values())
    tot = sp + sum(c["other"] for c in cnt.values())
    res["static_share"] = round(sp / tot, 4)
    for w in (4, 8):
        s = sum(c["spill"] * w ** d for d, c in cnt.items())
        a = sum((c["spill"] + c["other"]) * w ** d for d, c in cnt.items())
        res[f"weighted_share_{w}_per_level"] = round(s / a, 5)
    return res


def main(out=None):
    sys.path.insert(0, PKG)
    from rtmi._lib import kernel_source_hash
    res = {"source_hash": kernel_source_hash(), "kernels": {}}
    for src, (flags, pats) in KERNELS.items():
        lines = asm(src, flags)
        for pat in pats:
            res["kernels"][pat] = analyse(lines, pat)
    js = json.dumps(res, indent=1)
    print(js)
    if out:
        open(out, "w").write(js + "\n")


if __name__ == "__main__":
    main(*sys.argv[1:])
