"""Per-kernel register / spill / occupancy table of a HIP translation unit.

    python tools/kres.py [-D...] [--filter REGEX] [source.hip]

Compiles the device side with -Rpass-analysis=kernel-resource-usage (the
Makefile's float32 flags) and prints one line per kernel: VGPRs, AGPRs,
SGPRs, VGPR / SGPR spills, scratch bytes per lane, waves per SIMD.
"""
import re
import subprocess
import sys

args = sys.argv[1:]
flt = None
if "--filter" in args:
    i = args.index("--filter")
    flt = re.compile(args[i + 1])
    del args[i:i + 2]
src = [a for a in args if not a.startswith("-")] or ["csrc/rt_kernels_f32.hip"]
defs = [a for a in args if a.startswith("-")]
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast", "-Xclang",
       "-target-feature", "-Xclang", "-packed-fp32-ops", "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "--cuda-device-only",
       "-Rpass-analysis=kernel-resource-usage", "-c", src[0], "-o", "/dev/null"] + defs
out = subprocess.run(cmd, capture_output=True, text=True, cwd="/root/repo/nim-raytracer_amd").stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*?) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
print(f"{'VGPR':>4} {'AGPR':>4} {'SGPR':>4} {'Vsp':>4} {'Ssp':>4} {'scr':>4} {'occ':>3}  kernel")
for r in rows:
    n = subprocess.run(["c++filt", r["name"]], capture_output=True, text=True).stdout.strip()
    if flt and not flt.search(n):
        continue
    print(f"{r.get('VGPRs','?'):>4} {r.get('AGPRs','?'):>4} {r.get('TotalSGPRs','?'):>4} {r.get('VGPRs Spill','?'):>4} "
          f"{r.get('SGPRs Spill','?'):>4} {r.get('ScratchSize [bytes/lane]','?'):>4} {r.get('Occupancy [waves/SIMD]','?'):>3}  {n[:110]}")
