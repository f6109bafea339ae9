# kernel trace of rank-0 band launches at world 1/2/4/8 (tools/host_overhead.py loop)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/tb
rm -rf $O; mkdir -p $O
K=10 timeout -k 10 200 rocprofv3 --kernel-trace -d $O/t -o s -f csv -- python3 tools/host_overhead.py > $O/ho.json 2> $O/ho.err || exit 1
cat $O/ho.json
python - <<'PY'
import csv, glob, collections
rows = []
for p in glob.glob("gpurun_out/tb/t/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(p)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# group consecutive render kernels by grid size
seq = [(r["Kernel_Name"][:40], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
prev_end = None
stats = collections.defaultdict(list)
for name, dur, s, e in seq:
    gap = (s - prev_end) / 1e3 if prev_end else 0
    stats[name].append((dur, gap))
    prev_end = e
for name, v in stats.items():
    print(name, "n", len(v), "dur_us(median)", sorted(d for d, _ in v)[len(v)//2])
# last 30 entries
last = None
for name, dur, s, e in seq[-32:]:
    print(f"{name:40s} {dur:9.1f} us  gap {((s - last) / 1e3 if last else 0):7.1f} us")
    last = e
PY
