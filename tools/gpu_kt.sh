# per-kernel times of the C3 call (serial two-class launch) + call time serial vs concurrent
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/kt
rm -rf $O; mkdir -p $O
RTMI_SPLIT_SERIAL=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o s -f csv -- python3 tools/time_c3.py > $O/kt.json 2> $O/kt.err || exit 1
python - <<'PY'
import csv, glob
for p in glob.glob("gpurun_out/kt/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "render" in r["Name"]:
            print(f"{r['Name'][:60]:60s} calls={r['Calls']} avg_ms={float(r['AverageNs'])/1e6:.4f}")
PY
for i in 1 2; do
RTMI_SPLIT_SERIAL=1 REPS=7 timeout -k 10 120 python tools/time_c3.py || exit 1
REPS=7 timeout -k 10 120 python tools/time_c3.py || exit 1
done
