# Round 4: per-rank kernel traces at N = 2, 4, 8 (and lean lanes-per-pixel A/B), C3 bench.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4f}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_split.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_build.log 2>&1 || { tail -40 $O/tests_build.log; exit 1; }
tail -1 $O/tests_build.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/prof.err || exit 1
for cfg in "2 0" "4 0" "8 0" "8 4" "4 16" "2 16"; do
  set -- $cfg
  WORLD=$1 RTMI_LEAN_LP=$2 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p$1_$2 -o run -f csv -- python3 tools/rank_prof.py > $O/rp$1_$2.log 2> $O/rp$1_$2.err || exit 1
done
python3 - <<PY
import csv, glob
for d in sorted(glob.glob("$O/p*/run_kernel_stats.csv")):
    print(d)
    for r in csv.DictReader(open(d)):
        if 'frame' in r['Name'] or 'render' in r['Name']:
            print("  ", r['Name'][:58].ljust(58), r['Calls'], round(float(r['AverageNs'])/1000,2))
PY
