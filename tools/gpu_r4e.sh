# Round 4: build tests, C3 bench + kernel trace, per-rank (N=8) kernel trace, scaling projection.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4e}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_dropin.py tests/test_gpu_split.py -m gpu -x -q --timeout 200 --timeout-method thread > $O/tests_build.log 2>&1 || { tail -40 $O/tests_build.log; exit 1; }
tail -2 $O/tests_build.log
timeout -k 10 300 python bench.py --no-cpu > $O/bench_c3.json 2> $O/bench_c3.err || exit 1
cut -c1-300 $O/bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/bench_prof.json 2> $O/prof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run -f csv -- python3 tools/rank_prof.py > $O/rank_prof.log 2> $O/rank_prof.err || exit 1
BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/scaling_sim.json 2> $O/ss.err || exit 1
cat $O/scaling_sim.json
python3 - <<PY
import csv
for d in ("prof", "prof8"):
    print(d)
    for r in csv.DictReader(open("$O/%s/run_kernel_stats.csv" % d)):
        print(r['Name'][:60].ljust(60), r['Calls'], round(float(r['AverageNs'])/1000,2))
PY
