# Round 4: n1 / n2 on C5: lane occupancy of the general
# pixels' searches (RTMI_DIAG_LANES build), LDS staging A/B on C5 and C3;
# then the multi-GPU projection (per-rank times + rank-0 kernel trace at N=8).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4h}
mkdir -p $O
RTMI_LIB=tools/ab/lanes.so RTMI_STAT_FLUSH=1 timeout -k 10 300 python tools/lanes_probe.py > $O/lanes.jsonl 2> $O/lanes.err || { tail $O/lanes.err; exit 1; }
cat $O/lanes.jsonl
for v in base lds; do
  L=""; [ $v = lds ] && L=tools/ab/lds.so
  RTMI_LIB=$L timeout -k 10 300 python bench.py --config C5 --steps 3 --warmup 1 --no-cpu > $O/c5_$v.json 2> $O/c5_$v.err || exit 1
  RTMI_LIB=$L timeout -k 10 200 python bench.py --steps 10 --warmup 2 --no-cpu > $O/c3_$v.json 2> $O/c3_$v.err || exit 1
  echo $v; cut -c1-200 $O/c5_$v.json; cut -c1-200 $O/c3_$v.json
done
BANDS=4 timeout -k 10 300 python tools/scaling_sim.py > $O/scaling_sim.json 2> $O/ss.err || exit 1
cat $O/scaling_sim.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof8 -o run -f csv -- python3 tools/rank_prof.py > $O/rank_prof.log 2> $O/rank_prof.err || exit 1
python3 - <<PY
import csv
for r in csv.DictReader(open("$O/prof8/run_kernel_stats.csv")):
    print(r['Name'][:60].ljust(60), r['Calls'], round(float(r['AverageNs'])/1000,2))
PY
