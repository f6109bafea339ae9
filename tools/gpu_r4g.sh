# Round 4: render time against launch size / layout; build2 without per-pixel skip tests (diagnostic).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4g}
mkdir -p $O
timeout -k 10 300 python tools/render_curve.py > $O/render_curve.jsonl 2> $O/rc.err || { tail $O/rc.err; exit 1; }
cat $O/render_curve.jsonl
for sh in 8 16 32; do RTMI_SHARDS=$sh WORLDS=8 timeout -k 10 100 python tools/render_curve.py > $O/rc_sh$sh.jsonl 2>> $O/rc.err || exit 1; echo "shards $sh"; cat $O/rc_sh$sh.jsonl; done
for dg in 2 3; do RTMI_DIAG_B2=$dg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/pd8_$dg -o run -f csv -- python3 tools/rank_prof.py > $O/rd8_$dg.log 2>&1 || exit 1; done
for dg in 2 3; do RTMI_DIAG_B2=$dg timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/pd1_$dg -o run -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/rd1_$dg.log 2>&1 || exit 1; done
RTMI_B2_WAVES=8 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/pw8 -o run -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/bw8.json 2> $O/bw8.err || exit 1
RTMI_DIAG_B2=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/pdiag -o run -f csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/bdiag.json 2> $O/bdiag.err || exit 1
python3 - <<PY
import csv, glob
for d in sorted(glob.glob("$O/p*/run_kernel_stats.csv")):
    print(d)
    for r in csv.DictReader(open(d)):
        if 'frame' in r['Name'] or 'render' in r['Name']:
            print("  ", r['Name'][:58].ljust(58), r['Calls'], round(float(r['AverageNs'])/1000,2))
PY
