# SQ instruction mix per render kernel of the C3 call (default flags), one pass
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmck
rm -rf $O; mkdir -p $O
K='k_render_fast<false|k_render_lean|k_render_gen'
RTMI_MIX=0 timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "$K" -d $O/sq -o p -f csv -- python3 tools/time_c3.py > /dev/null 2> $O/sq.err || exit 1
python - <<'PY'
import glob, sys
sys.path.insert(0, "tools")
import pmc_summary as m
for p in glob.glob("gpurun_out/pmck/sq/**/*counter_collection.csv", recursive=True):
    for k, cs in m.means(p, r"k_render_fast<false|k_render_lean|k_render_gen").items():
        print(f"{k[:50]:50s}", {c: f"{v:.4g}" for c, v in sorted(cs.items())})
PY
# per-kernel durations of the same call, run serially (RTMI_SPLIT_SERIAL)
RTMI_MIX=0 RTMI_SPLIT_SERIAL=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt -o s -f csv -- python3 tools/time_c3.py > $O/kt.json 2> $O/kt.err || exit 1
python - <<'PY'
import csv, glob
for p in glob.glob("gpurun_out/pmck/kt/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "render" in r["Name"]:
            print(f"{r['Name'][:60]:60s} calls={r['Calls']} avg_ms={float(r['AverageNs'])/1e6:.4f}")
PY
