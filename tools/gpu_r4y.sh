# Round 4 diagnostic: C3's two pixel classes timed apart (RT_FLAG_NO_MIX with
# the lean kernel serialised behind the general one) + their VALU / SALU.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r4y}
mkdir -p $O
RTMI_SPLIT_SERIAL=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/t -o run -f csv -- python3 tools/scene_times.py mesh-bunny+0x400:1920x1080:16 mesh-bunny:1920x1080:16 > $O/st.log 2>&1 || { tail $O/st.log; exit 1; }
cat $O/st.log | tail -3
python3 - <<PY
import csv
for r in csv.DictReader(open("$O/t/run_kernel_stats.csv")):
    if 'render' in r['Name']: print(r['Name'][:60].ljust(60), r['Calls'], round(float(r['AverageNs'])/1000,1))
PY
RTMI_SPLIT_SERIAL=1 timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY --kernel-include-regex "k_render" -d $O/p -o p -f csv -- python3 tools/scene_times.py mesh-bunny+0x400:1920x1080:16 > /dev/null 2> $O/p.err || exit 1
python3 - <<PY
import csv, collections
agg=collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open("$O/p/p_counter_collection.csv")):
    agg[r['Kernel_Name'][:50]][r['Counter_Name']].append(float(r['Counter_Value']))
for k,cs in agg.items():
    print(k, {c: round(sum(v)/len(v)/1e6,2) for c,v in cs.items()})
PY
