# Per-kernel durations (serial two-class launch) and SQ instruction mix of
# the C3 render call, batched general kernel vs RT_FLAG_NO_BATCH.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/pmcgen
mkdir -p $O
K='k_render_fast<false|k_render_lean<|k_render_gen<'
for f in 0 0x20; do
  RTMI_FLAGS=$f RTMI_SPLIT_SERIAL=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/kt$f -o s -f csv -- python3 tools/time_c3.py > $O/t$f.json 2> $O/kt$f.err || exit 1
  RTMI_FLAGS=$f timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "$K" -d $O/pmc$f -o p -f csv -- python3 tools/time_c3.py > /dev/null 2> $O/pmc$f.err || exit 1
done
python - <<'PY'
import csv, glob, collections, sys
sys.path.insert(0, "tools")
import pmc_summary as m
O = "gpurun_out/pmcgen"
for f in ("0", "0x20"):
    print("== flags", f)
    for p in glob.glob(f"{O}/kt{f}/**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if "render" in r["Name"]:
                print(f"  {r['Name'][:60]:60s} calls={r['Calls']} avg_ms={float(r['AverageNs'])/1e6:.3f}")
    for p in glob.glob(f"{O}/pmc{f}/**/*counter_collection.csv", recursive=True):
        for k, cs in m.means(p, r"k_render_fast<false|k_render_lean<|k_render_gen<").items():
            print(f"  {k[:60]:60s}", {c: f"{v:.4g}" for c, v in sorted(cs.items())})
PY
