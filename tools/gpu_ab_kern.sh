# per-kernel durations (separate two-class kernels, serial: RTMI_MIX=0 RTMI_SPLIT_SERIAL=1) for each tools/ab/*.so
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/abk
rm -rf $O; mkdir -p $O
for so in tools/ab/*.so; do
  n=$(basename $so .so)
  RTMI_LIB=$PWD/$so RTMI_MIX=0 RTMI_SPLIT_SERIAL=1 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/$n -o s -f csv -- python3 tools/time_c3.py > $O/$n.json 2> $O/$n.err || exit 1
done
python - <<'PY'
import csv, glob, os
for d in sorted(glob.glob("gpurun_out/abk/*/")):
    n = os.path.basename(d.rstrip("/"))
    row = []
    for p in glob.glob(d + "**/*kernel_stats.csv", recursive=True):
        for r in csv.DictReader(open(p)):
            if "render" in r["Name"]:
                row.append(f"{r['Name'].split('::')[-1][:24]}={float(r['AverageNs'])/1e6:.3f}")
    print(n, " ".join(sorted(row)))
PY
