set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export CASES=bunny:16,bunny:8
for pol in "1 0.5" "3 0.5" "3 0.25" "3 0.75" "4 0.5" "4 0.25"; do
  set -- $pol
  RTMI_ORDER=$1 RTMI_ORDER_P=$2 timeout -k 10 200 python tools/tail_probe.py >> gpurun_out/pol.log 2>&1 || exit 1
done
cat gpurun_out/pol.log
